// bhtree.hip -- Barnes-Hut quadtree build + traversal (TsneHelpers.scala:227-264,
// QuadTree.scala:38-152, Cell.scala:31-36) on gfx950.
//
// Equivalence with the reference pointer quadtree (capacity 1, root
// Cell(0, 0, W) with W = max(dX, dY)):
//  * a point's Morton digits are computed by replaying the reference's own
//    fp64 cell arithmetic (child centres x -/+ 0.5*hW, closed containment
//    tests tried in the order NW, NE, SW, SE), so boundary ties and the
//    rounding of non-dyadic W land in the same cell as in the reference;
//  * the reference tree only splits cells holding >= 2 distinct points.
//    Cells with a single occupied child form chains with identical
//    (count, centre of mass); because the criterion max(hW,hH)/D < theta is
//    monotone along such a chain (h halves, D fixed), summarising the chain
//    at its deepest cell gives the same contribution as the reference's
//    walk down it.  The binary radix tree (Karras) over the sorted keys has
//    exactly one node per split; nodes that split inside a quad level are
//    transparent (always opened);
//  * leaves always interact directly; a leaf equal to the query contributes
//    nothing (QuadTree.scala:128); points outside the root cell are not in
//    the tree but still get a force (they are queries).
//  * exact duplicate embedding points get the reference's multiplicities
//    (dup_* kernels below: a leaf holding c copies re-inserts ONE of them
//    when it splits, QuadTree.scala:52-61), replayed from insertion rows.
// Known deviations (documented in DESIGN.md): cells deeper than 31 levels
// are not split further (keys tie: all points interact directly; duplicate
// groups sharing such a cell with other points keep full multiplicity);
// centres of mass are summed in tree order, not insertion order.
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>

#include "bhtree.hpp"

namespace tsne {
namespace {

constexpr int LEVELS = 31;                 // 62 key bits
constexpr uint64_t OUT_KEY = 1ull << 63;   // outside the root cell: sorts last
constexpr int STACK = 320;                 // batch pops (<= 8 cells) while <= STACK/2 entries, then
                                           // depth-first (+3 per level, <= 35 levels): never overflows
constexpr int QREC_V4 = sizeof(QRec) / 16; // 16-byte pieces of a record

// ---- Subtree moments (the all-open fast path, see bh_traverse)
// For a subtree every cell of which a query would open, the reference sums
// 1/(1+D) and (q-y)/(1+D)^2 over all of the subtree's points (A15 at every
// leaf).  With u = y - c about the subtree's bounding-box centre c, v = q - c,
// A = |v|^2, E = D - A = |u|^2 - 2 v.u and B = 1/(1+A):
//   1/(1+D)   = B   sum_k (-B E)^k,        1/(1+D)^2 = B^2 sum_k (k+1) (-B E)^k,
// a series in rho = B max|E| <= B (R^2 + 2 |v| R) (R = the box half-diagonal).
// Truncated at k = MOM_ORDER, every term is a polynomial of degree <= 2k+1 in
// u, so the subtree sums follow from its moments sum u_x^a u_y^b
// (a + b <= MOM_DEG), shifted to the query.  The path is taken only when the
// truncation bound (MOM_ORDER+2) rho^(MOM_ORDER+1) / (1-rho)^2 <= Options::mom_tol (1e-12),
// i.e. the result equals the reference's exact leaf sum to ~1e-14 relative
// (fp64 rounding level); otherwise the dense leaf tile runs.  This turns the
// near-exact O(N^2) phase of a small embedding into
// O(N) moment evaluations.
constexpr int MOM_ORDER = 4;
constexpr int MOM_DEG = 2 * MOM_ORDER + 1;
constexpr int MOM_K = (MOM_DEG + 1) * (MOM_DEG + 2) / 2;
constexpr int MOM_MIN_POINTS = 64;
constexpr int MOM_CHUNK = 2048;
constexpr int MOM_TASKS = 128;  // moment evaluations recorded per query; more -> dense tiles
// moment (a, b), a + b <= MOM_DEG: rows of decreasing length
__host__ __device__ constexpr int midx(int a, int b) { return a * (MOM_DEG + 1) - a * (a - 1) / 2 + b; }
__host__ __device__ constexpr double fact(int k) { return k <= 1 ? 1.0 : k * fact(k - 1); }
__host__ __device__ constexpr double binom(int k, int i) { return fact(k) / (fact(i) * fact(k - i)); }

__global__ void bbox_partial(const double *__restrict__ Y, int64_t n, double *__restrict__ part) {
    __shared__ double sm[4][4];
    double mnx = __builtin_inf(), mxx = -__builtin_inf(), mny = __builtin_inf(), mxy = -__builtin_inf();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double x = Y[2 * i], y = Y[2 * i + 1];
        mnx = fmin(mnx, x); mxx = fmax(mxx, x);
        mny = fmin(mny, y); mxy = fmax(mxy, y);
    }
    mnx = wave_min(mnx); mxx = wave_max(mxx); mny = wave_min(mny); mxy = wave_max(mxy);
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0) { sm[w][0] = mnx; sm[w][1] = mxx; sm[w][2] = mny; sm[w][3] = mxy; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 4; ++k) {
            sm[0][0] = fmin(sm[0][0], sm[k][0]); sm[0][1] = fmax(sm[0][1], sm[k][1]);
            sm[0][2] = fmin(sm[0][2], sm[k][2]); sm[0][3] = fmax(sm[0][3], sm[k][3]);
        }
        for (int k = 0; k < 4; ++k) part[blockIdx.x * 4 + k] = sm[0][k];
    }
}

// One 256-thread block folds the per-block partials.
// Thread 0 also resets the build's counters and takes the moment gate
// (moment_count): mom_flag[0] = the previous traversal saw enough tiles that
// moments would serve (mom_flag[1] >= mom_flag[2]), then mom_flag[1] restarts.
__global__ void bbox_final(const double *__restrict__ part, int nb, double *__restrict__ W,
                           int32_t *__restrict__ meta, double *__restrict__ bb, int32_t *__restrict__ mom_flag,
                           int32_t *__restrict__ mom_items) {
    __shared__ double sm[4][4];
    double mnx = __builtin_inf(), mxx = -__builtin_inf(), mny = __builtin_inf(), mxy = -__builtin_inf();
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        mnx = fmin(mnx, part[4 * b]); mxx = fmax(mxx, part[4 * b + 1]);
        mny = fmin(mny, part[4 * b + 2]); mxy = fmax(mxy, part[4 * b + 3]);
    }
    mnx = wave_min(mnx); mxx = wave_max(mxx); mny = wave_min(mny); mxy = wave_max(mxy);
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0) { sm[w][0] = mnx; sm[w][1] = mxx; sm[w][2] = mny; sm[w][3] = mxy; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 4; ++k) {
            sm[0][0] = fmin(sm[0][0], sm[k][0]); sm[0][1] = fmax(sm[0][1], sm[k][1]);
            sm[0][2] = fmin(sm[0][2], sm[k][2]); sm[0][3] = fmax(sm[0][3], sm[k][3]);
        }
        const double a = sm[0][1] - sm[0][0], c = sm[0][3] - sm[0][2];
        *W = a > c ? a : c;  // scala.math.max(maxX - minX, maxY - minY)
        for (int k = 0; k < 4; ++k) bb[k] = sm[0][k];
        meta[0] = 0;
        meta[2] = 0;
        meta[3] = 0;         // root replaced by its virtual chain top (duplicates, dup_apply)
        if (mom_flag) {
            mom_flag[0] = mom_flag[1] >= mom_flag[2];
            mom_flag[1] = 0;
        }
        if (mom_items) *mom_items = 0;
    }
}

// Morton key by replaying the reference cell arithmetic (no FMA contraction).
// Fast path: away from cell boundaries the replay's digits are those of the
// exact quantisation X = (p + W) / (2W) * 2^31 (every coarser boundary is
// also a level-31 boundary, and the reference's rounded cell centres sit
// within a few ulps of the exact ones), so a point whose fixed-point
// coordinates are more than 1e-4 of a level-31 cell away from every boundary
// takes the quantised digits; the rest (a fraction ~4e-4) and every
// out-of-range case replay the reference arithmetic.
__device__ __forceinline__ bool quant_digits(double p, double W, uint32_t &q) {
    const double t = (p + W) / (2.0 * W) * 2147483648.0;   // in [0, 2^31] for in-root points
    if (!(t >= 0.0 && t < 2147483648.0)) return false;
    const double f = floor(t);
    const double fr = t - f;
    // t carries <= ~3 ulp(2^31) = 1.4e-6 of rounding, the reference's cell
    // centres <= 31 roundings = 7.4e-6 (both in level-31 cell units): a band
    // of 1e-4 is far outside both
    if (fr < 1e-4 || fr > 1.0 - 1e-4) return false;          // near a boundary: replay
    q = (uint32_t)f;
    return true;
}

__global__ void morton_keys(const double *__restrict__ Y, int64_t n, const double *__restrict__ Wp,
                            uint64_t *__restrict__ keys, int32_t *__restrict__ idx,
                            int32_t *__restrict__ meta) {
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i0 < n;
    const int64_t i = live ? i0 : n - 1;
    const double W = *Wp;
    const double px = Y[2 * i], py = Y[2 * i + 1];
    double x = 0.0, y = 0.0, hw = W, hh = W;
    bool in = live && (__dsub_rn(x, hw) <= px) && (__dadd_rn(x, hw) >= px) && (__dsub_rn(y, hh) <= py) &&
              (__dadd_rn(y, hh) >= py);
    uint64_t key = 0;
    uint32_t qx, qy;
    if (in && W > 0.0 && quant_digits(px, W, qx) && quant_digits(py, W, qy)) {
        // digit l: (west/east from x, north/south from y): q = 2 * south + east,
        // south = y below the centre = high bit of qy clear
        uint64_t k = 0;
        for (int l = 30; l >= 0; --l) {
            const uint32_t east = (qx >> l) & 1u, south = 1u - ((qy >> l) & 1u);
            k = (k << 2) | (uint64_t)(2u * south + east);
        }
        key = k;
    } else if (in) {
        for (int l = 0; l < LEVELS; ++l) {
            const double nw = __dmul_rn(0.5, hw), nh = __dmul_rn(0.5, hw);
            const double xw = __dsub_rn(x, nw), xe = __dadd_rn(x, nw);
            const double yn = __dadd_rn(y, nh), ys = __dsub_rn(y, nh);
            const bool inW = (__dsub_rn(xw, nw) <= px) && (__dadd_rn(xw, nw) >= px);
            const bool inE = (__dsub_rn(xe, nw) <= px) && (__dadd_rn(xe, nw) >= px);
            const bool inN = (__dsub_rn(yn, nh) <= py) && (__dadd_rn(yn, nh) >= py);
            const bool inS = (__dsub_rn(ys, nh) <= py) && (__dadd_rn(ys, nh) >= py);
            int q;
            if (inN && inW) q = 0;        // NW
            else if (inN && inE) q = 1;   // NE
            else if (inS && inW) q = 2;   // SW
            else q = 3;                   // SE (or a rounding gap: see header)
            x = (q & 1) ? xe : xw;
            y = (q & 2) ? ys : yn;
            hw = nw;
            hh = nh;
            key = (key << 2) | (uint64_t)q;
        }
    } else {
        key = OUT_KEY;
    }
    if (live) {
        keys[i] = key;
        idx[i] = (int32_t)i;
    }
    (void)meta;   // the in-root count m is read off the sorted keys (count_in_root)
}

// m = number of in-root points = index of the first OUT_KEY in the sorted
// keys: a 64-ary search by one wave (4 rounds of one load per lane at 1M),
// instead of an atomic per wave on one counter (serialised in the L2).
__global__ void count_in_root(const uint64_t *__restrict__ ks, int64_t n, int32_t *__restrict__ meta) {
    const int lane = lane_id();
    int64_t lo = 0, hi = n;   // answer in [lo, hi]
    while (hi > lo) {
        const int64_t step = (hi - lo + 63) / 64;
        const int64_t p = lo + (int64_t)lane * step;   // probe: is ks[p] an out-of-root key?
        const bool out = p < hi && ks[p] >= OUT_KEY;
        const uint64_t b = __ballot(out || p >= hi);
        const int f = b ? __ffsll((long long)b) - 1 : 64;   // first lane whose probe is out (or past hi)
        // first out-of-root index lies in (lo + (f-1) step, lo + f step]
        const int64_t nlo = f == 0 ? lo : lo + (int64_t)(f - 1) * step + 1;
        const int64_t nhi = min(hi, lo + (int64_t)f * step);
        if (f == 0) { hi = lo; break; }
        lo = nlo;
        hi = nhi;
    }
    if (lane == 0) {
        meta[0] = (int32_t)lo;
        meta[1] = lo >= 2 ? 0 : (lo == 1 ? ~0 : INT32_MIN);   // the root ref
    }
}

__global__ void gather_sorted(const double *__restrict__ Y, const int32_t *__restrict__ idx_sorted,
                              int64_t n, double2 *__restrict__ pos, int32_t *__restrict__ inv,
                              const int32_t *__restrict__ pcost, int32_t *__restrict__ pred) {
    int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // (option trav_front_cur: each new 64-query wave's predicted cost, the
    // largest previous cost of its points -- lanes = the wave's queries)
    if (pred) {
        const int32_t c = s < n ? pcost[idx_sorted[s]] : 0;
        const int32_t m = wave_max(c);
        if (lane_id() == 0 && s < n) pred[s >> 6] = m;
    }
    if (s >= n) return;
    int32_t i = idx_sorted[s];
    const double x = Y[2 * i], y = Y[2 * i + 1];
    pos[s] = make_double2(x, y);
    inv[i] = (int32_t)s;
}

// delta between sorted keys i and j (bits of common prefix of the 62-bit
// Morton field; ties extend with the index bits); -1 out of range.
__device__ __forceinline__ int kdelta(const uint64_t *__restrict__ k, int m, int i, int j) {
    if (j < 0 || j >= m) return -1;
    uint64_t a = k[i], b = k[j];
    if (a == b) return 62 + __clz((unsigned)(i ^ j));
    return __clzll((long long)(a ^ b)) - 2;
}

// Bottom-up workgroup ranges (bottom_up_intra): the leaves are cut into
// "frontier" subtrees, the maximal subtrees of <= BU_FRONT leaves; workgroup b
// takes the frontier subtrees that start in [b BU_NB, (b + 1) BU_NB), so every
// node of <= BU_FRONT leaves is combined inside one workgroup (LDS hand-off)
// and only the nodes above the frontier cross workgroups.
constexpr int BU_NB = 1024;
constexpr int BU_FRONT = 512;
constexpr int BU_CAP = BU_NB + BU_FRONT;

// Karras (2012) binary radix tree over the m in-root points.  fstart[p] =
// gen marks p as the first leaf of a frontier subtree (gen: this build's
// number, so no clearing pass is needed).
__global__ void karras_build(const uint64_t *__restrict__ k, int64_t n, const int32_t *__restrict__ meta,
                             BHNode *__restrict__ nodes, int32_t *__restrict__ parent_leaf,
                             int32_t *__restrict__ parent_node, int32_t *__restrict__ arrive,
                             int32_t *__restrict__ arrive2, int32_t *__restrict__ fstart, int32_t gen,
                             int32_t *__restrict__ top_cnt) {
    const int m = meta[0];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m - 1) return;
    if (i == 0 && top_cnt) *top_cnt = 0;
    arrive[i] = 0;
    arrive2[i] = 0;
    const int dr = kdelta(k, m, i, i + 1), dl = kdelta(k, m, i, i - 1);
    const int d = (dr > dl) ? 1 : -1;
    const int dmin = d > 0 ? dl : dr;
    int lmax = 2;
    while (kdelta(k, m, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (kdelta(k, m, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = kdelta(k, m, i, j);
    int s = 0;
    int t = l;
    do {
        t = (t + 1) >> 1;
        if (kdelta(k, m, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + (d < 0 ? -1 : 0);
    const int lo = min(i, j), hi = max(i, j);
    int left, right;
    if (lo == gamma) { left = ~gamma; parent_leaf[gamma] = i; }
    else { left = gamma; parent_node[gamma] = i; }
    if (hi == gamma + 1) { right = ~(gamma + 1); parent_leaf[gamma + 1] = i; }
    else { right = gamma + 1; parent_node[gamma + 1] = i; }
    nodes[i].left = left;
    nodes[i].right = right;
    nodes[i].delta = dnode;
    nodes[i].first = lo;
    nodes[i].last = hi;
    if (i == 0) parent_node[0] = -1;
    if (fstart) {
        if (hi - lo + 1 <= BU_FRONT) {
            if (i == 0) fstart[0] = gen;   // the root is the only frontier subtree
        } else {
            if (gamma - lo + 1 <= BU_FRONT) fstart[lo] = gen;
            if (hi - gamma <= BU_FRONT) fstart[gamma + 1] = gen;
        }
    }
}

// Bottom-up count / sums / bounding box / hmin.  The second thread to reach a
// node computes it from its two children (fixed order: deterministic sums).
// Cross-workgroup hand-off without fences (MI355X_MICROARCH.md, "Valid forms"):
// the per-node aggregates that a sibling thread reads are written and read
// with system-scope (sc0 sc1, write-through / cache-bypassing) 8-byte
// accesses; every thread drains its stores (s_waitcnt vmcnt(0)) before its
// relaxed arrival atomic.  Agent-scope __threadfence() (or an acq_rel
// arrival: buffer_wbl2 + buffer_inv at agent scope) here wrote back the whole
// XCD L2 per wave and cost ~8 ms per build at 1M points.  What orders the
// hand-off instead: the writer's stores complete (vmcnt(0), an asm with a
// memory clobber: also a compiler barrier) before its arrival is issued; the
// reader's loads are issued after its arrival returned (a branch on the
// result, plus a compiler-only signal fence so that the relaxed loads cannot
// be hoisted above the relaxed atomic), and they bypass the non-coherent
// caches (system scope).  This relies on gfx950's in-order issue and
// write-through / bypassing system-scope accesses, not on the HIP memory
// model's release / acquire; it is gfx950-only code like the rest.  Since
// round 5 the default arrival is an agent-scope acquire-release RMW instead
// (bottom_up_top<true>, Options::bu_acqrel): the memory model's own ordering,
// at no measurable cost in the two-phase scheme (the round-1 figure above was
// for every level crossing workgroups); the relaxed form stays as option 0.
__device__ __forceinline__ void st_sys(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double ld_sys(const double *p) {
    return __hip_atomic_load(const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int AGG = 10;   // sx, sy, x0, x1, y0, y1, hmin, cnt, rball, (pad)

// rball: radius of a disc around the node's centre of mass inside which a
// query opens EVERY real cell of the subtree (so the subtree is all leaves
// for it).  A cell u is opened by q iff h_u / D(q, c_u) >= theta, i.e. q lies
// in the disc |q - c_u| <= sqrt(h_u / theta); ball(c_v, R_v) is inside
// ball(c_c, R_c) when R_v + |c_v - c_c| <= R_c, hence
// R_v = min(sqrt(h_v/theta) [real v], R_c - |c_v - c_c| over children c),
// shrunk by a relative 1e-9 per level for rounding.  Leaves impose nothing.
// Node p's aggregates from its two children's (child order fixed: the sums
// are deterministic whichever thread combines them); writes nodes[p] and
// returns the nine aggregates in o[] (sx, sy, x0, x1, y0, y1, hmin, cnt,
// rball) and p's parent.
__device__ __forceinline__ void bu_combine_d(int p, const double (&a)[2][7], const double (&c)[2], const double (&rb)[2],
                                             const int32_t (&ch)[2], int32_t dl, int par, int32_t pdelta, double W,
                                             double inv_theta, BHNode *nodes, double (&o)[9]) {
    const double cnt = c[0] + c[1];
    const double sx = a[0][0] + a[1][0], sy = a[0][1] + a[1][1];
    const double x0 = fmin(a[0][2], a[1][2]), x1 = fmax(a[0][3], a[1][3]);
    const double y0 = fmin(a[0][4], a[1][4]), y1 = fmax(a[0][5], a[1][5]);
    const int dlev = dl >> 1;
    bool real;
    if (dl >= 62) real = false;                      // keys tie below 31 levels
    else if (par < 0) real = true;                   // root cell chain
    else real = (pdelta >> 1) < dlev;                // first node of its quad level
    const double h = real ? ldexp(W, -dlev) : -1.0;  // -1 = transparent
    const double hmin = fmin(real ? h : __builtin_inf(), fmin(a[0][6], a[1][6]));
    const double cx = sx / cnt, cy = sy / cnt;       // centerOfMass = sum / cumSize
    double rball = real ? sqrt(h * inv_theta) : __builtin_inf();
    // the children's centres here only bound rball (shrunk by 1e-9 per level):
    // reciprocal + one Newton step instead of two IEEE divisions each
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (ch[k] >= 0) {
            const double r = __builtin_amdgcn_rcp(c[k]);
            const double ic = __fma_rn(r, __fma_rn(-c[k], r, 1.0), r);
            const double ccx = a[k][0] * ic, ccy = a[k][1] * ic;
            const double dd = sqrt((cx - ccx) * (cx - ccx) + (cy - ccy) * (cy - ccy));
            rball = fmin(rball, rb[k] - dd * (1.0 + 1e-12));
        }
    }
    rball = rball > 0.0 ? rball * (1.0 - 1e-9) : 0.0;
    BHNode &nd = nodes[p];                           // read by the traversal (later launches)
    nd.cx = cx;
    nd.cy = cy;
    nd.cnt = (int32_t)cnt;
    nd.h = h;
    nd.hmin = hmin;
    nd.rball = rball;
    nd.bx0 = x0; nd.bx1 = x1; nd.by0 = y0; nd.by1 = y1;
    o[0] = sx; o[1] = sy; o[2] = x0; o[3] = x1; o[4] = y0; o[5] = y1; o[6] = hmin; o[7] = cnt; o[8] = rball;
}
__device__ __forceinline__ int bu_combine(int p, const double (&a)[2][7], const double (&c)[2], const double (&rb)[2],
                                          const int32_t (&ch)[2], int32_t dl, double W, double inv_theta,
                                          BHNode *nodes, const int32_t *__restrict__ parent_node, double (&o)[9]) {
    const int par = parent_node[p];
    bu_combine_d(p, a, c, rb, ch, dl, par, par >= 0 ? nodes[par].delta : 0, W, inv_theta, nodes, o);
    return par;
}

__device__ __forceinline__ void bu_leaf(const double2 *__restrict__ pos, int s, double (&a)[7], double &c, double &rb) {
    const double2 q = pos[s];
    a[0] = q.x; a[1] = q.y; a[2] = q.x; a[3] = q.x; a[4] = q.y; a[5] = q.y;
    a[6] = __builtin_inf();
    c = 1.0;
    rb = __builtin_inf();
}

// Phase 1 of the bottom-up pass: every node inside the workgroup's leaf range
// [S0, S1) (whole frontier subtrees, see BU_FRONT) is combined through LDS
// arrival counters and aggregates.  A node whose parent lies outside the
// range publishes its aggregates to agg (plain stores: the next launch reads
// them) and appends the parent to the arrival list of phase 2, as does a leaf
// whose parent lies outside.  Nothing waits on another workgroup, so a
// workgroup's run is its own short climb.
// The climbs run in steps over an LDS queue of arrivals: each step every
// queued arrival is taken by one thread (the first arriver at a node stops,
// the second combines it and queues the parent for the next step), so the
// live climbers are packed into the first waves -- a climb per thread kept
// all 16 waves issuing every step for their one or two live lanes (round 5:
// 136 us at C3).  The sums are the same: each node is combined from its two
// children in a fixed order, whichever thread does it.
__global__ __launch_bounds__(BU_NB) void bottom_up_intra(const double2 *__restrict__ pos, const int32_t *__restrict__ meta,
                                                        const double *__restrict__ Wp, double inv_theta, BHNode *nodes,
                                                        double *__restrict__ agg, const int32_t *__restrict__ parent_leaf,
                                                        const int32_t *__restrict__ parent_node,
                                                        const int32_t *__restrict__ fstart, int32_t gen,
                                                        int32_t *__restrict__ top_list, int32_t *__restrict__ top_cnt) {
    // aggregates (sx, sy, x0, x1, y0, y1, hmin, rball) and the topology of the
    // range's nodes (ids [S0, S1), Karras: a node's id lies in its own leaf
    // range: count, children, delta, parent, whether the node lies inside the
    // range), staged once so that the climb never waits on global memory
    __shared__ double lagg[8][BU_CAP];
    __shared__ int32_t lleft[BU_CAP], lright[BU_CAP], ldelta[BU_CAP], lcnt[BU_CAP], lpar[BU_CAP];
    __shared__ int32_t larr[BU_CAP];
    __shared__ int32_t queue[2][BU_CAP];
    __shared__ uint8_t lself[BU_CAP];
    __shared__ int32_t sS[2], qn[2];
    const int m = meta[0];
    const int b = blockIdx.x;
    if (m < 2 || b * BU_NB >= m) return;
    const int t = threadIdx.x;
    if (t < 2) { sS[t] = INT32_MAX; qn[t] = 0; }
    __syncthreads();
    // a frontier subtree starts within any BU_FRONT + 1 consecutive leaves
    for (int j = t; j < 2 * (BU_FRONT + 1); j += BU_NB) {
        const int side = j / (BU_FRONT + 1);
        const int p = (b + side) * BU_NB + (j - side * (BU_FRONT + 1));
        if (p < m && fstart[p] == gen) atomicMin(&sS[side], p);
    }
    __syncthreads();
    const int S0 = b == 0 ? 0 : min(sS[0], m);
    const int S1 = (b + 1) * BU_NB >= m ? m : min(sS[1], m);
    for (int j = t; j < S1 - S0; j += BU_NB) {
        const int q = S0 + j;
        larr[j] = 0;
        if (q < m - 1) {
            const BHNode &nd = nodes[q];
            lleft[j] = nd.left; lright[j] = nd.right; ldelta[j] = nd.delta;
            lcnt[j] = nd.last - nd.first + 1; lpar[j] = parent_node[q];
            lself[j] = nd.first >= S0 && nd.last < S1;
        } else {
            lself[j] = 0;   // not a node: never in range
        }
    }
    __syncthreads();
    const double W = *Wp;
    auto in_blk = [&](int q) { return q >= S0 && q < S1 && lself[q - S0]; };
    // the leaves' arrivals: at a parent in the range (queue 0), or phase 2's
    for (int s = S0 + t; s < S1; s += BU_NB) {
        const int p = parent_leaf[s];
        if (p < 0) continue;
        if (!in_blk(p)) top_list[atomicAdd(top_cnt, 1)] = p;   // a leaf hanging off a node above the frontier
        else queue[0][atomicAdd(&qn[0], 1)] = p;
    }
    int cur = 0;
    while (true) {
        __syncthreads();   // the step's queue complete; the other queue empty
        const int na = qn[cur];
        if (na == 0) break;
        const int nxt = cur ^ 1;
        for (int e = t; e < na; e += BU_NB) {
            const int p = queue[cur][e];
            const int op = p - S0;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (__hip_atomic_fetch_add(&larr[op], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
                continue;                                // first arriver stops
            const int32_t ch[2] = {lleft[op], lright[op]};
            const int32_t dl = ldelta[op];
            double a[2][7], c[2], rb[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (ch[k] < 0) {
                    bu_leaf(pos, ~ch[k], a[k], c[k], rb[k]);
                } else {                                 // children of an in-range node are in range
                    const int o = ch[k] - S0;
#pragma unroll
                    for (int f = 0; f < 7; ++f) a[k][f] = lagg[f][o];
                    c[k] = (double)lcnt[o];
                    rb[k] = lagg[7][o];
                }
            }
            // bu_combine's global reads of the parent, from the staged topology
            const int par = lpar[op];
            const bool pin = par >= 0 && in_blk(par);
            const int32_t pdelta = pin ? ldelta[par - S0] : (par >= 0 ? nodes[par].delta : 0);
            double o9[9];
            bu_combine_d(p, a, c, rb, ch, dl, par, pdelta, W, inv_theta, nodes, o9);
            if (pin) {
#pragma unroll
                for (int f = 0; f < 7; ++f) lagg[f][op] = o9[f];
                lagg[7][op] = o9[8];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                queue[nxt][atomicAdd(&qn[nxt], 1)] = par;
            } else {
                double *g = agg + AGG * (int64_t)p;
#pragma unroll
                for (int f = 0; f < 9; ++f) g[f] = o9[f];
                if (par >= 0) top_list[atomicAdd(top_cnt, 1)] = par;
            }
        }
        __syncthreads();   // every push of the step done
        if (t == 0) qn[cur] = 0;   // consumed: the next step's push queue
        cur = nxt;
    }
}

// Phase 2: the nodes above the frontier.  Each arrival of phase 1 (a child
// published, the parent listed) starts a climb; the second arriver at a node
// combines it (agent-scope arrival counters, system-scope aggregates: the
// hand-off described above st_sys) and climbs on.  Only the top ~log2(m / BU_FRONT) levels remain
// for this cross-workgroup hand-off.
// ACQREL (Options::bu_acqrel = 1, the default): the arrival is an agent-scope
// acquire-release RMW -- the HIP memory model's own ordering of the
// aggregates' stores before it and the sibling's loads after it -- instead of
// relying on gfx950's in-order issue (0).  C3 whole schedule 5.46 / 5.45 s
// (ABAB, round 5): no measurable cost with the two-phase bottom-up, where
// only the top ~log2(m / 512) levels cross workgroups.
template <bool ACQREL>
__global__ __launch_bounds__(256) void bottom_up_top(const double2 *__restrict__ pos, const int32_t *__restrict__ meta,
                                                     const double *__restrict__ Wp, double inv_theta, BHNode *nodes,
                                                     double *agg, const int32_t *__restrict__ parent_node,
                                                     int32_t *arrive, const int32_t *__restrict__ top_list,
                                                     const int32_t *__restrict__ top_cnt) {
    if (meta[0] < 2) return;   // no karras launch reset the count
    const int ne = *top_cnt;
    const double W = *Wp;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += gridDim.x * blockDim.x) {
        int p = top_list[e];
        while (p >= 0) {
            if (ACQREL) {
                if (__hip_atomic_fetch_add(&arrive[p], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 0) break;
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (__hip_atomic_fetch_add(&arrive[p], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) break;
            }
            __atomic_signal_fence(__ATOMIC_SEQ_CST);   // the sibling's aggregates are read after the arrival
            const int32_t ch[2] = {nodes[p].left, nodes[p].right};
            const int32_t dl = nodes[p].delta;
            double a[2][7], c[2], rb[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (ch[k] < 0) {
                    bu_leaf(pos, ~ch[k], a[k], c[k], rb[k]);
                } else {
                    const double *g = agg + AGG * (int64_t)ch[k];
#pragma unroll
                    for (int f = 0; f < 7; ++f) a[k][f] = ld_sys(g + f);
                    c[k] = ld_sys(g + 7);
                    rb[k] = ld_sys(g + 8);
                }
            }
            double o9[9];
            const int par = bu_combine(p, a, c, rb, ch, dl, W, inv_theta, nodes, parent_node, o9);
            double *g = agg + AGG * (int64_t)p;
#pragma unroll
            for (int f = 0; f < 9; ++f) st_sys(g + f, o9[f]);
            p = par;
        }
    }
}

// 1/x for the BH terms: v_rcp_f64 + one Newton step, within 11 ulp of the
// IEEE quotient over the whole range (scripts/rcp_accuracy.hip: rcp alone
// 2.5e8 ulp, one step 11, two steps 0) -- ~2e-15 relative per term, far
// below the 1e-6 near-exact and 1e-4 gradient bars, two fp64 ops per term
// cheaper than the correctly rounded pair of steps.
__device__ __forceinline__ double recip_bh(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    return __fma_rn(r, __fma_rn(-x, r, 1.0), r);
}

// Direct interaction of one lane's query with one leaf point (QuadTree.scala:
// 128-142 at a leaf: cumSize 1, com = the point; zero if equal to the query).
__device__ __forceinline__ void leaf_force(double qx, double qy, double px, double py, double &fx,
                                           double &fy, double &zs) {
    if (px == qx && py == qy) return;
    const double dx = qx - px, dy = qy - py;
    const double D = __fma_rn(dx, dx, dy * dy);
    const double r = recip_bh(1.0 + D);
    const double sc = r * r;
    fx = __fma_rn(sc, dx, fx);
    fy = __fma_rn(sc, dy, fy);
    zs += r;
}

// Masked forms for the traversal's child loop: every lane evaluates, `take`
// selects whether the term is added (a zero term leaves the sums bit-equal).
// Branch-free, so the accumulators are updated in place -- the branchy forms
// made the compiler copy fx, fy, zs at every merge of the divergent paths.
__device__ __forceinline__ void leaf_force_m(bool take, double qx, double qy, double px, double py, double &fx,
                                             double &fy, double &zs) {
    take = take && !(px == qx && py == qy);
    const double dx = qx - px, dy = qy - py;
    const double D = __fma_rn(dx, dx, dy * dy);
    const double r = recip_bh(1.0 + D);
    const double sc = r * r;
    fx = __fma_rn(take ? sc : 0.0, dx, fx);
    fy = __fma_rn(take ? sc : 0.0, dy, fy);
    zs += take ? r : 0.0;
}

// Pair term for dense tiles, without the equality test (see the caller):
// r = 1/(1 + dx^2 + dy^2) with the 1 folded into the FMA chain.
__device__ __forceinline__ void pair_force(double qx, double qy, double px, double py, double &fx,
                                           double &fy, double &zs) {
    const double dx = qx - px, dy = qy - py;
    const double r = recip_bh(__fma_rn(dx, dx, __fma_rn(dy, dy, 1.0)));
    const double sc = r * r;
    fx = __fma_rn(sc, dx, fx);
    fy = __fma_rn(sc, dy, fy);
    zs += r;
}
// pair_force's term added only with `take` (else + 0: the sums bit-equal)
__device__ __forceinline__ void pair_force_m(bool take, double qx, double qy, double px, double py, double &fx,
                                             double &fy, double &zs) {
    const double dx = qx - px, dy = qy - py;
    const double r = recip_bh(__fma_rn(dx, dx, __fma_rn(dy, dy, 1.0)));
    const double sc = r * r;
    fx = __fma_rn(take ? sc : 0.0, dx, fx);
    fy = __fma_rn(take ? sc : 0.0, dy, fy);
    zs += take ? r : 0.0;
}

// Number of points whose coordinates equal pos[s] exactly (itself included);
// they sit in the same equal-key run of the sorted order.
__global__ void dup_count(const double2 *__restrict__ pos, const uint64_t *__restrict__ keys, int64_t n,
                          int32_t *__restrict__ dupc, int32_t *__restrict__ vid, int32_t *__restrict__ dflag) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const double2 q = pos[s];
    const uint64_t k = keys[s];
    int32_t c = 1;
    int64_t first = s;   // value id: the first sorted position holding this exact point
    for (int64_t t = s - 1; t >= 0 && keys[t] == k; --t) {
        const double2 p = pos[t];
        if (p.x == q.x && p.y == q.y) { ++c; first = t; }
    }
    for (int64_t t = s + 1; t < n && keys[t] == k; ++t) {
        const double2 p = pos[t];
        c += (p.x == q.x && p.y == q.y);
    }
    dupc[s] = c;
    vid[s] = (int32_t)first;
    if (c > 1) dflag[0] = 1;
}

// ---- Exact duplicates (QuadTree.scala:52-61).  The reference keeps one
// leaf per distinct point and counts every copy on the way down, but when a
// leaf holding c copies of v splits (a different point arrived) it re-inserts
// v ONCE into the new child: cells created after the first copy of v was
// inserted count only 1 + the copies inserted after their creation.  A cell
// is created when its parent cell splits, i.e. at the row t2(parent) of the
// first point in the parent's cell whose value differs from the value of the
// parent cell's first point.  So for a duplicate group of m copies (rows
// r_1 < ... < r_m) and a cell X on its path with parent cell P:
// count_v(X) = m - max(0, #{r_i < t2(P)} - 1)  (the root: m), and the leaf
// of v (the quad child of the deepest cell R that also holds other points)
// has multiplicity m - max(0, #{r_i < t2(R)} - 1).  Only work when some
// point has a duplicate (dflag); no tile or moment ever covers such a group
// (the cells above it are traversed the reference's way).

// t2 per binary node from (first row, its value id, t2) of the two children:
// the union's first value is the earlier child's; its second distinct value
// arrives at the earlier of that child's t2 and the other child's first row
// (different value) or t2 (same value).
// (It also clears the correction arrays of dup_fixup, as dup_clear did.)
__global__ void dup_bottom_up(const int32_t *__restrict__ meta, const int32_t *__restrict__ dflag,
                              const int32_t *__restrict__ idx_sorted, const int32_t *__restrict__ rowmap,
                              const int32_t *__restrict__ vid, const BHNode *__restrict__ nodes,
                              const int32_t *__restrict__ parent_leaf, const int32_t *__restrict__ parent_node,
                              int32_t *arrive2, int32_t *rmin, int32_t *rvid, int32_t *rt2, int32_t *__restrict__ cntcorr,
                              double *__restrict__ sumcorr, int32_t *__restrict__ tiecnt, int32_t *__restrict__ notile,
                              int32_t *__restrict__ vflag, int32_t *__restrict__ vcnt, double *__restrict__ vsum) {
    const int m = meta[0];
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (!dflag[0] || s >= m) return;
    cntcorr[s] = 0;
    sumcorr[2 * s] = 0.0;
    sumcorr[2 * s + 1] = 0.0;
    tiecnt[s] = 0;
    notile[s] = 0;
    vflag[s] = 0;
    vcnt[s] = 0;
    vsum[2 * s] = 0.0;
    vsum[2 * s + 1] = 0.0;
    if (m < 2) return;
    auto leaf = [&](int q, int &r, int &v, int &t) {
        const int32_t l = idx_sorted[q];
        r = rowmap ? rowmap[l] : l;
        v = vid[q];
        t = INT32_MAX;
    };
    auto ld = [](const int32_t *p) { return __hip_atomic_load(const_cast<int32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
    auto st = [](int32_t *p, int32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
    int p = parent_leaf[s];
    while (p >= 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (__hip_atomic_fetch_add(&arrive2[p], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
        int r[2], v[2], t[2];
        const int32_t ch[2] = {nodes[p].left, nodes[p].right};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (ch[k] < 0) leaf(~ch[k], r[k], v[k], t[k]);
            else { r[k] = ld(rmin + ch[k]); v[k] = ld(rvid + ch[k]); t[k] = ld(rt2 + ch[k]); }
        }
        const int a = r[0] < r[1] ? 0 : 1, b = 1 - a;   // a: the child holding the earlier first row
        const int other = v[b] != v[a] ? r[b] : t[b];
        st(rmin + p, r[a]);
        st(rvid + p, v[a]);
        st(rt2 + p, min(t[a], other));
        p = parent_node[p];
    }
}

__device__ __forceinline__ bool real_cell(const BHNode &nd) { return nd.h >= 0.0; }

// One thread per pure duplicate group (the first of m >= 2 exact copies that
// form a whole equal-key run): leaf multiplicity of its tie node, count / sum
// corrections and no-tile marks of the real cells above it.
__global__ void dup_fixup(const int32_t *__restrict__ meta, const int32_t *__restrict__ dflag,
                          const double2 *__restrict__ pos, const uint64_t *__restrict__ keys,
                          const int32_t *__restrict__ dupc, const int32_t *__restrict__ idx_sorted,
                          const int32_t *__restrict__ rowmap, const BHNode *__restrict__ nodes,
                          const int32_t *__restrict__ parent_leaf, const int32_t *__restrict__ parent_node,
                          const int32_t *__restrict__ rt2, int32_t *__restrict__ cntcorr, double *__restrict__ sumcorr,
                          int32_t *__restrict__ tiecnt, int32_t *__restrict__ notile, int32_t *__restrict__ vflag,
                          int32_t *__restrict__ vcnt, double *__restrict__ vsum) {
    const int mroot = meta[0];
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (!dflag[0] || s >= mroot || dupc[s] < 2) return;
    const double2 q = pos[s];
    if (s > 0 && pos[s - 1].x == q.x && pos[s - 1].y == q.y) return;   // not the group's first
    const int m = dupc[s], kb = s + m - 1;
    if (kb >= mroot) return;
    for (int u = s; u <= kb; ++u)
        if (pos[u].x != q.x || pos[u].y != q.y) return;                 // copies not contiguous: impure run
    if ((s > 0 && keys[s - 1] == keys[s]) || (kb + 1 < mroot && keys[kb + 1] == keys[s])) return;
    // the group's node: climb from its first leaf until the node spans [s, kb]
    int g = parent_leaf[s];
    while (g >= 0 && !(nodes[g].first == s && nodes[g].last == kb)) g = parent_node[g];
    if (g < 0 || g == 0) return;                                         // every point identical: root tie
    auto copies_before = [&](int t2) {
        int c = 0;
        for (int u = s; u <= kb; ++u) {
            const int32_t l = idx_sorted[u];
            c += (rowmap ? rowmap[l] : l) < t2;
        }
        return c;
    };
    auto real_above = [&](int x) {   // the nearest real cell strictly above binary node x, -1 if none
        int y = parent_node[x];
        while (y >= 0 && !real_cell(nodes[y])) y = parent_node[y];
        return y;
    };
    int R = real_above(g);
    if (R < 0) return;
    tiecnt[g] = m - max(0, copies_before(rt2[R]) - 1);   // the leaf: R's quad child, created at t2(R)
    // Real node X = the DEEPEST cell C_k of a chain C_1 > ... > C_k of
    // reference cells holding the same points (our binary node exists only
    // where they split).  C_1 (a quad child of the real cell P above) was
    // created at t2(P); C_2..C_k at t2(C_1) = t2(X), in one cascade.
    for (int X = R; X >= 0;) {
        notile[X] = 1;
        const int P = real_above(X);
        const int lx = nodes[X].delta >> 1;
        const int deep = max(0, copies_before(rt2[X]) - 1);
        int top, node_corr;
        bool chain;
        if (P < 0) {   // the root: C_1 is the reference root cell, which holds every copy
            top = 0;
            chain = lx > 0;
        } else {
            top = max(0, copies_before(rt2[P]) - 1);
            chain = lx > (nodes[P].delta >> 1) + 1;
        }
        node_corr = chain ? deep : top;
        if (node_corr > 0) {
            atomicAdd(&cntcorr[X], node_corr);
            atomicAdd(&sumcorr[2 * X], node_corr * q.x);
            atomicAdd(&sumcorr[2 * X + 1], node_corr * q.y);
        }
        if (chain) {   // the chain top's own count: a virtual record when it differs
            if (top > 0) {
                atomicAdd(&vcnt[X], top);
                atomicAdd(&vsum[2 * X], top * q.x);
                atomicAdd(&vsum[2 * X + 1], top * q.y);
            }
            if (top != deep) vflag[X] = 1;
        }
        X = P;
    }
}

// corrected counts / centres of mass of the cells above duplicate groups
__global__ void dup_apply(int32_t *__restrict__ meta, const int32_t *__restrict__ dflag,
                          const int32_t *__restrict__ cntcorr, const double *__restrict__ sumcorr,
                          const int32_t *__restrict__ vflag, const int32_t *__restrict__ vcnt,
                          const double *__restrict__ vsum, int32_t *__restrict__ vcntf, double *__restrict__ vcom,
                          BHNode *__restrict__ nodes) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (!dflag[0] || i >= meta[0] - 1 || (cntcorr[i] == 0 && !vflag[i])) return;
    BHNode &nd = nodes[i];
    const double c0 = nd.cnt, x0 = nd.cx * c0, y0 = nd.cy * c0;   // all copies
    if (vflag[i]) {   // the chain top C_1
        if (i == meta[1]) meta[3] = 1;   // the root's chain: the reference root cell holds every copy
        const int32_t ct = nd.cnt - vcnt[i];
        vcntf[i] = ct;
        vcom[2 * i] = (x0 - vsum[2 * i]) / ct;
        vcom[2 * i + 1] = (y0 - vsum[2 * i + 1]) / ct;
    }
    if (cntcorr[i] != 0) {
        const double c1 = nd.cnt - cntcorr[i];
        nd.cx = (x0 - sumcorr[2 * i]) / c1;
        nd.cy = (y0 - sumcorr[2 * i + 1]) / c1;
        nd.cnt -= cntcorr[i];
    }
}


// ---- subtree moments: chunk counts, item map, per-item partial sums, reduce
__device__ __forceinline__ void box_centre(double bx0, double bx1, double by0, double by1, double &cx, double &cy,
                                           double &R) {
    cx = 0.5 * (bx0 + bx1);
    cy = 0.5 * (by0 + by1);
    const double ex = 0.5 * (bx1 - bx0), ey = 0.5 * (by1 - by0);
    R = sqrt(ex * ex + ey * ey) * (1.0 + 1e-12);
}
__device__ __forceinline__ void box_centre(const BHNode &nd, double &cx, double &cy, double &R) {
    box_centre(nd.bx0, nd.bx1, nd.by0, nd.by1, cx, cy, R);
}

// Per binary node with >= MOM_MIN_POINTS points (when the gate is on, see
// bbox_final): its chunk count, its place in the list of moment nodes of
// several chunks (one atomic per block; moment_reduce's work list) and its item range (one atomic per block on the item
// counter off[n]; the placement of the ranges varies from run to run, a
// node's chunks are summed in chunk order, so the moments do not), with the
// item -> node map filled in.
__global__ __launch_bounds__(1024) void moment_count(const BHNode *__restrict__ nodes, int64_t n, const int32_t *__restrict__ meta,
                             const int32_t *__restrict__ mom_flag, int32_t *__restrict__ cnt,
                             int32_t *__restrict__ list, int32_t *__restrict__ meta_w, int32_t *__restrict__ off,
                             int32_t *__restrict__ item) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int m = meta[0];
    int32_t c = 0;
    if (i < m - 1 && mom_flag[0]) {
        const BHNode &nd = nodes[i];
        if (nd.cnt >= MOM_MIN_POINTS && nd.delta < 62) c = (nd.cnt + MOM_CHUNK - 1) / MOM_CHUNK;
    }
    if (i < n) cnt[i] = c;
    __shared__ int wcnt[16], wbase[16], wsum[16], wibase[16];
    const int w = threadIdx.x >> 6, lane = lane_id();
    const uint64_t bal = __ballot(c > 1);   // the list: nodes of several chunks (moment_reduce)
    int inc = c;   // inclusive scan of the chunk counts over the wave (item offsets)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(inc, o, 64);
        if (lane >= o) inc += v;
    }
    if (lane == 63) wsum[w] = inc;
    if (lane == 0) wcnt[w] = (int)__popcll(bal);
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0, itot = 0;
        for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
            wbase[k] = tot; tot += wcnt[k];
            wibase[k] = itot; itot += wsum[k];
        }
        const int base = tot ? atomicAdd(&meta_w[2], tot) : 0;
        const int ibase = itot ? atomicAdd(&off[n], itot) : 0;
        for (int k = 0; k < (int)(blockDim.x >> 6); ++k) { wbase[k] += base; wibase[k] += ibase; }
    }
    __syncthreads();
    if (c > 1) list[wbase[w] + __popcll(bal & lanemask_lt())] = (int32_t)i;
    if (c > 0) {
        const int o = wibase[w] + inc - c;
        off[i] = o;
        for (int k = 0; k < c; ++k) item[o + k] = (int32_t)i;
    }
}

// Fixed-order wave reduction of MOM_K per-lane partial sums to dst[0..MOM_K)
// (LDSRED: 8 moments at a time transposed through a per-wave LDS tile -- 8
// row sums per column + 3 shuffle stages, ~20 instructions per 8 moments --
// instead of a 6-stage shuffle tree per moment).
template <bool LDSRED>
__device__ __forceinline__ void moments_wave_store(const double (&acc)[MOM_K], double *rw, int lane,
                                                   double *__restrict__ dst) {
    if (LDSRED) {
        const int col = lane & 7, r0 = (lane >> 3) * 8;
#pragma unroll
        for (int k0 = 0; k0 < MOM_K; k0 += 8) {
#pragma unroll
            for (int j = 0; j < 8; ++j) rw[lane * 9 + j] = (k0 + j < MOM_K) ? acc[k0 + j] : 0.0;
            // the other lanes' stores must have landed before the cross-lane
            // loads (and those loads before the next round overwrites rw)
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
            __builtin_amdgcn_wave_barrier();
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < 8; ++r) v += rw[(r0 + r) * 9 + col];
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            v += __shfl_xor(v, 8, 64);
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            if (lane < 8 && k0 + lane < MOM_K) dst[k0 + lane] = v;
        }
    } else {
#pragma unroll
        for (int k = 0; k < MOM_K; ++k) {
            const double v = wave_sum(acc[k]);
            if (lane == 0) dst[k] = v;
        }
    }
}

// One wave per item (<= MOM_CHUNK points of one node): lanes accumulate the
// scaled moments u_x^a u_y^b / (a! b!) in registers, then the fixed-order
// wave reduction.  A node of one chunk (chunk counts cnt, when given) gets its
// moments written directly to mom; moment_reduce sums the others' chunks.
template <bool LDSRED>
__global__ __launch_bounds__(256) void moment_items(const double2 *__restrict__ pos,
                                                    const BHNode *__restrict__ nodes,
                                                    const int32_t *__restrict__ off, int64_t n,
                                                    const int32_t *__restrict__ item,
                                                    double *__restrict__ part, const int32_t *__restrict__ cnt,
                                                    double *__restrict__ mom) {
    __shared__ double red[4][64 * 9];
    double *rw = red[threadIdx.x >> 6];
    const int total = off[n];
    const int lane = lane_id();
    const int nw = gridDim.x * (blockDim.x >> 6);
    for (int it = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); it < total; it += nw) {
        const int node = __builtin_amdgcn_readfirstlane(item[it]);
        const int c = it - off[node];
        const BHNode &nd = nodes[node];
        double cx, cy, R;
        box_centre(nd, cx, cy, R);
        const int p0 = nd.first + c * MOM_CHUNK;
        const int p1 = min(nd.last + 1, p0 + MOM_CHUNK);
        double acc[MOM_K];
#pragma unroll
        for (int k = 0; k < MOM_K; ++k) acc[k] = 0.0;
        for (int p = p0 + lane; p < p1; p += 64) {
            const double2 q = pos[p];
            const double ux = q.x - cx, uy = q.y - cy;
            double X[MOM_DEG + 1], Yv[MOM_DEG + 1];
            X[0] = 1.0; Yv[0] = 1.0;
#pragma unroll
            for (int e = 1; e <= MOM_DEG; ++e) {
                X[e] = X[e - 1] * ux * (1.0 / e);
                Yv[e] = Yv[e - 1] * uy * (1.0 / e);
            }
#pragma unroll
            for (int a = 0; a <= MOM_DEG; ++a)
#pragma unroll
                for (int b = 0; b <= MOM_DEG; ++b)
                    if (a + b <= MOM_DEG) acc[midx(a, b)] = __fma_rn(X[a], Yv[b], acc[midx(a, b)]);
        }
        const bool single = cnt && __builtin_amdgcn_readfirstlane(cnt[node]) == 1;
        moments_wave_store<LDSRED>(acc, rw, lane, single ? mom + (int64_t)node * MOM_K : part + (int64_t)it * MOM_K);
    }
}

// One wave per moment node of several chunks (the list; single-chunk nodes
// were written by moment_items): each lane sums its chunks' partials (chunk j
// to lane j mod 64, in order), then the fixed-order wave reduction -- the
// root's ~500 chunks are no longer one lane's serial chain.
__global__ __launch_bounds__(256) void moment_reduce(const int32_t *__restrict__ meta, const int32_t *__restrict__ list,
                                                     const int32_t *__restrict__ cnt, const int32_t *__restrict__ off,
                                                     const double *__restrict__ part, double *__restrict__ mom) {
    __shared__ double red[4][64 * 9];
    double *rw = red[threadIdx.x >> 6];
    const int nl = meta[2];
    const int lane = lane_id();
    const int nw = gridDim.x * (blockDim.x >> 6);
    for (int e = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); e < nl; e += nw) {
        const int node = __builtin_amdgcn_readfirstlane(list[e]);
        const int c = __builtin_amdgcn_readfirstlane(cnt[node]);
        const int o = __builtin_amdgcn_readfirstlane(off[node]);
        double acc[MOM_K];
#pragma unroll
        for (int k = 0; k < MOM_K; ++k) acc[k] = 0.0;
        for (int j = lane; j < c; j += 64) {
            const double *pp = part + (int64_t)(o + j) * MOM_K;
#pragma unroll
            for (int k = 0; k < MOM_K; ++k) acc[k] += pp[k];
        }
        moments_wave_store<true>(acc, rw, lane, mom + (int64_t)node * MOM_K);
    }
}

// omega_i (z) and phi_i (F) weights of S_i = sum D^i, Sx_i = sum D^i w, for
// A = |v|^2.
__device__ __forceinline__ void moment_weights(double A, double *om, double *ph) {
    const double B = 1.0 / (1.0 + A);
    {
        double Ap[MOM_ORDER + 1], Bp[MOM_ORDER + 3];
        Ap[0] = 1.0; Bp[0] = 1.0;
#pragma unroll
        for (int k = 1; k <= MOM_ORDER; ++k) Ap[k] = Ap[k - 1] * A;
#pragma unroll
        for (int k = 1; k <= MOM_ORDER + 2; ++k) Bp[k] = Bp[k - 1] * B;
#pragma unroll
        for (int i = 0; i <= MOM_ORDER; ++i) {
            double so = 0.0, sp = 0.0;
#pragma unroll
            for (int k = 0; k <= MOM_ORDER; ++k) {
                if (k < i) continue;
                so += binom(k, i) * Ap[k - i] * Bp[k + 1];
                sp += (k + 1) * binom(k, i) * Ap[k - i] * Bp[k + 2];
            }
            om[i] = (i & 1) ? -so : so;
            ph[i] = (i & 1) ? sp : -sp;
        }
    }
}

// Subtree sums for one lane's query from the node's moments (see the header).
// Returns z += sum 1/(1+D), (fx, fy) += sum (q - y)/(1+D)^2 over the subtree's
// points, the query itself and its exact duplicates included (D = 0: they add
// 1 to z and 0 to F; the traversal subtracts them).
__device__ __forceinline__ void moment_eval(const double *mu, double vx, double vy, double &fx, double &fy,
                                            double &zs) {
    double om[MOM_ORDER + 1], ph[MOM_ORDER + 1];
    moment_weights(vx * vx + vy * vy, om, ph);
    // shift to the query: w = u - v; X[e] = (-v_x)^e / e!
    double X[MOM_DEG + 1], Yv[MOM_DEG + 1];
    X[0] = 1.0; Yv[0] = 1.0;
#pragma unroll
    for (int e = 1; e <= MOM_DEG; ++e) {
        X[e] = X[e - 1] * (-vx) * (1.0 / e);
        Yv[e] = Yv[e - 1] * (-vy) * (1.0 / e);
    }
    double z = 0.0, gx = 0.0, gy = 0.0;
#pragma unroll
    for (int a = 0; a <= MOM_DEG; ++a) {
        double lam[MOM_DEG + 1];         // lam[b'] = sum_a' mu(a', b') X[a - a']
#pragma unroll
        for (int b1 = 0; b1 <= MOM_DEG; ++b1) {
            if (a + b1 > MOM_DEG) continue;
            double t = 0.0;
#pragma unroll
            for (int a1 = 0; a1 <= MOM_DEG; ++a1)
                if (a1 <= a) t = __fma_rn(mu[midx(a1, b1)], X[a - a1], t);
            lam[b1] = t;
        }
#pragma unroll
        for (int b = 0; b <= MOM_DEG; ++b) {
            if (a + b > MOM_DEG) continue;
            if ((a & 1) && (b & 1)) continue;
            if (!(a & 1) && !(b & 1) && a + b > 2 * MOM_ORDER) continue;
            double nu = 0.0;   // nu(a, b) / (a! b!) = sum_j w_x^a w_y^b / (a! b!)
#pragma unroll
            for (int b1 = 0; b1 <= MOM_DEG; ++b1)
                if (b1 <= b) nu = __fma_rn(lam[b1], Yv[b - b1], nu);
            if (!(a & 1) && !(b & 1)) {
                const int i = (a + b) / 2;
                z = __fma_rn(om[i] * (binom(i, a / 2) * fact(a) * fact(b)), nu, z);
            } else if (a & 1) {
                const int i = (a + b - 1) / 2;
                gx = __fma_rn(ph[i] * (binom(i, (a - 1) / 2) * fact(a) * fact(b)), nu, gx);
            } else {
                const int i = (a + b - 1) / 2;
                gy = __fma_rn(ph[i] * (binom(i, a / 2) * fact(a) * fact(b)), nu, gy);
            }
        }
    }
    zs += z;
    fx += gx;
    fy += gy;
}

// ---- The same sums as polynomials in v (root-tile mode: ONE subtree for
// every query).  moment_eval computes z = sum_i om_i(A) Qz_i(v) with
//   Qz_i(v) = sum_{a+b=2i, a,b even} C(i, a/2) a! b! nu(a, b),
//   nu(a, b) = sum_{p<=a, q<=b} mu(a-p, b-q) (-v_x)^p (-v_y)^q / (p! q!),
// a polynomial of degree 2i in (v_x, v_y); gx / gy likewise with ph_i and
// Qx_i (a odd) / Qy_i (b odd) of degree 2i+1.  Their POLY_K coefficients
// depend on the subtree's moments only: poly_coef computes them once, and a
// query evaluates 3 (MOM_ORDER+1) small polynomials by Horner with uniform
// (scalar-loaded) coefficients instead of shifting the moments itself --
// ~40 VGPRs instead of 256 + spills.
__host__ __device__ constexpr int poly_len(int d) { return (d + 1) * (d + 2) / 2; }
__host__ __device__ constexpr int poly_off_z(int i) { return i == 0 ? 0 : poly_off_z(i - 1) + poly_len(2 * i - 2); }
constexpr int POLY_X = poly_off_z(MOM_ORDER + 1);
__host__ __device__ constexpr int poly_off_x(int i) { return i == 0 ? POLY_X : poly_off_x(i - 1) + poly_len(2 * i - 1); }
constexpr int POLY_Y = poly_off_x(MOM_ORDER + 1);
__host__ __device__ constexpr int poly_off_y(int i) { return POLY_Y + poly_off_x(i) - POLY_X; }
constexpr int POLY_K = POLY_Y + (POLY_Y - POLY_X);
static_assert(POLY_K == 345, "MOM_ORDER 4: 95 + 125 + 125 coefficients");

__device__ __forceinline__ double factd(int k) {
    double f = 1.0;
    for (int j = 2; j <= k; ++j) f *= j;
    return f;
}

// Coefficient c of the root polynomials from the node's moments mu (one
// thread per coefficient; (p, q) ordered like midx within each polynomial).
__global__ void poly_coef(const double *__restrict__ mu, double *__restrict__ coef) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= POLY_K) return;
    int kind = 0, i = 0, r = c;   // kind 0 z, 1 x, 2 y
    if (c >= POLY_Y) { kind = 2; r = c - POLY_Y; }
    else if (c >= POLY_X) { kind = 1; r = c - POLY_X; }
    for (;;) {
        const int len = poly_len(kind == 0 ? 2 * i : 2 * i + 1);
        if (r < len) break;
        r -= len;
        ++i;
    }
    const int d = kind == 0 ? 2 * i : 2 * i + 1;
    int p = 0;
    while (r >= d + 1 - p) { r -= d + 1 - p; ++p; }
    const int q = r;
    double s = 0.0;
    for (int a = p; a <= d; ++a) {
        const int b = d - a;
        const bool ok = kind == 0 ? !(a & 1) : kind == 1 ? (a & 1) : !(a & 1);
        if (!ok || b < q) continue;
        const int j = kind == 1 ? (a - 1) / 2 : a / 2;
        s += factd(i) / (factd(j) * factd(i - j)) * factd(a) * factd(b) * mu[midx(a - p, b - q)];
    }
    coef[c] = (((p + q) & 1) ? -s : s) / (factd(p) * factd(q));
}

template <int D>
__device__ __forceinline__ double poly_eval(const double *__restrict__ c, double vx, double vy) {
    double acc = 0.0;
#pragma unroll
    for (int p = D; p >= 0; --p) {
        const int o = p * (D + 1) - p * (p - 1) / 2;
        double r = c[o + D - p];
#pragma unroll
        for (int q = D - p - 1; q >= 0; --q) r = __fma_rn(r, vy, c[o + q]);
        acc = p == D ? r : __fma_rn(acc, vx, r);
    }
    return acc;
}

template <int I>
__device__ __forceinline__ void poly_terms(const double *__restrict__ c, double vx, double vy, const double *om,
                                           const double *ph, double &z, double &gx, double &gy) {
    if constexpr (I <= MOM_ORDER) {
        z = __fma_rn(om[I], poly_eval<2 * I>(c + poly_off_z(I), vx, vy), z);
        gx = __fma_rn(ph[I], poly_eval<2 * I + 1>(c + poly_off_x(I), vx, vy), gx);
        gy = __fma_rn(ph[I], poly_eval<2 * I + 1>(c + poly_off_y(I), vx, vy), gy);
        poly_terms<I + 1>(c, vx, vy, om, ph, z, gx, gy);
    }
}

// moment_eval from the subtree's polynomial coefficients (poly_coef).
__device__ __forceinline__ void poly_moment_eval(const double *__restrict__ coef, double vx, double vy, double &fx,
                                                 double &fy, double &zs) {
    double om[MOM_ORDER + 1], ph[MOM_ORDER + 1];
    moment_weights(vx * vx + vy * vy, om, ph);
    double z = 0.0, gx = 0.0, gy = 0.0;
    poly_terms<0>(coef, vx, vy, om, ph, z, gx, gy);
    zs += z;
    fx += gx;
    fy += gy;
}

// Truncation test of the moment path for query q and a subtree's bounding box.
__device__ __forceinline__ bool moment_ok(double bx0, double bx1, double by0, double by1, double qx, double qy,
                                          double tol) {
    double cx, cy, R;
    box_centre(bx0, bx1, by0, by1, cx, cy, R);
    const double vx = qx - cx, vy = qy - cy;
    const double A = vx * vx + vy * vy;
    const double rho = (R * R + 2.0 * sqrt(A) * R) / (1.0 + A) * (1.0 + 1e-12);
    if (!(rho < 0.25)) return false;
    double rp = rho;
#pragma unroll
    for (int k = 0; k < MOM_ORDER; ++k) rp *= rho;
    return (MOM_ORDER + 2) * rp <= tol * (1.0 - rho) * (1.0 - rho);
}

// Moment tasks of each query (query slots [g0, g1): sorted positions, or
// qlist[slot] when a rank computes a list of them), in traversal order, added
// to the traversal's F and z.
// Tile chunks (TSNE_TILE_CHUNK=0: off): a traversal wave whose tile cost
// (points + 16 per task) exceeds 2x the mean (and 4096) has its tile list cut
// into C contiguous index ranges, each a tile_apply wave of its own.  Chunk
// slots write partial sums (Fp, Zp) and moment lists per slot lane;
// chunk_combine adds them to F, Z in chunk order: deterministic.
struct ChunkView {
    const int32_t *slot_w = nullptr, *slot_c = nullptr, *nslots = nullptr;
    double2 *Fp = nullptr;
    double *Zp = nullptr;
};
constexpr int CHUNK_MAX = 32;
constexpr int CHUNK_MIN = 4096;
__global__ void chunk_total(const int32_t *__restrict__ tcost, int64_t waves, unsigned long long *__restrict__ total) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long c = w < waves ? (unsigned long long)max(tcost[w], 0) : 0ull;
    const unsigned long long ws = wave_sum(c);
    if (lane_id() == 0 && ws) atomicAdd(total, ws);
}
__global__ void chunk_parts(const int32_t *__restrict__ tcost, const unsigned long long *__restrict__ total,
                            int64_t waves, int32_t *__restrict__ Cw, const int32_t *__restrict__ claims, int32_t gen,
                            int32_t *__restrict__ wout, double frac) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w > waves) return;
    if (w == waves) { Cw[w] = 0; return; }
    // ceil(2 total / waves): the extra chunks sum to <= total / target <= waves / 2,
    // inside the slot capacity (waves + waves / 2 + 64, bh_alloc)
    const unsigned long long W = (unsigned long long)max<int64_t>(waves, 1);
    const long long target = max((long long)CHUNK_MIN, (long long)((2 * (*total) + W - 1) / W));
    if (wout && w == 0) *wout = (int32_t)min(2.0e9, frac * (double)target);
    // (tile streaming: a handed-over list is one chunk, whichever path sums it)
    Cw[w] = claims && (claims[w] >> 2) == gen ? 1
                                              : 1 + (int32_t)min((long long)(CHUNK_MAX - 1),
                                                                 (long long)max(tcost[w], 0) / target);
}
__global__ void chunk_fill(int32_t *__restrict__ Cw, int32_t *__restrict__ slot0,
                           const int32_t *__restrict__ tcost, int64_t waves, int32_t *__restrict__ slot_w,
                           int32_t *__restrict__ slot_c, int32_t *__restrict__ scost, int64_t slots_max,
                           int32_t *__restrict__ nslots) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // the plan fits by construction (chunk_parts); should it not, every wave
    // falls back to one slot (C = 1) rather than a chunk being dropped
    const bool fits = slot0[waves] <= slots_max;
    if (w == waves) *nslots = fits ? slot0[waves] : (int32_t)waves;
    if (w < waves && !fits) {
        Cw[w] = 1;
        slot0[w] = (int32_t)w;
        slot_w[w] = (int32_t)w;
        slot_c[w] = 1 << 16;
        scost[w] = tcost[w];
    } else if (w < waves) {
        const int C = Cw[w];
        for (int j = 0; j < C; ++j) {
            slot_w[slot0[w] + j] = (int32_t)w;
            slot_c[slot0[w] + j] = j | (C << 16);
            scost[slot0[w] + j] = tcost[w] / C;
        }
    }
    // slots past the plan: no work, lowest cost
    for (int64_t k = (fits ? slot0[waves] : waves) + w; w <= waves && k < slots_max; k += waves + 1) scost[k] = 0;
}
// The whole chunk plan and the longest-first tile_apply block order in ONE
// workgroup (replacing chunk_total / chunk_parts / a scan / chunk_fill and
// the block sort: ~13 launches of a few us each at 1M).  Same chunk counts,
// slots and fallback as those kernels; the block order is by cost bucket
// (4 per doubling, descending; the order within a bucket is unspecified --
// tile_apply's sums do not depend on the order its blocks run in).
constexpr int PLAN_WAVES_MAX = 16384;    // traversal waves whose costs the plan stages in LDS
constexpr int PLAN_BLOCKS_MAX = (PLAN_WAVES_MAX + PLAN_WAVES_MAX / 2 + 64 + 3) / 4;   // tile_apply blocks (4 slots each)
constexpr int PLAN_BUCKETS = 128;
__device__ __forceinline__ int plan_bucket(int32_t c) {
    return c <= 0 ? 0 : min(PLAN_BUCKETS - 1, 1 + (int)(4.0f * __log2f((float)c)));
}
// hist[key] += 1 for every active lane of the wave, one LDS atomic per
// distinct key (per-lane atomics serialise on the few cost buckets most
// entries share -- late in the schedule nearly all in bucket 0); returns the
// lane's slot (old value + its rank among the wave's lanes of that key).
__device__ __forceinline__ int32_t wave_bucket_add(int32_t *hist, int key, bool act) {
    const int lane = lane_id();
    int32_t res = 0;
    uint64_t rem = __ballot(act);
    while (rem) {
        const int leader = __builtin_ctzll(rem);
        const int kb = __shfl(key, leader, 64);
        const bool mine = act && key == kb;
        const uint64_t m = __ballot(mine);
        int32_t b0 = 0;
        if (lane == leader) b0 = atomicAdd(&hist[kb], (int32_t)__popcll(m));
        b0 = __shfl(b0, leader, 64);
        if (mine) res = b0 + (int32_t)__popcll(m & lanemask_lt());
        rem &= ~m;
    }
    return res;
}
__global__ __launch_bounds__(1024) void tile_plan(const int32_t *__restrict__ tcost, int64_t waves, int64_t slots_max,
                                                  int32_t *__restrict__ Cw, int32_t *__restrict__ slot0,
                                                  int32_t *__restrict__ slot_w, int32_t *__restrict__ slot_c,
                                                  int32_t *__restrict__ nslots, int32_t *__restrict__ torder,
                                                  const int32_t *__restrict__ claims, int32_t gen,
                                                  int32_t *__restrict__ wout, double frac) {
    __shared__ int32_t bc[PLAN_BLOCKS_MAX];
    __shared__ int32_t tc[PLAN_WAVES_MAX];
    __shared__ unsigned long long red[16];
    __shared__ int32_t wtot[16];
    __shared__ int32_t hist[PLAN_BUCKETS];
    __shared__ int32_t sfits;
    const int t = threadIdx.x, lane = lane_id(), w = t >> 6;
    const int64_t tblocks = (slots_max + 3) / 4;
    // total tile cost
    unsigned long long acc = 0;
    for (int64_t v = t; v < waves; v += 1024) {
        const int32_t c = max(tcost[v], 0);
        tc[v] = c;
        acc += (unsigned long long)c;
    }
    acc = wave_sum(acc);
    if (lane == 0) red[w] = acc;
    for (int64_t b = t; b < tblocks; b += 1024) bc[b] = 0;
    if (t < PLAN_BUCKETS) hist[t] = 0;
    __syncthreads();
    unsigned long long total = 0;
    for (int k = 0; k < 16; ++k) total += red[k];
    // ceil(2 total / waves): the extra chunks sum to <= waves / 2 (bh_alloc's slot capacity)
    const unsigned long long Wd = (unsigned long long)max<int64_t>(waves, 1);
    const long long target = max((long long)CHUNK_MIN, (long long)((2 * total + Wd - 1) / Wd));
    // (tile streaming: a handed-over list is one chunk, whichever path sums it)
    auto chunks = [&](int64_t v) {
        if (claims && (claims[v] >> 2) == gen) return 1;
        return 1 + (int32_t)min((long long)(CHUNK_MAX - 1), (long long)tc[v] / target);
    };
    if (wout && t == 0) *wout = (int32_t)min(2.0e9, frac * (double)target);
    // this thread's contiguous run of waves and its slot count
    const int64_t per = (waves + 1023) / 1024, v0 = min(waves, t * per), v1 = min(waves, v0 + per);
    int32_t loc = 0;
    for (int64_t v = v0; v < v1; ++v) loc += chunks(v);
    int32_t inc = loc;   // exclusive scan over the 1024 threads: waves, then wave totals
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t x = __shfl_up(inc, o, 64);
        if (lane >= o) inc += x;
    }
    if (lane == 63) wtot[w] = inc;
    __syncthreads();
    int32_t base = inc - loc, S = 0;
    for (int k = 0; k < 16; ++k) {
        if (k < w) base += wtot[k];
        S += wtot[k];
    }
    if (t == 0) sfits = S <= slots_max;
    __syncthreads();
    const bool fits = sfits != 0;   // else every wave one slot, rather than a chunk dropped
    int32_t run = base;
    for (int64_t v = v0; v < v1; ++v) {
        const int32_t c = fits ? chunks(v) : 1;
        const int32_t s0 = fits ? run : (int32_t)v;
        Cw[v] = c;
        slot0[v] = s0;
        const int32_t sc = tc[v] / c;
        for (int j = 0; j < c; ++j) {
            slot_w[s0 + j] = (int32_t)v;
            slot_c[s0 + j] = j | (c << 16);
            if (torder) atomicMax(&bc[(s0 + j) >> 2], sc);
        }
        run += c;
    }
    if (t == 0) {
        Cw[waves] = 0;
        slot0[waves] = fits ? S : (int32_t)waves;
        *nslots = fits ? S : (int32_t)waves;
    }
    if (!torder) return;
    __syncthreads();
    // the blocks' cost buckets (wave_bucket_add); the order within a bucket is free
    for (int64_t b0 = (int64_t)w * 64; b0 < tblocks; b0 += 1024) {
        const int64_t b = b0 + lane;
        (void)wave_bucket_add(hist, b < tblocks ? plan_bucket(bc[b]) : 0, b < tblocks);
    }
    __syncthreads();
    if (t == 0) {   // descending bucket starts
        int32_t r = 0;
        for (int k = PLAN_BUCKETS - 1; k >= 0; --k) { const int32_t c = hist[k]; hist[k] = r; r += c; }
    }
    __syncthreads();
    for (int64_t b0 = (int64_t)w * 64; b0 < tblocks; b0 += 1024) {
        const int64_t b = b0 + lane;
        const int32_t pos = wave_bucket_add(hist, b < tblocks ? plan_bucket(bc[b]) : 0, b < tblocks);
        if (b < tblocks) torder[pos] = (int32_t)b;
    }
}

// F, Z of each query += its chunks' partial sums, in chunk order
__global__ void chunk_combine(const double2 *__restrict__ Fp, const double *__restrict__ Zp,
                              const int32_t *__restrict__ Cw, const int32_t *__restrict__ slot0, int64_t g0, int64_t g1,
                              const int32_t *__restrict__ qlist, double2 *__restrict__ F, double *__restrict__ Z,
                              int32_t *__restrict__ pcost, const int32_t *__restrict__ idx_sorted,
                              const int32_t *__restrict__ wcost, const int32_t *__restrict__ nflag) {
    const int64_t k = g0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= g1) return;
    if (pcost) {   // option trav_front_cur: the point's wave cost (a narrow group's: heavy)
        const int64_t wq = (k - g0) >> 6;
        pcost[idx_sorted[k]] = nflag && nflag[wq] ? (1 << 29) : wcost[wq];
    }
    const int64_t w = (k - g0) >> 6, lane = (k - g0) & 63;
    const int64_t s = qlist ? (int64_t)qlist[k] : k;
    const int64_t b = (int64_t)slot0[w] * 64 + lane;
    double fx = 0.0, fy = 0.0, z = 0.0;
    for (int j = 0; j < Cw[w]; ++j) {
        const double2 g = Fp[b + 64 * j];
        fx += g.x; fy += g.y;
        z += Zp[b + 64 * j];
    }
    if (fx != 0.0 || fy != 0.0 || z != 0.0) {
        const double2 f = F[s];
        F[s] = make_double2(f.x + fx, f.y + fy);
        Z[s] = Z[s] + z;
    }
}

__global__ __launch_bounds__(256) void moment_apply(const double2 *__restrict__ pos,
                                                    const BHNode *__restrict__ nodes,
                                                    const double *__restrict__ mom,
                                                    const int32_t *__restrict__ mtask,
                                                    const int32_t *__restrict__ mtask_n, int64_t g0,
                                                    int64_t g1, const int32_t *__restrict__ qlist,
                                                    double2 *__restrict__ F, double *__restrict__ Z,
                                                    ChunkView cv) {
    // entry = query slot, or (tile chunks) chunk slot lane with partial sums Fp / Zp
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t k = g0 + i;
    if (cv.slot_w) {
        if ((i >> 6) >= *cv.nslots) return;
        k = g0 + (int64_t)cv.slot_w[i >> 6] * 64 + (i & 63);
    }
    if (k >= g1) return;
    const int64_t s = qlist ? (int64_t)qlist[k] : k;
    const int64_t e = cv.slot_w ? i : s;
    const int nt = mtask_n[e];
    if (nt == 0) return;
    const double2 q = pos[s];
    double fx = 0.0, fy = 0.0, zs = 0.0;
    for (int t = 0; t < nt; ++t) {
        const int node = mtask[e * MOM_TASKS + t];
        double cx, cy, R;
        box_centre(nodes[node], cx, cy, R);
        moment_eval(mom + (int64_t)node * MOM_K, q.x - cx, q.y - cy, fx, fy, zs);
    }
    double2 *Fo = cv.slot_w ? cv.Fp : F;
    double *Zo = cv.slot_w ? cv.Zp : Z;
    const double2 f = Fo[e];
    Fo[e] = make_double2(f.x + fx, f.y + fy);
    Zo[e] = Zo[e] + zs;
}

// Moment tasks of the narrow groups' queries (their own lists, entry = heavy
// slot x 64 + query), added to F, Z after the narrow traversal's sums.
__global__ __launch_bounds__(256) void narrow_moment_apply(const double2 *__restrict__ pos,
                                                           const BHNode *__restrict__ nodes,
                                                           const double *__restrict__ mom,
                                                           const int32_t *__restrict__ hlist,
                                                           const int32_t *__restrict__ hcount,
                                                           const int32_t *__restrict__ mtask,
                                                           const int32_t *__restrict__ mtask_n, int64_t g0, int64_t g1,
                                                           const int32_t *__restrict__ qlist, double2 *__restrict__ F,
                                                           double *__restrict__ Z) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((e >> 6) >= (int64_t)*hcount) return;
    const int64_t k = g0 + (int64_t)hlist[e >> 6] * 64 + (e & 63);
    if (k >= g1) return;
    const int nt = mtask_n[e];
    if (nt == 0) return;
    const int64_t s = qlist ? (int64_t)qlist[k] : k;
    const double2 q = pos[s];
    double fx = 0.0, fy = 0.0, zs = 0.0;
    for (int t = 0; t < nt; ++t) {
        const int node = mtask[e * MOM_TASKS + t];
        double cx, cy, R;
        box_centre(nodes[node], cx, cy, R);
        moment_eval(mom + (int64_t)node * MOM_K, q.x - cx, q.y - cy, fx, fy, zs);
    }
    const double2 f = F[s];
    F[s] = make_double2(f.x + fx, f.y + fy);
    Z[s] = Z[s] + zs;
}

// fl(h / D) < theta -- the reference's max(hHeigth, hWidth) / D < theta with
// an IEEE division -- decided by comparing h with theta * D outside a 1e-14
// relative band (where the rounded quotient cannot cross theta), and by the
// exact division inside it.  Df may be the FMA-evaluated D (within 1 ulp of
// the reference's dx*dx + dy*dy); the exact path recomputes the latter.
// D = 0 or denormal gives h > theta D: opened, as h / 0 = inf is not < theta.
__device__ __forceinline__ bool summarise(double h, double Df, double dx, double dy, double th_lo, double th_hi,
                                          double theta) {
    if (h < th_lo * Df) return true;
    if (h > th_hi * Df) return false;
    const double D = __dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy));
    return h / D < theta;
}

// One summarised cell (QuadTree.scala:134-142): Q = 1/(1+D), m = n Q.
__device__ __forceinline__ void cell_force(double dx, double dy, double D, int32_t n, double &fx, double &fy,
                                           double &zs) {
    const double Q = recip_bh(1.0 + D);
    const double mult = (double)n * Q;
    const double sc = mult * Q;
    fx = __fma_rn(sc, dx, fx);
    fy = __fma_rn(sc, dy, fy);
    zs += mult;
}

// Quad records: one per real node, children found through transparent nodes
// (build_qrec below).  Slots of transparent nodes are never written: only
// real cells are ever pushed (and their records read) by the traversal.
struct DupView {   // duplicate-multiplicity data for build_qrec (nullptr members when there is none)
    const int32_t *tiecnt, *notile, *vflag, *vcntf;
    const double *vcom;
    int32_t virt;   // record index offset of the virtual chain tops (= n)
};
__device__ __forceinline__ void build_qrec_reg(const BHNode *__restrict__ nodes, const double2 *__restrict__ pos, int i,
                                               double inv_theta, double near_dmax, const DupView &dv, QRec &r);
// One thread per binary node: it builds its record in registers
// (build_qrec_reg) and writes it as 16 contiguous 16-byte stores (the partial
// lines of a wave's stores merge in the L2), so the occupancy is set by
// registers -- an LDS-staged version (coalesced copies of 64 records per
// workgroup, 16 KB of LDS each) took 103 us at C3, this one 87 us (round 5).
__global__ __launch_bounds__(256) void build_qrec(const BHNode *__restrict__ nodes,
                                                         const double2 *__restrict__ pos,
                                                         const int32_t *__restrict__ meta, double inv_theta,
                                                         double near_dmax, const int32_t *__restrict__ dflag,
                                                         DupView dv, QRec *__restrict__ qrec) {
    const int m = meta[0];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m - 1) return;
    const bool dups = dflag[0] != 0;
    if (!dups) dv = DupView{nullptr, nullptr, nullptr, nullptr, nullptr, 0};
    if (nodes[i].h >= 0.0) {   // transparent / key-tie nodes get no record
        QRec r;
        build_qrec_reg(nodes, pos, i, inv_theta, near_dmax, dv, r);
        const uint4 *src = reinterpret_cast<const uint4 *>(&r);
        uint4 *dst = reinterpret_cast<uint4 *>(qrec + i);
#pragma unroll
        for (int k = 0; k < (int)(sizeof(QRec) / 16); ++k) dst[k] = src[k];
    }
    if (dups && dv.vflag[i]) {   // node i's chain top C_1 (as build_qrec)
        const BHNode &nd = nodes[i];
        QRec v;
        v.cx = dv.vcom[2 * i]; v.cy = dv.vcom[2 * i + 1]; v.rball = 0.0;
        v.hmin = fmax(nd.hmin * inv_theta * (1.0 - 1e-12), near_dmax) * (1.0 - 1.1e-12);
        v.bx0 = nd.bx0; v.bx1 = nd.bx1; v.by0 = nd.by0; v.by1 = nd.by1;
        v.ex = 1e-15 * (fabs(nd.bx0) + fabs(nd.bx1) + fabs(nd.by0) + fabs(nd.by1));
        v.lmask = 0;
        v.first = nd.first; v.last = nd.last; v.cnt = dv.vcntf[i]; v.nch = 1;
        v.ccx[0] = nd.cx; v.ccy[0] = nd.cy; v.cref[0] = i; v.ccnt[0] = nd.cnt;
        v.ca[0] = qacc_accept(nd.h, inv_theta);
        v.cb[0] = qacc_open(nd.h, inv_theta);
        for (int k = 1; k < 4; ++k) {
            v.ccx[k] = 0.0; v.ccy[k] = 0.0; v.cb[k] = 0.0; v.ca[k] = 0.0; v.cref[k] = 0; v.ccnt[k] = 0;
        }
        qrec[dv.virt + i] = v;
    }
}

// One quad record, every array of it indexed by compile-time constants (the
// children's refs collected first, then one unrolled slot per child), so that
// the record stays in registers (build_qrec).
__device__ __forceinline__ void build_qrec_reg(const BHNode *__restrict__ nodes, const double2 *__restrict__ pos, int i,
                                               double inv_theta, double near_dmax, const DupView &dv, QRec &r) {
    const int32_t *tiecnt = dv.tiecnt, *notile = dv.notile;
    const BHNode &nd = nodes[i];
    r.cx = nd.cx; r.cy = nd.cy; r.rball = nd.rball * nd.rball * (1.0 - 1e-9);
    r.hmin = fmax(nd.hmin * inv_theta * (1.0 - 1e-12), near_dmax) * (1.0 - 1.1e-12);
    r.bx0 = nd.bx0; r.bx1 = nd.bx1; r.by0 = nd.by0; r.by1 = nd.by1;
    r.ex = 1e-15 * (fabs(nd.bx0) + fabs(nd.bx1) + fabs(nd.by0) + fabs(nd.by1));
    r.lmask = 0;
    r.first = nd.first; r.last = nd.last; r.cnt = nd.cnt;
    auto transparent = [&](int32_t c) { return c >= 0 && nodes[c].delta < 62 && nodes[c].h < 0.0; };
    // the quad children in key order (<= 4: a 2-deep descent through transparent nodes)
    int32_t l0 = 0, l1 = 0, l2 = 0, l3 = 0;
    int nc = 0;
    auto add = [&](int32_t c) {
        l3 = nc == 3 ? c : l3; l2 = nc == 2 ? c : l2; l1 = nc == 1 ? c : l1; l0 = nc == 0 ? c : l0;
        ++nc;
    };
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int32_t c = k == 0 ? nd.left : nd.right;
        if (transparent(c)) {
            const int32_t l = nodes[c].left, rr = nodes[c].right;
            if (transparent(l)) { add(nodes[l].left); add(nodes[l].right); } else add(l);
            if (transparent(rr)) { add(nodes[rr].left); add(nodes[rr].right); } else add(rr);
        } else {
            add(c);
        }
    }
    int kinds = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int32_t c = k == 0 ? l0 : k == 1 ? l1 : k == 2 ? l2 : l3;
        double x = 0.0, y = 0.0, cb = 0.0, ca = 0.0;
        int32_t cref = 0, ccnt = 0;
        if (k < nc) {
            double chv;
            if (c < 0) {
                const double2 p = pos[~c];
                x = p.x; y = p.y; chv = QCH_LEAF; cref = c; ccnt = 1;
            } else {
                const BHNode &cn = nodes[c];
                x = cn.cx; y = cn.cy; chv = cn.delta >= 62 ? QCH_TIE : cn.h;
                cref = c; ccnt = cn.cnt;
                if (cn.delta >= 62 && tiecnt && tiecnt[c] > 0) {   // pure duplicate group: one leaf, its multiplicity
                    const double2 p = pos[cn.first];
                    x = p.x; y = p.y; chv = QCH_MULTI; ccnt = tiecnt[c];
                } else if (cn.delta < 62 && dv.vflag && dv.vflag[c]) {   // the chain top C_1 of real node c
                    x = dv.vcom[2 * c]; y = dv.vcom[2 * c + 1]; chv = 0.5 * nd.h;
                    cref = dv.virt + c; ccnt = dv.vcntf[c];
                }
                if (chv >= 0.0) { ca = qacc_accept(chv, inv_theta); cb = qacc_open(chv, inv_theta); }
            }
            kinds |= (chv == QCH_LEAF ? QK_LEAF : chv == QCH_TIE ? QK_TIE : chv == QCH_MULTI ? QK_MULTI : QK_CELL)
                     << (QNCH_KIND + 2 * k);
        }
        r.ccx[k] = x; r.ccy[k] = y; r.cb[k] = cb; r.ca[k] = ca; r.cref[k] = cref; r.ccnt[k] = ccnt;
    }
    const double hx = 0.5 * (nd.bx1 - nd.bx0), hy = 0.5 * (nd.by1 - nd.by0);
    const bool tile_possible = (nd.rball > 0.0 || (hx * hx + hy * hy) * (1.0 - 1e-9) <= fmax(nd.hmin * inv_theta, near_dmax))
                               && !(notile && notile[i]);
    r.nch = nc | (tile_possible ? QNCH_TILE : 0) | kinds;
}

// Traversal: one wave = 64 consecutive sorted queries sharing an LDS stack of
// (cell, lane mask) entries, one per cell that some lane OPENS.  Popping a
// cell loads its quad record once; every lane that opened it then takes its
// own reference decision for each quad child from the record (a leaf
// interacts; a cell is summarised when max(hW,hH)/D < theta, else pushed with
// the mask of the lanes that open it).  Fast path on pop: if for a lane EVERY
// real cell of the subtree would be opened, the reference would reach every
// leaf of it, so the lane sums the subtree's leaves directly (moment task or
// dense tile over the contiguous range of sorted points).  That is the
// near-exact regime of a small embedding.
// Two conservative all-open tests, either suffices (rounding margins kept):
//  * ball: |q - com|^2 <= rball^2, where ball(com, rball) lies inside every
//    descendant cell's "opened" disc |q - c_u|^2 <= h_u / theta (bottom_up);
//  * box: max squared distance from q to the subtree's bounding box
//    <= hmin / theta (hmin = smallest real cell half-width inside).
// A third test admits subtrees whose reference sum provably equals the exact
// leaf sum to BH_NEAR_TOL relative: a cell c is summarised only when
// h_c < theta D, and replacing its n_c points by their centre of mass changes
// sum 1/(1+D) by at most (8 + 32 D) h_c^2 n_c (second-order Taylor; the first
// order vanishes at the centre of mass) and sum (q-y)/(1+D)^2 by at most
// ~24 sqrt(D) h_c^2 n_c.  With every point of the subtree within
// D <= near_dmax of q (box corners), the relative deviation is below
// ~48 theta^2 near_dmax^2 <= BH_NEAR_TOL (bh_near_dmax).  In the tiny-embedding
// phase (extent ~1e-3) the root passes for every query: one moment task each.
// Dense leaf tiles are not run inside the traversal: the wave appends (leaf
// range, lane mask) to its own task list (DENSE_CAP entries; when full, the
// lanes simply keep traversing the subtree -- the reference's own path) and
// dense_apply sums the tiles afterwards.  This keeps the traversal at <= 64
// VGPRs (8 waves per SIMD to hide the record fetches) instead of ~100.

// ---- Narrow layout for heavy 64-query groups.
// A wave's BH work is the depth-first walk of its shared stack; its span is
// the serial chain pop -> record fetch -> child tests -> push.  In dense
// clusters a few 64-query groups carry 10-20x the mean work (DESIGN.md 6,
// "BH mid phase") and that chain alone sets the grid's span.  Such groups
// (previous traversal cost >= Options::narrow x the mean, narrow_select) run
// as NPARTS waves of NQ queries each, with the lanes laid out as (record k,
// query q, child c): one pass takes NKP stack entries at once and evaluates
// the 4 children of each for NQ queries in ONE sweep of the lanes, where the
// 64-query layout spends 4 sweeps (one per child) per entry with most lanes
// masked off.  The stack entries carry NQ-bit query masks.  All-open /
// near-exact tiles are summed inline (the 4 child lanes of a query split the
// subtree's points) or become moment tasks on the group's own lists
// (narrow_moment_apply).  Each lane keeps its own partial sums; the NKP x 4
// lanes of a query are added by a fixed xor butterfly at the end, so the
// result does not depend on timing (it differs from the 64-query layout's
// association only at rounding level: the same cells are summarised, the
// same leaves and tiles summed).
constexpr int NQ_LOG = 2;
constexpr int NQ = 1 << NQ_LOG;    // queries per narrow wave
constexpr int NKP = 16 / NQ;       // stack entries per narrow pass
constexpr int NPARTS = 64 / NQ;    // narrow waves per 64-query group (NPARTS / 4 workgroups)
static_assert(NKP * NQ * 4 == 64 && NPARTS % 4 == 0 && STACK / 2 + 4 * NKP + 3 * 32 <= STACK, "narrow lane layout, stack bound");

// bits {4 i : i < NQ} of x (one query per 4 lanes) -> bits {i}
__device__ __forceinline__ uint32_t narrow_compress(uint64_t x) {
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < NQ; ++i) m |= (uint32_t)((x >> (4 * i)) & 1ull) << i;
    return m;
}
// lanes (k, q, c = 0) for every record slot k: query q's first lane in each
__host__ __device__ constexpr uint64_t narrow_qcol0() {
    uint64_t m = 0;
    for (int k = 0; k < NKP; ++k) m |= 1ull << (k * 4 * NQ);
    return m;
}

struct NarrowView {
    const int32_t *hlist = nullptr;    // heavy slot -> 64-query group
    const int32_t *hcount = nullptr;   // [0] heavy groups this traversal
    int32_t *ncost = nullptr;          // per heavy slot x part: the narrow wave's cost (next selection)
    int32_t *mtask = nullptr;          // per heavy slot x 64 queries: moment tasks (MOM_TASKS each)
    int32_t *mtask_n = nullptr;
    const int32_t *nflag = nullptr;    // per group: heavy slot + 1, or 0 (the 64-query layout)
    int32_t nbn = 0;                   // workgroups of the narrow part of the grid (hmax x NPARTS / 4)
    unsigned long long *wlog = nullptr;   // STATS + option wave_log: per-wave timeline (wave_log_put)
};

// Option wave_log (counting calls only): every traversal / narrow / tile wave
// appends (start, end << 2 | kind) in 100 MHz wall ticks; wlog[0] counts.
constexpr int64_t WAVE_LOG_CAP = 1 << 17;
__device__ __forceinline__ void wave_log_put(unsigned long long *wlog, unsigned long long t0, unsigned long long t1,
                                             int kind) {
    if (!wlog) return;
    const unsigned long long k = atomicAdd(wlog, 1ull);
    if (k < (unsigned long long)WAVE_LOG_CAP) {
        wlog[1 + 2 * k] = t0;
        wlog[2 + 2 * k] = (t1 << 2) | (unsigned long long)kind;
    }
}

// Tree partition (several ranks, bh_repulsion with `plim`): rank r owns the
// sorted positions [lo, hi) and walks every query over the cells that hold
// points of its own.  The cuts sit on boundaries of level-PART_LEVEL cells
// (part_align), so at most PART_LEVEL levels of records straddle a cut.  A
// record inside [lo, hi) takes the normal path; a straddling ("shared") one
// the slow path of bh_traverse<., true>: a child without points of mine is
// skipped, an opened one pushed, and a child's term (summarised cell, leaf,
// duplicate leaf or key-tie group) is taken only by the rank owning the
// child's first point -- so over the ranks every term of the reference's sum
// is taken exactly once.  A shared record that passes the all-open /
// near-exact test for a lane is an exact leaf sum for it: its children are
// pushed with REF_FORCED (lanes in exact-sum mode); a forced record of mine
// becomes one tile task (the exact leaf sum over its range), a forced shared
// one is expanded again.  The sum over the ranks of these parts is the
// record's exact leaf sum, up to rounding and the moments' 1e-12 truncation.
constexpr int32_t REF_FORCED = 1 << 30;
constexpr int PART_LEVEL = 10;

// The traversal kernels' state (LDS per WPB-wave block): KB records per batch
// (4 in the 64-query layout, NKP in the narrow one).
template <int KB, int WPB = 4>
struct TravLDS_T {
    QRec srec[WPB][KB];          // first: the record fields' LDS offsets fit the ds_read2 immediates
    int32_t sref[WPB][STACK];
    uint64_t smask[WPB][STACK];
    int32_t bref[WPB][KB];       // the batch's refs (its masks ride in the records' lmask)
};
// Waves per block of the 64-query traversal (a block holds its LDS and wave
// slots until its last wave ends; 2 instead of 4: C3 loop 5.03 / 5.02 vs
// 5.03 / 5.04 s, t = 450 snapshot span 13.6 vs 13.5 ms -- not the limiter,
// round 6)
#ifndef TRAV_WPB
#define TRAV_WPB 4
#endif
using TravLDS = TravLDS_T<4, TRAV_WPB>;
using NarrowLDS = TravLDS_T<(NKP > 4 ? NKP : 4)>;

// Stage the records of stack entries [sp, sp + k) of wave w into LDS (one
// round of coalesced 16-byte loads; their latencies overlap), each with its
// entry's lane mask in the copy's lmask slot (read with the record's other
// fields from one LDS address).
template <class LDS>
__device__ __forceinline__ void stage_records(LDS &L, int w, int lane, int sp, int k,
                                              const QRec *__restrict__ qrec) {
    static_assert(offsetof(QRec, lmask) == 16 * (QREC_V4 - 1) + 8, "lmask: the upper half of the last 16 bytes");
    if (lane < k) L.bref[w][lane] = L.sref[w][sp + lane];
    for (int e = lane; e < QREC_V4 * k; e += 64) {
        const int rr = e / QREC_V4, part = e - rr * QREC_V4;
        const int rf = L.sref[w][sp + rr] & ~REF_FORCED;
        uint4 v = reinterpret_cast<const uint4 *>(qrec + rf)[part];
        if (part == QREC_V4 - 1) {
            const uint64_t m = L.smask[w][sp + rr];
            v.z = (uint32_t)m;
            v.w = (uint32_t)(m >> 32);
        }
        reinterpret_cast<uint4 *>(&L.srec[w][rr])[part] = v;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0);   // vmcnt = lgkmcnt = 0: batch staged in LDS
    __builtin_amdgcn_wave_barrier();
}

// The half width of cell child `cref` of record `ref` (flags stripped), for
// the exact-quotient band (QACC_BAND): a real node's own h, or for the
// virtual chain top of a duplicate group (cref >= virt) half its parent's
// (build_qrec_reg).  A virtual record's only child is a real node.
__device__ __forceinline__ double qrec_child_h(const BHNode *__restrict__ nodes, int32_t ref, int32_t cref,
                                               int32_t virt) {
    return cref < virt ? nodes[cref].h : 0.5 * nodes[ref & ~REF_FORCED].h;
}

// The reference's summarise decision for a cell child from D1 = 1 + D (see
// QACC_BAND): the two record bounds, the exact IEEE quotient in between.
__device__ __forceinline__ bool qrec_accept(const QRec &nd, int c, double D1, double dx, double dy, double theta,
                                            const BHNode *__restrict__ nodes, int32_t ref, int32_t virt) {
    if (D1 > nd.ca[c]) return true;
    if (D1 < nd.cb[c]) return false;
    return qrec_child_h(nodes, ref, nd.cref[c], virt) / __dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)) < theta;
}

// All-open / near-exact test of one (query, record) pair (see the comment above
// bh_traverse): the subtree's exact leaf sum replaces its walk.
// (The record carries the box's part of the rounding margin and the bound
// with its 1 + 1e-12 factor folded in: 5 fp64 operations fewer per lane.)
__device__ __forceinline__ bool tile_test(const QRec &nd, double qx, double qy, double qmag) {
    const double cdx = qx - nd.cx, cdy = qy - nd.cy;
    const double dc = cdx * cdx + cdy * cdy;
    bool tile = dc <= nd.rball;   // rball^2 (1 - 1e-9)
    if (!tile) {
        const double ex = __fma_rn(1e-15, qmag, nd.ex);   // 1e-15 (|q| + |box|)
        const double dxm = fmax(fabs(qx - nd.bx0), fabs(qx - nd.bx1)) + ex;
        const double dym = fmax(fabs(qy - nd.by0), fabs(qy - nd.by1)) + ex;
        tile = dxm * dxm + dym * dym <= nd.hmin;   // max(hmin / theta (1 - 1e-12), near_dmax) / (1 + 1e-12), rounded down
    }
    return tile;
}

// The root: a single point, a key-tie group, or a cell tested like any child.
// Lanes with `eval` take its term for their query (qx, qy); returns the lanes
// that open it (the caller pushes the root record) and its record ref.
template <bool STATS>
__device__ __forceinline__ uint64_t root_step(const double2 *__restrict__ pos, const BHNode *__restrict__ nodes,
                                              const QRec *__restrict__ qrec, const int32_t *__restrict__ meta,
                                              int32_t virt, bool eval, double qx, double qy, double theta,
                                              double th_lo, double th_hi, double &fx, double &fy, double &zs,
                                              unsigned long long &nvis, int32_t &rpush, bool own0 = true) {
    const int root = meta[1];
    rpush = root;
    if (root == ~0) {
        if (eval && own0) { if (STATS) ++nvis; const double2 p = pos[0]; leaf_force(qx, qy, p.x, p.y, fx, fy, zs); }
        return 0;
    }
    if (root < 0) return 0;
    const BHNode &rt = nodes[root];
    if (rt.delta >= 62) {
        for (int p = rt.first; p <= rt.last; ++p) {
            const double2 pp = pos[p];
            if (eval && own0) { if (STATS) ++nvis; leaf_force(qx, qy, pp.x, pp.y, fx, fy, zs); }
        }
        return 0;
    }
    // the root cell; with duplicates whose copies the reference root counts
    // differently from the cells below it: its virtual record (h = W, every
    // copy), opened into the real root node
    double rh = rt.h, rcx = rt.cx, rcy = rt.cy;
    int32_t rcnt = rt.cnt;
    if (meta[3]) {
        const QRec &vq = qrec[virt + root];
        rh = ldexp(rt.h, rt.delta >> 1);
        rcx = vq.cx; rcy = vq.cy; rcnt = vq.cnt; rpush = virt + root;
    }
    bool open = false;
    if (eval) {
        if (STATS) ++nvis;
        const double dx = qx - rcx, dy = qy - rcy;
        const double D = __fma_rn(dx, dx, dy * dy);
        if (summarise(rh, D, dx, dy, th_lo, th_hi, theta)) { if (own0) cell_force(dx, dy, D, rcnt, fx, fy, zs); }
        else open = true;
    }
    return __ballot(open);
}

// One narrow wave: part `part` (queries part*NQ .. +NQ-1) of heavy group `grp`
// (heavy slot h).  See "Narrow layout" above.
template <int MODE>
__device__ void narrow_wave(NarrowLDS &L, const double2 *__restrict__ pos, const int32_t *__restrict__ dupc,
                            const BHNode *__restrict__ nodes, const QRec *__restrict__ qrec,
                            const int32_t *__restrict__ meta, const double *__restrict__ unused_mom, bool mom_on,
                            double mom_tol, double theta, int64_t g0, int64_t g1, const int32_t *__restrict__ qlist,
                            int32_t virt, double2 *__restrict__ F, double *__restrict__ Z,
                            unsigned long long *__restrict__ visits, unsigned long long *__restrict__ bcost,
                            const int32_t *__restrict__ cost_lab, int32_t *__restrict__ ttask_n,
                            int32_t *__restrict__ tcost, int32_t *__restrict__ mom_flag, const NarrowView &nv,
                            int64_t h, int part, int w) {
    constexpr bool STATS = MODE == 2, COST = MODE >= 1;
    (void)unused_mom;
    const int lane = lane_id();
    const int c = lane & 3, q = (lane >> 2) & (NQ - 1), k = lane >> (2 + NQ_LOG);
    const int64_t grp = nv.hlist[h];
    const double th_lo = theta * (1.0 - 1e-14), th_hi = theta * (1.0 + 1e-14);
    const int64_t kq = g0 + grp * 64 + part * NQ + q;
    const bool valid = kq < g1;
    const int32_t s = valid ? (qlist ? qlist[kq] : (int32_t)kq) : -1;   // sorted position (< 2^31)
    // (the group's empty tile list and cost are the 64-query kernel's: tile_apply
    // need not wait for this kernel)
    const long long t_start = COST ? clock64() : 0;
    const unsigned long long w_start = STATS ? wall_clock64() : 0;
    double qx = 0.0, qy = 0.0;
    if (valid) { const double2 qq = pos[s]; qx = qq.x; qy = qq.y; }
    double fx = 0.0, fy = 0.0, zs = 0.0;
    unsigned long long nvis = 0;
    int32_t npops = 0, ntilepts = 0, ntask = 0, nwant = 0;
    int sp = 0;
    {
        int32_t rpush;
        const uint64_t om = root_step<STATS>(pos, nodes, qrec, meta, virt, valid && k == 0 && c == 0, qx, qy, theta,
                                             th_lo, th_hi, fx, fy, zs, nvis, rpush);
        const uint32_t qm = narrow_compress(om);
        if (qm) {
            if (lane == 0) { L.sref[w][0] = rpush; L.smask[w][0] = qm; }
            sp = 1;
        }
    }
    while (sp > 0) {
        const int kn = sp > STACK / 2 ? 1 : (sp < NKP ? sp : NKP);
        sp -= kn;
        stage_records(L, w, lane, sp, kn, qrec);
        npops += kn;
        const bool kin = k < kn;
        const int kk = kin ? k : 0;
        const QRec &nd = L.srec[w][kk];
        const uint32_t msk = (uint32_t)nd.lmask;
        bool act = kin && valid && ((msk >> q) & 1u);
        const int nflags = nd.nch;
        bool tile = false;
        if ((nflags & QNCH_TILE) && act) tile = tile_test(nd, qx, qy, fabs(qx) + fabs(qy));
        if (__ballot(tile)) {
            const int a = nd.first, b = nd.last, cnt = nd.cnt;
            // moment path: decided once per (record, query) by its child-0 lane,
            // tasks appended per query in record order (capped at MOM_TASKS)
            const bool mw = tile && c == 0 && cnt >= MOM_MIN_POINTS && moment_ok(nd.bx0, nd.bx1, nd.by0, nd.by1, qx, qy, mom_tol);
            nwant += mw ? 1 : 0;
            const uint64_t U = __ballot(mw && mom_on);
            // same-query lanes of earlier records: the task order within a pass
            const uint64_t qcol = narrow_qcol0() << (4 * q);
            const int before = __popcll(U & qcol & lanemask_lt());
            const bool usem = mw && mom_on && ntask + before < MOM_TASKS;
            if (usem) nv.mtask[(h * 64 + part * NQ + q) * MOM_TASKS + ntask + before] = L.bref[w][kk];
            ntask = min(MOM_TASKS, ntask + (int)__popcll(U & qcol));
            const uint64_t UM = __ballot(usem);
            const bool dense = tile && !((UM >> (lane & ~3)) & 1ull);
            // the range holds whole equal-key runs: the query's duplicates (itself
            // included) add exactly 1 each to z in the leaf sum, taken off here
            if (tile && c == 0 && s >= a && s <= b) zs -= (double)dupc[s];
            if (STATS && tile && c == 0) nvis += (unsigned long long)(b - a + 1);
            // dense: the query's 4 lanes split the subtree's points, summed
            // apart and added once (accumulating into fx / fy / zs inside the
            // divergent loop made the compiler copy them at every merge)
            // (a divergent do-while: lanes leave it one by one, no merge per point)
            double ux = 0.0, uy = 0.0, uq = 0.0;
            if (dense && a + c <= b) {
                int p = a + c;
                do {
                    const double2 pp = pos[p];
                    pair_force(qx, qy, pp.x, pp.y, ux, uy, uq);
                    p += 4;
                } while (p <= b);
            }
            if (dense) { fx += ux; fy += uy; zs += uq; }
            const uint64_t tm = __ballot(tile && c == 0);
            for (uint64_t r = tm; r; r &= r - 1) {   // cost: points per (record, query), as the 64-query layout's
                const int l = __ffsll((long long)r) - 1;
                ntilepts += __shfl(b - a + 1, l, 64);
            }
            act = act && !tile;
        }
        if (__ballot(act) == 0) continue;
        // child c of record k for query q
        const int nch = nflags & 0xff;
        const int kind = (nflags >> (QNCH_KIND + 2 * c)) & 3;
        const bool has = act && c < nch;
        const double dx = qx - nd.ccx[c], dy = qy - nd.ccy[c];
        const double D1 = __fma_rn(dx, dx, __fma_rn(dy, dy, 1.0));   // 1 + D (QACC_BAND)
        const bool isleaf = has && kind == QK_LEAF, iscell = has && kind == QK_CELL;
        bool acc = D1 > nd.ca[c];
        if (iscell && !acc && !(D1 < nd.cb[c]))
            acc = qrec_child_h(nodes, L.bref[w][kk], nd.cref[c], virt) / __dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)) <
                  theta;
        const bool takel = isleaf && !(dx == 0.0 && dy == 0.0);
        const bool takec = iscell && acc;
        const double wm = takel ? 1.0 : (takec ? (double)nd.ccnt[c] : 0.0);
        if (STATS && (isleaf || iscell)) ++nvis;
        const double Qv = recip_bh(D1);
        const double mult = wm * Qv;
        const double sc = mult * Qv;
        fx = __fma_rn(sc, dx, fx);
        fy = __fma_rn(sc, dy, fy);
        zs += mult;
        // duplicate kinds (rare)
        const bool dupk = has && (kind == QK_MULTI || kind == QK_TIE);
        if (__builtin_expect(__ballot(dupk) != 0, 0)) {
            if (dupk && kind == QK_MULTI) {   // a leaf of ccnt copies: 0 if it is the query's point
                if (!(nd.ccx[c] == qx && nd.ccy[c] == qy)) {
                    if (STATS) ++nvis;
                    cell_force(dx, dy, __fma_rn(dx, dx, dy * dy), nd.ccnt[c], fx, fy, zs);
                }
            } else if (dupk) {                // a key-tie group: every point directly
                const BHNode &tn = nodes[nd.cref[c]];
                for (int p = tn.first; p <= tn.last; ++p) {
                    const double2 pp = pos[p];
                    if (STATS) ++nvis;
                    leaf_force(qx, qy, pp.x, pp.y, fx, fy, zs);
                }
            }
        }
        // pushes: one entry per (record, child) that some query opens, in lane order
        const uint64_t O = __ballot(iscell && !acc);
        const bool pl = q == 0 && kin;
        const uint32_t m = pl ? narrow_compress(O >> (k * 4 * NQ + c)) : 0u;
        const uint64_t P = __ballot(m != 0u);
        if (m) {
            const int at = sp + (int)__popcll(P & lanemask_lt());
            L.sref[w][at] = nd.cref[c];
            L.smask[w][at] = m;
        }
        sp += (int)__popcll(P);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the pushes landed before the next pop
        __builtin_amdgcn_wave_barrier();
    }
    // the query's NKP x 4 lanes, in a fixed xor butterfly (every lane the same bits)
#pragma unroll
    for (int o = 1; o <= 2; o <<= 1) {
        fx += __shfl_xor(fx, o, 64); fy += __shfl_xor(fy, o, 64); zs += __shfl_xor(zs, o, 64);
    }
#pragma unroll
    for (int o = 4 * NQ; o < 64; o <<= 1) {
        fx += __shfl_xor(fx, o, 64); fy += __shfl_xor(fy, o, 64); zs += __shfl_xor(zs, o, 64);
    }
    if (k == 0 && c == 0 && valid) {
        F[s] = make_double2(fx, fy);
        Z[s] = zs;
    }
    if (k == 0 && c == 0) nv.mtask_n[h * 64 + part * NQ + q] = valid ? ntask : 0;
    const int wwant = wave_sum(nwant);
    if (lane == 0) {
        nv.ncost[h * NPARTS + part] = npops + (ntilepts >> 6);
        if (wwant && __hip_atomic_load(&mom_flag[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < mom_flag[2])
            atomicAdd(&mom_flag[1], wwant);
    }
    // this wave's run time into its queries' buckets (multi-GPU balancing); a
    // wave of the last, partial group may hold no query at all: nothing to add
    if (COST && bcost && __ballot(valid)) {
        const unsigned long long cc = ((unsigned long long)(clock64() - t_start) >> 6) + 1;
        if (cost_lab) {
            if (valid && k == 0 && c == 0) atomicAdd(&bcost[cost_lab[s] >> 8], (cc + NQ - 1) / NQ);
        } else {
            const int64_t sf = wave_min(valid ? s : ((int64_t)1 << 62));
            if (lane == 0) atomicAdd(&bcost[sf >> 8], cc);
        }
    }
    if (STATS && visits) {
        const unsigned long long tv = wave_sum(nvis);
        if (lane == 0) {
            atomicAdd(visits, tv);
            atomicAdd(visits + 3, (unsigned long long)npops);
            atomicAdd(visits + 4, (unsigned long long)ntilepts);
            atomicMax(visits + 8, (unsigned long long)npops);
            atomicAdd(visits + 30, 1ull);   // narrow waves run
            const unsigned long long w_end = wall_clock64();
            atomicMax(visits + 15, w_end - w_start);
            atomicMax(visits + 16, ~0ull - w_start);
            atomicMax(visits + 17, w_end);
            atomicAdd(visits + 18, w_end - w_start);
            atomicAdd(visits + 37, (unsigned long long)(clock64() - t_start));   // shader cycles (wave_mhz)
            atomicMax(visits + 31, w_end - w_start);   // longest narrow wave
            wave_log_put(nv.wlog, w_start, w_end, 1);
        }
    }
}

// The narrow waves of the heavy groups: 4 per workgroup, idle beyond the
// heavy count.  A kernel of its own (its ~78 VGPRs would cost the 64-query
// layout's 8 waves per SIMD), launched on a second stream beside bh_traverse.
template <int MODE>
#ifdef NARROW_WPE   // A/B builds: the narrow waves' occupancy bound (waves per SIMD)
#define NARROW_ATTR __attribute__((amdgpu_waves_per_eu(NARROW_WPE)))
#else
#define NARROW_ATTR
#endif
__global__ __launch_bounds__(256) NARROW_ATTR void bh_traverse_narrow(
    const double2 *__restrict__ pos, const int32_t *__restrict__ dupc, const BHNode *__restrict__ nodes,
    const QRec *__restrict__ qrec, int32_t *__restrict__ ttask_n, const int32_t *__restrict__ meta,
    int32_t *__restrict__ mom_flag, double mom_tol, double theta, int64_t g0, int64_t g1,
    const int32_t *__restrict__ qlist, int32_t virt, double2 *__restrict__ F, double *__restrict__ Z,
    unsigned long long *__restrict__ visits, unsigned long long *__restrict__ bcost, int32_t *__restrict__ tcost,
    const int32_t *__restrict__ cost_lab, NarrowView nv) {
    __shared__ NarrowLDS L;
    const int w = threadIdx.x >> 6;
    const int64_t slot = (int64_t)blockIdx.x * 4 + w;   // heavy slot x part
    const int64_t h = slot / NPARTS;
    if (h >= (int64_t)*nv.hcount) return;
    narrow_wave<MODE>(L, pos, dupc, nodes, qrec, meta, nullptr, mom_flag[0] != 0, mom_tol, theta, g0, g1, qlist, virt,
                      F, Z, visits, bcost, cost_lab, ttask_n, tcost, mom_flag, nv, h, (int)(slot % NPARTS), w);
}

// ---- Spill: splitting long walks over the chip (Options::spill; round 6).
// A walk -- a wave's own 64-query group, or a task -- that has popped its
// budget of records stops at the next batch boundary and hands its LDS stack
// (the rest of the walk: (cell record, lane mask) entries) to the task list of
// the next level, cut into tasks of consecutive entries (1, 1, 2, 4, 8, 16, 16,
// ... from the bottom of the stack, whose entries are the largest subtrees).
// Level l's tasks are taken by the l-th drain launch after the traversal: one
// atomic add per claim on the level's head, no waiting (the list is complete
// when the launch starts, as its producers ran in the previous launch); the
// task's entries become the wave's stack, the walk is the same loop -- the
// reference's opened / summarised cells (QuadTree.scala:123-152: a cell's
// decision depends on the query and the cell only, not on who walks it) --
// and splits again into level l + 1 (the last level never splits).  The split
// points depend on the pop counts of the walks alone (the tree and the
// queries), not on timing; the tasks' sums go to per-query fixed-point
// accumulators (2^-64 units in two carry-free words, fxp_add), whose integer
// adds are associative, so the result does not depend on which wave took which
// task.
// Tiles a task records go to 64-tile pages (tile_apply<true>), added the same
// way.  The heavy waves of the mid phase are one LDS stack walked serially
// (DESIGN 5, 6): this spreads their walks over the chip.
constexpr int SP_LMAX = 4;     // task levels (drain launches) at most
constexpr int SP_PAGES = 0, SP_B0 = 1, SP_B1 = 2, SP_OVF = 3, SP_TASKS = 4;
__host__ __device__ constexpr int sp_head(int l) { return 8 + 3 * (l - 1); }    // level l's next task to take
__host__ __device__ constexpr int sp_ttail(int l) { return 9 + 3 * (l - 1); }   // level l's tasks
__host__ __device__ constexpr int sp_etail(int l) { return 10 + 3 * (l - 1); }  // level l's stack entries
constexpr int SP_NCTL = 8 + 3 * SP_LMAX;
constexpr int SP_FRAC = 64;    // fixed-point fraction bits: |value| < 2^31, resolution 2^-64
constexpr int SP_PAGE = 64;    // tiles per task tile page
constexpr int SP_CHUNK = 16;   // stack entries per task at most (<= 64: one lane each)
struct SpillView {
    int32_t *ctl = nullptr;               // SP_* / sp_*(l) words
    int4 *task = nullptr;                 // level l's at [(l - 1) cap, l cap): {group, first entry, entries, 0}
    uint4 *ent = nullptr;                 // level l's at [(l - 1) cap, l cap): {ref, 0, mask lo, mask hi}
    int32_t *gflag = nullptr;             // group -> gen when it spilled
    unsigned long long *acc = nullptr;    // sorted position -> fx, fy, z as (lo, hi)
    TileTask *pg_tiles = nullptr;
    int32_t *pg_grp = nullptr, *pg_n = nullptr;
    int32_t cap = 0, pg_cap = 0, gen = 0;
    int32_t lin = 0;    // TASK launches: the level whose tasks they take
    int32_t lout = 0;   // the level a walk past its budget splits into (0: none, the last level)
    int32_t force = 0;  // > 0: both budgets this many pops
};

// ---- Tile streaming (option tile_stream, round 6)
// The 64-query traversal's tail -- its last, heavy waves finishing one by one
// -- leaves wave slots idle, while tile_apply's work waits for the whole grid.
// With streaming, a traversal wave whose list is short enough (st_streamed:
// tile cost <= maxcost, so the slot path would not chunk it) hands it over
// when it ends: its list stored, an agent-scope release, then the item
// gen << 32 | wave at items[tail++].  tile_apply<2>, a persistent grid of
// tile_stream workgroups per CU on a stream of its own, dispatched once every
// traversal block has started (hipStreamWaitValue32 on ST_STARTED, which the
// blocks count; tile_stream_gate 0: at once), takes items in order (head++);
// it waits a bounded while for a claimed item to appear and otherwise leaves.
// A list goes to whichever path claims its wave first (claims[wave]: gen << 2
// | 1 the slot path, | 2 a consumer; compare-and-swap), so a list published
// after the consumers left is summed by the slot path.  A consumer sums a list
// as the slot path does a one-chunk wave -- D (the dense terms, the same
// loops) into per-item partials and the moment list -- and stream_finish,
// after the traversal's launch and the consumers, adds M (the moment terms in
// list order, from 0) and then F += D + M, as moment_apply and chunk_combine
// would: the same bits, whichever path took a list and when.  Handed-over
// words are read through the vector path after the acquire (it does not
// invalidate the scalar cache).  Nothing waits on a later launch, so no
// consumer can hold resources another stream's kernel needs to finish.
constexpr int ST_STARTED = 0, ST_TAIL = 1, ST_HEAD = 2, ST_CUM = 9, ST_W = 10;
constexpr int ST_RESET = 8;     // words [0, 8) zeroed after every call (ST_CUM accumulates;
                                // ST_W: the streaming threshold the last tile plan set)
constexpr int ST_Q0 = 16;       // the claims (one word per wave slot) from word 16 on, then the items (8 B each)

#ifndef TSNE_ST_TRAV
#define TSNE_ST_TRAV 1   // 0: the traversal's hand-over hooks compiled out (A/B of their cost only)
#endif
struct StreamView {
    int32_t *ctl = nullptr;             // ST_* words, then the claims, then the items
    int32_t gen = 0;                    // this call's generation (never 0)
    int32_t maxcost = 0;                // > 0: streamed when the tile cost (points + 16 per task) <= maxcost;
                                        // 0: <= ctl[ST_W] (the previous plan's chunk unit x tile_stream_frac)
    int32_t cap = 0;                    // wave slots the claims and items have room for
    int32_t total = 0;                  // traversal wave slots of this call (blocks x TRAV_WPB)
    int32_t prio = 0;                   // the 64-query traversal waves' issue priority (s_setprio; option trav_prio)
    int32_t wait = 48;                  // polls (s_sleep 16 each, ~0.4 us) a consumer waits for a claimed item
    unsigned long long *wlog = nullptr; // the wave timeline (tile_apply's waves; see NarrowView::wlog)
    const int32_t *border = nullptr;    // the 64-query traversal's workgroup order (trav_front), or identity
};
__device__ __forceinline__ int32_t *st_claims(int32_t *ctl) { return ctl + ST_Q0; }
__device__ __forceinline__ unsigned long long *st_items(int32_t *ctl, int32_t cap) {
    return reinterpret_cast<unsigned long long *>(ctl + ST_Q0 + ((cap + 1) & ~1));
}
// A wave's claim word: gen << 2 when its list was handed over this call,
// | 1 once the slot path, | 2 once a consumer took it.  Claim for `who`: the
// owner (`who` itself for a list that was not handed over: the slot path's).
__device__ __forceinline__ int32_t st_claim(int32_t *claims, int64_t w, int32_t gen, int32_t who) {
    int32_t v = __hip_atomic_load(&claims[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
        if ((v >> 2) != gen) return who;
        if (v & 3) return v & 3;
        if (__hip_atomic_compare_exchange_strong(&claims[w], &v, (gen << 2) | who, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return who;
    }
}

// A load through the vector path: handed-over bytes read after the acquire
// must not come from the scalar cache, which the acquire does not invalidate
// (a wave-uniform address would otherwise make it an s_load).
template <class T> __device__ __forceinline__ T vec_load(const T *p) {
    asm volatile("" : "+v"(p));
    return *p;
}

// a += v as fixed point: X = v 2^64 truncated toward zero (|v| < 2^31), kept
// as two words that add without carries, so both atomics are independent
// (no returned value to wait for): a[0] += the low 32 bits of X (unsigned,
// < 2^32 per add), a[1] += X >> 32 (signed).  The value is a[1] 2^-32 +
// a[0] 2^-64, exact as a 128-bit integer; resolution 2^-64 absolute.
__device__ __forceinline__ void fxp_add(unsigned long long *a, double v) {
    if (v == 0.0) return;
    const unsigned long long bits = (unsigned long long)__double_as_longlong(v);
    const int ex = (int)((bits >> 52) & 0x7ff);
    const unsigned long long M = (bits & 0xFFFFFFFFFFFFFull) | (ex ? (1ull << 52) : 0ull);
    const int sh = (ex ? ex : 1) - 1075 + SP_FRAC;   // |v| 2^64 = M 2^sh
    unsigned long long lo, hi;                       // |X| = hi 2^32 + lo, lo < 2^32
    if (sh >= 32) { lo = (M << sh) & 0xFFFFFFFFull; hi = M << (sh - 32); }
    else if (sh >= 0) { const unsigned long long m = M << sh; lo = m & 0xFFFFFFFFull; hi = sh ? (M >> (32 - sh)) : (M >> 32); }
    else if (sh > -64) { const unsigned long long m = M >> (-sh); lo = m & 0xFFFFFFFFull; hi = m >> 32; }
    else { lo = 0; hi = 0; }
    if (bits >> 63) {   // X = -|X|: lo' = (2^32 - lo) mod 2^32, hi' = -hi - (lo != 0)
        hi = ~hi + (lo ? 0ull : 1ull);
        lo = (0x100000000ull - lo) & 0xFFFFFFFFull;
    }
    atomicAdd(a, lo);
    atomicAdd(a + 1, hi);
}
__device__ __forceinline__ double fxp_value(unsigned long long lo, unsigned long long hi) {
    return ldexp((double)(long long)hi, 32 - SP_FRAC) + ldexp((double)lo, -SP_FRAC);
}

// task k of a split: its first entry and size (1, 1, 2, 4, 8, 16, 16, ...)
__device__ __forceinline__ int sp_size(int k) { return k < 2 ? 1 : min(1 << (k - 1), SP_CHUNK); }
__device__ __forceinline__ int sp_start(int k) {
    int s = 0;
    for (int j = 0; j < k; ++j) s += sp_size(j);
    return s;
}
__device__ __forceinline__ int sp_ntasks(int n) {
    int k = 0;
    for (int c = 0; c < n; ++k) c += sp_size(k);
    return k;
}

// The next task of level sv.lin (wave-uniform; false when the level's list is
// taken): its group, and its entries pushed onto wave w's stack (sp).
template <class LDS>
__device__ __forceinline__ bool sp_next(const SpillView &sv, LDS &L, int w, int64_t &grp, int &sp) {
    int h = -1;
    if (lane_id() == 0) {
        h = atomicAdd(&sv.ctl[sp_head(sv.lin)], 1);
        if (h >= sv.ctl[sp_ttail(sv.lin)]) h = -1;
    }
    h = __builtin_amdgcn_readfirstlane(h);
    if (h < 0) return false;
    const int4 tk = sv.task[(int64_t)(sv.lin - 1) * sv.cap + h];
    grp = __builtin_amdgcn_readfirstlane(tk.x);
    const int e0 = __builtin_amdgcn_readfirstlane(tk.y), n = __builtin_amdgcn_readfirstlane(tk.z);
    if (lane_id() < n) {
        const uint4 v = sv.ent[(int64_t)(sv.lin - 1) * sv.cap + e0 + lane_id()];
        L.sref[w][lane_id()] = (int32_t)v.x;
        L.smask[w][lane_id()] = ((uint64_t)v.w << 32) | v.z;
    }
    sp = n;
    return true;
}

// Room for n stack entries (and their tasks) in level sv.lout's lists: the
// first entry and the first task (wave-uniform), or e = -1 when the entries
// do not fit (the walk goes on: nothing is lost).  Only the allocation runs
// inside the walk's loop (few registers); sp_write fills the slots after it.
__device__ __forceinline__ int sp_alloc(const SpillView &sv, int n, int &t) {
    int e = -1, tt = 0;
    if (lane_id() == 0) {
        int c = __hip_atomic_load(&sv.ctl[sp_etail(sv.lout)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int tries = 0; tries < 100000; ++tries) {
            if (c + n > sv.cap) break;
            if (__hip_atomic_compare_exchange_strong(&sv.ctl[sp_etail(sv.lout)], &c, c + n, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                e = c;
                break;
            }
        }
        if (e < 0) {
            atomicOr(&sv.ctl[SP_OVF], 1);
        } else {   // tasks <= entries <= cap: always room
            const int nt = sp_ntasks(n);
            tt = atomicAdd(&sv.ctl[sp_ttail(sv.lout)], nt);
            atomicAdd(&sv.ctl[SP_TASKS], nt);
        }
    }
    t = __builtin_amdgcn_readfirstlane(tt);
    return __builtin_amdgcn_readfirstlane(e);
}
// Stack entries [0, n) of wave w -> level sv.lout's entries [e, e + n) and
// tasks [t, t + ntasks(n)) of group grp (read by the next launch).
template <class LDS>
__device__ __forceinline__ void sp_write(const SpillView &sv, LDS &L, int w, int e, int t, int n, int32_t grp) {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the stack's last pushes landed
    __builtin_amdgcn_wave_barrier();
    if (lane_id() == 0) sv.gflag[grp] = sv.gen;
    const int64_t lb = (int64_t)(sv.lout - 1) * sv.cap;
    for (int i = lane_id(); i < n; i += 64) {
        const uint64_t m = L.smask[w][i];
        sv.ent[lb + e + i] = make_uint4((uint32_t)L.sref[w][i], 0u, (uint32_t)m, (uint32_t)(m >> 32));
    }
    const int nt = sp_ntasks(n);
    for (int k = lane_id(); k < nt; k += 64) {
        const int a = sp_start(k);
        sv.task[lb + t + k] = make_int4(grp, e + a, min(sp_size(k), n - a), 0);
    }
}

// Traversal kernel (see the comment above), one 64-query group per wave;
// groups the narrow waves take (nv.nflag) return at once.  MODE 0 plain; 1
// wave run times into the multi-GPU cost buckets; 2 every counter (profiling).
// With spill (sv.mode, never with a tree partition) a walk past its budget
// hands the rest to the task queue; TASK: the drain launches' instantiation,
// whose waves take tasks while the queue has any (see "Spill" above) -- a
// kernel of its own, so that the 64-query walk keeps its registers.
template <int MODE, bool PART, bool TASK>
__global__ __launch_bounds__(64 * TRAV_WPB) __attribute__((amdgpu_waves_per_eu(8))) void bh_traverse(
    const double2 *__restrict__ pos, const int32_t *__restrict__ dupc, const BHNode *__restrict__ nodes,
    const QRec *__restrict__ qrec, TileTask *__restrict__ ttask, int32_t *__restrict__ ttask_n,
    const int32_t *__restrict__ meta, int32_t *__restrict__ mom_flag, double mom_tol, double theta, int64_t g0,
    int64_t g1, const int32_t *__restrict__ qlist, int32_t virt, double2 *__restrict__ F, double *__restrict__ Z,
    unsigned long long *__restrict__ visits, unsigned long long *__restrict__ bcost, int32_t *__restrict__ wcost,
    int32_t *__restrict__ tcost, const int32_t *__restrict__ cost_lab, NarrowView nv, int32_t *__restrict__ plim,
    SpillView sv, StreamView stv) {
    constexpr bool STATS = MODE == 2, COST = MODE >= 1;
    if (!PART && !TASK && stv.prio > 0) {   // issue priority over the waves beside it (option trav_prio)
        if (stv.prio == 1) __builtin_amdgcn_s_setprio(1);
        else if (stv.prio == 2) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(3);
    }
    // tile streaming (see "Tile streaming"): every block counts its start
    if (TSNE_ST_TRAV && !PART && !TASK && stv.ctl && threadIdx.x == 0) atomicAdd(&stv.ctl[ST_STARTED], 1);
    // tree partition: this rank's sorted positions [plo, phi) (plim[2]: stack overflow flag)
    const int32_t plo = PART ? plim[0] : 0, phi = PART ? plim[1] : INT32_MAX;
    __shared__ TravLDS L;
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const double th_lo = theta * (1.0 - 1e-14), th_hi = theta * (1.0 + 1e-14);
    // (option trav_front: the previous traversal's heavy workgroups first)
    const int64_t blk = !PART && !TASK && stv.border ? (int64_t)stv.border[blockIdx.x] : (int64_t)blockIdx.x;
    const int64_t wid = blk * TRAV_WPB + w;   // query slots g0 + 64 wid .. + 63, tile list wid
    const bool spill_on = !PART && sv.lout != 0;
    int32_t bud = 0;   // pops after which a walk splits (0: never)
    if (spill_on) bud = sv.force > 0 ? sv.force : sv.ctl[TASK ? SP_B1 : SP_B0];
    // the wave's first item: its own group, or (TASK) a task
    int64_t grp = wid;
    constexpr bool task = TASK;
    int tsp = 0;   // TASK: the task's entries on the stack
    if (TASK) {
        if (!sp_next(sv, L, w, grp, tsp)) return;
    } else {
        if (g0 + wid * 64 >= g1) return;
        if (lane == 0) { ttask_n[wid] = 0; wcost[wid] = 0; tcost[wid] = 0; }
        if (nv.nflag && nv.nflag[wid]) return;   // a heavy group: the narrow waves take it (no tiles here)
    }
    for (;;) {
    // query slot k -> sorted position s (the identity, or this rank's list of
    // its own queries in sorted order: the waves stay Morton-coherent)
    const int64_t k = g0 + grp * 64 + lane;
    const bool valid = k < g1;
    const int64_t s = valid ? (qlist ? (int64_t)qlist[k] : k) : -1;
    const long long t_start = COST ? clock64() : 0;
    const unsigned long long w_start = STATS ? wall_clock64() : 0;
    int32_t npops = 0, ntilepts = 0;   // wave-uniform: this walk's cost for the next selection
    double qx = 0.0, qy = 0.0;
    if (valid) { double2 q = pos[s]; qx = q.x; qy = q.y; }
    const double qmag = fabs(qx) + fabs(qy);
    const int ndup = valid ? dupc[s] : 0;   // exact duplicates of the query (itself included)
    double fx = 0.0, fy = 0.0, zs = 0.0;
    unsigned long long nvis = 0, nevals = 0, wpops = 0, wtile = 0, wslots = 0;   // STATS only
    unsigned long long wtie = 0;                                               // STATS: key-tie points walked
    unsigned long long wfull = 0, wpart = 0;                                   // STATS only
    int sp = 0;
    int ntt = 0;
    // tile sink: a group's own list (TILE_CAP), or a task's current page
    TileTask *const mytt = ttask + wid * TILE_CAP;
    TileTask *tdst = task ? nullptr : mytt;
    int tcap = task ? 0 : TILE_CAP;
    int32_t page = -1;
    if (!task) {
        int32_t rpush;
        const uint64_t om = root_step<STATS>(pos, nodes, qrec, meta, virt, valid, qx, qy, theta, th_lo, th_hi, fx, fy,
                                             zs, nvis, rpush, plo <= 0 && phi > 0);
        if (om) {
            if (lane == 0) { L.sref[w][0] = rpush; L.smask[w][0] = om; }
            sp = 1;
        }
    } else {
        sp = tsp;   // (sp_next staged its entries)
    }
    // Pop up to 4 cells at a time (one while the stack is over half full: the
    // depth stays bounded): their records are fetched with one round of
    // coalesced 16-byte vector loads, then processed one by one from LDS
    // broadcasts.  (A software pipeline -- the next batch's records in flight
    // in registers while one is processed -- measured no gain: C3 loop 5.645
    // vs 5.643 s, BH snapshots within noise; removed.)
    int spe = -1, spt = 0;   // past the budget: where the rest of the walk goes (entries, tasks)
    int32_t wbud = bud;
    while (sp > 0) {
        if (!PART && wbud > 0 && npops >= wbud && sp >= 2) {
            spe = sp_alloc(sv, sp, spt);
            if (spe >= 0) break;
            wbud = 0;   // no room: walk on
        }
        const int kb = sp > STACK / 2 ? 1 : (sp < 4 ? sp : 4);
        sp -= kb;
        stage_records(L, w, lane, sp, kb, qrec);
        const QRec *brec = L.srec[w];
        const int32_t *bref_c = L.bref[w];
        npops += kb;
        for (int r = 0; r < kb; ++r) {
            if (STATS) ++wpops;
            const int ref = __builtin_amdgcn_readfirstlane(bref_c[r]);
            const uint64_t msk = brec[r].lmask;
            const uint64_t msk_s = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(msk >> 32)) << 32) |
                                   (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)msk);   // the wave's (scalar)
            bool act = __builtin_amdgcn_inverse_ballot_w64(msk_s);   // the mask's own SGPRs: no VALU
            const QRec &nd = brec[r];
            if (PART) {   // a shared or forced record: the tree partition's slow path (see REF_FORCED)
                const int rf = __builtin_amdgcn_readfirstlane(nd.first), rl = __builtin_amdgcn_readfirstlane(nd.last);
                const bool forced = (ref & REF_FORCED) != 0, mine_rec = rf >= plo && rl < phi;
                if (forced || !mine_rec) {
                    auto push = [&](int32_t pref, uint64_t pm) {
                        if (sp >= STACK) {   // the cut alignment bounds the depth: never expected
                            if (lane == 0) plim[2] = 1;
                            return;
                        }
                        if (lane == 0) { L.sref[w][sp] = pref; L.smask[w][sp] = pm; }
                        ++sp;
                    };
                    const int rref = ref & ~REF_FORCED;
                    const int nflags = __builtin_amdgcn_readfirstlane(nd.nch);
                    bool fm = forced && act, an = !forced && act;
                    if (forced && mine_rec && ntt < TILE_CAP) {   // exact sum over a subtree of mine: one tile
                        const uint64_t tm = __ballot(fm);
                        if (lane == 0) {
                            TileTask tt; tt.ref = rref; tt.first = rf; tt.last = rl; tt.pad = nd.cnt; tt.mask = tm;
                            mytt[ntt] = tt;
                        }
                        ++ntt;
                        ntilepts += rl - rf + 1;
                        if (STATS) wtile += (unsigned long long)(rl - rf + 1);
                        if (fm) {
                            if (STATS) nvis += (unsigned long long)(rl - rf + 1);
                            if (s >= rf && s <= rl) zs -= (double)ndup;
                        }
                        continue;
                    }
                    if (!forced && (nflags & QNCH_TILE) && an && tile_test(nd, qx, qy, qmag)) { fm = true; an = false; }
                    if (__ballot(an || fm) == 0) continue;
                    const int nch = nflags & 0xff;
                    for (int c = 0; c < nch; ++c) {
                        const int kind = (nflags >> (QNCH_KIND + 2 * c)) & 3;
                        const int32_t cref = __builtin_amdgcn_readfirstlane(nd.cref[c]);
                        int32_t c0, c1;   // the child's sorted range
                        if (kind == QK_LEAF) {
                            c0 = c1 = ~cref;
                        } else {
                            const BHNode &cn = nodes[cref >= virt ? cref - virt : cref];
                            c0 = __builtin_amdgcn_readfirstlane(cn.first);
                            c1 = __builtin_amdgcn_readfirstlane(cn.last);
                        }
                        if (c1 < plo || c0 >= phi) continue;         // no point of mine below
                        const bool own = c0 >= plo && c0 < phi;      // the term's owner: its first point's rank
                        const double dx = qx - nd.ccx[c], dy = qy - nd.ccy[c];
                        const double D1 = __fma_rn(dx, dx, __fma_rn(dy, dy, 1.0));   // 1 + D (QACC_BAND)
                        if (kind == QK_LEAF || kind == QK_CELL) {
                            bool take, acc = false;
                            if (kind == QK_LEAF) {
                                take = own && (an || fm) && !(dx == 0.0 && dy == 0.0);
                            } else {
                                if (an) acc = qrec_accept(nd, c, D1, dx, dy, theta, nodes, rref, virt);
                                take = own && an && acc;
                                const uint64_t om = __ballot(an && !acc), fmm = __ballot(fm);
                                if (om) push(cref, om);
                                if (fmm) push(cref | REF_FORCED, fmm);
                            }
                            if (STATS && (an || fm)) ++nvis;
                            const double wm = take ? (kind == QK_LEAF ? 1.0 : (double)nd.ccnt[c]) : 0.0;
                            const double Q = recip_bh(D1);
                            const double mult = wm * Q;
                            const double sc = mult * Q;
                            fx = __fma_rn(sc, dx, fx);
                            fy = __fma_rn(sc, dy, fy);
                            zs += mult;
                        } else if (kind == QK_MULTI) {   // a leaf of ccnt copies: 0 if it is the query's point
                            if (own && (an || fm) && !(nd.ccx[c] == qx && nd.ccy[c] == qy)) {
                                if (STATS) ++nvis;
                                cell_force(dx, dy, __fma_rn(dx, dx, dy * dy), nd.ccnt[c], fx, fy, zs);
                            }
                        } else if (own) {                // a key-tie group: every point directly
                            for (int p = c0; p <= c1; ++p) {
                                const double2 pp = pos[p];
                                if (an || fm) { if (STATS) ++nvis; leaf_force(qx, qy, pp.x, pp.y, fx, fy, zs); }
                            }
                        }
                    }
                    continue;
                }
            }
            // all-open / near-exact tests (per lane) -> the subtree's exact leaf sum;
            // both tests on every lane, their masks straight from the compares
            // (tile_test's branch and a ballot of the combined bool cost more).
            // Lane state is kept as scalar masks (amask: lanes that go on to the
            // children), turned into lane predicates by inverse ballots, which
            // read the mask's SGPRs directly: no VALU per conversion.
            uint64_t tm = 0;
            uint64_t amask = msk_s;
            const int nflags = __builtin_amdgcn_readfirstlane(nd.nch);   // the record is the wave's
            if (nflags & QNCH_TILE) {
                const double cdx = qx - nd.cx, cdy = qy - nd.cy;
                const double ex = __fma_rn(1e-15, qmag, nd.ex);
                const double dxm = fmax(fabs(qx - nd.bx0), fabs(qx - nd.bx1)) + ex;
                const double dym = fmax(fabs(qy - nd.by0), fabs(qy - nd.by1)) + ex;
                // (FMA forms: the bounds carry 1e-9 / 1.1e-12 relative margins)
                tm = msk_s & (__builtin_amdgcn_ballot_w64(__fma_rn(cdx, cdx, cdy * cdy) <= nd.rball) |
                              __builtin_amdgcn_ballot_w64(__fma_rn(dxm, dxm, dym * dym) <= nd.hmin));
            }
            if (!PART && tm && task && ntt == tcap) {   // a task's tile page is full (or none yet): the next one
                if (page >= 0 && lane == 0) { sv.pg_n[page] = ntt; sv.pg_grp[page] = (int32_t)grp; }
                int p = 0;
                if (lane == 0) p = atomicAdd(&sv.ctl[SP_PAGES], 1);
                p = __builtin_amdgcn_readfirstlane(p);
                ntt = 0;
                if (p < sv.pg_cap) {
                    page = p;
                    tdst = sv.pg_tiles + (int64_t)p * SP_PAGE;
                    tcap = SP_PAGE;
                } else {   // no page left: the lanes keep traversing (the reference's path; flagged)
                    page = -1;
                    tcap = 0;
                    if (lane == 0) atomicOr(&sv.ctl[SP_OVF], 2);
                }
            }
            if (tm && ntt < tcap) {
                // The wave records (subtree, lanes) for tile_apply, or, when its
                // list is full, the lanes keep traversing (the reference's path).
                // The range holds whole equal-key runs, so either all of the
                // query's exact duplicates (itself included) are in it or none
                // is; they add exactly 1 each to z in the leaf sum: taken off here.
                const int a = __builtin_amdgcn_readfirstlane(nd.first), b = __builtin_amdgcn_readfirstlane(nd.last);
                if (lane == 0) {
                    TileTask tt; tt.ref = ref; tt.first = a; tt.last = b; tt.pad = nd.cnt; tt.mask = tm;
                    tdst[ntt] = tt;
                }
                ++ntt;
                ntilepts += b - a + 1;
                if (STATS) wtile += (unsigned long long)(b - a + 1);
                if (__builtin_amdgcn_inverse_ballot_w64(tm)) {
                    if (STATS) nvis += (unsigned long long)(b - a + 1);
                    if (s >= a && s <= b) zs -= (double)ndup;
                }
                amask = msk_s & ~tm;
            }
            if (amask == 0) continue;
            act = __builtin_amdgcn_inverse_ballot_w64(amask);
            // the opened cell's quad children, from its record
            const int nch = nflags & 0xff;
            if (STATS) { wslots += (unsigned long long)nch; if (act) nevals += (unsigned long long)nch; }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (c >= nch) break;
                const int kind = (nflags >> (QNCH_KIND + 2 * c)) & 3;   // uniform: scalar branches
                if (kind == QK_CELL || kind == QK_LEAF) {
                    // A leaf (cumSize 1, com = the point) always interacts, zero if
                    // it is the query's own point (x - y == 0 iff x == y).  A cell is
                    // summarised when ch / D < theta (QACC_BAND: two compares of
                    // D1 = 1 + D against the record's bounds, the exact quotient only
                    // inside the band; at D = 0 never).  wm = the term's multiplicity
                    // where taken, else 0: a zero term leaves the sums bit-equal.
                    // Only wm is computed per kind (uniform branch), so the
                    // accumulators stay in place.
                    if (STATS && act) ++nvis;
                    const double dx = qx - nd.ccx[c], dy = qy - nd.ccy[c];
                    const double D1 = __fma_rn(dx, dx, __fma_rn(dy, dy, 1.0));   // 1 + D, the term's denominator
                    uint64_t takem;
                    double wm;
                    if (kind == QK_LEAF) {
                        takem = amask & ~(__builtin_amdgcn_ballot_w64(dx == 0.0) & __builtin_amdgcn_ballot_w64(dy == 0.0));
                        wm = __builtin_amdgcn_inverse_ballot_w64(takem) ? 1.0 : 0.0;
                    } else {
                        // the masks straight from the compares (scalar: a
                        // ballot of a combined bool costs two VALU per child)
                        uint64_t accm = __builtin_amdgcn_ballot_w64(D1 > nd.ca[c]);
                        const uint64_t band = amask & ~accm & ~__builtin_amdgcn_ballot_w64(D1 < nd.cb[c]);
                        if (band) {   // rare: inside the band the exact IEEE quotient decides
                            bool acc = false;
                            if (__builtin_amdgcn_inverse_ballot_w64(band))
                                acc = qrec_child_h(nodes, ref, nd.cref[c], virt) /
                                          __dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)) < theta;
                            accm |= band & __builtin_amdgcn_ballot_w64(acc);
                        }
                        takem = amask & accm;
                        wm = (double)(__builtin_amdgcn_inverse_ballot_w64(takem) ? nd.ccnt[c] : 0);
                        const uint64_t om = amask & ~accm;
                        if (om) {
                            if (PART && sp >= STACK) {
                                if (lane == 0) plim[2] = 1;
                            } else {
                                if (lane == 0) { L.sref[w][sp] = nd.cref[c]; L.smask[w][sp] = om; }
                                ++sp;
                            }
                        }
                    }
                    const double Q = recip_bh(D1);
                    const double mult = wm * Q;
                    const double sc = mult * Q;
                    fx = __fma_rn(sc, dx, fx);
                    fy = __fma_rn(sc, dy, fy);
                    zs += mult;
                    if (STATS) {   // children every active lane takes (summarised cell or leaf), full wave or not
                        if (takem == amask) {
                            if (amask == __ballot(valid)) ++wfull; else ++wpart;
                        }
                    }
                }
            }
            // duplicate kinds (rare), after the others: out of the main loop,
            // whose accumulators then stay in place
            if (__builtin_expect((nflags & (0xAA << QNCH_KIND)) != 0, 0)) {
                for (int c = 0; c < nch; ++c) {
                    const int kind = (nflags >> (QNCH_KIND + 2 * c)) & 3;
                    if (kind == QK_MULTI) {   // a leaf of ccnt copies: 0 if it is the query's point
                        if (act && !(nd.ccx[c] == qx && nd.ccy[c] == qy)) {
                            if (STATS) ++nvis;
                            const double dx = qx - nd.ccx[c], dy = qy - nd.ccy[c];
                            cell_force(dx, dy, __fma_rn(dx, dx, dy * dy), nd.ccnt[c], fx, fy, zs);
                        }
                    } else if (kind == QK_TIE) {
                        const BHNode &tn = nodes[__builtin_amdgcn_readfirstlane(nd.cref[c])];
                        if (STATS) wtie += (unsigned long long)(tn.last - tn.first + 1);
                        for (int p = tn.first; p <= tn.last; ++p) {
                            const double2 pp = pos[p];
                            if (act) { if (STATS) ++nvis; leaf_force(qx, qy, pp.x, pp.y, fx, fy, zs); }
                        }
                    }
                }
            }
        }
    }
    if (!PART && spe >= 0) sp_write(sv, L, w, spe, spt, sp, (int32_t)grp);
    if (!task) {
        if (valid) {
            F[s] = make_double2(fx, fy);
            Z[s] = zs;
        }
        if (lane == 0) {
            ttask_n[wid] = ntt;
            tcost[wid] = ntilepts + 16 * ntt;
            // (an add: the group's tasks add their pops too, possibly before this)
            if (spill_on) atomicAdd(&wcost[wid], npops + (ntilepts >> 6));
            else wcost[wid] = npops + (ntilepts >> 6);
        }
        if (TSNE_ST_TRAV && !PART && stv.ctl && ntt > 0 &&
            ntilepts + 16 * ntt <= (stv.maxcost > 0 ? stv.maxcost : stv.ctl[ST_W])) {
            // hand the list to the streaming consumers: every store of this
            // wave done, its claim word, an agent-scope release, then the item
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) {
                __hip_atomic_store(st_claims(stv.ctl) + wid, stv.gen << 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const int32_t k = atomicAdd(&stv.ctl[ST_TAIL], 1);
                __hip_atomic_store(st_items(stv.ctl, stv.cap) + k,
                                   ((unsigned long long)(uint32_t)stv.gen << 32) | (unsigned long long)wid,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    } else {
        if (page >= 0 && lane == 0) { sv.pg_n[page] = ntt; sv.pg_grp[page] = (int32_t)grp; }
        if (valid && (fx != 0.0 || fy != 0.0 || zs != 0.0)) {
            unsigned long long *a = sv.acc + 6 * s;
            fxp_add(a, fx);
            fxp_add(a + 2, fy);
            fxp_add(a + 4, zs);
        }
        if (lane == 0) atomicAdd(&wcost[grp], npops + (ntilepts >> 6));
    }
    if (COST && bcost) {   // cost of this walk into its queries' 256-query buckets
        // the walk's own run time (shader clock / 64; the slices only move work
        // between ranks, every query's sums are unchanged)
        const unsigned long long c = ((unsigned long long)(clock64() - t_start) >> 6) + 1;
        if (cost_lab) {   // by label: an equal share into each query's label bucket
            if (valid) atomicAdd(&bcost[cost_lab[s] >> 8], (c + 63) >> 6);
        } else {
            const int64_t sf = wave_min(valid ? s : ((int64_t)1 << 62));
            if (lane == 0) atomicAdd(&bcost[sf >> 8], c);
        }
    }
    if (STATS && visits) {   // [0] reference-equivalent node evaluations, [3] wave-level pops,
                             // [4] wave-level tile points, [5] lane child evaluations, [6] wave
                             // child slots, [7..9] heaviest wave ([1], [2]: tile_apply), [32] tasks run
        const unsigned long long tv = wave_sum(nvis), te = wave_sum(nevals);
        if (lane == 0) {
            atomicAdd(visits, tv);
            atomicAdd(visits + 3, wpops);
            atomicAdd(visits + 4, wtile);
            atomicAdd(visits + 5, te);
            atomicAdd(visits + 6, wslots);
            atomicMax(visits + 7, wpops + wtile / 16);   // heaviest wave (pops + tile points/16)
            atomicMax(visits + 8, wpops);
            atomicMax(visits + 9, wtile);
            atomicAdd(visits + 13, wfull);
            atomicAdd(visits + 14, wpart);
            const unsigned long long w_end = wall_clock64();   // [15] longest wave, [16] ~first start,
            atomicMax(visits + 15, w_end - w_start);            // [17] last end, [18] sum of wave times
            atomicMax(visits + 16, ~0ull - w_start);
            atomicMax(visits + 17, w_end);
            atomicAdd(visits + 18, w_end - w_start);
            if (task) atomicAdd(visits + 32, 1ull);
            atomicAdd(visits + 37, (unsigned long long)(clock64() - t_start));   // shader cycles (wave_mhz)
            if (!TASK) wave_log_put(nv.wlog, w_start, w_end, 0);
            // the slowest wave's own counts (ticks << 24 | count: the max keeps that wave's)
            const unsigned long long tk = min(w_end - w_start, (1ull << 40) - 1) << 24, cm = (1ull << 24) - 1;
            atomicMax(visits + 33, tk | min(wpops, cm));
            atomicMax(visits + 34, tk | min(wtie, cm));
            atomicMax(visits + 35, tk | min(wtile, cm));
            atomicMax(visits + 36, tk | min(wslots, cm));
        }
    }
    // TASK: the next one of the level (never waiting for one to appear)
    if (!TASK || !sp_next(sv, L, w, grp, tsp)) break;
    }
}

// The heavy groups of the next traversal, from this one's costs (one
// workgroup): a group's cost is its wave's (pops + tile points / 64), or for a
// group that ran narrow 2 x its heaviest narrow wave's (hysteresis: the
// narrow waves each walk a part of the 64-query union).  Heavy: cost >= fac x
// the mean over all groups (and >= NARROW_MIN); at most hmax of them, listed
// in group order.  nflag[g] = heavy slot + 1 or 0.
// Fill mode (hfill > 0: too few 64-query waves to occupy the chip, e.g. one
// rank's share of the queries): also the hfill most costly groups, whatever
// the factor -- the threshold is lowered to the cost bucket (4 per doubling,
// plan_bucket) where the count from the top reaches hfill.
constexpr int32_t NARROW_MIN = 32;
__global__ __launch_bounds__(1024) void narrow_select(int32_t *__restrict__ wcost, int64_t waves,
                                                      int32_t *__restrict__ nflag, const int32_t *__restrict__ ncost,
                                                      int32_t *__restrict__ hlist, int32_t *__restrict__ hcount,
                                                      int64_t hmax, double fac, int64_t hfill,
                                                      int32_t *__restrict__ border, double ffac) {
    __shared__ unsigned long long red[16];
    __shared__ int32_t wtot[16];
    __shared__ int32_t hist[PLAN_BUCKETS];
    __shared__ int32_t sbucket;
    __shared__ double sthr;
    const int t = threadIdx.x, lane = lane_id(), w = t >> 6;
    if (t < PLAN_BUCKETS) hist[t] = 0;
    __syncthreads();
    unsigned long long acc = 0;
    for (int64_t g0 = (int64_t)w * 64; g0 < waves; g0 += 1024) {
        const int64_t g = g0 + lane;
        int32_t c = 0;
        if (g < waves) {
            c = wcost[g];
            const int32_t f = nflag[g];
            if (f > 0) {
                int32_t mx = 0;
                for (int p = 0; p < NPARTS; ++p) mx = max(mx, ncost[(int64_t)(f - 1) * NPARTS + p]);
                c = 2 * mx;
                wcost[g] = c;
            }
            acc += (unsigned long long)max(c, 0);
        }
        if (hfill > 0) (void)wave_bucket_add(hist, plan_bucket(c), g < waves);
    }
    acc = wave_sum(acc);
    if (lane == 0) red[w] = acc;
    __syncthreads();
    if (t == 0) {
        unsigned long long total = 0;
        for (int j = 0; j < 16; ++j) total += red[j];
        sthr = fmax((double)NARROW_MIN, fac * (double)total / (double)max<int64_t>(waves, 1));
        // fill mode: buckets >= sbucket hold at most hfill groups
        int64_t run = 0;
        int b = PLAN_BUCKETS;
        if (hfill > 0)
            while (b > 1 && run + hist[b - 1] <= hfill) run += hist[--b];
        sbucket = b;
    }
    __syncthreads();
    const double thr = sthr;
    const int bmin = sbucket;
    int32_t base = 0;
    for (int64_t g0 = 0; g0 < waves; g0 += 1024) {
        const int64_t g = g0 + t;
        bool hv = false;
        if (fac > 0.0 && g < waves) {
            const int32_t c = wcost[g];
            hv = c >= NARROW_MIN && ((double)c >= thr || plan_bucket(c) >= bmin);
        }
        const uint64_t b = __ballot(hv);
        if (lane == 0) wtot[w] = (int32_t)__popcll(b);
        __syncthreads();
        int32_t off = base, tot = 0;
        for (int j = 0; j < 16; ++j) {
            if (j < w) off += wtot[j];
            tot += wtot[j];
        }
        const int32_t slot = off + (int32_t)__popcll(b & lanemask_lt());
        if (g < waves) {
            const bool take = hv && slot < hmax;
            nflag[g] = take ? slot + 1 : 0;
            if (take) hlist[slot] = (int32_t)g;
        }
        base += tot;
        __syncthreads();
    }
    if (t == 0) *hcount = (int32_t)min<int64_t>(base, hmax);
    if (!border) return;
    // The next traversal's block order (option trav_front): the 64-query
    // workgroups whose heaviest wave (narrow groups excluded: they leave at
    // once) cost >= ffac x the mean first, then the rest, each in Morton order
    __syncthreads();
    const int64_t nb = (waves + TRAV_WPB - 1) / TRAV_WPB;
    const double fthr = ffac * (double)sthr / fmax(fac, 1e-300);   // sthr = fac x mean (or NARROW_MIN)
    int32_t pos = 0;
    for (int pass = 0; pass < 2; ++pass) {
        for (int64_t b0 = 0; b0 < nb; b0 += 1024) {
            const int64_t b = b0 + t;
            bool in = false;
            if (b < nb) {
                int32_t c = 0;
                for (int k = 0; k < TRAV_WPB; ++k) {
                    const int64_t g = b * TRAV_WPB + k;
                    if (g < waves && nflag[g] == 0) c = max(c, wcost[g]);
                }
                const bool heavy = (double)c >= fthr;
                in = pass == 0 ? heavy : !heavy;
            }
            const uint64_t m = __ballot(in);
            if (lane == 0) wtot[w] = (int32_t)__popcll(m);
            __syncthreads();
            int32_t off = pos, tot = 0;
            for (int j = 0; j < 16; ++j) {
                if (j < w) off += wtot[j];
                tot += wtot[j];
            }
            if (in) border[off + (int32_t)__popcll(m & lanemask_lt())] = (int32_t)b;
            pos += tot;
            __syncthreads();
        }
    }
}

// Option trav_front_cur: the traversal's workgroup order from this build's
// predicted wave costs (gather_sorted): workgroups whose heaviest predicted
// 64-query wave (narrow groups excluded) is >= ffac x the mean first, the rest
// after, each in Morton order.  One workgroup, on the second stream during the build.
__global__ __launch_bounds__(1024) void trav_order_cur(const int32_t *__restrict__ pred,
                                                       const int32_t *__restrict__ nflag, int64_t waves, double ffac,
                                                       int32_t *__restrict__ border) {
    __shared__ unsigned long long red[16];
    __shared__ int32_t wtot[16];
    __shared__ double sthr;
    const int t = threadIdx.x, lane = lane_id(), w = t >> 6;
    unsigned long long acc = 0, cnt = 0;
    for (int64_t g = t; g < waves; g += 1024)
        if (!(nflag && nflag[g])) { acc += (unsigned long long)max(pred[g], 0); ++cnt; }
    acc = wave_sum(acc);
    cnt = wave_sum(cnt);
    if (lane == 0) { red[w] = acc; wtot[w] = (int32_t)cnt; }
    __syncthreads();
    if (t == 0) {
        unsigned long long a = 0, c = 0;
        for (int j = 0; j < 16; ++j) { a += red[j]; c += (unsigned long long)wtot[j]; }
        sthr = ffac * (double)a / (double)max(1ull, c);
    }
    __syncthreads();
    const double thr = sthr;
    const int64_t nb = (waves + TRAV_WPB - 1) / TRAV_WPB;
    int32_t pos = 0;
    for (int pass = 0; pass < 2; ++pass) {
        for (int64_t b0 = 0; b0 < nb; b0 += 1024) {
            const int64_t b = b0 + t;
            bool in = false;
            if (b < nb) {
                int32_t c = 0;
                for (int k = 0; k < TRAV_WPB; ++k) {
                    const int64_t g = b * TRAV_WPB + k;
                    if (g < waves && !(nflag && nflag[g])) c = max(c, pred[g]);
                }
                const bool heavy = c > 0 && (double)c >= thr;
                in = pass == 0 ? heavy : !heavy;
            }
            const uint64_t m = __ballot(in);
            __syncthreads();
            if (lane == 0) wtot[w] = (int32_t)__popcll(m);
            __syncthreads();
            int32_t off = pos, tot = 0;
            for (int j = 0; j < 16; ++j) {
                if (j < w) off += wtot[j];
                tot += wtot[j];
            }
            if (in) border[off + (int32_t)__popcll(m & lanemask_lt())] = (int32_t)b;
            pos += tot;
        }
    }
}

// The traversal waves' tiles, in recording order: one wave per traversal
// wave (same 64 queries).  For every (subtree, lanes) task each lane of the
// mask takes the subtree's exact leaf sum either from its moments -- when the
// series' truncation bound holds and moments were built this iteration, the
// lane appends the node to its own moment list, evaluated lane-parallel by
// moment_apply -- or densely: the points staged through LDS 64 at a time (one
// coalesced dwordx4 load per lane, the next chunk prefetched into registers)
// and read back as wave-uniform broadcasts.  Lanes whose bound holds are
// counted for the next iteration's moment gate.
// MODE 1 (PAGE): the spill tasks' tile pages instead (one wave per page, its
// group's 64 queries; moments evaluated in place; sums into the fixed-point
// accumulators, see "Spill").  MODE 2 (STREAM): the streaming consumer (see
// "Tile streaming"): persistent waves taking the handed-over lists, moments
// recorded per consumer lane and evaluated after its tiles, F += D + M.  MODE 0 skips the
// streamed waves' lists (st_streamed: their list length and tile cost).
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void tile_apply(
    const double2 *__restrict__ pos, const BHNode *__restrict__ nodes, const TileTask *__restrict__ ttask,
    const int32_t *__restrict__ ttask_n, int64_t g0, int64_t g1, const int32_t *__restrict__ qlist,
    int32_t *__restrict__ mom_flag, double mom_tol, int32_t *__restrict__ mtask, int32_t *__restrict__ mtask_n,
    double2 *__restrict__ F, double *__restrict__ Z, unsigned long long *__restrict__ visits,
    const int32_t *__restrict__ torder, ChunkView cv, const double *__restrict__ mom, SpillView sv,
    StreamView stv, const int32_t *__restrict__ tcost) {
    constexpr bool PAGE = MODE == 1, STREAM = MODE == 2;
    __shared__ double2 tbuf[4][64];
    __shared__ int smark[4][64];
    __shared__ int2 srng[4][64];
    constexpr float LW_COST = 1.0f;   // lane-wise cost per point relative to a sweep slot (gathers, refills;
                                      // 1.6 before the lane-wise loop lost its accumulator copies, round 5)
    const int lane = lane_id(), w = threadIdx.x >> 6;
    int64_t wid, qw;
    int tb, nt;
    const TileTask *mytt;
    // PAGE: pages blockIdx.x * 4 + w, + 4 gridDim.x, ... (the loop's end below)
    for (int64_t pit = (int64_t)blockIdx.x * 4 + w;; pit += (int64_t)gridDim.x * 4) {
    if (PAGE) {   // page wid of the spill tasks
        wid = pit;
        if (wid >= (int64_t)min(sv.ctl[SP_PAGES], sv.pg_cap)) return;
        qw = sv.pg_grp[wid];
        mytt = sv.pg_tiles + wid * SP_PAGE;
        tb = 0;
        nt = sv.pg_n[wid];
        if (nt == 0) return;
    } else if (STREAM) {   // the next handed-over list (see "Tile streaming")
        int32_t k = 0;
        if (lane == 0) k = atomicAdd(&stv.ctl[ST_HEAD], 1);
        k = __builtin_amdgcn_readfirstlane(k);
        int64_t got = -1;
        if (k < stv.total) {
            for (int poll = 0; poll < stv.wait; ++poll) {
                unsigned long long v = 0;
                if (lane == 0)
                    v = __hip_atomic_load(st_items(stv.ctl, stv.cap) + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t vhi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
                const uint32_t vlo = __builtin_amdgcn_readfirstlane((uint32_t)v);
                if (vhi == (uint32_t)stv.gen) { got = vlo; break; }
                __builtin_amdgcn_s_sleep(16);
            }
        }
        if (got < 0) return;   // nothing more for now: the slot path takes what comes later
        int32_t own = 0;
        if (lane == 0) own = st_claim(st_claims(stv.ctl), got, stv.gen, 2);
        if (__builtin_amdgcn_readfirstlane(own) != 2) continue;   // the slot path has it
        // the producer's release pairs with this acquire: its list, F and Z fresh
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wid = k;   // entries k x 64 + lane of the consumers' partial sums and moment lists
        qw = got;
        mytt = ttask + qw * TILE_CAP;
        tb = 0;
        nt = vec_load(ttask_n + qw);
        if (lane == 0) atomicAdd(&stv.ctl[ST_CUM], 1);
    } else {
        const int64_t blk = torder ? (int64_t)torder[blockIdx.x] : (int64_t)blockIdx.x;
        wid = blk * 4 + w;
        qw = wid;   // chunks: slot wid = chunk c of C of traversal wave qw's tile list
        int ch = 0, C = 1;
        if (cv.slot_w) {
            if (wid >= *cv.nslots) return;
            qw = cv.slot_w[wid];
            const int32_t v = cv.slot_c[wid];
            ch = v & 0xffff;
            C = v >> 16;
        }
        if (g0 + qw * 64 >= g1) return;
        mytt = ttask + qw * TILE_CAP;
        // (a list a streaming consumer claimed first: nothing here, zero partials)
        int ntw = ttask_n[qw];
        if (stv.ctl) {
            int32_t own = 0;
            if (lane == 0) own = st_claim(st_claims(stv.ctl), qw, stv.gen, 1);
            if (__builtin_amdgcn_readfirstlane(own) == 2) ntw = 0;
        }
        tb = (int)((int64_t)ntw * ch / C);
        nt = (int)((int64_t)ntw * (ch + 1) / C);
    }
    const int64_t kq = g0 + qw * 64 + lane;
    const bool valid = kq < g1;
    const int64_t s = valid ? (qlist ? (int64_t)qlist[kq] : kq) : -1;
    const int64_t e = STREAM || cv.slot_w ? wid * 64 + lane : s;   // moment list / partial-sum entry
    if (MODE == 0 && nt == tb) {
        if (valid) {
            mtask_n[e] = 0;
            if (cv.slot_w) { cv.Fp[e] = make_double2(0.0, 0.0); cv.Zp[e] = 0.0; }
        }
        return;
    }
    double qx = 0.0, qy = 0.0;
    if (valid) { const double2 q = pos[s]; qx = q.x; qy = q.y; }
    const bool mom_on = mom_flag[0] != 0;
    const unsigned long long w_start = visits ? wall_clock64() : 0;
    double fx = 0.0, fy = 0.0, zs = 0.0;
    int nwant = 0, ntask = 0;
    unsigned long long ndense = 0;
    unsigned long long wt_tasks = 0, wt_dense_pts = 0, wt_momchk = 0;   // wave-level diagnostics
    // per dense path (lane-wise, packed sweep, query-major, staged sweep): wave
    // steps (pair slots the wave issues) and this lane's useful pairs
    unsigned long long ps_steps[4] = {0, 0, 0, 0}, ps_pairs[4] = {0, 0, 0, 0};
    double2 *buf = tbuf[w];
    int masked_until = tb;   // tiles before this one take the masked sweep
    for (int t = tb; t < nt;) {
        const TileTask tt = STREAM ? vec_load(mytt + t) : mytt[t];
        if (t >= masked_until && tt.last - tt.first + 1 < MOM_MIN_POINTS) {
            // Lane-wise window: the run of <= 64 consecutive small tiles
            // starting at t.  Each lane walks only the points of ITS tiles
            // (its bits of the 64 masks, transposed by 64 ballots), gathering
            // them itself, so a sweep costs the busiest lane's point count
            // instead of every tile point with most lanes masked off (the
            // masks of small tiles hold ~1/4 of the lanes in the mid phase).
            // Per lane the order is fixed (tile order, then point order).
            const int ti = t + lane;
            bool sm = false;
            int a_i = 0, b_i = -1;
            uint64_t m_i = 0;
            if (ti < nt) {
                const TileTask h = mytt[ti];
                if (h.last - h.first + 1 < MOM_MIN_POINTS) { sm = true; a_i = h.first; b_i = h.last; m_i = h.mask; }
            }
            const uint64_t nsm = ~__ballot(sm);
            const int wn = nsm ? __ffsll((long long)nsm) - 1 : 64;   // >= 1: tile t is small
            if (lane >= wn) m_i = 0;
            // 64 x 64 bit transpose (row i = tile t + i's lane mask): six
            // butterfly stages swapping the off-diagonal blocks of halving size
            uint64_t W = m_i;
#pragma unroll
            for (int st = 0; st < 6; ++st) {
                const int j = 32 >> st;
                const uint64_t lo = st == 0 ? 0x00000000FFFFFFFFull : st == 1 ? 0x0000FFFF0000FFFFull
                                  : st == 2 ? 0x00FF00FF00FF00FFull : st == 3 ? 0x0F0F0F0F0F0F0F0Full
                                  : st == 4 ? 0x3333333333333333ull : 0x5555555555555555ull;
                const uint32_t ylo = __shfl_xor((uint32_t)W, j, 64), yhi = __shfl_xor((uint32_t)(W >> 32), j, 64);
                const uint64_t y = ((uint64_t)yhi << 32) | ylo;
                W = (lane & j) ? ((W & ~lo) | ((y & ~lo) >> j)) : ((W & lo) | ((y & lo) << j));
            }
            // W bit i: tile t + i is one of mine.  Lane-wise costs the busiest
            // lane's points, the masked 64-slot sweep every point: take the
            // cheaper (LW_COST: lane-wise cost per point relative to a sweep
            // slot, gathers and refills included), the sweep for the whole window.
            const int cnt_i = b_i - a_i + 1;
            __builtin_amdgcn_wave_barrier();
            srng[w][lane] = make_int2(a_i, b_i);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            int cl = 0;
            for (uint64_t wb = W; wb; wb &= wb - 1) {
                const int2 r = srng[w][__ffsll((long long)wb) - 1];
                cl += r.y - r.x + 1;
            }
            const int cmax = wave_max(cl), ctot = wave_sum(lane < wn ? cnt_i : 0);
            if ((float)cmax * LW_COST >= (float)ctot) {
                masked_until = t + wn;
                goto masked;
            }
            double ux = 0.0, uy = 0.0, uz = 0.0;
            int nmine = 0, nit = 0;
            // a divergent do-while per lane (two points of one tile per step,
            // the second masked at a tile's odd end): the accumulators are
            // updated in place, not copied at the merges of a wave-uniform loop
            if (W) {
                int i = __ffsll((long long)W) - 1;
                W &= W - 1;
                int2 r = srng[w][i];
                int p = r.x, last = r.y;
                bool more;
                do {
                    const bool two = p < last;
                    const double2 p0 = pos[p];
                    const double2 p1 = pos[two ? p + 1 : p];
                    pair_force(qx, qy, p0.x, p0.y, ux, uy, uz);
                    pair_force_m(two, qx, qy, p1.x, p1.y, ux, uy, uz);
                    nmine += two ? 2 : 1;
                    ++nit;
                    p += 2;
                    if (p > last && W) {
                        i = __ffsll((long long)W) - 1;
                        W &= W - 1;
                        r = srng[w][i];
                        p = r.x; last = r.y;
                    }
                    more = p <= last;
                } while (more);
            }
            if (visits) ps_steps[0] += 2ull * (unsigned long long)wave_max(nit);
            __builtin_amdgcn_wave_barrier();
            fx += ux; fy += uy; zs += uz;
            ndense += (unsigned long long)nmine;
            if (visits) {
                ps_pairs[0] += (unsigned long long)nmine;
                wt_tasks += (unsigned long long)wn;
                wt_dense_pts += (unsigned long long)wave_sum(lane < wn ? b_i - a_i + 1 : 0);
            }
            t += wn;
            continue;
        }
    masked:
        if (tt.last - tt.first + 1 < MOM_MIN_POINTS) {
            // Packed round: the run of consecutive small tiles (no moments below
            // MOM_MIN_POINTS) whose points fit 64 slots is staged as one batch of
            // (point, tile lane mask) and swept once, each lane taking the points
            // of its own tiles -- one staging round per <= 64 points instead of
            // one per tile (tiles average ~9 points in the mid phase).
            const int ti = t + lane;
            int c_i = 1 << 20, a_i = 0;
            uint64_t m_i = 0;
            if (ti < nt) {
                const TileTask h = mytt[ti];
                const int c = h.last - h.first + 1;
                if (c < MOM_MIN_POINTS) { c_i = c; a_i = h.first; m_i = h.mask; }
            }
            int S = c_i;   // inclusive prefix of the counts
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int v = __shfl_up(S, o, 64);
                if (lane >= o) S += v;
            }
            const int mtake = __popcll(__ballot(S <= 64));   // >= 1: tile t itself fits
            const int total = __shfl(S, mtake - 1, 64);
            __builtin_amdgcn_wave_barrier();
            smark[w][lane] = -1;
            __builtin_amdgcn_wave_barrier();
            if (lane < mtake) smark[w][S - c_i] = lane;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            int own = smark[w][lane];   // slot -> tile: running max of the start markers
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int v = __shfl_up(own, o, 64);
                if (lane >= o) own = max(own, v);
            }
            const int st = __shfl(S - c_i, own, 64), fa = __shfl(a_i, own, 64);
            const uint64_t mk = __shfl(m_i, own, 64);
            __builtin_amdgcn_wave_barrier();
            buf[lane] = lane < total ? pos[fa + lane - st] : make_double2(0.0, 0.0);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
            double ux = 0.0, uy = 0.0, uz = 0.0;
            int nmine = 0;
            // lane-wise over the staged slots: each lane walks only ITS slots
            // (the round's 64 slot masks transposed), two at a time, so the
            // round costs its busiest lane's slots instead of all of them;
            // a lane's order is still slot order (the same sums as the sweep)
            uint64_t M = lane < total ? mk : 0ull;
#pragma unroll
            for (int st2 = 0; st2 < 6; ++st2) {
                const int j = 32 >> st2;
                const uint64_t lo = st2 == 0 ? 0x00000000FFFFFFFFull : st2 == 1 ? 0x0000FFFF0000FFFFull
                                  : st2 == 2 ? 0x00FF00FF00FF00FFull : st2 == 3 ? 0x0F0F0F0F0F0F0F0Full
                                  : st2 == 4 ? 0x3333333333333333ull : 0x5555555555555555ull;
                const uint32_t ylo = __shfl_xor((uint32_t)M, j, 64), yhi = __shfl_xor((uint32_t)(M >> 32), j, 64);
                const uint64_t y = ((uint64_t)yhi << 32) | ylo;
                M = (lane & j) ? ((M & ~lo) | ((y & ~lo) >> j)) : ((M & lo) | ((y & lo) << j));
            }
            // a divergent do-while per lane, the next slot's point read before
            // the current one is summed: the accumulators are updated in place
            // (a wave-uniform loop with an `if (M)` body made the compiler copy
            // them at every merge -- ~20 moves per two pairs)
            if (M) {
                int j = __ffsll((long long)M) - 1;
                M &= M - 1;
                double2 pp = buf[j];
                bool more;
                do {
                    more = M != 0ull;
                    j = more ? __ffsll((long long)M) - 1 : j;
                    M &= M - 1;
                    const double2 pn = buf[j];
                    pair_force(qx, qy, pp.x, pp.y, ux, uy, uz);
                    if (visits) ++nmine;
                    pp = pn;
                } while (more);
            }
            if (visits) ps_steps[1] += (unsigned long long)wave_max(nmine);
            __builtin_amdgcn_wave_barrier();
            fx += ux; fy += uy; zs += uz;
            ndense += (unsigned long long)nmine;
            if (visits) {
                wt_tasks += (unsigned long long)mtake; wt_dense_pts += (unsigned long long)total;
                ps_pairs[1] += (unsigned long long)nmine;
            }
            t += mtake;
            continue;
        }
        ++t;
        const int ref = __builtin_amdgcn_readfirstlane(tt.ref);
        const int a = __builtin_amdgcn_readfirstlane(tt.first), b = __builtin_amdgcn_readfirstlane(tt.last);
        const int cnt = __builtin_amdgcn_readfirstlane(tt.pad);
        const bool mine = (tt.mask >> lane) & 1ull;
        bool usem = false;
        if (mine && cnt >= MOM_MIN_POINTS && (PAGE || ntask < MOM_TASKS)) {
            const BHNode &nd = nodes[ref];
            if (moment_ok(nd.bx0, nd.bx1, nd.by0, nd.by1, qx, qy, mom_tol)) {
                ++nwant;
                if (mom_on) {
                    usem = true;
                    if (PAGE) {   // evaluated here (no per-query list for pages)
                        double cx, cy, R;
                        box_centre(nd, cx, cy, R);
                        moment_eval(mom + (int64_t)ref * MOM_K, qx - cx, qy - cy, fx, fy, zs);
                        ++ntask;
                    } else {
                        mtask[e * MOM_TASKS + ntask++] = ref;
                    }
                }
            }
        }
        const bool dense = mine && !usem;
        const uint64_t dm = __ballot(dense);
        const int kq = __popcll(dm), cnt_t = b - a + 1;
        if (visits) {
            ++wt_tasks;
            if (dm) wt_dense_pts += (unsigned long long)cnt_t;
            if (cnt >= MOM_MIN_POINTS && (tt.mask != 0)) ++wt_momchk;
        }
        if (dm && kq * ((cnt_t + 63) / 64 + 6) < cnt_t) {
            // Few lanes, many points: query-major.  For each dense lane j in
            // turn, all 64 lanes split the tile's points and a butterfly sum
            // (fixed order: deterministic) hands lane j its total -- kq passes
            // of cnt/64 pairs instead of cnt pairs with most lanes masked off.
            uint64_t rem = dm;
            while (rem) {
                const int j = __ffsll((long long)rem) - 1;
                rem &= rem - 1;
                const double qjx = __shfl(qx, j, 64), qjy = __shfl(qy, j, 64);
                double ux = 0.0, uy = 0.0, uz = 0.0;
                int p = a + lane;
                for (; p + 64 <= b; p += 128) {
                    const double2 p0 = pos[p], p1 = pos[p + 64];
                    pair_force(qjx, qjy, p0.x, p0.y, ux, uy, uz);
                    pair_force(qjx, qjy, p1.x, p1.y, ux, uy, uz);
                }
                if (p <= b) {
                    const double2 p0 = pos[p];
                    pair_force(qjx, qjy, p0.x, p0.y, ux, uy, uz);
                }
                ux = wave_sum(ux); uy = wave_sum(uy); uz = wave_sum(uz);
                if (lane == j) { fx += ux; fy += uy; zs += uz; ndense += (unsigned long long)cnt_t; }
                if (visits) {
                    ps_steps[2] += (unsigned long long)((cnt_t + 63) / 64 + 6);
                    if (lane == j) ps_pairs[2] += (unsigned long long)cnt_t;
                }
            }
        } else if (dm) {
            double2 nxt = make_double2(0.0, 0.0);
            if (a + lane <= b) nxt = pos[a + lane];
            double ux = 0.0, uy = 0.0, uz = 0.0;
            for (int c0 = a; c0 <= b; c0 += 64) {
                const int cn = min(64, b - c0 + 1);
                __builtin_amdgcn_wave_barrier();
                buf[lane] = nxt;
                if (c0 + 64 + lane <= b) nxt = pos[c0 + 64 + lane];
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes landed
                __builtin_amdgcn_wave_barrier();
                int j = 0;
                for (; j + 4 <= cn; j += 4) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const double2 pp = buf[j + u];
                        pair_force(qx, qy, pp.x, pp.y, ux, uy, uz);
                    }
                }
                for (; j < cn; ++j) {
                    const double2 pp = buf[j];
                    pair_force(qx, qy, pp.x, pp.y, ux, uy, uz);
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (dense) { fx += ux; fy += uy; zs += uz; ndense += (unsigned long long)(b - a + 1); }
            if (visits) {
                ps_steps[3] += (unsigned long long)(b - a + 1);
                if (dense) ps_pairs[3] += (unsigned long long)(b - a + 1);
            }
        }
    }
    if (PAGE) {
        if (valid && (fx != 0.0 || fy != 0.0 || zs != 0.0)) {
            unsigned long long *a = sv.acc + 6 * s;
            fxp_add(a, fx);
            fxp_add(a + 2, fy);
            fxp_add(a + 4, zs);
        }
    } else if (valid && (STREAM || cv.slot_w)) {   // STREAM: item entries (stream_finish adds them)
        mtask_n[e] = ntask;
        cv.Fp[e] = make_double2(fx, fy);
        cv.Zp[e] = zs;
    } else if (valid) {
        mtask_n[s] = ntask;
        if (fx != 0.0 || fy != 0.0 || zs != 0.0) {
            const double2 f = F[s];
            F[s] = make_double2(f.x + fx, f.y + fy);
            Z[s] = Z[s] + zs;
        }
    }
    const int wwant = wave_sum(nwant);
    // (only until the gate's threshold is reached: one memory-side atomic
    // per wave on one word would serialise ~n / 64 of them)
    if (lane == 0 && wwant && __hip_atomic_load(&mom_flag[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < mom_flag[2])
        atomicAdd(&mom_flag[1], wwant);
    if (visits) {   // [1] moment evaluations, [2] dense pair terms; [10..12] diagnostics:
                    // tile tasks, wave-level dense points, tasks with a moment check
        const unsigned long long tm = wave_sum((unsigned long long)ntask), td = wave_sum(ndense);
        unsigned long long pp[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) pp[k] = wave_sum(ps_pairs[k]);
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {   // [24 + 2k] wave steps, [25 + 2k] lane pairs of dense path k
                atomicAdd(visits + 24 + 2 * k, ps_steps[k]);
                atomicAdd(visits + 25 + 2 * k, pp[k]);
            }
            atomicAdd(visits + 10, wt_tasks);
            atomicAdd(visits + 11, wt_dense_pts);
            atomicAdd(visits + 12, wt_momchk);
            atomicAdd(visits + 1, tm);
            atomicAdd(visits + 2, td);
            const unsigned long long w_end = wall_clock64();   // [19] longest wave, [20] ~first start,
            atomicMax(visits + 19, w_end - w_start);            // [21] last end, [22] sum of wave times
            atomicMax(visits + 20, ~0ull - w_start);
            atomicMax(visits + 21, w_end);
            atomicAdd(visits + 22, w_end - w_start);
            if (MODE == 0) wave_log_put(stv.wlog, w_start, w_end, 2);
        }
    }
    if (MODE == 0) break;
    }
}

// Tile streaming's last step (see "Tile streaming"), on the consumers' stream
// after them: per handed-over list's query, moment_apply's terms M over its
// moment list, then F += D + M as moment_apply + chunk_combine would for a
// one-chunk wave (Fp = D; Fp += M if any; F += 0 + Fp if nonzero): the same bits.
__global__ __launch_bounds__(256) void stream_finish(const double2 *__restrict__ pos, const BHNode *__restrict__ nodes,
                                                     const double *__restrict__ mom, int32_t *__restrict__ ctl,
                                                     const int32_t *__restrict__ mtask,
                                                     const int32_t *__restrict__ mtask_n, const double2 *__restrict__ Dp,
                                                     const double *__restrict__ Dz, int64_t g0, int64_t g1,
                                                     double2 *__restrict__ F, double *__restrict__ Z, int32_t cap,
                                                     int32_t gen) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t k = i >> 6;
    if (k >= ctl[ST_TAIL]) return;
    const int64_t w = (int64_t)(uint32_t)st_items(ctl, cap)[k];
    if (st_claims(ctl)[w] != ((gen << 2) | 2)) return;   // summed by the slot path
    const int64_t s = g0 + w * 64 + (i & 63);
    if (s >= g1) return;
    double2 d = Dp[i];
    double dz = Dz[i];
    const int nt = mtask_n[i];
    if (nt > 0) {
        const double2 qp = pos[s];
        double fx = 0.0, fy = 0.0, zs = 0.0;
        for (int t = 0; t < nt; ++t) {
            const int node = mtask[i * MOM_TASKS + t];
            double cx, cy, R;
            box_centre(nodes[node], cx, cy, R);
            moment_eval(mom + (int64_t)node * MOM_K, qp.x - cx, qp.y - cy, fx, fy, zs);
        }
        d = make_double2(d.x + fx, d.y + fy);
        dz = dz + zs;
    }
    const double sx = 0.0 + d.x, sy = 0.0 + d.y, sz = 0.0 + dz;
    if (sx != 0.0 || sy != 0.0 || sz != 0.0) {
        const double2 f = F[s];
        F[s] = make_double2(f.x + sx, f.y + sy);
        Z[s] = Z[s] + sz;
    }
}

// F, Z of the queries of every group that spilled += their tasks' fixed-point
// sums (then zeroed); thread 0 also empties the queue for the next traversal.
__global__ void spill_combine(const int32_t *__restrict__ gflag, int32_t gen, unsigned long long *__restrict__ acc,
                              int64_t g0, int64_t g1, const int32_t *__restrict__ qlist, double2 *__restrict__ F,
                              double *__restrict__ Z, int32_t *__restrict__ ctl) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {   // the lists are empty for the next traversal
        ctl[SP_PAGES] = 0;
        for (int l = 1; l <= SP_LMAX; ++l) { ctl[sp_head(l)] = 0; ctl[sp_ttail(l)] = 0; ctl[sp_etail(l)] = 0; }
    }
    const int64_t k = g0 + i;
    if (k >= g1 || gflag[i >> 6] != gen) return;
    const int64_t s = qlist ? (int64_t)qlist[k] : k;
    ulonglong2 *a = reinterpret_cast<ulonglong2 *>(acc + 6 * s);
    const ulonglong2 vx = a[0], vy = a[1], vz = a[2];
    if ((vx.x | vx.y | vy.x | vy.y | vz.x | vz.y) == 0ull) return;
    const double2 f = F[s];
    F[s] = make_double2(f.x + fxp_value(vx.x, vx.y), f.y + fxp_value(vy.x, vy.y));
    Z[s] = Z[s] + fxp_value(vz.x, vz.y);
    const ulonglong2 zero = make_ulonglong2(0ull, 0ull);
    a[0] = zero; a[1] = zero; a[2] = zero;
}

// The next traversal's budgets from this one's costs (one workgroup): the
// mean walk cost per group (pops + tile points / 64, the group's tasks
// included; groups without a cost -- narrow ones before their selection --
// left out), B0 = max(bmin, fac mean), B1 = max(8, ftask B0).
__global__ __launch_bounds__(1024) void spill_budget(const int32_t *__restrict__ wcost, int64_t waves, double fac,
                                                     double ftask, int32_t bmin, int32_t *__restrict__ ctl) {
    __shared__ unsigned long long rs[16], rc[16];
    const int t = threadIdx.x, lane = lane_id(), w = t >> 6;
    unsigned long long sum = 0, cnt = 0;
    for (int64_t g = t; g < waves; g += 1024) {
        const int32_t c = wcost[g];
        if (c > 0) { sum += (unsigned long long)c; ++cnt; }
    }
    sum = wave_sum(sum);
    cnt = wave_sum(cnt);
    if (lane == 0) { rs[w] = sum; rc[w] = cnt; }
    __syncthreads();
    if (t == 0) {
        unsigned long long S = 0, C = 0;
        for (int k = 0; k < 16; ++k) { S += rs[k]; C += rc[k]; }
        const double mean = C ? (double)S / (double)C : 0.0;
        const int32_t b0 = (int32_t)fmin(2e9, fmax((double)bmin, fac * mean));
        ctl[SP_B0] = b0;
        ctl[SP_B1] = (int32_t)fmax(8.0, ftask * (double)b0);
    }
}

// ---- Root-tile mode (the small-embedding phase).  When every point lies in
// the root cell, no point has an exact duplicate, the bounding box is so
// small that every query opens the root (4 theta max(dx, dy) < 1: a cell
// holding all points has half-width >= max(dx, dy) / 2 and D <= dx^2 + dy^2)
// and passes the near-exact test at it (every box corner within near_dmax),
// the normal path makes the root one tile for every lane, evaluated from the
// root's moments (tile_apply -> moment_apply).  This path computes that --
// the root's moments (moment_items / moment_reduce, chunks of the points in
// label order), the same per-query additions -- without the Morton sort, the
// radix tree, the bottom-up aggregates, the quad records or the moments of
// the other ~n/64 nodes.  Duplicates are found by a hash set instead of the
// sorted order (any duplicate: the full path).
//
// Exact-duplicate detection without sorting or atomics (device-scope atomics
// execute at the memory side, ~13 G/s for one CAS per point): rounds of a
// last-writer-wins table of 4n slots.  Round r: every open point stores its
// index at slot h_r(point) (plain stores; one of the points sharing a slot
// wins), then -- next kernel -- reads the slot back: the winner is done, a
// point that finds a point with its exact coordinates raises the flag, and a
// point that finds different coordinates stays open for the next round's
// hash.  Two copies of one position share every slot, so they stay open
// together until one of them wins one (found).  ~11 % of the points stay open
// after round 0, ~0.2 % after round 1; any still open after the last round
// raise the flag too (flag = "not shown duplicate-free": the full path, which
// handles every case).
constexpr int DUP_ROUNDS = 4;
__device__ __forceinline__ uint64_t hash_xy(double x, double y, uint64_t seed) {
    uint64_t h = ((uint64_t)__double_as_longlong(x) ^ seed) * 0x9E3779B97F4A7C15ull;
    h ^= (uint64_t)__double_as_longlong(y) + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2);
    h ^= h >> 31;
    h *= 0xD6E8FEB86659FD93ull;
    return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t dup_seed(int round) { return 0xA24BAED4963EE407ull * (uint64_t)(round + 1); }

__global__ __launch_bounds__(256) void dup_store(const double2 *__restrict__ Y, int64_t n, int32_t *__restrict__ tab,
                                                 uint64_t mask, const uint8_t *__restrict__ open, int round) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || (round > 0 && !open[i])) return;
    const double2 p = Y[i];
    tab[hash_xy(p.x, p.y, dup_seed(round)) & mask] = (int32_t)i;
}

__global__ __launch_bounds__(256) void dup_probe(const double2 *__restrict__ Y, int64_t n,
                                                 const int32_t *__restrict__ tab, uint64_t mask,
                                                 uint8_t *__restrict__ open, int round, int32_t *__restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || (round > 0 && !open[i])) return;
    const double2 p = Y[i];
    const int64_t w = tab[hash_xy(p.x, p.y, dup_seed(round)) & mask];
    bool still = false;
    if (w != i) {
        const double2 o = Y[w];
        if (o.x == p.x && o.y == p.y) flag[0] = 1;
        else still = true;
    }
    if (still && round == DUP_ROUNDS - 1) flag[0] = 1;
    if (round == 0 || !still) open[i] = still ? 1 : 0;
}

// The root's moments from its chunk partials (root-tile mode, ~n / MOM_CHUNK
// chunks): one block per moment, fixed strided + tree order.
__global__ __launch_bounds__(256) void root_moment_reduce(const int32_t *__restrict__ mom_off, int64_t n,
                                                          const double *__restrict__ part, double *__restrict__ mom) {
    __shared__ double red[256];
    const int k = blockIdx.x;
    const int K = mom_off[n];
    double s = 0.0;
    for (int it = threadIdx.x; it < K; it += 256) s += part[(int64_t)it * MOM_K + k];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) mom[k] = red[0];
}

__global__ void root_tile_check(const int32_t *__restrict__ dflag, const double *__restrict__ bb,
                                const double *__restrict__ Wp, int64_t n, double theta, double near_dmax,
                                int32_t *__restrict__ status) {
    const double W = *Wp, dx = bb[1] - bb[0], dy = bb[3] - bb[2];
    const double amax = fmax(fmax(fabs(bb[0]), fabs(bb[1])), fmax(fabs(bb[2]), fabs(bb[3])));
    const double ex = 6e-15 * amax;   // the traversal's rounding margin, bounded for every query in the box
    const double dmax = ((dx + ex) * (dx + ex) + (dy + ex) * (dy + ex)) * (1.0 + 1e-11);
    // every point inside the root cell Cell(0, 0, W) (closed, Cell.scala:31-36)
    const bool in_root = -W <= bb[0] && bb[1] <= W && -W <= bb[2] && bb[3] <= W;
    const double box = 4.0 * theta * fmax(dx, dy) * (1.0 + 1e-12);
    const bool ok = in_root && n >= MOM_MIN_POINTS && !dflag[0] && W > 0.0 && theta > 0.0 && box < 1.0 &&
                    dmax <= near_dmax;
    status[0] = ok ? 1 : 0;
    // how far the box is from the test: floor(log2) of the larger ratio (the
    // host skips the test for a while once the embedding has outgrown it)
    const double r = fmax(box, near_dmax > 0.0 ? dmax / near_dmax : 0.0);
    status[1] = r > 1.0 ? (int32_t)fmin(60.0, floor(log2(r))) : 0;
}

// The root's moment items: node 0 = all m sorted points, its bounding box.
__global__ void root_tile_prep(const double *__restrict__ bb, int64_t n, BHNode *__restrict__ nodes,
                               int32_t *__restrict__ mom_cnt, int32_t *__restrict__ mom_off,
                               int32_t *__restrict__ mom_list, int32_t *__restrict__ mom_item, int32_t *__restrict__ meta_w,
                               int32_t *__restrict__ inv, int32_t *__restrict__ idx_sorted,
                               int32_t *__restrict__ mom_flag) {
    const int m = (int)n;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        inv[i] = i;            // no sort: query / force slots are the labels
        idx_sorted[i] = i;
    }
    const int K = (m + MOM_CHUNK - 1) / MOM_CHUNK;
    for (int it = blockIdx.x * blockDim.x + threadIdx.x; it < K; it += gridDim.x * blockDim.x) mom_item[it] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        BHNode &r = nodes[0];
        r.first = 0; r.last = m - 1; r.cnt = m;
        r.bx0 = bb[0]; r.bx1 = bb[1]; r.by0 = bb[2]; r.by1 = bb[3];
        mom_cnt[0] = K;
        mom_off[0] = 0;
        mom_off[n] = K;
        mom_list[0] = 0;
        meta_w[0] = m;
        meta_w[2] = 1;
        // every query's tile is eligible: the next full build keeps moments on
        mom_flag[0] = 1;
        mom_flag[1] = mom_flag[2];
    }
}

// Per query: what the traversal (root tile, z -= the query itself: no
// duplicates in this mode), tile_apply (moment task, or the dense leaf sum)
// and moment_apply write for it -- the moment sums from the root's
// polynomial coefficients (poly_moment_eval).
template <bool STATS>
__global__ __launch_bounds__(256) void root_tile_eval(const double2 *__restrict__ pos, const BHNode *__restrict__ nodes,
                                                      const double *__restrict__ coef, const int32_t *__restrict__ meta,
                                                      int64_t g0, int64_t g1, const int32_t *__restrict__ qlist,
                                                      double2 *__restrict__ F, double *__restrict__ Z,
                                                      unsigned long long *__restrict__ visits, double mom_tol) {
    const int64_t k = g0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = k < g1;
    const int64_t s = valid ? (qlist ? (int64_t)qlist[k] : k) : 0;
    const int m = meta[0];
    const BHNode &rt = nodes[0];
    bool usem = false;
    double fx = 0.0, fy = 0.0, zs = 0.0;
    if (valid) {
        const double2 q = pos[s];
        usem = moment_ok(rt.bx0, rt.bx1, rt.by0, rt.by1, q.x, q.y, mom_tol);
        if (usem) {
            double cx, cy, R;
            box_centre(rt, cx, cy, R);
            poly_moment_eval(coef, q.x - cx, q.y - cy, fx, fy, zs);
            F[s] = make_double2(0.0 + fx, 0.0 + fy);
        } else {   // the exact leaf sum (only if the series bound fails: not expected here)
            for (int p = 0; p < m; ++p) { const double2 pp = pos[p]; pair_force(q.x, q.y, pp.x, pp.y, fx, fy, zs); }
            F[s] = make_double2(fx, fy);
        }
        Z[s] = -1.0 + zs;
    }
    if (STATS && visits) {   // block totals, one set of atomics per block
        __shared__ unsigned long long sv[4][2];
        const unsigned long long nv = __popcll(__ballot(valid)), nu = __popcll(__ballot(usem));
        if (lane_id() == 0) { sv[threadIdx.x >> 6][0] = nv; sv[threadIdx.x >> 6][1] = nu; }
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long bv = 0, bu = 0, bw = 0;
            for (int w = 0; w < 4; ++w) { bv += sv[w][0]; bu += sv[w][1]; bw += sv[w][0] ? 1 : 0; }
            if (bv) {
                atomicAdd(visits, bv * (unsigned long long)m);
                atomicAdd(visits + 1, bu);
                atomicAdd(visits + 2, (bv - bu) * (unsigned long long)m);
                atomicAdd(visits + 3, bw);
                atomicAdd(visits + 4, bw * (unsigned long long)m);
            }
        }
    }
}

// Sort keys of a longest-first block order: block b's cost = its heaviest wave.
__global__ void block_cost_keys(const int32_t *__restrict__ cost, int64_t nwaves, int64_t nblocks,
                                int32_t *__restrict__ key, int32_t *__restrict__ val) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblocks) return;
    int32_t c = 0;
    for (int w = 0; w < 4; ++w)
        if (4 * b + w < nwaves) c = max(c, cost[4 * b + w]);
    key[b] = c;
    val[b] = (int32_t)b;
}

// Heavy groups a traversal of `waves` 64-query waves turns narrow to fill the
// chip: narrowing h groups adds (NPARTS - 1) h waves; up to 8 waves per SIMD
// (32 per CU) in all.  0 once the 64-query waves alone fill it (one rank of
// 1M points: 15,625 waves).  Below half of that (one of 8 ranks at C3: 1,953
// waves) every group: there each 64-query wave is one latency-bound chain
// with ~2 waves per SIMD beside it, and the narrow layout cuts the chain
// (W = 8 projection, scripts/loop_projection.py: span 4.83 -> 3.99 s).
int64_t narrow_fill(const tsne_ctx *ctx, int64_t waves) {
    const int64_t cap = 32 * (int64_t)ctx->cu_count;
    if (waves >= cap) return 0;
    return waves < cap / 2 ? waves : (cap - waves) / (NPARTS - 1);
}

}  // namespace

// The Morton sort (64-bit keys, int32 payload).  rocPRIM's radix sort picks
// its merge sort below 2^20 items (22 launches, ~200 us at 1M; Onesweep
// measured ~300 us at 1M).
static void morton_sort(void *tmp, size_t &bytes, const uint64_t *k_in, uint64_t *k_out, const int32_t *v_in,
                        int32_t *v_out, int64_t n, hipStream_t st) {
    TSNE_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, bytes, k_in, k_out, v_in, v_out, (int)n, 0, 64, st));
}

// Longest-first order of nblocks blocks by the per-wave costs -> order.
static void block_order(tsne_ctx *ctx, BHTree &t, const int32_t *cost, int64_t nwaves, int64_t nblocks,
                        int32_t *order) {
    hipStream_t st = ctx->stream;
    hipLaunchKernelGGL(block_cost_keys, dim3(ceil_div(nblocks, 256)), dim3(256), 0, st, cost, nwaves, nblocks, t.okey,
                       t.oval);
    size_t tb = t.osort_tmp_bytes;
    TSNE_HIP(hipcub::DeviceRadixSort::SortPairsDescending(t.osort_tmp, tb, t.okey, t.okey2, t.oval, order,
                                                          (int)nblocks, 0, 32, st));
}

void bh_alloc(tsne_ctx *ctx, BHTree &t, int64_t n, const std::string &pre) {
    Workspace &ws = ctx->ws;
    t.n = n;
    t.keys = ws.get<uint64_t>(pre + "keys", n);
    t.keys_sorted = ws.get<uint64_t>(pre + "keys_sorted", n);
    t.idx = ws.get<int32_t>(pre + "idx", n);
    t.idx_sorted = ws.get<int32_t>(pre + "idx_sorted", n);
    t.inv = ws.get<int32_t>(pre + "inv", n);
    t.dupc = ws.get<int32_t>(pre + "dupc", n);
    t.vid = ws.get<int32_t>(pre + "vid", n);
    t.dflag = ws.get<int32_t>(pre + "dflag", 1);
    t.rmin = ws.get<int32_t>(pre + "rmin", n);
    t.rvid = ws.get<int32_t>(pre + "rvid", n);
    t.rt2 = ws.get<int32_t>(pre + "rt2", n);
    t.arrive2 = ws.get<int32_t>(pre + "arrive2", n);
    t.cntcorr = ws.get<int32_t>(pre + "cntcorr", n);
    t.tiecnt = ws.get<int32_t>(pre + "tiecnt", n);
    t.notile = ws.get<int32_t>(pre + "notile", n);
    t.sumcorr = ws.get<double>(pre + "sumcorr", 2 * (size_t)n);
    t.vflag = ws.get<int32_t>(pre + "vflag", n);
    t.vcnt = ws.get<int32_t>(pre + "vcnt", n);
    t.vcntf = ws.get<int32_t>(pre + "vcntf", n);
    t.vsum = ws.get<double>(pre + "vsum", 2 * (size_t)n);
    t.vcom = ws.get<double>(pre + "vcom", 2 * (size_t)n);
    t.pos = ws.get<double2>(pre + "pos", n);
    t.nodes = ws.get<BHNode>(pre + "nodes", n);
    t.qrec = ws.get<QRec>(pre + "qrec", 2 * (size_t)n);   // [n, 2n): virtual chain-top records (duplicates)
    t.agg = ws.get<double>(pre + "agg", AGG * (size_t)n);
    t.parent_leaf = ws.get<int32_t>(pre + "parent_leaf", n);
    t.parent_node = ws.get<int32_t>(pre + "parent_node", n);
    t.arrive = ws.get<int32_t>(pre + "arrive", n);
    t.fstart = ws.get<int32_t>(pre + "fstart", n);
    TSNE_HIP(hipMemsetAsync(t.fstart, 0, sizeof(int32_t) * n, ctx->stream));
    t.gen = 0;
    t.rt_skip = 0;
    t.top_list = ws.get<int32_t>(pre + "top_list", 2 * (size_t)n);
    t.top_cnt = ws.get<int32_t>(pre + "top_cnt", 1);
    t.meta = ws.get<int32_t>(pre + "meta", 4);
    t.mom = ws.get<double>(pre + "mom", (size_t)n * MOM_K);
    t.mom_cnt = ws.get<int32_t>(pre + "mom_cnt", n + 1);
    t.mom_off = ws.get<int32_t>(pre + "mom_off", n + 1);
    t.mom_list = ws.get<int32_t>(pre + "mom_list", n);
    // items <= sum over moment nodes of (cnt / MOM_CHUNK + 1); every point lies in
    // at most 94 nested nodes (62 key bits + 32 tie-break bits)
    t.mom_items_cap = n + ceil_div(n * 94, MOM_CHUNK);
    t.mom_item = ws.get<int32_t>(pre + "mom_item", t.mom_items_cap);
    t.mom_part = ws.get<double>(pre + "mom_part", (size_t)t.mom_items_cap * MOM_K);
    t.mom_flag = ws.get<int32_t>(pre + "mom_flag", 3);
    const int32_t flag_init[3] = {1, INT32_MAX, (int32_t)std::min<int64_t>(INT32_MAX, (n >> 6) + 1)};   // first build: moments on
    TSNE_HIP(hipMemcpyAsync(t.mom_flag, flag_init, sizeof(flag_init), hipMemcpyHostToDevice, ctx->stream));
    TSNE_HIP(hipStreamSynchronize(ctx->stream));
    // tile_apply slots: traversal waves + at most half as many extra chunks (+ margin)
    const int64_t qwaves = ceil_div(n, 64) + 4;
    t.tile_waves = qwaves + qwaves / 2 + 64;
    t.mtask = ws.get<int32_t>(pre + "mtask", (size_t)std::max<int64_t>(n, t.tile_waves * 64) * MOM_TASKS);
    t.mtask_n = ws.get<int32_t>(pre + "mtask_n", std::max<int64_t>(n, t.tile_waves * 64));
    t.ttask = ws.get<TileTask>(pre + "ttask", (size_t)t.tile_waves * TILE_CAP);
    t.ttask_n = ws.get<int32_t>(pre + "ttask_n", t.tile_waves);
    size_t sb = 0;
    TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, sb, t.mom_cnt, t.mom_off, (int)(n + 1), ctx->stream));
    t.scan_tmp_bytes = sb;
    t.scan_tmp = ws.get<uint8_t>(pre + "scan_tmp", sb);
    t.bbox_blocks = (int)std::min<int64_t>(1024, std::max<int64_t>(1, ceil_div(n, 256)));
    t.bbox_part = ws.get<double>(pre + "bbox_part", 4 * (size_t)t.bbox_blocks);
    t.W = ws.get<double>(pre + "W", 1);
    t.bb = ws.get<double>(pre + "bb", 4);
    t.status = ws.get<int32_t>(pre + "status", 4);
    t.status_h = ctx->pinned;
    t.rcoef = ws.get<double>(pre + "rcoef", POLY_K);
    t.dup_mask = ((uint64_t)1 << (64 - __builtin_clzll((uint64_t)std::max<int64_t>(2, 4 * n) - 1))) - 1;
    t.dup_tab = ws.get<int32_t>(pre + "dup_tab", t.dup_mask + 1);
    t.dup_open = ws.get<uint8_t>(pre + "dup_open", n);
    size_t tb = 0;
    morton_sort(nullptr, tb, t.keys, t.keys_sorted, t.idx, t.idx_sorted, n, ctx->stream);
    t.sort_tmp_bytes = tb;
    t.sort_tmp = ws.get<uint8_t>(pre + "sort_tmp", tb);
    csort_alloc(ctx, t.cs, n, pre);
    t.cs_primed = false;
    const int64_t nb = ceil_div(t.tile_waves, 4);
    t.wcost = ws.get<int32_t>(pre + "wcost", t.tile_waves);
    t.tcost = ws.get<int32_t>(pre + "tcost", t.tile_waves);
    t.okey = ws.get<int32_t>(pre + "okey", nb);
    t.okey2 = ws.get<int32_t>(pre + "okey2", nb);
    t.oval = ws.get<int32_t>(pre + "oval", nb);
    t.border = ws.get<int32_t>(pre + "border", nb);
    t.torder = ws.get<int32_t>(pre + "torder", nb);
    size_t ob = 0;
    TSNE_HIP(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, ob, t.okey, t.okey2, t.oval, t.border, (int)nb, 0,
                                                          32, ctx->stream));
    t.osort_tmp_bytes = ob;
    t.osort_tmp = ws.get<uint8_t>(pre + "osort_tmp", ob);
    t.sel_waves = 0;
    t.ran_narrow = false;
    t.ch_C = ws.get<int32_t>(pre + "ch_C", qwaves + 1);
    t.ch_slot0 = ws.get<int32_t>(pre + "ch_slot0", qwaves + 1);
    t.ch_slot_w = ws.get<int32_t>(pre + "ch_slot_w", t.tile_waves);
    t.ch_slot_c = ws.get<int32_t>(pre + "ch_slot_c", t.tile_waves);
    t.ch_scost = ws.get<int32_t>(pre + "ch_scost", t.tile_waves);
    t.ch_nslots = ws.get<int32_t>(pre + "ch_nslots", 1);
    t.ch_total = ws.get<unsigned long long>(pre + "ch_total", 1);
    t.ch_Fp = ws.get<double2>(pre + "ch_Fp", (size_t)t.tile_waves * 64);
    t.ch_Zp = ws.get<double>(pre + "ch_Zp", (size_t)t.tile_waves * 64);
    size_t cb = 0;
    TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, cb, t.ch_C, t.ch_slot0, (int)(qwaves + 1), ctx->stream));
    t.ch_scan_bytes = cb;
    t.ch_scan_tmp = ws.get<uint8_t>(pre + "ch_scan_tmp", cb);
    // narrow layout of heavy groups: at most 1/8 of the groups, their moment lists
    t.nar_hmax = std::max<int64_t>({(int64_t)1, ceil_div(qwaves, 8), std::min<int64_t>(qwaves, 16 * (int64_t)ctx->cu_count)});
    t.nflag = ws.get<int32_t>(pre + "nflag", t.tile_waves);
    TSNE_HIP(hipMemsetAsync(t.nflag, 0, sizeof(int32_t) * t.tile_waves, ctx->stream));
    t.hlist = ws.get<int32_t>(pre + "hlist", t.nar_hmax);
    t.hcount = ws.get<int32_t>(pre + "hcount", 1);
    t.hran = ws.get<int32_t>(pre + "hran", 1);
    TSNE_HIP(hipMemsetAsync(t.hcount, 0, sizeof(int32_t), ctx->stream));
    t.ncost = ws.get<int32_t>(pre + "ncost", (size_t)t.nar_hmax * NPARTS);
    t.nmtask = ws.get<int32_t>(pre + "nmtask", (size_t)t.nar_hmax * 64 * MOM_TASKS);
    t.nmtask_n = ws.get<int32_t>(pre + "nmtask_n", (size_t)t.nar_hmax * 64);
    t.pre = pre;
    t.sp_ctl = nullptr;   // spill buffers: on first use (bh_spill_alloc)
    t.pcost_valid = false;   // (trav_front_cur: no previous costs for this size)
    t.order_ready = false;
    t.sp_gen = 0;
    t.sp_waves = 0;
    t.ran_spill = false;
    TSNE_HIP(hipStreamSynchronize(ctx->stream));
}

// The spill buffers (see "Spill"): per level, stack entries and tasks for
// max(16 per query group, 2^18) entries (far more than the budgets produce),
// 64-tile pages for n / 4 + 16384 pages of task tiles, 48 B of accumulators
// per point.
static void bh_spill_alloc(tsne_ctx *ctx, BHTree &t) {
    if (t.sp_ctl) return;
    Workspace &ws = ctx->ws;
    const std::string &pre = t.pre;
    const int64_t n = t.n, qwaves = ceil_div(n, 64) + 4;
    t.sp_cap = (int32_t)std::min<int64_t>(1 << 26, std::max<int64_t>(1 << 18, 16 * qwaves));
    t.sp_pg_cap = (int32_t)std::min<int64_t>(1 << 24, n / 4 + (1 << 14));
    t.sp_ctl = ws.get<int32_t>(pre + "sp_ctl", SP_NCTL);
    t.sp_task = ws.get<int4>(pre + "sp_task", (size_t)SP_LMAX * t.sp_cap);
    t.sp_ent = ws.get<uint4>(pre + "sp_ent", (size_t)SP_LMAX * t.sp_cap);
    t.sp_gflag = ws.get<int32_t>(pre + "sp_gflag", t.tile_waves);
    t.sp_acc = ws.get<unsigned long long>(pre + "sp_acc", 6 * (size_t)n);
    t.sp_pg_tiles = ws.get<TileTask>(pre + "sp_pg_tiles", (size_t)t.sp_pg_cap * SP_PAGE);
    t.sp_pg_grp = ws.get<int32_t>(pre + "sp_pg_grp", t.sp_pg_cap);
    t.sp_pg_n = ws.get<int32_t>(pre + "sp_pg_n", t.sp_pg_cap);
    hipStream_t st = ctx->stream;
    TSNE_HIP(hipMemsetAsync(t.sp_ctl, 0, sizeof(int32_t) * SP_NCTL, st));
    TSNE_HIP(hipMemsetAsync(t.sp_gflag, 0, sizeof(int32_t) * t.tile_waves, st));
    TSNE_HIP(hipMemsetAsync(t.sp_acc, 0, sizeof(unsigned long long) * 6 * n, st));
    t.sp_gen = 0;
}

// Tile streaming: control words, one item and one flag per traversal wave;
// the consumers' stream and events on the context.
static void bh_stream_alloc(tsne_ctx *ctx, BHTree &t) {
    if (!ctx->st_stream) {
        TSNE_HIP(hipStreamCreateWithFlags(&ctx->st_stream, hipStreamNonBlocking));
        for (auto &e : ctx->st_ev) TSNE_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    Workspace &ws = ctx->ws;
    // control words, the claims, the items; kept (with ST_W, the threshold
    // the last plan set) while the tree keeps its size
    const size_t words = ST_Q0 + 3 * (size_t)t.tile_waves + 2;
    int32_t *c = ws.get<int32_t>(t.pre + "st_ctl", words);
    const bool fresh = c != t.st_ctl || t.st_words != words;
    t.st_ctl = c;
    t.st_words = words;
    // per item (<= one per traversal wave slot) and lane: partial sums D and moment lists
    const size_t ent = (size_t)(ceil_div(t.n, 64) + TRAV_WPB) * 64;
    t.st_Dp = ws.get<double2>(t.pre + "st_Dp", ent);
    t.st_Dz = ws.get<double>(t.pre + "st_Dz", ent);
    t.st_mtask_n = ws.get<int32_t>(t.pre + "st_mtask_n", ent);
    t.st_mtask = ws.get<int32_t>(t.pre + "st_mtask", ent * MOM_TASKS);
    if (fresh) {
        TSNE_HIP(hipMemsetAsync(t.st_ctl, 0, sizeof(int32_t) * words, ctx->stream));
        t.st_gen = 0;
    }
}

int64_t bh_stream_counter(tsne_ctx *ctx, BHTree &t) {
    if (!t.st_ctl) return 0;
    int32_t c[ST_Q0];
    TSNE_HIP(hipMemcpyAsync(c, t.st_ctl, sizeof(c), hipMemcpyDeviceToHost, ctx->stream));
    TSNE_HIP(hipStreamSynchronize(ctx->stream));
    return (int64_t)c[ST_CUM];
}

int64_t bh_spill_counter(tsne_ctx *ctx, BHTree &t, bool flags) {
    if (!t.sp_ctl) return 0;
    int32_t c[SP_NCTL];
    TSNE_HIP(hipMemcpyAsync(c, t.sp_ctl, sizeof(c), hipMemcpyDeviceToHost, ctx->stream));
    TSNE_HIP(hipStreamSynchronize(ctx->stream));
    return flags ? (int64_t)c[SP_OVF] : (int64_t)c[SP_TASKS];
}

int64_t bh_narrow_groups(tsne_ctx *ctx, BHTree &t) {
    if (!t.ran_narrow || !t.hran) return 0;
    int32_t h = 0;
    TSNE_HIP(hipMemcpyAsync(&h, t.hran, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    TSNE_HIP(hipStreamSynchronize(ctx->stream));
    return h;
}

BHTree &bh_single_tree(tsne_ctx *ctx, int64_t n) {
    if (!ctx->single_tree) ctx->single_tree = new BHTree();
    BHTree &t = *ctx->single_tree;
    if (t.n != n) bh_alloc(ctx, t, n, "bh1.");
    // a single call is a function of its input alone unless the caller asked
    // for the previous call's costs (Options::reuse_costs): without costs the
    // traversal takes the 64-query layout everywhere
    if (!ctx->opts.reuse_costs) { t.sel_waves = 0; t.sp_waves = 0; t.front_waves = 0; }
    return t;
}

// Cost-balanced query slices for the next iteration: one 1024-thread block
// scans the (all-reduced, so identical on every rank) 256-query bucket costs
// and cuts the sorted order into world pieces of equal cost.
__global__ __launch_bounds__(1024) void balance_slices(const unsigned long long *__restrict__ bcost, int64_t nb,
                                                       int64_t n, int world, int64_t *__restrict__ bounds) {
    __shared__ unsigned long long part[1024];
    __shared__ unsigned long long total;
    const int t = threadIdx.x;
    const int64_t per = (nb + 1023) / 1024, b0 = t * per, b1 = min(nb, b0 + per);
    unsigned long long acc = 0;
    for (int64_t b = b0; b < b1; ++b) acc += bcost[b];
    part[t] = acc;
    __syncthreads();
    if (t == 0) {
        unsigned long long run = 0;
        for (int k = 0; k < 1024; ++k) { const unsigned long long v = part[k]; part[k] = run; run += v; }
        total = run;
        bounds[0] = 0;
        bounds[world] = n;
        for (int r = 1; r < world; ++r)   // a zero target cuts at 0; the scan sets the others
            bounds[r] = (run / world * r + (run % world) * r / world) == 0 ? 0 : n;
    }
    __syncthreads();
    // thread t owns buckets [b0, b1) with exclusive prefix part[t]
    unsigned long long run = part[t];
    for (int64_t b = b0; b < b1; ++b) {
        const unsigned long long nxt = run + bcost[b];
        for (int r = 1; r < world; ++r) {
            const unsigned long long target = total / world * r + (total % world) * r / world;
            if (run < target && nxt >= target) bounds[r] = min(n, (b + 1) << 8);
        }
        run = nxt;
    }
    __syncthreads();
    if (t == 0) {   // all-zero costs: equal counts; keep the cuts monotone
        for (int r = 1; r < world; ++r) {
            if (total == 0) bounds[r] = n * r / world;
            if (bounds[r] < bounds[r - 1]) bounds[r] = bounds[r - 1];
        }
    }
}

void bh_balance(tsne_ctx *ctx, const unsigned long long *bcost, int64_t n, int world, int64_t *bounds) {
    hipLaunchKernelGGL(balance_slices, dim3(1), dim3(1024), 0, ctx->stream, bcost, ceil_div(n, 256), n, world, bounds);
    TSNE_LAUNCH_CHECK();
}

// ---- tree partition (several ranks; see REF_FORCED)
// One wave: cut r (1 <= r < world) moved forward to the first sorted position p
// with p == m or a level-PART_LEVEL cell boundary between keys p - 1 and p.
__global__ void part_align_kernel(const uint64_t *__restrict__ keys, const int32_t *__restrict__ meta,
                                  const int64_t *__restrict__ cuts, int world, int rank, int32_t *__restrict__ plim) {
    const int lane = lane_id();
    const int64_t m = meta[0];
    constexpr int SH = 62 - 2 * PART_LEVEL;
    auto align = [&](int r) -> int64_t {
        if (r <= 0) return 0;
        if (r >= world) return INT32_MAX;
        int64_t c = min(max(cuts[r], (int64_t)0), m);
        if (c <= 0 || c >= m) return c;
        for (int64_t b = c; b < m; b += 64) {
            const int64_t p = b + lane;
            const bool hit = p >= m || (keys[p - 1] >> SH) != (keys[p] >> SH);
            const uint64_t bl = __ballot(hit);
            if (bl) return b + __ffsll((long long)bl) - 1;
        }
        return m;
    };
    const int64_t lo = align(rank), hi = align(rank + 1);
    if (lane == 0) {
        plim[0] = (int32_t)lo;
        plim[1] = (int32_t)max(lo, hi);
    }
}

// One thread: equal-cost cuts of the cumulative cost, linear inside each
// rank's current range, moved half way from the current cuts.
__global__ void part_recut_kernel(const unsigned long long *__restrict__ cost, int world, int64_t n,
                                  int64_t *__restrict__ cuts) {
    if (threadIdx.x != 0) return;
    double total = 0.0;
    for (int r = 0; r < world; ++r) total += (double)cost[r];
    if (!(total > 0.0)) return;
    double nc[64];
    int r = 0;
    double cum = 0.0;
    for (int k = 1; k < world && k < 64; ++k) {
        const double T = total * k / world;
        while (r < world - 1 && cum + (double)cost[r] <= T) cum += (double)cost[r++];
        const double x0 = (double)cuts[r], x1 = (double)(r + 1 < world ? cuts[r + 1] : n);
        const double f = cost[r] > 0 ? (T - cum) / (double)cost[r] : 0.5;
        nc[k] = x0 + f * (x1 - x0);
    }
    for (int k = 1; k < world && k < 64; ++k) {
        int64_t v = (int64_t)(0.5 * ((double)cuts[k] + nc[k]));
        v = max(v, cuts[k - 1]);
        cuts[k] = min(v, n);
    }
}

// Sum of the traversal waves' costs (pops + tile points / 64).
__global__ __launch_bounds__(1024) void part_cost_kernel(const int32_t *__restrict__ wcost, int64_t waves,
                                                         unsigned long long *__restrict__ out) {
    __shared__ unsigned long long red[16];
    unsigned long long a = 0;
    for (int64_t i = threadIdx.x; i < waves; i += 1024) a += (unsigned long long)max(wcost[i], 0);
    a = wave_sum(a);
    if (lane_id() == 0) red[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int k = 0; k < 16; ++k) t += red[k];
        *out = t;
    }
}

// The near-exact tolerance of a build (Options::near_tol_early / near_tol_late;
// 0 disables the test)
double bh_near_tol(const tsne_ctx *ctx, bool late) { return late ? ctx->opts.near_tol_late : ctx->opts.near_tol_early; }

// Largest D for which 48 theta^2 D^2 (1 + 8 D) <= tol (see bh_traverse).
double bh_near_dmax(double theta, double tol) {
    if (!(theta > 0.0)) return __builtin_inf();   // theta = 0: the reference opens every cell
    if (!(tol > 0.0)) return -1.0;
    double d = std::sqrt(tol / (48.0 * theta * theta));
    while (48.0 * theta * theta * d * d * (1.0 + 8.0 * d) > tol) d *= 0.99;
    return d;
}

void bh_build(tsne_ctx *ctx, BHTree &t, const double *dY, double theta, const int32_t *rowmap, bool root_tile_ok,
              double near_tol) {
    if (near_tol < 0.0) near_tol = bh_near_tol(ctx, false);
    t.near_dmax = bh_near_dmax(theta, near_tol);
    hipStream_t st = ctx->stream;
    const int64_t n = t.n;
    t.rowmap = rowmap;
    t.root_tile = false;
    TSNE_HIP(hipMemsetAsync(t.dflag, 0, sizeof(int32_t), st));
    hipLaunchKernelGGL(bbox_partial, dim3(t.bbox_blocks), dim3(256), 0, st, dY, n, t.bbox_part);
    hipLaunchKernelGGL(bbox_final, dim3(1), dim3(256), 0, st, t.bbox_part, t.bbox_blocks, t.W, t.meta, t.bb,
                       t.mom_flag, t.mom_off + n);
    // once the box failed the root-tile test by 2^k (k >= 3), the next 4 (k - 2)
    // builds (<= 64) skip the test and its host read-back: the embedding
    // shrinks by a few % per iteration at most (C3: extent 1e-3 -> 9e-5 over
    // t = 10..100), and a skipped test only means the full build, whose sums
    // the root-tile path reproduces (performance, not results)
    if (root_tile_ok && t.rt_skip > 0) {
        --t.rt_skip;
        root_tile_ok = false;
    }
    if (root_tile_ok) {   // small read-backs decide the path (the host must know which kernels to launch)
        // the box conditions first (dflag still 0): once the embedding has
        // outgrown the root tile, the duplicate rounds (~90 us at 1M) are skipped
        hipLaunchKernelGGL(root_tile_check, dim3(1), dim3(1), 0, st, t.dflag, t.bb, t.W, n, theta, t.near_dmax,
                           t.status);
        TSNE_HIP(hipMemcpyAsync(t.status_h, t.status, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        TSNE_HIP(hipStreamSynchronize(st));
        if (!t.status_h[0]) {
            root_tile_ok = false;
            if (t.status_h[1] >= 3) t.rt_skip = std::min(64, 4 * (t.status_h[1] - 2));
        }
    }
    if (root_tile_ok) {
        const auto Y2 = reinterpret_cast<const double2 *>(dY);
        for (int r = 0; r < DUP_ROUNDS; ++r) {
            hipLaunchKernelGGL(dup_store, dim3(ceil_div(n, 256)), dim3(256), 0, st, Y2, n, t.dup_tab, t.dup_mask,
                               t.dup_open, r);
            hipLaunchKernelGGL(dup_probe, dim3(ceil_div(n, 256)), dim3(256), 0, st, Y2, n, t.dup_tab, t.dup_mask,
                               t.dup_open, r, t.dflag);
        }
        hipLaunchKernelGGL(root_tile_check, dim3(1), dim3(1), 0, st, t.dflag, t.bb, t.W, n, theta, t.near_dmax,
                           t.status);
        TSNE_HIP(hipMemcpyAsync(t.status_h, t.status, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        TSNE_HIP(hipStreamSynchronize(st));
        if (t.status_h[0]) {
            t.root_tile = true;
            hipLaunchKernelGGL(root_tile_prep, dim3(std::min<int64_t>(1024, ceil_div(n, 256))), dim3(256), 0, st, t.bb,
                               n, t.nodes, t.mom_cnt, t.mom_off, t.mom_list, t.mom_item, t.meta, t.inv, t.idx_sorted,
                               t.mom_flag);
            const int mgrid = (int)std::min<int64_t>(2048, std::max<int64_t>(1, ceil_div(n, 256)));
            hipLaunchKernelGGL(moment_items<true>, dim3(mgrid), dim3(256), 0, st, Y2, t.nodes, t.mom_off, n,
                               t.mom_item, t.mom_part, nullptr, nullptr);
            hipLaunchKernelGGL(root_moment_reduce, dim3(MOM_K), dim3(256), 0, st, t.mom_off, n, t.mom_part, t.mom);
            hipLaunchKernelGGL(poly_coef, dim3(ceil_div(POLY_K, 128)), dim3(128), 0, st, t.mom, t.rcoef);
            t.root_pos = Y2;
            TSNE_LAUNCH_CHECK();
            return;
        }
        TSNE_HIP(hipMemsetAsync(t.dflag, 0, sizeof(int32_t), st));   // dup_count recomputes it
    }
    hipLaunchKernelGGL(morton_keys, dim3(ceil_div(n, 256)), dim3(256), 0, st, dY, n, t.W, t.keys, t.idx, t.meta);
    TSNE_LAUNCH_CHECK();
    // the previous full build's order buckets the keys (csort.hpp); the first
    // build, small trees and Options::coherent_sort = 0: rocPRIM's sort (the same
    // result: keys ascending, ties by point index)
    if (t.cs.P > 0 && t.cs_primed && ctx->opts.coherent_sort) {
        csort_run(ctx, t.cs, t.keys, t.idx_sorted, t.keys_sorted, t.idx_sorted, st);
    } else {
        size_t tb = t.sort_tmp_bytes;
        morton_sort(t.sort_tmp, tb, t.keys, t.keys_sorted, t.idx, t.idx_sorted, n, st);
    }
    t.cs_primed = true;
    hipLaunchKernelGGL(count_in_root, dim3(1), dim3(64), 0, st, t.keys_sorted, n, t.meta);
    // (trav_front_cur: predictions from the previous traversal's per-point costs,
    // the order made on the second stream while the build goes on)
    const bool cur_order = ctx->opts.trav_front_cur > 0.0 && t.pcost_valid && t.sel_waves == ceil_div(n, 64);
    hipLaunchKernelGGL(gather_sorted, dim3(ceil_div(n, 256)), dim3(256), 0, st, dY, t.idx_sorted, n, t.pos, t.inv,
                       cur_order ? t.pcost : nullptr, cur_order ? t.pred : nullptr);
    t.order_ready = false;
    if (cur_order) {
        TSNE_HIP(hipEventRecord(ctx->aux_ev[0], st));
        TSNE_HIP(hipStreamWaitEvent(ctx->aux_stream, ctx->aux_ev[0], 0));
        hipLaunchKernelGGL(trav_order_cur, dim3(1), dim3(1024), 0, ctx->aux_stream, t.pred, t.nflag, ceil_div(n, 64),
                           ctx->opts.trav_front_cur, t.trav_order);
        if (!t.ord_ev) TSNE_HIP(hipEventCreateWithFlags(&t.ord_ev, hipEventDisableTiming));
        TSNE_HIP(hipEventRecord(t.ord_ev, ctx->aux_stream));
        t.order_ready = true;
    }
    hipLaunchKernelGGL(dup_count, dim3(ceil_div(n, 256)), dim3(256), 0, st, t.pos, t.keys_sorted, n, t.dupc, t.vid,
                       t.dflag);
    if (++t.gen <= 0) {   // wrapped: clear the marks once
        TSNE_HIP(hipMemsetAsync(t.fstart, 0, sizeof(int32_t) * n, st));
        t.gen = 1;
    }
    hipLaunchKernelGGL(karras_build, dim3(ceil_div(n, 256)), dim3(256), 0, st, t.keys_sorted, n, t.meta,
                       t.nodes, t.parent_leaf, t.parent_node, t.arrive, t.arrive2, t.fstart, t.gen, t.top_cnt);
    const double inv_theta = theta > 0.0 ? 1.0 / theta : __builtin_inf();
    hipLaunchKernelGGL(bottom_up_intra, dim3(ceil_div(n, BU_NB)), dim3(BU_NB), 0, st, t.pos, t.meta, t.W, inv_theta,
                       t.nodes, t.agg, t.parent_leaf, t.parent_node, t.fstart, t.gen, t.top_list, t.top_cnt);
    hipLaunchKernelGGL(ctx->opts.bu_acqrel ? bottom_up_top<true> : bottom_up_top<false>,
                       dim3(std::max(1, ctx->cu_count * 4)), dim3(256), 0, st, t.pos, t.meta, t.W,
                       inv_theta, t.nodes, t.agg, t.parent_node, t.arrive, t.top_list, t.top_cnt);
    // exact duplicates: the reference's multiplicities (each kernel returns
    // at once unless dup_count saw a duplicate)
    hipLaunchKernelGGL(dup_bottom_up, dim3(ceil_div(n, 256)), dim3(256), 0, st, t.meta, t.dflag, t.idx_sorted, rowmap,
                       t.vid, t.nodes, t.parent_leaf, t.parent_node, t.arrive2, t.rmin, t.rvid, t.rt2, t.cntcorr,
                       t.sumcorr, t.tiecnt, t.notile, t.vflag, t.vcnt, t.vsum);
    hipLaunchKernelGGL(dup_fixup, dim3(ceil_div(n, 256)), dim3(256), 0, st, t.meta, t.dflag, t.pos, t.keys_sorted,
                       t.dupc, t.idx_sorted, rowmap, t.nodes, t.parent_leaf, t.parent_node, t.rt2, t.cntcorr,
                       t.sumcorr, t.tiecnt, t.notile, t.vflag, t.vcnt, t.vsum);
    hipLaunchKernelGGL(dup_apply, dim3(ceil_div(n, 256)), dim3(256), 0, st, t.meta, t.dflag, t.cntcorr, t.sumcorr,
                       t.vflag, t.vcnt, t.vsum, t.vcntf, t.vcom, t.nodes);
    const DupView dv{t.tiecnt, t.notile, t.vflag, t.vcntf, t.vcom, (int32_t)n};
    hipLaunchKernelGGL(build_qrec, dim3(ceil_div(n, 256)), dim3(256), 0, st, t.nodes, t.pos, t.meta, inv_theta,
                       t.near_dmax, t.dflag, dv, t.qrec);
    // subtree moments for the all-open fast path
    hipLaunchKernelGGL(moment_count, dim3(ceil_div(n + 1, 1024)), dim3(1024), 0, st, t.nodes, n, t.meta, t.mom_flag,
                       t.mom_cnt, t.mom_list, t.meta, t.mom_off, t.mom_item);
    const int mgrid = (int)std::min<int64_t>(2048, std::max<int64_t>(1, ceil_div(n, 256)));
    hipLaunchKernelGGL(moment_items<true>, dim3(mgrid), dim3(256), 0, st, t.pos, t.nodes, t.mom_off, n, t.mom_item,
                       t.mom_part, t.mom_cnt, t.mom);
    hipLaunchKernelGGL(moment_reduce, dim3(mgrid), dim3(256), 0, st, t.meta, t.mom_list, t.mom_cnt, t.mom_off,
                       t.mom_part, t.mom);
    TSNE_LAUNCH_CHECK();
}

void bh_repulsion(tsne_ctx *ctx, BHTree &t, double theta, int64_t s0, int64_t s1,
                  double2 *dF, double *dz, unsigned long long *visits, const int32_t *qlist,
                  unsigned long long *bcost, bool cost_by_label, int32_t *plim) {
    if (s1 <= s0) return;
    hipStream_t st = ctx->stream;
    const double mom_tol = ctx->opts.mom_tol;
    if (t.root_tile) {
        if (visits)
            hipLaunchKernelGGL(root_tile_eval<true>, dim3(ceil_div(s1 - s0, 256)), dim3(256), 0, st, t.root_pos,
                               t.nodes, t.rcoef, t.meta, s0, s1, qlist, dF, dz, visits, mom_tol);
        else
            hipLaunchKernelGGL(root_tile_eval<false>, dim3(ceil_div(s1 - s0, 256)), dim3(256), 0, st, t.root_pos,
                               t.nodes, t.rcoef, t.meta, s0, s1, qlist, dF, dz, visits, mom_tol);
        TSNE_LAUNCH_CHECK();
        return;
    }
    // counters only when asked for: visits need every counter, the multi-GPU
    // cost buckets only the waves' run times
    const int mode = visits ? 2 : (bcost ? 1 : 0);
    auto kern = plim ? (mode == 2 ? bh_traverse<2, true, false> : mode == 1 ? bh_traverse<1, true, false>
                                                                         : bh_traverse<0, true, false>)
                     : (mode == 2 ? bh_traverse<2, false, false> : mode == 1 ? bh_traverse<1, false, false>
                                                                           : bh_traverse<0, false, false>);
    auto tkern = mode == 2 ? bh_traverse<2, false, true> : mode == 1 ? bh_traverse<1, false, true>
                                                                     : bh_traverse<0, false, true>;
    const int64_t waves = ceil_div(s1 - s0, 64), nblocks = ceil_div(waves, TRAV_WPB);
    TSNE_REQUIRE(waves <= t.tile_waves, "tile task lists sized for fewer queries");
    // heavy groups: selected after the previous traversal of the same query
    // count from its costs (narrow_select at the end of this function, so
    // that nothing delays this traversal's dispatch behind the tree build);
    // none on a tree's first traversal or with Options::narrow = 0
    NarrowView nv;
    unsigned long long *wlog = visits && ctx->opts.wave_log ? ctx->ws.get<unsigned long long>("rep.wavelog", 1 + 2 * WAVE_LOG_CAP)
                                                             : nullptr;
    nv.wlog = wlog;
    const double nfac = ctx->opts.narrow;
    // (not with a tree partition: every rank walks all queries, the 64-query grid fills the chip)
    const bool narrow = nfac > 0.0 && t.sel_waves == waves && !plim;
    if (narrow) {
        nv.hlist = t.hlist; nv.hcount = t.hcount; nv.ncost = t.ncost; nv.mtask = t.nmtask; nv.mtask_n = t.nmtask_n;
        nv.nflag = t.nflag;
        nv.nbn = (int32_t)ceil_div(t.nar_hmax * NPARTS, 4);
    }
    t.ran_narrow = narrow;
    // work splitting of long walks (see "Spill"): budgets from the previous
    // traversal of the same query count (spill_budget), or forced (tests)
    const Options &o = ctx->opts;
    const bool spill = !plim && (o.spill_force > 0 || (o.spill > 0.0 && t.sp_waves == waves));
    SpillView sv;
    if (spill) {
        bh_spill_alloc(ctx, t);
        ++t.sp_gen;
        sv.ctl = t.sp_ctl; sv.task = t.sp_task; sv.ent = t.sp_ent; sv.gflag = t.sp_gflag; sv.acc = t.sp_acc;
        sv.pg_tiles = t.sp_pg_tiles; sv.pg_grp = t.sp_pg_grp; sv.pg_n = t.sp_pg_n;
        sv.cap = t.sp_cap; sv.pg_cap = t.sp_pg_cap; sv.gen = t.sp_gen;
        sv.lin = 0;
        sv.lout = 1;
        sv.force = o.spill_force;
    }
    t.ran_spill = spill;
    // tile streaming (see "Tile streaming"): one rank's own queries only (a
    // rank's list, a tree partition and spill keep the slot path)
    StreamView stv;
    const bool stream = o.tile_stream > 0 && !plim && !spill && !qlist;
    const int cblocks = std::max(1, ctx->cu_count * o.tile_stream);
    if (stream) {
        bh_stream_alloc(ctx, t);
        stv.ctl = t.st_ctl;
        stv.gen = ++t.st_gen;
        if (t.st_gen >= (1 << 29)) t.st_gen = 1;   // (claims hold gen << 2; 0: never claimed)
        stv.gen = t.st_gen;
        stv.maxcost = o.tile_stream_max;
        stv.wait = o.tile_stream_wait;
        stv.total = (int32_t)(nblocks * TRAV_WPB);
        stv.cap = (int32_t)t.tile_waves;
        // ungated, the consumers' stream starts behind everything before the
        // traversal (gated, the traversal's start implies that; and no marker
        // goes between the build and the traversal on this stream, which lets
        // the side stream's attraction reach the CUs first)
        if (!o.tile_stream_gate) {
            TSNE_HIP(hipEventRecord(ctx->st_ev[0], st));
            TSNE_HIP(hipStreamWaitEvent(ctx->st_stream, ctx->st_ev[0], 0));
        }
    }
    t.ran_stream = stream;
    stv.prio = o.trav_prio;   // (also without streaming)
    if (o.trav_front > 0.0 && narrow && t.front_waves == waves) stv.border = t.trav_order;
    if (t.order_ready && narrow && !plim && !qlist && s0 == 0 && waves == ceil_div(t.n, 64)) {
        TSNE_HIP(hipStreamWaitEvent(st, t.ord_ev, 0));   // (done long before: made during the build)
        stv.border = t.trav_order;
    }
    stv.wlog = wlog;
    const int32_t *clab = cost_by_label ? t.idx_sorted : nullptr;
    if (narrow) {   // the narrow waves on the second stream, beside the 64-query grid
        TSNE_HIP(hipEventRecord(ctx->aux_ev[0], st));
        TSNE_HIP(hipStreamWaitEvent(ctx->aux_stream, ctx->aux_ev[0], 0));
        auto nk = mode == 2 ? bh_traverse_narrow<2> : mode == 1 ? bh_traverse_narrow<1> : bh_traverse_narrow<0>;
        hipLaunchKernelGGL(nk, dim3(nv.nbn), dim3(256), 0, ctx->aux_stream, t.pos, t.dupc, t.nodes, t.qrec, t.ttask_n,
                           t.meta, t.mom_flag, mom_tol, theta, s0, s1, qlist, (int32_t)t.n, dF, dz, visits, bcost,
                           t.tcost, clab, nv);
        TSNE_HIP(hipEventRecord(ctx->aux_ev[1], ctx->aux_stream));
    }
    hipLaunchKernelGGL(kern, dim3(nblocks), dim3(64 * TRAV_WPB), 0, st, t.pos, t.dupc, t.nodes, t.qrec, t.ttask, t.ttask_n,
                       t.meta, t.mom_flag, mom_tol, theta, s0, s1, qlist, (int32_t)t.n, dF, dz, visits, bcost, t.wcost,
                       t.tcost, clab, nv, plim, sv, stv);
    if (stream) {   // the consumers beside the traversal, then their moments and sums into F, Z
        // (tile_stream_gate: dispatched once every traversal block has started,
        // so that they take the slots its tail frees, not slots its blocks need)
        if (o.tile_stream_gate)
            TSNE_HIP(hipStreamWaitValue32(ctx->st_stream, t.st_ctl + ST_STARTED, (uint32_t)nblocks,
                                          hipStreamWaitValueGte, 0xffffffffu));
        ChunkView scv;
        scv.Fp = t.st_Dp;
        scv.Zp = t.st_Dz;
        hipLaunchKernelGGL(tile_apply<2>, dim3(cblocks), dim3(256), 0, ctx->st_stream, t.pos, t.nodes, t.ttask,
                           t.ttask_n, s0, s1, qlist, t.mom_flag, mom_tol, t.st_mtask, t.st_mtask_n, dF, dz, visits,
                           nullptr, scv, t.mom, SpillView(), stv, t.tcost);
        // (F, Z of the traversal itself: read after its launch has ended)
        TSNE_HIP(hipEventRecord(ctx->st_ev[2], st));
        TSNE_HIP(hipStreamWaitEvent(ctx->st_stream, ctx->st_ev[2], 0));
        hipLaunchKernelGGL(stream_finish, dim3(ceil_div((int64_t)stv.total * 64, 256)), dim3(256), 0, ctx->st_stream,
                           t.pos, t.nodes, t.mom, t.st_ctl, t.st_mtask, t.st_mtask_n, t.st_Dp, t.st_Dz, s0, s1,
                           dF, dz, stv.cap, stv.gen);
        // the per-call words zeroed for the next call (after the traversal and the consumers)
        TSNE_HIP(hipMemsetAsync(t.st_ctl, 0, sizeof(int32_t) * ST_RESET, ctx->st_stream));
        TSNE_HIP(hipEventRecord(ctx->st_ev[1], ctx->st_stream));
    }
    // the levels' tasks: drain launch l takes level l (one wave per slot),
    // splitting into level l + 1; the last one without splits
    const int levels = std::min(o.spill_drains, SP_LMAX);
    for (int d = 1; spill && d <= levels; ++d) {
        SpillView dv = sv;
        dv.lin = d;
        dv.lout = d < levels ? d + 1 : 0;
        hipLaunchKernelGGL(tkern, dim3(std::max(1, ctx->cu_count * 32 / TRAV_WPB)), dim3(64 * TRAV_WPB), 0, st, t.pos,
                           t.dupc, t.nodes,
                           t.qrec, t.ttask, t.ttask_n, t.meta, t.mom_flag, mom_tol, theta, s0, s1, qlist, (int32_t)t.n,
                           dF, dz, visits, bcost, t.wcost, t.tcost, clab, nv, plim, dv, StreamView());
    }
    // tile chunks of heavy waves (ChunkView): the single-workgroup plan while
    // the per-wave costs fit its LDS, else the multi-launch plan and block sort
    ChunkView cv;
    const int64_t tslots = std::min<int64_t>(t.tile_waves, waves + waves / 2 + 64);
    const int32_t *torder = t.torder;
    if (waves <= PLAN_WAVES_MAX && ceil_div(tslots, 4) <= PLAN_BLOCKS_MAX) {
        hipLaunchKernelGGL(tile_plan, dim3(1), dim3(1024), 0, st, t.tcost, waves, tslots, t.ch_C, t.ch_slot0,
                           t.ch_slot_w, t.ch_slot_c, t.ch_nslots, t.torder, stream ? t.st_ctl + ST_Q0 : nullptr,
                           stv.gen, stream ? t.st_ctl + ST_W : nullptr, o.tile_stream_frac);
    } else {
        const int64_t wb = ceil_div(waves + 1, 256);
        TSNE_HIP(hipMemsetAsync(t.ch_total, 0, sizeof(unsigned long long), st));
        hipLaunchKernelGGL(chunk_total, dim3(wb), dim3(256), 0, st, t.tcost, waves, t.ch_total);
        hipLaunchKernelGGL(chunk_parts, dim3(wb), dim3(256), 0, st, t.tcost, t.ch_total, waves, t.ch_C,
                           stream ? t.st_ctl + ST_Q0 : nullptr, stv.gen, stream ? t.st_ctl + ST_W : nullptr,
                           o.tile_stream_frac);
        size_t tb = t.ch_scan_bytes;
        TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(t.ch_scan_tmp, tb, t.ch_C, t.ch_slot0, (int)(waves + 1), st));
        hipLaunchKernelGGL(chunk_fill, dim3(wb), dim3(256), 0, st, t.ch_C, t.ch_slot0, t.tcost, waves, t.ch_slot_w,
                           t.ch_slot_c, t.ch_scost, tslots, t.ch_nslots);
        block_order(ctx, t, t.ch_scost, tslots, ceil_div(tslots, 4), t.torder);
    }
    cv.slot_w = t.ch_slot_w; cv.slot_c = t.ch_slot_c; cv.nslots = t.ch_nslots;
    cv.Fp = t.ch_Fp; cv.Zp = t.ch_Zp;
    hipLaunchKernelGGL(tile_apply<0>, dim3(ceil_div(tslots, 4)), dim3(256), 0, st, t.pos, t.nodes, t.ttask,
                       t.ttask_n, s0, s1, qlist, t.mom_flag, mom_tol, t.mtask, t.mtask_n, dF, dz, visits, torder, cv,
                       t.mom, SpillView(), stv, t.tcost);
    hipLaunchKernelGGL(moment_apply, dim3(ceil_div(tslots * 64, 256)), dim3(256), 0, st, t.pos, t.nodes, t.mom,
                       t.mtask, t.mtask_n, s0, s1, qlist, dF, dz, cv);
    const bool keep_pcost = o.trav_front_cur > 0.0 && !plim && !qlist && s0 == 0 && s1 == t.n;
    if (keep_pcost) {
        t.pcost = ctx->ws.get<int32_t>(t.pre + "pcost", (size_t)t.n);
        t.pred = ctx->ws.get<int32_t>(t.pre + "pred", (size_t)ceil_div(t.n, 64) + 1);
        t.trav_order = ctx->ws.get<int32_t>(t.pre + "trav_order", ceil_div(t.tile_waves, TRAV_WPB) + 1);
    }
    hipLaunchKernelGGL(chunk_combine, dim3(ceil_div(s1 - s0, 256)), dim3(256), 0, st, t.ch_Fp, t.ch_Zp, t.ch_C,
                       t.ch_slot0, s0, s1, qlist, dF, dz, keep_pcost ? t.pcost : nullptr, t.idx_sorted, t.wcost,
                       narrow ? t.nflag : nullptr);
    t.pcost_valid = keep_pcost;
    if (spill) {   // the tasks' tile pages, then their sums into F, Z
        hipLaunchKernelGGL(tile_apply<1>, dim3(std::max(1, ctx->cu_count * 4)), dim3(256), 0, st, t.pos, t.nodes,
                           t.ttask, t.ttask_n, s0, s1, qlist, t.mom_flag, mom_tol, t.mtask, t.mtask_n, dF, dz, visits,
                           nullptr, ChunkView(), t.mom, sv, StreamView(), t.tcost);
        hipLaunchKernelGGL(spill_combine, dim3(ceil_div(s1 - s0, 256)), dim3(256), 0, st, t.sp_gflag, t.sp_gen,
                           t.sp_acc, s0, s1, qlist, dF, dz, t.sp_ctl);
    }
    // the narrow waves' own queries from here on (their F / Z entries are
    // disjoint from the 64-query waves' above, so the tiles did not wait for them)
    if (narrow) {
        TSNE_HIP(hipStreamWaitEvent(st, ctx->aux_ev[1], 0));
        hipLaunchKernelGGL(narrow_moment_apply, dim3(ceil_div(t.nar_hmax * 64, 256)), dim3(256), 0, st, t.pos,
                           t.nodes, t.mom, t.hlist, t.hcount, t.nmtask, t.nmtask_n, s0, s1, qlist, dF, dz);
        TSNE_HIP(hipMemcpyAsync(t.hran, t.hcount, sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    }
    // the next traversal's heavy groups (of the same query count) from this one's costs
    if (nfac > 0.0 && !plim) {
        if (!narrow) TSNE_HIP(hipMemsetAsync(t.nflag, 0, sizeof(int32_t) * waves, st));   // no stale slots
        const bool front = o.trav_front > 0.0;
        if (front) t.trav_order = ctx->ws.get<int32_t>(t.pre + "trav_order", ceil_div(t.tile_waves, TRAV_WPB) + 1);
        hipLaunchKernelGGL(narrow_select, dim3(1), dim3(1024), 0, st, t.wcost, waves, t.nflag, t.ncost, t.hlist,
                           t.hcount, t.nar_hmax, nfac, std::min<int64_t>(t.nar_hmax, narrow_fill(ctx, waves)),
                           front ? t.trav_order : nullptr, o.trav_front);
        t.sel_waves = waves;
        t.front_waves = front ? waves : 0;
    } else {
        t.sel_waves = 0;
        t.front_waves = 0;
    }
    // the next traversal's split budgets (of the same query count) from this one's costs
    if (o.spill > 0.0 && o.spill_force == 0 && !plim) {
        bh_spill_alloc(ctx, t);
        hipLaunchKernelGGL(spill_budget, dim3(1), dim3(1024), 0, st, t.wcost, waves, o.spill, o.spill_task,
                           (int32_t)o.spill_min, t.sp_ctl);
        t.sp_waves = waves;
    } else {
        t.sp_waves = 0;
    }
    // the streamed lists' sums are in F, Z (and the control words zeroed)
    // before anything after this call reads them
    if (stream) TSNE_HIP(hipStreamWaitEvent(st, ctx->st_ev[1], 0));
    TSNE_LAUNCH_CHECK();
}

void part_align(tsne_ctx *ctx, BHTree &t, const int64_t *cuts, int world, int rank, int32_t *plim) {
    TSNE_REQUIRE(world <= 64, "tree partition: at most 64 ranks");
    TSNE_REQUIRE(2 * t.n < (int64_t)REF_FORCED, "tree partition: too many points for the record flags");
    hipLaunchKernelGGL(part_align_kernel, dim3(1), dim3(64), 0, ctx->stream, t.keys_sorted, t.meta, cuts, world, rank,
                       plim);
    TSNE_LAUNCH_CHECK();
}

void part_recut(tsne_ctx *ctx, const unsigned long long *cost, int world, int64_t n, int64_t *cuts) {
    hipLaunchKernelGGL(part_recut_kernel, dim3(1), dim3(64), 0, ctx->stream, cost, world, n, cuts);
    TSNE_LAUNCH_CHECK();
}

void part_cost(tsne_ctx *ctx, BHTree &t, int64_t waves, unsigned long long *out) {
    hipLaunchKernelGGL(part_cost_kernel, dim3(1), dim3(1024), 0, ctx->stream, t.wcost, waves, out);
    TSNE_LAUNCH_CHECK();
}

}  // namespace tsne
