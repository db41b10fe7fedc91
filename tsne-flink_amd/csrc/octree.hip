// octree.hip -- Barnes-Hut octree build + traversal for 3-D embeddings on
// gfx950 (the SURVEY.md 8f extension of QuadTree.scala:38-152 /
// Cell.scala:31-36 to nComponents = 3; restated in oracle/tsne_oracle.c).
//
// Same equivalence argument as bhtree.hip: Morton digits replay the cell
// arithmetic (child centres c -/+ 0.5 h, closed containment tried in the
// order upper NW, NE, SW, SE, lower NW, NE, SW, SE), so cells are the
// restatement's; a cell whose points all sit in one child forms a chain
// summarised at its deepest cell (the criterion is monotone along it);
// leaves interact directly, a leaf equal to the query contributes nothing;
// points outside the root cell are queries only.  Deviations:
// exact duplicates count with full multiplicity, cells deeper than 21 levels
// are not split (all their points interact directly), and subtrees entirely
// within D <= near_dmax of a query are summed exactly (<= Options::
// near_tol3_early (1e-7) / near_tol3_late (5e-6: C4 loop 29.7 -> 19.5 s,
// losses to 6 digits) relative from the restatement's cell sums).
//
// The traversal is the 2-D design without its quad-collapsed records and
// moments: a wave of 64 Morton-consecutive queries shares an LDS stack of
// (node, lane mask); per popped node each lane first tries the all-open /
// near-exact tile test (exact leaf sum over the node's contiguous range,
// points staged through LDS), then evaluates the node's two binary children.
#include <hipcub/hipcub.hpp>

#include "bhtree.hpp"   // qacc_open / qacc_accept (the records' child bounds)
#include "octree.hpp"

namespace tsne {
namespace {

constexpr int LEVELS3 = 21;                 // 63 key bits
constexpr uint64_t OUT_KEY3 = 1ull << 63;   // outside the root cell: sorts last
constexpr int STACK3 = 256;                 // single pops, <= 2 pushes each: depth-bounded
constexpr int AGG3 = 12;                    // sx, sy, sz, x0, x1, y0, y1, z0, z1, hmin, cnt, rball

__global__ void bbox3_partial(const double *__restrict__ Y, int64_t n, double *__restrict__ part) {
    __shared__ double sm[4][6];
    double mn[3], mx[3];
    for (int k = 0; k < 3; ++k) { mn[k] = __builtin_inf(); mx[k] = -__builtin_inf(); }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        for (int k = 0; k < 3; ++k) { mn[k] = fmin(mn[k], Y[3 * i + k]); mx[k] = fmax(mx[k], Y[3 * i + k]); }
    const int w = threadIdx.x >> 6;
    for (int k = 0; k < 3; ++k) {
        mn[k] = wave_min(mn[k]);
        mx[k] = wave_max(mx[k]);
        if (lane_id() == 0) { sm[w][2 * k] = mn[k]; sm[w][2 * k + 1] = mx[k]; }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int v = 1; v < 4; ++v)
            for (int k = 0; k < 3; ++k) {
                sm[0][2 * k] = fmin(sm[0][2 * k], sm[v][2 * k]);
                sm[0][2 * k + 1] = fmax(sm[0][2 * k + 1], sm[v][2 * k + 1]);
            }
        for (int k = 0; k < 6; ++k) part[blockIdx.x * 6 + k] = sm[0][k];
    }
}

__global__ void bbox3_final(const double *__restrict__ part, int nb, double *__restrict__ W,
                            int32_t *__restrict__ meta) {
    __shared__ double sm[4][6];
    double mn[3], mx[3];
    for (int k = 0; k < 3; ++k) { mn[k] = __builtin_inf(); mx[k] = -__builtin_inf(); }
    for (int b = threadIdx.x; b < nb; b += blockDim.x)
        for (int k = 0; k < 3; ++k) { mn[k] = fmin(mn[k], part[6 * b + 2 * k]); mx[k] = fmax(mx[k], part[6 * b + 2 * k + 1]); }
    const int w = threadIdx.x >> 6;
    for (int k = 0; k < 3; ++k) {
        mn[k] = wave_min(mn[k]);
        mx[k] = wave_max(mx[k]);
        if (lane_id() == 0) { sm[w][2 * k] = mn[k]; sm[w][2 * k + 1] = mx[k]; }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int v = 1; v < 4; ++v)
            for (int k = 0; k < 3; ++k) {
                sm[0][2 * k] = fmin(sm[0][2 * k], sm[v][2 * k]);
                sm[0][2 * k + 1] = fmax(sm[0][2 * k + 1], sm[v][2 * k + 1]);
            }
        const double a = sm[0][1] - sm[0][0], b = sm[0][3] - sm[0][2], c = sm[0][5] - sm[0][4];
        const double ab = a > b ? a : b;
        *W = ab > c ? ab : c;   // max(maxX - minX, maxY - minY, maxZ - minZ)
        meta[0] = 0;
    }
}

// fixed-point digits away from cell boundaries (see bhtree.hip quant_digits):
// 21 levels, band 1e-4 of a level-21 cell
__device__ __forceinline__ bool quant21(double p, double W, uint32_t &q) {
    const double t = (p + W) / (2.0 * W) * 2097152.0;   // 2^21
    if (!(t >= 0.0 && t < 2097152.0)) return false;
    const double f = floor(t);
    const double fr = t - f;
    if (fr < 1e-4 || fr > 1.0 - 1e-4) return false;
    q = (uint32_t)f;
    return true;
}

// digit c = 4 lower + 2 south + east, tried in ascending c (the child order)
__global__ void morton3_keys(const double *__restrict__ Y, int64_t n, const double *__restrict__ Wp,
                             uint64_t *__restrict__ keys, int32_t *__restrict__ idx, int32_t *__restrict__ meta) {
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i0 < n;
    const int64_t i = live ? i0 : n - 1;
    const double W = *Wp;
    const double px = Y[3 * i], py = Y[3 * i + 1], pz = Y[3 * i + 2];
    double x = 0.0, y = 0.0, z = 0.0, h = W;
    bool in = live && (__dsub_rn(x, h) <= px) && (__dadd_rn(x, h) >= px) && (__dsub_rn(y, h) <= py) &&
              (__dadd_rn(y, h) >= py) && (__dsub_rn(z, h) <= pz) && (__dadd_rn(z, h) >= pz);
    uint64_t key = 0;
    uint32_t qx, qy, qz;
    if (in && W > 0.0 && quant21(px, W, qx) && quant21(py, W, qy) && quant21(pz, W, qz)) {
        for (int l = LEVELS3 - 1; l >= 0; --l) {
            const uint32_t east = (qx >> l) & 1u, south = 1u - ((qy >> l) & 1u), lower = 1u - ((qz >> l) & 1u);
            key = (key << 3) | (uint64_t)(4u * lower + 2u * south + east);
        }
    } else if (in) {
        for (int l = 0; l < LEVELS3; ++l) {
            const double nh = __dmul_rn(0.5, h);
            const double xw = __dsub_rn(x, nh), xe = __dadd_rn(x, nh);
            const double yn = __dadd_rn(y, nh), ys = __dsub_rn(y, nh);
            const double zu = __dadd_rn(z, nh), zl = __dsub_rn(z, nh);
            const bool inW = (__dsub_rn(xw, nh) <= px) && (__dadd_rn(xw, nh) >= px);
            const bool inE = (__dsub_rn(xe, nh) <= px) && (__dadd_rn(xe, nh) >= px);
            const bool inN = (__dsub_rn(yn, nh) <= py) && (__dadd_rn(yn, nh) >= py);
            const bool inS = (__dsub_rn(ys, nh) <= py) && (__dadd_rn(ys, nh) >= py);
            const bool inU = (__dsub_rn(zu, nh) <= pz) && (__dadd_rn(zu, nh) >= pz);
            const bool inL = (__dsub_rn(zl, nh) <= pz) && (__dadd_rn(zl, nh) >= pz);
            int c = 7;   // lower SE, or a rounding gap (see bhtree.hip)
            for (int t = 0; t < 8; ++t) {
                const bool ok = ((t & 1) ? inE : inW) && ((t & 2) ? inS : inN) && ((t & 4) ? inL : inU);
                if (ok) { c = t; break; }
            }
            x = (c & 1) ? xe : xw;
            y = (c & 2) ? ys : yn;
            z = (c & 4) ? zl : zu;
            h = nh;
            key = (key << 3) | (uint64_t)c;
        }
    } else {
        key = OUT_KEY3;
    }
    if (live) {
        keys[i] = key;
        idx[i] = (int32_t)i;
    }
    (void)meta;   // in-root count: count_in_root3 on the sorted keys
}

// m = index of the first OUT_KEY3 in the sorted keys (64-ary search by one
// wave; see bhtree.hip count_in_root)
__global__ void count_in_root3(const uint64_t *__restrict__ ks, int64_t n, int32_t *__restrict__ meta) {
    const int lane = lane_id();
    int64_t lo = 0, hi = n;
    while (hi > lo) {
        const int64_t step = (hi - lo + 63) / 64;
        const int64_t p = lo + (int64_t)lane * step;
        const bool out = p >= hi || ks[p] >= OUT_KEY3;
        const uint64_t b = __ballot(out);
        const int f = b ? __ffsll((long long)b) - 1 : 64;
        if (f == 0) break;
        const int64_t nlo = lo + (int64_t)(f - 1) * step + 1;
        hi = min(hi, lo + (int64_t)f * step);
        lo = nlo;
    }
    if (lane == 0) meta[0] = (int32_t)lo;
}

__global__ void gather3(const double *__restrict__ Y, const int32_t *__restrict__ idx_sorted, int64_t n,
                        double4 *__restrict__ pos, int32_t *__restrict__ inv) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const int32_t i = idx_sorted[s];
    pos[s] = make_double4(Y[3 * i], Y[3 * i + 1], Y[3 * i + 2], 0.0);
    inv[i] = (int32_t)s;
}

__global__ void dup_count3(const double4 *__restrict__ pos, const uint64_t *__restrict__ keys, int64_t n,
                           int32_t *__restrict__ dupc) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const double4 q = pos[s];
    const uint64_t k = keys[s];
    int32_t c = 1;
    for (int64_t t = s - 1; t >= 0 && keys[t] == k; --t) {
        const double4 p = pos[t];
        c += (p.x == q.x && p.y == q.y && p.z == q.z);
    }
    for (int64_t t = s + 1; t < n && keys[t] == k; ++t) {
        const double4 p = pos[t];
        c += (p.x == q.x && p.y == q.y && p.z == q.z);
    }
    dupc[s] = c;
}

// common-prefix bits of sorted keys i and j within the 63-bit Morton field
// (ties extend with the index bits); -1 out of range
__device__ __forceinline__ int kdelta3(const uint64_t *__restrict__ k, int m, int i, int j) {
    if (j < 0 || j >= m) return -1;
    const uint64_t a = k[i], b = k[j];
    if (a == b) return 63 + __clz((unsigned)(i ^ j));
    return __clzll((long long)(a ^ b)) - 1;
}

__global__ void karras3(const uint64_t *__restrict__ k, const int32_t *__restrict__ meta, OctNode *__restrict__ nodes,
                        int32_t *__restrict__ parent_leaf, int32_t *__restrict__ parent_node,
                        int32_t *__restrict__ arrive) {
    const int m = meta[0];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m - 1) return;
    arrive[i] = 0;
    const int dr = kdelta3(k, m, i, i + 1), dl = kdelta3(k, m, i, i - 1);
    const int d = (dr > dl) ? 1 : -1;
    const int dmin = d > 0 ? dl : dr;
    int lmax = 2;
    while (kdelta3(k, m, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (kdelta3(k, m, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = kdelta3(k, m, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (kdelta3(k, m, i, i + (s + t) * d) > dnode) s += t;
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
}

__device__ __forceinline__ void st_sys3(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double ld_sys3(const double *p) {
    return __hip_atomic_load(const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Bottom-up sums / boxes / hmin / rball (bhtree.hip bottom_up, one more axis;
// the same LDS hand-off for nodes inside the workgroup's BLK leaves).
template <int BLK>
__global__ __launch_bounds__(BLK) void bottom_up3(const double4 *__restrict__ pos, const int32_t *__restrict__ meta,
                           const double *__restrict__ Wp, double inv_theta, OctNode *nodes, double *agg,
                           const int32_t *__restrict__ parent_leaf, const int32_t *__restrict__ parent_node,
                           int32_t *arrive) {
    __shared__ double lagg[AGG3][BLK];
    __shared__ int32_t larr[BLK];
    const int m = meta[0];
    const int S0 = blockIdx.x * BLK;
    larr[threadIdx.x] = 0;
    __syncthreads();
    const int s = S0 + threadIdx.x;
    if (s >= m || m < 2) return;
    const double W = *Wp;
    auto in_blk = [&](int q) { return nodes[q].first >= S0 && nodes[q].last < S0 + BLK; };
    int p = parent_leaf[s];
    bool intra = p >= 0 && in_blk(p);
    while (p >= 0) {
        if (intra) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (__hip_atomic_fetch_add(&larr[p - S0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
                return;
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (__hip_atomic_fetch_add(&arrive[p], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
        }
        const int32_t ch[2] = {nodes[p].left, nodes[p].right};
        const int32_t dl = nodes[p].delta;
        double a[2][10];   // sx, sy, sz, x0, x1, y0, y1, z0, z1, hmin
        double c[2], rb[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (ch[k] < 0) {
                const double4 q = pos[~ch[k]];
                a[k][0] = q.x; a[k][1] = q.y; a[k][2] = q.z;
                a[k][3] = q.x; a[k][4] = q.x; a[k][5] = q.y; a[k][6] = q.y; a[k][7] = q.z; a[k][8] = q.z;
                a[k][9] = __builtin_inf();
                c[k] = 1.0;
                rb[k] = __builtin_inf();
            } else if (intra) {
                const int o = ch[k] - S0;
#pragma unroll
                for (int f = 0; f < 10; ++f) a[k][f] = lagg[f][o];
                c[k] = lagg[10][o];
                rb[k] = lagg[11][o];
            } else {
                const double *g = agg + AGG3 * (int64_t)ch[k];
#pragma unroll
                for (int f = 0; f < 10; ++f) a[k][f] = ld_sys3(g + f);
                c[k] = ld_sys3(g + 10);
                rb[k] = ld_sys3(g + 11);
            }
        }
        const double cnt = c[0] + c[1];
        const double sx = a[0][0] + a[1][0], sy = a[0][1] + a[1][1], sz = a[0][2] + a[1][2];
        const double x0 = fmin(a[0][3], a[1][3]), x1 = fmax(a[0][4], a[1][4]);
        const double y0 = fmin(a[0][5], a[1][5]), y1 = fmax(a[0][6], a[1][6]);
        const double z0 = fmin(a[0][7], a[1][7]), z1 = fmax(a[0][8], a[1][8]);
        const int par = parent_node[p];
        const int dlev = dl / 3;
        bool real;
        if (dl >= 63) real = false;                       // keys tie below 21 levels
        else if (par < 0) real = true;                    // root cell chain
        else real = (nodes[par].delta / 3) < dlev;        // first node of its level
        const double h = real ? ldexp(W, -dlev) : -1.0;
        const double hmin = fmin(real ? h : __builtin_inf(), fmin(a[0][9], a[1][9]));
        const double cx = sx / cnt, cy = sy / cnt, cz = sz / cnt;
        double rball = real ? sqrt(h * inv_theta) : __builtin_inf();
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (ch[k] >= 0) {
                const double ex = cx - a[k][0] / c[k], ey = cy - a[k][1] / c[k], ez = cz - a[k][2] / c[k];
                rball = fmin(rball, rb[k] - sqrt(ex * ex + ey * ey + ez * ez));
            }
        }
        rball = rball > 0.0 ? rball * (1.0 - 1e-9) : 0.0;
        const bool pintra = par >= 0 && in_blk(par);
        if (pintra) {
            const int o = p - S0;
            lagg[0][o] = sx; lagg[1][o] = sy; lagg[2][o] = sz;
            lagg[3][o] = x0; lagg[4][o] = x1; lagg[5][o] = y0; lagg[6][o] = y1;
            lagg[7][o] = z0; lagg[8][o] = z1; lagg[9][o] = hmin;
            lagg[10][o] = cnt; lagg[11][o] = rball;
        } else {
            double *g = agg + AGG3 * (int64_t)p;
            st_sys3(g + 0, sx); st_sys3(g + 1, sy); st_sys3(g + 2, sz);
            st_sys3(g + 3, x0); st_sys3(g + 4, x1); st_sys3(g + 5, y0); st_sys3(g + 6, y1);
            st_sys3(g + 7, z0); st_sys3(g + 8, z1); st_sys3(g + 9, hmin);
            st_sys3(g + 10, cnt); st_sys3(g + 11, rball);
        }
        OctNode &nd = nodes[p];
        nd.cx = cx; nd.cy = cy; nd.cz = cz;
        nd.cnt = (int32_t)cnt;
        nd.h = h;
        nd.hmin = hmin;
        nd.rball = rball;
        nd.bx0 = x0; nd.bx1 = x1; nd.by0 = y0; nd.by1 = y1; nd.bz0 = z0; nd.bz1 = z1;
        p = par;
        intra = pintra;
    }
}

__global__ void set_root3(int32_t *meta) {
    const int m = meta[0];
    meta[1] = (m >= 2) ? 0 : (m == 1 ? ~0 : INT32_MIN);
}

// 1 / x for the BH terms: v_rcp_f64 + one Newton step, within 11 ulp of the
// IEEE quotient (bhtree.hip recip_bh, scripts/rcp_accuracy.hip): ~2e-15
// relative per term, two fp64 ops per term cheaper than the second step
__device__ __forceinline__ double rcp2(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    return __fma_rn(r, __fma_rn(-x, r, 1.0), r);
}

// a leaf point (zero if equal to the query)
__device__ __forceinline__ void leaf3(double qx, double qy, double qz, double px, double py, double pz, double &fx,
                                      double &fy, double &fz, double &zs) {
    if (px == qx && py == qy && pz == qz) return;
    const double dx = qx - px, dy = qy - py, dz = qz - pz;
    const double r = rcp2(1.0 + (dx * dx + dy * dy + dz * dz));
    const double sc = r * r;
    fx = __fma_rn(sc, dx, fx);
    fy = __fma_rn(sc, dy, fy);
    fz = __fma_rn(sc, dz, fz);
    zs += r;
}

// a summarised cell: Q = 1/(1+D), m = n Q, F += m Q (q - com)
__device__ __forceinline__ void cell3(double dx, double dy, double dz, double D, int32_t n, double &fx, double &fy,
                                      double &fz, double &zs) {
    const double Q = rcp2(1.0 + D);
    const double mult = (double)n * Q;
    const double sc = mult * Q;
    fx = __fma_rn(sc, dx, fx);
    fy = __fma_rn(sc, dy, fy);
    fz = __fma_rn(sc, dz, fz);
    zs += mult;
}

// fl(h / D) < theta (bhtree.hip summarise, 3-D D)
__device__ __forceinline__ bool summarise3(double h, double dx, double dy, double dz, double th_lo, double th_hi,
                                           double theta) {
    const double D = __dadd_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)), __dmul_rn(dz, dz));
    if (h < th_lo * D) return true;
    if (h > th_hi * D) return false;
    return h / D < theta;
}

// ---- Subtree moments in 3-D (the 2-D moment path of bhtree.hip, restated
// for the octree).  For a node with box centre c and a query q: v = q - c,
// A = |v|^2, B = 1 / (1 + A), and per point P = p - c, s = |P|^2,
// delta = D - A = s - 2 v.P.  Then
//   1 / (1 + D) = B sum_k (-B delta)^k,
//   z = B sum_k (-B)^k T_k,            T_k = sum_p delta^k,
//   F = B^2 sum_k (k + 1) (-B)^k (v T_k - U_k),   U_k = sum_p P delta^k,
// and T_k, U_k are polynomials in v whose coefficients are the moments
// M(a; b) = sum_p s^a P^b (a + |b| <= MOM3_ORDER + 1).  Truncated at
// k <= MOM3_ORDER; with rho = B (R^2 + 2 |v| R) >= |B delta| (R: the box's
// half-diagonal) the remainder is below (K + 2) rho^(K+1) / (1 - rho)^2
// relative, taken only when that is <= Options::mom3_tol (1e-12).  A
// subtree evaluated this way is one the traversal sums exactly (an all-open or
// near-exact tile), so the result equals that exact leaf sum to 1e-14.
constexpr int MOM3_ORDER = 3;
constexpr int MOM3_K = 70;          // (a, bx, by, bz) with a + bx + by + bz <= 4
constexpr int MOM3_MIN = 64;        // nodes of >= 64 points carry moments
constexpr int MOM3_CHUNK = 1024;    // points per moment item
constexpr int MOM3_TASKS = 512;     // moment tiles recorded per query; more -> dense tiles
constexpr int DENSE3_MAX = 2048;    // larger tiles only by moments (else traversed)

struct M3Tab {
    int8_t a[MOM3_K], bx[MOM3_K], by[MOM3_K], bz[MOM3_K];
    int8_t idx[5][5][5][5];
};
__host__ __device__ constexpr M3Tab make_m3tab() {
    M3Tab t{};
    int k = 0;
    for (int a = 0; a <= 4; ++a)
        for (int j = 0; j <= 4 - a; ++j)
            for (int bx = j; bx >= 0; --bx)
                for (int by = j - bx; by >= 0; --by) {
                    const int bz = j - bx - by;
                    t.a[k] = (int8_t)a; t.bx[k] = (int8_t)bx; t.by[k] = (int8_t)by; t.bz[k] = (int8_t)bz;
                    t.idx[a][bx][by][bz] = (int8_t)k;
                    ++k;
                }
    return t;
}
__constant__ M3Tab kM3 = make_m3tab();
static_assert(make_m3tab().a[MOM3_K - 1] == 4, "70 moments");

__device__ __forceinline__ bool mom3_node(const OctNode &nd) { return nd.cnt >= MOM3_MIN && nd.delta < 63; }

// items: node i (an internal node, i < m - 1) gets ceil(cnt / CHUNK) of them
__global__ void oct_mom_count(const OctNode *__restrict__ nodes, int64_t n, const int32_t *__restrict__ meta,
                              const int32_t *__restrict__ mom_flag, int32_t *__restrict__ mcnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t c = 0;
    if (mom_flag[0] && i < (int64_t)meta[0] - 1 && mom3_node(nodes[i])) c = (nodes[i].cnt + MOM3_CHUNK - 1) / MOM3_CHUNK;
    mcnt[i] = c;
}
__global__ void oct_mom_fill(const int32_t *__restrict__ mcnt, const int32_t *__restrict__ moff, int64_t n,
                             int64_t cap, int32_t *__restrict__ item_node) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int c = 0; c < mcnt[i]; ++c)
        if (moff[i] + c < cap) item_node[moff[i] + c] = (int32_t)i;
}
__device__ __forceinline__ void box3(const OctNode &nd, double &cx, double &cy, double &cz, double &R) {
    cx = 0.5 * (nd.bx0 + nd.bx1);
    cy = 0.5 * (nd.by0 + nd.by1);
    cz = 0.5 * (nd.bz0 + nd.bz1);
    const double ex = 0.5 * (nd.bx1 - nd.bx0), ey = 0.5 * (nd.by1 - nd.by0), ez = 0.5 * (nd.bz1 - nd.bz0);
    R = sqrt(ex * ex + ey * ey + ez * ez) * (1.0 + 1e-12);
}
__host__ __device__ constexpr double factd3(int k) { return k <= 1 ? 1.0 : k * factd3(k - 1); }
__device__ __forceinline__ double ipow(double x, int e) {
    double r = 1.0;
    for (int k = 0; k < e; ++k) r *= x;
    return r;
}
// One wave per item: lanes over the item's points, all MOM3_K moments in
// registers in one pass (the powers from tables: the same products, in the
// same order, as repeated multiplication), a fixed-order wave reduction per
// moment.
__global__ __launch_bounds__(256) void oct_mom_items(const double4 *__restrict__ pos, const OctNode *__restrict__ nodes,
                                                     const int32_t *__restrict__ mcnt, const int32_t *__restrict__ moff,
                                                     int64_t n, const int32_t *__restrict__ item_node, int64_t cap,
                                                     double *__restrict__ part, double *__restrict__ mom,
                                                     int32_t *__restrict__ mlist, int32_t *__restrict__ mlist_n) {
    constexpr M3Tab T = make_m3tab();
    const int64_t total = min((int64_t)moff[n - 1] + mcnt[n - 1], cap);
    const int lane = lane_id();
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t it = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); it < total; it += nw) {
        const int node = __builtin_amdgcn_readfirstlane(item_node[it]);
        const OctNode &nd = nodes[node];
        double cx, cy, cz, R;
        box3(nd, cx, cy, cz, R);
        const int c = (int)(it - moff[node]);
        const int p0 = nd.first + c * MOM3_CHUNK, p1 = min(nd.last + 1, p0 + MOM3_CHUNK);
        double acc[MOM3_K];
#pragma unroll
        for (int k = 0; k < MOM3_K; ++k) acc[k] = 0.0;
        for (int p = p0 + lane; p < p1; p += 64) {
            const double4 q = pos[p];
            const double ux = q.x - cx, uy = q.y - cy, uz = q.z - cz;
            const double s = ux * ux + uy * uy + uz * uz;
            double S[5], X[5], Yp[5], Zp[5];
            S[0] = 1.0; X[0] = 1.0; Yp[0] = 1.0; Zp[0] = 1.0;
#pragma unroll
            for (int e = 1; e <= 4; ++e) {
                S[e] = S[e - 1] * s; X[e] = X[e - 1] * ux; Yp[e] = Yp[e - 1] * uy; Zp[e] = Zp[e - 1] * uz;
            }
#pragma unroll
            for (int k = 0; k < MOM3_K; ++k)
                acc[k] = __fma_rn(S[T.a[k]] * X[T.bx[k]] * Yp[T.by[k]], Zp[T.bz[k]], acc[k]);
        }
        // a node of one item: its moments directly; of several: listed once for oct_mom_reduce
        const int nc = __builtin_amdgcn_readfirstlane(mcnt[node]);
        double *dst = nc == 1 ? mom + (int64_t)node * MOM3_K : part + it * MOM3_K;
        if (nc > 1 && c == 0 && lane == 0) mlist[atomicAdd(mlist_n, 1)] = node;
#pragma unroll
        for (int k = 0; k < MOM3_K; ++k) {
            const double v = wave_sum(acc[k]);
            if (lane == 0) dst[k] = v;
        }
    }
}
// moments of the nodes of several items (the list, any order): their items'
// partials summed in item order (thread per (node, moment))
__global__ void oct_mom_reduce(const int32_t *__restrict__ mcnt, const int32_t *__restrict__ moff,
                               const int32_t *__restrict__ mlist, const int32_t *__restrict__ mlist_n, int64_t cap,
                               const double *__restrict__ part, double *__restrict__ mom) {
    const int64_t total = (int64_t)*mlist_n * MOM3_K;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = mlist[e / MOM3_K];
        const int k = (int)(e % MOM3_K);
        if (moff[i] + mcnt[i] > cap) continue;
        double s = 0.0;
        for (int c = 0; c < mcnt[i]; ++c) s += part[(moff[i] + c) * MOM3_K + k];
        mom[i * MOM3_K + k] = s;
    }
}
// the moments exist this iteration if the previous traversal had demand for
// them (lanes whose tile could use them: >= n / 64), or at the first build
__global__ void oct_mom_gate(int32_t *mom_flag) {
    mom_flag[0] = mom_flag[1] >= mom_flag[2];
    mom_flag[1] = 0;
    mom_flag[3] = 0;   // oct_mom_items' list of nodes of several items
}

__device__ __forceinline__ bool mom3_ok(double vx, double vy, double vz, double R, double tol) {
    const double A = vx * vx + vy * vy + vz * vz;
    const double rho = (R * R + 2.0 * sqrt(A) * R) / (1.0 + A) * (1.0 + 1e-12);
    if (!(rho < 0.25)) return false;
    double rp = rho;
#pragma unroll
    for (int k = 0; k < MOM3_ORDER; ++k) rp *= rho;
    return (MOM3_ORDER + 2) * rp <= tol * (1.0 - rho) * (1.0 - rho);
}
// z += sum 1/(1+D), F += sum (q - p)/(1+D)^2 over the node's points from its
// moments mu (wave-uniform: scalar loads), the query itself included (D = 0:
// 1 to z, 0 to F -- taken off by the caller like the dense tile)
__device__ __forceinline__ void mom3_eval(const double *__restrict__ mu, double vx, double vy, double vz, double &fx,
                                          double &fy, double &fz, double &zs) {
    const double A = vx * vx + vy * vy + vz * vz;
    const double B = rcp2(1.0 + A);
    double px[4], py[4], pz[4];
    px[0] = py[0] = pz[0] = 1.0;
#pragma unroll
    for (int e = 1; e < 4; ++e) { px[e] = px[e - 1] * vx; py[e] = py[e - 1] * vy; pz[e] = pz[e - 1] * vz; }
    double T[MOM3_ORDER + 1], Ux[MOM3_ORDER + 1], Uy[MOM3_ORDER + 1], Uz[MOM3_ORDER + 1];
#pragma unroll
    for (int k = 0; k <= MOM3_ORDER; ++k) {
        double t = 0.0, ux = 0.0, uy = 0.0, uz = 0.0;
        double ckj = 1.0, m2 = 1.0;   // C(k, j), (-2)^j
#pragma unroll
        for (int j = 0; j <= k; ++j) {
            // sum over |b| = j of multinom(j; b) v^b M(k - j; b) (and b + e_x, e_y, e_z)
            double st = 0.0, sx = 0.0, sy = 0.0, sz = 0.0;
#pragma unroll
            for (int bx = j; bx >= 0; --bx)
#pragma unroll
                for (int by = j - bx; by >= 0; --by) {
                    const int bz = j - bx - by;
                    const double mult = factd3(j) / (factd3(bx) * factd3(by) * factd3(bz));   // multinomial
                    const double w = mult * px[bx] * py[by] * pz[bz];
                    const int a = k - j;
                    st = __fma_rn(w, mu[kM3.idx[a][bx][by][bz]], st);
                    sx = __fma_rn(w, mu[kM3.idx[a][bx + 1][by][bz]], sx);
                    sy = __fma_rn(w, mu[kM3.idx[a][bx][by + 1][bz]], sy);
                    sz = __fma_rn(w, mu[kM3.idx[a][bx][by][bz + 1]], sz);
                }
            const double c = ckj * m2;
            t = __fma_rn(c, st, t);
            ux = __fma_rn(c, sx, ux);
            uy = __fma_rn(c, sy, uy);
            uz = __fma_rn(c, sz, uz);
            ckj = ckj * (double)(k - j) / (double)(j + 1);
            m2 *= -2.0;
        }
        T[k] = t; Ux[k] = ux; Uy[k] = uy; Uz[k] = uz;
    }
    double z = 0.0, gx = 0.0, gy = 0.0, gz = 0.0, bk = 1.0;   // bk = (-B)^k
#pragma unroll
    for (int k = 0; k <= MOM3_ORDER; ++k) {
        z = __fma_rn(bk, T[k], z);
        const double c = (double)(k + 1) * bk;
        gx = __fma_rn(c, vx * T[k] - Ux[k], gx);
        gy = __fma_rn(c, vy * T[k] - Uy[k], gy);
        gz = __fma_rn(c, vz * T[k] - Uz[k], gz);
        bk *= -B;
    }
    const double B2 = B * B;
    zs += B * z;
    fx += B2 * gx;
    fy += B2 * gy;
    fz += B2 * gz;
}

template <bool DBG>
__global__ __launch_bounds__(256) void oct_traverse(const double4 *__restrict__ pos, const int32_t *__restrict__ dupc,
                                                    const OctNode *__restrict__ nodes,
                                                    const int32_t *__restrict__ meta, double theta, double near_dmax,
                                                    int64_t g0, int64_t g1, const int32_t *__restrict__ qlist,
                                                    int32_t *__restrict__ mom_flag, int32_t *__restrict__ mtask,
                                                    int32_t *__restrict__ mtask_n, double *__restrict__ F,
                                                    double *__restrict__ Z, unsigned long long *__restrict__ dbg,
                                                    double mom_tol) {
    __shared__ int32_t sref[4][STACK3];
    __shared__ uint64_t smask[4][STACK3];
    __shared__ double4 tbuf[4][64];
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const int64_t wid = (int64_t)blockIdx.x * 4 + w;
    const int64_t k = g0 + wid * 64 + lane;   // query slot -> sorted position (qlist: a rank's own queries)
    const bool valid = k < g1;
    const int64_t s = valid ? (qlist ? (int64_t)qlist[k] : k) : -1;
    if (__ballot(valid) == 0) return;
    const int root = meta[1];
    const double inv_theta = theta > 0.0 ? 1.0 / theta : __builtin_inf();
    const double th_lo = theta * (1.0 - 1e-14), th_hi = theta * (1.0 + 1e-14);
    double qx = 0.0, qy = 0.0, qz = 0.0;
    if (valid) { const double4 q = pos[s]; qx = q.x; qy = q.y; qz = q.z; }
    const double qmag = fabs(qx) + fabs(qy) + fabs(qz);
    const int ndup = valid ? dupc[s] : 0;
    double fx = 0.0, fy = 0.0, fz = 0.0, zs = 0.0;
    double4 *buf = tbuf[w];
    int sp = 0;
    const bool mom_on = mom_flag[0] != 0;
    int nwant = 0;   // tiles whose moments this lane could take (the next build's gate)
    int ntask = 0;
    unsigned long long d_pops = 0, d_childs = 0, d_dense = 0, d_declined = 0;   // TSNE_DEBUG_OCT counters
    if (root == ~0) {
        if (valid) { const double4 p = pos[0]; leaf3(qx, qy, qz, p.x, p.y, p.z, fx, fy, fz, zs); }
    } else if (root >= 0) {
        const OctNode &rt = nodes[root];
        if (rt.delta >= 63) {
            for (int p = rt.first; p <= rt.last; ++p) {
                const double4 pp = pos[p];
                if (valid) leaf3(qx, qy, qz, pp.x, pp.y, pp.z, fx, fy, fz, zs);
            }
        } else {
            bool open = false;
            if (valid) {
                const double dx = qx - rt.cx, dy = qy - rt.cy, dz = qz - rt.cz;
                if (summarise3(rt.h, dx, dy, dz, th_lo, th_hi, theta))
                    cell3(dx, dy, dz, dx * dx + dy * dy + dz * dz, rt.cnt, fx, fy, fz, zs);
                else
                    open = true;
            }
            const uint64_t om = __ballot(open);
            if (om) {
                if (lane == 0) { sref[w][0] = root; smask[w][0] = om; }
                sp = 1;
            }
        }
    }
    while (sp > 0) {
        --sp;
        const int ref = __builtin_amdgcn_readfirstlane(sref[w][sp]);
        const uint64_t msk = smask[w][sp];
        bool act = (msk >> lane) & 1ull;
        const OctNode &nd = nodes[ref];
        // all-open (ball / box with hmin) or near-exact: the exact leaf sum
        bool tile = false;
        if (act) {
            const double cdx = qx - nd.cx, cdy = qy - nd.cy, cdz = qz - nd.cz;
            tile = cdx * cdx + cdy * cdy + cdz * cdz <= nd.rball * nd.rball * (1.0 - 1e-9);
            if (!tile) {
                const double ex = 1e-15 * (qmag + fabs(nd.bx0) + fabs(nd.bx1) + fabs(nd.by0) + fabs(nd.by1) +
                                           fabs(nd.bz0) + fabs(nd.bz1));
                const double dxm = fmax(fabs(qx - nd.bx0), fabs(qx - nd.bx1)) + ex;
                const double dym = fmax(fabs(qy - nd.by0), fabs(qy - nd.by1)) + ex;
                const double dzm = fmax(fabs(qz - nd.bz0), fabs(qz - nd.bz1)) + ex;
                const double dmax = (dxm * dxm + dym * dym + dzm * dzm) * (1.0 + 1e-12);
                tile = dmax <= nd.hmin * inv_theta * (1.0 - 1e-12) || dmax <= near_dmax;
            }
        }
        // a tile from the node's moments when the truncation bound holds: a
        // task of this query's list (oct_mom_apply evaluates it afterwards)
        bool usem = false;
        if (tile && mom3_node(nd)) {
            double cx, cy, cz, R;
            box3(nd, cx, cy, cz, R);
            if (mom3_ok(qx - cx, qy - cy, qz - cz, R, mom_tol)) {
                ++nwant;
                if (mom_on && ntask < MOM3_TASKS) {
                    usem = true;
                    mtask[s * MOM3_TASKS + ntask++] = ref;
                    zs -= (s >= nd.first && s <= nd.last) ? (double)ndup : 0.0;
                }
            }
        }
        if (usem) act = false;
        // a large tile the moments cannot take is declined: the lane keeps
        // traversing it (the reference's own path), and its sub-tiles are
        // taken further down -- by moments, or densely once small
        if (tile && !usem && nd.cnt > DENSE3_MAX) { tile = false; if (DBG) ++d_declined; }
        const bool dense = tile && !usem;
        if (DBG) {
            ++d_pops;
            if (dense) d_dense += (unsigned long long)(nd.last - nd.first + 1);
        }
        if (__ballot(dense)) {
            // points staged through LDS 64 at a time, read back as broadcasts; the
            // query's exact duplicates (itself included) add 1 each to z: taken off
            const int a = nd.first, b = nd.last;
            double ux = 0.0, uy = 0.0, uz = 0.0, uq = 0.0;
            for (int c0 = a; c0 <= b; c0 += 64) {
                const int cn = min(64, b - c0 + 1);
                __builtin_amdgcn_wave_barrier();
                if (lane < cn) buf[lane] = pos[c0 + lane];
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_s_waitcnt(0);
                __builtin_amdgcn_wave_barrier();
                if (dense) {
                    for (int j = 0; j < cn; ++j) {
                        const double4 pp = buf[j];
                        const double dx = qx - pp.x, dy = qy - pp.y, dz = qz - pp.z;
                        const double r = rcp2(__fma_rn(dx, dx, __fma_rn(dy, dy, __fma_rn(dz, dz, 1.0))));
                        const double sc = r * r;
                        ux = __fma_rn(sc, dx, ux);
                        uy = __fma_rn(sc, dy, uy);
                        uz = __fma_rn(sc, dz, uz);
                        uq += r;
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (dense) {
                fx += ux; fy += uy; fz += uz;
                zs += uq - ((s >= a && s <= b) ? (double)ndup : 0.0);
                act = false;
            }
        }
        if (__ballot(act) == 0) continue;
        const int32_t chs[2] = {nd.left, nd.right};
        if (DBG && act) d_childs += 2;
        // push order: right first, so the left (lower keys: earlier children) pops first
        int32_t push_ref[2];
        uint64_t push_mask[2] = {0ull, 0ull};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int32_t ch = chs[k];
            push_ref[k] = ch;
            if (ch < 0) {
                const double4 p = pos[~ch];
                if (act) leaf3(qx, qy, qz, p.x, p.y, p.z, fx, fy, fz, zs);
                continue;
            }
            const OctNode &cn = nodes[ch];
            if (cn.delta >= 63) {                       // key-tie group: all points interact
                for (int p = cn.first; p <= cn.last; ++p) {
                    const double4 pp = pos[p];
                    if (act) leaf3(qx, qy, qz, pp.x, pp.y, pp.z, fx, fy, fz, zs);
                }
            } else if (cn.h < 0.0) {                    // transparent: opened with its parent
                push_mask[k] = __ballot(act);
            } else {
                bool open = false;
                if (act) {
                    const double dx = qx - cn.cx, dy = qy - cn.cy, dz = qz - cn.cz;
                    if (summarise3(cn.h, dx, dy, dz, th_lo, th_hi, theta))
                        cell3(dx, dy, dz, __fma_rn(dx, dx, __fma_rn(dy, dy, dz * dz)), cn.cnt, fx, fy, fz, zs);
                    else
                        open = true;
                }
                push_mask[k] = __ballot(open);
            }
        }
#pragma unroll
        for (int k = 1; k >= 0; --k) {
            if (push_mask[k]) {
                if (lane == 0) { sref[w][sp] = push_ref[k]; smask[w][sp] = push_mask[k]; }
                ++sp;
            }
        }
    }
    if (valid) {
        F[3 * s] = fx;
        F[3 * s + 1] = fy;
        F[3 * s + 2] = fz;
        Z[s] = zs;
        mtask_n[s] = ntask;
    }
    // demand for the next build's moments (only until the gate's threshold:
    // one memory-side atomic per wave on one word would serialise n / 64 of them)
    if (DBG) {   // [0] wave pops, [1] lane child evaluations, [2] lane dense tile points, [3] lane declined tiles, [4] moment tasks
        const unsigned long long a = wave_sum(d_childs), b = wave_sum(d_dense), c = wave_sum(d_declined),
                                 e = wave_sum((unsigned long long)ntask);
        if (lane == 0) {
            atomicAdd(dbg, d_pops);
            atomicAdd(dbg + 1, a);
            atomicAdd(dbg + 2, b);
            atomicAdd(dbg + 3, c);
            atomicAdd(dbg + 4, e);
        }
    }
    const int ww = wave_sum(nwant);
    if (lane == 0 && ww && __hip_atomic_load(&mom_flag[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < mom_flag[2])
        atomicAdd(&mom_flag[1], ww);
}

// Each query's moment tasks (in traversal order), added to its F and z.
__global__ __launch_bounds__(256) void oct_mom_apply(const double4 *__restrict__ pos, const OctNode *__restrict__ nodes,
                                                     const double *__restrict__ mom, const int32_t *__restrict__ mtask,
                                                     const int32_t *__restrict__ mtask_n, int64_t g0, int64_t g1,
                                                     const int32_t *__restrict__ qlist, double *__restrict__ F,
                                                     double *__restrict__ Z) {
    const int64_t k = g0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= g1) return;
    const int64_t s = qlist ? (int64_t)qlist[k] : k;
    const int nt = mtask_n[s];
    if (nt == 0) return;
    const double4 q = pos[s];
    double fx = 0.0, fy = 0.0, fz = 0.0, zs = 0.0;
    for (int i = 0; i < nt; ++i) {
        const int node = mtask[s * MOM3_TASKS + i];
        double cx, cy, cz, R;
        box3(nodes[node], cx, cy, cz, R);
        mom3_eval(mom + (int64_t)node * MOM3_K, q.x - cx, q.y - cy, q.z - cz, fx, fy, fz, zs);
    }
    F[3 * s] += fx;
    F[3 * s + 1] += fy;
    F[3 * s + 2] += fz;
    Z[s] += zs;
}

// ---- Octal records and the record traversal (the 2-D design of bhtree.hip:
// quad records + batched record fetches, with the narrow lane layout).

// One thread per binary node: the record of every real cell (h >= 0, no key
// tie); its children found through <= 2 levels of transparent nodes, in key
// order.  Records are assembled in LDS and copied out as coalesced 16-byte
// pieces (ORec is 496 bytes).
constexpr int OREC_BLK = 64;
__global__ __launch_bounds__(OREC_BLK) void build_orec(const OctNode *__restrict__ nodes,
                                                       const double4 *__restrict__ pos,
                                                       const int32_t *__restrict__ meta, double inv_theta,
                                                       double near_dmax, ORec *__restrict__ orec) {
    __shared__ ORec sr[OREC_BLK];
    __shared__ int32_t sreal[OREC_BLK];
    const int m = meta[0];
    const int b0 = blockIdx.x * OREC_BLK;
    const int nrec = min(OREC_BLK, m - 1 - b0);
    if (nrec <= 0) return;
    const int i = b0 + threadIdx.x;
    if (threadIdx.x < nrec) {
        const OctNode &nd = nodes[i];
        const bool real = nd.h >= 0.0 && nd.delta < 63;
        sreal[threadIdx.x] = real;
        if (real) {
            ORec &r = sr[threadIdx.x];
            r.cx = nd.cx; r.cy = nd.cy; r.cz = nd.cz;
            r.rball2 = nd.rball * nd.rball * (1.0 - 1e-9);
            r.thr = fmax(nd.hmin * inv_theta * (1.0 - 1e-12), near_dmax);
            r.bx0 = nd.bx0; r.bx1 = nd.bx1; r.by0 = nd.by0; r.by1 = nd.by1; r.bz0 = nd.bz0; r.bz1 = nd.bz1;
            r.first = nd.first; r.last = nd.last; r.cnt = nd.cnt; r.pad = 0;
            int nc = 0, kinds = 0;
            auto put = [&](int32_t c) {
                if (c < 0) {
                    const double4 p = pos[~c];
                    r.ccx[nc] = p.x; r.ccy[nc] = p.y; r.ccz[nc] = p.z;
                    r.cb[nc] = 0.0; r.ca[nc] = 0.0; r.cref[nc] = c; r.ccnt[nc] = 1;
                    kinds |= OK_LEAF << (2 * nc);
                } else {
                    const OctNode &cn = nodes[c];
                    r.ccx[nc] = cn.cx; r.ccy[nc] = cn.cy; r.ccz[nc] = cn.cz;
                    r.cref[nc] = c; r.ccnt[nc] = cn.cnt;
                    if (cn.delta >= 63) {
                        r.cb[nc] = 0.0; r.ca[nc] = 0.0;
                        kinds |= OK_TIE << (2 * nc);
                    } else {
                        r.cb[nc] = qacc_open(cn.h, inv_theta); r.ca[nc] = qacc_accept(cn.h, inv_theta);
                        kinds |= OK_CELL << (2 * nc);
                    }
                }
                ++nc;
            };
            auto transparent = [&](int32_t c) { return c >= 0 && nodes[c].delta < 63 && nodes[c].h < 0.0; };
            const int32_t top[2] = {nd.left, nd.right};
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int32_t c = top[k];
                if (transparent(c)) {
                    const int32_t sub[2] = {nodes[c].left, nodes[c].right};
#pragma unroll
                    for (int k2 = 0; k2 < 2; ++k2) {
                        const int32_t c2 = sub[k2];
                        if (transparent(c2)) { put(nodes[c2].left); put(nodes[c2].right); }
                        else put(c2);
                    }
                } else {
                    put(c);
                }
            }
            for (int k = nc; k < 8; ++k) {
                r.ccx[k] = 0.0; r.ccy[k] = 0.0; r.ccz[k] = 0.0; r.cb[k] = 0.0; r.ca[k] = 0.0;
                r.cref[k] = 0; r.ccnt[k] = 0;
            }
            // a tile test can pass here unless the box's half-diagonal alone
            // (the least max-corner distance of any query) exceeds both bounds
            const double hx = 0.5 * (nd.bx1 - nd.bx0), hy = 0.5 * (nd.by1 - nd.by0), hz = 0.5 * (nd.bz1 - nd.bz0);
            const bool tile = nd.rball > 0.0 || (hx * hx + hy * hy + hz * hz) * (1.0 - 1e-9) <= r.thr;
            r.nch = nc | (tile ? ONCH_TILE : 0);
            r.kinds = kinds;
        }
    }
    __syncthreads();
    constexpr int V = sizeof(ORec) / 16;
    const uint4 *src = reinterpret_cast<const uint4 *>(sr);
    uint4 *dst = reinterpret_cast<uint4 *>(orec + b0);
    for (int k = threadIdx.x; k < nrec * V; k += OREC_BLK)
        if (sreal[k / V]) dst[k] = src[k];
}

// Record traversal: one wave = 8 queries x 8 children (lane = 8 q + c).  The
// wave's LDS stack holds (record, 8-bit query mask) entries, one per cell some
// query opens; up to OKPOP records are fetched per round (coalesced 16-byte
// pieces, latencies overlapped), then each is one sweep of the lanes: lane
// (q, c) takes child c of the record for query q -- a leaf interacts (zero if
// it is the query's own point), a cell is summarised when h / D < theta
// (QuadTree.scala:133-134, 3-D D) or pushed, a key-tie group interacts point
// by point.  Before that, per (record, query), the all-open / near-exact tests
// (the 2-D path's, bhtree.hip): the subtree's exact leaf sum from its moments
// (a task of the query's list, oct_mom_apply) or densely, the query's 8 lanes
// splitting its points; a large tile the moments cannot take is traversed.
// Each lane keeps its own partial sums; the query's 8 lanes are added by a
// fixed xor butterfly at the end (deterministic).
constexpr int OQ = 8;          // queries per wave
constexpr int OKPOP = 4;       // records per fetch round
constexpr int OSTACK = 512;    // batch rounds while <= OSTACK / 2 entries, then depth-first (+7 per level)
template <bool DBG>
__global__ __launch_bounds__(256) void oct_traverse_rec(
    const double4 *__restrict__ pos, const int32_t *__restrict__ dupc, const OctNode *__restrict__ nodes,
    const ORec *__restrict__ orec, const int32_t *__restrict__ meta, double theta, int64_t g0, int64_t g1,
    const int32_t *__restrict__ qlist, int32_t *__restrict__ mom_flag, int32_t *__restrict__ mtask,
    int32_t *__restrict__ mtask_n, double *__restrict__ F, double *__restrict__ Z,
    unsigned long long *__restrict__ dbg, double mom_tol, const double *__restrict__ Wp, double wthr, int regime) {
    __shared__ int32_t sref[4][OSTACK];
    __shared__ uint32_t smask[4][OSTACK];
    __shared__ ORec srec[4][OKPOP];
    __shared__ int32_t bref[4][OKPOP];
    __shared__ uint32_t bmask[4][OKPOP];
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const int q = lane >> 3, c = lane & 7;
    const int64_t wid = (int64_t)blockIdx.x * 4 + w;
    const int64_t kq = g0 + wid * OQ + q;
    const bool valid = kq < g1;
    if (__ballot(valid) == 0) return;
    // per-iteration layout choice (oct_repulsion): regime 1 runs below the
    // root half-width wthr, regime 2 at or above it, 0 always
    if (regime != 0 && (regime == 1) != (*Wp < wthr)) return;
    const int64_t s = valid ? (qlist ? (int64_t)qlist[kq] : kq) : -1;
    const double th_lo = theta * (1.0 - 1e-14), th_hi = theta * (1.0 + 1e-14);
    double qx = 0.0, qy = 0.0, qz = 0.0;
    if (valid) { const double4 p = pos[s]; qx = p.x; qy = p.y; qz = p.z; }
    const double qmag = fabs(qx) + fabs(qy) + fabs(qz);
    const int ndup = valid ? dupc[s] : 0;
    const bool mom_on = mom_flag[0] != 0;
    double fx = 0.0, fy = 0.0, fz = 0.0, zs = 0.0;
    int ntask = 0, nwant = 0;
    unsigned long long d_pops = 0, d_childs = 0, d_dense = 0, d_declined = 0;   // Options-free debug counters
    int sp = 0;
    // the root: a single point, a key-tie group, or a cell tested like any child
    // (lane c = 0 of each query)
    const int root = meta[1];
    const bool r0 = valid && c == 0;
    if (root == ~0) {
        if (r0) { const double4 p = pos[0]; leaf3(qx, qy, qz, p.x, p.y, p.z, fx, fy, fz, zs); }
    } else if (root >= 0) {
        const OctNode &rt = nodes[root];
        if (rt.delta >= 63) {
            for (int p = rt.first; p <= rt.last; ++p) {
                const double4 pp = pos[p];
                if (r0) leaf3(qx, qy, qz, pp.x, pp.y, pp.z, fx, fy, fz, zs);
            }
        } else {
            bool open = false;
            if (r0) {
                const double dx = qx - rt.cx, dy = qy - rt.cy, dz = qz - rt.cz;
                if (summarise3(rt.h, dx, dy, dz, th_lo, th_hi, theta))
                    cell3(dx, dy, dz, dx * dx + dy * dy + dz * dz, rt.cnt, fx, fy, fz, zs);
                else
                    open = true;
            }
            const uint64_t om = __ballot(open);
            uint32_t qm = 0;
#pragma unroll
            for (int k = 0; k < OQ; ++k) qm |= (uint32_t)((om >> (8 * k)) & 1ull) << k;
            if (qm) {
                if (lane == 0) { sref[w][0] = root; smask[w][0] = qm; }
                sp = 1;
            }
        }
    }
    while (sp > 0) {
        const int kb = sp > OSTACK / 2 ? 1 : (sp < OKPOP ? sp : OKPOP);
        sp -= kb;
        if (lane < kb) { bref[w][lane] = sref[w][sp + lane]; bmask[w][lane] = smask[w][sp + lane]; }
        constexpr int V = sizeof(ORec) / 16;
        for (int e = lane; e < V * kb; e += 64) {
            const int rr = e / V, part = e - rr * V;
            const int rf = sref[w][sp + rr];
            reinterpret_cast<uint4 *>(&srec[w][rr])[part] = reinterpret_cast<const uint4 *>(orec + rf)[part];
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0);   // vmcnt = lgkmcnt = 0: the batch is in LDS
        __builtin_amdgcn_wave_barrier();
        for (int r = 0; r < kb; ++r) {
            if (DBG && lane == 0) ++d_pops;
            const int ref = __builtin_amdgcn_readfirstlane(bref[w][r]);
            const uint32_t msk = bmask[w][r];
            bool act = valid && ((msk >> q) & 1u);
            const ORec &nd = srec[w][r];
            const int nflags = __builtin_amdgcn_readfirstlane(nd.nch);
            // all-open / near-exact tests, per (record, query): the subtree's exact leaf sum
            bool tile = false;
            if ((nflags & ONCH_TILE) && act) {
                const double cdx = qx - nd.cx, cdy = qy - nd.cy, cdz = qz - nd.cz;
                tile = cdx * cdx + cdy * cdy + cdz * cdz <= nd.rball2;
                if (!tile) {
                    const double ex = 1e-15 * (qmag + fabs(nd.bx0) + fabs(nd.bx1) + fabs(nd.by0) + fabs(nd.by1) +
                                               fabs(nd.bz0) + fabs(nd.bz1));
                    const double dxm = fmax(fabs(qx - nd.bx0), fabs(qx - nd.bx1)) + ex;
                    const double dym = fmax(fabs(qy - nd.by0), fabs(qy - nd.by1)) + ex;
                    const double dzm = fmax(fabs(qz - nd.bz0), fabs(qz - nd.bz1)) + ex;
                    tile = (dxm * dxm + dym * dym + dzm * dzm) * (1.0 + 1e-12) <= nd.thr;
                }
            }
            if (__ballot(tile)) {
                const int a = __builtin_amdgcn_readfirstlane(nd.first), b = __builtin_amdgcn_readfirstlane(nd.last);
                const int cnt = __builtin_amdgcn_readfirstlane(nd.cnt);
                // moments: decided by the query's lane c = 0 (one record per sweep: list order = record order)
                bool usem = false;
                if (tile && c == 0 && cnt >= MOM3_MIN) {
                    double bcx, bcy, bcz, R;
                    box3(nodes[ref], bcx, bcy, bcz, R);
                    if (mom3_ok(qx - bcx, qy - bcy, qz - bcz, R, mom_tol)) {
                        ++nwant;
                        if (mom_on && ntask < MOM3_TASKS) {
                            usem = true;
                            mtask[s * MOM3_TASKS + ntask] = ref;
                        }
                    }
                }
                const uint64_t UM = __ballot(usem);
                const bool mq = (UM >> (lane & ~7)) & 1ull;   // the query's moment decision
                if (mq) ++ntask;                              // (every lane of the query: the same count)
                // a large tile the moments cannot take: the lane keeps traversing it
                const bool dense = tile && !mq && (b - a + 1) <= DENSE3_MAX;
                if (DBG && tile && !mq && !dense && c == 0) ++d_declined;
                const bool taken = mq || dense;
                if (taken && c == 0 && s >= a && s <= b) zs -= (double)ndup;   // the query's own copies add 1 each
                if (DBG && dense && c == 0) d_dense += (unsigned long long)(b - a + 1);
                // the query's 8 lanes split the points; summed apart in a divergent
                // do-while (no merge of the accumulators per point), added once
                double ux = 0.0, uy = 0.0, uz = 0.0, uq = 0.0;
                if (dense && a + c <= b) {
                    int p = a + c;
                    do {
                        const double4 pp = pos[p];
                        const double dx = qx - pp.x, dy = qy - pp.y, dz = qz - pp.z;
                        const double rr = rcp2(__fma_rn(dx, dx, __fma_rn(dy, dy, __fma_rn(dz, dz, 1.0))));
                        const double sc = rr * rr;
                        ux = __fma_rn(sc, dx, ux);
                        uy = __fma_rn(sc, dy, uy);
                        uz = __fma_rn(sc, dz, uz);
                        uq += rr;
                        p += 8;
                    } while (p <= b);
                }
                if (dense) { fx += ux; fy += uy; fz += uz; zs += uq; }
                act = act && !taken;
            }
            if (__ballot(act) == 0) continue;
            // child c of the record for query q
            const int nch = nflags & 0xff;
            const int kind = (__builtin_amdgcn_readfirstlane(nd.kinds) >> (2 * c)) & 3;
            const bool has = act && c < nch;
            if (DBG && has) ++d_childs;
            const double dx = qx - nd.ccx[c], dy = qy - nd.ccy[c], dz = qz - nd.ccz[c];
            const double D1 = __fma_rn(dx, dx, __fma_rn(dy, dy, __fma_rn(dz, dz, 1.0)));   // 1 + D (QACC_BAND)
            const bool isleaf = has && kind == OK_LEAF, iscell = has && kind == OK_CELL;
            bool acc = D1 > nd.ca[c];
            if (iscell && !acc && !(D1 < nd.cb[c]))
                acc = nodes[nd.cref[c]].h / __dadd_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)), __dmul_rn(dz, dz)) <
                      theta;
            const bool takel = isleaf && !(dx == 0.0 && dy == 0.0 && dz == 0.0);
            const bool takec = iscell && acc;
            const double wm = takel ? 1.0 : (takec ? (double)nd.ccnt[c] : 0.0);
            const double Qv = rcp2(D1);
            const double mult = wm * Qv;
            const double sc = mult * Qv;
            fx = __fma_rn(sc, dx, fx);
            fy = __fma_rn(sc, dy, fy);
            fz = __fma_rn(sc, dz, fz);
            zs += mult;
            const bool tie = has && kind == OK_TIE;
            if (__builtin_expect(__ballot(tie) != 0, 0) && tie) {   // a key-tie group: every point directly
                const OctNode &tn = nodes[nd.cref[c]];
                for (int p = tn.first; p <= tn.last; ++p) {
                    const double4 pp = pos[p];
                    leaf3(qx, qy, qz, pp.x, pp.y, pp.z, fx, fy, fz, zs);
                }
            }
            // pushes: one entry per child some query opens, in child order
            const uint64_t O = __ballot(iscell && !acc);
            uint32_t mcq = 0;
            if (q == 0 && c < nch) {
#pragma unroll
                for (int k = 0; k < OQ; ++k) mcq |= (uint32_t)((O >> (8 * k + c)) & 1ull) << k;
            }
            const uint64_t P = __ballot(mcq != 0u);
            if (mcq) {
                const int at = sp + (int)__popcll(P & lanemask_lt());
                sref[w][at] = nd.cref[c];
                smask[w][at] = mcq;
            }
            sp += (int)__popcll(P);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the pushes landed before the next reads
            __builtin_amdgcn_wave_barrier();
        }
    }
    // the query's 8 lanes in a fixed xor butterfly (every lane the same bits)
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
        fx += __shfl_xor(fx, o, 64); fy += __shfl_xor(fy, o, 64);
        fz += __shfl_xor(fz, o, 64); zs += __shfl_xor(zs, o, 64);
    }
    if (valid && c == 0) {
        F[3 * s] = fx;
        F[3 * s + 1] = fy;
        F[3 * s + 2] = fz;
        Z[s] = zs;
        mtask_n[s] = ntask;
    }
    if (DBG) {   // [0] wave pops, [1] lane child evaluations, [2] dense tile points, [3] declined tiles, [4] moment tasks
        const unsigned long long a = wave_sum(d_childs), b2 = wave_sum(d_dense), c2 = wave_sum(d_declined),
                                 e = wave_sum((unsigned long long)(c == 0 ? ntask : 0));
        if (lane == 0) {
            atomicAdd(dbg, d_pops * (64 / OQ));   // in 64-query-wave units, as the binary traversal's
            atomicAdd(dbg + 1, a);
            atomicAdd(dbg + 2, b2);
            atomicAdd(dbg + 3, c2);
            atomicAdd(dbg + 4, e);
        }
    }
    const int ww = wave_sum(nwant);
    if (lane == 0 && ww && __hip_atomic_load(&mom_flag[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < mom_flag[2])
        atomicAdd(&mom_flag[1], ww);
}


// Record traversal, 64-query layout: one wave = 64 consecutive sorted queries
// (lane = query) sharing an LDS stack of (record, 64-bit lane mask) entries,
// the 2-D traversal's design (bhtree.hip bh_traverse) on octal records.  A
// popped record serves every lane that opened it: one record fetch per 64
// queries (the 8-query layout fetches it per 8), so the transition phase --
// extents ~0.05-5, where nearly every cell near a query opens and the
// neighbouring queries open the same ones -- moves 8x fewer record bytes.
// Each lane evaluates the record's <= 8 children in order.  All-open /
// near-exact tiles: per lane a moment task (oct_mom_apply) or the dense leaf
// sum, which all lanes of the tile walk together: the points are wave-uniform
// (scalar loads), each lane adds its own pair terms.  Identical decisions to
// the 8-query layout (same tests, same records); the sums differ from it only
// in association.
constexpr int O64_STACK = 256;   // entries; batches of O64_KB while sp <= O64_BATCH, then depth-first
constexpr int O64_KB = 2;        // records per fetch round (2 x 31 16-byte pieces: one round of the lanes)
constexpr int O64_BATCH = 64;    // depth bound: 64 + 2 x 8 + 7 per level x 21 levels < O64_STACK
static_assert(O64_BATCH + O64_KB * 8 + 7 * LEVELS3 < O64_STACK, "64-query octal stack bound");
static_assert(O64_KB * (int)(sizeof(ORec) / 16) <= 64, "one fetch round per batch");
template <bool DBG>
__global__ __launch_bounds__(256) void oct_traverse64(
    const double4 *__restrict__ pos, const int32_t *__restrict__ dupc, const OctNode *__restrict__ nodes,
    const ORec *__restrict__ orec, const int32_t *__restrict__ meta, double theta, int64_t g0, int64_t g1,
    const int32_t *__restrict__ qlist, int32_t *__restrict__ mom_flag, int32_t *__restrict__ mtask,
    int32_t *__restrict__ mtask_n, double *__restrict__ F, double *__restrict__ Z,
    unsigned long long *__restrict__ dbg, double mom_tol, const double *__restrict__ Wp, double wthr, int regime) {
    __shared__ int32_t sref[4][O64_STACK];
    __shared__ uint64_t smask[4][O64_STACK];
    __shared__ ORec srec[4][O64_KB];
    __shared__ int32_t bref[4][O64_KB];
    __shared__ uint64_t bmask[4][O64_KB];
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const int64_t wid = (int64_t)blockIdx.x * 4 + w;
    const int64_t kq = g0 + wid * 64 + lane;
    const bool valid = kq < g1;
    if (__ballot(valid) == 0) return;
    // per-iteration layout choice (oct_repulsion): regime 1 runs below the
    // root half-width wthr, regime 2 at or above it, 0 always
    if (regime != 0 && (regime == 1) != (*Wp < wthr)) return;
    const int64_t s = valid ? (qlist ? (int64_t)qlist[kq] : kq) : -1;
    const double th_lo = theta * (1.0 - 1e-14), th_hi = theta * (1.0 + 1e-14);
    double qx = 0.0, qy = 0.0, qz = 0.0;
    if (valid) { const double4 p = pos[s]; qx = p.x; qy = p.y; qz = p.z; }
    const double qmag = fabs(qx) + fabs(qy) + fabs(qz);
    const int ndup = valid ? dupc[s] : 0;
    const bool mom_on = mom_flag[0] != 0;
    double fx = 0.0, fy = 0.0, fz = 0.0, zs = 0.0;
    int ntask = 0, nwant = 0;
    unsigned long long d_pops = 0, d_childs = 0, d_dense = 0, d_declined = 0;
    int sp = 0;
    const int root = meta[1];
    if (root == ~0) {
        if (valid) { const double4 p = pos[0]; leaf3(qx, qy, qz, p.x, p.y, p.z, fx, fy, fz, zs); }
    } else if (root >= 0) {
        const OctNode &rt = nodes[root];
        if (rt.delta >= 63) {
            for (int p = rt.first; p <= rt.last; ++p) {
                const double4 pp = pos[p];
                if (valid) leaf3(qx, qy, qz, pp.x, pp.y, pp.z, fx, fy, fz, zs);
            }
        } else {
            bool open = false;
            if (valid) {
                const double dx = qx - rt.cx, dy = qy - rt.cy, dz = qz - rt.cz;
                if (summarise3(rt.h, dx, dy, dz, th_lo, th_hi, theta))
                    cell3(dx, dy, dz, dx * dx + dy * dy + dz * dz, rt.cnt, fx, fy, fz, zs);
                else
                    open = true;
            }
            const uint64_t om = __ballot(open);
            if (om) {
                if (lane == 0) { sref[w][0] = root; smask[w][0] = om; }
                sp = 1;
            }
        }
    }
    while (sp > 0) {
        const int kb = sp > O64_BATCH ? 1 : (sp < O64_KB ? sp : O64_KB);
        sp -= kb;
        if (lane < kb) { bref[w][lane] = sref[w][sp + lane]; bmask[w][lane] = smask[w][sp + lane]; }
        constexpr int V = sizeof(ORec) / 16;
        if (lane < V * kb) {
            const int rr = lane / V, part = lane - rr * V;
            reinterpret_cast<uint4 *>(&srec[w][rr])[part] = reinterpret_cast<const uint4 *>(orec + sref[w][sp + rr])[part];
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0);   // vmcnt = lgkmcnt = 0: the batch is in LDS
        __builtin_amdgcn_wave_barrier();
        for (int r = 0; r < kb; ++r) {
            if (DBG && lane == 0) ++d_pops;
            const int ref = __builtin_amdgcn_readfirstlane(bref[w][r]);
            const uint64_t msk = bmask[w][r];
            bool act = valid && ((msk >> lane) & 1ull);
            const ORec &nd = srec[w][r];
            const int nflags = __builtin_amdgcn_readfirstlane(nd.nch);
            bool tile = false;
            if ((nflags & ONCH_TILE) && act) {
                const double cdx = qx - nd.cx, cdy = qy - nd.cy, cdz = qz - nd.cz;
                tile = cdx * cdx + cdy * cdy + cdz * cdz <= nd.rball2;
                if (!tile) {
                    const double ex = 1e-15 * (qmag + fabs(nd.bx0) + fabs(nd.bx1) + fabs(nd.by0) + fabs(nd.by1) +
                                               fabs(nd.bz0) + fabs(nd.bz1));
                    const double dxm = fmax(fabs(qx - nd.bx0), fabs(qx - nd.bx1)) + ex;
                    const double dym = fmax(fabs(qy - nd.by0), fabs(qy - nd.by1)) + ex;
                    const double dzm = fmax(fabs(qz - nd.bz0), fabs(qz - nd.bz1)) + ex;
                    tile = (dxm * dxm + dym * dym + dzm * dzm) * (1.0 + 1e-12) <= nd.thr;
                }
            }
            if (__ballot(tile)) {
                const int a = __builtin_amdgcn_readfirstlane(nd.first), b = __builtin_amdgcn_readfirstlane(nd.last);
                const int cnt = __builtin_amdgcn_readfirstlane(nd.cnt);
                bool usem = false;
                if (tile && cnt >= MOM3_MIN) {
                    double bcx, bcy, bcz, R;
                    box3(nodes[ref], bcx, bcy, bcz, R);
                    if (mom3_ok(qx - bcx, qy - bcy, qz - bcz, R, mom_tol)) {
                        ++nwant;
                        if (mom_on && ntask < MOM3_TASKS) {
                            usem = true;
                            mtask[s * MOM3_TASKS + ntask++] = ref;
                        }
                    }
                }
                // a large tile the moments cannot take: the lane keeps traversing it
                const bool dense = tile && !usem && (b - a + 1) <= DENSE3_MAX;
                if (DBG && tile && !usem && !dense) ++d_declined;
                const bool taken = usem || dense;
                if (taken && s >= a && s <= b) zs -= (double)ndup;   // the query's own copies add 1 each
                if (__ballot(dense)) {
                    if (DBG && dense) d_dense += (unsigned long long)(b - a + 1);
                    // the points are the wave's (uniform index: scalar loads), every
                    // lane of the tile adds its own terms
                    double ux = 0.0, uy = 0.0, uz = 0.0, uq = 0.0;
                    for (int p = a; p <= b; ++p) {
                        const double4 pp = pos[p];
                        const double dx = qx - pp.x, dy = qy - pp.y, dz = qz - pp.z;
                        const double rr = rcp2(__fma_rn(dx, dx, __fma_rn(dy, dy, __fma_rn(dz, dz, 1.0))));
                        const double sc = rr * rr;
                        ux = __fma_rn(sc, dx, ux);
                        uy = __fma_rn(sc, dy, uy);
                        uz = __fma_rn(sc, dz, uz);
                        uq += rr;
                    }
                    if (dense) { fx += ux; fy += uy; fz += uz; zs += uq; }
                }
                act = act && !taken;
            }
            const uint64_t amask = __ballot(act);   // the lanes that go on to the children
            if (amask == 0) continue;
            const int nch = nflags & 0xff;
            const int kinds = __builtin_amdgcn_readfirstlane(nd.kinds);
            if (DBG && act) d_childs += (unsigned long long)nch;
            for (int c = 0; c < nch; ++c) {
                const int kind = (kinds >> (2 * c)) & 3;   // uniform: scalar branches
                if (kind == OK_TIE) continue;                // after the loop (rare)
                const double dx = qx - nd.ccx[c], dy = qy - nd.ccy[c], dz = qz - nd.ccz[c];
                const double D1 = __fma_rn(dx, dx, __fma_rn(dy, dy, __fma_rn(dz, dz, 1.0)));   // 1 + D (QACC_BAND)
                // lane predicates from scalar masks (inverse ballots: no VALU),
                // the masks straight from the compares, as in bh_traverse
                double wm;
                if (kind == OK_LEAF) {
                    const uint64_t takem = amask & ~(__builtin_amdgcn_ballot_w64(dx == 0.0) &
                                                     __builtin_amdgcn_ballot_w64(dy == 0.0) &
                                                     __builtin_amdgcn_ballot_w64(dz == 0.0));
                    wm = __builtin_amdgcn_inverse_ballot_w64(takem) ? 1.0 : 0.0;
                } else {
                    uint64_t accm = __builtin_amdgcn_ballot_w64(D1 > nd.ca[c]);
                    const uint64_t band = amask & ~accm & ~__builtin_amdgcn_ballot_w64(D1 < nd.cb[c]);
                    if (band) {   // rare: inside the band the exact IEEE quotient decides
                        bool acc = false;
                        if (__builtin_amdgcn_inverse_ballot_w64(band))
                            acc = nodes[nd.cref[c]].h /
                                      __dadd_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)), __dmul_rn(dz, dz)) <
                                  theta;
                        accm |= band & __builtin_amdgcn_ballot_w64(acc);
                    }
                    wm = (double)(__builtin_amdgcn_inverse_ballot_w64(amask & accm) ? nd.ccnt[c] : 0);
                    const uint64_t om = amask & ~accm;
                    if (om) {
                        if (lane == 0) { sref[w][sp] = nd.cref[c]; smask[w][sp] = om; }
                        ++sp;
                    }
                }
                const double Qv = rcp2(D1);
                const double mult = wm * Qv;
                const double sc = mult * Qv;
                fx = __fma_rn(sc, dx, fx);
                fy = __fma_rn(sc, dy, fy);
                fz = __fma_rn(sc, dz, fz);
                zs += mult;
            }
            if (__builtin_expect(kinds & 0xAAAA, 0)) {   // key-tie groups: every point directly
                for (int c = 0; c < nch; ++c) {
                    if (((kinds >> (2 * c)) & 3) != OK_TIE) continue;
                    const OctNode &tn = nodes[__builtin_amdgcn_readfirstlane(nd.cref[c])];
                    for (int p = tn.first; p <= tn.last; ++p) {
                        const double4 pp = pos[p];
                        if (__builtin_amdgcn_inverse_ballot_w64(amask)) leaf3(qx, qy, qz, pp.x, pp.y, pp.z, fx, fy, fz, zs);
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the pushes landed before the next reads
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (valid) {
        F[3 * s] = fx;
        F[3 * s + 1] = fy;
        F[3 * s + 2] = fz;
        Z[s] = zs;
        mtask_n[s] = ntask;
    }
    if (DBG) {   // [0] wave pops, [1] lane child evaluations, [2] dense tile points, [3] declined tiles, [4] moment tasks
        const unsigned long long a = wave_sum(d_childs), b2 = wave_sum(d_dense), c2 = wave_sum(d_declined),
                                 e = wave_sum((unsigned long long)ntask);
        if (lane == 0) {
            atomicAdd(dbg, d_pops);
            atomicAdd(dbg + 1, a);
            atomicAdd(dbg + 2, b2);
            atomicAdd(dbg + 3, c2);
            atomicAdd(dbg + 4, e);
        }
    }
    const int ww = wave_sum(nwant);
    if (lane == 0 && ww && __hip_atomic_load(&mom_flag[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < mom_flag[2])
        atomicAdd(&mom_flag[1], ww);
}

}  // namespace

void oct_alloc(tsne_ctx *ctx, OctTree &t, int64_t n, const std::string &pre) {
    Workspace &ws = ctx->ws;
    t.n = n;
    t.keys = ws.get<uint64_t>(pre + "keys", n);
    t.keys_sorted = ws.get<uint64_t>(pre + "keys_sorted", n);
    t.idx = ws.get<int32_t>(pre + "idx", n);
    t.idx_sorted = ws.get<int32_t>(pre + "idx_sorted", n);
    t.inv = ws.get<int32_t>(pre + "inv", n);
    t.dupc = ws.get<int32_t>(pre + "dupc", n);
    t.pos = ws.get<double4>(pre + "pos", n);
    t.nodes = ws.get<OctNode>(pre + "nodes", n);
    t.orec = ws.get<ORec>(pre + "orec", n);
    t.agg = ws.get<double>(pre + "agg", AGG3 * (size_t)n);
    t.parent_leaf = ws.get<int32_t>(pre + "parent_leaf", n);
    t.parent_node = ws.get<int32_t>(pre + "parent_node", n);
    t.arrive = ws.get<int32_t>(pre + "arrive", n);
    t.meta = ws.get<int32_t>(pre + "meta", 4);
    t.bbox_blocks = (int)std::min<int64_t>(1024, std::max<int64_t>(1, ceil_div(n, 256)));
    t.bbox_part = ws.get<double>(pre + "bbox_part", 6 * (size_t)t.bbox_blocks);
    t.W = ws.get<double>(pre + "W", 1);
    size_t tb = 0;
    TSNE_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, t.keys, t.keys_sorted, t.idx, t.idx_sorted, (int)n, 0,
                                               64, ctx->stream));
    t.sort_tmp_bytes = tb;
    t.sort_tmp = ws.get<uint8_t>(pre + "sort_tmp", tb);
    csort_alloc(ctx, t.cs, n, pre);
    t.cs_primed = false;
    t.mom = ws.get<double>(pre + "mom", (size_t)MOM3_K * n);
    t.mcnt = ws.get<int32_t>(pre + "mcnt", n);
    t.moff = ws.get<int32_t>(pre + "moff", n);
    t.item_cap = n / 8 + 64;
    t.item_node = ws.get<int32_t>(pre + "item_node", t.item_cap);
    t.mom_part = ws.get<double>(pre + "mom_part", (size_t)MOM3_K * t.item_cap);
    t.mom_flag = ws.get<int32_t>(pre + "mom_flag", 4);
    t.mlist = ws.get<int32_t>(pre + "mlist", n / 256 + 64);   // nodes of > MOM3_CHUNK points: < 2 n / MOM3_CHUNK
    t.mtask = ws.get<int32_t>(pre + "mtask", (size_t)MOM3_TASKS * n);
    t.mtask_n = ws.get<int32_t>(pre + "mtask_n", n);
    size_t mb = 0;
    TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, mb, t.mcnt, t.moff, (int)n, ctx->stream));
    t.mscan_tmp_bytes = mb;
    t.mscan_tmp = ws.get<uint8_t>(pre + "mscan_tmp", mb);
    // the first build computes moments (demand := threshold); threshold n / 64
    // lanes; Options::oct_moments = 0 turns the path off
    const bool on = ctx->opts.oct_moments != 0;
    const int32_t thr = (int32_t)std::max<int64_t>(1, n / 64);
    const int32_t f[4] = {0, on ? thr : 0, on ? thr : INT32_MAX, 0};
    TSNE_HIP(hipMemcpyAsync(t.mom_flag, f, sizeof(f), hipMemcpyHostToDevice, ctx->stream));
    TSNE_HIP(hipStreamSynchronize(ctx->stream));
}

static double oct_near_dmax(const tsne_ctx *ctx, double theta, bool late);

void oct_build(tsne_ctx *ctx, OctTree &t, const double *dY, double theta, bool late) {
    hipStream_t st = ctx->stream;
    const int64_t n = t.n;
    hipLaunchKernelGGL(bbox3_partial, dim3(t.bbox_blocks), dim3(256), 0, st, dY, n, t.bbox_part);
    hipLaunchKernelGGL(bbox3_final, dim3(1), dim3(256), 0, st, t.bbox_part, t.bbox_blocks, t.W, t.meta);
    hipLaunchKernelGGL(morton3_keys, dim3(ceil_div(n, 256)), dim3(256), 0, st, dY, n, t.W, t.keys, t.idx, t.meta);
    TSNE_LAUNCH_CHECK();
    if (t.cs.P > 0 && t.cs_primed && ctx->opts.coherent_sort) {   // from the previous build's order (csort.hpp)
        csort_run(ctx, t.cs, t.keys, t.idx_sorted, t.keys_sorted, t.idx_sorted, st);
    } else {
        size_t tb = t.sort_tmp_bytes;
        TSNE_HIP(hipcub::DeviceRadixSort::SortPairs(t.sort_tmp, tb, t.keys, t.keys_sorted, t.idx, t.idx_sorted, (int)n,
                                                   0, 64, st));
    }
    t.cs_primed = true;
    hipLaunchKernelGGL(count_in_root3, dim3(1), dim3(64), 0, st, t.keys_sorted, n, t.meta);
    hipLaunchKernelGGL(gather3, dim3(ceil_div(n, 256)), dim3(256), 0, st, dY, t.idx_sorted, n, t.pos, t.inv);
    hipLaunchKernelGGL(dup_count3, dim3(ceil_div(n, 256)), dim3(256), 0, st, t.pos, t.keys_sorted, n, t.dupc);
    hipLaunchKernelGGL(karras3, dim3(ceil_div(n, 256)), dim3(256), 0, st, t.keys_sorted, t.meta, t.nodes,
                       t.parent_leaf, t.parent_node, t.arrive);
    const double inv_theta = theta > 0.0 ? 1.0 / theta : __builtin_inf();
    hipLaunchKernelGGL(bottom_up3<512>, dim3(ceil_div(n, 512)), dim3(512), 0, st, t.pos, t.meta, t.W, inv_theta, t.nodes,
                       t.agg, t.parent_leaf, t.parent_node, t.arrive);
    hipLaunchKernelGGL(set_root3, dim3(1), dim3(1), 0, st, t.meta);
    t.near_dmax = oct_near_dmax(ctx, theta, late);
    if (ctx->opts.oct_records)
        hipLaunchKernelGGL(build_orec, dim3(ceil_div(n, OREC_BLK)), dim3(OREC_BLK), 0, st, t.nodes, t.pos, t.meta,
                           inv_theta, t.near_dmax, t.orec);
    // subtree moments (when the last traversal wanted them)
    hipLaunchKernelGGL(oct_mom_gate, dim3(1), dim3(1), 0, st, t.mom_flag);
    hipLaunchKernelGGL(oct_mom_count, dim3(ceil_div(n, 256)), dim3(256), 0, st, t.nodes, n, t.meta, t.mom_flag, t.mcnt);
    size_t mb = t.mscan_tmp_bytes;
    TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(t.mscan_tmp, mb, t.mcnt, t.moff, (int)n, st));
    hipLaunchKernelGGL(oct_mom_fill, dim3(ceil_div(n, 256)), dim3(256), 0, st, t.mcnt, t.moff, n, t.item_cap,
                       t.item_node);
    hipLaunchKernelGGL(oct_mom_items, dim3(std::max<int64_t>(1, std::min<int64_t>(4096, ceil_div(t.item_cap, 4)))),
                       dim3(256), 0, st, t.pos, t.nodes, t.mcnt, t.moff, n, t.item_node, t.item_cap, t.mom_part, t.mom,
                       t.mlist, t.mom_flag + 3);
    hipLaunchKernelGGL(oct_mom_reduce, dim3(256), dim3(256), 0, st, t.mcnt, t.moff, t.mlist, t.mom_flag + 3, t.item_cap,
                       t.mom_part, t.mom);
    TSNE_LAUNCH_CHECK();
}

// Largest D with 72 theta^2 D^2 (1 + 8 D) <= the near-exact tolerance
// (Options::near_tol3_early / near_tol3_late): the 2-D bound (bhtree.hip
// bh_near_dmax) scaled by 12/8 for the larger 3-D cell diagonal (second-order
// remainder (2 + 8D) r^2 / 2 with r^2 <= 12 h^2 instead of 8 h^2).
static double oct_near_dmax(const tsne_ctx *ctx, double theta, bool late) {
    if (!(theta > 0.0)) return __builtin_inf();
    const double tol = late ? ctx->opts.near_tol3_late : ctx->opts.near_tol3_early;
    if (!(tol > 0.0)) return -1.0;
    double d = std::sqrt(tol / (72.0 * theta * theta));
    while (72.0 * theta * theta * d * d * (1.0 + 8.0 * d) > tol) d *= 0.99;
    return d;
}

void oct_repulsion(tsne_ctx *ctx, const OctTree &t, double theta, int64_t s0, int64_t s1, double *dF, double *dz,
                   const int32_t *qlist) {
    if (s1 <= s0) return;
    static const bool debug = getenv("TSNE_DEBUG_OCT") != nullptr;   // traversal counters on stderr (synchronises)
    unsigned long long *dbg = nullptr;
    if (debug) {
        dbg = ctx->ws.get<unsigned long long>("oct.dbg", 8);
        TSNE_HIP(hipMemsetAsync(dbg, 0, 8 * sizeof(unsigned long long), ctx->stream));
    }
    // the record traversals: 64 queries per wave (oct_records 2), or 8 (1);
    // with oct_layout_switch > 0 the layout follows the embedding's size each
    // iteration (device-side: both launched, one returns at once): the
    // 8-query one while the root half-width is below oct_layout_switch x the
    // near-exact radius (its dense tiles have sparse lane masks there), the
    // 64-query one above (C4 transition, profiles/r04_s16_c4_probe_layouts.jsonl)
    const bool sw = ctx->opts.oct_records == 2 && ctx->opts.oct_layout_switch > 0.0 && t.near_dmax > 0.0;
    const double wthr = sw ? ctx->opts.oct_layout_switch * std::sqrt(t.near_dmax) : 0.0;
    if (ctx->opts.oct_records == 2) {
        const int64_t nw = ceil_div(s1 - s0, 64);
        auto k64 = debug ? oct_traverse64<true> : oct_traverse64<false>;
        hipLaunchKernelGGL(k64, dim3(ceil_div(nw, 4)), dim3(256), 0, ctx->stream, t.pos, t.dupc, t.nodes, t.orec,
                           t.meta, theta, s0, s1, qlist, t.mom_flag, t.mtask, t.mtask_n, dF, dz, dbg,
                           ctx->opts.mom3_tol, t.W, wthr, sw ? 2 : 0);
    }
    if (ctx->opts.oct_records == 1 || sw) {
        const int64_t rw = ceil_div(s1 - s0, OQ);
        auto k8 = debug ? oct_traverse_rec<true> : oct_traverse_rec<false>;
        hipLaunchKernelGGL(k8, dim3(ceil_div(rw, 4)), dim3(256), 0, ctx->stream, t.pos, t.dupc, t.nodes, t.orec,
                           t.meta, theta, s0, s1, qlist, t.mom_flag, t.mtask, t.mtask_n, dF, dz, dbg,
                           ctx->opts.mom3_tol, t.W, wthr, sw ? 1 : 0);
    }
    if (ctx->opts.oct_records == 0) {   // the binary-node walk
        auto kb = debug ? oct_traverse<true> : oct_traverse<false>;
        hipLaunchKernelGGL(kb, dim3(ceil_div(ceil_div(s1 - s0, 64), 4)), dim3(256), 0, ctx->stream, t.pos, t.dupc,
                           t.nodes, t.meta, theta, t.near_dmax, s0, s1, qlist, t.mom_flag, t.mtask, t.mtask_n, dF, dz,
                           dbg, ctx->opts.mom3_tol);
    }
    hipLaunchKernelGGL(oct_mom_apply, dim3(ceil_div(s1 - s0, 256)), dim3(256), 0, ctx->stream, t.pos, t.nodes, t.mom,
                       t.mtask, t.mtask_n, s0, s1, qlist, dF, dz);
    if (debug) {
        unsigned long long h[8];
        TSNE_HIP(hipMemcpy(h, dbg, sizeof(h), hipMemcpyDeviceToHost));
        const double q = (double)(s1 - s0);
        fprintf(stderr, "[oct] queries=%lld pops/wave=%.1f child_evals/query=%.1f dense_pts/query=%.1f "
                "declined/query=%.2f moment_tasks/query=%.2f\n", (long long)(s1 - s0), h[0] / (q / 64.0), h[1] / q,
                h[2] / q, h[3] / q, h[4] / q);
    }
    TSNE_LAUNCH_CHECK();
}

}  // namespace tsne
