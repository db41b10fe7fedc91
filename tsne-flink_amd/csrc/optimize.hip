// optimize.hip -- gradient combine, updateEmbedding, centerEmbedding and the
// device-resident optimize loop (TsneHelpers.scala:221-430) on gfx950.
//
// Per global iteration t (1-based, TsneHelpers.scala:403-427 phases):
//   ex  = earlyExaggeration if t <= min(T,20) + min(T-20, 81) else 1
//   mom = initialMomentum if t <= min(T,20) else finalMomentum
//   1. quadtree of the full Y (every rank builds the identical tree), or the
//      root-tile shortcut while the embedding is small (bhtree.hip)
//   2. BH repulsion for this rank's own points (its query list)
//   3. Z = sum z (TsneHelpers.scala:266): the per-iteration all-reduce
//   4. attraction per owned row of P over the CSR row (q = 1/(1+metric(y_i,
//      y_j)), TsneHelpers.scala:290-302; side stream outside loss
//      iterations), loss terms every 10th iteration, then combine_update:
//      grad = attr - F/Z (:311-317), gains/momentum/step (:341-369) -> Ynew
//   5. [multi-GPU] ragged all-gather of the owned Ynew slices
//   6. centre: Y = Ynew - mean(Ynew) (:320-329)
//
// Internal labels.  The optimizer keeps its own copy of P (full, every rank)
// and of the working set, indexed by internal point labels: P's graph order
// at setup (connected components, BFS levels), then every RELABEL_EVERY
// iterations the current Morton order of the embedding when that keeps more
// of P's edges local -- rows consecutive in memory gather Y_j from nearby
// labels, so the CSR attraction's gathers hit the L2.  Rank r owns a range of
// labels (cost-balanced cuts at relabels).  The caller's Y, upd and gains
// are written back in the original order by tsne_dev_opt_sync.
#include <hipcub/hipcub.hpp>

#include "bhtree.hpp"
#include "octree.hpp"

namespace tsne {

// one tile of the tiled attraction (attract_tiles): the entries of a row
// block whose column lies in one window of labels, as 64-row slices
struct ATile {
    int32_t s0;    // first slice
    int32_t ns;    // slices
    int32_t cb;    // column window
    int32_t rb;    // row block
};
struct ASlice {
    int64_t base;    // first entry (step 0, lane 0)
    int32_t width;   // steps: entries of the slice's first (longest) lane
    int32_t wide;    // 1: one long row split over the 64 lanes (wave-reduced)
    int32_t j0;      // first (sorted) segment
    int32_t cnt;     // segments (rows): <= 64, or 1 for a wide slice
};

struct OptState {
    tsne_params p{};
    int C = 2;
    int64_t n = 0, nnz = 0;
    // caller buffers (original order, n x C)
    double *Yu = nullptr, *updu = nullptr, *gainsu = nullptr;
    // the caller's P (original point order, every rank holds it), copied once
    int64_t *rp0 = nullptr;
    int32_t *col0 = nullptr;
    double *val0 = nullptr;
    // 2-D: this rank's rows (labels [L0, L1)) with columns in labels, rebuilt
    // from P0 at every relabel; row pointer local (rpw[r] for label L0 + r)
    int64_t *rpw = nullptr;
    int32_t *colw = nullptr;
    double *valw = nullptr;
    // labels: working set in label order (full n on every rank; upd / gains
    // are current on a rank only for its own labels between relabels)
    double *Y[2] = {nullptr, nullptr}, *upd[2] = {nullptr, nullptr}, *gains[2] = {nullptr, nullptr};
    int32_t *orig[2] = {nullptr, nullptr};   // label -> original index
    int32_t *lab = nullptr;                  // original index -> label
    int cur = 0;
    std::vector<int64_t> own;                // world + 1 label cuts (identical on every rank)
    int64_t L0 = 0, L1 = 0;
    int64_t *rowlen = nullptr;
    void *scan_tmp = nullptr;
    size_t scan_tmp_bytes = 0;
    int32_t *qlist = nullptr, *qcnt = nullptr, *qoff = nullptr;   // world > 1: this rank's BH queries
    void *qscan_tmp = nullptr;
    size_t qscan_tmp_bytes = 0;
    unsigned long long *lscore = nullptr;    // locality_score counters
    int relabels = 0, relabel_checks = 0;

    double *Ynew = nullptr;   // n x C (label order)
    double2 *F = nullptr;     // n, sorted order
    double2 *attr = nullptr;  // owned rows
    unsigned long long *bcost = nullptr;   // 256-position bucket costs of the last traversal
    int64_t *bounds = nullptr;             // world + 1 (device): cost-balanced cuts
    double *z = nullptr;      // n, sorted order
    double *scal = nullptr;   // [0] Z, [1] loss, [2..4] mean
    double *part = nullptr;   // reduction partials
    double *part2 = nullptr;  // second-level partials (NPART)
    double *loss = nullptr;   // per loss slot
    int32_t loss_slots = 0;
    std::vector<int32_t> loss_written;
    unsigned long long *visits = nullptr;
    BHTree tree;
    // 3-D embeddings (nComponents = 3, the SURVEY.md 8f octree extension):
    // labels stay the original indices (no relabel); owned rows are read
    // straight from P0; F3 (n x 3, sorted order) and attr3 (owned x 3).
    OctTree otree;
    double *F3 = nullptr, *attr3 = nullptr;
    bool profile = false;
    hipEvent_t ev[6] = {};
    // The attraction sums need only Y and P (not F or Z), so outside loss
    // iterations they run on a second stream concurrently with the BH
    // traversal (a latency-bound kernel that leaves CUs idle).
    hipStream_t side = nullptr;
    hipEvent_t ev_y = nullptr, ev_attr = nullptr;
    // per launch of the attraction kernel (ctx->timers "opt.attract"): its
    // iteration and whether it ran alone on the main stream (loss iterations)
    // or on the side stream concurrently with the BH traversal
    // (kept in step with the stage timer: its last StageTimers::CAP launches)
    std::deque<std::pair<int32_t, int32_t>> attract_iter;
    void log_attract(int32_t t, int32_t kind) {
        attract_iter.push_back({t, kind});
        while (attract_iter.size() > StageTimers::CAP) attract_iter.pop_front();
    }
    double *mpart = nullptr;  // centring mean: block partials of combine_update
    // tiled attraction layout of the owned rows (attract_tiles), rebuilt with them
    bool at_on = false;
    int64_t at_nrb = 0, at_ncb = 0;
    int64_t at_rbs = 0;       // rows per row block (<= the config's RB: the grid covers the CUs)
    int at_cfg = 0;
    int at_pipe = 0;   // Options::attract_pipe when the layout was built
    int at_dyn = 0;    // Options::attract_dyn
    bool morton_labels = false;   // the labels follow the embedding's Morton order (a relabel happened)
    ATile *at_tiles = nullptr;
    int32_t *at_rbt = nullptr;
    ASlice *at_slices = nullptr;
    uint32_t *at_srow = nullptr;
    uint16_t *at_pk = nullptr;
    double *at_pv = nullptr;
    double last_ms[5] = {0, 0, 0, 0, 0};
    int64_t last_visits[10] = {};
    int64_t last_mhz = 0;   // the traced traversal's waves' shader clock (MHz)
    // tree partition (Options::bh_split, several ranks, 2-D): cuts of the sorted
    // points (world + 1), this rank's aligned [lo, hi) + overflow flag, the
    // ranks' traversal costs (all-reduced), F in label order (reduce-scatter)
    int64_t *pcuts = nullptr;
    int32_t *plim = nullptr;
    unsigned long long *pcost = nullptr;
    double2 *Fl = nullptr;
    bool split_last = false;   // the last iteration used the tree partition
};

// The sharded code path (query lists, collectives, centring from the gathered
// embedding) runs whenever the context has a communicator: world > 1, or a
// world-1 communicator made with Options::comm_world1 (transport tests).
static inline bool sharded(const tsne_ctx *ctx) { return ctx->comm != nullptr; }

// TSNE_DEBUG_TILES=1: layout and per-iteration BH / tile diagnostics on stderr
// (synchronises; a debug print, no effect on results)
static bool debug_tiles() {
    static const bool on = getenv("TSNE_DEBUG_TILES") != nullptr;
    return on;
}

namespace {

constexpr int NPART = 512;
constexpr int RELABEL_EVERY = 25;

__device__ __forceinline__ double jmax(double a, double b) {  // java.lang.Math.max
    if (a != a) return a;
    if (b != b) return b;
    return a >= b ? a : b;
}

// Deterministic sum of v[0..n) (stride elements, component c) into part[block].
__global__ void reduce_partial(const double *__restrict__ v, int64_t n, int stride, int c,
                               double *__restrict__ part) {
    __shared__ double sw[4];
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        s += v[i * stride + c];
    s = wave_sum(s);
    if (lane_id() == 0) sw[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (sw[0] + sw[1]) + (sw[2] + sw[3]);
}

// Sum of v[0 .. *np) into NPART block partials (reduce_partial with a device count).
__global__ void reduce_partial_devn(const double *__restrict__ v, const int64_t *__restrict__ np,
                                    double *__restrict__ part) {
    __shared__ double sw[4];
    const int64_t n = *np;
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        s += v[i];
    s = wave_sum(s);
    if (lane_id() == 0) sw[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (sw[0] + sw[1]) + (sw[2] + sw[3]);
}

// Z-free KL terms: the kernels summed P ln(P (1 + metric)); the loss adds
// ln(Z) sum p (p = ex P over this rank's owned entries, sum P in scal[6])
// once Z is known.
__global__ void loss_add_lnz(double *scal, double ex) {
    if (threadIdx.x == 0) scal[1] += log(scal[0]) * (scal[6] * ex);
}
__global__ void set_unit(double *x) {
    if (threadIdx.x == 0) *x = 1.0;
}

__global__ void reduce_final(const double *__restrict__ part, int np, double *__restrict__ out,
                             double scale_div) {
    __shared__ double sw[4];
    double s = 0.0;
    for (int b = threadIdx.x; b < np; b += blockDim.x) s += part[b];
    s = wave_sum(s);
    if (lane_id() == 0) sw[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = (sw[0] + sw[1]) + (sw[2] + sw[3]);
        *out = scale_div > 0.0 ? t / scale_div : t;
    }
}

// q = 1 / (1 + metric(y_i, y_j)) with the input metric on 2-D points
// (TsneHelpers.scala:293), metric fixed at compile time; v_rcp_f64 + two
// Newton steps.
template <int MET>
__device__ __forceinline__ double qterm_t(double ax, double ay, double bx, double by, double &x) {
    double m;
    if (MET == TSNE_METRIC_COSINE) {
        const double dt = __dadd_rn(__dmul_rn(ax, bx), __dmul_rn(ay, by));
        const double na = sqrt(__dadd_rn(__dmul_rn(ax, ax), __dmul_rn(ay, ay)));
        const double nb = sqrt(__dadd_rn(__dmul_rn(bx, bx), __dmul_rn(by, by)));
        m = 1.0 - dt / (na * nb);
    } else {
        const double dx = __dsub_rn(ax, bx), dy = __dsub_rn(ay, by);
        const double s2 = __dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy));
        m = MET == TSNE_METRIC_EUCLIDEAN ? sqrt(s2) : s2;
    }
    x = 1.0 + m;
    double r = __builtin_amdgcn_rcp(x);
    r = __fma_rn(r, __fma_rn(-x, r, 1.0), r);
    r = __fma_rn(r, __fma_rn(-x, r, 1.0), r);
    return r;
}
// The tiled attraction's q (attract_tiles), given d = a - b: the sqeuclidean
// 1 + |d|^2 as an FMA chain and v_rcp_f64 + one Newton step (within 11 ulp,
// as recip_bh) -- 4 fp64 operations fewer per entry than qterm_t; x = 1 + metric.
template <int MET>
__device__ __forceinline__ double qforce_t(double ax, double ay, double bx, double by, double dx, double dy,
                                           double &x) {
    if (MET == TSNE_METRIC_COSINE) {
        const double dt = __dadd_rn(__dmul_rn(ax, bx), __dmul_rn(ay, by));
        const double na = sqrt(__dadd_rn(__dmul_rn(ax, ax), __dmul_rn(ay, ay)));
        const double nb = sqrt(__dadd_rn(__dmul_rn(bx, bx), __dmul_rn(by, by)));
        x = 1.0 + (1.0 - dt / (na * nb));
    } else if (MET == TSNE_METRIC_EUCLIDEAN) {
        x = 1.0 + sqrt(__fma_rn(dx, dx, dy * dy));
    } else {
        x = __fma_rn(dx, dx, __fma_rn(dy, dy, 1.0));
    }
    const double r = __builtin_amdgcn_rcp(x);
    return __fma_rn(r, __fma_rn(-x, r, 1.0), r);
}
template <int MET>
__device__ __forceinline__ double qterm_t(double ax, double ay, double bx, double by) {
    double x;
    return qterm_t<MET>(ax, ay, bx, by, x);
}

// ln x in fp64 for the KL terms (the loss), ~4x fewer instructions than the
// libm log: x = 2^e m with m in [1/sqrt2, sqrt2), ln m = 2 atanh(s),
// s = (m - 1) / (m + 1) (|s| <= 0.1716, v_rcp_f64 + two Newton steps), the
// odd series to s^21 (remainder < 3e-17 relative), e ln2 in two parts
// (fdlibm's split).  Within a few ulp of log(); zero, negative, infinite
// and NaN arguments take log() itself (0 ln 0 stays NaN).
__device__ __forceinline__ double log_kl(double x) {
    if (!(x >= 0x1p-1022 && x < INFINITY)) return log(x);
    const long long b = __double_as_longlong(x);
    int e = (int)((b >> 52) & 0x7ff) - 1023;
    double m = __longlong_as_double((b & 0x000fffffffffffffll) | 0x3ff0000000000000ll);
    if (m > 1.4142135623730951) { m *= 0.5; ++e; }
    const double f = m - 1.0;   // exact
    const double d = 2.0 + f;
    double r = __builtin_amdgcn_rcp(d);
    r = __fma_rn(r, __fma_rn(-d, r, 1.0), r);
    r = __fma_rn(r, __fma_rn(-d, r, 1.0), r);
    const double s = f * r, s2 = s * s;
    double p = 2.0 / 21.0;
    p = __fma_rn(p, s2, 2.0 / 19.0);
    p = __fma_rn(p, s2, 2.0 / 17.0);
    p = __fma_rn(p, s2, 2.0 / 15.0);
    p = __fma_rn(p, s2, 2.0 / 13.0);
    p = __fma_rn(p, s2, 2.0 / 11.0);
    p = __fma_rn(p, s2, 2.0 / 9.0);
    p = __fma_rn(p, s2, 2.0 / 7.0);
    p = __fma_rn(p, s2, 2.0 / 5.0);
    p = __fma_rn(p, s2, 2.0 / 3.0);
    const double lnm = __fma_rn(s * s2, p, 2.0 * s);
    const double de = (double)e;
    return __fma_rn(de, 6.93147180369123816490e-01, __fma_rn(de, 1.90821492927058770002e-10, lnm));
}

// Attraction over the CSR rows [r0, r1) (TsneHelpers.scala:269-306):
// attr_i = sum_j ex P_ij q_ij (y_i - y_j), and with LOSS the KL terms
// ex P_ij ln(ex P_ij / (q_ij / Z)).  LPR lanes per row, 64/LPR rows per wave
// step; each lane issues U (col, val) loads and then U dependent Y_j gathers
// before any arithmetic, so a row of <= LPR*U entries costs two memory round
// trips.  Tail slots gather Y_i with P = 0 (exact no-ops in the sums).
// Persistent, XCD-partitioned grid (gridDim.x a multiple of 8): the blocks
// the dispatcher places on XCD x (blockIdx % 8 == x) stride over the x-th
// contiguous eighth of the Morton-ordered rows, so that XCD's L2 holds the
// spatially local Y_j of its rows, and waves stay resident across rows (PMC:
// one-row-per-wave launches kept only ~3.7 waves per SIMD in flight).
template <int LPR, int U, bool LOSS, int MET>
__global__ __launch_bounds__(256) void attract_rows(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col, const double *__restrict__ val,
    int64_t r0, int64_t r1, const double *__restrict__ Y, const double *__restrict__ scal, double ex,
    double2 *__restrict__ attr, double *__restrict__ lpart) {
    __shared__ double sl[4];
    constexpr int RPW = 64 / LPR;   // rows per wave step
    const int sub = threadIdx.x & (LPR - 1);
    const int x = blockIdx.x % NUM_XCD;
    const int64_t bpx = gridDim.x / NUM_XCD;                   // blocks per XCD
    const int64_t nrows = r1 - r0;
    const int64_t q0 = r0 + nrows * x / NUM_XCD, q1 = r0 + nrows * (x + 1) / NUM_XCD;
    const int64_t wv = (int64_t)(blockIdx.x / NUM_XCD) * 4 + (threadIdx.x >> 6);
    const int64_t nwv = bpx * 4;
    const int rsub = (threadIdx.x & 63) / LPR;
    const double Z = LOSS ? scal[0] : 1.0;
    double lsum = 0.0;
    for (int64_t i = q0 + wv * RPW + rsub; i - rsub < q1; i += nwv * RPW) {
        const bool live = i < q1;
        double fx = 0.0, fy = 0.0;
        double yx = 0.0, yy = 0.0;
        if (live) {
            const double2 yi = *reinterpret_cast<const double2 *>(Y + 2 * i);
            yx = yi.x; yy = yi.y;
            const int64_t e1 = row_ptr[i + 1];
            for (int64_t e = row_ptr[i] + sub; e < e1; e += LPR * U) {
                int32_t j[U];
                double pv[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int64_t o = e + LPR * u;
                    const bool in = o < e1;
                    j[u] = in ? col[o] : (int32_t)i;
                    pv[u] = in ? val[o] : 0.0;
                }
                double jx[U], jy[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const double2 yj = *reinterpret_cast<const double2 *>(Y + 2 * (int64_t)j[u]);
                    jx[u] = yj.x; jy[u] = yj.y;
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const double pij = __dmul_rn(pv[u], ex);
                    const double q = qterm_t<MET>(yx, yy, jx[u], jy[u]);
                    const double sc = __dmul_rn(pij, q);
                    fx = __dadd_rn(fx, __dmul_rn(sc, __dsub_rn(yx, jx[u])));
                    fy = __dadd_rn(fy, __dmul_rn(sc, __dsub_rn(yy, jy[u])));
                    if (LOSS && e + LPR * u < e1) lsum += pij * log(pij / (q / Z));
                }
            }
        }
#pragma unroll
        for (int o = LPR / 2; o > 0; o >>= 1) {
            fx += __shfl_xor(fx, o, LPR);
            fy += __shfl_xor(fy, o, LPR);
        }
        if (live && sub == 0) attr[i - r0] = make_double2(fx, fy);
    }
    if (LOSS) {
        lsum = wave_sum(lsum);
        if (lane_id() == 0) sl[threadIdx.x >> 6] = lsum;
        __syncthreads();
        if (threadIdx.x == 0) lpart[blockIdx.x] = (sl[0] + sl[1]) + (sl[2] + sl[3]);
    }
}

// ---- Tiled attraction (the optimizer's own rows of P, rebuilt with the labels)
// attract_rows is bound by its Y_j gathers: 16 B from a random line of a
// 1.6 MB blob of Y per entry, each an L1 miss served by the L2, at the CU's
// outstanding-miss limit (~0.11 misses/cycle/CU) -- 0.17 of the HBM roofline.
// Here the owned rows are cut into row blocks of RB rows and their entries
// regrouped by column window of W labels.  A "tile" (row block, window) is
// processed by one workgroup: it copies the window's Y into LDS (coalesced
// 16-byte loads, from L2), then sums the tile's entries with Y_j from LDS.
// Within a tile each row is one lane of a 64-row slice, the tile's rows sorted
// by their entry count (descending), and a slice is stored in jagged-diagonal
// order: step k holds the k-th entry of every lane whose row has more than k,
// contiguously (those lanes are a prefix, as the counts descend) -- the
// loads of a step are coalesced and no slot is padding.  Per entry only the
// bytes of a CSR pair cross HBM: a 16-bit column offset within the window and
// the value (10 B instead of 12).  A lane sums its row's entries of the tile
// in the row's own order and adds the sum to the row's LDS accumulator; every
// row has exactly one lane per tile, so nothing is shared and every sum runs
// in one fixed order (bit-reproducible).
template <int RB_, int W_, int NT_>
struct ATCfg {
    static constexpr int RB = RB_, W = W_, NT = NT_, WAVES = NT_ / 64;
    static constexpr int ROWBITS = __builtin_ctz(RB_);
    static_assert((RB_ & (RB_ - 1)) == 0 && RB_ <= 4096 && W_ <= 65536, "tile packing");
};
// Measured at C3 (window loss launch / non-loss launch): 4096 x 5888 1.12 /
// 0.77 ms, 4096 x 5632 1.45 / 0.79 (before the division-free loss), 2048 x
// 3840 1.59 / 1.14, 1024 x 3840 (2 workgroups per CU) 2.28 / 1.13: fewer,
// longer row segments per tile win over occupancy.
// The row block shrinks with the owned rows (a rank of a multi-GPU run) so
// that the grid still covers the CUs: the largest of 4096 / 2048 / 1024 / 512
// rows giving at least one workgroup per CU.
using ATCfg0 = ATCfg<512, 5888, 1024>;    // 102 KB LDS
using ATCfg1 = ATCfg<1024, 5888, 1024>;   // 110 KB
using ATCfg2 = ATCfg<2048, 5888, 1024>;   // 126 KB
using ATCfg3 = ATCfg<4096, 5888, 1024>;   // 156 KB
// 3-D (attract_tiles3): 24-byte points, so a smaller window
using ATCfg3D = ATCfg<2048, 4096, 1024>;   // 96 KB window + 48 KB accumulators
using ATCfg3Ds = ATCfg<512, 4096, 1024>;   // 96 + 12 KB: a rank's share of the rows
#ifndef AT_DIAG
#define AT_DIAG 0   // 1 / 2 / 3: diagnostic builds of attract_tiles (timing only; see DESIGN.md 6, rounds 5 and 6)
#endif
#ifndef AT_UNROLL
#define AT_UNROLL 12
#endif
constexpr int AT_U = AT_UNROLL;   // jagged steps whose loads are issued together
#ifndef AT_NT
#define AT_NT 1   // attract_tiles' entry loads nontemporal (round 6)
#endif
constexpr int AT_LENBITS = 20;    // slice lane word: local row << 20 | entries in the tile

constexpr uint32_t AT_OOB = 0x80000000u;   // >= the descriptors' range: reads 0

__device__ __forceinline__ __amdgpu_buffer_rsrc_t at_rsrc(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, 0x7ffffff0, 0x00020000);
}
// the tile window into LDS: all loads before the first store, every store
// unconditional (indices past the window clamped onto its last point, whose
// writers all hold the same value), so no load can sink into a branch
template <int WN, int NT>
__device__ __forceinline__ void at_window_regs(double2 (&yv)[(WN + NT - 1) / NT], const double2 *src, int wn, int tid) {
#pragma unroll
    for (int k = 0; k < (WN + NT - 1) / NT; ++k) yv[k] = src[min(tid + k * NT, wn - 1)];
}
template <int WN, int NT>
__device__ __forceinline__ void at_window_store(double2 *win, const double2 (&yv)[(WN + NT - 1) / NT], int tid) {
#pragma unroll
    for (int k = 0; k < (WN + NT - 1) / NT; ++k) win[min(tid + k * NT, WN - 1)] = yv[k];
}

// A wave's next slice of the current tile: an LDS counter per tile parity
// (lane 0's atomic, broadcast)
__device__ __forceinline__ int at_claim(int *c) {
    int v = 0;
    if (lane_id() == 0) v = atomicAdd(c, 1);
    return __builtin_amdgcn_readfirstlane(v);
}

// One workgroup per row block (owned rows [b0, b0 + RB) of [0, rows), label
// r0 + local row); XCD-chunked block order.  attr / lpart as attract_rows.
// DYN (Options::attract_dyn, round 6): a tile's slices are claimed by the
// waves from a counter instead of dealt round-robin.  The slices come sorted
// by descending width, so round-robin gives wave 0 the widest of every 16 and
// the other waves wait for it at the tile's barrier (PMC: waves wait 58 % of
// their lifetime, 22 % on their own loads).  Every row has one slice per tile
// and the tiles keep their order, so each accumulator receives the same terms
// in the same order: the sums are bit-identical either way.  (Not for the
// loss: a wave's partial would sum whichever slices it claimed, so loss
// launches keep the round-robin deal.)
template <class CF, bool LOSS, int MET, bool DYN = false>
__global__ __launch_bounds__(CF::NT) void attract_tiles(
    const ATile *__restrict__ tiles, const int32_t *__restrict__ rbt, const ASlice *__restrict__ slices,
    const uint32_t *__restrict__ srow, int64_t rows, int64_t r0, int64_t n, const uint16_t *__restrict__ pk,
    const double *__restrict__ pv, const double *__restrict__ Y, const double *__restrict__ scal, double ex,
    int64_t xcd_chunk, double2 *__restrict__ attr, double *__restrict__ lpart, int64_t rbs) {
    constexpr int RB = CF::RB, W = CF::W, NT = CF::NT, WAVES = CF::WAVES;
    __shared__ double2 win[W];
    __shared__ double2 acc[RB];
    __shared__ double sl[WAVES];
    __shared__ int claim[2];
    const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const int64_t rb = xcd_chunk > 0 ? xcd_block_chunked(blockIdx.x, gridDim.x, xcd_chunk) : (int64_t)blockIdx.x;
    const int64_t b0 = rb * rbs;   // rbs <= RB rows per block (build_attract_tiles)
    const int nr = (int)min(rbs, rows - b0);
    const double2 *Y2 = reinterpret_cast<const double2 *>(Y);
    const double2 *Yrow = Y2 + r0 + b0;
    for (int i = tid; i < nr; i += NT) acc[i] = make_double2(0.0, 0.0);
    if (DYN && tid < 2) claim[tid] = 0;
    const double Z = LOSS ? scal[0] : 1.0;
    double lsum = 0.0;
    constexpr int WL = (W + NT - 1) / NT;
    const int t0 = rbt[rb], t1 = rbt[rb + 1];
    for (int t = t0; t < t1; ++t) {
        const ATile tl = tiles[t];
#if AT_DIAG != 3
        {   // the tile's window: all of a thread's loads in flight before its LDS stores
            // (round 6: unconditional stores; with `if (i < wn)` the compiler sank each
            // load into its store's branch and the copy took WL dependent round trips)
            const int64_t base = (int64_t)tl.cb * W;
            double2 yv[WL];
            at_window_regs<W, NT>(yv, Y2 + base, (int)min((int64_t)W, n - base), tid);
            at_window_store<W, NT>(win, yv, tid);
        }
#endif
        __syncthreads();
        const int s0 = tl.s0, send = tl.s0 + tl.ns;
        // the wave's slices s0 + w, s0 + w + WAVES, ... (DYN: claimed); the next
        // slice's record and lane word are fetched during the current one
        if (DYN && tid == 0) claim[(t + 1) & 1] = 0;   // the next tile's counter: its last claim was before this barrier
        int s = DYN ? s0 + at_claim(&claim[t & 1]) : s0 + w;
        ASlice sd{};
        uint32_t rl = 0;
        if (s < send) {
            sd = slices[s];
            rl = srow[(int64_t)s * 64 + lane];
        }
        while (s < send) {
            const int len = (int)(rl & ((1u << AT_LENBITS) - 1)), lrow = (int)(rl >> AT_LENBITS);
            double2 yi = make_double2(0.0, 0.0);
#if AT_DIAG != 3
            if (len > 0) yi = Yrow[lrow];
#endif
            const int sn = DYN ? s0 + at_claim(&claim[t & 1]) : s + WAVES;
            ASlice sdn{};
            uint32_t rln = 0;
            double fx = 0.0, fy = 0.0;
            int64_t off = sd.base;   // wave-uniform: the current step's first entry
            for (int k0 = 0; k0 < sd.width; k0 += AT_U) {
                uint32_t cu[AT_U];   // one register each: a packed 16-bit array would wait on every load
                double vu[AT_U];
#pragma unroll
                for (int u = 0; u < AT_U; ++u) {
                    const int k = k0 + u;
                    cu[u] = 0;
                    vu[u] = 0.0;
#if AT_DIAG == 2   // diagnostic build: no entry loads
                    if (k < len) { cu[u] = (uint32_t)((lane * 97 + k * 31) % W); vu[u] = 1e-9; }
#elif AT_NT   // entries read once per launch (1.6 GB at C3, past the Infinity Cache): nontemporal
                    if (k < len) {
                        cu[u] = __builtin_nontemporal_load(pk + off + lane);
                        vu[u] = __builtin_nontemporal_load(pv + off + lane);
                    }
#else
                    if (k < len) { cu[u] = pk[off + lane]; vu[u] = pv[off + lane]; }
#endif
                    off += __popcll(__ballot(len > k));   // the step's active lanes (a prefix)
                }
                if (k0 == 0 && sn < send) {
                    sdn = slices[sn];
                    rln = srow[(int64_t)sn * 64 + lane];
                }
#pragma unroll
                for (int u = 0; u < AT_U; ++u) {
#if AT_DIAG == 1 || AT_DIAG == 3   // diagnostic builds: loads only, no window reads or pair terms
                                    // (3: no window copy or Y_i either -- the entry stream's own rate)
                    if (k0 + u < len) { fx += vu[u]; fy += (double)cu[u]; }
                    continue;
#endif
                    if (k0 + u < len) {
                        // P q d with P's exaggeration applied to the row's total
                        // (attr below), the q d terms accumulated by FMA
                        const double2 yj = win[cu[u]];
                        const double dx = __dsub_rn(yi.x, yj.x), dy = __dsub_rn(yi.y, yj.y);
                        double x1m;   // 1 + metric = 1 / q
                        const double q = qforce_t<MET>(yi.x, yi.y, yj.x, yj.y, dx, dy, x1m);
                        const double sc = __dmul_rn(vu[u], q);
                        fx = __fma_rn(sc, dx, fx);
                        fy = __fma_rn(sc, dy, fy);
                        // P ln(P / (q / Z)) = P ln(P Z (1 + metric)): no divisions
                        // (0 ln 0 = NaN for an underflowed P, as the reference)
                        if (LOSS) {
                            const double pij = __dmul_rn(vu[u], ex);
                            lsum += pij * log_kl(pij * Z * x1m);
                        }
                    }
                }
            }
            if (sd.wide) {   // one row over the 64 lanes: a fixed-order tree
                fx = wave_sum(fx);
                fy = wave_sum(fy);
                if (lane == 0) {
                    const double2 o = acc[lrow];
                    acc[lrow] = make_double2(__dadd_rn(o.x, fx), __dadd_rn(o.y, fy));
                }
            } else if (len > 0) {
                const double2 o = acc[lrow];
                acc[lrow] = make_double2(__dadd_rn(o.x, fx), __dadd_rn(o.y, fy));
            }
            s = sn;
            sd = sdn;
            rl = rln;
        }
        __syncthreads();
    }
    for (int i = tid; i < nr; i += NT) attr[b0 + i] = make_double2(acc[i].x * ex, acc[i].y * ex);
    if (LOSS) {
        lsum = wave_sum(lsum);
        if (lane == 0) sl[w] = lsum;
        __syncthreads();
        if (tid == 0) {
            double s = 0.0;
            for (int k = 0; k < WAVES; ++k) s += sl[k];
            lpart[blockIdx.x] = s;
        }
    }
}

// ---- attract_tiles, pipelined (Options::attract_pipe, round 6)
// attract_tiles' ISA waits once per slice for ALL of that slice's loads (its
// entries and the next slice's prefetched record alike: the entry loads sit in
// exec-masked branches, so the compiler's wait counts fall back to vmcnt(0)),
// and nothing is in flight while the slice is summed; each tile's window
// copy also ran as WL dependent load -> wait -> store round trips (the loads
// were sunk into the stores' branches).  Here a wave has the entries of its
// next D slices in flight while it sums the current one, the slice records
// 2D ahead, and the next tile's window is loaded into registers during the
// current tile (WPF).  Every slice issues the same instructions: the entry
// loads are buffer loads whose lanes past their row's entries address out of
// range (0, no memory request), so the compiler's wait counts stay exact.
// A slice wider than U steps loads and sums its remaining steps in place.
// Each lane sums its row's entries in the same order as attract_tiles, so the
// results are bit-identical.
// The wave's cursor over the row block's tiles (tile t, slice s < send;
// t == t1: none)
struct ATCur {
    int t, s, send;
};
// ring R (records and lane words, 2D + 1 slices ahead) and ring E (entries
// of the first U steps and y_i, D slices ahead)
struct ATRSlot {
    uint32_t lo;   // the slice record as loaded (every lane the same address):
    int2 wd;       // first entry (< 2^31: build_attract_tiles), width, wide
    uint32_t rl;   // lane word: local row << AT_LENBITS | entries
    ATCur c;
};
template <int U>
struct ATESlot {
    uint16_t cu[U];   // widened where summed: a widening here waits for the load
    double vu[U];
    double2 yi;
    int base, width, wide, rU;   // wave-uniform; rU: entries of the first U steps
};
constexpr int AT_RU = 4;   // steps past U: loaded and summed 4 at a time

// the wave's first slice in tiles t.. (scalar loads: every value wave-uniform)
__device__ __forceinline__ ATCur atp_first(const ATile *__restrict__ tiles, int t, int t1, int w) {
    ATCur c{__builtin_amdgcn_readfirstlane(t), 0, 0};
    for (; c.t < t1; c.t = __builtin_amdgcn_readfirstlane(c.t + 1)) {
        const int s0 = __builtin_amdgcn_readfirstlane(tiles[c.t].s0);
        const int ns = __builtin_amdgcn_readfirstlane(tiles[c.t].ns);
        c.s = s0 + w;
        c.send = s0 + ns;
        if (c.s < c.send) break;
    }
    return c;
}
template <int WAVES>
__device__ __forceinline__ ATCur atp_next(const ATile *__restrict__ tiles, const ATCur &c, int t1, int w) {
    if (c.t >= t1) return c;
    ATCur d = c;
    d.s += WAVES;
    return d.s < d.send ? d : atp_first(tiles, c.t + 1, t1, w);
}
// ring R's loads: unconditional, so that every step issues the same
// instructions (past the wave's last slice a dummy slice's, whose entries are
// loaded but never summed); nothing consumes them until the entries' issue
// (a select on the lane word here would wait for it at once).  The record
// goes through buffer loads: vector memory, counted in order with the rest
// (scalar loads share their counter with the LDS reads of the sums).
__device__ __forceinline__ void atp_issue_rec(ATRSlot &x, const ASlice *__restrict__ slices,
                                              const uint32_t *__restrict__ srow, int t1, int sdummy, int lane) {
    const int s = x.c.t < t1 ? x.c.s : sdummy;
    const __amdgpu_buffer_rsrc_t rr = at_rsrc(slices + s);
    x.lo = __builtin_amdgcn_raw_buffer_load_b32(rr, 0u, 0, 0);   // base (low word)
    typedef uint32_t u2v __attribute__((ext_vector_type(2)));
    const u2v wd = __builtin_amdgcn_raw_buffer_load_b64(rr, 8u, 0, 0);
    x.wd = make_int2((int)wd.x, (int)wd.y);
    x.rl = srow[(int64_t)s * 64 + lane];
}
template <int U>
__device__ __forceinline__ void atp_issue_entries(const ATRSlot &x, ATESlot<U> &e, const uint16_t *__restrict__ pk,
                                                  const double *__restrict__ pv, const double2 *__restrict__ Yrow,
                                                  int lane) {
    e.base = __builtin_amdgcn_readfirstlane((int)x.lo);
    e.width = __builtin_amdgcn_readfirstlane(x.wd.x);
    e.wide = __builtin_amdgcn_readfirstlane(x.wd.y);
    const int len = (int)(x.rl & ((1u << AT_LENBITS) - 1)), lrow = (int)(x.rl >> AT_LENBITS);
    const __amdgpu_buffer_rsrc_t rk = at_rsrc(pk + e.base), rv = at_rsrc(pv + e.base);
    int r = 0;   // wave-uniform: the step's first entry, relative to base
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const bool act = len > u;
        const uint32_t o = (uint32_t)(r + lane);
        e.cu[u] = __builtin_amdgcn_raw_buffer_load_b16(rk, act ? 2u * o : AT_OOB, 0, 0);
        typedef uint32_t u2v __attribute__((ext_vector_type(2)));
        const u2v v = __builtin_amdgcn_raw_buffer_load_b64(rv, act ? 8u * o : AT_OOB, 0, 0);
        e.vu[u] = __longlong_as_double((long long)(((uint64_t)v.y << 32) | v.x));
        r += __popcll(__ballot(act));
    }
    e.rU = r;
    e.yi = Yrow[lrow];   // lrow = 0 for a lane without a row: a valid point
}
template <bool LOSS, int MET>
__device__ __forceinline__ void atp_term(const double2 *win, double2 yi, uint32_t c, double v, double ex, double Z,
                                         double &fx, double &fy, double &lsum) {
    const double2 yj = win[c];
    const double dx = __dsub_rn(yi.x, yj.x), dy = __dsub_rn(yi.y, yj.y);
    double x1m;
    const double q = qforce_t<MET>(yi.x, yi.y, yj.x, yj.y, dx, dy, x1m);
    const double sc = __dmul_rn(v, q);
    fx = __fma_rn(sc, dx, fx);
    fy = __fma_rn(sc, dy, fy);
    if (LOSS) {
        const double pij = __dmul_rn(v, ex);
        lsum += pij * log_kl(pij * Z * x1m);
    }
}
// a slice's sums into its rows' accumulators (steps past U loaded in place)
template <int U, bool LOSS, int MET>
__device__ __forceinline__ void atp_sum(const ATRSlot &x, const ATESlot<U> &e, const double2 *win, double2 *acc,
                                        const uint16_t *__restrict__ pk, const double *__restrict__ pv, double ex,
                                        double Z, int lane, double &lsum) {
    const int len = (int)(x.rl & ((1u << AT_LENBITS) - 1)), lrow = (int)(x.rl >> AT_LENBITS);
    double fx = 0.0, fy = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (u < len) atp_term<LOSS, MET>(win, e.yi, e.cu[u], e.vu[u], ex, Z, fx, fy, lsum);
    if (e.width > U) {
        int64_t off = (int64_t)e.base + e.rU;
        for (int k0 = U; k0 < e.width; k0 += AT_RU) {
            uint32_t cu[AT_RU];
            double vu[AT_RU];
#pragma unroll
            for (int u = 0; u < AT_RU; ++u) {
                const int k = k0 + u;
                cu[u] = 0;
                vu[u] = 0.0;
                if (k < len) { cu[u] = pk[off + lane]; vu[u] = pv[off + lane]; }
                off += __popcll(__ballot(len > k));
            }
#pragma unroll
            for (int u = 0; u < AT_RU; ++u)
                if (k0 + u < len) atp_term<LOSS, MET>(win, e.yi, cu[u], vu[u], ex, Z, fx, fy, lsum);
        }
        // vmcnt(0): the remainder's loads are consumed in exec-masked branches,
        // so past this block the compiler would count them as outstanding and
        // make every later step wait for nearly everything in flight
        __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    if (e.wide) {   // one row over the 64 lanes: a fixed-order tree
        fx = wave_sum(fx);
        fy = wave_sum(fy);
        if (lane == 0) {
            const double2 o = acc[lrow];
            acc[lrow] = make_double2(__dadd_rn(o.x, fx), __dadd_rn(o.y, fy));
        }
    } else if (len > 0) {
        const double2 o = acc[lrow];
        acc[lrow] = make_double2(__dadd_rn(o.x, fx), __dadd_rn(o.y, fy));
    }
}
// tile t's window into LDS, then the barrier (every wave has left the previous one)
template <int W, int NT>
__device__ __forceinline__ void atp_tile_begin(double2 *win, const ATile *__restrict__ tiles, const double2 *Y2,
                                               int64_t n, int t, int tid) {
    const int64_t nb = (int64_t)__builtin_amdgcn_readfirstlane(tiles[t].cb) * W;
    double2 yv[(W + NT - 1) / NT];
    at_window_regs<W, NT>(yv, Y2 + nb, (int)min((int64_t)W, n - nb), tid);
    at_window_store<W, NT>(win, yv, tid);
    __syncthreads();
}

template <class CF, int D, int U, bool LOSS, int MET>
__global__ __launch_bounds__(CF::NT) void attract_tiles_pipe(
    const ATile *__restrict__ tiles, const int32_t *__restrict__ rbt, const ASlice *__restrict__ slices,
    const uint32_t *__restrict__ srow, int64_t rows, int64_t r0, int64_t n, const uint16_t *__restrict__ pk,
    const double *__restrict__ pv, const double *__restrict__ Y, const double *__restrict__ scal, double ex,
    int64_t xcd_chunk, double2 *__restrict__ attr, double *__restrict__ lpart, int64_t rbs) {
    constexpr int RB = CF::RB, W = CF::W, NT = CF::NT, WAVES = CF::WAVES;
    constexpr int NE = D + 1, NR = 2 * (D + 1);   // the step loop is unrolled over NR
    static_assert(D >= 1 && D <= 3 && U >= 1, "pipeline shape");
    __shared__ double2 win[W];
    __shared__ double2 acc[RB];
    __shared__ double sl[WAVES];
    const int tid = threadIdx.x, lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform for the compiler
    const int64_t rb = xcd_chunk > 0 ? xcd_block_chunked(blockIdx.x, gridDim.x, xcd_chunk) : (int64_t)blockIdx.x;
    const int64_t b0 = rb * rbs;
    const int nr = (int)min(rbs, rows - b0);
    const double2 *Y2 = reinterpret_cast<const double2 *>(Y);
    const double2 *Yrow = Y2 + r0 + b0;
    for (int i = tid; i < nr; i += NT) acc[i] = make_double2(0.0, 0.0);
    const double Z = LOSS ? scal[0] : 1.0;
    double lsum = 0.0;
    const int t0 = __builtin_amdgcn_readfirstlane(rbt[rb]), t1 = __builtin_amdgcn_readfirstlane(rbt[rb + 1]);
    if (t0 < t1) {
        const int sdummy = __builtin_amdgcn_readfirstlane(tiles[t0].s0);   // a valid slice for "no slice"
        ATRSlot R[NR];
        ATESlot<U> E[NE];
        // prologue: slices 0 .. 2D: records; 0 .. D-1: entries, issued in the
        // steps' own order (entries of j, then the record of j + D + 1), so
        // that the compiler's outstanding-load counts agree at the loop head
        R[0].c = atp_first(tiles, t0, t1, w);
#pragma unroll
        for (int j = 1; j <= 2 * D; ++j) R[j].c = atp_next<WAVES>(tiles, R[j - 1].c, t1, w);
#pragma unroll
        for (int j = 0; j <= D; ++j) atp_issue_rec(R[j], slices, srow, t1, sdummy, lane);
#pragma unroll
        for (int j = 0; j < D; ++j) {
            atp_issue_entries<U>(R[j], E[j], pk, pv, Yrow, lane);
            atp_issue_rec(R[j + D + 1], slices, srow, t1, sdummy, lane);
        }
        int tcur = t0;
        atp_tile_begin<W, NT>(win, tiles, Y2, n, t0, tid);
        // Rounds of NR steps; every step issues its loads whether or not its
        // slice exists (past the wave's last slice: dummies), only the sum is
        // conditional -- a step skipped as a whole would make the compiler
        // count fewer loads after each outstanding one and wait for nearly all
        do {
#pragma unroll
            for (int r = 0; r < NR; ++r) {   // the step of slice i, r = i mod NR
                const bool live = R[r].c.t < t1;
                while (live && tcur != R[r].c.t) {   // the wave's next slice is in a later tile
                    __syncthreads();
                    tcur = __builtin_amdgcn_readfirstlane(tcur + 1);
                    atp_tile_begin<W, NT>(win, tiles, Y2, n, tcur, tid);
                }
                atp_issue_entries<U>(R[(r + D) % NR], E[(r + D) % NE], pk, pv, Yrow, lane);   // slice i + D
                if (live) atp_sum<U, LOSS, MET>(R[r], E[r % NE], win, acc, pk, pv, ex, Z, lane, lsum);
                // slice i - 1's record slot is free: slice i + 2D + 1
                R[(r + NR - 1) % NR].c = atp_next<WAVES>(tiles, R[(r + 2 * D) % NR].c, t1, w);
                atp_issue_rec(R[(r + NR - 1) % NR], slices, srow, t1, sdummy, lane);
            }
        } while (R[0].c.t < t1);
        while (tcur + 1 < t1) {   // the barriers of the tiles this wave has no slice in
            __syncthreads();
            tcur = __builtin_amdgcn_readfirstlane(tcur + 1);
            atp_tile_begin<W, NT>(win, tiles, Y2, n, tcur, tid);
        }
        __syncthreads();
    }
    for (int i = tid; i < nr; i += NT) attr[b0 + i] = make_double2(acc[i].x * ex, acc[i].y * ex);
    if (LOSS) {
        lsum = wave_sum(lsum);
        if (lane == 0) sl[tid >> 6] = lsum;
        __syncthreads();
        if (tid == 0) {
            double s = 0.0;
            for (int k = 0; k < WAVES; ++k) s += sl[k];
            lpart[blockIdx.x] = s;
        }
    }
}

// ---- tile layout build (at every relabel; see build_attract_tiles)
// 1. key (row block * ncb + window) << rowbits | local row of every owned
//    entry (wave per row), for a stable radix sort
__global__ void at_keys(const int64_t *__restrict__ rpw, const int32_t *__restrict__ colw, int64_t rows, int64_t ncb,
                        int rowbits, int64_t rbs, int64_t W, uint64_t *__restrict__ key, int32_t *__restrict__ idx) {
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int64_t rb = r / rbs;   // row block of rbs (<= 2^rowbits) rows
    const uint64_t hi = (uint64_t)(rb * ncb);
    const uint64_t lr = (uint64_t)(r - rb * rbs);
    for (int64_t e = rpw[r] + lane_id(); e < rpw[r + 1]; e += 64) {
        key[e] = ((hi + (uint64_t)(colw[e] / W)) << rowbits) | lr;
        idx[e] = (int32_t)e;
    }
}

// 2. sorted position p <- entry perm[p]: column offset in the window, value,
//    and the start flag of each (tile, row) segment
__global__ void at_gather(const uint64_t *__restrict__ ks, const int32_t *__restrict__ perm, int64_t m, int64_t ncb,
                          int rowbits, int64_t W, const int32_t *__restrict__ colw, const double *__restrict__ valw,
                          uint16_t *__restrict__ cs, double *__restrict__ vs, int32_t *__restrict__ flag) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= m) return;
    const int64_t e = perm[p];
    const uint64_t k = ks[p];
    const int64_t cb = (int64_t)((k >> rowbits) % (uint64_t)ncb);
    cs[p] = (uint16_t)(colw[e] - cb * W);
    vs[p] = valw[e];
    flag[p] = (p == 0 || ks[p - 1] != k) ? 1 : 0;
}

// 3. segments: start, key; then (next kernel) length and the sort key
//    (tile << 20 | ~length) that orders a tile's rows by descending count
__global__ void at_segs(const uint64_t *__restrict__ ks, const int32_t *__restrict__ flag,
                        const int32_t *__restrict__ sid, int64_t m, int32_t *__restrict__ sstart,
                        uint64_t *__restrict__ skey) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= m || !flag[p]) return;
    sstart[sid[p]] = (int32_t)p;
    skey[sid[p]] = ks[p];
}
__global__ void at_seglen(const int32_t *__restrict__ sstart, const uint64_t *__restrict__ skey, int32_t ns, int64_t m,
                          int rowbits, int32_t *__restrict__ slen, uint64_t *__restrict__ okey,
                          int32_t *__restrict__ oval) {
    const int32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ns) return;
    const int32_t len = (int32_t)((g + 1 < ns ? (int64_t)sstart[g + 1] : m) - sstart[g]);
    slen[g] = len;
    okey[g] = ((skey[g] >> rowbits) << AT_LENBITS) | (uint64_t)((1u << AT_LENBITS) - 1 - (uint32_t)len);
    oval[g] = g;
}

// 4. over the sorted segments j: lengths in sorted order and tile-start flags
__global__ void at_sorted(const uint64_t *__restrict__ okey, const int32_t *__restrict__ og,
                          const int32_t *__restrict__ slen, int32_t ns, int64_t *__restrict__ lenj,
                          int32_t *__restrict__ tflag) {
    const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ns) return;
    lenj[j] = slen[og[j]];
    tflag[j] = (j == 0 || (okey[j - 1] >> AT_LENBITS) != (okey[j] >> AT_LENBITS)) ? 1 : 0;
}
// 5. tiles: first sorted segment, segment count -> slices (count / 64, scanned)
__global__ void at_tilefirst(const uint64_t *__restrict__ okey, const int32_t *__restrict__ tflag,
                             const int32_t *__restrict__ tix, int32_t ns, int64_t ncb, int32_t *__restrict__ tfirst,
                             ATile *__restrict__ tiles) {
    const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ns || !tflag[j]) return;
    const uint64_t tile = okey[j] >> AT_LENBITS;
    const int32_t t = tix[j];
    tfirst[t] = j;
    tiles[t].cb = (int32_t)(tile % (uint64_t)ncb);
    tiles[t].rb = (int32_t)(tile / (uint64_t)ncb);
}
// A row with more than AT_WIDE_MIN entries in a tile gets a slice of its own:
// the row cut into 64 consecutive pieces, one per lane, summed by a wave
// reduction -- a hub row would otherwise keep one wave busy while the
// workgroup waits for it at the tile's barrier.  (Measured at C3: wide above
// 48 entries 1.11 ms per loss launch; wide only above max(64, twice the
// slice's 64th row) 1.31 ms -- balanced lanes beat fewer slices.)
constexpr int AT_WIDE_MIN = 48;
__global__ void at_tilecount(const int32_t *__restrict__ tfirst, const int64_t *__restrict__ lenj, int32_t nt,
                             int32_t ns, int32_t *__restrict__ tns, int32_t *__restrict__ twide) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nt) return;
    const int32_t j0 = tfirst[t], cnt = (t + 1 < nt ? tfirst[t + 1] : ns) - j0;
    int32_t nw = 0;   // segments sorted by descending length
    while (nw < cnt && lenj[j0 + nw] > AT_WIDE_MIN) ++nw;
    twide[t] = nw;
    tns[t] = nw + (cnt - nw + 63) / 64;
}
// 6. slice records (one thread per tile writes its slices)
__global__ void at_slices(const int32_t *__restrict__ tfirst, const int32_t *__restrict__ tns,
                          const int32_t *__restrict__ twide, const int32_t *__restrict__ ts0,
                          const int64_t *__restrict__ lenj, const int64_t *__restrict__ ebase, int32_t nt, int32_t ns,
                          ATile *__restrict__ tiles, ASlice *__restrict__ slices) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nt) return;
    tiles[t].s0 = ts0[t];
    tiles[t].ns = tns[t];
    const int32_t j0 = tfirst[t], jend = t + 1 < nt ? tfirst[t + 1] : ns, nw = twide[t];
    for (int32_t q = 0; q < tns[t]; ++q) {
        ASlice sd;
        if (q < nw) {
            sd.j0 = j0 + q;
            sd.cnt = 1;
            sd.wide = 1;
            sd.width = (int32_t)((lenj[sd.j0] + 63) / 64);
        } else {
            sd.j0 = j0 + nw + 64 * (q - nw);
            sd.cnt = min(64, jend - sd.j0);
            sd.wide = 0;
            sd.width = (int32_t)lenj[sd.j0];
        }
        sd.base = ebase[sd.j0];
        slices[ts0[t] + q] = sd;
    }
}
// 7. one wave per slice: lane words and the jagged-diagonal scatter of the
//    lanes' rows (step k: the k-th entry of each row longer than k)
__global__ void at_fill(const ASlice *__restrict__ slices, int32_t nsl, const int32_t *__restrict__ og,
                        const int32_t *__restrict__ sstart, const uint64_t *__restrict__ skey,
                        const int64_t *__restrict__ lenj, int rowbits, const uint16_t *__restrict__ cs,
                        const double *__restrict__ vs, uint32_t *__restrict__ srow, uint16_t *__restrict__ pk,
                        double *__restrict__ pv) {
    const int64_t s = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (s >= nsl) return;
    const int lane = lane_id();
    const ASlice sd = slices[s];
    int len = 0, lrow = 0;
    int64_t src = 0;
    if (sd.wide) {   // piece `lane` of the row: entries [lane * width, ...)
        const int32_t g = og[sd.j0];
        const int64_t L = lenj[sd.j0];
        len = (int)max((int64_t)0, min((int64_t)sd.width, L - (int64_t)lane * sd.width));
        lrow = (int)(skey[g] & ((1u << rowbits) - 1));
        src = sstart[g] + (int64_t)lane * sd.width;
    } else if (lane < sd.cnt) {
        const int32_t g = og[sd.j0 + lane];
        len = (int)lenj[sd.j0 + lane];
        lrow = (int)(skey[g] & ((1u << rowbits) - 1));
        src = sstart[g];
    }
    srow[s * 64 + lane] = ((uint32_t)lrow << AT_LENBITS) | (uint32_t)len;
    int64_t off = sd.base;
    for (int k = 0; k < sd.width; ++k) {
        if (k < len) {
            pk[off + lane] = cs[src + k];
            pv[off + lane] = vs[src + k];
        }
        off += __popcll(__ballot(k < len));
    }
}

// 8. the row blocks' tile ranges: rbt[rb] = first tile of a row block >= rb
__global__ void at_ranges(const ATile *__restrict__ tiles, int32_t nt, int64_t nrb, int32_t *__restrict__ rbt) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > nt) return;
    const int64_t lo = t == 0 ? 0 : (int64_t)tiles[t - 1].rb + 1;
    const int64_t hi = t < nt ? (int64_t)tiles[t].rb : nrb;
    for (int64_t r = lo; r <= hi; ++r) rbt[r] = (int32_t)t;
}

// grad = attr - F / Z (TsneHelpers.scala:311-317); MODE 0 writes it, MODE 1
// applies updateEmbedding (TsneHelpers.scala:341-369) -> Ynew.  One thread
// per row, all accesses coalesced except F[inv[i]] (near-identity gather).
// With `mpart` (MODE 1) each block also writes the sum of its rows' Ynew
// (x, y) to mpart[2 * block]: the centring mean's partials, fused into the
// update so that centerEmbedding costs one more pass (center2); the
// mean itself is mean2_final (finalising it in the last block instead saved a
// launch but cost 3,907 same-address arrival atomics: 0.062 -> 0.085 ms).
template <int MODE>
__global__ __launch_bounds__(256) void combine_update(
    int64_t r0, int64_t r1, const double2 *__restrict__ attr, const int32_t *__restrict__ inv,
    const double2 *__restrict__ F, const double *__restrict__ scal, const double *__restrict__ Y,
    double *__restrict__ grad, double *__restrict__ Ynew, double *__restrict__ upd, double *__restrict__ gains,
    double min_gain, double mom, double lr, double *__restrict__ mpart) {
    __shared__ double sm[2][4];
    const int64_t i = r0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < r1;
    double yn[2] = {0.0, 0.0};
    if (live) {
        const double Z = scal[0];
        const double2 at = attr[i - r0];
        const double2 f = F[inv ? inv[i] : i];   // sorted order, or already by label (inv = nullptr)
        const double gx = at.x - f.x / Z, gy = at.y - f.y / Z;  // attrForce - repForce / sumQ
        if (MODE == 0) {
            grad[2 * i] = gx;
            grad[2 * i + 1] = gy;
        } else {
            const double g[2] = {gx, gy};
            const double2 u2 = *reinterpret_cast<const double2 *>(upd + 2 * i);
            const double2 g2 = *reinterpret_cast<const double2 *>(gains + 2 * i);
            const double2 y2 = *reinterpret_cast<const double2 *>(Y + 2 * i);
            const double uu[2] = {u2.x, u2.y}, gg[2] = {g2.x, g2.y}, yy[2] = {y2.x, y2.y};
            double un[2], gn[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                gn[c] = ((g[c] > 0.0) == (uu[c] > 0.0)) ? jmax(gg[c] * 0.8, min_gain) : jmax(gg[c] + 0.2, min_gain);
                un[c] = __dsub_rn(__dmul_rn(mom, uu[c]), __dmul_rn(__dmul_rn(lr, gn[c]), g[c]));
                yn[c] = __dadd_rn(un[c], yy[c]);
            }
            *reinterpret_cast<double2 *>(gains + 2 * i) = make_double2(gn[0], gn[1]);
            *reinterpret_cast<double2 *>(upd + 2 * i) = make_double2(un[0], un[1]);
            *reinterpret_cast<double2 *>(Ynew + 2 * i) = make_double2(yn[0], yn[1]);
        }
    }
    if (MODE == 1 && mpart) {
        const double sx = wave_sum(yn[0]), sy = wave_sum(yn[1]);
        if (lane_id() == 0) { sm[0][threadIdx.x >> 6] = sx; sm[1][threadIdx.x >> 6] = sy; }
        __syncthreads();
        if (threadIdx.x == 0) {
            const double px = (sm[0][0] + sm[0][1]) + (sm[0][2] + sm[0][3]);
            const double py = (sm[1][0] + sm[1][1]) + (sm[1][2] + sm[1][3]);
            mpart[2 * blockIdx.x] = px;
            mpart[2 * blockIdx.x + 1] = py;
        }
    }
}

// mean[c] = (sum of the nb block partials of component c, fixed order) / n
__global__ __launch_bounds__(256) void mean2_final(const double *__restrict__ mpart, int64_t nb, double n,
                                                   double *__restrict__ mean) {
    __shared__ double sm[2][4];
    double s[2] = {0.0, 0.0};
    for (int64_t b = threadIdx.x; b < nb; b += blockDim.x) { s[0] += mpart[2 * b]; s[1] += mpart[2 * b + 1]; }
    s[0] = wave_sum(s[0]);
    s[1] = wave_sum(s[1]);
    if (lane_id() == 0) { sm[0][threadIdx.x >> 6] = s[0]; sm[1][threadIdx.x >> 6] = s[1]; }
    __syncthreads();
    if (threadIdx.x < 2) mean[threadIdx.x] = ((sm[threadIdx.x][0] + sm[threadIdx.x][1]) + (sm[threadIdx.x][2] + sm[threadIdx.x][3])) / n;
}

// centerEmbedding (TsneHelpers.scala:320-329): Y = Ynew - mean, label order.
// The caller's copy (original point order) is written by tsne_dev_opt_sync
// (opt_sync), not here: its scattered 16-byte writes were a third of the
// update's HBM traffic per iteration (round 4: 69 of 250 MB).
__global__ __launch_bounds__(256) void center2(const double *__restrict__ Ynew, int64_t n,
                                               const double *__restrict__ mean, double *__restrict__ Y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double2 v = *reinterpret_cast<const double2 *>(Ynew + 2 * i);
    *reinterpret_cast<double2 *>(Y + 2 * i) = make_double2(v.x - mean[0], v.y - mean[1]);
}

__global__ void center_apply(const double *__restrict__ src, int64_t n, int32_t c,
                             const double *__restrict__ mean, double *__restrict__ dst) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * c) return;
    dst[e] = src[e] - mean[e % c];
}

__global__ void update_kernel(int64_t ne, const double *__restrict__ grad, double *__restrict__ Y,
                              double *__restrict__ upd, double *__restrict__ gains, double min_gain,
                              double mom, double lr) {
    int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= ne) return;
    const double g = grad[o], u = upd[o], gn0 = gains[o];
    const double gn = ((g > 0.0) == (u > 0.0)) ? jmax(gn0 * 0.8, min_gain) : jmax(gn0 + 0.2, min_gain);
    const double un = __dsub_rn(__dmul_rn(mom, u), __dmul_rn(__dmul_rn(lr, gn), g));
    gains[o] = gn;
    upd[o] = un;
    Y[o] = __dadd_rn(un, Y[o]);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// N(0, 1e-4^2) by Box-Muller on a counter-based stream keyed by seed.
__global__ void init_ws_kernel(int64_t ne, uint64_t seed, double *__restrict__ Y,
                               double *__restrict__ upd, double *__restrict__ gains) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint64_t a = splitmix64(seed ^ splitmix64(2 * (uint64_t)e));
    const uint64_t b = splitmix64(seed ^ splitmix64(2 * (uint64_t)e + 1));
    const double u1 = ((double)(a >> 11) + 1.0) * 0x1.0p-53;
    const double u2 = (double)(b >> 11) * 0x1.0p-53;
    Y[e] = 1e-4 * sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
    upd[e] = 0.0;
    gains[e] = 1.0;
}

// ---- internal labels
__global__ void iota_i32(int32_t *p, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = (int32_t)i;
}

// new label s <- old label order[s]: working set (C components) and the label
// maps orig1 (label -> original point) and lab (original point -> label)
__global__ void relabel_state(const int32_t *__restrict__ order, int64_t n, int C, const double *__restrict__ Y0,
                              const double *__restrict__ u0, const double *__restrict__ g0,
                              const int32_t *__restrict__ o0, double *__restrict__ Y1, double *__restrict__ u1,
                              double *__restrict__ g1, int32_t *__restrict__ o1, int32_t *__restrict__ lab) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const int64_t i = order[s];
    for (int c = 0; c < C; ++c) {
        Y1[C * s + c] = Y0[C * i + c];
        u1[C * s + c] = u0[C * i + c];
        g1[C * s + c] = g0[C * i + c];
    }
    const int32_t o = o0[i];
    o1[s] = o;
    lab[o] = (int32_t)s;
}

// Row lengths of the owned labels [L0, L1) from the caller's P (original order)
__global__ void own_rowlen(const int32_t *__restrict__ orig, const int64_t *__restrict__ rp0, int64_t L0, int64_t L1,
                           int64_t *__restrict__ len) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > L1 - L0) return;
    if (r == L1 - L0) { len[r] = 0; return; }
    const int64_t o = orig[L0 + r];
    len[r] = rp0[o + 1] - rp0[o];
}

// One wave per owned row: the caller's row of its original point, columns
// renamed into labels (entry order kept: the attraction sums run in the
// reference's row order whatever the labelling).
__global__ void own_rows(const int32_t *__restrict__ orig, const int32_t *__restrict__ lab,
                         const int64_t *__restrict__ rp0, const int32_t *__restrict__ c0,
                         const double *__restrict__ v0, int64_t L0, int64_t L1, const int64_t *__restrict__ rpw,
                         int32_t *__restrict__ cw, double *__restrict__ vw) {
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (r >= L1 - L0) return;
    const int64_t o = orig[L0 + r];
    const int64_t a = rp0[o], len = rp0[o + 1] - a, b = rpw[r];
    for (int64_t e = lane_id(); e < len; e += 64) {
        cw[b + e] = lab[c0[a + e]];
        vw[b + e] = v0[a + e];
    }
}

// This rank's queries: the sorted positions whose label it owns, ascending
// (a stable compaction: flags, block counts, scan, scatter).
__global__ void qlist_count(const int32_t *__restrict__ idx_sorted, int64_t n, int64_t L0, int64_t L1,
                            int32_t *__restrict__ bcnt) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool f = s < n && idx_sorted[s] >= L0 && idx_sorted[s] < L1;
    __shared__ int wc[4];
    const int c = __popcll(__ballot(f));
    if (lane_id() == 0) wc[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) bcnt[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}
__global__ void qlist_fill(const int32_t *__restrict__ idx_sorted, int64_t n, int64_t L0, int64_t L1,
                           const int32_t *__restrict__ boff, int32_t *__restrict__ qlist) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool f = s < n && idx_sorted[s] >= L0 && idx_sorted[s] < L1;
    __shared__ int wc[4];
    const uint64_t bal = __ballot(f);
    if (lane_id() == 0) wc[threadIdx.x >> 6] = __popcll(bal);
    __syncthreads();
    const int w = threadIdx.x >> 6;
    int base = boff[blockIdx.x];
    for (int k = 0; k < w; ++k) base += wc[k];
    if (f) qlist[base + __popcll(bal & lanemask_lt())] = (int32_t)s;
}

// F in label order: Fl[l] = F[inv[l]] (the tree partition's reduce-scatter
// buffer: each rank's partial sums of every point, summed at the row owners)
__global__ void f_to_label(const int32_t *__restrict__ inv, int64_t n, const double2 *__restrict__ F,
                           double2 *__restrict__ Fl) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l < n) Fl[l] = F[inv[l]];
}

// Z partial of a rank: sum of z over its query list (fixed order per block)
__global__ void reduce_list_partial(const double *__restrict__ z, const int32_t *__restrict__ qlist, int64_t m,
                                    double *__restrict__ part) {
    __shared__ double sw[4];
    double acc = 0.0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
        acc += z[qlist[k]];
    acc = wave_sum(acc);
    if (lane_id() == 0) sw[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (sw[0] + sw[1]) + (sw[2] + sw[3]);
}

// ---- locality of the CSR attraction's gathers (relabel decisions)
// Connected components (minimum original index) and BFS level from that
// root over the symmetric P: fixpoint iterations, deterministic.
__global__ void cc_pull(const int64_t *__restrict__ rp, const int32_t *__restrict__ col, int64_t n,
                        int32_t *__restrict__ comp, int32_t *__restrict__ changed) {
    const int64_t i = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (i >= n) return;
    int32_t m = comp[i];
    for (int64_t e = rp[i] + lane_id(); e < rp[i + 1]; e += 64) m = min(m, comp[col[e]]);
    m = wave_min(m);
    if (lane_id() == 0 && m < comp[i]) {
        atomicMin(&comp[i], m);
        changed[0] = 1;
    }
}
__global__ void cc_jump(int32_t *__restrict__ comp, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    comp[i] = comp[comp[comp[i]]];
}
__global__ void level_init(const int32_t *__restrict__ comp, int64_t n, int32_t *__restrict__ lev) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) lev[i] = comp[i] == (int32_t)i ? 0 : INT32_MAX;
}
__global__ void level_pull(const int64_t *__restrict__ rp, const int32_t *__restrict__ col, int64_t n,
                           int32_t *__restrict__ lev, int32_t *__restrict__ changed) {
    const int64_t i = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (i >= n) return;
    int32_t m = INT32_MAX;
    for (int64_t e = rp[i] + lane_id(); e < rp[i + 1]; e += 64) m = min(m, lev[col[e]]);
    m = wave_min(m);
    if (lane_id() == 0 && m != INT32_MAX && m + 1 < lev[i]) {
        atomicMin(&lev[i], m + 1);
        changed[0] = 1;
    }
}
__global__ void graph_keys(const int32_t *__restrict__ comp, const int32_t *__restrict__ lev, int64_t n,
                           uint64_t *__restrict__ key, int32_t *__restrict__ val) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    key[i] = ((uint64_t)(uint32_t)comp[i] << 24) | (uint64_t)min(lev[i], (1 << 24) - 1);
    val[i] = (int32_t)i;
}

// Fraction of P's edges (a fixed sample of rows) whose endpoints lie within
// `win` labels of each other: under the current labels (cnt[0]) and under the
// Morton order of this iteration's tree (cnt[1]: label l -> inv[l]).
__global__ void locality_score(const int64_t *__restrict__ rp0, const int32_t *__restrict__ c0,
                               const int32_t *__restrict__ lab, const int32_t *__restrict__ inv, int64_t n,
                               int64_t stride, int64_t nsamp, int64_t win, unsigned long long *__restrict__ cnt) {
    const int64_t k = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (k >= nsamp) return;
    const int64_t o = k * stride;
    const int64_t li = lab[o], mi = inv[li];
    unsigned long long a = 0, b = 0;
    for (int64_t e = rp0[o] + lane_id(); e < rp0[o + 1]; e += 64) {
        const int64_t lj = lab[c0[e]];
        const int64_t da = li - lj, db = mi - (int64_t)inv[lj];
        a += (da <= win && -da <= win);
        b += (db <= win && -db <= win);
    }
    a = wave_sum(a);
    b = wave_sum(b);
    if (lane_id() == 0) { atomicAdd(cnt, a); atomicAdd(cnt + 1, b); }
}

// dst[orig[i]] = src[i], c components
__global__ void scatter_to_user_c(const double *__restrict__ src, const int32_t *__restrict__ orig, int64_t n,
                                  int32_t c, double *__restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t o = orig[i];
    for (int k = 0; k < c; ++k) dst[c * o + k] = src[c * i + k];
}

// ---- 3-D (nComponents = 3) optimizer kernels
// q = 1 / (1 + metric(y_i, y_j)) on 3-D points (TsneHelpers.scala:293)
template <int MET>
__device__ __forceinline__ double qterm3(const double *a, const double *b) {
    double m;
    if (MET == TSNE_METRIC_COSINE) {
        double dt = 0.0, na = 0.0, nb = 0.0;
        for (int k = 0; k < 3; ++k) {
            dt = __dadd_rn(dt, __dmul_rn(a[k], b[k]));
            na = __dadd_rn(na, __dmul_rn(a[k], a[k]));
            nb = __dadd_rn(nb, __dmul_rn(b[k], b[k]));
        }
        m = 1.0 - dt / (sqrt(na) * sqrt(nb));
    } else {
        double s2 = 0.0;
        for (int k = 0; k < 3; ++k) {
            const double d = __dsub_rn(a[k], b[k]);
            s2 = __dadd_rn(s2, __dmul_rn(d, d));
        }
        m = MET == TSNE_METRIC_EUCLIDEAN ? sqrt(s2) : s2;
    }
    const double x = 1.0 + m;
    double r = __builtin_amdgcn_rcp(x);
    r = __fma_rn(r, __fma_rn(-x, r, 1.0), r);
    r = __fma_rn(r, __fma_rn(-x, r, 1.0), r);
    return r;
}

// qterm3's q with x = 1 + metric returned too (the tiled 3-D attraction's
// loss terms P ln(P Z x) need no division); the same arithmetic as qterm3.
template <int MET>
__device__ __forceinline__ double qforce3_t(const double *a, const double *b, double &x) {
    double m;
    if (MET == TSNE_METRIC_COSINE) {
        double dt = 0.0, na = 0.0, nb = 0.0;
        for (int k = 0; k < 3; ++k) {
            dt = __dadd_rn(dt, __dmul_rn(a[k], b[k]));
            na = __dadd_rn(na, __dmul_rn(a[k], a[k]));
            nb = __dadd_rn(nb, __dmul_rn(b[k], b[k]));
        }
        m = 1.0 - dt / (sqrt(na) * sqrt(nb));
    } else {
        double s2 = 0.0;
        for (int k = 0; k < 3; ++k) {
            const double d = __dsub_rn(a[k], b[k]);
            s2 = __dadd_rn(s2, __dmul_rn(d, d));
        }
        m = MET == TSNE_METRIC_EUCLIDEAN ? sqrt(s2) : s2;
    }
    x = 1.0 + m;
    double r = __builtin_amdgcn_rcp(x);
    r = __fma_rn(r, __fma_rn(-x, r, 1.0), r);
    r = __fma_rn(r, __fma_rn(-x, r, 1.0), r);
    return r;
}

// The tiled attraction in 3-D (round 6; the 2-D kernel attract_tiles above,
// same layout and loop): per tile the window's W points (24 B each, copied
// from Y as 16-byte pieces) and the row block's RB accumulators sit in LDS;
// each row of a 64-row slice is one lane, summing its entries of the tile in
// its own order with attract3's pair term (qterm3), then adding the sum to
// its accumulator -- one fixed order per row, no atomics.  Replaces
// attract3's Y_j gathers (24 B from a random line per entry: 0.03 of the
// HBM roofline in the C4 loop) by LDS reads.
template <class CF, bool LOSS, int MET>
__global__ __launch_bounds__(CF::NT) void attract_tiles3(
    const ATile *__restrict__ tiles, const int32_t *__restrict__ rbt, const ASlice *__restrict__ slices,
    const uint32_t *__restrict__ srow, int64_t rows, int64_t r0, int64_t n, const uint16_t *__restrict__ pk,
    const double *__restrict__ pv, const double *__restrict__ Y, const double *__restrict__ scal, double ex,
    int64_t xcd_chunk, double *__restrict__ attr, double *__restrict__ lpart, int64_t rbs) {
    constexpr int RB = CF::RB, W = CF::W, NT = CF::NT, WAVES = CF::WAVES;
    static_assert(W % 2 == 0, "window as 16-byte pieces (aligned)");
    __shared__ double2 win2[3 * W / 2];
    __shared__ double acc[3 * RB];
    __shared__ double sl[WAVES];
    const double *win = reinterpret_cast<const double *>(win2);
    const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const int64_t rb = xcd_chunk > 0 ? xcd_block_chunked(blockIdx.x, gridDim.x, xcd_chunk) : (int64_t)blockIdx.x;
    const int64_t b0 = rb * rbs;   // rbs <= RB rows per block (build_attract_tiles)
    const int nr = (int)min(rbs, rows - b0);
    const double *Yrow = Y + 3 * (r0 + b0);
    for (int i = tid; i < 3 * nr; i += NT) acc[i] = 0.0;
    const double Z = LOSS ? scal[0] : 1.0;
    double lsum = 0.0;
    constexpr int WL = (3 * W / 2 + NT - 1) / NT;
    const int t0 = rbt[rb], t1 = rbt[rb + 1];
    for (int t = t0; t < t1; ++t) {
        const ATile tl = tiles[t];
        {   // the window's 3 wn doubles: 16-byte pieces (the odd last double of the last window alone)
            const int64_t base = (int64_t)tl.cb * W;
            const int wn = (int)min((int64_t)W, n - base);
            const int np = 3 * wn / 2;
            const double2 *src = reinterpret_cast<const double2 *>(Y + 3 * base);
            double2 yv[WL];
#pragma unroll
            for (int k = 0; k < WL; ++k) yv[k] = src[min(tid + k * NT, np - 1)];
#pragma unroll
            for (int k = 0; k < WL; ++k) {
                const int i = tid + k * NT;
                if (i < np) win2[i] = yv[k];
            }
            if ((3 * wn) & 1) {
                if (tid == 0) reinterpret_cast<double *>(win2)[3 * wn - 1] = Y[3 * (base + wn) - 1];
            }
        }
        __syncthreads();
        const int s0 = tl.s0, send = tl.s0 + tl.ns;
        int s = s0 + w;
        ASlice sd{};
        uint32_t rl = 0;
        if (s < send) {
            sd = slices[s];
            rl = srow[(int64_t)s * 64 + lane];
        }
        while (s < send) {
            const int len = (int)(rl & ((1u << AT_LENBITS) - 1)), lrow = (int)(rl >> AT_LENBITS);
            double yi[3] = {0.0, 0.0, 0.0};
            if (len > 0) { yi[0] = Yrow[3 * lrow]; yi[1] = Yrow[3 * lrow + 1]; yi[2] = Yrow[3 * lrow + 2]; }
            const int sn = s + WAVES;
            ASlice sdn{};
            uint32_t rln = 0;
            double f0 = 0.0, f1 = 0.0, f2 = 0.0;
            int64_t off = sd.base;
            for (int k0 = 0; k0 < sd.width; k0 += AT_U) {
                uint32_t cu[AT_U];
                double vu[AT_U];
#pragma unroll
                for (int u = 0; u < AT_U; ++u) {
                    const int k = k0 + u;
                    cu[u] = 0;
                    vu[u] = 0.0;
                    if (k < len) { cu[u] = pk[off + lane]; vu[u] = pv[off + lane]; }
                    off += __popcll(__ballot(len > k));
                }
                if (k0 == 0 && sn < send) {
                    sdn = slices[sn];
                    rln = srow[(int64_t)sn * 64 + lane];
                }
#pragma unroll
                for (int u = 0; u < AT_U; ++u) {
                    if (k0 + u < len) {
                        const double yj[3] = {win[3 * cu[u]], win[3 * cu[u] + 1], win[3 * cu[u] + 2]};
                        double x1m;
                        const double q = qforce3_t<MET>(yi, yj, x1m);
                        const double sc = __dmul_rn(vu[u], q);
                        f0 = __fma_rn(sc, __dsub_rn(yi[0], yj[0]), f0);
                        f1 = __fma_rn(sc, __dsub_rn(yi[1], yj[1]), f1);
                        f2 = __fma_rn(sc, __dsub_rn(yi[2], yj[2]), f2);
                        if (LOSS) {
                            const double pij = __dmul_rn(vu[u], ex);
                            lsum += pij * log_kl(pij * Z * x1m);
                        }
                    }
                }
            }
            if (sd.wide) {   // one row over the 64 lanes: a fixed-order tree
                f0 = wave_sum(f0);
                f1 = wave_sum(f1);
                f2 = wave_sum(f2);
                if (lane == 0) {
                    acc[3 * lrow] = __dadd_rn(acc[3 * lrow], f0);
                    acc[3 * lrow + 1] = __dadd_rn(acc[3 * lrow + 1], f1);
                    acc[3 * lrow + 2] = __dadd_rn(acc[3 * lrow + 2], f2);
                }
            } else if (len > 0) {
                acc[3 * lrow] = __dadd_rn(acc[3 * lrow], f0);
                acc[3 * lrow + 1] = __dadd_rn(acc[3 * lrow + 1], f1);
                acc[3 * lrow + 2] = __dadd_rn(acc[3 * lrow + 2], f2);
            }
            s = sn;
            sd = sdn;
            rl = rln;
        }
        __syncthreads();
    }
    for (int i = tid; i < 3 * nr; i += NT) attr[3 * b0 + i] = acc[i] * ex;
    if (LOSS) {
        lsum = wave_sum(lsum);
        if (lane == 0) sl[w] = lsum;
        __syncthreads();
        if (tid == 0) {
            double s = 0.0;
            for (int k = 0; k < WAVES; ++k) s += sl[k];
            lpart[blockIdx.x] = s;
        }
    }
}

// One wave per row (grid-stride), lanes over the row's entries, then a
// wave reduction: attr_i = sum_j ex P_ij q_ij (y_i - y_j); LOSS adds the KL
// terms into one partial per block (TsneHelpers.scala:269-306).  A lane's
// entries e, e + 64, ... are taken ATTR3_U at a time: their column and value
// loads, then their Y_j gathers, are all in flight before the first term is
// summed (C4: ~163 entries per row, one round); the sums keep the lane's
// entry order, so the result is the same to the bit.
constexpr int ATTR3_U = 4;
template <bool LOSS, int MET>
__global__ __launch_bounds__(256) void attract3(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
                                                const double *__restrict__ val, int64_t r0, int64_t r1,
                                                const double *__restrict__ Y, const double *__restrict__ scal,
                                                double ex, double *__restrict__ attr, double *__restrict__ lpart) {
    __shared__ double sl[4];
    const int lane = lane_id();
    const double Z = LOSS ? scal[0] : 1.0;
    double lsum = 0.0;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t i = r0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < r1; i += nw) {
        const double yi[3] = {Y[3 * i], Y[3 * i + 1], Y[3 * i + 2]};
        double f[3] = {0.0, 0.0, 0.0};
        const int64_t e1 = row_ptr[i + 1];
        for (int64_t eb = row_ptr[i] + lane; eb < e1; eb += 64 * ATTR3_U) {
            int64_t j[ATTR3_U];
            double pv[ATTR3_U];
#pragma unroll
            for (int u = 0; u < ATTR3_U; ++u) {
                const int64_t e = eb + 64 * u;
                j[u] = e < e1 ? (int64_t)col[e] : i;
                pv[u] = e < e1 ? val[e] : 0.0;
            }
            double yj[ATTR3_U][3];
#pragma unroll
            for (int u = 0; u < ATTR3_U; ++u)
#pragma unroll
                for (int k = 0; k < 3; ++k) yj[u][k] = Y[3 * j[u] + k];
#pragma unroll
            for (int u = 0; u < ATTR3_U; ++u) {
                if (eb + 64 * u >= e1) break;
                const double pij = __dmul_rn(pv[u], ex);
                const double q = qterm3<MET>(yi, yj[u]);
                const double sc = __dmul_rn(pij, q);
                for (int k = 0; k < 3; ++k) f[k] = __dadd_rn(f[k], __dmul_rn(sc, __dsub_rn(yi[k], yj[u][k])));
                if (LOSS) lsum += pij * log(pij / (q / Z));
            }
        }
        for (int k = 0; k < 3; ++k) {
            const double v = wave_sum(f[k]);
            if (lane == 0) attr[3 * (i - r0) + k] = v;
        }
    }
    if (LOSS) {
        lsum = wave_sum(lsum);
        if (lane == 0) sl[threadIdx.x >> 6] = lsum;
        __syncthreads();
        if (threadIdx.x == 0) lpart[blockIdx.x] = (sl[0] + sl[1]) + (sl[2] + sl[3]);
    }
}

// grad = attr - F / Z, then (MODE 1) updateEmbedding -> Ynew (3 components).
// With `mpart` (MODE 1, one rank) each block also writes the sums of its
// rows' Ynew to mpart[3 * block + c]: the centring mean's partials, as
// combine_update in 2-D (meanC_final, center3_scatter).
template <int MODE>
__global__ __launch_bounds__(256) void combine_update3(int64_t r0, int64_t r1, const double *__restrict__ attr,
                                                       const int32_t *__restrict__ inv, const double *__restrict__ F,
                                                       const double *__restrict__ scal, const double *__restrict__ Y,
                                                       double *__restrict__ grad, double *__restrict__ Ynew,
                                                       double *__restrict__ upd, double *__restrict__ gains,
                                                       double min_gain, double mom, double lr,
                                                       double *__restrict__ mpart) {
    __shared__ double sm[3][4];
    const int64_t i = r0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double yn[3] = {0.0, 0.0, 0.0};
    if (i < r1) {
        const double Z = scal[0];
        const int64_t si = inv[i];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double g = attr[3 * (i - r0) + c] - F[3 * si + c] / Z;
            const int64_t o = 3 * i + c;
            if (MODE == 0) { grad[o] = g; continue; }
            const double u = upd[o], gn0 = gains[o];
            const double gn = ((g > 0.0) == (u > 0.0)) ? jmax(gn0 * 0.8, min_gain) : jmax(gn0 + 0.2, min_gain);
            const double un = __dsub_rn(__dmul_rn(mom, u), __dmul_rn(__dmul_rn(lr, gn), g));
            gains[o] = gn;
            upd[o] = un;
            yn[c] = __dadd_rn(un, Y[o]);
            Ynew[o] = yn[c];
        }
    }
    if (MODE == 1 && mpart) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double v = wave_sum(yn[c]);
            if (lane_id() == 0) sm[c][threadIdx.x >> 6] = v;
        }
        __syncthreads();
        if (threadIdx.x < 3)
            mpart[3 * blockIdx.x + threadIdx.x] =
                (sm[threadIdx.x][0] + sm[threadIdx.x][1]) + (sm[threadIdx.x][2] + sm[threadIdx.x][3]);
    }
}

// mean[c] = (sum of the nb block partials mpart[3 b + c], fixed order) / n
__global__ __launch_bounds__(256) void mean3_final(const double *__restrict__ mpart, int64_t nb, double n,
                                                   double *__restrict__ mean) {
    __shared__ double sm[3][4];
    double s[3] = {0.0, 0.0, 0.0};
    for (int64_t b = threadIdx.x; b < nb; b += blockDim.x)
        for (int c = 0; c < 3; ++c) s[c] += mpart[3 * b + c];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double v = wave_sum(s[c]);
        if (lane_id() == 0) sm[c][threadIdx.x >> 6] = v;
    }
    __syncthreads();
    if (threadIdx.x < 3)
        mean[threadIdx.x] = ((sm[threadIdx.x][0] + sm[threadIdx.x][1]) + (sm[threadIdx.x][2] + sm[threadIdx.x][3])) / n;
}

// centerEmbedding (TsneHelpers.scala:320-329), 3-D: Y = Ynew - mean (the
// caller's copy at tsne_dev_opt_sync, as in 2-D)
__global__ __launch_bounds__(256) void center3(const double *__restrict__ Ynew, int64_t n,
                                               const double *__restrict__ mean, double *__restrict__ Y) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= 3 * n) return;
    Y[e] = Ynew[e] - mean[e % 3];
}

static int64_t attract3_blocks(int64_t rows) { return std::max<int64_t>(1, std::min<int64_t>(8192, ceil_div(rows, 4))); }

// attract_tiles3 over the tiled layout of the owned rows (3-D); returns the
// workgroups (the loss partials)
template <class CF, bool LOSS, int MET>
static void attract_tiles3_c(hipStream_t st, const OptState *s, const double *Y, const double *scal, double ex,
                             double *attr, double *lpart) {
    const int64_t nb = s->at_nrb;
    hipLaunchKernelGGL((attract_tiles3<CF, LOSS, MET>), dim3(nb), dim3(CF::NT), 0, st, s->at_tiles, s->at_rbt,
                       s->at_slices, s->at_srow, s->L1 - s->L0, s->L0, s->n, s->at_pk, s->at_pv, Y, scal, ex,
                       nb / NUM_XCD, attr, lpart, s->at_rbs);
}
template <bool LOSS, int MET>
static void attract_tiles3_m(hipStream_t st, const OptState *s, const double *Y, const double *scal, double ex,
                             double *attr, double *lpart) {
    if (s->at_cfg == 4) attract_tiles3_c<ATCfg3D, LOSS, MET>(st, s, Y, scal, ex, attr, lpart);
    else attract_tiles3_c<ATCfg3Ds, LOSS, MET>(st, s, Y, scal, ex, attr, lpart);
}
static int64_t attract_tiles3_launch(hipStream_t st, const OptState *s, const double *Y, const double *scal,
                                     int metric, double ex, double *attr, double *lpart, bool loss) {
#define TSNE_AT3(L, M) attract_tiles3_m<L, M>(st, s, Y, scal, ex, attr, lpart)
    if (metric == TSNE_METRIC_EUCLIDEAN) { if (loss) TSNE_AT3(true, TSNE_METRIC_EUCLIDEAN); else TSNE_AT3(false, TSNE_METRIC_EUCLIDEAN); }
    else if (metric == TSNE_METRIC_COSINE) { if (loss) TSNE_AT3(true, TSNE_METRIC_COSINE); else TSNE_AT3(false, TSNE_METRIC_COSINE); }
    else { if (loss) TSNE_AT3(true, TSNE_METRIC_SQEUCLIDEAN); else TSNE_AT3(false, TSNE_METRIC_SQEUCLIDEAN); }
#undef TSNE_AT3
    TSNE_LAUNCH_CHECK();
    return s->at_nrb;
}

static int64_t attract3_launch(hipStream_t st, const int64_t *rp, const int32_t *col, const double *val, int64_t r0,
                               int64_t r1, const double *Y, const double *scal, int metric, double ex, double *attr,
                               double *lpart, bool loss) {
    const int64_t blocks = attract3_blocks(r1 - r0);
    if (r1 <= r0) return 0;
#define TSNE_A3(L, M) \
    hipLaunchKernelGGL((attract3<L, M>), dim3(blocks), dim3(256), 0, st, rp, col, val, r0, r1, Y, scal, ex, attr, lpart)
    if (metric == TSNE_METRIC_EUCLIDEAN) { if (loss) TSNE_A3(true, TSNE_METRIC_EUCLIDEAN); else TSNE_A3(false, TSNE_METRIC_EUCLIDEAN); }
    else if (metric == TSNE_METRIC_COSINE) { if (loss) TSNE_A3(true, TSNE_METRIC_COSINE); else TSNE_A3(false, TSNE_METRIC_COSINE); }
    else { if (loss) TSNE_A3(true, TSNE_METRIC_SQEUCLIDEAN); else TSNE_A3(false, TSNE_METRIC_SQEUCLIDEAN); }
#undef TSNE_A3
    return blocks;
}

// Attraction launch: variant (lanes per row x unroll) from TSNE_ATTRACT
// ("16x4", "32x4", "64x4", "16x8", "32x8", "16x12"); returns the block count
// (loss partials).
struct AttractArgs {
    const int64_t *rp; const int32_t *col; const double *val; int64_t r0, r1; const double *Y;
    const double *scal; int metric; double ex; double2 *attr; double *lpart;
    int bpc = 0;   // blocks per CU of the persistent grid (0: 8 = every wave slot)
};

// persistent grid: bpc 256-thread blocks per CU (8: every wave slot), a
// multiple of the XCD count.  The gathers are bound by the CU's outstanding
// misses, not its waves: 3-4 blocks per CU run as fast as 8 and leave slots
// to a concurrent tree build.
static int64_t attract_grid(int64_t rows, int lpr, int bpc_req) {
    static const int cus = [] {
        int dev = 0, c = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
        return c;
    }();
    const int bpc = bpc_req > 0 ? std::min(bpc_req, 8) : 8;
    const int64_t full = round_up(cus * bpc, NUM_XCD);
    const int64_t need = round_up(std::max<int64_t>(1, ceil_div(rows * lpr, 256)), NUM_XCD);
    return std::min(full, need);
}

template <int LPR, int U, int MET>
static int64_t attract_launch_m(hipStream_t st, const AttractArgs &a, bool loss) {
    const int64_t rows = a.r1 - a.r0;
    const int64_t blocks = attract_grid(rows, LPR, a.bpc);
    if (loss)
        hipLaunchKernelGGL((attract_rows<LPR, U, true, MET>), dim3(blocks), dim3(256), 0, st, a.rp, a.col, a.val,
                           a.r0, a.r1, a.Y, a.scal, a.ex, a.attr, a.lpart);
    else
        hipLaunchKernelGGL((attract_rows<LPR, U, false, MET>), dim3(blocks), dim3(256), 0, st, a.rp, a.col, a.val,
                           a.r0, a.r1, a.Y, a.scal, a.ex, a.attr, a.lpart);
    return blocks;
}

template <int LPR, int U>
static int64_t attract_launch_v(hipStream_t st, const AttractArgs &a, bool loss) {
    switch (a.metric) {
        case TSNE_METRIC_EUCLIDEAN: return attract_launch_m<LPR, U, TSNE_METRIC_EUCLIDEAN>(st, a, loss);
        case TSNE_METRIC_COSINE: return attract_launch_m<LPR, U, TSNE_METRIC_COSINE>(st, a, loss);
        default: return attract_launch_m<LPR, U, TSNE_METRIC_SQEUCLIDEAN>(st, a, loss);
    }
}

// attract_rows: 64 lanes per row, 4 (col, val) loads then 4 Y_j gathers in
// flight per lane (16/32 lanes, 8/12 in flight measured slower, round 1)
static int64_t attract_launch(hipStream_t st, const AttractArgs &a, bool loss) {
    return attract_launch_v<64, 4>(st, a, loss);
}

template <int MODE>
static void combine_launch(hipStream_t st, int64_t r0, int64_t r1, const double2 *attr, const int32_t *inv,
                           const double2 *F, const double *scal, const double *Y, double *grad, double *Ynew,
                           double *upd, double *gains, double min_gain, double mom, double lr,
                           double *mpart = nullptr) {
    if (r1 <= r0) return;
    hipLaunchKernelGGL(combine_update<MODE>, dim3(ceil_div(r1 - r0, 256)), dim3(256), 0, st, r0, r1, attr, inv, F,
                       scal, Y, grad, Ynew, upd, gains, min_gain, mom, lr, mpart);
}

// Upper bound of attract_launch's block count for rows rows.
// (rounded up to the XCD count like attract_grid's launch)
static int64_t attract_max_blocks(int64_t rows) {
    return round_up(std::max<int64_t>(1, ceil_div(rows * 64, 256)), NUM_XCD);
}
}  // namespace

// ------------------------------------------------------------ single ops

void update_device(tsne_ctx *ctx, int64_t n, int32_t c, const double *dgrad, double *dY,
                   double *dupd, double *dgains, double min_gain, double momentum, double lr) {
    const int64_t ne = n * c;
    if (ne <= 0) return;
    hipLaunchKernelGGL(update_kernel, dim3(ceil_div(ne, 256)), dim3(256), 0, ctx->stream, ne, dgrad,
                       dY, dupd, dgains, min_gain, momentum, lr);
    TSNE_LAUNCH_CHECK();
}

void center_device(tsne_ctx *ctx, int64_t n, int32_t c, double *dY) {
    if (n <= 0) return;
    TSNE_REQUIRE(c >= 1 && c <= 8, "n_components out of range");
    double *part = ctx->ws.get<double>("ctr.part", NPART);
    double *mean = ctx->ws.get<double>("ctr.mean", 8);
    double *tmp = ctx->ws.get<double>("ctr.tmp", (size_t)n * c);
    for (int k = 0; k < c; ++k) {
        hipLaunchKernelGGL(reduce_partial, dim3(NPART), dim3(256), 0, ctx->stream, dY, n, c, k, part);
        hipLaunchKernelGGL(reduce_final, dim3(1), dim3(256), 0, ctx->stream, part, NPART, mean + k, (double)n);
    }
    TSNE_HIP(hipMemcpyAsync(tmp, dY, sizeof(double) * n * c, hipMemcpyDeviceToDevice, ctx->stream));
    hipLaunchKernelGGL(center_apply, dim3(ceil_div(n * c, 256)), dim3(256), 0, ctx->stream, tmp, n, c, mean, dY);
    TSNE_LAUNCH_CHECK();
}

void init_working_set_device(tsne_ctx *ctx, int64_t n, int32_t c, uint64_t seed, double *dY,
                             double *dupd, double *dgains) {
    const int64_t ne = n * c;
    if (ne <= 0) return;
    hipLaunchKernelGGL(init_ws_kernel, dim3(ceil_div(ne, 256)), dim3(256), 0, ctx->stream, ne, seed, dY,
                       dupd, dgains);
    TSNE_LAUNCH_CHECK();
}

// The root-tile shortcut of bh_build while the embedding is small
// (Options::root_tile = 0: always the full tree).
static bool root_tile_enabled(const tsne_ctx *ctx) { return ctx->opts.root_tile != 0; }

void gradient_device(tsne_ctx *ctx, const int64_t *d_row_ptr, const int32_t *d_col,
                     const double *d_P, int64_t n, const double *dY, int32_t metric, double theta,
                     double exaggeration, double *d_grad, double *h_sumq, double *h_loss) {
    TSNE_REQUIRE(n >= 1, "empty embedding");
    hipStream_t st = ctx->stream;
    BHTree &t = bh_single_tree(ctx, n);
    bh_build(ctx, t, dY, theta, nullptr, root_tile_enabled(ctx));
    double2 *F = ctx->ws.get<double2>("grad.F", n);
    double *z = ctx->ws.get<double>("grad.z", n);
    double *part = ctx->ws.get<double>("grad.part", NPART);
    double *scal = ctx->ws.get<double>("grad.scal", 4);
    bh_repulsion(ctx, t, theta, 0, n, F, z, nullptr);
    hipLaunchKernelGGL(reduce_partial, dim3(NPART), dim3(256), 0, st, z, n, 1, 0, part);
    hipLaunchKernelGGL(reduce_final, dim3(1), dim3(256), 0, st, part, NPART, scal, 0.0);
    double *lpart = ctx->ws.get<double>("grad.lpart", attract_max_blocks(n));
    const bool want_loss = h_loss != nullptr;
    double2 *attr = ctx->ws.get<double2>("grad.attr", n);
    AttractArgs aa{d_row_ptr, d_col, d_P, 0, n, dY, scal, metric, exaggeration, attr, lpart};
    const int64_t blocks = attract_launch(st, aa, want_loss);
    combine_launch<0>(st, 0, n, attr, t.inv, F, scal, dY, d_grad, nullptr, nullptr, nullptr, 0.0, 0.0, 0.0);
    TSNE_LAUNCH_CHECK();
    if (want_loss) {   // two-level: block partials -> NPART -> 1
        hipLaunchKernelGGL(reduce_partial, dim3(NPART), dim3(256), 0, st, lpart, blocks, 1, 0, part);
        hipLaunchKernelGGL(reduce_final, dim3(1), dim3(256), 0, st, part, NPART, scal + 1, 0.0);
    }
    double hs[2] = {0, 0};
    TSNE_HIP(hipMemcpyAsync(hs, scal, 2 * sizeof(double), hipMemcpyDeviceToHost, st));
    TSNE_HIP(hipStreamSynchronize(st));
    if (h_sumq) *h_sumq = hs[0];
    if (h_loss) *h_loss = hs[1];
}

// per-point results from sorted order back to the original order
__global__ void unsort_fz(const int32_t *__restrict__ inv, int64_t n, int c, const double *__restrict__ Fs,
                          const double *__restrict__ zs, double *__restrict__ Fo, double *__restrict__ zo) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t si = inv[i];
    for (int k = 0; k < c; ++k) Fo[c * i + k] = Fs[c * si + k];
    zo[i] = zs[si];
}

// QuadTree.computeRepulsiveForce (QuadTree.scala:123-152) for every point of
// Y against the tree of all of them (c = 2), or the octree extension (c = 3):
// F (n x c) and z (sumQ contribution) per point, original order.
void repulsion_device(tsne_ctx *ctx, const double *dY, int64_t n, int32_t c, double theta, double *dF,
                      double *dz) {
    TSNE_REQUIRE(n >= 1, "empty embedding");
    hipStream_t st = ctx->stream;
    double *Fs = ctx->ws.get<double>("rep.F", (size_t)c * n);
    double *zs = ctx->ws.get<double>("rep.z", n);
    const int32_t *inv;
    if (c == 2) {
        BHTree &t = bh_single_tree(ctx, n);
        bh_build(ctx, t, dY, theta, nullptr, root_tile_enabled(ctx));
        unsigned long long *vis = nullptr;   // Options::rep_stats: the counting traversal
        if (ctx->opts.rep_stats) {
            vis = ctx->ws.get<unsigned long long>("rep.visits", VIS_N);
            TSNE_HIP(hipMemsetAsync(vis, 0, sizeof(unsigned long long) * VIS_N, st));
            if (ctx->opts.wave_log)   // (the log's count; bh_repulsion takes the buffer)
                TSNE_HIP(hipMemsetAsync(ctx->ws.get<unsigned long long>("rep.wavelog", 1), 0, 8, st));
        }
        bh_repulsion(ctx, t, theta, 0, n, reinterpret_cast<double2 *>(Fs), zs, vis);
        inv = t.inv;
    } else {
        OctTree t;
        oct_alloc(ctx, t, n, "oct1.");
        oct_build(ctx, t, dY, theta);
        oct_repulsion(ctx, t, theta, 0, n, Fs, zs);
        inv = t.inv;
    }
    hipLaunchKernelGGL(unsort_fz, dim3(ceil_div(n, 256)), dim3(256), 0, st, inv, n, c, Fs, zs, dF, dz);
    TSNE_LAUNCH_CHECK();
}

int64_t opt_wave_mhz(tsne_ctx *ctx) { return ctx->opt ? ctx->opt->last_mhz : 0; }

bool repulsion_stat(tsne_ctx *ctx, const std::string &name, int64_t *value_out) {
    // indices of bh_traverse's counters (its STATS block): wave pops, tile
    // points, wave child slots, reference-equivalent evaluations
    const int at = name == "bh.pops" ? 3 : name == "bh.tile_points" ? 4 : name == "bh.child_slots" ? 6
                 : name == "bh.visits" ? 0 : name == "bh.wave_ticks_max" ? 15 : name == "bh.wave_ticks_sum" ? 18
                 : name == "bh.span_ticks" ? 17 : name == "bh.dense_pairs" ? 2 : name == "bh.moment_evals" ? 1
                 : name == "bh.tile_ticks_max" ? 19 : name == "bh.tile_ticks_sum" ? 22 : name == "bh.tile_span_ticks" ? 21
                 : name == "bh.slow_wave_ticks" ? 33 : name == "bh.slow_wave_pops" ? 33 : name == "bh.slow_wave_ties" ? 34
                 : name == "bh.slow_wave_tile_points" ? 35 : name == "bh.slow_wave_slots" ? 36
                 : name == "bh.wave_mhz" ? 37 : -1;
    // tile_apply's dense paths k = 0..3 (lane-wise, packed, query-major, staged
    // sweep): "bh.tile_steps<k>" wave steps issued, "bh.tile_pairs<k>" useful lane pairs
    int atk = at;
    if (at < 0 && name.size() == 14 && name.compare(0, 13, "bh.tile_steps") == 0) atk = 24 + 2 * (name[13] - '0');
    if (at < 0 && name.size() == 14 && name.compare(0, 13, "bh.tile_pairs") == 0) atk = 25 + 2 * (name[13] - '0');
    if (atk < 0 || atk >= VIS_N) return false;
    TSNE_REQUIRE(ctx->opts.rep_stats && ctx->ws.has("rep.visits"), "counter '" + name + "' needs option rep_stats");
    unsigned long long v[VIS_N];
    TSNE_HIP(hipMemcpyAsync(v, ctx->ws.get<unsigned long long>("rep.visits", VIS_N), sizeof(v), hipMemcpyDeviceToHost,
                            ctx->stream));
    TSNE_HIP(hipStreamSynchronize(ctx->stream));
    // span: last wave end - first wave start ([16] holds ~first start), 100 MHz ticks
    *value_out = atk == 17 ? (int64_t)(v[17] - (~0ull - v[16])) : atk == 21 ? (int64_t)(v[21] - (~0ull - v[20]))
                                                                              : (int64_t)v[atk];
    if (atk == 37) *value_out = v[18] ? (int64_t)(100.0 * (double)v[37] / (double)v[18]) : 0;
    if (atk >= 33 && atk <= 36)   // (ticks << 24 | count) of the slowest wave
        *value_out = name == "bh.slow_wave_ticks" ? (int64_t)(v[atk] >> 24) : (int64_t)(v[atk] & ((1ull << 24) - 1));
    return true;
}

// 3-D gradient (octree): same contract as gradient_device, Y / grad n x 3.
void gradient3_device(tsne_ctx *ctx, const int64_t *d_row_ptr, const int32_t *d_col, const double *d_P, int64_t n,
                      const double *dY, int32_t metric, double theta, double exaggeration, double *d_grad,
                      double *h_sumq, double *h_loss) {
    TSNE_REQUIRE(n >= 1, "empty embedding");
    hipStream_t st = ctx->stream;
    OctTree t;
    oct_alloc(ctx, t, n, "oct1.");
    oct_build(ctx, t, dY, theta);
    double *F = ctx->ws.get<double>("grad3.F", 3 * (size_t)n);
    double *z = ctx->ws.get<double>("grad.z", n);
    double *part = ctx->ws.get<double>("grad.part", NPART);
    double *scal = ctx->ws.get<double>("grad.scal", 4);
    oct_repulsion(ctx, t, theta, 0, n, F, z);
    hipLaunchKernelGGL(reduce_partial, dim3(NPART), dim3(256), 0, st, z, n, 1, 0, part);
    hipLaunchKernelGGL(reduce_final, dim3(1), dim3(256), 0, st, part, NPART, scal, 0.0);
    const bool want_loss = h_loss != nullptr;
    double *lpart = ctx->ws.get<double>("grad3.lpart", attract3_blocks(n));
    double *attr = ctx->ws.get<double>("grad3.attr", 3 * (size_t)n);
    const int64_t blocks = attract3_launch(st, d_row_ptr, d_col, d_P, 0, n, dY, scal, metric, exaggeration, attr,
                                           lpart, want_loss);
    hipLaunchKernelGGL(combine_update3<0>, dim3(ceil_div(n, 256)), dim3(256), 0, st, 0, n, attr, t.inv, F, scal, dY,
                       d_grad, nullptr, nullptr, nullptr, 0.0, 0.0, 0.0, nullptr);
    TSNE_LAUNCH_CHECK();
    if (want_loss) {
        hipLaunchKernelGGL(reduce_partial, dim3(NPART), dim3(256), 0, st, lpart, blocks, 1, 0, part);
        hipLaunchKernelGGL(reduce_final, dim3(1), dim3(256), 0, st, part, NPART, scal + 1, 0.0);
    }
    double hs[2] = {0, 0};
    TSNE_HIP(hipMemcpyAsync(hs, scal, 2 * sizeof(double), hipMemcpyDeviceToHost, st));
    TSNE_HIP(hipStreamSynchronize(st));
    if (h_sumq) *h_sumq = hs[0];
    if (h_loss) *h_loss = hs[1];
}

// ------------------------------------------------------------ optimizer

void opt_destroy(tsne_ctx *ctx) {
    if (!ctx->opt) return;
    OptState *s = ctx->opt;
    for (auto &e : s->ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {s->ev_y, s->ev_attr})
        if (e) (void)hipEventDestroy(e);
    if (s->side) {
        (void)hipStreamSynchronize(s->side);
        (void)hipStreamDestroy(s->side);
    }
    delete ctx->opt;
    ctx->opt = nullptr;
}

// cuts of [0, n) into world equal label ranges
static std::vector<int64_t> equal_cuts(int64_t n, int world) {
    std::vector<int64_t> c(world + 1);
    const int64_t chunk = ceil_div(n, world);
    for (int r = 0; r <= world; ++r) c[r] = std::min<int64_t>(n, chunk * r);
    return c;
}

// make every rank's upd / gains current for all labels (each rank updates
// only its own labels between relabels): ragged all-gather of the slices
static void gather_working_set(tsne_ctx *ctx, OptState *s) {
    if (!sharded(ctx)) return;
    const int c = s->cur;
    std::vector<int64_t> off(ctx->world + 1);
    for (int r = 0; r <= ctx->world; ++r) off[r] = s->own[r] * s->C * (int64_t)sizeof(double);
    comm_allgatherv(ctx, s->upd[c], off.data());
    comm_allgatherv(ctx, s->gains[c], off.data());
}

// Tile configuration for `rows` owned rows (Options::attract_cfg 0..3 forces one);
// 3-D: 4 (ATCfg3D) when its row blocks cover the CUs, else 5 (ATCfg3Ds)
static int at_cfg(tsne_ctx *ctx, int64_t rows, int C = 2) {
    if (C == 3) return ceil_div(rows, (int64_t)ATCfg3D::RB) >= ctx->cu_count - ctx->cu_count / 16 ? 4 : 5;
    if (ctx->opts.attract_cfg >= 0) return ctx->opts.attract_cfg;
    for (int c = 3; c > 0; --c)
        if (ceil_div(rows, (int64_t)512 << c) >= ctx->cu_count - ctx->cu_count / 16) return c;
    return 0;
}

// The tiled layout of the owned rows (attract_tiles): a stable radix sort of
// the entries by (row block, column window, local row) -- within a row the
// entries keep their order -- then per tile its rows sorted by entry count
// (a second radix sort of the (tile, row) segments), 64-row slices, and the
// jagged-diagonal scatter of the column offsets and values.
// Skipped (attract_rows runs) for dense rows over a small embedding (C5: all
// of Y sits in one L2), for >= 2^31 owned entries, or with Options::attract_tiles = 0.
static void build_attract_tiles(tsne_ctx *ctx, OptState *s) {
    const bool on = ctx->opts.attract_tiles != 0;
    hipStream_t st = ctx->stream;
    Workspace &ws = ctx->ws;
    const int64_t rows = s->L1 - s->L0, n = s->n;
    s->at_on = false;
    // Only while the labels are P's graph order: once they follow the
    // embedding's Morton order, a row's Y_j are spatially local and
    // attract_rows' gathers hit the L2 (C3 loss launches: attract_rows 1.58
    // ms, attract_tiles 2.4 ms over t = 300..1000; in graph order 1.45 vs 1.11).
    // 3-D only with Options::attract_tiles3 (measured slower than attract3 at C4)
    if (!on || rows <= 0 || s->morton_labels || (s->C == 3 && !ctx->opts.attract_tiles3)) return;
    if (s->nnz / std::max<int64_t>(1, n) > 1024 && n * 16 <= (2 << 20)) return;
    int64_t m = 0;
    TSNE_HIP(hipMemcpyAsync(&m, s->rpw + rows, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    TSNE_HIP(hipStreamSynchronize(st));
    if (m <= 0 || m >= (int64_t)INT32_MAX) return;
    const int cfg = at_cfg(ctx, rows, s->C);
    const int rowbits = cfg == 0 ? ATCfg0::ROWBITS : cfg == 1 ? ATCfg1::ROWBITS : cfg == 2 ? ATCfg2::ROWBITS
                      : cfg == 3 ? ATCfg3::ROWBITS : cfg == 4 ? ATCfg3D::ROWBITS : ATCfg3Ds::ROWBITS;
    const int64_t W = cfg == 0 ? ATCfg0::W : cfg == 1 ? ATCfg1::W : cfg == 2 ? ATCfg2::W : cfg == 3 ? ATCfg3::W
                    : cfg == 4 ? ATCfg3D::W : ATCfg3Ds::W;
    // rows per block: the config's 2^rowbits, or fewer (a multiple of 64) so
    // that the row blocks cover every CU (C3: 3968 rows, 253 blocks, instead
    // of 245 blocks of 4096)
    const int64_t rbs = std::min<int64_t>((int64_t)1 << rowbits, round_up(ceil_div(rows, (int64_t)ctx->cu_count), 64));
    const int64_t nrb = ceil_div(rows, rbs), ncb = ceil_div(n, W);
    int bits = rowbits;
    for (uint64_t v = (uint64_t)(nrb * ncb - 1); v; v >>= 1) ++bits;
    uint64_t *key = ws.get<uint64_t>("opt.at.key", m), *key2 = ws.get<uint64_t>("opt.at.key2", m);
    int32_t *idx = ws.get<int32_t>("opt.at.idx", m), *idx2 = ws.get<int32_t>("opt.at.idx2", m);
    auto scan_i32 = [&](const int32_t *in, int32_t *out, int64_t cnt) {
        size_t b = 0;
        TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b, in, out, (int)cnt, st));
        TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(ws.get<uint8_t>("opt.at.stmp", b), b, in, out, (int)cnt, st));
    };
    auto total = [&](const int32_t *excl, const int32_t *in, int64_t cnt) {   // excl[cnt-1] + in[cnt-1]
        int32_t h[2] = {0, 0};
        TSNE_HIP(hipMemcpyAsync(h, excl + cnt - 1, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        TSNE_HIP(hipMemcpyAsync(h + 1, in + cnt - 1, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        TSNE_HIP(hipStreamSynchronize(st));
        return h[0] + h[1];
    };
    // 1-2: entries sorted by (tile, local row), row order kept within a row
    hipLaunchKernelGGL(at_keys, dim3(ceil_div(rows, 4)), dim3(256), 0, st, s->rpw, s->colw, rows, ncb, rowbits, rbs, W,
                       key, idx);
    size_t tb = 0;
    TSNE_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, key2, idx, idx2, (int)m, 0, bits, st));
    TSNE_HIP(hipcub::DeviceRadixSort::SortPairs(ws.get<uint8_t>("opt.at.tmp", tb), tb, key, key2, idx, idx2, (int)m, 0,
                                                bits, st));
    uint16_t *cs = ws.get<uint16_t>("opt.at.cs", m);
    double *vs = ws.get<double>("opt.at.vs", m);
    int32_t *flag = ws.get<int32_t>("opt.at.flag", m), *sid = ws.get<int32_t>("opt.at.sid", m);
    hipLaunchKernelGGL(at_gather, dim3(ceil_div(m, 256)), dim3(256), 0, st, key2, idx2, m, ncb, rowbits, W, s->colw,
                       s->valw, cs, vs, flag);
    // 3: (tile, row) segments, sorted by tile and descending length
    scan_i32(flag, sid, m);
    const int32_t ns = total(sid, flag, m);
    int32_t *sstart = ws.get<int32_t>("opt.at.sstart", ns), *slen = ws.get<int32_t>("opt.at.slen", ns);
    uint64_t *skey = ws.get<uint64_t>("opt.at.skey", ns);
    uint64_t *okey = ws.get<uint64_t>("opt.at.okey", ns), *okey2 = ws.get<uint64_t>("opt.at.okey2", ns);
    int32_t *oval = ws.get<int32_t>("opt.at.oval", ns), *og = ws.get<int32_t>("opt.at.og", ns);
    hipLaunchKernelGGL(at_segs, dim3(ceil_div(m, 256)), dim3(256), 0, st, key2, flag, sid, m, sstart, skey);
    hipLaunchKernelGGL(at_seglen, dim3(ceil_div(ns, 256)), dim3(256), 0, st, sstart, skey, ns, m, rowbits, slen, okey,
                       oval);
    const int obits = bits - rowbits + AT_LENBITS;
    tb = 0;
    TSNE_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, okey, okey2, oval, og, (int)ns, 0, obits, st));
    TSNE_HIP(hipcub::DeviceRadixSort::SortPairs(ws.get<uint8_t>("opt.at.tmp", tb), tb, okey, okey2, oval, og, (int)ns,
                                                0, obits, st));
    // 4-5: tiles, their slices, slice bases (prefix of the sorted lengths)
    int64_t *lenj = ws.get<int64_t>("opt.at.lenj", ns), *ebase = ws.get<int64_t>("opt.at.ebase", ns);
    int32_t *tflag = ws.get<int32_t>("opt.at.tflag", ns), *tix = ws.get<int32_t>("opt.at.tix", ns);
    hipLaunchKernelGGL(at_sorted, dim3(ceil_div(ns, 256)), dim3(256), 0, st, okey2, og, slen, ns, lenj, tflag);
    {
        size_t b = 0;
        TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b, lenj, ebase, (int)ns, st));
        TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(ws.get<uint8_t>("opt.at.stmp", b), b, lenj, ebase, (int)ns, st));
    }
    scan_i32(tflag, tix, ns);
    const int32_t nt = total(tix, tflag, ns);
    int32_t *tfirst = ws.get<int32_t>("opt.at.tfirst", nt), *tns = ws.get<int32_t>("opt.at.tns", nt);
    int32_t *ts0 = ws.get<int32_t>("opt.at.ts0", nt), *twide = ws.get<int32_t>("opt.at.twide", nt);
    s->at_tiles = ws.get<ATile>("opt.at.tiles", nt);
    hipLaunchKernelGGL(at_tilefirst, dim3(ceil_div(ns, 256)), dim3(256), 0, st, okey2, tflag, tix, ns, ncb, tfirst,
                       s->at_tiles);
    hipLaunchKernelGGL(at_tilecount, dim3(ceil_div(nt, 256)), dim3(256), 0, st, tfirst, lenj, nt, ns, tns, twide);
    scan_i32(tns, ts0, nt);
    const int32_t nsl = total(ts0, tns, nt);
    s->at_slices = ws.get<ASlice>("opt.at.slices", nsl);
    hipLaunchKernelGGL(at_slices, dim3(ceil_div(nt, 256)), dim3(256), 0, st, tfirst, tns, twide, ts0, lenj, ebase, nt,
                       ns, s->at_tiles, s->at_slices);
    // 6-7: the jagged-diagonal entries and the lane words
    s->at_srow = ws.get<uint32_t>("opt.at.srow", (size_t)nsl * 64);
    s->at_pk = ws.get<uint16_t>("opt.at.pk", m);
    s->at_pv = ws.get<double>("opt.at.pv", m);
    hipLaunchKernelGGL(at_fill, dim3(ceil_div(nsl, 4)), dim3(256), 0, st, s->at_slices, nsl, og, sstart, skey, lenj,
                       rowbits, cs, vs, s->at_srow, s->at_pk, s->at_pv);
    s->at_rbt = ws.get<int32_t>("opt.at.rbt", nrb + 1);
    hipLaunchKernelGGL(at_ranges, dim3(ceil_div(nt + 1, 256)), dim3(256), 0, st, s->at_tiles, nt, nrb, s->at_rbt);
    TSNE_LAUNCH_CHECK();
    if (debug_tiles()) {   // layout statistics: tiles, segments, slices, slice widths
        std::vector<ASlice> hs(nsl);
        TSNE_HIP(hipMemcpyAsync(hs.data(), s->at_slices, sizeof(ASlice) * nsl, hipMemcpyDeviceToHost, st));
        TSNE_HIP(hipStreamSynchronize(st));
        int64_t wsum = 0, wmax = 0;
        for (const ASlice &x : hs) { wsum += x.width; wmax = std::max<int64_t>(wmax, x.width); }

        fprintf(stderr, "[attract tiles] cfg=%d rows=%lld m=%lld nrb=%lld ncb=%lld tiles=%d segments=%d slices=%d "
                "width avg=%.2f max=%lld entries/slice=%.1f\n", cfg, (long long)rows, (long long)m, (long long)nrb,
                (long long)ncb, nt, ns, nsl, nsl ? (double)wsum / nsl : 0.0, (long long)wmax,
                nsl ? (double)m / nsl : 0.0);
    }
    s->at_nrb = nrb;
    s->at_ncb = ncb;
    s->at_rbs = rbs;
    s->at_cfg = cfg;
    s->at_pipe = ctx->opts.attract_pipe;
    s->at_dyn = ctx->opts.attract_dyn;
    s->at_on = true;
}

// this rank's rows of P in the current labels (2-D)
static void build_own_rows(tsne_ctx *ctx, OptState *s) {
    hipStream_t st = ctx->stream;
    const int64_t m = s->L1 - s->L0;
    const int32_t *orig = s->orig[s->cur];
    hipLaunchKernelGGL(own_rowlen, dim3(ceil_div(m + 1, 256)), dim3(256), 0, st, orig, s->rp0, s->L0, s->L1, s->rowlen);
    size_t tb = s->scan_tmp_bytes;
    TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(s->scan_tmp, tb, s->rowlen, s->rpw, (int)(m + 1), st));
    if (m > 0)
        hipLaunchKernelGGL(own_rows, dim3(ceil_div(m, 4)), dim3(256), 0, st, orig, s->lab, s->rp0, s->col0, s->val0,
                           s->L0, s->L1, s->rpw, s->colw, s->valw);
    TSNE_LAUNCH_CHECK();
    // sum of the owned P entries (scal[6]) and Z = 1 (scal[7]) for the Z-free
    // loss terms of an attraction launched before this iteration's Z
    hipLaunchKernelGGL(reduce_partial_devn, dim3(NPART), dim3(256), 0, st, s->valw, s->rpw + m, s->part2);
    hipLaunchKernelGGL(reduce_final, dim3(1), dim3(256), 0, st, s->part2, NPART, s->scal + 6, 0.0);
    hipLaunchKernelGGL(set_unit, dim3(1), dim3(64), 0, st, s->scal + 7);
    build_attract_tiles(ctx, s);
}

// world > 1: the sorted positions of this rank's labels, ascending
static void build_qlist(tsne_ctx *ctx, OptState *s, const int32_t *idx_sorted) {
    hipStream_t st = ctx->stream;
    const int64_t n = s->n, nb = ceil_div(n, 256);
    hipLaunchKernelGGL(qlist_count, dim3(nb), dim3(256), 0, st, idx_sorted, n, s->L0, s->L1, s->qcnt);
    size_t tb = s->qscan_tmp_bytes;
    TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(s->qscan_tmp, tb, s->qcnt, s->qoff, (int)nb, st));
    hipLaunchKernelGGL(qlist_fill, dim3(nb), dim3(256), 0, st, idx_sorted, n, s->L0, s->L1, s->qoff, s->qlist);
    TSNE_LAUNCH_CHECK();
}

// Renumber labels: new label j holds old label order[j] (device); new cuts.
static void relabel(tsne_ctx *ctx, OptState *s, const int32_t *order, const std::vector<int64_t> &cuts) {
    hipStream_t st = ctx->stream;
    const int a = s->cur, b = 1 - a;
    gather_working_set(ctx, s);   // full upd / gains under the old cuts
    hipLaunchKernelGGL(relabel_state, dim3(ceil_div(s->n, 256)), dim3(256), 0, st, order, s->n, s->C, s->Y[a],
                       s->upd[a], s->gains[a], s->orig[a], s->Y[b], s->upd[b], s->gains[b], s->orig[b], s->lab);
    TSNE_LAUNCH_CHECK();
    s->cur = b;
    s->own = cuts;
    s->L0 = cuts[ctx->rank];
    s->L1 = cuts[ctx->rank + 1];
    build_own_rows(ctx, s);
    ++s->relabels;
}

// Initial labels: P's connected components (smallest original index), then
// the BFS level from that root, then the original index -- points that
// share neighbourhoods in P get nearby labels, so each XCD's rows gather
// their Y_j from a few components instead of the whole embedding while the
// embedding itself is still unrelated to P (the first ~150 iterations, before
// the Morton relabelling below takes over).  Deterministic fixpoints.
static void graph_order(tsne_ctx *ctx, OptState *s, int32_t *order) {
    hipStream_t st = ctx->stream;
    Workspace &ws = ctx->ws;
    const int64_t n = s->n;
    int32_t *comp = ws.get<int32_t>("opt.g.comp", n);
    int32_t *lev = ws.get<int32_t>("opt.g.lev", n);
    int32_t *flag = ws.get<int32_t>("opt.g.flag", 1);
    uint64_t *key = ws.get<uint64_t>("opt.g.key", n), *key2 = ws.get<uint64_t>("opt.g.key2", n);
    int32_t *val = ws.get<int32_t>("opt.g.val", n);
    hipLaunchKernelGGL(iota_i32, dim3(ceil_div(n, 256)), dim3(256), 0, st, comp, n);
    auto fixpoint = [&](auto &&pass) {
        for (int it = 0; it < 10000; ++it) {
            int32_t h = 0;
            TSNE_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), st));
            pass();
            TSNE_HIP(hipMemcpyAsync(&h, flag, sizeof(int32_t), hipMemcpyDeviceToHost, st));
            TSNE_HIP(hipStreamSynchronize(st));
            if (!h) return;
        }
        fail(TSNE_ERR_HIP, "graph ordering did not converge");
    };
    fixpoint([&] {
        hipLaunchKernelGGL(cc_pull, dim3(ceil_div(n, 4)), dim3(256), 0, st, s->rp0, s->col0, n, comp, flag);
        hipLaunchKernelGGL(cc_jump, dim3(ceil_div(n, 256)), dim3(256), 0, st, comp, n);
    });
    hipLaunchKernelGGL(level_init, dim3(ceil_div(n, 256)), dim3(256), 0, st, comp, n, lev);
    fixpoint([&] { hipLaunchKernelGGL(level_pull, dim3(ceil_div(n, 4)), dim3(256), 0, st, s->rp0, s->col0, n, lev, flag); });
    hipLaunchKernelGGL(graph_keys, dim3(ceil_div(n, 256)), dim3(256), 0, st, comp, lev, n, key, val);
    size_t tb = 0;
    TSNE_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, key2, val, order, (int)n, 0, 64, st));
    void *tmp = ws.get<uint8_t>("opt.g.tmp", tb);
    TSNE_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, key2, val, order, (int)n, 0, 64, st));
    TSNE_LAUNCH_CHECK();
}

void opt_setup(tsne_ctx *ctx, const tsne_params *p, const int64_t *d_row_ptr, const int32_t *d_col,
               const double *d_P, int64_t n, double *dY, double *dupd, double *dgains) {
    TSNE_REQUIRE(p != nullptr, "params is NULL");
    if (p->n_components != 2 && p->n_components != 3)
        fail(TSNE_ERR_UNSUPPORTED, "n_components must be 2 (quadtree) or 3 (octree extension)");
    TSNE_REQUIRE(n >= 1, "empty embedding");
    TSNE_REQUIRE(p->metric >= 0 && p->metric <= 2, "unknown metric");
    TSNE_REQUIRE(n < (int64_t)INT32_MAX, "n must fit int32 point ids");
    hipStream_t st = ctx->stream;
    opt_destroy(ctx);
    OptState *s = new OptState();
    ctx->opt = s;
    s->p = *p;
    s->C = p->n_components;
    const int C = s->C;
    const int world = ctx->world;
    s->n = n;
    s->Yu = dY;
    s->updu = dupd;
    s->gainsu = dgains;
    int64_t nnz = 0;
    TSNE_HIP(hipMemcpyAsync(&nnz, d_row_ptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    TSNE_HIP(hipStreamSynchronize(st));
    s->nnz = nnz;
    Workspace &ws = ctx->ws;
    s->rp0 = ws.get<int64_t>("opt.rp0", n + 1);
    s->col0 = ws.get<int32_t>("opt.col0", nnz + 1);
    s->val0 = ws.get<double>("opt.val0", nnz + 1);
    TSNE_HIP(hipMemcpyAsync(s->rp0, d_row_ptr, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToDevice, st));
    TSNE_HIP(hipMemcpyAsync(s->col0, d_col, sizeof(int32_t) * nnz, hipMemcpyDeviceToDevice, st));
    TSNE_HIP(hipMemcpyAsync(s->val0, d_P, sizeof(double) * nnz, hipMemcpyDeviceToDevice, st));
    for (int b = 0; b < 2; ++b) {
        const std::string k = std::to_string(b);
        s->Y[b] = ws.get<double>("opt.Y" + k, C * n);
        s->upd[b] = ws.get<double>("opt.upd" + k, C * n);
        s->gains[b] = ws.get<double>("opt.gains" + k, C * n);
        s->orig[b] = ws.get<int32_t>("opt.orig" + k, n);
    }
    s->lab = ws.get<int32_t>("opt.lab", n);
    s->cur = 0;
    TSNE_HIP(hipMemcpyAsync(s->Y[0], dY, sizeof(double) * C * n, hipMemcpyDeviceToDevice, st));
    TSNE_HIP(hipMemcpyAsync(s->upd[0], dupd, sizeof(double) * C * n, hipMemcpyDeviceToDevice, st));
    TSNE_HIP(hipMemcpyAsync(s->gains[0], dgains, sizeof(double) * C * n, hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(iota_i32, dim3(ceil_div(n, 256)), dim3(256), 0, st, s->orig[0], n);
    hipLaunchKernelGGL(iota_i32, dim3(ceil_div(n, 256)), dim3(256), 0, st, s->lab, n);
    s->own = equal_cuts(n, world);
    s->L0 = s->own[ctx->rank];
    s->L1 = s->own[ctx->rank + 1];
    const int64_t rows_cap = n;   // owned rows (cost-balanced cuts may give one rank most of them)
    s->rowlen = ws.get<int64_t>("opt.rowlen", rows_cap + 1);
    size_t tb = 0;
    TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, s->rowlen, s->rowlen, (int)(rows_cap + 1), st));
    s->scan_tmp_bytes = tb;
    s->scan_tmp = ws.get<uint8_t>("opt.scan_tmp", tb);
    s->Ynew = ws.get<double>("opt.Ynew", C * n);
    s->attr = ws.get<double2>("opt.attr", rows_cap);
    s->F = ws.get<double2>("opt.F", n);
    s->z = ws.get<double>("opt.z", n);
    s->scal = ws.get<double>("opt.scal", 8);
    s->part = ws.get<double>("opt.part", std::max<int64_t>(NPART, attract_max_blocks(rows_cap)));
    s->part2 = ws.get<double>("opt.part2", NPART);
    s->mpart = ws.get<double>("opt.mpart", 3 * ceil_div(rows_cap, 256) + 3);   // C <= 3 components
    s->bcost = ws.get<unsigned long long>("opt.bcost", ceil_div(n, 256) + 1);
    s->bounds = ws.get<int64_t>("opt.bounds", world + 1);
    s->lscore = ws.get<unsigned long long>("opt.lscore", 2);
    s->loss_slots = std::max(1, p->iterations / 10 + 1);
    s->loss = ws.get<double>("opt.loss", s->loss_slots);
    s->loss_written.assign(s->loss_slots, 0);
    s->visits = ws.get<unsigned long long>("opt.visits", VIS_N);
    if (sharded(ctx)) {
        const int64_t nb = ceil_div(n, 256);
        if (C == 2) {
            s->pcuts = ws.get<int64_t>("opt.pcuts", world + 1);
            s->plim = ws.get<int32_t>("opt.plim", 4);
            s->pcost = ws.get<unsigned long long>("opt.pcost", world);
            s->Fl = ws.get<double2>("opt.Fl", n);
            std::vector<int64_t> c0(world + 1);
            for (int r = 0; r <= world; ++r) c0[r] = n * r / world;
            TSNE_HIP(hipMemcpyAsync(s->pcuts, c0.data(), sizeof(int64_t) * (world + 1), hipMemcpyHostToDevice, st));
            TSNE_HIP(hipMemsetAsync(s->plim, 0, 4 * sizeof(int32_t), st));
            TSNE_HIP(hipStreamSynchronize(st));
        }
        s->qlist = ws.get<int32_t>("opt.qlist", n);
        s->qcnt = ws.get<int32_t>("opt.qcnt", nb);
        s->qoff = ws.get<int32_t>("opt.qoff", nb);
        size_t qb = 0;
        TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, qb, s->qcnt, s->qoff, (int)nb, st));
        s->qscan_tmp_bytes = qb;
        s->qscan_tmp = ws.get<uint8_t>("opt.qscan_tmp", qb);
    }
    TSNE_HIP(hipMemsetAsync(s->Ynew, 0, sizeof(double) * C * n, st));
    TSNE_HIP(hipMemsetAsync(s->F, 0, sizeof(double2) * n, st));
    TSNE_HIP(hipMemsetAsync(s->z, 0, sizeof(double) * n, st));
    if (C == 3) {
        oct_alloc(ctx, s->otree, n);
        s->F3 = ws.get<double>("opt.F3", 3 * (size_t)n);
        s->attr3 = ws.get<double>("opt.attr3", 3 * (size_t)rows_cap);
        s->part = ws.get<double>("opt.part", std::max<int64_t>(NPART, attract3_blocks(rows_cap)));
        TSNE_HIP(hipMemsetAsync(s->F3, 0, sizeof(double) * 3 * n, st));
    } else {
        bh_alloc(ctx, s->tree, n);
    }
    s->rpw = ws.get<int64_t>("opt.rpw", rows_cap + 1);
    s->colw = ws.get<int32_t>("opt.colw", nnz + 1);
    s->valw = ws.get<double>("opt.valw", nnz + 1);
    {   // initial labels in P's graph order (Options::graph_order = 0: the original order);
        // in 3-D too since round 6 (attract3's Y_j gathers then hit the L2 as in 2-D)
        const bool gorder = ctx->opts.graph_order != 0;
        const bool dense_small = s->nnz / n > 1024 && n * 16 <= (2 << 20);   // see maybe_relabel
        if (gorder && n >= 2 && !(dense_small && !sharded(ctx))) {
            int32_t *order = ws.get<int32_t>("opt.g.order", n);
            graph_order(ctx, s, order);
            relabel(ctx, s, order, s->own);
        } else {
            build_own_rows(ctx, s);
        }
    }
    for (auto &e : s->ev) TSNE_HIP(hipEventCreate(&e));
    TSNE_HIP(hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking));   // the attraction's (stream priorities: no gain, round 1)
    TSNE_HIP(hipEventCreateWithFlags(&s->ev_y, hipEventDisableTiming));
    TSNE_HIP(hipEventCreateWithFlags(&s->ev_attr, hipEventDisableTiming));
    ctx->timers.reset("opt.attract");
    ctx->timers.reset("opt.update");
    TSNE_LAUNCH_CHECK();
}

// Z = sum of z over all queries: locally (one rank) or this rank's partial
// over its query list + an all-reduce of one double
static void reduce_Z(tsne_ctx *ctx, OptState *s, const double *z, bool all_points = false) {
    hipStream_t st = ctx->stream;
    if (!sharded(ctx) || all_points) {   // every point (a tree partition: this rank's partial sums)
        hipLaunchKernelGGL(reduce_partial, dim3(NPART), dim3(256), 0, st, z, s->n, 1, 0, s->part2);
    } else {
        hipLaunchKernelGGL(reduce_list_partial, dim3(NPART), dim3(256), 0, st, z, s->qlist, s->L1 - s->L0, s->part2);
    }
    hipLaunchKernelGGL(reduce_final, dim3(1), dim3(256), 0, st, s->part2, NPART, s->scal, 0.0);
    if (sharded(ctx)) comm_allreduce_sum_f64(ctx, s->scal, 1);
}

// loss of this iteration (all ranks' partial sums) into its slot
static void record_loss(tsne_ctx *ctx, OptState *s, int32_t t, int64_t blocks, bool zfree = false,
                        double ex = 1.0) {
    hipStream_t st = ctx->stream;
    hipLaunchKernelGGL(reduce_partial, dim3(NPART), dim3(256), 0, st, s->part, blocks, 1, 0, s->part2);
    hipLaunchKernelGGL(reduce_final, dim3(1), dim3(256), 0, st, s->part2, NPART, s->scal + 1, 0.0);
    if (zfree) hipLaunchKernelGGL(loss_add_lnz, dim3(1), dim3(64), 0, st, s->scal, ex);
    if (sharded(ctx)) comm_allreduce_sum_f64(ctx, s->scal + 1, 1);
    const int slot = t / 10 - 1;
    if (slot >= 0 && slot < s->loss_slots) {
        TSNE_HIP(hipMemcpyAsync(s->loss + slot, s->scal + 1, sizeof(double), hipMemcpyDeviceToDevice, st));
        s->loss_written[slot] = t;
    }
}

// the updated embedding of every rank's labels on every rank
static void gather_Ynew(tsne_ctx *ctx, OptState *s) {
    std::vector<int64_t> off(ctx->world + 1);
    for (int r = 0; r <= ctx->world; ++r) off[r] = s->own[r] * s->C * (int64_t)sizeof(double);
    comm_allgatherv(ctx, s->Ynew, off.data());
}

static void finish_profile(tsne_ctx *ctx, OptState *s, int32_t t) {
    TSNE_HIP(hipEventRecord(s->ev[5], ctx->stream));
    TSNE_HIP(hipEventSynchronize(s->ev[5]));
    for (int k = 0; k < 5; ++k) {   // [3]: the attraction kernel alone, on its own stream
        float ms = 0.f;
        if (k != 3) TSNE_HIP(hipEventElapsedTime(&ms, s->ev[k], s->ev[k + 1]));
        s->last_ms[k] = ms;
    }
    s->last_ms[3] = ctx->timers.last_ms("opt.attract");
    if (s->C == 3) {
        for (int k = 0; k < 10; ++k) s->last_visits[k] = 0;
        return;
    }
    unsigned long long v[VIS_N] = {};
    TSNE_HIP(hipMemcpy(v, s->visits, sizeof(v), hipMemcpyDeviceToHost));
    for (int k = 0; k < 10; ++k) s->last_visits[k] = (int64_t)v[k];
    // the traversal waves' shader clock: their cycles over their 100 MHz wall ticks
    s->last_mhz = v[18] ? (int64_t)(100.0 * (double)v[37] / (double)v[18]) : 0;
    const bool dbg = debug_tiles();   // tile_apply diagnostics
    if (dbg)
        fprintf(stderr, "[tiles] t=%d tasks=%llu dense_pts=%llu momchk=%llu moment_evals=%llu dense_pairs=%llu "
                "pops=%llu child_slots=%llu all_take_full=%llu all_take_partial=%llu\n", t,
                v[10], v[11], v[12], v[1], v[2], v[3], v[6], v[13], v[14]);
    if (dbg && v[17] > 0)   // traversal wave times (100 MHz wall clock): span of the grid vs its waves
        fprintf(stderr, "[waves] t=%d span_us=%.1f max_wave_us=%.1f mean_wave_us=%.2f\n", t,
                (double)(v[17] - (~0ull - v[16])) * 0.01, (double)v[15] * 0.01,
                (double)v[18] * 0.01 / (double)std::max<int64_t>(1, ceil_div(s->L1 - s->L0, 64)));
    if (dbg)   // tile_apply dense paths: wave steps / useful lane pairs
        fprintf(stderr, "[tpaths] t=%d lanewise %llu/%llu packed %llu/%llu qmajor %llu/%llu staged %llu/%llu\n", t,
                v[24], v[25], v[26], v[27], v[28], v[29], v[30], v[31]);
    if (dbg && v[21] > 0)   // tile_apply waves (only waves with tiles report)
        fprintf(stderr, "[twaves] t=%d span_us=%.1f max_wave_us=%.1f\n", t,
                (double)(v[21] - (~0ull - v[20])) * 0.01, (double)v[19] * 0.01);
}

// One iteration of the 3-D (octree) optimizer: labels are P's graph order
// (set once at setup, as in 2-D; no Morton relabels), rank r owns labels
// [L0, L1) -- its rows of P in labels (rpw / colw / valw) -- and computes BH
// for exactly those points (its query list in octree order); only Z, the loss
// and the updated embedding cross ranks.
static void opt_step3(tsne_ctx *ctx, OptState *s, int32_t t) {
    hipStream_t st = ctx->stream;
    const tsne_params &p = s->p;
    const int32_t T = p.iterations;
    const int32_t n1 = std::min(T, 20);
    const int32_t n2 = std::min(T - n1, 81);
    const double ex = (t <= n1 + n2) ? p.early_exaggeration : 1.0;
    const double mom = (t <= n1) ? p.initial_momentum : p.final_momentum;
    const bool want_loss = (t % 10 == 0);
    const int64_t n = s->n;
    const int c = s->cur;
    double *Y = s->Y[c];
    const int64_t *rpl = s->rpw - s->L0;   // this rank's rows by label (rpl[L0] = 0)
    if (s->profile) TSNE_HIP(hipEventRecord(s->ev[0], st));
    oct_build(ctx, s->otree, Y, p.theta, ex == 1.0);
    if (s->profile) TSNE_HIP(hipEventRecord(s->ev[1], st));
    // the attraction of a non-loss iteration needs no Z: on the side stream,
    // beside the traversal (after the build, whose latency-bound kernels it
    // would stretch; the 2-D rule); a loss iteration's after Z, as before
    const bool side = !want_loss;
    int64_t blocks = 0;
    if (side) {
        TSNE_HIP(hipEventRecord(s->ev_y, st));
        TSNE_HIP(hipStreamWaitEvent(s->side, s->ev_y, 0));
        ctx->timers.begin("opt.attract", s->side);
        blocks = s->at_on ? attract_tiles3_launch(s->side, s, Y, s->scal, p.metric, ex, s->attr3, s->part, false)
                          : attract3_launch(s->side, rpl, s->colw, s->valw, s->L0, s->L1, Y, s->scal, p.metric, ex,
                                            s->attr3, s->part, false);
        ctx->timers.end("opt.attract", s->side);
        TSNE_HIP(hipEventRecord(s->ev_attr, s->side));
    }
    if (sharded(ctx)) {
        build_qlist(ctx, s, s->otree.idx_sorted);
        oct_repulsion(ctx, s->otree, p.theta, 0, s->L1 - s->L0, s->F3, s->z, s->qlist);
    } else {
        oct_repulsion(ctx, s->otree, p.theta, 0, n, s->F3, s->z, nullptr);
    }
    if (s->profile) TSNE_HIP(hipEventRecord(s->ev[2], st));
    reduce_Z(ctx, s, s->z);
    if (s->profile) TSNE_HIP(hipEventRecord(s->ev[3], st));
    if (side) {
        TSNE_HIP(hipStreamWaitEvent(st, s->ev_attr, 0));
    } else {
        ctx->timers.begin("opt.attract", st);
        blocks = s->at_on ? attract_tiles3_launch(st, s, Y, s->scal, p.metric, ex, s->attr3, s->part, want_loss)
                          : attract3_launch(st, rpl, s->colw, s->valw, s->L0, s->L1, Y, s->scal, p.metric, ex,
                                            s->attr3, s->part, want_loss);
        ctx->timers.end("opt.attract", st);
    }
    s->log_attract(t, side ? 0 : 1);   // 0: beside the traversal (side stream); 1: loss launch alone after Z
    if (s->profile) TSNE_HIP(hipEventRecord(s->ev[4], st));
    ctx->timers.begin("opt.update", st);
    // one rank: the mean's block partials from combine_update3, one
    // workgroup for the mean, one pass for the centring
    const bool fused_mean = !sharded(ctx);
    if (s->L1 > s->L0)
        hipLaunchKernelGGL(combine_update3<1>, dim3(ceil_div(s->L1 - s->L0, 256)), dim3(256), 0, st, s->L0, s->L1,
                           s->attr3, s->otree.inv, s->F3, s->scal, Y, nullptr, s->Ynew, s->upd[c], s->gains[c],
                           p.min_gain, mom, p.learning_rate, fused_mean ? s->mpart : nullptr);
    TSNE_LAUNCH_CHECK();
    if (want_loss) record_loss(ctx, s, t, blocks);
    if (fused_mean) {
        hipLaunchKernelGGL(mean3_final, dim3(1), dim3(256), 0, st, s->mpart, ceil_div(s->L1 - s->L0, 256), (double)n,
                           s->scal + 2);
        hipLaunchKernelGGL(center3, dim3(ceil_div(n * 3, 256)), dim3(256), 0, st, s->Ynew, n, s->scal + 2, Y);
    } else {
        gather_Ynew(ctx, s);
        for (int k = 0; k < 3; ++k) {
            hipLaunchKernelGGL(reduce_partial, dim3(NPART), dim3(256), 0, st, s->Ynew, n, 3, k, s->part2);
            hipLaunchKernelGGL(reduce_final, dim3(1), dim3(256), 0, st, s->part2, NPART, s->scal + 2 + k, (double)n);
        }
        hipLaunchKernelGGL(center_apply, dim3(ceil_div(n * 3, 256)), dim3(256), 0, st, s->Ynew, n, 3, s->scal + 2, Y);
    }
    ctx->timers.end("opt.update", st);
    TSNE_LAUNCH_CHECK();
    if (s->profile) finish_profile(ctx, s, t);
}

// Several ranks with the tiled layout keep P's graph order (TSNE_RELABEL
// unset): the ownership is re-cut in that order instead of a Morton relabel,
// which would hand the attraction back to attract_rows (C3 standalone: 2.35 vs
// 0.77 ms).  Each query's traversal cost goes to its label's 256-label bucket
// (an equal share of its wave's time); the all-reduced buckets give cuts of
// equal cost, applied (owned rows and their tiles rebuilt) when a cut moves
// by more than 1/16 of a rank's share.
// The tree partition (Options::bh_split): several ranks, 2-D.
static bool split_mode(const tsne_ctx *ctx, const OptState *s) {
    return sharded(ctx) && ctx->opts.bh_split && s->C == 2 && s->pcuts != nullptr;
}

static bool recut_mode(tsne_ctx *ctx, OptState *s) {
    if (split_mode(ctx, s)) return false;   // BH cost does not follow the row ownership there
    return ctx->opts.recut && ctx->opts.relabel == -1 && sharded(ctx) && s->at_on && !s->morton_labels;
}
static void recut(tsne_ctx *ctx, OptState *s, const std::vector<int64_t> &cuts) {
    gather_working_set(ctx, s);   // full upd / gains under the old cuts
    s->own = cuts;
    s->L0 = cuts[ctx->rank];
    s->L1 = cuts[ctx->rank + 1];
    build_own_rows(ctx, s);
    ++s->relabels;
}
static void maybe_recut(tsne_ctx *ctx, OptState *s) {
    hipStream_t st = ctx->stream;
    const int64_t n = s->n;
    ++s->relabel_checks;
    std::vector<int64_t> cuts(ctx->world + 1);
    comm_allreduce_sum_u64(ctx, s->bcost, (size_t)ceil_div(n, 256));
    bh_balance(ctx, s->bcost, n, ctx->world, s->bounds);
    TSNE_HIP(hipMemcpyAsync(cuts.data(), s->bounds, sizeof(int64_t) * (ctx->world + 1), hipMemcpyDeviceToHost, st));
    TSNE_HIP(hipStreamSynchronize(st));
    int64_t moved = 0;
    for (int r = 1; r < ctx->world; ++r) moved = std::max<int64_t>(moved, std::llabs(cuts[r] - s->own[r]));
    if (moved * 16 * ctx->world > n) recut(ctx, s, cuts);   // identical decision on every rank
}

// Relabel check (every RELABEL_EVERY iterations, 2-D): renumber the labels
// into this iteration's Morton order when that order keeps more of P's edges
// within a window of labels than the current one (identical decision on
// every rank: the score reads only replicated data).  With several ranks the
// new cuts balance the BH cost measured in this iteration (all-reduced
// 256-position bucket costs); the qlist waves of the NEXT iterations follow.
static void maybe_relabel(tsne_ctx *ctx, OptState *s) {
    hipStream_t st = ctx->stream;
    const int64_t n = s->n;
    if (recut_mode(ctx, s)) {   // several ranks on the tiled layout: re-cut the graph order by cost
        maybe_recut(ctx, s);
        return;
    }
    // dense rows over a small embedding (the distance-matrix mode, C5): every
    // row gathers all of Y, which sits in one XCD's L2 (n * 16 B <= 2 MiB)
    // whatever the labels, so a relabel (a copy of the whole P) buys nothing
    if (!sharded(ctx) && s->nnz / std::max<int64_t>(1, n) > 1024 && n * 16 <= (2 << 20)) return;
    // Options::relabel: 0 never, 1 by the locality score, 2 always; -1: by the
    // score, except on one rank with the tiled layout, which keeps P's graph
    // order (attract_tiles reads Y in label windows; a Morton relabel hands
    // the attraction back to attract_rows: whole C3 schedule 7.23 -> 7.01 s
    // without relabels, A/B on one box)
    const int mode = ctx->opts.relabel;
    if (mode == 0 || (mode == -1 && !sharded(ctx) && s->at_on)) return;
    // a fixed sample of rows, ~1 << 22 entries at most (dense rows: fewer rows)
    const int64_t avg = std::max<int64_t>(1, s->nnz / std::max<int64_t>(1, n));
    const int64_t nsamp = std::max<int64_t>(1, std::min<int64_t>({n, 1 << 16, (1 << 22) / avg}));
    const int64_t stride = std::max<int64_t>(1, n / nsamp);
    const int64_t win = std::max<int64_t>(64, n / 64);
    TSNE_HIP(hipMemsetAsync(s->lscore, 0, 2 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(locality_score, dim3(ceil_div(nsamp, 4)), dim3(256), 0, st, s->rp0, s->col0, s->lab,
                       s->tree.inv, n, stride, nsamp, win, s->lscore);
    unsigned long long sc[2] = {0, 0};
    TSNE_HIP(hipMemcpyAsync(sc, s->lscore, sizeof(sc), hipMemcpyDeviceToHost, st));
    TSNE_HIP(hipStreamSynchronize(st));
    ++s->relabel_checks;
    const bool go = mode == 2 || sc[1] > sc[0];
    if (!go) return;
    std::vector<int64_t> cuts = s->own;
    if (sharded(ctx) && !split_mode(ctx, s)) {   // (tree partition: the rows keep equal label cuts)
        comm_allreduce_sum_u64(ctx, s->bcost, (size_t)ceil_div(n, 256));
        bh_balance(ctx, s->bcost, n, ctx->world, s->bounds);
        TSNE_HIP(hipMemcpyAsync(cuts.data(), s->bounds, sizeof(int64_t) * (ctx->world + 1), hipMemcpyDeviceToHost, st));
        TSNE_HIP(hipStreamSynchronize(st));
    }
    s->morton_labels = true;
    relabel(ctx, s, s->tree.idx_sorted, cuts);
}

// The optimizer's attraction: attract_tiles over the tiled layout when it was
// built, else attract_rows over the owned CSR rows.  Returns the blocks (loss
// partials) written.
template <class CF, bool LOSS, int MET>
static void attract_tiles_launch_c(hipStream_t st, const OptState *s, const AttractArgs &a) {
    const int64_t nb = s->at_nrb;
#define TSNE_ATP(K)                                                                                            \
    hipLaunchKernelGGL(K, dim3(nb), dim3(CF::NT), 0, st, s->at_tiles, s->at_rbt, s->at_slices, s->at_srow,    \
                       a.r1 - a.r0, a.r0, s->n, s->at_pk, s->at_pv, a.Y, a.scal, a.ex, nb / NUM_XCD, a.attr, \
                       a.lpart, s->at_rbs)
    if constexpr (CF::RB == 4096 && !LOSS) {
        switch (s->at_pipe) {
            case 1: TSNE_ATP((attract_tiles_pipe<CF, 1, 6, LOSS, MET>)); return;
            case 2: TSNE_ATP((attract_tiles_pipe<CF, 1, 8, LOSS, MET>)); return;
            case 3: TSNE_ATP((attract_tiles_pipe<CF, 2, 4, LOSS, MET>)); return;
            case 4: TSNE_ATP((attract_tiles_pipe<CF, 2, 6, LOSS, MET>)); return;
            case 5: TSNE_ATP((attract_tiles_pipe<CF, 3, 4, LOSS, MET>)); return;
            default: break;
        }
    }
    // loss launches deal the slices round-robin: a wave's loss partial sums the
    // slices it ran, so claimed slices would make the loss's rounding vary
    if (s->at_dyn && !LOSS) TSNE_ATP((attract_tiles<CF, LOSS, MET, true>));
    else TSNE_ATP((attract_tiles<CF, LOSS, MET, false>));
#undef TSNE_ATP
}
template <bool LOSS, int MET>
static void attract_tiles_launch_m(hipStream_t st, const OptState *s, const AttractArgs &a) {
    switch (s->at_cfg) {
        case 0: attract_tiles_launch_c<ATCfg0, LOSS, MET>(st, s, a); break;
        case 1: attract_tiles_launch_c<ATCfg1, LOSS, MET>(st, s, a); break;
        case 3: attract_tiles_launch_c<ATCfg3, LOSS, MET>(st, s, a); break;
        default: attract_tiles_launch_c<ATCfg2, LOSS, MET>(st, s, a); break;
    }
}
template <bool LOSS>
static void attract_tiles_launch_l(hipStream_t st, const OptState *s, const AttractArgs &a) {
    switch (a.metric) {
        case TSNE_METRIC_EUCLIDEAN: attract_tiles_launch_m<LOSS, TSNE_METRIC_EUCLIDEAN>(st, s, a); break;
        case TSNE_METRIC_COSINE: attract_tiles_launch_m<LOSS, TSNE_METRIC_COSINE>(st, s, a); break;
        default: attract_tiles_launch_m<LOSS, TSNE_METRIC_SQEUCLIDEAN>(st, s, a); break;
    }
}
// attract_tiles only while the tree build takes the root-tile path: beside
// the BH traversal of the later phases its 156 KB of LDS per CU keeps the
// traversal's workgroups off those CUs (t = 180..300 at C3: 5.4 ms per
// concurrent launch vs 3.1 for attract_rows), and there the attraction is
// hidden behind the traversal anyway.
static int64_t attract_launch_opt(hipStream_t st, const OptState *s, const AttractArgs &a, bool loss) {
    // tiles in every phase while the labels are P's graph order (only in the
    // root-tile phase, attract_rows after it: whole C3 schedule 5.94 -> 6.40 s)
    if (!s->at_on) return attract_launch(st, a, loss);
    if (loss) attract_tiles_launch_l<true>(st, s, a);
    else attract_tiles_launch_l<false>(st, s, a);
    return s->at_nrb;
}

void opt_step(tsne_ctx *ctx, int32_t t) {
    OptState *s = ctx->opt;
    TSNE_REQUIRE(s != nullptr, "tsne_dev_opt_setup has not been called");
    TSNE_REQUIRE(t >= 1, "iteration numbers start at 1");
    if (s->C == 3) {
        opt_step3(ctx, s, t);
        return;
    }
    hipStream_t st = ctx->stream;
    const tsne_params &p = s->p;
    const int32_t T = p.iterations;
    const int32_t n1 = std::min(T, 20);
    const int32_t n2 = std::min(T - n1, 81);
    const double ex = (t <= n1 + n2) ? p.early_exaggeration : 1.0;
    const double mom = (t <= n1) ? p.initial_momentum : p.final_momentum;
    const int want_loss = (t % 10 == 0);
    const bool check_relabel = t % RELABEL_EVERY == 0;
    const int64_t n = s->n;
    double *Y = s->Y[s->cur];
    if (s->profile) {
        TSNE_HIP(hipMemsetAsync(s->visits, 0, VIS_N * sizeof(unsigned long long), st));
        TSNE_HIP(hipEventRecord(s->ev[0], st));
    }
    // attraction over this rank's rows (row pointer local to L0)
    AttractArgs aa{s->rpw - s->L0, s->colw, s->valw, s->L0, s->L1, Y, s->scal, p.metric, ex, s->attr, s->part};
    // 0. attraction sums on the side stream, concurrent with the BH
    // traversal (in loss iterations with Z-free KL terms, P ln(P (1 + metric)):
    // ln(Z) sum P is added once Z is known; the loss launch alone after Z:
    // whole schedule +1 %) -- or, while the last build took the root-tile
    // path, already with the tree build, on 3 blocks per CU (as fast as 8:
    // miss-bound) so that the build's short kernels keep the other slots.  A
    // full build is not overlapped: its latency-bound kernels stretch under
    // the attraction (morton_keys 15 -> 800 us; whole schedule 8.53 -> 8.97 s).
    const bool rt_phase = s->tree.root_tile;
    if (want_loss) aa.scal = s->scal + 7;   // Z = 1 in the kernel
    int64_t blocks = 0;
    if (rt_phase) aa.bpc = 3;
    auto side_attract = [&] {
        TSNE_HIP(hipEventRecord(s->ev_y, st));
        TSNE_HIP(hipStreamWaitEvent(s->side, s->ev_y, 0));
        ctx->timers.begin("opt.attract", s->side);
        blocks = attract_launch_opt(s->side, s, aa, want_loss != 0);
        TSNE_LAUNCH_CHECK();
        ctx->timers.end("opt.attract", s->side);
        s->log_attract(t, want_loss ? 2 : 0);
        TSNE_HIP(hipEventRecord(s->ev_attr, s->side));
    };
    // (attract_serial_t0 <= t <= attract_serial_t1: the attraction alone on
    // this stream after the BH kernels instead -- an A/B of the overlap's cost)
    const bool serial_at = t >= ctx->opts.attract_serial_t0 && t <= ctx->opts.attract_serial_t1 && !rt_phase;
    if (rt_phase) side_attract();
    // 1. tree (identical on every rank)
    // insertion rows = original indices; the root-tile shortcut while the
    // embedding is small
    // the strict near-exact tolerance while P is exaggerated (the dynamics
    // amplify any difference fastest there), the late one after
    bh_build(ctx, s->tree, Y, p.theta, s->orig[s->cur], root_tile_enabled(ctx), bh_near_tol(ctx, ex == 1.0));
    if (sharded(ctx)) comm_mark(ctx, s->tree.root_tile ? "tree_rt" : "tree");
    if (!rt_phase && !serial_at) side_attract();
    if (s->profile) TSNE_HIP(hipEventRecord(s->ev[1], st));
    // 2. repulsion for this rank's points: all of them, or its query list
    // (its labels' sorted positions, ascending: the waves stay Morton-local);
    // bucket costs only where a relabel may re-cut the ownership
    // tree partition: every query over this rank's cells (sorted-position
    // range, re-cut by the ranks' traversal costs every iteration)
    const bool split = split_mode(ctx, s) && !s->tree.root_tile;
    s->split_last = split;
    unsigned long long *bcost = (sharded(ctx) && check_relabel && !split_mode(ctx, s)) ? s->bcost : nullptr;
    if (bcost) TSNE_HIP(hipMemsetAsync(bcost, 0, sizeof(unsigned long long) * ceil_div(n, 256), st));
    if (split) {
        part_align(ctx, s->tree, s->pcuts, ctx->world, ctx->rank, s->plim);
        bh_repulsion(ctx, s->tree, p.theta, 0, n, s->F, s->z, s->profile ? s->visits : nullptr, nullptr, nullptr, false,
                     s->plim);
        comm_mark(ctx, "bh");
    } else if (sharded(ctx)) {
        build_qlist(ctx, s, s->tree.idx_sorted);
        bh_repulsion(ctx, s->tree, p.theta, 0, s->L1 - s->L0, s->F, s->z, s->profile ? s->visits : nullptr, s->qlist,
                     bcost, recut_mode(ctx, s));
        comm_mark(ctx, s->tree.root_tile ? "bh_rt" : "bh");
    } else {
        bh_repulsion(ctx, s->tree, p.theta, 0, n, s->F, s->z, s->profile ? s->visits : nullptr);
    }
    if (serial_at) side_attract();   // (the side stream waits for everything above)
    if (s->profile) TSNE_HIP(hipEventRecord(s->ev[2], st));
    // 3. Z (TsneHelpers.scala:266): the only per-iteration all-reduce
    reduce_Z(ctx, s, s->z, split);
    const double2 *Fc = s->F;           // combine_update's forces: sorted order (inv) ...
    const int32_t *Finv = s->tree.inv;
    if (split) {
        // the next iteration's cuts from this traversal's costs (identical on every rank)
        TSNE_HIP(hipMemsetAsync(s->pcost, 0, sizeof(unsigned long long) * ctx->world, st));
        part_cost(ctx, s->tree, ceil_div(n, 64), s->pcost + ctx->rank);
        comm_allreduce_sum_u64(ctx, s->pcost, (size_t)ctx->world);
        part_recut(ctx, s->pcost, ctx->world, n, s->pcuts);
        // ... or, with the tree partition, by label after the reduce-scatter of
        // every rank's partial sums to the row owners
        hipLaunchKernelGGL(f_to_label, dim3(ceil_div(n, 256)), dim3(256), 0, st, s->tree.inv, n, s->F, s->Fl);
        std::vector<int64_t> off(ctx->world + 1);
        for (int r = 0; r <= ctx->world; ++r) off[r] = 2 * s->own[r];
        comm_reduce_scatterv_f64(ctx, reinterpret_cast<double *>(s->Fl), off.data());
        Fc = s->Fl;
        Finv = nullptr;
    }
    if (s->profile) TSNE_HIP(hipEventRecord(s->ev[3], st));
    // 4. the attraction's sums + update for owned rows
    TSNE_HIP(hipStreamWaitEvent(st, s->ev_attr, 0));
    if (s->profile) TSNE_HIP(hipEventRecord(s->ev[4], st));
    // update + centre: combine_update (with the mean's block partials when one
    // rank holds every row), mean, centre + write-back of the caller's Y
    ctx->timers.begin("opt.update", st);
    const bool fused_mean = !sharded(ctx);
    const int c = s->cur;
    combine_launch<1>(st, s->L0, s->L1, s->attr, Finv, Fc, s->scal, Y, nullptr, s->Ynew, s->upd[c],
                      s->gains[c], p.min_gain, mom, p.learning_rate, fused_mean ? s->mpart : nullptr);
    if (want_loss) record_loss(ctx, s, t, blocks, true, ex);
    // 5. exchange (all-gather of the owned slices) + 6. centre
    if (fused_mean) {
        hipLaunchKernelGGL(mean2_final, dim3(1), dim3(256), 0, st, s->mpart, ceil_div(s->L1 - s->L0, 256),
                           (double)n, s->scal + 2);
    } else {
        gather_Ynew(ctx, s);
        for (int k = 0; k < 2; ++k) {
            hipLaunchKernelGGL(reduce_partial, dim3(NPART), dim3(256), 0, st, s->Ynew, n, 2, k, s->part2);
            hipLaunchKernelGGL(reduce_final, dim3(1), dim3(256), 0, st, s->part2, NPART, s->scal + 2 + k, (double)n);
        }
    }
    hipLaunchKernelGGL(center2, dim3(ceil_div(n, 256)), dim3(256), 0, st, s->Ynew, n, s->scal + 2, Y);
    ctx->timers.end("opt.update", st);
    TSNE_LAUNCH_CHECK();
    if (check_relabel) maybe_relabel(ctx, s);
    if (s->profile) finish_profile(ctx, s, t);
}

// The tree partition's traversal stack guard (bh_traverse<., true>): never
// expected to trip (the cut alignment bounds the shared depth); loud if it did.
static void check_split_overflow(tsne_ctx *ctx, const OptState *s) {
    if (!s->plim) return;
    int32_t f = 0;
    TSNE_HIP(hipMemcpyAsync(&f, s->plim + 2, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    TSNE_HIP(hipStreamSynchronize(ctx->stream));
    if (f) fail(TSNE_ERR_HIP, "tree-partition traversal stack overflow (results invalid)");
}

// Write upd / gains (and Y) back to the caller's buffers in the original order.
void opt_sync(tsne_ctx *ctx) {
    OptState *s = ctx->opt;
    TSNE_REQUIRE(s != nullptr, "tsne_dev_opt_setup has not been called");
    check_split_overflow(ctx, s);
    hipStream_t st = ctx->stream;
    gather_working_set(ctx, s);
    const int c = s->cur;
    const int64_t n = s->n;
    const int C = s->C;
    hipLaunchKernelGGL(scatter_to_user_c, dim3(ceil_div(n, 256)), dim3(256), 0, st, s->Y[c], s->orig[c], n, C, s->Yu);
    hipLaunchKernelGGL(scatter_to_user_c, dim3(ceil_div(n, 256)), dim3(256), 0, st, s->upd[c], s->orig[c], n, C,
                       s->updu);
    hipLaunchKernelGGL(scatter_to_user_c, dim3(ceil_div(n, 256)), dim3(256), 0, st, s->gains[c], s->orig[c], n, C,
                       s->gainsu);
    TSNE_LAUNCH_CHECK();
}

int32_t opt_losses(tsne_ctx *ctx, int32_t *keys, double *vals, int32_t cap) {
    OptState *s = ctx->opt;
    TSNE_REQUIRE(s != nullptr, "tsne_dev_opt_setup has not been called");
    check_split_overflow(ctx, s);
    std::vector<double> h(s->loss_slots);
    TSNE_HIP(hipMemcpyAsync(h.data(), s->loss, sizeof(double) * s->loss_slots, hipMemcpyDeviceToHost, ctx->stream));
    TSNE_HIP(hipStreamSynchronize(ctx->stream));
    int32_t k = 0;
    for (int32_t i = 0; i < s->loss_slots; ++i) {
        if (!s->loss_written[i]) continue;
        if (k < cap) {
            if (keys) keys[k] = s->loss_written[i];
            if (vals) vals[k] = h[i];
        }
        ++k;
    }
    return k;
}

int32_t opt_attract_log(tsne_ctx *ctx, int32_t *iters, int32_t *standalone, double *ms, int32_t cap) {
    OptState *s = ctx->opt;
    TSNE_REQUIRE(s != nullptr, "tsne_dev_opt_setup has not been called");
    const std::vector<double> v = ctx->timers.ms("opt.attract");
    TSNE_REQUIRE(v.size() == s->attract_iter.size(), "attraction timer log out of step");
    const int32_t k = (int32_t)v.size();
    for (int32_t e = 0; e < k && e < cap; ++e) {
        if (iters) iters[e] = s->attract_iter[e].first;
        if (standalone) standalone[e] = s->attract_iter[e].second;
        if (ms) ms[e] = v[e];
    }
    return k;
}

int64_t opt_attract_kernel(tsne_ctx *ctx) {
    OptState *s = ctx->opt;
    if (!s) return -1;
    return s->C == 3 ? (s->at_on ? 3 : 2) : (s->at_on ? 1 : 0);
}

BHTree *opt_tree(tsne_ctx *ctx) {
    OptState *s = ctx->opt;
    return (s && s->C == 2) ? &s->tree : nullptr;
}

double opt_last_z(tsne_ctx *ctx) {
    OptState *s = ctx->opt;
    TSNE_REQUIRE(s != nullptr, "tsne_dev_opt_setup has not been called");
    double z = 0.0;
    TSNE_HIP(hipMemcpyAsync(&z, s->scal, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    TSNE_HIP(hipStreamSynchronize(ctx->stream));
    return z;
}

void opt_profile(tsne_ctx *ctx, int enable, double *ms5, int64_t *visits) {
    OptState *s = ctx->opt;
    TSNE_REQUIRE(s != nullptr, "tsne_dev_opt_setup has not been called");
    if (enable >= 0) s->profile = enable != 0;
    if (ms5)
        for (int k = 0; k < 5; ++k) ms5[k] = s->last_ms[k];
    if (visits)
        for (int k = 0; k < 10; ++k) visits[k] = s->last_visits[k];
}

}  // namespace tsne
