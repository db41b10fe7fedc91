// common.hpp -- shared plumbing for libtsne_hip (gfx950 / MI355X only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/tsne_hip.h"

namespace tsne {

// Internal error type; converted to a tsne_status at the C ABI boundary.
struct Error : std::runtime_error {
    int status;
    Error(int s, const std::string &m) : std::runtime_error(m), status(s) {}
};

[[noreturn]] void fail(int status, const std::string &msg);

#define TSNE_HIP(expr)                                                                     \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            ::tsne::fail(TSNE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define TSNE_LAUNCH_CHECK() TSNE_HIP(hipGetLastError())

#define TSNE_REQUIRE(cond, msg)                                         \
    do {                                                                \
        if (!(cond)) ::tsne::fail(TSNE_ERR_ARG, std::string(msg));     \
    } while (0)

// Growable device allocation owned by the context.
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    void *ensure(size_t b) {
        if (b > bytes) {
            release();
            size_t want = b < 256 ? 256 : b;
            hipError_t e = hipMalloc(&p, want);
            if (e != hipSuccess) {
                p = nullptr;
                fail(TSNE_ERR_NOMEM, "hipMalloc(" + std::to_string(want) + ") failed: " + hipGetErrorString(e));
            }
            bytes = want;
        }
        return p;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

// Named workspace: each stage grabs buffers by name; they persist across calls.
struct Workspace {
    std::map<std::string, std::unique_ptr<DevBuf>> bufs;
    template <class T> T *get(const std::string &name, size_t count) {
        auto &b = bufs[name];
        if (!b) b.reset(new DevBuf());
        return static_cast<T *>(b->ensure(count * sizeof(T)));
    }
    bool has(const std::string &name) const { return bufs.count(name) != 0; }
    void clear() { bufs.clear(); }
    // free every buffer whose name starts with prefix (large one-time temporaries)
    void release_prefix(const std::string &prefix) {
        for (auto it = bufs.begin(); it != bufs.end();)
            it = it->first.compare(0, prefix.size(), prefix) == 0 ? bufs.erase(it) : std::next(it);
    }
};

// Named kernel-stage timers: HIP event pairs recorded on the stream the
// stage's kernels run on, read (and synchronised) only when asked for, so a
// timed loop never waits on them.  Events are pooled and reused; a stage keeps
// its last CAP intervals (older pairs are recycled), so a long device loop
// holds a bounded number of events.
struct StageTimers {
    static constexpr size_t CAP = 1 << 14;
    std::map<std::string, std::deque<std::pair<hipEvent_t, hipEvent_t>>> rec;
    std::vector<hipEvent_t> pool;
    hipEvent_t take() {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) fail(TSNE_ERR_HIP, "hipEventCreate failed");
        return e;
    }
    void reset(const std::string &name) {
        auto it = rec.find(name);
        if (it == rec.end()) return;
        for (auto &p : it->second) { pool.push_back(p.first); pool.push_back(p.second); }
        it->second.clear();
    }
    // begin(): opens a new interval (recycling the oldest beyond CAP); end() closes it.
    void begin(const std::string &name, hipStream_t st) {
        auto &v = rec[name];
        if (v.size() >= CAP) {   // the oldest interval's events are complete or reusable: re-recorded below
            pool.push_back(v.front().first);
            pool.push_back(v.front().second);
            v.pop_front();
        }
        v.push_back({take(), take()});
        if (hipEventRecord(v.back().first, st) != hipSuccess) fail(TSNE_ERR_HIP, "hipEventRecord failed");
    }
    void end(const std::string &name, hipStream_t st) {
        auto &v = rec[name];
        if (v.empty()) fail(TSNE_ERR_HIP, "stage timer " + name + " not started");
        if (hipEventRecord(v.back().second, st) != hipSuccess) fail(TSNE_ERR_HIP, "hipEventRecord failed");
    }
    static double elapsed(const std::pair<hipEvent_t, hipEvent_t> &p) {
        if (hipEventSynchronize(p.second) != hipSuccess) fail(TSNE_ERR_HIP, "hipEventSynchronize failed");
        float f = 0.f;
        if (hipEventElapsedTime(&f, p.first, p.second) != hipSuccess) fail(TSNE_ERR_HIP, "hipEventElapsedTime failed");
        return f;
    }
    // elapsed ms of every kept interval of `name` (synchronises on their events)
    std::vector<double> ms(const std::string &name) {
        std::vector<double> out;
        auto it = rec.find(name);
        if (it == rec.end()) return out;
        for (auto &p : it->second) out.push_back(elapsed(p));
        return out;
    }
    // elapsed ms of the last interval only (0 if none)
    double last_ms(const std::string &name) {
        auto it = rec.find(name);
        if (it == rec.end() || it->second.empty()) return 0.0;
        return elapsed(it->second.back());
    }
    size_t count(const std::string &name) const {
        auto it = rec.find(name);
        return it == rec.end() ? 0 : it->second.size();
    }
    void clear() {
        for (auto &kv : rec)
            for (auto &p : kv.second) { (void)hipEventDestroy(p.first); (void)hipEventDestroy(p.second); }
        rec.clear();
        for (hipEvent_t e : pool) (void)hipEventDestroy(e);
        pool.clear();
    }
    ~StageTimers() { clear(); }
};

struct Comm;      // collective backend: RCCL or in-process loopback (comm.cpp)
struct OptState;  // device-resident optimizer state (optimize.hip)
struct BHTree;    // Barnes-Hut tree (bhtree.hpp)

// Per-context tunables (tsne_ctx_set_option): the library's defaults, set per
// handle by the caller -- nothing here is process-static.  DESIGN.md 3a gives
// the tolerances' derivations and measurements.
struct Options {
    // near-exact BH subtrees (bh_traverse): relative bound per summarised cell,
    // single gradients and the early-exaggeration phase / the optimizer after it
    double near_tol_early = 1e-6, near_tol_late = 5e-6;
    double mom_tol = 1e-12;                               // subtree-moment truncation bound (2-D)
    double near_tol3_early = 1e-7, near_tol3_late = 5e-6;  // the 3-D octree's
    double mom3_tol = 1e-12;
    int oct_moments = 1;      // 3-D subtree moments
    int coherent_sort = 1;    // the trees' Morton sort from the previous build's order (csort.hpp; 0: rocPRIM's radix sort)
    double oct_layout_switch = 6.0;   // 3-D: the 8-query layout while the root half-width < this x sqrt(near_dmax)
    int oct_records = 2;      // 3-D: octal records + the 64-query record traversal (1: the 8-query one; 0: the binary-node walk)
    int root_tile = 1;        // root-tile shortcut of the small-embedding phase
    int attract_tiles = 1;    // tiled attraction (attract_tiles) where the labels allow it
    int attract_tiles3 = 0;   // 3-D: the tiled attraction (attract_tiles3) instead of attract3 (C4: 6.7 vs 3.7 ms
                              // per launch beside the octree traversal; round 6)
    int attract_cfg = -1;     // its tile shape: -1 by rows per rank, else ATCfg0..3
    int attract_pipe = 0;     // 2-D tiled attraction: 0 attract_tiles, 1..5 attract_tiles_pipe shapes (round 6)
    int attract_dyn = 1;      // attract_tiles: a tile's slices claimed by the waves (round 6; same sums)
    int graph_order = 1;      // P's graph order (components + BFS) as the initial labels
    int relabel = -1;         // -1 automatic, 0 never, 1 by the locality score, 2 always
    int recut = 0;            // several ranks on the tiled layout: re-cut by BH cost instead of relabels
    int knn_bf16 = 1;         // kNN threshold filter: bf16x3 MFMA (0: f32-input MFMA)
    double narrow = 3.0;      // BH: 64-query groups costing >= narrow x the mean run in the narrow layout (0: off)
    int bh_split = 0;         // several ranks: 1 = partition the BH tree by sorted-position ranges (every rank walks
                              // every query over its own cells; F summed by a reduce-scatter) instead of the queries
                              // (0; measured faster at 8 projected ranks)
    int bu_acqrel = 1;        // bottom-up hand-off: 1 = agent-scope acquire-release arrivals (HIP memory model),
                              // 0 = relaxed arrivals + gfx950 in-order issue (no measurable difference)
    int loop_serial = 0;      // loopback groups: ranks take turns on the device and log their work between
                              // collectives (tsne_ctx_loop_profile; a one-GPU projection of N GPUs)
    int rep_stats = 0;        // tsne_repulsion / tsne_dev_repulsion (2-D): count the traversal's pops, child slots and
                              // tile points (the counting kernel variant) for tsne_ctx_counter "bh.*"
    int comm_world1 = 0;      // tsne_ctx_init_comm / _callbacks at world 1 still create the communicator, and
                              // the optimizer runs its sharded code path through it (tests the transport)
    int reuse_costs = 0;      // single-call BH (tsne_gradient / tsne_repulsion): select narrow groups from the
                              // previous call's costs (results then depend on the call history at rounding level)
    // BH work splitting (bhtree.hip "Spill"): a 64-query wave stops after spill x the previous
    // traversal's mean wave cost (in record pops, >= spill_min) and hands its stack to idle waves as
    // tasks, which split again after spill_task x that budget (0: off); spill_force > 0 sets both
    // budgets to that many pops from the first traversal on (tests); spill_drains follow-up launches
    // take the tasks left when the traversal's waves ended (the last one never splits)
    double spill = 0.0, spill_task = 0.25;
    int spill_min = 256, spill_force = 0, spill_drains = 2;
    // tile streaming (2-D BH, one rank): tile_stream > 0 launches that many
    // consumer workgroups per CU on their own stream beside the traversal;
    // they sum the tile lists of traversal waves
    // whose tile cost is <= tile_stream_max while the traversal's last waves
    // run (4095: only lists the slot path would not chunk, so the sums are
    // bit-identical to tile_stream 0)
    int tile_stream = 0, tile_stream_max = 0;
    double tile_stream_frac = 1.0;   // tile_stream_max 0: streamed up to this x the previous plan's chunk unit
    int tile_stream_wait = 48;   // polls (~0.4 us each) a consumer waits for the next list before it leaves
    int attract_serial_t0 = 0, attract_serial_t1 = -1;   // 2-D: the attraction after BH for t in [t0, t1] (A/B)
    int wave_log = 0;            // with rep_stats: the counting call logs every BH wave's start / end (tsne_debug_wave_log)
    double trav_front = 0.0;     // > 0: the 64-query traversal's workgroups whose heaviest wave cost >= this x the
                                 // previous traversal's mean first (the order made with the narrow selection)
    double trav_front_cur = 0.0; // > 0: as trav_front, the order predicted from the points' previous costs
                                 // through this build's Morton order (made during the build, second stream)
    int trav_prio = 0;           // 1-3: the 64-query BH traversal's waves at that issue priority (s_setprio)
    int tile_stream_gate = 1;    // 1: the consumers wait (on the device) until every traversal block has started
};

}  // namespace tsne

struct tsne_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    hipStream_t aux_stream = nullptr;   // second stream of one operator (the narrow BH waves)
    hipEvent_t aux_ev[2] = {nullptr, nullptr};
    // third stream: the tile-streaming consumers (created on first use)
    hipStream_t st_stream = nullptr;
    hipEvent_t st_ev[3] = {nullptr, nullptr, nullptr};
    int rank = 0, world = 1;
    tsne::Comm *comm = nullptr;
    tsne::Workspace ws;
    tsne::OptState *opt = nullptr;
    tsne::Options opts;
    tsne::BHTree *single_tree = nullptr;   // bh_single_tree (owned; freed by tsne_ctx_destroy)
    std::string loop_profile_pending;      // tsne_ctx_loop_profile: a summary read for its length, not yet copied out
    tsne::StageTimers timers;
    int32_t *pinned = nullptr;   // small pinned host scratch (per-iteration read-backs)
    int cu_count = 256;
    // tsne_ctx_create_multi: the per-device contexts (ranks) of a group
    // handle; host-buffer operators fan out over them, one thread per rank
    std::vector<tsne_ctx *> group;
};

namespace tsne {

// RAII guard that makes ctx->device current for the calling thread.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) TSNE_HIP(hipSetDevice(dev));
    }
    ~DeviceGuard() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

// ---- stage entry points (device pointers, enqueue on ctx->stream) ----
void knn_device(tsne_ctx *ctx, const double *dX, int64_t n, int32_t d, int32_t metric,
                int32_t k, int64_t q0, int64_t q1, int32_t *d_idx, double *d_dist);
void project_knn_device(tsne_ctx *ctx, const double *dX, int64_t n, int32_t d, int32_t metric, int32_t k,
                        int32_t iterations, const double *d_shifts, int32_t *d_idx, double *d_dist);
void affinities_device(tsne_ctx *ctx, const int64_t *d_row_ptr, const double *d_dist,
                       int64_t nrows, double perplexity, double *d_p);
int64_t joint_device(tsne_ctx *ctx, const int64_t *d_row_ptr, const int32_t *d_col,
                     const double *d_p, int64_t n, int64_t cap, int64_t *d_out_row_ptr,
                     int32_t *d_out_col, double *d_out_val);
void init_working_set_device(tsne_ctx *ctx, int64_t n, int32_t c, uint64_t seed, double *dY,
                             double *dupd, double *dgains);
void update_device(tsne_ctx *ctx, int64_t n, int32_t c, const double *dgrad, double *dY,
                   double *dupd, double *dgains, double min_gain, double momentum, double lr);
void center_device(tsne_ctx *ctx, int64_t n, int32_t c, double *dY);
// single gradient evaluation (whole problem on this device)
void gradient_device(tsne_ctx *ctx, const int64_t *d_row_ptr, const int32_t *d_col,
                     const double *d_P, int64_t n, const double *dY, int32_t metric,
                     double theta, double exaggeration, double *d_grad, double *h_sumq,
                     double *h_loss);

// "bh.pops" / "bh.child_slots" / "bh.tile_points" / "bh.visits" of the last 2-D
// repulsion_device call with Options::rep_stats; false for other names.
bool repulsion_stat(tsne_ctx *ctx, const std::string &name, int64_t *value_out);
int64_t opt_wave_mhz(tsne_ctx *ctx);   // the last traced 2-D traversal's waves' shader clock (MHz), 0 if none
void repulsion_device(tsne_ctx *ctx, const double *dY, int64_t n, int32_t c, double theta, double *dF,
                      double *dz);
void gradient3_device(tsne_ctx *ctx, const int64_t *d_row_ptr, const int32_t *d_col, const double *d_P, int64_t n,
                      const double *dY, int32_t metric, double theta, double exaggeration, double *d_grad,
                      double *h_sumq, double *h_loss);

void opt_setup(tsne_ctx *ctx, const tsne_params *p, const int64_t *d_row_ptr,
               const int32_t *d_col, const double *d_P, int64_t n, double *dY, double *dupd,
               double *dgains);
void opt_step(tsne_ctx *ctx, int32_t t);
void opt_sync(tsne_ctx *ctx);
int32_t opt_losses(tsne_ctx *ctx, int32_t *keys, double *vals, int32_t cap);
void opt_profile(tsne_ctx *ctx, int enable, double *ms5, int64_t *visits);
double opt_last_z(tsne_ctx *ctx);
int32_t opt_attract_log(tsne_ctx *ctx, int32_t *iters, int32_t *standalone, double *ms, int32_t cap);
void opt_destroy(tsne_ctx *ctx);
int64_t opt_attract_kernel(tsne_ctx *ctx);   // the optimizer's attraction: 0 attract_rows, 1 attract_tiles, 2 attract3,
                                              // 3 attract_tiles3 (-1: none)
BHTree *opt_tree(tsne_ctx *ctx);   // the optimizer's 2-D tree (nullptr without one)

// comm.cpp
void comm_unique_id(uint8_t *out);
void comm_init(tsne_ctx *ctx, int rank, int world, const uint8_t *id);
void comm_destroy(tsne_ctx *ctx);
void comm_init_group(const std::vector<tsne_ctx *> &subs, bool loopback);
void comm_init_callbacks(tsne_ctx *ctx, int rank, int world, const tsne_comm_ops *ops, void *user);
// in place: on rank r, doubles [off[r], off[r+1]) of buf become their sum over the ranks
void comm_reduce_scatterv_f64(tsne_ctx *ctx, double *buf, const int64_t *off_elems);
// the context's communicator: kind (0 none, 1 RCCL, 2 loopback, 3 callbacks) or collectives issued
int64_t comm_counter(const tsne_ctx *ctx, bool calls);
// the loopback group's serial-mode summary (JSON; empty for other transports), then cleared
std::string comm_loop_profile(tsne_ctx *ctx);
void comm_abort(tsne_ctx *ctx);
void comm_release(tsne_ctx *ctx);
void comm_mark(tsne_ctx *ctx, const char *what);   // phase boundary (loopback serial timing)   // end of a rank's group call (loopback serial timing)
// in place: rank r's bytes [off_bytes[r], off_bytes[r+1]) of buf reach every rank
void comm_allgatherv(tsne_ctx *ctx, void *buf, const int64_t *off_bytes);
void comm_allreduce_sum_f64(tsne_ctx *ctx, double *buf, size_t count);
void comm_allreduce_sum_u64(tsne_ctx *ctx, unsigned long long *buf, size_t count);

}  // namespace tsne

// ---------------------------------------------------------------- device helpers
namespace tsne {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// XCD-aware block order: the dispatcher places block b on XCD b % 8, so map
// the blocks of one XCD onto one contiguous 1/8 of [0, nb) -- neighbouring
// work items (Morton-ordered rows / queries) then share that XCD's L2.
constexpr int NUM_XCD = 8;
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
    const int64_t per = nb / NUM_XCD, rem = nb % NUM_XCD;
    const int64_t x = b % NUM_XCD, k = b / NUM_XCD;
    return x * per + (x < rem ? x : rem) + k;
}
// Chunked variant: runs of C consecutive logical blocks go to one XCD and the
// runs rotate over the XCDs (locality within a run, balance across XCDs);
// bijective on [0, nb), identity on the tail that does not fill 8 runs.
__device__ __forceinline__ int64_t xcd_block_chunked(int64_t b, int64_t nb, int64_t C) {
    const int64_t G = (int64_t)NUM_XCD * C, full = (nb / G) * G;
    if (b >= full) return b;
    const int64_t x = b % NUM_XCD, k = b / NUM_XCD;
    return (k / C) * G + x * C + (k % C);
}

template <class T> __device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <class T> __device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        T w = __shfl_xor(v, o, 64);
        v = v > w ? v : w;
    }
    return v;
}

template <class T> __device__ __forceinline__ T wave_min(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        T w = __shfl_xor(v, o, 64);
        v = v < w ? v : w;
    }
    return v;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    const int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Order-preserving map of a double to uint64 (NaN canonicalised, sorts last).
__device__ __forceinline__ uint64_t dkey(double d) {
    uint64_t u = __double_as_longlong(d);
    if (d != d) u = 0x7FF8000000000000ull;
    return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ uint32_t fkey(float f) {
    uint32_t u = __float_as_uint(f);
    if (f != f) return 0xFFFFFFFFu;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
    uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
    return __uint_as_float(u);
}

}  // namespace tsne
