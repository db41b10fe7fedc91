/*
 * tsne_hip.h -- C ABI of libtsne_hip, the MI355X-native hot path of
 * tsne-flink (ChristophAl/tsne-flink): brute-force kNN, perplexity-calibrated
 * affinities, and the Barnes-Hut gradient / optimizer loop.
 *
 * The reference exposes this path as Scala object methods over Flink
 * DataSets (TsneHelpers.scala).  Each entry point below replaces exactly one
 * of them; a JNI shim turns the DataSet partition into the
 * flat arrays used here.  Conventions:
 *   - point ids are dense 0..n-1 (the host mirror remaps arbitrary int ids);
 *   - sparse matrices are CSR: row_ptr[n+1] (int64), col[nnz] (int32),
 *     val[nnz] (double);
 *   - embeddings are row-major n x n_components doubles;
 *   - every call returns a tsne_status; on error tsne_last_error() holds a
 *     thread-local message.  No C++ exception crosses this boundary.
 *   - tsne_* functions take HOST buffers (caller-owned); tsne_dev_* take
 *     DEVICE buffers on the context's device and enqueue on its stream.
 * Numerics are fp64 everywhere except the kNN candidate filter: a bf16x3
 * split-precision MFMA pass (each fp32 coordinate as two bf16 parts, three
 * bf16 products per term, fp32 accumulation) with a rigorous error bound,
 * followed by an exact fp64 re-rank of the survivors.
 */
#ifndef TSNE_HIP_H
#define TSNE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSNE_HIP_ABI_VERSION 2
#define TSNE_UNIQUE_ID_BYTES 128

typedef enum {
    TSNE_OK = 0,
    TSNE_ERR_ARG = -1,          /* IllegalArgumentException in the reference */
    TSNE_ERR_HIP = -2,          /* HIP runtime / kernel launch failure */
    TSNE_ERR_NOMEM = -3,
    TSNE_ERR_UNSUPPORTED = -4,  /* e.g. n_components not 2 or 3 (Cell.scala:32 requires 2) */
    TSNE_ERR_CAPACITY = -5,     /* caller buffer too small; required size reported */
    TSNE_ERR_COMM = -6,         /* RCCL failure */
    TSNE_ERR_NO_DEVICE = -7
} tsne_status;

/* Tsne.getMetric (Tsne.scala:161-168) */
typedef enum {
    TSNE_METRIC_SQEUCLIDEAN = 0,
    TSNE_METRIC_EUCLIDEAN = 1,
    TSNE_METRIC_COSINE = 2
} tsne_metric;

/* Optimizer parameters; defaults = Tsne.scala:47-63 + TsneHelpers.scala:386. */
typedef struct {
    int32_t n_components;       /* --nComponents, 2 (3: octree extension) */
    int32_t metric;             /* --metric, sqeuclidean (used for the attractive q) */
    double learning_rate;       /* --learningRate, 1000 */
    int32_t iterations;         /* --iterations, 300 */
    double early_exaggeration;  /* --earlyExaggeration, 4 */
    double initial_momentum;    /* --initialMomentum, 0.5 */
    double final_momentum;      /* --finalMomentum, 0.8 */
    double theta;               /* --theta, 0.25 */
    double min_gain;            /* hard-coded 0.01 (TsneHelpers.scala:386) */
} tsne_params;

typedef struct tsne_ctx tsne_ctx;

/* ---------------------------------------------------------------- basics */
int tsne_abi_version(void);
const char *tsne_last_error(void);
void tsne_params_default(tsne_params *p);
/* Tsne.getMetric (Tsne.scala:161-168): unknown name -> TSNE_ERR_ARG. */
int tsne_metric_from_name(const char *name, int32_t *metric_out);
/* Host-side CSR from COO triples, for callers that receive a DataSet's
 * triples one at a time (the JNI operator bodies stream a Flink iterator into
 * off-heap arrays: TsneHelpers.scala:162-196's groupBy(0) without JVM arrays,
 * so nothing is bounded by 2^31 elements).  row[e] in [0, n); rows come out
 * in index order, each row's entries in input order (a stable counting sort,
 * the reference's group order).  row_ptr_out: n + 1; col_out / val_out: nnz
 * (val / val_out may be NULL).  No context, no device. */
int tsne_coo_to_csr(const int32_t *row, const int32_t *col, const double *val, int64_t nnz, int64_t n,
                    int64_t *row_ptr_out, int32_t *col_out, double *val_out);
/* Row shard [r0, r1) of rank `rank` out of `world` (contiguous, balanced). */
int tsne_shard_rows(int64_t n, int32_t world, int32_t rank, int64_t *r0, int64_t *r1);
/* Cost-balanced cuts of the Morton-sorted BH queries (the rule the multi-GPU
 * optimizer applies on the device every iteration): bcost[b] = cost of the
 * queries [b*bucket, (b+1)*bucket); bounds[0..world] with bounds[0] = 0,
 * bounds[world] = n and bounds[r] = min(n, (b+1)*bucket) for the first bucket
 * b whose inclusive cost prefix reaches total*r/world (a zero target cuts at
 * 0; all-zero costs cut equal counts). */
int tsne_balance_cuts(const uint64_t *bcost, int64_t nb, int64_t n, int32_t world, int32_t bucket,
                      int64_t *bounds);
/* The same cuts computed by the device kernel (bucket 256) from device
 * buffers; for testing the kernel against tsne_balance_cuts. */
int tsne_dev_balance_cuts(tsne_ctx *ctx, const uint64_t *d_bcost, int64_t n, int32_t world, int64_t *d_bounds);

/* ---------------------------------------------------------------- context */
int tsne_ctx_create(int32_t device, tsne_ctx **out);
/* One caller, several GPUs (SURVEY.md 8b "Threading": a Flink operator at
 * parallelism 1 drives the node).  Creates one rank context per entry of
 * devices[0..ndev) and their communicator: RCCL (ncclCommInitAll, over xGMI)
 * when all devices are distinct, an in-process loopback when all are the same
 * device (ndev ranks sharing one GPU -- executes the multi-GPU code path on a
 * single GPU, for testing).  On the returned handle tsne_knn splits the query
 * rows and tsne_optimize shards the rows of P and the BH queries over the
 * ranks, one host thread per rank, results written to the caller's buffers
 * once; every other host-buffer operator, and the single-device tsne_dev_*
 * calls (kNN, affinities, joint, repulsion), run on the first device.  The
 * device-resident optimizer (tsne_dev_opt_*) holds one rank's state and
 * returns TSNE_ERR_UNSUPPORTED on a handle of ndev > 1: use tsne_optimize
 * there, or one context per rank.  Destroy with tsne_ctx_destroy. */
int tsne_ctx_create_multi(const int32_t *devices, int32_t ndev, tsne_ctx **out);
int tsne_ctx_destroy(tsne_ctx *ctx);
/* Enqueue on a caller-owned hipStream_t (e.g. torch's current stream). NULL = own stream. */
int tsne_ctx_set_stream(tsne_ctx *ctx, void *hip_stream);
void *tsne_ctx_stream(tsne_ctx *ctx);
int tsne_ctx_synchronize(tsne_ctx *ctx);
/* Per-handle tunables (no reference counterpart: the reference has no BH
 * shortcuts).  The defaults are the library's choices; a setting applies to
 * every later call on this handle (every rank of a tsne_ctx_create_multi
 * handle), never to other handles or threads.  Keys:
 *   "near_tol_early" 1e-6, "near_tol_late" 5e-6   near-exact BH subtrees:
 *       relative bound per summarised cell, for single gradients and the
 *       optimizer's early-exaggeration phase / after it (0: the test is off);
 *   "mom_tol" 1e-12           subtree-moment truncation bound (2-D);
 *   "near_tol3_early" 1e-7, "near_tol3_late" 5e-6, "mom3_tol" 1e-12, and
 *   "oct_moments" 1           the same for the 3-D octree;
 *   "oct_records" 2           3-D: octal records and the 64-query record
 *                             traversal (1: the 8-query one; 0: the
 *                             binary-node walk);
 *   "oct_layout_switch" 6     3-D with oct_records 2: the 8-query layout
 *                             while the octree's root half-width is below
 *                             this x the near-exact radius (0: never);
 *   "coherent_sort" 1         the trees' Morton sort from the previous build's
 *                             order (0: rocPRIM's radix sort; the same
 *                             permutation);
 *   "root_tile" 1             root-tile shortcut of the small-embedding phase;
 *   "attract_tiles" 1         tiled attraction where the labels allow it;
 *   "attract_tiles3" 0        3-D: the tiled attraction too (slower than the
 *                             row kernel beside the octree traversal at C4);
 *   "attract_cfg" -1          its tile shape (-1 automatic, 0..3);
 *   "attract_pipe" 0          2-D tiled attraction: 0 attract_tiles; 1..5 the
 *                             pipelined kernel (entries of the next 1 or 2
 *                             slices in flight; identical results);
 *   "attract_dyn" 1           attract_tiles: the waves claim a tile's slices
 *                             instead of taking every 16th (non-loss launches;
 *                             identical results);
 *   "graph_order" 1           P's graph order as the initial labels;
 *   "relabel" -1              Morton relabels: -1 automatic, 0 never, 1 by
 *                             locality score, 2 always;
 *   "recut" 0                 several ranks on the tiled layout: re-cut the
 *                             row ownership by BH cost instead of relabels;
 *   "knn_bf16" 1              kNN threshold filter on bf16x3 MFMA (0: the
 *                             f32-input MFMA; results are identical);
 *   "narrow" 3                BH: 64-query groups costing >= this x the mean
 *                             run in the narrow layout (0: off).  The
 *                             selection reads the previous traversal's costs:
 *                             the optimizer's previous iteration, and for the
 *                             single-call operators only with
 *   "spill" 0, "spill_task" 0.25, "spill_min" 256, "spill_force" 0,
 *   "spill_drains" 2          BH work splitting (2-D): a walk past spill x the
 *                             previous traversal's mean cost (>= spill_min
 *                             record pops; spill_force: a fixed budget) hands
 *                             the rest of its stack to task lists that
 *                             spill_drains follow-up launches take, splitting
 *                             again past spill_task x that budget; the sums are
 *                             deterministic, equal to the unsplit walk to
 *                             rounding (0: off, the default: slower at C3);
 *   "tile_stream" 0, "tile_stream_max" 0, "tile_stream_frac" 1,
 *   "tile_stream_wait" 48, "tile_stream_gate" 1, "trav_prio" 0
 *                             BH tile streaming (2-D, one rank): tile_stream
 *                             workgroups per CU (<= 8), on a stream of their
 *                             own and (gate 1) dispatched once every traversal
 *                             block has started, sum the finished traversal
 *                             waves' tile lists of cost (points + 16 per task)
 *                             <= tile_stream_max (0: tile_stream_frac x the
 *                             previous tile plan's chunk unit) while the
 *                             traversal's last waves run, leaving after
 *                             tile_stream_wait polls (~0.4 us each) without a
 *                             list; the slot path sums the rest.  Deterministic;
 *                             tile_stream_max <= 4095: the bits of 0 (off, the
 *                             default: measured slower at C3).
 *                             trav_prio 1-3: the 64-query traversal's waves at
 *                             that issue priority (no measured effect);
 *   "trav_front" 0             > 0: the 64-query traversal's workgroups whose
 *                             heaviest wave cost >= this x the previous
 *                             traversal's mean are dispatched first (the order
 *                             is made with the narrow selection; same sums; no
 *                             measured gain);
 *   "trav_front_cur" 0         > 0: as trav_front with the order predicted from
 *                             each point's previous cost through the current
 *                             Morton order (made during the build; slower);
 *   "attract_serial_t0" 0, "attract_serial_t1" -1
 *                             2-D optimizer: for t in [t0, t1] the attraction
 *                             runs after the BH kernels instead of beside them
 *                             (an A/B of the overlap; slower);
 *   "wave_log" 0               with "rep_stats": the counting call logs every
 *                             BH wave's start and end (tsne_debug_wave_log);
 *   "bh_split" 0              several ranks (2-D), 1: partition the Barnes-Hut
 *                             tree by ranges of its sorted points -- every rank
 *                             walks every query over the cells holding its own
 *                             points, each term taken by one rank, and the
 *                             forces are summed by a reduce-scatter to the row
 *                             owners (0: partition the queries, Z-only exchange);
 *   "bu_acqrel" 1             the tree build's cross-workgroup bottom-up
 *                             hand-off uses agent-scope acquire-release
 *                             arrivals (the HIP memory model's ordering); 0:
 *                             relaxed arrivals ordered by gfx950's in-order
 *                             issue (the same trees; no measurable cost
 *                             difference);
 *   "loop_serial" 0           1 (a loopback tsne_ctx_create_multi group, set
 *                             before tsne_optimize): the ranks take turns on the
 *                             device and log their work between collectives --
 *                             a one-GPU projection of N GPUs, read with
 *                             tsne_ctx_loop_profile;
 *   "comm_world1" 0           1: tsne_ctx_init_comm / tsne_ctx_init_comm_callbacks
 *                             at world 1 still create the communicator (RCCL:
 *                             a one-rank ncclCommInitRankConfig, id may be
 *                             NULL), and the optimizer runs its sharded path
 *                             through it -- the transport's own test;
 *   "rep_stats" 0             1: tsne_repulsion / tsne_dev_repulsion (2-D) run
 *                             the traversal's counting variant, read with the
 *                             "bh.*" counters below (diagnostics; the same sums);
 *   "reuse_costs" 0           1: tsne_gradient / tsne_repulsion select from the
 *                             previous call's costs (results then depend on
 *                             the call history at rounding level; 0 keeps
 *                             every single call a function of its input).
 * Unknown keys and out-of-range values return TSNE_ERR_ARG. */
int tsne_ctx_set_option(tsne_ctx *ctx, const char *key, double value);
/* HIP runtime versions (HIP_VERSION encoding, major * 10^7 + minor * 10^5 +
 * patch): the headers this library was built with, and the runtime the
 * process loaded (e.g. a host framework's bundled libamdhip64).  The
 * bindings refuse a different major version.  No device needed. */
int tsne_hip_versions(int32_t *built_out, int32_t *runtime_out);
int tsne_ctx_get_option(tsne_ctx *ctx, const char *key, double *value_out);
/* The loopback group's "loop_serial" summary (JSON: the span of the ranks'
 * work between collectives, per collective and per 100 occurrences) of the
 * segments logged since the last read; *len_out = its length (buf may be NULL
 * to ask: the summary is then kept for the next call, which copies it out), at
 * most cap - 1 bytes + NUL written.  Empty for other handles. */
int tsne_ctx_loop_profile(tsne_ctx *ctx, char *buf, int64_t cap, int64_t *len_out);
/* Diagnostic counters of the last call (synchronises the context's stream):
 *   "bh.narrow_groups"   64-query groups the last single-call BH traversal
 *                        (tsne_gradient / tsne_repulsion) ran in the narrow layout;
 *   "opt.narrow_groups"  the same for the optimizer's last iteration;
 *   "bh.pops", "bh.child_slots", "bh.tile_points", "bh.visits"  with option
 *                        "rep_stats": the last 2-D single-call repulsion's
 *                        traversal stack pops (wave level), child slots
 *                        evaluated (wave level), tile points, and
 *                        reference-equivalent node evaluations;
 *   "bh.wave_ticks_max", "bh.wave_ticks_sum", "bh.span_ticks"  (rep_stats) the
 *                        traversal waves' longest and summed run time and
 *                        the grid's span, in 100 MHz ticks (both layouts);
 *   "bh.tile_ticks_max", "bh.tile_ticks_sum", "bh.tile_span_ticks"  (rep_stats)
 *                        the same for tile_apply's waves;
 *   "bh.dense_pairs", "bh.moment_evals", "bh.tile_steps0".."bh.tile_steps3",
 *   "bh.tile_pairs0".."bh.tile_pairs3"  (rep_stats) exact-sum work: pair terms,
 *                        moment evaluations, and per dense path of tile_apply
 *                        (lane-wise, packed, query-major, staged sweep) the
 *                        wave steps issued and the useful lane pairs;
 *   "comm.kind"          the context's communicator: 0 none, 1 RCCL, 2 loopback,
 *                        3 caller callbacks; "comm.calls" collectives it issued;
 *   "opt.attract_kernel" the optimizer's attraction kernel: 0 attract_rows,
 *                        1 attract_tiles, 2 attract3 (3-D), 3 attract_tiles3
 *                        (3-D, tiled), -1 no optimizer;
 *   "opt.csort_oversized_total"  the same summed over every build of the optimizer's tree;
 *   "bh.csort_oversized", "opt.csort_oversized"  buckets of the last coherent
 *                        Morton sort (csort.hpp) beyond its LDS capacity;
 *   "bh.spill_tasks", "opt.spill_tasks"  BH walks split off as tasks (option
 *                        "spill"), summed over every traversal of the tree;
 *   "bh.spill_flags", "opt.spill_flags"  1 a task list full, 2 task tile pages
 *                        exhausted (those walks went on unsplit / untiled: the
 *                        same sums, but their split points then depend on timing);
 *   "bh.stream_lists", "opt.stream_lists"  tile lists the streaming consumers
 *                        summed (option "tile_stream"), over every traversal. */
int tsne_ctx_counter(tsne_ctx *ctx, const char *name, int64_t *value_out);

/* Diagnostics (option "wave_log" with "rep_stats"): the last counting
 * repulsion call's BH waves as (start, end << 2 | kind) pairs in 100 MHz wall
 * ticks, kind 0 64-query traversal, 1 narrow, 2 tile_apply; up to cap pairs
 * copied to out, *count = the pairs logged (<= 2^17). */
int tsne_debug_wave_log(tsne_ctx *ctx, uint64_t *out, int64_t cap, int64_t *count);

/* Multi-GPU, one process per GPU over RCCL.  Rank 0 calls
 * tsne_comm_unique_id and ships the bytes to the other ranks out of band
 * (torch.distributed / MPI / a file); every rank then calls
 * tsne_ctx_init_comm.  Afterwards tsne_optimize / tsne_dev_opt_* shard the
 * rows of P and the BH queries (each rank owns a range of internal labels,
 * re-cut by measured BH cost when the labels are renumbered); per iteration
 * only the updated embedding slices (all-gather) and Z (all-reduce) cross
 * ranks.  Results are replicated on every rank.  (tsne_knn takes explicit
 * query ranges per rank.) */
int tsne_comm_unique_id(uint8_t id_out[TSNE_UNIQUE_ID_BYTES]);
int tsne_ctx_init_comm(tsne_ctx *ctx, int32_t rank, int32_t world,
                       const uint8_t id[TSNE_UNIQUE_ID_BYTES]);
int tsne_ctx_rank(tsne_ctx *ctx, int32_t *rank, int32_t *world);

/* Collectives supplied by the host dataflow instead of RCCL (e.g. carried by
 * the JVM's own network stack across nodes, or torch.distributed in tests).
 * Each operates in place on a HOST buffer and returns 0 on success; every
 * rank calls them in the same order.  allgatherv: rank r's bytes
 * [off[r], off[r+1]) of buf (off has world + 1 entries) must reach every
 * rank's buf. */
typedef struct {
    int (*allreduce_sum_f64)(void *user, double *buf, int64_t count);
    int (*allreduce_sum_u64)(void *user, uint64_t *buf, int64_t count);
    int (*allgatherv)(void *user, void *buf, const int64_t *off);
} tsne_comm_ops;
int tsne_ctx_init_comm_callbacks(tsne_ctx *ctx, int32_t rank, int32_t world, const tsne_comm_ops *ops,
                                 void *user);

/* ------------------------------------------------- host-buffer operators */

/* kNearestNeighbors (TsneHelpers.scala:41-59).  X: n x d row-major.
 * For query rows [q0, q1): the kk = min(k, n-1) nearest j != i, ascending by
 * (metric value, j).  idx_out / dist_out: (q1-q0) x kk.  Distances are the
 * exact fp64 breeze metric values (sequential sums). */
int tsne_knn(tsne_ctx *ctx, const double *X, int64_t n, int32_t d, int32_t metric,
             int32_t k, int64_t q0, int64_t q1, int32_t *idx_out, double *dist_out);

/* projectKnn (TsneHelpers.scala:93-160, ZOrder.scala:25-42; --knnMethod
 * project): candidates = the k Z-order neighbours on either side of each
 * point in the input and in `iterations - 1` shifted copies x + r_s (shifts:
 * (iterations-1) x d, uniform [0,1) vectors supplied by the caller -- the
 * reference draws them unseeded), ranked by the exact fp64 metric; idx_out /
 * dist_out: n x min(k, n-1), ascending by (distance, j).  The Z-order
 * comparator is the reference's (signed XOR of the raw bit patterns) and is a
 * total order for nonnegative inputs.  2*k*iterations <= 1024. */
int tsne_project_knn(tsne_ctx *ctx, const double *X, int64_t n, int32_t d, int32_t metric, int32_t k,
                     int32_t iterations, const double *shifts, int32_t *idx_out, double *dist_out);
/* pairwiseAffinities (TsneHelpers.scala:162-180 + 434-504): per CSR row the
 * beta binary search to entropy ln(perplexity); p_out has the layout of dist. */
int tsne_pairwise_affinities(tsne_ctx *ctx, const int64_t *row_ptr, const double *dist,
                             int64_t nrows, double perplexity, double *p_out);

/* jointDistribution (TsneHelpers.scala:182-196): P = (C + C^T) / sum over the
 * union pattern (explicit zeros kept); output rows sorted by column.  If
 * cap < nnz returns TSNE_ERR_CAPACITY with *nnz_out set (cap = 2*nnz_in
 * always suffices). */
int tsne_joint_distribution(tsne_ctx *ctx, const int64_t *row_ptr, const int32_t *col,
                            const double *p, int64_t n, int64_t cap, int64_t *out_row_ptr,
                            int32_t *out_col, double *out_val, int64_t *nnz_out);

/* gradient (TsneHelpers.scala:221-318): Barnes-Hut with the reference
 * quadtree semantics and opening criterion.  P values are multiplied by
 * `exaggeration`.  Y, grad_out: n x 2.  sumq_out (Z) and loss_out (KL term
 * of TsneHelpers.scala:297-299) are optional (NULL). */
int tsne_gradient(tsne_ctx *ctx, const int64_t *row_ptr, const int32_t *col, const double *P,
                  int64_t n, const double *Y, int32_t metric, double theta, double exaggeration,
                  double *grad_out, double *sumq_out, double *loss_out);

/* gradient for c = 2 (== tsne_gradient) or c = 3: the 3-D octree extension
 * (the reference itself requires 2-D, Cell.scala:32): root
 * Cell(0,0,0,W) with W = max(dX, dY, dZ), 8 children (upper/lower x NW, NE,
 * SW, SE), the same max(h)/D < theta criterion on squared 3-D distances.
 * Y, grad_out: n x c.  Other c -> TSNE_ERR_UNSUPPORTED. */
int tsne_gradient_c(tsne_ctx *ctx, const int64_t *row_ptr, const int32_t *col, const double *P, int64_t n,
                    int32_t c, const double *Y, int32_t metric, double theta, double exaggeration,
                    double *grad_out, double *sumq_out, double *loss_out);
/* QuadTree.computeRepulsiveForce (QuadTree.scala:123-152; tree built as in
 * TsneHelpers.scala:227-256) for every point: F_out (n x c, the repulsive
 * force sum before the 1/Z normalisation) and z_out (n, the point's sumQ
 * contribution; Z = their sum, TsneHelpers.scala:266), original order.
 * c = 2, or 3 for the octree extension. */
int tsne_repulsion(tsne_ctx *ctx, const double *Y, int64_t n, int32_t c, double theta, double *F_out,
                   double *z_out);

/* updateEmbedding (TsneHelpers.scala:341-369), in place on Y, upd, gains. */
int tsne_update_embedding(tsne_ctx *ctx, int64_t n, int32_t c, const double *grad, double *Y,
                          double *upd, double *gains, double min_gain, double momentum,
                          double learning_rate);

/* centerEmbedding (TsneHelpers.scala:320-329), in place. */
int tsne_center_embedding(tsne_ctx *ctx, int64_t n, int32_t c, double *Y);

/* initWorkingSet (TsneHelpers.scala:198-219): Y ~ N(0, 1e-4^2) from a
 * counter-based generator keyed by `seed` (the reference ignores
 * --randomState; this build honours it), upd = 0, gains = 1. */
int tsne_init_working_set(tsne_ctx *ctx, int64_t n, int32_t c, uint64_t seed, double *Y,
                          double *upd, double *gains);

/* optimize (TsneHelpers.scala:396-430): all iterations on the device; Y,
 * upd and gains (n x n_components, 2 or 3) are read and written back.  loss_keys / loss_vals
 * receive (t, KL) for every t % 10 == 0 (the "loss" accumulator,
 * TsneHelpers.scala:297-300), at most loss_cap entries. */
int tsne_optimize(tsne_ctx *ctx, const tsne_params *params, const int64_t *row_ptr,
                  const int32_t *col, const double *P, int64_t n, double *Y, double *upd,
                  double *gains, int32_t *loss_keys, double *loss_vals, int32_t loss_cap,
                  int32_t *n_loss);

/* ----------------------------------------------------- device-buffer API */
/* Same operators, pointers on the context's device, enqueued on its stream.
 * They do not synchronise unless a result size must reach the host. */
int tsne_dev_knn(tsne_ctx *ctx, const double *dX, int64_t n, int32_t d, int32_t metric,
                 int32_t k, int64_t q0, int64_t q1, int32_t *d_idx, double *d_dist);
int tsne_dev_project_knn(tsne_ctx *ctx, const double *dX, int64_t n, int32_t d, int32_t metric, int32_t k,
                         int32_t iterations, const double *d_shifts, int32_t *d_idx, double *d_dist);
int tsne_dev_repulsion(tsne_ctx *ctx, const double *dY, int64_t n, int32_t c, double theta, double *d_F,
                       double *d_z);
int tsne_dev_pairwise_affinities(tsne_ctx *ctx, const int64_t *d_row_ptr, const double *d_dist,
                                 int64_t nrows, double perplexity, double *d_p);
/* Fixed-k conditional rows (row i = entries [i*k, (i+1)*k)), symmetrised into
 * caller-allocated CSR (capacity 2*n*k); *nnz_out is synchronised to host. */
int tsne_dev_joint_distribution(tsne_ctx *ctx, const int64_t *d_row_ptr, const int32_t *d_col,
                                const double *d_p, int64_t n, int64_t cap, int64_t *d_out_row_ptr,
                                int32_t *d_out_col, double *d_out_val, int64_t *nnz_out);

/* Device-resident optimizer.  setup copies the FULL P (every rank holds it;
 * rank r computes the rows of its range of the optimizer's internal point
 * labels) and the working set (Y, upd, gains: n x n_components, original
 * point order) into its own state and allocates the workspace; step runs
 * global iteration t (1-based) with the reference phase schedule; sync
 * writes the working set back to the caller's Y, upd and gains (original
 * order; with several ranks a collective call).  The caller's buffers are
 * not touched by a step (round 5: the per-step scatter of Y was a third of
 * the update's HBM traffic).  Losses for t % 10 == 0 stay on the device
 * and are read by tsne_dev_opt_losses.  Internal labels (2-D): P's graph
 * order at setup (connected components, BFS level), then every 25
 * iterations the Morton order of the embedding when it keeps more of P's
 * edges local -- cache locality of the CSR attraction's gathers; results do
 * not depend on the labelling beyond summation order.  n_components = 3 runs
 * the octree extension (see tsne_gradient_c). */
int tsne_dev_opt_setup(tsne_ctx *ctx, const tsne_params *params, const int64_t *d_row_ptr,
                       const int32_t *d_col, const double *d_P, int64_t n, double *d_Y,
                       double *d_upd, double *d_gains);
int tsne_dev_opt_step(tsne_ctx *ctx, int32_t t);
int tsne_dev_opt_sync(tsne_ctx *ctx);
int tsne_dev_opt_losses(tsne_ctx *ctx, int32_t *loss_keys, double *loss_vals, int32_t cap,
                        int32_t *n_loss);
/* The Z normaliser (sum of the BH sumQ over all points, TsneHelpers.scala:266)
 * of the last tsne_dev_opt_step: the value its gradient and loss used.
 * Synchronises the context stream. */
int tsne_dev_opt_last_z(tsne_ctx *ctx, double *z_out);
/* Per-stage timing of the last step (HIP events on the ctx stream), in ms:
 * [0] tree build, [1] BH repulsion (traversal + tile and moment kernels),
 * [2] Z reduce (+ its all-reduce with several ranks), [3] attraction kernel
 * (attract_tiles / attract_rows, timed on the stream it runs on -- a side
 * stream when it overlaps [0]-[2]), [4] wait for it, combine + update, loss,
 * embedding exchange, centring.
 * Also BH work counters of the last step (counters_out5, may be NULL):
 * [0] reference-equivalent node evaluations (lane visits; a leaf tile of m
 * points counts m), [1] subtree-moment evaluations, [2] dense pair terms,
 * [3] wave-level cell pops, [4] wave-level tile points, [5] lane child
 * evaluations, [6] wave child slots (lane utilisation = [5] / (64 * [6])),
 * [7] heaviest wave (its pops + tile points / 16), [8] most pops of a
 * wave, [9] most tile points of a wave.
 * enable: 1 on, 0 off, -1 leave unchanged. */
int tsne_dev_opt_profile(tsne_ctx *ctx, int32_t enable, double *ms_out5, int64_t *counters_out10);
/* Kernel time of every attraction launch since tsne_dev_opt_setup (HIP
 * events on the stream it ran on): its iteration t, a placement code
 * (0 non-loss launch on the side stream, concurrent with the tree build / BH
 * traversal; 1 loss launch alone on the context stream after Z; 2 loss launch
 * on the side stream with Z-free KL terms; 3 non-loss launch alone on the
 * context stream), ms.  Synchronises on the recorded events; *count = number
 * of launches kept (the last 16384; entries beyond cap are not written). */
int tsne_dev_opt_attract_log(tsne_ctx *ctx, int32_t *iters, int32_t *standalone, double *ms, int32_t cap,
                             int32_t *count);
/* Stage timers of the context (HIP events around the stage's kernels, on
 * their stream), in ms per interval since the stage was last reset:
 * "knn.filter" (the fp32-MFMA distance filter launches of the last kNN call),
 * "opt.attract" (see above), "opt.update" (combine + updateEmbedding +
 * centerEmbedding + write-back, per iteration).  *count = intervals. */
int tsne_ctx_stage_ms(tsne_ctx *ctx, const char *stage, double *ms_out, int32_t cap, int32_t *count);

#ifdef __cplusplus
}
#endif
#endif /* TSNE_HIP_H */
