// bhtree.hpp -- GPU Barnes-Hut quadtree with the reference's semantics.
#pragma once
#include "common.hpp"
#include "csort.hpp"

namespace tsne {

// A leaf tile of one traversal wave: the subtree (node, leaf range) whose
// exact leaf sum the lanes of `mask` take (by moments or densely, tile_apply).
constexpr int TILE_CAP = 8192;   // tiles per wave; beyond, lanes keep traversing
struct TileTask {
    int32_t ref, first, last, pad;
    uint64_t mask;
};

// Internal node of the binary radix tree over sorted Morton keys.  A node
// whose common prefix ends inside a quad level is "transparent" (h == 0:
// always opened); otherwise it IS the reference quadtree cell of half width
// h = W / 2^level (QuadTree.scala subDivide halves hWidth per level).
struct __attribute__((aligned(16))) BHNode {
    double cx, cy;    // centre of mass (sum / count)
    double h;         // half width of the quad cell, 0 = transparent
    double hmin;      // min h over the real internal nodes of this subtree (+inf if none)
    double bx0, bx1, by0, by1;  // bounding box of the subtree's points
    int32_t cnt;      // cumSize
    int32_t left;     // child refs: >= 0 internal node, < 0 leaf ~ref
    int32_t right;
    int32_t delta;    // common-prefix length in bits (62+ = key tie)
    int32_t first, last;  // leaf range [first, last] in sorted order
    double rball;     // all-open ball radius around (cx, cy), see bottom_up
};

// Quad-collapsed record of a real node (a reference quadtree cell): its own
// tile-test data plus the summaries of its <= 4 quad children (found by
// descending through transparent binary nodes), so that the traversal
// evaluates all children of an opened cell from one record load and pushes
// only children that some lane opens.  Child kinds (ch): >= 0 real cell of
// half width ch (cref = node id); QCH_LEAF one point (cref = ~sorted index,
// com = the point); QCH_TIE a key-tie group (cref = node id, all points
// interact directly).
constexpr double QCH_LEAF = -1.0;
constexpr double QCH_TIE = -2.0;
constexpr double QCH_MULTI = -3.0;   // a leaf holding ccnt copies of one point (reference multiplicity)
constexpr int32_t QNCH_TILE = 0x100;   // nch flag: an all-open tile test can pass here
// nch bits 16 + 2c: child c's kind, wave-uniform in the traversal (scalar
// branches instead of per-lane compares of ch[c])
constexpr int QNCH_KIND = 16;
constexpr int QK_CELL = 0, QK_LEAF = 1, QK_TIE = 2, QK_MULTI = 3;
struct __attribute__((aligned(16))) QRec {
    double cx, cy;              // centre of mass
    double rball, hmin;         // all-open tests, precomputed (build_qrec): rball^2 (1 - 1e-9) and
                                // max(hmin / theta (1 - 1e-12), near_dmax) (1 - 1.1e-12) (see bottom_up)
    double bx0, bx1, by0, by1;  // bounding box of the subtree's points
    int32_t first, last;        // leaf range in sorted order
    int32_t cnt, nch;           // cumSize, number of quad children | QNCH_TILE
    double ccx[4], ccy[4];
    double cb[4];               // cells: the sure-open bound on 1 + D (see QACC_BAND)
    double ca[4];               // cells: the sure-accept bound on 1 + D
    int32_t cref[4], ccnt[4];
    double ex;                  // the box test's rounding margin, record part: 1e-15 (|bx0| + |bx1| + |by0| + |by1|)
    uint64_t lmask;             // 0 in HBM; the LDS copy of a popped record: its stack entry's lane mask
};
// A cell child is tested on D1 = fma(dx, dx, fma(dy, dy, 1)) ~ 1 + D, the
// denominator its term needs anyway (one fp64 add per child fewer than
// testing D and forming 1 + D apart).  It is summarised for sure when
// D1 > ca, opened for sure when D1 < cb, with
//   ca = (1 + ch / theta (1 + 2.5e-14)) (1 + 1e-15)  (rounded: > the bound),
//   cb = (1 + ch / theta (1 - 2.5e-14)) (1 - 1e-15)  (rounded: < the bound);
// the 1e-15 factors cover D1's two roundings (<= 2^-52 relative), the
// 2.5e-14 ones the distance between the reference's D and the exact one and
// the quotient's rounding.  In between, the exact IEEE quotient ch / D < theta
// decides (the reference's test, QuadTree.scala:134), with ch read from the
// node (qrec_child_h: rare, so the record does not carry it).
constexpr double QACC_MARGIN = 2.5e-14;
constexpr double QACC_BAND = (1.0 - QACC_MARGIN) / (1.0 + QACC_MARGIN);
__host__ __device__ inline double qacc_accept(double ch, double inv_theta) {
    return (1.0 + ch * inv_theta * (1.0 + QACC_MARGIN)) * (1.0 + 1e-15);
}
__host__ __device__ inline double qacc_open(double ch, double inv_theta) {
    return (1.0 + ch * inv_theta * (1.0 - QACC_MARGIN)) * (1.0 - 1e-15);
}

// counters of the BH kernels' STATS blocks (visits arrays: bh_traverse,
// tile_apply; repulsion_stat names them)
constexpr int VIS_N = 48;

struct BHTree {
    int64_t n = 0;           // points (queries)
    // device arrays (ctx workspace)
    uint64_t *keys = nullptr, *keys_sorted = nullptr;
    int32_t *idx = nullptr, *idx_sorted = nullptr;  // sorted position -> original row
    int32_t *inv = nullptr;                         // original row -> sorted position
    int32_t *dupc = nullptr;                        // exact duplicates of each sorted point (incl. itself)
    // exact-duplicate multiplicities of the reference (QuadTree.scala:52-61):
    // dflag[0] = some point has a duplicate; per binary node: first inserted
    // row, its value id, the row at which a second distinct value arrived
    // (t2: when the reference cell splits); count / sum corrections of real
    // cells, the leaf multiplicity of a pure duplicate group's tie node,
    // and a no-tile mark on the cells above such a group
    int32_t *dflag = nullptr, *vid = nullptr, *rmin = nullptr, *rvid = nullptr, *rt2 = nullptr, *arrive2 = nullptr;
    int32_t *cntcorr = nullptr, *tiecnt = nullptr, *notile = nullptr;
    double *sumcorr = nullptr;
    // a reference cell chain C_1 > ... > C_k (same points, one binary node)
    // whose top cell counts different duplicate copies than the rest: a
    // virtual record (qrec[n + node]) for C_1 with its own count / centre
    int32_t *vflag = nullptr, *vcnt = nullptr, *vcntf = nullptr;
    double *vsum = nullptr, *vcom = nullptr;
    const int32_t *rowmap = nullptr;                // label -> insertion row (nullable: identity)
    double2 *pos = nullptr;                         // sorted positions (leaves + queries)
    BHNode *nodes = nullptr;
    QRec *qrec = nullptr;       // per binary node id, valid for real nodes; [n, 2n): virtual chain tops
    double *agg = nullptr;      // per-node bottom-up aggregates (AGG doubles)
    int32_t *parent_leaf = nullptr, *parent_node = nullptr;
    int32_t *arrive = nullptr;
    // two-phase bottom-up (bottom_up_intra / bottom_up_top): frontier-subtree
    // start marks (= gen of the build that set them), phase-2 arrival list
    int32_t *fstart = nullptr, *top_list = nullptr, *top_cnt = nullptr;
    int32_t gen = 0;
    int rt_skip = 0;            // builds left before the root-tile test is tried again
    double near_dmax = 0.0;     // this build's near-exact radius (squared distance), bh_near_dmax
    int32_t *meta = nullptr;    // [0] = m (in-root points), [1] = root ref, [2] = moment nodes
    // subtree moments (see bhtree.hip "Subtree moments"): per internal node
    // MOM_K scaled moments about its bounding-box centre, for nodes of
    // >= MOM_MIN_POINTS points; built in chunks of MOM_CHUNK points.
    double *mom = nullptr;       // n x MOM_K
    double *mom_part = nullptr;  // item x MOM_K partial sums
    int32_t *mom_cnt = nullptr, *mom_off = nullptr;  // chunks per node, exclusive scan (n + 1)
    int32_t *mom_list = nullptr;                     // nodes that carry moments
    int32_t *mom_item = nullptr;                     // item -> node
    int32_t *mom_flag = nullptr;                     // [0] moments built, [1] eligible tiles seen,
                                                     // [2] tiles needed to build them (n / 64 + 1)
    int32_t *mtask = nullptr, *mtask_n = nullptr;    // per query: moment evaluations (node ids), count
    TileTask *ttask = nullptr;                       // per traversal wave: tile list
    int32_t *ttask_n = nullptr;
    int64_t tile_waves = 0;
    int64_t mom_items_cap = 0;
    void *scan_tmp = nullptr;
    size_t scan_tmp_bytes = 0;
    double *bbox_part = nullptr, *W = nullptr;
    double *bb = nullptr;        // bounding box of all points: x0, x1, y0, y1
    int32_t *status = nullptr;   // [0] root-tile mode possible (see bh_root_tile)
    int32_t *status_h = nullptr; // pinned host copy
    bool root_tile = false;      // this build took the root-tile path (no sort: slots = labels)
    const double2 *root_pos = nullptr;   // root-tile mode: the points in label order
    double *rcoef = nullptr;             // root-tile mode: the root's sums as polynomials in v (POLY_K)
    int32_t *dup_tab = nullptr;          // root-tile duplicate check: 4n-slot table
    uint8_t *dup_open = nullptr;         // ... per point: still unresolved
    uint64_t dup_mask = 0;
    void *sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    CoherentSort cs;             // the Morton sort from the previous build's order (csort.hpp)
    bool cs_primed = false;      // idx_sorted holds a previous build's permutation
    int bbox_blocks = 0;
    // longest-first block order of the traversal (by each wave's pops + tile
    // points in the previous traversal) and of tile_apply (by this
    // traversal's tile points): heavy waves start first instead of forming
    // a low-occupancy tail
    int32_t *wcost = nullptr, *tcost = nullptr;    // per wave
    int32_t *okey = nullptr, *okey2 = nullptr, *oval = nullptr;   // per block: sort scratch
    int32_t *border = nullptr, *torder = nullptr;  // per block: traversal / tile_apply order
    void *osort_tmp = nullptr;
    size_t osort_tmp_bytes = 0;
    // tile chunks (bhtree.hip ChunkView): chunks per traversal wave, first
    // chunk slot (waves + 1), slot -> wave and chunk | C << 16, slot costs,
    // slot count; partial sums per chunk slot lane
    int32_t *ch_C = nullptr, *ch_slot0 = nullptr, *ch_slot_w = nullptr, *ch_slot_c = nullptr;
    int32_t *ch_scost = nullptr, *ch_nslots = nullptr;
    unsigned long long *ch_total = nullptr;
    double2 *ch_Fp = nullptr;
    double *ch_Zp = nullptr;
    void *ch_scan_tmp = nullptr;
    size_t ch_scan_bytes = 0;
    // narrow layout of heavy 64-query groups (bhtree.hip "Narrow layout"):
    // per group its heavy slot + 1 (or 0), the heavy list and count, per
    // narrow wave its cost, per narrow query its moment tasks
    int32_t *nflag = nullptr, *hlist = nullptr, *hcount = nullptr, *ncost = nullptr;
    int32_t *hran = nullptr;     // heavy groups the last traversal ran narrow
    int32_t *nmtask = nullptr, *nmtask_n = nullptr;
    int64_t nar_hmax = 0;
    int64_t sel_waves = 0;       // query waves the current selection is for (0: none)
    bool ran_narrow = false;     // the last traversal used a selection
    // work splitting of long traversals (bhtree.hip "Spill"): a walk past its
    // pop budget hands its stack entries to the next level's task list, taken
    // by drain launches; task sums go to per-query fixed-point accumulators
    // (order-free, so the result does not depend on which wave ran which task)
    int32_t *sp_ctl = nullptr;            // control words (levels' heads and tails, pages, budgets, flags)
    int4 *sp_task = nullptr;              // per level: task -> {group, first entry, entries}
    uint4 *sp_ent = nullptr;              // per level: stack entry -> {ref, 0, mask lo, mask hi}
    int32_t *sp_gflag = nullptr;          // per 64-query group: generation of its last spill
    unsigned long long *sp_acc = nullptr; // per sorted position: fx, fy, z as (lo, hi) pairs
    TileTask *sp_pg_tiles = nullptr;      // task tile pages (64 tiles each)
    int32_t *sp_pg_grp = nullptr, *sp_pg_n = nullptr;
    int32_t sp_cap = 0, sp_pg_cap = 0;
    int32_t sp_gen = 0;
    int64_t sp_waves = 0;                 // query waves the budget words are for (0: none yet)
    bool ran_spill = false;               // the last traversal split work
    // tile streaming (option tile_stream; bhtree.hip "Tile streaming")
    int32_t *st_ctl = nullptr;            // ST_* control words (zero between calls), then the items
    double2 *st_Dp = nullptr;             // per item x 64: the consumers' dense sums (F part)
    double *st_Dz = nullptr;              // per item x 64: (z part)
    int32_t *st_mtask = nullptr, *st_mtask_n = nullptr;   // per item x 64: moment lists
    int32_t st_gen = 0;
    size_t st_words = 0;
    int32_t *trav_order = nullptr;        // option trav_front: the next traversal's workgroup order
    int64_t front_waves = 0;              // query waves that order is for (0: none)
    // option trav_front_cur: per point (Y row) the previous traversal's wave
    // cost, per new wave its prediction, the order event
    int32_t *pcost = nullptr, *pred = nullptr;
    bool pcost_valid = false, order_ready = false;
    hipEvent_t ord_ev = nullptr;
    bool ran_stream = false;              // the last traversal streamed its lists
    std::string pre;                      // the workspace prefix of this tree's buffers
};

// Allocate (from ctx->ws, buffers named pre + field) for n points.  One
// prefix per tree that must persist alongside another (the optimizer's "bh.",
// the single-call operators' "bh1.").
void bh_alloc(tsne_ctx *ctx, BHTree &t, int64_t n, const std::string &pre = "bh.");
// The single-call operators' tree (tsne_gradient / tsne_repulsion): kept in
// the context, so that consecutive calls of one size reuse its buffers and the
// previous traversal's wave costs (the narrow layout's selection).
BHTree &bh_single_tree(tsne_ctx *ctx, int64_t n);
// Build the tree of all n points of Y (n x 2, device).  rowmap (device,
// nullable = identity) gives each point's insertion row in the reference
// (its original index): the order that decides duplicate multiplicities.
// With root_tile_ok, the build stops after the sort when every query's whole
// tree is one near-exact subtree evaluated from the root's moments (the
// small-embedding phase, see bh_root_tile): t.root_tile tells which.
// near_tol: the near-exact tolerance of this build and the traversals on it
// (< 0: bh_near_tol(ctx, false), the strict one).
void bh_build(tsne_ctx *ctx, BHTree &t, const double *dY, double theta, const int32_t *rowmap = nullptr,
              bool root_tile_ok = false, double near_tol = -1.0);
double bh_near_tol(const tsne_ctx *ctx, bool late);
// Repulsion for the query slots [s0, s1): sorted positions, or with qlist
// (device, ascending sorted positions: one rank's own queries) the positions
// qlist[s0..s1).  F (double2) and z (sum of Q) are written at the sorted
// position; visits (nullable) += node evaluations; bcost (nullable)
// accumulates each wave's cost into the 256-position bucket of its first query
// (cost_by_label: an equal share into each query's 256-label bucket).
// plim (device, nullable): the tree partition -- plim[0..1] = this rank's
// sorted positions [lo, hi) (part_cuts), plim[2] a stack-overflow flag; every
// query then gets this rank's PART of its sums (the cells holding its points,
// see bhtree.hip REF_FORCED), to be added over the ranks.
void bh_repulsion(tsne_ctx *ctx, BHTree &t, double theta, int64_t s0, int64_t s1,
                  double2 *dF, double *dz, unsigned long long *visits, const int32_t *qlist = nullptr,
                  unsigned long long *bcost = nullptr, bool cost_by_label = false, int32_t *plim = nullptr);
// Tree partition cuts: cuts[0..world] (device int64, sorted positions of the
// previous build, refined by part_recut) -> this rank's [lo, hi) in plim,
// each cut moved forward to the next boundary of level-10 cells of this
// build's sorted keys (so no record below level 10 straddles a cut), within [0, m].
void part_align(tsne_ctx *ctx, BHTree &t, const int64_t *cuts, int world, int rank, int32_t *plim);
// New cuts from the ranks' traversal costs (cost[r], all-reduced): the
// cumulative cost, linear inside each rank's current range, cut at equal
// shares (moved half way: damped); identical on every rank.
void part_recut(tsne_ctx *ctx, const unsigned long long *cost, int world, int64_t n, int64_t *cuts);
// This traversal's cost (sum over its waves of pops + tile points / 64) into *out.
void part_cost(tsne_ctx *ctx, BHTree &t, int64_t waves, unsigned long long *out);
// Spill counters of t (synchronises the stream): tasks split off over all its
// traversals, or (flags) 1 a level's list full, 2 tile pages exhausted (those
// walks went on unsplit / untiled: the same sums).
int64_t bh_spill_counter(tsne_ctx *ctx, BHTree &t, bool flags);
// tile streaming: the lists the consumers summed over every call of the tree
int64_t bh_stream_counter(tsne_ctx *ctx, BHTree &t);
// Heavy groups the last traversal on t ran narrow (synchronises the stream).
int64_t bh_narrow_groups(tsne_ctx *ctx, BHTree &t);
// Cut [0, n) into world slices of equal bucket cost -> bounds[0..world] (device).
void bh_balance(tsne_ctx *ctx, const unsigned long long *bcost, int64_t n, int world, int64_t *bounds);

}  // namespace tsne
