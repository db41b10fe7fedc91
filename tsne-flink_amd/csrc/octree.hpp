// octree.hpp -- GPU Barnes-Hut octree for 3-D embeddings (nComponents = 3).
//
// The reference supports only 2-D embeddings (Cell.scala:32 requires
// len == 2).  SURVEY.md section 8f asks for the natural generalisation, which
// oracle/tsne_oracle.c restates (root Cell(0, 0, 0, W), W = max(dX, dY, dZ),
// capacity 1, children upper/lower x NW, NE, SW, SE, criterion h / D < theta
// with D the squared 3-D distance).  The GPU build follows bhtree.hpp's
// design: Morton keys replaying the cell arithmetic (21 levels x 3 bits), a
// Karras binary radix tree whose nodes at a level boundary are the octree
// cells (the rest transparent), and a wave-shared traversal stack.
#pragma once
#include "common.hpp"
#include "csort.hpp"

namespace tsne {

struct __attribute__((aligned(16))) OctNode {
    double cx, cy, cz;            // centre of mass
    double h;                     // half width of the cell, < 0 = transparent
    double hmin;                  // min h over the real cells of the subtree (+inf if none)
    double rball;                 // all-open ball radius around the centre of mass
    double bx0, bx1, by0, by1, bz0, bz1;   // bounding box of the subtree's points
    int32_t cnt;                  // cumSize
    int32_t left, right;          // >= 0 internal node, < 0 leaf ~sorted index
    int32_t delta;                // common-prefix bits (63+ = key tie)
    int32_t first, last;          // leaf range in sorted order
};

// Octal record of a real octree cell (the 2-D QRec's design, bhtree.hpp):
// its own tile-test data plus the summaries of its <= 8 octree children,
// found by descending through the transparent binary nodes of its level
// (<= 2 binary levels: 3 key bits per octal level), so that the traversal
// evaluates all children of an opened cell from one record load.  Child kinds
// (bits 2c of `kinds`): OK_CELL a real cell (cref = node id), OK_LEAF one
// point (cref = ~sorted index), OK_TIE a key-tie group (cref = node id: all
// its points interact directly).
constexpr int OK_CELL = 0, OK_LEAF = 1, OK_TIE = 2;
constexpr int32_t ONCH_TILE = 0x100;   // nch flag: an all-open / near-exact tile test can pass here
struct __attribute__((aligned(16))) ORec {
    double cx, cy, cz;                     // centre of mass
    double rball2, thr;                    // tile tests: rball^2 (1 - 1e-9); max(hmin / theta (1 - 1e-12), near_dmax)
    double bx0, bx1, by0, by1, bz0, bz1;   // bounding box of the subtree's points
    int32_t first, last, cnt, nch;         // leaf range, cumSize, children | ONCH_TILE
    int32_t kinds, pad;
    double ccx[8], ccy[8], ccz[8];         // child centres of mass (leaf: the point)
    double cb[8], ca[8];                   // cells: sure-open / sure-accept bounds on 1 + D (bhtree.hpp QACC_BAND:
                                           // qacc_open / qacc_accept; the band's exact quotient reads h from the node)
    int32_t cref[8], ccnt[8];
};
static_assert(sizeof(ORec) % 16 == 0, "records are fetched in 16-byte pieces");

struct OctTree {
    int64_t n = 0;
    uint64_t *keys = nullptr, *keys_sorted = nullptr;
    int32_t *idx = nullptr, *idx_sorted = nullptr;   // sorted position -> original row
    int32_t *inv = nullptr;                          // original row -> sorted position
    int32_t *dupc = nullptr;                         // exact duplicates of each sorted point
    double4 *pos = nullptr;                          // sorted positions (x, y, z, 0)
    OctNode *nodes = nullptr;
    ORec *orec = nullptr;                            // per binary node id, valid for real cells
    double near_dmax = 0.0;                          // the records' near-exact radius (this build)
    double *agg = nullptr;
    int32_t *parent_leaf = nullptr, *parent_node = nullptr, *arrive = nullptr;
    int32_t *meta = nullptr;                         // [0] in-root points m, [1] root ref
    double *bbox_part = nullptr, *W = nullptr;
    void *sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    CoherentSort cs;             // the Morton sort from the previous build's order (csort.hpp)
    bool cs_primed = false;
    int bbox_blocks = 0;
    // subtree moments (70 per node of >= MOM3_MIN points, about its box
    // centre), built in chunks; gated by the previous traversal's demand
    double *mom = nullptr, *mom_part = nullptr;
    int32_t *mlist = nullptr;   // nodes whose moments sum several items (oct_mom_reduce)
    int32_t *mcnt = nullptr, *moff = nullptr, *item_node = nullptr, *mom_flag = nullptr;
    int32_t *mtask = nullptr, *mtask_n = nullptr;   // per query: nodes evaluated from their moments
    void *mscan_tmp = nullptr;
    size_t mscan_tmp_bytes = 0;
    int64_t item_cap = 0;
};

// Allocate (from ctx->ws, buffers named pre + field) for n points: the
// optimizer's tree "oct.", the single-call operators' "oct1." (the coherent
// sort reads the previous build's order, so two trees never share buffers).
void oct_alloc(tsne_ctx *ctx, OctTree &t, int64_t n, const std::string &pre = "oct.");
// Octree of all n points of Y (n x 3, device); late: the optimizer after
// early exaggeration (the near-exact tolerance the records are built for).
void oct_build(tsne_ctx *ctx, OctTree &t, const double *dY, double theta, bool late = false);
// Repulsion for the query slots [s0, s1) (sorted positions, or qlist[slot]:
// a rank's own queries, ascending): F (n x 3, sorted order) and z written
// at the sorted position (the near-exact tolerance of the build).
void oct_repulsion(tsne_ctx *ctx, const OctTree &t, double theta, int64_t s0, int64_t s1, double *dF,
                   double *dz, const int32_t *qlist = nullptr);

}  // namespace tsne
