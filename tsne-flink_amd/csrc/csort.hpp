// csort.hpp -- the trees' Morton sort, using the previous build's order.
//
// Every optimizer iteration sorts all n points by their Morton key (bhtree /
// octree builds).  rocPRIM's radix sort of 64-bit keys takes ~190 us at
// n = 1M (its merge-sort path: ~20 launches), a quarter of the 2-D build.
// The embedding moves little between iterations, so the previous build's
// sorted order nearly sorts the new keys: P splitters taken from it at equal
// steps (oversampled 4x) cut the key range into buckets of ~1024 points, the points are
// scattered to their buckets (in the previous order: a workgroup's points
// fall into a few adjacent buckets), and each bucket is sorted in LDS.
// Output: keys ascending, ties by point index -- exactly the stable radix
// sort of (keys[i], i), whatever the previous order was (it only sets the
// bucket sizes; a bucket beyond the LDS capacity is sorted in global memory
// by its workgroup, correct and slower).
#pragma once
#include "common.hpp"

namespace tsne {

struct CoherentSort {
    int64_t n = 0;
    int32_t P = 0;                  // buckets
    uint64_t *split = nullptr;      // P sorted splitters (bucket b holds keys in [split[b], split[b + 1]))
    uint64_t *runs = nullptr;       // the sorted sample runs the splitters are merged from
    int32_t *cnt = nullptr;         // P bucket sizes
    int32_t *off = nullptr;         // P + 1 bucket offsets
    int32_t *cur = nullptr;         // P scatter cursors
    int32_t *bkt = nullptr;         // n: bucket of element j (the previous order's j-th point)
    uint64_t *kb = nullptr;         // 3n: bucketed keys [0, n), then the oversized buckets' scratch
                                    // (bucket at offset o: [n + 2 o, n + 2 o + 2 m), power-of-two padded)
    int32_t *vb = nullptr;          // 3n: bucketed point indices, the same layout
    int32_t *stat = nullptr;        // [0] oversized buckets of the last sort, [1] their running total (diagnostics)
};

// Buffers for n points (ctx workspace, names pre + field).  n outside
// [CSORT_MIN_N, CSORT_MAX_N]: nothing (the callers keep rocPRIM's sort).
constexpr int64_t CSORT_MIN_N = 16384;
// Above 1024 x 1.2k points the mean bucket outgrows the LDS sort's 4k capacity
// at the measured 3.3x bucket skew (cs_split_runs) and whole buckets would take the
// slow global-memory bitonic path: rocPRIM's sort there.
constexpr int64_t CSORT_MAX_N = 1250000;
void csort_alloc(tsne_ctx *ctx, CoherentSort &cs, int64_t n, const std::string &pre);
// keys[p] for points p < n -> keys_sorted / idx_sorted ascending by (key, p).
// prev_idx_sorted: the previous sort's idx_sorted (a permutation of [0, n));
// it may be the same buffer as idx_sorted (read before it is written).
void csort_run(tsne_ctx *ctx, CoherentSort &cs, const uint64_t *keys, const int32_t *prev_idx_sorted,
               uint64_t *keys_sorted, int32_t *idx_sorted, hipStream_t st);
// Oversized buckets of the last csort_run, or (total) of every run since the
// allocation (synchronises the context's stream; 0 if none ran).
int64_t csort_oversized(tsne_ctx *ctx, const CoherentSort &cs, bool total = false);

}  // namespace tsne
