// device_pipeline.hpp -- the CLI's chain kNN -> pairwiseAffinities ->
// jointDistribution -> optimize (Tsne.scala:80-86, TsneHelpers.scala:41-196,
// 396-430) with every intermediate resident in HBM: the tsne_dev_* entry
// points of the C ABI, so the host sees the input once (one H2D copy of X) and
// the embedding once (one D2H copy of Y), instead of the DataSet-shaped host
// round trips of the TsneHelpers mirror between the operators.  The results
// are those of the mirror's chain (the same library calls on the same data).
#pragma once

#include <cstdint>
#include <map>
#include <vector>

#include "tsne_hip.h"

namespace tsne_flink {

struct DeviceRun {
    std::vector<double> y;             // n x n_components, rows in the input's id order
    std::map<int32_t, double> loss;    // the optimizer's "loss" accumulator
    int64_t nnz = 0;                   // entries of the joint distribution P
    double t_knn = 0, t_aff = 0, t_loop = 0;   // seconds, each stage to its completion
};

// X: n x d row-major (rows = the sorted ids).  Exact kNN (k neighbours, as
// TsneHelpers.kNearestNeighbors), affinities at `perplexity`, the joint P, the
// working set initWorkingSet(randomState), then p.iterations of the optimizer.
// Requires n >= 2 (every row then has k >= 1 neighbours: no empty row of P).
DeviceRun runOnDevice(tsne_ctx *ctx, const std::vector<double> &X, int64_t n, int32_t d, int32_t k,
                      double perplexity, const tsne_params &p, int64_t randomState);

}  // namespace tsne_flink
