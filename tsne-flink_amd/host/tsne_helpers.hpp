// tsne_helpers.hpp -- C++ host mirror of the reference's TsneHelpers object
// (TsneHelpers.scala) over the libtsne_hip C ABI.
//
// The reference's methods take and return Flink DataSets of tuples; here the
// same tuples are std::vectors, point ids are arbitrary int32 (remapped to
// dense indices at the ABI), and every method keeps the reference's name,
// argument meaning and error behaviour (std::invalid_argument where the
// reference throws IllegalArgumentException).
#pragma once

#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "tsne_hip.h"

namespace tsne_flink {

// (i, j, value): kNN distance, p_j|i, or joint p_ij -- DataSet[(Int, Int, Double)]
struct Triple {
    int32_t i, j;
    double v;
};

// DataSet[(Int, Vector[Double])]
using Vectors = std::vector<std::pair<int32_t, std::vector<double>>>;

// DataSet[(Int, Vector, Vector, Vector)]: (id, embedding, last update, gains)
struct WorkingSet {
    std::vector<int32_t> ids;
    int32_t n_components = 2;
    std::vector<double> y, upd, gains;  // ids.size() x n_components, row-major
};

// CSR of triples over a dense id map (ids sorted ascending).
struct Csr {
    std::vector<int32_t> ids;        // dense index -> original id
    std::vector<int64_t> row_ptr;
    std::vector<int32_t> col;        // dense indices
    std::vector<double> val;
};

// Tsne.getMetric (Tsne.scala:161-168): the name validated, the id returned.
int32_t getMetric(const std::string &name);

class TsneHelpers {
  public:
    explicit TsneHelpers(int device = 0);
    tsne_ctx *context() const { return ctx_; }   // the handle its calls run on
    ~TsneHelpers();
    TsneHelpers(const TsneHelpers &) = delete;
    TsneHelpers &operator=(const TsneHelpers &) = delete;

    // TsneHelpers.scala:41-59
    std::vector<Triple> kNearestNeighbors(const Vectors &input, int32_t k, int32_t metric);
    // TsneHelpers.scala:61-91: same exact result; `blocks` is only a tiling hint
    std::vector<Triple> partitionKnn(const Vectors &input, int32_t k, int32_t metric, int32_t blocks);
    std::vector<Triple> projectKnn(const Vectors &input, int32_t k, int32_t metric, int32_t iterations,
                                   int64_t randomState);
    // TsneHelpers.scala:162-180
    std::vector<Triple> pairwiseAffinities(const std::vector<Triple> &knn, double perplexity);
    // TsneHelpers.scala:182-196
    std::vector<Triple> jointDistribution(const std::vector<Triple> &affinities);
    // TsneHelpers.scala:198-219 (randomState honoured: seeded generator)
    WorkingSet initWorkingSet(const std::vector<int32_t> &ids, int32_t nComponents, int64_t randomState);
    // TsneHelpers.scala:221-318 (one evaluation; exaggeration multiplies P)
    std::vector<std::pair<int32_t, std::vector<double>>> gradient(const std::vector<Triple> &P,
                                                                  const WorkingSet &embedding,
                                                                  int32_t metric, double theta,
                                                                  double exaggeration = 1.0);
    // TsneHelpers.scala:341-369 (in place)
    void updateEmbedding(const std::vector<double> &grad, WorkingSet &ws, double minGain,
                         double momentum, double learningRate);
    // TsneHelpers.scala:320-329 (in place)
    void centerEmbedding(WorkingSet &ws);
    // TsneHelpers.scala:396-430; `loss` receives the "loss" accumulator {iteration -> KL}
    void optimize(const std::vector<Triple> &P, WorkingSet &ws, double learningRate,
                  int32_t iterations, int32_t metric, double earlyExaggeration,
                  double initialMomentum, double finalMomentum, double theta,
                  std::map<int32_t, double> *loss);

    // The same operators on CSR (rows = the sorted ids, columns dense row
    // indices): the CLI's path, without materialising 10^8 triples per stage.
    // knnMethod: "bruteforce" / "partition" (exact) or "project".
    Csr kNearestNeighborsCsr(const Vectors &input, int32_t k, int32_t metric, const std::string &method = "bruteforce",
                             int32_t iterations = 3, int64_t randomState = 0);
    // the same on the input already dense: ids ascending, X ids.size() x d (readInputDense)
    Csr kNearestNeighborsCsr(std::vector<int32_t> ids, const std::vector<double> &X, int32_t d, int32_t k,
                             int32_t metric, const std::string &method = "bruteforce", int32_t iterations = 3,
                             int64_t randomState = 0);
    Csr pairwiseAffinitiesCsr(const Csr &knn, double perplexity);
    Csr jointDistributionCsr(const Csr &affinities);
    void optimizeCsr(const Csr &P, WorkingSet &ws, double learningRate, int32_t iterations, int32_t metric,
                     double earlyExaggeration, double initialMomentum, double finalMomentum, double theta,
                     std::map<int32_t, double> *loss);

    tsne_ctx *ctx() { return ctx_; }

  private:
    tsne_ctx *ctx_ = nullptr;
};

// Throws std::invalid_argument for TSNE_ERR_ARG, std::runtime_error otherwise.
void check(int status);

Csr toCsr(const std::vector<Triple> &t, const std::vector<int32_t> *ids = nullptr);
// CSR -> triples (ids restored), row by row
std::vector<Triple> fromCsr(const Csr &c);

// java.lang.Double.toString formatting and java.util.HashMap<Integer,Double>.toString
std::string javaDouble(double v);
std::string javaHashMapString(const std::map<int32_t, double> &m);

}  // namespace tsne_flink
