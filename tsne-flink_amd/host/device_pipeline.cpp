// device_pipeline.cpp -- see device_pipeline.hpp.
#include "device_pipeline.hpp"

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <stdexcept>
#include <string>

namespace tsne_flink {
namespace {

void hipCheck(hipError_t e, const char *what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void libCheck(int rc) {
    if (rc != TSNE_OK) throw std::runtime_error("libtsne_hip status " + std::to_string(rc) + ": " + tsne_last_error());
}

// one device allocation, freed on scope exit
template <class T> struct DevArray {
    T *p = nullptr;
    explicit DevArray(size_t count) { hipCheck(hipMalloc(reinterpret_cast<void **>(&p), sizeof(T) * (count ? count : 1)), "hipMalloc"); }
    ~DevArray() { if (p) (void)hipFree(p); }
    DevArray(const DevArray &) = delete;
    DevArray &operator=(const DevArray &) = delete;
    void release() { if (p) (void)hipFree(p); p = nullptr; }
};

double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

DeviceRun runOnDevice(tsne_ctx *ctx, const std::vector<double> &X, int64_t n, int32_t d, int32_t k,
                      double perplexity, const tsne_params &p, int64_t randomState) {
    if (n < 2) throw std::invalid_argument("the device pipeline needs at least two points");
    DeviceRun out;
    const int64_t kk = std::min<int64_t>(k, n - 1);
    const int32_t C = p.n_components;
    double t0 = now();
    // kNearestNeighbors (TsneHelpers.scala:41-59)
    DevArray<int32_t> idx((size_t)(n * kk));
    DevArray<double> dist((size_t)(n * kk));
    {
        DevArray<double> dX((size_t)n * d);
        hipCheck(hipMemcpy(dX.p, X.data(), sizeof(double) * (size_t)n * d, hipMemcpyHostToDevice), "H2D X");
        libCheck(tsne_dev_knn(ctx, dX.p, n, d, p.metric, k, 0, n, idx.p, dist.p));
        libCheck(tsne_ctx_synchronize(ctx));
    }
    out.t_knn = now() - t0;
    t0 = now();
    // pairwiseAffinities (:162-180) over the kNN rows, jointDistribution (:182-196)
    std::vector<int64_t> hrp((size_t)n + 1);
    for (int64_t r = 0; r <= n; ++r) hrp[(size_t)r] = r * kk;
    DevArray<int64_t> rp((size_t)n + 1);
    hipCheck(hipMemcpy(rp.p, hrp.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice), "H2D row_ptr");
    DevArray<double> cond((size_t)(n * kk));
    libCheck(tsne_dev_pairwise_affinities(ctx, rp.p, dist.p, n, perplexity, cond.p));
    dist.release();
    const int64_t cap = 2 * n * kk + 1;
    DevArray<int64_t> prp((size_t)n + 1);
    DevArray<int32_t> pcol((size_t)cap);
    DevArray<double> pval((size_t)cap);
    int64_t nnz = 0;
    libCheck(tsne_dev_joint_distribution(ctx, rp.p, idx.p, cond.p, n, cap, prp.p, pcol.p, pval.p, &nnz));
    if (nnz > cap) throw std::runtime_error("joint distribution larger than its bound");
    libCheck(tsne_ctx_synchronize(ctx));
    idx.release();
    cond.release();
    out.nnz = nnz;
    out.t_aff = now() - t0;
    t0 = now();
    // initWorkingSet (:198-219) + optimize (:396-430), the state resident in HBM
    const size_t ne = (size_t)n * C;
    std::vector<double> y(ne), upd(ne), gains(ne);
    libCheck(tsne_init_working_set(ctx, n, C, (uint64_t)randomState, y.data(), upd.data(), gains.data()));
    DevArray<double> dY(ne), dU(ne), dG(ne);
    hipCheck(hipMemcpy(dY.p, y.data(), sizeof(double) * ne, hipMemcpyHostToDevice), "H2D Y");
    hipCheck(hipMemcpy(dU.p, upd.data(), sizeof(double) * ne, hipMemcpyHostToDevice), "H2D upd");
    hipCheck(hipMemcpy(dG.p, gains.data(), sizeof(double) * ne, hipMemcpyHostToDevice), "H2D gains");
    libCheck(tsne_dev_opt_setup(ctx, &p, prp.p, pcol.p, pval.p, n, dY.p, dU.p, dG.p));
    for (int32_t t = 1; t <= p.iterations; ++t) libCheck(tsne_dev_opt_step(ctx, t));
    libCheck(tsne_dev_opt_sync(ctx));
    libCheck(tsne_ctx_synchronize(ctx));
    out.y.resize(ne);
    hipCheck(hipMemcpy(out.y.data(), dY.p, sizeof(double) * ne, hipMemcpyDeviceToHost), "D2H Y");
    const int32_t lcap = p.iterations / 10 + 1;
    std::vector<int32_t> keys((size_t)lcap);
    std::vector<double> vals((size_t)lcap);
    int32_t nl = 0;
    libCheck(tsne_dev_opt_losses(ctx, keys.data(), vals.data(), lcap, &nl));
    for (int32_t i = 0; i < std::min(nl, lcap); ++i) out.loss[keys[(size_t)i]] += vals[(size_t)i];
    out.t_loop = now() - t0;
    return out;
}

}  // namespace tsne_flink
