// project.hip -- approximate kNN by Z-order projections (projectKnn,
// TsneHelpers.scala:93-160, with the comparator of ZOrder.scala:25-42), the
// --knnMethod project path, on gfx950.
//
// For the input and each of the iterations-1 shifted copies x + r_s (r_s
// caller-supplied uniform [0,1)^d vectors; the reference draws them
// unseeded), the points are sorted by the Z-order comparator and the k
// points on either side of each point become its candidates; the union is
// ranked by the exact fp64 metric on the ORIGINAL vectors and the k nearest
// are kept, ordered by (distance, j).
//
// The comparator is the reference's: XOR of the raw IEEE bit patterns as
// SIGNED 64-bit integers, the dimension with the most significant differing
// bit decides (less_msb), a(j) > b(j) is "greater".  It is a total order on
// nonnegative inputs (the defined case; exact duplicates are ordered by index
// here, the reference leaves them to TimSort's input order).  The sort is a
// merge sort of row indices (rocPRIM) with that comparator: one O(d) row
// comparison per merge step, the rows read from L2 / HBM.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace tsne {
namespace {

constexpr int PROJ_CAP = 1024;   // candidates per query (2 k iterations <= PROJ_CAP)

// strict weak order on row indices: Z-order of the rows, index on ties
struct ZLess {
    const double *X;
    int32_t d;
    __device__ bool operator()(const int32_t &i, const int32_t &j) const {
        const double *a = X + (int64_t)i * d, *b = X + (int64_t)j * d;
        int32_t m = 0;
        int64_t x = 0;
        for (int32_t c = 0; c < d; ++c) {
            const int64_t y = __double_as_longlong(a[c]) ^ __double_as_longlong(b[c]);
            if ((x < y) && (x < (x ^ y))) { m = c; x = y; }   // less_msb (signed longs)
        }
        if (b[m] > a[m]) return true;    // compareByZorder(b, a)
        if (a[m] > b[m]) return false;   // compareByZorder(a, b)
        return i < j;
    }
};

__global__ void shift_rows(const double *__restrict__ X, int64_t ne, int32_t d, const double *__restrict__ r,
                           double *__restrict__ Xs, int32_t *__restrict__ order, int64_t n) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < ne) Xs[e] = r ? __dadd_rn(X[e], r[e % d]) : X[e];   // breeze x + randomVector
    if (e < n) order[e] = (int32_t)e;
}

__global__ void rank_of(const int32_t *__restrict__ order, int64_t n, int32_t *__restrict__ rank) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) rank[order[p]] = (int32_t)p;
}

__device__ __forceinline__ double metric_rows(const double *__restrict__ a, const double *__restrict__ b, int32_t d,
                                              int32_t metric) {
    if (metric == TSNE_METRIC_COSINE) {
        double s = 0.0, na = 0.0, nb = 0.0;
        for (int32_t t = 0; t < d; ++t) {
            s = __dadd_rn(s, __dmul_rn(a[t], b[t]));
            na = __dadd_rn(na, __dmul_rn(a[t], a[t]));
            nb = __dadd_rn(nb, __dmul_rn(b[t], b[t]));
        }
        return 1.0 - s / (sqrt(na) * sqrt(nb));
    }
    double s = 0.0;
    for (int32_t t = 0; t < d; ++t) {
        const double df = __dsub_rn(a[t], b[t]);
        s = __dadd_rn(s, __dmul_rn(df, df));
    }
    return metric == TSNE_METRIC_EUCLIDEAN ? sqrt(s) : s;
}

// One 64-thread workgroup per query: gather the 2 k S neighbour slots, sort
// and de-duplicate the ids, exact metric per distinct candidate, sort by
// (key(d), j) and keep kk.  Bitonic sorts in LDS over the padded power of two.
__global__ __launch_bounds__(64) void project_select(const double *__restrict__ X, int64_t n, int32_t d,
                                                     int32_t metric, int32_t k, int32_t S, int32_t P,
                                                     const int32_t *__restrict__ order,
                                                     const int32_t *__restrict__ rank, int32_t kk,
                                                     int32_t *__restrict__ out_idx, double *__restrict__ out_dist) {
    __shared__ int32_t cj[PROJ_CAP];
    __shared__ uint64_t ck[PROJ_CAP];
    __shared__ double cd[PROJ_CAP];
    const int lane = threadIdx.x;
    const int64_t i = blockIdx.x;
    if (i >= n) return;
    const int slots = 2 * k * S;
    for (int e = lane; e < P; e += 64) {
        int32_t j = INT32_MAX;
        if (e < slots) {
            const int s = e / (2 * k), off = e - s * 2 * k;
            const int64_t p = rank[(int64_t)s * n + i];
            const int64_t q = off < k ? p - k + off : p + 1 + (off - k);
            if (q >= 0 && q < n) j = order[(int64_t)s * n + q];
        }
        cj[e] = j;
    }
    __builtin_amdgcn_wave_barrier();
    for (int size = 2; size <= P; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int e = lane; e < P; e += 64) {
                const int o = e ^ stride;
                if (o > e) {
                    const int32_t u = cj[e], v = cj[o];
                    if (((e & size) == 0) == (u > v)) { cj[e] = v; cj[o] = u; }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    // distinct candidates: compact in sorted order
    int m = 0;
    for (int base = 0; base < P; base += 64) {
        const int e = base + lane;
        const int32_t j = cj[e];
        const bool keep = j != INT32_MAX && (e == 0 || cj[e - 1] != j);
        const uint64_t b = __ballot(keep);
        __builtin_amdgcn_wave_barrier();
        if (keep) {
            const int t = m + __popcll(b & lanemask_lt());
            ck[t] = (uint64_t)j;   // staged ids
        }
        m += __popcll(b);
        __builtin_amdgcn_wave_barrier();
    }
    const double *xi = X + i * d;
    for (int e = lane; e < P; e += 64) {
        if (e < m) {
            const int32_t j = (int32_t)ck[e];
            const double v = metric_rows(xi, X + (int64_t)j * d, d, metric);
            cd[e] = v;
            cj[e] = j;
        } else {
            cd[e] = __builtin_inf();
            cj[e] = INT32_MAX;
        }
    }
    __builtin_amdgcn_wave_barrier();
    for (int e = lane; e < P; e += 64) ck[e] = e < m ? dkey(cd[e]) : ~0ull;
    __builtin_amdgcn_wave_barrier();
    for (int size = 2; size <= P; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int e = lane; e < P; e += 64) {
                const int o = e ^ stride;
                if (o > e) {
                    const uint64_t ku = ck[e], kv = ck[o];
                    const int32_t ju = cj[e], jv = cj[o];
                    const bool gt = ku > kv || (ku == kv && ju > jv);
                    if (((e & size) == 0) == gt) {
                        ck[e] = kv; ck[o] = ku;
                        cj[e] = jv; cj[o] = ju;
                        const double t = cd[e]; cd[e] = cd[o]; cd[o] = t;
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    for (int t = lane; t < kk; t += 64) {
        out_idx[i * kk + t] = cj[t];
        out_dist[i * kk + t] = cd[t];
    }
}

}  // namespace

void project_knn_device(tsne_ctx *ctx, const double *dX, int64_t n, int32_t d, int32_t metric, int32_t k,
                        int32_t iterations, const double *d_shifts, int32_t *d_idx, double *d_dist) {
    TSNE_REQUIRE(n >= 2 && d >= 1 && k >= 1 && iterations >= 1, "bad projectKnn arguments");
    TSNE_REQUIRE(metric >= 0 && metric <= 2, "unknown metric");
    TSNE_REQUIRE(n < INT32_MAX, "too many points");
    if ((int64_t)2 * k * iterations > PROJ_CAP)
        fail(TSNE_ERR_UNSUPPORTED, "projectKnn: 2 * k * knnIterations must be <= " + std::to_string(PROJ_CAP));
    hipStream_t st = ctx->stream;
    Workspace &ws = ctx->ws;
    const int32_t S = iterations;
    double *Xs = ws.get<double>("proj.Xs", (size_t)(n * d));
    int32_t *order = ws.get<int32_t>("proj.order", (size_t)(S * n));
    int32_t *rank = ws.get<int32_t>("proj.rank", (size_t)(S * n));
    size_t tb = 0;
    ZLess cmp0{Xs, d};
    TSNE_HIP(hipcub::DeviceMergeSort::SortKeys(nullptr, tb, order, (int)n, cmp0, st));
    void *tmp = ws.get<uint8_t>("proj.sort_tmp", tb);
    const int64_t ne = n * d;
    for (int32_t s = 0; s < S; ++s) {
        int32_t *ord = order + (int64_t)s * n;
        hipLaunchKernelGGL(shift_rows, dim3(ceil_div(std::max(ne, n), 256)), dim3(256), 0, st, dX, ne, d,
                           s == 0 ? nullptr : d_shifts + (int64_t)(s - 1) * d, Xs, ord, n);
        size_t b = tb;
        TSNE_HIP(hipcub::DeviceMergeSort::SortKeys(tmp, b, ord, (int)n, ZLess{Xs, d}, st));
        hipLaunchKernelGGL(rank_of, dim3(ceil_div(n, 256)), dim3(256), 0, st, ord, n, rank + (int64_t)s * n);
    }
    int P = 64;
    while (P < 2 * k * S) P <<= 1;
    const int32_t kk = (int32_t)std::min<int64_t>(k, n - 1);
    hipLaunchKernelGGL(project_select, dim3(n), dim3(64), 0, st, dX, n, d, metric, k, S, P, order, rank, kk, d_idx,
                       d_dist);
    TSNE_LAUNCH_CHECK();
}

}  // namespace tsne
