// affinity.hip -- perplexity calibration (TsneHelpers.scala:162-180, 434-504)
// and symmetrisation (TsneHelpers.scala:182-196) on gfx950.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace tsne {
namespace {

// ------------------------------------------------------------ beta search
// One wavefront per CSR row.  Rows of up to 64*RREG entries stay in
// registers across the (at most 51) entropy evaluations; longer rows
// (distance-matrix mode) are re-read from memory.  The two sums of computeH
// are wave reductions (DPP/shuffle tree) -- the branch structure, the 1e-7
// guard, the strict |H - target| < 1e-5 test and the 50-update budget are
// exactly approximateBeta's.
template <int RREG>
__global__ __launch_bounds__(256) void beta_search(const int64_t *__restrict__ row_ptr,
                                                   const double *__restrict__ dist, int64_t nrows,
                                                   double target, double *__restrict__ pout) {
    const int lane = lane_id();
    const int64_t row = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (row >= nrows) return;
    const int64_t b = row_ptr[row], len = row_ptr[row + 1] - b;
    const double *d = dist + b;
    const bool inreg = len <= 64 * RREG;
    double dr[RREG];
#pragma unroll
    for (int r = 0; r < RREG; ++r) {
        int64_t e = r * 64 + lane;
        dr[r] = (inreg && e < len) ? d[e] : 0.0;
    }
    auto sums = [&](double beta, double &s, double &sdp) {
        s = 0.0;
        sdp = 0.0;
        if (inreg) {
#pragma unroll
            for (int r = 0; r < RREG; ++r) {
                if (r * 64 + lane < len) {
                    double p = exp(-dr[r] * beta);
                    s += p;
                    sdp += dr[r] * p;
                }
            }
        } else {
            for (int64_t e = lane; e < len; e += 64) {
                double dv = d[e];
                double p = exp(-dv * beta);
                s += p;
                sdp += dv * p;
            }
        }
        s = wave_sum(s);
        sdp = wave_sum(sdp);
    };
    double beta = 1.0, mn = -__builtin_inf(), mx = __builtin_inf();
    int budget = 50;
    double s, sdp;
    for (;;) {
        sums(beta, s, sdp);
        double sp = (s == 0.0) ? 1e-7 : s;
        double h = log(sp) + beta * sdp / sp;
        if (fabs(h - target) < 1e-5 || budget == 0) break;
        double nb;
        if (h - target > 0) {
            nb = isinf(mx) ? beta * 2 : (beta + mx) / 2;
            mn = beta;
        } else {
            nb = isinf(mn) ? beta / 2 : (beta + mn) / 2;
            mx = beta;
        }
        beta = nb;
        --budget;
    }
    // computeP: recompute S at the final beta (identical to the last H pass)
    double sp = (s == 0.0) ? 1e-7 : s;
    double *p = pout + b;
    if (inreg) {
#pragma unroll
        for (int r = 0; r < RREG; ++r) {
            int64_t e = r * 64 + lane;
            if (e < len) p[e] = exp(-dr[r] * beta) / sp;
        }
    } else {
        for (int64_t e = lane; e < len; e += 64) p[e] = exp(-d[e] * beta) / sp;
    }
}

// ------------------------------------------------------------ symmetrise
// Row i of J = its own entries (J_ij = p_j|i + p_i|j if i is in row j, else
// p_j|i) followed by the non-mutual reverse entries (j -> i, J_ij = p_i|j).
// Needs each input row sorted by column for the mutual lookup.

__global__ void seg_offsets(const int64_t *__restrict__ row_ptr, int64_t n, int *__restrict__ b,
                            int *__restrict__ e) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { b[i] = (int)row_ptr[i]; e[i] = (int)row_ptr[i + 1]; }
}

__device__ __forceinline__ int64_t find_in_row(const int32_t *__restrict__ scol, int64_t b,
                                               int64_t e, int32_t key) {
    while (b < e) {
        int64_t m = (b + e) >> 1;
        int32_t v = scol[m];
        if (v < key) b = m + 1;
        else e = m;
    }
    return b;
}

// pass 1: per entry (i, j): mutual?  count reverse entries per target row.
__global__ void sym_count(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ scol,
                          int64_t n, int32_t *__restrict__ mutual_pos,
                          int32_t *__restrict__ rev_cnt) {
    const int64_t i = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (i >= n) return;
    const int lane = lane_id();
    for (int64_t t = row_ptr[i] + lane; t < row_ptr[i + 1]; t += 64) {
        int32_t j = scol[t];
        int64_t jb = row_ptr[j], je = row_ptr[j + 1];
        int64_t pos = find_in_row(scol, jb, je, (int32_t)i);
        bool mutual = pos < je && scol[pos] == (int32_t)i;
        mutual_pos[t] = mutual ? (int32_t)(pos - jb) : -1;
        if (!mutual) atomicAdd(&rev_cnt[j], 1);
    }
}

__global__ void sym_rowlen(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ rev_cnt,
                           int64_t n, int64_t *__restrict__ out_len) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out_len[i] = (row_ptr[i + 1] - row_ptr[i]) + rev_cnt[i];
}

// pass 2: write own entries in place and scatter reverse entries.
__global__ void sym_fill(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ scol,
                         const double *__restrict__ sval, const int32_t *__restrict__ mutual_pos,
                         int64_t n, const int64_t *__restrict__ out_ptr,
                         int32_t *__restrict__ rev_fill, int32_t *__restrict__ ocol,
                         double *__restrict__ oval) {
    const int64_t i = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (i >= n) return;
    const int lane = lane_id();
    const int64_t rb = row_ptr[i], len = row_ptr[i + 1] - rb;
    for (int64_t t = rb + lane; t < rb + len; t += 64) {
        int32_t j = scol[t];
        double v = sval[t];
        int32_t mp = mutual_pos[t];
        const int64_t o = out_ptr[i] + (t - rb);
        if (mp >= 0) {
            ocol[o] = j;
            oval[o] = v + sval[row_ptr[j] + mp];  // p_j|i + p_i|j
        } else {
            ocol[o] = j;
            oval[o] = v;
            int slot = atomicAdd(&rev_fill[j], 1);
            int64_t oj = out_ptr[j] + (row_ptr[j + 1] - row_ptr[j]) + slot;
            ocol[oj] = (int32_t)i;
            oval[oj] = v;
        }
    }
}

__global__ void sum_partial(const double *__restrict__ v, int64_t n, double *__restrict__ part) {
    __shared__ double s_w[4];
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        s += v[i];
    s = wave_sum(s);
    if (lane_id() == 0) s_w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (s_w[0] + s_w[1]) + (s_w[2] + s_w[3]);
}

__global__ void scale_by_sum(double *__restrict__ v, int64_t n, const double *__restrict__ part,
                             int nparts) {
    __shared__ double tot;
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int b = 0; b < nparts; ++b) s += part[b];
        tot = s;
    }
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        v[i] = v[i] / tot;
}

__global__ void copy_row_ptr(const int64_t *__restrict__ excl, int64_t n, int64_t total,
                             int64_t *__restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = excl[i];
    if (i == n) out[n] = total;
}

}  // namespace

void affinities_device(tsne_ctx *ctx, const int64_t *d_row_ptr, const double *d_dist,
                       int64_t nrows, double perplexity, double *d_p) {
    TSNE_REQUIRE(perplexity > 0.0, "perplexity must be positive");
    if (nrows <= 0) return;
    hipLaunchKernelGGL(beta_search<2>, dim3(ceil_div(nrows, 4)), dim3(256), 0, ctx->stream,
                       d_row_ptr, d_dist, nrows, log(perplexity), d_p);
    TSNE_LAUNCH_CHECK();
}

int64_t joint_device(tsne_ctx *ctx, const int64_t *d_row_ptr, const int32_t *d_col,
                     const double *d_p, int64_t n, int64_t cap, int64_t *d_out_row_ptr,
                     int32_t *d_out_col, double *d_out_val) {
    hipStream_t st = ctx->stream;
    Workspace &ws = ctx->ws;
    int64_t nnz = 0;
    TSNE_HIP(hipMemcpyAsync(&nnz, d_row_ptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    TSNE_HIP(hipStreamSynchronize(st));
    TSNE_REQUIRE(nnz < (int64_t)INT32_MAX, "nnz must fit int32 offsets for the segmented sort");
    // 1. sort every input row by column (stable, so duplicate columns keep order)
    int *sb = ws.get<int>("sym.sb", n), *se = ws.get<int>("sym.se", n);
    hipLaunchKernelGGL(seg_offsets, dim3(ceil_div(n, 256)), dim3(256), 0, st, d_row_ptr, n, sb, se);
    int32_t *scol = ws.get<int32_t>("sym.scol", nnz + 1);
    double *sval = ws.get<double>("sym.sval", nnz + 1);
    size_t tb = 0;
    TSNE_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, tb, d_col, scol, d_p, sval, (int)nnz,
                                                         (int)n, sb, se, 0, 32, st));
    void *tmp = ws.get<uint8_t>("sym.tmp", tb);
    TSNE_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(tmp, tb, d_col, scol, d_p, sval, (int)nnz,
                                                         (int)n, sb, se, 0, 32, st));
    // 2. mutual lookup + reverse counts
    int32_t *mpos = ws.get<int32_t>("sym.mpos", nnz + 1);
    int32_t *rev = ws.get<int32_t>("sym.rev", n);
    TSNE_HIP(hipMemsetAsync(rev, 0, n * sizeof(int32_t), st));
    hipLaunchKernelGGL(sym_count, dim3(ceil_div(n, 4)), dim3(256), 0, st, d_row_ptr, scol, n, mpos, rev);
    int64_t *len = ws.get<int64_t>("sym.len", n + 1);
    hipLaunchKernelGGL(sym_rowlen, dim3(ceil_div(n, 256)), dim3(256), 0, st, d_row_ptr, rev, n, len);
    int64_t *excl = ws.get<int64_t>("sym.excl", n + 1);
    size_t tb2 = 0;
    TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, len, excl, (int)n + 1, st));
    void *tmp2 = ws.get<uint8_t>("sym.tmp2", tb2);
    TSNE_HIP(hipMemsetAsync(len + n, 0, sizeof(int64_t), st));
    TSNE_HIP(hipcub::DeviceScan::ExclusiveSum(tmp2, tb2, len, excl, (int)n + 1, st));
    int64_t total = 0;
    TSNE_HIP(hipMemcpyAsync(&total, excl + n, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    TSNE_HIP(hipStreamSynchronize(st));
    if (total > cap) return total;
    // 3. fill (unsorted reverse part), then sort each output row by column
    int32_t *ucol = ws.get<int32_t>("sym.ucol", total + 1);
    double *uval = ws.get<double>("sym.uval", total + 1);
    TSNE_HIP(hipMemsetAsync(rev, 0, n * sizeof(int32_t), st));
    hipLaunchKernelGGL(sym_fill, dim3(ceil_div(n, 4)), dim3(256), 0, st, d_row_ptr, scol, sval, mpos,
                       n, excl, rev, ucol, uval);
    TSNE_LAUNCH_CHECK();
    hipLaunchKernelGGL(copy_row_ptr, dim3(ceil_div(n + 1, 256)), dim3(256), 0, st, excl, n, total,
                       d_out_row_ptr);
    hipLaunchKernelGGL(seg_offsets, dim3(ceil_div(n, 256)), dim3(256), 0, st, d_out_row_ptr, n, sb, se);
    size_t tb3 = 0;
    TSNE_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, tb3, ucol, d_out_col, uval, d_out_val,
                                                         (int)total, (int)n, sb, se, 0, 32, st));
    void *tmp3 = ws.get<uint8_t>("sym.tmp3", tb3);
    TSNE_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(tmp3, tb3, ucol, d_out_col, uval, d_out_val,
                                                         (int)total, (int)n, sb, se, 0, 32, st));
    // 4. normalise by the global sum
    const int nparts = 1024;
    double *part = ws.get<double>("sym.part", nparts);
    hipLaunchKernelGGL(sum_partial, dim3(nparts), dim3(256), 0, st, d_out_val, total, part);
    hipLaunchKernelGGL(scale_by_sum, dim3(1024), dim3(256), 0, st, d_out_val, total, part, nparts);
    TSNE_LAUNCH_CHECK();
    return total;
}

}  // namespace tsne
