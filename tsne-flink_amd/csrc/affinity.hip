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

// Long rows (the distance-matrix mode: a row holds every other point,
// Tsne.scala:155-159): one BT-thread workgroup per row.  The first
// BT * RREG entries stay in registers across the (<= 51) entropy
// evaluations, the next LDSN in LDS, any rest is re-read per evaluation; the
// two sums of computeH are reduced through LDS in a fixed order.  One HBM
// read of the row instead of one per evaluation.  <58, 512, 20000> holds
// 49,696 entries (all but ~300 of C5's 50,000-point rows): 2 waves per SIMD
// leave 256 VGPRs per lane (116 for the row, the fp64 exp / log / division
// code takes the rest without spilling), and the single resident workgroup
// owns the CU's 160 KiB of LDS.
template <int RREG, int BT, int LDSN>
__global__ __launch_bounds__(BT) void beta_search_block(const int64_t *__restrict__ row_ptr,
                                                        const double *__restrict__ dist, int64_t row0,
                                                        double target, double *__restrict__ pout) {
    __shared__ double red[2][BT / 64];
    __shared__ double bc[2];
    __shared__ double lrow[LDSN > 0 ? LDSN : 1];
    const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const int64_t row = row0 + blockIdx.x;
    const int64_t b = row_ptr[row], len = row_ptr[row + 1] - b;
    const double *d = dist + b;
    constexpr int64_t RN = (int64_t)RREG * BT;          // entries in registers
    double dr[RREG];
#pragma unroll
    for (int r = 0; r < RREG; ++r) {
        const int64_t e = (int64_t)r * BT + tid;
        dr[r] = e < len ? d[e] : 0.0;
    }
    const int64_t nl = LDSN > 0 ? (len - RN < LDSN ? (len > RN ? len - RN : 0) : LDSN) : 0;
    for (int64_t e = tid; e < nl; e += BT) lrow[e] = d[RN + e];
    __syncthreads();
    auto sums = [&](double beta, double &s, double &sdp) {
        double a = 0.0, c = 0.0;
#pragma unroll
        for (int r = 0; r < RREG; ++r) {
            if ((int64_t)r * BT + tid < len) {
                const double p = exp(-dr[r] * beta);
                a += p;
                c += dr[r] * p;
            }
        }
        for (int64_t e = tid; e < nl; e += BT) {
            const double dv = lrow[e];
            const double p = exp(-dv * beta);
            a += p;
            c += dv * p;
        }
        for (int64_t e = RN + nl + tid; e < len; e += BT) {   // beyond registers + LDS: re-read
            const double dv = d[e];
            const double p = exp(-dv * beta);
            a += p;
            c += dv * p;
        }
        a = wave_sum(a);
        c = wave_sum(c);
        if (lane == 0) { red[0][w] = a; red[1][w] = c; }
        __syncthreads();
        if (tid < 2) {
            double t = 0.0;
            for (int k = 0; k < BT / 64; ++k) t += red[tid][k];
            bc[tid] = t;
        }
        __syncthreads();
        s = bc[0];
        sdp = bc[1];
        __syncthreads();   // red / bc are rewritten by the next evaluation
    };
    double beta = 1.0, mn = -__builtin_inf(), mx = __builtin_inf();
    int budget = 50;
    double s, sdp;
    for (;;) {
        sums(beta, s, sdp);
        const double sp = (s == 0.0) ? 1e-7 : s;
        const double h = log(sp) + beta * sdp / sp;
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
    const double sp = (s == 0.0) ? 1e-7 : s;
    double *p = pout + b;
#pragma unroll
    for (int r = 0; r < RREG; ++r) {
        const int64_t e = (int64_t)r * BT + tid;
        if (e < len) p[e] = exp(-dr[r] * beta) / sp;
    }
    for (int64_t e = tid; e < nl; e += BT) p[RN + e] = exp(-lrow[e] * beta) / sp;
    for (int64_t e = RN + nl + tid; e < len; e += BT) p[e] = exp(-d[e] * beta) / sp;
}

// longest row of a CSR (the dispatch of the beta search)
__global__ void max_row_len(const int64_t *__restrict__ row_ptr, int64_t n, unsigned long long *__restrict__ out) {
    unsigned long long m = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        m = max(m, (unsigned long long)(row_ptr[i + 1] - row_ptr[i]));
    m = wave_max(m);
    if (lane_id() == 0) atomicMax(out, m);
}

// ------------------------------------------------------------ symmetrise
// Row i of J = its own entries (J_ij = p_j|i + p_i|j if i is in row j, else
// p_j|i) followed by the non-mutual reverse entries (j -> i, J_ij = p_i|j).
// Needs each input row sorted by column for the mutual lookup.

// int32 segment offsets of rows [r0, r0 + m), relative to row_ptr[r0]
// (the segmented sorts run over row chunks of < 2^31 entries)
__global__ void seg_offsets(const int64_t *__restrict__ row_ptr, int64_t r0, int64_t m, int *__restrict__ b,
                            int *__restrict__ e) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) {
        const int64_t base = row_ptr[r0];
        b[i] = (int)(row_ptr[r0 + i] - base);
        e[i] = (int)(row_ptr[r0 + i + 1] - base);
    }
}

// flag[0] = 1 if some row's columns are not ascending (the sort is needed)
__global__ void rows_unsorted(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col, int64_t n,
                              int32_t *__restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (i >= n) return;
    bool bad = false;
    for (int64_t t = row_ptr[i] + 1 + lane_id(); t < row_ptr[i + 1]; t += 64) bad |= col[t - 1] > col[t];
    if (__ballot(bad) && lane_id() == 0) flag[0] = 1;
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
    hipStream_t st = ctx->stream;
    unsigned long long *dm = ctx->ws.get<unsigned long long>("aff.maxlen", 1);
    TSNE_HIP(hipMemsetAsync(dm, 0, sizeof(unsigned long long), st));
    hipLaunchKernelGGL(max_row_len, dim3(std::min<int64_t>(1024, ceil_div(nrows, 256))), dim3(256), 0, st, d_row_ptr,
                       nrows, dm);
    unsigned long long maxlen = 0;
    TSNE_HIP(hipMemcpyAsync(&maxlen, dm, sizeof(maxlen), hipMemcpyDeviceToHost, st));
    TSNE_HIP(hipStreamSynchronize(st));
    const double target = log(perplexity);
    // kNN rows (<= 128 entries): a wave per row; distance-matrix rows: a
    // workgroup per row with the row in registers + LDS (the tail re-read)
    if (maxlen <= 128) {
        hipLaunchKernelGGL(beta_search<2>, dim3(ceil_div(nrows, 4)), dim3(256), 0, st, d_row_ptr, d_dist, nrows, target,
                           d_p);
    } else {
        auto kern = maxlen <= 4096 ? beta_search_block<4, 1024, 0> : maxlen <= 16384 ? beta_search_block<16, 1024, 0>
                  : beta_search_block<58, 512, 20000>;
        const int bt = maxlen <= 16384 ? 1024 : 512;
        for (int64_t r0 = 0; r0 < nrows; r0 += 1 << 20)   // grid.x chunks
            hipLaunchKernelGGL(kern, dim3(std::min<int64_t>(1 << 20, nrows - r0)), dim3(bt), 0, st, d_row_ptr, d_dist,
                               r0, target, d_p);
    }
    TSNE_LAUNCH_CHECK();
}

// Stable per-row sort of (col, val) by column for every CSR row, in row
// chunks of < 2^31 entries (hipcub's segmented sort takes int offsets; the
// distance-matrix mode reaches N^2 = 2.5e9 entries at 50k points).
static void sort_rows(tsne_ctx *ctx, const std::vector<int64_t> &hrp, const int64_t *d_rp, int64_t n,
                      const int32_t *kin, int32_t *kout, const double *vin, double *vout, const char *tag) {
    hipStream_t st = ctx->stream;
    Workspace &ws = ctx->ws;
    const int64_t LIM = (int64_t)INT32_MAX - 1;
    int64_t r0 = 0;
    while (r0 < n) {
        int64_t r1 = r0;   // largest r1 with hrp[r1] - hrp[r0] <= LIM (at least one row)
        {
            int64_t lo = r0 + 1, hi = n;
            while (lo < hi) {
                const int64_t mid = (lo + hi + 1) / 2;
                if (hrp[mid] - hrp[r0] <= LIM) lo = mid; else hi = mid - 1;
            }
            r1 = lo;
        }
        TSNE_REQUIRE(hrp[r1] - hrp[r0] <= LIM, "a single row holds 2^31 or more entries");
        const int64_t m = r1 - r0, base = hrp[r0], cnt = hrp[r1] - hrp[r0];
        int *sb = ws.get<int>("sym.sb", m), *se = ws.get<int>("sym.se", m);
        hipLaunchKernelGGL(seg_offsets, dim3(ceil_div(m, 256)), dim3(256), 0, st, d_rp, r0, m, sb, se);
        size_t tb = 0;
        TSNE_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, tb, kin + base, kout + base, vin + base,
                                                             vout + base, (int)cnt, (int)m, sb, se, 0, 32, st));
        void *tmp = ws.get<uint8_t>(std::string("sym.tmp.") + tag, tb);
        TSNE_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(tmp, tb, kin + base, kout + base, vin + base,
                                                             vout + base, (int)cnt, (int)m, sb, se, 0, 32, st));
        TSNE_LAUNCH_CHECK();
        r0 = r1;
    }
}

int64_t joint_device(tsne_ctx *ctx, const int64_t *d_row_ptr, const int32_t *d_col,
                     const double *d_p, int64_t n, int64_t cap, int64_t *d_out_row_ptr,
                     int32_t *d_out_col, double *d_out_val) {
    hipStream_t st = ctx->stream;
    Workspace &ws = ctx->ws;
    std::vector<int64_t> hrp(n + 1);
    TSNE_HIP(hipMemcpyAsync(hrp.data(), d_row_ptr, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, st));
    int32_t *flag = ws.get<int32_t>("sym.flag", 1);
    TSNE_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), st));
    hipLaunchKernelGGL(rows_unsorted, dim3(ceil_div(n, 4)), dim3(256), 0, st, d_row_ptr, d_col, n, flag);
    int32_t unsorted = 0;
    TSNE_HIP(hipMemcpyAsync(&unsorted, flag, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    TSNE_HIP(hipStreamSynchronize(st));
    const int64_t nnz = hrp[n];
    TSNE_REQUIRE(hrp[0] == 0, "row_ptr[0] must be 0");
    // 1. every input row sorted by column (stable, so duplicate columns keep
    // order); rows that already are (a full distance matrix) are used in place
    const int32_t *scol = d_col;
    const double *sval = d_p;
    if (unsorted) {
        int32_t *c2 = ws.get<int32_t>("sym.scol", nnz + 1);
        double *v2 = ws.get<double>("sym.sval", nnz + 1);
        sort_rows(ctx, hrp, d_row_ptr, n, d_col, c2, d_p, v2, "in");
        scol = c2;
        sval = v2;
    }
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
    if (total > cap) { ws.release_prefix("sym."); return total; }
    // 3. fill (own entries in place, reverse entries appended), then sort each
    // output row by column -- not needed when no row received a reverse entry
    // (every pair mutual, e.g. a full distance matrix: rows stay sorted)
    const bool any_rev = total > nnz;
    int32_t *ucol = any_rev ? ws.get<int32_t>("sym.ucol", total + 1) : d_out_col;
    double *uval = any_rev ? ws.get<double>("sym.uval", total + 1) : d_out_val;
    TSNE_HIP(hipMemsetAsync(rev, 0, n * sizeof(int32_t), st));
    hipLaunchKernelGGL(sym_fill, dim3(ceil_div(n, 4)), dim3(256), 0, st, d_row_ptr, scol, sval, mpos,
                       n, excl, rev, ucol, uval);
    TSNE_LAUNCH_CHECK();
    hipLaunchKernelGGL(copy_row_ptr, dim3(ceil_div(n + 1, 256)), dim3(256), 0, st, excl, n, total,
                       d_out_row_ptr);
    if (any_rev) {
        std::vector<int64_t> hor(n + 1);
        TSNE_HIP(hipMemcpyAsync(hor.data(), d_out_row_ptr, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, st));
        TSNE_HIP(hipStreamSynchronize(st));
        sort_rows(ctx, hor, d_out_row_ptr, n, ucol, d_out_col, uval, d_out_val, "out");
    }
    // 4. normalise by the global sum
    const int nparts = 1024;
    double *part = ws.get<double>("sym.part", nparts);
    hipLaunchKernelGGL(sum_partial, dim3(nparts), dim3(256), 0, st, d_out_val, total, part);
    hipLaunchKernelGGL(scale_by_sum, dim3(1024), dim3(256), 0, st, d_out_val, total, part, nparts);
    TSNE_LAUNCH_CHECK();
    TSNE_HIP(hipStreamSynchronize(st));
    ws.release_prefix("sym.");   // N^2-sized temporaries in the distance-matrix mode
    return total;
}

}  // namespace tsne
