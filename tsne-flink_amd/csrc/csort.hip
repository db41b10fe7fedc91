// csort.hip -- the trees' Morton sort from the previous build's order (csort.hpp).
#include "csort.hpp"

namespace tsne {
namespace {

constexpr int CS_BLK = 1024;      // elements per count / scatter workgroup
constexpr int CS_TARGET = 1024;   // points per bucket
constexpr int CS_PMAX = 1024;     // buckets at most
constexpr int CS_OVS = 4;         // samples per bucket (splitters: every CS_OVS-th sorted sample)
constexpr int CS_CAP = 4096;      // bucket capacity of the LDS sort (48 KB)
constexpr int CS_SORT_T = 1024;   // threads of a bucket's sort

// (k, v) < (k2, v2) lexicographically
__device__ __forceinline__ bool kv_less(uint64_t k, int32_t v, uint64_t k2, int32_t v2) {
    return k < k2 || (k == k2 && v < v2);
}

// Bitonic sorts of N (a power of two) entries, T threads: stage (k, j) has
// N / 2 compare-exchange pairs (i, i + j), i = the pair index p with a zero
// bit inserted at j, taken p = tid, tid + T, ... (every thread busy).
__device__ __forceinline__ int bitonic_lo(int p, int j) { return ((p & ~(j - 1)) << 1) | (p & (j - 1)); }

// Stage boundary of the bitonic networks below.  A stage of partner distance
// j <= 64 pairs, in each wave's share (pairs p = 64 w .. 64 w + 63, + T per
// round), exactly the elements 128 w .. 128 w + 127 (+ 2 T per round),
// whatever j: consecutive such stages touch only the wave's own elements, so
// a wave-level boundary (its LDS operations complete, in order) suffices; a
// stage crossing waves (j > 64) and the one after it need the workgroup
// barrier.  In LDS this drops ~4/5 of the barriers (N = 4096: 15 of 78
// stages keep one).  Global scratch (oversized buckets) keeps every barrier.
template <bool LDS>
__device__ __forceinline__ void bitonic_boundary(int j, int jn) {
    if (!LDS || j > 64 || jn > 64) {
        __syncthreads();
    } else {
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
}
// the partner distance of the stage after (k, j): 0 after the last
__device__ __forceinline__ int bitonic_next_j(int k, int j, int N) { return j > 1 ? j >> 1 : (k < N ? k : 0); }

// (key, value) pairs ascending by (key, value); a / b in LDS or in global
// memory private to the workgroup (one network, instantiated per space)
template <int T, bool LDS, class KP, class VP>
__device__ __forceinline__ void bitonic_kv(KP a, VP b, int N) {
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int p = threadIdx.x; p < (N >> 1); p += T) {
                const int i = bitonic_lo(p, j), l = i + j;
                const uint64_t ka = a[i], kl = a[l];
                const int32_t va = b[i], vl = b[l];
                if (kv_less(kl, vl, ka, va) == ((i & k) == 0)) {
                    a[i] = kl; a[l] = ka;
                    b[i] = vl; b[l] = va;
                }
            }
            const int jn = bitonic_next_j(k, j, N);
            bitonic_boundary<LDS>(j, jn == 0 ? (1 << 30) : jn);   // after the last stage: the workgroup barrier
        }
    }
}

// keys ascending (LDS)
template <int T>
__device__ __forceinline__ void bitonic_k(uint64_t *a, int N) {
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int p = threadIdx.x; p < (N >> 1); p += T) {
                const int i = bitonic_lo(p, j), l = i + j;
                const uint64_t ka = a[i], kl = a[l];
                if ((kl < ka) == ((i & k) == 0)) { a[i] = kl; a[l] = ka; }
            }
            const int jn = bitonic_next_j(k, j, N);
            bitonic_boundary<true>(j, jn == 0 ? (1 << 30) : jn);
        }
    }
}

// P splitters: CS_OVS x P samples of the keys at equal steps of the previous
// order, sorted; every CS_OVS-th.  The previous order keeps the coarse Morton
// cells in place, but inside a dense cell the order is new every iteration
// (the box moves its deep cell boundaries), so the samples there are random
// ones: 4x oversampling keeps the buckets within ~3.3x of their mean on the
// C3 snapshots (max 3290 of 1024 at t = 650, CS_CAP 4096).
//
// Two launches over CS_RUNS compute units instead of one workgroup's 4096-entry
// network (LDS-bound on one CU, 47 us at n = 1M): cs_split_runs sorts CS_RUNS
// runs of <= CS_RUN samples, one workgroup each (at n = 1M: 488); cs_split_rank places every
// sample at its rank in the merged order (its index in its run + the entries
// before it in every other run: binary searches, equal keys ordered by run)
// and keeps the ranks that are multiples of CS_OVS -- the same splitters as
// sorting all samples.
constexpr int CS_RUNS = 8;
constexpr int CS_RUN = CS_OVS * CS_PMAX / CS_RUNS;   // 512 samples per run at most
constexpr int CS_RANK_T = 256;

__global__ __launch_bounds__(CS_RUN / 2) void cs_split_runs(const uint64_t *__restrict__ keys,
                                                            const int32_t *__restrict__ prev, int64_t n, int32_t P,
                                                            uint64_t *__restrict__ runs) {
    __shared__ uint64_t s[CS_RUN];
    const int S = CS_OVS * P, L = (S + CS_RUNS - 1) / CS_RUNS;
    const int j0 = blockIdx.x * L, m = max(0, min(S, j0 + L) - j0);
    int N = 2;
    while (N < L) N <<= 1;
    int32_t pi[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int i = threadIdx.x + (CS_RUN / 2) * e;
        pi[e] = i < m ? prev[(int64_t)(j0 + i) * n / S] : 0;
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int i = threadIdx.x + (CS_RUN / 2) * e;
        if (i < N) s[i] = i < m ? keys[pi[e]] : ~0ull;
    }
    __syncthreads();
    bitonic_k<CS_RUN / 2>(s, N);
    for (int i = threadIdx.x; i < m; i += CS_RUN / 2) runs[blockIdx.x * CS_RUN + i] = s[i];
}

__global__ __launch_bounds__(CS_RANK_T) void cs_split_rank(const uint64_t *__restrict__ runs, int32_t P,
                                                           uint64_t *__restrict__ split) {
    __shared__ uint64_t s[CS_RUNS * CS_RUN];
    const int S = CS_OVS * P, L = (S + CS_RUNS - 1) / CS_RUNS;
    for (int i = threadIdx.x; i < CS_RUNS * CS_RUN; i += CS_RANK_T) {
        const int r = i / CS_RUN, k = i - r * CS_RUN;
        if (r * L + k < S && k < L) s[i] = runs[i];
    }
    __syncthreads();
    const int j = blockIdx.x * CS_RANK_T + threadIdx.x;
    if (j >= S) return;
    const int r = j / L, i = j - r * L;
    const uint64_t x = s[r * CS_RUN + i];
    int rank = i;
    for (int q = 0; q < CS_RUNS; ++q) {
        if (q == r) continue;
        const int m = max(0, min(S, q * L + L) - q * L);
        const uint64_t *a = s + q * CS_RUN;
        int lo = 0, hi = m;   // entries of run q before x: keys < x, or <= x for an earlier run
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (q < r ? a[mid] <= x : a[mid] < x) lo = mid + 1;
            else hi = mid;
        }
        rank += lo;
    }
    if (rank % CS_OVS == 0) split[rank / CS_OVS] = x;
}

// bucket of key k: the number of splitters split[1..P-1] <= k; guess g first
// (the bucket the previous order puts element j in)
__device__ __forceinline__ int cs_find(const uint64_t *__restrict__ split, int32_t P, uint64_t k, int g) {
    if ((g == 0 || split[g] <= k) && (g == P - 1 || k < split[g + 1])) return g;
    int lo = 0, hi = P - 1;   // answer in [lo, hi]
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (split[mid] <= k) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ __launch_bounds__(CS_BLK) void cs_count(const uint64_t *__restrict__ keys, const int32_t *__restrict__ prev,
                                                   int64_t n, int32_t P, const uint64_t *__restrict__ split,
                                                   int32_t *__restrict__ bkt, int32_t *__restrict__ cnt) {
    __shared__ int32_t h[CS_PMAX];
    for (int b = threadIdx.x; b < P; b += CS_BLK) h[b] = 0;
    __syncthreads();
    const int64_t j = (int64_t)blockIdx.x * CS_BLK + threadIdx.x;
    if (j < n) {
        const uint64_t k = keys[prev[j]];
        const int b = cs_find(split, P, k, (int)(j * P / n));
        bkt[j] = b;
        atomicAdd(&h[b], 1);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < P; b += CS_BLK)
        if (h[b]) atomicAdd(&cnt[b], h[b]);
}

// exclusive scan of the bucket sizes -> off[0..P], cur = off; stat[0] = oversized buckets
__global__ __launch_bounds__(1024) void cs_scan(const int32_t *__restrict__ cnt, int32_t P, int32_t *__restrict__ off,
                                                int32_t *__restrict__ cur, int32_t *__restrict__ stat) {
    __shared__ int32_t s[1024];
    __shared__ int32_t nover;
    const int t = threadIdx.x;
    if (t == 0) nover = 0;
    const int per = (P + 1023) / 1024;   // <= 2
    int loc[2] = {0, 0}, sum = 0;
    for (int e = 0; e < per; ++e) {
        const int b = t * per + e;
        loc[e] = b < P ? cnt[b] : 0;
        sum += loc[e];
    }
    s[t] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {   // inclusive Hillis-Steele scan
        const int v = t >= d ? s[t - d] : 0;
        __syncthreads();
        s[t] += v;
        __syncthreads();
    }
    int run = s[t] - sum;
    for (int e = 0; e < per; ++e) {
        const int b = t * per + e;
        if (b < P) {
            off[b] = run;
            cur[b] = run;
            if (loc[e] > CS_CAP) atomicAdd(&nover, 1);
        }
        run += loc[e];
    }
    if (t == 1023) off[P] = s[1023];
    __syncthreads();
    if (t == 0) { stat[0] = nover; stat[1] += nover; }   // the last sort's, and the running total
}

__global__ __launch_bounds__(CS_BLK) void cs_scatter(const uint64_t *__restrict__ keys, const int32_t *__restrict__ prev,
                                                     int64_t n, int32_t P, const int32_t *__restrict__ bkt,
                                                     int32_t *__restrict__ cur, uint64_t *__restrict__ kb,
                                                     int32_t *__restrict__ vb) {
    __shared__ int32_t h[CS_PMAX], base[CS_PMAX];
    for (int b = threadIdx.x; b < P; b += CS_BLK) h[b] = 0;
    __syncthreads();
    const int64_t j = (int64_t)blockIdx.x * CS_BLK + threadIdx.x;
    int b = 0, r = 0;
    if (j < n) {
        b = bkt[j];
        r = atomicAdd(&h[b], 1);   // rank within this workgroup's share of the bucket (any order: sorted below)
    }
    __syncthreads();
    for (int c = threadIdx.x; c < P; c += CS_BLK)
        if (h[c]) base[c] = atomicAdd(&cur[c], h[c]);
    __syncthreads();
    if (j < n) {
        const int32_t p = prev[j];
        const int32_t slot = base[b] + r;
        kb[slot] = keys[p];
        vb[slot] = p;
    }
}

// One workgroup per bucket: its (key, point) pairs sorted and written to the
// output at the bucket's offset.  Over CS_CAP: the same bitonic network in
// the bucket's private scratch (kb / vb + n + 2 off: disjoint, N <= 2 m).
__global__ __launch_bounds__(CS_SORT_T) void cs_bucket(const int32_t *__restrict__ cnt, const int32_t *__restrict__ off,
                                                       int64_t n, uint64_t *kb, int32_t *vb,
                                                       uint64_t *__restrict__ keys_sorted,
                                                       int32_t *__restrict__ idx_sorted) {
    __shared__ uint64_t sk[CS_CAP];
    __shared__ int32_t sv[CS_CAP];
    const int b = blockIdx.x;
    const int m = cnt[b], o = off[b];
    if (m == 0) return;
    int N = 2;
    while (N < m) N <<= 1;
    if (m <= CS_CAP) {   // LDS (its own instantiation: ds_ instructions, not flat ones)
        for (int i = threadIdx.x; i < N; i += CS_SORT_T) {
            sk[i] = i < m ? kb[o + i] : ~0ull;
            sv[i] = i < m ? vb[o + i] : INT32_MAX;
        }
        __syncthreads();
        bitonic_kv<CS_SORT_T, true>(sk, sv, N);
        for (int i = threadIdx.x; i < m; i += CS_SORT_T) {
            keys_sorted[o + i] = sk[i];
            idx_sorted[o + i] = sv[i];
        }
    } else {
        uint64_t *a = kb + n + 2 * (int64_t)o;
        int32_t *v = vb + n + 2 * (int64_t)o;
        for (int i = threadIdx.x; i < N; i += CS_SORT_T) {
            a[i] = i < m ? kb[o + i] : ~0ull;
            v[i] = i < m ? vb[o + i] : INT32_MAX;
        }
        __syncthreads();
        bitonic_kv<CS_SORT_T, false>(a, v, N);
        for (int i = threadIdx.x; i < m; i += CS_SORT_T) {
            keys_sorted[o + i] = a[i];
            idx_sorted[o + i] = v[i];
        }
    }
}

}  // namespace

void csort_alloc(tsne_ctx *ctx, CoherentSort &cs, int64_t n, const std::string &pre) {
    cs.n = n;
    cs.P = 0;
    if (n < CSORT_MIN_N || n > CSORT_MAX_N) return;   // rocPRIM's sort
    cs.P = (int32_t)std::min<int64_t>(CS_PMAX, std::max<int64_t>(2, n / CS_TARGET));
    Workspace &ws = ctx->ws;
    cs.split = ws.get<uint64_t>(pre + "cs.split", cs.P);
    cs.runs = ws.get<uint64_t>(pre + "cs.runs", CS_RUNS * CS_RUN);
    cs.cnt = ws.get<int32_t>(pre + "cs.cnt", cs.P);
    cs.off = ws.get<int32_t>(pre + "cs.off", cs.P + 1);
    cs.cur = ws.get<int32_t>(pre + "cs.cur", cs.P);
    cs.bkt = ws.get<int32_t>(pre + "cs.bkt", n);
    cs.kb = ws.get<uint64_t>(pre + "cs.kb", 3 * (size_t)n);
    cs.vb = ws.get<int32_t>(pre + "cs.vb", 3 * (size_t)n);
    cs.stat = ws.get<int32_t>(pre + "cs.stat", 2);
    TSNE_HIP(hipMemsetAsync(cs.stat, 0, 2 * sizeof(int32_t), ctx->stream));
}

int64_t csort_oversized(tsne_ctx *ctx, const CoherentSort &cs, bool total) {
    if (cs.P <= 0 || !cs.stat) return 0;
    int32_t h = 0;
    TSNE_HIP(hipMemcpyAsync(&h, cs.stat + (total ? 1 : 0), sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    TSNE_HIP(hipStreamSynchronize(ctx->stream));
    return h;
}

void csort_run(tsne_ctx *ctx, CoherentSort &cs, const uint64_t *keys, const int32_t *prev, uint64_t *keys_sorted,
               int32_t *idx_sorted, hipStream_t st) {
    (void)ctx;
    TSNE_REQUIRE(cs.P > 0, "coherent sort not allocated");
    const int64_t n = cs.n;
    const int64_t nb = ceil_div(n, CS_BLK);
    hipLaunchKernelGGL(cs_split_runs, dim3(CS_RUNS), dim3(CS_RUN / 2), 0, st, keys, prev, n, cs.P, cs.runs);
    hipLaunchKernelGGL(cs_split_rank, dim3(ceil_div(CS_OVS * cs.P, CS_RANK_T)), dim3(CS_RANK_T), 0, st, cs.runs, cs.P,
                       cs.split);
    TSNE_HIP(hipMemsetAsync(cs.cnt, 0, sizeof(int32_t) * cs.P, st));
    hipLaunchKernelGGL(cs_count, dim3(nb), dim3(CS_BLK), 0, st, keys, prev, n, cs.P, cs.split, cs.bkt, cs.cnt);
    hipLaunchKernelGGL(cs_scan, dim3(1), dim3(1024), 0, st, cs.cnt, cs.P, cs.off, cs.cur, cs.stat);
    hipLaunchKernelGGL(cs_scatter, dim3(nb), dim3(CS_BLK), 0, st, keys, prev, n, cs.P, cs.bkt, cs.cur, cs.kb, cs.vb);
    hipLaunchKernelGGL(cs_bucket, dim3(cs.P), dim3(CS_SORT_T), 0, st, cs.cnt, cs.off, n, cs.kb, cs.vb, keys_sorted,
                       idx_sorted);
    TSNE_LAUNCH_CHECK();
}

}  // namespace tsne
