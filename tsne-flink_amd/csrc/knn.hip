// knn.hip -- brute-force kNN (TsneHelpers.scala:41-59) on gfx950.
//
// The reference crosses all N^2 pairs, filters i != j, sorts each group by
// the fp64 breeze metric and keeps the first k.  Here:
//   1. prep:   centre X (or L2-normalise for cosine) and round to fp32, with
//              fp32 squared norms; rows padded to a multiple of 32 columns.
//   2. filter: MFMA fp32 tiles (v_mfma_f32_32x32x2_f32) compute
//              d32 = |q|^2 + |c|^2 - 2 q.c for a 128x128 (query x candidate)
//              tile staged through LDS; every pair with d32 <= tau_q (the
//              query's running threshold) is appended to the query's
//              candidate buffer.  The N x N matrix is never materialised.
//              Candidates are swept in doubling ranges; after each range a
//   3. compact kernel (one wave per query) radix-selects the kk-th smallest
//              d32, sets tau_q = kth + 2*delta_q and drops everything above.
//              delta_q is a rigorous bound on |d32 - d64| (fp32 rounding of
//              the inputs, the K-term fp32 FMA chain, the final add), so the
//              buffer always holds every j whose exact distance can be in the
//              top kk -- including exact ties at the k-th distance.
//   4. rerank: one wave per query recomputes the surviving candidates with
//              the exact breeze fp64 metric (sequential sum, no FMA
//              contraction) and bitonic-sorts them by (d, j) in LDS.
//   5. fallback: a query whose buffer overflows (only pathological crowds of
//              near-equal distances, e.g. many duplicate points) is redone by
//              an exact fp64 scan + stable radix sort.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace tsne {
namespace {

constexpr int TQ = 128;   // queries per workgroup tile
constexpr int TC = 128;   // candidates per workgroup tile
constexpr int KC = 32;    // k-chunk staged in LDS
constexpr int LDSW = KC + 1;  // padded LDS row (bank-conflict free column reads)

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));   // 8 bf16: one 32x32x16 MFMA operand fragment
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// bf16x3 filter tiles (knn_filter_glds): 256 queries x 256 candidates per
// 1024-thread workgroup, dims staged 32 at a time (two 16-deep MFMA steps).
constexpr int FT = 256;
constexpr int FK = 32;
constexpr int FTPB = 8;        // candidate tiles per workgroup (cross-tile prefetch)
constexpr int FSQ = 64, FSC = 4;   // super-tile: query tiles x candidate groups

// ---------------------------------------------------------------- prep
// Column partial sums for the mean (deterministic two-level reduction).
__global__ void colsum_partial(const double *__restrict__ X, int64_t n, int32_t d,
                               int64_t rows_per_block, double *__restrict__ part) {
    const int64_t r0 = blockIdx.x * rows_per_block;
    const int64_t r1 = min(n, r0 + rows_per_block);
    for (int32_t c = threadIdx.x; c < d; c += blockDim.x) {
        double s = 0.0;
        for (int64_t r = r0; r < r1; ++r) s += X[r * d + c];
        part[(int64_t)blockIdx.x * d + c] = s;
    }
}

__global__ void colsum_final(const double *__restrict__ part, int64_t nblocks, int32_t d,
                             int64_t n, double *__restrict__ mean) {
    for (int32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < d; c += gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int64_t b = 0; b < nblocks; ++b) s += part[b * d + c];
        mean[c] = s / (double)n;
    }
}

// One wave per row: X32 = fp32(x - mean) (or fp32(x / |x|) for cosine),
// norm32 = fp32(sum X32^2) (0.5 for cosine), norm64 = sqrt(sum x^2) fp64
// sequential (cosine rerank).  Rows >= n are zero.
__global__ void prep_rows(const double *__restrict__ X, int64_t n, int32_t d, int32_t dpad,
                          int64_t npad, int32_t metric, const double *__restrict__ mean,
                          float *__restrict__ X32, float *__restrict__ norm32,
                          double *__restrict__ norm64, unsigned int *__restrict__ nmax_bits) {
    const int64_t row = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x / 64);
    const int lane = lane_id();
    if (row >= npad) return;
    float *out = X32 + row * dpad;
    if (row >= n) {
        for (int c = lane; c < dpad; c += 64) out[c] = 0.f;
        if (lane == 0) { norm32[row] = 0.f; norm64[row] = 0.0; }
        return;
    }
    const double *x = X + row * d;
    double scale = 1.0;
    if (metric == TSNE_METRIC_COSINE) {
        if (lane == 0) {  // exact sequential norm, as breeze norm()
            double s = 0.0;
            for (int c = 0; c < d; ++c) s = __dadd_rn(s, __dmul_rn(x[c], x[c]));
            norm64[row] = sqrt(s);
        }
        double s = 0.0;
        for (int c = lane; c < d; c += 64) s += x[c] * x[c];
        s = wave_sum(s);
        scale = s > 0.0 ? 1.0 / sqrt(s) : 0.0;
    }
    double acc = 0.0;
    for (int c = lane; c < dpad; c += 64) {
        float v = 0.f;
        if (c < d) v = (metric == TSNE_METRIC_COSINE) ? (float)(x[c] * scale) : (float)(x[c] - mean[c]);
        out[c] = v;
        acc += (double)v * (double)v;
    }
    acc = wave_sum(acc);
    if (lane == 0) {
        float nv = (metric == TSNE_METRIC_COSINE) ? 0.5f : (float)acc;
        norm32[row] = nv;
        if (metric != TSNE_METRIC_COSINE) norm64[row] = 0.0;
        atomicMax(nmax_bits, __float_as_uint(nv));  // non-negative floats order as uints
    }
}

// fp32 -> bf16, round to nearest even (finite inputs).
__device__ __forceinline__ unsigned short bf16_rn(float f) {
    const uint32_t u = __float_as_uint(f);
    return (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_to_f(unsigned short h) { return __uint_as_float((uint32_t)h << 16); }

// X32 -> (hi, mid) bf16 pair per element: x = hi + mid + e, |e| <= 2^-16 |x|
// (two bf16 roundings of 8 significant bits each).
__global__ void split_bf16(const float *__restrict__ X32, int64_t count, unsigned short *__restrict__ Xh,
                           unsigned short *__restrict__ Xm) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
        const float x = X32[i];
        const unsigned short h = bf16_rn(x);
        Xh[i] = h;
        Xm[i] = bf16_rn(x - bf16_to_f(h));   // exact difference in fp32
    }
}

// ------------------------------------------------------------- filter
// Workgroup = 4 waves in a 2x2 arrangement; wave tile 64x64 = 2x2 MFMA
// 32x32 tiles (64 accumulators per lane).  MODE 0 = dense first pass
// (every candidate written at slot c - c0, self = +inf); MODE 1 = threshold
// filter with wave-aggregated atomic appends.
template <int MODE>
__global__ __launch_bounds__(256) void knn_filter(
    const float *__restrict__ X32, const float *__restrict__ norm32, int32_t dpad,
    int64_t q0, int64_t q1, int64_t c0, int64_t c1, float dot_scale,
    const float *__restrict__ tau, int32_t *__restrict__ cnt, float *__restrict__ cand_d,
    int32_t *__restrict__ cand_j, int32_t *__restrict__ flags, int32_t cap) {
    __shared__ float Qs[TQ * LDSW];
    __shared__ float Cs[TC * LDSW];
    __shared__ float nq_s[TQ], tau_s[TQ], nc_s[TC];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int64_t qb = q0 + (int64_t)blockIdx.y * TQ;   // query tile base (global row)
    const int64_t cb = c0 + (int64_t)blockIdx.x * TC;   // candidate tile base

    if (tid < TQ) {
        int64_t q = qb + tid;
        nq_s[tid] = norm32[q];  // padded arrays: q < npad always
        tau_s[tid] = (MODE == 1 && q < q1) ? tau[q - q0] : 0.f;
    } else {
        int64_t c = cb + (tid - TQ);
        nc_s[tid - TQ] = norm32[c];
    }

    floatx16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

    // K chunks of 32 staged through LDS; the next chunk's global loads are
    // issued into registers before the current chunk's MFMAs (software
    // pipelining: the loads' latency hides behind the matrix work).
    float4 pq[4], pc[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int idx = tid + it * 256;
        const int r = idx >> 3, c4 = (idx & 7) * 4;
        pq[it] = *reinterpret_cast<const float4 *>(X32 + (qb + r) * dpad + c4);
        pc[it] = *reinterpret_cast<const float4 *>(X32 + (cb + r) * dpad + c4);
    }
    for (int k0 = 0; k0 < dpad; k0 += KC) {
        // stage 128 x 32 of queries and of candidates: 1024 float4 each, 4 per thread
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int idx = tid + it * 256;
            const int r = idx >> 3, c4 = (idx & 7) * 4;
            float *dq = Qs + r * LDSW + c4;
            float *dc = Cs + r * LDSW + c4;
            dq[0] = pq[it].x; dq[1] = pq[it].y; dq[2] = pq[it].z; dq[3] = pq[it].w;
            dc[0] = pc[it].x; dc[1] = pc[it].y; dc[2] = pc[it].z; dc[3] = pc[it].w;
        }
        __syncthreads();
        if (k0 + KC < dpad) {
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                const int idx = tid + it * 256;
                const int r = idx >> 3, c4 = (idx & 7) * 4;
                pq[it] = *reinterpret_cast<const float4 *>(X32 + (qb + r) * dpad + k0 + KC + c4);
                pc[it] = *reinterpret_cast<const float4 *>(X32 + (cb + r) * dpad + k0 + KC + c4);
            }
        }
        const int lr = lane & 31, lk = lane >> 5;
#pragma unroll
        for (int s = 0; s < KC / 2; ++s) {
            const int kk = 2 * s + lk;
            float a0 = Qs[(wr * 64 + lr) * LDSW + kk];
            float a1 = Qs[(wr * 64 + 32 + lr) * LDSW + kk];
            float b0 = Cs[(wc * 64 + lr) * LDSW + kk];
            float b1 = Cs[(wc * 64 + 32 + lr) * LDSW + kk];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        __syncthreads();
    }

    // epilogue: C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
    const int half = lane >> 5, lcol = lane & 31;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti) {
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
            const int lc = wc * 64 + tj * 32 + lcol;
            const int64_t c = cb + lc;
            const float ncv = nc_s[lc];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int lrow = wr * 64 + ti * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                const int64_t q = qb + lrow;
                float dv = nq_s[lrow] + ncv - dot_scale * acc[ti][tj][r];
                if (MODE == 0) {
                    if (q < q1 && c < c1) {
                        float w = (c == q) ? __builtin_inff() : dv;
                        int64_t o = (q - q0) * (int64_t)cap + (c - c0);
                        cand_d[o] = w;
                        cand_j[o] = (int32_t)c;
                    }
                } else {
                    bool ok = (q < q1) && (c < c1) && (c != q) && (dv <= tau_s[lrow]);
                    uint64_t m = __ballot(ok);
                    if (m) {
                        uint32_t mine = half ? (uint32_t)(m >> 32) : (uint32_t)m;
                        int leader = __ffs(mine) - 1;  // -1 if none in this half
                        int base = 0;
                        if (ok && lcol == leader) base = atomicAdd(&cnt[q - q0], __popc(mine));
                        base = __shfl(base, (half << 5) + (leader < 0 ? 0 : leader), 64);
                        if (ok) {
                            int slot = base + __popc(mine & ((1u << lcol) - 1u));
                            if (slot < cap) {
                                int64_t o = (q - q0) * (int64_t)cap + slot;
                                cand_d[o] = dv;
                                cand_j[o] = (int32_t)c;
                            } else {
                                flags[q - q0] = 1;
                            }
                        }
                    }
                }
            }
        }
    }
}

// Threshold filter with bf16x3 products (the MFMA rate of bf16 is 16x that
// of the f32-input MFMA): q.c ~ qh.ch + qh.cm + qm.ch over the (hi, mid)
// splits, fp32 accumulation.  The dropped qm.cm and split-residual terms
// are <= 3.02 * 2^-16 |q_k||c_k| each, so |d - d32| grows by at most
// 3.02 * 2^-16 (|q|^2 + |c|^2) (+ the fp32 accumulation of 3K products):
// knn_run's delta_coef covers both, and the exact fp64 re-rank restores
// the exact order -- the filter only decides who is re-ranked.
// Workgroup: 16 waves as 4 (queries) x 4 (candidates), wave tile 64 x 64 =
// 2 x 2 MFMA 32x32 tiles.  The 32-dim stages are copied global -> LDS by the
// LDS DMA (global_load_lds_dwordx4): no staging registers (a register-staged
// form spilled at 4 waves/SIMD, and each spill reload's vmcnt(0) drained the
// prefetch), two LDS stage buffers, stage g+1 issued before stage g is
// waited for.  LDS rows are 64 B with the 16-B slots XOR-swizzled by row
// bits 2..3 (conflict-free ds_read_b128 fragment reads); the DMA writes each
// wave-instruction's 1 KB linearly, so the swizzle is applied to the global
// source address.  One __shared__ array (a second one makes hipcc wait
// vmcnt(0) before LDS reads); barriers are raw s_barrier with an
// lgkmcnt(0) wait only -- __syncthreads() would wait vmcnt(0) too.
constexpr int GROW = 32;                         // bf16 per LDS row
constexpr int GARR = FT * GROW * 2;              // one array of a stage: 16 KB
constexpr int GSTAGE = 4 * GARR;                 // Qh, Qm, Ch, Cm: 64 KB
constexpr int G_NQ = 2 * GSTAGE, G_TAU = G_NQ + FT * 4, G_QOFF = G_TAU + FT * 4, G_NC = G_QOFF + FT * 8;
constexpr int G_THR = G_NC + FTPB * FT * 4, G_LDS = G_THR + FT * 4;   // 141 KB
__device__ __forceinline__ int gslot(int row, int part) { return part ^ ((row >> 2) & 3); }
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

__global__ __launch_bounds__(1024) void knn_filter_glds(
    const unsigned short *__restrict__ Xh, const unsigned short *__restrict__ Xm, const float *__restrict__ norm32,
    int32_t dpad, int64_t q0, int64_t q1, int64_t c0, int64_t c1, float dot_scale, const float *__restrict__ tau,
    int32_t *__restrict__ cnt, float *__restrict__ cand_d, int32_t *__restrict__ cand_j, int32_t *__restrict__ flags,
    int32_t cap, float nmax) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[G_LDS];
    float *nq_s = reinterpret_cast<float *>(lds + G_NQ);
    float *thr_s = reinterpret_cast<float *>(lds + G_THR);
    float *tau_s = reinterpret_cast<float *>(lds + G_TAU);
    int64_t *qoff_s = reinterpret_cast<int64_t *>(lds + G_QOFF);
    float *nc_s = reinterpret_cast<float *>(lds + G_NC);
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    // Super-tile raster over a 1-D grid: FSQ query tiles x FSC candidate
    // groups per super-tile, query tile fastest (the XCD = block % 8 keeps
    // neighbouring query tiles' candidate stages in its L2)
    const int64_t nqt = (q1 - q0 + FT - 1) / FT;
    const int64_t ncg = (c1 - c0 + (int64_t)FT * FTPB - 1) / ((int64_t)FT * FTPB);
    const int64_t nqt_pad = (nqt + FSQ - 1) / FSQ * FSQ;
    const int64_t bid = blockIdx.x, sts = (int64_t)FSQ * FSC;
    const int64_t stn = bid / sts, inner = bid % sts, nst_q = nqt_pad / FSQ;
    const int64_t qt = (stn % nst_q) * FSQ + inner % FSQ, cg = (stn / nst_q) * FSC + inner / FSQ;
    if (qt >= nqt || cg >= ncg) return;
    const int64_t qb = q0 + qt * FT;
    const int64_t cfirst = c0 + cg * FTPB * FT;
    const int ntile = (int)min<int64_t>(FTPB, (c1 - cfirst + FT - 1) / FT);
    const int qlim = (int)min<int64_t>(FT, q1 - qb), qi0 = (int)(qb - q0);
    if (tid < FT) {
        const int64_t q = qb + tid;
        const float nq = norm32[q], t = q < q1 ? tau[q - q0] : 0.f;
        nq_s[tid] = nq;
        tau_s[tid] = t;
        qoff_s[tid] = (q - q0) * (int64_t)cap;
        // screening threshold of the epilogue: fma(-s, dot, |c|^2) <= thr
        // holds whenever the exact test (|q|^2 + |c|^2) - s dot <= tau does.
        // The two differ by the roundings of |q|^2 + |c|^2, s dot, their
        // difference, the fma and tau - |q|^2: at most 4 u (|tau| + |q|^2 +
        // max |c|^2) (|s dot| <= |q|^2 + |c|^2); 2^-19 is 8x that.
        thr_s[tid] = tid < qlim ? (t - nq) + 1.9073486328125e-06f * (fabsf(t) + nq + nmax) : -__builtin_inff();
    }
    for (int i = tid; i < ntile * FT; i += 1024) nc_s[i] = norm32[cfirst + i];
    __syncthreads();   // nothing in flight yet
    // this wave's DMA share of a stage: array ga, rows grb .. grb + 63 (4 x 16 rows)
    const int ga = wave >> 2, grb = (wave & 3) * 64;
    const unsigned short *gsrc = (ga & 1) ? Xm : Xh;
    const int nks = dpad / FK, nstage = ntile * nks;

    // The DMA is inline asm: seen by the compiler, an LDS DMA in flight
    // makes it wait vmcnt(0) before every LDS access (it cannot tell the
    // two stage buffers apart), draining the prefetch.  The wait for it is
    // therefore explicit: vmcnt(4) = this wave's stage-g copies (stage
    // g+1's four are the newer ones), then the barrier for the other waves'.
    const uint32_t lds0 = lds_addr(lds);
    auto issue = [&](int g, int ln) {   // stage g -> LDS buffer g & 1
        const int drow = ln >> 2, dslot = ln & 3;
        const int it = g / nks, k0 = (g - it * nks) * FK;
        const int64_t rbase = ga < 2 ? qb : cfirst + (int64_t)it * FT;
        const uint32_t dst = lds0 + (uint32_t)((g & 1) * GSTAGE + ga * GARR + grb * (GROW * 2));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int R = grb + i * 16 + drow;
            const uint32_t e = (uint32_t)(rbase + R) * (uint32_t)dpad + (uint32_t)(k0 + 8 * gslot(R, dslot));
            const uint64_t src = (uint64_t)(uintptr_t)(gsrc + e);
            const uint32_t m0v = __builtin_amdgcn_readfirstlane(dst + i * 1024);
            asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(src), "s"(m0v) : "memory");
        }
    };
    issue(0, lane);
    for (int it = 0; it < ntile; ++it) {
    floatx16 acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int nn = 0; nn < 2; ++nn)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][nn][r] = 0.f;
    for (int kstage = 0; kstage < nks; ++kstage) {
        const int g = it * nks + kstage;
        // lane-derived addresses are recomputed from an opaque copy of the
        // lane id every stage: hoisted out of the loop they would stay live
        // beside the 64 accumulators and spill (each spill reload's
        // compiler-inserted vmcnt(0) would drain the stage prefetch)
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int lr = ln & 31, lh = ln >> 5;
        if (g + 1 < nstage) {
            issue(g + 1, ln);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // this wave's stage-g copies landed
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_barrier" ::: "memory");                // every wave's stage-g copies landed
        // fragment reads are ordinary LDS loads (the compiler tracks their
        // lgkmcnt waits and the MFMA source hazards; it cannot see the DMA,
        // so it inserts no vmcnt for it -- the asm waits above order them)
        const unsigned short *sb = reinterpret_cast<const unsigned short *>(lds + (g & 1) * GSTAGE);
#pragma unroll
        for (int stp = 0; stp < 2; ++stp) {
            const int part = 2 * stp + lh;
            const int c0r = wc * 64 + lr, c1r = c0r + 32;
            const int co0 = 2 * FT * GROW + c0r * GROW + 8 * gslot(c0r, part);
            const int co1 = 2 * FT * GROW + c1r * GROW + 8 * gslot(c1r, part);
            const bf16x8 bh0 = *reinterpret_cast<const bf16x8 *>(sb + co0);
            const bf16x8 bm0 = *reinterpret_cast<const bf16x8 *>(sb + co0 + FT * GROW);
            const bf16x8 bh1 = *reinterpret_cast<const bf16x8 *>(sb + co1);
            const bf16x8 bm1 = *reinterpret_cast<const bf16x8 *>(sb + co1 + FT * GROW);
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const int qrow = wr * 64 + m * 32 + lr;
                const int qo = qrow * GROW + 8 * gslot(qrow, part);
                const bf16x8 ah = *reinterpret_cast<const bf16x8 *>(sb + qo);
                const bf16x8 am = *reinterpret_cast<const bf16x8 *>(sb + qo + FT * GROW);
                acc[m][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh0, acc[m][0], 0, 0, 0);
                acc[m][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm0, acc[m][0], 0, 0, 0);
                acc[m][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh0, acc[m][0], 0, 0, 0);
                acc[m][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh1, acc[m][1], 0, 0, 0);
                acc[m][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm1, acc[m][1], 0, 0, 0);
                acc[m][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh1, acc[m][1], 0, 0, 0);
            }
        }
        // every wave is done reading buffer g & 1 before stage g + 2 is copied into it
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
        // epilogue of candidate tile it.  Screening: one fma and one compare
        // per element against the row's thr_s (a superset of the exact
        // test); only a wave with a screened element runs the exact test
        // and the candidate append (rare: a few in 10^4 elements).
        const int64_t cb = cfirst + (int64_t)it * FT;
        const float *ncb = nc_s + it * FT;
        const int clim = (int)min<int64_t>(FT, c1 - cb);
        const int64_t dqc = qb - cb;
        const int dself = (dqc > -FT && dqc < FT) ? (int)dqc : (1 << 20);
        // lane-derived row / column bases from an opaque lane id: otherwise
        // they are hoisted out of the tile loop and spilled (and the spill
        // reload's vmcnt(0) waits for the next tile's first stage)
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int lh = ln >> 5, lr = ln & 31;
        const int rbase = wr * 64 + 4 * lh, cbase = wc * 64 + lr;
        float cv[2];
#pragma unroll
        for (int nn = 0; nn < 2; ++nn) {
            const int lc = cbase + nn * 32;
            cv[nn] = lc < clim ? ncb[lc] : __builtin_inff();
        }
#pragma unroll
        for (int m = 0; m < 2; ++m) {
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                const float4 th4 = *reinterpret_cast<const float4 *>(thr_s + rbase + m * 32 + 8 * rq);
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4) {
                    const int r = 4 * rq + r4;
                    const float th = r4 == 0 ? th4.x : r4 == 1 ? th4.y : r4 == 2 ? th4.z : th4.w;
#pragma unroll
                    for (int nn = 0; nn < 2; ++nn) {
                        const float a = acc[m][nn][r];
                        if (__builtin_expect(__ballot(__builtin_fmaf(-dot_scale, a, cv[nn]) <= th) != 0, 0)) {
                            // bases re-made opaque inside the branch: nothing
                            // of this cold path is computed ahead of the test
                            int rb = rbase, cbs = cbase;
                            asm volatile("" : "+v"(rb), "+v"(cbs));
                            const int lrow = rb + m * 32 + (r & 3) + 8 * (r >> 2);
                            const int lc = cbs + nn * 32;
                            const float dv = nq_s[lrow] + ncb[lc] - dot_scale * a;
                            const bool ok = lrow < qlim && lc < clim && lc != lrow + dself && dv <= tau_s[lrow];
                            const uint64_t msk = __ballot(ok);
                            const uint32_t mine = lh ? (uint32_t)(msk >> 32) : (uint32_t)msk;
                            const int leader = __ffs(mine) - 1;
                            int base = 0;
                            if (ok && lr == leader) base = atomicAdd(&cnt[qi0 + lrow], __popc(mine));
                            base = __shfl(base, (lh << 5) + (leader < 0 ? 0 : leader), 64);
                            if (ok) {
                                const int slot = base + __popc(mine & ((1u << lr) - 1u));
                                if (slot < cap) {
                                    const int64_t o = qoff_s[lrow] + slot;
                                    cand_d[o] = dv;
                                    cand_j[o] = (int32_t)(cb + lc);
                                } else {
                                    flags[qi0 + lrow] = 1;
                                }
                            }
                        }
                    }
                }
            }
        }
    }
}

// ------------------------------------------------------------- compact
// One wave per query: radix-select the kk-th smallest d32 among the first
// min(cnt, CAP) entries, tau = kth + 2 delta, keep entries <= tau in place.
template <int CAP>
__global__ __launch_bounds__(256) void knn_compact(
    int64_t nq, int32_t kk, const float *__restrict__ norm32, int64_t q0, float nmax,
    float delta_coef, float *__restrict__ tau, int32_t *__restrict__ cnt,
    float *__restrict__ cand_d, int32_t *__restrict__ cand_j, int32_t *__restrict__ flags) {
    constexpr int R = CAP / 64;
    __shared__ unsigned int hist_s[4][256];
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const int64_t qi = (int64_t)blockIdx.x * 4 + w;
    if (qi >= nq) return;
    unsigned int *hist = hist_s[w];
    if (flags[qi]) { if (lane == 0) tau[qi] = -__builtin_inff(); return; }
    const int m = min(cnt[qi], CAP);
    float *bd = cand_d + qi * CAP;
    int32_t *bj = cand_j + qi * CAP;
    float dv[R];
    int32_t jv[R];
    uint32_t key[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int e = r * 64 + lane;
        dv[r] = e < m ? bd[e] : __builtin_inff();
        jv[r] = e < m ? bj[e] : 0;
        key[r] = e < m ? fkey(dv[r]) : 0xFFFFFFFFu;
    }
    float t;
    if (m < kk) {
        t = __builtin_inff();
    } else {
        uint32_t prefix = 0, pmask = 0;
        int rank = kk;  // 1-based rank of the wanted element
        for (int shift = 24; shift >= 0; shift -= 8) {
            for (int b = lane; b < 256; b += 64) hist[b] = 0;
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < R; ++r)
                if ((key[r] & pmask) == prefix && (r * 64 + lane) < m)
                    atomicAdd(&hist[(key[r] >> shift) & 255u], 1u);
            __builtin_amdgcn_wave_barrier();
            unsigned int h0 = hist[lane * 4], h1 = hist[lane * 4 + 1], h2 = hist[lane * 4 + 2],
                         h3 = hist[lane * 4 + 3];
            unsigned int s = h0 + h1 + h2 + h3, incl = s;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                unsigned int y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            unsigned int excl = incl - s;
            // the lane whose [excl, incl) covers rank
            bool here = (excl < (unsigned)rank) && ((unsigned)rank <= incl);
            uint64_t hm = __ballot(here);
            int src = __ffsll((unsigned long long)hm) - 1;
            int bin = 0;
            unsigned int below = excl;
            if (here) {
                unsigned int acc2 = excl;
                if ((unsigned)rank <= acc2 + h0) { bin = lane * 4; }
                else if ((unsigned)rank <= acc2 + h0 + h1) { bin = lane * 4 + 1; below = acc2 + h0; }
                else if ((unsigned)rank <= acc2 + h0 + h1 + h2) { bin = lane * 4 + 2; below = acc2 + h0 + h1; }
                else { bin = lane * 4 + 3; below = acc2 + h0 + h1 + h2; }
            }
            bin = __shfl(bin, src, 64);
            below = __shfl(below, src, 64);
            prefix |= (uint32_t)bin << shift;
            pmask |= 255u << shift;
            rank -= (int)below;
            __builtin_amdgcn_wave_barrier();
        }
        float kth = fkey_inv(prefix);
        float delta = delta_coef * (norm32[q0 + qi] + nmax);
        t = (kth + 2.0f * delta) * 1.000001f + 1e-30f;
        if (!(t == t)) t = __builtin_inff();
    }
    // compaction in place (all reads are in registers already)
    int out = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        bool keep = (r * 64 + lane) < m && dv[r] <= t;
        uint64_t km = __ballot(keep);
        if (keep) {
            int pos = out + __popcll(km & lanemask_lt());
            bd[pos] = dv[r];
            bj[pos] = jv[r];
        }
        out += __popcll(km);
    }
    if (lane == 0) {
        cnt[qi] = out;
        tau[qi] = t;
        if (out > CAP / 2) { flags[qi] = 1; tau[qi] = -__builtin_inff(); }
    }
}

// -------------------------------------------------------------- rerank
// Exact breeze metric in fp64, sequential over the coordinates (no FMA).
__device__ __forceinline__ double exact_metric(const double *__restrict__ a,
                                               const double *__restrict__ b, int32_t d,
                                               int32_t metric, double na, double nb) {
    if (metric == TSNE_METRIC_COSINE) {
        double s = 0.0;
        for (int32_t t = 0; t < d; ++t) s = __dadd_rn(s, __dmul_rn(a[t], b[t]));
        return 1.0 - s / (na * nb);
    }
    double s = 0.0;
    for (int32_t t = 0; t < d; ++t) {
        double df = __dsub_rn(a[t], b[t]);
        s = __dadd_rn(s, __dmul_rn(df, df));
    }
    return metric == TSNE_METRIC_EUCLIDEAN ? sqrt(s) : s;
}

// One wave per query (WG of 64 threads), bitonic sort of (key(d), j) in LDS.
template <int CAP>
__global__ __launch_bounds__(64) void knn_rerank(
    const double *__restrict__ X, int32_t d, int32_t metric, const double *__restrict__ norm64,
    int64_t q0, int64_t nq, int32_t kk, const int32_t *__restrict__ cnt,
    const float *__restrict__ cand_d, const int32_t *__restrict__ cand_j,
    int32_t *__restrict__ flags, int32_t *__restrict__ out_idx, double *__restrict__ out_dist) {
    __shared__ uint64_t ks[CAP];
    __shared__ int32_t js[CAP];
    __shared__ double ds[CAP];
    const int lane = threadIdx.x;
    const int64_t qi = blockIdx.x;
    if (qi >= nq || flags[qi]) return;
    const int m = min(cnt[qi], CAP);
    if (m < kk) { if (lane == 0) flags[qi] = 1; return; }
    int P = 64;
    while (P < m) P <<= 1;
    const int64_t q = q0 + qi;
    const double *xq = X + q * d;
    const double nqv = norm64[q];
    for (int e = lane; e < P; e += 64) {
        if (e < m) {
            int32_t j = cand_j[qi * CAP + e];
            double dv = exact_metric(xq, X + (int64_t)j * d, d, metric, nqv, norm64[j]);
            ks[e] = dkey(dv);
            js[e] = j;
            ds[e] = dv;
        } else {
            ks[e] = ~0ull;
            js[e] = 0x7FFFFFFF;
            ds[e] = 0.0;
        }
    }
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int e = lane; e < P / 2; e += 64) {
                int lo = 2 * e - (e & (stride - 1));
                int hi = lo + stride;
                bool up = ((lo & size) == 0);
                uint64_t ka = ks[lo], kb = ks[hi];
                int32_t ja = js[lo], jb = js[hi];
                bool gt = (ka > kb) || (ka == kb && ja > jb);
                if (gt == up) {
                    ks[lo] = kb; ks[hi] = ka;
                    js[lo] = jb; js[hi] = ja;
                    double t = ds[lo]; ds[lo] = ds[hi]; ds[hi] = t;
                }
            }
            __syncthreads();
        }
    }
    for (int t = lane; t < kk; t += 64) {
        out_idx[qi * kk + t] = js[t];
        out_dist[qi * kk + t] = ds[t];
    }
}

// ------------------------------------------------------------ fallback
__global__ void fallback_dist(const double *__restrict__ X, int64_t n, int32_t d, int32_t metric,
                              const double *__restrict__ norm64, int64_t q,
                              uint64_t *__restrict__ keys, int32_t *__restrict__ vals,
                              double *__restrict__ dist) {
    int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    double dv = exact_metric(X + q * d, X + j * d, d, metric, norm64[q], norm64[j]);
    keys[j] = (j == q) ? ~0ull : dkey(dv);
    vals[j] = (int32_t)j;
    dist[j] = dv;
}

__global__ void fallback_emit(const uint64_t *__restrict__ keys, const int32_t *__restrict__ vals,
                              const double *__restrict__ dist, int32_t kk,
                              int32_t *__restrict__ out_idx, double *__restrict__ out_dist) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= kk) return;
    int32_t j = vals[t];
    out_idx[t] = j;
    out_dist[t] = dist[j];
}

__global__ void fill_i32(int32_t *p, int64_t n, int32_t v) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}
__global__ void fill_f32(float *p, int64_t n, float v) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

template <int CAP>
void knn_run(tsne_ctx *ctx, const double *dX, int64_t n, int32_t d, int32_t metric, int32_t kk,
             int64_t q0, int64_t q1, int32_t *d_idx, double *d_dist) {
    hipStream_t st = ctx->stream;
    Workspace &ws = ctx->ws;
    const int64_t nq = q1 - q0;
    const int32_t dpad = (int32_t)round_up(d, KC);
    // rows up to the last 256-tile of a candidate range starting anywhere
    const int64_t npad = round_up(n, FT) + FT;
    // bf16x3 threshold passes (Options::knn_bf16 = 0: f32-input MFMA only)
    const int bf_mode = ctx->opts.knn_bf16;
    const bool use_bf = bf_mode != 0 && 2 * npad * (int64_t)round_up(d, KC) < ((int64_t)1 << 31);   // 32-bit offsets

    // --- prep
    double *mean = ws.get<double>("knn.mean", d);
    if (metric != TSNE_METRIC_COSINE) {
        const int64_t rpb = 2048;
        const int64_t nb = ceil_div(n, rpb);
        double *part = ws.get<double>("knn.colpart", (size_t)nb * d);
        hipLaunchKernelGGL(colsum_partial, dim3(nb), dim3(256), 0, st, dX, n, d, rpb, part);
        hipLaunchKernelGGL(colsum_final, dim3(ceil_div(d, 256)), dim3(256), 0, st, part, nb, d, n, mean);
        TSNE_LAUNCH_CHECK();
    }
    float *X32 = ws.get<float>("knn.x32", (size_t)npad * dpad);
    float *norm32 = ws.get<float>("knn.norm32", npad);
    double *norm64 = ws.get<double>("knn.norm64", npad);
    unsigned int *nmax_bits = ws.get<unsigned int>("knn.nmax", 1);
    TSNE_HIP(hipMemsetAsync(nmax_bits, 0, sizeof(unsigned int), st));
    hipLaunchKernelGGL(prep_rows, dim3(ceil_div(npad, 4)), dim3(256), 0, st, dX, n, d, dpad, npad,
                       metric, mean, X32, norm32, norm64, nmax_bits);
    TSNE_LAUNCH_CHECK();
    unsigned short *Xh = nullptr, *Xm = nullptr;
    if (use_bf) {
        Xh = ws.get<unsigned short>("knn.xh", (size_t)npad * dpad);
        Xm = ws.get<unsigned short>("knn.xm", (size_t)npad * dpad);
        hipLaunchKernelGGL(split_bf16, dim3(2048), dim3(256), 0, st, X32, npad * dpad, Xh, Xm);
        TSNE_LAUNCH_CHECK();
    }
    unsigned int nmax_h = 0;
    TSNE_HIP(hipMemcpyAsync(&nmax_h, nmax_bits, sizeof(unsigned int), hipMemcpyDeviceToHost, st));
    TSNE_HIP(hipStreamSynchronize(st));
    float nmax;
    std::memcpy(&nmax, &nmax_h, sizeof(float));
    // |d32 - d64| <= (K + 8) u (|a|^2 + |b|^2) (see header); use K + 32 for slack.
    // bf16x3 passes: + 3.02 * 2^-16 (split) and the fp32 accumulation of 3K
    // products (3.06 K u): 2^-14 + (5K + 64) u covers both.
    const float delta_coef = use_bf ? (float)(6.103515625e-05 + (5.0 * dpad + 64) * 5.9604644775390625e-8)
                                    : (float)((dpad + 32) * 5.9604644775390625e-8);
    const float dot_scale = metric == TSNE_METRIC_COSINE ? 1.0f : 2.0f;

    // --- per-query state
    float *tau = ws.get<float>("knn.tau", nq);
    int32_t *cnt = ws.get<int32_t>("knn.cnt", nq);
    int32_t *flags = ws.get<int32_t>("knn.flags", nq);
    float *cand_d = ws.get<float>("knn.cand_d", (size_t)nq * CAP);
    int32_t *cand_j = ws.get<int32_t>("knn.cand_j", (size_t)nq * CAP);
    TSNE_HIP(hipMemsetAsync(flags, 0, nq * sizeof(int32_t), st));

    const int64_t qtiles = ceil_div(nq, TQ);
    // dense first range
    int64_t s0 = round_up(std::max<int64_t>(kk + 1, 256), TC);
    s0 = std::min<int64_t>(std::min<int64_t>(s0, CAP), n);
    hipLaunchKernelGGL(fill_i32, dim3(ceil_div(nq, 256)), dim3(256), 0, st, cnt, nq, (int32_t)s0);
    // "knn.filter": the MFMA filter launches alone (their sum is the kNN's
    // dense-contraction time, tsne_ctx_stage_ms)
    ctx->timers.reset("knn.filter");
    ctx->timers.begin("knn.filter", st);
    hipLaunchKernelGGL(knn_filter<0>, dim3(ceil_div(s0, TC), qtiles), dim3(256), 0, st, X32, norm32,
                       dpad, q0, q1, (int64_t)0, s0, dot_scale, tau, cnt, cand_d, cand_j, flags,
                       (int32_t)CAP);
    ctx->timers.end("knn.filter", st);
    TSNE_LAUNCH_CHECK();
    auto compact = [&]() {
        hipLaunchKernelGGL(knn_compact<CAP>, dim3(ceil_div(nq, 4)), dim3(256), 0, st, nq, kk, norm32,
                           q0, nmax, delta_coef, tau, cnt, cand_d, cand_j, flags);
        TSNE_LAUNCH_CHECK();
    };
    compact();
    int64_t seen = s0;
    while (seen < n) {
        int64_t r = std::min<int64_t>(seen, n - seen);
        ctx->timers.begin("knn.filter", st);
        if (use_bf)
            hipLaunchKernelGGL(knn_filter_glds,
                               dim3(round_up(ceil_div(nq, FT), FSQ) * round_up(ceil_div(r, (int64_t)FT * FTPB), FSC)),
                               dim3(1024), 0, st, Xh, Xm, norm32, dpad, q0, q1, seen, seen + r, dot_scale, tau, cnt,
                               cand_d, cand_j, flags, (int32_t)CAP, nmax);
        else
            hipLaunchKernelGGL(knn_filter<1>, dim3(ceil_div(r, TC), qtiles), dim3(256), 0, st, X32,
                               norm32, dpad, q0, q1, seen, seen + r, dot_scale, tau, cnt, cand_d,
                               cand_j, flags, (int32_t)CAP);
        ctx->timers.end("knn.filter", st);
        TSNE_LAUNCH_CHECK();
        compact();
        seen += r;
    }
    hipLaunchKernelGGL(knn_rerank<CAP>, dim3(nq), dim3(64), 0, st, dX, d, metric, norm64, q0, nq,
                       kk, cnt, cand_d, cand_j, flags, d_idx, d_dist);
    TSNE_LAUNCH_CHECK();

    // --- exact fallback for flagged queries
    std::vector<int32_t> hflags(nq);
    TSNE_HIP(hipMemcpyAsync(hflags.data(), flags, nq * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    TSNE_HIP(hipStreamSynchronize(st));
    bool any = false;
    for (int64_t i = 0; i < nq && !any; ++i) any = hflags[i] != 0;
    if (!any) return;
    uint64_t *keys = ws.get<uint64_t>("knn.fb_keys", n);
    uint64_t *keys2 = ws.get<uint64_t>("knn.fb_keys2", n);
    int32_t *vals = ws.get<int32_t>("knn.fb_vals", n);
    int32_t *vals2 = ws.get<int32_t>("knn.fb_vals2", n);
    double *dist = ws.get<double>("knn.fb_dist", n);
    size_t tmp_bytes = 0;
    TSNE_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys, keys2, vals, vals2, (int)n, 0, 64, st));
    void *tmp = ws.get<uint8_t>("knn.fb_tmp", tmp_bytes);
    for (int64_t i = 0; i < nq; ++i) {
        if (!hflags[i]) continue;
        hipLaunchKernelGGL(fallback_dist, dim3(ceil_div(n, 256)), dim3(256), 0, st, dX, n, d, metric,
                           norm64, q0 + i, keys, vals, dist);
        TSNE_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys2, vals, vals2, (int)n, 0, 64, st));
        hipLaunchKernelGGL(fallback_emit, dim3(ceil_div(kk, 256)), dim3(256), 0, st, keys2, vals2, dist,
                           kk, d_idx + i * kk, d_dist + i * kk);
        TSNE_LAUNCH_CHECK();
    }
}

}  // namespace

void knn_device(tsne_ctx *ctx, const double *dX, int64_t n, int32_t d, int32_t metric, int32_t k,
                int64_t q0, int64_t q1, int32_t *d_idx, double *d_dist) {
    TSNE_REQUIRE(n >= 2, "kNN needs at least two points");
    TSNE_REQUIRE(d >= 1, "dimension must be positive");
    TSNE_REQUIRE(k >= 1, "k must be positive");
    TSNE_REQUIRE(metric >= 0 && metric <= 2, "unknown metric");
    TSNE_REQUIRE(q0 >= 0 && q1 <= n && q0 <= q1, "query range out of bounds");
    TSNE_REQUIRE(n < (int64_t)INT32_MAX, "n must fit int32 point ids");
    const int32_t kk = (int32_t)std::min<int64_t>(k, n - 1);
    if (q1 == q0) return;
    if (4 * kk + 256 <= 1024)
        knn_run<1024>(ctx, dX, n, d, metric, kk, q0, q1, d_idx, d_dist);
    else if (4 * kk + 512 <= 4096)
        knn_run<4096>(ctx, dX, n, d, metric, kk, q0, q1, d_idx, d_dist);
    else
        fail(TSNE_ERR_UNSUPPORTED, "k too large (max 896)");
}

}  // namespace tsne
