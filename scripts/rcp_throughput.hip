#include <hip/hip_runtime.h>
#include <cstdio>
// Throughput of reciprocal variants on fp64: 8 independent chains per lane.
template <int V>
__global__ void k(double *out, int iters) {
    double x[8];
    for (int c = 0; c < 8; ++c) x[c] = 1.0 + 1e-3 * (threadIdx.x + c);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const double d = 1.0 + x[c];
            double r;
            if (V == 0) {   // v_rcp_f64 + 1 Newton
                r = __builtin_amdgcn_rcp(d);
                r = __fma_rn(r, __fma_rn(-d, r, 1.0), r);
            } else if (V == 1) {   // f32 rcp seed + 2 Newton in f64
                r = (double)__builtin_amdgcn_rcpf((float)d);
                r = __fma_rn(r, __fma_rn(-d, r, 1.0), r);
                r = __fma_rn(r, __fma_rn(-d, r, 1.0), r);
            } else if (V == 2) {   // v_rcp_f64 alone
                r = __builtin_amdgcn_rcp(d);
            } else {   // 2 fma (baseline)
                r = __fma_rn(d, 0.5, 0.25);
                r = __fma_rn(r, 0.5, 0.25);
            }
            x[c] = r;
        }
    }
    double s = 0; for (int c = 0; c < 8; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
    double *o; hipMalloc(&o, 8 * 256 * 1024 * 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int iters = 4000, blocks = 256 * 4;
    for (int v = 0; v < 4; ++v) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            if (v == 0) k<0><<<blocks, 256>>>(o, iters);
            if (v == 1) k<1><<<blocks, 256>>>(o, iters);
            if (v == 2) k<2><<<blocks, 256>>>(o, iters);
            if (v == 3) k<3><<<blocks, 256>>>(o, iters);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            const double ops = (double)blocks * 256 * iters * 8;
            if (rep) printf("variant %d: %.3f ms, %.2f G recips/s\n", v, ms, ops / ms / 1e6);
        }
    }
}
