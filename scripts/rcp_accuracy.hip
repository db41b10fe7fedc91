// Accuracy of v_rcp_f64 (+ Newton steps) against IEEE division on gfx950,
// over x = 1 + D, D in [0, 1e8) log-uniform (the BH pair term's range).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>

__global__ void k(int64_t n, unsigned long long *maxulp) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
    double u = (double)(h >> 11) * 0x1.0p-53;
    double D = pow(10.0, -12.0 + 20.0 * u);
    double x = 1.0 + D;
    double e = 1.0 / x;
    double r0 = __builtin_amdgcn_rcp(x);
    double r1 = fma(r0, fma(-x, r0, 1.0), r0);
    double r2 = fma(r1, fma(-x, r1, 1.0), r1);
    long long b = __double_as_longlong(e);
    unsigned long long d0 = llabs(__double_as_longlong(r0) - b);
    unsigned long long d1 = llabs(__double_as_longlong(r1) - b);
    unsigned long long d2 = llabs(__double_as_longlong(r2) - b);
    atomicMax(&maxulp[0], d0); atomicMax(&maxulp[1], d1); atomicMax(&maxulp[2], d2);
}

int main() {
    unsigned long long *d, h[3] = {0, 0, 0};
    hipMalloc(&d, sizeof(h));
    hipMemset(d, 0, sizeof(h));
    int64_t n = 1 << 26;
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, n, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("max ulp vs IEEE 1/x: rcp %llu, rcp+1NR %llu, rcp+2NR %llu\n", h[0], h[1], h[2]);
    return 0;
}
