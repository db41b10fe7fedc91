// Microbenchmark of the CSR attraction's memory pattern on gfx950 (diagnostic,
// not product code): 1M rows x ~160 nnz, variants isolate the col/val stream,
// the Y_j gathers and the arithmetic.  Usage: ./attract_micro [n] [deg] [local]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int MODE>   // 0 full, 1 no gather (Y_i), 2 gather only (hashed j), 3 stream only
__global__ __launch_bounds__(256) void attr(const int64_t *__restrict__ rp, const int32_t *__restrict__ col,
                                            const double *__restrict__ val, int64_t n, const double *__restrict__ Y,
                                            double2 *__restrict__ out) {
    const int sub = threadIdx.x & 63;
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (i >= n) return;
    const double2 yi = *reinterpret_cast<const double2 *>(Y + 2 * i);
    double fx = 0, fy = 0;
    const int64_t e1 = rp[i + 1];
    for (int64_t e = rp[i] + sub; e < e1; e += 256) {
        int32_t j[4]; double pv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t o = e + 64 * u; const bool in = o < e1;
            if (MODE == 2) { j[u] = in ? (int32_t)(((uint64_t)o * 2654435761ull) % (uint64_t)n) : (int32_t)i; pv[u] = in ? 1e-9 : 0.0; }
            else { j[u] = in ? col[o] : (int32_t)i; pv[u] = in ? val[o] : 0.0; }
        }
        double jx[4], jy[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (MODE == 1 || MODE == 3) { jx[u] = yi.x + 1e-3 * j[u]; jy[u] = yi.y; }
            else { const double2 yj = *reinterpret_cast<const double2 *>(Y + 2 * (int64_t)j[u]); jx[u] = yj.x; jy[u] = yj.y; }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (MODE == 3) { fx += pv[u] * jx[u]; continue; }
            const double dx = yi.x - jx[u], dy = yi.y - jy[u];
            const double x = 1.0 + (dx * dx + dy * dy);
            double r = __builtin_amdgcn_rcp(x);
            r = __fma_rn(r, __fma_rn(-x, r, 1.0), r);
            r = __fma_rn(r, __fma_rn(-x, r, 1.0), r);
            const double s = pv[u] * r;
            fx += s * dx; fy += s * dy;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { fx += __shfl_xor(fx, o, 64); fy += __shfl_xor(fy, o, 64); }
    if (sub == 0) out[i] = make_double2(fx, fy);
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
    const int deg = argc > 2 ? atoi(argv[2]) : 160;
    const int local = argc > 3 ? atoi(argv[3]) : 0;   // 1: columns within +-2048 of the row
    std::vector<int64_t> rp(n + 1);
    std::vector<int32_t> col((size_t)n * deg);
    std::vector<double> val((size_t)n * deg, 1e-9), Y(2 * n);
    uint64_t h = 88172645463325252ull;
    auto rnd = [&]() { h ^= h << 13; h ^= h >> 7; h ^= h << 17; return h; };
    for (int64_t i = 0; i <= n; ++i) rp[i] = i * deg;
    for (int64_t i = 0; i < n; ++i)
        for (int k = 0; k < deg; ++k) {
            int64_t j = local ? (i + (int64_t)(rnd() % 4096) - 2048) : (int64_t)(rnd() % n);
            if (j < 0) j += n; if (j >= n) j -= n;
            col[i * deg + k] = (int32_t)j;
        }
    for (auto &y : Y) y = (double)(rnd() % 1000000) * 1e-5;
    int64_t *drp; int32_t *dcol; double *dval, *dY; double2 *dout;
    CK(hipMalloc(&drp, 8 * (n + 1))); CK(hipMalloc(&dcol, 4 * col.size())); CK(hipMalloc(&dval, 8 * val.size()));
    CK(hipMalloc(&dY, 8 * Y.size())); CK(hipMalloc(&dout, 16 * n));
    CK(hipMemcpy(drp, rp.data(), 8 * (n + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(dcol, col.data(), 4 * col.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dval, val.data(), 8 * val.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dY, Y.data(), 8 * Y.size(), hipMemcpyHostToDevice));
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const double bytes = (double)n * deg * 12 + n * 8.0 + n * 32.0 + n * 16.0;
    const char *names[4] = {"full", "no-gather", "gather-only", "stream-only"};
    for (int m = 0; m < 4; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(a));
            for (int it = 0; it < 10; ++it) {
                dim3 g((unsigned)((n * 64 + 255) / 256));
                if (m == 0) hipLaunchKernelGGL(attr<0>, g, dim3(256), 0, 0, drp, dcol, dval, n, dY, dout);
                if (m == 1) hipLaunchKernelGGL(attr<1>, g, dim3(256), 0, 0, drp, dcol, dval, n, dY, dout);
                if (m == 2) hipLaunchKernelGGL(attr<2>, g, dim3(256), 0, 0, drp, dcol, dval, n, dY, dout);
                if (m == 3) hipLaunchKernelGGL(attr<3>, g, dim3(256), 0, 0, drp, dcol, dval, n, dY, dout);
            }
            CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
            float ms; hipEventElapsedTime(&ms, a, b); ms /= 10;
            if (rep) printf("n=%ld deg=%d local=%d %-12s %.3f ms  %.0f GB/s (algorithmic)\n", (long)n, deg, local, names[m], ms, bytes / ms / 1e6);
        }
    }
    return 0;
}
