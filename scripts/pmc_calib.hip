// pmc_calib.hip -- calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950
// for the access widths of attract_rows (MI355X_MICROARCH.md "HBM": only the
// 16-B/lane streaming read is calibrated there).  Each kernel reads a known
// number of bytes (arrays of 512 MiB, beyond the 256 MiB MALL) with one
// element per lane per step, in the widths the attraction kernel uses:
//   read4   int32 stream   (col)
//   read8   double stream  (val, row_ptr)
//   read16  double2 stream (own Y_i)
//   gather16 random double2 gathers from a 16 MiB table (Y_j at 1M points),
//            one per lane, 64 Mi gathers
//   write16 double2 stream (attr out)
// The per-kernel FETCH_SIZE (KiB) / known bytes gives the width's factor.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/pmc_calib.hip -o scripts/pmc_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } \
    } while (0)

template <class T>
__global__ void read_stream(const T *__restrict__ a, int64_t n, double *__restrict__ sink) {
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const T v = a[i];
        acc += (double)reinterpret_cast<const int32_t *>(&v)[0];
    }
    if (acc == 12345.678) sink[0] = acc;   // never true: keeps the loads
}

__global__ void gather16(const double2 *__restrict__ tab, int64_t ntab, int64_t n, double *__restrict__ sink) {
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        acc += tab[h % (uint64_t)ntab].x;
    }
    if (acc == 12345.678) sink[0] = acc;
}

__global__ void write_stream16(double2 *__restrict__ a, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        a[i] = make_double2((double)i, 1.0);
}

int main() {
    const size_t bytes = 512ull << 20;
    void *buf = nullptr, *tab = nullptr;
    double *sink = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&tab, 16ull << 20));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 1, bytes));
    CK(hipMemset(tab, 1, 16ull << 20));
    const dim3 grid(2048), blk(256);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(read_stream<int32_t>, grid, blk, 0, 0, (const int32_t *)buf, (int64_t)(bytes / 4), sink);
        hipLaunchKernelGGL(read_stream<double>, grid, blk, 0, 0, (const double *)buf, (int64_t)(bytes / 8), sink);
        hipLaunchKernelGGL(read_stream<double2>, grid, blk, 0, 0, (const double2 *)buf, (int64_t)(bytes / 16), sink);
        hipLaunchKernelGGL(gather16, grid, blk, 0, 0, (const double2 *)tab, (int64_t)(1 << 20), (int64_t)(64ll << 20),
                           sink);
        hipLaunchKernelGGL(write_stream16, grid, blk, 0, 0, (double2 *)buf, (int64_t)(bytes / 16));
    }
    CK(hipDeviceSynchronize());
    std::printf("known bytes: read4/read8/read16/write16 %zu each; gather16 %lld gathers x 16 B = %lld B "
                "(table 16 MiB)\n", bytes, (long long)(64ll << 20), (long long)(64ll << 20) * 16);
    CK(hipFree(buf));
    CK(hipFree(tab));
    CK(hipFree(sink));
    return 0;
}
