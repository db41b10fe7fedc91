// Probe: hipStreamWaitValue32 on ordinary device memory that a running
// kernel increments (the gate the tile-streaming consumers would use).
// Stream 1 runs `work`: every block adds 1 to a counter at its start, then
// spins ~spin_us.  Stream 2 waits for counter >= nblocks, then `mark` writes
// the wall clock.  Prints when the last block started, when mark ran and when
// work ended (wall clock ticks, 100 MHz), or "UNSUPPORTED".
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void work(int *cnt, unsigned long long *t_last_start, unsigned long long *t_end, long long spin) {
    if (threadIdx.x == 0) {
        atomicAdd(cnt, 1);
        atomicMax(t_last_start, (unsigned long long)wall_clock64());
    }
    const long long t0 = clock64();
    while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(4);
    if (threadIdx.x == 0) atomicMax(t_end, (unsigned long long)wall_clock64());
}

__global__ void mark(unsigned long long *t_mark) { if (threadIdx.x == 0) *t_mark = wall_clock64(); }

int main(int argc, char **argv) {
    const int nblocks = argc > 1 ? std::atoi(argv[1]) : 8192;
    int sup = 0;
    CK(hipDeviceGetAttribute(&sup, hipDeviceAttributeCanUseStreamWaitValue, 0));
    std::printf("CanUseStreamWaitValue %d\n", sup);
    if (!sup) { std::printf("UNSUPPORTED\n"); return 0; }
    int *cnt;
    unsigned long long *ts;
    CK(hipMalloc(&cnt, 256));
    CK(hipMalloc(&ts, 256));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(cnt, 0, 256));
        CK(hipMemset(ts, 0, 256));
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(work, dim3(nblocks), dim3(256), 0, s1, cnt, ts + 0, ts + 1, 2000000LL);
        CK(hipStreamWaitValue32(s2, cnt, (uint32_t)nblocks, hipStreamWaitValueGte, 0xffffffffu));
        hipLaunchKernelGGL(mark, dim3(1), dim3(64), 0, s2, ts + 2);
        CK(hipDeviceSynchronize());
        unsigned long long h[3];
        int c = 0;
        CK(hipMemcpy(h, ts, sizeof(h), hipMemcpyDeviceToHost));
        CK(hipMemcpy(&c, cnt, sizeof(int), hipMemcpyDeviceToHost));
        std::printf("rep %d: count %d  last start -> mark %+lld ticks, mark -> work end %+lld ticks\n", rep, c,
                    (long long)(h[2] - h[0]), (long long)(h[1] - h[2]));
    }
    return 0;
}
