// Probe: LDS-DMA (global_load_lds_dwordx4 via M0) at LDS offsets below and
// above 64 KiB; prints mismatches per destination offset.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ __launch_bounds__(64) void probe(const uint32_t *src, uint32_t *out, uint32_t dst_off) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[140 * 1024];
    const int lane = threadIdx.x;
    for (int i = lane; i < 140 * 1024 / 4; i += 64) reinterpret_cast<uint32_t *>(lds)[i] = 0xDEADBEEFu;
    __syncthreads();
    const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)lds + dst_off;
    const uint64_t s = (uint64_t)(uintptr_t)(src + lane * 4);
    const uint32_t m0v = __builtin_amdgcn_readfirstlane(base);
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(s), "s"(m0v) : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = lane; i < 256; i += 64) out[i] = reinterpret_cast<const uint32_t *>(lds + dst_off)[i];
}

int main() {
    std::vector<uint32_t> h(256);
    for (int i = 0; i < 256; ++i) h[i] = 1000 + i;
    uint32_t *s, *o;
    hipMalloc(&s, 1024); hipMalloc(&o, 1024);
    hipMemcpy(s, h.data(), 1024, hipMemcpyHostToDevice);
    for (uint32_t off : {0u, 1024u, 32768u, 64512u, 65536u, 66560u, 98304u, 131072u}) {
        hipMemset(o, 0, 1024);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, s, o, off);
        std::vector<uint32_t> r(256);
        hipMemcpy(r.data(), o, 1024, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < 256; ++i) bad += r[i] != h[i];
        printf("dst_off %6u: %d of 256 words wrong (first %u)\n", off, bad, r[0]);
    }
    return 0;
}
