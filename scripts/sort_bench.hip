// Microbenchmark: 1M (uint64 Morton key, int32 index) pairs sorted by
// hipcub::DeviceRadixSort (rocPRIM merge sort below 2^20 items) vs
// rocprim::radix_sort_pairs with merge_sort_limit = 0 (Onesweep).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)
using onesweep_cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;
int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1000000;
    std::vector<uint64_t> hk(n);
    uint64_t s = 12345;
    for (int i = 0; i < n; ++i) { s = s * 6364136223846793005ull + 1442695040888963407ull; hk[i] = s >> 2; }
    uint64_t *k, *k2; int *v, *v2;
    CK(hipMalloc(&k, 8 * n)); CK(hipMalloc(&k2, 8 * n)); CK(hipMalloc(&v, 4 * n)); CK(hipMalloc(&v2, 4 * n));
    CK(hipMemcpy(k, hk.data(), 8 * n, hipMemcpyHostToDevice));
    std::vector<int> hv(n); for (int i = 0; i < n; ++i) hv[i] = i;
    CK(hipMemcpy(v, hv.data(), 4 * n, hipMemcpyHostToDevice));
    size_t t1 = 0, t2 = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, t1, k, k2, v, v2, n, 0, 64));
    CK(rocprim::radix_sort_pairs<onesweep_cfg>(nullptr, t2, k, k2, v, v2, (size_t)n, 0, 64));
    void *tmp; CK(hipMalloc(&tmp, std::max(t1, t2)));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int mode = 0; mode < 3; ++mode) {
        float best = 1e9;
        for (int r = 0; r < 20; ++r) {
            CK(hipEventRecord(a));
            size_t tb = std::max(t1, t2);
            if (mode == 0) CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k, k2, v, v2, n, 0, 64));
            else if (mode == 1) CK(rocprim::radix_sort_pairs<onesweep_cfg>(tmp, tb, k, k2, v, v2, (size_t)n, 0, 64));
            else CK(rocprim::radix_sort_pairs<onesweep_cfg>(tmp, tb, k, k2, v, v2, (size_t)n, 0, 62));
            CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b)); best = std::min(best, ms);
        }
        std::vector<uint64_t> out(n); CK(hipMemcpy(out.data(), k2, 8 * n, hipMemcpyDeviceToHost));
        printf("mode %d (%s): %.1f us sorted=%d\n", mode, mode == 0 ? "hipcub" : mode == 1 ? "onesweep 64b" : "onesweep 62b",
               best * 1e3, (int)std::is_sorted(out.begin(), out.end()));
    }
    return 0;
}
