// Radix sort of 2^28 (u32 key, u32 value) pairs with 23-bit keys (the MSM digit sort of one
// batch): rocprim default onesweep vs wider digits per pass.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_fill(uint32_t* k, uint32_t* v, uint32_t n, uint32_t bits) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t x = i * 0x9E3779B97F4A7C15ull;
    x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
    k[i] = (uint32_t)x & ((1u << bits) - 1);
    v[i] = i;
}

template <unsigned RB, unsigned BS, unsigned IPT>
using OneCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>, rocprim::kernel_config<BS, IPT>, RB,
                                        rocprim::block_radix_rank_algorithm::match>>;

template <class Cfg>
int run(const char* name, uint32_t* k, uint32_t* v, uint32_t* k2, uint32_t* v2, uint32_t n, uint32_t bits) {
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, k, k2, v, v2, n, 0, bits));
    void* tmp; CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    float best = 1e9;
    for (int r = 0; r < 4; r++) {
        hipLaunchKernelGGL(k_fill, dim3((n + 255) / 256), dim3(256), 0, 0, k, v, n, bits);
        hipEventRecord(a);
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, k, k2, v, v2, n, 0, bits));
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); if (r) best = ms < best ? ms : best;
    }
    std::vector<uint32_t> h(1 << 20);
    CK(hipMemcpy(h.data(), k2 + (n - h.size()), h.size() * 4, hipMemcpyDeviceToHost));
    bool ok = true;
    for (size_t i = 1; i < h.size(); i++) ok &= h[i - 1] <= h[i];
    printf("{\"cfg\":\"%s\",\"bits\":%u,\"n\":%u,\"ms\":%.3f,\"sorted_tail\":%d}\n", name, bits, n, best, ok);
    hipFree(tmp);
    return 0;
}

__global__ void k_offsets(uint32_t* off, uint32_t segs, uint32_t len) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= segs) off[i] = i * len;
}

int run_seg(uint32_t* k, uint32_t* v, uint32_t* k2, uint32_t* v2, uint32_t n, uint32_t segs, uint32_t bits) {
    uint32_t* off; CK(hipMalloc(&off, (segs + 1) * 4));
    hipLaunchKernelGGL(k_offsets, dim3((segs + 256) / 256), dim3(256), 0, 0, off, segs, n / segs);
    size_t tb = 0;
    CK(rocprim::segmented_radix_sort_pairs(nullptr, tb, k, k2, v, v2, n, segs, off, off + 1, 0, bits));
    void* tmp; CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    float best = 1e9;
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(k_fill, dim3((n + 255) / 256), dim3(256), 0, 0, k, v, n, bits);
        hipEventRecord(a);
        CK(rocprim::segmented_radix_sort_pairs(tmp, tb, k, k2, v, v2, n, segs, off, off + 1, 0, bits));
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); if (r) best = ms < best ? ms : best;
    }
    printf("{\"cfg\":\"segmented\",\"segs\":%u,\"bits\":%u,\"n\":%u,\"ms\":%.3f}\n", segs, bits, n, best);
    hipFree(tmp); hipFree(off);
    return 0;
}

int main() {
    const uint32_t n = 1u << 28;
    uint32_t *k, *v, *k2, *v2;
    CK(hipMalloc(&k, n * 4ull)); CK(hipMalloc(&v, n * 4ull)); CK(hipMalloc(&k2, n * 4ull)); CK(hipMalloc(&v2, n * 4ull));
    // the MSM digit sort: 2^28 pairs, low 16 key bits (c = 16)
    for (uint32_t bits : {16u}) {
        run<rocprim::default_config>("default", k, v, k2, v2, n, bits);
        run<OneCfg<8, 256, 16>>("rb8_256x16", k, v, k2, v2, n, bits);
        run<OneCfg<8, 512, 12>>("rb8_512x12", k, v, k2, v2, n, bits);
        run<OneCfg<8, 512, 16>>("rb8_512x16", k, v, k2, v2, n, bits);
        run<OneCfg<8, 1024, 8>>("rb8_1024x8", k, v, k2, v2, n, bits);
        run<OneCfg<8, 1024, 12>>("rb8_1024x12", k, v, k2, v2, n, bits);
        run<OneCfg<8, 256, 24>>("rb8_256x24", k, v, k2, v2, n, bits);
        run<OneCfg<8, 512, 20>>("rb8_512x20", k, v, k2, v2, n, bits);
        run<OneCfg<7, 512, 16>>("rb7_512x16", k, v, k2, v2, n, bits);
        run<OneCfg<6, 512, 16>>("rb6_512x16", k, v, k2, v2, n, bits);
    }
    return 0;
}
