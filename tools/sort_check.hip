// Correctness + timing of csrc/sort.hip (the MSM's own radix sort and scan) against the host and
// against rocPRIM's onesweep (the library sort it replaces; the comparison lives in this tool
// only).  Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/sort_check.hip -o
// tools/sort_check.  Prints one JSON line per case.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <vector>

#include "../plonky3_eon_amd/csrc/sort.hip"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            printf("{\"error\":\"%s\",\"line\":%d}\n", hipGetErrorString(e_), __LINE__);       \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

// keys like k_msm_digits': (group << c) | (|digit| - 1), zero digits 0xFFFFFFFF (1 in 2^15),
// group-major; values = the input index (so stability is checkable)
__global__ void k_fill(uint32_t* k, uint32_t* v, uint32_t n, uint32_t c, uint32_t per_group, uint32_t mode) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t x = (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 32;
    uint32_t key;
    if (mode == 0) {
        const uint32_t mag = (uint32_t)x & ((1u << (c - 1)) - 1);
        key = ((uint32_t)(x >> 40) & 0x7fff) == 0 ? 0xFFFFFFFFu : ((i / per_group) << c) | mag;
    } else if (mode == 1) {
        key = (uint32_t)x;  // uniform
    } else {
        key = (uint32_t)(x & 7);  // heavy duplicates
    }
    k[i] = key;
    v[i] = i;
}

// device check of a sort too large for the host: out[i] is input pair v[i] (k2[i] == k[v2[i]]),
// keys non-decreasing on the sorted bits, values increasing within equal keys (stability), every
// input index exactly once (bitmap)
__global__ void k_check_big(const uint32_t* k, const uint32_t* k2, const uint32_t* v2, uint64_t n, uint32_t m,
                            uint32_t* seen, unsigned long long* bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t vi = v2[i];
    bool ok = vi < n && k2[i] == k[vi];
    if (i > 0) {
        const uint32_t a = k2[i - 1] & m, b = k2[i] & m;
        ok = ok && (a < b || (a == b && v2[i - 1] < vi));
    }
    if (vi < n && (atomicOr(seen + vi / 32, 1u << (vi % 32)) >> (vi % 32) & 1)) ok = false;
    if (!ok) atomicAdd(bad, 1ull);
}

static bool check(const std::vector<uint32_t>& kin, const std::vector<uint32_t>& kout, const std::vector<uint32_t>& vout,
                  uint32_t bits) {
    const size_t n = kin.size();
    const uint32_t m = bits >= 32 ? 0xFFFFFFFFu : (1u << bits) - 1;
    std::vector<uint32_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0u);
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return (kin[a] & m) < (kin[b] & m); });
    for (size_t i = 0; i < n; i++)
        if (vout[i] != idx[i] || kout[i] != kin[idx[i]]) return false;
    return true;
}

int main(int argc, char** argv) {
    const bool big = argc > 1 && std::string(argv[1]) == "big";
    if (argc > 1 && std::string(argv[1]) == "huge") {
        // beyond the 30-bit look-back counts of the round-3 sort: 2^30 + 4097 and
        // 2^31 + 3 pairs, 16 key bits, checked on the device
        for (uint64_t n : {(1ull << 30) + 4097, (1ull << 31) + 3}) {
            const uint32_t bits = 16;
            uint32_t *k, *v, *k2, *v2, *seen;
            unsigned long long* bad;
            CK(hipMalloc(&k, n * 4));
            CK(hipMalloc(&v, n * 4));
            CK(hipMalloc(&k2, n * 4));
            CK(hipMalloc(&v2, n * 4));
            CK(hipMalloc(&seen, (n / 32 + 1) * 4));
            CK(hipMalloc(&bad, 8));
            CK(hipMemset(seen, 0, (n / 32 + 1) * 4));
            CK(hipMemset(bad, 0, 8));
            hipLaunchKernelGGL(k_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, k, v, (uint32_t)n, bits,
                               1u << 21, 0);
            void* tmp;
            CK(hipMalloc(&tmp, eon::radix_sort_temp_bytes(n, bits)));
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipEventRecord(a);
            CK(eon::radix_sort_pairs(tmp, k, k2, v, v2, n, bits, 0));
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            hipLaunchKernelGGL(k_check_big, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, k, k2, v2, n,
                               (1u << bits) - 1, seen, bad);
            unsigned long long nbad = 1;
            CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
            printf("{\"case\":\"huge\",\"n\":%llu,\"bits\":%u,\"ms\":%.3f,\"bad\":%llu,\"ok\":%d}\n",
                   (unsigned long long)n, bits, ms, nbad, (int)(nbad == 0));
            // one past the limit must be refused, not sorted
            const hipError_t e = eon::radix_sort_pairs(tmp, k, k2, v, v2, eon::RADIX_SORT_MAX_PAIRS + 1, bits, 0);
            printf("{\"case\":\"limit\",\"n\":%llu,\"refused\":%d}\n",
                   (unsigned long long)eon::RADIX_SORT_MAX_PAIRS + 1, (int)(e == hipErrorInvalidValue));
            hipFree(tmp); hipFree(k); hipFree(v); hipFree(k2); hipFree(v2); hipFree(seen); hipFree(bad);
        }
        return 0;
    }
    struct Case { uint32_t n, bits, mode; };
    std::vector<Case> cases = {{0, 16, 0}, {1, 16, 0}, {1000, 16, 0}, {8191, 16, 1}, {8192, 16, 0}, {8193, 16, 2},
                               {100003, 8, 1}, {100003, 19, 0}, {100003, 23, 1}, {1u << 20, 16, 0}, {(1u << 20) + 7, 32, 1},
                               {3u << 20, 5, 2}, {(1u << 22) + 3, 16, 0},
                               // 17..20 key bits (three passes)
                               {8193, 19, 2}, {100003, 17, 0}, {100003, 18, 1}, {(1u << 20) + 5, 20, 0},
                               {3u << 20, 19, 1}, {(1u << 22) + 1, 20, 2},
                               // the edges of a 16384-pair tile (1024 threads x 16)
                               {16383, 16, 0}, {16384, 16, 1}, {16385, 16, 2}, {32769, 19, 0}};
    for (const Case& cs : cases) {
        uint32_t *k, *v, *k2, *v2;
        const size_t nb = std::max<size_t>(cs.n, 1) * 4;
        CK(hipMalloc(&k, nb));
        CK(hipMalloc(&v, nb));
        CK(hipMalloc(&k2, nb));
        CK(hipMalloc(&v2, nb));
        if (cs.n)
            hipLaunchKernelGGL(k_fill, dim3((cs.n + 255) / 256), dim3(256), 0, 0, k, v, cs.n, std::min(std::max(16u, cs.bits), 24u),
                               1u << 17, cs.mode);
        void* tmp;
        CK(hipMalloc(&tmp, eon::radix_sort_temp_bytes(cs.n, cs.bits) + 256));
        CK(eon::radix_sort_pairs(tmp, k, k2, v, v2, cs.n, cs.bits, 0));
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> hk(cs.n), hv(cs.n), hk2(cs.n);
        if (cs.n) {
            CK(hipMemcpy(hk.data(), k, nb, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hk2.data(), k2, nb, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hv.data(), v2, nb, hipMemcpyDeviceToHost));
        }
        printf("{\"case\":\"sort\",\"n\":%u,\"bits\":%u,\"mode\":%u,\"ok\":%d}\n", cs.n, cs.bits, cs.mode,
               (int)check(hk, hk2, hv, cs.bits));
        // scan of the keys' low 8 bits
        std::vector<uint32_t> hs(cs.n);
        for (uint32_t i = 0; i < cs.n; i++) hs[i] = hk[i] & 0xff;
        uint32_t* so;
        CK(hipMalloc(&so, nb));
        void* stmp;
        CK(hipMalloc(&stmp, eon::exclusive_scan_temp_bytes(cs.n)));
        if (cs.n) CK(hipMemcpy(k2, hs.data(), nb, hipMemcpyHostToDevice));
        CK(eon::exclusive_scan_u32(stmp, k2, so, cs.n, 0));
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> got(cs.n);
        if (cs.n) CK(hipMemcpy(got.data(), so, nb, hipMemcpyDeviceToHost));
        uint32_t run = 0;
        bool ok = true;
        for (uint32_t i = 0; i < cs.n; i++) {
            ok &= got[i] == run;
            run += hs[i];
        }
        printf("{\"case\":\"scan\",\"n\":%u,\"ok\":%d}\n", cs.n, (int)ok);
        hipFree(so); hipFree(stmp); hipFree(tmp); hipFree(k); hipFree(v); hipFree(k2); hipFree(v2);
    }
    if (!big) return 0;
    // timing at the prove's batch size: 2^28 MSM-like pairs, 16 key bits (c = 16)
    for (uint32_t bits : {16u, 19u, 20u}) {
        const uint32_t n = 1u << 28;
        uint32_t *k, *v, *k2, *v2;
        CK(hipMalloc(&k, n * 4ull));
        CK(hipMalloc(&v, n * 4ull));
        CK(hipMalloc(&k2, n * 4ull));
        CK(hipMalloc(&v2, n * 4ull));
        hipLaunchKernelGGL(k_fill, dim3((n + 255) / 256), dim3(256), 0, 0, k, v, n, bits, 1u << 21, 0);
        void* tmp;
        CK(hipMalloc(&tmp, eon::radix_sort_temp_bytes(n, bits)));
        size_t rb = 0;
        CK(rocprim::radix_sort_pairs(nullptr, rb, k, k2, v, v2, (size_t)n, 0u, bits, 0));
        void* rtmp;
        CK(hipMalloc(&rtmp, rb));
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        float best_own = 1e9, best_roc = 1e9;
        for (int r = 0; r < 5; r++) {
            hipEventRecord(a);
            CK(eon::radix_sort_pairs(tmp, k, k2, v, v2, n, bits, 0));
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (r) best_own = std::min(best_own, ms);
            hipEventRecord(a);
            CK(rocprim::radix_sort_pairs(rtmp, rb, k, k2, v, v2, (size_t)n, 0u, bits, 0));
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
            if (r) best_roc = std::min(best_roc, ms);
        }
        // correctness of the big run on a 2^20 window (sortedness + stability by the value index)
        CK(eon::radix_sort_pairs(tmp, k, k2, v, v2, n, bits, 0));
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> hk(1 << 20), hv(1 << 20);
        CK(hipMemcpy(hk.data(), k2 + n / 2, hk.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hv.data(), v2 + n / 2, hv.size() * 4, hipMemcpyDeviceToHost));
        const uint32_t m = (1u << bits) - 1;
        bool ok = true;
        for (size_t i = 1; i < hk.size(); i++) {
            ok &= (hk[i - 1] & m) <= (hk[i] & m);
            if ((hk[i - 1] & m) == (hk[i] & m)) ok &= hv[i - 1] < hv[i];
        }
        printf("{\"case\":\"time\",\"n\":%u,\"bits\":%u,\"own_ms\":%.3f,\"rocprim_default_ms\":%.3f,\"ok\":%d}\n", n, bits,
               best_own, best_roc, (int)ok);
        hipFree(rtmp); hipFree(tmp); hipFree(k); hipFree(v); hipFree(k2); hipFree(v2);
    }
    return 0;
}
