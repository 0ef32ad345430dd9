// cumask_probe.hip — what hipExtStreamCreateWithCUMask does on this box (r05 diagnostic).
//  1. placement: blocks launched on a stream with a CU mask record their XCC / SE / CU
//     (s_getreg HW_ID, XCC_ID), so the mask-bit -> CU map and the restriction itself are visible;
//  2. queues: two single-block spin kernels on two streams that may share a hardware queue
//     (GPU_MAX_HW_QUEUES 4), plain and CU-masked: overlapped start times = separate queues.
// Build: hipcc --offload-arch=gfx950 -O2 tools/cumask_probe.hip -o build/cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <tuple>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

// per block: start, end (100 MHz ticks), HW_ID, XCC_ID
__global__ void k_probe(unsigned long long *out, int spin_ticks) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
    unsigned long long t = t0;
    while (t - t0 < static_cast<unsigned long long>(spin_ticks)) {
        __builtin_amdgcn_s_sleep(8);
        t = __builtin_amdgcn_s_memrealtime();
    }
    out[4 * blockIdx.x + 0] = t0;
    out[4 * blockIdx.x + 1] = t;
    out[4 * blockIdx.x + 2] = hw;
    out[4 * blockIdx.x + 3] = xcc;
}

static std::tuple<int, int, int> cu_of(unsigned long long hw, unsigned long long xcc) {
    const int cu = static_cast<int>((hw >> 8) & 0xF), sh = static_cast<int>((hw >> 12) & 1), se = static_cast<int>((hw >> 13) & 7);
    return {static_cast<int>(xcc & 0xF), se, cu | (sh << 4)};
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    std::printf("device %s, %d CUs\n", prop.gcnArchName, ncu);
    const int words = (ncu + 31) / 32;
    unsigned long long *d = nullptr;
    const int nb = 256;
    CK(hipMalloc(&d, sizeof(unsigned long long) * 4 * nb));
    std::vector<unsigned long long> h(4 * nb);

    // 1. placement under a mask
    auto place = [&](const std::vector<uint32_t> &mask, const char *what, int blocks) {
        hipStream_t s;
        CK(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask.size()), mask.data()));
        CK(hipMemsetAsync(d, 0, sizeof(unsigned long long) * 4 * nb, s));
        hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(64), 0, s, d, 2000);   // 20 us each
        CK(hipGetLastError());
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), d, sizeof(unsigned long long) * 4 * nb, hipMemcpyDeviceToHost));
        std::set<std::tuple<int, int, int>> cus;
        std::set<int> xccs;
        for (int b = 0; b < blocks; ++b) { cus.insert(cu_of(h[4 * b + 2], h[4 * b + 3])); xccs.insert(static_cast<int>(h[4 * b + 3] & 0xF)); }
        std::printf("%-28s blocks %3d -> %3zu distinct CUs over %zu XCCs:", what, blocks, cus.size(), xccs.size());
        int shown = 0;
        for (auto &c : cus) { if (shown++ < 6) std::printf(" (x%d s%d c%d)", std::get<0>(c), std::get<1>(c), std::get<2>(c)); }
        std::printf("\n");
        CK(hipStreamDestroy(s));
    };
    for (int bit : {0, 1, 2, 3, 7, 8, 31, 32, 33, 64, 128, 255}) {
        if (bit >= ncu) continue;
        std::vector<uint32_t> m(words, 0);
        m[bit / 32] |= 1u << (bit % 32);
        char w[64];
        std::snprintf(w, sizeof w, "mask bit %d", bit);
        place(m, w, 16);
    }
    for (int lo_hi : {8, 32, 64}) {
        std::vector<uint32_t> m(words, 0);
        for (int b = 0; b < lo_hi; ++b) m[b / 32] |= 1u << (b % 32);
        char w[64];
        std::snprintf(w, sizeof w, "mask bits 0..%d", lo_hi - 1);
        place(m, w, 256);
    }
    {
        std::vector<uint32_t> m(words, 0xFFFFFFFFu);
        place(m, "full mask", 256);
    }

    // 2. hardware queues: streams made in a row; pairs (0, k) with k = 1..8, plain, then CU-masked
    auto overlap = [&](hipStream_t a, hipStream_t b) {
        unsigned long long *d2 = d + 4 * 128;
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, a, d, 20000);    // 200 us
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, b, d2, 20000);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        unsigned long long r[8];
        CK(hipMemcpy(r, d, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        CK(hipMemcpy(r + 4, d2, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        const long long gap = static_cast<long long>(r[4]) - static_cast<long long>(r[0]);
        return gap;   // ticks between the two starts: ~0 overlapped, ~20000 serialised
    };
    std::vector<hipStream_t> plain(9);
    for (auto &s : plain) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::printf("plain streams, start gap (us) of stream 0 and stream k:");
    for (int k = 1; k < 9; ++k) std::printf(" k%d %.0f", k, overlap(plain[0], plain[k]) / 100.0);
    std::printf("\n");
    std::vector<hipStream_t> masked(9);
    std::vector<uint32_t> full(words, 0xFFFFFFFFu);
    for (auto &s : masked) CK(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(full.size()), full.data()));
    std::printf("full-mask streams, start gap (us) of masked 0 and masked k:");
    for (int k = 1; k < 9; ++k) std::printf(" k%d %.0f", k, overlap(masked[0], masked[k]) / 100.0);
    std::printf("\n");
    std::printf("plain 0 vs masked k:");
    for (int k = 0; k < 9; ++k) std::printf(" k%d %.0f", k, overlap(plain[0], masked[k]) / 100.0);
    std::printf("\n");
    for (auto &s : plain) CK(hipStreamDestroy(s));
    for (auto &s : masked) CK(hipStreamDestroy(s));
    CK(hipFree(d));
    std::printf("done\n");
    return 0;
}
