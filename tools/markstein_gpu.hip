// markstein_gpu.hip (r05, a checker, not product code): the triangle test's s and t divisions
// (raytracing.cpp:144, :148) as q = RN(n rD), q' = fma(fma(-q, D, n), rD, q) with rD = RN(1/D)
// taken from the triangle record, against the correctly rounded n / D, for EVERY pair of float
// significands (2^23 x 2^23). Every step is invariant under scaling n and D by powers of two while
// all intermediates stay normal, which the kernel's range check (|q| in [2^-30, 2^30], |D| in
// [2^-30, 2^30]) guarantees, so a clean sweep proves the fast path exact on the whole domain it takes.
// One thread per divisor significand, numerators in launches of 2^16; per-thread counts in a buffer
// (plain vector stores). Usage: markstein_gpu [control]: "control" also sweeps the uncorrected q over
// one launch, which must report mismatches (the check can fail).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/markstein_gpu.hip -o tools/bin/markstein_gpu
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 2; } } while (0)

constexpr uint32_t kSig = 1u << 23;
constexpr uint32_t kChunk = 1u << 16;

template <bool kCorrect>
__global__ void __launch_bounds__(256) sweep(uint32_t a0, unsigned long long *bad, uint32_t *first) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= kSig) return;
    const float D = __uint_as_float(0x3f800000u | d);
    const float rD = 1.0f / D;                      // correctly rounded (IEEE division, no fast math)
    unsigned long long nb = 0;
    uint32_t f = first[d];
    for (uint32_t a = a0; a < a0 + kChunk; ++a) {
        const float n = __uint_as_float(0x3f800000u | a);
        const float q = n * rD;
        const float res = kCorrect ? fmaf(fmaf(-q, D, n), rD, q) : q;
        const float ref = n / D;
        if (__float_as_uint(res) != __float_as_uint(ref)) {
            ++nb;
            if (f == 0xffffffffu) f = a;
        }
    }
    bad[d] += nb;
    first[d] = f;
}

int main(int argc, char **argv) {
    const bool control = argc > 1 && std::strcmp(argv[1], "control") == 0;
    unsigned long long *d_bad = nullptr;
    uint32_t *d_first = nullptr;
    CHECK(hipMalloc(&d_bad, sizeof(unsigned long long) * kSig));
    CHECK(hipMalloc(&d_first, sizeof(uint32_t) * kSig));
    const dim3 grid(kSig / 256), block(256);
    if (control) {
        CHECK(hipMemset(d_bad, 0, sizeof(unsigned long long) * kSig));
        CHECK(hipMemset(d_first, 0xff, sizeof(uint32_t) * kSig));
        sweep<false><<<grid, block>>>(0, d_bad, d_first);
        CHECK(hipGetLastError());
        std::vector<unsigned long long> b(kSig);
        CHECK(hipMemcpy(b.data(), d_bad, sizeof(unsigned long long) * kSig, hipMemcpyDeviceToHost));
        unsigned long long t = 0;
        for (auto v : b) t += v;
        std::printf("control (uncorrected q, numerators [0, 2^16)): %llu of %llu wrong\n", t,
                    static_cast<unsigned long long>(kSig) * kChunk);
    }
    CHECK(hipMemset(d_bad, 0, sizeof(unsigned long long) * kSig));
    CHECK(hipMemset(d_first, 0xff, sizeof(uint32_t) * kSig));
    for (uint32_t a0 = 0; a0 < kSig; a0 += kChunk) {
        sweep<true><<<grid, block>>>(a0, d_bad, d_first);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        if ((a0 / kChunk) % 16 == 15) { std::printf("numerators up to %u done\n", a0 + kChunk); std::fflush(stdout); }
    }
    std::vector<unsigned long long> b(kSig);
    std::vector<uint32_t> f(kSig);
    CHECK(hipMemcpy(b.data(), d_bad, sizeof(unsigned long long) * kSig, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(f.data(), d_first, sizeof(uint32_t) * kSig, hipMemcpyDeviceToHost));
    unsigned long long t = 0;
    long long ex = -1;
    for (uint32_t d = 0; d < kSig; ++d) { t += b[d]; if (b[d] && ex < 0) ex = d; }
    std::printf("corrected: %llu of %llu significand pairs wrong\n", t, static_cast<unsigned long long>(kSig) * kSig);
    if (ex >= 0) std::printf("first: divisor significand %lld numerator %u\n", ex, f[ex]);
    CHECK(hipFree(d_bad));
    CHECK(hipFree(d_first));
    return t ? 1 : 0;
}
