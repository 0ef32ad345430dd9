// FP32 VALU issue-rate probe for the roofline denominators in bench.py: chains of independent
// v_add_f32, v_mul_f32 and v_fma_f32 (8 accumulators per lane, no memory traffic in the loop) at
// 8 waves per SIMD on every CU. Prints one JSON line of lane-op rates (T op/s) and the clock the
// rates imply against 256 CUs x 4 SIMDs x 32 lanes.
// Built twice: with -fno-slp-vectorize (one v_add/v_mul/v_fma_f32 per op) and without (the
// compiler packs pairs into v_pk_add/v_pk_mul/v_pk_fma_f32); argv[1] labels the line.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -o valu_rate tools/valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int kOp>
__global__ __launch_bounds__(256) void k_rate(float *out, float b, float c, int iters) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 1e-3f + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (kOp == 0) a[i] = a[i] + b;
                else if (kOp == 1) a[i] = a[i] * b;
                else a[i] = __builtin_fmaf(a[i], b, c);
            }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;   // vector store; keeps the chains live
}

template <int kOp>
static int run(const char *name, float *d, int blocks, int iters, double *rate) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_rate<kOp>, dim3(blocks), dim3(256), 0, 0, d, 1.0000001f, 1e-7f, iters);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k_rate<kOp>, dim3(blocks), dim3(256), 0, 0, d, 1.0000001f, 1e-7f, iters);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    const double lane_ops = double(blocks) * 256 * iters * 16 * 8;
    *rate = lane_ops / (best * 1e-3) / 1e12;
    std::printf("%s\"%s_Tops\": %.2f, \"%s_ms\": %.3f", kOp ? ", " : "", name, *rate, name, best);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return 0;
}

int main(int argc, char **argv) {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8;            // 8 blocks x 4 waves per CU = 8 waves per SIMD
    const int iters = 4096;
    float *d = nullptr;
    CHECK(hipMalloc(&d, size_t(blocks) * 256 * sizeof(float)));
    double add = 0, mul = 0, fma = 0;
    std::printf("{\"variant\": \"%s\", ", argc > 1 ? argv[1] : "");
    if (run<0>("add", d, blocks, iters, &add) || run<1>("mul", d, blocks, iters, &mul) ||
        run<2>("fma", d, blocks, iters, &fma))
        return 1;
    // lanes per clock per CU if the clock were 2.4 GHz
    std::printf(", \"cus\": %d, \"add_lane_ops_per_clk_per_cu_at_2p4GHz\": %.1f, \"fma_TFLOPs\": %.2f}\n",
                cus, add * 1e12 / (cus * 2.4e9), 2 * fma);
    CHECK(hipFree(d));
    return 0;
}
