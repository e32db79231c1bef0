// Calibration microbenchmark (tools only): sustained f32 MFMA rate at one wave per SIMD, with and
// without scalar "cursor" work between the MFMAs, to size the conv kernel's per-chunk budget.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_calib.hip -o /tmp/mfma_calib && /tmp/mfma_calib
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int NACC, int FILL>
__global__ __launch_bounds__(256) void k16(float* out, int iters, int s0) {
    floatx4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = floatx4{0, 0, 0, 0};
    float a = threadIdx.x * 1e-3f, b = 1.0f;
    int s = s0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc[j % NACC] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j % NACC], 0, 0, 0);
#pragma unroll
            for (int f = 0; f < FILL; ++f) s = __builtin_amdgcn_readfirstlane(s * 3 + it);
        }
    }
    float r = s;
    for (int i = 0; i < NACC; ++i) r += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int NACC>
__global__ __launch_bounds__(256) void k32(float* out, int iters) {
    floatx16 acc[NACC];
    for (int i = 0; i < NACC; ++i)
        for (int r = 0; r < 16; ++r) acc[i][r] = 0;
    float a = threadIdx.x * 1e-3f, b = 1.0f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            acc[j % NACC] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j % NACC], 0, 0, 0);
    }
    float r = 0;
    for (int i = 0; i < NACC; ++i)
        for (int q = 0; q < 16; ++q) r += acc[i][q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <typename F>
static double time_ms(F f) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    f();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    f();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    float* out;
    hipMalloc(&out, 1 << 24);
    const int blocks = 256, iters = 4000;   // 256 blocks x 4 waves = 1024 waves = 1 per SIMD
    const double mf = (double)blocks * 4 * iters * 8;   // MFMAs
    auto rep16 = [&](const char* name, double ms) {
        printf("%-34s %8.3f ms  %7.1f TF/s  %6.1f cyc/MFMA@2.1GHz\n", name, ms, mf * 2048 / (ms * 1e-3) / 1e12,
               ms * 1e-3 * 2.1e9 / (iters * 8.0));
    };
    rep16("16x16x4 1 acc", time_ms([&] { k16<1, 0><<<blocks, 256>>>(out, iters, 1); }));
    rep16("16x16x4 2 acc", time_ms([&] { k16<2, 0><<<blocks, 256>>>(out, iters, 1); }));
    rep16("16x16x4 4 acc", time_ms([&] { k16<4, 0><<<blocks, 256>>>(out, iters, 1); }));
    rep16("16x16x4 2 acc + 2 scalar/MFMA", time_ms([&] { k16<2, 2><<<blocks, 256>>>(out, iters, 1); }));
    rep16("16x16x4 2 acc + 5 scalar/MFMA", time_ms([&] { k16<2, 5><<<blocks, 256>>>(out, iters, 1); }));
    rep16("16x16x4 2 acc + 10 scalar/MFMA", time_ms([&] { k16<2, 10><<<blocks, 256>>>(out, iters, 1); }));
    auto rep32 = [&](const char* name, double ms) {
        printf("%-34s %8.3f ms  %7.1f TF/s  %6.1f cyc/MFMA@2.1GHz\n", name, ms, mf * 4096 / (ms * 1e-3) / 1e12,
               ms * 1e-3 * 2.1e9 / (iters * 8.0));
    };
    rep32("32x32x2 1 acc", time_ms([&] { k32<1><<<blocks, 256>>>(out, iters); }));
    rep32("32x32x2 2 acc", time_ms([&] { k32<2><<<blocks, 256>>>(out, iters); }));
    hipFree(out);
    return 0;
}
