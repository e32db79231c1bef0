// The data formats either side of the path: the 8-bit mel-spectrogram PNG the
// reference's dataset is made of (audio_processor.py:55-73 quantisation, :81-100 its inverse) and the
// [0,1] float tensors the model consumes (dataset.py:252-260, torchvision ToTensor).  Elementwise and
// HBM-bound: one float4 / uchar4 per lane, grid-stride, the reference's fp32 operation order.
#include "common.h"

#pragma clang fp contract(off)

namespace ldm {
namespace {

// uint8(clip((db + max_db) * (255 / max_db), 0, 255) + 0.5): numpy float32 arithmetic, truncating cast
__device__ __forceinline__ unsigned char quant1(float v, float max_db, float scale) {
    float s = v + max_db;
    s = s * scale;
    s = s < 0.f ? 0.f : (s > 255.f ? 255.f : s);
    s = s + 0.5f;
    return (unsigned char)(int)s;
}

__global__ __launch_bounds__(256) void mel_quantize_kernel(const float* __restrict__ db, unsigned char* __restrict__ out,
                                                           int64_t n, float max_db, float scale) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
    for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
        if (i + 3 < n && ((uintptr_t)(db + i) & 15) == 0) {
            const floatx4 v = *reinterpret_cast<const floatx4*>(db + i);
            uchar4 o;
            o.x = quant1(v[0], max_db, scale);
            o.y = quant1(v[1], max_db, scale);
            o.z = quant1(v[2], max_db, scale);
            o.w = quant1(v[3], max_db, scale);
            if (((uintptr_t)(out + i) & 3) == 0) {
                *reinterpret_cast<uchar4*>(out + i) = o;
                continue;
            }
            out[i] = o.x, out[i + 1] = o.y, out[i + 2] = o.z, out[i + 3] = o.w;
        } else {
            for (int64_t j = i; j < i + 4 && j < n; ++j) out[j] = quant1(db[j], max_db, scale);
        }
    }
}

// db = u8 * (max_db / 255) - max_db  (the inverse, before db_to_power)
__global__ __launch_bounds__(256) void mel_dequantize_kernel(const unsigned char* __restrict__ in, float* __restrict__ db,
                                                             int64_t n, float max_db, float scale) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float v = (float)in[i] * scale;
        db[i] = v - max_db;
    }
}

// ToTensor: u8 / 255 in fp32
__global__ __launch_bounds__(256) void u8_to_unit_kernel(const unsigned char* __restrict__ in, float* __restrict__ out,
                                                         int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = (float)in[i] / 255.0f;
}

unsigned grid_for(int64_t n, int per_lane) {
    int64_t b = (n + 256LL * per_lane - 1) / (256LL * per_lane);
    return (unsigned)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}

}  // namespace
}  // namespace ldm

using namespace ldm;

extern "C" int ldm_mel_quantize(const float* db, uint8_t* out, int64_t n, float max_db, void* stream) {
    LDM_REQUIRE(db && out && n >= 0 && max_db > 0.f, "mel_quantize: bad argument");
    if (n == 0) return 0;
    hipLaunchKernelGGL(mel_quantize_kernel, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, db,
                       reinterpret_cast<unsigned char*>(out), n, max_db, (float)(255.0 / (double)max_db));
    LDM_CHECK_LAUNCH("mel_quantize_kernel");
    return 0;
}

extern "C" int ldm_mel_dequantize(const uint8_t* in, float* db, int64_t n, float max_db, void* stream) {
    LDM_REQUIRE(in && db && n >= 0 && max_db > 0.f, "mel_dequantize: bad argument");
    if (n == 0) return 0;
    hipLaunchKernelGGL(mel_dequantize_kernel, dim3(grid_for(n, 1)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const unsigned char*>(in), db, n, max_db, (float)((double)max_db / 255.0));
    LDM_CHECK_LAUNCH("mel_dequantize_kernel");
    return 0;
}

extern "C" int ldm_u8_to_unit(const uint8_t* in, float* out, int64_t n, void* stream) {
    LDM_REQUIRE(in && out && n >= 0, "u8_to_unit: bad argument");
    if (n == 0) return 0;
    hipLaunchKernelGGL(u8_to_unit_kernel, dim3(grid_for(n, 1)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const unsigned char*>(in), out, n);
    LDM_CHECK_LAUNCH("u8_to_unit_kernel");
    return 0;
}
