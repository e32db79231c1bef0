// Multi-tensor weight re-pack: every packed conv weight of a train step refreshed by ONE launch after the
// optimizer step (the train path packs each trainable conv / convT weight, and its data-gradient dual, into
// the MFMA fragment order of its plan; one small launch per weight was 51 launches per step at B = 32).
// Same element formulas as conv_pack_kernel (conv.hip) and tconv_pack_kernel (tconv.hip).  Each job owns a
// whole number of blocks (kBlockElems elements each), so a block finds its job with a uniform binary search
// and indexes with 32-bit magic-number divisions (the per-element int64 divisions of the single-weight
// kernels would make this launch ALU-bound).  The job table is built on the host once and kept on the device.
#include "common.h"

namespace ldm {
namespace {

constexpr int kThreads = 256;
constexpr int kPerThread = 4;
constexpr int kBlockElems = kThreads * kPerThread;

__device__ __forceinline__ float pack_source(const PackJob& j, int m, int ci, int kk) {
    return j.transposed ? j.w[((size_t)ci * j.Cout + m) * j.KK + kk] : j.w[((size_t)m * j.Cin + ci) * j.KK + kk];
}

__global__ __launch_bounds__(kThreads) void pack_many_kernel(const PackJob* __restrict__ jobs, int njobs) {
    const int b = blockIdx.x;
    int lo = 0, hi = njobs - 1;   // the job owning block b (jobs sorted by first_block)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (jobs[mid].first_block <= b) lo = mid;
        else hi = mid - 1;
    }
    const PackJob& j = jobs[lo];
    const uint32_t total = (uint32_t)j.total;
    const uint32_t base = (uint32_t)(b - j.first_block) * kBlockElems + threadIdx.x;
#pragma unroll
    for (int e = 0; e < kPerThread; ++e) {
        const uint32_t idx = base + e * kThreads;
        if (idx >= total) return;
        int ph = 0;
        for (int p = 1; p < j.nphase; ++p)
            if (idx >= (uint32_t)j.wofs[p]) ph = p;
        const uint32_t local = idx - (uint32_t)j.wofs[ph];
        float v = 0.f;
        if (j.kind == 3) {   // tconv.hip: [phase][chunk = cc*ntap + t][Mpad][32], 16-bit
            const int el = (int)(local & 31u);
            const int row = (int)(local >> 5);
            const int c = j.fd_mpad.div(row);
            const int m = row - c * j.Mpad;
            const int cc = j.fd_ntap[ph].div(c);
            const int t = c - cc * j.ntap[ph];
            if (m < j.Cout) v = pack_source(j, m, cc * 32 + el, j.kk[ph][t]);
            unsigned short* o = reinterpret_cast<unsigned short*>(j.out);
            o[idx] = j.dt == LDM_DT_F16 ? __builtin_bit_cast(unsigned short, (_Float16)v)
                                        : __builtin_bit_cast(unsigned short, (__bf16)v);
            continue;
        }
        // conv.hip: [phase][chunk][Mpad][CK], k = chunk*CK + slot, tap-major over Cin
        const int lck = j.kind == 1 ? 3 : 4;
        const int slot = (int)(local & ((1u << lck) - 1));
        const int rowid = (int)(local >> lck);
        const int c = j.fd_mpad.div(rowid);
        const int m = rowid - c * j.Mpad;
        const int k = (c << lck) + slot;
        const int t = j.fd_cin.div(k);
        const int ci = k - t * j.Cin;
        if (m < j.Cout && t < j.ntap[ph]) v = pack_source(j, m, ci, j.kk[ph][t]);
        reinterpret_cast<float*>(j.out)[idx] = v;
    }
}

}  // namespace
}  // namespace ldm

using namespace ldm;

extern "C" int64_t ldm_pack_job_bytes(void) { return (int64_t)sizeof(PackJob); }

extern "C" int ldm_pack_many_prepare(const ldm_conv_desc* descs, const ldm_conv_plan* plans, const float* const* w,
                                     void* const* out, int32_t n, void* host_jobs, int64_t* launch_size) {
    LDM_REQUIRE(descs && plans && w && out && host_jobs && launch_size && n > 0, "pack_many_prepare: bad argument");
    PackJob* jobs = reinterpret_cast<PackJob*>(host_jobs);
    int64_t blocks = 0;
    for (int i = 0; i < n; ++i) {
        PackJob j{};
        LDM_REQUIRE(w[i] && out[i], "pack_many_prepare: null weight / output");
        int rc = plans[i].kind == 3 ? tconv_pack_job(descs[i], plans[i], j) : conv_pack_job(descs[i], plans[i], j);
        if (rc) return rc;
        LDM_REQUIRE(j.total > 0 && j.total < (1LL << 31) - kBlockElems, "pack_many_prepare: weight too large");
        j.w = w[i];
        j.out = out[i];
        j.first_block = blocks;
        j.fd_mpad = FastDiv::make(j.Mpad);
        j.fd_cin = FastDiv::make(j.Cin);
        for (int p = 0; p < kMaxPhase; ++p) j.fd_ntap[p] = FastDiv::make(j.ntap[p] > 0 ? j.ntap[p] : 1);
        blocks += (j.total + kBlockElems - 1) / kBlockElems;
        jobs[i] = j;
    }
    LDM_REQUIRE(blocks < (1LL << 31), "pack_many_prepare: launch too large");
    *launch_size = blocks;
    return 0;
}

extern "C" int ldm_pack_many(const void* device_jobs, int32_t n, int64_t launch_size, void* stream) {
    LDM_REQUIRE(device_jobs && n > 0 && launch_size > 0 && launch_size < (1LL << 31), "pack_many: bad argument");
    hipLaunchKernelGGL(pack_many_kernel, dim3((unsigned)launch_size), dim3(kThreads), 0, (hipStream_t)stream,
                       reinterpret_cast<const PackJob*>(device_jobs), n);
    LDM_CHECK_LAUNCH("pack_many_kernel");
    return 0;
}
