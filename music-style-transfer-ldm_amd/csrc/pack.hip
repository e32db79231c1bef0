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
constexpr int kRun = 8;                           // consecutive packed elements per run (one 16- or 32-byte store)
constexpr int kRunsPerThread = 1;                 // runs per thread, kThreads runs apart (4: 54 -> 62 us per step)
constexpr int kBlockElems = kThreads * kRun * kRunsPerThread;

__device__ __forceinline__ float pack_source(const PackJob& j, int m, int ci, int kk) {
    return j.transposed ? j.w[((size_t)ci * j.Cout + m) * j.KK + kk] : j.w[((size_t)m * j.Cin + ci) * j.KK + kk];
}

// Run idx (an 8-element run of the job's packed weight; the runs of a phase are enumerated tap-fastest, see
// below): the run lies inside one phase and one packed row (phase segments and rows are multiples of 8
// elements), so the index arithmetic is done once per run, the eight source loads are independent, and the run
// is written with one 16-byte store (16-bit kind 3) or two (fp32).  Round 4: one element per thread at a
// 256-element stride (a 2-byte store per element, the taps of a source line read by different blocks) took 63-68
// us per step for 19.9 M elements; 8-element runs 59-63 us; runs tap-fastest 51-55 us (profiles/r04/pack_runs).
__device__ __forceinline__ void pack_run(const PackJob& j, uint32_t idx) {
    int ph = 0;
    for (int p = 1; p < j.nphase; ++p)
        if (idx >= (uint32_t)j.wofs[p]) ph = p;
    const uint32_t local = idx - (uint32_t)j.wofs[ph];
    float v[kRun];
    if (j.kind == 3) {   // tconv.hip: [phase][chunk = cc*ntap + t][Mpad][32], 16-bit
        // runs in (cc, m, 8-channel quarter, tap) order, the tap fastest: neighbouring lanes read the taps of the
        // same source rows (w[m][ci][0..KK) contiguous), so a wave's loads cover whole source lines once instead
        // of one tap's word of every line (the lines' other taps re-fetched by other blocks)
        const uint32_t run = local / kRun;
        const int nt = j.ntap[ph];
        const uint32_t q = j.fd_ntap[ph].div(run);
        const int t = (int)(run - q * (uint32_t)nt);
        const int el = (int)(q & 3u) * kRun;
        const int row2 = (int)(q >> 2);              // cc * Mpad + m
        const int cc = j.fd_mpad.div(row2);
        const int m = row2 - cc * j.Mpad;
        const int kk = j.kk[ph][t];
#pragma unroll
        for (int e = 0; e < kRun; ++e) v[e] = m < j.Cout ? pack_source(j, m, cc * 32 + el + e, kk) : 0.f;
        uint32_t u[kRun / 2];
#pragma unroll
        for (int e = 0; e < kRun / 2; ++e) {
            const float a0 = v[2 * e], a1 = v[2 * e + 1];
            const uint32_t h0 = j.dt == LDM_DT_F16 ? __builtin_bit_cast(unsigned short, (_Float16)a0)
                                                   : __builtin_bit_cast(unsigned short, (__bf16)a0);
            const uint32_t h1 = j.dt == LDM_DT_F16 ? __builtin_bit_cast(unsigned short, (_Float16)a1)
                                                   : __builtin_bit_cast(unsigned short, (__bf16)a1);
            u[e] = h0 | (h1 << 16);
        }
        const size_t o = (size_t)j.wofs[ph] + ((size_t)(cc * nt + t) * j.Mpad + m) * 32 + el;
        *reinterpret_cast<uint4*>(reinterpret_cast<unsigned short*>(j.out) + o) = make_uint4(u[0], u[1], u[2], u[3]);
        return;
    }
    // conv.hip: [phase][chunk][Mpad][CK], k = chunk*CK + slot, tap-major over Cin
    const int lck = j.kind == 1 ? 3 : 4;
    int c, m, slot, t, ci;
    if (j.remap) {
        // one phase, Cin % 8 == 0: runs in (m, run of K) order with the K runs tap-fastest (as kind 3 above),
        // the K padding past ntap * Cin last; a run never crosses a tap or a chunk
        const uint32_t run = local / kRun;
        m = j.fd_kr.div(run);
        const int kr = (int)(run - (uint32_t)m * (uint32_t)j.fd_kr.d);
        const int nt = j.ntap[0], nval = nt * (j.Cin / kRun);
        int k0;
        if (kr < nval) {
            const int cir = j.fd_ntap[0].div(kr);
            t = kr - cir * nt;
            ci = cir * kRun;
            k0 = t * j.Cin + ci;
        } else {
            k0 = kr * kRun;
            t = nt;   // padding: zeros
            ci = 0;
        }
        c = k0 >> lck;
        slot = k0 & ((1 << lck) - 1);
    } else {
        slot = (int)(local & ((1u << lck) - 1));
        const int rowid = (int)(local >> lck);
        c = j.fd_mpad.div(rowid);
        m = rowid - c * j.Mpad;
        const int k = (c << lck) + slot;
        t = j.fd_cin.div(k);
        ci = k - t * j.Cin;
    }
#pragma unroll
    for (int e = 0; e < kRun; ++e) {
        v[e] = m < j.Cout && t < j.ntap[ph] ? pack_source(j, m, ci, j.kk[ph][t < kMaxTap ? t : 0]) : 0.f;
        if (++ci == j.Cin) ci = 0, ++t;
    }
    float* o = reinterpret_cast<float*>(j.out) + (j.remap ? ((size_t)c * j.Mpad + m) * (1 << lck) + slot : idx);
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
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
    const uint32_t r0 = (uint32_t)(b - j.first_block) * (kThreads * kRunsPerThread) + threadIdx.x;
#pragma unroll
    for (int i = 0; i < kRunsPerThread; ++i) {
        const uint32_t idx = (r0 + i * kThreads) * kRun;
        if (idx < total) pack_run(j, idx);
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
        ldm_conv_plan pl = plans[i];
        if (pl.kind == 4) pl.kind = 3, pl.tm = 1;   // sconv.hip reads the kind-3 pack (64-row padding)
        int rc = pl.kind == 3 ? tconv_pack_job(descs[i], pl, j) : conv_pack_job(descs[i], pl, j);
        if (rc) return rc;
        LDM_REQUIRE(j.total > 0 && j.total < (1LL << 31) - kBlockElems, "pack_many_prepare: weight too large");
        // the kernel writes whole 8-element runs: phase segments (and so the total) are multiples of 8 elements
        for (int p = 0; p < j.nphase; ++p) LDM_REQUIRE(j.wofs[p] % kRun == 0, "pack_many_prepare: unaligned phase");
        LDM_REQUIRE(j.total % kRun == 0, "pack_many_prepare: unaligned total");
        LDM_REQUIRE(((uintptr_t)out[i] & 15) == 0, "pack_many_prepare: output must be 16-byte aligned");
        j.w = w[i];
        j.out = out[i];
        j.first_block = blocks;
        j.fd_mpad = FastDiv::make(j.Mpad);
        j.fd_cin = FastDiv::make(j.Cin);
        for (int p = 0; p < kMaxPhase; ++p) j.fd_ntap[p] = FastDiv::make(j.ntap[p] > 0 ? j.ntap[p] : 1);
        j.remap = j.kind != 3 && j.nphase == 1 && j.Cin % kRun == 0;
        j.fd_kr = FastDiv::make(j.remap ? (int32_t)(j.total / j.Mpad / kRun) : 1);
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
