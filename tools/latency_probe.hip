// Calibration (tools only): where the fixed cost of a short kernel goes on this box.
// Per block, wall-clock stamps (s_memrealtime, 100 MHz) around: the first kernarg read, a second
// kernarg read 1.2 KB further, a load from a buffer the previous kernel wrote, a load from a buffer
// nobody touched for a while, and the final store.  Kernels are chained back to back in a hipGraph
// (as in the sampler); the stamps of the last launch are reported (median over blocks).
//   hipcc -O3 --offload-arch=gfx950 tools/latency_probe.hip -o tools/bin/latency_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

struct BigArgs {
    const float* warm;
    const float* cold;
    float* out;
    unsigned long long* stamps;
    int pad[300];
    int far_field;
};

struct SmallArgs {
    const float* warm;
    const float* cold;
    float* out;
    unsigned long long* stamps;
    int far_field;
};

template <typename A>
__global__ __launch_bounds__(256) void probe(A a, int write_stamps) {
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const float* warm = a.warm;   // first kernarg read
    const int i = blockIdx.x * 256 + threadIdx.x;
    float v0 = __builtin_nontemporal_load(&warm[i]);
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    int ff = __builtin_amdgcn_readfirstlane(a.far_field);   // kernarg 1.2 KB away (BigArgs)
    unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    float v1 = warm[i + ff];                                  // written by the previous launch
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    float v2 = a.cold[(size_t)i * 16 + ff];                   // far, rarely touched
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
    a.out[i] = v0 + v1 + v2;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t5 = __builtin_amdgcn_s_memrealtime();
    if (write_stamps && threadIdx.x == 0) {
        unsigned long long* s = a.stamps + blockIdx.x * 6;
        s[0] = t0; s[1] = t1; s[2] = t2; s[3] = t3; s[4] = t4; s[5] = t5;
    }
}

template <typename A>
static void run(const char* name, A a, int blocks) {
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipGraph_t g;
    hipGraphExec_t x;
    const int reps = 30;
    (void)hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
    for (int r = 0; r < reps; ++r) {
        A b = a;
        if (r & 1) { const float* t = b.warm; b.warm = b.out; b.out = const_cast<float*>(t); }   // read what the previous launch wrote
        hipLaunchKernelGGL(probe<A>, dim3(blocks), dim3(256), 0, st, b, r == reps - 1);
    }
    (void)hipStreamEndCapture(st, &g);
    (void)hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipGraphLaunch(x, st);
    (void)hipStreamSynchronize(st);
    (void)hipEventRecord(e0, st);
    (void)hipGraphLaunch(x, st);
    (void)hipEventRecord(e1, st);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(blocks * 6);
    (void)hipMemcpy(h.data(), a.stamps, h.size() * 8, hipMemcpyDeviceToHost);
    auto med = [&](int k0, int k1) {
        std::vector<double> v;
        for (int b = 0; b < blocks; ++b) v.push_back((double)(h[b * 6 + k1] - h[b * 6 + k0]) * 0.01);
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    unsigned long long mn = ~0ull, mx = 0;
    for (int b = 0; b < blocks; ++b) mn = std::min(mn, h[b * 6]), mx = std::max(mx, h[b * 6 + 5]);
    printf("%-26s blocks %5d  per-launch %6.2f us | kernarg+ld %5.2f  kernarg2 %5.2f  warm-ld %5.2f  cold-ld %5.2f  "
           "store %5.2f  block %5.2f  span %5.2f us\n",
           name, blocks, ms * 1e3 / reps, med(0, 1), med(1, 2), med(2, 3), med(3, 4), med(4, 5), med(0, 5),
           (mx - mn) * 0.01);
}

int main() {
    const int maxb = 2048;
    float *warm, *out, *cold;
    unsigned long long* st;
    (void)hipMalloc(&warm, maxb * 256 * 4 * 2);
    (void)hipMalloc(&out, maxb * 256 * 4 * 2);
    (void)hipMalloc(&cold, (size_t)maxb * 256 * 16 * 4 * 2);
    (void)hipMalloc(&st, maxb * 6 * 8);
    (void)hipMemset(warm, 0, maxb * 256 * 4 * 2);
    (void)hipMemset(out, 0, maxb * 256 * 4 * 2);
    (void)hipMemset(cold, 0, (size_t)maxb * 256 * 16 * 4 * 2);
    for (int blocks : {256, 1024}) {
        BigArgs b{};
        b.warm = warm; b.cold = cold; b.out = out; b.stamps = st; b.far_field = 0;
        SmallArgs s{warm, cold, out, st, 0};
        run("big kernargs (1.2 KB)", b, blocks);
        run("small kernargs (36 B)", s, blocks);
    }
    return 0;
}
