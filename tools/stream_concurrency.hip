// Calibration (tools only): do kernels on two HIP streams overlap on this box — eagerly, and when each
// stream replays its own hipGraph?  One single-block spin kernel of ~100 us per stream.
//   hipcc -O3 --offload-arch=gfx950 tools/stream_concurrency.hip -o tools/bin/stream_concurrency
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void spin(unsigned long long cycles, int* out) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < cycles) {
    }
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

static float run(hipStream_t a, hipStream_t b, bool two, unsigned long long cyc, int* out, int reps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, a);
    (void)hipStreamWaitEvent(b, e0, 0);
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, cyc, out);
        if (two) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, b, cyc, out + 1);
    }
    hipEvent_t eb;
    (void)hipEventCreate(&eb);
    (void)hipEventRecord(eb, b);
    (void)hipStreamWaitEvent(a, eb, 0);
    (void)hipEventRecord(e1, a);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    int* out;
    (void)hipMalloc(&out, 4096);
    hipStream_t a, b;
    (void)hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
    const unsigned long long cyc = 200000;   // ~100 us at ~2 GHz
    run(a, b, true, cyc, out, 2);
    printf("eager  one stream x10 : %.3f ms\n", run(a, b, false, cyc, out, 10));
    printf("eager  two streams x10: %.3f ms (overlap if ~= one stream)\n", run(a, b, true, cyc, out, 10));
    // graphs: each stream captures 10 launches, then both graphs are launched on their streams
    hipGraph_t ga, gb;
    hipGraphExec_t xa, xb;
    (void)hipStreamBeginCapture(a, hipStreamCaptureModeGlobal);
    for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, cyc, out);
    (void)hipStreamEndCapture(a, &ga);
    (void)hipStreamBeginCapture(b, hipStreamCaptureModeGlobal);
    for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, b, cyc, out + 1);
    (void)hipStreamEndCapture(b, &gb);
    (void)hipGraphInstantiate(&xa, ga, nullptr, nullptr, 0);
    (void)hipGraphInstantiate(&xb, gb, nullptr, nullptr, 0);
    for (int pass = 0; pass < 2; ++pass) {
        hipEvent_t e0, e1, eb;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventCreate(&eb);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0, a);
        (void)hipStreamWaitEvent(b, e0, 0);
        (void)hipGraphLaunch(xa, a);
        if (pass == 1) (void)hipGraphLaunch(xb, b);
        (void)hipEventRecord(eb, b);
        (void)hipStreamWaitEvent(a, eb, 0);
        (void)hipEventRecord(e1, a);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("graphs %s: %.3f ms\n", pass ? "two streams x10" : "one stream x10 ", ms);
    }
    return 0;
}
