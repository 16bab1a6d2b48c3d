// Probe: are parallel branches of a hipGraph dispatched concurrently (ROCm 7.2, MI355X)?
// Each branch is one single-workgroup kernel that idles ~20 us (s_memrealtime).  A second test
// has branch A poll (bounded) a flag that branch B sets: concurrent dispatch => A sees it.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_idle(long ticks) {
    const long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}
__global__ void k_wait(unsigned* flag, unsigned* result, long max_ticks) {
    const long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned seen = 0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < max_ticks) {
        seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (seen) break;
        __builtin_amdgcn_s_sleep(2);
    }
    *result = seen ? 1u : 2u;
}
__global__ void k_set(unsigned* flag, long delay) {
    const long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < delay) __builtin_amdgcn_s_sleep(2);
    __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
    const long T20 = 2000;  // s_memrealtime runs at 100 MHz: 2000 ticks = 20 us
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t fork, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    unsigned *flag, *res;
    CK(hipMalloc(&flag, 4));
    CK(hipMalloc(&res, 4));
    for (int par = 0; par < 2; ++par) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
        hipLaunchKernelGGL(k_idle, dim3(1), dim3(64), 0, s0, T20);
        if (par) {
            CK(hipEventRecord(fork, s0));
            CK(hipStreamWaitEvent(s1, fork, 0));
            hipLaunchKernelGGL(k_idle, dim3(1), dim3(64), 0, s0, T20);
            hipLaunchKernelGGL(k_idle, dim3(1), dim3(64), 0, s1, T20);
            CK(hipEventRecord(join, s1));
            CK(hipStreamWaitEvent(s0, join, 0));
        } else {
            hipLaunchKernelGGL(k_idle, dim3(1), dim3(64), 0, s0, T20);
            hipLaunchKernelGGL(k_idle, dim3(1), dim3(64), 0, s0, T20);
        }
        CK(hipStreamEndCapture(s0, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s0));
        CK(hipStreamSynchronize(s0));
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, s0));
        CK(hipStreamSynchronize(s0));
        double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 20;
        printf("%s: %.1f us per replay (3 x 20 us kernels; serial ~60, 2 concurrent ~40)\n",
               par ? "branches" : "serial", us);
    }
    // flag hand-off across branches: A waits (<= 2 ms) for B, which sets the flag after 10 us
    {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
        CK(hipMemsetAsync(flag, 0, 4, s0));
        CK(hipEventRecord(fork, s0));
        CK(hipStreamWaitEvent(s1, fork, 0));
        hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, s0, flag, res, 200000L);
        hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, s1, flag, 1000L);
        CK(hipEventRecord(join, s1));
        CK(hipStreamWaitEvent(s0, join, 0));
        CK(hipStreamEndCapture(s0, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        int ok = 0;
        for (int i = 0; i < 10; ++i) {
            CK(hipGraphLaunch(ge, s0));
            CK(hipStreamSynchronize(s0));
            unsigned r;
            CK(hipMemcpy(&r, res, 4, hipMemcpyDeviceToHost));
            ok += (r == 1);
        }
        printf("cross-branch flag seen while waiting: %d / 10 replays\n", ok);
    }
    return 0;
}
