// mall_probe.hip -- does a default-policy read of a weight slice make a later read of it faster
// (Infinity Cache / L3 hit), for plain and non-temporal 16-B loads?  Standalone probe.
// build: hipcc --offload-arch=gfx950 -O3 mall_probe.hip -o mall_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void __launch_bounds__(256) k_read(const uint4* __restrict__ p, long n16, unsigned* sink) {
    const long per = (long)gridDim.x * 256;
    unsigned acc = 0;
    long e = (long)blockIdx.x * 256 + threadIdx.x;
    for (; e + 7 * per < n16; e += 8 * per) {
        uint4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (NT) {
                u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + e + j * per));
                v[j] = make_uint4(t.x, t.y, t.z, t.w);
            } else {
                v[j] = p[e + j * per];
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc ^= v[j].x ^ v[j].w;
    }
    for (; e < n16; e += per) acc ^= p[e].x;
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const long big = 2L << 30;  // 2 GiB flush buffer
    uint8_t *flush, *w;
    unsigned* sink;
    CK(hipMalloc(&flush, big));
    CK(hipMalloc(&w, 512L << 20));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(flush, 1, big));
    CK(hipMemset(w, 2, 512L << 20));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](bool nt, const void* p, long bytes, int blocks) {
        if (nt) hipLaunchKernelGGL(k_read<true>, dim3(blocks), dim3(256), 0, 0, (const uint4*)p, bytes / 16, sink);
        else hipLaunchKernelGGL(k_read<false>, dim3(blocks), dim3(256), 0, 0, (const uint4*)p, bytes / 16, sink);
    };
    auto timed = [&](bool nt, const void* p, long bytes, int blocks) {
        hipEventRecord(a, 0);
        run(nt, p, bytes, blocks);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        return ms * 1000.f;
    };
    for (long mb : {16L, 32L, 64L, 128L, 200L}) {
        const long bytes = mb << 20;
        for (int warm_nt = 0; warm_nt < 2; ++warm_nt)
            for (int read_nt = 0; read_nt < 2; ++read_nt) {
                float cold = 0, hot = 0, warm_t = 0;
                const int reps = 5;
                for (int r = 0; r < reps; ++r) {
                    run(false, flush, big, 2048);  // evict
                    cold += timed(read_nt, w, bytes, 1024);
                    run(false, flush, big, 2048);
                    warm_t += timed(warm_nt, w, bytes, 1024);  // warm pass
                    hot += timed(read_nt, w, bytes, 1024);
                }
                printf("%4ld MB  warm %s read %s : cold %7.2f us (%5.0f GB/s)  warm-pass %7.2f us  after-warm %7.2f us (%5.0f GB/s)\n",
                       mb, warm_nt ? "nt " : "def", read_nt ? "nt " : "def", cold / reps, bytes / (cold / reps) / 1e3,
                       warm_t / reps, hot / reps, bytes / (hot / reps) / 1e3);
            }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
