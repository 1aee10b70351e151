// Throughput of coalesced global atomics (a wave adds 64 consecutive words at a random 256-B or
// 512-B aligned segment of a 256 MB buffer): f32 add, u64 add, u32 add, plain f32 stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ __launch_bounds__(256) void k_atom(void* buf, uint64_t nseg, int iters) {
    uint32_t s = blockIdx.x * 2654435761u + (threadIdx.x >> 6) * 40503u + 12345u;
    const int lane = threadIdx.x & 63;
    for (int i = 0; i < iters; ++i) {
        s = s * 1664525u + 1013904223u;
        const uint64_t seg = (uint64_t)(__builtin_amdgcn_readfirstlane(s) % (uint32_t)nseg);
        if (MODE == 0) atomicAdd(reinterpret_cast<float*>(buf) + seg * 64 + lane, 1.0f);
        if (MODE == 1) atomicAdd(reinterpret_cast<unsigned long long*>(buf) + seg * 64 + lane, 1ull);
        if (MODE == 2) atomicAdd(reinterpret_cast<unsigned*>(buf) + seg * 64 + lane, 1u);
        if (MODE == 3) reinterpret_cast<float*>(buf)[seg * 64 + lane] = (float)i;
    }
}

int main() {
    void* buf;
    const size_t bytes = 512ull << 20;
    hipMalloc(&buf, bytes);
    hipMemset(buf, 0, bytes);
    const char* names[] = {"f32 atomic add", "u64 atomic add", "u32 atomic add", "f32 store"};
    const int iters = 256, blocks = 8192;
    for (int m = 0; m < 4; ++m) {
        const uint64_t nseg = (256ull << 20) / (m == 1 ? 512 : 256);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0, 0);
            if (m == 0) hipLaunchKernelGGL(k_atom<0>, dim3(blocks), dim3(256), 0, 0, buf, nseg, iters);
            if (m == 1) hipLaunchKernelGGL(k_atom<1>, dim3(blocks), dim3(256), 0, 0, buf, nseg, iters);
            if (m == 2) hipLaunchKernelGGL(k_atom<2>, dim3(blocks), dim3(256), 0, 0, buf, nseg, iters);
            if (m == 3) hipLaunchKernelGGL(k_atom<3>, dim3(blocks), dim3(256), 0, 0, buf, nseg, iters);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
        }
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double ops = (double)blocks * 256 * iters;
        printf("%-16s %.3f ms  %.3g lane-ops/s  %.3g wave-ops/s  %.1f GB/s payload\n", names[m], ms, ops / ms * 1e3,
               ops / 64 / ms * 1e3, ops * (m == 1 ? 8 : 4) / ms / 1e6);
    }
    return 0;
}
