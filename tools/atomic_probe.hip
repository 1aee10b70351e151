// Throughput of scattered global atomics on MI355X: float vs uint32 vs uint64
// adds to random addresses of a film-sized buffer (tools/, not part of the engine).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}

template <int KIND>
__global__ void probe(void* buf, uint32_t mask, int iters, int walk) {
    uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a = hash32(tid) & mask;
    for (int i = 0; i < iters; ++i) {
        // walk: consecutive visits move to a neighbour (x / y / z step of a 400^3 grid) like a DDA
        uint32_t h = hash32(tid * 977u + i);
        if (walk) a = (a + ((h & 3) == 0 ? 1u : (h & 3) == 1 ? 400u : 160000u)) & mask;
        else a = h & mask;
        if (KIND == 0) atomicAdd(reinterpret_cast<float*>(buf) + a, 1.0f);
        if (KIND == 1) atomicAdd(reinterpret_cast<unsigned*>(buf) + a, 1u);
        if (KIND == 2) atomicAdd(reinterpret_cast<unsigned long long*>(buf) + (a >> 1), 1ull);
        if (KIND == 3) __hip_atomic_fetch_add(reinterpret_cast<float*>(buf) + a, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int main() {
    const uint32_t n = 1u << 26;  // 64M words = 256 MB
    void* buf;
    hipMalloc(&buf, (size_t)n * 8);
    hipMemset(buf, 0, (size_t)n * 8);
    hipEvent_t s, e;
    hipEventCreate(&s);
    hipEventCreate(&e);
    const int threads = 256 * 4096, iters = 64;
    const char* names[] = {"float atomicAdd", "u32 atomicAdd", "u64 atomicAdd", "float hip_atomic relaxed agent"};
    for (int walk = 0; walk < 2; ++walk)
        for (int kind = 0; kind < 4; ++kind) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(s);
                switch (kind) {
                    case 0: hipLaunchKernelGGL(probe<0>, dim3(4096), dim3(256), 0, 0, buf, n - 1, iters, walk); break;
                    case 1: hipLaunchKernelGGL(probe<1>, dim3(4096), dim3(256), 0, 0, buf, n - 1, iters, walk); break;
                    case 2: hipLaunchKernelGGL(probe<2>, dim3(4096), dim3(256), 0, 0, buf, n - 1, iters, walk); break;
                    default: hipLaunchKernelGGL(probe<3>, dim3(4096), dim3(256), 0, 0, buf, n - 1, iters, walk); break;
                }
                hipEventRecord(e);
                hipEventSynchronize(e);
                float ms;
                hipEventElapsedTime(&ms, s, e);
                if (rep) printf("%-34s %s: %.2f ms, %.2f G atomics/s\n", names[kind], walk ? "walk  " : "random", ms,
                                (double)threads * iters / ms / 1e6);
            }
        }
    hipFree(buf);
    return 0;
}
