// Microbenchmark: which lanes of a ds_read_b128 share an LDS cycle (bank-conflict groups).
// Each lane reads 16 bytes at chunk c(lane) (address 16 c); cycles per read by pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(1024) void probe(const int* __restrict__ chunk, long long* __restrict__ out, float* sink) {
    __shared__ __attribute__((aligned(16))) float lds[8192 * 4];
    for (int i = threadIdx.x; i < 8192 * 4; i += 1024) lds[i] = (float)i;
    __syncthreads();
    const int a = chunk[threadIdx.x & 63] * 16 + (int)(size_t)(&lds[0]);
    float acc = 0.0f;
    const long long t0 = clock64();
#pragma unroll 1
    for (int it = 0; it < 16384; ++it) {
        float4 v0, v1, v2, v3;
        asm volatile("ds_read_b128 %0, %4\n ds_read_b128 %1, %4 offset:4096\n ds_read_b128 %2, %4 offset:8192\n ds_read_b128 %3, %4 offset:12288\n ds_read_b128 %0, %4 offset:16\n ds_read_b128 %1, %4 offset:4112\n ds_read_b128 %2, %4 offset:8208\n ds_read_b128 %3, %4 offset:12304\n s_waitcnt lgkmcnt(0)"
                     : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3) : "v"(a));
        acc += v0.x + v1.y + v2.z + v3.w;
    }
    const long long t1 = clock64();
    __syncthreads();
    const long long t2 = clock64();
    if (threadIdx.x == 0) out[blockIdx.x] = t2 - t0;
    sink[threadIdx.x & 63] = acc + lds[(threadIdx.x * 37) & 8191];
}

int main() {
    static const int LG[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                  {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                  {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                  {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
    const char* names[] = {"lane%16 (contiguous groups distinct)", "LG-distinct", "all same address", "lane (64 chunks)",
                           "LG-distinct, one 2-way pair per LG group", "contiguous 16s, 2-way pairs (l, l+8)",
                           "lane%16 + 16*(lane/16) (distinct residues in contiguous 16s, different rows)",
                           "LG-distinct + 16*lane (different rows)", "16*lane (all residue 0)",
                           "(l%16)/2 + 16*l (2-way both models)", "LG pos j/2 + 8*(g&1) + 16*l (2-way in LG only?)"};
    const int NP = 11;
    int *d_c;
    long long* d_o;
    float* d_s;
    hipMalloc(&d_c, 64 * sizeof(int));
    hipMalloc(&d_o, 256 * sizeof(long long));
    hipMalloc(&d_s, 64 * sizeof(float));
    for (int p = 0; p < NP; ++p) {
        std::vector<int> c(64);
        for (int l = 0; l < 64; ++l) c[l] = 0;
        for (int g = 0; g < 4; ++g)
            for (int j = 0; j < 16; ++j) {
                const int l = LG[g][j];
                switch (p) {
                    case 0: c[l] = l % 16; break;
                    case 1: c[l] = j; break;
                    case 2: c[l] = 0; break;
                    case 3: c[l] = l; break;
                    case 4: c[l] = j == 1 ? 0 : j; break;
                    case 5: c[l] = (l % 16) % 8; break;
                    case 6: c[l] = l % 16 + 16 * (l / 16); break;
                    case 7: c[l] = j + 16 * l; break;
                    case 8: c[l] = 16 * l; break;
                    case 9: c[l] = (l % 16) / 2 + 16 * l; break;
                    case 10: c[l] = j / 2 + 8 * (g & 1) + 16 * l; break;
                }
            }
        hipMemcpy(d_c, c.data(), 64 * sizeof(int), hipMemcpyHostToDevice);
        hipLaunchKernelGGL(probe, dim3(256), dim3(1024), 0, 0, d_c, d_o, d_s);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(probe, dim3(256), dim3(1024), 0, 0, d_c, d_o, d_s);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        long long t;
        hipMemcpy(&t, d_o, sizeof(long long), hipMemcpyDeviceToHost);
        printf("  %.3f ms = %.2f ns per wave-read per CU; clock64 %.3g\n", ms, ms * 1e6 / (16384.0 * 8 * 16), (double)t);
        printf("%-80s\n", names[p]);
    }
    return 0;
}
