// Prototype (not part of libtvam): the per-forward pattern binning of the voxel-driven planar
// forward (tvam_slice_bin_kernel, tvam_planar.hip: [angle][row][column] -> [angle][column][slice],
// one DMD row per slice in config 2) as a plain transpose, in the production kernel's shape
// (64 x 64 tiles through LDS, one float per thread and step) and with 16-byte accesses (each
// thread loads four columns of a row and stores four slices of a column; the LDS tile is read
// back transposed).  Both write the same layout; the check compares them bit for bit.  Config 2's
// size: 400 angles x 400 rows x 400 columns (256 MB in, 256 MB out).
//
// usage: proto_slice_bin [A R C]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

// the production scheme: block (64 columns, 64 rows, angle), 256 threads, scalar loads / stores
__global__ __launch_bounds__(256) void bin_scalar(const float* __restrict__ in, float* __restrict__ out, int R, int C) {
    __shared__ float t[64][65];
    const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64, a = blockIdx.z;
    const int lc = threadIdx.x & 63, lr = threadIdx.x >> 6;
    const float* pa = in + (size_t)a * R * C;
#pragma unroll 4
    for (int rr = lr; rr < 64; rr += 4) {
        const int r = r0 + rr, c = c0 + lc;
        t[lc][rr] = (r < R && c < C) ? pa[(size_t)r * C + c] : 0.0f;
    }
    __syncthreads();
    float* po = out + (size_t)a * C * R;
    const int r = r0 + lc;
    if (r >= R) return;
    for (int cc = lr; cc < 64; cc += 4)
        if (c0 + cc < C) po[(size_t)(c0 + cc) * R + r] = t[cc][lc];
}

// 16-byte accesses: a thread loads 4 consecutive columns of one row (float4) and stores 4
// consecutive rows (slices) of one column (float4); R and C multiples of 4
__global__ __launch_bounds__(256) void bin_vec4(const float* __restrict__ in, float* __restrict__ out, int R, int C) {
    __shared__ float t[64][65];
    const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64, a = blockIdx.z;
    const int q = threadIdx.x & 15, lr = threadIdx.x >> 4;  // 16 float4 per 64-wide row, 16 rows per step
    const float* pa = in + (size_t)a * R * C;
#pragma unroll
    for (int rr = lr; rr < 64; rr += 16) {
        const int r = r0 + rr, c = c0 + 4 * q;
        float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (r < R && c < C) v = *reinterpret_cast<const float4*>(pa + (size_t)r * C + c);
        t[4 * q + 0][rr] = v.x;
        t[4 * q + 1][rr] = v.y;
        t[4 * q + 2][rr] = v.z;
        t[4 * q + 3][rr] = v.w;
    }
    __syncthreads();
    float* po = out + (size_t)a * C * R;
#pragma unroll
    for (int cc = lr; cc < 64; cc += 16) {
        const int c = c0 + cc, r = r0 + 4 * q;
        if (c < C && r < R)
            *reinterpret_cast<float4*>(po + (size_t)c * R + r) =
                make_float4(t[cc][4 * q], t[cc][4 * q + 1], t[cc][4 * q + 2], t[cc][4 * q + 3]);
    }
}

int main(int argc, char** argv) {
    const int A = argc > 3 ? atoi(argv[1]) : 400, R = argc > 3 ? atoi(argv[2]) : 400, C = argc > 3 ? atoi(argv[3]) : 400;
    if (R % 4 || C % 4) {
        fprintf(stderr, "R and C must be multiples of 4\n");
        return 1;
    }
    const size_t n = (size_t)A * R * C;
    std::vector<float> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000003u) * 1e-6f;
    float *in, *o1, *o2;
    CHECK(hipMalloc(&in, n * 4));
    CHECK(hipMalloc(&o1, n * 4));
    CHECK(hipMalloc(&o2, n * 4));
    CHECK(hipMemcpy(in, h.data(), n * 4, hipMemcpyHostToDevice));
    const dim3 grid((C + 63) / 64, (R + 63) / 64, A);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timeit = [&](int which) {
        float best = 1e30f;
        for (int rep = 0; rep < 20; ++rep) {
            CHECK(hipEventRecord(e0));
            if (which == 0)
                hipLaunchKernelGGL(bin_scalar, grid, dim3(256), 0, 0, in, o1, R, C);
            else
                hipLaunchKernelGGL(bin_vec4, grid, dim3(256), 0, 0, in, o2, R, C);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 3 && ms < best) best = ms;
        }
        return best;
    };
    const float t0 = timeit(0), t1 = timeit(1);
    std::vector<float> r1(n), r2(n);
    CHECK(hipMemcpy(r1.data(), o1, n * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(r2.data(), o2, n * 4, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < n; ++i) diff += r1[i] != r2[i];
    bool ok = diff == 0;
    for (int a = 0; a < A && ok; a += 97)  // spot check against the definition
        for (int r = 0; r < R && ok; r += 13)
            for (int c = 0; c < C; c += 7)
                if (r1[((size_t)a * C + c) * R + r] != h[((size_t)a * R + r) * C + c]) ok = false;
    const double gb = 2.0 * n * 4 / 1e9;
    printf("{\"A\": %d, \"R\": %d, \"C\": %d, \"scalar_us\": %.1f, \"scalar_TBps\": %.2f, \"vec4_us\": %.1f, "
           "\"vec4_TBps\": %.2f, \"identical\": %s}\n",
           A, R, C, t0 * 1e3, gb / t0, t1 * 1e3, gb / t1, ok ? "true" : "false");
    return ok ? 0 : 2;
}
