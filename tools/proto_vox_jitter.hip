// Prototype (not part of libtvam): a voxel-driven (gather-form) forward for JITTERED parallel rays,
// measured at config 5's size to see whether it could replace the per-ray tile kernels of the
// jittered first segments.  It is a LOWER BOUND on such a
// kernel's cost: straight rays (no vial refraction, no occluder), every ray inside its DMD row's
// slice (no vertical jitter across slices), no absorption (a per-ray factor and a per-voxel factor,
// both outside the candidate loop, would add nothing per candidate).  What it does keep is the part
// that jitter makes per slice: each (angle, row, column) has spp rays at independent lateral
// positions u, so every voxel of every slice tests the ~3 columns x spp rays whose band can reach it
// and adds chord length x value (the chord of a line through a unit square is a trapezoid in the
// lateral offset d: min(Lmax, (hw - |d|) / (|cos| |sin|)), clamped at 0).
//
//   grid N^3 voxels (unit cells, centred), A angles, C = N columns, spp rays per pixel;
//   workgroup: a 32 x 32 voxel tile x ZS slices, all angles; per angle the rays of the tile's
//   column window (ZS slices x W columns x spp float2 {u, value}) are staged in LDS (double
//   buffered), each thread owns 4 voxel columns x ZS slices of accumulators.
//
// usage: proto_vox_jitter N A SPP [check]   (check: a small case against a CPU Liang-Barsky clip)
#include <hip/hip_runtime.h>

#include <cmath>
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

constexpr int TX = 32, TY = 32, ZS = 8, NT = 256, WMAX = 52, SPPMAX = 4;

__host__ __device__ inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// ray (a, z, c, s): u = c - C/2 + jitter, value in [0, 1)
__host__ __device__ inline void ray_of(uint64_t i, int C, float2& r) {
    const uint32_t h1 = hash32((uint32_t)i * 2u + 1u), h2 = hash32((uint32_t)(i >> 31) ^ ((uint32_t)i * 2u + 2u) * 0x9e3779b9u);
    const int c = (int)((i / SPPMAX) % (uint64_t)C);
    r.x = (float)c - 0.5f * (float)C + (float)(h1 >> 8) * (1.0f / 16777216.0f);
    r.y = (float)(h2 >> 8) * (1.0f / 16777216.0f);
}

__global__ void fill_rays(float2* rays, uint64_t n, int C) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        ray_of(i, C, rays[i]);
}

// rays: [A][N slices][C][SPPMAX] float2; out: [N][N][N] (z, y, x)
__global__ __launch_bounds__(NT) void gather_fwd(const float2* __restrict__ rays, const float2* __restrict__ cs,
                                                 int N, int A, float* __restrict__ out) {
    __shared__ float4 sh[2][ZS][WMAX][SPPMAX / 2];
    const int ntx = N / TX;
    const int tile = blockIdx.x % (ntx * (N / TY)), zc = blockIdx.x / (ntx * (N / TY));
    const int x0 = (tile % ntx) * TX, y0 = (tile / ntx) * TY, z0 = zc * ZS;
    const int C = N;
    const int tx = threadIdx.x % TX, ty4 = (threadIdx.x / TX) * 4;
    const float half = 0.5f * (float)N;
    float acc[4][ZS];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int z = 0; z < ZS; ++z) acc[i][z] = 0.0f;
    // window base column of angle a (tile corners' lateral extent)
    auto wbase = [&](float c, float s) {
        const float xa = (float)x0 - half, xb = xa + (float)TX, ya = (float)y0 - half, yb = ya + (float)TY;
        const float u0 = fminf(fminf(-xa * s + ya * c, -xb * s + ya * c), fminf(-xa * s + yb * c, -xb * s + yb * c));
        return (int)floorf(u0 - 1.0f + half);
    };
    auto stage = [&](int a, int buf) {
        const float2 t = cs[a];
        const int cb = wbase(t.x, t.y);
        // ZS x WMAX columns x 2 float4 (4 rays)
        for (int q = threadIdx.x; q < ZS * WMAX * 2; q += NT) {
            const int h = q & 1, col = (q >> 1) % WMAX, z = (q >> 1) / WMAX;
            const int cc = cb + col;
            float4 v = make_float4(1e30f, 0.0f, 1e30f, 0.0f);  // outside the film: no contribution
            if (cc >= 0 && cc < C)
                v = reinterpret_cast<const float4*>(rays)[((((size_t)a * N + (z0 + z)) * C + cc) * SPPMAX) / 2 + h];
            sh[buf][z][col][h] = v;
        }
    };
    stage(0, 0);
    __syncthreads();
    for (int a = 0; a < A; ++a) {
        const int buf = a & 1;
        if (a + 1 < A) stage(a + 1, buf ^ 1);
        const float2 t = cs[a];
        const float c = t.x, s = t.y, ac = fabsf(c), as = fabsf(s);
        const float hw = 0.5f * (ac + as), lmax = 1.0f / fmaxf(ac, as), k = fminf(1.0f / (ac * as), 1e30f);
        const int cb = wbase(c, s);
        const float xc = (float)(x0 + tx) + 0.5f - half;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float yc = (float)(y0 + ty4 + i) + 0.5f - half;
            const float uc = -xc * s + yc * c;
            const int clo = (int)floorf(uc - hw + half) - cb;  // first candidate column in the window
#pragma unroll
            for (int z = 0; z < ZS; ++z) {
                float sum = 0.0f;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int col = min(clo + j, WMAX - 1);
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const float4 r = sh[buf][z][col][h];
                        const float l0 = fminf(fmaxf(k * (hw - fabsf(r.x - uc)), 0.0f), lmax);
                        const float l1 = fminf(fmaxf(k * (hw - fabsf(r.z - uc)), 0.0f), lmax);
                        sum = fmaf(l0, r.y, sum);
                        sum = fmaf(l1, r.w, sum);
                    }
                }
                acc[i][z] += sum;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int z = 0; z < ZS; ++z)
            out[(((size_t)(z0 + z) * N) + (y0 + ty4 + i)) * N + (x0 + tx)] = acc[i][z];
}

// chord of the line {p : -p.x s + p.y c = u} through the unit cell centred at (xc, yc) (Liang-Barsky)
static double clip_len(double u, double c, double s, double xc, double yc) {
    // a point on the line and its direction (c, s)
    const double px = -u * s, py = u * c;
    double t0 = -1e30, t1 = 1e30;
    const double lo[2] = {xc - 0.5, yc - 0.5}, hi[2] = {xc + 0.5, yc + 0.5}, p[2] = {px, py}, d[2] = {c, s};
    for (int a = 0; a < 2; ++a) {
        if (std::fabs(d[a]) < 1e-15) {
            if (p[a] < lo[a] || p[a] > hi[a]) return 0.0;
            continue;
        }
        double ta = (lo[a] - p[a]) / d[a], tb = (hi[a] - p[a]) / d[a];
        if (ta > tb) std::swap(ta, tb);
        t0 = std::max(t0, ta);
        t1 = std::min(t1, tb);
    }
    return t1 > t0 ? t1 - t0 : 0.0;
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 800, A = argc > 2 ? atoi(argv[2]) : 800;
    const int spp = argc > 3 ? atoi(argv[3]) : 4;
    const bool check = argc > 4;
    if (N % TX || N % ZS || spp != SPPMAX) {
        fprintf(stderr, "N must be a multiple of 32 and of %d, spp %d\n", ZS, SPPMAX);
        return 1;
    }
    const int C = N;
    const uint64_t nr = (uint64_t)A * N * C * SPPMAX;
    std::vector<float2> hcs(A);
    for (int a = 0; a < A; ++a) {
        const double th = 2.0 * M_PI * (a + 0.37) / A;
        hcs[a] = make_float2((float)std::cos(th), (float)std::sin(th));
    }
    float2 *rays, *cs;
    float* out;
    CHECK(hipMalloc(&rays, nr * sizeof(float2)));
    CHECK(hipMalloc(&cs, A * sizeof(float2)));
    CHECK(hipMalloc(&out, (size_t)N * N * N * sizeof(float)));
    CHECK(hipMemcpy(cs, hcs.data(), A * sizeof(float2), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(fill_rays, dim3(8192), dim3(256), 0, 0, rays, nr, C);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    const int nblk = (N / TX) * (N / TY) * (N / ZS);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = check ? 1 : 3;
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(gather_fwd, dim3(nblk), dim3(NT), 0, 0, rays, cs, N, A, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.0f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms);
        printf("{\"N\": %d, \"angles\": %d, \"spp\": %d, \"rep\": %d, \"ms\": %.3f}\n", N, A, spp, r, ms);
        fflush(stdout);
    }
    const double vox_ang = (double)N * N * N * A;
    printf("{\"N\": %d, \"angles\": %d, \"spp\": %d, \"best_ms\": %.3f, \"voxel_angles_per_s\": %.4g}\n", N, A, spp, best,
           vox_ang / (best * 1e-3));
    if (check) {  // a few slices against the CPU clip over every ray of the slice
        std::vector<float> h((size_t)N * N * N);
        CHECK(hipMemcpy(h.data(), out, h.size() * sizeof(float), hipMemcpyDeviceToHost));
        double err = 0.0, ref2 = 0.0;
        for (int z : {0, N / 2 + 3, N - 1}) {
            std::vector<double> ref((size_t)N * N, 0.0);
            for (int a = 0; a < A; ++a)
                for (int c = 0; c < C; ++c)
                    for (int s = 0; s < SPPMAX; ++s) {
                        float2 r;
                        ray_of((((uint64_t)a * N + z) * C + c) * SPPMAX + s, C, r);
                        for (int y = 0; y < N; ++y)
                            for (int x = 0; x < N; ++x)
                                ref[(size_t)y * N + x] += r.y * clip_len(r.x, hcs[a].x, hcs[a].y, x + 0.5 - 0.5 * N,
                                                                         y + 0.5 - 0.5 * N);
                    }
            for (size_t i = 0; i < ref.size(); ++i) {
                const double d = h[(size_t)z * N * N + i] - ref[i];
                err += d * d;
                ref2 += ref[i] * ref[i];
            }
        }
        const double rel = std::sqrt(err / ref2);
        printf("{\"check_rel_l2\": %.3e}\n", rel);
        return rel < 1e-5 ? 0 : 2;
    }
    return 0;
}
