// Radon filter (integrators/radon.py:47-106, optimize.py:143-163):
// one thread per DMD pixel of the plan's shard, summing its samples'
// weighted target-and-medium absorption (tvam_radon_ray).  The optimiser
// keeps the pixels with radon > 0 ('filter_radon').  Setup-time work: the
// target mesh is tested triangle by triangle (no BVH).
#include "tvam_internal.h"

namespace {

__global__ __launch_bounds__(256) void tvam_radon_kernel(TvamConsts k, TvamTiles tp, const float* __restrict__ tgt,
                                                         int ntgt, int max_depth, float wray,
                                                         float* __restrict__ radon) {
    const int spp = (int)tp.spp;
    const int64_t per_angle = (int64_t)k.crop_y * k.crop_x;
    const int64_t n = (int64_t)tp.n_shard * per_angle;
    for (int64_t local = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; local < n;
         local += (int64_t)gridDim.x * blockDim.x) {
        const int al = (int)(local / per_angle);
        const int64_t pix = local - (int64_t)al * per_angle;
        const int rowc = (int)(pix / k.crop_x), colc = (int)(pix - (int64_t)rowc * k.crop_x);
        const int64_t dense = local + k.shard_base;
        const float2 csv = tp.cs[al];
        float acc = 0.0f;
        for (int smp = 0; smp < spp; ++smp) {
            float jx = 0.5f, jy = 0.5f;
            if (!k.regular) {
                TvamPcg rng;
                rng.seed(tp.seed, (uint64_t)dense * (uint64_t)spp + (uint64_t)smp);
                jx = rng.next_float();
                jy = rng.next_float();
            }
            float xc, yc, ox, oy, oz, dx, dy;
            tvam_ray_camera(k, k.crop_off_x + colc, k.crop_off_y + rowc, jx, jy, xc, yc);
            tvam_ray_world(k, csv.x, csv.y, xc, yc, ox, oy, oz, dx, dy);
            acc += tvam_radon_ray(k, tgt, ntgt, max_depth, ox, oy, oz, dx, dy);
        }
        radon[local] = wray * acc;
    }
}

}  // namespace

hipError_t tvam_launch_radon(const TvamConsts& k, const TvamTiles& t, const float* tgt, int ntgt, int max_depth,
                             float wray, float* radon, hipStream_t stream) {
    const int64_t n = (int64_t)t.n_shard * k.crop_y * k.crop_x;
    int64_t g = (n + 255) / 256;
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(tvam_radon_kernel, dim3((unsigned)g), dim3(256), 0, stream, k, t, tgt, ntgt, max_depth, wray,
                       radon);
    return hipGetLastError();
}
