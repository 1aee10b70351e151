// tvam_internal.h — plan layout and kernel launchers shared by tvam_plan.hip
// and tvam_kernels.hip (not part of the public ABI).
#pragma once
#include "tvam_common.h"
#include "../../include/tvam.h"

// Device tables that drive one tile launch.
struct TvamTiles {
    const float2* cs;          // [n_shard] (cos, sin) of each angle of the shard
    const int32_t* slice_off;  // [res_z + 1] CSR offsets into slice_rows
    const int32_t* slice_rows; // crop-local DMD rows feeding each z-slice
    const int32_t* col_lo;     // [ntiles][n_shard] first crop-local column crossing the tile
    const int32_t* col_hi;     // [ntiles][n_shard] last crop-local column crossing the tile
    const int32_t* col_off;    // [ntiles][n_shard + 1] prefix sums of column-PAIR counts ceil(n/2)
    const float4* ang;         // [n_shard] {tstep_x, tstep_y, step_x, step_y} (sensor.py:343, :360)
    const float4* ray_f;       // [n_shard*crop_y*crop_x*spp] {t_start, tau_end, dtmax0_x, dtmax0_y}
    const int2* ray_i;         // same index: {start voxel x | y << 16, z-slice or -1}
    int32_t ntx, nty, tsx, tsy;
    int32_t n_shard;
    uint32_t spp, seed;
};

enum TvamMode { TVAM_MODE_FWD = 0, TVAM_MODE_ADJ = 1, TVAM_MODE_COUNT = 2 };

hipError_t tvam_launch_tiles(int mode, const TvamConsts& k, const TvamTiles& t, size_t lds_bytes,
                             const float* pat, const int32_t* idxmap, const float* gin, float* out,
                             unsigned long long* counter, hipStream_t stream);

// Per-ray pre-pass: ray generation, vial segment and DDA initialisation of
// every ray of the shard, stored as the records the tile kernels resume from.
hipError_t tvam_launch_ray_setup(const TvamConsts& k, const TvamTiles& t, float4* ray_f, int2* ray_i,
                                 hipStream_t stream);

hipError_t tvam_launch_scatter(const TvamConsts& k, const float* data, const uint32_t* pixels,
                               uint64_t n, float* dense, int32_t* idxmap, hipStream_t stream);

hipError_t tvam_launch_gather(const TvamConsts& k, const float* dense, const uint32_t* pixels,
                              uint64_t n, float* out, hipStream_t stream);

hipError_t tvam_launch_loss_threshold(const float* dose, const float* ddose, float alpha,
                                      const float* target, uint64_t n, int K, float tl, float tu,
                                      float w_object, float w_void, float w_limit, float scale,
                                      double* out, float* grad, hipStream_t stream);
