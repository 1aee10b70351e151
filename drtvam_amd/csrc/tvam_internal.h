// tvam_internal.h — plan layout and kernel launchers shared by tvam_plan.hip
// and tvam_kernels.hip (not part of the public ABI).
#pragma once

// Row pitch (voxels) of the per-ray tile kernels' LDS tile (tile + 1-voxel guard band): odd, so
// that lanes stepping through one tile column (stride = pitch) never share an LDS bank.  An even
// pitch of 64 (800^3 tiles of 62) put a whole column on one bank: 86 % of the forward's LDS cycles
// were bank-conflict stalls.
#define TVAM_TILE_PITCH(tsx) (((tsx) + 2) | 1)

#include <vector>

#include "tvam_common.h"
#include "../../include/tvam.h"

// A tuning knob: the environment variable `name` under TVAM_EXPERIMENTAL=1 (logged), else `def`
// (tvam_plan.hip).
int tvam_knob(const char* name, int def);
// Launch timer of the dominant forward kernel (tvam_plan_kernel_time): while enabled, each launch
// of the measured plan's dominant kind -- the voxel-driven planar forward, the per-ray tile
// forward or the forward brick march -- is bracketed by two HIP events on its stream.
enum TvamKtKind { TVAM_KT_PLANAR = 0, TVAM_KT_TILE = 1, TVAM_KT_BRICK = 2 };
void tvam_kt_begin(hipStream_t stream, int kind);
void tvam_kt_end(hipStream_t stream, int kind);
// the next timer event pair for a launch that records them itself (hipExtLaunchKernelGGL); false: untimed
bool tvam_kt_take(int kind, hipEvent_t* start, hipEvent_t* stop);

// Device tables that drive one tile launch.
struct TvamTiles {
    const float2* cs;          // [n_shard] (cos, sin) of each angle of the shard
    const int32_t* slice_off;  // [res_z + 1] CSR offsets into slice_rows
    const int32_t* slice_rows; // crop-local DMD rows feeding each z-slice
    const uint32_t* slots;     // per tile: (shard angle << 16 | crop column) of every ray crossing it,
                               // sorted by predicted in-tile visits (longest first)
    const int64_t* slot_off;   // [ntiles + 1] offsets into slots
    const float4* ang;         // [n_shard] {tstep_x, tstep_y, step_x, step_y} (sensor.py:343, :360)
    const float4* ray_f;       // [n_shard*crop_y*crop_x*spp] {t_start, tau_end, dtmax0_x, dtmax0_y}
    const int2* ray_i;         // same index: {start voxel x | y << 16, z-slice or -1}
    const float4* ray_g;       // same index, refracting vials only: {+-tstep_x, +-tstep_y (sign = step),
                               // interface weight, 0}; nullptr: straight rays (per-angle ang[])
    int32_t ntx, nty, tsx, tsy;
    int32_t n_shard;
    uint32_t spp, seed;
    int64_t* frozen;              // ray indices marked frozen by the ray setup (ray_i.y <= -2), appended
    unsigned long long* frozen_n; // their count (beyond frozen_cap: the frozen kernel scans ray_i instead)
    int64_t frozen_cap;
    int32_t kz0, kz1;             // forward launches: local film slices [kz0, kz1) (tvam_forward_slices)
    // Jittered rows whose rays reach neighbouring slices only at the sampler's extreme jitters
    // (config 4 / 5: 1:1 rows, one ray in ~10^4 elsewhere; tvam_plan.hip): each slice then enumerates
    // its main rows (row_main: the slice of the row's centre ray), and the few rays outside their
    // row's main slice ("strays", listed by the ray setup, sorted by slice per record set) join the
    // workgroup of their slice.  slice_moff = nullptr: every slice enumerates its full row list.
    const int32_t* slice_moff;    // [res_z + 1] CSR offsets into slice_mrows
    const int32_t* slice_mrows;
    const int32_t* row_main;      // [crop_y] local main slice of each crop row (-1: none)
    uint32_t* stray_idx;          // ray setup: stray record indices, appended (capacity stray_cap)
    uint32_t* stray_cnt;          // [res_z + 1] strays per local slice (the scan's cursor afterwards)
    uint32_t* stray_off;          // [res_z + 1] CSR offsets into stray_list
    uint32_t* stray_list;         // stray record indices by slice
    unsigned long long* stray_n;  // strays found (beyond stray_cap: the workgroups use the full row lists)
    uint32_t stray_cap;
};

// Planar fast path of regular sampling (tvam_planar.hip): one ray record per
// (angle, DMD column), shared by every DMD row.
struct TvamPlanar {
    const float2* cs;          // [ns] (cos, sin) of each angle of the shard
    float4* vox;               // [ns][crop_x] {qx, qy, t_end, 0} (voxel-driven forward)
    float4* rec_f;             // [ns][crop_x] {t_start, tau_end, dtmax0_x, dtmax0_y} (tile DDA resume)
    int32_t* rec_i;            // [ns][crop_x] start voxel x | y << 16, -1 if the ray misses
    float4* rec_g;             // [ns][crop_x] refracting vials: {+-tstep_x, +-tstep_y, weight, 0}; else nullptr
    const int32_t* slice_off;  // [res_z + 1] CSR: DMD rows whose rays lie in each slice
    const int32_t* slice_rows;
    int32_t ns;
    int32_t ncmax;             // forward: DMD columns staged per (16 x 16 tile, angle)
    float marg_u;              // forward: candidate-column margin (spawn offset of o2 + rounding), in columns
    float u0;                  // forward: crop column of lateral coordinate 0 (0.5 W - 0.5 - crop_off_x)
    int32_t fwd_nc;            // forward: candidate columns per (voxel, angle)
    int32_t fwd_multi;         // forward: some slice collects several DMD rows
    const float4* fwd_ang;     // forward: [ns][2] {s du, -c du, 1/d.x, 1/d.y}, {half width + margin, axis flags}
    const int32_t* fwd_cb;     // forward: [16 x 16 tiles][ns] first column of the staged window
    int32_t fwd_pf;            // forward: staged values per thread and angle (2 or 4)
    int32_t max_rows_chunk;    // adjoint: most DMD rows in one chunk of Z slices
    int32_t adj_pitch;         // adjoint: LDS row pitch of the gradient tile in voxels (>= tile + 2)
    int32_t max_rows_slice;    // ray-driven forward: most DMD rows in one slice (fixed-point bound)
    int32_t adj_split;         // adjoint: workgroups sharing one (tile, slice chunk)'s ray list (thin slabs)
    int32_t adj_nt;            // adjoint: threads per workgroup (256 or 512)
    int32_t rayfwd_pitch;      // ray-driven forward: LDS row pitch of its dose tile (>= tile + 2)
    int32_t rayfwd_nt;         // ray-driven forward: threads per workgroup (256 or 512)
    int32_t fwd_parts;         // forward: angle parts per (tile, slice chunk) (thin slabs; 1 = none)
    int32_t fwd_ab;            // forward: angles per barrier (1 or 2)
    int32_t fwd_dma;           // forward: binned slabs staged by LDS-DMA (tvam_planar_fwd_dma_ok)
    float* fwd_part;           // forward: [fwd_parts][nz][res_y][res_x] partial doses when fwd_parts > 1
    float* fwd_bin;            // forward: [ns][crop_x + 2 bin_pad][bin_nz] slice-binned patterns (nullptr: staged
                               // from the [row][col] patterns directly)
    int32_t bin_pad;           // forward: zero columns on either side of the binned patterns (= ncmax)
    int32_t bin_nz;            // forward: slices per binned column (nz rounded up to the slab depth Z)
    // voxel-driven forward behind a refracting vial (fwd_refr = 1): every column's chord has its
    // own direction, and the candidate columns of a voxel come from a per-(16x16 tile, angle)
    // bilinear model of the chord index u(x, y) (tvam_refr_model_kernel)
    int32_t fwd_zc0, fwd_nzc;  // voxel-driven forward launch: slice chunks [zc0, zc0 + nzc) of Z slices (0, 0: all)
    int32_t adj_zc0, adj_nzc;  // planar adjoint launch: slice chunks [zc0, zc0 + nzc) of Z slices (0, 0: all)
    int32_t fwd_refr;
    float4* vox2;              // [ns][crop_x] {1/d.x, 1/d.y, axis flags (int bits), interface weight}
    float4* chord;             // plan creation only: [ns][crop_x] {o2.x, o2.y, d2.x, d2.y} of the medium chord
    const float4* fwd_model;   // [16x16 tiles][ns][2] {u00, du/dlx, du/dly, d2u/dlx dly},
                               //   {half width + model error, candidates (int bits), first window column (int bits), 0}
    // adjoint over slice-invariant visit lists (tvam_adjlist.hip; adjl_ngroups = 0: the tile adjoint)
    const int32_t* adjl_gchunk;  // [ngroups + 1] first chunk of each (tile, part) group
    const int64_t* adjl_coff;    // [nchunks + 1] first float4 row of each chunk's weights
    const int4* adjl_hdr;        // [nchunks][64] {entry LDS offset, slot, interface weight bits, x | y step << 16}
    const float4* adjl_w;        // [rows][64] weights, 4 visits per float4, LSB = y step after the visit
    const int32_t* adjl_glist;   // [nlist] the groups that hold chunks, in group order (the grid's groups)
    int32_t adjl_ngroups, adjl_parts;  // groups = (tile, step quadrant, part)
    int32_t adjl_nlist;                // groups that hold chunks
    int32_t adjl_tw0, adjl_tw1;        // row pitch (voxels) for equal / opposite step signs: 1 / 15 (mod 16)
    int32_t adjl_slack;                // zeroed bytes around each plane (padding visits walk there)
    int32_t adjl_z;                    // slices per workgroup (8 or 16)
};

// Device buffers of the visit lists (owned by the plan).
struct TvamAdjListBufs {
    int32_t* gchunk = nullptr;
    int32_t* glist = nullptr;
    int64_t* coff = nullptr;
    int4* hdr = nullptr;
    float4* w = nullptr;
    size_t bytes = 0;
    int64_t visits_padded = 0;
};
size_t tvam_adjl_lds(const TvamPlanar& pl, const TvamTiles& t, int Z);
hipError_t tvam_build_adj_lists(const TvamConsts& k, TvamPlanar& pl, const TvamTiles& t, int parts, size_t max_bytes,
                                TvamAdjListBufs& bufs, hipStream_t stream);
hipError_t tvam_launch_adj_lists(const TvamConsts& k, const TvamPlanar& pl, const TvamTiles& t, int Z,
                                 const int32_t* idxmap, const float* gin, float* out, hipStream_t stream);

hipError_t tvam_launch_planar_rays(const TvamConsts& k, const TvamPlanar& pl, hipStream_t stream);
// Refracted voxel-driven forward: per (16x16 tile, angle) model of the chord index (needs pl.chord);
// model: [tiles][ns][2] float4, need: [tiles][ns] window width in columns.  range: [ns] first / last
// column whose chord reaches the medium.
hipError_t tvam_launch_refr_model(const TvamConsts& k, const TvamPlanar& pl, const int2* range, float4* model,
                                  int32_t* need, hipStream_t stream);
size_t tvam_planar_fwd_lds(const TvamPlanar& pl, int Z);
bool tvam_planar_fwd_fits(const TvamPlanar& pl, int Z);
bool tvam_planar_fwd_dma_ok(const TvamPlanar& pl, int Z);
bool tvam_planar_fwd_dma_window(const TvamPlanar& pl, int Z);
hipError_t tvam_launch_fwd_planar(const TvamConsts& k, const TvamPlanar& pl, int Z, const float* pat, float* dose,
                                  hipStream_t stream);
size_t tvam_planar_adj_lds(const TvamPlanar& pl, const TvamTiles& t, int Z);
hipError_t tvam_launch_adj_planar(const TvamConsts& k, const TvamPlanar& pl, const TvamTiles& t, int Z,
                                  const int32_t* idxmap, const float* gin, float* out, hipStream_t stream);
// Ray-driven planar forward (refracted rays, fine DMDs): per-angle max |pattern| ->
// fixed-point scale (amax: [ns] scratch, scale: [2]) -> Z-slice-sharing march.
size_t tvam_planar_rayfwd_lds(const TvamPlanar& pl, const TvamTiles& t, int Z);
hipError_t tvam_launch_fwd_rays_planar(const TvamConsts& k, const TvamPlanar& pl, const TvamTiles& t, int Z,
                                       const float* pat, unsigned* amax, float* scale, float* dose,
                                       hipStream_t stream);

enum TvamMode { TVAM_MODE_FWD = 0, TVAM_MODE_ADJ = 1, TVAM_MODE_COUNT = 2, TVAM_MODE_EMIT = 3 };

// float4s per brick-bin segment record (48 B; 64-B aligned records measured +0.4 % on config 4:
// their third more bytes leave fewer chunks in the forward bin cache)
#define TVAM_REC_F4 3
// Brick of the binned scattered-segment forward (LDS int64 tile: 128 KB)
#define TVAM_BX 32
#define TVAM_BY 32
#define TVAM_BZ 16
// brick-bin sort keys: brick id << TVAM_BIN_CLASS_BITS | class of the entry's predicted in-brick
// visit count (entries of one brick run in class order: similar march lengths per wave)
#define TVAM_BIN_CLASS_BITS 4

// Scattered segments of paths [p0, p1): `slots` records per path
// (a = {t_start, tau_end, dtm0_x, dtm0_y}, b = {dtm0_z, +-ts_x, +-ts_y, +-ts_z},
// c = {start voxel x | y << 11 | z << 22, weight bits}), m = bricks crossed (0: empty).
struct TvamSegBuf {
    int64_t p0, p1;
    int32_t slots;
    int32_t adj;                  // records for the adjoint (weight att * wscale)
    float4* r;                    // [slots][3] segment records (48 B, one cache-line span per gather)
    uint32_t* m;
    uint32_t* wmax;               // forward: max |record weight| of the chunk (float bits, atomicMax)
    // counting-sort bins (tvam_scatter_binned without TVAM_BIN_SORT): the record writer's per
    // (brick, workgroup) entry counts, [nbricks][gridDim.x]; nullptr: the radix-sort path
    uint32_t* hist;
    int32_t nbricks;
    uint32_t* bad;                // bin fill: slots whose walk disagreed with the writer's count
};
// a radix-path bin entry (segment slot) that marches nothing: padding of a slot whose walk fell
// short of its count (slots stay below 2^31)
#define TVAM_ENT_NULL 0x80000000u

// One chunk of forward bins kept in HBM for the next forward of the same (seed, spp): an
// optimiser iteration renders seed i twice (the forward and the line-search forward, the
// paths' geometry does not depend on the pattern), so the second call skips the path replay,
// the scan, the bin fill and the sort, rescales the records' weights to the new pattern and
// marches.  c.z of each record holds the path attenuation for that rescale.
struct TvamBinChunk {
    float4* r = nullptr;          // [3 * cap_slots] records
    int64_t cap_slots = 0;
    uint32_t* vals = nullptr;     // [cap_vals] sorted segment slots, or counting-sort entries (ws)
    int64_t cap_vals = 0;
    uint32_t* bstart = nullptr;   // [nbricks + 1]
    int64_t cap_bricks = 0;
    uint32_t total = 0;
    bool valid = false;
    bool ws = false;              // vals are tvam_bin_fill2_kernel entries (slot | class << 28)
};

// Scratch of the binned forward (owned by the plan, grown on demand).
struct TvamBinScratch {
    TvamSegBuf sb;
    int64_t cap_slots = 0;
    uint32_t* off = nullptr;      // [cap_slots + 1] exclusive scan of m
    uint32_t* keys[2] = {nullptr, nullptr};
    uint32_t* vals[2] = {nullptr, nullptr};
    int64_t cap_entries = 0, cap_entries2 = 0;
    uint32_t* bstart = nullptr;   // [nbricks + 1]
    int32_t cap_bricks = 0;
    void* temp = nullptr;
    size_t temp_bytes = 0;
    int acc_float = 0;            // 1: float LDS adds instead of int64 fixed point (TVAM_BIN_FLOAT)
    float* part = nullptr;        // [cap_entries] adjoint partial of each entry
    uint32_t* hist = nullptr;     // [nbricks * G + 1] writer counts per (brick, workgroup), then their scan
    uint32_t* hbase = nullptr;
    int64_t cap_hist = 0;
    // forward bin cache (TvamBinChunk), keyed on the call's constants, seed, spp and chunking
    std::vector<TvamBinChunk> fc;
    bool fc_key = false;
    TvamConsts fc_k{};
    uint32_t fc_seed = 0, fc_spp = 0;
    int64_t fc_chunk = 0, fc_npaths = 0;
    // last call's chunking (tvam_plan_bin_stats): chunks, chunks served from the cache,
    // chunks stored into it, brick entries sorted, paths per chunk
    int64_t st[5] = {0, 0, 0, 0, 0};
    // the bin-fill count check (sb.bad, cumulative since the scratch was allocated) is read lazily:
    // each binned call ends with an async copy into pinned host memory and an event, and the next
    // call checks the copy once its event has completed -- no stream synchronisation on the hot path
    uint32_t* bad_host = nullptr;
    hipEvent_t bad_ev = nullptr;
    bool bad_pending = false;
    int64_t temp_cap() const { return (int64_t)temp_bytes; }
};

hipError_t tvam_launch_tiles(int mode, const TvamConsts& k, const TvamTiles& t, size_t lds_bytes,
                             const float* pat, const int32_t* idxmap, const float* gin, float* out,
                             unsigned long long* counter, hipStream_t stream);

// Scattering media: every path's segments after its first medium segment
// (free flights, phase sampling, 3-D DDA; tvam_scatter.hip).
hipError_t tvam_launch_scatter_paths(int mode, const TvamConsts& k, const TvamTiles& t, const float* pat,
                                     const int32_t* idxmap, const float* gin, float* out,
                                     unsigned long long* counter, hipStream_t stream);
// Forward of the scattered segments through brick bins (chunks of paths; host
// syncs once per chunk to size the bins).  Returns hipErrorNotSupported when
// the grid is too large for the packed records (callers then use the atomics).
hipError_t tvam_scatter_binned(int mode, const TvamConsts& k, const TvamTiles& t, const float* pat,
                               const int32_t* idxmap, const float* gin, float* out, TvamBinScratch& s,
                               hipStream_t stream);
void tvam_bin_scratch_free(TvamBinScratch& s);

// Surface-aware films (film_channels 2): every path's medium segment cut at the
// target mesh, channel 0 inside / 1 outside, global atomics / gathers; vols =
// the per-(voxel, channel) volumes (tvam_scatter.hip).  The forward adds the
// unscaled film (caller zeroes `out`) and tvam_launch_scale_volumes divides it.
hipError_t tvam_launch_surface_paths(int mode, const TvamConsts& k, const TvamTiles& t, const float* pat,
                                     const int32_t* idxmap, const float* gin, const float* vols, float* out,
                                     unsigned long long* counter, hipStream_t stream);
// General per-path kernel (sample_time, 'ratio' / 'delta' sensors): the whole path
// loop per (ray, sample), global atomics / gathers (tvam_scatter.hip).
hipError_t tvam_launch_general_paths(int mode, const TvamConsts& k, const TvamTiles& t, const float* pat,
                                     const int32_t* idxmap, const float* gin, float* out,
                                     unsigned long long* counter, hipStream_t stream);
hipError_t tvam_launch_scale_volumes(int64_t n, const float* vols, float* dose, hipStream_t stream);
// compute_volume (sensor.py:47-110): volumes [res z][y][x][2]
hipError_t tvam_launch_volumes(const TvamConsts& k, uint32_t sample_count, float* volumes, hipStream_t stream);
hipError_t tvam_launch_frozen(int mode, const TvamConsts& k, const TvamTiles& t, const float* pat,
                              const int32_t* idxmap, const float* gin, float* out, unsigned long long* counter,
                              hipStream_t stream);
hipError_t tvam_launch_discretize(const TvamConsts& k, const float* h_tris, float* occ, hipStream_t stream);

// Radon filter image of the shard's DMD pixels (tvam_radon.hip).
hipError_t tvam_launch_radon(const TvamConsts& k, const TvamTiles& t, const float* tgt, int ntgt, int max_depth,
                             float wray, float* radon, hipStream_t stream);

// Per-ray pre-pass: ray generation, vial segment and DDA initialisation of
// every ray of the shard, stored as the records the tile kernels resume from.
hipError_t tvam_launch_stray_lists(const TvamConsts& k, const TvamTiles& t, hipStream_t stream);
hipError_t tvam_launch_ray_setup(const TvamConsts& k, const TvamTiles& t, float4* ray_f, int2* ray_i,
                                 float4* ray_g, const int32_t* idxmap, hipStream_t stream);

hipError_t tvam_launch_scatter(const TvamConsts& k, const float* data, const uint32_t* pixels,
                               uint64_t n, float* dense, int32_t* idxmap, hipStream_t stream);

hipError_t tvam_launch_gather(const TvamConsts& k, const float* dense, const uint32_t* pixels,
                              uint64_t n, float* out, hipStream_t stream);

#define TVAM_MAX_PROBES 8
// target: f32 (> 0 = object), or mask != nullptr: its bit mask (tvam_launch_target_mask) read from bit mbit0
hipError_t tvam_launch_loss_probes(const float* dose, const float* ddose, const float* alphas, int na,
                                   const float* target, const uint32_t* mask, uint64_t mbit0, uint64_t n, int K,
                                   float tl, float tu, float w_object, float w_void, float w_limit, float scale,
                                   double* out, hipStream_t stream);
hipError_t tvam_launch_loss_threshold(const float* dose, const float* ddose, float alpha, const float* target,
                                      const uint32_t* mask, uint64_t mbit0, uint64_t n, int K, float tl, float tu,
                                      float w_object, float w_void, float w_limit, float scale, double* out,
                                      float* grad, hipStream_t stream);
hipError_t tvam_launch_target_mask(const float* target, uint64_t n, uint32_t* mask, hipStream_t stream);

// Fused L-BFGS vector kernels (tvam_vec.hip).
hipError_t tvam_launch_lbfgs_history(uint64_t n, const float* p, const float* p_old, const float* g,
                                     const float* g_old, int h, const float* const* S, const float* const* Y,
                                     float* s_new, float* y_new, double* work, double* dots, hipStream_t stream,
                                     uint64_t nseg = 0, uint64_t seg_len = 0, uint64_t seg_stride = 0,
                                     uint64_t seg_off = 0);
hipError_t tvam_launch_lbfgs_direction(uint64_t n, const float* g, int h, const float* const* S,
                                       const float* const* Y, float cg, const float* cs, const float* cy, float* d,
                                       hipStream_t stream);
hipError_t tvam_launch_lbfgs_coef(int h, int is_new, int first, const int* order, const double* dots, double* gram,
                                  float* coef, double* gdz, hipStream_t stream);
hipError_t tvam_launch_lbfgs_direction_dev(uint64_t n, const float* g, int h, const float* const* S,
                                           const float* const* Y, const float* coef, float* d, hipStream_t stream,
                                           uint64_t nseg = 0, uint64_t seg_len = 0, uint64_t seg_stride = 0,
                                           uint64_t seg_off = 0);
hipError_t tvam_launch_axpy_clamp(uint64_t n, const float* p, float alpha, const float* d, float lo, float* out,
                                  hipStream_t stream, const float* alpha_dev = nullptr, float* s_out = nullptr);
hipError_t tvam_launch_armijo(int nprobe, double a0, const double* probes, const double* loss_dev, double loss_host,
                              double loss_div, const double* gdz, double c1, float* alpha, double* report,
                              hipStream_t stream);
