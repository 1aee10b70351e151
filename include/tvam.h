/*
 * tvam.h — C ABI of the MI355X-native TVAM projection engine (libtvam.so).
 *
 * This is the drop-in boundary for Dr.TVAM's hot path: the per-angle voxel-grid
 * ray march behind the `volume` integrator + `dda` sensor + `vfilm` film +
 * `collimated` projector plugins.  Every entry point names the reference
 * interface it replaces (paths relative to the drtvam source tree):
 *
 *   tvam_plan_create   <- scene assembly: optimize.py:15-79 (load_scene),
 *                         TVAMProjector.__init__ projector.py:41-139,
 *                         CollimatedProjector.__init__ projector.py:167-182,
 *                         CircularMotion motion.py:19-36,
 *                         VolumetricSensor.__init__ sensor.py:5-22,
 *                         VolumetricFilm.__init__ film.py:4-21,
 *                         IndexMatchedVial.to_dict geometry.py:75-96,
 *                         TVAMIntegrator.__init__ integrators/common.py:6-22
 *   tvam_forward       <- VolumeIntegrator.render integrators/volume.py:18-56
 *                         (+ sample() :136-282, DDAVolumetricSensor.accumulate
 *                         sensor.py:306-440 primal branch, VolumetricFilm.write
 *                         film.py:40-41)
 *   tvam_adjoint       <- VolumeIntegrator.render_backward integrators/volume.py:97-134
 *                         (+ accumulate backward branch sensor.py:417-423 and
 *                         dr.backward_from(Le * em_grad) volume.py:274-276)
 *   tvam_count_visits  <- (new) exact DDA visit count H used for the roofline
 *   tvam_loss_threshold<- ThresholdedLoss.__call__ loss.py:28-59, :119-132 (fused
 *                         value + dL/dx, also used for the Armijo probes of
 *                         LinearLBFGS.step lbfgs.py:256-266)
 *   tvam_loss_threshold_probes <- the same Armijo probes, up to 8 step sizes per pass
 *                         (lbfgs.py:255-268: one loss pass and one host read per batch)
 *   tvam_plan_destroy, tvam_last_error  <- Python exception plumbing
 *
 * All buffers are caller-owned device pointers (e.g. torch tensors' data_ptr()).
 * Calls are asynchronous on the given HIP stream; a plan is bound to one device
 * and is not thread-safe.  Functions return 0 on success and a negative
 * TVAM_ERR_* code on failure; tvam_last_error() then returns a thread-local
 * message (the Python shim re-raises it with the reference's wording).
 */
#ifndef TVAM_H_
#define TVAM_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TVAM_ABI_VERSION 12

/* error codes */
#define TVAM_OK               0
#define TVAM_ERR_INVALID     -1   /* bad descriptor / argument (ValueError)  */
#define TVAM_ERR_UNSUPPORTED -2   /* configuration not implemented yet        */
#define TVAM_ERR_HIP         -3   /* HIP runtime failure (RuntimeError)      */
#define TVAM_ERR_TOO_LARGE   -4   /* > 2^32 samples, common.py:60-65          */

/* projector kinds (projector.py:300-302) */
#define TVAM_PROJECTOR_COLLIMATED 0
/* vial / container kinds (geometry.py:312-318) */
#define TVAM_VIAL_INDEX_MATCHED   0
#define TVAM_VIAL_CYLINDRICAL     1
#define TVAM_VIAL_SQUARE          2  /* glass cuboids w_ext / w_int (vial_r = w_int/2, vial_r_ext = w_ext/2) */

/* medium phase functions (Mitsuba 'isotropic', 'rayleigh', 'hg'; geometry.py:29-39) */
#define TVAM_PHASE_ISOTROPIC      0
#define TVAM_PHASE_RAYLEIGH       1
#define TVAM_PHASE_HG             2
/* sensor kinds (sensor.py:442-444) */
#define TVAM_SENSOR_DDA           0  /* analytic absorption per voxel visit (sensor.py:297-440) */
#define TVAM_SENSOR_RATIO         1  /* ratio tracking at a majorant (sensor.py:193-295) */
#define TVAM_SENSOR_DELTA         2  /* collision estimator at the medium interactions (sensor.py:112-191) */

/*
 * Scene + integrator description.  Plain old data; every field mirrors a
 * reference property of the same meaning.
 */
typedef struct tvam_desc {
    int32_t abi_version;          /* must be TVAM_ABI_VERSION */

    /* projector: TVAMProjector props (projector.py:73-99) */
    int32_t projector_type;       /* TVAM_PROJECTOR_* */
    int32_t n_patterns;           /* 'n_patterns' (A) */
    int32_t res_x, res_y;         /* 'resx', 'resy' (full DMD W, H) */
    int32_t crop_x, crop_y;       /* 'cropx', 'cropy' */
    int32_t crop_offset_x, crop_offset_y; /* 'crop_offset_x/_y' */
    float   pixel_size_x, pixel_size_y;   /* 'pixel_size' (projector.py:171-175) */

    /* motion: CircularMotion (motion.py:19-24) */
    float   distance;             /* 'distance' */
    int32_t clockwise;            /* 'clockwise' */

    /* sensor + film: bbox = to_world @ [-0.5,0.5]^3 (sensor.py:14-16);
       film resolution in film order: res.x = props['resy'],
       res.y = props['resx'], res.z = props['resz'] (film.py:9-14) */
    int32_t sensor_type;          /* TVAM_SENSOR_* */
    float   bbox_min[3], bbox_max[3];
    int32_t film_res[3];
    int32_t film_channels;        /* 1, or 2 = 'surface_aware' (film.py:16-21): channel 0 collects
                                     the segments inside the target mesh, 1 those outside
                                     (sensor.py:405-409); needs target_tris */

    /* container (geometry.py:20-35, :75-96, :142-183) */
    int32_t vial_type;            /* TVAM_VIAL_* */
    float   vial_r;               /* index_matched 'r' (or cylindrical 'r_int') */
    float   vial_r_ext;           /* cylindrical 'r_ext' */
    float   vial_height;          /* 'height' (default 40) */
    float   vial_ior;             /* cylindrical 'ior' */
    float   medium_ior;           /* medium 'ior' */
    float   sigma_t;              /* medium 'extinction' */
    float   albedo;               /* medium 'albedo' */

    /* integrator props (integrators/common.py:6-22, optimize.py:96-128) */
    float   print_time;           /* 'print_time' (config 'time') */
    int32_t regular_sampling;     /* 'regular_sampling' */
    int32_t sample_time;          /* 'sample_time' */
    int32_t max_depth;            /* 'max_depth' */
    int32_t rr_depth;             /* 'rr_depth' */
    int32_t transmission_only;    /* 'transmission_only' */

    /* execution (new): angle shard [angle_begin, angle_end) of this rank and
       the LDS tile edge in voxels (0 = auto) */
    int32_t angle_begin, angle_end;
    int32_t tile;
    int32_t flags;                /* TVAM_FLAG_* */
    /* film slab [slab_begin, slab_end) of z-slices this plan renders (-1 =
       whole film): the dose / grad_dose buffers hold only these slices, and
       rays of other slices are skipped (z-slab sharding of planar scenes) */
    int32_t slab_begin, slab_end;
    /* scattering media (albedo > 0): medium 'phase' {'type', 'g'} */
    int32_t phase_type;           /* TVAM_PHASE_* */
    float   phase_g;              /* 'hg' asymmetry g */
    /* occluder meshes ('occlusions', geometry.py:55-72): black diffuse
       triangles; host array [n_occluder_tris][3 vertices][x, y, z], read by
       tvam_plan_create (not kept) */
    const float* occluder_tris;
    int32_t n_occluder_tris;
    /* target mesh (optimize.py:64-73: null BSDF, kept in the scene when the
       film is surface-aware, optimize.py:188-191): host array
       [n_target_tris][3 vertices][x, y, z] in world space, read by
       tvam_plan_create (not kept).  Used when film_channels == 2. */
    const float* target_tris;
    int32_t n_target_tris;
    /* 'ratio' sensor: its 'majorant' (sensor.py:195) */
    float   majorant;
    int32_t reserved0;
    /* Position of a sparse active_pixels[0] in the whole projector.active_pixels
       when the active set is split over plans (angle shards): the sampler stream of
       entry i is (active_base + i) * spp + sample, as TVAMIntegrator.prepare /
       sample_rays seed it (common.py:57-67, :81).  Dense calls (active_pixels ==
       NULL) use the global dense crop index, which is that position already. */
    int64_t active_base;
    /* len(projector.active_data) of the whole (unsharded) active set: the ray weight
       inv_pdf / n_samples = pixel area * active_total / (active_total * spp)
       (projector.py:164-165, :187) in the reference's fp32 rounding; 0 = the call's
       n_active. */
    int64_t active_total;
} tvam_desc;

/* tvam_desc.flags */
#define TVAM_FLAG_NO_ZERO_SKIP 1  /* forward: march rays whose pattern value is 0 too */
#define TVAM_FLAG_FWD_STATS    2  /* forward: count tiles that fell back to float LDS atomics */
#define TVAM_FLAG_NO_PLANAR    4  /* use the per-ray tile kernels even where the planar path applies */
#define TVAM_FLAG_RAY_FWD      8  /* planar path: ray-driven forward instead of the voxel-driven one */
#define TVAM_FLAG_SCATTER_ATOMIC 16 /* scattering media: per-path global atomics / gathers instead of brick bins */

typedef struct tvam_plan tvam_plan;

/* Fill *desc with the reference defaults (scene-independent fields). */
void tvam_desc_init(tvam_desc* desc);

/* Validate desc, build per-angle / per-slice / per-tile tables on `device`. */
int  tvam_plan_create(const tvam_desc* desc, int device, tvam_plan** plan);
void tvam_plan_destroy(tvam_plan* plan);

/*
 * Forward projection (primal render).  Writes the whole film
 * dose[z][y][x][C] (film order) = inv_vol * sum over rays of this plan's
 * angle shard; every voxel is overwritten (no pre-zeroing needed).
 *   active_data   : f32, n_active entries (projector.active_data)
 *   active_pixels : u32 flat indices angle*H*W + row*W + col into the full DMD
 *                   (projector.active_pixels); NULL means the dense crop order
 *                   produced by TVAMProjector.__init__ (projector.py:90-98),
 *                   in which case n_active must equal A*crop_y*crop_x.
 *                   Jittered sampling: the plan keeps the per-ray records of a sparse set
 *                   keyed on (active_pixels pointer, n_active, seed, spp) and reuses them
 *                   (slice ranges, the line-search forward of one seed); after changing the
 *                   array's contents in place, or before passing a different array (a new
 *                   allocation can land on a freed one's address), call
 *                   tvam_plan_set_active, which drops them.
 * spp / seed follow TVAMIntegrator.prepare (common.py:41-68).
 */
int tvam_forward(tvam_plan* plan, const float* active_data,
                 const uint32_t* active_pixels, uint64_t n_active,
                 uint32_t spp, uint32_t seed, float* dose, void* hip_stream);

/*
 * Forward projection of film slices [z_begin, z_end) only (relative to the plan's slab): the
 * same values tvam_forward writes there, the other slices of dose untouched.  Lets a caller
 * all-reduce a finished slice range of an angle shard's partial dose while the next range is
 * computed.  The range must lie on the forward's slice chunks
 * (tvam_plan_fwd_chunk); TVAM_ERR_UNSUPPORTED when the plan's forward cannot be split (0).
 */
int tvam_forward_slices(tvam_plan* plan, const float* active_data,
                        const uint32_t* active_pixels, uint64_t n_active,
                        uint32_t spp, uint32_t seed, int32_t z_begin, int32_t z_end,
                        float* dose, void* hip_stream);
/* Slice granularity of tvam_forward_slices (0: the plan's forward covers every slice at once:
   scattering media, per-path kernels, the ray-driven planar forward). */
int tvam_plan_fwd_chunk(const tvam_plan* plan);

/*
 * Adjoint projection (render_backward).  grad_active[i] (overwritten, f32,
 * n_active entries) = d<grad_dose, forward(active_data)>/d active_data[i],
 * i.e. the gradient Dr.TVAM accumulates into projector.active_data.grad.
 */
int tvam_adjoint(tvam_plan* plan, const float* grad_dose,
                 const uint32_t* active_pixels, uint64_t n_active,
                 uint32_t spp, uint32_t seed, float* grad_active,
                 void* hip_stream);

/* Update desc.active_base / desc.active_total of a plan (after the active set was
   compacted, e.g. by 'filter_radon', optimize.py:143-163); later calls seed and
   weight their rays with them. */
int tvam_plan_set_active(tvam_plan* plan, int64_t active_base, int64_t active_total);

/* Diagnostics (host-synchronous): number of (slice, tile) workgroups of the
   last forward that accumulated with float atomics instead of fixed point
   (needs TVAM_FLAG_FWD_STATS). */
int tvam_plan_stats(tvam_plan* plan, uint64_t* fallback_tiles);

/* Radon filter (integrators/radon.py:47-106, optimize.py:143-163, 'filter_radon'):
   for every DMD pixel of the plan's shard (dense crop order [angle][row][col],
   n = shard angles * crop_y * crop_x), the sum over `spp` samples of the ray
   weight times the absorption on the ray's segments inside both the medium
   and the target mesh (null BSDF); the optimiser keeps the pixels with a
   positive value.  target_tris: host array [n_target_tris][3][3] of
   world-space triangles.  radon: device, n floats, overwritten.  Synchronous. */
int tvam_radon(tvam_plan* plan, const float* target_tris, int32_t n_target_tris, uint32_t spp, uint32_t seed,
               int32_t max_depth, float* radon, void* stream);

/* Surface-aware discretisation (film_channels == 2; VolumetricSensor.compute_volume,
   sensor.py:47-110): volumes[z][y][x][2] (device, f32, overwritten) = the voxel volume
   inside (channel 0) / outside (1) the target mesh, estimated from sample_count points per
   voxel (independent sampler seeded (0, voxel)), each classified by the orientation of the
   first target hit along a uniform random direction.  Synchronous. */
int tvam_compute_volume(tvam_plan* plan, uint32_t sample_count, float* volumes, void* hip_stream);

/* Target discretisation (utils.py:83-128 discretize; the target transform of
   optimize.py:30-50 is applied by the caller): occ[z][y][x] (device, f32, overwritten)
   = 1 where the voxel centre bbox_min + (0.5 + i) h lies strictly inside the target
   mesh's bbox and the first hit of a ray from it along square_to_uniform_sphere(next_2d)
   (independent sampler seeded (0, voxels), lane = flat voxel index) faces away from the
   ray (dot(n, d) > 0), else 0.  Uses desc->film_res, bbox_min/max and target_tris
   (host, world space).  Runs on the current HIP device; synchronous. */
int tvam_discretize(const tvam_desc* desc, float* occ, void* hip_stream);

/* Diagnostics (host-synchronous): the fixed-point scale of the last forward of a plan
   served by the ray-driven planar forward (tvam_plan_path == 1): scale[0] = 2^e with
   |every voxel's scaled sum| < 2^30 guaranteed, scale[1] = 1 (exact int32 fixed point)
   or 0 (the bound was not finite: float LDS adds). */
int tvam_plan_fwd_scale(tvam_plan* plan, float* scale);

/* Diagnostics (host-synchronous): the chunking of the last brick-binned call of a plan with
   a scattering medium (the later segments of every path, tvam_scatter.hip).  stats[0] =
   chunks of paths, [1] = chunks served from the forward bin cache (weights rescaled to the
   new pattern, no replay / sort), [2] = chunks stored into the cache, [3] = brick entries
   marched, [4] = paths per chunk (all 0 when the plan's last call binned nothing), [5] = device
   bytes the forward bin cache holds, [6] = device bytes of the chunk scratch, [7] = slots whose
   bin-fill walk disagreed with the record writer's closed-form brick count, summed over the calls
   since the chunk scratch was allocated (0 by construction; host-synchronous read; a binned call
   that finds an earlier call's count nonzero fails with TVAM_ERR_HIP).  stats has 8 entries.
   (ABI v10) */
int tvam_plan_bin_stats(tvam_plan* plan, int64_t* stats);

/* Diagnostics (host-synchronous): the per-ray tile kernels' row walks for the plan's most
   recent ray records (jittered sampling).  stats[0] = rays the ray setup listed as strays
   (outside their row's main slice; -1 when the plan keeps no stray lists: regular sampling,
   rows whose interior jitters already change slice, or > 2^32 records), [1] = the stray-list
   capacity (beyond it every workgroup walks its slice's full row list), [2] = the (tile, slice)
   workgroups' stray walk summed over the launch (each walks its slice's whole stray list:
   strays x tiles), [3] = their main-row slot walk (rows x slots x spp over all workgroups),
   [4] = frozen-axis rays, [5] = spp of the records, [6] = tiles, [7] = (angle, column) slots
   over all tiles.  stats has 8 entries.  (ABI v11) */
int tvam_plan_tile_stats(tvam_plan* plan, int64_t* stats);

/* Measurement (host-synchronous): launch time of the plan's dominant forward kernel -- the
   forward brick march of a scattering medium, else the voxel-driven planar forward where it
   serves, else the per-ray tile forward -- from HIP events recorded on its stream around each
   launch.  Returns the launches recorded since the previous call and their summed time in ms (at
   most 1024 per measurement), then stops recording, or (enable != 0) starts a new measurement of
   the kernel kind of `plan`.  One timer per process, owned by the plan that enabled it (another
   plan's call fails while it runs; launches on other devices are not recorded); reading it
   (enable == 0) releases it, and so does destroying the owning plan.  (ABI v11) */
int tvam_plan_kernel_time(tvam_plan* plan, int32_t enable, double* total_ms, int64_t* launches);

/* Surface-aware plans: the per-channel voxel volumes the forward divides by and the
   adjoint multiplies the incoming gradient with (inv_vol = 1/volume, 0 where volume
   is 0: volume.py:41-42, :130).  Device pointer [z][y][x][2], caller-owned, kept by
   the plan until replaced; must be set before tvam_forward / tvam_adjoint. */
int tvam_plan_set_volumes(tvam_plan* plan, const float* volumes);

/* Which kernels serve this plan (bit mask; 0 = per-ray tile kernels):
   bit 0 = planar adjoint (regular sampling: one ray record per (angle,
   column), Z-slice-sharing adjoint); bit 1 = voxel-driven planar forward
   (straight rays only: not behind a refracting vial). */
int tvam_plan_path(const tvam_plan* plan);

/*
 * Fused vector kernels of the linear L-BFGS step (lbfgs.py:146-275,
 * optimize.py:316-318).  All vectors are f32, n entries, 16-byte aligned.
 *
 * tvam_lbfgs_history: with p_old != NULL forms s_new = p - p_old and
 *   y_new = g - g_old (written to s_new / y_new) and, over the h retained
 *   pairs S[j], Y[j] (oldest first, 0 <= h <= 7) followed by the new pair,
 *   writes to dots (f64): s_j.g | y_j.g | s_new.y_j | s_j.y_new | y_new.y_j
 *   (h + 1 entries each) | g.g.  With p_old == NULL only s_j.g | y_j.g | g.g
 *   (h entries each).  With p_old == NULL and g_old != NULL (ABI v12): the new
 *   pair's s_new already holds p - p_old (tvam_axpy_clamp_dev's s_out) and is
 *   read, y_new formed; the same dots as the p_old path.  work: >=
 *   TVAM_LBFGS_WORK_DOUBLES f64 of scratch.
 * tvam_lbfgs_direction: d = cg g + sum_j (cs[j] S[j] + cy[j] Y[j]), h <= 8.
 * tvam_axpy_clamp: out = max(p + alpha d, lo) (out may alias p).
 * tvam_lbfgs_coef: the two-loop recursion (lbfgs.py:221-243) on the device, in
 *   Gram form, one lane: order[h] = the ring slots (0..7) of the pairs, oldest
 *   first, the new pair last when is_new; dots = tvam_lbfgs_history's output
 *   for those pairs (device, after any all-reduce); gram (device, 128 f64) keeps
 *   s_a.y_b / y_a.y_b by slot across steps (the new pair's entries are stored
 *   into it).  Writes coef (device, 17 f32: cg | cs[8] | cy[8]) and gdz (device
 *   f64: g.d).  first: the first step (gamma = 1).  No host synchronisation.
 * tvam_lbfgs_direction_dev: tvam_lbfgs_direction with coef read from device
 *   memory (tvam_lbfgs_coef's output).
 * tvam_lbfgs_history_rows: tvam_lbfgs_history over the entries seg_off +
 *   a * seg_stride + [0, seg_len) of every a < nseg only (a band of DMD rows):
 *   s_new / y_new of those entries and the band's dots (summed over the bands by
 *   the caller, in band order, before tvam_lbfgs_coef).
 * tvam_lbfgs_direction_rows: the same for the entries seg_off + a * seg_stride +
 *   [0, seg_len) of every a < nseg only (a band of DMD rows of every angle:
 *   seg_stride = rows * columns), so that the forward of one band's slices can
 *   start while the next band's direction is formed (all multiples of 4).
 * tvam_lbfgs_armijo: the first batch of backtracking Armijo probes (lbfgs.py:256-266)
 *   decided on the device, one lane: alpha[0] (device f32) = a_j = alpha0 / 2^j
 *   for the first j < nprobe with probes[j] <= loss + c1 a_j gdz[0] (device f64
 *   probes and g.d; loss = loss_dev[0] / loss_div, or loss_host when loss_dev is
 *   NULL), evaluated as the host loop evaluates it in f64; 0 when none passes.
 *   report (may be NULL; device-visible, e.g. pinned host memory the host polls):
 *   loss_dev[0] (or loss_host) | gdz[0] | probes[0..nprobe) | alpha | 1.0, f64, the
 *   final 1.0 written after the others are visible system-wide.
 * tvam_axpy_clamp_dev: tvam_axpy_clamp with alpha read from device memory
 *   (tvam_lbfgs_armijo's output), so the update follows the probes on the stream
 *   without a host round trip; s_out (may be NULL, no alias of p / d / out) =
 *   out - p, the next step's s_new.  (Both ABI v12.)
 */
#define TVAM_LBFGS_WORK_DOUBLES (2048 * 64)
int tvam_lbfgs_history(uint64_t n, const float* p, const float* p_old, const float* g, const float* g_old,
                       int32_t h, const float* const* S, const float* const* Y, float* s_new, float* y_new,
                       double* work, double* dots, void* hip_stream);
int tvam_lbfgs_history_rows(uint64_t nseg, uint64_t seg_len, uint64_t seg_stride, uint64_t seg_off, const float* p,
                            const float* p_old, const float* g, const float* g_old, int32_t h, const float* const* S,
                            const float* const* Y, float* s_new, float* y_new, double* work, double* dots,
                            void* hip_stream);
int tvam_lbfgs_direction(uint64_t n, const float* g, int32_t h, const float* const* S, const float* const* Y,
                         float cg, const float* cs, const float* cy, float* d, void* hip_stream);
int tvam_lbfgs_coef(int32_t h, int32_t is_new, int32_t first, const int32_t* order, const double* dots,
                    double* gram, float* coef, double* gdz, void* hip_stream);
int tvam_lbfgs_direction_dev(uint64_t n, const float* g, int32_t h, const float* const* S, const float* const* Y,
                             const float* coef, float* d, void* hip_stream);
int tvam_lbfgs_direction_rows(uint64_t nseg, uint64_t seg_len, uint64_t seg_stride, uint64_t seg_off,
                              const float* g, int32_t h, const float* const* S, const float* const* Y,
                              const float* coef, float* d, void* hip_stream);
int tvam_axpy_clamp(uint64_t n, const float* p, float alpha, const float* d, float lo, float* out,
                    void* hip_stream);
int tvam_axpy_clamp_dev(uint64_t n, const float* p, const float* alpha, const float* d, float lo, float* out,
                        float* s_out, void* hip_stream);
int tvam_lbfgs_armijo(int32_t nprobe, double alpha0, const double* probes, const double* loss_dev, double loss_host,
                      double loss_div, const double* gdz, double c1, float* alpha, double* report,
                      void* hip_stream);

/* Global film z-slice of every crop row's rays under regular sampling
   (slice_of_row[crop_y]; -1 when the row's rays miss the grid or the vial),
   computed with the plan's own fp32 ray generation: the row <-> slice map
   that z-slab sharding of planar scenes partitions. */
int tvam_row_slices(const tvam_desc* desc, int32_t* slice_of_row);

/* The planar adjoint of film slices [z_begin, z_end) alone (tvam_adjoint of a dense set restricted
   to them), into DMD rows [row_begin, row_end) of every angle of grad_active (n_active = the dense
   crop count; those rows zeroed first, the others untouched).  The rows must be exactly the rows
   whose rays lie in those slices (tvam_row_slices); slices on tvam_plan_adj_chunk's chunks.  With
   tvam_forward_slices it lets a caller pipeline a slab's forward, loss and adjoint with the vector
   passes of the neighbouring slabs.  TVAM_ERR_UNSUPPORTED off the planar path. */
int tvam_adjoint_slices(tvam_plan* plan, const float* grad_dose, uint64_t n_active, int32_t z_begin, int32_t z_end,
                        int32_t row_begin, int32_t row_end, float* grad_active, void* hip_stream);
/* Slice granularity of tvam_adjoint_slices (0: not available). */
int tvam_plan_adj_chunk(const tvam_plan* plan);

/* Exact number of DDA voxel visits of one pass (host-synchronous). */
int tvam_count_visits(tvam_plan* plan, uint32_t spp, uint32_t seed,
                      uint64_t* visits);

/*
 * ThresholdedLoss (loss.py:82-132) over a binary target, fused.
 *   x = dose + alpha * ddose (ddose may be NULL), target: f32 (>0 = object).
 *   out[0] += sum of the per-voxel loss (f64 accumulation, caller zeroes out);
 *   grad (may be NULL) = dL/dx per voxel (sum reduction; scale = 1/n for mean
 *   is applied by the caller through `scale`).
 */
int tvam_loss_threshold(const float* dose, const float* ddose, float alpha,
                        const float* target, uint64_t n, int32_t K,
                        float tl, float tu, float w_object, float w_void,
                        float w_limit, float scale, double* out, float* grad,
                        void* hip_stream);

/*
 * Armijo probes of LinearLBFGS's line search (lbfgs.py:255-268), fused: the
 * ThresholdedLoss of dose + alphas[j] * ddose for j < n_alpha (<= 8, alphas on
 * the host) in one pass; out[j] += the sum for alphas[j] (f64, caller zeroes
 * out[0..n_alpha)), scaled like tvam_loss_threshold.  Per element the same
 * arithmetic as tvam_loss_threshold with that alpha.
 */
int tvam_loss_threshold_probes(const float* dose, const float* ddose,
                               const float* alphas, int32_t n_alpha,
                               const float* target, uint64_t n, int32_t K,
                               float tl, float tu, float w_object, float w_void,
                               float w_limit, float scale, double* out,
                               void* hip_stream);

/*
 * The object test of both loss kernels (target > 0, loss.py:119) from a bit mask
 * of the target, 1/32 of its bytes (ABI v12):
 *   tvam_target_mask: mask[(n + 31) / 32] (device u32), bit j of word w =
 *   target[32 w + j] > 0 (0 past n).
 *   tvam_loss_threshold_mask / tvam_loss_threshold_probes_mask: tvam_loss_threshold /
 *   tvam_loss_threshold_probes with voxel i's object bit read at bit mask_bit0 + i
 *   of mask (a slab of the film: mask_bit0 = its first voxel's index).
 */
int tvam_target_mask(const float* target, uint64_t n, uint32_t* mask, void* hip_stream);
int tvam_loss_threshold_mask(const float* dose, const float* ddose, float alpha,
                             const uint32_t* mask, uint64_t mask_bit0, uint64_t n, int32_t K,
                             float tl, float tu, float w_object, float w_void,
                             float w_limit, float scale, double* out, float* grad,
                             void* hip_stream);
int tvam_loss_threshold_probes_mask(const float* dose, const float* ddose,
                                    const float* alphas, int32_t n_alpha,
                                    const uint32_t* mask, uint64_t mask_bit0, uint64_t n,
                                    int32_t K, float tl, float tu, float w_object,
                                    float w_void, float w_limit, float scale,
                                    double* out, void* hip_stream);

/* Thread-local message describing the last error ("" if none). */
const char* tvam_last_error(void);

/* ABI version of the loaded library. */
int tvam_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* TVAM_H_ */
