// tvam_plan.hip — plan construction and the extern "C" boundary (include/tvam.h).
//
// The plan turns a tvam_desc (the reference's scene / plugin properties) into
// the small constant tables the tile kernels consume:
//   * per-angle (cos, sin) of the shard, computed like CircularMotion.eval
//     (motion.py:26-36: alpha = 2*pi*time, time = angle / n_patterns);
//   * per-z-slice list of DMD rows whose (planar) rays lie in that slice;
//   * per-(xy-tile, angle) range of DMD columns whose rays can cross the tile.
// Caller buffers are never allocated or copied here on the hot path; only the
// sparse active-set path uses a lazily allocated dense scratch.
#include "tvam_internal.h"

#include <algorithm>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(TVAM_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

struct tvam_plan {
    tvam_desc desc;
    int device;
    TvamConsts k;
    TvamTiles tiles;
    int32_t ntiles;
    size_t lds_bytes;
    int32_t max_rows_per_slice;
    int64_t n_slots_all = 0;  // (angle, column) slots over every tile (tvam_plan_tile_stats)
    int64_t n_main_rows = 0;  // main-row list entries over every slice (0: no main-row lists)
    int64_t n_rows_all = 0;   // row list entries over every slice
    bool empty;  // max_depth too small for any ray to reach the medium
    bool cyl;    // refracting (cylindrical / square) vial: per-ray directions and weights
    bool surface = false;    // surface-aware film (2 channels): per-path kernels cut at the target mesh
    bool general = false;    // sample_time or a ratio / delta sensor: the general per-path kernel
    float* d_tgt = nullptr;  // target mesh triangles (surface-aware films)
    const float* vols = nullptr;  // caller's compute_volume() output (tvam_plan_set_volumes)
    float* d_occ = nullptr;  // occluder triangles
    // device tables
    float2* d_cs = nullptr;
    int32_t* d_slice_off = nullptr;
    int32_t* d_slice_rows = nullptr;
    int32_t* d_slice_moff = nullptr;   // main-row lists (TvamTiles::slice_moff)
    int32_t* d_slice_mrows = nullptr;
    int32_t* d_row_main = nullptr;
    uint32_t* d_slots = nullptr;
    int64_t* d_slot_off = nullptr;
    unsigned long long* d_counter = nullptr;
    float4* d_ang = nullptr;
    // per-ray records (tvam_ray_setup_kernel), cached: regular sampling makes
    // them call-independent; otherwise they are keyed on (spp, seed).  Two slots (LRU) when memory
    // allows: an optimiser iteration renders seed i, back-projects seed i', renders seed i again
    struct RaySlot {
        float4* f = nullptr;
        int2* i = nullptr;
        float4* g = nullptr;
        int64_t* frozen = nullptr;  // frozen-axis rays of the ray records (tvam_frozen_kernel)
        unsigned long long* frozen_n = nullptr;
        uint32_t* stray = nullptr;  // stray rays (TvamTiles::stray_*): [cap] appended, [cap] by slice,
        uint32_t* stray_cs = nullptr;  // [2 (nz + 1)] counts / cursors, offsets
        unsigned long long* stray_n = nullptr;
        uint64_t cap = 0;
        bool valid = false;
        uint32_t spp = 0, seed = 0;
        bool sparse = false;  // records built for a sparse active set (streams by active position)
        const void* pix = nullptr;  // ... that set (active_pixels pointer and count: the records'
        uint64_t npix = 0;          // key; tvam_plan_set_active drops them after in-place changes)
        hipEvent_t ready = nullptr;
        uint64_t used = 0;
    };
    RaySlot rs[2];
    uint64_t ray_tick = 0;
    // planar fast path (regular sampling; tvam_planar.hip)
    bool planar = false;      // planar adjoint
    bool planar_fwd = false;  // voxel-driven planar forward (straight rays only)
    int32_t planar_fz = 16, planar_az = 4;
    TvamPlanar pl{};
    int32_t* d_pl_slice_off = nullptr;
    int32_t* d_pl_slice_rows = nullptr;
    float4* d_pl_vox = nullptr;
    float4* d_pl_fwd_ang = nullptr;
    int32_t* d_pl_fwd_cb = nullptr;
    float4* d_pl_rec_f = nullptr;
    int32_t* d_pl_rec_i = nullptr;
    float4* d_pl_rec_g = nullptr;
    float* d_pl_part = nullptr;  // voxel-driven forward: partial doses of the angle parts
    float* d_pl_bin = nullptr;   // voxel-driven forward: slice-binned patterns
    float4* d_pl_vox2 = nullptr;      // refracted voxel-driven forward: per-column 1/d, flags, weight
    float4* d_pl_fwd_model = nullptr; // refracted voxel-driven forward: per-(tile, angle) chord-index models
    unsigned* d_amax = nullptr;  // ray-driven forward: per-angle max |pattern|, fixed-point scale
    float* d_fscale = nullptr;
    int32_t planar_rz = 4;
    TvamAdjListBufs adjl;  // planar adjoint: slice-invariant visit lists (tvam_adjlist.hip)
    bool adjl_pending = false;  // the lists are to be built by the first adjoint call
    int adjl_parts = 1;
    TvamBinScratch bins;  // scattering media: brick-binned forward scratch
    std::vector<float4> fwd_ang_h;  // host staging of the forward tables (plan creation only)
    std::vector<int32_t> fwd_cb_h;
    // sparse scratch (dense crop layout), allocated on first sparse call
    float* d_dense = nullptr;
    int32_t* d_idxmap = nullptr;
    uint64_t dense_n = 0;
};

extern "C" void tvam_desc_init(tvam_desc* d) {
    std::memset(d, 0, sizeof(*d));
    d->abi_version = TVAM_ABI_VERSION;
    d->projector_type = TVAM_PROJECTOR_COLLIMATED;
    d->n_patterns = 1000;            // projector.py:73
    d->res_x = d->res_y = 256;       // projector.py:74-75
    d->crop_x = d->crop_y = 256;
    d->pixel_size_x = d->pixel_size_y = 1.0f;
    d->distance = 20.0f;
    d->sensor_type = TVAM_SENSOR_DDA;
    for (int a = 0; a < 3; ++a) {
        d->bbox_min[a] = -0.5f;
        d->bbox_max[a] = 0.5f;
        d->film_res[a] = 256;        // film.py:9-11
    }
    d->film_channels = 1;
    d->vial_type = TVAM_VIAL_INDEX_MATCHED;
    d->vial_height = 40.0f;          // geometry.py:80
    d->medium_ior = 1.0f;
    d->vial_ior = 1.5f;
    d->print_time = 1.0f;            // common.py:13
    d->regular_sampling = 0;         // common.py:22
    d->sample_time = 0;              // common.py:10
    d->max_depth = 6;                // optimize.py:99
    d->rr_depth = 6;                 // optimize.py:100
    d->transmission_only = 1;        // common.py:19
    d->angle_begin = 0;
    d->angle_end = -1;               // -1: all angles
    d->tile = 0;
    d->slab_begin = 0;
    d->slab_end = -1;                // -1: all slices
}

extern "C" const char* tvam_last_error(void) { return g_err.c_str(); }
extern "C" int tvam_abi_version(void) { return TVAM_ABI_VERSION; }

static void adjl_free(TvamAdjListBufs& b) {
    (void)hipFree(b.gchunk);
    (void)hipFree(b.glist);
    (void)hipFree(b.coff);
    (void)hipFree(b.hdr);
    (void)hipFree(b.w);
    b = TvamAdjListBufs{};
}

static void plan_free(tvam_plan* p) {
    if (!p) return;
    (void)hipFree(p->d_cs);
    (void)hipFree(p->d_slice_off);
    (void)hipFree(p->d_slice_rows);
    (void)hipFree(p->d_slice_moff);
    (void)hipFree(p->d_slice_mrows);
    (void)hipFree(p->d_row_main);
    (void)hipFree(p->d_slots);
    (void)hipFree(p->d_slot_off);
    (void)hipFree(p->d_counter);
    (void)hipFree(p->d_ang);
    for (auto& r : p->rs) {
        (void)hipFree(r.f);
        (void)hipFree(r.i);
        (void)hipFree(r.g);
        (void)hipFree(r.frozen);
        (void)hipFree(r.frozen_n);
        (void)hipFree(r.stray);
        (void)hipFree(r.stray_cs);
        (void)hipFree(r.stray_n);
        if (r.ready) (void)hipEventDestroy(r.ready);
    }
    (void)hipFree(p->d_dense);
    (void)hipFree(p->d_idxmap);
    (void)hipFree(p->d_pl_slice_off);
    (void)hipFree(p->d_pl_slice_rows);
    (void)hipFree(p->d_pl_vox);
    (void)hipFree(p->d_pl_fwd_ang);
    (void)hipFree(p->d_pl_fwd_cb);
    (void)hipFree(p->d_pl_rec_f);
    (void)hipFree(p->d_pl_rec_i);
    (void)hipFree(p->d_pl_rec_g);
    (void)hipFree(p->d_pl_part);
    (void)hipFree(p->d_pl_bin);
    adjl_free(p->adjl);
    (void)hipFree(p->d_pl_vox2);
    (void)hipFree(p->d_pl_fwd_model);
    (void)hipFree(p->d_amax);
    (void)hipFree(p->d_occ);
    (void)hipFree(p->d_tgt);
    tvam_bin_scratch_free(p->bins);
    (void)hipFree(p->d_fscale);
    delete p;
}

static void kt_plan_gone(const tvam_plan* p);  // the kernel timer's events go with their owning plan

extern "C" void tvam_plan_destroy(tvam_plan* p) {
    if (!p) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(p->device);
    kt_plan_gone(p);
    plan_free(p);
    (void)hipSetDevice(cur);
}

static int validate(const tvam_desc& d) {
    if (d.abi_version != TVAM_ABI_VERSION) return fail(TVAM_ERR_INVALID, "tvam_desc.abi_version mismatch");
    if (d.projector_type != TVAM_PROJECTOR_COLLIMATED)
        return fail(TVAM_ERR_UNSUPPORTED, "only the 'collimated' projector is implemented on the GPU path");
    if (d.sensor_type != TVAM_SENSOR_DDA && d.sensor_type != TVAM_SENSOR_RATIO && d.sensor_type != TVAM_SENSOR_DELTA)
        return fail(TVAM_ERR_INVALID, "unknown sensor type");
    if (d.sensor_type == TVAM_SENSOR_DELTA && d.albedo == 0.0f)  // volume.py:160-161
        return fail(TVAM_ERR_INVALID, "Tried to render a purely absorptive volume with a delta tracking sensor. This is not supported.");
    if (d.sensor_type == TVAM_SENSOR_RATIO && !(d.majorant > 0.0f))
        return fail(TVAM_ERR_INVALID, "the 'ratio' sensor needs a positive majorant");
    if (d.sample_time && d.film_channels != 1)
        return fail(TVAM_ERR_UNSUPPORTED, "sample_time needs a one-channel film");
    if ((d.sensor_type != TVAM_SENSOR_DDA || d.sample_time) &&
        (d.slab_begin != 0 || (d.slab_end >= 0 && d.slab_end != d.film_res[2])))
        return fail(TVAM_ERR_UNSUPPORTED, "sample_time and the ratio / delta sensors need a film without slabs");
    if (d.vial_type != TVAM_VIAL_INDEX_MATCHED && d.vial_type != TVAM_VIAL_CYLINDRICAL &&
        d.vial_type != TVAM_VIAL_SQUARE)
        return fail(TVAM_ERR_UNSUPPORTED, "only the 'index_matched', 'cylindrical' and 'square' containers are implemented on the GPU path");
    if (d.n_occluder_tris < 0 || (d.n_occluder_tris > 0 && !d.occluder_tris))
        return fail(TVAM_ERR_INVALID, "occluder_tris is null");
    if (d.film_channels != 1 && d.film_channels != 2) return fail(TVAM_ERR_INVALID, "film_channels must be 1 or 2");
    if (d.film_channels == 2) {
        if (d.n_target_tris <= 0 || !d.target_tris)
            return fail(TVAM_ERR_INVALID, "No target shape found in the scene");  // sensor.py:60-61
        if (d.slab_begin != 0 || (d.slab_end >= 0 && d.slab_end != d.film_res[2]))
            return fail(TVAM_ERR_UNSUPPORTED, "surface-aware films cannot be split into slabs");
    }
    if (!(d.albedo >= 0.0f && d.albedo <= 1.0f)) return fail(TVAM_ERR_INVALID, "medium albedo must lie in [0, 1]");
    if (d.albedo != 0.0f) {
        if (!(d.sigma_t > 0.0f)) return fail(TVAM_ERR_INVALID, "scattering medium: extinction must be positive");
        if (d.phase_type < TVAM_PHASE_ISOTROPIC || d.phase_type > TVAM_PHASE_HG)
            return fail(TVAM_ERR_UNSUPPORTED, "unknown phase function");
        if (d.slab_begin != 0 || (d.slab_end >= 0 && d.slab_end != d.film_res[2]))
            return fail(TVAM_ERR_UNSUPPORTED, "scattered paths leave their slice: film slabs need a non-scattering medium");
    }
    // the medium segment is path vertex 1 (index matched) or 2 (behind two glass
    // surfaces); Russian roulette starts at depth > rr_depth (volume.py:182-185)
    if (d.rr_depth < (d.vial_type == TVAM_VIAL_INDEX_MATCHED ? 1 : 2))
        return fail(TVAM_ERR_UNSUPPORTED, "Russian roulette before the medium segment (rr_depth too small) is not implemented");
    if (d.n_patterns <= 0 || d.res_x <= 0 || d.res_y <= 0) return fail(TVAM_ERR_INVALID, "projector resolution and n_patterns must be positive");
    if (d.crop_x <= 0 || d.crop_y <= 0 || d.crop_x > d.res_x || d.crop_y > d.res_y)
        return fail(TVAM_ERR_INVALID, "Crop resolution must be smaller than the base resolution.");  // projector.py:81-82
    if (d.crop_offset_x < 0 || d.crop_offset_y < 0 || d.crop_offset_x + d.crop_x > d.res_x ||
        d.crop_offset_y + d.crop_y > d.res_y)
        return fail(TVAM_ERR_INVALID, "With the specified crop offset, the cropped region extends beyond the base resolution.");  // projector.py:87-88
    for (int a = 0; a < 3; ++a) {
        if (d.film_res[a] <= 0) return fail(TVAM_ERR_INVALID, "film resolution must be positive");
        if (!(d.bbox_max[a] > d.bbox_min[a])) return fail(TVAM_ERR_INVALID, "sensor bounding box is empty");
    }
    if (!(d.vial_r > 0.0f)) return fail(TVAM_ERR_INVALID, "vial radius must be positive");
    if (d.vial_type != TVAM_VIAL_INDEX_MATCHED &&
        !(d.vial_r_ext > d.vial_r && d.vial_ior > 0.0f && d.medium_ior > 0.0f && d.vial_height > 0.0f))
        return fail(TVAM_ERR_INVALID, "glass vial: need r_ext > r_int > 0 (w_ext > w_int) and positive IORs");
    {
        const int z1 = d.slab_end < 0 ? d.film_res[2] : d.slab_end;
        if (d.slab_begin < 0 || z1 > d.film_res[2] || d.slab_begin >= z1)
            return fail(TVAM_ERR_INVALID, "invalid film slab [slab_begin, slab_end)");
    }
    if (!(d.pixel_size_x > 0.0f && d.pixel_size_y > 0.0f)) return fail(TVAM_ERR_INVALID, "pixel_size must be positive");
    if (d.active_base < 0 || d.active_total < 0) return fail(TVAM_ERR_INVALID, "active_base / active_total must be >= 0");
    return 0;
}

static TvamConsts make_consts(const tvam_desc& d, int a0, int a1) {
    TvamConsts k;
    std::memset(&k, 0, sizeof(k));
    for (int a = 0; a < 3; ++a) {
        k.bmin[a] = d.bbox_min[a];
        k.bmax[a] = d.bbox_max[a];
        k.res[a] = d.film_res[a];
        k.h[a] = (d.bbox_max[a] - d.bbox_min[a]) / (float)d.film_res[a];  // sensor.py:19
    }
    k.z0 = d.slab_begin;
    k.nz = (d.slab_end < 0 ? d.film_res[2] : d.slab_end) - d.slab_begin;
    float vol = k.h[0] * k.h[1] * k.h[2];
    k.inv_vol = vol != 0.0f ? 1.0f / vol : 0.0f;  // volume.py:41-42
    k.res_x = d.res_x;
    k.res_y = d.res_y;
    k.crop_x = d.crop_x;
    k.crop_y = d.crop_y;
    k.crop_off_x = d.crop_offset_x;
    k.crop_off_y = d.crop_offset_y;
    k.n_patterns = d.n_patterns;
    k.a0 = a0;
    k.a1 = a1;
    k.shard_base = (int64_t)a0 * d.crop_y * d.crop_x;
    k.stream_base = d.active_base;
    k.ex = (float)d.res_x * d.pixel_size_x;
    k.ey = (float)d.res_y * d.pixel_size_y;
    k.inv_w = 1.0f / (float)d.res_x;
    k.inv_h = 1.0f / (float)d.res_y;
    k.dist_m_zc = d.distance - 0.005f;
    k.clockwise = d.clockwise;
    k.regular = d.regular_sampling;
    k.sample_time = d.sample_time;
    k.skip_zero = (d.flags & TVAM_FLAG_NO_ZERO_SKIP) ? 0 : 1;
    k.vial_type = d.vial_type;
    k.max_depth = d.max_depth;
    k.vial_r = d.vial_r;
    k.vial_half_h = 0.5f * d.vial_height;
    k.vial_r_ext = d.vial_r_ext;
    k.vial_hz_int = (float)(0.5 * 0.9 * (double)d.vial_height);  // geometry.py:207 (inner cuboid)
    k.eta_ext = d.vial_ior / TVAM_IOR_AIR;   // int/ext IOR of the outer surface (geometry.py:160-170)
    k.eta_int = d.medium_ior / d.vial_ior;   // and of the inner one (geometry.py:171-183)
    k.nsig2 = -d.sigma_t * 1.44269504088896340736f;
    k.sig_t = d.sigma_t;
    k.sig_s = d.albedo * d.sigma_t;
    k.rr_depth = d.rr_depth;
    k.phase_type = d.phase_type;
    k.phase_g = d.phase_g;
    k.sensor_type = d.sensor_type;
    k.majorant = d.majorant;
    k.wscale = 0.0f;  // per call
    {
        double hxy = std::max((double)k.h[0], (double)k.h[1]);
        k.vox_chord = (float)std::min(1.0, (double)d.sigma_t * std::sqrt(2.0) * hxy);
        k.rays_per_voxel = (float)((double)(a1 - a0) * (std::ceil(std::sqrt(2.0) * hxy / d.pixel_size_x) + 1.0));
    }
    return k;
}

template <typename T>
static int upload(T** dst, const std::vector<T>& v) {
    size_t bytes = std::max<size_t>(v.size(), 1) * sizeof(T);
    hipError_t e = hipMalloc((void**)dst, bytes);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc");
    if (!v.empty()) {
        e = hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpy");
    }
    return 0;
}

// Tuning knobs (TVAM_<NAME> environment variables) are honoured only under TVAM_EXPERIMENTAL=1 --
// A/B runs and the tests that force a code path (work splits, slab depths, chunk sizes) -- and
// each honoured one is logged; production plans take the defaults whatever the environment holds.
int tvam_knob(const char* name, int def) {
    const char* x = std::getenv("TVAM_EXPERIMENTAL");  // read per call: a test process sets it per test
    if (!(x && std::atoi(x) == 1)) return def;
    const char* v = std::getenv(name);
    if (!(v && *v)) return def;
    const int r = std::atoi(v);
    std::fprintf(stderr, "[tvam] TVAM_EXPERIMENTAL: %s=%d (default %d)\n", name, r, def);
    return r;
}
#define env_int tvam_knob

// Launch timer of the dominant forward kernel (tvam_plan_kernel_time): event pairs recorded on the
// launching stream around each launch while enabled (up to 1024 launches per measurement).  One
// timer per process, owned by the plan that enabled it: launches on another device are not
// recorded, the state is guarded by a mutex (plans on other host threads may launch meanwhile),
// and the events are destroyed with the owning plan.
namespace {
struct KernelTimer {
    std::mutex mu;
    bool on = false;
    int kind = 0;  // TvamKtKind of the measured plan's dominant forward kernel
    int device = -1;
    const tvam_plan* owner = nullptr;
    std::vector<hipEvent_t> ev;
    size_t n = 0;
};
KernelTimer g_kt;

bool kt_here(int kind) {
    if (!g_kt.on || kind != g_kt.kind || g_kt.n + 2 > g_kt.ev.size()) return false;
    int cur = -1;
    return hipGetDevice(&cur) == hipSuccess && cur == g_kt.device;
}

// the owner's events (every recorded pair complete first); caller holds the mutex
void kt_release() {
    for (size_t i = 0; i < g_kt.n; ++i) (void)hipEventSynchronize(g_kt.ev[i]);
    for (hipEvent_t e : g_kt.ev) (void)hipEventDestroy(e);
    g_kt.ev.clear();
    g_kt.n = 0;
    g_kt.on = false;
    g_kt.owner = nullptr;
    g_kt.device = -1;
}
}  // namespace

static void kt_plan_gone(const tvam_plan* p) {
    std::lock_guard<std::mutex> lk(g_kt.mu);
    if (g_kt.owner == p) kt_release();
}

void tvam_kt_begin(hipStream_t stream, int kind) {
    std::lock_guard<std::mutex> lk(g_kt.mu);
    if (kt_here(kind)) (void)hipEventRecord(g_kt.ev[g_kt.n], stream);
}

bool tvam_kt_take(int kind, hipEvent_t* start, hipEvent_t* stop) {
    std::lock_guard<std::mutex> lk(g_kt.mu);
    if (!kt_here(kind)) return false;
    *start = g_kt.ev[g_kt.n];
    *stop = g_kt.ev[g_kt.n + 1];
    g_kt.n += 2;
    return true;
}

void tvam_kt_end(hipStream_t stream, int kind) {
    std::lock_guard<std::mutex> lk(g_kt.mu);
    if (!kt_here(kind)) return;
    (void)hipEventRecord(g_kt.ev[g_kt.n + 1], stream);
    g_kt.n += 2;
}

// Planar fast path: regular sampling and rows whose vial entry offset is
// row-independent (|z| <= 0.7 r < r / sqrt(2) <= max(|p_x|, |p_y|) on the
// vial wall).  Builds the row -> slice CSR of valid rows and the per-(angle,
// column) ray table (computed once, here).
static bool planar_fwd_setup(tvam_plan* p, const std::vector<float2>& cs, const std::vector<int32_t>& off);
static int fwd_buffers(tvam_plan* p);
static int choose_fwd_z(tvam_plan* p);
static int refr_fwd_setup(tvam_plan* p, const std::vector<int32_t>& off);

static int planar_setup(tvam_plan* p, const std::vector<float2>& cs) {
    const tvam_desc& d = p->desc;
    const TvamConsts& k = p->k;
    // occluders end segments at z-dependent points: rows no longer share a path
    if (!d.regular_sampling || (d.flags & TVAM_FLAG_NO_PLANAR) || p->empty || d.n_occluder_tris > 0) return 0;
    std::vector<std::vector<int32_t>> rows_of(k.nz);
    for (int rc = 0; rc < d.crop_y; ++rc) {
        float xc, yc;
        tvam_ray_camera(k, 0, d.crop_offset_y + rc, 0.5f, 0.5f, xc, yc);
        const int s = tvam_slice_of(k, yc) - k.z0;
        if (s < 0 || s >= k.nz || !(yc >= -k.vial_half_h && yc <= k.vial_half_h)) continue;  // misses grid / vial / slab
        if (!(std::fabs(yc) <= 0.7f * d.vial_r)) return 0;  // spawn offset would depend on z
        rows_of[s].push_back(rc);
    }
    std::vector<int32_t> off(k.nz + 1, 0), rows;
    for (int s = 0; s < k.nz; ++s) {
        off[s] = (int32_t)rows.size();
        rows.insert(rows.end(), rows_of[s].begin(), rows_of[s].end());
    }
    off[k.nz] = (int32_t)rows.size();
    p->planar_fz = env_int("TVAM_PLANAR_FWD_Z", 0);  // 0: chosen from the slab depth (planar_fwd_setup)
    // adjoint slices per workgroup: 8 (one march gathers 8 slices: measured 5.2 -> 3.9 ms on
    // config 2 with 1024-thread workgroups and 45 x 45 tiles), 4 for films under 8 slices
    // (TVAM_PLANAR_ADJ_Z: 4 = the tile adjoint at 4 slices, 8 / 16 = the list adjoint's slices per workgroup)
    const int az_knob = env_int("TVAM_PLANAR_ADJ_Z", 0);
    p->planar_az = az_knob == 4 || k.nz < 8 ? 4 : 8;
    if (p->planar_fz != 8 && p->planar_fz != 16 && p->planar_fz != 24 && p->planar_fz != 28 && p->planar_fz != 32 &&
        p->planar_fz != 40 && p->planar_fz != 48 && p->planar_fz != 52 && p->planar_fz != 60)
        p->planar_fz = 0;
    const int ns = (int)cs.size();
    int32_t mrc = 0;
    for (int z0 = 0; z0 < k.nz; z0 += p->planar_az)
        mrc = std::max<int32_t>(mrc, off[std::min(z0 + p->planar_az, k.nz)] - off[z0]);
    p->pl.ns = ns;
    p->pl.max_rows_chunk = mrc;
    p->pl.max_rows_slice = 0;
    for (int z = 0; z < k.nz; ++z) p->pl.max_rows_slice = std::max(p->pl.max_rows_slice, off[z + 1] - off[z]);
    p->planar_rz = 4;
    p->pl.adj_pitch = p->tiles.tsx + 2;
    p->pl.rayfwd_pitch = p->pl.adj_pitch;
    // Refracted rays are not parallel, and a DMD much finer than the voxels
    // overflows the voxel-driven forward's column window: there the forward
    // is ray-driven like the adjoint (one record per (angle, column), shared
    // by all slices).
    p->planar_fwd = !p->cyl && !(d.flags & TVAM_FLAG_RAY_FWD);
    if (p->planar_fwd && !planar_fwd_setup(p, cs, off)) p->planar_fwd = false;
    if (tvam_planar_adj_lds(p->pl, p->tiles, p->planar_az) > 160 * 1024) p->planar_az = 4;
    if (tvam_planar_adj_lds(p->pl, p->tiles, p->planar_az) > 160 * 1024) return 0;  // tile too large: general path
    {
        // Split each tile's ray list over up to 8 workgroups until there are >= ~16K in
        // all: a thin slab (z-slab sharding) leaves few (tile, chunk) workgroups for 256
        // CUs, and even the full film (10K at 400^3) ends with a ragged last round
        // (measured 5.30 -> 5.20 ms at split 2 on config 2).  1024-thread workgroups each
        // reload a 71 KB gradient tile, so they aim at half as many: >= ~8K (config 2:
        // split 3 instead of 5, adjoint 3.98 -> 3.72 ms; split 8: 4.29 ms).  At most 4: the thin
        // slabs of 4 / 8 z-slab ranks (split 8 by the rule) measured adjoint 1.15 / 0.63 ms at
        // split 8, 1.01 / 0.57 ms at 4, 1.00 / 0.59 ms at 2 (profiles/r03/s2/slab_split_ab.jsonl)
        // 1024 threads at Z = 8: the 71 KB tile admits 2 workgroups per CU = 8 waves per SIMD
        const int ant = env_int("TVAM_ADJ_NT", p->planar_az >= 8 ? 1024 : 512);
        p->pl.adj_nt = ant == 1024 ? 1024 : 512;
        const int64_t want = p->pl.adj_nt >= 1024 ? 8192 : 16384;
        const int64_t nwg = (int64_t)p->tiles.ntx * p->tiles.nty * ((k.nz + p->planar_az - 1) / p->planar_az);
        int split = (int)std::min<int64_t>(4, std::max<int64_t>(1, (want + nwg - 1) / std::max<int64_t>(nwg, 1)));
        const int es = env_int("TVAM_ADJ_SPLIT", 0);
        if (es >= 1 && es <= 64) split = es;
        p->pl.adj_split = split;
        p->pl.rayfwd_nt = 512;
    }
    if (tvam_planar_rayfwd_lds(p->pl, p->tiles, p->planar_rz) > 160 * 1024) p->planar_rz = 4;
    if (tvam_planar_rayfwd_lds(p->pl, p->tiles, p->planar_rz) > 160 * 1024) return 0;
    int rc;
    const size_t nrec = (size_t)std::max(ns, 1) * d.crop_x;
    hipError_t e;
    if ((rc = upload(&p->d_pl_slice_off, off)) || (rc = upload(&p->d_pl_slice_rows, rows))) return rc;
    if (p->planar_fwd) {
        // the forward's scalar loads read two angles' constants at a time: pad both tables so the pair
        // of the last angle stays inside its allocation
        p->fwd_ang_h.resize(p->fwd_ang_h.size() + 4, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
        p->fwd_cb_h.resize(p->fwd_cb_h.size() + 2, 0);
        if ((rc = upload(&p->d_pl_fwd_ang, p->fwd_ang_h)) || (rc = upload(&p->d_pl_fwd_cb, p->fwd_cb_h))) return rc;
        p->pl.fwd_ang = p->d_pl_fwd_ang;
        p->pl.fwd_cb = p->d_pl_fwd_cb;
    }
    p->fwd_ang_h.clear();
    p->fwd_cb_h.clear();
    p->pl.fwd_parts = 1;
    if (p->planar_fwd && (rc = fwd_buffers(p))) return rc;
    if ((e = hipMalloc((void**)&p->d_pl_vox, nrec * sizeof(float4))) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_pl_rec_f, nrec * sizeof(float4))) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_pl_rec_i, nrec * sizeof(int32_t))) != hipSuccess ||
        (p->cyl && (e = hipMalloc((void**)&p->d_pl_rec_g, nrec * sizeof(float4))) != hipSuccess) ||
        (e = hipMalloc((void**)&p->d_amax, (size_t)std::max(ns, 1) * sizeof(unsigned))) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_fscale, 2 * sizeof(float))) != hipSuccess)
        return hip_fail(e, "hipMalloc (planar tables)");
    // refracting vial: the voxel-driven forward over per-column chords (tvam_refr_model_kernel)
    const bool try_refr = p->cyl && !(d.flags & TVAM_FLAG_RAY_FWD) && ns > 0;
    float4* d_chord = nullptr;
    if (try_refr && ((e = hipMalloc((void**)&p->d_pl_vox2, nrec * sizeof(float4))) != hipSuccess ||
                     (e = hipMalloc((void**)&d_chord, nrec * sizeof(float4))) != hipSuccess)) {
        (void)hipFree(d_chord);
        return hip_fail(e, "hipMalloc (refracted forward tables)");
    }
    p->pl.vox2 = p->d_pl_vox2;
    p->pl.chord = d_chord;
    p->pl.cs = p->d_cs;
    p->pl.vox = p->d_pl_vox;
    p->pl.rec_f = p->d_pl_rec_f;
    p->pl.rec_i = p->d_pl_rec_i;
    p->pl.rec_g = p->d_pl_rec_g;
    p->pl.slice_off = p->d_pl_slice_off;
    p->pl.slice_rows = p->d_pl_slice_rows;
    if (ns > 0) {
        if ((e = tvam_launch_planar_rays(k, p->pl, nullptr)) != hipSuccess) return hip_fail(e, "planar ray table");
        if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(e, "planar ray table");
        // A column whose DDA starts with a frozen axis (sensor.py:358, see tvam_frozen_kernel) leaves
        // its chord; the planar kernels cannot follow it, so such a plan runs the per-ray tile path
        // (none occurs in the BASELINE configs under regular sampling).
        std::vector<int32_t> ri((size_t)ns * k.crop_x);
        if ((e = hipMemcpy(ri.data(), p->d_pl_rec_i, ri.size() * sizeof(int32_t), hipMemcpyDeviceToHost)) != hipSuccess)
            return hip_fail(e, "hipMemcpy");
        for (int32_t v : ri)
            if (v == -2) {
                (void)hipFree(d_chord);
                p->pl.chord = nullptr;
                return 0;
            }
    }
    if (try_refr) {
        rc = refr_fwd_setup(p, off);
        (void)hipFree(d_chord);
        p->pl.chord = nullptr;
        if (rc) return rc;
    }
    // the adjoint over slice-invariant visit lists (tvam_adjlist.hip), when they fit in a quarter of
    // the free device memory (config 2: ~0.5 GB); else the tile adjoint re-derives the visits.
    // Groups = (tile, step quadrant, part), parts until the grid holds >= 8K workgroups.
    p->pl.adjl_ngroups = 0;
    if (p->planar_az == 8 && ns > 0 && env_int("TVAM_ADJ_LISTS", 1)) {
        // 16 slices per workgroup (one per CU) on deep films, 8 (two per CU) on thin ones: the
        // 50-slice slabs of 8 ranks ran 0.68 ms at 16 (four chunks, the last 2 slices deep) and
        // 0.47 ms at 8; 400 slices 3.20 ms at 16, 3.29 at 8 (profiles/r05/slab_adjoint_z/)
        p->pl.adjl_z = env_int("TVAM_ADJL_Z", az_knob == 8 || k.nz < 256 ? 8 : 16) == 8 ? 8 : 16;
        const int64_t nwg4 = (int64_t)p->tiles.ntx * p->tiles.nty * 4 * ((k.nz + p->pl.adjl_z - 1) / p->pl.adjl_z);
        // built by the first adjoint call (ensure_adj_lists): a forward-only plan (final_render) never
        // pays for them
        p->adjl_parts = (int)std::min<int64_t>(4, std::max<int64_t>(1, (4096 + nwg4 - 1) / std::max<int64_t>(nwg4, 1)));
        p->adjl_pending = true;
    }
    p->planar = true;
    return 0;
}


// Buffers of the voxel-driven forward (straight or refracted): angle parts of thin slabs and
// the slice-binned patterns.
static int fwd_buffers(tvam_plan* p) {
    const tvam_desc& d = p->desc;
    const TvamConsts& k = p->k;
    const int ns = p->pl.ns;
    hipError_t e;
    // A thin slab leaves few (16x16 tile, slice chunk) workgroups, each running
    // every angle: at 3 resident workgroups per CU, 1250 of them (400^2 film,
    // 50 slices) fill 1.6 rounds of the 768 slots.  Split the angles into parts
    // until >= 4 rounds; the partial doses are summed in fixed order.
    const int tw = 16;
    const int64_t nwg = (int64_t)((k.res[0] + tw - 1) / tw) * ((k.res[1] + 15) / 16) *
                        ((k.nz + p->planar_fz - 1) / p->planar_fz);
    int parts = (int)std::min<int64_t>(4, std::max<int64_t>(1, (4 * 768 + nwg - 1) / std::max<int64_t>(nwg, 1)));
    const int ep = env_int("TVAM_FWD_PARTS", 0);
    if (ep >= 1 && ep <= 16) parts = ep;
    parts = std::max(1, std::min(parts, ns));
    if (parts > 1) {
        const size_t bytes = (size_t)parts * k.nz * k.res[0] * k.res[1] * sizeof(float);
        if ((e = hipMalloc((void**)&p->d_pl_part, bytes)) != hipSuccess) return hip_fail(e, "hipMalloc (forward parts)");
        p->pl.fwd_part = p->d_pl_part;
    }
    p->pl.fwd_parts = parts;
    // Slice-binned patterns ([angle][pad + column][slice], tvam_slice_bin_kernel): the
    // forward stages each window column's Z slices with 16-byte loads and stores
    const int Z = p->planar_fz;
    const int nq = (p->pl.ncmax * (Z / 4) + 255) / 256;
    if (env_int("TVAM_FWD_BIN", 1) && nq <= 2 && ns > 0) {
        if (p->pl.fwd_ab > 2 || (nq == 2 && p->pl.fwd_ab != 2)) p->pl.fwd_ab = 2;  // the instantiated variants
        p->pl.bin_pad = p->pl.ncmax;
        p->pl.bin_nz = (k.nz + Z - 1) / Z * Z;
        const size_t bytes = (size_t)ns * (d.crop_x + 2 * p->pl.bin_pad) * p->pl.bin_nz * sizeof(float);
        if ((e = hipMalloc((void**)&p->d_pl_bin, bytes)) != hipSuccess) return hip_fail(e, "hipMalloc (binned patterns)");
        if ((e = hipMemset(p->d_pl_bin, 0, bytes)) != hipSuccess) return hip_fail(e, "hipMemset (binned patterns)");
        p->pl.fwd_bin = p->d_pl_bin;
        p->pl.fwd_pf = nq;
    }
    // binned slabs staged by LDS-DMA where the window fits (tvam_planar_fwd_dma_ok; wider windows
    // keep the register staging)
    p->pl.fwd_dma = tvam_planar_fwd_dma_ok(p->pl, Z) ? 1 : 0;
    return 0;
}


// Slices per workgroup of the voxel-driven forward: the fewest padded slice-passes
// ceil(nz / Z) * (Z + 12) (the +12 prices the per-angle candidate geometry and staging shared by
// the Z slices), register-staged depths (windows the LDS-DMA staging cannot take) priced 25 %
// higher, among the depths whose staging fits.  With the DMA staging, Z = 52 on 400-slice films
// (8 chunks; Z = 60, 7 chunks, measured a tie: kernel 2294 against 2306 us, its 420-slice binning
// 110 against 93 us, profiles/r06/; round 5: Z = 52 2.68, 40 2.72, 32 2.81 ms, profiles/r05/fwd_depth/),
// and Z = 60 / 48 on films of <= 60 / 48 slices (the slabs of 8 ranks, 48-57 slices: one chunk).
// Returns false when none fits.
static int choose_fwd_z(tvam_plan* p) {
    const TvamConsts& k = p->k;
    if (p->planar_fz == 0) {
        int best = 8;
        int64_t bcost = INT64_MAX;
        const bool deep = env_int("TVAM_FWD_BIN", 1) != 0;
        for (int Z : {60, 52, 48, 40, 32, 28, 24, 16, 8}) {
            if ((Z > 32 && !deep) || !tvam_planar_fwd_fits(p->pl, Z)) continue;
            if (Z == 60 && k.nz > 60) continue;  // one-chunk slabs only (400 slices: a tie with 52, binning +15 %)
            const int64_t cost =
                (int64_t)((k.nz + Z - 1) / Z) * (Z + 12) * (deep && tvam_planar_fwd_dma_window(p->pl, Z) ? 4 : 5);
            if (cost < bcost) bcost = cost, best = Z;
        }
        p->planar_fz = best;
    }
    for (int Z : {60, 52, 48, 40, 32, 28, 24, 16, 8})  // the deepest instantiated depth <= the choice that fits
        if (Z <= p->planar_fz && tvam_planar_fwd_fits(p->pl, Z)) {
            p->planar_fz = Z;
            break;
        }
    return tvam_planar_fwd_fits(p->pl, p->planar_fz) ? 1 : 0;
}

// Refracted voxel-driven forward (after the planar ray table, with pl.chord filled): the
// per-angle run of columns whose chords reach the medium (contiguous, else no voxel-driven
// forward), the per-(tile, angle) chord-index models and the staged window width.  Leaves
// planar_fwd false (the ray-driven forward serves) when the tables do not fit.
static int refr_fwd_setup(tvam_plan* p, const std::vector<int32_t>& off) {
    const tvam_desc& d = p->desc;
    const TvamConsts& k = p->k;
    const int ns = p->pl.ns;
    hipError_t e;
    std::vector<float4> vox((size_t)ns * d.crop_x);
    if ((e = hipMemcpy(vox.data(), p->d_pl_vox, vox.size() * sizeof(float4), hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_fail(e, "hipMemcpy");
    std::vector<int2> range(ns);
    for (int a = 0; a < ns; ++a) {
        int c0 = -1, c1 = -2;
        for (int c = 0; c < d.crop_x; ++c)
            if (vox[(size_t)a * d.crop_x + c].z >= 0.0f) {
                if (c0 < 0) c0 = c;
                if (c1 >= 0 && c1 != c - 1) return 0;  // a gap in the run: the bisection needs one
                c1 = c;
            }
        range[a] = make_int2(c0, c1);
    }
    // The chord-index model needs chords that do not cross inside the grid: every chord's end
    // points must lie on one side of its predecessor's line, the same side for the whole angle
    // (strong refraction can fold the beam; the ray-driven forward then serves).
    {
        std::vector<float4> chord((size_t)ns * d.crop_x);
        if ((e = hipMemcpy(chord.data(), p->pl.chord, chord.size() * sizeof(float4), hipMemcpyDeviceToHost)) != hipSuccess)
            return hip_fail(e, "hipMemcpy");
        for (int a = 0; a < ns; ++a) {
            int orient = 0;
            for (int c = range[a].x; c < range[a].y; ++c) {
                const float4 A = chord[(size_t)a * d.crop_x + c], B = chord[(size_t)a * d.crop_x + c + 1];
                const double tb = vox[(size_t)a * d.crop_x + c + 1].z;
                const double pts[2][2] = {{B.x, B.y}, {B.x + tb * B.z, B.y + tb * B.w}};
                for (const auto& q : pts) {
                    const double sd = (q[0] - A.x) * (double)A.w - (q[1] - A.y) * (double)A.z;
                    const int sg = sd > 0.0 ? 1 : (sd < 0.0 ? -1 : 0);
                    if (sg == 0 || (orient != 0 && sg != orient)) return 0;
                    orient = sg;
                }
            }
        }
    }
    const int ntiles = ((k.res[0] + 15) / 16) * ((k.res[1] + 15) / 16);
    const size_t nm = (size_t)ntiles * ns;
    int2* d_range = nullptr;
    int32_t* d_need = nullptr;
    int rc = upload(&d_range, range);
    if (rc) return rc;
    if ((e = hipMalloc((void**)&p->d_pl_fwd_model, 2 * nm * sizeof(float4))) != hipSuccess ||
        (e = hipMalloc((void**)&d_need, nm * sizeof(int32_t))) != hipSuccess) {
        (void)hipFree(d_range);
        (void)hipFree(d_need);
        return hip_fail(e, "hipMalloc (refracted forward models)");
    }
    e = tvam_launch_refr_model(k, p->pl, d_range, p->d_pl_fwd_model, d_need, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    std::vector<int32_t> need(nm);
    std::vector<float4> mdl(2 * nm);
    if (e == hipSuccess) e = hipMemcpy(need.data(), d_need, nm * sizeof(int32_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(mdl.data(), p->d_pl_fwd_model, 2 * nm * sizeof(float4), hipMemcpyDeviceToHost);
    (void)hipFree(d_range);
    (void)hipFree(d_need);
    if (e != hipSuccess) return hip_fail(e, "refracted forward models");
    int ncm = 1, ncmax_c = 1;
    for (size_t i = 0; i < nm; ++i) {
        int nc;
        std::memcpy(&nc, &mdl[2 * i + 1].y, sizeof(int));
        ncm = std::max(ncm, need[i]);
        ncmax_c = std::max(ncmax_c, nc);
        // windows wholly outside the crop stage only the binned patterns' zero pads
        int cb;
        std::memcpy(&cb, &mdl[2 * i + 1].z, sizeof(int));
        (void)cb;
    }
    TvamPlanar save = p->pl;
    p->pl.fwd_refr = 1;
    p->pl.ncmax = ncm;
    p->pl.fwd_nc = ncmax_c;
    p->pl.fwd_ab = 2;
    p->pl.fwd_model = p->d_pl_fwd_model;
    {
        bool multi = false;
        for (int z = 0; z < k.nz; ++z) multi |= off[z + 1] - off[z] > 1;
        p->pl.fwd_multi = multi ? 1 : 0;
    }
    // clamp windows into the binned patterns' zero pads (bin_pad = ncmax on either side)
    bool changed = false;
    for (size_t i = 0; i < nm; ++i) {
        int cb;
        std::memcpy(&cb, &mdl[2 * i + 1].z, sizeof(int));
        const int cl = std::min(std::max(cb, -ncm), (int)d.crop_x);
        if (cl != cb) {
            std::memcpy(&mdl[2 * i + 1].z, &cl, sizeof(int));
            changed = true;
        }
    }
    if (changed && (e = hipMemcpy(p->d_pl_fwd_model, mdl.data(), 2 * nm * sizeof(float4), hipMemcpyHostToDevice)) !=
                       hipSuccess)
        return hip_fail(e, "hipMemcpy");
    if (!choose_fwd_z(p)) {
        p->pl = save;
        (void)hipFree(p->d_pl_fwd_model);
        p->d_pl_fwd_model = nullptr;
        return 0;
    }
    const int nq = (p->pl.ncmax * (p->planar_fz / 4) + 255) / 256;
    p->pl.fwd_pf = nq;
    p->planar_fwd = true;
    if ((rc = fwd_buffers(p))) return rc;
    if (!p->pl.fwd_bin) return fail(TVAM_ERR_INVALID, "refracted voxel-driven forward needs the binned patterns");
    return 0;
}

// Voxel-driven forward tables (straight rays); false when the DMD is too fine
// for the staged column window.
static bool planar_fwd_setup(tvam_plan* p, const std::vector<float2>& cs, const std::vector<int32_t>& off) {
    const tvam_desc& d = p->desc;
    const TvamConsts& k = p->k;
    const int ns = (int)cs.size();
    // Forward (voxel-driven) tables.  Per angle, in the kernel's fp32 ops:
    // u(X, Y) = X * (s du) + Y * (-c du) + u0 is the crop column whose ray has
    // lateral coordinate X s - Y c (common.py:96-99: x_c = W a (0.5 - u));
    // w = half the voxel's lateral width in columns + the spawn-offset margin.
    // A voxel's candidates are the NC columns from ceil(u - w) on; every
    // (16x16 tile, angle) stages a window of ncmax columns from fwd_cb.
    // The spawn offset moves a planar ray's line sideways by at most its length
    // (1 + max|p|) * RayEpsilon, max|p| = r on the vial wall (|p_z| <= 0.7 r here).
    const double marg_u = 1.5 * (1.0 + (double)d.vial_r) * (double)TVAM_RAY_EPS * (double)d.res_x / (double)k.ex + 1e-3;
    const float du = -(float)d.res_x / k.ex;
    const float u0 = 0.5f * (float)d.res_x - 0.5f - (float)d.crop_offset_x;
    std::vector<float4> fang(2 * (size_t)std::max(ns, 1));
    double wmax = 0.0;
    for (int i = 0; i < ns; ++i) {
        const float c = cs[i].x, sn = cs[i].y, dxr = -c, dyr = -sn;
        const int fl = (std::fabs(dxr) > 1e-8f ? 1 : 0) | (std::fabs(dyr) > 1e-8f ? 2 : 0);
        const float w = 0.5f * (k.h[0] * std::fabs(sn) + k.h[1] * std::fabs(c)) * std::fabs(du) + (float)marg_u;
        int32_t flb = fl;
        float flf;
        std::memcpy(&flf, &flb, sizeof(flf));
        fang[2 * (size_t)i] = make_float4(sn * du, -c * du, 1.0f / dxr, 1.0f / dyr);
        fang[2 * (size_t)i + 1] = make_float4(w, flf, 0.0f, 0.0f);
        wmax = std::max(wmax, (double)w);
    }
    const int nc = (int)std::floor(2.0 * wmax + 1e-3) + 1;
    // per (16 px x 16 tile, angle): the first staged column and the window width that holds every
    // voxel's candidates (px = 2: 32 x 16 tiles of voxel pairs)
    auto windows = [&](std::vector<int32_t>& fcb) {
        const int tw = 16;
        const int ntx = (k.res[0] + tw - 1) / tw, nty = (k.res[1] + 15) / 16;
        fcb.assign((size_t)ntx * nty * std::max(ns, 1), 0);
        int need = 0;
        for (int t = 0; t < ntx * nty; ++t) {
            const int bx = t % ntx, by = t / ntx;
            const double xc0 = (double)k.bmin[0] + (bx * tw + 0.5) * k.h[0], xc1 = xc0 + (tw - 1.0) * k.h[0];
            const double yc0 = (double)k.bmin[1] + (by * 16 + 0.5) * k.h[1], yc1 = yc0 + 15.0 * k.h[1];
            for (int i = 0; i < ns; ++i) {
                const double A = fang[2 * (size_t)i].x, B = fang[2 * (size_t)i].y, w = fang[2 * (size_t)i + 1].x;
                const double uc[4] = {xc0 * A + yc0 * B, xc1 * A + yc0 * B, xc0 * A + yc1 * B, xc1 * A + yc1 * B};
                const double umin = *std::min_element(uc, uc + 4) + u0, umax = *std::max_element(uc, uc + 4) + u0;
                const int cb = (int)std::floor(umin - w) - 1;  // 1 column of slack for fp32 rounding in the kernel
                fcb[(size_t)t * ns + i] = cb;
                need = std::max(need, (int)std::ceil(umax - w) + 1 + nc - cb);
            }
        }
        // a window wholly outside the crop stages only zero columns: clamp it into the
        // slice-binned patterns' zero pads (ncmax columns either side)
        for (auto& cb : fcb) cb = std::min(std::max(cb, -need), (int)d.crop_x);
        return need;
    };
    std::vector<int32_t> fcb;
    const int need = windows(fcb);
    p->pl.marg_u = (float)marg_u;
    p->pl.u0 = u0;
    p->pl.fwd_nc = nc;
    p->pl.ncmax = need;
    {
        bool multi = false;
        for (int z = 0; z < k.nz; ++z) multi |= off[z + 1] - off[z] > 1;
        p->pl.fwd_multi = multi ? 1 : 0;
    }
    p->pl.fwd_ab = 2;  // two angles per barrier (4.34 -> 3.80 ms on config 2)
    if (!choose_fwd_z(p)) return false;
    p->pl.fwd_pf = (p->pl.ncmax * p->planar_fz + 255) / 256 <= 2 ? 2 : 4;
    p->fwd_ang_h = std::move(fang);
    p->fwd_cb_h = std::move(fcb);
    return true;
}


// Slot lists behind a refracting (cylindrical) vial.  A column's rays are no
// longer one straight line per angle: each sub-pixel position u is traced
// through the glass (tvam_segment, the kernels' own fp32 code) to its medium
// chord, and the tiles within `marg` of that chord are marked.  Jittered
// sampling covers u in [0, 1] by bisection until neighbouring chords' end
// points are within a quarter voxel (or their hit status flips at a grazing /
// total-internal-reflection boundary, refined to 2^-12 of a pixel), and marks
// each pair with their end-point distance as extra margin: the chords of the
// rays in between lie in the quadrilateral the pair spans.
namespace {
struct CylChord {
    bool hit;
    double ax, ay, bx, by;
    float w;  // interface weight
};

CylChord cyl_chord(const TvamConsts& k, float c, float s, int col, float u) {
    CylChord ch{false, 0, 0, 0, 0, 0.0f};
    float xc, yc, ox, oy, oz, dx, dy, o2x, o2y, d2x, d2y, maxt, w;
    tvam_ray_camera(k, col, 0, u, 0.5f, xc, yc);
    tvam_ray_world(k, c, s, xc, 0.0f, ox, oy, oz, dx, dy);
    if (!tvam_segment(k, ox, oy, 0.0f, dx, dy, o2x, o2y, d2x, d2y, maxt, w)) return ch;
    ch.hit = true;
    ch.ax = o2x;
    ch.ay = o2y;
    ch.bx = (double)o2x + (double)maxt * d2x;
    ch.by = (double)o2y + (double)maxt * d2y;
    ch.w = w;
    return ch;
}

double chord_dist(const CylChord& a, const CylChord& b) {
    return std::max(std::hypot(a.ax - b.ax, a.ay - b.ay), std::hypot(a.bx - b.bx, a.by - b.by));
}

struct TileGrid {
    double x0, y0, wx, wy;  // origin and tile size
    int ntx, nty;
};

// Mark the tiles whose box, grown by m, meets the segment a -> b (slab clip), with the length of
// the segment inside the tile itself (0 where only the grown box meets it).  (The length in the
// grown box made a chord pair at a square vial's corner, marked with a margin of their millimetre
// apart end points, the longest of the tile, and the length classes of the other slots collapsed:
// config 5's waves held whole within-angle length ramps, 0.57 of the march lanes busy.)
template <typename F>
void mark_tiles(const TileGrid& g, const CylChord& ch, double m, F&& mark) {
    const double lox = std::min(ch.ax, ch.bx) - m, hix = std::max(ch.ax, ch.bx) + m;
    const double loy = std::min(ch.ay, ch.by) - m, hiy = std::max(ch.ay, ch.by) + m;
    const int tx0 = std::max(0, (int)std::floor((lox - g.x0) / g.wx)), tx1 = std::min(g.ntx - 1, (int)std::floor((hix - g.x0) / g.wx));
    const int ty0 = std::max(0, (int)std::floor((loy - g.y0) / g.wy)), ty1 = std::min(g.nty - 1, (int)std::floor((hiy - g.y0) / g.wy));
    const double dx = ch.bx - ch.ax, dy = ch.by - ch.ay;
    for (int ty = ty0; ty <= ty1; ++ty)
        for (int tx = tx0; tx <= tx1; ++tx) {
            const double bx0 = g.x0 + tx * g.wx - m, bx1 = g.x0 + (tx + 1) * g.wx + m;
            const double by0 = g.y0 + ty * g.wy - m, by1 = g.y0 + (ty + 1) * g.wy + m;
            double t0 = 0.0, t1 = 1.0;
            auto clip = [&](double o, double d, double lo, double hi) {
                if (std::fabs(d) < 1e-300) return o >= lo && o <= hi;
                double a = (lo - o) / d, b = (hi - o) / d;
                if (a > b) std::swap(a, b);
                t0 = std::max(t0, a);
                t1 = std::min(t1, b);
                return t0 <= t1;
            };
            if (clip(ch.ax, dx, bx0, bx1) && clip(ch.ay, dy, by0, by1)) {
                t0 = 0.0;
                t1 = 1.0;
                const bool in = clip(ch.ax, dx, bx0 + m, bx1 - m) && clip(ch.ay, dy, by0 + m, by1 - m);
                mark(ty * g.ntx + tx, in ? (t1 - t0) * std::hypot(dx, dy) : 0.0);  // the chord's length in the tile
            }
        }
}
}  // namespace

// Fixed-point bound behind a refracting vial (replaces TvamConsts::rays_per_voxel):
// the beam converges, and a cuboid splits it into sub-beams that cross, so
// more than one ray per pixel pitch of one angle may cross a voxel.  From the
// chords of an angle at 1 (regular) or 8 (jittered) positions per column, in
// column order, split into runs of neighbours that keep one side of each
// other along the whole chord (the distance of a point moving along one chord
// to the other's line is linear, so checking both end points suffices; a miss,
// a crossing or a change of side starts a new run).  A run whose least
// neighbour spacing is s contributes at most ceil(sqrt2 h / s) + 2 columns'
// rays to a voxel (a factor 2 covers the approximation); the runs add up.
// The largest interface weight scales the bound.  A tube is rotation
// invariant (one angle); a cuboid is not (every angle, the largest sum).
static float cyl_rays_per_voxel(const tvam_desc& d, const TvamConsts& k, const std::vector<float2>& cs) {
    const int sub = d.regular_sampling ? 1 : 8;
    const int ns = (int)cs.size();
    const int nang = d.vial_type == TVAM_VIAL_SQUARE ? ns : std::min(ns, 1);
    const double hxy = std::max((double)k.h[0], (double)k.h[1]);
    const double D = 2.0 * std::sqrt(2.0) * hxy;
    double wmax = 1.0, worst = 0.0;
    std::vector<CylChord> ch;
    for (int ai = 0; ai < nang; ++ai) {
        const bool sq = d.vial_type == TVAM_VIAL_SQUARE;
        const float c = sq ? cs[ai].x : 1.0f, sn = sq ? cs[ai].y : 0.0f;
        ch.clear();
        for (int col = 0; col < d.crop_x; ++col)
            for (int j = 0; j < sub; ++j)
                ch.push_back(cyl_chord(k, c, sn, d.crop_offset_x + col, ((float)j + 0.5f) / (float)sub));
        double total = 0.0, run_s = INFINITY;
        int run_sign = 0;
        bool in_run = false;
        auto close_run = [&]() {
            if (in_run) total += (run_s < INFINITY ? std::ceil(D / run_s) : 0.0) + 2.0;
            in_run = false;
            run_s = INFINITY;
            run_sign = 0;
        };
        for (size_t i = 0; i < ch.size(); ++i) {
            if (!ch[i].hit) {
                close_run();
                continue;
            }
            wmax = std::max(wmax, (double)ch[i].w);
            in_run = true;
            if (i + 1 == ch.size() || !ch[i + 1].hit) continue;
            const double dx = ch[i].bx - ch[i].ax, dy = ch[i].by - ch[i].ay, L = std::hypot(dx, dy);
            if (!(L > 1e-12)) continue;
            const double nx = -dy / L, ny = dx / L;
            const double da = (ch[i + 1].ax - ch[i].ax) * nx + (ch[i + 1].ay - ch[i].ay) * ny;
            const double db = (ch[i + 1].bx - ch[i].ax) * nx + (ch[i + 1].by - ch[i].ay) * ny;
            const int sg = da > 0.0 ? 1 : -1;
            if (!(da * db > 0.0) || (run_sign != 0 && sg != run_sign)) {
                close_run();  // the next chord crosses (or turns): a new run starts with it
                in_run = false;
                continue;
            }
            run_sign = sg;
            run_s = std::min(run_s, std::min(std::fabs(da), std::fabs(db)) * sub);
        }
        close_run();
        worst = std::max(worst, total);
    }
    if (!(worst > 0.0)) return k.rays_per_voxel;  // no chord: the straight-ray bound
    return (float)((double)ns * worst * wmax * 1.01);
}

// Within each angle a tile's slots are ordered by decreasing predicted in-tile chord length
// (the longest of the column's traced sub-pixel chords): the per-ray tile kernels' waves take 64
// consecutive slots of one angle, which then march similar lengths (the columns of an angle
// crossing a tile have a trapezoid of lengths; in column order every wave held both ramps and the
// long middle), while neighbouring lanes still read neighbouring columns' records.
static void cyl_slot_lists(const tvam_desc& d, const TvamConsts& k, const std::vector<float2>& cs, int tsx, int tsy,
                           int ntx, int nty, double marg, std::vector<std::vector<uint32_t>>& per_tile) {
    const TileGrid g{(double)k.bmin[0], (double)k.bmin[1], tsx * (double)k.h[0], tsy * (double)k.h[1], ntx, nty};
    const double hmin = std::min(k.h[0], k.h[1]);
    per_tile.assign((size_t)ntx * nty, {});
    std::vector<std::vector<float>> len_of((size_t)ntx * nty);
    std::vector<uint32_t> last((size_t)ntx * nty, 0xffffffffu);
    std::vector<size_t> angle_start((size_t)ntx * nty, 0);
    const int ns = (int)cs.size();
    const int sort_mode = env_int("TVAM_SLOT_SORT", 3);
    const bool sort_len = sort_mode != 0;
    for (int i = 0; i < ns; ++i) {
        for (size_t t = 0; t < per_tile.size(); ++t) angle_start[t] = per_tile[t].size();
        for (int col = 0; col < d.crop_x; ++col) {
            const uint32_t key = ((uint32_t)i << 16) | (uint32_t)col;
            auto mark = [&](int t, double len) {
                if (last[t] != key) {
                    last[t] = key;
                    per_tile[t].push_back(key);
                    len_of[t].push_back((float)len);
                } else {
                    len_of[t].back() = std::max(len_of[t].back(), (float)len);
                }
            };
            const float c = cs[i].x, s = cs[i].y;
            const int colg = d.crop_offset_x + col;
            if (d.regular_sampling) {
                const CylChord ch = cyl_chord(k, c, s, colg, 0.5f);
                if (ch.hit) mark_tiles(g, ch, marg, mark);
                continue;
            }
            struct Iv {
                float u0, u1;
                CylChord a, b;
                int depth;
            };
            std::vector<Iv> st;
            st.push_back({0.0f, 1.0f, cyl_chord(k, c, s, colg, 0.0f), cyl_chord(k, c, s, colg, 1.0f), 0});
            while (!st.empty()) {
                Iv v = st.back();
                st.pop_back();
                if (!v.a.hit && !v.b.hit && v.depth >= 4) continue;  // both miss on a 1/16 pixel: between them too
                const bool mixed = v.a.hit != v.b.hit;
                const double dd = (v.a.hit && v.b.hit) ? chord_dist(v.a, v.b) : 0.0;
                if ((mixed || dd > 0.25 * hmin || v.depth < 4) && v.depth < 12) {
                    const float um = 0.5f * (v.u0 + v.u1);
                    const CylChord cm = cyl_chord(k, c, s, colg, um);
                    st.push_back({v.u0, um, v.a, cm, v.depth + 1});
                    st.push_back({um, v.u1, cm, v.b, v.depth + 1});
                    continue;
                }
                const double m = marg + (mixed ? hmin : dd);
                if (v.a.hit) mark_tiles(g, v.a, m, mark);
                if (v.b.hit) mark_tiles(g, v.b, m, mark);
            }
        }
        if (!sort_len) continue;
        for (size_t t = 0; t < per_tile.size(); ++t) {  // this angle's slots of tile t, longest first
            const size_t b = angle_start[t], e = per_tile[t].size();
            if (e - b < 2) continue;
            std::vector<size_t> ord(e - b);
            for (size_t j = 0; j < ord.size(); ++j) ord[j] = b + j;
            std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return len_of[t][x] > len_of[t][y]; });
            std::vector<uint32_t> keys(ord.size());
            std::vector<float> lens(ord.size());
            for (size_t j = 0; j < ord.size(); ++j) {
                keys[j] = per_tile[t][ord[j]];
                lens[j] = len_of[t][ord[j]];
            }
            std::copy(keys.begin(), keys.end(), per_tile[t].begin() + (std::ptrdiff_t)b);
            std::copy(lens.begin(), lens.end(), len_of[t].begin() + (std::ptrdiff_t)b);
        }
    }
    // TVAM_SLOT_SORT=2: length classes (eighths of the tile's longest chord) over all angles,
    // longest class first; angle order and the within-angle order are kept inside a class, so a
    // wave's lanes march similar lengths without mixing far-apart angles (config 4 first segments,
    // 40-angle shard: forward 32.0 -> 28.7 ms, adjoint 35.4 -> 30.8 ms; config 5 unchanged)
    // TVAM_SLOT_SORT=3 (default): the same classes within blocks of 16 angles, so the tiles of a
    // slice (one XCD's, tvam_tile_kernel) walk the angles in step and re-read each other's ray
    // records from L2 (config 5, 200-angle shard: adjoint 211 -> 206 ms, forward -0.5 %; config 4
    // unchanged; profiles/r05/ab_slot_blocks/)
    const int ablk = sort_mode == 3 ? std::max(1, env_int("TVAM_SLOT_BLOCK", 16)) : (1 << 30);
    if ((sort_mode == 2 || sort_mode == 3) && !d.regular_sampling)  // (the planar adjoint keeps the per-angle order: 3.9 -> 8.2 ms)
        for (size_t t = 0; t < per_tile.size(); ++t) {
            const size_t n = per_tile[t].size();
            if (n < 2) continue;
            const float lmax = *std::max_element(len_of[t].begin(), len_of[t].end());
            if (!(lmax > 0.0f)) continue;
            std::vector<int> cls(n);
            for (size_t j = 0; j < n; ++j)
                cls[j] = std::min(7, (int)(8.0f * len_of[t][j] / lmax)) - 8 * (int)((per_tile[t][j] >> 16) / (uint32_t)ablk);
            std::vector<size_t> ord(n);
            for (size_t j = 0; j < n; ++j) ord[j] = j;
            std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return cls[x] > cls[y]; });
            std::vector<uint32_t> keys(n);
            for (size_t j = 0; j < n; ++j) keys[j] = per_tile[t][ord[j]];
            per_tile[t].swap(keys);
        }
    for (auto& v : len_of) std::vector<float>().swap(v);
}

extern "C" int tvam_plan_create(const tvam_desc* desc, int device, tvam_plan** out) {
    if (!desc || !out) return fail(TVAM_ERR_INVALID, "null argument");
    *out = nullptr;
    int rc = validate(*desc);
    if (rc) return rc;
    const tvam_desc& d = *desc;
    int a0 = d.angle_begin, a1 = d.angle_end < 0 ? d.n_patterns : d.angle_end;
    if (a0 < 0 || a1 > d.n_patterns || a0 > a1) return fail(TVAM_ERR_INVALID, "invalid angle shard");

    if (a1 - a0 > 65536 || d.crop_x > 65536)  // slot entries pack (angle << 16 | column)
        return fail(TVAM_ERR_UNSUPPORTED, "more than 65536 angles per shard or DMD columns");

    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");

    tvam_plan* p = new tvam_plan();
    p->desc = d;
    p->device = device;
    p->k = make_consts(d, a0, a1);
    p->cyl = d.vial_type == TVAM_VIAL_CYLINDRICAL || d.vial_type == TVAM_VIAL_SQUARE;
    // index matched: entry bounce + medium segment; glass vials: two glass
    // surfaces + medium segment (volume.py:179, :271-272)
    p->empty = d.max_depth < (p->cyl ? 3 : 2);
    p->surface = d.film_channels == 2;
    p->general = !p->surface && (d.sample_time || d.sensor_type != TVAM_SENSOR_DDA);
    if (p->surface) {  // target mesh to the device (TvamConsts::tgt)
        std::vector<float> tri(d.target_tris, d.target_tris + 9 * (size_t)d.n_target_tris);
        if ((rc = upload(&p->d_tgt, tri))) {
            plan_free(p);
            return rc;
        }
        p->k.tgt = p->d_tgt;
        p->k.n_tgt = d.n_target_tris;
    }
    if (d.n_occluder_tris > 0) {  // occluder triangles to the device (TvamConsts::occ)
        std::vector<float> tri(d.occluder_tris, d.occluder_tris + 9 * (size_t)d.n_occluder_tris);
        if ((rc = upload(&p->d_occ, tri))) {
            plan_free(p);
            return rc;
        }
        p->k.occ = p->d_occ;
        p->k.n_occ = d.n_occluder_tris;
        for (int a = 0; a < 3; ++a) {
            p->k.occ_lo[a] = TVAM_INF;
            p->k.occ_hi[a] = -TVAM_INF;
        }
        for (size_t i = 0; i < tri.size(); ++i) {
            p->k.occ_lo[i % 3] = std::min(p->k.occ_lo[i % 3], tri[i]);
            p->k.occ_hi[i % 3] = std::max(p->k.occ_hi[i % 3], tri[i]);
        }
    }
    const TvamConsts& k = p->k;
    const int ns = a1 - a0;

    // tile geometry: LDS-resident xy tile of one z-slice
    auto pick = [&](int res) {
        // measured optima: the planar adjoint (regular sampling, 8 interleaved slices in LDS) at
        // <= 48 (45 at 400^3: two 71 KB tiles per CU); the per-ray tile kernels of the jittered
        // configs at 73 (config 5, 800^3: 11 tiles of 73 -> 3.15 s per iteration vs 3.35 s at 13
        // tiles of 62, 3.24 s at 80, 3.50 s at 89; config 4: 6 tiles of 67 within 1 % of 5 of 80)
        int ts = d.tile > 0 ? d.tile : (d.regular_sampling && !(d.flags & TVAM_FLAG_NO_PLANAR) ? 48 : 73);
        int nt = (res + ts - 1) / ts;
        return (res + nt - 1) / nt;
    };
    int tsx = pick(k.res[0]), tsy = pick(k.res[1]);
    int ntx = (k.res[0] + tsx - 1) / tsx, nty = (k.res[1] + tsy - 1) / tsy;
    p->ntiles = ntx * nty;
    // tile (+ guard band) + reduction scratch + per-angle max |p|
    p->lds_bytes = (size_t)TVAM_TILE_PITCH(tsx) * (tsy + 2) * sizeof(float) +
                   16 * sizeof(float) + (size_t)ns * sizeof(float);
    if (p->lds_bytes > 160 * 1024) {
        plan_free(p);
        return fail(TVAM_ERR_INVALID, "tile too large for LDS; lower tvam_desc.tile");
    }

    // per-angle rotation (motion.py:26-36)
    std::vector<float2> cs(ns);
    for (int i = 0; i < ns; ++i) {
        float time = (float)(a0 + i) / (float)d.n_patterns;
        float alpha = TVAM_TWO_PI * time;
        if (d.clockwise) alpha = -alpha;
        cs[i] = make_float2(cosf(alpha), sinf(alpha));
    }

    // per-angle DDA stepping (sensor.py:343, :357-360): d = (-c, -s)
    std::vector<float4> ang(ns);
    for (int i = 0; i < ns; ++i) {
        float d[2] = {-cs[i].x, -cs[i].y}, ts[2], st[2];
        for (int a = 0; a < 2; ++a) {
            int step = d[a] > 0.0f ? 1 : -1;
            bool valid = fabsf(d[a]) > 1e-8f;
            ts[a] = valid ? (k.h[a] / d[a]) * (float)step : TVAM_INF;
            st[a] = (float)step;
        }
        ang[i] = make_float4(ts[0], ts[1], st[0], st[1]);
    }

    // per-slice DMD rows.  A ray's height is y_c of its row (+ jitter); its
    // slice is the DDA start voxel z (tvam_slice_of).
    // (local slice s of the slab = global slice k.z0 + s)
    std::vector<std::vector<int32_t>> rows_of(k.nz);
    for (int rc = 0; rc < d.crop_y; ++rc) {
        int row = d.crop_offset_y + rc;
        if (d.regular_sampling) {
            float xc, yc;
            tvam_ray_camera(k, 0, row, 0.5f, 0.5f, xc, yc);
            int s = tvam_slice_of(k, yc) - k.z0;
            if (s >= 0 && s < k.nz) rows_of[s].push_back(rc);
        } else {
            // jittered rows: a ray's height yc(jy) is monotone in jy in fp32 (tvam_ray_camera), and so is
            // its slice (int)((yc - bmin) / h) (tvam_slice_of), so the slices of the sampler's jy in
            // [0, 1 - 2^-23] (TvamPcg::next_float) lie between those of its two ends, computed with the
            // kernels' own fp32 expressions (a slice list with a +-1 margin made two of every three row
            // slots of the tile kernels idle at 1:1 rows; jy = 1 itself, never drawn, listed a row in
            // the next slice wherever row and slice boundaries coincide)
            float xc, ytop, ybot;
            tvam_ray_camera(k, 0, row, 0.5f, 0.0f, xc, ytop);
            tvam_ray_camera(k, 0, row, 0.5f, 0.99999988f, xc, ybot);
            if (!(ytop > k.bmin[2] && ybot < k.bmax[2])) continue;  // every jittered ray misses the grid
            const float zlo = ybot > k.bmin[2] ? ybot : k.bmin[2], zhi = ytop < k.bmax[2] ? ytop : k.bmax[2];
            int s0 = (int)((zlo - k.bmin[2]) / k.h[2]), s1 = (int)((zhi - k.bmin[2]) / k.h[2]);
            s0 = std::max(k.z0, std::max(s0, 0));
            s1 = std::min(k.z0 + k.nz - 1, std::min(s1, k.res[2] - 1));
            for (int s = s0; s <= s1; ++s) rows_of[s - k.z0].push_back(rc);
        }
    }
    // Main rows of jittered plans (TvamTiles::slice_moff): a row's main slice is its centre ray's;
    // used when the row lists hold rows that only the extreme jitters take into a slice (config 5:
    // 1:1 rows list two per slice, and half of the tile kernels' slots were rays of the other
    // slice, tools/tile_diag.py) and 32 interior jitters of every row stay in its main slice.
    std::vector<int32_t> row_main(d.crop_y, -1), slice_moff(k.nz + 1, 0), slice_mrows;
    bool main_rows = false;
    if (!d.regular_sampling && env_int("TVAM_TILE_MAIN", 1) != 0) {
        std::vector<std::vector<int32_t>> mrows(k.nz);
        bool split = false;
        for (int rc = 0; rc < d.crop_y && !split; ++rc) {
            float xc, yc;
            tvam_ray_camera(k, 0, d.crop_offset_y + rc, 0.5f, 0.5f, xc, yc);
            const int sg = tvam_slice_of(k, yc);
            for (int j = 0; j < 32 && !split; ++j) {
                tvam_ray_camera(k, 0, d.crop_offset_y + rc, 0.5f, ((float)j + 0.5f) / 32.0f, xc, yc);
                split = tvam_slice_of(k, yc) != sg;
            }
            if (sg >= k.z0 && sg < k.z0 + k.nz) {
                row_main[rc] = sg - k.z0;
                mrows[sg - k.z0].push_back(rc);
            }
        }
        bool gain = false;
        for (int z = 0; z < k.nz; ++z) gain = gain || mrows[z].size() < rows_of[z].size();
        main_rows = gain && !split;
        for (int z = 0; z < k.nz && main_rows; ++z) {
            slice_moff[z] = (int32_t)slice_mrows.size();
            slice_mrows.insert(slice_mrows.end(), mrows[z].begin(), mrows[z].end());
        }
        slice_moff[k.nz] = (int32_t)slice_mrows.size();
    }
    std::vector<int32_t> slice_off(k.nz + 1, 0), slice_rows;
    p->max_rows_per_slice = 0;
    for (int s = 0; s < k.nz; ++s) {
        slice_off[s] = (int32_t)slice_rows.size();
        slice_rows.insert(slice_rows.end(), rows_of[s].begin(), rows_of[s].end());
        p->max_rows_per_slice = std::max<int32_t>(p->max_rows_per_slice, (int32_t)rows_of[s].size());
    }
    slice_off[k.nz] = (int32_t)slice_rows.size();

    // Per-tile slot lists: every (angle, DMD column) whose ray crosses the
    // tile, in (angle, column) order so that consecutive lanes read
    // consecutive ray records.  A collimated ray's lateral coordinate is
    // l = dot(o, (s,-c,0)) = x_c; the spawn offset moves it by less than
    // (1+max|p|)*RayEpsilon, covered by the margin.  (Sorting the slots by
    // predicted in-tile length balances the lanes of a wave — 0.98 instead of
    // 0.64 of the lanes busy in the march loop — but scatters the record reads
    // and the adjoint's atomics over angles, which costs more than it gains.)
    double rmax = std::max({std::fabs((double)k.bmin[0]), std::fabs((double)k.bmax[0]), std::fabs((double)k.bmin[1]),
                            std::fabs((double)k.bmax[1]), (double)d.vial_r, (double)k.vial_half_h});
    double marg_l = 4.0 * (1.0 + rmax) * (double)TVAM_RAY_EPS;
    const double W = d.res_x, ex = k.ex;
    const double vr = d.vial_r;
    std::vector<int64_t> slot_off((size_t)p->ntiles + 1, 0);
    std::vector<uint32_t> slots;
    int64_t max_nrt = 0;
    if (p->cyl) {
        std::vector<std::vector<uint32_t>> per_tile;
        // host tracing without occluders (device memory; they only shorten chords: a superset)
        TvamConsts kh = k;
        kh.occ = nullptr;
        kh.n_occ = 0;
        cyl_slot_lists(d, kh, cs, tsx, tsy, ntx, nty, marg_l + 1e-3 * std::min(k.h[0], k.h[1]), per_tile);
        p->k.rays_per_voxel = cyl_rays_per_voxel(d, kh, cs);
        for (int t = 0; t < p->ntiles; ++t) {
            slots.insert(slots.end(), per_tile[t].begin(), per_tile[t].end());
            slot_off[(size_t)t + 1] = (int64_t)slots.size();
            max_nrt = std::max<int64_t>(max_nrt, (int64_t)per_tile[t].size());
        }
    } else {
    for (int ty = 0; ty < nty; ++ty)
        for (int tx = 0; tx < ntx; ++tx) {
            int tile = ty * ntx + tx;
            double X0 = (double)k.bmin[0] + (double)(tx * tsx) * k.h[0];
            double X1 = (double)k.bmin[0] + (double)std::min((tx + 1) * tsx, k.res[0]) * k.h[0];
            double Y0 = (double)k.bmin[1] + (double)(ty * tsy) * k.h[1];
            double Y1 = (double)k.bmin[1] + (double)std::min((ty + 1) * tsy, k.res[1]) * k.h[1];
            const size_t first = slots.size();
            for (int i = 0; i < ns; ++i) {
                double c = cs[i].x, s = cs[i].y;
                double l[4] = {X0 * s - Y0 * c, X1 * s - Y0 * c, X0 * s - Y1 * c, X1 * s - Y1 * c};
                double L0 = *std::min_element(l, l + 4) - marg_l, L1 = *std::max_element(l, l + 4) + marg_l;
                L0 = std::max(L0, -vr - marg_l);
                L1 = std::min(L1, vr + marg_l);
                if (!(L0 <= L1)) continue;
                double c_lo = W * (0.5 - L1 / ex) - 1.0, c_hi = W * (0.5 - L0 / ex);
                int cl = std::max((int)std::floor(c_lo) - 1 - d.crop_offset_x, 0);
                int ch = std::min((int)std::ceil(c_hi) + 1 - d.crop_offset_x, d.crop_x - 1);
                // (column order: ordering by in-tile chord length, as behind refracting vials, made the
                // planar adjoint slower, 3.82 -> 3.96 ms on config 2)
                for (int col = cl; col <= ch; ++col) slots.push_back(((uint32_t)i << 16) | (uint32_t)col);
            }
            slot_off[(size_t)tile + 1] = (int64_t)slots.size();
            max_nrt = std::max<int64_t>(max_nrt, (int64_t)(slots.size() - first));
        }
    }
    // flat slot count per workgroup must fit int32 (rows * slots * spp)
    if ((int64_t)p->max_rows_per_slice * max_nrt * 64 > (int64_t)0x7fffffff) {
        plan_free(p);
        return fail(TVAM_ERR_TOO_LARGE, "too many rays per tile for one launch");
    }

    if ((rc = upload(&p->d_cs, cs)) || (rc = upload(&p->d_slice_off, slice_off)) ||
        (rc = upload(&p->d_slice_rows, slice_rows)) || (rc = upload(&p->d_slots, slots)) ||
        (rc = upload(&p->d_slot_off, slot_off)) || (rc = upload(&p->d_ang, ang))) {
        plan_free(p);
        return rc;
    }
    e = hipMalloc((void**)&p->d_counter, sizeof(unsigned long long));
    if (e != hipSuccess) {
        plan_free(p);
        return hip_fail(e, "hipMalloc");
    }
    p->tiles.cs = p->d_cs;
    p->tiles.slice_off = p->d_slice_off;
    p->tiles.slice_rows = p->d_slice_rows;
    p->tiles.slots = p->d_slots;
    p->tiles.slot_off = p->d_slot_off;
    p->tiles.ang = p->d_ang;
    p->n_slots_all = (int64_t)slots.size();
    p->n_main_rows = main_rows ? (int64_t)slice_mrows.size() : 0;
    p->n_rows_all = (int64_t)slice_rows.size();
    if (main_rows) {
        if (slice_mrows.empty()) slice_mrows.push_back(0);
        if ((rc = upload(&p->d_slice_moff, slice_moff)) || (rc = upload(&p->d_slice_mrows, slice_mrows)) ||
            (rc = upload(&p->d_row_main, row_main))) {
            plan_free(p);
            return rc;
        }
        p->tiles.slice_moff = p->d_slice_moff;
        p->tiles.slice_mrows = p->d_slice_mrows;
        p->tiles.row_main = p->d_row_main;
    }
    for (auto& r : p->rs)
        if ((e = hipEventCreateWithFlags(&r.ready, hipEventDisableTiming)) != hipSuccess) {
            plan_free(p);
            return hip_fail(e, "hipEventCreate");
        }
    p->tiles.ntx = ntx;
    p->tiles.nty = nty;
    p->tiles.tsx = tsx;
    p->tiles.tsy = tsy;
    p->tiles.n_shard = ns;
    if (!p->surface && !p->general && (rc = planar_setup(p, cs))) {
        plan_free(p);
        return rc;
    }
    *out = p;
    return 0;
}

// tvam_scatter_binned found brick walks that disagree with the record writer's counts
static int bin_mismatch_fail(tvam_plan* p) {
    uint32_t bad = 0;
    if (p->bins.sb.bad) (void)hipMemcpy(&bad, p->bins.sb.bad, sizeof(uint32_t), hipMemcpyDeviceToHost);
    return fail(TVAM_ERR_HIP, "brick bins: " + std::to_string(bad) +
                                  " scattered segments' brick walks disagree with their closed-form brick counts "
                                  "(entries would be lost); rerun with TVAM_FLAG_SCATTER_ATOMIC");
}

// per-call constants: spp forced to 1 under regular sampling (common.py:49-51),
// weight = inv_pdf / n_samples * print_time (projector.py:164-165, :187; common.py:111)
static int call_setup(tvam_plan* p, uint64_t n_active, const uint32_t* active_pixels, uint32_t& spp, TvamConsts& k) {
    const tvam_desc& d = p->desc;
    uint64_t dense_n = (uint64_t)(p->k.a1 - p->k.a0) * d.crop_y * d.crop_x;  // this shard's angles
    if (!active_pixels && n_active != dense_n)
        return fail(TVAM_ERR_INVALID, "active_data and active_pixels must have the same length.");  // projector.py:137-138
    if (d.regular_sampling) spp = 1;
    if (spp == 0) spp = 4;  // optimize.py:96
    if ((d.active_total > 0 ? (uint64_t)d.active_total : n_active) * (uint64_t)spp > (1ull << 32))
        return fail(TVAM_ERR_TOO_LARGE,
                    "The total number of Monte Carlo samples required by this rendering task exceeds 2^32 = "
                    "4294967296. Please use fewer samples per pixel or render using multiple passes.");  // common.py:60-65
    k = p->k;
    // inv_pdf / n_samples over the whole active set (projector.py:164-165, :187): a shard's
    // call carries its own n_active, the reference's len(active_data) is desc.active_total
    const uint64_t n_all = d.active_total > 0 ? (uint64_t)d.active_total : n_active;
    float area = d.pixel_size_x * d.pixel_size_y * (float)n_all;
    float w = area / (float)(n_all * (uint64_t)spp);
    w = w * d.print_time;
    float ss = d.albedo * d.sigma_t;
    float sa_st = d.sigma_t != 0.0f ? (float)(((double)d.sigma_t - (double)ss) / (double)d.sigma_t) : 0.0f;
    k.wscale = w * sa_st;
    hipError_t e = hipSetDevice(p->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    return 0;
}

static int ensure_dense(tvam_plan* p) {
    const tvam_desc& d = p->desc;
    uint64_t n = (uint64_t)(p->k.a1 - p->k.a0) * d.crop_y * d.crop_x;
    if (p->d_dense && p->dense_n == n) return 0;
    hipError_t e;
    if ((e = hipMalloc((void**)&p->d_dense, n * sizeof(float))) != hipSuccess) return hip_fail(e, "hipMalloc");
    if ((e = hipMalloc((void**)&p->d_idxmap, n * sizeof(int32_t))) != hipSuccess) return hip_fail(e, "hipMalloc");
    p->dense_n = n;
    return 0;
}

// Make the per-ray records of (spp, seed) available on `stream`.  The
// buffer grows on demand (first call with a larger spp); the pre-pass runs
// only when the cached records do not match the call.
#define TVAM_FROZEN_CAP (1 << 20)
#define TVAM_STRAY_CAP (1 << 22)  // stray rays per record set (more: the tile kernels use the full row lists)

static int ensure_rays(tvam_plan* p, const TvamConsts& k, TvamTiles& t, const int32_t* idxmap, hipStream_t stream,
                       const uint32_t* active_pixels = nullptr, uint64_t n_active = 0) {
    const uint64_t n = (uint64_t)(k.a1 - k.a0) * k.crop_y * k.crop_x * t.spp;
    if (n > 0xFFFFFFFFull) {  // stray lists hold 32-bit record indices: every slice walks its full row list
        t.slice_moff = nullptr;
        t.row_main = nullptr;
    }
    hipError_t e;
    auto bind = [&](tvam_plan::RaySlot& r) {
        t.ray_f = r.f;
        t.ray_i = r.i;
        t.ray_g = r.g;
        t.frozen = r.frozen;
        t.frozen_n = r.frozen_n;
        t.frozen_cap = TVAM_FROZEN_CAP;
        if (t.slice_moff) {
            t.stray_idx = r.stray;
            t.stray_list = r.stray + TVAM_STRAY_CAP;
            t.stray_cnt = r.stray_cs;
            t.stray_off = r.stray_cs + (k.nz + 1);
            t.stray_n = r.stray_n;
            t.stray_cap = TVAM_STRAY_CAP;
        }
        r.used = ++p->ray_tick;
    };
    // jittered records of a sparse active set depend on the set (sampler streams by active
    // position): reused for the same set (pointer and count; the slice ranges of one forward,
    // the line-search forward of the same seed), like a dense set's for the same seed and spp
    auto same_set = [&](const tvam_plan::RaySlot& r) {
        return idxmap ? (r.sparse && r.pix == (const void*)active_pixels && r.npix == n_active) : !r.sparse;
    };
    for (auto& r : p->rs)
        if (r.valid && r.spp == t.spp && (k.regular || (r.seed == t.seed && same_set(r)))) {
            bind(r);
            e = hipStreamWaitEvent(stream, r.ready, 0);
            return e == hipSuccess ? 0 : hip_fail(e, "hipStreamWaitEvent");
        }
    const size_t per_ray = sizeof(float4) + sizeof(int2) + (p->cyl ? sizeof(float4) : 0);
    auto alloc = [&](tvam_plan::RaySlot& r) -> int {
        (void)hipFree(r.f);
        (void)hipFree(r.i);
        (void)hipFree(r.g);
        r.f = nullptr;
        r.i = nullptr;
        r.g = nullptr;
        r.cap = 0;
        r.valid = false;
        if ((e = hipMalloc((void**)&r.f, std::max<uint64_t>(n, 1) * sizeof(float4))) != hipSuccess ||
            (e = hipMalloc((void**)&r.i, std::max<uint64_t>(n, 1) * sizeof(int2))) != hipSuccess ||
            (p->cyl && (e = hipMalloc((void**)&r.g, std::max<uint64_t>(n, 1) * sizeof(float4))) != hipSuccess))
            return hip_fail(e, "hipMalloc (ray records)");
        if (!r.frozen &&
            ((e = hipMalloc((void**)&r.frozen, (size_t)TVAM_FROZEN_CAP * sizeof(int64_t))) != hipSuccess ||
             (e = hipMalloc((void**)&r.frozen_n, sizeof(unsigned long long))) != hipSuccess))
            return hip_fail(e, "hipMalloc (frozen-ray list)");
        if (t.slice_moff && !r.stray &&
            ((e = hipMalloc((void**)&r.stray, (size_t)2 * TVAM_STRAY_CAP * sizeof(uint32_t))) != hipSuccess ||
             (e = hipMalloc((void**)&r.stray_cs, (size_t)2 * (k.nz + 1) * sizeof(uint32_t))) != hipSuccess ||
             (e = hipMalloc((void**)&r.stray_n, sizeof(unsigned long long))) != hipSuccess))
            return hip_fail(e, "hipMalloc (stray-ray lists)");
        r.cap = n;
        return 0;
    };
    // the slot to fill: the first one; a second only for jittered records and while a quarter
    // of the device memory stays free after it; else the least recently used one that holds n
    tvam_plan::RaySlot* r = &p->rs[0];
    if (p->rs[0].cap > 0) {
        bool second = p->rs[1].cap >= n;
        if (!second && !k.regular && p->rs[1].cap == 0) {
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr > (size_t)n * per_ray + tot / 4 + ((size_t)16 << 20)) {
                int rc;
                if ((rc = alloc(p->rs[1]))) return rc;
                second = true;
            }
        }
        if (second && (p->rs[1].used < p->rs[0].used || !p->rs[1].valid)) r = &p->rs[1];
    }
    if (r->cap < n) {
        int rc;
        if ((rc = alloc(*r))) return rc;
    }
    bind(*r);
    if ((e = hipMemsetAsync(r->frozen_n, 0, sizeof(unsigned long long), stream)) != hipSuccess)
        return hip_fail(e, "hipMemsetAsync");
    if (t.slice_moff && ((e = hipMemsetAsync(r->stray_n, 0, sizeof(unsigned long long), stream)) != hipSuccess ||
                         (e = hipMemsetAsync(r->stray_cs, 0, (size_t)(k.nz + 1) * sizeof(uint32_t), stream)) != hipSuccess))
        return hip_fail(e, "hipMemsetAsync");
    if ((e = tvam_launch_ray_setup(k, t, r->f, r->i, r->g, idxmap, stream)) != hipSuccess)
        return hip_fail(e, "ray setup launch");
    if (t.slice_moff && (e = tvam_launch_stray_lists(k, t, stream)) != hipSuccess)
        return hip_fail(e, "stray list launch");
    if ((e = hipEventRecord(r->ready, stream)) != hipSuccess) return hip_fail(e, "hipEventRecord");
    r->valid = true;
    r->spp = t.spp;
    r->seed = t.seed;
    r->sparse = idxmap != nullptr;
    r->pix = idxmap ? (const void*)active_pixels : nullptr;
    r->npix = idxmap ? n_active : 0;
    return 0;
}

extern "C" int tvam_plan_set_active(tvam_plan* p, int64_t active_base, int64_t active_total) {
    if (!p) return fail(TVAM_ERR_INVALID, "null argument");
    if (active_base < 0 || active_total < 0) return fail(TVAM_ERR_INVALID, "active_base / active_total must be >= 0");
    p->desc.active_base = active_base;
    p->desc.active_total = active_total;
    p->k.stream_base = active_base;
    for (auto& r : p->rs) r.valid = false;
    return 0;
}

// Slice granularity of tvam_forward_slices: the voxel-driven forward's Z, 1 for the per-ray tile
// kernels, 0 when the plan's forward cannot be split by slices (scattered paths and per-path
// kernels add into every slice; the ray-driven planar forward).
static int fwd_chunk(const tvam_plan* p) {
    if (p->surface || p->general || p->desc.albedo != 0.0f) return 0;
    if (p->planar_fwd) return p->planar_fz;
    return p->planar ? 0 : 1;
}

extern "C" int tvam_plan_fwd_chunk(const tvam_plan* p) { return p ? fwd_chunk(p) : 0; }

static int forward_impl(tvam_plan* p, const float* active_data, const uint32_t* active_pixels, uint64_t n_active,
                        uint32_t spp, uint32_t seed, float* dose, void* stream_, int zb, int ze);

extern "C" int tvam_forward(tvam_plan* p, const float* active_data, const uint32_t* active_pixels, uint64_t n_active,
                            uint32_t spp, uint32_t seed, float* dose, void* stream_) {
    return forward_impl(p, active_data, active_pixels, n_active, spp, seed, dose, stream_, 0, -1);
}

extern "C" int tvam_forward_slices(tvam_plan* p, const float* active_data, const uint32_t* active_pixels,
                                   uint64_t n_active, uint32_t spp, uint32_t seed, int32_t z_begin, int32_t z_end,
                                   float* dose, void* stream) {
    if (!p) return fail(TVAM_ERR_INVALID, "null argument");
    const int ch = fwd_chunk(p), nz = p->k.nz;
    if (ch == 0) return fail(TVAM_ERR_UNSUPPORTED, "this plan's forward cannot be split into slice ranges");
    if (z_begin < 0 || z_end > nz || z_begin >= z_end || z_begin % ch != 0 || (z_end % ch != 0 && z_end != nz))
        return fail(TVAM_ERR_INVALID, "slice range must lie in the film and on the forward's slice chunks");
    return forward_impl(p, active_data, active_pixels, n_active, spp, seed, dose, stream, z_begin, z_end);
}

static int forward_impl(tvam_plan* p, const float* active_data, const uint32_t* active_pixels, uint64_t n_active,
                        uint32_t spp, uint32_t seed, float* dose, void* stream_, int zb, int ze) {
    if (!p || !dose || (!active_data && n_active)) return fail(TVAM_ERR_INVALID, "null argument");
    hipStream_t stream = (hipStream_t)stream_;
    TvamConsts k;
    int rc = call_setup(p, n_active, active_pixels, spp, k);
    if (rc) return rc;
    const TvamConsts& kc = k;
    size_t V = (size_t)kc.res[0] * kc.res[1] * kc.nz * (p->surface ? 2 : 1);
    const bool ranged = ze >= 0;  // tvam_forward_slices: only slices [zb, ze) of dose are written
    hipError_t e;
    if (p->surface && !p->vols) return fail(TVAM_ERR_INVALID, "surface-aware film: call tvam_plan_set_volumes first");
    if (p->empty || n_active == 0 || p->surface || p->general) {
        const size_t plane = (size_t)kc.res[0] * kc.res[1];
        e = ranged ? hipMemsetAsync(dose + (size_t)zb * plane, 0, (size_t)(ze - zb) * plane * sizeof(float), stream)
                   : hipMemsetAsync(dose, 0, V * sizeof(float), stream);
        if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync");
        if (p->empty || n_active == 0) return 0;
    }
    const float* pat = active_data;
    const int32_t* idxmap = nullptr;
    if (active_pixels) {
        if ((rc = ensure_dense(p))) return rc;
        if ((e = hipMemsetAsync(p->d_dense, 0, p->dense_n * sizeof(float), stream)) != hipSuccess ||
            (e = hipMemsetAsync(p->d_idxmap, 0xff, p->dense_n * sizeof(int32_t), stream)) != hipSuccess)
            return hip_fail(e, "hipMemsetAsync");
        if ((e = tvam_launch_scatter(kc, active_data, active_pixels, n_active, p->d_dense, p->d_idxmap, stream)) !=
            hipSuccess)
            return hip_fail(e, "scatter launch");
        pat = p->d_dense;
        idxmap = p->d_idxmap;
    }
    if (p->general) {
        TvamTiles t = p->tiles;
        t.spp = spp;
        t.seed = seed;
        e = tvam_launch_general_paths(TVAM_MODE_FWD, kc, t, pat, idxmap, nullptr, dose, nullptr, stream);
        return e == hipSuccess ? 0 : hip_fail(e, "path forward launch");
    }
    if (p->surface) {
        TvamTiles t = p->tiles;
        t.spp = spp;
        t.seed = seed;
        e = tvam_launch_surface_paths(TVAM_MODE_FWD, kc, t, pat, idxmap, nullptr, p->vols, dose, nullptr, stream);
        if (e == hipSuccess) e = tvam_launch_scale_volumes((int64_t)V, p->vols, dose, stream);
        return e == hipSuccess ? 0 : hip_fail(e, "surface-aware forward launch");
    }
    if (p->planar_fwd) {
        if (p->desc.flags & TVAM_FLAG_FWD_STATS) {
            if ((e = hipMemsetAsync(p->d_counter, 0, sizeof(unsigned long long), stream)) != hipSuccess)
                return hip_fail(e, "hipMemsetAsync");
        }
        TvamPlanar pl = p->pl;
        if (ranged) {
            pl.fwd_zc0 = zb / p->planar_fz;
            pl.fwd_nzc = (ze - zb + p->planar_fz - 1) / p->planar_fz;
        }
        e = tvam_launch_fwd_planar(kc, pl, p->planar_fz, pat, dose, stream);
        if (e != hipSuccess) return hip_fail(e, "planar forward launch");
    } else if (p->planar) {
        e = tvam_launch_fwd_rays_planar(kc, p->pl, p->tiles, p->planar_rz, pat, p->d_amax, p->d_fscale, dose, stream);
        if (e != hipSuccess) return hip_fail(e, "planar ray forward launch");
    } else {
        TvamTiles t = p->tiles;
        t.spp = spp;
        t.seed = seed;
        if (ranged) {
            t.kz0 = zb;
            t.kz1 = ze;
        }
        if ((rc = ensure_rays(p, kc, t, idxmap, stream, active_pixels, n_active))) return rc;
        unsigned long long* stats = nullptr;
        if (p->desc.flags & TVAM_FLAG_FWD_STATS) {
            if ((e = hipMemsetAsync(p->d_counter, 0, sizeof(unsigned long long), stream)) != hipSuccess)
                return hip_fail(e, "hipMemsetAsync");
            stats = p->d_counter;
        }
        tvam_kt_begin(stream, TVAM_KT_TILE);
        e = tvam_launch_tiles(TVAM_MODE_FWD, kc, t, p->lds_bytes, pat, idxmap, nullptr, dose, stats, stream);
        tvam_kt_end(stream, TVAM_KT_TILE);
        if (e == hipSuccess) e = tvam_launch_frozen(TVAM_MODE_FWD, kc, t, pat, idxmap, nullptr, dose, nullptr, stream);
        if (e != hipSuccess) return hip_fail(e, "forward launch");
    }
    if (p->desc.albedo != 0.0f) {  // scattered segments (after each path's first medium segment)
        TvamTiles t = p->tiles;
        t.spp = spp;
        t.seed = seed;
        e = hipErrorNotSupported;
        p->bins.acc_float = env_int("TVAM_BIN_FLOAT", 0);
        if (p->desc.flags & TVAM_FLAG_SCATTER_ATOMIC)
            for (auto& v : p->bins.st) v = 0;  // nothing binned
        else
            e = tvam_scatter_binned(TVAM_MODE_FWD, kc, t, pat, idxmap, nullptr, dose, p->bins, stream);
        if (e == hipErrorNotSupported)
            e = tvam_launch_scatter_paths(TVAM_MODE_FWD, kc, t, pat, idxmap, nullptr, dose, nullptr, stream);
        if (e == hipErrorIllegalState) return bin_mismatch_fail(p);
        if (e != hipSuccess) return hip_fail(e, "scatter forward launch");
    }
    return 0;
}

// The planar adjoint of film slices [z_begin, z_end) alone, into the DMD rows [row_begin, row_end) of every
// angle of grad_active (dense crop order; those rows zeroed first, the others untouched): the caller's rows
// are exactly the rows whose rays lie in those slices (tvam_row_slices), so the rows hold their whole
// gradient.  Regular-sampling planar plans of a dense set; slices on the adjoint's Z-slice chunks.
// The planar adjoint's visit lists, built at the plan's first adjoint call when they fit in a
// quarter of the free device memory (else the tile adjoint serves).  16 slices per workgroup where
// the tile's 4 planes fit in LDS, else 8 (the weights are the same; the adjoint's chunk reported
// before the build, max(8, adjl_z), stays a multiple of the one the kernel then runs).
static int ensure_adj_lists(tvam_plan* p) {
    if (!p->adjl_pending) return 0;
    p->adjl_pending = false;
    size_t fr = 0, tot = 0;
    hipError_t e = hipMemGetInfo(&fr, &tot);
    if (e != hipSuccess) return hip_fail(e, "hipMemGetInfo");
    e = tvam_build_adj_lists(p->k, p->pl, p->tiles, p->adjl_parts, fr / 4, p->adjl, nullptr);
    if (e == hipSuccess && p->pl.adjl_z == 16 && tvam_adjl_lds(p->pl, p->tiles, 16) > 160 * 1024) p->pl.adjl_z = 8;
    if (e == hipSuccess && tvam_adjl_lds(p->pl, p->tiles, p->pl.adjl_z) > 160 * 1024) e = hipErrorOutOfMemory;
    if (e != hipSuccess) {
        adjl_free(p->adjl);
        p->pl.adjl_ngroups = 0;
        if (e != hipErrorOutOfMemory) return hip_fail(e, "adjoint visit lists");
        (void)hipGetLastError();
    }
    return 0;
}

extern "C" int tvam_adjoint_slices(tvam_plan* p, const float* grad_dose, uint64_t n_active, int32_t z_begin,
                                   int32_t z_end, int32_t row_begin, int32_t row_end, float* grad_active,
                                   void* stream_) {
    if (!p || !grad_dose || !grad_active) return fail(TVAM_ERR_INVALID, "null argument");
    if (!p->planar || p->general || p->surface || p->desc.albedo != 0.0f || p->empty)
        return fail(TVAM_ERR_UNSUPPORTED, "tvam_adjoint_slices: planar plans only");
    hipStream_t stream = (hipStream_t)stream_;
    TvamConsts k;
    uint32_t spp = 1;
    int rc = call_setup(p, n_active, nullptr, spp, k);
    if (rc) return rc;
    const int Z = p->pl.adjl_ngroups > 0 || p->adjl_pending ? std::max(p->planar_az, p->pl.adjl_z) : p->planar_az,
              nz = k.nz;
    if ((rc = ensure_adj_lists(p))) return rc;
    const int64_t R = k.crop_y, C = k.crop_x, A = (int64_t)p->tiles.n_shard;
    if (z_begin < 0 || z_end > nz || z_begin >= z_end || z_begin % Z != 0 || (z_end % Z != 0 && z_end != nz) ||
        row_begin < 0 || row_end > R || row_begin > row_end || (int64_t)n_active != A * R * C)
        return fail(TVAM_ERR_INVALID, "tvam_adjoint_slices: slices on the adjoint's chunks, rows in the crop, dense set");
    hipError_t e = hipSuccess;
    if (row_end > row_begin)
        e = hipMemset2DAsync(grad_active + (size_t)row_begin * C, (size_t)(R * C) * sizeof(float), 0,
                             (size_t)(row_end - row_begin) * C * sizeof(float), (size_t)A, stream);
    if (e != hipSuccess) return hip_fail(e, "hipMemset2DAsync");
    TvamPlanar pl = p->pl;
    pl.adj_zc0 = z_begin / p->planar_az;  // (in the tile adjoint's chunks; the list adjoint converts)
    pl.adj_nzc = (z_end - z_begin + p->planar_az - 1) / p->planar_az;
    e = tvam_launch_adj_planar(k, pl, p->tiles, p->planar_az, nullptr, grad_dose, grad_active, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "planar adjoint launch");
}

extern "C" int tvam_plan_adj_chunk(const tvam_plan* p) {
    if (!p || !p->planar || p->general || p->surface || p->desc.albedo != 0.0f) return 0;
    return p->pl.adjl_ngroups > 0 || p->adjl_pending ? std::max(p->planar_az, p->pl.adjl_z) : p->planar_az;
}

extern "C" int tvam_adjoint(tvam_plan* p, const float* grad_dose, const uint32_t* active_pixels, uint64_t n_active,
                            uint32_t spp, uint32_t seed, float* grad_active, void* stream_) {
    if (!p || !grad_dose || (!grad_active && n_active)) return fail(TVAM_ERR_INVALID, "null argument");
    hipStream_t stream = (hipStream_t)stream_;
    TvamConsts k;
    int rc = call_setup(p, n_active, active_pixels, spp, k);
    if (rc) return rc;
    hipError_t e;
    if (n_active == 0) return 0;
    const int32_t* idxmap = nullptr;
    if (active_pixels) {
        // dense (angle,row,col) -> active index map; the kernel adds each
        // ray's gradient straight into grad_active[active index]
        if ((rc = ensure_dense(p))) return rc;
        if ((e = hipMemsetAsync(p->d_idxmap, 0xff, p->dense_n * sizeof(int32_t), stream)) != hipSuccess)
            return hip_fail(e, "hipMemsetAsync");
        if ((e = tvam_launch_scatter(k, nullptr, active_pixels, n_active, p->d_dense, p->d_idxmap, stream)) !=
            hipSuccess)
            return hip_fail(e, "scatter launch");
        idxmap = p->d_idxmap;
    }
    if ((rc = ensure_adj_lists(p))) return rc;
    if ((e = hipMemsetAsync(grad_active, 0, n_active * sizeof(float), stream)) != hipSuccess)
        return hip_fail(e, "hipMemsetAsync");
    if (p->general) {
        if (p->empty) return 0;
        TvamTiles t = p->tiles;
        t.spp = spp;
        t.seed = seed;
        e = tvam_launch_general_paths(TVAM_MODE_ADJ, k, t, nullptr, idxmap, grad_dose, grad_active, nullptr, stream);
        return e == hipSuccess ? 0 : hip_fail(e, "path adjoint launch");
    }
    if (p->surface) {
        if (!p->vols) return fail(TVAM_ERR_INVALID, "surface-aware film: call tvam_plan_set_volumes first");
        if (p->empty) return 0;
        TvamTiles t = p->tiles;
        t.spp = spp;
        t.seed = seed;
        e = tvam_launch_surface_paths(TVAM_MODE_ADJ, k, t, nullptr, idxmap, grad_dose, p->vols, grad_active, nullptr,
                                      stream);
        return e == hipSuccess ? 0 : hip_fail(e, "surface-aware adjoint launch");
    }
    if (p->planar) {
        e = tvam_launch_adj_planar(k, p->pl, p->tiles, p->planar_az, idxmap, grad_dose, grad_active, stream);
        if (e != hipSuccess) return hip_fail(e, "planar adjoint launch");
    } else if (!p->empty) {
        TvamTiles t = p->tiles;
        t.spp = spp;
        t.seed = seed;
        if ((rc = ensure_rays(p, k, t, idxmap, stream, active_pixels, n_active))) return rc;
        e = tvam_launch_tiles(TVAM_MODE_ADJ, k, t, p->lds_bytes, nullptr, idxmap, grad_dose, grad_active, nullptr,
                              stream);
        if (e == hipSuccess)
            e = tvam_launch_frozen(TVAM_MODE_ADJ, k, t, nullptr, idxmap, grad_dose, grad_active, nullptr, stream);
        if (e != hipSuccess) return hip_fail(e, "adjoint launch");
    }
    if (p->desc.albedo != 0.0f && !p->empty) {
        TvamTiles t = p->tiles;
        t.spp = spp;
        t.seed = seed;
        e = hipErrorNotSupported;
        if (p->desc.flags & TVAM_FLAG_SCATTER_ATOMIC)
            for (auto& v : p->bins.st) v = 0;  // nothing binned
        else
            e = tvam_scatter_binned(TVAM_MODE_ADJ, k, t, nullptr, idxmap, grad_dose, grad_active, p->bins, stream);
        if (e == hipErrorNotSupported)
            e = tvam_launch_scatter_paths(TVAM_MODE_ADJ, k, t, nullptr, idxmap, grad_dose, grad_active, nullptr, stream);
        if (e == hipErrorIllegalState) return bin_mismatch_fail(p);
        if (e != hipSuccess) return hip_fail(e, "scatter adjoint launch");
    }
    return 0;
}

extern "C" int tvam_count_visits(tvam_plan* p, uint32_t spp, uint32_t seed, uint64_t* visits) {
    if (!p || !visits) return fail(TVAM_ERR_INVALID, "null argument");
    TvamConsts k;
    const tvam_desc& d = p->desc;
    uint64_t n = (uint64_t)(p->k.a1 - p->k.a0) * d.crop_y * d.crop_x;
    int rc = call_setup(p, n, nullptr, spp, k);
    if (rc) return rc;
    *visits = 0;
    if (p->empty) return 0;
    hipError_t e = hipMemset(p->d_counter, 0, sizeof(unsigned long long));
    if (e != hipSuccess) return hip_fail(e, "hipMemset");
    TvamTiles t = p->tiles;
    t.spp = spp;
    t.seed = seed;
    if (p->general) {
        e = tvam_launch_general_paths(TVAM_MODE_COUNT, k, t, nullptr, nullptr, nullptr, nullptr, p->d_counter, nullptr);
    } else if (p->surface) {
        e = tvam_launch_surface_paths(TVAM_MODE_COUNT, k, t, nullptr, nullptr, nullptr, nullptr, nullptr, p->d_counter,
                                      nullptr);
    } else {
        if ((rc = ensure_rays(p, k, t, nullptr, nullptr))) return rc;
        e = tvam_launch_tiles(TVAM_MODE_COUNT, k, t, p->lds_bytes, nullptr, nullptr, nullptr, nullptr, p->d_counter,
                              nullptr);
        if (e == hipSuccess)
            e = tvam_launch_frozen(TVAM_MODE_COUNT, k, t, nullptr, nullptr, nullptr, nullptr, p->d_counter, nullptr);
    }
    if (e != hipSuccess) return hip_fail(e, "count launch");
    if (p->desc.albedo != 0.0f && !p->general && !p->surface) {  // (the surface kernel runs whole paths)
        e = tvam_launch_scatter_paths(TVAM_MODE_COUNT, k, t, nullptr, nullptr, nullptr, nullptr, p->d_counter, nullptr);
        if (e != hipSuccess) return hip_fail(e, "scatter count launch");
    }
    unsigned long long h = 0;
    e = hipMemcpy(&h, p->d_counter, sizeof(h), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpy");
    *visits = h;
    return 0;
}

extern "C" int tvam_radon(tvam_plan* p, const float* target_tris, int32_t n_target_tris, uint32_t spp, uint32_t seed,
                          int32_t max_depth, float* radon, void* stream_) {
    if (!p || !radon || n_target_tris < 0 || (n_target_tris > 0 && !target_tris))
        return fail(TVAM_ERR_INVALID, "null argument");
    const tvam_desc& d = p->desc;
    const uint64_t n = (uint64_t)(p->k.a1 - p->k.a0) * d.crop_y * d.crop_x;
    TvamConsts k;
    int rc = call_setup(p, n, nullptr, spp, k);
    if (rc) return rc;
    hipStream_t stream = (hipStream_t)stream_;
    float* dt = nullptr;
    hipError_t e = hipSuccess;
    if (n_target_tris > 0) {
        const size_t bytes = (size_t)n_target_tris * 9 * sizeof(float);
        if ((e = hipMalloc((void**)&dt, bytes)) != hipSuccess) return hip_fail(e, "hipMalloc (target mesh)");
        if ((e = hipMemcpy(dt, target_tris, bytes, hipMemcpyHostToDevice)) != hipSuccess) {
            (void)hipFree(dt);
            return hip_fail(e, "hipMemcpy (target mesh)");
        }
    }
    // ray weight inv_pdf / n / spp * print_time (projector.py:164-165, common.py:111)
    const float area = d.pixel_size_x * d.pixel_size_y * (float)n;
    const float wray = area / (float)(n * (uint64_t)spp) * d.print_time;
    TvamTiles t = p->tiles;
    t.spp = spp;
    t.seed = seed;
    e = tvam_launch_radon(k, t, dt, n_target_tris, max_depth, wray, radon, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    (void)hipFree(dt);
    return e == hipSuccess ? 0 : hip_fail(e, "radon launch");
}

extern "C" int tvam_compute_volume(tvam_plan* p, uint32_t sample_count, float* volumes, void* stream_) {
    if (!p || !volumes) return fail(TVAM_ERR_INVALID, "null argument");
    if (!p->surface) return fail(TVAM_ERR_INVALID, "compute_volume needs a surface-aware film (film_channels 2)");
    if (sample_count == 0) return fail(TVAM_ERR_INVALID, "sample_count must be positive");
    hipError_t e = hipSetDevice(p->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    hipStream_t stream = (hipStream_t)stream_;
    e = tvam_launch_volumes(p->k, sample_count, volumes, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    return e == hipSuccess ? 0 : hip_fail(e, "compute_volume launch");
}

extern "C" int tvam_plan_set_volumes(tvam_plan* p, const float* volumes) {
    if (!p) return fail(TVAM_ERR_INVALID, "null argument");
    if (!p->surface) return fail(TVAM_ERR_INVALID, "volumes apply to surface-aware films (film_channels 2)");
    p->vols = volumes;
    return 0;
}

extern "C" int tvam_discretize(const tvam_desc* desc, float* occ, void* stream_) {
    if (!desc || !occ) return fail(TVAM_ERR_INVALID, "null argument");
    const tvam_desc& d = *desc;
    if (d.abi_version != TVAM_ABI_VERSION) return fail(TVAM_ERR_INVALID, "tvam_desc.abi_version mismatch");
    if (d.n_target_tris <= 0 || !d.target_tris) return fail(TVAM_ERR_INVALID, "No target shape found in the scene");
    for (int a = 0; a < 3; ++a)
        if (d.film_res[a] <= 0 || !(d.bbox_max[a] > d.bbox_min[a]))
            return fail(TVAM_ERR_INVALID, "film resolution and sensor bbox must be positive");
    if ((int64_t)d.film_res[0] * d.film_res[1] * d.film_res[2] > (int64_t)1 << 32)
        return fail(TVAM_ERR_TOO_LARGE, "discretize: more than 2^32 voxels");
    hipStream_t stream = (hipStream_t)stream_;
    TvamConsts k{};
    for (int a = 0; a < 3; ++a) {
        k.res[a] = d.film_res[a];
        k.bmin[a] = d.bbox_min[a];
        k.h[a] = (d.bbox_max[a] - d.bbox_min[a]) / (float)d.film_res[a];  // utils.py:104
    }
    const size_t nb = (size_t)d.n_target_tris * 9 * sizeof(float);
    float* d_tris = nullptr;
    hipError_t e = hipMalloc((void**)&d_tris, nb);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc");
    e = hipMemcpyAsync(d_tris, d.target_tris, nb, hipMemcpyHostToDevice, stream);
    k.tgt = d_tris;
    k.n_tgt = d.n_target_tris;
    if (e == hipSuccess) e = tvam_launch_discretize(k, d.target_tris, occ, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    (void)hipFree(d_tris);
    return e == hipSuccess ? 0 : hip_fail(e, "discretize launch");
}

extern "C" int tvam_plan_fwd_scale(tvam_plan* p, float* scale) {
    if (!p || !scale) return fail(TVAM_ERR_INVALID, "null argument");
    if (!p->planar || p->planar_fwd)
        return fail(TVAM_ERR_INVALID, "tvam_plan_fwd_scale: this plan's forward is not the ray-driven planar kernel");
    hipError_t e = hipSetDevice(p->device);
    if (e == hipSuccess) e = hipMemcpy(scale, p->d_fscale, 2 * sizeof(float), hipMemcpyDeviceToHost);
    return e == hipSuccess ? 0 : hip_fail(e, "hipMemcpy");
}

// bit 0: planar adjoint (+ ray-driven planar forward unless bit 1), bit 1: voxel-driven planar forward
extern "C" int tvam_plan_path(const tvam_plan* p) { return p ? (p->planar ? 1 : 0) | (p->planar_fwd ? 2 : 0) : 0; }

extern "C" int tvam_plan_stats(tvam_plan* p, uint64_t* fallback_tiles) {
    if (!p || !fallback_tiles) return fail(TVAM_ERR_INVALID, "null argument");
    unsigned long long h = 0;
    hipError_t e = hipMemcpy(&h, p->d_counter, sizeof(h), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpy");
    *fallback_tiles = h;
    return 0;
}

extern "C" int tvam_plan_bin_stats(tvam_plan* p, int64_t* stats) {
    if (!p || !stats) return fail(TVAM_ERR_INVALID, "null argument");
    const TvamBinScratch& b = p->bins;
    for (int i = 0; i < 5; ++i) stats[i] = b.st[i];
    int64_t cache = 0;  // device bytes the forward bin cache holds
    for (const TvamBinChunk& c : b.fc)
        cache += c.cap_slots * TVAM_REC_F4 * (int64_t)sizeof(float4) + (c.cap_vals + c.cap_bricks) * (int64_t)sizeof(uint32_t);
    stats[5] = cache;
    // the chunk scratch: records, brick counts and offsets, sort keys / values, adjoint partials
    stats[6] = b.cap_slots * (TVAM_REC_F4 * (int64_t)sizeof(float4) + 2 * (int64_t)sizeof(uint32_t)) +
               b.cap_entries * (int64_t)(4 * sizeof(uint32_t) + sizeof(float)) + b.cap_bricks * 4 + b.temp_cap();
    // slots whose bin-fill walk disagreed with the record writer's closed-form brick count
    // (sc_brick_count; 0 by construction, checked by the tests), summed over the calls since the
    // chunk scratch was allocated
    stats[7] = 0;
    if (b.sb.bad) {
        uint32_t bad = 0;
        if (hipMemcpy(&bad, b.sb.bad, sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
            return fail(TVAM_ERR_HIP, "tvam_plan_bin_stats: reading the count check");
        stats[7] = bad;
    }
    return 0;
}

// The per-ray tile kernels' row walks for the plan's most recent ray records (jittered plans):
// how many rays the ray setup listed as strays (rays outside their row's main slice) and what
// the (tile, slice) workgroups walk because of them -- every workgroup of a slice walks that
// slice's whole stray list, against its main rows' slots.
extern "C" int tvam_plan_tile_stats(tvam_plan* p, int64_t* stats) {
    if (!p || !stats) return fail(TVAM_ERR_INVALID, "null argument");
    for (int i = 0; i < 8; ++i) stats[i] = 0;
    stats[0] = -1;
    const tvam_plan::RaySlot* r = nullptr;
    for (const auto& s : p->rs)
        if (s.valid && (!r || s.used > r->used)) r = &s;
    if (!r) return 0;
    unsigned long long ns = 0, nf = 0;
    hipError_t e = hipSuccess;
    if (r->stray_n && p->n_main_rows > 0) e = hipMemcpy(&ns, r->stray_n, sizeof(ns), hipMemcpyDeviceToHost);
    if (e == hipSuccess && r->frozen_n) e = hipMemcpy(&nf, r->frozen_n, sizeof(nf), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpy");
    const bool lists = r->stray_n && p->n_main_rows > 0;
    stats[0] = lists ? (int64_t)ns : -1;
    stats[1] = lists ? (int64_t)TVAM_STRAY_CAP : 0;
    // strays beyond the cap: the workgroups walk the full row lists instead (no stray walk)
    const bool used = lists && ns <= (unsigned long long)TVAM_STRAY_CAP;
    stats[2] = used ? (int64_t)ns * p->ntiles : 0;
    stats[3] = (used ? p->n_main_rows : p->n_rows_all) * p->n_slots_all * (int64_t)r->spp;
    stats[4] = (int64_t)nf;
    stats[5] = (int64_t)r->spp;
    stats[6] = p->ntiles;
    stats[7] = p->n_slots_all;
    return 0;
}

extern "C" int tvam_plan_kernel_time(tvam_plan* p, int32_t enable, double* total_ms, int64_t* launches) {
    if (!p || !total_ms || !launches) return fail(TVAM_ERR_INVALID, "null argument");
    *total_ms = 0.0;
    *launches = 0;
    std::lock_guard<std::mutex> lk(g_kt.mu);
    if (g_kt.owner && g_kt.owner != p) return fail(TVAM_ERR_INVALID, "tvam_plan_kernel_time: another plan owns the timer");
    hipError_t e = hipSuccess;
    for (size_t i = 0; e == hipSuccess && i < g_kt.n; i += 2) {  // each pair's end complete before it is read
        float ms = 0.0f;
        e = hipEventSynchronize(g_kt.ev[i + 1]);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, g_kt.ev[i], g_kt.ev[i + 1]);
        *total_ms += ms;
    }
    *launches = (int64_t)(g_kt.n / 2);
    if (e != hipSuccess) return hip_fail(e, "tvam_plan_kernel_time");
    g_kt.n = 0;
    g_kt.on = false;
    if (!enable) {  // measurement read: the events go with it
        kt_release();
        return 0;
    }
    {
        g_kt.owner = p;
        g_kt.device = p->device;
        while (g_kt.ev.size() < 2048) {
            hipEvent_t ev;
            if ((e = hipEventCreate(&ev)) != hipSuccess) return hip_fail(e, "hipEventCreate");
            g_kt.ev.push_back(ev);
        }
        // the plan's dominant forward kernel: the brick march of a scattering medium, else the
        // voxel-driven planar forward where it serves, else the per-ray tile forward
        g_kt.kind = p->desc.albedo != 0.0f ? TVAM_KT_BRICK : (p->planar_fwd ? TVAM_KT_PLANAR : TVAM_KT_TILE);
        g_kt.on = true;
    }
    return 0;
}

extern "C" int tvam_loss_threshold(const float* dose, const float* ddose, float alpha, const float* target, uint64_t n,
                                   int32_t K, float tl, float tu, float w_object, float w_void, float w_limit,
                                   float scale, double* out, float* grad, void* stream) {
    if (!dose || !target || !out) return fail(TVAM_ERR_INVALID, "null argument");
    if (K < 1 || K > 16) return fail(TVAM_ERR_UNSUPPORTED, "ThresholdedLoss: integer K in [1, 16] required on the GPU path");
    hipError_t e = tvam_launch_loss_threshold(dose, ddose, alpha, target, nullptr, 0, n, K, tl, tu, w_object, w_void,
                                              w_limit, scale, out, grad, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "loss launch");
}

extern "C" int tvam_target_mask(const float* target, uint64_t n, uint32_t* mask, void* stream) {
    if (!target || !mask) return fail(TVAM_ERR_INVALID, "null argument");
    hipError_t e = tvam_launch_target_mask(target, n, mask, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "target mask launch");
}

extern "C" int tvam_loss_threshold_mask(const float* dose, const float* ddose, float alpha, const uint32_t* mask,
                                        uint64_t mask_bit0, uint64_t n, int32_t K, float tl, float tu, float w_object,
                                        float w_void, float w_limit, float scale, double* out, float* grad,
                                        void* stream) {
    if (!dose || !mask || !out) return fail(TVAM_ERR_INVALID, "null argument");
    if (K < 1 || K > 16) return fail(TVAM_ERR_UNSUPPORTED, "ThresholdedLoss: integer K in [1, 16] required on the GPU path");
    hipError_t e = tvam_launch_loss_threshold(dose, ddose, alpha, nullptr, mask, mask_bit0, n, K, tl, tu, w_object,
                                              w_void, w_limit, scale, out, grad, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "loss launch");
}

extern "C" int tvam_loss_threshold_probes_mask(const float* dose, const float* ddose, const float* alphas,
                                               int32_t n_alpha, const uint32_t* mask, uint64_t mask_bit0, uint64_t n,
                                               int32_t K, float tl, float tu, float w_object, float w_void,
                                               float w_limit, float scale, double* out, void* stream) {
    if (!dose || !ddose || !alphas || !mask || !out) return fail(TVAM_ERR_INVALID, "null argument");
    if (n_alpha < 1 || n_alpha > TVAM_MAX_PROBES)
        return fail(TVAM_ERR_INVALID, "tvam_loss_threshold_probes_mask: 1 <= n_alpha <= 8");
    if (K < 1 || K > 16) return fail(TVAM_ERR_UNSUPPORTED, "ThresholdedLoss: integer K in [1, 16] required on the GPU path");
    hipError_t e = tvam_launch_loss_probes(dose, ddose, alphas, n_alpha, nullptr, mask, mask_bit0, n, K, tl, tu,
                                           w_object, w_void, w_limit, scale, out, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "loss probes launch");
}

extern "C" int tvam_loss_threshold_probes(const float* dose, const float* ddose, const float* alphas, int32_t n_alpha,
                                          const float* target, uint64_t n, int32_t K, float tl, float tu,
                                          float w_object, float w_void, float w_limit, float scale, double* out,
                                          void* stream) {
    if (!dose || !ddose || !alphas || !target || !out) return fail(TVAM_ERR_INVALID, "null argument");
    if (n_alpha < 1 || n_alpha > TVAM_MAX_PROBES) return fail(TVAM_ERR_INVALID, "tvam_loss_threshold_probes: 1 <= n_alpha <= 8");
    if (K < 1 || K > 16) return fail(TVAM_ERR_UNSUPPORTED, "ThresholdedLoss: integer K in [1, 16] required on the GPU path");
    hipError_t e = tvam_launch_loss_probes(dose, ddose, alphas, n_alpha, target, nullptr, 0, n, K, tl, tu, w_object,
                                           w_void, w_limit, scale, out, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "loss probes launch");
}

static bool aligned16(const void* q) { return ((uintptr_t)q & 15u) == 0; }

extern "C" int tvam_lbfgs_history(uint64_t n, const float* p, const float* p_old, const float* g, const float* g_old,
                                  int32_t h, const float* const* S, const float* const* Y, float* s_new,
                                  float* y_new, double* work, double* dots, void* stream) {
    if (!g || !work || !dots || (h > 0 && (!S || !Y))) return fail(TVAM_ERR_INVALID, "null argument");
    if (h < 0 || h > 7) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_history: 0 <= h <= 7 retained pairs");
    if (p_old && (!p || !g_old || !s_new || !y_new)) return fail(TVAM_ERR_INVALID, "null argument");
    // p_old NULL with g_old given: a new pair whose s_new already holds p - p_old (read, not written)
    const bool spre = !p_old && g_old;
    if (spre && (!s_new || !y_new)) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_history: precomputed s_new needs s_new, y_new");
    bool ok = aligned16(g) && (!p_old || (aligned16(p) && aligned16(p_old) && aligned16(g_old) &&
                                          aligned16(s_new) && aligned16(y_new))) &&
              (!spre || (aligned16(g_old) && aligned16(s_new) && aligned16(y_new)));
    for (int j = 0; j < h; ++j) ok = ok && S[j] && Y[j] && aligned16(S[j]) && aligned16(Y[j]);
    if (!ok) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_history: vectors must be 16-byte aligned");
    hipError_t e = tvam_launch_lbfgs_history(n, p, p_old, g, g_old, h, S, Y, s_new, y_new, work, dots,
                                             (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "lbfgs history launch");
}

extern "C" int tvam_lbfgs_history_rows(uint64_t nseg, uint64_t seg_len, uint64_t seg_stride, uint64_t seg_off,
                                       const float* p, const float* p_old, const float* g, const float* g_old,
                                       int32_t h, const float* const* S, const float* const* Y, float* s_new,
                                       float* y_new, double* work, double* dots, void* stream) {
    if (!g || !work || !dots || (h > 0 && (!S || !Y))) return fail(TVAM_ERR_INVALID, "null argument");
    if (h < 0 || h > 7) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_history_rows: 0 <= h <= 7 retained pairs");
    if (p_old && (!p || !g_old || !s_new || !y_new)) return fail(TVAM_ERR_INVALID, "null argument");
    if (!p_old && g_old) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_history_rows: g_old without p_old");
    if (nseg == 0 || seg_len == 0 || seg_len % 4 || seg_stride % 4 || seg_off % 4 || seg_len > seg_stride ||
        seg_len / 4 > 0xffffffffull)
        return fail(TVAM_ERR_INVALID, "tvam_lbfgs_history_rows: segments of a multiple of 4 entries, 4-aligned");
    bool ok = aligned16(g) && (!p_old || (aligned16(p) && aligned16(p_old) && aligned16(g_old) &&
                                          aligned16(s_new) && aligned16(y_new)));
    for (int j = 0; j < h; ++j) ok = ok && S[j] && Y[j] && aligned16(S[j]) && aligned16(Y[j]);
    if (!ok) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_history_rows: vectors must be 16-byte aligned");
    hipError_t e = tvam_launch_lbfgs_history(0, p, p_old, g, g_old, h, S, Y, s_new, y_new, work, dots,
                                             (hipStream_t)stream, nseg, seg_len, seg_stride, seg_off);
    return e == hipSuccess ? 0 : hip_fail(e, "lbfgs history launch");
}

extern "C" int tvam_lbfgs_direction(uint64_t n, const float* g, int32_t h, const float* const* S,
                                    const float* const* Y, float cg, const float* cs, const float* cy, float* d,
                                    void* stream) {
    if (!g || !d || (h > 0 && (!S || !Y || !cs || !cy))) return fail(TVAM_ERR_INVALID, "null argument");
    if (h < 0 || h > 8) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_direction: 0 <= h <= 8 pairs");
    bool ok = aligned16(g) && aligned16(d);
    for (int j = 0; j < h; ++j) ok = ok && S[j] && Y[j] && aligned16(S[j]) && aligned16(Y[j]);
    if (!ok) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_direction: vectors must be 16-byte aligned");
    hipError_t e = tvam_launch_lbfgs_direction(n, g, h, S, Y, cg, cs, cy, d, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "lbfgs direction launch");
}

extern "C" int tvam_lbfgs_coef(int32_t h, int32_t is_new, int32_t first, const int32_t* order, const double* dots,
                               double* gram, float* coef, double* gdz, void* stream) {
    if (h < 0 || h > 8) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_coef: 0 <= h <= 8 pairs");
    if (!dots || !gram || !coef || !gdz || (h > 0 && !order)) return fail(TVAM_ERR_INVALID, "null argument");
    if (is_new && h == 0) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_coef: a new pair needs h >= 1");
    for (int j = 0; j < h; ++j)
        if (order[j] < 0 || order[j] >= 8) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_coef: ring slots are 0..7");
    hipError_t e = tvam_launch_lbfgs_coef(h, is_new ? 1 : 0, first ? 1 : 0, order, dots, gram, coef, gdz,
                                          (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "lbfgs coefficient launch");
}

extern "C" int tvam_lbfgs_direction_dev(uint64_t n, const float* g, int32_t h, const float* const* S,
                                        const float* const* Y, const float* coef, float* d, void* stream) {
    if (!g || !d || !coef || (h > 0 && (!S || !Y))) return fail(TVAM_ERR_INVALID, "null argument");
    if (h < 0 || h > 8) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_direction_dev: 0 <= h <= 8 pairs");
    bool ok = aligned16(g) && aligned16(d);
    for (int j = 0; j < h; ++j) ok = ok && S[j] && Y[j] && aligned16(S[j]) && aligned16(Y[j]);
    if (!ok) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_direction_dev: vectors must be 16-byte aligned");
    hipError_t e = tvam_launch_lbfgs_direction_dev(n, g, h, S, Y, coef, d, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "lbfgs direction launch");
}

extern "C" int tvam_lbfgs_direction_rows(uint64_t nseg, uint64_t seg_len, uint64_t seg_stride, uint64_t seg_off,
                                         const float* g, int32_t h, const float* const* S, const float* const* Y,
                                         const float* coef, float* d, void* stream) {
    if (!g || !d || !coef || (h > 0 && (!S || !Y))) return fail(TVAM_ERR_INVALID, "null argument");
    if (h < 0 || h > 8) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_direction_rows: 0 <= h <= 8 pairs");
    if (nseg == 0 || seg_len == 0 || seg_len % 4 || seg_stride % 4 || seg_off % 4 || seg_len > seg_stride ||
        seg_len / 4 > 0xffffffffull)
        return fail(TVAM_ERR_INVALID, "tvam_lbfgs_direction_rows: segments of a multiple of 4 entries, 4-aligned");
    bool ok = aligned16(g) && aligned16(d);
    for (int j = 0; j < h; ++j) ok = ok && S[j] && Y[j] && aligned16(S[j]) && aligned16(Y[j]);
    if (!ok) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_direction_rows: vectors must be 16-byte aligned");
    hipError_t e = tvam_launch_lbfgs_direction_dev(0, g, h, S, Y, coef, d, (hipStream_t)stream, nseg, seg_len,
                                                   seg_stride, seg_off);
    return e == hipSuccess ? 0 : hip_fail(e, "lbfgs direction launch");
}

extern "C" int tvam_axpy_clamp(uint64_t n, const float* p, float alpha, const float* d, float lo, float* out,
                               void* stream) {
    if (!p || !d || !out) return fail(TVAM_ERR_INVALID, "null argument");
    if (!aligned16(p) || !aligned16(d) || !aligned16(out))
        return fail(TVAM_ERR_INVALID, "tvam_axpy_clamp: vectors must be 16-byte aligned");
    hipError_t e = tvam_launch_axpy_clamp(n, p, alpha, d, lo, out, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "axpy launch");
}

extern "C" int tvam_axpy_clamp_dev(uint64_t n, const float* p, const float* alpha, const float* d, float lo,
                                   float* out, float* s_out, void* stream) {
    if (!p || !alpha || !d || !out) return fail(TVAM_ERR_INVALID, "null argument");
    if (!aligned16(p) || !aligned16(d) || !aligned16(out) || (s_out && !aligned16(s_out)))
        return fail(TVAM_ERR_INVALID, "tvam_axpy_clamp_dev: vectors must be 16-byte aligned");
    if (s_out && (s_out == p || s_out == out || s_out == d))
        return fail(TVAM_ERR_INVALID, "tvam_axpy_clamp_dev: s_out must not alias p, d or out");
    hipError_t e = tvam_launch_axpy_clamp(n, p, 0.0f, d, lo, out, (hipStream_t)stream, alpha, s_out);
    return e == hipSuccess ? 0 : hip_fail(e, "axpy launch");
}

extern "C" int tvam_lbfgs_armijo(int32_t nprobe, double alpha0, const double* probes, const double* loss_dev,
                                 double loss_host, double loss_div, const double* gdz, double c1, float* alpha,
                                 double* report, void* stream) {
    if (!probes || !gdz || !alpha) return fail(TVAM_ERR_INVALID, "null argument");
    if (nprobe < 1 || nprobe > 64) return fail(TVAM_ERR_INVALID, "tvam_lbfgs_armijo: 1 <= nprobe <= 64");
    if (!(alpha0 > 0.0) || !(loss_div > 0.0))
        return fail(TVAM_ERR_INVALID, "tvam_lbfgs_armijo: alpha0 and loss_div must be positive");
    hipError_t e = tvam_launch_armijo(nprobe, alpha0, probes, loss_dev, loss_host, loss_div, gdz, c1, alpha, report,
                                      (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "armijo launch");
}

extern "C" int tvam_row_slices(const tvam_desc* desc, int32_t* slice_of_row) {
    if (!desc || !slice_of_row) return fail(TVAM_ERR_INVALID, "null argument");
    int rc = validate(*desc);
    if (rc) return rc;
    const tvam_desc& d = *desc;
    const TvamConsts k = make_consts(d, 0, d.n_patterns);
    for (int r = 0; r < d.crop_y; ++r) {
        float xc, yc;
        tvam_ray_camera(k, 0, d.crop_offset_y + r, 0.5f, 0.5f, xc, yc);
        const int s = tvam_slice_of(k, yc);
        slice_of_row[r] = (s >= 0 && yc >= -k.vial_half_h && yc <= k.vial_half_h) ? s : -1;
    }
    return 0;
}
