// tvam_kernels.hip — gfx950 kernels of the TVAM projection engine.
//
// Hot path: the DDA ray march of DDAVolumetricSensor.accumulate
// (sensor.py:383-438) for every ray of every projector angle.
//
// Design (MI355X-first):
//  * Collimated rays under circular motion around a vertical vial are planar
//    (d.z == 0), so every ray stays in ONE z-slice of the film.  A workgroup
//    owns one (z-slice, xy-tile) pair and keeps that tile resident in LDS.
//  * Forward: every ray crossing the tile marches only its in-tile part and
//    accumulates exp(-st t)(1 - exp(-st dt)) * Le into LDS with ds_add_f32;
//    the tile is written to HBM once with coalesced stores (no global
//    atomics, no pre-zeroing of the film).
//  * Adjoint: the workgroup stages dL/dD * inv_vol for its tile in LDS, each
//    ray gathers its in-tile sum from LDS and adds it to its pattern gradient
//    with one coalesced global float atomic per (ray, tile).
//  * The march is resumed at the tile entry in closed form: the reference
//    DDA steps axis a at t_start + dtm0[a] + n*ts[a], so the voxel index and
//    dtmax at any time follow without marching the skipped part.
#include "tvam_internal.h"

#define TVAM_BLOCK 256
#define TVAM_WAVES (TVAM_BLOCK / 64)


__device__ __forceinline__ float tvam_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// floor(x + 0.5) in one instruction (round to nearest, ties up).
__device__ __forceinline__ int tvam_rint(float x) {
    int r;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// How the in-tile march consumes one visit.
enum TvamAcc { ACC_FLOAT = 0, ACC_FIXED = 1, ACC_GATHER = 2, ACC_COUNT = 3 };



// March state of one ray inside one tile (times measured from the tile entry).
struct TvamMarchRay {
    char* pv;        // LDS address of the current voxel
    float Tx, Ty;    // next x / y boundary crossing
    float rem;       // in-tile exit: tile exit or segment end, whichever is first
    float stop;      // rem - 1e-6: the reference's "remaining <= 1e-6" end test (sensor.py:427)
    float nt0;       // -st * log2(e) * (distance travelled at the tile entry)
    float e0;        // em * exp(-st * t) at the tile entry
    float ems;       // em, pre-scaled for the accumulator
};

// In-tile DDA march (sensor.py:383-438) from a resumed state.  The march
// tracks the NEXT x / y boundary crossing and the in-tile exit, so a visit is
// [tp, tn = min(Tx, Ty, rem)] and one test ends the ray.  The reference
// decrements per-axis countdowns by dt instead; both are the same DDA up to
// fp32 rounding of the step times.  One axis steps per visit: on an exact tie
// the other axis steps on the next visit, whose dt is exactly 0 (c == 0), i.e.
// the reference's diagonal step.  Rounding can let the last step cross the
// tile edge one visit early; the tile carries a 1-voxel guard band that
// absorbs that visit (its dt is at rounding level, and guard cells are never
// stored / read as 0).  Visit weight e0 (1 - e^{-st dt}) from the tile-relative
// dt = tn - tp (tvam_omexp: no cancellation), then e0 *= e^{-st dt} (= e0 - c);
// e0 restarts exactly from exp2 at every tile entry.
// W2 (plans with st * voxel diagonal < TVAM_W2_MAX): e0 carries st e^{-st t} and a visit costs
// c = e0 dt (1 - st dt / 2), e0 -= st c (the planar kernels' form; five full-rate instructions
// in place of the degree-4 polynomial, its range test and the cancellation-free product).
template <int ACC, bool W2 = false>
__device__ __forceinline__ void tvam_march(TvamMarchRay a, const float tsx, const float tsy, const int sxb,
                                           const int syb, const float sig, float& acc,
                                           unsigned long long& nvis, const char* tile = nullptr, const int tw = 0,
                                           const int wx = 0, const int wy = 0) {
    constexpr int ESZ = 4;
    const float mhs = -0.5f * sig, msig = -sig;
    float tp = 0.0f;
    for (;;) {
        const float tn = fminf(fminf(a.Tx, a.Ty), a.rem);
        // tn never decreases (the crossings only grow, tp starts at the clamped tile entry 0)
        const float dt = tn - tp;
        const float c = W2 ? a.e0 * dt * fmaf(mhs, dt, 1.0f) : a.e0 * tvam_omexp(sig * fmaxf(dt, 0.0f));
        const float e1 = W2 ? fmaf(msig, c, a.e0) : a.e0 - c;
        if (ACC == ACC_FLOAT) atomicAdd(reinterpret_cast<float*>(a.pv), c);
        else if (ACC == ACC_FIXED) atomicAdd(reinterpret_cast<int*>(a.pv), tvam_rint(c));
        else if (ACC == ACC_GATHER) acc = fmaf(c, *reinterpret_cast<const float*>(a.pv), acc);
        else {  // interior visits of nonzero length (guard-band visits carry rounding-level dt)
            const int li = (int)(a.pv - tile) / ESZ, ly = li / tw, lx = li - ly * tw;
            nvis += (tn > tp && lx >= 1 && lx <= wx && ly >= 1 && ly <= wy) ? 1 : 0;
        }
        tp = tn;
        const bool mx = a.Tx <= a.Ty;
        a.Tx = mx ? a.Tx + tsx : a.Tx;
        a.Ty = mx ? a.Ty : a.Ty + tsy;
        a.pv += mx ? sxb : syb;
        a.e0 = e1;
        if (!(tn < a.stop)) break;
    }
}

// Ray slot enumeration of one workgroup: slot f -> (slice row ri, entry g of
// the tile's slot list, sample smp).  Slots advance by the block size, so
// (ri, rrem) are updated incrementally.
struct TvamSlot {
    int ri, rrem;
};

__device__ __forceinline__ void tvam_slot_init(TvamSlot& sl, int f, int per_row) {
    sl.ri = f / per_row;
    sl.rrem = f - sl.ri * per_row;
}

__device__ __forceinline__ void tvam_slot_next(TvamSlot& sl, int per_row, int step = TVAM_BLOCK) {
    sl.rrem += step;
    while (sl.rrem >= per_row) {
        sl.rrem -= per_row;
        ++sl.ri;
    }
}

// Everything of one ray inside one tile.
struct TvamTileRay {
    int64_t local, act;
    int lidx, sx, sy;
    float t, rem, dtx, dty, tsx, tsy;
    float weight;  // interfaces' transmission weight (refracting vials; 1 otherwise)
    int why;       // diagnostic builds: why the ray does not reach the tile (1 inactive, 2 slice, 3 window)
};

// Appends this wave's stray rays (s: the lane's ray lies outside its row's main slice zl) to the
// stray list with one atomic per wave, and adds the per-slice counts with one atomic per distinct
// slice among them (a wave's lanes are neighbouring pixels of one row, so its strays share one or
// two slices) instead of one per stray on the single list counter (no measurable change on
// config 5, whose strays are few).  List order is the atomics' (the tile kernels' sums ignore it).
__device__ __forceinline__ void tvam_append_strays(const TvamTiles& tp, bool s, int zl, uint32_t idx) {
    const unsigned long long m = __ballot(s);
    if (m == 0) return;
    const int lane = (int)__lane_id(), leader = __ffsll((long long)m) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(tp.stray_n, (unsigned long long)__popcll(m));
    base = ((unsigned long long)(unsigned)__shfl((int)(base >> 32), leader, 64) << 32) |
           (unsigned long long)(unsigned)__shfl((int)(unsigned)base, leader, 64);
    const unsigned long long j = base + (unsigned long long)__popcll(m & ((1ull << lane) - 1ull));
    const bool kept = s && j < (unsigned long long)tp.stray_cap;
    if (kept) tp.stray_idx[j] = idx;
    unsigned long long left = __ballot(kept);
    while (left) {  // per-slice counts of the kept strays
        const int l0 = __ffsll((long long)left) - 1;
        const int z0 = __shfl(zl, l0, 64);
        const unsigned long long same = __ballot(kept && zl == z0) & left;
        if (lane == l0) atomicAdd(&tp.stray_cnt[z0], (unsigned)__popcll(same));
        left &= ~same;
    }
}

// Ray record pre-pass (one thread per ray of the shard): ray generation
// (common.py:81-108), index-matched vial segment (volume.py:179-216) and DDA
// initialisation (sensor.py:327-365).  Record index = sample * n_local + local.
__global__ __launch_bounds__(256) void tvam_ray_setup_kernel(TvamConsts k, TvamTiles tp, float4* __restrict__ ray_f,
                                                             int2* __restrict__ ray_i, float4* __restrict__ ray_g,
                                                             const int32_t* __restrict__ idxmap) {
    const int spp = (int)tp.spp;
    const int64_t per_angle = (int64_t)k.crop_y * k.crop_x;
    const int64_t n_local = (int64_t)tp.n_shard * per_angle;
    const int64_t n = n_local * spp;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        // record i = smp * n_local + local (sample-major: the tile kernels' lanes, which enumerate
        // the sample slowest, read consecutive records of neighbouring pixels)
        int smp, al, rowc, colc;
        int64_t local;
        if (n <= (int64_t)0xffffffff) {  // 32-bit index arithmetic (a 64-bit division is ~3x the code)
            const uint32_t ii = (uint32_t)i, nl = (uint32_t)n_local, pa = (uint32_t)per_angle, cx = (uint32_t)k.crop_x;
            const uint32_t s32 = ii / nl, l32 = ii - s32 * nl, a32 = l32 / pa, p32 = l32 - a32 * pa, r32 = p32 / cx;
            smp = (int)s32;
            local = (int64_t)l32;
            al = (int)a32;
            rowc = (int)r32;
            colc = (int)(p32 - r32 * cx);
        } else {
            smp = (int)(i / n_local);
            local = i - (int64_t)smp * n_local;
            al = (int)(local / per_angle);
            const int64_t pix = local - (int64_t)al * per_angle;
            rowc = (int)(pix / k.crop_x);
            colc = (int)(pix - (int64_t)rowc * k.crop_x);
        }
        float jx = 0.5f, jy = 0.5f;
        if (!k.regular) {
            TvamPcg rng;
            rng.seed(tp.seed, tvam_stream(k, idxmap, local, (uint32_t)spp, smp));
            jx = rng.next_float();
            jy = rng.next_float();
        }
        const float2 csv = tp.cs[al];
        float xc, yc, ox, oy, oz, dx, dy;
        tvam_ray_camera(k, k.crop_off_x + colc, k.crop_off_y + rowc, jx, jy, xc, yc);
        tvam_ray_world(k, csv.x, csv.y, xc, yc, ox, oy, oz, dx, dy);
        int slice = tvam_slice_of(k, oz);
        float o2x, o2y, d2x, d2y, maxt, wgt;
        TvamDda q;
        if (slice < 0 || !tvam_segment(k, ox, oy, oz, dx, dy, o2x, o2y, d2x, d2y, maxt, wgt) ||
            !tvam_dda_init(k, o2x, o2y, d2x, d2y, maxt, q)) {
            ray_f[i] = make_float4(0.0f, -1.0f, 0.0f, 0.0f);
            ray_i[i] = make_int2(0, -1);
            if (ray_g) ray_g[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            continue;
        }
        ray_f[i] = make_float4(q.t_start, q.tau_end, q.dtm0[0], q.dtm0[1]);
        // an axis that moves but whose first crossing rounded negative never steps (sensor.py:358):
        // the ray leaves its chord, so tvam_frozen_kernel marches it instead of the tile kernels
        const bool frozen = (fabsf(d2x) > 1e-8f && !(q.dtm0[0] < TVAM_INF)) ||
                            (fabsf(d2y) > 1e-8f && !(q.dtm0[1] < TVAM_INF));
        ray_i[i] = make_int2(q.sv[0] | (q.sv[1] << 16), frozen ? -2 - slice : slice);
        if (frozen && tp.frozen) {
            const unsigned long long j = atomicAdd(tp.frozen_n, 1ull);
            if ((int64_t)j < tp.frozen_cap) tp.frozen[j] = i;
        }
        bool stray = false;
        const int zl = slice - k.z0;
        if (tp.row_main && !frozen) {  // a ray outside its row's main slice (TvamTiles::slice_moff)
            stray = zl >= 0 && zl < k.nz && zl != tp.row_main[rowc];
        }
        if (ray_g)
            ray_g[i] = make_float4(q.step[0] > 0 ? q.ts[0] : -q.ts[0], q.step[1] > 0 ? q.ts[1] : -q.ts[1], wgt, 0.0f);
        if (tp.row_main) tvam_append_strays(tp, stray, zl, (uint32_t)i);
    }
}

hipError_t tvam_launch_ray_setup(const TvamConsts& k, const TvamTiles& t, float4* ray_f, int2* ray_i,
                                 float4* ray_g, const int32_t* idxmap, hipStream_t stream) {
    const int64_t n = (int64_t)t.n_shard * k.crop_y * k.crop_x * t.spp;
    int64_t g = (n + 255) / 256;
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(tvam_ray_setup_kernel, dim3((unsigned)g), dim3(256), 0, stream, k, t, ray_f, ray_i, ray_g, idxmap);
    return hipGetLastError();
}

// Stray rays by slice (one workgroup): offsets from the ray setup's counts, then every stray
// record index into its slice's range (order inside a slice: atomic; the tile kernels' sums do
// not depend on it).  Beyond stray_cap the lists stay unused (the tile kernels test stray_n).
__global__ __launch_bounds__(1024) void tvam_stray_lists_kernel(TvamTiles tp, int nz, int z0) {
    __shared__ uint32_t s_part[1024];
    const unsigned long long n_all = *tp.stray_n;
    if (n_all > tp.stray_cap) return;
    const int n = (int)n_all;
    // exclusive scan of stray_cnt[0, nz): per-thread chunks, then the chunk totals
    const int per = (nz + 1023) / 1024, b = (int)threadIdx.x * per;
    uint32_t sum = 0;
    for (int z = b; z < min(b + per, nz); ++z) sum += tp.stray_cnt[z];
    s_part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int t = 0; t < 1024; ++t) {
            const uint32_t v = s_part[t];
            s_part[t] = acc;
            acc += v;
        }
    }
    __syncthreads();
    uint32_t acc = s_part[threadIdx.x];
    for (int z = b; z < min(b + per, nz); ++z) {
        const uint32_t c = tp.stray_cnt[z];
        tp.stray_off[z] = acc;
        tp.stray_cnt[z] = 0;  // the fill's cursor
        acc += c;
    }
    if (b < nz && b + per >= nz) tp.stray_off[nz] = acc;
    if (nz == 0 && threadIdx.x == 0) tp.stray_off[0] = 0;
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += 1024) {
        const uint32_t i = tp.stray_idx[j];
        const int zl = tp.ray_i[i].y - z0;
        const uint32_t pos = atomicAdd(&tp.stray_cnt[zl], 1u);
        tp.stray_list[tp.stray_off[zl] + pos] = i;
    }
}

hipError_t tvam_launch_stray_lists(const TvamConsts& k, const TvamTiles& t, hipStream_t stream) {
    hipLaunchKernelGGL(tvam_stray_lists_kernel, dim3(1), dim3(1024), 0, stream, t, k.nz, k.z0);
    return hipGetLastError();
}

// Resume one ray (pre-computed record) at the tile entry, in closed form of
// the reference march.  Returns false when the ray does not reach the tile.
__device__ __forceinline__ bool tvam_tile_ray(const TvamConsts& k, const TvamTiles& tp, int kz, int x0, int x1, int y0,
                                              int y1, int rowc, int al, int colc, int smp,
                                              const int32_t* __restrict__ idxmap, TvamTileRay& r) {
    r.local = ((int64_t)(k.a0 + al) * k.crop_y + rowc) * k.crop_x + colc - k.shard_base;
    r.act = r.local;
    if (idxmap) {
        r.act = idxmap[r.local];
        r.why = 1;
        if (r.act < 0) return false;  // inactive pixel
    }
    const int64_t ri = (int64_t)smp * ((int64_t)tp.n_shard * k.crop_y * k.crop_x) + r.local;  // sample-major records
    const int2 ii = tp.ray_i[ri];
    r.why = 2;
    if (ii.y != kz + k.z0) return false;  // misses the grid / vial, or lies in another z-slice
    const float4 ff = tp.ray_f[ri];
    float4 an;
    r.weight = 1.0f;
    if (tp.ray_g) {  // refracted ray: its own direction (signed step times) and weight
        const float4 gg = tp.ray_g[ri];
        an = make_float4(fabsf(gg.x), fabsf(gg.y), gg.x < 0.0f ? -1.0f : 1.0f, gg.y < 0.0f ? -1.0f : 1.0f);
        r.weight = gg.z;
    } else {
        an = tp.ang[al];
    }
    const int svx = ii.x & 0xffff, svy = ii.x >> 16;
    const int stx = (int)an.z, sty = (int)an.w;
    float tin0, tout0, tin1, tout1;
    int nin0, nout0, nin1, nout1;
    tvam_axis_window(svx, stx, ff.z, an.x, x0, x1, tin0, tout0, nin0, nout0);
    tvam_axis_window(svy, sty, ff.w, an.y, y0, y1, tin1, tout1, nin1, nout1);
    const float tau_e = fmaxf(fmaxf(tin0, tin1), 0.0f);
    const float tau_x = fminf(fminf(tout0, tout1), ff.y);
    r.why = 3;
    if (!(tau_e < tau_x)) return false;
    const int n0 = tvam_axis_steps(tau_e, ff.z, an.x, nin0, nout0);
    const int n1 = tvam_axis_steps(tau_e, ff.w, an.y, nin1, nout1);
    const int vx = svx + stx * n0;
    const int vy = svy + sty * n1;
    r.dtx = ff.z < TVAM_INF ? fmaxf(fmaf((float)n0, an.x, ff.z) - tau_e, 0.0f) : TVAM_INF;
    r.dty = ff.w < TVAM_INF ? fmaxf(fmaf((float)n1, an.y, ff.w) - tau_e, 0.0f) : TVAM_INF;
    r.tsx = an.x;
    r.tsy = an.y;
    const int tw = TVAM_TILE_PITCH(tp.tsx);  // guard band of one voxel on every side, odd pitch
    r.sx = stx;
    r.sy = sty * tw;
    r.lidx = (vy - y0 + 1) * tw + (vx - x0 + 1);
    r.rem = tau_x - tau_e;  // distance left inside this tile
    r.t = ff.x + tau_e;
    return true;
}

__device__ __forceinline__ float tvam_block_max(float v, float* red) {
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float m = red[0];
    for (int w = 1; w < TVAM_WAVES; ++w) m = fmaxf(m, red[w]);
    return m;
}

__device__ __forceinline__ float tvam_block_sum(float v, float* red) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float m = red[0];
    for (int w = 1; w < TVAM_WAVES; ++w) m += red[w];
    return m;
}

// Record index (sample-major, tvam_ray_setup_kernel) -> (shard angle, crop row, crop column, sample).
__device__ __forceinline__ void tvam_ray_of(const TvamConsts& k, const TvamTiles& tp, uint32_t i, int& al, int& rowc,
                                            int& colc, int& smp) {
    const int64_t n_local = (int64_t)tp.n_shard * k.crop_y * k.crop_x;
    smp = (int)((int64_t)i / n_local);
    const int64_t g = (int64_t)i - (int64_t)smp * n_local + k.shard_base;
    const int64_t t = g / k.crop_x;
    colc = (int)(g - t * k.crop_x);
    const int64_t a = t / k.crop_y;
    rowc = (int)(t - a * k.crop_y);
    al = (int)a - k.a0;
}

// Slot setup of the per-ray tile kernels: slot f -> (sample, slice row, list entry) -> the ray's
// resumed march state in this tile.  false: nothing to march (zero pattern under skip_zero,
// inactive pixel, other slice, or the ray misses the tile).
template <int MODE, bool W2>
__device__ __forceinline__ bool tvam_tile_slot(const TvamConsts& k, const TvamTiles& tp, const float* __restrict__ pat,
                                               const int32_t* __restrict__ idxmap, int kz, int x0, int x1, int y0,
                                               int y1, int al, int colc, int rowc, int smp, int acc_mode, float fscale,
                                               TvamTileRay& r, float& e0, int& why) {
    float em = 1.0f;
    if (MODE == TVAM_MODE_FWD && k.skip_zero) {
        const int64_t local = ((int64_t)(k.a0 + al) * k.crop_y + rowc) * k.crop_x + colc - k.shard_base;
        why = 4;
        if (pat[local] == 0.0f) return false;  // contributes exactly zero dose
    }
    const bool reach = tvam_tile_ray(k, tp, kz, x0, x1, y0, y1, rowc, al, colc, smp, idxmap, r);
    why = reach ? 0 : r.why;
    if (!reach) return false;
    if (MODE == TVAM_MODE_FWD) {  // (after the slice test: half of config 5's slots lie in another slice)
        em = pat[r.local] * k.wscale;  // Le * weight (common.py:108-111, volume.py:49)
        if (acc_mode != ACC_FLOAT) em *= fscale;
        em *= r.weight;  // attenuation of the vial's interfaces (sensor.py:404)
    }
    e0 = (W2 ? em * k.sig_t : em) * tvam_exp2(k.nsig2 * r.t);
    return true;
}

// One workgroup per (xy tile, z-slice); the tile (+ guard band) resident in LDS.
template <int MODE, bool W2>
__global__ __launch_bounds__(TVAM_BLOCK) void tvam_tile_kernel(
    TvamConsts k, TvamTiles tp, const float* __restrict__ pat, const int32_t* __restrict__ idxmap,
    const float* __restrict__ gin, float* __restrict__ out, unsigned long long* __restrict__ counter, int nzl) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* tile = reinterpret_cast<float*>(smem);
    const int tsx = tp.tsx, tsy = tp.tsy, ns = tp.n_shard;
    const int tw = TVAM_TILE_PITCH(tsx), th = tsy + 2;  // tile + 1-voxel guard band, odd row pitch
    const int tile_words = tw * th;
    float* s_red = tile + tile_words;
    unsigned* s_amax = reinterpret_cast<unsigned*>(s_red + 16);  // forward: per-angle max |p|

    // XCD-aware order: workgroup b runs on XCD b % 8; XCD x takes slices x, x + 8, x + 16, ..., all
    // tiles of a slice in turn, so the tiles re-reading one slice's ray records (every tile a ray
    // crosses reads its record) share that XCD's L2 instead of fetching it into all eight, and the
    // XCDs' loads stay even where the work per slice is not (contiguous slice runs per XCD left the
    // XCDs of a sparse active set's empty slices idle: config 5 with filter_radon 11 % slower)
    const int ntl = tp.ntx * tp.nty;
    const int bi = (int)(blockIdx.x >> 3);
    const int zloc = (bi / ntl) * 8 + (int)(blockIdx.x & 7);
    const int tile_id = bi - (bi / ntl) * ntl;
    if (zloc >= nzl) return;
    const int kz = zloc + (MODE == TVAM_MODE_FWD ? tp.kz0 : 0);
    const int x0 = (tile_id % tp.ntx) * tsx, y0 = (tile_id / tp.ntx) * tsy;
    const int x1 = min(x0 + tsx, k.res[0]), y1 = min(y0 + tsy, k.res[1]);
    const int wx = x1 - x0, wy = y1 - y0;
    const size_t slice_base = (size_t)kz * (size_t)k.res[0] * (size_t)k.res[1];

    int nonzero = 0;
    for (int i = threadIdx.x; i < tile_words; i += TVAM_BLOCK) {
        float v = 0.0f;
        if (MODE == TVAM_MODE_ADJ) {
            int ly = i / tw - 1, lx = i - (ly + 1) * tw - 1;
            if (lx >= 0 && ly >= 0 && lx < wx && ly < wy)
                v = gin[slice_base + (size_t)(y0 + ly) * k.res[0] + (x0 + lx)] * k.inv_vol;  // volume.py:130
            nonzero |= v != 0.0f ? 1 : 0;
        }
        tile[i] = v;
    }
    if (MODE == TVAM_MODE_FWD)
        for (int i = threadIdx.x; i < ns; i += TVAM_BLOCK) s_amax[i] = 0u;
    if (MODE == TVAM_MODE_ADJ) {
        // an all-zero gradient tile (the thresholded loss is flat wherever the dose meets its
        // bounds) gathers exactly 0 on every ray, which adds nothing: no march
        if (!__syncthreads_or(nonzero)) return;
    } else {
        __syncthreads();
    }

    // this tile's (angle, column) slots, longest predicted in-tile march first
    const uint32_t* slots = tp.slots + tp.slot_off[tile_id];
    const int nrt = (int)(tp.slot_off[tile_id + 1] - tp.slot_off[tile_id]);
    // rows: the slice's main rows plus its stray rays (TvamTiles::slice_moff), else its full row list
    const bool main_rows = tp.slice_moff && *tp.stray_n <= (unsigned long long)tp.stray_cap;
    const int32_t* rows = main_rows ? tp.slice_mrows : tp.slice_rows;
    const int rbeg = main_rows ? tp.slice_moff[kz] : tp.slice_off[kz];
    const int rend = main_rows ? tp.slice_moff[kz + 1] : tp.slice_off[kz + 1];
    const int nrows = rend - rbeg;
    const int nrows_all = tp.slice_off[kz + 1] - tp.slice_off[kz];  // (every marched ray comes from these)
    const int sbeg = main_rows ? (int)tp.stray_off[kz] : 0, send = main_rows ? (int)tp.stray_off[kz + 1] : 0;
    const int spp = (int)tp.spp;
    // slot f -> (sample, slice row, list entry) with the sample slowest: the lanes of a wave march
    // different pixels.  With the sample fastest, spp neighbouring lanes marched one pixel's
    // jittered rays through the same voxels, and their LDS atomics / the adjoint's per-pixel
    // global atomics hit the same addresses (90 % of the forward's LDS cycles were bank conflicts).
    const int per_row = nrt;
    const int first = nrows * per_row;  // the slots of sample 0
    const int total = first * spp;

    // Forward: pick the accumulator.  Fixed point (int32 ds_add: ~4x the
    // throughput of ds_add_f32 on gfx950) with a per-workgroup scale 2^e
    // chosen so that |sum| < 2^30 is guaranteed: at most rays_per_voxel/n_shard
    // rays of one angle (and sample, and row) cross a voxel, each adding at
    // most |em| * min(1, st*sqrt2*h), so
    //   |voxel sum| <= vox_chord * (rays_per_voxel/n_shard) * spp * rows * sum_a max|em|_a.
    // Two's complement sums are exact and order-independent (deterministic);
    // the step is ~1e-9 of the tile's largest possible voxel sum.  When fewer
    // than 1/64 of the rays are within 2^10 of the largest |value| (a few
    // outliers would set the step), the workgroup uses ds_add_f32 instead.
    int acc_mode = ACC_GATHER;
    float fscale = 1.0f;
    if (MODE == TVAM_MODE_FWD) {
        float nz = 0.0f;
        TvamSlot sl;
        tvam_slot_init(sl, threadIdx.x, max(per_row, 1));
        for (int f = threadIdx.x; f < first; f += TVAM_BLOCK, tvam_slot_next(sl, per_row)) {  // one look per (angle, column)
            const uint32_t e = slots[sl.rrem];
            const int al = (int)(e >> 16), colc = (int)(e & 0xffffu);
            const int rowc = rows[rbeg + sl.ri];
            const int64_t local = ((int64_t)(k.a0 + al) * k.crop_y + rowc) * k.crop_x + colc - k.shard_base;
            if (idxmap && idxmap[local] < 0) continue;
            const float v = fabsf(pat[local]);
            if (v > 0.0f) {
                atomicMax(&s_amax[al], __float_as_uint(v));  // non-negative floats order like their bits
                nz += 1.0f;
            }
        }
        for (int f = sbeg + (int)threadIdx.x; f < send; f += TVAM_BLOCK) {  // the stray rays
            int al, rowc, colc, smp;
            tvam_ray_of(k, tp, tp.stray_list[f], al, rowc, colc, smp);
            const int64_t local = ((int64_t)(k.a0 + al) * k.crop_y + rowc) * k.crop_x + colc - k.shard_base;
            if (idxmap && idxmap[local] < 0) continue;
            const float v = fabsf(pat[local]);
            if (v > 0.0f) {
                atomicMax(&s_amax[al], __float_as_uint(v));
                nz += 1.0f;
            }
        }
        __syncthreads();
        float am = 0.0f, amx = 0.0f;
        for (int a = threadIdx.x; a < ns; a += TVAM_BLOCK) {
            const float v = __uint_as_float(s_amax[a]);
            am += v;
            amx = fmaxf(amx, v);
        }
        const float amax_sum = tvam_block_sum(am, s_red);
        const float pmax = tvam_block_max(amx, s_red);
        const float pcnt = tvam_block_sum(nz, s_red);
        // outlier test: how many rays are within 2^10 of the largest |value|
        float nbig = 0.0f;
        if (pmax > 0.0f && isfinite(pmax)) {
            const float thr = pmax * (1.0f / 1024.0f);
            tvam_slot_init(sl, threadIdx.x, max(per_row, 1));
            for (int f = threadIdx.x; f < first; f += TVAM_BLOCK, tvam_slot_next(sl, per_row)) {
                const uint32_t e = slots[sl.rrem];
                const int al = (int)(e >> 16), colc = (int)(e & 0xffffu);
                const int rowc = rows[rbeg + sl.ri];
                const int64_t local = ((int64_t)(k.a0 + al) * k.crop_y + rowc) * k.crop_x + colc - k.shard_base;
                if (idxmap && idxmap[local] < 0) continue;
                nbig += fabsf(pat[local]) >= thr ? 1.0f : 0.0f;
            }
            for (int f = sbeg + (int)threadIdx.x; f < send; f += TVAM_BLOCK) {
                int al, rowc, colc, smp;
                tvam_ray_of(k, tp, tp.stray_list[f], al, rowc, colc, smp);
                const int64_t local = ((int64_t)(k.a0 + al) * k.crop_y + rowc) * k.crop_x + colc - k.shard_base;
                if (idxmap && idxmap[local] < 0) continue;
                nbig += fabsf(pat[local]) >= thr ? 1.0f : 0.0f;
            }
            nbig = tvam_block_sum(nbig, s_red);
        }
        const float per_angle = k.rays_per_voxel / (float)ns;
        const float bound = amax_sum * fabsf(k.wscale) * k.vox_chord * per_angle * (float)(nrows_all * spp);
        const int headroom = 30;
        if (!(amax_sum > 0.0f)) {
            acc_mode = ACC_FIXED;  // all-zero tile: every contribution is 0
        } else if (64.0f * nbig >= pcnt && isfinite(bound)) {
            int e;
            frexpf(bound, &e);  // bound < 2^e
            e = headroom - e;
            e = e > 126 ? 126 : (e < -126 ? -126 : e);
            fscale = ldexpf(1.0f, e);
            acc_mode = ACC_FIXED;
        } else {
            acc_mode = ACC_FLOAT;
            if (counter && threadIdx.x == 0) atomicAdd(counter, 1ull);  // fallback statistics
        }
        __syncthreads();
    }

    constexpr int ESZ = 4;
    unsigned long long nvis = 0;
    // one march from a resumed state, into the tile (forward / count) or gathering from it (adjoint)
    auto march = [&](TvamMarchRay& m, float rtsx, float rtsy, int sxb, int syb) -> float {
        float acc = 0.0f;
        if (MODE == TVAM_MODE_FWD) {
            if (acc_mode == ACC_FIXED)
                tvam_march<ACC_FIXED, W2>(m, rtsx, rtsy, sxb, syb, k.sig_t, acc, nvis);
            else
                tvam_march<ACC_FLOAT, W2>(m, rtsx, rtsy, sxb, syb, k.sig_t, acc, nvis);
        } else if (MODE == TVAM_MODE_ADJ) {
            tvam_march<ACC_GATHER, W2>(m, rtsx, rtsy, sxb, syb, k.sig_t, acc, nvis);
        } else {
            tvam_march<ACC_COUNT, W2>(m, rtsx, rtsy, sxb, syb, k.sig_t, acc, nvis, reinterpret_cast<const char*>(tile),
                                      tw, wx, wy);
        }
        return acc;
    };

    // Adjoint with spp a power of two <= 64: the sample FASTEST instead (lanes of a group of spp march
    // one pixel's jittered rays), so the group sums its partials with shuffles and adds them to the
    // pixel's gradient with one global atomic per tile instead of spp (config 4: 16 atomics on one
    // address per workgroup).  The gather reads the same LDS words on the group's near-identical
    // paths: broadcasts, not conflicts (the forward's LDS atomics are why it keeps the sample slowest).
    const bool sfast = MODE == TVAM_MODE_ADJ && spp > 1 && spp <= 64 && (spp & (spp - 1)) == 0;
    const int sshift = sfast ? __ffs(spp) - 1 : 0;
    TvamSlot sl;
    tvam_slot_init(sl, (int)threadIdx.x >> sshift, max(per_row, 1));
    for (int f = threadIdx.x; f < total; f += TVAM_BLOCK, tvam_slot_next(sl, per_row, TVAM_BLOCK >> sshift)) {
        const int smp = sfast ? (f & (spp - 1)) : (spp == 1 ? 0 : sl.ri / nrows);
        const int rowi = sfast ? sl.ri : sl.ri - smp * nrows;
        const uint32_t e = slots[sl.rrem];
        TvamTileRay r;
        float e0;
        int why = 5;
        float part = 0.0f;  // sfast: this lane's weighted partial
        if (tvam_tile_slot<MODE, W2>(k, tp, pat, idxmap, kz, x0, x1, y0, y1, (int)(e >> 16), (int)(e & 0xffffu),
                                     rows[rbeg + rowi], smp, acc_mode, fscale, r, e0, why)) {
            TvamMarchRay m;
            m.pv = reinterpret_cast<char*>(tile) + r.lidx * ESZ;
            m.Tx = r.dtx;
            m.Ty = r.dty;
            m.rem = r.rem;
            m.stop = r.rem - 1e-6f;
            m.e0 = e0;
            const float acc = march(m, r.tsx, r.tsy, r.sx * ESZ, r.sy * ESZ);
            if (MODE == TVAM_MODE_ADJ) {
                const float v = acc * (k.wscale * r.weight);  // backward_from(Le * em_grad), volume.py:274-276
                if (sfast)
                    part = v;
                else
                    atomicAdd(&out[r.act], v);
            }
        }
        if (MODE == TVAM_MODE_ADJ && sfast) {  // the pixel's spp partials (groups are whole: total = first * spp)
            for (int o = 1; o < spp; o <<= 1) part += __shfl_xor(part, o, 64);
            if (smp == 0 && part != 0.0f) {
                const int64_t local = ((int64_t)(k.a0 + (int)(e >> 16)) * k.crop_y + rows[rbeg + rowi]) * k.crop_x +
                                      (int)(e & 0xffffu) - k.shard_base;
                const int64_t act = idxmap ? (int64_t)idxmap[local] : local;
                if (act >= 0) atomicAdd(&out[act], part);
            }
        }
    }
    for (int f = sbeg + (int)threadIdx.x; f < send; f += TVAM_BLOCK) {  // the slice's stray rays
        int al, rowc, colc, smp;
        tvam_ray_of(k, tp, tp.stray_list[f], al, rowc, colc, smp);
        TvamTileRay r;
        float e0;
        int why = 5;
        if (tvam_tile_slot<MODE, W2>(k, tp, pat, idxmap, kz, x0, x1, y0, y1, al, colc, rowc, smp, acc_mode, fscale, r,
                                     e0, why)) {
            TvamMarchRay m;
            m.pv = reinterpret_cast<char*>(tile) + r.lidx * ESZ;
            m.Tx = r.dtx;
            m.Ty = r.dty;
            m.rem = r.rem;
            m.stop = r.rem - 1e-6f;
            m.e0 = e0;
            const float acc = march(m, r.tsx, r.tsy, r.sx * ESZ, r.sy * ESZ);
            if (MODE == TVAM_MODE_ADJ) atomicAdd(&out[r.act], acc * (k.wscale * r.weight));
        }
    }

    if (MODE == TVAM_MODE_FWD) {
        __syncthreads();
        const float outscale = k.inv_vol / fscale;
        const int* itile = reinterpret_cast<const int*>(tile);
        for (int i = threadIdx.x; i < wx * wy; i += TVAM_BLOCK) {
            int ly = i / wx, lx = i - ly * wx;
            const int li = (ly + 1) * tw + (lx + 1);
            float v = acc_mode == ACC_FIXED ? (float)itile[li] * outscale : tile[li] * k.inv_vol;
            out[slice_base + (size_t)(y0 + ly) * k.res[0] + (x0 + lx)] = v;
        }
    } else if (MODE == TVAM_MODE_COUNT) {
        for (int off = 32; off > 0; off >>= 1) nvis += __shfl_down(nvis, off, 64);
        if ((threadIdx.x & 63) == 0 && nvis) atomicAdd(counter, nvis);
    }
}

hipError_t tvam_launch_tiles(int mode, const TvamConsts& k, const TvamTiles& t, size_t lds_bytes,
                             const float* pat, const int32_t* idxmap, const float* gin, float* out,
                             unsigned long long* counter, hipStream_t stream) {
    // forward launches may cover a slice range [kz0, kz1) (tvam_forward_slices); the others every slice
    const int nzl = mode == TVAM_MODE_FWD && t.kz1 > t.kz0 ? t.kz1 - t.kz0 : k.nz;
    TvamTiles tl = t;
    if (!(mode == TVAM_MODE_FWD && t.kz1 > t.kz0)) tl.kz0 = 0;
    const int64_t nwg = (int64_t)t.ntx * t.nty * ((nzl + 7) / 8 * 8);
    dim3 grid((unsigned)nwg);  // slices rounded up to a multiple of 8 (the kernel's XCD-aware order)
    dim3 block(TVAM_BLOCK);
    const bool w2 = k.vox_chord < TVAM_W2_MAX;
#define TVAM_TILE_LAUNCH(M)                                                                                      \
    if (w2)                                                                                                      \
        hipLaunchKernelGGL((tvam_tile_kernel<M, true>), grid, block, lds_bytes, stream, k, tl, pat, idxmap, gin, out, \
                           counter, nzl);                                                                        \
    else                                                                                                         \
        hipLaunchKernelGGL((tvam_tile_kernel<M, false>), grid, block, lds_bytes, stream, k, tl, pat, idxmap, gin, out, \
                           counter, nzl);
    switch (mode) {
        case TVAM_MODE_FWD:
            TVAM_TILE_LAUNCH(TVAM_MODE_FWD)
            break;
        case TVAM_MODE_ADJ:
            TVAM_TILE_LAUNCH(TVAM_MODE_ADJ)
            break;
        default:
            TVAM_TILE_LAUNCH(TVAM_MODE_COUNT)
            break;
    }
#undef TVAM_TILE_LAUNCH
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Sparse active set <-> dense crop layout (projector.py:90-98 order)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t tvam_dense_index(const TvamConsts& k, uint32_t p) {
    uint32_t hw = (uint32_t)k.res_x * (uint32_t)k.res_y;
    uint32_t a = p / hw, r = p - a * hw;
    uint32_t row = r / (uint32_t)k.res_x, col = r - row * (uint32_t)k.res_x;
    int rc = (int)row - k.crop_off_y, cc = (int)col - k.crop_off_x;
    if (a < (uint32_t)k.a0 || a >= (uint32_t)k.a1 || rc < 0 || rc >= k.crop_y || cc < 0 || cc >= k.crop_x) return -1;
    return ((int64_t)(a - (uint32_t)k.a0) * k.crop_y + rc) * k.crop_x + cc;  // shard-local
}

__global__ void tvam_scatter_kernel(TvamConsts k, const float* __restrict__ data,
                                    const uint32_t* __restrict__ pixels, uint64_t n, float* __restrict__ dense,
                                    int32_t* __restrict__ idxmap) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        int64_t di = tvam_dense_index(k, pixels[i]);
        if (di < 0) continue;
        dense[di] = data ? data[i] : 0.0f;
        idxmap[di] = (int32_t)i;
    }
}

__global__ void tvam_gather_kernel(TvamConsts k, const float* __restrict__ dense, const uint32_t* __restrict__ pixels,
                                   uint64_t n, float* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        int64_t di = tvam_dense_index(k, pixels[i]);
        out[i] = di < 0 ? 0.0f : dense[di];
    }
}

static unsigned tvam_grid_for(uint64_t n) {
    uint64_t g = (n + 255) / 256;
    return (unsigned)(g < 4096 ? (g ? g : 1) : 4096);
}

hipError_t tvam_launch_scatter(const TvamConsts& k, const float* data, const uint32_t* pixels, uint64_t n,
                               float* dense, int32_t* idxmap, hipStream_t stream) {
    hipLaunchKernelGGL(tvam_scatter_kernel, dim3(tvam_grid_for(n)), dim3(256), 0, stream, k, data, pixels, n, dense,
                       idxmap);
    return hipGetLastError();
}

hipError_t tvam_launch_gather(const TvamConsts& k, const float* dense, const uint32_t* pixels, uint64_t n, float* out,
                              hipStream_t stream) {
    hipLaunchKernelGGL(tvam_gather_kernel, dim3(tvam_grid_for(n)), dim3(256), 0, stream, k, dense, pixels, n, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// ThresholdedLoss (loss.py:82-132), binary target: fused value + gradient.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float tvam_powi(float x, int K) {
    float r = 1.0f;
    for (int i = 0; i < K; ++i) r *= x;
    return r;
}

// The object test of a voxel: target > 0 (loss.py:119), from the f32 target or from its bit mask
// (tvam_target_mask: bit i of word i / 32 = target[i] > 0, read at bit offset mbit0 + i): the same
// predicate from 1/32 of the bytes.
template <bool MASK>
__device__ __forceinline__ bool tvam_is_obj(const float* __restrict__ target, const uint32_t* __restrict__ mask,
                                            uint64_t mbit0, uint64_t i) {
    if (MASK) {
        const uint64_t b = mbit0 + i;
        return (mask[b >> 5] >> (b & 31)) & 1u;
    }
    return target[i] > 0.0f;
}

// four consecutive voxels' object bits (bit j = voxel i + j); i = 4 t, mbit0 % 4 == 0 on the float4 path of a mask
template <bool MASK>
__device__ __forceinline__ uint32_t tvam_obj4(const float* __restrict__ target, const uint32_t* __restrict__ mask,
                                              uint64_t mbit0, uint64_t t) {
    if (MASK) {
        const uint64_t b = mbit0 + 4 * t;
        return (mask[b >> 5] >> (b & 31)) & 15u;
    }
    const float4 tg = reinterpret_cast<const float4*>(target)[t];
    return (tg.x > 0.0f ? 1u : 0u) | (tg.y > 0.0f ? 2u : 0u) | (tg.z > 0.0f ? 4u : 0u) | (tg.w > 0.0f ? 8u : 0u);
}

__global__ __launch_bounds__(256) void tvam_target_mask_kernel(const float* __restrict__ target, uint64_t n,
                                                               uint32_t* __restrict__ mask) {
    // one word per thread: 32 voxels, the last word's bits past n are 0
    const uint64_t nw = (n + 31) / 32, stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
        uint32_t m = 0;
        for (int j = 0; j < 32; ++j) {
            const uint64_t i = 32 * w + j;
            if (i < n && target[i] > 0.0f) m |= 1u << j;
        }
        mask[w] = m;
    }
}

hipError_t tvam_launch_target_mask(const float* target, uint64_t n, uint32_t* mask, hipStream_t stream) {
    const uint64_t nw = (n + 31) / 32;
    unsigned g = (unsigned)((nw + 255) / 256);
    if (g > 4096) g = 4096;
    if (g == 0) g = 1;
    hipLaunchKernelGGL(tvam_target_mask_kernel, dim3(g), dim3(256), 0, stream, target, n, mask);
    return hipGetLastError();
}

// KC: the exponent K as a compile-time constant (1..4: tvam_powi unrolled, the same products in the same
// order), or 0: K at run time
template <int KC>
__device__ __forceinline__ float tvam_loss_grad_elem(float x, bool obj, int Kr, float tl, float tu, float w_object,
                                                     float w_void, float w_limit, float& gr) {
    const int K = KC ? KC : Kr;
    if (obj) {
        const float zo = tu - x, zl = x - 1.0f;
        const float ro = zo > 0.0f ? zo : 0.0f, rl = zl > 0.0f ? zl : 0.0f;
        gr = (zo > 0.0f ? -w_object * (float)K * tvam_powi(ro, K - 1) : 0.0f) +
             (zl > 0.0f ? w_limit * (float)K * tvam_powi(rl, K - 1) : 0.0f);
        return w_object * tvam_powi(ro, K) + w_limit * tvam_powi(rl, K);
    }
    const float zv = x - tl;
    const float rv = zv > 0.0f ? zv : 0.0f;
    gr = zv > 0.0f ? w_void * (float)K * tvam_powi(rv, K - 1) : 0.0f;
    return w_void * tvam_powi(rv, K);
}

// n4: elements / 4 when dose, ddose, grad (and the f32 target, or a mask offset % 4 == 0) allow
// float4 accesses, else 0
template <bool MASK, int KC>
__global__ __launch_bounds__(256) void tvam_loss_threshold_kernel(
    const float* __restrict__ dose, const float* __restrict__ ddose, float alpha, const float* __restrict__ target,
    const uint32_t* __restrict__ mask, uint64_t mbit0, uint64_t n, uint64_t n4, int K, float tl, float tu,
    float w_object, float w_void, float w_limit, float scale, double* __restrict__ out, float* __restrict__ grad) {
    __shared__ double red[256 / 64];
    double acc = 0.0;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = tid; t < n4; t += stride) {
        float4 x = reinterpret_cast<const float4*>(dose)[t];
        if (ddose) {  // vol + alpha * dvol (lbfgs.py:258)
            const float4 dx = reinterpret_cast<const float4*>(ddose)[t];
            x = make_float4(fmaf(alpha, dx.x, x.x), fmaf(alpha, dx.y, x.y), fmaf(alpha, dx.z, x.z), fmaf(alpha, dx.w, x.w));
        }
        const uint32_t ob = tvam_obj4<MASK>(target, mask, mbit0, t);
        float4 g;
        acc += (double)tvam_loss_grad_elem<KC>(x.x, ob & 1u, K, tl, tu, w_object, w_void, w_limit, g.x);
        acc += (double)tvam_loss_grad_elem<KC>(x.y, ob & 2u, K, tl, tu, w_object, w_void, w_limit, g.y);
        acc += (double)tvam_loss_grad_elem<KC>(x.z, ob & 4u, K, tl, tu, w_object, w_void, w_limit, g.z);
        acc += (double)tvam_loss_grad_elem<KC>(x.w, ob & 8u, K, tl, tu, w_object, w_void, w_limit, g.w);
        if (grad)
            reinterpret_cast<float4*>(grad)[t] = make_float4(g.x * scale, g.y * scale, g.z * scale, g.w * scale);
    }
    for (uint64_t i = 4 * n4 + tid; i < n; i += stride) {
        float x = dose[i];
        if (ddose) x = fmaf(alpha, ddose[i], x);
        float gr;
        acc += (double)tvam_loss_grad_elem<KC>(x, tvam_is_obj<MASK>(target, mask, mbit0, i), K, tl, tu, w_object, w_void,
                                           w_limit, gr);
        if (grad) grad[i] = gr * scale;
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int w = 0; w < 256 / 64; ++w) s += red[w];
        atomicAdd(out, s * (double)scale);
    }
}

// Armijo probes of the linear line search (lbfgs.py:255-268): the loss of dose + alpha_j * ddose for
// up to TVAM_MAX_PROBES step sizes in one pass over dose / ddose / target (per element the same
// arithmetic as tvam_loss_threshold_kernel), out[j] += sum_j * scale.
struct TvamProbeAlphas {
    float a[TVAM_MAX_PROBES];
};

template <int KC>
__device__ __forceinline__ float tvam_loss_elem(float x, bool obj, int Kr, float tl, float tu, float w_object,
                                                float w_void, float w_limit) {
    const int K = KC ? KC : Kr;
    if (obj) {
        const float zo = tu - x, zl = x - 1.0f;
        const float ro = zo > 0.0f ? zo : 0.0f, rl = zl > 0.0f ? zl : 0.0f;
        return w_object * tvam_powi(ro, K) + w_limit * tvam_powi(rl, K);
    }
    const float zv = x - tl;
    const float rv = zv > 0.0f ? zv : 0.0f;
    return w_void * tvam_powi(rv, K);
}

template <bool MASK, int KC>
__global__ __launch_bounds__(256) void tvam_loss_probes_kernel(
    const float* __restrict__ dose, const float* __restrict__ ddose, TvamProbeAlphas al, int na,
    const float* __restrict__ target, const uint32_t* __restrict__ mask, uint64_t mbit0, uint64_t n, uint64_t n4, int K,
    float tl, float tu, float w_object, float w_void, float w_limit, float scale, double* __restrict__ out) {
    __shared__ double red[TVAM_MAX_PROBES][256 / 64];
    double acc[TVAM_MAX_PROBES];
#pragma unroll
    for (int j = 0; j < TVAM_MAX_PROBES; ++j) acc[j] = 0.0;
    auto elem = [&](float x0, float dx, bool obj) {
#pragma unroll
        for (int j = 0; j < TVAM_MAX_PROBES; ++j)
            if (j < na) acc[j] += (double)tvam_loss_elem<KC>(fmaf(al.a[j], dx, x0), obj, K, tl, tu, w_object, w_void, w_limit);
    };
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    // n4: elements / 4 when the arrays allow float4 loads, else 0
    const float4* d4 = reinterpret_cast<const float4*>(dose);
    const float4* dd4 = reinterpret_cast<const float4*>(ddose);
    for (uint64_t i = tid; i < n4; i += stride) {
        const float4 x = d4[i], dx = dd4[i];
        const uint32_t ob = tvam_obj4<MASK>(target, mask, mbit0, i);
        elem(x.x, dx.x, ob & 1u);
        elem(x.y, dx.y, ob & 2u);
        elem(x.z, dx.z, ob & 4u);
        elem(x.w, dx.w, ob & 8u);
    }
    for (uint64_t i = 4 * n4 + tid; i < n; i += stride) elem(dose[i], ddose[i], tvam_is_obj<MASK>(target, mask, mbit0, i));
#pragma unroll
    for (int j = 0; j < TVAM_MAX_PROBES; ++j) {
        double v = acc[j];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
        if ((threadIdx.x & 63) == 0) red[j][threadIdx.x >> 6] = v;
    }
    __syncthreads();
    if ((int)threadIdx.x < na) {
        double s = 0.0;
        for (int w = 0; w < 256 / 64; ++w) s += red[threadIdx.x][w];
        atomicAdd(out + threadIdx.x, s * (double)scale);
    }
}

static bool tvam_al16(const void* a, const void* b, const void* c) {
    return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15) == 0;
}

hipError_t tvam_launch_loss_probes(const float* dose, const float* ddose, const float* alphas, int na,
                                   const float* target, const uint32_t* mask, uint64_t mbit0, uint64_t n, int K,
                                   float tl, float tu, float w_object, float w_void, float w_limit, float scale,
                                   double* out, hipStream_t stream) {
    TvamProbeAlphas al{};
    for (int j = 0; j < na; ++j) al.a[j] = alphas[j];
    const bool v4 = tvam_al16(dose, ddose, mask ? nullptr : target) && (!mask || mbit0 % 4 == 0);
    const uint64_t n4 = v4 ? n / 4 : 0;
    unsigned g = (unsigned)(((v4 ? n4 : n) + 255) / 256);
    if (g > 2048) g = 2048;
    if (g == 0) g = 1;
#define TVAM_PROBES(M, KC)                                                                                    \
    hipLaunchKernelGGL((tvam_loss_probes_kernel<M, KC>), dim3(g), dim3(256), 0, stream, dose, ddose, al, na, target, \
                       mask, mbit0, n, n4, K, tl, tu, w_object, w_void, w_limit, scale, out)
#define TVAM_PROBES_K(M)                     \
    switch (K) {                             \
        case 1: TVAM_PROBES(M, 1); break;    \
        case 2: TVAM_PROBES(M, 2); break;    \
        case 3: TVAM_PROBES(M, 3); break;    \
        case 4: TVAM_PROBES(M, 4); break;    \
        default: TVAM_PROBES(M, 0); break;   \
    }
    if (mask) {
        TVAM_PROBES_K(true)
    } else {
        TVAM_PROBES_K(false)
    }
#undef TVAM_PROBES_K
#undef TVAM_PROBES
    return hipGetLastError();
}

hipError_t tvam_launch_loss_threshold(const float* dose, const float* ddose, float alpha, const float* target,
                                      const uint32_t* mask, uint64_t mbit0, uint64_t n, int K, float tl, float tu,
                                      float w_object, float w_void, float w_limit, float scale, double* out,
                                      float* grad, hipStream_t stream) {
    const bool v4 = tvam_al16(dose, ddose, grad) && tvam_al16(mask ? nullptr : target, nullptr, nullptr) &&
                    (!mask || mbit0 % 4 == 0);
    const uint64_t n4 = v4 ? n / 4 : 0;
    unsigned g = (unsigned)(((v4 ? n4 : n) + 255) / 256);
    if (g > 2048) g = 2048;
    if (g == 0) g = 1;
#define TVAM_LOSS(M, KC)                                                                                           \
    hipLaunchKernelGGL((tvam_loss_threshold_kernel<M, KC>), dim3(g), dim3(256), 0, stream, dose, ddose, alpha, target, \
                       mask, mbit0, n, n4, K, tl, tu, w_object, w_void, w_limit, scale, out, grad)
#define TVAM_LOSS_K(M)                     \
    switch (K) {                           \
        case 1: TVAM_LOSS(M, 1); break;    \
        case 2: TVAM_LOSS(M, 2); break;    \
        case 3: TVAM_LOSS(M, 3); break;    \
        case 4: TVAM_LOSS(M, 4); break;    \
        default: TVAM_LOSS(M, 0); break;   \
    }
    if (mask) {
        TVAM_LOSS_K(true)
    } else {
        TVAM_LOSS_K(false)
    }
#undef TVAM_LOSS_K
#undef TVAM_LOSS
    return hipGetLastError();
}
