// Scattering media (BASELINE config 4): the part of every
// path after its first medium segment.
//
// With has_scattering (sigma_s != 0) the reference's path loop
// (integrators/volume.py:179-272) deposits, for every medium segment, the
// analytic absorption along the whole segment up to the next surface
// (sensor.py:383-438 with maxt = si.t), weighted by the path attenuation, and
// continues the path from a free-flight sample (homogeneous medium:
// t = -log(1 - u) / sigma_t) in a phase-function direction.  The first medium
// segment is the planar, non-scattering one: the planar / tile kernels
// already deposit it (weight = the interfaces' attenuation).  This kernel
// replays each path's sampler stream to that segment, then runs the free
// flights and the 3-D DDA of every later segment:
//   forward:  global float atomics into the dose (scattered segments leave
//             their slice and tile, so there is no LDS tile to own them);
//   adjoint:  gathers of grad * inv_vol, one atomic per path into its pattern
//             gradient;
//   count:    visits of the later segments.
// One thread per (ray, sample); the stream is `active position * spp +
// sample` (tvam_stream), as for the ray records.  Draw order per loop iteration (restated
// in oracle/tvam_oracle.c, or_trace_scatter): RR next_1d, medium next_1d,
// BSDF next_1d + next_2d on surfaces, phase next_1d + next_2d on scattering.
#include "tvam_internal.h"

#include <algorithm>
#include <vector>

#include "tvam_bricks.h"

namespace {

__device__ __forceinline__ float sc_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Nearest hit t >= 0 of the open tube (radius r, |z| <= half) for a 3-D ray
// (Mitsuba cylinder restated; oracle or_tube_hit).
__device__ __forceinline__ float sc_tube_hit(float ox, float oy, float oz, float dx, float dy, float dz, float r,
                                             float half) {
    float t0, t1;
    if (!tvam_cyl_roots(ox, oy, dx, dy, r, t0, t1)) return TVAM_INF;
    if (!(t1 >= 0.0f)) return TVAM_INF;
    const float zn = fmaf(dz, t0, oz), zf = fmaf(dz, t1, oz);
    if (t0 >= 0.0f && zn >= -half && zn <= half) return t0;
    if (zf >= -half && zf <= half) return t1;
    return TVAM_INF;
}

// Next container surface from inside the medium (the inner / index-matched tube
// comes first; the outer tube is only reached through it).
// Square vial: the inner cuboid (closed: its top and bottom faces end a
// segment too).  Occluders end a segment where they are nearer.
__device__ __forceinline__ float sc_container_hit(const TvamConsts& k, float ox, float oy, float oz, float dx,
                                                  float dy, float dz) {
    float t;
    if (k.vial_type == 2) {
        float nx, ny, nz;
        t = tvam_box_hit(ox, oy, oz, dx, dy, dz, k.vial_r, k.vial_r, k.vial_hz_int, nx, ny, nz);
    } else {
        t = sc_tube_hit(ox, oy, oz, dx, dy, dz, k.vial_r, k.vial_half_h);
        if (k.vial_type == 1) {
            const float te = sc_tube_hit(ox, oy, oz, dx, dy, dz, k.vial_r_ext, k.vial_half_h);
            if (!(t <= te)) t = te;  // (never from inside; kept like the oracle)
        }
    }
    if (k.n_occ) t = fminf(t, tvam_occ_hit(k, ox, oy, oz, dx, dy, dz));
    return t;
}

// Mitsuba coordinate_system() (Duff et al. 2017) and the phase functions'
// sample(): isotropic (square_to_uniform_sphere, world space), rayleigh (cbrt
// inversion of the (3/8)(1 + mu^2) CDF), hg (-cos_theta in the frame of wi).
__device__ __forceinline__ void sc_phase(const TvamConsts& k, float dx, float dy, float dz, float u1, float u2,
                                         float& wx, float& wy, float& wz) {
    float lx, ly, lz;
    if (k.phase_type == TVAM_PHASE_ISOTROPIC) {  // square_to_uniform_sphere(u): z = 1 - 2 u.y, phi = 2 pi u.x
        const float z = 1.0f - 2.0f * u2;
        const float r = sqrtf(fmaxf(1.0f - z * z, 0.0f));
        const float sp = sinf(TVAM_TWO_PI * u1), cp = cosf(TVAM_TWO_PI * u1);
        wx = r * cp;
        wy = r * sp;
        wz = z;
        return;
    }
    if (k.phase_type == TVAM_PHASE_RAYLEIGH) {
        const float z = 2.0f * (2.0f * u1 - 1.0f);
        const float tmp = sqrtf(z * z + 1.0f);
        const float ct = cbrtf(z + tmp) + cbrtf(z - tmp);
        const float st = sqrtf(fmaxf(1.0f - ct * ct, 0.0f));
        const float sp = sinf(TVAM_TWO_PI * u2), cp = cosf(TVAM_TWO_PI * u2);
        lx = st * cp;
        ly = st * sp;
        lz = ct;
    } else {
        const float g = k.phase_g;
        float ct;
        if (fabsf(g) < 5.9604644775390625e-08f) {
            ct = 1.0f - 2.0f * u1;
        } else {
            const float sq = (1.0f - g * g) / (1.0f - g + 2.0f * g * u1);
            ct = (1.0f + g * g - sq * sq) / (2.0f * g);
        }
        const float st = sqrtf(fmaxf(1.0f - ct * ct, 0.0f));
        const float sp = sinf(TVAM_TWO_PI * u2), cp = cosf(TVAM_TWO_PI * u2);
        lx = st * cp;
        ly = st * sp;
        lz = -ct;
    }
    const float nx = -dx, ny = -dy, nz = -dz;  // Frame3f(wi = -d)
    const float sg = copysignf(1.0f, nz);
    const float a = -1.0f / (sg + nz);
    const float b = nx * ny * a;
    const float sx = sg * (nx * nx * a) + 1.0f, sy = sg * b, sz = -sg * nx;
    const float tx = b, ty = fmaf(ny, ny * a, sg), tz = -ny;
    wx = sx * lx + tx * ly + nx * lz;
    wy = sy * lx + ty * ly + ny * lz;
    wz = sz * lx + tz * ly + nz * lz;
}

// ---------------------------------------------------------------------------
// Brick-binned forward of the scattered segments.  A segment's DDA state after
// the box clip and initialisation (sensor.py:327-365) is stored as a record;
// its visits inside a brick of TVAM_BX x TVAM_BY x TVAM_BZ voxels follow in
// closed form from the per-axis crossing times t_a(k) = dtm0_a + (k - 1) ts_a
// (relative to t_start; the resume of the tile kernels, in 3-D), so each brick
// workgroup marches only its part of every segment crossing it, adding into an
// LDS tile, and writes the tile once.
// ---------------------------------------------------------------------------
// SegDda, sc_dda_init, sc_walk_bricks, sc_brick_count: tvam_bricks.h

// The visits of a segment inside the voxel box [lo, hi) (a brick), resumed in
// closed form at the box entry: per axis the step count n at the entry time,
// the next crossing at t = dtm0 + n ts (fmaf from the count, so a visit splits
// at a brick face exactly where the neighbouring brick resumes), one axis per
// visit (ties: x before y before z).  Axes are kept in scalars (dynamically
// indexed arrays would be promoted to LDS).  F(local x, y, z, weight
// e^{-st t0} - e^{-st t1}).
template <typename F>
__device__ __forceinline__ void sc_box_march(const TvamConsts& k, const SegDda& q, const int lo[3], const int hi[3],
                                             F&& f) {
    float tin[3], tout[3];
    int nin[3], nout[3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
        tvam_axis_window(q.sv[a], q.step[a], q.dtm0[a], q.ts[a], lo[a], hi[a], tin[a], tout[a], nin[a], nout[a]);
    const float tau_e = fmaxf(fmaxf(fmaxf(tin[0], tin[1]), tin[2]), 0.0f);
    const float tau_x = fminf(fminf(fminf(tout[0], tout[1]), tout[2]), q.tau_end);
    if (!(tau_e < tau_x)) return;
    int n0 = tvam_axis_steps(tau_e, q.dtm0[0], q.ts[0], nin[0], nout[0]);
    int n1 = tvam_axis_steps(tau_e, q.dtm0[1], q.ts[1], nin[1], nout[1]);
    int n2 = tvam_axis_steps(tau_e, q.dtm0[2], q.ts[2], nin[2], nout[2]);
    int x = q.sv[0] + q.step[0] * n0 - lo[0];
    int y = q.sv[1] + q.step[1] * n1 - lo[1];
    int z = q.sv[2] + q.step[2] * n2 - lo[2];
    const float ts0 = q.ts[0], ts1 = q.ts[1], ts2 = q.ts[2];
    const float d0 = q.dtm0[0], d1 = q.dtm0[1], d2 = q.dtm0[2];
    float T0 = d0 < TVAM_INF ? fmaf((float)n0, ts0, d0) : TVAM_INF;
    float T1 = d1 < TVAM_INF ? fmaf((float)n1, ts1, d1) : TVAM_INF;
    float T2 = d2 < TVAM_INF ? fmaf((float)n2, ts2, d2) : TVAM_INF;
    const int s0 = q.step[0], s1 = q.step[1], s2 = q.step[2];
    const float stop = tau_x - 1e-6f;
    const float base = k.nsig2 * q.t_start;
    float ea = sc_exp2(fmaf(k.nsig2, tau_e, base)), tp = tau_e;
    for (int guard = 0; guard < 3 * 4096; ++guard) {
        const bool m0 = T0 <= T1 && T0 <= T2;
        const bool m1 = !m0 && T1 <= T2;
        const float tmin = m0 ? T0 : (m1 ? T1 : T2);
        const float tn = tmin < tau_x ? tmin : tau_x;
        // e^{-st t} (1 - e^{-st dt}) without cancellation (tvam_omexp); ea tracks e^{-st t}
        const float c = ea * tvam_omexp(k.sig_t * fmaxf(tn - tp, 0.0f));
        const float eb = ea - c;
        tp = tn;
        f(x, y, z, c);
        if (!(tn < stop)) break;
        if (m0) {
            x += s0;
            ++n0;
            T0 = fmaf((float)n0, ts0, d0);
        } else if (m1) {
            y += s1;
            ++n1;
            T1 = fmaf((float)n1, ts1, d1);
        } else {
            z += s2;
            ++n2;
            T2 = fmaf((float)n2, ts2, d2);
        }
        ea = eb;
    }
}

// sc_box_march for the brick kernels: the same visits (the same crossing times fmaf(n, ts, dtm0)
// and axis choices), stepped without divergent branches (every axis' candidate next crossing is
// formed and selected), with the visit's index into a TVAM_BX x TVAM_BY x TVAM_BZ tile carried
// incrementally.  W2: the degree-2 visit weight of tvam_common.h on E = st e^{-st t} (used when
// st * sqrt(3) * max h < TVAM_W2_MAX3, a relative weight error < 4.2e-6), restarted from exp2 at
// every brick entry; else tvam_omexp as sc_box_march.  F(tile index, weight).
#define TVAM_W2_MAX3 5.0e-3f
template <bool W2, typename F>
__device__ __forceinline__ void sc_brick_march(const TvamConsts& k, const SegDda& q, const int lo[3], const int hi[3],
                                               F&& f) {
    float tin[3], tout[3];
    int nin[3], nout[3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
        tvam_axis_window(q.sv[a], q.step[a], q.dtm0[a], q.ts[a], lo[a], hi[a], tin[a], tout[a], nin[a], nout[a]);
    const float tau_e = fmaxf(fmaxf(fmaxf(tin[0], tin[1]), tin[2]), 0.0f);
    const float tau_x = fminf(fminf(fminf(tout[0], tout[1]), tout[2]), q.tau_end);
    if (!(tau_e < tau_x)) return;
    int n0 = tvam_axis_steps(tau_e, q.dtm0[0], q.ts[0], nin[0], nout[0]);
    int n1 = tvam_axis_steps(tau_e, q.dtm0[1], q.ts[1], nin[1], nout[1]);
    int n2 = tvam_axis_steps(tau_e, q.dtm0[2], q.ts[2], nin[2], nout[2]);
    constexpr int SY = TVAM_BX, SZ = TVAM_BX * TVAM_BY;
    int li = (q.sv[0] + q.step[0] * n0 - lo[0]) + (q.sv[1] + q.step[1] * n1 - lo[1]) * SY +
             (q.sv[2] + q.step[2] * n2 - lo[2]) * SZ;
    const int dl0 = q.step[0], dl1 = q.step[1] * SY, dl2 = q.step[2] * SZ;
    const float ts0 = q.ts[0], ts1 = q.ts[1], ts2 = q.ts[2];
    const float d0 = q.dtm0[0], d1 = q.dtm0[1], d2 = q.dtm0[2];
    // a frozen axis (dtm0 = inf) never steps: its T stays inf
    const bool f0 = d0 < TVAM_INF, f1 = d1 < TVAM_INF, f2 = d2 < TVAM_INF;
    float T0 = f0 ? fmaf((float)n0, ts0, d0) : TVAM_INF;
    float T1 = f1 ? fmaf((float)n1, ts1, d1) : TVAM_INF;
    float T2 = f2 ? fmaf((float)n2, ts2, d2) : TVAM_INF;
    const float stop = tau_x - 1e-6f;
    const float base = k.nsig2 * q.t_start;
    const float e_in = sc_exp2(fmaf(k.nsig2, tau_e, base));
    float ea = W2 ? k.sig_t * e_in : e_in, tp = tau_e;
    const float mhs = -0.5f * k.sig_t, msig = -k.sig_t;
    for (int guard = 0; guard < 3 * 4096; ++guard) {
        const bool m0 = T0 <= T1 && T0 <= T2;
        const bool m1 = !m0 && T1 <= T2;
        const float tmin = m0 ? T0 : (m1 ? T1 : T2);
        const float tn = tmin < tau_x ? tmin : tau_x;
        const float dt = fmaxf(tn - tp, 0.0f);
        float c;
        if (W2) {
            c = ea * dt * fmaf(mhs, dt, 1.0f);
            ea = fmaf(msig, c, ea);
        } else {
            c = ea * tvam_omexp(k.sig_t * dt);
            ea = ea - c;
        }
        tp = tn;
        f(li, c);
        if (!(tn < stop)) break;
        const bool m2 = !m0 && !m1;
        n0 += m0 ? 1 : 0;
        n1 += m1 ? 1 : 0;
        n2 += m2 ? 1 : 0;
        li += m0 ? dl0 : (m1 ? dl1 : dl2);
        T0 = m0 ? fmaf((float)n0, ts0, d0) : T0;
        T1 = m1 ? fmaf((float)n1, ts1, d1) : T1;
        T2 = m2 ? fmaf((float)n2, ts2, d2) : T2;
    }
}

// The whole segment, brick by brick (the binned forward's visits exactly).
template <typename F>
__device__ __forceinline__ void sc_seg_march(const TvamConsts& k, const SegDda& q, F&& f) {
    const int B[3] = {TVAM_BX, TVAM_BY, TVAM_BZ};
    const int nb[3] = {sc_nbr(k, 0), sc_nbr(k, 1), sc_nbr(k, 2)};
    sc_walk_bricks(k, q, [&](int bid, float, float) {
        const int bx = bid % nb[0], by = (bid / nb[0]) % nb[1], bz = bid / (nb[0] * nb[1]);
        const int lo[3] = {bx * B[0], by * B[1], bz * B[2]};
        const int hi[3] = {min(lo[0] + B[0], k.res[0]), min(lo[1] + B[1], k.res[1]), min(lo[2] + B[2], k.res[2])};
        sc_box_march(k, q, lo, hi, [&](int x, int y, int z, float c) { f(lo[0] + x, lo[1] + y, lo[2] + z, c); });
    });
}

// One medium segment's 3-D DDA (sensor.py:327-438, op for op like the oracle's
// or_dda): MODE FWD adds em * (e^{-st t} - e^{-st (t + dt)}) * inv_vol into the
// dose, ADJ returns sum (...) * grad * inv_vol, COUNT counts visits.
template <int MODE>
__device__ float sc_dda(const TvamConsts& k, float ox, float oy, float oz, float dx, float dy, float dz, float maxt,
                        float em, float* __restrict__ dose, const float* __restrict__ gin, uint64_t& nvis) {
    const float o[3] = {ox, oy, oz}, d[3] = {dx, dy, dz};
    SegDda q;
    if (!sc_dda_init(k, o, d, maxt, q)) return 0.0f;
    float acc = 0.0f;
    const int64_t sy = k.res[0], sz = (int64_t)k.res[0] * k.res[1];
    sc_seg_march(k, q, [&](int x, int y, int z, float c) {
        const int64_t idx = x + y * sy + z * sz;
        if (MODE == TVAM_MODE_FWD) atomicAdd(&dose[idx], em * c);
        else if (MODE == TVAM_MODE_ADJ) acc = fmaf(c, gin[idx] * k.inv_vol, acc);
        ++nvis;
    });
    return acc;
}

// The largest of a 256-thread workgroup's non-negative values into *dst (float bits, which order
// like the floats): one device atomic per workgroup (one per wave put ~10^6 atomics on a single
// address per chunk)
__device__ __forceinline__ void sc_block_max(float v, uint32_t* dst) {
    __shared__ float s_max[4];
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        v = fmaxf(fmaxf(s_max[0], s_max[1]), fmaxf(s_max[2], s_max[3]));
        if (v > 0.0f) atomicMax(dst, __float_as_uint(v));
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void tvam_scatter_kernel(TvamConsts k, TvamTiles tp, const float* __restrict__ pat,
                                                           const int32_t* __restrict__ idxmap,
                                                           const float* __restrict__ gin, float* __restrict__ out,
                                                           unsigned long long* __restrict__ counter, TvamSegBuf sb) {
    const int spp = (int)tp.spp;
    const int64_t per_angle = (int64_t)k.crop_y * k.crop_x;
    const int64_t n = MODE == TVAM_MODE_EMIT ? sb.p1 : (int64_t)tp.n_shard * per_angle * spp;
    const int64_t i0 = MODE == TVAM_MODE_EMIT ? sb.p0 : 0;
    const float st = k.sig_t, ss = k.sig_s;
    const int nsurf = k.vial_type == 0 ? 1 : 2;  // glass vials: two surfaces before the medium
    uint64_t nvis = 0;
    float wmax = 0.0f;  // EMIT (forward): largest |record weight| of this thread's paths
    // EMIT with sb.hist: this workgroup's entries per brick (LDS), written to hist[brick][block]:
    // the counting sort of tvam_scatter_binned places the workgroup's entries of a brick after
    // those of the lower-numbered workgroups (tvam_bin_fill2_kernel walks the same paths)
    extern __shared__ uint32_t s_hist[];
    const bool hist = MODE == TVAM_MODE_EMIT && sb.hist != nullptr;
    if (hist) {
        for (int b = threadIdx.x; b < sb.nbricks; b += blockDim.x) s_hist[b] = 0u;
        __syncthreads();
    }
    for (int64_t i = i0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (MODE == TVAM_MODE_EMIT && !sb.adj)  // slots without a segment: attenuation 0 (the cache's rescale)
            for (int q = 0; q < sb.slots; ++q) reinterpret_cast<float*>(&sb.r[TVAM_REC_F4 * ((i - sb.p0) * sb.slots + q) + 2])[2] = 0.0f;
        int64_t local;
        int smp, al, rowc, colc;
        if (n <= (int64_t)0xffffffff) {  // 32-bit index arithmetic (a 64-bit division is ~3x the code)
            const uint32_t ii = (uint32_t)i, sp = (uint32_t)spp, pa = (uint32_t)per_angle, cx = (uint32_t)k.crop_x;
            const uint32_t l32 = ii / sp, a32 = l32 / pa, p32 = l32 - a32 * pa, r32 = p32 / cx;
            local = (int64_t)l32;
            smp = (int)(ii - l32 * sp);
            al = (int)a32;
            rowc = (int)r32;
            colc = (int)(p32 - r32 * cx);
        } else {
            local = i / spp;
            smp = (int)(i - local * spp);
            al = (int)(local / per_angle);
            const int64_t pix = local - (int64_t)al * per_angle;
            rowc = (int)(pix / k.crop_x);
            colc = (int)(pix - (int64_t)rowc * k.crop_x);
        }
        float em = 1.0f;
        int64_t act = local;
        if (MODE == TVAM_MODE_FWD || (MODE == TVAM_MODE_EMIT && !sb.adj)) {
            const float p = pat[local];
            if (p == 0.0f && k.skip_zero) continue;
            em = p * k.wscale * k.inv_vol;
        } else if (MODE == TVAM_MODE_EMIT) {  // adjoint records: weight att * wscale (grad * inv_vol gathered)
            em = k.wscale;
            if (idxmap && idxmap[local] < 0) continue;
        } else if (idxmap) {
            act = idxmap[local];
            if (act < 0) continue;
        }
        TvamPcg rng;
        rng.seed(tp.seed, tvam_stream(k, idxmap, local, (uint32_t)spp, smp));
        float jx = 0.5f, jy = 0.5f;
        if (!k.regular) {
            jx = rng.next_float();
            jy = rng.next_float();
        }
        (void)rng.next_float();  // aperture sample (projector.py:160)
        (void)rng.next_float();
        const float2 csv = tp.cs[al];
        float xc, yc, ox, oy, oz, dx, dy;
        tvam_ray_camera(k, k.crop_off_x + colc, k.crop_off_y + rowc, jx, jy, xc, yc);
        tvam_ray_world(k, csv.x, csv.y, xc, yc, ox, oy, oz, dx, dy);
        float o2x, o2y, d2x, d2y, maxt, wgt;
        if (!tvam_segment(k, ox, oy, oz, dx, dy, o2x, o2y, d2x, d2y, maxt, wgt)) continue;
        for (int q = 0; q < 5 * nsurf; ++q) (void)rng.next_float();  // surface iterations: RR, medium, BSDF
        float px = o2x, py = o2y, pz = oz, vx = d2x, vy = d2y, vz = 0.0f;
        float att = wgt;
        int depth = nsurf;
        float acc = 0.0f;
        for (int seg = 0;; ++seg) {
            const float q = fminf(0.99f, att);
            const float u_rr = rng.next_float();
            if (depth > k.rr_depth) {  // Russian roulette (volume.py:182-185)
                if (!(u_rr < q)) break;
                att = att * (1.0f / q);
            }
            if (!(att != 0.0f)) break;
            float tsi = maxt;
            if (seg > 0) {
                tsi = sc_container_hit(k, px, py, pz, vx, vy, vz);
                if (!(tsi < TVAM_INF)) break;  // escapes through an open end: no surface, no deposit
            }
            const float u_m = rng.next_float();
            const float tmi = -logf(1.0f - u_m) / st;
            if (seg > 0 && MODE == TVAM_MODE_EMIT) {
                const float o[3] = {px, py, pz}, dv[3] = {vx, vy, vz};
                SegDda q;
                if (seg <= sb.slots && sc_dda_init(k, o, dv, tsi, q)) {
                    const int64_t slot = (i - sb.p0) * sb.slots + (seg - 1);
                    sb.r[TVAM_REC_F4 * slot] = make_float4(q.t_start, q.tau_end, q.dtm0[0], q.dtm0[1]);
                    sb.r[TVAM_REC_F4 * slot + 1] = make_float4(q.dtm0[2], q.ts[0] * (float)q.step[0], q.ts[1] * (float)q.step[1],
                                             q.ts[2] * (float)q.step[2]);
                    // .z: the attenuation alone, for the cached forward's rescale (tvam_bin_reweight_kernel)
                    sb.r[TVAM_REC_F4 * slot + 2] = make_float4(__int_as_float(q.sv[0] | (q.sv[1] << 11) | (q.sv[2] << 22)), em * att, att, 0.0f);
                    // the bricks it crosses: counted in closed form (the bin fill does the only walk),
                    // or walked when the counting sort needs each brick's count
                    sb.m[slot] = hist ? (uint32_t)sc_walk_bricks(k, q, [&](int bid, float, float) {
                        atomicAdd(&s_hist[bid], 1u);
                    })
                                      : (uint32_t)sc_brick_count(k, q);
                    wmax = fmaxf(wmax, fabsf(em * att));
                }
            } else if (seg > 0) {
                const float r = sc_dda<MODE>(k, px, py, pz, vx, vy, vz, tsi, em * att, out, gin, nvis);
                if (MODE == TVAM_MODE_ADJ) acc = fmaf(att, r, acc);
            }
            if (tsi < tmi) break;  // leaves the medium for good (transmission only, convex tubes)
            const float tr = expf(-tmi * st);
            const float pdf = tr * st;
            const float inv = pdf > 0.0f ? 1.0f / pdf : 0.0f;
            float w = tr * inv;
            w = w * ss;
            (void)rng.next_float();  // phase next_1d
            const float u1 = rng.next_float(), u2 = rng.next_float();
            float wx, wy, wz;
            sc_phase(k, vx, vy, vz, u1, u2, wx, wy, wz);
            px = fmaf(vx, tmi, px);
            py = fmaf(vy, tmi, py);
            pz = fmaf(vz, tmi, pz);
            vx = wx;
            vy = wy;
            vz = wz;
            att = att * w;
            ++depth;
            if (depth >= k.max_depth) break;
        }
        if (MODE == TVAM_MODE_ADJ && acc != 0.0f) atomicAdd(&out[act], acc * k.wscale);
    }
    if (MODE == TVAM_MODE_COUNT) {
        for (int off = 32; off > 0; off >>= 1) nvis += __shfl_down(nvis, off, 64);
        if ((threadIdx.x & 63) == 0 && nvis) atomicAdd(counter, (unsigned long long)nvis);
    }
    if (MODE == TVAM_MODE_EMIT && !sb.adj) sc_block_max(wmax, sb.wmax);
    if (hist) {
        __syncthreads();
        for (int b = threadIdx.x; b < sb.nbricks; b += blockDim.x)
            sb.hist[(size_t)b * gridDim.x + blockIdx.x] = s_hist[b];
    }
}

// ---------------------------------------------------------------------------
// Frozen-axis rays of the per-ray tile path.  The reference's DDA initialises
// an axis's first crossing time as (next boundary - start) / d and disables the
// axis when that comes out negative in fp32 (sensor.py:358: the start point
// rounds past the boundary of its start voxel): the ray then never steps on
// that axis and marches along the other one, off its geometric chord.  The
// tile kernels only visit tiles on the chord (host-traced slot lists), so
// tvam_ray_setup_kernel marks such rays (ray_i.y = -2 - slice) and this kernel
// marches each of them over the whole grid (the brick walk's closed-form
// stepping keeps a frozen axis frozen), with global atomics (forward), a
// gather (adjoint) or a visit count.  About 3e-5 of the jittered rays of
// BASELINE configs 4-5; none under regular sampling.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void tvam_frozen_kernel(TvamConsts k, TvamTiles tp, const float* __restrict__ pat,
                                                          const int32_t* __restrict__ idxmap,
                                                          const float* __restrict__ gin, float* __restrict__ out,
                                                          unsigned long long* __restrict__ counter) {
    const int spp = (int)tp.spp;
    const int64_t per_angle = (int64_t)k.crop_y * k.crop_x;
    // the appended list when it held every frozen ray, else a scan of all ray records
    const unsigned long long nf = *tp.frozen_n;
    const bool list = (int64_t)nf <= tp.frozen_cap;
    const int64_t n = list ? (int64_t)nf : (int64_t)tp.n_shard * per_angle * spp;
    uint64_t nvis = 0;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = list ? tp.frozen[j] : j;
        const int iy = tp.ray_i[i].y;
        if (iy > -2) continue;
        if (MODE == TVAM_MODE_FWD && tp.kz1 > tp.kz0 && !(-2 - iy >= k.z0 + tp.kz0 && -2 - iy < k.z0 + tp.kz1))
            continue;  // a slice-range forward: another range's frozen ray (it stays in its slice)
        const int64_t n_local = (int64_t)tp.n_shard * per_angle;  // sample-major ray records
        const int smp = (int)(i / n_local);
        const int64_t local = i - (int64_t)smp * n_local;
        float em = 1.0f;
        int64_t act = local;
        if (MODE == TVAM_MODE_FWD) {
            const float p = pat[local];
            if (p == 0.0f && k.skip_zero) continue;
            em = p * k.wscale * k.inv_vol;
        } else if (MODE == TVAM_MODE_ADJ && idxmap) {
            act = idxmap[local];
            if (act < 0) continue;
        }
        const int al = (int)(local / per_angle);
        const int64_t pix = local - (int64_t)al * per_angle;
        const int rowc = (int)(pix / k.crop_x), colc = (int)(pix - (int64_t)rowc * k.crop_x);
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
        float o2x, o2y, d2x, d2y, maxt, wgt;
        if (!tvam_segment(k, ox, oy, oz, dx, dy, o2x, o2y, d2x, d2y, maxt, wgt)) continue;
        const float o[3] = {o2x, o2y, oz}, dv[3] = {d2x, d2y, 0.0f};
        SegDda q;
        if (!sc_dda_init(k, o, dv, maxt, q)) continue;
        const int64_t sy = k.res[0], sz = (int64_t)k.res[0] * k.res[1];
        const float emw = em * wgt;
        float acc = 0.0f;
        sc_seg_march(k, q, [&](int x, int y, int z, float c) {
            if (z < k.z0 || z >= k.z0 + k.nz) return;  // outside this plan's film slab
            const int64_t idx = x + y * sy + (int64_t)(z - k.z0) * sz;
            if (MODE == TVAM_MODE_FWD) atomicAdd(&out[idx], emw * c);
            else if (MODE == TVAM_MODE_ADJ) acc = fmaf(c, gin[idx] * k.inv_vol, acc);
            ++nvis;
        });
        if (MODE == TVAM_MODE_ADJ && acc != 0.0f) atomicAdd(&out[act], acc * wgt * k.wscale);
    }
    if (MODE == TVAM_MODE_COUNT) {
        for (int off = 32; off > 0; off >>= 1) nvis += __shfl_down(nvis, off, 64);
        if ((threadIdx.x & 63) == 0 && nvis) atomicAdd(counter, (unsigned long long)nvis);
    }
}

// ---------------------------------------------------------------------------
// Surface-aware films (film.py:16-21, sensor.py:405-409, volume.py:175-218):
// the target mesh stays in the scene with a null BSDF, so a path's medium
// segment is cut at every target hit; each piece restarts its DDA from the
// spawned origin (offset_p along the face normal), deposits into channel 0
// while inside the target and 1 outside, and the attenuation picks up
// e^{-st si.t} per piece (volume.py:263).  Non-scattering media; one thread
// per (ray, sample); restated op for op in oracle or_trace_surface.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sf_target_hit(const TvamConsts& k, float ox, float oy, float oz, float dx, float dy,
                                               float dz, int& tri) {
    float best = TVAM_INF;
    tri = -1;
    for (int i = 0; i < k.n_tgt; ++i) {
        const float t = tvam_tri_hit(k.tgt + 9 * i, ox, oy, oz, dx, dy, dz);
        if (t < best) {
            best = t;
            tri = i;
        }
    }
    return best;
}

// sc_dda with the film index x + y res.x + z res.x res.y times 2 plus the channel;
// FWD adds em * c (unscaled film), ADJ gathers grad / volume of the channel.
template <int MODE>
__device__ float sf_dda(const TvamConsts& k, float ox, float oy, float oz, float dx, float dy, float dz, float maxt,
                        float em, int ch, float* __restrict__ film, const float* __restrict__ gin,
                        const float* __restrict__ vols, uint64_t& nvis) {
    const float o[3] = {ox, oy, oz}, d[3] = {dx, dy, dz};
    SegDda q;
    if (!sc_dda_init(k, o, d, maxt, q)) return 0.0f;
    float acc = 0.0f;
    const int64_t sy = k.res[0], sz = (int64_t)k.res[0] * k.res[1];
    sc_seg_march(k, q, [&](int x, int y, int z, float c) {
        const int64_t idx = 2 * (x + y * sy + z * sz) + ch;
        if (MODE == TVAM_MODE_FWD) atomicAdd(&film[idx], em * c);
        else if (MODE == TVAM_MODE_ADJ) {
            const float v = vols[idx];
            const float iv = v != 0.0f ? 1.0f / v : 0.0f;  // volume.py:41-42
            acc = fmaf(c, gin[idx] * iv, acc);
        }
        ++nvis;
    });
    return acc;
}

// A point deposit of the ratio / delta sensors on a surface-aware film (sensor.py:143-151,
// :248-260): voxel floor((p - bbox.min) / h), skipped outside the grid, index 2 voxel + channel.
template <int MODE>
__device__ __forceinline__ float sf_point(const TvamConsts& k, float px, float py, float pz, float w, int ch,
                                          float* __restrict__ film, const float* __restrict__ gin,
                                          const float* __restrict__ vols, uint64_t& nvis) {
    const int vx = (int)floorf((px - k.bmin[0]) / k.h[0]);
    const int vy = (int)floorf((py - k.bmin[1]) / k.h[1]);
    const int vz = (int)floorf((pz - k.bmin[2]) / k.h[2]);
    if (vx < 0 || vy < 0 || vz < 0 || vx >= k.res[0] || vy >= k.res[1] || vz >= k.res[2]) return 0.0f;
    const int64_t idx = 2 * (vx + (int64_t)vy * k.res[0] + (int64_t)vz * k.res[0] * k.res[1]) + ch;
    ++nvis;
    if (MODE == TVAM_MODE_FWD) atomicAdd(&film[idx], w);
    else if (MODE == TVAM_MODE_ADJ) {
        const float v = vols[idx];
        return w * (gin[idx] * (v != 0.0f ? 1.0f / v : 0.0f));
    }
    return 0.0f;
}

// RNG (a scattering medium or the ratio / delta sensor; oracle or_trace_surface_scatter /
// or_trace_estimator): the path loop of tvam_scatter_kernel in which each segment ends at the
// nearer of the target mesh and the container; the draws per iteration are RR, the medium's
// (scattering media), the ratio sensor's steps, then BSDF 1d + 2d at a surface or the phase
// function's 1d + 2d at a medium event.  A target hit before the free flight ends passes the null
// BSDF with weight tr / pdf (pdf = tr, volume.py:206-208; e^{-st t} without scattering, :263),
// toggles the channel and does not count towards max_depth.
template <int MODE, bool RNG>
__global__ __launch_bounds__(256) void tvam_surface_kernel(TvamConsts k, TvamTiles tp, const float* __restrict__ pat,
                                                           const int32_t* __restrict__ idxmap,
                                                           const float* __restrict__ gin,
                                                           const float* __restrict__ vols, float* __restrict__ out,
                                                           unsigned long long* __restrict__ counter) {
    const int spp = (int)tp.spp;
    const int64_t per_angle = (int64_t)k.crop_y * k.crop_x;
    const int64_t n = (int64_t)tp.n_shard * per_angle * spp;
    const float st = k.sig_t, ss = k.sig_s, mj = k.majorant;
    const bool has_sc = ss != 0.0f;
    uint64_t nvis = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t local = i / spp;
        const int smp = (int)(i - local * spp);
        float em = 1.0f;
        int64_t act = local;
        if (MODE == TVAM_MODE_FWD) {
            const float p = pat[local];
            if (p == 0.0f && k.skip_zero) continue;
            em = p * k.wscale;
        } else if (idxmap) {
            act = idxmap[local];
            if (act < 0) continue;
        }
        const int al = (int)(local / per_angle);
        const int64_t pix = local - (int64_t)al * per_angle;
        const int rowc = (int)(pix / k.crop_x), colc = (int)(pix - (int64_t)rowc * k.crop_x);
        float jx = 0.5f, jy = 0.5f;
        TvamPcg rng;
        if (!k.regular || RNG) {
            rng.seed(tp.seed, tvam_stream(k, idxmap, local, (uint32_t)spp, smp));
            if (!k.regular) {
                jx = rng.next_float();
                jy = rng.next_float();
            }
        }
        const float2 csv = tp.cs[al];
        float xc, yc, ox, oy, oz, dx, dy;
        tvam_ray_camera(k, k.crop_off_x + colc, k.crop_off_y + rowc, jx, jy, xc, yc);
        tvam_ray_world(k, csv.x, csv.y, xc, yc, ox, oy, oz, dx, dy);
        float o2x, o2y, d2x, d2y, maxt, wgt;
        if (!tvam_segment(k, ox, oy, oz, dx, dy, o2x, o2y, d2x, d2y, maxt, wgt)) continue;
        const int nsurf = k.vial_type == 0 ? 1 : 2;
        if (RNG) {
            (void)rng.next_float();  // aperture sample (projector.py:160)
            (void)rng.next_float();
            for (int q = 0; q < (has_sc ? 5 : 4) * nsurf; ++q) (void)rng.next_float();  // RR, (medium), BSDF
        }
        float px = o2x, py = o2y, pz = oz;
        float vx = d2x, vy = d2y, vz = 0.0f;
        float att = wgt, tcont = maxt, acc = 0.0f;
        int inside = 0, depth = nsurf;
        for (int it = 0; it < 4096; ++it) {
            if (RNG) {
                const float q = fminf(0.99f, att);
                const float u_rr = rng.next_float();
                if (depth > k.rr_depth) {  // Russian roulette (volume.py:182-185)
                    if (!(u_rr < q)) break;
                    att = att * (1.0f / q);
                }
                if (!(att != 0.0f)) break;
            }
            int tri;
            const float tt = sf_target_hit(k, px, py, pz, vx, vy, vz, tri);
            const bool hit = tt < tcont;
            const float tsi = hit ? tt : tcont;
            float tmi = TVAM_INF;
            if (RNG && has_sc) tmi = -logf(1.0f - rng.next_float()) / st;
            const bool reached = !(tmi <= tsi);
            const int ch = inside ? 0 : 1;
            if (k.sensor_type == TVAM_SENSOR_DDA) {
                const float r = sf_dda<MODE>(k, px, py, pz, vx, vy, vz, tsi, em * att, ch, out, gin, vols, nvis);
                if (MODE == TVAM_MODE_ADJ) acc = fmaf(att, r, acc);
            } else if (RNG && k.sensor_type == TVAM_SENSOR_RATIO) {
                const float ratio = st / mj, keep = 1.0f - ratio;
                float t = 0.0f, pk = 1.0f;
                for (int s2 = 0; s2 < (1 << 20); ++s2) {
                    t = t + (-logf(1.0f - rng.next_float()) / mj);
                    if (!(t < tsi)) break;
                    const float w = att * pk * ratio;
                    const float r = sf_point<MODE>(k, fmaf(vx, t, px), fmaf(vy, t, py), fmaf(vz, t, pz), em * w, ch, out,
                                                   gin, vols, nvis);
                    if (MODE == TVAM_MODE_ADJ) acc += r;
                    pk = pk * keep;
                }
            } else if (RNG && !reached) {  // delta: the medium interaction ray(mei.t)
                const float r = sf_point<MODE>(k, fmaf(vx, tmi, px), fmaf(vy, tmi, py), fmaf(vz, tmi, pz), em * att, ch,
                                               out, gin, vols, nvis);
                if (MODE == TVAM_MODE_ADJ) acc += r;
            }
            if (RNG && !reached) {  // a medium event before the surface: phase sampling
                const float tr = expf(-tmi * st);
                const float pdf = tr * st;
                const float inv = pdf > 0.0f ? 1.0f / pdf : 0.0f;
                float w = tr * inv;
                w = w * ss;
                (void)rng.next_float();  // phase next_1d
                const float u1 = rng.next_float(), u2 = rng.next_float();
                float wx, wy, wz;
                sc_phase(k, vx, vy, vz, u1, u2, wx, wy, wz);
                px = fmaf(vx, tmi, px);
                py = fmaf(vy, tmi, py);
                pz = fmaf(vz, tmi, pz);
                vx = wx;
                vy = wy;
                vz = wz;
                att = att * w;
                ++depth;
                if (depth >= k.max_depth) break;
                tcont = sc_container_hit(k, px, py, pz, vx, vy, vz);
                if (!(tcont < TVAM_INF)) break;  // escapes through an open end
                continue;
            }
            if (!hit) break;  // the container or an occluder: leaves the medium for good
            if (RNG && has_sc) {
                const float tr = expf(-tsi * st);
                const float inv = tr > 0.0f ? 1.0f / tr : 0.0f;
                att = att * (tr * inv);
            } else {
                att = att * expf(-k.sig_t * tsi);
            }
            if (RNG) {
                (void)rng.next_float();  // BSDF next_1d + next_2d (null BSDF)
                (void)rng.next_float();
                (void)rng.next_float();
            }
            inside ^= 1;
            // spawn_ray at the target hit: offset_p along the geometric normal (oracle or_spawn_target)
            const float* v = k.tgt + 9 * tri;
            const float e1x = v[3] - v[0], e1y = v[4] - v[1], e1z = v[5] - v[2];
            const float e2x = v[6] - v[0], e2y = v[7] - v[1], e2z = v[8] - v[2];
            const float cx = e1y * e2z - e1z * e2y, cy = e1z * e2x - e1x * e2z, cz = e1x * e2y - e1y * e2x;
            const float inv = 1.0f / sqrtf(cx * cx + cy * cy + cz * cz);
            const float nx = cx * inv, ny = cy * inv, nz = cz * inv;
            const float hx = fmaf(vx, tt, px), hy = fmaf(vy, tt, py), hz = fmaf(vz, tt, pz);
            const float m = fmaxf(fmaxf(fabsf(hx), fabsf(hy)), fabsf(hz));
            float mag = (1.0f + m) * TVAM_RAY_EPS;
            if (__builtin_signbit(nx * vx + ny * vy + nz * vz)) mag = -mag;
            px = fmaf(mag, nx, hx);
            py = fmaf(mag, ny, hy);
            pz = fmaf(mag, nz, hz);
            tcont = sc_container_hit(k, px, py, pz, vx, vy, vz);
            if (!(tcont < TVAM_INF)) break;
        }
        if (MODE == TVAM_MODE_ADJ && acc != 0.0f) atomicAdd(&out[act], acc * k.wscale);
    }
    if (MODE == TVAM_MODE_COUNT) {
        for (int off = 32; off > 0; off >>= 1) nvis += __shfl_down(nvis, off, 64);
        if ((threadIdx.x & 63) == 0 && nvis) atomicAdd(counter, (unsigned long long)nvis);
    }
}

// ---------------------------------------------------------------------------
// General per-path kernel: the whole path loop of volume.py:179-272 per (ray,
// sample), every medium segment included, for the configurations the planar /
// tile kernels do not serve:
//   * sample_time (common.py:101-104): each ray's own rotation angle
//     2 pi (angle + u) / A, so the rays of one pattern are not parallel;
//   * the 'ratio' sensor (sensor.py:193-295): deposits at ray(t), t stepping
//     by -log(1 - u) / majorant (draws inside accumulate), weight
//     (1 - st / mu)^k st / mu;
//   * the 'delta' sensor (sensor.py:112-191): a deposit at each medium
//     interaction (collision estimator, weight 1 with sa / st in wscale).
// Forward: global float atomics; adjoint: gathers, one atomic per path.
// Restated op for op in oracle or_trace_estimator / or_trace_scatter.
// ---------------------------------------------------------------------------
template <int MODE>
__device__ __forceinline__ float gp_point(const TvamConsts& k, float px, float py, float pz, float w,
                                          float* __restrict__ out, const float* __restrict__ gin, uint64_t& nvis) {
    const int vx = (int)floorf((px - k.bmin[0]) / k.h[0]);
    const int vy = (int)floorf((py - k.bmin[1]) / k.h[1]);
    const int vz = (int)floorf((pz - k.bmin[2]) / k.h[2]);
    if (vx < 0 || vy < 0 || vz < 0 || vx >= k.res[0] || vy >= k.res[1] || vz >= k.res[2]) return 0.0f;
    const int64_t idx = vx + (int64_t)vy * k.res[0] + (int64_t)vz * k.res[0] * k.res[1];
    ++nvis;
    if (MODE == TVAM_MODE_FWD) atomicAdd(&out[idx], w);
    else if (MODE == TVAM_MODE_ADJ) return w * (gin[idx] * k.inv_vol);
    return 0.0f;
}

template <int MODE>
__global__ __launch_bounds__(256) void tvam_path_kernel(TvamConsts k, TvamTiles tp, const float* __restrict__ pat,
                                                        const int32_t* __restrict__ idxmap,
                                                        const float* __restrict__ gin, float* __restrict__ out,
                                                        unsigned long long* __restrict__ counter) {
    const int spp = (int)tp.spp;
    const int64_t per_angle = (int64_t)k.crop_y * k.crop_x;
    const int64_t n = (int64_t)tp.n_shard * per_angle * spp;
    const float st = k.sig_t, ss = k.sig_s, mj = k.majorant;
    const bool has_sc = ss != 0.0f;
    const int nsurf = k.vial_type == 0 ? 1 : 2;
    uint64_t nvis = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t local = i / spp;
        const int smp = (int)(i - local * spp);
        float em = 1.0f;
        int64_t act = local;
        if (MODE == TVAM_MODE_FWD) {
            const float p = pat[local];
            if (p == 0.0f && k.skip_zero) continue;
            em = p * k.wscale * k.inv_vol;
        } else if (idxmap) {
            act = idxmap[local];
            if (act < 0) continue;
        }
        const int al = (int)(local / per_angle);
        const int64_t pix = local - (int64_t)al * per_angle;
        const int rowc = (int)(pix / k.crop_x), colc = (int)(pix - (int64_t)rowc * k.crop_x);
        TvamPcg rng;
        rng.seed(tp.seed, tvam_stream(k, idxmap, local, (uint32_t)spp, smp));
        float jx = 0.5f, jy = 0.5f;
        if (!k.regular) {
            jx = rng.next_float();
            jy = rng.next_float();
        }
        float c, sn;
        if (k.sample_time) {  // common.py:101-104: time = (angle + u) / n_patterns
            float time = (float)(k.a0 + al);
            time = time + rng.next_float();
            time = time / (float)k.n_patterns;
            float alpha = TVAM_TWO_PI * time;
            if (k.clockwise) alpha = -alpha;
            c = cosf(alpha);
            sn = sinf(alpha);
        } else {
            const float2 csv = tp.cs[al];
            c = csv.x;
            sn = csv.y;
        }
        (void)rng.next_float();  // aperture sample (projector.py:160)
        (void)rng.next_float();
        float xc, yc, ox, oy, oz, dx, dy;
        tvam_ray_camera(k, k.crop_off_x + colc, k.crop_off_y + rowc, jx, jy, xc, yc);
        tvam_ray_world(k, c, sn, xc, yc, ox, oy, oz, dx, dy);
        float o2x, o2y, d2x, d2y, maxt, wgt;
        if (!tvam_segment(k, ox, oy, oz, dx, dy, o2x, o2y, d2x, d2y, maxt, wgt)) continue;
        for (int q = 0; q < (has_sc ? 5 : 4) * nsurf; ++q) (void)rng.next_float();  // RR, (medium), BSDF
        float px = o2x, py = o2y, pz = oz, vx = d2x, vy = d2y, vz = 0.0f;
        float att = wgt;
        int depth = nsurf;
        float acc = 0.0f;
        for (int seg = 0;; ++seg) {
            const float q = fminf(0.99f, att);
            const float u_rr = rng.next_float();
            if (depth > k.rr_depth) {  // Russian roulette (volume.py:182-185)
                if (!(u_rr < q)) break;
                att = att * (1.0f / q);
            }
            if (!(att != 0.0f)) break;
            float tsi = maxt;
            if (seg > 0) {
                tsi = sc_container_hit(k, px, py, pz, vx, vy, vz);
                if (!(tsi < TVAM_INF)) break;
            }
            float tmi = TVAM_INF;
            if (has_sc) tmi = -logf(1.0f - rng.next_float()) / st;
            const bool reached = !(tmi <= tsi);
            if (k.sensor_type == TVAM_SENSOR_DDA) {
                const float r = sc_dda<MODE>(k, px, py, pz, vx, vy, vz, tsi, em * att, out, gin, nvis);
                if (MODE == TVAM_MODE_ADJ) acc = fmaf(att, r, acc);
            } else if (k.sensor_type == TVAM_SENSOR_RATIO) {
                const float ratio = st / mj, keep = 1.0f - ratio;
                float t = 0.0f, pk = 1.0f;
                for (int it = 0; it < (1 << 20); ++it) {
                    t = t + (-logf(1.0f - rng.next_float()) / mj);
                    if (!(t < tsi)) break;
                    const float w = att * pk * ratio;
                    const float r = gp_point<MODE>(k, fmaf(vx, t, px), fmaf(vy, t, py), fmaf(vz, t, pz), em * w, out,
                                                   gin, nvis);
                    if (MODE == TVAM_MODE_ADJ) acc += r;  // w * grad * inv_vol (em = 1 in the adjoint)
                    pk = pk * keep;
                }
            } else if (!reached) {  // delta: the medium interaction ray(mei.t)
                const float r = gp_point<MODE>(k, fmaf(vx, tmi, px), fmaf(vy, tmi, py), fmaf(vz, tmi, pz), em * att,
                                               out, gin, nvis);
                if (MODE == TVAM_MODE_ADJ) acc += r;
            }
            if (reached) break;  // leaves the medium (transmission only, convex containers)
            const float tr = expf(-tmi * st);
            const float pdf = tr * st;
            const float inv = pdf > 0.0f ? 1.0f / pdf : 0.0f;
            float w = tr * inv;
            w = w * ss;
            (void)rng.next_float();  // phase next_1d
            const float u1 = rng.next_float(), u2 = rng.next_float();
            float wx, wy, wz;
            sc_phase(k, vx, vy, vz, u1, u2, wx, wy, wz);
            px = fmaf(vx, tmi, px);
            py = fmaf(vy, tmi, py);
            pz = fmaf(vz, tmi, pz);
            vx = wx;
            vy = wy;
            vz = wz;
            att = att * w;
            ++depth;
            if (depth >= k.max_depth) break;
        }
        if (MODE == TVAM_MODE_ADJ && acc != 0.0f) atomicAdd(&out[act], acc * k.wscale);
    }
    if (MODE == TVAM_MODE_COUNT) {
        for (int off = 32; off > 0; off >>= 1) nvis += __shfl_down(nvis, off, 64);
        if ((threadIdx.x & 63) == 0 && nvis) atomicAdd(counter, (unsigned long long)nvis);
    }
}

__global__ __launch_bounds__(256) void tvam_scale_volumes_kernel(int64_t n, const float* __restrict__ vols,
                                                                 float* __restrict__ dose) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const float v = vols[i];
        dose[i] = dose[i] * (v != 0.0f ? 1.0f / v : 0.0f);
    }
}

// One compute_volume sample (sensor.py:89-104): 1 = inside the target mesh.
__device__ __forceinline__ int sf_volume_sample(const TvamConsts& k, TvamPcg& rng, int vx, int vy, int vz,
                                                const float3 mb0, const float3 mb1) {
    const float fx = rng.next_float(), fy = rng.next_float(), fz = rng.next_float();
    const float sx = rng.next_float(), sy = rng.next_float();
    const float ox = k.bmin[0] + k.h[0] * ((float)vx + fx);
    const float oy = k.bmin[1] + k.h[1] * ((float)vy + fy);
    const float oz = k.bmin[2] + k.h[2] * ((float)vz + fz);
    if (!(ox > mb0.x && oy > mb0.y && oz > mb0.z && ox < mb1.x && oy < mb1.y && oz < mb1.z)) return 0;
    // warp::square_to_uniform_sphere(sample): z = 1 - 2 y, phi = 2 pi x
    const float dz = 1.0f - 2.0f * sy, r = sqrtf(fmaxf(1.0f - dz * dz, 0.0f));
    const float dx = r * cosf(TVAM_TWO_PI * sx), dy = r * sinf(TVAM_TWO_PI * sx);
    int tri;
    const float t = sf_target_hit(k, ox, oy, oz, dx, dy, dz, tri);
    if (!(t < TVAM_INF)) return 0;
    const float* p = k.tgt + 9 * tri;
    const float e1x = p[3] - p[0], e1y = p[4] - p[1], e1z = p[5] - p[2];
    const float e2x = p[6] - p[0], e2y = p[7] - p[1], e2z = p[8] - p[2];
    const float cx = e1y * e2z - e1z * e2y, cy = e1z * e2x - e1x * e2z, cz = e1x * e2y - e1y * e2x;
    return cx * dx + cy * dy + cz * dz > 0.0f ? 1 : 0;
}

// compute_volume (sensor.py:47-110): one thread per voxel, sample_count points.
// A voxel whose box misses the open mesh bbox has every point outside; one whose
// box meets no triangle's bounding box lies on one side of the (closed) mesh, so
// every one of its points gets the same answer: its first three samples decide
// (majority, against a ray grazing an edge).  The others run every sample.
__global__ __launch_bounds__(256) void tvam_volume_kernel(TvamConsts k, float3 mb0, float3 mb1, uint32_t sample_count,
                                                          const float* __restrict__ tri_box,
                                                          float* __restrict__ volumes) {
    const int64_t V = (int64_t)k.res[0] * k.res[1] * k.res[2];
    const float vvol = k.h[0] * k.h[1] * k.h[2];
    for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < V; v += (int64_t)gridDim.x * 256) {
        const int vx = (int)(v % k.res[0]), vy = (int)((v / k.res[0]) % k.res[1]);
        const int vz = (int)(v / ((int64_t)k.res[0] * k.res[1]));
        uint32_t cin = 0;
        const float x0 = k.bmin[0] + k.h[0] * (float)vx, x1 = k.bmin[0] + k.h[0] * ((float)vx + 1.0f);
        const float y0 = k.bmin[1] + k.h[1] * (float)vy, y1 = k.bmin[1] + k.h[1] * ((float)vy + 1.0f);
        const float z0 = k.bmin[2] + k.h[2] * (float)vz, z1 = k.bmin[2] + k.h[2] * ((float)vz + 1.0f);
        const bool may = x1 >= mb0.x && x0 <= mb1.x && y1 >= mb0.y && y0 <= mb1.y && z1 >= mb0.z && z0 <= mb1.z;
        if (may) {
            bool touch = false;  // some triangle's (slightly grown) bounding box meets the voxel
            for (int i = 0; i < k.n_tgt && !touch; ++i) {
                const float* b = tri_box + 6 * i;
                touch = x1 >= b[0] && x0 <= b[3] && y1 >= b[1] && y0 <= b[4] && z1 >= b[2] && z0 <= b[5];
            }
            TvamPcg rng;
            rng.seed(0u, (uint64_t)v);
            if (touch || sample_count < 3) {
                for (uint32_t i = 0; i < sample_count; ++i) cin += sf_volume_sample(k, rng, vx, vy, vz, mb0, mb1);
            } else {
                int c3 = 0;
                for (int i = 0; i < 3; ++i) c3 += sf_volume_sample(k, rng, vx, vy, vz, mb0, mb1);
                cin = c3 >= 2 ? sample_count : 0;
            }
        }
        const uint32_t cout = sample_count - cin;
        volumes[2 * v] = (float)cin * vvol / (float)sample_count;
        volumes[2 * v + 1] = (float)cout * vvol / (float)sample_count;
    }
}

// discretize (utils.py:83-128): one thread per voxel, one ray from the voxel centre
// bmin + (0.5 + i) h along square_to_uniform_sphere(next_2d) of the independent
// sampler seeded (0, voxels) at lane = voxel index; inside when the centre is
// strictly inside the mesh bbox and the first target hit faces away from the ray.
// A voxel whose box meets no triangle's (grown) bounding box is decided the same way
// (one ray, like the reference), so the result is exactly the per-voxel predicate.
__global__ __launch_bounds__(256) void tvam_discretize_kernel(TvamConsts k, float3 mb0, float3 mb1,
                                                              float* __restrict__ occ) {
    const int64_t V = (int64_t)k.res[0] * k.res[1] * k.res[2];
    for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < V; v += (int64_t)gridDim.x * 256) {
        const int vx = (int)(v % k.res[0]), vy = (int)((v / k.res[0]) % k.res[1]);
        const int vz = (int)(v / ((int64_t)k.res[0] * k.res[1]));
        const float ox = k.bmin[0] + (0.5f + (float)vx) * k.h[0];
        const float oy = k.bmin[1] + (0.5f + (float)vy) * k.h[1];
        const float oz = k.bmin[2] + (0.5f + (float)vz) * k.h[2];
        float inside = 0.0f;
        if (ox > mb0.x && oy > mb0.y && oz > mb0.z && ox < mb1.x && oy < mb1.y && oz < mb1.z) {
            TvamPcg rng;
            rng.seed(0u, (uint64_t)v);
            const float sx = rng.next_float(), sy = rng.next_float();
            const float dz = 1.0f - 2.0f * sy, r = sqrtf(fmaxf(1.0f - dz * dz, 0.0f));
            const float dx = r * cosf(TVAM_TWO_PI * sx), dy = r * sinf(TVAM_TWO_PI * sx);
            int tri;
            const float t = sf_target_hit(k, ox, oy, oz, dx, dy, dz, tri);
            if (t < TVAM_INF) {
                const float* p = k.tgt + 9 * tri;
                const float e1x = p[3] - p[0], e1y = p[4] - p[1], e1z = p[5] - p[2];
                const float e2x = p[6] - p[0], e2y = p[7] - p[1], e2z = p[8] - p[2];
                const float cx = e1y * e2z - e1z * e2y, cy = e1z * e2x - e1x * e2z, cz = e1x * e2y - e1y * e2x;
                inside = cx * dx + cy * dy + cz * dz > 0.0f ? 1.0f : 0.0f;
            }
        }
        occ[v] = inside;
    }
}

}  // namespace

hipError_t tvam_launch_surface_paths(int mode, const TvamConsts& k, const TvamTiles& t, const float* pat,
                                     const int32_t* idxmap, const float* gin, const float* vols, float* out,
                                     unsigned long long* counter, hipStream_t stream) {
    const int64_t n = (int64_t)t.n_shard * k.crop_y * k.crop_x * t.spp;
    int64_t g = (n + 255) / 256;
    if (g > 262144) g = 262144;
    if (g < 1) g = 1;
    // draws beyond the ray's own: a scattering medium (volume.py:159) or the ratio / delta sensor
    const bool scat = k.sig_s != 0.0f || k.sensor_type != TVAM_SENSOR_DDA;
#define TVAM_SF_LAUNCH(M)                                                                                          \
    if (scat)                                                                                                      \
        hipLaunchKernelGGL((tvam_surface_kernel<M, true>), dim3((unsigned)g), dim3(256), 0, stream, k, t, pat, idxmap, \
                           gin, vols, out, counter);                                                               \
    else                                                                                                           \
        hipLaunchKernelGGL((tvam_surface_kernel<M, false>), dim3((unsigned)g), dim3(256), 0, stream, k, t, pat, idxmap, \
                           gin, vols, out, counter);
    switch (mode) {
        case TVAM_MODE_FWD: TVAM_SF_LAUNCH(TVAM_MODE_FWD) break;
        case TVAM_MODE_ADJ: TVAM_SF_LAUNCH(TVAM_MODE_ADJ) break;
        default: TVAM_SF_LAUNCH(TVAM_MODE_COUNT)
    }
#undef TVAM_SF_LAUNCH
    return hipGetLastError();
}

hipError_t tvam_launch_general_paths(int mode, const TvamConsts& k, const TvamTiles& t, const float* pat,
                                     const int32_t* idxmap, const float* gin, float* out,
                                     unsigned long long* counter, hipStream_t stream) {
    const int64_t n = (int64_t)t.n_shard * k.crop_y * k.crop_x * t.spp;
    int64_t g = (n + 255) / 256;
    if (g > 262144) g = 262144;
    if (g < 1) g = 1;
    switch (mode) {
        case TVAM_MODE_FWD:
            hipLaunchKernelGGL(tvam_path_kernel<TVAM_MODE_FWD>, dim3((unsigned)g), dim3(256), 0, stream, k, t, pat,
                               idxmap, gin, out, counter);
            break;
        case TVAM_MODE_ADJ:
            hipLaunchKernelGGL(tvam_path_kernel<TVAM_MODE_ADJ>, dim3((unsigned)g), dim3(256), 0, stream, k, t, pat,
                               idxmap, gin, out, counter);
            break;
        default:
            hipLaunchKernelGGL(tvam_path_kernel<TVAM_MODE_COUNT>, dim3((unsigned)g), dim3(256), 0, stream, k, t, pat,
                               idxmap, gin, out, counter);
    }
    return hipGetLastError();
}

hipError_t tvam_launch_scale_volumes(int64_t n, const float* vols, float* dose, hipStream_t stream) {
    const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 16384);
    hipLaunchKernelGGL(tvam_scale_volumes_kernel, dim3(g), dim3(256), 0, stream, n, vols, dose);
    return hipGetLastError();
}

hipError_t tvam_launch_volumes(const TvamConsts& k, uint32_t sample_count, float* volumes, hipStream_t stream) {
    float3 mb0 = make_float3(TVAM_INF, TVAM_INF, TVAM_INF), mb1 = make_float3(-TVAM_INF, -TVAM_INF, -TVAM_INF);
    // the mesh bbox on the host copy is not kept: read it back from the device triangles
    std::vector<float> h((size_t)k.n_tgt * 9);
    hipError_t e = hipMemcpy(h.data(), k.tgt, h.size() * sizeof(float), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    for (size_t i = 0; i < h.size(); i += 3) {
        mb0.x = fminf(mb0.x, h[i]);
        mb0.y = fminf(mb0.y, h[i + 1]);
        mb0.z = fminf(mb0.z, h[i + 2]);
        mb1.x = fmaxf(mb1.x, h[i]);
        mb1.y = fmaxf(mb1.y, h[i + 1]);
        mb1.z = fmaxf(mb1.z, h[i + 2]);
    }
    // per-triangle bounding boxes, grown by 1e-4 of the mesh extent (+ an absolute 1e-6)
    const float ext = fmaxf(fmaxf(mb1.x - mb0.x, mb1.y - mb0.y), mb1.z - mb0.z);
    const float grow = 1e-4f * ext + 1e-6f;
    std::vector<float> box((size_t)k.n_tgt * 6);
    for (int i = 0; i < k.n_tgt; ++i) {
        const float* t = h.data() + 9 * (size_t)i;
        for (int a = 0; a < 3; ++a) {
            box[6 * (size_t)i + a] = fminf(fminf(t[a], t[3 + a]), t[6 + a]) - grow;
            box[6 * (size_t)i + 3 + a] = fmaxf(fmaxf(t[a], t[3 + a]), t[6 + a]) + grow;
        }
    }
    float* d_box = nullptr;
    if ((e = hipMalloc((void**)&d_box, box.size() * sizeof(float))) != hipSuccess) return e;
    if ((e = hipMemcpy(d_box, box.data(), box.size() * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess) {
        (void)hipFree(d_box);
        return e;
    }
    const int64_t V = (int64_t)k.res[0] * k.res[1] * k.res[2];
    const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>((V + 255) / 256, 1), 1 << 20);
    hipLaunchKernelGGL(tvam_volume_kernel, dim3(g), dim3(256), 0, stream, k, mb0, mb1, sample_count, d_box, volumes);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    (void)hipFree(d_box);
    return e;
}

hipError_t tvam_launch_discretize(const TvamConsts& k, const float* h_tris, float* occ, hipStream_t stream) {
    float3 mb0 = make_float3(TVAM_INF, TVAM_INF, TVAM_INF), mb1 = make_float3(-TVAM_INF, -TVAM_INF, -TVAM_INF);
    for (size_t i = 0; i < (size_t)k.n_tgt * 9; i += 3) {  // the target bbox (utils.py:98, :118)
        mb0.x = fminf(mb0.x, h_tris[i]);
        mb0.y = fminf(mb0.y, h_tris[i + 1]);
        mb0.z = fminf(mb0.z, h_tris[i + 2]);
        mb1.x = fmaxf(mb1.x, h_tris[i]);
        mb1.y = fmaxf(mb1.y, h_tris[i + 1]);
        mb1.z = fmaxf(mb1.z, h_tris[i + 2]);
    }
    const int64_t V = (int64_t)k.res[0] * k.res[1] * k.res[2];
    const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>((V + 255) / 256, 1), 1 << 20);
    hipLaunchKernelGGL(tvam_discretize_kernel, dim3(g), dim3(256), 0, stream, k, mb0, mb1, occ);
    return hipGetLastError();
}

hipError_t tvam_launch_frozen(int mode, const TvamConsts& k, const TvamTiles& t, const float* pat,
                              const int32_t* idxmap, const float* gin, float* out, unsigned long long* counter,
                              hipStream_t stream) {
    if (!t.frozen || !t.frozen_n) return hipErrorInvalidValue;
    const int64_t n = (int64_t)t.n_shard * k.crop_y * k.crop_x * t.spp;
    int64_t g = (n + 255) / 256;
    if (g > 4096) g = 4096;  // the list is short; a scan (list overflow) grid-strides
    if (g < 1) g = 1;
    switch (mode) {
        case TVAM_MODE_FWD:
            hipLaunchKernelGGL(tvam_frozen_kernel<TVAM_MODE_FWD>, dim3((unsigned)g), dim3(256), 0, stream, k, t, pat,
                               idxmap, gin, out, counter);
            break;
        case TVAM_MODE_ADJ:
            hipLaunchKernelGGL(tvam_frozen_kernel<TVAM_MODE_ADJ>, dim3((unsigned)g), dim3(256), 0, stream, k, t, pat,
                               idxmap, gin, out, counter);
            break;
        default:
            hipLaunchKernelGGL(tvam_frozen_kernel<TVAM_MODE_COUNT>, dim3((unsigned)g), dim3(256), 0, stream, k, t,
                               pat, idxmap, gin, out, counter);
    }
    return hipGetLastError();
}

hipError_t tvam_launch_scatter_paths(int mode, const TvamConsts& k, const TvamTiles& t, const float* pat,
                                     const int32_t* idxmap, const float* gin, float* out,
                                     unsigned long long* counter, hipStream_t stream) {
    const int64_t n = (int64_t)t.n_shard * k.crop_y * k.crop_x * t.spp;
    int64_t g = (n + 255) / 256;
    if (g > 262144) g = 262144;
    if (g < 1) g = 1;
    const TvamSegBuf none{};
    switch (mode) {
        case TVAM_MODE_FWD:
            hipLaunchKernelGGL(tvam_scatter_kernel<TVAM_MODE_FWD>, dim3((unsigned)g), dim3(256), 0, stream, k, t, pat,
                               idxmap, gin, out, counter, none);
            break;
        case TVAM_MODE_ADJ:
            hipLaunchKernelGGL(tvam_scatter_kernel<TVAM_MODE_ADJ>, dim3((unsigned)g), dim3(256), 0, stream, k, t, pat,
                               idxmap, gin, out, counter, none);
            break;
        default:
            hipLaunchKernelGGL(tvam_scatter_kernel<TVAM_MODE_COUNT>, dim3((unsigned)g), dim3(256), 0, stream, k, t,
                               pat, idxmap, gin, out, counter, none);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Brick bins: fill (segment, brick) pairs, sort by brick, march per brick.
// ---------------------------------------------------------------------------
#include <hipcub/hipcub.hpp>

namespace {

__device__ __forceinline__ void sc_unpack(const float4 a, const float4 b, const float4 cf, SegDda& q, float& w) {
    const int2 c = make_int2(__float_as_int(cf.x), __float_as_int(cf.y));
    q.t_start = a.x;
    q.tau_end = a.y;
    q.dtm0[0] = a.z;
    q.dtm0[1] = a.w;
    q.dtm0[2] = b.x;
    const float tsv[3] = {b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        q.step[i] = tsv[i] < 0.0f ? -1 : 1;
        q.ts[i] = fabsf(tsv[i]);
    }
    q.sv[0] = c.x & 0x7ff;
    q.sv[1] = (c.x >> 11) & 0x7ff;
    q.sv[2] = (c.x >> 22) & 0x3ff;
    w = __int_as_float(c.y);
}

// (brick, entry) pairs; an entry is one (segment, brick) crossing, entries of
// a segment are contiguous from off[slot].  The value is the segment slot.
// Lane balance: a workgroup takes TVAM_FILL_T consecutive slots, orders them in LDS by their
// brick count (counting sort, longest first; empty slots last) and its lanes walk them in that
// order, so the lanes of a wave walk segments of similar length.  In slot order the lanes of a
// wave idled on empty slots and on the wave's longest walk (lane utilisation 0.12).  Every
// slot writes its own entries [off[slot], off[slot] + m[slot]): the order does not change the
// output.
#define TVAM_FILL_T 1024
__global__ __launch_bounds__(256) void tvam_bin_fill_kernel(TvamConsts k, TvamSegBuf sb, const uint32_t* __restrict__ off,
                                                            int64_t nslots, uint32_t* __restrict__ keys,
                                                            uint32_t* __restrict__ vals, int cbits) {
    constexpr int U = TVAM_FILL_T / 256;
    __shared__ uint32_t s_cnt[256];
    __shared__ uint32_t s_ord[TVAM_FILL_T];
    for (int64_t t0 = (int64_t)blockIdx.x * TVAM_FILL_T; t0 < nslots; t0 += (int64_t)gridDim.x * TVAM_FILL_T) {
        s_cnt[threadIdx.x] = 0;
        __syncthreads();
        uint32_t bin[U], rk[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t s = t0 + threadIdx.x + u * 256;
            const uint32_t m = s < nslots ? sb.m[s] : 0u;
            bin[u] = m == 0 ? 255u : 254u - min(m - 1u, 254u);  // longest first, empty slots last (bin 255)
            rk[u] = atomicAdd(&s_cnt[bin[u]], 1u);
        }
        __syncthreads();
        if (threadIdx.x < 64) {  // exclusive scan of the 256 bin counts (one wave, 4 bins per lane)
            const int l = threadIdx.x;
            uint32_t c[4], tot = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                c[j] = s_cnt[4 * l + j];
                tot += c[j];
            }
            uint32_t inc = tot;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t v = __shfl_up(inc, d, 64);
                if (l >= d) inc += v;
            }
            uint32_t run = inc - tot;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t cj = c[j];
                s_cnt[4 * l + j] = run;
                run += cj;
            }
        }
        __syncthreads();
        // non-empty slots: those before bin 255's start
        const uint32_t nne = s_cnt[255];
#pragma unroll
        for (int u = 0; u < U; ++u) s_ord[s_cnt[bin[u]] + rk[u]] = threadIdx.x + u * 256;
        __syncthreads();
        for (uint32_t r = threadIdx.x; r < nne; r += 256) {
            const int64_t s = t0 + s_ord[r];
            SegDda q;
            float w;
            sc_unpack(sb.r[TVAM_REC_F4 * s], sb.r[TVAM_REC_F4 * s + 1], sb.r[TVAM_REC_F4 * s + 2], q, w);
            uint32_t o = off[s];
            const uint32_t oe = o + sb.m[s];  // the record writer's closed-form count (sc_brick_count)
            // visits per unit length: one per voxel-face crossing of each moving axis
            float rate = 0.0f;
#pragma unroll
            for (int a = 0; a < 3; ++a) rate += q.ts[a] < TVAM_INF ? 1.0f / q.ts[a] : 0.0f;
            uint32_t klast = 0u;
            sc_walk_bricks(k, q, [&](int bid, float ta, float tb) {
                // low key bits: a class of the predicted in-brick visit count, so that the lanes of a
                // wave of the brick kernel march entries of similar length
                // classes of 4 visits (16 classes) or 8 (8 classes)
                const int cls = (int)fminf((float)((1 << cbits) - 1),
                                           fmaxf(tb - ta, 0.0f) * rate * (0.015625f * (float)(1 << cbits)));
                klast = ((uint32_t)bid << cbits) | (uint32_t)cls;
                if (o < oe) {
                    keys[o] = klast;
                    vals[o] = (uint32_t)s;
                }
                ++o;
            });
            // the walk and the count disagree (never, by construction: counted for the tests,
            // tvam_plan_bin_stats): the slot keeps its own range, short ranges padded with null
            // entries (TVAM_ENT_NULL: marched with weight 0)
            if (o != oe) atomicAdd(sb.bad, 1u);
            for (; o < oe; ++o) {
                keys[o] = klast;
                vals[o] = (uint32_t)s | TVAM_ENT_NULL;
            }
        }
        __syncthreads();
    }
}

// Counting-sort fill (no radix sort): workgroup b of the record writer's grid walks the same
// paths' segments again (its 256-path groups g = b, b + G, ...; in rounds of TVAM_FILL_T slots
// ordered by brick count, as tvam_bin_fill_kernel) and writes each (segment, brick) entry at its
// brick's next position among this workgroup's (base: the scan of the writer's per-(brick,
// workgroup) counts, cursors in LDS).  An entry is its slot | class << 28 (the class of its
// predicted in-brick visit count, 16 classes: the brick kernel orders each wave's entries by it).
// The order of one workgroup's entries within a brick follows its LDS atomics: the forward sums
// them exactly (int64 fixed point) and the adjoint reduces each pixel's partials in (slot, brick)
// order through inv (inv[off[slot] + j] = position of the slot's j-th entry), so results do
// not depend on it.
#define TVAM_ENT_SLOT_BITS 28
__global__ __launch_bounds__(256) void tvam_bin_fill2_kernel(TvamConsts k, TvamSegBuf sb, int64_t nslots,
                                                             const uint32_t* __restrict__ base,
                                                             uint32_t* __restrict__ ent,
                                                             const uint32_t* __restrict__ off,
                                                             uint32_t* __restrict__ inv) {
    constexpr int U = TVAM_FILL_T / 256;
    extern __shared__ uint32_t s_cur[];  // [nbricks]
    __shared__ uint32_t s_cnt[256];
    __shared__ uint32_t s_ord[TVAM_FILL_T];
    const int G = (int)gridDim.x, beta = (int)blockIdx.x;
    for (int b = threadIdx.x; b < sb.nbricks; b += 256) s_cur[b] = base[(size_t)b * G + beta];
    const int64_t gslots = (int64_t)256 * sb.slots;  // one writer group: 256 paths
    for (int64_t s0 = (int64_t)beta * gslots; s0 < nslots; s0 += (int64_t)G * gslots) {
        const int64_t s1 = min(nslots, s0 + gslots);
        for (int64_t t0 = s0; t0 < s1; t0 += TVAM_FILL_T) {
            __syncthreads();  // s_cur ready; the previous round's s_ord consumed
            s_cnt[threadIdx.x] = 0;
            __syncthreads();
            uint32_t bin[U], rk[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t si = t0 + threadIdx.x + u * 256;
                const uint32_t m = si < s1 ? sb.m[si] : 0u;
                bin[u] = m == 0 ? 255u : 254u - min(m - 1u, 254u);  // longest first, empty slots last
                rk[u] = atomicAdd(&s_cnt[bin[u]], 1u);
            }
            __syncthreads();
            if (threadIdx.x < 64) {  // exclusive scan of the 256 bin counts
                const int l = threadIdx.x;
                uint32_t c[4], tot = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    c[j] = s_cnt[4 * l + j];
                    tot += c[j];
                }
                uint32_t inc = tot;
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t v = __shfl_up(inc, d, 64);
                    if (l >= d) inc += v;
                }
                uint32_t run = inc - tot;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t cj = c[j];
                    s_cnt[4 * l + j] = run;
                    run += cj;
                }
            }
            __syncthreads();
            const uint32_t nne = s_cnt[255];
#pragma unroll
            for (int u = 0; u < U; ++u) s_ord[s_cnt[bin[u]] + rk[u]] = threadIdx.x + u * 256;
            __syncthreads();
            for (uint32_t r = threadIdx.x; r < nne; r += 256) {
                const int64_t si = t0 + s_ord[r];
                SegDda q;
                float w;
                sc_unpack(sb.r[TVAM_REC_F4 * si], sb.r[TVAM_REC_F4 * si + 1], sb.r[TVAM_REC_F4 * si + 2], q, w);
                uint32_t o = inv ? off[si] : 0u;
                float rate = 0.0f;
#pragma unroll
                for (int a = 0; a < 3; ++a) rate += q.ts[a] < TVAM_INF ? 1.0f / q.ts[a] : 0.0f;
                sc_walk_bricks(k, q, [&](int bid, float ta, float tb) {
                    const int cls = (int)fminf(15.0f, fmaxf(tb - ta, 0.0f) * rate * 0.25f);  // classes of 4 visits
                    const uint32_t pos = atomicAdd(&s_cur[bid], 1u);
                    ent[pos] = (uint32_t)si | ((uint32_t)cls << TVAM_ENT_SLOT_BITS);
                    if (inv) inv[o++] = pos;
                });
            }
        }
    }
}

// bstart[b] = the first entry of brick b (the scan of the per-(brick, workgroup) counts at
// workgroup 0), bstart[nbricks] = the total
__global__ void tvam_bin_bstart_kernel(const uint32_t* __restrict__ base, int G, int nbricks,
                                       uint32_t* __restrict__ bstart) {
    for (int b = blockIdx.x * blockDim.x + threadIdx.x; b <= nbricks; b += gridDim.x * blockDim.x)
        bstart[b] = base[(size_t)b * G];
}

// Adjoint of the counting-sort bins: per DMD pixel of the chunk (one wave), the sum of its slots'
// entry partials in (slot, brick) order -- inv lists each slot's entry positions contiguously
// from off[slot], and a pixel's slots are contiguous -- added to the pattern gradient.
__global__ __launch_bounds__(256) void tvam_bin_reduce2_kernel(TvamSegBuf sb, int spp, const uint32_t* __restrict__ off,
                                                               const uint32_t* __restrict__ inv,
                                                               const float* __restrict__ part,
                                                               const int32_t* __restrict__ idxmap,
                                                               float* __restrict__ grad) {
    const int64_t l0 = sb.p0 / spp, l1 = sb.p1 / spp;
    const int64_t pslots = (int64_t)spp * sb.slots;
    const int lane = (int)(threadIdx.x & 63);
    const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, ws = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t local = l0 + w0; local < l1; local += ws) {
        const int64_t i = local - l0;
        const uint32_t a = off[i * pslots], b = off[(i + 1) * pslots];
        if (a == b) continue;  // (uniform over the wave)
        float acc = 0.0f;
        for (uint32_t e = a + (uint32_t)lane; e < b; e += 64) acc += part[inv[e]];
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
        if (lane == 0) {
            int64_t act = local;
            if (idxmap) {
                act = idxmap[local];
                if (act < 0) continue;
            }
            grad[act] += acc;
        }
    }
}

__global__ void tvam_bin_start_kernel(const uint32_t* __restrict__ keys, int64_t n, int nbricks, uint32_t kmask,
                                      int cbits, uint32_t* __restrict__ bstart) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x) {
        const int kc = i < n ? (int)((keys[i] & kmask) >> cbits) : nbricks;
        const int kp = i > 0 ? (int)((keys[i - 1] & kmask) >> cbits) : -1;
        for (int b = kp + 1; b <= kc; ++b) bstart[b] = (uint32_t)i;  // bricks (kp, kc] start here
    }
}

// One workgroup per brick.  Forward (ACC 0: exact int64 fixed point; every add
// rounds to int32 with a per-brick scale 2^e from max |w| * the largest
// per-visit weight min(1, st sqrt3 h), so the step is 2^-30 of the largest
// single add and the int64 sums cannot overflow; ACC 1: float adds): the brick's visits
// added in LDS, then dose += tile (the brick is this launch's alone).
// Adjoint (ACC 2): the brick's grad * inv_vol staged in LDS, each entry's weighted gather
// written at its own sorted position e with its DMD pixel (the chunk-local pixel of its slot,
// slot / pslots): coalesced stores, no atomics.  tvam_scatter_binned then sorts the
// (pixel, partial) pairs by pixel and sums each pixel's run (a partial stored at the
// segment's own entry index instead -- one random 4-byte store per entry -- took 57 % of
// this kernel's time on config 4).
//
// WS (counting-sort bins): vals are tvam_bin_fill2_kernel's entries (slot | class << 28, a brick's
// entries in fill order).  Each wave takes batches of 256 of its brick's entries, orders a batch
// by class in LDS (ballot counting sort, longest first; no workgroup barrier) and marches its lanes'
// four entries in that order, so the lanes of a step march similar lengths.
template <int ACC, int NT, bool WS = false>
__global__ __launch_bounds__(NT) void tvam_bin_march_kernel(TvamConsts k, TvamSegBuf sb,
                                                             const uint32_t* __restrict__ vals,
                                                             const uint32_t* __restrict__ bstart,
                                                             float* __restrict__ dose, const float* __restrict__ gin,
                                                             uint32_t pslots, uint32_t* __restrict__ ppix,
                                                             float* __restrict__ part) {
    constexpr int NV = TVAM_BX * TVAM_BY * TVAM_BZ;
    __shared__ __attribute__((aligned(16))) unsigned char smem[NV * (ACC == 0 ? 8 : 4)];
    constexpr int WSB = 256;  // entries per wave batch (WS): the batch order in LDS as byte offsets (4 KB;
                              // the adjoint's two 64 KB tiles per CU stay resident)
    __shared__ uint8_t s_wo[WS ? (NT / 64) * WSB : 1];
    long long* ltile = reinterpret_cast<long long*>(smem);
    float* ftile = reinterpret_cast<float*>(smem);
    const int nbx = sc_nbr(k, 0), nby = sc_nbr(k, 1);
    const int bid = blockIdx.x;
    const uint32_t e0 = bstart[bid], e1 = bstart[bid + 1];
    if (e0 == e1) return;
    const int bx = bid % nbx, by = (bid / nbx) % nby, bz = bid / (nbx * nby);
    const int lo[3] = {bx * TVAM_BX, by * TVAM_BY, bz * TVAM_BZ};
    const int hi[3] = {min(lo[0] + TVAM_BX, k.res[0]), min(lo[1] + TVAM_BY, k.res[1]), min(lo[2] + TVAM_BZ, k.res[2])};
    const int wx = hi[0] - lo[0], wy = hi[1] - lo[1], wz = hi[2] - lo[2];
    const int sy = TVAM_BX, sz = TVAM_BX * TVAM_BY;
    const bool w2 = k.sig_t * 1.7320508f * fmaxf(fmaxf(k.h[0], k.h[1]), k.h[2]) < TVAM_W2_MAX3;
    float scale = 1.0f;
    if (ACC == 0) {
        // per-add bound: each add rounds to int32 (one v_cvt), the int64 sums cannot overflow; the
        // chunk's largest |weight| (from the record writer: no gather pass over the brick's entries)
        for (int i = threadIdx.x; i < NV; i += NT) ltile[i] = 0;
        __syncthreads();
        const float tot = __uint_as_float(*sb.wmax);
        const float hmax = fmaxf(fmaxf(k.h[0], k.h[1]), k.h[2]);
        const float bound = tot * fminf(1.0f, k.sig_t * 1.7320508f * hmax) * 1.001f;
        if (bound > 0.0f && isfinite(bound)) {
            int ex;
            frexpf(bound, &ex);
            ex = 30 - ex;
            ex = ex > 126 ? 126 : (ex < -126 ? -126 : ex);
            scale = ldexpf(1.0f, ex);
        }
    } else if (ACC == 1) {
        for (int i = threadIdx.x; i < NV; i += NT) ftile[i] = 0.0f;
        __syncthreads();
    } else {
        int nonzero = 0;
        for (int i = threadIdx.x; i < wx * wy * wz; i += NT) {
            const int x = i % wx, y = (i / wx) % wy, z = i / (wx * wy);
            const size_t g = ((size_t)(lo[2] + z) * k.res[1] + (lo[1] + y)) * k.res[0] + (lo[0] + x);
            const float v = gin[g] * k.inv_vol;  // volume.py:130
            ftile[z * sz + y * sy + x] = v;
            nonzero |= v != 0.0f ? 1 : 0;
        }
        if (!__syncthreads_or(nonzero) && !WS) {
            // an all-zero gradient brick (the thresholded loss is flat wherever the dose meets its
            // bounds): every entry's partial is exactly 0 -- written with its pixel for the sort
            for (uint32_t e = e0 + threadIdx.x; e < e1; e += NT) {
                part[e] = 0.0f;
                ppix[e] = (vals[e] & ~TVAM_ENT_NULL) / pslots;
            }
            return;
        }
    }
    // Load pipeline over this thread's entries e, e + S, e + 2S, ... (S = NT), unrolled by two with
    // two record register sets: while one entry marches, the records of the next are in flight and
    // the slot of the one after (vals -> record is two dependent gathers).  Indices are clamped to the brick's last entry, so every load is
    // issued unconditionally (no branch around it: the compiler's vmcnt waits then count only the
    // loads a use needs; a single register set with conditional loads had it wait for the next
    // entry's records at the top of every entry).
    constexpr uint32_t S = NT;
    const uint32_t et = e0 + threadIdx.x, el = e1 - 1;
    struct Ent {
        float4 a, b, c;
        uint32_t slot;
    };
    auto load = [&](uint32_t v, uint32_t e, Ent& r) {
        (void)e;
        const uint32_t slot = v & ~TVAM_ENT_NULL;
        r.a = sb.r[TVAM_REC_F4 * slot];
        r.b = sb.r[TVAM_REC_F4 * slot + 1];
        r.c = sb.r[TVAM_REC_F4 * slot + 2];
        r.slot = v;
    };
    auto run = [&](const Ent& r, uint32_t e) {
        SegDda q;
        float w;
        sc_unpack(r.a, r.b, r.c, q, w);
        if (r.slot & TVAM_ENT_NULL) w = 0.0f;  // a null entry (tvam_bin_fill_kernel's padding)
        const float ws = w * scale;
        float acc = 0.0f;
        // adjoint: each visit's LDS value is consumed one visit later, so its read latency overlaps
        // the next DDA step (the sum keeps its order: bit-identical)
        float pc = 0.0f, pv = 0.0f;
        auto visit = [&](int li, float c) {
            if (ACC == 0) {
                __hip_atomic_fetch_add(&ltile[li], (long long)__float2int_rn(ws * c), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if (ACC == 1) {
                __hip_atomic_fetch_add(&ftile[li], w * c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                const float v = ftile[li];
                acc = fmaf(pc, pv, acc);
                pc = c;
                pv = v;
            }
        };
        if (w2)
            sc_brick_march<true>(k, q, lo, hi, visit);
        else
            sc_brick_march<false>(k, q, lo, hi, visit);
        if (ACC == 2) {
            part[e] = w * fmaf(pc, pv, acc);
            if (!WS) ppix[e] = (r.slot & ~TVAM_ENT_NULL) / pslots;
        }
    };
    if constexpr (WS) {
        constexpr int U = WSB / 64, NW = NT / 64;
        constexpr uint32_t SMASK = (1u << TVAM_ENT_SLOT_BITS) - 1u;
        const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
        uint8_t* so = s_wo + wv * WSB;
        const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));  // the lanes below this one
        for (uint32_t b0 = e0 + (uint32_t)wv * WSB; b0 < e1; b0 += (uint32_t)NW * WSB) {
            uint32_t v[U];
            int key[U], pos[U];
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const uint32_t idx = b0 + (uint32_t)(j * 64 + lane);
                const bool ok = idx < e1;
                v[j] = ok ? vals[idx] : 0u;
                key[j] = ok ? 15 - (int)(v[j] >> TVAM_ENT_SLOT_BITS) : 16;  // longest class first, past e1 last
                pos[j] = 0;
            }
            int run_ = 0;
            for (int c = 0; c <= 16; ++c) {
#pragma unroll
                for (int j = 0; j < U; ++j) {
                    const uint64_t m = __ballot(key[j] == c);
                    if (key[j] == c) pos[j] = run_ + (int)__popcll(m & lt);
                    run_ += (int)__popcll(m);
                }
            }
#pragma unroll
            for (int j = 0; j < U; ++j) so[pos[j]] = (uint8_t)(j * 64 + lane);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t nval = min(e1 - b0, (uint32_t)WSB);
            uint32_t sl[U], eo[U];
#pragma unroll
            for (int j = 0; j < U; ++j) {  // the batch's entry at sorted position j * 64 + lane (re-read: L1)
                eo[j] = b0 + (uint32_t)so[j * 64 + lane];
                sl[j] = (uint32_t)(j * 64 + lane) < nval ? vals[eo[j]] & SMASK : 0u;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();  // every lane has read the batch before the next one is written
            Ent rA, rB;
            load(sl[0], 0u, rA);
            load(sl[1], 0u, rB);
            if ((uint32_t)lane < nval) run(rA, eo[0]);
            load(sl[2], 0u, rA);
            if ((uint32_t)(64 + lane) < nval) run(rB, eo[1]);
            load(sl[3], 0u, rB);
            if ((uint32_t)(128 + lane) < nval) run(rA, eo[2]);
            if ((uint32_t)(192 + lane) < nval) run(rB, eo[3]);
        }
    } else if (et < e1) {
        uint32_t sB = vals[min(et + S, el)];
        Ent rA, rB;
        load(vals[et], et, rA);
        for (uint32_t e = et;; e += 2 * S) {
            load(sB, e + S, rB);
            const uint32_t sC = vals[min(e + 2 * S, el)];
            run(rA, e);
            if (e + S >= e1) break;
            load(sC, e + 2 * S, rA);
            sB = vals[min(e + 3 * S, el)];
            run(rB, e + S);
            if (e + 2 * S >= e1) break;
        }
    }
    if (ACC == 2) return;
    __syncthreads();
    const float inv = 1.0f / scale;
    for (int i = threadIdx.x; i < wx * wy * wz; i += NT) {
        const int x = i % wx, y = (i / wx) % wy, z = i / (wx * wy);
        const int li = z * sz + y * sy + x;
        const float v = ACC == 0 ? (float)ltile[li] * inv : ftile[li];
        if (v != 0.0f) {
            const size_t g = ((size_t)(lo[2] + z) * k.res[1] + (lo[1] + y)) * k.res[0] + (lo[0] + x);
            dose[g] += v;
        }
    }
}

// Adjoint: per DMD pixel of the chunk, the sum of its samples' segment-brick partials (its
// run [pstart[i], pstart[i + 1]) of the pixel-sorted partials; one wave per pixel, coalesced
// reads, a fixed butterfly order), added to the pattern gradient after the first-segment
// kernels (same stream, one writer per pixel).
__global__ __launch_bounds__(256) void tvam_bin_reduce_kernel(TvamSegBuf sb, int spp, const uint32_t* __restrict__ pstart,
                                                              const float* __restrict__ part,
                                                              const int32_t* __restrict__ idxmap,
                                                              float* __restrict__ grad) {
    const int64_t l0 = sb.p0 / spp, l1 = sb.p1 / spp;
    const int lane = (int)(threadIdx.x & 63);
    const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, ws = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t local = l0 + w0; local < l1; local += ws) {
        const int64_t i = local - l0;
        const uint32_t a = pstart[i], b = pstart[i + 1];
        if (a == b) continue;  // (uniform over the wave)
        float acc = 0.0f;
        for (uint32_t e = a + (uint32_t)lane; e < b; e += 64) acc += part[e];
        for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
        if (lane == 0) {
            int64_t act = local;
            if (idxmap) {
                act = idxmap[local];
                if (act < 0) continue;
            }
            grad[act] += acc;
        }
    }
}

// Cached forward bins, new pattern: each record's weight em * att with em of the new pattern,
// the same expression as tvam_scatter_kernel<EMIT> (bit-identical records), and the chunk's
// largest |weight| (EMIT clears the attenuation of slots without a segment: the same max as
// EMIT's).  32-bit slot indices (a chunk holds < 2^31 slots; chunks are whole pixels, so a slot's
// pixel is the chunk's first pixel + s / (spp * slots)), one block-max atomic per workgroup.
__global__ __launch_bounds__(256) void tvam_bin_reweight_kernel(TvamConsts k, TvamSegBuf sb, int spp,
                                                                const float* __restrict__ pat) {
    const uint32_t ns = (uint32_t)((sb.p1 - sb.p0) * sb.slots), per = (uint32_t)spp * (uint32_t)sb.slots;
    const float* __restrict__ pc = pat + sb.p0 / spp;
    float wmax = 0.0f;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < ns; s += gridDim.x * blockDim.x) {
        const float em = pc[s / per] * k.wscale * k.inv_vol;
        float* c = reinterpret_cast<float*>(&sb.r[TVAM_REC_F4 * (size_t)s + 2]);
        const float w = em * c[2];  // c[2] = 0 for slots without a segment
        c[1] = w;
        wmax = fmaxf(wmax, fabsf(w));
    }
    sc_block_max(wmax, sb.wmax);
}

template <typename T>
hipError_t grow(T** p, int64_t& cap, int64_t need) {
    if (need <= cap) return hipSuccess;
    (void)hipFree(*p);
    *p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc((void**)p, (size_t)need * sizeof(T));
    if (e == hipSuccess) cap = need;
    return e;
}

}  // namespace

void tvam_bin_scratch_free(TvamBinScratch& s) {
    (void)hipFree(s.sb.r);
    (void)hipFree(s.sb.m);
    (void)hipFree(s.sb.wmax);
    (void)hipFree(s.sb.bad);
    (void)hipFree(s.off);
    for (int i = 0; i < 2; ++i) {
        (void)hipFree(s.keys[i]);
        (void)hipFree(s.vals[i]);
    }
    (void)hipFree(s.bstart);
    (void)hipFree(s.temp);
    (void)hipFree(s.part);
    (void)hipFree(s.hist);
    (void)hipFree(s.hbase);
    for (auto& c : s.fc) {
        (void)hipFree(c.r);
        (void)hipFree(c.vals);
        (void)hipFree(c.bstart);
    }
    if (s.bad_ev) (void)hipEventSynchronize(s.bad_ev);
    (void)hipHostFree(s.bad_host);
    if (s.bad_ev) (void)hipEventDestroy(s.bad_ev);
    s = TvamBinScratch{};
}

hipError_t tvam_scatter_binned(int mode, const TvamConsts& k, const TvamTiles& t, const float* pat,
                               const int32_t* idxmap, const float* gin, float* out, TvamBinScratch& s,
                               hipStream_t stream) {
    for (int i = 0; i < 5; ++i) s.st[i] = 0;  // stats of this call, also when it bins nothing
    // an earlier call's count check, if its copy has landed: a slot whose brick walk disagreed with
    // the writer's closed-form count (never, by construction) may have dropped entries -- fail loudly
    if (s.bad_pending && hipEventQuery(s.bad_ev) == hipSuccess) {
        s.bad_pending = false;
        if (*s.bad_host) return hipErrorIllegalState;
    }
    const int nsurf = k.vial_type == 0 ? 1 : 2;
    const int slots = k.max_depth - nsurf - 1;  // later medium segments per path
    if (slots <= 0) return hipSuccess;
    if (k.res[0] > 2048 || k.res[1] > 2048 || k.res[2] > 1024) return hipErrorNotSupported;
    const bool adj = mode == TVAM_MODE_ADJ;
    const int nbx = (k.res[0] + TVAM_BX - 1) / TVAM_BX, nby = (k.res[1] + TVAM_BY - 1) / TVAM_BY,
              nbz = (k.res[2] + TVAM_BZ - 1) / TVAM_BZ;
    const int nbricks = nbx * nby * nbz;
    // brick-march workgroup: 1024 threads double the waves per SIMD under the one 128 KB int64
    // tile per CU (forward) and the two 64 KB gradient tiles (adjoint); TVAM_BIN_NT=512 for A/B
    static const int bin_nt = tvam_knob("TVAM_BIN_NT", 1024) == 512 ? 512 : 1024;
    int bits = 1;
    while ((1 << bits) < nbricks) ++bits;
    // length classes: 16, or 8 / 4 where that keeps the sort key within 16 bits (two radix passes
    // instead of three; config 4: 4225 bricks); TVAM_BIN_CBITS overrides (2..4)
    int cbits = bits <= 14 ? std::min(4, 16 - bits) : TVAM_BIN_CLASS_BITS;
    if (const int cb = tvam_knob("TVAM_BIN_CBITS", 0)) cbits = std::min(4, std::max(2, cb));
    bits += cbits;
    const uint32_t kmask = bits >= 32 ? 0xffffffffu : ((1u << bits) - 1u);
    const int spp = (int)t.spp;
    const int64_t npaths = (int64_t)t.n_shard * k.crop_y * k.crop_x * spp;
    // chunk of paths: a whole number of pixels (the adjoint reduces a pixel's samples together)
    int64_t max_slots = (int64_t)1 << 27;  // 128M slots (TVAM_BIN_CHUNK_SLOTS: smaller, for tests)
    if (const int cs = tvam_knob("TVAM_BIN_CHUNK_SLOTS", 0)) max_slots = std::max<int64_t>(1, cs);
    int64_t chunk = std::max<int64_t>(1, max_slots / slots);
    chunk = std::max<int64_t>(spp, chunk / spp * spp);
    chunk = std::min(npaths, chunk);
    const int64_t nsl = chunk * slots;
    if (nsl >= ((int64_t)1 << 31)) return hipErrorNotSupported;  // 32-bit slot indices (reweight)
    // counting-sort bins (TVAM_BIN_SORT=0; the radix sort stays the default): the record writer
    // counts each workgroup's entries per brick, a scan of those counts places every entry, and each
    // brick wave orders its entries by class itself -- no radix sort of (brick, class) keys and, in
    // the adjoint, none of (pixel, partial) pairs.  Measured on config 4 (profiles/r04/ab3): the
    // sorts' 8.4 ms per chunk go, but the fill's scattered 4-byte entry stores take 10.0 ms instead
    // of 5.6, and the brick marches lose the record-line sharing of the class-sorted fill order
    // (forward 18.8 -> 23.7 ms, adjoint 16.2 -> 20.1 ms per chunk): 0.2856 -> 0.2853 it/s.
    static const bool bin_sort = tvam_knob("TVAM_BIN_SORT", 1) != 0;
    const bool csort = !bin_sort && !s.acc_float && bin_nt == 1024 && nbricks <= 16384 &&
                       nsl <= ((int64_t)1 << TVAM_ENT_SLOT_BITS);
    hipError_t e;
    if (nsl > s.cap_slots) {
        const int keep_float = s.acc_float;
        tvam_bin_scratch_free(s);
        s.acc_float = keep_float;
        if ((e = hipMalloc((void**)&s.sb.r, TVAM_REC_F4 * nsl * sizeof(float4))) != hipSuccess ||
            (e = hipMalloc((void**)&s.sb.m, (nsl + 1) * sizeof(uint32_t))) != hipSuccess ||
            (e = hipMalloc((void**)&s.off, (nsl + 1) * sizeof(uint32_t))) != hipSuccess ||
            (e = hipMalloc((void**)&s.sb.wmax, sizeof(uint32_t))) != hipSuccess ||
            (e = hipMalloc((void**)&s.sb.bad, sizeof(uint32_t))) != hipSuccess ||
            (e = hipHostMalloc((void**)&s.bad_host, sizeof(uint32_t))) != hipSuccess ||
            (e = hipEventCreateWithFlags(&s.bad_ev, hipEventDisableTiming)) != hipSuccess)
            return e;
        *s.bad_host = 0;
        // the fill walks that disagreed with the record writer's brick counts, summed over the calls
        // (bin stats [7])
        if ((e = hipMemsetAsync(s.sb.bad, 0, sizeof(uint32_t), stream)) != hipSuccess) return e;
        s.cap_slots = nsl;
    }
    int64_t capb = s.cap_bricks;
    if ((e = grow(&s.bstart, capb, (int64_t)nbricks + 1)) != hipSuccess) return e;
    s.cap_bricks = (int32_t)capb;
    // forward bin cache: dense pattern sets only (a sparse set's streams follow the set), and not
    // with skip_zero (then the paths depend on the pattern); TVAM_BIN_CACHE=0 turns it off
    const bool cacheable = !adj && !idxmap && !k.skip_zero && tvam_knob("TVAM_BIN_CACHE", 1) != 0;
    if (cacheable) {
        const bool same = s.fc_key && s.fc_seed == t.seed && s.fc_spp == t.spp && s.fc_chunk == chunk &&
                          s.fc_npaths == npaths && std::memcmp(&s.fc_k, &k, sizeof(TvamConsts)) == 0;
        if (!same) {
            for (auto& c : s.fc) c.valid = false;
            s.fc_key = true;
            s.fc_k = k;
            s.fc_seed = t.seed;
            s.fc_spp = t.spp;
            s.fc_chunk = chunk;
            s.fc_npaths = npaths;
        }
        const size_t nch = (size_t)((npaths + chunk - 1) / chunk);
        if (s.fc.size() < nch) s.fc.resize(nch);
    }
    // a chunk is cached while an eighth of the device memory (+ 1 GB) stays free after its buffers
    // (the call's other buffers, e.g. the ray records and this scratch, are allocated before)
    auto room = [](size_t bytes) {
        size_t fr = 0, tot = 0;
        return hipMemGetInfo(&fr, &tot) == hipSuccess && fr > bytes + tot / 8 + ((size_t)1 << 30);
    };
    // forward brick march: int64 fixed point (default) or float LDS adds (TVAM_BIN_FLOAT)
    auto march_fwd = [&](const TvamSegBuf& sb, const uint32_t* vals, const uint32_t* bstart, bool ws) {
        const dim3 grid((unsigned)nbricks), blk(bin_nt);
        tvam_kt_begin(stream, TVAM_KT_BRICK);
        if (ws)  // counting-sort entries (csort: int64 tiles, 1024 threads)
            hipLaunchKernelGGL((tvam_bin_march_kernel<0, 1024, true>), grid, dim3(1024), 0, stream, k, sb, vals,
                               bstart, out, nullptr, 0u, nullptr, nullptr);
        else if (s.acc_float && bin_nt == 1024)
            hipLaunchKernelGGL((tvam_bin_march_kernel<1, 1024>), grid, blk, 0, stream, k, sb, vals, bstart, out,
                               nullptr, 0u, nullptr, nullptr);
        else if (s.acc_float)
            hipLaunchKernelGGL((tvam_bin_march_kernel<1, 512>), grid, blk, 0, stream, k, sb, vals, bstart, out,
                               nullptr, 0u, nullptr, nullptr);
        else if (bin_nt == 1024)
            hipLaunchKernelGGL((tvam_bin_march_kernel<0, 1024>), grid, blk, 0, stream, k, sb, vals, bstart, out,
                               nullptr, 0u, nullptr, nullptr);
        else
            hipLaunchKernelGGL((tvam_bin_march_kernel<0, 512>), grid, blk, 0, stream, k, sb, vals, bstart, out,
                               nullptr, 0u, nullptr, nullptr);
        tvam_kt_end(stream, TVAM_KT_BRICK);
    };
    s.st[4] = chunk;
    for (int64_t p0 = 0; p0 < npaths; p0 += chunk) {
        const int64_t p1 = std::min(npaths, p0 + chunk);
        const int64_t ns = (p1 - p0) * slots;
        ++s.st[0];
        TvamSegBuf sb = s.sb;
        sb.p0 = p0;
        sb.p1 = p1;
        sb.slots = slots;
        sb.adj = adj ? 1 : 0;
        if (!adj && (e = hipMemsetAsync(sb.wmax, 0, sizeof(uint32_t), stream)) != hipSuccess) return e;
        TvamBinChunk* cc = cacheable ? &s.fc[(size_t)(p0 / chunk)] : nullptr;
        if (cc && cc->valid) {  // same paths as the cached chunk: new weights, then the march
            ++s.st[1];
            s.st[3] += cc->total;
            if (cc->total == 0) continue;
            sb.r = cc->r;
            int64_t g = std::min<int64_t>((ns + 255) / 256, 8192);
            hipLaunchKernelGGL(tvam_bin_reweight_kernel, dim3((unsigned)g), dim3(256), 0, stream, k, sb, spp, pat);
            march_fwd(sb, cc->vals, cc->bstart, cc->ws);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            continue;
        }
        if (cc && cc->cap_slots < nsl) {
            (void)hipFree(cc->r);
            cc->r = nullptr;
            cc->cap_slots = 0;
            if (room(TVAM_REC_F4 * (size_t)nsl * sizeof(float4)) &&
                hipMalloc((void**)&cc->r, TVAM_REC_F4 * (size_t)nsl * sizeof(float4)) == hipSuccess)
                cc->cap_slots = nsl;
            else
                cc->r = nullptr;
        }
        if (cc && !cc->r) cc = nullptr;  // no room: this chunk runs from the scratch
        if (cc) sb.r = cc->r;
        if ((e = hipMemsetAsync(sb.m, 0, (ns + 1) * sizeof(uint32_t), stream)) != hipSuccess) return e;
        int64_t g = std::min<int64_t>((p1 - p0 + 255) / 256, 262144);
        const int G = csort ? (int)std::min<int64_t>((p1 - p0 + 255) / 256, 2048) : 0;
        const int64_t nh = (int64_t)nbricks * G + 1;  // per-(brick, workgroup) counts + the total
        if (csort) {
            if (nh > s.cap_hist) {
                (void)hipFree(s.hist);
                (void)hipFree(s.hbase);
                s.hist = s.hbase = nullptr;
                s.cap_hist = 0;
                if ((e = hipMalloc((void**)&s.hist, nh * sizeof(uint32_t))) != hipSuccess ||
                    (e = hipMalloc((void**)&s.hbase, nh * sizeof(uint32_t))) != hipSuccess)
                    return e;
                s.cap_hist = nh;
            }
            if ((e = hipMemsetAsync(s.hist + (nh - 1), 0, sizeof(uint32_t), stream)) != hipSuccess) return e;
            sb.hist = s.hist;
            sb.nbricks = nbricks;
            g = G;
        } else {
            sb.hist = nullptr;
        }
        hipLaunchKernelGGL(tvam_scatter_kernel<TVAM_MODE_EMIT>, dim3((unsigned)g), dim3(256),
                           csort ? (size_t)nbricks * sizeof(uint32_t) : 0, stream, k, t, pat, idxmap, nullptr, nullptr,
                           nullptr, sb);
        sb.hist = nullptr;  // the march kernels read none of it
        if (csort) {
            size_t tbh = 0;
            if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, tbh, s.hist, s.hbase, (int)nh, stream)) != hipSuccess)
                return e;
            if (tbh > s.temp_bytes) {
                (void)hipFree(s.temp);
                s.temp = nullptr;
                s.temp_bytes = 0;
                if ((e = hipMalloc(&s.temp, tbh)) != hipSuccess) return e;
                s.temp_bytes = tbh;
            }
            if ((e = hipcub::DeviceScan::ExclusiveSum(s.temp, tbh, s.hist, s.hbase, (int)nh, stream)) != hipSuccess)
                return e;
        }
        // exclusive scan of the brick counts (ns + 1 entries: the last gives the total); the
        // counting-sort forward needs none (its positions come from the histogram scan)
        size_t tb = 0;
        if (!csort || adj) {
            if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, sb.m, s.off, (int)(ns + 1), stream)) != hipSuccess)
                return e;
            if (tb > s.temp_bytes) {
                (void)hipFree(s.temp);
                s.temp = nullptr;
                s.temp_bytes = 0;
                if ((e = hipMalloc(&s.temp, tb)) != hipSuccess) return e;
                s.temp_bytes = tb;
            }
            if ((e = hipcub::DeviceScan::ExclusiveSum(s.temp, tb, sb.m, s.off, (int)(ns + 1), stream)) != hipSuccess)
                return e;
        }
        uint32_t total = 0;
        if ((e = hipMemcpyAsync(&total, csort ? s.hbase + (nh - 1) : s.off + ns, sizeof(uint32_t),
                                hipMemcpyDeviceToHost, stream)) != hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(stream)) != hipSuccess) return e;
        if (cc && (int64_t)total > cc->cap_vals) {
            (void)hipFree(cc->vals);
            cc->vals = nullptr;
            cc->cap_vals = 0;
            const int64_t cap = (int64_t)total + total / 8;
            if (room((size_t)cap * sizeof(uint32_t)) &&
                hipMalloc((void**)&cc->vals, (size_t)cap * sizeof(uint32_t)) == hipSuccess)
                cc->cap_vals = cap;
            else
                cc->vals = nullptr;
        }
        if (cc && cc->cap_bricks < (int64_t)nbricks + 1) {
            (void)hipFree(cc->bstart);
            cc->bstart = nullptr;
            cc->cap_bricks = 0;
            if (hipMalloc((void**)&cc->bstart, ((size_t)nbricks + 1) * sizeof(uint32_t)) == hipSuccess)
                cc->cap_bricks = (int64_t)nbricks + 1;
            else
                cc->bstart = nullptr;
        }
        // a chunk whose sorted slots find no room runs from the scratch arrays, uncached
        const bool keep = cc && (total == 0 || (cc->vals && cc->bstart));
        if (keep) cc->total = total;
        if (keep) cc->ws = csort;
        if (keep) ++s.st[2];
        s.st[3] += total;
        if (total == 0) {
            if (keep) cc->valid = true;
            continue;
        }
        // entry arrays: keys[0] (sort keys / the counting-sort adjoint's inv), vals[1] (sorted slots /
        // entries), part (adjoint partials); the radix sort's second buffers keys[1] / vals[0] only
        // on that path (cap_entries2)
        if ((int64_t)total > s.cap_entries) {
            (void)hipFree(s.keys[0]);
            (void)hipFree(s.vals[1]);
            (void)hipFree(s.part);
            s.keys[0] = s.vals[1] = nullptr;
            s.part = nullptr;
            s.cap_entries = 0;
            const int64_t cap = (int64_t)total + total / 4;
            if ((e = hipMalloc((void**)&s.keys[0], cap * sizeof(uint32_t))) != hipSuccess ||
                (e = hipMalloc((void**)&s.vals[1], cap * sizeof(uint32_t))) != hipSuccess ||
                (e = hipMalloc((void**)&s.part, cap * sizeof(float))) != hipSuccess)
                return e;
            s.cap_entries = cap;
        }
        if (!csort && (int64_t)total > s.cap_entries2) {
            (void)hipFree(s.keys[1]);
            (void)hipFree(s.vals[0]);
            s.keys[1] = s.vals[0] = nullptr;
            s.cap_entries2 = 0;
            const int64_t cap = (int64_t)total + total / 4;
            if ((e = hipMalloc((void**)&s.keys[1], cap * sizeof(uint32_t))) != hipSuccess ||
                (e = hipMalloc((void**)&s.vals[0], cap * sizeof(uint32_t))) != hipSuccess)
                return e;
            s.cap_entries2 = cap;
        }
        if (csort) {
            uint32_t* ent = keep ? cc->vals : s.vals[1];
            uint32_t* bstart = keep ? cc->bstart : s.bstart;
            uint32_t* inv = adj ? s.keys[0] : nullptr;
            hipLaunchKernelGGL(tvam_bin_bstart_kernel, dim3((unsigned)((nbricks + 256) / 256)), dim3(256), 0, stream,
                               s.hbase, G, nbricks, bstart);
            hipLaunchKernelGGL(tvam_bin_fill2_kernel, dim3((unsigned)G), dim3(256), (size_t)nbricks * sizeof(uint32_t),
                               stream, k, sb, ns, s.hbase, ent, adj ? s.off : nullptr, inv);
            if (adj) {
                hipLaunchKernelGGL((tvam_bin_march_kernel<2, 1024, true>), dim3((unsigned)nbricks), dim3(1024), 0,
                                   stream, k, sb, ent, bstart, nullptr, gin, 0u, nullptr, s.part);
                const int64_t npix = (p1 - p0) / spp;
                g = std::min<int64_t>((npix + 3) / 4, 65536);  // a wave per pixel
                hipLaunchKernelGGL(tvam_bin_reduce2_kernel, dim3((unsigned)g), dim3(256), 0, stream, sb, spp, s.off,
                                   inv, s.part, idxmap, out);
            } else {
                march_fwd(sb, ent, bstart, true);
            }
            if ((e = hipGetLastError()) != hipSuccess) return e;
            if (keep) cc->valid = true;
            continue;
        }
        size_t tb2 = 0;
        if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, s.keys[0], s.keys[1], s.vals[0], s.vals[1],
                                                    (int)total, 0, bits, stream)) != hipSuccess)
            return e;
        if (tb2 > s.temp_bytes) {
            (void)hipFree(s.temp);
            s.temp = nullptr;
            s.temp_bytes = 0;
            if ((e = hipMalloc(&s.temp, tb2)) != hipSuccess) return e;
            s.temp_bytes = tb2;
        }
        g = std::min<int64_t>((ns + TVAM_FILL_T - 1) / TVAM_FILL_T, 65536);
        hipLaunchKernelGGL(tvam_bin_fill_kernel, dim3((unsigned)g), dim3(256), 0, stream, k, sb, s.off, ns, s.keys[0],
                           s.vals[0], cbits);
        uint32_t* vals_out = keep ? cc->vals : s.vals[1];
        uint32_t* bstart = keep ? cc->bstart : s.bstart;
        if ((e = hipcub::DeviceRadixSort::SortPairs(s.temp, tb2, s.keys[0], s.keys[1], s.vals[0], vals_out,
                                                    (int)total, 0, bits, stream)) != hipSuccess)
            return e;
        g = std::min<int64_t>(((int64_t)total + 256) / 256, 65536);
        hipLaunchKernelGGL(tvam_bin_start_kernel, dim3((unsigned)g), dim3(256), 0, stream, s.keys[1], (int64_t)total,
                           nbricks, kmask, cbits, bstart);
        if (adj) {
            // partials at their sorted positions with their pixel (s.keys[1]: read by the start
            // kernel above, free now), sorted by pixel into keys[0] / vals[0] (free since the
            // sort), each pixel's run start in s.off (free since the fill), summed per pixel
            uint32_t* ppix = s.keys[1];
            const uint32_t pslots = (uint32_t)spp * (uint32_t)slots;
            if (bin_nt == 1024)
                hipLaunchKernelGGL((tvam_bin_march_kernel<2, 1024>), dim3((unsigned)nbricks), dim3(1024), 0, stream, k,
                                   sb, s.vals[1], s.bstart, nullptr, gin, pslots, ppix, s.part);
            else
                hipLaunchKernelGGL((tvam_bin_march_kernel<2, 512>), dim3((unsigned)nbricks), dim3(512), 0, stream, k,
                                   sb, s.vals[1], s.bstart, nullptr, gin, pslots, ppix, s.part);
            const int64_t npix = (p1 - p0) / spp;
            int pbits = 1;
            while (((int64_t)1 << pbits) < npix) ++pbits;
            float* psort = reinterpret_cast<float*>(s.vals[0]);
            size_t tb3 = 0;
            if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb3, ppix, s.keys[0], s.part, psort, (int)total, 0,
                                                        pbits, stream)) != hipSuccess)
                return e;
            if (tb3 > s.temp_bytes) {
                (void)hipFree(s.temp);
                s.temp = nullptr;
                s.temp_bytes = 0;
                if ((e = hipMalloc(&s.temp, tb3)) != hipSuccess) return e;
                s.temp_bytes = tb3;
            }
            if ((e = hipcub::DeviceRadixSort::SortPairs(s.temp, tb3, ppix, s.keys[0], s.part, psort, (int)total, 0,
                                                        pbits, stream)) != hipSuccess)
                return e;
            g = std::min<int64_t>(((int64_t)total + 256) / 256, 65536);
            hipLaunchKernelGGL(tvam_bin_start_kernel, dim3((unsigned)g), dim3(256), 0, stream, s.keys[0],
                               (int64_t)total, (int)npix, 0xffffffffu, 0, s.off);
            g = std::min<int64_t>((npix + 3) / 4, 65536);  // a wave per pixel
            hipLaunchKernelGGL(tvam_bin_reduce_kernel, dim3((unsigned)g), dim3(256), 0, stream, sb, spp, s.off, psort,
                               idxmap, out);
        } else {
            march_fwd(sb, vals_out, bstart, false);
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (keep) cc->valid = true;
    }
    // the count check, read by a later call (above) or tvam_plan_bin_stats, without a sync here
    if (s.sb.bad && s.st[0] > 0 && !s.bad_pending) {
        if ((e = hipMemcpyAsync(s.bad_host, s.sb.bad, sizeof(uint32_t), hipMemcpyDeviceToHost, stream)) != hipSuccess ||
            (e = hipEventRecord(s.bad_ev, stream)) != hipSuccess)
            return e;
        s.bad_pending = true;
    }
    return hipSuccess;
}
