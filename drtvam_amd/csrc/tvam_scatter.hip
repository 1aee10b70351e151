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
// One thread per (ray, sample); the stream is `dense crop index * spp +
// sample`, as for the ray records.  Draw order per loop iteration (restated
// in oracle/tvam_oracle.c, or_trace_scatter): RR next_1d, medium next_1d,
// BSDF next_1d + next_2d on surfaces, phase next_1d + next_2d on scattering.
#include "tvam_internal.h"

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
    if (k.phase_type == TVAM_PHASE_ISOTROPIC) {
        const float z = 1.0f - 2.0f * u1;
        const float r = sqrtf(fmaxf(1.0f - z * z, 0.0f));
        const float sp = sinf(TVAM_TWO_PI * u2), cp = cosf(TVAM_TWO_PI * u2);
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

// One medium segment's 3-D DDA (sensor.py:327-438, op for op like the oracle's
// or_dda): MODE FWD adds em * (e^{-st t} - e^{-st (t + dt)}) * inv_vol into the
// dose, ADJ returns sum (...) * grad * inv_vol, COUNT counts visits.
template <int MODE>
__device__ float sc_dda(const TvamConsts& k, float ox, float oy, float oz, float dx, float dy, float dz, float maxt,
                        float em, float* __restrict__ dose, const float* __restrict__ gin, uint64_t& nvis) {
    const float o[3] = {ox, oy, oz}, d[3] = {dx, dy, dz};
    float lo[3], hi[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float tb0 = (k.bmin[a] - o[a]) / d[a];
        const float tb1 = (k.bmax[a] - o[a]) / d[a];
        lo[a] = fminf(tb0, tb1);
        hi[a] = fmaxf(tb0, tb1);
    }
    const float t_start = fmaxf(fmaxf(fmaxf(fmaxf(lo[0], lo[1]), lo[2]), 0.0f), 0.0f);
    const float t_end = fminf(fminf(fminf(hi[0], hi[1]), hi[2]), maxt);
    if (!(isfinite(t_start) && isfinite(t_end) && t_start < t_end)) return 0.0f;
    int cur[3], endv[3], step[3];
    float dtmax[3], tstep[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float gs = fmaf(d[a], t_start, o[a]);
        const float ge = fmaf(d[a], t_end, o[a]);
        step[a] = d[a] > 0.0f ? 1 : -1;
        int sv = (int)((gs - k.bmin[a]) / k.h[a]);
        int ev = (int)((ge - k.bmin[a]) / k.h[a]);
        sv = sv < 0 ? 0 : (sv > k.res[a] - 1 ? k.res[a] - 1 : sv);
        ev = ev < 0 ? 0 : (ev > k.res[a] - 1 ? k.res[a] - 1 : ev);
        cur[a] = sv;
        endv[a] = ev;
        float next = k.bmin[a] + (float)(sv + step[a]) * k.h[a];
        if (d[a] < 0.0f) next = next + k.h[a];
        const bool valid = fabsf(d[a]) > 1e-8f;
        float dtm = valid ? (next - gs) / d[a] : TVAM_INF;
        if (dtm < 0.0f) dtm = TVAM_INF;
        dtmax[a] = dtm;
        tstep[a] = valid ? (k.h[a] / d[a]) * (float)step[a] : TVAM_INF;
    }
    float t = t_start, remaining = t_end - t_start;
    float e0 = sc_exp2(k.nsig2 * t);
    float acc = 0.0f;
    const int64_t sx = 1, sy = k.res[0], sz = (int64_t)k.res[0] * k.res[1];
    for (;;) {
        const float dt = fminf(fminf(fminf(dtmax[0], dtmax[1]), dtmax[2]), remaining);
        remaining = remaining - dt;
        const float e1 = sc_exp2(k.nsig2 * (t + fmaxf(dt, 0.0f)));
        const int64_t idx = cur[0] * sx + cur[1] * sy + cur[2] * sz;
        if (MODE == TVAM_MODE_FWD) atomicAdd(&dose[idx], em * (e0 - e1));
        else if (MODE == TVAM_MODE_ADJ) acc = fmaf(e0 - e1, gin[idx] * k.inv_vol, acc);
        ++nvis;
        if (!((cur[0] != endv[0] || cur[1] != endv[1] || cur[2] != endv[2]) && remaining > 1e-6f)) break;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const bool m = dtmax[a] == dt;
            dtmax[a] = m ? tstep[a] : dtmax[a] - dt;
            cur[a] += m ? step[a] : 0;
        }
        if (cur[0] < 0 || cur[1] < 0 || cur[2] < 0 || cur[0] >= k.res[0] || cur[1] >= k.res[1] || cur[2] >= k.res[2])
            break;
        t = t + dt;
        e0 = e1;
    }
    return acc;
}

template <int MODE>
__global__ __launch_bounds__(256) void tvam_scatter_kernel(TvamConsts k, TvamTiles tp, const float* __restrict__ pat,
                                                           const int32_t* __restrict__ idxmap,
                                                           const float* __restrict__ gin, float* __restrict__ out,
                                                           unsigned long long* __restrict__ counter) {
    const int spp = (int)tp.spp;
    const int64_t per_angle = (int64_t)k.crop_y * k.crop_x;
    const int64_t n = (int64_t)tp.n_shard * per_angle * spp;
    const float st = k.sig_t, ss = k.sig_s;
    const int nsurf = k.vial_type == 0 ? 1 : 2;  // glass vials: two surfaces before the medium
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
        const int64_t dense = local + k.shard_base;
        TvamPcg rng;
        rng.seed(tp.seed, (uint64_t)dense * (uint64_t)spp + (uint64_t)smp);
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
            if (seg > 0) {
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
}

}  // namespace

hipError_t tvam_launch_scatter_paths(int mode, const TvamConsts& k, const TvamTiles& t, const float* pat,
                                     const int32_t* idxmap, const float* gin, float* out,
                                     unsigned long long* counter, hipStream_t stream) {
    const int64_t n = (int64_t)t.n_shard * k.crop_y * k.crop_x * t.spp;
    int64_t g = (n + 255) / 256;
    if (g > 262144) g = 262144;
    if (g < 1) g = 1;
    switch (mode) {
        case TVAM_MODE_FWD:
            hipLaunchKernelGGL(tvam_scatter_kernel<TVAM_MODE_FWD>, dim3((unsigned)g), dim3(256), 0, stream, k, t, pat,
                               idxmap, gin, out, counter);
            break;
        case TVAM_MODE_ADJ:
            hipLaunchKernelGGL(tvam_scatter_kernel<TVAM_MODE_ADJ>, dim3((unsigned)g), dim3(256), 0, stream, k, t, pat,
                               idxmap, gin, out, counter);
            break;
        default:
            hipLaunchKernelGGL(tvam_scatter_kernel<TVAM_MODE_COUNT>, dim3((unsigned)g), dim3(256), 0, stream, k, t,
                               pat, idxmap, gin, out, counter);
    }
    return hipGetLastError();
}
