// tvam_common.h — scene constants and the per-ray fp32 geometry shared by the
// host-side plan builder and the gfx950 kernels.
//
// Every function here follows one reference routine op for op (fp32, no
// implicit FMA: the library is built with -ffp-contract=off and FMAs are
// written out where Mitsuba/Dr.Jit form them):
//   tvam_ray_camera    integrators/common.py:81-108 + projector.py:184-188
//                      (collimated get_ray through sample_to_camera)
//   tvam_ray_world     projector.py:160-162 + motion.py:26-36 (look_at)
//   tvam_segment_im    geometry.py:75-96 index-matched vial: null-BSDF open
//                      cylinder entry, spawn_ray offset, exit (volume.py:191,
//                      :237, :247) -> the one medium segment of the ray
//   tvam_dda_init      sensor.py:327-365 (box clip, start/end voxel, dtmax,
//                      tstep) restricted to planar rays (d.z == 0)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#define TVAM_HD __host__ __device__ __forceinline__

#define TVAM_RAY_EPS (1500.0f * 5.9604644775390625e-08f)  // math::RayEpsilon<float>
#define TVAM_TWO_PI 6.2831855f                            // float(2*pi), motion.py:28
#define TVAM_INF __builtin_huge_valf()

// 1 - e^{-x} for x >= 0 without the cancellation of the direct form: a visit's
// weight e^{-st t} (1 - e^{-st dt}) (sensor.py:404) has st dt ~ 1e-3 on the
// BASELINE grids, where 1 - exp() in fp32 keeps only ~4 significant digits
// (and e^{-st t_in} - e^{-st t_out} alike).  Degree-4 Taylor form below 0.05
// (relative error < x^4 / 120 < 6e-8), the direct form above (no cancellation
// there).  nlog2e = -log2(e): e^{-x} = exp2(nlog2e x).
// Kernels whose plan has st * (voxel xy diagonal) = vox_chord < TVAM_W2_MAX (every BASELINE
// grid) use the degree-2 form on E = st e^{-st t}: c = E dt (1 - st dt / 2), E -= st c: five
// full-rate instructions in place of an exp2 and its cancellation; the visit weight is low by a
// relative (st dt)^2 / 6 < 2.7e-6, E drifts by (st dt)^3 / 6 per visit (< 1e-8) and restarts
// from exp2 at every tile entry.
#define TVAM_W2_MAX 4.0e-3f
#define TVAM_NLOG2E (-1.4426950408889634f)
__device__ __forceinline__ float tvam_omexp(float x) {
    if (__builtin_expect(x < 0.05f, 1))
        return x * fmaf(x, fmaf(x, fmaf(x, -4.1666668e-2f, 0.16666667f), -0.5f), 1.0f);
    return 1.0f - __builtin_amdgcn_exp2f(TVAM_NLOG2E * x);
}

struct TvamConsts {
    // film / sensor (sensor.py:14-19, film.py:9-14)
    float bmin[3], bmax[3], h[3];
    int32_t res[3];      // whole film (res[2] = all z-slices: the row -> slice map)
    int32_t z0, nz;      // film slab rendered by this plan: slices [z0, z0 + nz)
    float inv_vol;       // volume.py:41-42 (fp32, like the reference)
    // projector (projector.py:73-99, :171-182)
    int32_t res_x, res_y, crop_x, crop_y, crop_off_x, crop_off_y;
    int32_t n_patterns;  // A
    int32_t a0, a1;      // angle shard
    int64_t shard_base;  // a0 * crop_y * crop_x: first dense index of the shard
    int64_t stream_base; // sparse active sets: position of this plan's first active entry (desc.active_base)
    float ex, ey;        // emitter size W*a_x, H*a_y
    float inv_w, inv_h;  // rcp(ScalarVector2f(w, h)) (common.py:98)
    float dist_m_zc;     // distance - 0.005 (camera-space z of ray origins)
    int32_t clockwise, regular, sample_time;
    int32_t skip_zero;   // forward: rays with pattern value 0 add exactly 0 -> skipped
    // container (geometry.py:75-96, :142-183)
    int32_t vial_type;   // TVAM_VIAL_*
    int32_t max_depth;   // path depth limit (volume.py:272)
    float vial_r, vial_half_h;  // index-matched r / cylindrical r_int; half height
    float vial_r_ext;    // cylindrical: outer glass radius; square: w_ext / 2 (vial_r = w_int / 2)
    float vial_hz_int;   // square: half height of the inner cuboid (0.45 height, geometry.py:207)
    const float* occ;    // occluder triangles [n_occ][3][3] (device; geometry.py:55-72), nullptr if none
    int32_t n_occ;
    float occ_lo[3], occ_hi[3];  // the occluder triangles' bounding box (tvam_occ_hit's early out)
    const float* tgt;    // surface-aware films: target mesh triangles [n_tgt][3][3] (device), else nullptr
    int32_t n_tgt;
    int32_t sensor_type; // TVAM_SENSOR_* (dda / ratio / delta)
    float majorant;      // 'ratio' sensor majorant
    float eta_ext, eta_int;     // cylindrical: int/ext IOR of the outer (glass/air) and inner (medium/glass) surface
    // medium / weights
    float sig_t, sig_s;  // scattering media: sigma_t, sigma_s = albedo * sigma_t (fp32, Mitsuba homogeneous)
    int32_t rr_depth;    // Russian roulette from depth > rr_depth (volume.py:182)
    int32_t phase_type;  // TVAM_PHASE_*
    float phase_g;       // hg asymmetry
    float nsig2;         // -sigma_t * log2(e): exp(-st t) == exp2(nsig2 t)
    float wscale;        // inv_pdf/n_samples * print_time * sa/st (projector.py:164-165,187; common.py:111; sensor.py:404)
    // fixed-point forward bound: |voxel sum| <= max|em| * vox_chord * rays_per_voxel * rows * spp
    float vox_chord;      // min(1, sigma_t * sqrt(2) * max(hx, hy)): bound of 1 - exp(-st dt) in a voxel
    float rays_per_voxel; // n_shard * (ceil(sqrt(2) * max(hx, hy) / pixel_size_x) + 1)
};

// --------------------------------------------------------------------------
// Sampler: TEA-scrambled PCG32 (Mitsuba 'independent' sampler, restated)
// --------------------------------------------------------------------------
struct TvamPcg {
    uint64_t state, inc;
    TVAM_HD uint32_t next() {
        uint64_t old = state;
        state = old * 0x5851f42d4c957f2dULL + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((~rot + 1u) & 31u));
    }
    TVAM_HD float next_float() {
        uint32_t bits = (next() >> 9) | 0x3f800000u;
        return __builtin_bit_cast(float, bits) - 1.0f;
    }
    TVAM_HD void seed(uint32_t seed_value, uint64_t wave_index) {
        uint32_t v0 = seed_value, v1 = (uint32_t)wave_index, sum = 0;
        for (int i = 0; i < 4; ++i) {
            sum += 0x9e3779b9u;
            v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + sum) ^ ((v1 >> 5) + 0xc8013ea4u);
            v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7e95761eu);
        }
        state = 0u;
        inc = ((uint64_t)v1 << 1u) | 1u;
        (void)next();
        state += (uint64_t)v0;
        (void)next();
    }
};

// Sampler stream of the ray of dense shard entry `local`, sample `smp`: the
// reference seeds stream i * spp + smp for entry i of projector.active_pixels
// (common.py:57-67 sampler.seed(seed, active_size * spp), :81 dr.repeat).  A
// sparse active set (idxmap = dense -> active position) uses that position; the
// dense crop order's position is the global dense index itself.
TVAM_HD uint64_t tvam_stream(const TvamConsts& k, const int32_t* idxmap, int64_t local, uint32_t spp, int smp) {
    int64_t pos = local + k.shard_base;
    if (idxmap) {
        const int32_t a = idxmap[local];
        pos = k.stream_base + (a < 0 ? 0 : a);  // inactive entries never reach the film
    }
    return (uint64_t)pos * (uint64_t)spp + (uint64_t)smp;
}

// --------------------------------------------------------------------------
// Ray generation
// --------------------------------------------------------------------------
// Camera-space origin of the collimated ray through (col + jx, row + jy).
TVAM_HD void tvam_ray_camera(const TvamConsts& k, int col, int row, float jx, float jy,
                             float& xc, float& yc) {
    float u = ((float)col + jx) * k.inv_w;
    float v = ((float)row + jy) * k.inv_h;
    xc = (0.5f - u) * k.ex;
    yc = (0.5f - v) * k.ey;
}

// World-space ray for rotation (c, s): o = look_at(dist*(c,s,0) -> 0, up z) @ (xc, yc, 0.005)
TVAM_HD void tvam_ray_world(const TvamConsts& k, float c, float s, float xc, float yc,
                            float& ox, float& oy, float& oz, float& dx, float& dy) {
    ox = c * k.dist_m_zc + s * xc;
    oy = s * k.dist_m_zc - c * xc;
    oz = yc;
    dx = -c;
    dy = -s;
}

// Mitsuba math::solve_quadratic (stable form).
TVAM_HD bool tvam_quadratic(float a, float b, float c, float& x0, float& x1) {
    float disc = b * b - 4.0f * a * c;
    if (!(disc >= 0.0f)) return false;
    float sq = sqrtf(disc);
    float temp = -0.5f * (b + copysignf(sq, b));
    float r0 = temp / a, r1 = c / temp;
    x0 = fminf(r0, r1);
    x1 = fmaxf(r0, r1);
    return true;
}

TVAM_HD bool tvam_cyl_roots(float ox, float oy, float dx, float dy, float r, float& t0, float& t1) {
    float A = dx * dx + dy * dy;
    float B = 2.0f * (dx * ox + dy * oy);
    float C = ox * ox + oy * oy - r * r;
    return tvam_quadratic(A, B, C, t0, t1);
}

TVAM_HD float tvam_occ_hit(const TvamConsts& k, float ox, float oy, float oz, float dx, float dy, float dz);

// Index-matched vial: the medium segment (o2, maxt) of a projector ray.
TVAM_HD bool tvam_segment_im(const TvamConsts& k, float ox, float oy, float oz, float dx, float dy,
                             float& o2x, float& o2y, float& maxt) {
    if (!(oz >= -k.vial_half_h && oz <= k.vial_half_h)) return false;
    float t0, t1;
    if (!tvam_cyl_roots(ox, oy, dx, dy, k.vial_r, t0, t1)) return false;
    if (!(t0 >= 0.0f)) return false;
    if (k.n_occ && tvam_occ_hit(k, ox, oy, oz, dx, dy, 0.0f) < t0) return false;  // blocked before the vial
    float px = fmaf(dx, t0, ox), py = fmaf(dy, t0, oy), pz = oz;
    float rp = sqrtf(px * px + py * py);
    float nx = px / rp, ny = py / rp;
    float m = fmaxf(fmaxf(fabsf(px), fabsf(py)), fabsf(pz));
    float mag = (1.0f + m) * TVAM_RAY_EPS;
    float ndd = nx * dx + ny * dy + 0.0f;  // n.z * d.z == +0
    if (__builtin_signbit(ndd)) mag = -mag;
    o2x = fmaf(mag, nx, px);
    o2y = fmaf(mag, ny, py);
    float u0, u1;
    if (!tvam_cyl_roots(o2x, o2y, dx, dy, k.vial_r, u0, u1)) return false;
    if (!(u1 > 0.0f)) return false;
    maxt = u1;
    if (k.n_occ) maxt = fminf(u1, tvam_occ_hit(k, o2x, o2y, oz, dx, dy, 0.0f));  // ends on an occluder
    return true;
}

#define TVAM_IOR_AIR 1.000277f  // Mitsuba ior table: 'air'

// Nearest hit t >= 0 of the open tube of radius r (Mitsuba cylinder restated;
// planar rays: the z test is the caller's).
TVAM_HD float tvam_tube_hit(float ox, float oy, float dx, float dy, float r) {
    float t0, t1;
    if (!tvam_cyl_roots(ox, oy, dx, dy, r, t0, t1)) return TVAM_INF;
    if (!(t1 >= 0.0f)) return TVAM_INF;
    return t0 >= 0.0f ? t0 : t1;
}

// Mitsuba dielectric sample() with only the transmission lobe, in the tube's
// shading frame (s = dp_du / |dp_du| = (-n.y, n.x), n outward): fresnel(),
// refract(wi, cos_t, eta_ti), weight (1 - F) eta_ti^2 (Radiance mode).
// eta = int_ior / ext_ior.  Returns the weight, 0 on total internal reflection.
TVAM_HD float tvam_transmit(float nx, float ny, float dx, float dy, float eta, float& wx, float& wy) {
    const float sx = -ny, sy = nx;
    const float wl_x = -(dx * sx + dy * sy);  // wi = to_local(-d)
    const float cos_i = -(dx * nx + dy * ny);
    const bool outside = cos_i >= 0.0f;
    const float rcp_eta = 1.0f / eta;
    const float eta_it = outside ? eta : rcp_eta, eta_ti = outside ? rcp_eta : eta;
    const float ct2 = 1.0f - (1.0f - cos_i * cos_i) * (eta_ti * eta_ti);
    const float ci = fabsf(cos_i), ct = sqrtf(fmaxf(ct2, 0.0f));
    float r;
    if (eta == 1.0f) r = 0.0f;
    else if (ci == 0.0f) r = 1.0f;
    else {
        const float a_s = (ci - eta_it * ct) / (ci + eta_it * ct);
        const float a_p = (ct - eta_it * ci) / (ct + eta_it * ci);
        r = 0.5f * (a_s * a_s + a_p * a_p);
    }
    const float cos_t = outside ? -ct : ct;
    const float t = 1.0f - r;
    if (!(t > 0.0f)) return 0.0f;
    const float ox = -eta_ti * wl_x;  // refract: (-eta_ti wi.x, -eta_ti wi.y, cos_t)
    wx = sx * ox + nx * cos_t;        // to_world
    wy = sy * ox + ny * cos_t;
    return t * (eta_ti * eta_ti);
}

// Occluders: nearest triangle hit (Mitsuba ray_intersect_triangle restated,
// Moller-Trumbore, t >= 0); oracle or_tri_hit / or_occ_hit.
TVAM_HD float tvam_tri_hit(const float* v, float ox, float oy, float oz, float dx, float dy, float dz) {
    const float e1x = v[3] - v[0], e1y = v[4] - v[1], e1z = v[5] - v[2];
    const float e2x = v[6] - v[0], e2y = v[7] - v[1], e2z = v[8] - v[2];
    const float tx = ox - v[0], ty = oy - v[1], tz = oz - v[2];
    const float px = dy * e2z - dz * e2y, py = dz * e2x - dx * e2z, pz = dx * e2y - dy * e2x;
    const float inv_det = 1.0f / (e1x * px + e1y * py + e1z * pz);
    const float u = (tx * px + ty * py + tz * pz) * inv_det;
    if (!(u >= 0.0f && u <= 1.0f)) return TVAM_INF;
    const float qx = ty * e1z - tz * e1y, qy = tz * e1x - tx * e1z, qz = tx * e1y - ty * e1x;
    const float w = (dx * qx + dy * qy + dz * qz) * inv_det;
    if (!(w >= 0.0f && u + w <= 1.0f)) return TVAM_INF;
    const float t = (e2x * qx + e2y * qy + e2z * qz) * inv_det;
    return t >= 0.0f ? t : TVAM_INF;
}

TVAM_HD float tvam_occ_hit(const TvamConsts& k, float ox, float oy, float oz, float dx, float dy, float dz) {
    float best = TVAM_INF;
    if (dz == 0.0f) {
        // a planar ray that passes the occluders' bounding box, grown by the per-triangle skip's
        // margin below, misses every triangle (same argument): most rays never test one
        const float o[2] = {ox, oy}, d[2] = {dx, dy};
        const float mz = 1e-3f * (1.0f + fabsf(k.occ_lo[2]) + fabsf(k.occ_hi[2]));
        if (oz < k.occ_lo[2] - mz || oz > k.occ_hi[2] + mz) return TVAM_INF;
        float t0 = 0.0f, t1 = TVAM_INF;  // tvam_tri_hit reports t >= 0 only
        for (int a = 0; a < 2; ++a) {
            const float m = 1e-3f * (1.0f + fabsf(k.occ_lo[a]) + fabsf(k.occ_hi[a]));
            const float lo = k.occ_lo[a] - m, hi = k.occ_hi[a] + m;
            if (d[a] == 0.0f) {
                if (o[a] < lo || o[a] > hi) return TVAM_INF;
                continue;
            }
            const float ta = (lo - o[a]) / d[a], tb = (hi - o[a]) / d[a];
            t0 = fmaxf(t0, fminf(ta, tb));
            t1 = fminf(t1, fmaxf(ta, tb));
        }
        if (t0 > t1) return TVAM_INF;
    }
    for (int i = 0; i < k.n_occ; ++i) {
        const float* v = k.occ + 9 * i;
        // a planar ray (d.z = 0) far outside the triangle's z range misses it: Moller-Trumbore's
        // barycentric test fails there by orders of magnitude more than its rounding (the margin),
        // so skipping the test returns the same t (most of a wave's rays pass below / above)
        if (dz == 0.0f) {
            const float zlo = fminf(fminf(v[2], v[5]), v[8]), zhi = fmaxf(fmaxf(v[2], v[5]), v[8]);
            const float mg = 1e-3f * (1.0f + fabsf(zlo) + fabsf(zhi));
            if (oz < zlo - mg || oz > zhi + mg) continue;
        }
        best = fminf(best, tvam_tri_hit(v, ox, oy, oz, dx, dy, dz));
    }
    return best;
}

// Closed box [-h, h] (Mitsuba 'cube' scaled): nearest t >= 0, outward face
// normal (oracle or_box_hit; same axis order and tie rule).
TVAM_HD float tvam_box_hit(float ox, float oy, float oz, float dx, float dy, float dz, float hx, float hy, float hz,
                           float& nx, float& ny, float& nz) {
    const float o[3] = {ox, oy, oz}, d[3] = {dx, dy, dz}, h[3] = {hx, hy, hz};
    float tn = -TVAM_INF, tf = TVAM_INF;
    int an = 0, af = 0;
    for (int a = 0; a < 3; ++a) {
        if (d[a] == 0.0f) {
            if (!(o[a] >= -h[a] && o[a] <= h[a])) return TVAM_INF;
            continue;
        }
        const float t0 = (-h[a] - o[a]) / d[a], t1 = (h[a] - o[a]) / d[a];
        const float lo = fminf(t0, t1), hi = fmaxf(t0, t1);
        if (lo > tn) {
            tn = lo;
            an = a;
        }
        if (hi < tf) {
            tf = hi;
            af = a;
        }
    }
    if (!(tn <= tf)) return TVAM_INF;
    float n[3] = {0.0f, 0.0f, 0.0f};
    float t = TVAM_INF;
    if (tn >= 0.0f) {
        n[an] = d[an] > 0.0f ? -1.0f : 1.0f;
        t = tn;
    } else if (tf >= 0.0f) {
        n[af] = d[af] > 0.0f ? 1.0f : -1.0f;
        t = tf;
    }
    nx = n[0];
    ny = n[1];
    nz = n[2];
    return t;
}

// Mitsuba fresnel() (oracle or_fresnel): reflectance, signed cos_theta_t, eta_ti.
TVAM_HD float tvam_fresnel(float cos_i, float eta, float& cos_t, float& eta_ti) {
    const bool outside = cos_i >= 0.0f;
    const float rcp_eta = 1.0f / eta;
    const float eta_it = outside ? eta : rcp_eta;
    eta_ti = outside ? rcp_eta : eta;
    const float ct2 = 1.0f - (1.0f - cos_i * cos_i) * (eta_ti * eta_ti);
    const float ci = fabsf(cos_i), ct = sqrtf(fmaxf(ct2, 0.0f));
    float r;
    if (eta == 1.0f) r = 0.0f;
    else if (ci == 0.0f) r = 1.0f;
    else {
        const float a_s = (ci - eta_it * ct) / (ci + eta_it * ct);
        const float a_p = (ct - eta_it * ci) / (ct + eta_it * ci);
        r = 0.5f * (a_s * a_s + a_p * a_p);
    }
    cos_t = outside ? -ct : ct;
    return r;
}

// Transmission in world space (the cube's faces; oracle or_transmit_world):
// wo = -eta_ti wi + (eta_ti cos_i + cos_t) n, weight (1 - F) eta_ti^2.
TVAM_HD float tvam_transmit_world(float nx, float ny, float nz, float dx, float dy, float dz, float eta, float& wx,
                                  float& wy, float& wz) {
    const float cos_i = -(dx * nx + dy * ny + dz * nz);
    float cos_t, eta_ti;
    const float r = tvam_fresnel(cos_i, eta, cos_t, eta_ti);
    const float t = 1.0f - r;
    if (!(t > 0.0f)) return 0.0f;
    const float c = eta_ti * cos_i + cos_t;
    wx = eta_ti * dx + c * nx;
    wy = eta_ti * dy + c * ny;
    wz = eta_ti * dz + c * nz;
    return t * (eta_ti * eta_ti);
}

// Square vial (geometry.py:186-219; oracle or_segment_square): the glass
// cuboids' faces in order, transmission and spawn_ray at each, until the ray
// runs inside the inner cuboid; the segment ends at its next hit (or an
// occluder).  Planar rays (d.z = 0) meet only vertical faces.
TVAM_HD bool tvam_segment_square(const TvamConsts& k, float ox, float oy, float oz, float dx, float dy, float& o2x,
                                 float& o2y, float& d2x, float& d2y, float& maxt, float& weight) {
    float px = ox, py = oy, vx = dx, vy = dy, att = 1.0f;
    bool in_medium = false;
    for (int depth = 0; depth < k.max_depth; ++depth) {
        float nex, ney, nez, nix, niy, niz;
        const float te = tvam_box_hit(px, py, oz, vx, vy, 0.0f, k.vial_r_ext, k.vial_r_ext, k.vial_half_h, nex, ney,
                                      nez);
        const float ti = tvam_box_hit(px, py, oz, vx, vy, 0.0f, k.vial_r, k.vial_r, k.vial_hz_int, nix, niy, niz);
        const bool inner = ti <= te;
        float t = inner ? ti : te;
        if (k.n_occ) {
            const float toc = tvam_occ_hit(k, px, py, oz, vx, vy, 0.0f);
            if (toc < t) {
                if (!in_medium) return false;
                t = toc;
            }
        }
        if (!(t < TVAM_INF)) return false;
        if (in_medium) {
            o2x = px;
            o2y = py;
            d2x = vx;
            d2y = vy;
            maxt = t;
            weight = att;
            return true;
        }
        const float nx = inner ? nix : nex, ny = inner ? niy : ney, nz = inner ? niz : nez;
        const float hx = fmaf(vx, t, px), hy = fmaf(vy, t, py), hz = fmaf(0.0f, t, oz);
        float wx, wy, wz;
        const float w = tvam_transmit_world(nx, ny, nz, vx, vy, 0.0f, inner ? k.eta_int : k.eta_ext, wx, wy, wz);
        if (!(w > 0.0f)) return false;
        att = att * w;
        const float m = fmaxf(fmaxf(fabsf(hx), fabsf(hy)), fabsf(hz));
        float mag = (1.0f + m) * TVAM_RAY_EPS;
        const float nwo = nx * wx + ny * wy + nz * wz;
        if (__builtin_signbit(nwo)) mag = -mag;
        px = fmaf(mag, nx, hx);
        py = fmaf(mag, ny, hy);
        vx = wx;
        vy = wy;
        in_medium = inner && nwo < 0.0f;
    }
    return false;
}

// Cylindrical vial (geometry.py:142-183, volume.py:179-272 transmission-only):
// surface hits in order (nearest of the r_ext / r_int tubes), transmission
// and spawn_ray at each, until the ray runs inside r_int; the medium segment
// (o2, d2, [0, maxt]) ends at its next hit.  weight = product of the
// interfaces' transmission weights.
TVAM_HD bool tvam_segment_cyl(const TvamConsts& k, float ox, float oy, float oz, float dx, float dy, float& o2x,
                              float& o2y, float& d2x, float& d2y, float& maxt, float& weight) {
    if (!(oz >= -k.vial_half_h && oz <= k.vial_half_h)) return false;  // passes above / below the tubes
    float px = ox, py = oy, vx = dx, vy = dy, att = 1.0f;
    bool in_medium = false;
    for (int depth = 0; depth < k.max_depth; ++depth) {
        const float te = tvam_tube_hit(px, py, vx, vy, k.vial_r_ext), ti = tvam_tube_hit(px, py, vx, vy, k.vial_r);
        const bool inner = ti <= te;
        float t = inner ? ti : te;
        if (k.n_occ) {
            const float toc = tvam_occ_hit(k, px, py, oz, vx, vy, 0.0f);
            if (toc < t) {  // an occluder: the segment ends there, or the ray dies outside the medium
                if (!in_medium) return false;
                t = toc;
            }
        }
        if (!(t < TVAM_INF)) return false;
        if (in_medium) {
            o2x = px;
            o2y = py;
            d2x = vx;
            d2y = vy;
            maxt = t;
            weight = att;
            return true;
        }
        const float hx = fmaf(vx, t, px), hy = fmaf(vy, t, py);
        const float rp = sqrtf(hx * hx + hy * hy);
        const float nx = hx / rp, ny = hy / rp;
        float wx, wy;
        const float w = tvam_transmit(nx, ny, vx, vy, inner ? k.eta_int : k.eta_ext, wx, wy);
        if (!(w > 0.0f)) return false;
        att = att * w;
        const float m = fmaxf(fmaxf(fabsf(hx), fabsf(hy)), fabsf(oz));
        float mag = (1.0f + m) * TVAM_RAY_EPS;
        const float nwo = nx * wx + ny * wy + 0.0f;
        if (__builtin_signbit(nwo)) mag = -mag;
        px = fmaf(mag, nx, hx);
        py = fmaf(mag, ny, hy);
        vx = wx;
        vy = wy;
        in_medium = inner && nwo < 0.0f;
    }
    return false;
}

// Radon filter path (integrators/radon.py:77-106; oracle or_radon_ray): a
// planar projector ray through the scene (container surfaces, occluders, the
// target mesh with its null BSDF), summing throughput e^{-st t}(1 - e^{-st
// si.t}) over the segments inside both the medium and the target (t = the
// distance travelled so far, from the ray origin).  Target hits toggle
// inside_target and do not count as depth.  Only L > 0 matters to the filter
// (optimize.py:143-163).
TVAM_HD float tvam_radon_ray(const TvamConsts& k, const float* tgt, int ntgt, int max_depth, float ox, float oy,
                             float oz, float dx, float dy) {
    float px = ox, py = oy, vx = dx, vy = dy;
    float thr = 1.0f, L = 0.0f, t = 0.0f;
    bool in_medium = false, inside = false;
    int depth = 0;
    for (int it = 0; it < 4096; ++it) {
        // nearest surface: container (kind 0 outer glass, 1 medium boundary), occluder (2), target (3)
        float tb = TVAM_INF, nx = 0.0f, ny = 0.0f;
        int kind = -1, tri = -1;
        if (k.vial_type == 2) {
            float ax, ay, az, bx, by, bz;
            const float te = tvam_box_hit(px, py, oz, vx, vy, 0.0f, k.vial_r_ext, k.vial_r_ext, k.vial_half_h, ax, ay, az);
            const float ti = tvam_box_hit(px, py, oz, vx, vy, 0.0f, k.vial_r, k.vial_r, k.vial_hz_int, bx, by, bz);
            if (ti <= te) {
                tb = ti;
                kind = 1;
                nx = bx;
                ny = by;
            } else {
                tb = te;
                kind = 0;
                nx = ax;
                ny = ay;
            }
        } else if (oz >= -k.vial_half_h && oz <= k.vial_half_h) {
            const float ti = tvam_tube_hit(px, py, vx, vy, k.vial_r);
            const float te = k.vial_type == 1 ? tvam_tube_hit(px, py, vx, vy, k.vial_r_ext) : TVAM_INF;
            tb = ti <= te ? ti : te;
            kind = ti <= te ? 1 : 0;
        }
        if (k.n_occ) {
            const float toc = tvam_occ_hit(k, px, py, oz, vx, vy, 0.0f);
            if (toc < tb) {
                tb = toc;
                kind = 2;
            }
        }
        for (int i = 0; i < ntgt; ++i) {
            const float tt = tvam_tri_hit(tgt + 9 * i, px, py, oz, vx, vy, 0.0f);
            if (tt < tb) {
                tb = tt;
                kind = 3;
                tri = i;
            }
        }
        if (!(tb < TVAM_INF)) break;
        const float contrib = thr * expf(-k.sig_t * t) * (1.0f - expf(-k.sig_t * tb));
        if (inside && in_medium) L = L + contrib;
        t = t + tb;
        const float hx = fmaf(vx, tb, px), hy = fmaf(vy, tb, py);
        float wx = vx, wy = vy, wz = 0.0f, nz = 0.0f;
        if (kind == 3) {  // target: null BSDF; geometric normal of the triangle for the spawn offset
            const float* v = tgt + 9 * tri;
            const float e1x = v[3] - v[0], e1y = v[4] - v[1], e1z = v[5] - v[2];
            const float e2x = v[6] - v[0], e2y = v[7] - v[1], e2z = v[8] - v[2];
            float cx = e1y * e2z - e1z * e2y, cy = e1z * e2x - e1x * e2z, cz = e1x * e2y - e1y * e2x;
            const float inv = 1.0f / sqrtf(cx * cx + cy * cy + cz * cz);
            nx = cx * inv;
            ny = cy * inv;
            nz = cz * inv;
            inside = !inside;
        } else if (kind == 2) {
            break;  // black occluder: throughput 0 from here on
        } else {
            if (k.vial_type == 1 || (k.vial_type == 0)) {  // tubes: outward normal
                const float rp = sqrtf(hx * hx + hy * hy);
                nx = hx / rp;
                ny = hy / rp;
            }
            if (k.vial_type != 0) {
                const float eta = kind == 1 ? k.eta_int : k.eta_ext;
                const float w = k.vial_type == 2 ? tvam_transmit_world(nx, ny, 0.0f, vx, vy, 0.0f, eta, wx, wy, wz)
                                                 : tvam_transmit(nx, ny, vx, vy, eta, wx, wy);
                if (!(w > 0.0f)) break;
                thr = thr * w;
            }
            ++depth;
        }
        const float m = fmaxf(fmaxf(fabsf(hx), fabsf(hy)), fabsf(oz));
        float mag = (1.0f + m) * TVAM_RAY_EPS;
        const float nwo = nx * wx + ny * wy + nz * wz;
        if (__builtin_signbit(nwo)) mag = -mag;
        px = fmaf(mag, nx, hx);
        py = fmaf(mag, ny, hy);
        // (the offset's z component moves oz by mag * nz for a tilted target face)
        oz = fmaf(mag, nz, oz);
        vx = wx;
        vy = wy;
        if (depth >= max_depth) break;
        if (kind == 1) in_medium = nwo < 0.0f;  // the medium boundary is the only medium transition
    }
    return L;
}

// The medium segment of a planar projector ray for the plan's container.
TVAM_HD bool tvam_segment(const TvamConsts& k, float ox, float oy, float oz, float dx, float dy, float& o2x,
                          float& o2y, float& d2x, float& d2y, float& maxt, float& weight) {
    if (k.vial_type == 1 /* TVAM_VIAL_CYLINDRICAL */)
        return tvam_segment_cyl(k, ox, oy, oz, dx, dy, o2x, o2y, d2x, d2y, maxt, weight);
    if (k.vial_type == 2 /* TVAM_VIAL_SQUARE */)
        return tvam_segment_square(k, ox, oy, oz, dx, dy, o2x, o2y, d2x, d2y, maxt, weight);
    d2x = dx;
    d2y = dy;
    weight = 1.0f;
    return tvam_segment_im(k, ox, oy, oz, dx, dy, o2x, o2y, maxt);
}

// z slice of a planar ray with origin height oz: the DDA's start voxel z
// (sensor.py:345) when the box clip admits the ray, else -1.  For d.z == +0
// the z slab test (bmin.z - oz)/0 admits exactly bmin.z < oz < bmax.z.
TVAM_HD int tvam_slice_of(const TvamConsts& k, float oz) {
    if (!(oz > k.bmin[2] && oz < k.bmax[2])) return -1;
    int sv = (int)((oz - k.bmin[2]) / k.h[2]);
    sv = sv < 0 ? 0 : (sv > k.res[2] - 1 ? k.res[2] - 1 : sv);
    return sv;
}

// In-plane DDA initialisation of the medium segment (o, d, [0, maxt]) of a
// planar ray.  Times are kept relative to t_start.
struct TvamDda {
    float t_start, tau_end;   // tau_end = t_end - t_start
    float dtm0[2], ts[2];     // dtmax at t_start, tstep (inf on invalid axes)
    int32_t sv[2], ev[2], step[2];
};

TVAM_HD bool tvam_dda_init(const TvamConsts& k, float ox, float oy, float dx, float dy, float maxt,
                           TvamDda& q) {
    float o[2] = {ox, oy}, d[2] = {dx, dy};
    float lo[2], hi[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        float tb0 = (k.bmin[a] - o[a]) / d[a];
        float tb1 = (k.bmax[a] - o[a]) / d[a];
        lo[a] = fminf(tb0, tb1);
        hi[a] = fmaxf(tb0, tb1);
    }
    // z axis: admitted (-inf, +inf) once tvam_slice_of() >= 0
    float mint_box = fmaxf(fmaxf(fmaxf(lo[0], lo[1]), -TVAM_INF), 0.0f);
    float maxt_box = fminf(fminf(hi[0], hi[1]), TVAM_INF);
    float t_start = fmaxf(mint_box, 0.0f);
    float t_end = fminf(maxt_box, maxt);
    if (!(isfinite(t_start) && isfinite(t_end) && t_start < t_end)) return false;
    q.t_start = t_start;
    q.tau_end = t_end - t_start;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        float gs = fmaf(d[a], t_start, o[a]);
        float ge = fmaf(d[a], t_end, o[a]);
        int step = d[a] > 0.0f ? 1 : -1;
        int sv = (int)((gs - k.bmin[a]) / k.h[a]);
        int ev = (int)((ge - k.bmin[a]) / k.h[a]);
        sv = sv < 0 ? 0 : (sv > k.res[a] - 1 ? k.res[a] - 1 : sv);
        ev = ev < 0 ? 0 : (ev > k.res[a] - 1 ? k.res[a] - 1 : ev);
        float next = k.bmin[a] + (float)(sv + step) * k.h[a];
        if (d[a] < 0.0f) next = next + k.h[a];
        bool valid = fabsf(d[a]) > 1e-8f;
        float dtm = valid ? (next - gs) / d[a] : TVAM_INF;
        if (dtm < 0.0f) dtm = TVAM_INF;
        q.dtm0[a] = dtm;
        q.ts[a] = valid ? (k.h[a] / d[a]) * (float)step : TVAM_INF;
        q.sv[a] = sv;
        q.ev[a] = ev;
        q.step[a] = step;
    }
    return true;
}

// Axis interval (relative times) during which the DDA's voxel index on one
// axis lies in [lo, hi).  The reference steps this axis at relative times
// T(n) = dtm0 + n*ts, n >= 0 (sensor.py:430-434 in exact arithmetic).
TVAM_HD void tvam_axis_window(int sv, int step, float dtm0, float ts, int lo, int hi,
                              float& tin, float& tout, int& nin, int& nout) {
    if (!(dtm0 < TVAM_INF)) {  // axis never steps
        bool inside = sv >= lo && sv < hi;
        tin = -TVAM_INF;
        tout = inside ? TVAM_INF : -TVAM_INF;
        nin = 0;
        nout = inside ? 0x7fffffff : 0;
        return;
    }
    if (step > 0) {
        nin = lo - sv;
        nout = hi - sv;
    } else {
        nin = sv - hi + 1;
        nout = sv - lo + 1;
    }
    tin = nin > 0 ? fmaf((float)(nin - 1), ts, dtm0) : -TVAM_INF;
    tout = nout > 0 ? fmaf((float)(nout - 1), ts, dtm0) : -TVAM_INF;
}

// Steps taken on an axis by relative time tau, clamped to the window.
TVAM_HD int tvam_axis_steps(float tau, float dtm0, float ts, int nin, int nout) {
    int n = tau < dtm0 ? 0 : (int)floorf((tau - dtm0) / ts) + 1;
    int nlo = nin > 0 ? nin : 0;
    n = n < nlo ? nlo : n;
    n = n > nout - 1 ? nout - 1 : n;
    return n;
}
