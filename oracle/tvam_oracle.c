/*
 * tvam_oracle.c — CPU restatement of Dr.TVAM's forward/adjoint ray march.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in drtvam_amd/ links, loads or calls this
 * file; it is used by tests/ (as the parity checker), by
 * __graft_entry__.smoke() (as the checker) and by bench.py's cpu_baseline leg
 * (as the timed CPU port).  It is an independent re-statement of the
 * reference algorithm, written from the reference sources:
 *
 *   ray generation    integrators/common.py:70-116 (sample_rays)
 *   collimated rays   projector.py:148-188 (+ Mitsuba orthographic_projection,
 *                     restated: x_c = W*a_x*(0.5-u), y_c = H*a_y*(0.5-v),
 *                     z_c = 0.005, dir (0,0,1))
 *   circular motion   motion.py:26-36 (+ Mitsuba look_at, restated:
 *                     left = (s,-c,0), up = (0,0,1), dir = (-c,-s,0))
 *   index-matched     geometry.py:75-96: open cylinder r, height h, null BSDF;
 *     vial            Mitsuba cylinder intersection + SurfaceInteraction
 *                     spawn_ray/offset_p restated (RayEpsilon = 1500*2^-24)
 *   cylindrical vial  geometry.py:142-183: glass tubes r_ext (air|glass) and
 *                     r_int (glass|medium), 'dielectric' BSDFs; the path loop
 *                     of volume.py:179-272 with transmission_only (common.py:19):
 *                     Mitsuba dielectric sample() restated (fresnel(), refract()
 *                     in the cylinder's shading frame s = dp_du, n outward,
 *                     weight (1 - F) * eta_ti^2 in Radiance mode), ior 'air' =
 *                     1.000277 (Mitsuba ior table).  UNPINNED like the rest of
 *                     the Mitsuba internals.
 *   path loop         integrators/volume.py:136-282 for the non-scattering,
 *                     transmission-only case: one medium segment per ray
 *   DDA accumulate    sensor.py:306-440 (op for op, fp32 geometry)
 *   ratio / delta     sensor.py:193-295 (ratio tracking at a majorant) and
 *     sensors         :112-191 (collision estimator), or_trace_estimator
 *   film              film.py:9-21, :40-41 (layout, scatter-add)
 *   render scale      integrators/volume.py:41-54 (inv_vol), :130 (adjoint)
 *   sampler           Mitsuba 'independent' sampler (TEA-scrambled PCG32),
 *                     restated from its published algorithm; draw order of
 *                     common.py:92-108.  Parity with Mitsuba's own stream is
 *                     UNPINNED (mitsuba/drjit are not installed here).
 *
 * Geometry (ray origins, box clip, DDA stepping, voxel choice) is computed in
 * fp32 with the same operation order the reference uses; the per-visit
 * weight exp(-st t)(1-exp(-st dt)) and all sums are evaluated in fp64.
 * Compile with -ffp-contract=off so no FMA is formed implicitly.
 */
#include "../include/tvam.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_RAY_EPS (1500.0f * 5.9604644775390625e-08f) /* math::RayEpsilon<float> */
#define OR_TWO_PI 6.2831855f                           /* float(2*pi) */

/* ------------------------------------------------------------------------ */
/* Sampler: TEA-scrambled PCG32 (Mitsuba IndependentSampler restated)        */
/* ------------------------------------------------------------------------ */
typedef struct { uint64_t state, inc; } or_pcg32;

static uint32_t or_pcg_next(or_pcg32* r) {
    uint64_t old = r->state;
    r->state = old * 0x5851f42d4c957f2dULL + r->inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((~rot + 1u) & 31u));
}

static void or_pcg_seed(or_pcg32* r, uint64_t initstate, uint64_t initseq) {
    r->state = 0u;
    r->inc = (initseq << 1u) | 1u;
    (void)or_pcg_next(r);
    r->state += initstate;
    (void)or_pcg_next(r);
}

static float or_pcg_float(or_pcg32* r) {
    uint32_t bits = (or_pcg_next(r) >> 9) | 0x3f800000u;
    float f;
    memcpy(&f, &bits, 4);
    return f - 1.0f;
}

static void or_tea(uint32_t* v0p, uint32_t* v1p) {
    uint32_t v0 = *v0p, v1 = *v1p, sum = 0;
    for (int i = 0; i < 4; ++i) {
        sum += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + sum) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    *v0p = v0;
    *v1p = v1;
}

static void or_sampler_seed(or_pcg32* r, uint32_t seed, uint64_t wave_index) {
    uint32_t v0 = seed, v1 = (uint32_t)wave_index;
    or_tea(&v0, &v1);
    or_pcg_seed(r, v0, v1);
}

/* ------------------------------------------------------------------------ */
/* Scene constants                                                          */
/* ------------------------------------------------------------------------ */
typedef struct {
    const tvam_desc* d;
    float h[3];         /* voxel size (sensor.py:19)            */
    int res[3];
    float ex, ey;       /* emitter size W*a_x, H*a_y            */
    float inv_w, inv_h; /* rcp(ScalarVector2f(w, h)) (common.py:98) */
    double inv_vol;     /* volume.py:41-42                      */
    double sa_over_st;  /* sensor.py:400, :404                  */
    float st;
    int part;           /* scattering paths: -1 all segments, 0 all but the first, 1 the first only */
    int C;              /* film channels: 1, or 2 = surface-aware (film.py:16-21) */
    const float* inv_volumes; /* surface-aware: 1 / compute_volume() per (voxel, channel), 0 where 0 */
} or_scene;

static void or_scene_init(or_scene* s, const tvam_desc* d) {
    s->d = d;
    for (int k = 0; k < 3; ++k) {
        s->res[k] = d->film_res[k];
        s->h[k] = (d->bbox_max[k] - d->bbox_min[k]) / (float)d->film_res[k];
    }
    s->ex = (float)d->res_x * d->pixel_size_x;
    s->ey = (float)d->res_y * d->pixel_size_y;
    s->inv_w = 1.0f / (float)d->res_x;
    s->inv_h = 1.0f / (float)d->res_y;
    float vol = s->h[0] * s->h[1] * s->h[2];
    s->inv_vol = vol != 0.0f ? 1.0 / (double)vol : 0.0;
    s->st = d->sigma_t;
    s->part = -1;
    s->C = d->film_channels == 2 ? 2 : 1;
    s->inv_volumes = NULL;
    float ss = d->albedo * d->sigma_t;
    s->sa_over_st = d->sigma_t != 0.0f ? ((double)d->sigma_t - (double)ss) / (double)d->sigma_t : 0.0;
}

/* per-ray constant weight: inv_pdf / n_samples * print_time (projector.py:164-165,187; common.py:111) */
static double or_ray_weight(const tvam_desc* d, uint64_t n_active, uint32_t spp) {
    float area = d->pixel_size_x * d->pixel_size_y * (float)n_active;
    float w = area / (float)(n_active * (uint64_t)spp);
    w = w * d->print_time;
    return (double)w;
}

/* ------------------------------------------------------------------------ */
/* Ray generation: common.py:70-116 + projector.py:148-188 + motion.py:26-36 */
/* ------------------------------------------------------------------------ */
typedef struct { float o[3], d[3]; } or_ray;

/* Ray of `pixel` for sampler stream `wave_index`.  Draw order of
   common.py:92-108: position (next_2d, jittered sampling only), time
   (next_1d, sample_time only), then the aperture sample of sample_ray
   (next_2d, always drawn, unused by the collimated projector).  If rng is
   given, it is left after those draws (the path loop continues the stream). */
static void or_gen_ray_rng(const or_scene* s, uint32_t pixel, uint64_t wave_index, uint32_t seed,
                           or_ray* ray, or_pcg32* rng_out) {
    const tvam_desc* d = s->d;
    uint32_t hw = (uint32_t)d->res_y * (uint32_t)d->res_x;
    uint32_t angle = pixel / hw;
    uint32_t pix = pixel % hw;
    uint32_t row = pix / (uint32_t)d->res_x;
    uint32_t col = pix - row * (uint32_t)d->res_x;

    float ox = 0.5f, oy = 0.5f, ot = 0.0f;
    if (!d->regular_sampling || d->sample_time || rng_out) {
        or_pcg32 rng;
        or_sampler_seed(&rng, seed, wave_index);
        if (!d->regular_sampling) {
            ox = or_pcg_float(&rng);
            oy = or_pcg_float(&rng);
        }
        if (d->sample_time) ot = or_pcg_float(&rng);
        if (rng_out) {
            (void)or_pcg_float(&rng); /* aperture sample (projector.py:160) */
            (void)or_pcg_float(&rng);
            *rng_out = rng;
        }
    }
    float u = ((float)col + ox) * s->inv_w;
    float v = ((float)row + oy) * s->inv_h;
    float time = (float)angle;
    if (d->sample_time) time = time + ot;
    time = time / (float)d->n_patterns;

    float alpha = OR_TWO_PI * time;
    if (d->clockwise) alpha = -alpha;
    float c = cosf(alpha), sn = sinf(alpha);

    float xc = (0.5f - u) * s->ex;
    float yc = (0.5f - v) * s->ey;
    const float zc = 0.005f;
    float dz = d->distance - zc;
    ray->o[0] = c * dz + sn * xc;
    ray->o[1] = sn * dz - c * xc;
    ray->o[2] = yc;
    ray->d[0] = -c;
    ray->d[1] = -sn;
    ray->d[2] = 0.0f;
}

static void or_gen_ray(const or_scene* s, uint32_t pixel, uint64_t wave_index, uint32_t seed, or_ray* ray) {
    or_gen_ray_rng(s, pixel, wave_index, seed, ray, NULL);
}

/* ------------------------------------------------------------------------ */
/* Index-matched vial: open cylinder of radius r, |z| <= height/2            */
/* ------------------------------------------------------------------------ */
/* Numerically stable quadratic (Mitsuba math::solve_quadratic restated). */
static int or_solve_quadratic(float a, float b, float c, float* x0, float* x1) {
    float disc = b * b - 4.0f * a * c;
    if (!(disc >= 0.0f)) return 0;
    float sq = sqrtf(disc);
    float temp = -0.5f * (b + copysignf(sq, b));
    float r0 = temp / a, r1 = c / temp;
    *x0 = fminf(r0, r1);
    *x1 = fmaxf(r0, r1);
    return 1;
}

static int or_cyl_roots(const float o[3], const float dd[3], float r, float* t0, float* t1) {
    float A = dd[0] * dd[0] + dd[1] * dd[1];
    float B = 2.0f * (dd[0] * o[0] + dd[1] * o[1]);
    float C = o[0] * o[0] + o[1] * o[1] - r * r;
    return or_solve_quadratic(A, B, C, t0, t1);
}

/* ------------------------------------------------------------------------ */
/* Occluders ('occlusions', geometry.py:55-72): black diffuse triangle       */
/* meshes.  Mitsuba's ray_intersect_triangle restated (Moller-Trumbore,     */
/* t in [0, maxt]); a path that reaches one ends there (black BSDF: weight   */
/* 0, volume.py:245-266).  UNPINNED (OptiX does this on the reference's GPU).*/
/* ------------------------------------------------------------------------ */
static float or_tri_hit(const float o[3], const float dd[3], const float* v) {
    float e1[3], e2[3], tv[3];
    for (int k = 0; k < 3; ++k) {
        e1[k] = v[3 + k] - v[k];
        e2[k] = v[6 + k] - v[k];
        tv[k] = o[k] - v[k];
    }
    float pv[3] = {dd[1] * e2[2] - dd[2] * e2[1], dd[2] * e2[0] - dd[0] * e2[2], dd[0] * e2[1] - dd[1] * e2[0]};
    float inv_det = 1.0f / (e1[0] * pv[0] + e1[1] * pv[1] + e1[2] * pv[2]);
    float u = (tv[0] * pv[0] + tv[1] * pv[1] + tv[2] * pv[2]) * inv_det;
    if (!(u >= 0.0f && u <= 1.0f)) return INFINITY;
    float qv[3] = {tv[1] * e1[2] - tv[2] * e1[1], tv[2] * e1[0] - tv[0] * e1[2], tv[0] * e1[1] - tv[1] * e1[0]};
    float w = (dd[0] * qv[0] + dd[1] * qv[1] + dd[2] * qv[2]) * inv_det;
    if (!(w >= 0.0f && u + w <= 1.0f)) return INFINITY;
    float t = (e2[0] * qv[0] + e2[1] * qv[1] + e2[2] * qv[2]) * inv_det;
    return t >= 0.0f ? t : INFINITY;
}

static float or_occ_hit(const tvam_desc* d, const float o[3], const float dd[3]) {
    float best = INFINITY;
    for (int i = 0; i < d->n_occluder_tris; ++i) best = fminf(best, or_tri_hit(o, dd, d->occluder_tris + 9 * i));
    return best;
}

/* Closed axis-aligned box [-h, h] (Mitsuba 'cube' scaled, geometry.py:186-219):
   nearest t >= 0 (entry from outside, exit from inside), outward face normal. */
static float or_box_hit(const float o[3], const float dd[3], const float h[3], float n[3]) {
    float tn = -INFINITY, tf = INFINITY;
    int an = -1, af = -1;
    for (int a = 0; a < 3; ++a) {
        if (dd[a] == 0.0f) {
            if (!(o[a] >= -h[a] && o[a] <= h[a])) return INFINITY;
            continue;
        }
        float t0 = (-h[a] - o[a]) / dd[a], t1 = (h[a] - o[a]) / dd[a];
        float lo = fminf(t0, t1), hi = fmaxf(t0, t1);
        if (lo > tn) {
            tn = lo;
            an = a;
        }
        if (hi < tf) {
            tf = hi;
            af = a;
        }
    }
    if (!(tn <= tf)) return INFINITY;
    n[0] = n[1] = n[2] = 0.0f;
    if (tn >= 0.0f) {
        n[an] = dd[an] > 0.0f ? -1.0f : 1.0f;
        return tn;
    }
    if (tf >= 0.0f) {
        n[af] = dd[af] > 0.0f ? 1.0f : -1.0f;
        return tf;
    }
    return INFINITY;
}

/* In-medium segment of a projector ray: origin o', maxt.  Returns 0 on miss. */
static int or_segment_index_matched(const or_scene* s, const or_ray* ray, float o2[3], float* maxt) {
    const tvam_desc* d = s->d;
    float half = 0.5f * d->vial_height;
    if (!(ray->o[2] >= -half && ray->o[2] <= half)) return 0; /* passes above/below the open tube */
    float t0, t1;
    if (!or_cyl_roots(ray->o, ray->d, d->vial_r, &t0, &t1)) return 0;
    if (!(t0 >= 0.0f)) return 0; /* projector outside the vial: the entry is the near root */
    if (d->n_occluder_tris && or_occ_hit(d, ray->o, ray->d) < t0) return 0; /* blocked before the vial */
    float p[3];
    for (int k = 0; k < 3; ++k) p[k] = fmaf(ray->d[k], t0, ray->o[k]);
    float rp = sqrtf(p[0] * p[0] + p[1] * p[1]);
    float n[3] = {p[0] / rp, p[1] / rp, 0.0f};
    float m = fmaxf(fmaxf(fabsf(p[0]), fabsf(p[1])), fabsf(p[2]));
    float mag = (1.0f + m) * OR_RAY_EPS;
    float ndd = n[0] * ray->d[0] + n[1] * ray->d[1] + n[2] * ray->d[2];
    if (signbit(ndd)) mag = -mag;
    for (int k = 0; k < 3; ++k) o2[k] = fmaf(mag, n[k], p[k]);
    float u0, u1;
    if (!or_cyl_roots(o2, ray->d, d->vial_r, &u0, &u1)) return 0;
    if (!(u1 > 0.0f)) return 0;
    *maxt = u1;
    if (d->n_occluder_tris) *maxt = fminf(u1, or_occ_hit(d, o2, ray->d)); /* ends on an occluder */
    return 1;
}

/* ------------------------------------------------------------------------ */
/* Cylindrical vial (geometry.py:142-183): glass tube between r_int and r_ext */
/* ------------------------------------------------------------------------ */
#define OR_IOR_AIR 1.000277f

/* Nearest hit t >= 0 of an open tube |z| <= half (Mitsuba cylinder restated). */
static float or_tube_hit(const float o[3], const float dd[3], float r, float half) {
    float t0, t1;
    if (!or_cyl_roots(o, dd, r, &t0, &t1)) return INFINITY;
    if (!(t1 >= 0.0f)) return INFINITY;
    float zn = fmaf(dd[2], t0, o[2]), zf = fmaf(dd[2], t1, o[2]);
    if (t0 >= 0.0f && zn >= -half && zn <= half) return t0;
    if (zf >= -half && zf <= half) return t1;
    return INFINITY;
}

/* Mitsuba fresnel(cos_theta_i, eta): reflectance, cos_theta_t, eta_ti. */
static float or_fresnel(float cos_i, float eta, float* cos_t, float* eta_ti) {
    int outside = cos_i >= 0.0f;
    float rcp_eta = 1.0f / eta;
    float eta_it = outside ? eta : rcp_eta;
    *eta_ti = outside ? rcp_eta : eta;
    float ct2 = 1.0f - (1.0f - cos_i * cos_i) * (*eta_ti * *eta_ti);
    float ci = fabsf(cos_i), ct = sqrtf(fmaxf(ct2, 0.0f));
    float r;
    if (eta == 1.0f) r = 0.0f;
    else if (ci == 0.0f) r = 1.0f;
    else {
        float a_s = (ci - eta_it * ct) / (ci + eta_it * ct);
        float a_p = (ct - eta_it * ci) / (ct + eta_it * ci);
        r = 0.5f * (a_s * a_s + a_p * a_p);
    }
    *cos_t = outside ? -ct : ct;
    return r;
}

/* Transmission through the tube surface point p (outward normal n) for a ray
   of direction d; eta = int_ior / ext_ior.  Mitsuba dielectric sample() with
   only the transmission lobe (volume.py:230-237): wo = refract(wi) in the
   frame (s = dp_du/|dp_du|, t = z, n), weight (1 - F) * eta_ti^2.  Returns
   the weight (0 on total internal reflection). */
static float or_transmit(const float n[3], const float d[3], float eta, float wo[3]) {
    float sx = -n[1], sy = n[0];                           /* dp_du = (-y, x, 0) normalised */
    float wl_x = -(d[0] * sx + d[1] * sy);                 /* wi = to_local(-d) */
    float wl_y = -d[2];
    float wl_z = -(d[0] * n[0] + d[1] * n[1]);
    float cos_t, eta_ti;
    float r = or_fresnel(wl_z, eta, &cos_t, &eta_ti);
    float t = 1.0f - r;
    if (!(t > 0.0f)) return 0.0f;
    float ox = -eta_ti * wl_x, oy = -eta_ti * wl_y;        /* refract(wi, cos_t, eta_ti) */
    wo[0] = sx * ox + n[0] * cos_t;                        /* to_world */
    wo[1] = sy * ox + n[1] * cos_t;
    wo[2] = oy;
    return t * (eta_ti * eta_ti);
}

/* Medium segment of a projector ray through the glass tube: surface hits in
   order (nearest of the two tubes), transmission at each, until the ray runs
   inside the inner tube; the segment ends at its next hit.  Returns 0 when
   the ray never enters the medium (misses, TIR, or runs out of max_depth). */
static int or_segment_cylindrical(const or_scene* s, const or_ray* ray, float o2[3], float d2[3], float* maxt,
                                  double* weight) {
    const tvam_desc* d = s->d;
    float half = 0.5f * d->vial_height;
    float o[3] = {ray->o[0], ray->o[1], ray->o[2]}, dd[3] = {ray->d[0], ray->d[1], ray->d[2]};
    float att = 1.0f; /* Spectrum attenuation: fp32 products (volume.py:265) */
    int in_medium = 0;
    for (int depth = 0; depth < d->max_depth; ++depth) {
        float te = or_tube_hit(o, dd, d->vial_r_ext, half), ti = or_tube_hit(o, dd, d->vial_r, half);
        int inner = ti <= te;
        float t = inner ? ti : te;
        if (d->n_occluder_tris) {
            float toc = or_occ_hit(d, o, dd);
            if (toc < t) { /* an occluder: the segment ends there, or the ray dies outside the medium */
                if (!in_medium) return 0;
                t = toc;
            }
        }
        if (!(t < INFINITY)) return 0;
        if (in_medium) { /* the medium segment [0, t] (volume.py:209-216) */
            for (int k = 0; k < 3; ++k) {
                o2[k] = o[k];
                d2[k] = dd[k];
            }
            *maxt = t;
            *weight = (double)att;
            return 1;
        }
        float p[3];
        for (int k = 0; k < 3; ++k) p[k] = fmaf(dd[k], t, o[k]);
        float rp = sqrtf(p[0] * p[0] + p[1] * p[1]);
        float n[3] = {p[0] / rp, p[1] / rp, 0.0f};
        float eta = inner ? d->medium_ior / d->vial_ior : d->vial_ior / OR_IOR_AIR;
        float wo[3];
        float w = or_transmit(n, dd, eta, wo);
        if (!(w > 0.0f)) return 0;
        att = att * w;
        /* spawn_ray(si.to_world(bs.wo)): offset_p along n, towards wo */
        float m = fmaxf(fmaxf(fabsf(p[0]), fabsf(p[1])), fabsf(p[2]));
        float mag = (1.0f + m) * OR_RAY_EPS;
        float nwo = n[0] * wo[0] + n[1] * wo[1] + n[2] * wo[2];
        if (signbit(nwo)) mag = -mag;
        for (int k = 0; k < 3; ++k) {
            o[k] = fmaf(mag, n[k], p[k]);
            dd[k] = wo[k];
        }
        /* the inner tube's interior is the printing medium (volume.py:268) */
        in_medium = inner && nwo < 0.0f;
    }
    return 0;
}

/* Diagnostics: segments whose DDA starts with a valid axis that never steps because its
   first crossing time came out negative in fp32 (sensor.py:358). */
static uint64_t or_frozen_axes = 0;
uint64_t oracle_frozen_axes(int reset) {
    uint64_t v = or_frozen_axes;
    if (reset) or_frozen_axes = 0;
    return v;
}

/* DDA declared ahead for the scattering path */
static double or_dda(const or_scene* s, const float o[3], const float dd[3], float maxt, double em,
                     int mode, double* film, const float* grad, int only_slice, uint64_t* visits);

/* Square vial (geometry.py:186-219): glass cuboids, outer [-w_ext/2, w_ext/2]^2
   x [-h/2, h/2] (dielectric air|glass), inner [-w_int/2, w_int/2]^2 x
   [-0.45 h, 0.45 h] (glass|medium, interior = the medium).  Same loop as the
   tubes; the transmission uses the world-space form of Mitsuba's refract()
   (wo = -eta_ti wi + (eta_ti cos_i + cos_t) n, frame-independent for the
   cube's faces). */
static float or_transmit_world(const float n[3], const float dd[3], float eta, float wo[3]) {
    float cos_i = -(dd[0] * n[0] + dd[1] * n[1] + dd[2] * n[2]);
    float cos_t, eta_ti;
    float r = or_fresnel(cos_i, eta, &cos_t, &eta_ti);
    float t = 1.0f - r;
    if (!(t > 0.0f)) return 0.0f;
    float c = eta_ti * cos_i + cos_t;
    for (int k = 0; k < 3; ++k) wo[k] = eta_ti * dd[k] + c * n[k];
    return t * (eta_ti * eta_ti);
}

static void or_square_extents(const tvam_desc* d, float he[3], float hi[3]) {
    he[0] = he[1] = d->vial_r_ext;
    he[2] = 0.5f * d->vial_height;
    hi[0] = hi[1] = d->vial_r;
    hi[2] = (float)(0.5 * 0.9 * (double)d->vial_height);
}

static int or_segment_square(const or_scene* s, const or_ray* ray, float o2[3], float d2[3], float* maxt,
                             double* weight) {
    const tvam_desc* d = s->d;
    float he[3], hi[3];
    or_square_extents(d, he, hi);
    float o[3] = {ray->o[0], ray->o[1], ray->o[2]}, dd[3] = {ray->d[0], ray->d[1], ray->d[2]};
    float att = 1.0f;
    int in_medium = 0;
    for (int depth = 0; depth < d->max_depth; ++depth) {
        float ne[3], ni[3];
        float te = or_box_hit(o, dd, he, ne), ti = or_box_hit(o, dd, hi, ni);
        int inner = ti <= te;
        float t = inner ? ti : te;
        if (d->n_occluder_tris) {
            float toc = or_occ_hit(d, o, dd);
            if (toc < t) {
                if (!in_medium) return 0;
                t = toc;
            }
        }
        if (!(t < INFINITY)) return 0;
        if (in_medium) {
            for (int k = 0; k < 3; ++k) {
                o2[k] = o[k];
                d2[k] = dd[k];
            }
            *maxt = t;
            *weight = (double)att;
            return 1;
        }
        const float* n = inner ? ni : ne;
        float p[3];
        for (int k = 0; k < 3; ++k) p[k] = fmaf(dd[k], t, o[k]);
        float eta = inner ? d->medium_ior / d->vial_ior : d->vial_ior / OR_IOR_AIR;
        float wo[3];
        float w = or_transmit_world(n, dd, eta, wo);
        if (!(w > 0.0f)) return 0;
        att = att * w;
        float m = fmaxf(fmaxf(fabsf(p[0]), fabsf(p[1])), fabsf(p[2]));
        float mag = (1.0f + m) * OR_RAY_EPS;
        float nwo = n[0] * wo[0] + n[1] * wo[1] + n[2] * wo[2];
        if (signbit(nwo)) mag = -mag;
        for (int k = 0; k < 3; ++k) {
            o[k] = fmaf(mag, n[k], p[k]);
            dd[k] = wo[k];
        }
        in_medium = inner && nwo < 0.0f;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Scattering media: the full path loop of volume.py:179-272  */
/* with has_scattering (sigma_s != 0).  Mitsuba internals restated (UNPINNED):*/
/*   homogeneous medium  sample_interaction: t = -log(1 - u) / sigma_t        */
/*                       (mint 0, unbounded medium); transmittance_eval_pdf:  */
/*                       tr = exp(-min(t_mi, t_si) sigma_t), pdf = tr at a    */
/*                       surface, tr * sigma_t at a medium interaction;       */
/*                       sigma_s = albedo * sigma_t                          */
/*   phase functions     isotropic (square_to_uniform_sphere), rayleigh      */
/*                       (cbrt inversion of the (1 + cos^2) CDF), hg; local   */
/*                       directions mapped by Frame3f(wi = -d) built with     */
/*                       coordinate_system() (Duff et al.)                    */
/*   medium spawn_ray    origin p = o + t d, no offset (n = 0)               */
/* Draw order per loop iteration: RR next_1d (every iteration), the medium   */
/* next_1d (every iteration), BSDF next_1d + next_2d (surface lanes only),   */
/* phase next_1d + next_2d (scattering lanes only).                          */
/* Every medium segment deposits its analytic absorption up to the next      */
/* surface (sensor.py:383-438 with maxt = si.t), weighted by the path        */
/* attenuation (sensor.py:367-381: throughput * exp(-st t_prev) * ss^n_scat  */
/* == attenuation in primal mode); the path continues from the sampled       */
/* interaction.  A segment whose ray escapes through an open tube end has no */
/* surface (si invalid) and deposits nothing (volume.py:191-196).            */
/* ------------------------------------------------------------------------ */
static void or_coordinate_system(const float n[3], float s[3], float t[3]) {
    float sign = copysignf(1.0f, n[2]);
    float a = -1.0f / (sign + n[2]);
    float b = n[0] * n[1] * a;
    s[0] = copysignf(1.0f, n[2]) * (n[0] * n[0] * a) + 1.0f; /* mulsign(x^2 a, n.z) + 1 */
    s[1] = copysignf(1.0f, n[2]) * b;
    s[2] = -copysignf(1.0f, n[2]) * n[0];                   /* mulsign_neg(n.x, n.z) */
    t[0] = b;
    t[1] = fmaf(n[1], n[1] * a, sign);
    t[2] = -n[1];
}

/* Phase-function sample: direction wo for a ray of direction dd (wi = -dd). */
static void or_phase_sample(const tvam_desc* d, const float dd[3], float u1, float u2, float wo[3]) {
    float lx, ly, lz;
    if (d->phase_type == TVAM_PHASE_ISOTROPIC) {
        /* warp::square_to_uniform_sphere(sample) in world space: z = 1 - 2 sample.y,
           phi = 2 pi sample.x */
        float z = 1.0f - 2.0f * u2;
        float r = sqrtf(fmaxf(1.0f - z * z, 0.0f));
        float sp = sinf(OR_TWO_PI * u1), cp = cosf(OR_TWO_PI * u1);
        wo[0] = r * cp;
        wo[1] = r * sp;
        wo[2] = z;
        return;
    }
    if (d->phase_type == TVAM_PHASE_RAYLEIGH) {
        float z = 2.0f * (2.0f * u1 - 1.0f);
        float tmp = sqrtf(z * z + 1.0f);
        float A = cbrtf(z + tmp), B = cbrtf(z - tmp);
        float ct = A + B;
        float st = sqrtf(fmaxf(1.0f - ct * ct, 0.0f));
        float sp = sinf(OR_TWO_PI * u2), cp = cosf(OR_TWO_PI * u2);
        lx = st * cp;
        ly = st * sp;
        lz = ct;
    } else { /* Henyey-Greenstein */
        float g = d->phase_g;
        float ct;
        if (fabsf(g) < 5.9604644775390625e-08f) {
            ct = 1.0f - 2.0f * u1;
        } else {
            float sq = (1.0f - g * g) / (1.0f - g + 2.0f * g * u1);
            ct = (1.0f + g * g - sq * sq) / (2.0f * g);
        }
        float st = sqrtf(fmaxf(1.0f - ct * ct, 0.0f));
        float sp = sinf(OR_TWO_PI * u2), cp = cosf(OR_TWO_PI * u2);
        lx = st * cp;
        ly = st * sp;
        lz = -ct;
    }
    float n[3] = {-dd[0], -dd[1], -dd[2]}, sv[3], tv[3];
    or_coordinate_system(n, sv, tv);
    for (int k = 0; k < 3; ++k) wo[k] = sv[k] * lx + tv[k] * ly + n[k] * lz;
}

/* Nearest container surface along (o, dd): t, hit point, outward normal and
   which tube (0 outer glass, 1 inner / index-matched tube).  INFINITY on a miss. */
static float or_container_hit(const or_scene* s, const float o[3], const float dd[3], int* which) {
    const tvam_desc* d = s->d;
    float half = 0.5f * d->vial_height;
    float t;
    *which = 1;
    if (d->vial_type == TVAM_VIAL_SQUARE) {
        float he[3], hi[3], n[3];
        or_square_extents(d, he, hi);
        t = or_box_hit(o, dd, hi, n);
    } else {
        t = or_tube_hit(o, dd, d->vial_r, half);
        if (d->vial_type == TVAM_VIAL_CYLINDRICAL) {
            float te = or_tube_hit(o, dd, d->vial_r_ext, half);
            if (!(t <= te)) {
                *which = 0;
                t = te;
            }
        }
    }
    if (d->n_occluder_tris) {
        float toc = or_occ_hit(d, o, dd);
        if (toc < t) {
            *which = 2;
            t = toc;
        }
    }
    return t;
}

/* One scattering path (volume.py:179-272).  The first medium segment is the
   non-scattering one (or_segment_*), then free flights until the path
   leaves the medium, escapes, hits max_depth, or Russian roulette ends it.
   first_only < 0: every segment; 0: all but the first (the GPU's scatter
   pass); 1: only the first. */
static double or_trace_scatter(const or_scene* s, uint32_t pixel, uint64_t wave_index, uint32_t seed, double em,
                               int mode, double* film, const float* grad, uint64_t* visits, int first_only) {
    const tvam_desc* d = s->d;
    or_ray ray;
    or_pcg32 rng;
    or_gen_ray_rng(s, pixel, wave_index, seed, &ray, &rng);
    float o[3], dd[3], maxt;
    double attd = 1.0;
    int nsurf;
    if (d->vial_type == TVAM_VIAL_CYLINDRICAL || d->vial_type == TVAM_VIAL_SQUARE) {
        if (!(d->vial_type == TVAM_VIAL_SQUARE ? or_segment_square(s, &ray, o, dd, &maxt, &attd)
                                               : or_segment_cylindrical(s, &ray, o, dd, &maxt, &attd)))
            return 0.0;
        nsurf = 2;
    } else {
        if (d->max_depth < 2 || !or_segment_index_matched(s, &ray, o, &maxt)) return 0.0;
        for (int k = 0; k < 3; ++k) dd[k] = ray.d[k];
        nsurf = 1;
    }
    /* the surface iterations before the medium: RR, medium, BSDF 1d + 2d */
    for (int i = 0; i < 5 * nsurf; ++i) (void)or_pcg_float(&rng);
    float att = (float)attd;
    int depth = nsurf;
    const float st = d->sigma_t, ss = d->albedo * d->sigma_t;
    double acc = 0.0;
    for (int seg = 0;; ++seg) {
        const float q = fminf(0.99f, att);
        const float u_rr = or_pcg_float(&rng);
        if (depth > d->rr_depth) { /* volume.py:182-185 */
            if (!(u_rr < q)) break;
            att = att * (1.0f / q);
        }
        if (!(att != 0.0f)) break;
        float tsi = maxt;
        if (seg > 0) {
            int which;
            tsi = or_container_hit(s, o, dd, &which);
            if (!(tsi < INFINITY)) break; /* escapes through an open end: no surface, no deposit */
        }
        const float u_m = or_pcg_float(&rng);
        const float tmi = -logf(1.0f - u_m) / st;
        const int reached = tsi < tmi;
        /* deposit along [0, si.t] */
        if (first_only < 0 || (first_only == 0 && seg > 0) || (first_only == 1 && seg == 0)) {
            if (mode == 0 || mode == 3) (void)or_dda(s, o, dd, tsi, em * (double)att, mode, film, NULL, -1, visits);
            else acc += (double)att * or_dda(s, o, dd, tsi, em, mode, NULL, grad, -1, visits);
        }
        if (reached || first_only == 1) break; /* leaves the medium for good (transmission only, convex) */
        const float tr = expf(-tmi * st);
        const float pdf = tr * st;
        const float inv = pdf > 0.0f ? 1.0f / pdf : 0.0f;
        float w = tr * inv;
        w = w * ss;
        (void)or_pcg_float(&rng); /* phase next_1d (unused) */
        const float u1 = or_pcg_float(&rng), u2 = or_pcg_float(&rng);
        float wo[3];
        or_phase_sample(d, dd, u1, u2, wo);
        for (int k = 0; k < 3; ++k) {
            o[k] = fmaf(dd[k], tmi, o[k]);
            dd[k] = wo[k];
        }
        att = att * w;
        ++depth;
        if (depth >= d->max_depth) break;
    }
    return acc;
}

/* ------------------------------------------------------------------------ */
/* DDA (sensor.py:327-438).  mode 0: forward (accumulate into film),          */
/* mode 1: adjoint (gather grad), mode 2: count only.                        */
/* ------------------------------------------------------------------------ */
static double or_dda(const or_scene* s, const float o[3], const float dd[3], float maxt, double em,
                     int mode, double* film, const float* grad, int only_slice, uint64_t* visits) {
    const tvam_desc* d = s->d;
    float tbmin[3], tbmax[3];
    for (int k = 0; k < 3; ++k) {
        tbmin[k] = (d->bbox_min[k] - o[k]) / dd[k];
        tbmax[k] = (d->bbox_max[k] - o[k]) / dd[k];
    }
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        lo[k] = fminf(tbmin[k], tbmax[k]);
        hi[k] = fmaxf(tbmin[k], tbmax[k]);
    }
    float mint_box = fmaxf(fmaxf(fmaxf(lo[0], lo[1]), lo[2]), 0.0f);
    float maxt_box = fminf(fminf(hi[0], hi[1]), hi[2]);
    float t_start = fmaxf(mint_box, 0.0f);
    float t_end = fminf(maxt_box, maxt);
    if (!(isfinite(t_start) && isfinite(t_end) && t_start < t_end)) return 0.0;

    float gs[3], ge[3];
    int step[3], cur[3], endv[3];
    float dtmax[3], tstep[3];
    for (int k = 0; k < 3; ++k) {
        gs[k] = fmaf(dd[k], t_start, o[k]);
        ge[k] = fmaf(dd[k], t_end, o[k]);
        step[k] = dd[k] > 0.0f ? 1 : -1;
        int sv = (int)((gs[k] - d->bbox_min[k]) / s->h[k]);
        int ev = (int)((ge[k] - d->bbox_min[k]) / s->h[k]);
        sv = sv < 0 ? 0 : (sv > s->res[k] - 1 ? s->res[k] - 1 : sv);
        ev = ev < 0 ? 0 : (ev > s->res[k] - 1 ? s->res[k] - 1 : ev);
        cur[k] = sv;
        endv[k] = ev;
        float next = d->bbox_min[k] + (float)(sv + step[k]) * s->h[k];
        if (dd[k] < 0.0f) next = next + s->h[k];
        int valid = fabsf(dd[k]) > 1e-8f;
        dtmax[k] = valid ? (next - gs[k]) / dd[k] : INFINITY;
        if (dtmax[k] < 0.0f) { /* sensor.py:358: the axis never steps ("frozen") */
            dtmax[k] = INFINITY;
            if (valid) {
#ifdef _OPENMP
#pragma omp atomic
#endif
                ++or_frozen_axes;
            }
        }
        tstep[k] = valid ? (s->h[k] / dd[k]) * (float)step[k] : INFINITY;
    }
    if (only_slice >= 0 && cur[2] != only_slice) return 0.0;

    float t = t_start;
    float remaining = t_end - t_start;
    double st = (double)s->st;
    double acc = 0.0;
    uint64_t nv = 0;
    for (;;) {
        float dt = fminf(fminf(fminf(dtmax[0], dtmax[1]), dtmax[2]), remaining);
        remaining = remaining - dt;
        double w = s->sa_over_st * exp(-st * (double)t) * (1.0 - exp(-st * (double)fmaxf(dt, 0.0f)));
        /* film index (sensor.py:405-409): x + y res.x + z res.x res.y, times C; the
           surface-aware channel offset is folded into the film / grad pointer */
        size_t idx = ((size_t)cur[0] + (size_t)cur[1] * (size_t)s->res[0] +
                      (size_t)cur[2] * (size_t)s->res[0] * (size_t)s->res[1]) * (size_t)s->C;
        if (mode == 0) film[idx] += em * w;
        else if (mode == 3) {
#ifdef _OPENMP
#pragma omp atomic
#endif
            film[idx] += em * w;
        }
        else if (mode == 1) acc += w * (double)grad[idx];
        ++nv;
        int alive = (cur[0] != endv[0] || cur[1] != endv[1] || cur[2] != endv[2]) && (remaining > 1e-6f);
        if (!alive) break;
        for (int k = 0; k < 3; ++k) {
            int m = dtmax[k] == dt;
            dtmax[k] = m ? tstep[k] : dtmax[k] - dt;
            if (m) cur[k] += step[k];
        }
        if (cur[0] < 0 || cur[1] < 0 || cur[2] < 0 || cur[0] >= s->res[0] || cur[1] >= s->res[1] ||
            cur[2] >= s->res[2])
            break;
        t = t + dt;
    }
    if (visits) *visits += nv;
    return acc;
}

/* pixel index of active entry i (dense crop order if active_pixels is NULL, projector.py:90-98) */
static uint32_t or_pixel(const tvam_desc* d, const uint32_t* active_pixels, uint64_t i) {
    if (active_pixels) return active_pixels[i];
    uint64_t cs = (uint64_t)d->crop_x * (uint64_t)d->crop_y;
    uint64_t a = i / cs, r = i % cs;
    uint64_t row = r / (uint64_t)d->crop_x, col = r % (uint64_t)d->crop_x;
    return (uint32_t)(a * (uint64_t)d->res_x * (uint64_t)d->res_y +
                      ((uint64_t)d->crop_offset_y + row) * (uint64_t)d->res_x + col +
                      (uint64_t)d->crop_offset_x);
}

/* Sampler stream of active entry i (before the * spp + sample): the reference seeds
   sampler.seed(seed, active_size * spp) and repeats active_pixels spp times
   (common.py:57-67, :81), so entry i of projector.active_pixels draws streams
   i*spp .. i*spp+spp-1.  For the dense crop order i is the dense crop index; a
   sparse set that is one shard of a larger one starts at desc.active_base. */
static uint64_t or_stream(const tvam_desc* d, const uint32_t* active_pixels, uint64_t i) {
    return active_pixels ? (uint64_t)d->active_base + i : i;
}

/* len(projector.active_data) the ray weight divides by (projector.py:164-165, :187) */
static uint64_t or_n_total(const tvam_desc* d, uint64_t n_active) {
    return d->active_total > 0 ? (uint64_t)d->active_total : n_active;
}

static int or_check(const tvam_desc* d) {
    if (d->vial_type != TVAM_VIAL_INDEX_MATCHED && d->vial_type != TVAM_VIAL_CYLINDRICAL &&
        d->vial_type != TVAM_VIAL_SQUARE)
        return TVAM_ERR_UNSUPPORTED;
    if (d->n_occluder_tris < 0 || (d->n_occluder_tris > 0 && !d->occluder_tris)) return TVAM_ERR_INVALID;
    if (d->projector_type != TVAM_PROJECTOR_COLLIMATED) return TVAM_ERR_UNSUPPORTED;
    if (d->film_channels != 1 && d->film_channels != 2) return TVAM_ERR_UNSUPPORTED;
    if (d->film_channels == 2 && (d->n_target_tris <= 0 || !d->target_tris)) return TVAM_ERR_INVALID;
    if (d->sensor_type != TVAM_SENSOR_DDA && d->sensor_type != TVAM_SENSOR_RATIO && d->sensor_type != TVAM_SENSOR_DELTA)
        return TVAM_ERR_INVALID;
    if (d->sensor_type == TVAM_SENSOR_DELTA && d->albedo == 0.0f) return TVAM_ERR_INVALID; /* volume.py:160-161 */
    if (d->sensor_type == TVAM_SENSOR_RATIO && !(d->majorant > 0.0f)) return TVAM_ERR_INVALID;
    if (d->albedo < 0.0f || d->albedo > 1.0f) return TVAM_ERR_INVALID;
    if (d->albedo != 0.0f && !(d->sigma_t > 0.0f)) return TVAM_ERR_INVALID;
    if (d->phase_type < TVAM_PHASE_ISOTROPIC || d->phase_type > TVAM_PHASE_HG) return TVAM_ERR_INVALID;
    /* Russian roulette (volume.py:182-185, depth > rr_depth) before the medium
       segment (path vertex 1 index matched, 2 behind the glass) is not restated */
    if (d->rr_depth < (d->vial_type == TVAM_VIAL_INDEX_MATCHED ? 1 : 2)) return TVAM_ERR_UNSUPPORTED;
    return 0;
}

/* Deposit / gather at point p of a medium segment (ratio / delta sensors: the voxel is
   floor((p - bbox.min) / voxel_size), skipped outside the grid; sensor.py:143-146, :248-252). */
static double or_point(const or_scene* s, const float p[3], double w, int mode, double* film, const float* grad,
                       uint64_t* visits) {
    const tvam_desc* d = s->d;
    int v[3];
    for (int k = 0; k < 3; ++k) {
        v[k] = (int)floorf((p[k] - d->bbox_min[k]) / s->h[k]);
        if (v[k] < 0 || v[k] >= s->res[k]) return 0.0;
    }
    size_t idx = ((size_t)v[0] + (size_t)v[1] * (size_t)s->res[0] + (size_t)v[2] * (size_t)s->res[0] * (size_t)s->res[1]) *
                 (size_t)s->C;
    if (visits) ++*visits;
    if (mode == 0) film[idx] += w;
    else if (mode == 3) {
#ifdef _OPENMP
#pragma omp atomic
#endif
        film[idx] += w;
    } else if (mode == 1) return w * (double)grad[idx];
    return 0.0;
}

/* spawn_ray at a target hit (t along (o, dd), triangle tri): offset_p along the geometric
   normal, away from the side the ray came from; o becomes the new origin. */
static void or_spawn_target(const tvam_desc* d, int tri, float t, float o[3], const float dd[3]) {
    const float* v = d->target_tris + 9 * tri;
    float e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]}, e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
    float c[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
    float ninv = 1.0f / sqrtf(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    float n[3], p[3];
    for (int k = 0; k < 3; ++k) {
        n[k] = c[k] * ninv;
        p[k] = fmaf(dd[k], t, o[k]);
    }
    float m = fmaxf(fmaxf(fabsf(p[0]), fabsf(p[1])), fabsf(p[2]));
    float mag = (1.0f + m) * OR_RAY_EPS;
    if (signbit(n[0] * dd[0] + n[1] * dd[1] + n[2] * dd[2])) mag = -mag;
    for (int k = 0; k < 3; ++k) o[k] = fmaf(mag, n[k], p[k]);
}

static float or_target_hit(const tvam_desc* d, const float o[3], const float dd[3], int* tri);

/* The path loop (volume.py:179-272) with the 'ratio' or 'delta' sensor (sensor.py:112-295):
   every medium segment [0, si.t) of the path either
     ratio:  steps t += -log(1 - u) / majorant (one sampler draw per step, inside accumulate,
             i.e. after the free-flight draw and before the BSDF / phase draws) and deposits
             att * (sa / st) * em * (1 - st / majorant)^k * st / majorant at ray(t), k = the
             step's index, while t < si.t;
     delta:  deposits att * (sa / st) * em at the medium interaction ray(mei.t) when the free
             flight ends before the surface (mei valid; tr * inv_pdf = 1 / st).
   Scattering continues the path as in or_trace_scatter; non-scattering media (ratio only:
   delta needs scattering, volume.py:160-161) have one segment and no free-flight draw. */
static double or_trace_estimator(const or_scene* s, uint32_t pixel, uint64_t wave_index, uint32_t seed, double em,
                                 int mode, double* film, const float* grad, uint64_t* visits) {
    const tvam_desc* d = s->d;
    or_ray ray;
    or_pcg32 rng;
    or_gen_ray_rng(s, pixel, wave_index, seed, &ray, &rng);
    const int has_sc = d->albedo != 0.0f;
    float o[3], dd[3], maxt;
    double attd = 1.0;
    int nsurf;
    if (d->vial_type == TVAM_VIAL_CYLINDRICAL || d->vial_type == TVAM_VIAL_SQUARE) {
        if (!(d->vial_type == TVAM_VIAL_SQUARE ? or_segment_square(s, &ray, o, dd, &maxt, &attd)
                                               : or_segment_cylindrical(s, &ray, o, dd, &maxt, &attd)))
            return 0.0;
        nsurf = 2;
    } else {
        if (d->max_depth < 2 || !or_segment_index_matched(s, &ray, o, &maxt)) return 0.0;
        for (int k = 0; k < 3; ++k) dd[k] = ray.d[k];
        nsurf = 1;
    }
    /* the surface iterations before the medium: RR, (medium), BSDF 1d + 2d */
    for (int i = 0; i < (has_sc ? 5 : 4) * nsurf; ++i) (void)or_pcg_float(&rng);
    float att = (float)attd;
    int depth = nsurf;
    const float st = d->sigma_t, ss = d->albedo * d->sigma_t;
    const float mj = d->majorant;
    double acc = 0.0;
    /* surface-aware film (C = 2): the target mesh cuts the segments as in or_trace_surface_scatter;
       the deposits go to channel 0 inside the target, 1 outside (sensor.py:148-151, :257-260) */
    const int sa = s->C == 2;
    int inside = 0, cut = 0;
    for (int seg = 0;; ++seg) {
        const float q = fminf(0.99f, att);
        const float u_rr = or_pcg_float(&rng);
        if (depth > d->rr_depth) {
            if (!(u_rr < q)) break;
            att = att * (1.0f / q);
        }
        if (!(att != 0.0f)) break;
        float tsi = maxt;
        if (seg > 0 || cut) {
            int which;
            tsi = or_container_hit(s, o, dd, &which);
            if (!(tsi < INFINITY)) break;
        }
        int tri = -1, hit = 0;
        float tt = INFINITY;
        if (sa) {
            tt = or_target_hit(d, o, dd, &tri);
            hit = tt < tsi;
            if (hit) tsi = tt;
        }
        double* film_c = film ? film + (inside ? 0 : 1) * sa : NULL;
        const float* grad_c = grad ? grad + (inside ? 0 : 1) * sa : NULL;
        float tmi = INFINITY;
        if (has_sc) {
            const float u_m = or_pcg_float(&rng);
            tmi = -logf(1.0f - u_m) / st;
        }
        const int reached = !(tmi <= tsi);
        const double wseg = (double)att * s->sa_over_st;
        if (d->sensor_type == TVAM_SENSOR_RATIO) {
            float t = 0.0f;
            double pk = 1.0;
            const double ratio = (double)st / (double)mj;
            for (int it = 0; it < (1 << 20); ++it) {
                const float u = or_pcg_float(&rng);
                t = t + (-logf(1.0f - u) / mj);
                if (!(t < tsi)) break;
                float p[3];
                for (int k = 0; k < 3; ++k) p[k] = fmaf(dd[k], t, o[k]);
                const double w = wseg * pk * ratio;
                if (mode == 1) acc += or_point(s, p, w, 1, NULL, grad_c, visits);
                else or_point(s, p, w * em, mode, film_c, NULL, visits);
                pk *= 1.0 - ratio;
            }
        } else if (!reached) { /* delta: the medium interaction */
            float p[3];
            for (int k = 0; k < 3; ++k) p[k] = fmaf(dd[k], tmi, o[k]);
            if (mode == 1) acc += or_point(s, p, wseg, 1, NULL, grad_c, visits);
            else or_point(s, p, wseg * em, mode, film_c, NULL, visits);
        }
        if (reached && hit) { /* the target's null BSDF: pass through, depth unchanged (volume.py:271) */
            if (has_sc) {
                const float tr = expf(-tsi * st);
                const float inv = tr > 0.0f ? 1.0f / tr : 0.0f;
                att = att * (tr * inv); /* transmittance_eval_pdf: tr / pdf, pdf = tr */
            } else {
                att = att * expf(-st * tsi); /* volume.py:263 */
            }
            for (int i = 0; i < 3; ++i) (void)or_pcg_float(&rng); /* BSDF next_1d + next_2d */
            inside = !inside;
            cut = 1;
            or_spawn_target(d, tri, tt, o, dd);
            continue;
        }
        if (reached) break;
        const float tr = expf(-tmi * st);
        const float pdf = tr * st;
        const float inv = pdf > 0.0f ? 1.0f / pdf : 0.0f;
        float w = tr * inv;
        w = w * ss;
        (void)or_pcg_float(&rng); /* phase next_1d (unused) */
        const float u1 = or_pcg_float(&rng), u2 = or_pcg_float(&rng);
        float wo[3];
        or_phase_sample(d, dd, u1, u2, wo);
        for (int k = 0; k < 3; ++k) {
            o[k] = fmaf(dd[k], tmi, o[k]);
            dd[k] = wo[k];
        }
        att = att * w;
        ++depth;
        if (depth >= d->max_depth) break;
    }
    return acc;
}

/* Nearest target-mesh hit along (o, dd) (Moller-Trumbore over every triangle); *tri = its index. */
static float or_target_hit(const tvam_desc* d, const float o[3], const float dd[3], int* tri) {
    float best = INFINITY;
    *tri = -1;
    for (int i = 0; i < d->n_target_tris; ++i) {
        float t = or_tri_hit(o, dd, d->target_tris + 9 * i);
        if (t < best) {
            best = t;
            *tri = i;
        }
    }
    return best;
}

/* Surface-aware path (film_channels 2, non-scattering; volume.py:179-272 with the target
   mesh in the scene, null BSDF): the medium segment is cut at every target hit.  Each
   piece deposits from its own origin into channel 0 while inside the target, 1 outside
   (inside_target toggles on each hit, starting outside: volume.py:175, :218); reaching a
   surface multiplies the attenuation by e^{-st si.t} (:263, :266); a target hit spawns the
   next piece at the hit point offset along the face normal (spawn_ray / offset_p) and does
   not count towards max_depth (:271); the piece ending at the container (or an occluder)
   is the last one deposited. */
static double or_trace_surface(const or_scene* s, uint32_t pixel, uint64_t wave_index, uint32_t seed, double em,
                               int mode, double* film, const float* grad, int only_slice, uint64_t* visits) {
    const tvam_desc* d = s->d;
    or_ray ray;
    or_gen_ray(s, pixel, wave_index, seed, &ray);
    float o[3], dd[3], maxt;
    double attd = 1.0;
    if (d->vial_type == TVAM_VIAL_CYLINDRICAL || d->vial_type == TVAM_VIAL_SQUARE) {
        if (!(d->vial_type == TVAM_VIAL_SQUARE ? or_segment_square(s, &ray, o, dd, &maxt, &attd)
                                               : or_segment_cylindrical(s, &ray, o, dd, &maxt, &attd)))
            return 0.0;
    } else {
        if (d->max_depth < 2 || !or_segment_index_matched(s, &ray, o, &maxt)) return 0.0;
        for (int k = 0; k < 3; ++k) dd[k] = ray.d[k];
    }
    float att = (float)attd;
    int inside = 0;
    double acc = 0.0;
    float tcont = maxt;
    for (int it = 0; it < 4096; ++it) {
        int tri;
        const float tt = or_target_hit(d, o, dd, &tri);
        const int hit = tt < tcont;
        const float tsi = hit ? tt : tcont;
        const int ch = inside ? 0 : 1;
        if (mode == 0 || mode == 3)
            (void)or_dda(s, o, dd, tsi, em * (double)att, mode, film + ch, NULL, only_slice, visits);
        else if (mode == 1)
            acc += (double)att * or_dda(s, o, dd, tsi, em, mode, NULL, grad + ch, only_slice, visits);
        else
            (void)or_dda(s, o, dd, tsi, em, mode, NULL, NULL, only_slice, visits);
        att = att * expf(-d->sigma_t * tsi);
        if (!hit) break;
        inside = !inside;
        const float* v = d->target_tris + 9 * tri;
        float e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]}, e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
        float c[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        float inv = 1.0f / sqrtf(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
        float n[3], p[3];
        for (int k = 0; k < 3; ++k) {
            n[k] = c[k] * inv;
            p[k] = fmaf(dd[k], tt, o[k]);
        }
        float m = fmaxf(fmaxf(fabsf(p[0]), fabsf(p[1])), fabsf(p[2]));
        float mag = (1.0f + m) * OR_RAY_EPS;
        if (signbit(n[0] * dd[0] + n[1] * dd[1] + n[2] * dd[2])) mag = -mag;
        for (int k = 0; k < 3; ++k) o[k] = fmaf(mag, n[k], p[k]);
        int which;
        tcont = or_container_hit(s, o, dd, &which);
        if (!(tcont < INFINITY)) break;
    }
    return acc;
}

/* Surface-aware film in a scattering medium (film_channels 2, has_scattering; volume.py:179-272
   with the target mesh in the scene, null BSDF).  The loop of or_trace_scatter in which the
   nearest surface of every medium segment is the nearer of the target mesh and the container
   (or an occluder); every segment deposits from its origin up to that surface (sensor.py with
   maxt = si.t) into channel 0 while inside the target, 1 outside (sensor.py:405-409;
   inside_target starts outside and toggles at each target hit, volume.py:175, :218).  Per loop
   iteration the draws are RR next_1d, the medium next_1d (volume.py:200), then BSDF next_1d +
   next_2d at a surface (:225-226) or the phase function's next_1d + next_2d at a medium event
   (:247-251).  A target hit before the free flight ends (reached_surface) passes the null BSDF:
   the attenuation takes transmittance_eval_pdf's tr / pdf with pdf = tr (:206-208), the next
   segment starts at the hit point offset along the face normal (spawn_ray), and depth is not
   incremented (:271); the container or an occluder ends the path (transmission only, convex). */
static double or_trace_surface_scatter(const or_scene* s, uint32_t pixel, uint64_t wave_index, uint32_t seed,
                                       double em, int mode, double* film, const float* grad, uint64_t* visits) {
    const tvam_desc* d = s->d;
    or_ray ray;
    or_pcg32 rng;
    or_gen_ray_rng(s, pixel, wave_index, seed, &ray, &rng);
    float o[3], dd[3], maxt;
    double attd = 1.0;
    int nsurf;
    if (d->vial_type == TVAM_VIAL_CYLINDRICAL || d->vial_type == TVAM_VIAL_SQUARE) {
        if (!(d->vial_type == TVAM_VIAL_SQUARE ? or_segment_square(s, &ray, o, dd, &maxt, &attd)
                                               : or_segment_cylindrical(s, &ray, o, dd, &maxt, &attd)))
            return 0.0;
        nsurf = 2;
    } else {
        if (d->max_depth < 2 || !or_segment_index_matched(s, &ray, o, &maxt)) return 0.0;
        for (int k = 0; k < 3; ++k) dd[k] = ray.d[k];
        nsurf = 1;
    }
    for (int i = 0; i < 5 * nsurf; ++i) (void)or_pcg_float(&rng); /* the surface iterations before the medium */
    float att = (float)attd;
    int depth = nsurf, inside = 0;
    const float st = d->sigma_t, ss = d->albedo * d->sigma_t;
    double acc = 0.0;
    float tcont = maxt;
    for (int it = 0; it < 4096; ++it) {
        const float q = fminf(0.99f, att);
        const float u_rr = or_pcg_float(&rng);
        if (depth > d->rr_depth) { /* volume.py:182-185 */
            if (!(u_rr < q)) break;
            att = att * (1.0f / q);
        }
        if (!(att != 0.0f)) break;
        int tri;
        const float tt = or_target_hit(d, o, dd, &tri);
        const int hit = tt < tcont;
        const float tsi = hit ? tt : tcont;
        const float u_m = or_pcg_float(&rng);
        const float tmi = -logf(1.0f - u_m) / st;
        const int reached = tsi < tmi;
        const int ch = inside ? 0 : 1;
        if (mode == 0 || mode == 3)
            (void)or_dda(s, o, dd, tsi, em * (double)att, mode, film + ch, NULL, -1, visits);
        else if (mode == 1)
            acc += (double)att * or_dda(s, o, dd, tsi, em, mode, NULL, grad + ch, -1, visits);
        else
            (void)or_dda(s, o, dd, tsi, em, mode, NULL, NULL, -1, visits);
        if (reached) {
            if (!hit) break; /* the container or an occluder: leaves the medium for good */
            const float tr = expf(-tsi * st);
            const float inv = tr > 0.0f ? 1.0f / tr : 0.0f;
            att = att * (tr * inv);
            for (int i = 0; i < 3; ++i) (void)or_pcg_float(&rng); /* BSDF next_1d + next_2d */
            inside = !inside;
            const float* v = d->target_tris + 9 * tri;
            float e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]}, e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
            float c[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
            float ninv = 1.0f / sqrtf(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
            float n[3], p[3];
            for (int k = 0; k < 3; ++k) {
                n[k] = c[k] * ninv;
                p[k] = fmaf(dd[k], tt, o[k]);
            }
            float m = fmaxf(fmaxf(fabsf(p[0]), fabsf(p[1])), fabsf(p[2]));
            float mag = (1.0f + m) * OR_RAY_EPS;
            if (signbit(n[0] * dd[0] + n[1] * dd[1] + n[2] * dd[2])) mag = -mag;
            for (int k = 0; k < 3; ++k) o[k] = fmaf(mag, n[k], p[k]);
        } else {
            const float tr = expf(-tmi * st);
            const float pdf = tr * st;
            const float inv = pdf > 0.0f ? 1.0f / pdf : 0.0f;
            float w = tr * inv;
            w = w * ss;
            (void)or_pcg_float(&rng); /* phase next_1d (unused) */
            const float u1 = or_pcg_float(&rng), u2 = or_pcg_float(&rng);
            float wo[3];
            or_phase_sample(d, dd, u1, u2, wo);
            for (int k = 0; k < 3; ++k) {
                o[k] = fmaf(dd[k], tmi, o[k]);
                dd[k] = wo[k];
            }
            att = att * w;
            ++depth;
            if (depth >= d->max_depth) break;
        }
        int which;
        tcont = or_container_hit(s, o, dd, &which);
        if (!(tcont < INFINITY)) break; /* escapes through an open end: no surface, no deposit */
    }
    return acc;
}

/* one ray: generate + segment + DDA.  Returns the adjoint sum (mode 1).
   mode 0: forward, 3: forward with atomic film adds (shared film). */
static double or_trace(const or_scene* s, uint32_t pixel, uint64_t wave_index, uint32_t seed, double em,
                       int mode, double* film, const float* grad, int only_slice, uint64_t* visits) {
    if (s->d->sensor_type != TVAM_SENSOR_DDA)
        return or_trace_estimator(s, pixel, wave_index, seed, em, mode, film, grad, visits);
    if (s->d->albedo != 0.0f && s->C == 2)  /* has_scattering, surface-aware film */
        return or_trace_surface_scatter(s, pixel, wave_index, seed, em, mode, film, grad, visits);
    if (s->d->albedo != 0.0f)  /* has_scattering (volume.py:159) */
        return or_trace_scatter(s, pixel, wave_index, seed, em, mode, film, grad, visits, s->part);
    if (s->C == 2) return or_trace_surface(s, pixel, wave_index, seed, em, mode, film, grad, only_slice, visits);
    or_ray ray;
    or_gen_ray(s, pixel, wave_index, seed, &ray);
    float o2[3], maxt;
    if (s->d->vial_type == TVAM_VIAL_CYLINDRICAL || s->d->vial_type == TVAM_VIAL_SQUARE) {
        float d2[3];
        double att;
        if (!(s->d->vial_type == TVAM_VIAL_SQUARE ? or_segment_square(s, &ray, o2, d2, &maxt, &att)
                                                  : or_segment_cylindrical(s, &ray, o2, d2, &maxt, &att)))
            return 0.0;
        /* the interfaces' attenuation scales every contribution (sensor.py:404) */
        if (mode == 0) return or_dda(s, o2, d2, maxt, em * att, mode, film, grad, only_slice, visits);
        return att * or_dda(s, o2, d2, maxt, em, mode, film, grad, only_slice, visits);
    }
    if (s->d->max_depth < 2) return 0.0;
    if (!or_segment_index_matched(s, &ray, o2, &maxt)) return 0.0;
    return or_dda(s, o2, ray.d, maxt, em, mode, film, grad, only_slice, visits);
}

/* ------------------------------------------------------------------------ */
/* Radon filter (integrators/radon.py:47-106, optimize.py:143-163; SURVEY    */
/* 8f-f4): per DMD pixel, the sum over samples of the ray's weighted         */
/* absorption on the segments inside both the medium and the target mesh     */
/* (null BSDF; t counts from the ray origin).  Pixels with radon > 0 stay    */
/* active under 'filter_radon'.  Draw order: sample_rays only (the BSDF      */
/* draws of the loop do not change transmission-only / null outcomes).      */
/* ------------------------------------------------------------------------ */
static double or_radon_ray(const or_scene* s, const or_ray* ray, const float* tgt, int ntgt, int max_depth) {
    const tvam_desc* d = s->d;
    float o[3] = {ray->o[0], ray->o[1], ray->o[2]}, dd[3] = {ray->d[0], ray->d[1], ray->d[2]};
    const float half = 0.5f * d->vial_height;
    float thr = 1.0f, L = 0.0f, t = 0.0f;
    int in_medium = 0, inside = 0, depth = 0;
    float he[3], hi[3];
    or_square_extents(d, he, hi);
    for (int it = 0; it < 4096; ++it) {
        float tb = INFINITY, n[3] = {0.0f, 0.0f, 0.0f};
        int kind = -1, tri = -1;
        if (d->vial_type == TVAM_VIAL_SQUARE) {
            float ne[3], ni[3];
            float te = or_box_hit(o, dd, he, ne), ti = or_box_hit(o, dd, hi, ni);
            if (ti <= te) {
                tb = ti;
                kind = 1;
                memcpy(n, ni, sizeof(n));
            } else {
                tb = te;
                kind = 0;
                memcpy(n, ne, sizeof(n));
            }
        } else if (o[2] >= -half && o[2] <= half) {
            float t0, t1, ti = INFINITY, te = INFINITY;
            if (or_cyl_roots(o, dd, d->vial_r, &t0, &t1) && t1 >= 0.0f) ti = t0 >= 0.0f ? t0 : t1;
            if (d->vial_type == TVAM_VIAL_CYLINDRICAL && or_cyl_roots(o, dd, d->vial_r_ext, &t0, &t1) && t1 >= 0.0f)
                te = t0 >= 0.0f ? t0 : t1;
            tb = ti <= te ? ti : te;
            kind = ti <= te ? 1 : 0;
        }
        if (d->n_occluder_tris) {
            float toc = or_occ_hit(d, o, dd);
            if (toc < tb) {
                tb = toc;
                kind = 2;
            }
        }
        for (int i = 0; i < ntgt; ++i) {
            float tt = or_tri_hit(o, dd, tgt + 9 * i);
            if (tt < tb) {
                tb = tt;
                kind = 3;
                tri = i;
            }
        }
        if (!(tb < INFINITY)) break;
        float contrib = thr * expf(-d->sigma_t * t) * (1.0f - expf(-d->sigma_t * tb));
        if (inside && in_medium) L = L + contrib;
        t = t + tb;
        float p[3];
        for (int k = 0; k < 3; ++k) p[k] = fmaf(dd[k], tb, o[k]);
        float wo[3] = {dd[0], dd[1], dd[2]};
        if (kind == 3) {
            const float* v = tgt + 9 * tri;
            float e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]}, e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
            float c[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
            float inv = 1.0f / sqrtf(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
            for (int k = 0; k < 3; ++k) n[k] = c[k] * inv;
            inside = !inside;
        } else if (kind == 2) {
            break;
        } else {
            if (d->vial_type != TVAM_VIAL_SQUARE) {
                float rp = sqrtf(p[0] * p[0] + p[1] * p[1]);
                n[0] = p[0] / rp;
                n[1] = p[1] / rp;
                n[2] = 0.0f;
            }
            if (d->vial_type != TVAM_VIAL_INDEX_MATCHED) {
                float eta = kind == 1 ? d->medium_ior / d->vial_ior : d->vial_ior / OR_IOR_AIR;
                float w = d->vial_type == TVAM_VIAL_SQUARE ? or_transmit_world(n, dd, eta, wo) : or_transmit(n, dd, eta, wo);
                if (!(w > 0.0f)) break;
                thr = thr * w;
            }
            ++depth;
        }
        float m = fmaxf(fmaxf(fabsf(p[0]), fabsf(p[1])), fabsf(p[2]));
        float mag = (1.0f + m) * OR_RAY_EPS;
        float nwo = n[0] * wo[0] + n[1] * wo[1] + n[2] * wo[2];
        if (signbit(nwo)) mag = -mag;
        for (int k = 0; k < 3; ++k) {
            o[k] = fmaf(mag, n[k], p[k]);
            dd[k] = wo[k];
        }
        if (depth >= max_depth) break;
        if (kind == 1) in_medium = nwo < 0.0f;
    }
    return (double)L;
}

/* radon[i] for every pixel of the dense crop (angle, row, col): sum over spp samples of
   ray weight * L (radon.py:72-78: imgs[idx] += L * weight). */
int oracle_radon(const tvam_desc* d, const float* tgt, int ntgt, uint32_t spp, uint32_t seed, int max_depth,
                 double* radon, int nthreads) {
    int rc = or_check(d);
    if (rc) return rc;
    if (d->regular_sampling) spp = 1;
    or_scene s;
    or_scene_init(&s, d);
    const uint64_t n = (uint64_t)d->n_patterns * d->crop_y * d->crop_x;
    const double wr = or_ray_weight(d, n, spp);
    if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 256) num_threads(nthreads)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        uint32_t pixel = or_pixel(d, NULL, (uint64_t)i);
        uint64_t st = or_stream(d, NULL, (uint64_t)i);
        double acc = 0.0;
        for (uint32_t k = 0; k < spp; ++k) {
            or_ray ray;
            or_gen_ray(&s, pixel, st * spp + k, seed, &ray);
            acc += or_radon_ray(&s, &ray, tgt, ntgt, max_depth);
        }
        radon[i] = wr * acc;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Public oracle entry points (called from tests/ and bench.py via ctypes)   */
/* ------------------------------------------------------------------------ */
static int or_forward_impl(const tvam_desc* d, const float* active_data, const uint32_t* active_pixels,
                           uint64_t n_active, uint32_t spp, uint32_t seed, double* dose, uint64_t* visits,
                           int nthreads, int part, const float* inv_volumes, const uint64_t* streams) {
    int rc = or_check(d);
    if (rc) return rc;
    if (d->regular_sampling) spp = 1;
    or_scene s;
    or_scene_init(&s, d);
    s.part = part;
    s.inv_volumes = inv_volumes;
    if (s.C == 2 && !inv_volumes) return TVAM_ERR_INVALID;
    size_t V = (size_t)s.res[0] * s.res[1] * s.res[2];
    memset(dose, 0, V * (size_t)s.C * sizeof(double));
    double wr = or_ray_weight(d, or_n_total(d, n_active), spp);
    uint64_t nv_total = 0;
    if ((d->albedo != 0.0f || d->sensor_type != TVAM_SENSOR_DDA) && nthreads > 1) {
        /* scattered paths leave their slice: per-thread films (static
           schedule, fixed-order reduction), or atomics when those would not fit */
        const size_t VC = V * (size_t)s.C;  /* film entries (2 channels on surface-aware films) */
        const int priv = (double)VC * (double)nthreads * 8.0 <= 2.0e9;
        double* films = priv ? (double*)calloc(VC * (size_t)nthreads, sizeof(double)) : NULL;
        if (priv && !films) return TVAM_ERR_INVALID;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads) reduction(+ : nv_total)
#endif
        {
#ifdef _OPENMP
            const int tid = omp_get_thread_num();
#else
            const int tid = 0;
#endif
            double* mine = priv ? films + (size_t)tid * VC : dose;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
            for (int64_t i = 0; i < (int64_t)n_active; ++i) {
                uint32_t pixel = or_pixel(d, active_pixels, (uint64_t)i);
                double em = (double)active_data[i] * wr;
                uint64_t st = streams ? streams[i] : or_stream(d, active_pixels, (uint64_t)i);
                for (uint32_t k = 0; k < spp; ++k)
                    or_trace(&s, pixel, st * spp + k, seed, em, priv ? 0 : 3, mine, NULL, -1, &nv_total);
            }
        }
        if (priv) {
            for (int t = 0; t < nthreads; ++t)
                for (size_t v = 0; v < VC; ++v) dose[v] += films[(size_t)t * VC + v];
            free(films);
        }
    } else if (nthreads <= 1) {
        for (uint64_t i = 0; i < n_active; ++i) {
            uint32_t pixel = or_pixel(d, active_pixels, i);
            double em = (double)active_data[i] * wr;
            uint64_t st = streams ? streams[i] : or_stream(d, active_pixels, (uint64_t)i);
            for (uint32_t k = 0; k < spp; ++k)
                or_trace(&s, pixel, st * spp + k, seed, em, 0, dose, NULL, -1, &nv_total);
        }
    } else {
        /* Rays are planar (collimated + circular motion + vertical vial axis):
           every ray stays in its start z-slice, so threads own whole slices and
           accumulate without atomics (the "z-slab private" CPU baseline).
           Active entries are bucketed by DMD row first (CSR), so each slice
           only visits the rows whose rays can reach it. */
        uint32_t H = (uint32_t)d->res_y, hw = (uint32_t)d->res_y * (uint32_t)d->res_x;
        uint64_t* row_off = (uint64_t*)calloc((size_t)H + 1, sizeof(uint64_t));
        uint64_t* row_idx = (uint64_t*)malloc((size_t)(n_active ? n_active : 1) * sizeof(uint64_t));
        if (!row_off || !row_idx) {
            free(row_off);
            free(row_idx);
            return TVAM_ERR_INVALID;
        }
        for (uint64_t i = 0; i < n_active; ++i) row_off[(or_pixel(d, active_pixels, i) % hw) / (uint32_t)d->res_x + 1]++;
        for (uint32_t r = 0; r < H; ++r) row_off[r + 1] += row_off[r];
        {
            uint64_t* fill = (uint64_t*)malloc((size_t)H * sizeof(uint64_t));
            memcpy(fill, row_off, (size_t)H * sizeof(uint64_t));
            for (uint64_t i = 0; i < n_active; ++i) {
                uint32_t r = (or_pixel(d, active_pixels, i) % hw) / (uint32_t)d->res_x;
                row_idx[fill[r]++] = i;
            }
            free(fill);
        }
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(+ : nv_total)
#endif
        for (int k = 0; k < s.res[2]; ++k) {
            float z0 = d->bbox_min[2] + (float)k * s.h[2];
            float z1 = z0 + s.h[2];
            float marg = 2.0f * s.h[2];
            for (uint32_t row = 0; row < H; ++row) {
                /* z of this row's rays lies in [(0.5-(row+1)/H)*ey, (0.5-row/H)*ey] */
                float zt = (0.5f - (float)row * s.inv_h) * s.ey;
                float zb = (0.5f - (float)(row + 1) * s.inv_h) * s.ey;
                if (zb > z1 + marg || zt < z0 - marg) continue;
                for (uint64_t j = row_off[row]; j < row_off[row + 1]; ++j) {
                    uint64_t i = row_idx[j];
                    uint32_t pixel = or_pixel(d, active_pixels, i);
                    double em = (double)active_data[i] * wr;
                    uint64_t st = streams ? streams[i] : or_stream(d, active_pixels, (uint64_t)i);
                    for (uint32_t q = 0; q < spp; ++q)
                        or_trace(&s, pixel, st * spp + q, seed, em, 0, dose, NULL, k, &nv_total);
                }
            }
        }
        free(row_off);
        free(row_idx);
    }
    if (s.C == 2)  /* volume.py:41-42 with the surface-aware volumes (sensor.py:47-110) */
        for (size_t v = 0; v < 2 * V; ++v) dose[v] *= (double)inv_volumes[v];
    else
        for (size_t v = 0; v < V; ++v) dose[v] *= s.inv_vol;
    if (visits) *visits = nv_total;
    return 0;
}

int oracle_forward_part(const tvam_desc* d, const float* active_data, const uint32_t* active_pixels,
                        uint64_t n_active, uint32_t spp, uint32_t seed, double* dose, uint64_t* visits,
                        int nthreads, int part) {
    return or_forward_impl(d, active_data, active_pixels, n_active, spp, seed, dose, visits, nthreads, part, NULL, NULL);
}

/* Surface-aware forward: dose [V][2] = film / volume per channel (inv_volumes [V][2]). */
int oracle_forward_surface(const tvam_desc* d, const float* active_data, const uint32_t* active_pixels,
                           uint64_t n_active, uint32_t spp, uint32_t seed, const float* inv_volumes, double* dose,
                           uint64_t* visits, int nthreads) {
    return or_forward_impl(d, active_data, active_pixels, n_active, spp, seed, dose, visits, nthreads, -1,
                           inv_volumes, NULL);
}

int oracle_forward(const tvam_desc* d, const float* active_data, const uint32_t* active_pixels,
                   uint64_t n_active, uint32_t spp, uint32_t seed, double* dose, uint64_t* visits,
                   int nthreads) {
    return oracle_forward_part(d, active_data, active_pixels, n_active, spp, seed, dose, visits, nthreads, -1);
}

/* Phase-function sample for a ray of direction dd (tests: distribution KATs). */
int oracle_phase(const tvam_desc* d, const float* dd, float u1, float u2, float* wo) {
    or_phase_sample(d, dd, u1, u2, wo);
    return 0;
}

static int or_adjoint_impl(const tvam_desc* d, const float* grad_dose, const uint32_t* active_pixels,
                           uint64_t n_active, uint32_t spp, uint32_t seed, double* grad, uint64_t* visits,
                           int nthreads, const float* inv_volumes, const uint64_t* streams) {
    int rc = or_check(d);
    if (rc) return rc;
    if (d->regular_sampling) spp = 1;
    or_scene s;
    or_scene_init(&s, d);
    s.inv_volumes = inv_volumes;
    if (s.C == 2 && !inv_volumes) return TVAM_ERR_INVALID;
    double wr = or_ray_weight(d, or_n_total(d, n_active), spp);
    /* delta_L = grad_in * inv_vol (volume.py:130), in fp32 like the reference */
    size_t V = (size_t)s.res[0] * s.res[1] * s.res[2] * (size_t)s.C;
    float* dl = (float*)malloc(V * sizeof(float));
    if (!dl) return TVAM_ERR_INVALID;
    float inv_vol_f = (float)s.inv_vol;
    for (size_t v = 0; v < V; ++v) dl[v] = grad_dose[v] * (s.C == 2 ? inv_volumes[v] : inv_vol_f);
    uint64_t nv_total = 0;
    if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 256) num_threads(nthreads) reduction(+ : nv_total)
#endif
    for (int64_t i = 0; i < (int64_t)n_active; ++i) {
        uint32_t pixel = or_pixel(d, active_pixels, (uint64_t)i);
        double g = 0.0;
        uint64_t st = streams ? streams[i] : or_stream(d, active_pixels, (uint64_t)i);
        for (uint32_t k = 0; k < spp; ++k)
            g += or_trace(&s, pixel, st * spp + k, seed, 1.0, 1, NULL, dl, -1, &nv_total);
        grad[i] = wr * g;
    }
    free(dl);
    if (visits) *visits = nv_total;
    return 0;
}

int oracle_adjoint(const tvam_desc* d, const float* grad_dose, const uint32_t* active_pixels,
                   uint64_t n_active, uint32_t spp, uint32_t seed, double* grad, uint64_t* visits,
                   int nthreads) {
    return or_adjoint_impl(d, grad_dose, active_pixels, n_active, spp, seed, grad, visits, nthreads, NULL, NULL);
}

int oracle_adjoint_surface(const tvam_desc* d, const float* grad_dose, const uint32_t* active_pixels,
                           uint64_t n_active, uint32_t spp, uint32_t seed, const float* inv_volumes, double* grad,
                           uint64_t* visits, int nthreads) {
    return or_adjoint_impl(d, grad_dose, active_pixels, n_active, spp, seed, grad, visits, nthreads, inv_volumes, NULL);
}

/* Test infrastructure: the forward / adjoint of a subset of a larger set's pixels, each
   active entry i drawing the sampler streams streams[i]*spp .. +spp-1 of its position in the
   larger set (common.py:57-67, :81).  A test can thus check the pixels it picks out of a
   plan's whole dense shard without the oracle tracing every path of the shard. */
int oracle_forward_streams(const tvam_desc* d, const float* active_data, const uint32_t* active_pixels,
                           const uint64_t* streams, uint64_t n_active, uint32_t spp, uint32_t seed, double* dose,
                           uint64_t* visits, int nthreads) {
    return or_forward_impl(d, active_data, active_pixels, n_active, spp, seed, dose, visits, nthreads, -1, NULL,
                           streams);
}

int oracle_adjoint_streams(const tvam_desc* d, const float* grad_dose, const uint32_t* active_pixels,
                           const uint64_t* streams, uint64_t n_active, uint32_t spp, uint32_t seed, double* grad,
                           uint64_t* visits, int nthreads) {
    return or_adjoint_impl(d, grad_dose, active_pixels, n_active, spp, seed, grad, visits, nthreads, NULL, streams);
}

/* ------------------------------------------------------------------------ */
/* Surface-aware discretisation (VolumetricSensor.compute_volume,           */
/* sensor.py:47-110): per voxel, sample_count points (independent sampler    */
/* seeded (0, wavefront = voxels), lane = flat voxel index; draws: offset     */
/* x, y, z, then next_2d), each shot along square_to_uniform_sphere; a point  */
/* is inside when its origin is strictly inside the mesh bbox and the first  */
/* target hit faces away (dot(d, n) > 0, n the geometric normal).            */
/* volumes[2v] = inside, [2v+1] = outside, count * voxel_vol / sample_count  */
/* in fp32.  UNPINNED like every Mitsuba internal (ray-triangle, sampler).   */
/* ------------------------------------------------------------------------ */
int oracle_compute_volume(const tvam_desc* d, uint32_t sample_count, float* volumes, int nthreads) {
    if (d->n_target_tris <= 0 || !d->target_tris || sample_count == 0) return TVAM_ERR_INVALID;
    or_scene s;
    or_scene_init(&s, d);
    float mb0[3] = {INFINITY, INFINITY, INFINITY}, mb1[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < 3 * d->n_target_tris; ++i)
        for (int k = 0; k < 3; ++k) {
            mb0[k] = fminf(mb0[k], d->target_tris[3 * i + k]);
            mb1[k] = fmaxf(mb1[k], d->target_tris[3 * i + k]);
        }
    const float vvol = s.h[0] * s.h[1] * s.h[2];
    const int64_t V = (int64_t)s.res[0] * s.res[1] * s.res[2];
    if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
#endif
    for (int64_t v = 0; v < V; ++v) {
        const int vx = (int)(v % s.res[0]), vy = (int)((v / s.res[0]) % s.res[1]), vz = (int)(v / ((int64_t)s.res[0] * s.res[1]));
        const float vox[3] = {(float)vx, (float)vy, (float)vz};
        or_pcg32 rng;
        or_sampler_seed(&rng, 0u, (uint64_t)v);
        uint32_t cin = 0, cout = 0;
        for (uint32_t i = 0; i < sample_count; ++i) {
            float off[3];
            for (int k = 0; k < 3; ++k) off[k] = or_pcg_float(&rng);
            const float sx = or_pcg_float(&rng), sy = or_pcg_float(&rng);
            float o[3], dd[3];
            for (int k = 0; k < 3; ++k) o[k] = d->bbox_min[k] + s.h[k] * (vox[k] + off[k]);
            const float z = 1.0f - 2.0f * sy, r = sqrtf(fmaxf(1.0f - z * z, 0.0f));
            dd[0] = r * cosf(OR_TWO_PI * sx);
            dd[1] = r * sinf(OR_TWO_PI * sx);
            dd[2] = z;
            int inside = 0;
            if (o[0] > mb0[0] && o[1] > mb0[1] && o[2] > mb0[2] && o[0] < mb1[0] && o[1] < mb1[1] && o[2] < mb1[2]) {
                int tri;
                const float t = or_target_hit(d, o, dd, &tri);
                if (t < INFINITY) {
                    const float* p = d->target_tris + 9 * tri;
                    float e1[3] = {p[3] - p[0], p[4] - p[1], p[5] - p[2]}, e2[3] = {p[6] - p[0], p[7] - p[1], p[8] - p[2]};
                    float c[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                                  e1[0] * e2[1] - e1[1] * e2[0]};
                    inside = c[0] * dd[0] + c[1] * dd[1] + c[2] * dd[2] > 0.0f;
                }
            }
            if (inside) ++cin;
            else ++cout;
        }
        volumes[2 * v] = (float)cin * vvol / (float)sample_count;
        volumes[2 * v + 1] = (float)cout * vvol / (float)sample_count;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Target discretisation (utils.py:83-128): one ray per voxel centre         */
/* pos = bbox.min + (0.5 + (x, y, z)) * voxel_size (:106-112), direction     */
/* square_to_uniform_sphere(next_2d) of the independent sampler seeded       */
/* (0, wavefront = voxels), lane = flat voxel index (:114-117); a voxel is   */
/* tested only when its centre lies strictly inside the target bbox (:118)   */
/* and is inside when the first target hit faces away from the ray,         */
/* dot(n, d) > 0 with n the geometric normal (:120-122).  occ[z][y][x] = 0/1 */
/* (float).  Target triangles: d->target_tris (world space).                 */
/* ------------------------------------------------------------------------ */
int oracle_discretize(const tvam_desc* d, float* occ, int nthreads) {
    if (d->n_target_tris <= 0 || !d->target_tris || !occ) return TVAM_ERR_INVALID;
    or_scene s;
    or_scene_init(&s, d);
    float mb0[3] = {INFINITY, INFINITY, INFINITY}, mb1[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < 3 * d->n_target_tris; ++i)
        for (int k = 0; k < 3; ++k) {
            mb0[k] = fminf(mb0[k], d->target_tris[3 * i + k]);
            mb1[k] = fmaxf(mb1[k], d->target_tris[3 * i + k]);
        }
    const int64_t V = (int64_t)s.res[0] * s.res[1] * s.res[2];
    if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads)
#endif
    for (int64_t v = 0; v < V; ++v) {
        const int vx = (int)(v % s.res[0]), vy = (int)((v / s.res[0]) % s.res[1]), vz = (int)(v / ((int64_t)s.res[0] * s.res[1]));
        const float vox[3] = {(float)vx, (float)vy, (float)vz};
        or_pcg32 rng;
        or_sampler_seed(&rng, 0u, (uint64_t)v);
        const float sx = or_pcg_float(&rng), sy = or_pcg_float(&rng);
        float o[3], dd[3];
        for (int k = 0; k < 3; ++k) o[k] = d->bbox_min[k] + (0.5f + vox[k]) * s.h[k];
        const float z = 1.0f - 2.0f * sy, r = sqrtf(fmaxf(1.0f - z * z, 0.0f));
        dd[0] = r * cosf(OR_TWO_PI * sx);
        dd[1] = r * sinf(OR_TWO_PI * sx);
        dd[2] = z;
        int inside = 0;
        if (o[0] > mb0[0] && o[1] > mb0[1] && o[2] > mb0[2] && o[0] < mb1[0] && o[1] < mb1[1] && o[2] < mb1[2]) {
            int tri;
            const float t = or_target_hit(d, o, dd, &tri);
            if (t < INFINITY) {
                const float* p = d->target_tris + 9 * tri;
                float e1[3] = {p[3] - p[0], p[4] - p[1], p[5] - p[2]}, e2[3] = {p[6] - p[0], p[7] - p[1], p[8] - p[2]};
                float c[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                              e1[0] * e2[1] - e1[1] * e2[0]};
                inside = c[0] * dd[0] + c[1] * dd[1] + c[2] * dd[2] > 0.0f;
            }
        }
        occ[v] = inside ? 1.0f : 0.0f;
    }
    return 0;
}

/* Ray of one sample, for property tests (test_projector.py:7-38 analogue):
   out = {o.x,o.y,o.z, d.x,d.y,d.z, hit, o'.x,o'.y,o'.z, maxt, d'.x,d'.y,d'.z, weight}
   (o', d', maxt: the medium segment; weight: the interfaces' attenuation). */
int oracle_ray(const tvam_desc* d, uint32_t pixel, uint64_t wave_index, uint32_t seed, float* out) {
    or_scene s;
    or_scene_init(&s, d);
    or_ray ray;
    or_gen_ray(&s, pixel, wave_index, seed, &ray);
    for (int k = 0; k < 3; ++k) {
        out[k] = ray.o[k];
        out[3 + k] = ray.d[k];
    }
    float o2[3] = {0, 0, 0}, d2[3] = {ray.d[0], ray.d[1], ray.d[2]}, maxt = 0.0f;
    double att = 1.0;
    int hit = 0;
    if (d->vial_type == TVAM_VIAL_INDEX_MATCHED) hit = or_segment_index_matched(&s, &ray, o2, &maxt);
    else if (d->vial_type == TVAM_VIAL_CYLINDRICAL) hit = or_segment_cylindrical(&s, &ray, o2, d2, &maxt, &att);
    else if (d->vial_type == TVAM_VIAL_SQUARE) hit = or_segment_square(&s, &ray, o2, d2, &maxt, &att);
    out[6] = (float)hit;
    out[7] = o2[0];
    out[8] = o2[1];
    out[9] = o2[2];
    out[10] = maxt;
    out[11] = d2[0];
    out[12] = d2[1];
    out[13] = d2[2];
    out[14] = (float)att;
    return 0;
}

/* DDA of an explicit ray (for analytic known-answer tests). */
int oracle_dda_ray(const tvam_desc* d, const float* o, const float* dir, float maxt, double em, double* film,
                   uint64_t* visits) {
    or_scene s;
    or_scene_init(&s, d);
    size_t V = (size_t)s.res[0] * s.res[1] * s.res[2];
    memset(film, 0, V * sizeof(double));
    or_dda(&s, o, dir, maxt, em, 0, film, NULL, -1, visits);
    return 0;
}

int oracle_version(void) { return 1; }
