// tvam_planar.hip — the planar fast path of regular sampling.
//
// With a collimated projector and regular sampling every ray of DMD column
// `col` at angle `a` has the same xy path whatever its DMD row: origin
// o = look_at(...) @ (x_c, y_c, 0.005) differs between rows only in z
// (common.py:81-108 with jitter 0.5), the index-matched vial is a vertical
// cylinder (geometry.py:75-96) so the medium segment [o2, o2 + maxt d] is
// row-independent, and the DDA (sensor.py:327-438) of a planar ray never
// steps in z.  The spawn offset (1 + max|p|) * RayEpsilon of the vial entry
// point p is row-independent as long as |p_z| < max(|p_x|, |p_y|), which the
// plan guarantees (|z| <= 0.7 r <= r / sqrt(2)).  So one (angle, column)
// record serves every row, and the per-visit weight
//     c = exp(-st t_in) - exp(-st t_out)
// of voxel (x, y) is the same for every z-slice.  Two kernels use that:
//
//   * forward, voxel-driven: a thread owns a voxel column (x, y) and Z
//     z-slices; for every angle it finds the 1-3 DMD columns whose ray
//     crosses the voxel, computes that ray's exact segment [t_in, t_out] in
//     the voxel (what one DDA visit accumulates), and adds c * P(slice) for
//     its Z slices from a per-angle pattern slab staged in LDS.  No atomics,
//     no per-ray resume, deterministic.
//   * adjoint, ray-driven with Z-slice sharing: the tile DDA of
//     tvam_kernels.hip, but the LDS tile holds Z interleaved slices, so one
//     march computes c once per visit and gathers Z gradient values with one
//     or two ds_read_b128.
//
// Both work in slice space: a slice's pattern is the sum of the DMD rows
// whose rays lie in it (usually exactly one), and a row's gradient is its
// slice's.
#include "tvam_internal.h"

#include <hip/hip_ext.h>

#include <algorithm>

#define TVAM_PB 256

__device__ __forceinline__ float pl_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
// native 4-vector for staged registers (HIP's float4 is a union wrapper that can keep a
// staged copy out of registers)
typedef float pl_f4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// (angle, column) table: ray generation (common.py:81-108, jitter 0.5), vial
// segment (volume.py:179-216) and DDA initialisation (sensor.py:327-365),
// evaluated once per column instead of once per (row, column).
//   vox[i]   = {qx, qy, maxt, 0}: t(X) = fma(X, 1/d.x, qx) is the distance
//              from o2 at which the ray crosses x = X (likewise y); an axis
//              with |d| <= 1e-8 (never stepped by the DDA) stores the DDA's
//              fixed voxel index instead; maxt < 0 marks a ray that misses.
//   rec_f[i] = {t_start, tau_end, dtmax0_x, dtmax0_y}, rec_i[i] = start voxel
//              x | y << 16 (or -1): the tile DDA's resume record.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void tvam_planar_rays_kernel(TvamConsts k, const float2* __restrict__ cs, int ns,
                                                               float4* __restrict__ vox, float4* __restrict__ rec_f,
                                                               int32_t* __restrict__ rec_i,
                                                               float4* __restrict__ rec_g, float4* __restrict__ vox2,
                                                               float4* __restrict__ chord) {
    const int64_t n = (int64_t)ns * k.crop_x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int al = (int)(i / k.crop_x), col = (int)(i - (int64_t)al * k.crop_x);
        const float2 csv = cs[al];
        float xc, yc, ox, oy, oz, dx, dy;
        tvam_ray_camera(k, k.crop_off_x + col, k.crop_off_y, 0.5f, 0.5f, xc, yc);
        tvam_ray_world(k, csv.x, csv.y, xc, 0.0f, ox, oy, oz, dx, dy);
        float o2x, o2y, d2x, d2y, maxt, wgt;
        TvamDda q;
        if (!tvam_segment(k, ox, oy, 0.0f, dx, dy, o2x, o2y, d2x, d2y, maxt, wgt) ||
            !tvam_dda_init(k, o2x, o2y, d2x, d2y, maxt, q)) {
            vox[i] = make_float4(0.0f, 0.0f, -1.0f, 0.0f);
            rec_f[i] = make_float4(0.0f, -1.0f, 0.0f, 0.0f);
            rec_i[i] = -1;
            if (rec_g) rec_g[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (vox2) vox2[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (chord) chord[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            continue;
        }
        if (rec_g)
            rec_g[i] = make_float4(q.step[0] > 0 ? q.ts[0] : -q.ts[0], q.step[1] > 0 ? q.ts[1] : -q.ts[1], wgt, 0.0f);
        if ((fabsf(d2x) > 1e-8f && !(q.dtm0[0] < TVAM_INF)) || (fabsf(d2y) > 1e-8f && !(q.dtm0[1] < TVAM_INF))) {
            vox[i] = make_float4(0.0f, 0.0f, -1.0f, 0.0f);  // frozen axis (sensor.py:358): the plan
            rec_i[i] = -2;                                  // falls back to the per-ray tile path
            continue;
        }
        dx = d2x;  // the medium chord's direction (the straight rays' own behind an index-matched vial)
        dy = d2y;
        const bool vx = fabsf(dx) > 1e-8f, vy = fabsf(dy) > 1e-8f;
        const float qx = vx ? -o2x * (1.0f / dx) : (float)q.sv[0];
        const float qy = vy ? -o2y * (1.0f / dy) : (float)q.sv[1];
        vox[i] = make_float4(qx, qy, q.t_start + q.tau_end, 0.0f);
        if (vox2)  // refracted forward: the column's own 1 / d, axis flags and interface weight
            vox2[i] = make_float4(vx ? 1.0f / dx : 0.0f, vy ? 1.0f / dy : 0.0f, __int_as_float((vx ? 1 : 0) | (vy ? 2 : 0)),
                                  wgt);
        if (chord) chord[i] = make_float4(o2x, o2y, d2x, d2y);
        rec_f[i] = make_float4(q.t_start, q.tau_end, q.dtm0[0], q.dtm0[1]);
        rec_i[i] = q.sv[0] | (q.sv[1] << 16);
    }
}

hipError_t tvam_launch_planar_rays(const TvamConsts& k, const TvamPlanar& pl, hipStream_t stream) {
    const int64_t n = (int64_t)pl.ns * k.crop_x;
    int64_t g = (n + 255) / 256;
    g = g > 65536 ? 65536 : (g < 1 ? 1 : g);
    hipLaunchKernelGGL(tvam_planar_rays_kernel, dim3((unsigned)g), dim3(256), 0, stream, k, pl.cs, pl.ns, pl.vox,
                       pl.rec_f, pl.rec_i, pl.rec_g, pl.vox2, pl.chord);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Forward, voxel-driven.  Workgroup = 16 x 16 voxel columns x Z slices.
// Per angle the workgroup stages, for the DMD columns whose rays can cross
// its tile (a window of pl.ncmax columns), the slice-binned pattern
// P[col][z] and the ray table entry; each thread then visits its 1-3
// candidate columns.  The DDA's visit of ray (a, col) in voxel (x, y) covers
// [max(t_x,near, t_y,near, 0), min(t_x,far, t_y,far, t_end)] (sensor.py:383-438
// in exact arithmetic), so the dose is the same sum of telescoped weights
// the DDA forms, up to fp32 rounding of the crossing times.
// ---------------------------------------------------------------------------
#define TVAM_PF 4     // most staged pattern values per thread and angle (host: ncmax * Z <= TVAM_PF * TVAM_PB)
// slab row stride (words) of Z slices: an odd number of 16-byte groups, so 16
// consecutive columns' ds_read_b128 hit 16 different bank groups
__host__ __device__ constexpr int tvam_fwd_zs(int Z) { return ((Z + 4) / 4) % 2 ? Z + 4 : Z + 8; }

// LDS-DMA staging of the binned slabs (straight rays): global_load_lds writes a
// wave's 64 lanes' 16-byte loads to 64 consecutive 16-byte LDS slots, so a buffer is laid out in
// whole wave-instructions: the slab's ncm * ZS / 4 slots (a column's Z / 4 data slots and its pad
// slots) rounded up to 64, and 64 record slots.  Each lane loads the global float4 its slot holds
// (a pad or round-up slot re-loads a data slot; nothing reads it).
// The DMA slab's column stride needs no pad when Z / 4 is odd (Z = 52: 13 float4 groups); slots are
// exact (ncm columns x ZS / 4 groups, the last wave-instruction's surplus lanes masked), so 6
// workgroups' LDS fits a CU at Z = 52 (4 with 64-slot rounding and a Z + 8 stride).
__host__ __device__ constexpr int tvam_fwd_zs_dma(int Z) { return (Z / 4) % 2 ? Z : Z + 4; }
__host__ __device__ constexpr int tvam_fwd_dma_np(int ncm, int Z) { return ncm * (tvam_fwd_zs_dma(Z) / 4); }
// One wave-instruction of LDS-DMA: each active lane's 16 bytes at g land at LDS byte l + 16 * lane
// (l wave-uniform, in M0).  Issued as inline asm so the compiler does not see an LDS write pending
// on vmcnt: with __builtin_amdgcn_global_load_lds it waits vmcnt(0) before the next ds_read of any
// LDS address, i.e. before computing the current buffer, which serialised the next angles' loads
// with this angle's compute.  The kernel drains the loads itself (s_waitcnt vmcnt(0) before the
// barrier that precedes their reads).
__device__ __forceinline__ void tvam_lds_dma16(const void* g, void* l) {
    const unsigned m = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)l;
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m) : "memory");
}
// a staged column outside the crop: no chord ({q, t_end < 0}; refracted: the second record zero)
__device__ float4 tvam_null_rec[2] = {{0.0f, 0.0f, -1.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
// super-block edge (tiles) of the forward's workgroup order: 5 x 5 (2.39-2.42 -> 2.36 ms on config 2;
// 8 x 8 2.36-2.43, 12 x 12 2.43-2.45; profiles/r06/ab_fwd/)
#define TVAM_FWD_SB 5
#define TVAM_ACH 64  // angles per LDS chunk of per-angle constants (paths without the SGPR constants)

// Z: slices per thread; NC: candidate DMD columns per (voxel, angle), a
// bound the plan derives from the voxel's lateral width in columns; MULTI:
// some slice collects several DMD rows; PF: staged values per thread (BIN:
// staged float4s); BIN: the window is staged from the slice-binned patterns
// (pl.fwd_bin, [angle][column][slice]) with one 16-byte load and store per slot.
//
// REFR (refracted rays, pl.fwd_refr): every staged column carries two records (its chord's
// crossing-time offsets / end and its own 1 / d, axis flags and interface weight), the
// per-angle constants are the (tile, angle) model of the chord index u (tvam_refr_model_kernel),
// and each voxel visits a per-(tile, angle) number of candidates (the same for the whole
// workgroup) from ceil(u - w).
template <int Z, int NC, bool MULTI, int PF, int AB, bool BIN = false, bool REFR = false, bool DMAP = false>
__global__ __launch_bounds__(TVAM_PB) void tvam_fwd_planar_kernel(TvamConsts k, TvamPlanar pl,
                                                                  const float* __restrict__ pat,
                                                                  float* __restrict__ dose) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int ncm = pl.ncmax;
    constexpr int RW = REFR ? 2 : 1;  // records (float4) per staged column
    constexpr bool DMA = BIN && DMAP && AB <= 2;  // LDS-DMA staging (pl.fwd_dma)
    constexpr bool SCONST = DMA && !REFR && AB == 2;  // per-angle constants in SGPRs
    // [2][AB][ncm * ZS + 4] (double buffer of AB angles per barrier), ZS = tvam_fwd_zs(Z);
    // the 4 words past a buffer's slab take the BIN staging's idle slots.  DMA: [2][AB][np] float4
    // slab slots (ZS = tvam_fwd_zs_dma(Z)) and [2][AB][RW ncm] record slots (refracted: record h of
    // column j at ncm h + j)
    constexpr int ZS = DMA ? tvam_fwd_zs_dma(Z) : tvam_fwd_zs(Z);
    const int np = DMA ? tvam_fwd_dma_np(ncm, Z) : 0;
    const int bstride = DMA ? 4 * np : ncm * ZS + 4;
    const int rstride = ncm * RW;
    const int rhalf = ncm;  // refracted: the second records' offset
    float* s_p = reinterpret_cast<float*>(smem);
    float4* s_r = reinterpret_cast<float4*>(s_p + 2 * AB * bstride);  // [2][AB][rstride]
    // per-angle constants of TVAM_ACH (+2 look-ahead) angles, copied to LDS so the
    // angle loop issues no scalar loads (an s_load's lgkmcnt wait would also
    // drain every outstanding LDS read)
    float4* s_ang = reinterpret_cast<float4*>(s_r + 2 * AB * rstride);  // [TVAM_ACH + 4][2]
    int* s_cb = reinterpret_cast<int*>(s_ang + 2 * (TVAM_ACH + 4)); // [TVAM_ACH + 4]
    int* s_row = s_cb + (TVAM_ACH + 4);                            // [Z]: the slice's row, -1 none, -2 several

    const int ntx = (k.res[0] + 15) >> 4, nty = (k.res[1] + 15) >> 4;
    // slice chunks of this launch: [fwd_zc0, fwd_zc0 + fwd_nzc) (tvam_forward_slices), else all
    const int nzc = pl.fwd_nzc > 0 ? pl.fwd_nzc : (k.nz + Z - 1) / Z;
    const int ntiles = ntx * nty, nwg1 = ntiles * nzc;
    const int parts = pl.fwd_parts > 1 ? pl.fwd_parts : 1, nwg = nwg1 * parts;
    // XCD-aware order: workgroup b runs on XCD b % 8; give each XCD a contiguous
    // run of (z-chunk, tile) pairs so the tiles sharing a z-chunk's pattern rows
    // share that XCD's L2
    const int L0 = (int)(gridDim.x >> 3);
    int L = (int)(blockIdx.x & 7) * L0 + (int)(blockIdx.x >> 3);
    if (L >= nwg) return;
    // angle part [ab, ae) of this workgroup (thin slabs: parts > 1 workgroups per
    // (tile, chunk), partial doses summed in fixed order by tvam_fwd_parts_kernel)
    const int part = L / nwg1;
    L -= part * nwg1;
    const int ab = (int)(((int64_t)pl.ns * part) / parts), ae = (int)(((int64_t)pl.ns * (part + 1)) / parts);
    // tiles in super-blocks of SB x SB (row-major blocks, row-major inside): the ~128 workgroups of a
    // z-chunk resident on one XCD cover a square of tiles, which rays of every angle cross several
    // tiles deep, so a staged column's slab is re-read from that XCD's L2 (a band of tile rows
    // shares it only along rays near the x axis)
    int bx, by;
    {
        const int t = L % ntiles;
        constexpr int SB = TVAM_FWD_SB;
        if (SB > 1) {
            const int sr = t / (ntx * SB), h = min(SB, nty - sr * SB);
            const int r2 = t - sr * ntx * SB, bc = r2 / (SB * h), w = min(SB, ntx - bc * SB);
            const int r3 = r2 - bc * SB * h;
            by = sr * SB + r3 / w;
            bx = bc * SB + r3 % w;
        } else {
            bx = t % ntx;
            by = t / ntx;
        }
    }
    const int tile = by * ntx + bx;
    const int ix = bx * 16 + (threadIdx.x & 15), iy = by * 16 + (threadIdx.x >> 4);
    const int z0 = ((pl.fwd_nzc > 0 ? pl.fwd_zc0 : 0) + L / ntiles) * Z;
    const float hx = k.h[0], hy = k.h[1];
    // voxel edges exactly as the DDA places them (bmin + i * h, sensor.py:357)
    const float X0 = k.bmin[0] + (float)ix * hx, X1 = k.bmin[0] + (float)(ix + 1) * hx;
    const float Y0 = k.bmin[1] + (float)iy * hy, Y1 = k.bmin[1] + (float)(iy + 1) * hy;
    const float Xc = k.bmin[0] + ((float)ix + 0.5f) * hx, Yc = k.bmin[1] + ((float)iy + 0.5f) * hy;
    const float u0 = pl.u0;
    const int32_t* cbt = pl.fwd_cb + (size_t)tile * pl.ns;  // first window column per angle

    if (threadIdx.x < Z) {
        const int s = z0 + threadIdx.x;
        int r = -1;
        if (s < k.nz) {
            const int b = pl.slice_off[s], e = pl.slice_off[s + 1];
            r = e - b == 1 ? pl.slice_rows[b] : (e - b == 0 ? -1 : -2);
        }
        s_row[threadIdx.x] = r;
    }
    const int ns = pl.ns;
    int tbase = ab;
    const float4* mdl = REFR ? pl.fwd_model + (size_t)tile * pl.ns * 2 : nullptr;  // this tile's models
    auto load_table = [&](int base) {
        for (int i = threadIdx.x; i < TVAM_ACH + 4; i += TVAM_PB) {
            const int a = base + i;
            if (a < ns) {
                if (REFR) {
                    const float4 m1 = mdl[2 * a + 1];
                    s_ang[2 * i] = mdl[2 * a];
                    s_ang[2 * i + 1] = m1;
                    s_cb[i] = __float_as_int(m1.z);
                } else {
                    s_ang[2 * i] = pl.fwd_ang[2 * a];
                    s_ang[2 * i + 1] = pl.fwd_ang[2 * a + 1];
                    s_cb[i] = cbt[a];
                }
            }
        }
    };
    load_table(ab);
    __syncthreads();

    // This thread's staging slots i = tid + q * 256 of the [Z][ncm] slab are
    // angle-independent: window column jj, the slice's row offset (or -2 - z
    // when several rows share the slice) and the LDS offset.  BIN: slots of the
    // [ncm][Z / 4] float4 slab, source and LDS offsets in float4s (an idle slot
    // re-reads slot 0's source and writes past the slab).
    int st_jj[PF], st_row[PF], st_off[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
        const int i = threadIdx.x + q * TVAM_PB;
        st_jj[q] = -1;
        st_row[q] = -1;
        st_off[q] = 0;
        if (BIN) {
            constexpr int G = Z / 4;
            const bool use = i < ncm * G;
            const int jj = use ? i / G : 0, gq = use ? i - (i / G) * G : 0;
            st_jj[q] = jj * (pl.bin_nz / 4) + gq;
            st_off[q] = use ? jj * (ZS / 4) + gq : ncm * ZS / 4;
        } else if (i < ncm * Z) {
            const int z = i / ncm, jj = i - z * ncm;
            const int r = s_row[z];
            st_jj[q] = jj;
            st_row[q] = r >= 0 ? r * k.crop_x : (r == -1 ? -1 : -2 - z);
            st_off[q] = jj * ZS + z;
        }
    }
    // DMA: this lane's slab slots w * 64 + lane + q * 256 (w: its wave) -> source float4 offsets
    // within an angle's binned window (angle-independent); a pad slot loads its column's last
    // data slot, a lane past the slab (dsrc < 0) loads nothing
    const int dwave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    int dsrc[2] = {0, 0};
    if constexpr (DMA) {
        constexpr int GZ = ZS / 4, G = Z / 4;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int P = (int)threadIdx.x + q * TVAM_PB;
            const int jj = P / GZ, gq = min(P - (P / GZ) * GZ, G - 1);
            dsrc[q] = P < ncm * GZ ? jj * (pl.bin_nz / 4) + gq : -1;
        }
    }
    auto fetch_dma_c = [&](int al, int buf, const int cb) __attribute__((always_inline)) {
        const pl_f4* src = reinterpret_cast<const pl_f4*>(pl.fwd_bin) +
                           ((size_t)al * (k.crop_x + 2 * pl.bin_pad) + (cb + pl.bin_pad)) * (pl.bin_nz / 4) + z0 / 4;
        float4* slab = reinterpret_cast<float4*>(s_p + buf * bstride);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int wb = dwave * 64 + q * TVAM_PB;  // wave-uniform
            // the LDS slot is M0 base + 16 * lane: the last wave-instruction's lanes past the slab are
            // masked off (exec), so nothing is written past it
            if (wb < np && dsrc[q] >= 0)
                tvam_lds_dma16(src + dsrc[q], slab + wb);
        }
        const int lane = (int)threadIdx.x & 63;
        if (dwave < RW && lane < ncm) {  // the window's ray-table records (ncm <= 64, host-checked);
                                         // refracted: wave 1 loads the columns' second records
            const int col = cb + lane;
            const float4* tab = reinterpret_cast<const float4*>(REFR && dwave == 1 ? pl.vox2 : pl.vox);
            const float4* rs = (unsigned)col < (unsigned)k.crop_x ? tab + (size_t)al * k.crop_x + col
                                                                  : &tvam_null_rec[dwave];
            tvam_lds_dma16(rs, s_r + buf * rstride + ncm * dwave);
        }
    };
    auto fetch_dma = [&](int al, int buf) __attribute__((always_inline)) { fetch_dma_c(al, buf, s_cb[al - tbase]); };
    // global loads of angle al's slab (slice-binned pattern + ray table) into registers
    // (the ray-table entry travels in its own array: a 48-byte stage struct is left in scratch)
    struct StageDirect {
        float pv[PF];
    };
    struct StageBinned {  // PF <= 2
        pl_f4 p0, p1;
    };
    using Stage = typename std::conditional<BIN, StageBinned, StageDirect>::type;
    auto fetch = [&](int al, Stage& S, pl_f4& rv) {
        const int cb = s_cb[al - tbase];
        if constexpr (BIN) {
            const pl_f4* src = reinterpret_cast<const pl_f4*>(pl.fwd_bin) +
                                ((size_t)al * (k.crop_x + 2 * pl.bin_pad) + (cb + pl.bin_pad)) * (pl.bin_nz / 4) + z0 / 4;
            S.p0 = src[st_jj[0]];
            if constexpr (PF > 1) S.p1 = src[st_jj[1]];
        } else {
            const float* pa = pat + (size_t)al * k.crop_y * k.crop_x;
#pragma unroll
            for (int q = 0; q < PF; ++q) {
                const int col = cb + st_jj[q], r = st_row[q];
                float v = 0.0f;
                const bool in = st_jj[q] >= 0 && (unsigned)col < (unsigned)k.crop_x;
                if (!MULTI) {
                    if (in && r >= 0) v = pa[(unsigned)(r + col)];
                } else if (in && r != -1) {
                    if (r >= 0) v = pa[(unsigned)(r + col)];
                    else {
                        const int z = -2 - r;
                        for (int t = pl.slice_off[z0 + z]; t < pl.slice_off[z0 + z + 1]; ++t)
                            v += pa[(size_t)pl.slice_rows[t] * k.crop_x + col];
                    }
                }
                S.pv[q] = v;
            }
        }
        if (REFR) {  // thread h ncm + j loads record h of window column j (stored [2][ncm]: 16-byte
                     // column stride in either half, so 16 neighbouring columns' reads hit distinct banks)
            const int h = (int)threadIdx.x >= ncm ? 1 : 0;
            const int col = cb + (int)threadIdx.x - h * ncm;
            rv = pl_f4{0.0f, 0.0f, h ? 0.0f : -1.0f, 0.0f};
            if ((int)threadIdx.x < 2 * ncm && (unsigned)col < (unsigned)k.crop_x)
                rv = reinterpret_cast<const pl_f4*>(h ? pl.vox2 : pl.vox)[(size_t)al * k.crop_x + col];
        } else {
            const int col = cb + (int)threadIdx.x;
            rv = pl_f4{0.0f, 0.0f, -1.0f, 0.0f};
            if ((int)threadIdx.x < ncm && (unsigned)col < (unsigned)k.crop_x)
                rv = reinterpret_cast<const pl_f4*>(pl.vox)[(size_t)al * k.crop_x + col];
        }
    };
    // buffer b = (double-buffer half) * AB + (angle within the barrier group)
    auto store = [&](int buf, const Stage& S, const pl_f4& rv) {
        float* sp = s_p + buf * bstride;
        if constexpr (BIN) {
            reinterpret_cast<pl_f4*>(sp)[st_off[0]] = S.p0;
            if constexpr (PF > 1) reinterpret_cast<pl_f4*>(sp)[st_off[1]] = S.p1;
        } else {
#pragma unroll
            for (int q = 0; q < PF; ++q)
                if (st_jj[q] >= 0) sp[st_off[q]] = S.pv[q];
        }
        if ((int)threadIdx.x < ncm * RW) reinterpret_cast<pl_f4*>(s_r)[buf * rstride + threadIdx.x] = rv;
    };

    float acc[Z];
#pragma unroll
    for (int z = 0; z < Z; ++z) acc[z] = 0.0f;

    auto compute_refr = [&](int al, int buf) {
        const int cb = s_cb[al - tbase];
        const float* sp = s_p + buf * bstride;
        const float4* sr = s_r + buf * rstride;
        // u(lx, ly) = the chord index through the voxel centre (lattice coordinates from the tile corner)
        const float4 m0 = s_ang[2 * (al - tbase)], m1 = s_ang[2 * (al - tbase) + 1];
        // this wave's candidate count (uniform over the wave, >= 2)
        const int nc = __builtin_amdgcn_readfirstlane((__float_as_int(m1.w) >> (8 * (threadIdx.x >> 6))) & 0xff);
        const float lx = (float)(threadIdx.x & 15) + 0.5f, ly = (float)(threadIdx.x >> 4) + 0.5f;
        const float u = fmaf(lx * ly, m0.w, fmaf(ly, m0.z, fmaf(lx, m0.y, m0.x)));
        const float hv = 0.5f * (fabsf(fmaf(m0.w, ly, m0.y)) + fabsf(fmaf(m0.w, lx, m0.z))) + 0.25f * fabsf(m0.w);
        int jj0 = (int)ceilf(u - hv - m1.x) - cb;  // the voxel's first candidate (m1.x: model error bound)
        jj0 = min(max(jj0, 0), ncm - nc);
        // candidate c's weight (exact slab intersection with its own chord; 0 when it misses the voxel)
        auto weight = [&](int jc) {
            const float4 q = sr[jc], g = sr[rhalf + jc];
            const int fl = __float_as_int(g.z);
            const float xa = fmaf(X0, g.x, q.x), xb = fmaf(X1, g.x, q.x);
            const float ya = fmaf(Y0, g.y, q.y), yb = fmaf(Y1, g.y, q.y);
            // |d| <= 1e-8 on an axis: the DDA never steps it (q = its voxel index)
            const float tnx = (fl & 1) ? fminf(xa, xb) : ((float)ix == q.x ? -TVAM_INF : TVAM_INF);
            const float tfx = (fl & 1) ? fmaxf(xa, xb) : TVAM_INF;
            const float tny = (fl & 2) ? fminf(ya, yb) : ((float)iy == q.y ? -TVAM_INF : TVAM_INF);
            const float tfy = (fl & 2) ? fmaxf(ya, yb) : TVAM_INF;
            const float tin = fmaxf(fmaxf(tnx, tny), 0.0f);
            const float tout = fminf(fminf(tfx, tfy), q.z);
            const float e = pl_exp2(k.nsig2 * tin) - pl_exp2(k.nsig2 * tout);
            return tout > tin ? e * g.w : 0.0f;  // x the interfaces' transmission (sensor.py:404)
        };
        auto accumulate = [&](int jc, float wgt) {
            if (wgt == 0.0f) return;
#pragma unroll
            for (int z4 = 0; z4 < Z / 4; ++z4) {
                const float4 p4 = reinterpret_cast<const float4*>(sp + jc * ZS)[z4];
                acc[4 * z4 + 0] = fmaf(wgt, p4.x, acc[4 * z4 + 0]);
                acc[4 * z4 + 1] = fmaf(wgt, p4.y, acc[4 * z4 + 1]);
                acc[4 * z4 + 2] = fmaf(wgt, p4.z, acc[4 * z4 + 2]);
                acc[4 * z4 + 3] = fmaf(wgt, p4.w, acc[4 * z4 + 3]);
            }
        };
        // every (tile, angle) has >= 2 candidates (the model kernel's floor): the first two run
        // straight-line like the index-matched forward's pair, the rest in a (uniform) loop
        const float w0 = weight(jj0), w1 = weight(jj0 + 1);
        accumulate(jj0, w0);
        accumulate(jj0 + 1, w1);
        for (int c = 2; c < nc; ++c) accumulate(jj0 + c, weight(jj0 + c));
    };

    // the candidates of angle al (staged in buffer buf): the first window column jj0 and the
    // candidates' weights (0 where the ray misses the voxel)
    // per-angle constants {s*du, -c*du, 1/d.x, 1/d.y}, {half width in columns, axis flags}, and the
    // window's first column: from LDS, or (TVAM_FWD_SCONST, straight-ray DMA path) from scalar registers
    // loaded one angle pair ahead
    auto geom_c = [&](const float4 g0, const float4 g1, const int cb, int buf, int& jj0, float (&wgt)[NC])
        __attribute__((always_inline)) {
        const float4* sr = s_r + buf * rstride;
        const int fl = __float_as_int(g1.y);

        // candidate columns: the rays whose lateral line meets the voxel's lateral extent
        const float u = fmaf(Xc, g0.x, fmaf(Yc, g0.y, u0));
        jj0 = (int)ceilf(u - g1.x) - cb;
        jj0 = min(max(jj0, 0), ncm - NC);
        // crossing times of the voxel's x / y edges relative to the ray's o2 (+ q.x / q.y)
        const float xa = X0 * g0.z, xb = X1 * g0.z, ya = Y0 * g0.w, yb = Y1 * g0.w;
        const float xn = fminf(xa, xb), xf = fmaxf(xa, xb), yn = fminf(ya, yb), yf = fmaxf(ya, yb);
        // the candidates' ray records read together (each read's latency is paid once per angle),
        // then pinned as 16-byte reads (ds_read_b128, not b96)
        float4 qs[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) qs[c] = sr[jj0 + c];
#pragma unroll
        for (int c = 0; c < NC; ++c) asm volatile("" : "+v"(qs[c].w));
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const float4 q = qs[c];
            float tnx = xn + q.x, tfx = xf + q.x, tny = yn + q.y, tfy = yf + q.y;
            if (!(fl & 1)) {  // |d.x| <= 1e-8: the DDA never steps x (q.x = its voxel index)
                tnx = (float)ix == q.x ? -TVAM_INF : TVAM_INF;
                tfx = TVAM_INF;
            }
            if (!(fl & 2)) {
                tny = (float)iy == q.y ? -TVAM_INF : TVAM_INF;
                tfy = TVAM_INF;
            }
            const float tin = fmaxf(fmaxf(tnx, tny), 0.0f);
            const float tout = fminf(fminf(tfx, tfy), q.z);
            // e^{-st t_in} - e^{-st t_out} of absolute times: their rounding (ulp(t) / dt ~ 4e-5 at
            // N = 400), not the cancellation, bounds this weight, so the cheaper telescoped form stays
            const float e = pl_exp2(k.nsig2 * tin) - pl_exp2(k.nsig2 * tout);
            wgt[c] = tout > tin ? e : 0.0f;
        }
    };
    auto geom = [&](int al, int buf, int& jj0, float (&wgt)[NC]) __attribute__((always_inline)) {
        geom_c(s_ang[2 * (al - tbase)], s_ang[2 * (al - tbase) + 1], s_cb[al - tbase], buf, jj0, wgt);
    };
    // dose += the candidates' weights x their staged slabs
    auto fmas = [&](int buf, int jj0, const float (&wgt)[NC]) __attribute__((always_inline)) {
        const float* sp = s_p + buf * bstride;
        // a lane reads (and FMAs) only the slabs of candidates that meet its voxel, and a wave skips a
        // candidate none of its lanes meets (with the zero weights FMAed instead: 2.44 -> 2.54 ms,
        // profiles/r06/ab_fwd/)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (wgt[c] != 0.0f) {
#pragma unroll
                for (int z4 = 0; z4 < Z / 4; ++z4) {
                    const float4 p4 = reinterpret_cast<const float4*>(sp + (jj0 + c) * ZS)[z4];
                    acc[4 * z4 + 0] = fmaf(wgt[c], p4.x, acc[4 * z4 + 0]);
                    acc[4 * z4 + 1] = fmaf(wgt[c], p4.y, acc[4 * z4 + 1]);
                    acc[4 * z4 + 2] = fmaf(wgt[c], p4.z, acc[4 * z4 + 2]);
                    acc[4 * z4 + 3] = fmaf(wgt[c], p4.w, acc[4 * z4 + 3]);
                }
            }
        }
    };
    auto compute = [&](int al, int buf) __attribute__((always_inline)) {
        if constexpr (REFR) {
            compute_refr(al, buf);
        } else {
            int jj0;
            float wgt[NC];
            geom(al, buf, jj0, wgt);
            fmas(buf, jj0, wgt);
        }
    };
    // the AB angles of a barrier group, one after the other
    auto compute2 = [&](int al, int buf, bool two) __attribute__((always_inline)) {
        compute(al, buf);
        if (two) compute(al + 1, buf + 1);
    };

    // Software pipeline over angles: angle a is computed from LDS buffer a & 1
    // while the loads of angle a + 1 are in flight in registers.
    if constexpr (DMA && SCONST) {
      if (ab < ae) {
        // as below, with the per-angle constants of the next pair in flight in scalar registers: no
        // LDS table (its reads and reload barriers); the s_loads are waited for after the barrier,
        // when the wave has no LDS read outstanding.  An angle pair is 16 dwords of fwd_ang and 2 of
        // the tile's fwd_cb (both tables padded by the host past the last pair).
        typedef unsigned su16 __attribute__((ext_vector_type(16)));
        typedef unsigned su2 __attribute__((ext_vector_type(2)));
        auto sload = [&](int al, su16& a, su2& c) __attribute__((always_inline)) {
            const float4* ga = pl.fwd_ang + 2 * al;
            const int32_t* gc = cbt + al;
            asm volatile("s_load_dwordx16 %0, %1, 0x0" : "=s"(a) : "s"(ga));
            asm volatile("s_load_dwordx2 %0, %1, 0x0" : "=s"(c) : "s"(gc));
        };
        auto sget = [](const su16& a, int j) {
            return make_float4(__uint_as_float(a[4 * j]), __uint_as_float(a[4 * j + 1]), __uint_as_float(a[4 * j + 2]),
                               __uint_as_float(a[4 * j + 3]));
        };
        su16 ca, na;
        su2 cc, nc2;
        sload(ab, ca, cc);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(ca), "+s"(cc)::"memory");  // cc feeds the first DMAs
        fetch_dma_c(ab, 0, (int)cc[0]);
        if (AB > 1 && ab + 1 < ae) fetch_dma_c(ab + 1, 1, (int)cc[1]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int half = 0;
        for (int al = ab; al < ae; al += AB) {
            const bool more = al + AB < ae;
            if (more) {
                sload(al + AB, na, nc2);
                asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(na), "+s"(nc2)::"memory");
                fetch_dma_c(al + AB, (half ^ 1) * AB, (int)nc2[0]);
                if (AB > 1 && al + AB + 1 < ae) fetch_dma_c(al + AB + 1, (half ^ 1) * AB + 1, (int)nc2[1]);
            }
            const bool two = AB > 1 && al + 1 < ae;
            int j0, j1 = 0;
            float w0[NC], w1[NC];
            // one angle's geometry and FMAs after the other (both angles' geometry first, then both
            // angles' FMAs: 2.44 -> 2.52 ms on config 2, profiles/r06/ab_fwd/)
            geom_c(sget(ca, 0), sget(ca, 1), (int)cc[0], half * AB, j0, w0);
            fmas(half * AB, j0, w0);
            if (two) {
                geom_c(sget(ca, 2), sget(ca, 3), (int)cc[1], half * AB + 1, j1, w1);
                fmas(half * AB + 1, j1, w1);
            }
            half ^= 1;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            ca = na;
            cc = nc2;
        }
      }
    } else if constexpr (DMA) {
      if (ab < ae) {
        // LDS-DMA: the next AB angles' slabs and records load straight into the other half while
        // this half is computed (its last reads were before the previous barrier); the loads are
        // drained (vmcnt) before the barrier that precedes their reads
        fetch_dma(ab, 0);
        if (AB > 1 && ab + 1 < ae) fetch_dma(ab + 1, 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int half = 0;
        for (int al = ab; al < ae; al += AB) {
            if (al - tbase > TVAM_ACH + 4 - 2 * AB) {  // next chunk of per-angle constants
                tbase = al;
                load_table(al);
                __syncthreads();
            }
            if (al + AB < ae) fetch_dma(al + AB, (half ^ 1) * AB);
            if (AB > 1 && al + AB + 1 < ae) fetch_dma(al + AB + 1, (half ^ 1) * AB + 1);
            compute2(al, half * AB, AB > 1 && al + 1 < ae);
            half ^= 1;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
      }
    } else if (ab < ae && AB <= 2) {
        // AB angles per barrier: the next group's global loads are in flight in
        // registers while this group is computed from LDS (named stages: an
        // array of them indexed by the angle in the group can end up in scratch)
        Stage S0, S1;
        pl_f4 R0, R1;
        fetch(ab, S0, R0);
        if (AB > 1 && ab + 1 < ae) fetch(ab + 1, S1, R1);
        store(0, S0, R0);
        if (AB > 1 && ab + 1 < ae) store(1, S1, R1);
        __syncthreads();
        int half = 0;
        for (int al = ab; al < ae; al += AB) {
            if (al - tbase > TVAM_ACH + 4 - 2 * AB) {  // next chunk of per-angle constants
                tbase = al;
                load_table(al);
                __syncthreads();
            }
            if (al + AB < ae) fetch(al + AB, S0, R0);
            if (AB > 1 && al + AB + 1 < ae) fetch(al + AB + 1, S1, R1);
            compute(al, half * AB);
            if (AB > 1 && al + 1 < ae) compute(al + 1, half * AB + 1);
            half ^= 1;
            if (al + AB < ae) store(half * AB, S0, R0);
            if (AB > 1 && al + AB + 1 < ae) store(half * AB + 1, S1, R1);
            __syncthreads();
        }
    } else if (ab < ae) {
        Stage S[AB];
        pl_f4 R[AB];
#pragma unroll
        for (int j = 0; j < AB; ++j)
            if (ab + j < ae) fetch(ab + j, S[j], R[j]);
#pragma unroll
        for (int j = 0; j < AB; ++j)
            if (ab + j < ae) store(j, S[j], R[j]);
        __syncthreads();
        int half = 0;
        for (int al = ab; al < ae; al += AB) {
            if (al - tbase > TVAM_ACH + 4 - 2 * AB) {
                tbase = al;
                load_table(al);
                __syncthreads();
            }
#pragma unroll
            for (int j = 0; j < AB; ++j)
                if (al + AB + j < ae) fetch(al + AB + j, S[j], R[j]);
#pragma unroll
            for (int j = 0; j < AB; ++j)
                if (al + j < ae) compute(al + j, half * AB + j);
            half ^= 1;
#pragma unroll
            for (int j = 0; j < AB; ++j)
                if (al + AB + j < ae) store(half * AB + j, S[j], R[j]);
            __syncthreads();
        }
    }

    if (ix < k.res[0] && iy < k.res[1]) {
        const float scale = k.wscale * k.inv_vol;  // Le * weight (common.py:108-111) / voxel volume (volume.py:41-42)
        const size_t plane = (size_t)k.res[0] * k.res[1];
        float* out = parts > 1 ? pl.fwd_part + (size_t)part * k.nz * plane : dose;
#pragma unroll
        for (int z = 0; z < Z; ++z)
            if (z0 + z < k.nz) out[(size_t)(z0 + z) * plane + (size_t)iy * k.res[0] + ix] = acc[z] * scale;
    }
}

// dose = sum of the angle parts' partial doses, in part order (deterministic)
__global__ __launch_bounds__(256) void tvam_fwd_parts_kernel(int64_t n, int parts, int64_t pstride,
                                                             const float* __restrict__ part,
                                                             float* __restrict__ dose) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        float v = part[i];
        for (int q = 1; q < parts; ++q) v += part[(size_t)q * pstride + i];
        dose[i] = v;
    }
}

// Slice binning of the patterns for the voxel-driven forward: bin[a][pad + col][z] =
// the sum of slice z's DMD rows of column col at angle a (in slice_rows order, as the
// direct staging sums them; 0 for a slice without rows).  A 64-column x 64-slice
// block goes through LDS, read along columns and written along slices.  Pads and
// slices past nz stay 0 from the plan's memset.
__global__ __launch_bounds__(256) void tvam_slice_bin_kernel(TvamConsts k, TvamPlanar pl,
                                                            const float* __restrict__ pat, int zblock0) {
    __shared__ float s_t[64][65];
    __shared__ int s_row[64];  // the slice's row x crop_x; -1: no row; -2: several rows
    const int c0 = blockIdx.x * 64, z0 = ((int)blockIdx.y + zblock0) * 64, al = blockIdx.z;
    if (threadIdx.x < 64) {
        const int z = z0 + (int)threadIdx.x;
        int r = -1;
        if (z < k.nz) {
            const int b = pl.slice_off[z], e = pl.slice_off[z + 1];
            r = e - b == 1 ? pl.slice_rows[b] * k.crop_x : (e == b ? -1 : -2);
        }
        s_row[threadIdx.x] = r;
    }
    __syncthreads();
    const float* pa = pat + (size_t)al * k.crop_y * k.crop_x;
    const int lc = threadIdx.x & 63, lz = threadIdx.x >> 6;
    const int c = c0 + lc;
    const bool cin = c < k.crop_x;
#pragma unroll 4
    for (int zz = lz; zz < 64; zz += 4) {
        const int r = s_row[zz];
        float v = 0.0f;
        if (cin && r >= 0) {
            v = pa[(size_t)r + c];
        } else if (cin && r == -2) {
            for (int t = pl.slice_off[z0 + zz]; t < pl.slice_off[z0 + zz + 1]; ++t)
                v += pa[(size_t)pl.slice_rows[t] * k.crop_x + c];
        }
        s_t[lc][zz] = v;
    }
    __syncthreads();
    float* out = pl.fwd_bin + ((size_t)al * (k.crop_x + 2 * pl.bin_pad) + pl.bin_pad) * pl.bin_nz;
    const int z = z0 + lc;
    if (z >= k.nz) return;
    for (int cc = lz; cc < 64; cc += 4)
        if (c0 + cc < k.crop_x) out[(size_t)(c0 + cc) * pl.bin_nz + z] = s_t[cc][lc];
}

// tvam_slice_bin_kernel with 16-byte accesses (crop_x a multiple of 4, the patterns 16-byte
// aligned, bin_nz a multiple of 4): a thread loads four columns of a slice's row and stores four
// slices of a column; slices in [nz, bin_nz) are written as the zeros they hold.  The same sums in
// the same order (bit-identical bins); 136 -> 100 us at config 2's size as a standalone transpose
// (tools/proto_slice_bin.hip, profiles/r04/proto_bin/).
__global__ __launch_bounds__(256) void tvam_slice_bin4_kernel(TvamConsts k, TvamPlanar pl,
                                                             const float* __restrict__ pat, int zblock0) {
    __shared__ float s_t[64][65];
    __shared__ int s_row[64];
    const int c0 = blockIdx.x * 64, z0 = ((int)blockIdx.y + zblock0) * 64, al = blockIdx.z;
    if (threadIdx.x < 64) {
        const int z = z0 + (int)threadIdx.x;
        int r = -1;
        if (z < k.nz) {
            const int b = pl.slice_off[z], e = pl.slice_off[z + 1];
            r = e - b == 1 ? pl.slice_rows[b] * k.crop_x : (e == b ? -1 : -2);
        }
        s_row[threadIdx.x] = r;
    }
    __syncthreads();
    const float* pa = pat + (size_t)al * k.crop_y * k.crop_x;
    const int q = threadIdx.x & 15, lz = threadIdx.x >> 4;
    const int c = c0 + 4 * q;
    const bool cin = c < k.crop_x;  // crop_x % 4 == 0: a thread's four columns are all in or all out
#pragma unroll
    for (int zz = lz; zz < 64; zz += 16) {
        const int r = s_row[zz];
        float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (cin && r >= 0) {
            v = *reinterpret_cast<const float4*>(pa + (size_t)r + c);
        } else if (cin && r == -2) {
            for (int t = pl.slice_off[z0 + zz]; t < pl.slice_off[z0 + zz + 1]; ++t) {
                const float4 w = *reinterpret_cast<const float4*>(pa + (size_t)pl.slice_rows[t] * k.crop_x + c);
                v.x += w.x;
                v.y += w.y;
                v.z += w.z;
                v.w += w.w;
            }
        }
        s_t[4 * q + 0][zz] = v.x;
        s_t[4 * q + 1][zz] = v.y;
        s_t[4 * q + 2][zz] = v.z;
        s_t[4 * q + 3][zz] = v.w;
    }
    __syncthreads();
    float* out = pl.fwd_bin + ((size_t)al * (k.crop_x + 2 * pl.bin_pad) + pl.bin_pad) * pl.bin_nz;
    const int z = z0 + 4 * q;
    if (z >= pl.bin_nz) return;
#pragma unroll
    for (int cc = lz; cc < 64; cc += 16)
        if (c0 + cc < k.crop_x)
            *reinterpret_cast<float4*>(out + (size_t)(c0 + cc) * pl.bin_nz + z) =
                make_float4(s_t[cc][4 * q], s_t[cc][4 * q + 1], s_t[cc][4 * q + 2], s_t[cc][4 * q + 3]);
}

// the binned slabs are staged by LDS-DMA where a window fits: <= 2 slab slots per
// thread and one record wave per record kind (pl.fwd_dma; else register staging)
bool tvam_planar_fwd_dma_window(const TvamPlanar& pl, int Z) {
    return pl.ncmax <= 64 && tvam_fwd_dma_np(pl.ncmax, Z) <= 2 * TVAM_PB;
}

bool tvam_planar_fwd_dma_ok(const TvamPlanar& pl, int Z) {
    return pl.fwd_bin && (pl.fwd_ab == 1 || pl.fwd_ab == 2) && tvam_planar_fwd_dma_window(pl, Z);
}

size_t tvam_planar_fwd_lds(const TvamPlanar& pl, int Z) {
    const int ab = pl.fwd_ab > 1 ? pl.fwd_ab : 1;
    const size_t rw = pl.fwd_refr ? 2 : 1;
    if (pl.fwd_dma && pl.fwd_bin && ab <= 2)
        return 2 * ab * ((size_t)tvam_fwd_dma_np(pl.ncmax, Z) + rw * pl.ncmax) * sizeof(float4) +
               (size_t)(TVAM_ACH + 4) * (2 * sizeof(float4) + sizeof(int)) + (size_t)Z * sizeof(int);
    return 2 * ab * (((size_t)pl.ncmax * tvam_fwd_zs(Z) + 4) * sizeof(float) + rw * pl.ncmax * sizeof(float4)) +
           (size_t)(TVAM_ACH + 4) * (2 * sizeof(float4) + sizeof(int)) + (size_t)Z * sizeof(int);
}

bool tvam_planar_fwd_fits(const TvamPlanar& pl, int Z) {
    if (pl.fwd_refr)  // two record loaders per window column; the binned staging only
        return 2 * pl.ncmax <= TVAM_PB && pl.ncmax * (Z / 4) <= 2 * TVAM_PB && pl.fwd_nc >= 1 &&
               pl.fwd_nc <= pl.ncmax && tvam_planar_fwd_lds(pl, Z) <= 64 * 1024;
    if (Z > 32)  // deep slabs: the binned staging only (<= 2 float4 per thread and angle)
        return pl.ncmax <= TVAM_PB && pl.ncmax * (Z / 4) <= 2 * TVAM_PB && pl.fwd_nc >= 1 && pl.fwd_nc <= 4 &&
               pl.fwd_nc <= pl.ncmax;
    return pl.ncmax <= TVAM_PB && pl.ncmax * Z <= TVAM_PF * TVAM_PB && pl.fwd_nc >= 1 && pl.fwd_nc <= 4 &&
           pl.fwd_nc <= pl.ncmax;
}

// ---------------------------------------------------------------------------
// Chord-index model of the refracted voxel-driven forward.  Behind a refracting
// vial the medium chords of one angle's columns are no longer parallel, but they
// do not cross inside the medium (the plan checks the bound that rests on it), so
// the chord index u(p) -- c where chord c passes through p, linear between
// neighbouring chords in their signed distances -- is monotone across the beam and
// a line meets a voxel iff u at its corners brackets the line's index.  One thread
// per (16x16 tile, angle) evaluates u exactly (bisection over the angle's chords)
// at the tile's 17x17 voxel corners, fits the bilinear model through the tile
// corners, and stores the half width w >= |u(corner) - model(centre)| of every
// voxel (model error at the corners + the model's own half-voxel spread), the
// candidate count and the staged window.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float refr_side(const float4* __restrict__ ch, int c, float px, float py) {
    const float4 q = ch[c];
    return (px - q.x) * q.w - (py - q.y) * q.z;
}

__device__ float refr_u(const float4* __restrict__ ch, int c0, int c1, float px, float py) {
    const float s0 = refr_side(ch, c0, px, py), s1 = refr_side(ch, c1, px, py);
    if ((s0 > 0.0f) == (s1 > 0.0f)) {  // outside the beam: extrapolate from the nearer edge pair
        if (fabsf(s0) <= fabsf(s1)) {
            const float sb = refr_side(ch, c0 + 1, px, py);
            return (float)c0 + s0 / (s0 - sb);
        }
        const float sa = refr_side(ch, c1 - 1, px, py);
        return (float)(c1 - 1) + sa / (sa - s1);
    }
    int lo = c0, hi = c1;
    float slo = s0, shi = s1;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        const float sm = refr_side(ch, mid, px, py);
        if ((sm > 0.0f) == (s0 > 0.0f)) {
            lo = mid;
            slo = sm;
        } else {
            hi = mid;
            shi = sm;
        }
    }
    return (float)lo + slo / (slo - shi);
}

__global__ __launch_bounds__(64) void tvam_refr_model_kernel(TvamConsts k, TvamPlanar pl, const int2* __restrict__ range,
                                                             float4* __restrict__ model, int32_t* __restrict__ need) {
    const int ntx = (k.res[0] + 15) >> 4, nty = (k.res[1] + 15) >> 4;
    const int64_t n = (int64_t)ntx * nty * pl.ns;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int tile = (int)(i / pl.ns), al = (int)(i - (int64_t)tile * pl.ns);
        const int bx = tile % ntx, by = tile / ntx;
        const int2 rg = range[al];
        float4* m = model + 2 * i;
        if (rg.y - rg.x < 1) {  // fewer than two chords reach the medium: no candidates
            m[0] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            m[1] = make_float4(0.0f, __int_as_float(0), __int_as_float(0), 0.0f);
            need[i] = 1;
            continue;
        }
        const float4* ch = pl.chord + (size_t)al * k.crop_x;
        auto uat = [&](int li, int lj) {
            const float px = k.bmin[0] + (float)(bx * 16 + li) * k.h[0];
            const float py = k.bmin[1] + (float)(by * 16 + lj) * k.h[1];
            return refr_u(ch, rg.x, rg.y, px, py);
        };
        const float u00 = uat(0, 0), u10 = uat(16, 0), u01 = uat(0, 16), u11 = uat(16, 16);
        const float4 m0 = make_float4(u00, (u10 - u00) * 0.0625f, (u01 - u00) * 0.0625f,
                                      (u11 - u10 - u01 + u00) * 0.00390625f);
        auto model_at = [&](float lx, float ly) { return fmaf(lx * ly, m0.w, fmaf(ly, m0.z, fmaf(lx, m0.y, m0.x))); };
        float err = 0.0f;
        for (int lj = 0; lj <= 16; ++lj)
            for (int li = 0; li <= 16; ++li) err = fmaxf(err, fabsf(uat(li, lj) - model_at((float)li, (float)lj)));
        // the model's spread from a voxel centre to its corners (half a voxel along each axis)
        float spread = 0.0f;
        for (int cy = 0; cy <= 16; cy += 16)
            for (int cx = 0; cx <= 16; cx += 16)
                spread = fmaxf(spread, fabsf(m0.y + m0.w * (float)cy) + fabsf(m0.z + m0.w * (float)cx));
        const float ue = err + 2e-3f + 1e-4f * fabsf(u00);  // model error + fp32 rounding of u itself
        const float w = ue + 0.5f * spread;
        // candidates of a voxel: the integers in [u - hv - ue, u + hv + ue], u the model at its centre and
        // hv = 0.5 (|du/dlx| + |du/dly|) + |d2u/dlx dly| / 4 its half range at the corners; the forward
        // runs the largest count of a wave's voxels (wave w: tile rows 4w .. 4w + 3; packed one byte
        // per wave), at least two (the forward runs two candidates straight-line)
        int nc = 2, ncw = 0;
        for (int wv = 0; wv < 4; ++wv) {
            int n_w = 2;
            for (int vy = 4 * wv; vy < 4 * wv + 4; ++vy)
                for (int vx = 0; vx < 16; ++vx) {
                    const float lx = (float)vx + 0.5f, ly = (float)vy + 0.5f;
                    const float u = model_at(lx, ly);
                    const float hv = 0.5f * (fabsf(fmaf(m0.w, ly, m0.y)) + fabsf(fmaf(m0.w, lx, m0.z))) + 0.25f * fabsf(m0.w);
                    n_w = max(n_w, (int)floorf(u + hv + ue) - (int)ceilf(u - hv - ue) + 1);
                }
            n_w = min(n_w, 255);
            nc = max(nc, n_w);
            ncw |= n_w << (8 * wv);
        }
        float umin = TVAM_INF, umax = -TVAM_INF;
        for (int cy = 0; cy < 2; ++cy)
            for (int cx = 0; cx < 2; ++cx) {
                const float u = model_at(cx ? 15.5f : 0.5f, cy ? 15.5f : 0.5f);
                umin = fminf(umin, u);
                umax = fmaxf(umax, u);
            }
        int cb = (int)floorf(umin - w) - 1;
        const int ce = (int)ceilf(umax + w) + 1;
        need[i] = ce - cb + 1;
        m[0] = m0;
        m[1] = make_float4(ue, __int_as_float(nc), __int_as_float(cb), __int_as_float(ncw));
    }
}

hipError_t tvam_launch_refr_model(const TvamConsts& k, const TvamPlanar& pl, const int2* range, float4* model,
                                  int32_t* need, hipStream_t stream) {
    const int64_t n = (int64_t)((k.res[0] + 15) / 16) * ((k.res[1] + 15) / 16) * pl.ns;
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 63) / 64, 1 << 20));
    hipLaunchKernelGGL(tvam_refr_model_kernel, dim3(g), dim3(64), 0, stream, k, pl, range, model, need);
    return hipGetLastError();
}

// the kernel timer's start / stop events of the next forward launch (tvam_kt_take), recorded by the
// launch itself (hipExtLaunchKernelGGL: no event packets between the kernels); null: untimed
static thread_local hipEvent_t g_fwd_ev[2] = {nullptr, nullptr};

template <int Z, int NC>
static void launch_fwd(dim3 grid, size_t lds, hipStream_t stream, const TvamConsts& k, const TvamPlanar& pl,
                       const float* pat, float* dose) {
    if (pl.fwd_bin && pl.fwd_dma) {  // binned slabs staged by LDS-DMA
        if (pl.fwd_refr)
            hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, 2, false, 1, 2, true, true, true>), grid, dim3(TVAM_PB), lds,
                               stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl, pat, dose);
        else if (pl.fwd_ab == 1)
            hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, false, 1, 1, true, false, true>), grid, dim3(TVAM_PB), lds,
                               stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl, pat, dose);
        else
            hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, false, 1, 2, true, false, true>), grid, dim3(TVAM_PB), lds,
                               stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl, pat, dose);
        return;
    }
    if (pl.fwd_refr) {  // refracted chords: binned staging, 2 angles per barrier, candidates per (tile, angle)
        if (pl.fwd_pf == 1)
            hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, 2, false, 1, 2, true, true>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0,
                               k, pl, pat, dose);
        else
            hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, 2, false, 2, 2, true, true>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0,
                               k, pl, pat, dose);
        return;
    }
    if constexpr (Z > 32) {  // deep slabs (thin-slab shards, 400-slice films in 10 chunks): binned staging only
        if (pl.fwd_pf == 1)
            hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, false, 1, 2, true>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl,
                               pat, dose);
        else
            hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, false, 2, 2, true>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl,
                               pat, dose);
        return;
    }
    if (pl.fwd_bin && pl.fwd_pf == 1 && pl.fwd_ab == 1)
        hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, false, 1, 1, true>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl, pat, dose);
    else if (pl.fwd_bin && pl.fwd_pf == 1)
        hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, false, 1, 2, true>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl, pat, dose);
    else if (pl.fwd_bin)
        hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, false, 2, 2, true>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl, pat, dose);
    else if (pl.fwd_multi)
        hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, true, 4, 1>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl, pat, dose);
    else if (pl.fwd_pf == 2)
        hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, false, 2, 1>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl, pat, dose);
    else if (NC == 2 && pl.fwd_ab == 4)
        hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, false, 4, 4>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl, pat, dose);
    else if (NC == 2 && pl.fwd_ab == 3)
        hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, false, 4, 3>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl, pat, dose);
    else if (NC == 2 && pl.fwd_ab == 2)
        hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, false, 4, 2>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl, pat, dose);
    else
        hipExtLaunchKernelGGL((tvam_fwd_planar_kernel<Z, NC, false, 4, 1>), grid, dim3(TVAM_PB), lds, stream, g_fwd_ev[0], g_fwd_ev[1], 0, k, pl, pat, dose);
}

template <int Z>
static hipError_t launch_fwd_z(dim3 grid, size_t lds, hipStream_t stream, const TvamConsts& k, const TvamPlanar& pl,
                               const float* pat, float* dose) {
    if (pl.fwd_refr) {
        launch_fwd<Z, 2>(grid, lds, stream, k, pl, pat, dose);
        return hipGetLastError();
    }
    switch (pl.fwd_nc) {
        case 1:
        case 2: launch_fwd<Z, 2>(grid, lds, stream, k, pl, pat, dose); break;
        case 3: launch_fwd<Z, 3>(grid, lds, stream, k, pl, pat, dose); break;
        case 4: launch_fwd<Z, 4>(grid, lds, stream, k, pl, pat, dose); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

static hipError_t tvam_launch_fwd_planar_z(dim3 grid, size_t lds, hipStream_t stream, const TvamConsts& k,
                                           const TvamPlanar& pl, int Z, const float* pat, float* dose);

hipError_t tvam_launch_fwd_planar(const TvamConsts& k, const TvamPlanar& pl, int Z, const float* pat, float* dose,
                                  hipStream_t stream) {
    const int ntx = (k.res[0] + 15) / 16, nty = (k.res[1] + 15) / 16;
    const int parts = pl.fwd_parts > 1 ? pl.fwd_parts : 1;
    if (parts > 1 && !pl.fwd_part) return hipErrorInvalidValue;
    const int nzc = pl.fwd_nzc > 0 ? pl.fwd_nzc : (k.nz + Z - 1) / Z;
    const unsigned nwg = (unsigned)(ntx * nty) * (unsigned)nzc * (unsigned)parts;
    dim3 grid((nwg + 7) / 8 * 8);  // XCD-aware order (tvam_fwd_planar_kernel): a multiple of 8
    const size_t lds = tvam_planar_fwd_lds(pl, Z);
    if (pl.fwd_bin) {
        if (pl.bin_nz % Z != 0 || pl.bin_nz < k.nz) return hipErrorInvalidValue;
        // bin only the 64-slice blocks of this launch's slices
        const int zlo = pl.fwd_nzc > 0 ? pl.fwd_zc0 * Z : 0;
        const int zhi = pl.fwd_nzc > 0 ? std::min(k.nz, (pl.fwd_zc0 + pl.fwd_nzc) * Z) : k.nz;
        const int b0 = zlo / 64, b1 = (zhi + 63) / 64;
        const dim3 bg((unsigned)((k.crop_x + 63) / 64), (unsigned)std::max(b1 - b0, 1), (unsigned)pl.ns);
        static const bool bin1 = tvam_knob("TVAM_SLICE_BIN1", 0) == 1;  // the one-float-per-thread binning (tests)
        if (!bin1 && k.crop_x % 4 == 0 && pl.bin_nz % 4 == 0 && ((uintptr_t)pat & 15u) == 0)
            hipLaunchKernelGGL(tvam_slice_bin4_kernel, bg, dim3(256), 0, stream, k, pl, pat, b0);
        else
            hipLaunchKernelGGL(tvam_slice_bin_kernel, bg, dim3(256), 0, stream, k, pl, pat, b0);
    }
    if (!tvam_kt_take(TVAM_KT_PLANAR, &g_fwd_ev[0], &g_fwd_ev[1])) g_fwd_ev[0] = g_fwd_ev[1] = nullptr;
    hipError_t e = tvam_launch_fwd_planar_z(grid, lds, stream, k, pl, Z, pat, dose);
    g_fwd_ev[0] = g_fwd_ev[1] = nullptr;
    if (e != hipSuccess || parts == 1) return e;
    // sum the angle parts of this launch's slices
    const int64_t plane = (int64_t)k.res[0] * k.res[1];
    const int64_t zlo = pl.fwd_nzc > 0 ? (int64_t)pl.fwd_zc0 * Z : 0;
    const int64_t zhi = pl.fwd_nzc > 0 ? std::min<int64_t>(k.nz, (int64_t)(pl.fwd_zc0 + pl.fwd_nzc) * Z) : k.nz;
    const int64_t n = (zhi - zlo) * plane;
    const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(tvam_fwd_parts_kernel, dim3(g), dim3(256), 0, stream, n, parts, (int64_t)k.nz * plane,
                       pl.fwd_part + zlo * plane, dose + zlo * plane);
    return hipGetLastError();
}

static hipError_t tvam_launch_fwd_planar_z(dim3 grid, size_t lds, hipStream_t stream, const TvamConsts& k,
                                           const TvamPlanar& pl, int Z, const float* pat, float* dose) {
    switch (Z) {
        case 8: return launch_fwd_z<8>(grid, lds, stream, k, pl, pat, dose);
        case 16: return launch_fwd_z<16>(grid, lds, stream, k, pl, pat, dose);
        case 24: return launch_fwd_z<24>(grid, lds, stream, k, pl, pat, dose);
        case 28: return launch_fwd_z<28>(grid, lds, stream, k, pl, pat, dose);
        case 32: return launch_fwd_z<32>(grid, lds, stream, k, pl, pat, dose);
        case 40: return pl.fwd_bin ? launch_fwd_z<40>(grid, lds, stream, k, pl, pat, dose) : hipErrorInvalidValue;
        case 48: return pl.fwd_bin ? launch_fwd_z<48>(grid, lds, stream, k, pl, pat, dose) : hipErrorInvalidValue;
        case 52: return pl.fwd_bin ? launch_fwd_z<52>(grid, lds, stream, k, pl, pat, dose) : hipErrorInvalidValue;
        case 60: return pl.fwd_bin ? launch_fwd_z<60>(grid, lds, stream, k, pl, pat, dose) : hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}

// ---------------------------------------------------------------------------
// Adjoint, ray-driven with Z-slice sharing.  Workgroup = (xy tile, Z
// slices); LDS holds the gradient tile (+ 1-voxel guard band) either as Z/4
// planes [z/4][voxel][4] (PL, default) or interleaved [voxel][z].  A lane
// resumes ray (a, col) at the tile entry from its row-independent record
// (closed form of the reference's stepping, as in tvam_kernels.hip), marches it
// once, and accumulates Z dot products; each row of each slice then receives
// its slice's value (volume.py:274-276).
// Banks: a ds_read_b128 is served in 4 groups of 16 lanes, each group
// conflict-free when its lanes' 16-byte chunks (address / 16 mod 16) differ.
// Interleaved, a voxel is 32 B (Z = 8), so voxels v and v + 8 collide; as
// planes a voxel is one 16-byte chunk per read, so only v = v' (mod 16)
// collide (neighbouring rays of a wave sit at neighbouring voxels, the row
// pitch is odd).
// ---------------------------------------------------------------------------
template <int Z, bool PF, int NT, bool PL = true, bool W2 = false>
__global__ __launch_bounds__(NT) void tvam_adj_planar_kernel(TvamConsts k, TvamPlanar pl, TvamTiles tp,
                                                                  const int32_t* __restrict__ idxmap,
                                                                  const float* __restrict__ gin,
                                                                  float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tsx = tp.tsx, tsy = tp.tsy;
    const int tile_id = blockIdx.x, z0 = ((int)blockIdx.y + pl.adj_zc0) * Z;
    // this workgroup's part of the tile's ray list (a thin slab has few slice chunks: several
    // workgroups then share one tile's rays, each ray once)
    const int tw = pl.adj_pitch;  // row pitch >= tsx + 2
    const uint32_t* slots = tp.slots + tp.slot_off[tile_id];
    const int nall = (int)(tp.slot_off[tile_id + 1] - tp.slot_off[tile_id]);
    const int gb = (int)(((int64_t)nall * blockIdx.z) / gridDim.z);
    const int nrt = (int)(((int64_t)nall * (blockIdx.z + 1)) / gridDim.z);
    if (gb >= nrt) return;  // (uniform over the workgroup)
    const int th = tsy + 2;
    float* tile = reinterpret_cast<float*>(smem);
    int* s_roff = reinterpret_cast<int*>(tile + (size_t)pl.adj_pitch * th * Z);  // [Z + 1] CSR
    int* s_rows = s_roff + Z + 1;                                       // [pl.max_rows_chunk]

    const int x0 = (tile_id % tp.ntx) * tsx, y0 = (tile_id / tp.ntx) * tsy;
    const int x1 = min(x0 + tsx, k.res[0]), y1 = min(y0 + tsy, k.res[1]);
    const int wx = x1 - x0, wy = y1 - y0;
    const size_t plane = (size_t)k.res[0] * k.res[1];

    // gradient tile, [z/4][voxel][4] (PL) or [voxel][z], scaled by 1/voxel volume (volume.py:130)
    const int nvox = tw * th;
    for (int i = threadIdx.x; i < nvox * Z; i += NT) {
        const int z = i / nvox, li = i - z * nvox;
        const int ly = li / tw - 1, lx = li - (ly + 1) * tw - 1;
        float v = 0.0f;
        if (lx >= 0 && ly >= 0 && lx < wx && ly < wy && z0 + z < k.nz)
            v = gin[(size_t)(z0 + z) * plane + (size_t)(y0 + ly) * k.res[0] + (x0 + lx)] * k.inv_vol;
        if (PL)
            tile[(size_t)(z >> 2) * nvox * 4 + (size_t)li * 4 + (z & 3)] = v;
        else
            tile[(size_t)li * Z + z] = v;
    }
    if (threadIdx.x == 0) {
        int n = 0;
        for (int z = 0; z < Z; ++z) {
            s_roff[z] = n;
            if (z0 + z < k.nz)
                for (int q = pl.slice_off[z0 + z]; q < pl.slice_off[z0 + z + 1]; ++q) s_rows[n++] = pl.slice_rows[q];
        }
        s_roff[Z] = n;
    }
    __syncthreads();
    if (s_roff[Z] == 0) return;  // no DMD row lies in these slices

    // PF: a two-stage software pipeline over this lane's rays -- the slot of ray
    // k + 2 and the records of ray k + 1 are loaded while ray k marches.  A lane's rays are list
    // entries gb + lane + q NT
    auto at = [&](int q) { return gb + (int)threadIdx.x + q * NT; };
    int qi = 0;
    int g = at(0);
    uint32_t e_n = 0, e_nn = 0;
    int ri_n = -1;
    float4 ff_n = make_float4(0.0f, 0.0f, 0.0f, 0.0f), an_n = ff_n;
    float w_n = 1.0f;
    auto records = [&](uint32_t e, int& ri, float4& ff, float4& an, float& wray) {
        const int al = (int)(e >> 16), colc = (int)(e & 0xffffu);
        ri = pl.rec_i[(size_t)al * k.crop_x + colc];
        ff = pl.rec_f[(size_t)al * k.crop_x + colc];
        wray = 1.0f;
        if (pl.rec_g) {  // refracted ray: its own direction (signed step times) and weight
            const float4 gg = pl.rec_g[(size_t)al * k.crop_x + colc];
            an = make_float4(fabsf(gg.x), fabsf(gg.y), gg.x < 0.0f ? -1.0f : 1.0f, gg.y < 0.0f ? -1.0f : 1.0f);
            wray = gg.z;
        } else {
            an = tp.ang[al];
        }
    };
    if (PF) {
        if (g < nrt) {
            e_n = slots[g];
            records(e_n, ri_n, ff_n, an_n, w_n);
        }
        if (at(1) < nrt) e_nn = slots[at(1)];
    }
    for (; g < nrt; g = at(++qi)) {
        uint32_t e;
        int ri;
        float4 ff, an;
        float wray;
        if (PF) {
            e = e_n;
            ri = ri_n;
            ff = ff_n;
            an = an_n;
            wray = w_n;
            if (at(qi + 1) < nrt) {
                e_n = e_nn;
                records(e_n, ri_n, ff_n, an_n, w_n);
            }
            if (at(qi + 2) < nrt) e_nn = slots[at(qi + 2)];
        } else {
            e = slots[g];
            records(e, ri, ff, an, wray);
        }
        const int al = (int)(e >> 16), colc = (int)(e & 0xffffu);
        if (ri < 0) continue;  // misses the vial / grid
        const int svx = ri & 0xffff, svy = ri >> 16;
        const int stx = (int)an.z, sty = (int)an.w;
        float tin0, tout0, tin1, tout1;
        int nin0, nout0, nin1, nout1;
        tvam_axis_window(svx, stx, ff.z, an.x, x0, x1, tin0, tout0, nin0, nout0);
        tvam_axis_window(svy, sty, ff.w, an.y, y0, y1, tin1, tout1, nin1, nout1);
        const float tau_e = fmaxf(fmaxf(tin0, tin1), 0.0f);
        const float tau_x = fminf(fminf(tout0, tout1), ff.y);
        if (!(tau_e < tau_x)) continue;
        const int n0 = tvam_axis_steps(tau_e, ff.z, an.x, nin0, nout0);
        const int n1 = tvam_axis_steps(tau_e, ff.w, an.y, nin1, nout1);
        const int vx = svx + stx * n0, vy = svy + sty * n1;
        float Tx = ff.z < TVAM_INF ? fmaxf(fmaf((float)n0, an.x, ff.z) - tau_e, 0.0f) : TVAM_INF;
        float Ty = ff.w < TVAM_INF ? fmaxf(fmaf((float)n1, an.y, ff.w) - tau_e, 0.0f) : TVAM_INF;
        const float rem = tau_x - tau_e, stop = rem - 1e-6f;
        const float nt0 = k.nsig2 * (ff.x + tau_e);
        constexpr int VB = PL ? 16 : Z * 4;  // bytes per voxel in one read's plane
        const int sxb = stx * VB, syb = sty * tw * VB;
        const int qstride = PL ? nvox * 16 : 16;  // bytes between a voxel's 4-slice groups
        const char* pv = reinterpret_cast<const char*>(tile) + (size_t)((vy - y0 + 1) * tw + (vx - x0 + 1)) * VB;
        float acc[Z];
#pragma unroll
        for (int z = 0; z < Z; ++z) acc[z] = 0.0f;
        // e0 = e^{-st t} (W2: st e^{-st t}, see TVAM_W2_MAX), restarted from exp2 at every tile entry
        float e0 = W2 ? k.sig_t * pl_exp2(nt0) : pl_exp2(nt0), tp = 0.0f;
        const float mhs = -0.5f * k.sig_t, msig = -k.sig_t;
        // one march, Z gathers per visit (see tvam_march in tvam_kernels.hip)
        for (;;) {
            const float tn = fminf(fminf(Tx, Ty), rem);
            const float dt = fmaxf(tn - tp, 0.0f);
            const float cw = W2 ? e0 * dt * fmaf(mhs, dt, 1.0f) : e0 * tvam_omexp(k.sig_t * dt);
            const float e1 = W2 ? fmaf(msig, cw, e0) : e0 - cw;
            tp = tn;
#pragma unroll
            for (int z4 = 0; z4 < Z / 4; ++z4) {
                const float4 gv = *reinterpret_cast<const float4*>(pv + z4 * qstride);
                acc[4 * z4 + 0] = fmaf(cw, gv.x, acc[4 * z4 + 0]);
                acc[4 * z4 + 1] = fmaf(cw, gv.y, acc[4 * z4 + 1]);
                acc[4 * z4 + 2] = fmaf(cw, gv.z, acc[4 * z4 + 2]);
                acc[4 * z4 + 3] = fmaf(cw, gv.w, acc[4 * z4 + 3]);
            }
            const bool mx = Tx <= Ty;
            Tx = mx ? Tx + an.x : Tx;
            Ty = mx ? Ty : Ty + an.y;
            pv += mx ? sxb : syb;
            e0 = e1;
            if (!(tn < stop)) break;
        }
        const int64_t base = (int64_t)(k.a0 + al) * k.crop_y * k.crop_x + colc - k.shard_base;
#pragma unroll
        for (int z = 0; z < Z; ++z) {
            const float v = acc[z] * (k.wscale * wray);
            for (int q = s_roff[z]; q < s_roff[z + 1]; ++q) {
                int64_t act = base + (int64_t)s_rows[q] * k.crop_x;
                if (idxmap) {
                    act = idxmap[act];
                    if (act < 0) continue;
                }
                atomicAdd(&out[act], v);  // backward_from(Le * em_grad), volume.py:274-276
            }
        }
    }
}

size_t tvam_planar_adj_lds(const TvamPlanar& pl, const TvamTiles& t, int Z) {
    return (size_t)pl.adj_pitch * (t.tsy + 2) * Z * sizeof(float) +
           (size_t)(Z + 1 + pl.max_rows_chunk) * sizeof(int);
}

hipError_t tvam_launch_adj_planar(const TvamConsts& k, const TvamPlanar& pl, const TvamTiles& t, int Z,
                                  const int32_t* idxmap, const float* gin, float* out, hipStream_t stream) {
    if (pl.adjl_ngroups > 0) return tvam_launch_adj_lists(k, pl, t, Z, idxmap, gin, out, stream);
    // slice chunks of this launch: [adj_zc0, adj_zc0 + adj_nzc) (tvam_adjoint_slices), else all
    const int nzc = pl.adj_nzc > 0 ? pl.adj_nzc : (k.nz + Z - 1) / Z;
    dim3 grid((unsigned)(t.ntx * t.nty), (unsigned)nzc, (unsigned)std::max(pl.adj_split, 1));
    const size_t lds = tvam_planar_adj_lds(pl, t, Z);
    const bool w2 = k.vox_chord < TVAM_W2_MAX;
    // Z = 8 (the list adjoint's fallback): 1024-thread workgroups, [z/4][voxel][4] planes; films
    // under 8 slices: Z = 4, 512 threads
    if (Z == 8 && pl.adj_nt == 1024 && w2)
        hipLaunchKernelGGL((tvam_adj_planar_kernel<8, true, 1024, true, true>), grid, dim3(1024), lds, stream, k, pl, t,
                           idxmap, gin, out);
    else if (Z == 8 && pl.adj_nt == 1024)
        hipLaunchKernelGGL((tvam_adj_planar_kernel<8, true, 1024, true, false>), grid, dim3(1024), lds, stream, k, pl, t,
                           idxmap, gin, out);
    else if (Z == 8)
        hipLaunchKernelGGL((tvam_adj_planar_kernel<8, true, 512, true, false>), grid, dim3(512), lds, stream, k, pl, t,
                           idxmap, gin, out);
    else if (Z == 4)
        hipLaunchKernelGGL((tvam_adj_planar_kernel<4, true, 512, false, false>), grid, dim3(512), lds, stream, k, pl, t,
                           idxmap, gin, out);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Forward, ray-driven with Z-slice sharing: the adjoint's march with its
// gathers turned into LDS adds.  Serves the planar scenes the voxel-driven
// forward cannot: refracted rays (cylindrical vial: not parallel) and DMDs
// finer than the voxels.  Per visit, Z adds of cw * E[z], E[z] = the sum of
// the slice's rows' pattern values (every row of a slice shares the ray's xy
// path).  The LDS dose tile is slice-major ([z][voxel], plane pitch padded):
// a wave's Z adds then hit Z planes with the lanes' voxels spread over the
// banks (the adjoint's [voxel][z] interleave would put every 4th voxel on one
// bank).  Fixed point (ds_add_u32, exact and order-independent) with the
// call's scale 2^e from tvam_fwd_scale_kernel; float adds when that bound is
// not finite.
// ---------------------------------------------------------------------------

// Per-angle max |pattern| of the shard (bits of non-negative floats order like
// the floats): grid (chunks, angles).
__global__ __launch_bounds__(256) void tvam_pattern_amax_kernel(int64_t per_angle, const float* __restrict__ pat,
                                                               unsigned* __restrict__ amax) {
    __shared__ unsigned s_m[4];
    const int al = blockIdx.y;
    const float* pa = pat + (int64_t)al * per_angle;
    float m = 0.0f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < per_angle; i += (int64_t)gridDim.x * 256)
        m = fmaxf(m, fabsf(pa[i]));
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_down(m, off, 64));
    if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = __float_as_uint(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned v = max(max(s_m[0], s_m[1]), max(s_m[2], s_m[3]));
        if (v) atomicMax(&amax[al], v);
    }
}

// scale[0] = 2^e with |voxel sum| < 2^30 / 2^e guaranteed, scale[1] = 1
// (fixed point) or 0 (float adds).  Bound as in tvam_tile_kernel: per angle at
// most rays_per_voxel / ns lines cross a voxel (rays_per_voxel includes the
// refracting vial's beam compression and interface weight), each adding at
// most vox_chord * rows * max|em|.  Deterministic: fixed-order sum.
__global__ __launch_bounds__(256) void tvam_fwd_scale_kernel(TvamConsts k, int ns, int rows,
                                                            const unsigned* __restrict__ amax,
                                                            float* __restrict__ scale) {
    __shared__ float s_sum[256];
    float a = 0.0f;
    for (int i = threadIdx.x; i < ns; i += 256) a += __uint_as_float(amax[i]);
    s_sum[threadIdx.x] = a;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) s_sum[threadIdx.x] += s_sum[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float sum = s_sum[0];
        const float bound = sum * fabsf(k.wscale) * k.vox_chord * (k.rays_per_voxel / (float)ns) * (float)rows;
        if (!(sum > 0.0f)) {
            scale[0] = 1.0f;
            scale[1] = 1.0f;
        } else if (isfinite(bound) && bound > 0.0f) {
            int e;
            frexpf(bound, &e);
            e = 30 - e;
            e = e > 126 ? 126 : (e < -126 ? -126 : e);
            scale[0] = ldexpf(1.0f, e);
            scale[1] = 1.0f;
        } else {
            scale[0] = 1.0f;
            scale[1] = 0.0f;
        }
    }
}

// LDS plane pitch (words) of the ray-driven forward's [z][voxel] tile: the
// (tile + guard) area rounded up to 32 words + 8 (planes start 8 banks apart).
static __host__ __device__ inline int tvam_ray_fwd_plane(int tw, int th) { return (tw * th + 31) / 32 * 32 + 8; }

size_t tvam_planar_rayfwd_lds(const TvamPlanar& pl, const TvamTiles& t, int Z) {
    return (size_t)tvam_ray_fwd_plane(pl.rayfwd_pitch, t.tsy + 2) * Z * sizeof(float) +
           (size_t)(Z + 1 + pl.max_rows_chunk) * sizeof(int);
}

__device__ __forceinline__ int pl_rint(float x) {
    int r;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

template <int Z, bool FIXED, bool W2>
__device__ __forceinline__ void fwd_rays_body(const TvamConsts& k, const TvamPlanar& pl, const TvamTiles& tp,
                                              const float* __restrict__ pat, float fscale, unsigned char* smem,
                                              const int* s_roff, const int* s_rows, int tile_id, int tw,
                                              int pstride, int x0, int x1, int y0, int y1) {
    float* tile = reinterpret_cast<float*>(smem);
    const uint32_t* slots = tp.slots + tp.slot_off[tile_id];
    const int nrt = (int)(tp.slot_off[tile_id + 1] - tp.slot_off[tile_id]);
    const int64_t per_angle = (int64_t)k.crop_y * k.crop_x;
    for (int g = threadIdx.x; g < nrt; g += (int)blockDim.x) {
        const uint32_t e = slots[g];
        const int al = (int)(e >> 16), colc = (int)(e & 0xffffu);
        const int ri = pl.rec_i[(size_t)al * k.crop_x + colc];
        if (ri < 0) continue;  // misses the vial / grid
        // the Z slices' pattern sums (volume.py:49: Le of every row's ray)
        const float* pc = pat + (int64_t)al * per_angle + colc;
        float em[Z];
        bool any = false;
#pragma unroll
        for (int z = 0; z < Z; ++z) {
            float v = 0.0f;
            for (int q = s_roff[z]; q < s_roff[z + 1]; ++q) v += pc[(int64_t)s_rows[q] * k.crop_x];
            em[z] = v;
            any |= v != 0.0f;
        }
        if (!any && k.skip_zero) continue;  // contributes exactly zero dose
        const float4 ff = pl.rec_f[(size_t)al * k.crop_x + colc];
        float4 an;
        float wray = 1.0f;
        if (pl.rec_g) {
            const float4 gg = pl.rec_g[(size_t)al * k.crop_x + colc];
            an = make_float4(fabsf(gg.x), fabsf(gg.y), gg.x < 0.0f ? -1.0f : 1.0f, gg.y < 0.0f ? -1.0f : 1.0f);
            wray = gg.z;
        } else {
            an = tp.ang[al];
        }
        const float sc = k.wscale * wray * fscale;  // weight (common.py:111) x interfaces (sensor.py:404)
#pragma unroll
        for (int z = 0; z < Z; ++z) em[z] *= sc;
        const int svx = ri & 0xffff, svy = ri >> 16;
        const int stx = (int)an.z, sty = (int)an.w;
        float tin0, tout0, tin1, tout1;
        int nin0, nout0, nin1, nout1;
        tvam_axis_window(svx, stx, ff.z, an.x, x0, x1, tin0, tout0, nin0, nout0);
        tvam_axis_window(svy, sty, ff.w, an.y, y0, y1, tin1, tout1, nin1, nout1);
        const float tau_e = fmaxf(fmaxf(tin0, tin1), 0.0f);
        const float tau_x = fminf(fminf(tout0, tout1), ff.y);
        if (!(tau_e < tau_x)) continue;
        const int n0 = tvam_axis_steps(tau_e, ff.z, an.x, nin0, nout0);
        const int n1 = tvam_axis_steps(tau_e, ff.w, an.y, nin1, nout1);
        const int vx = svx + stx * n0, vy = svy + sty * n1;
        float Tx = ff.z < TVAM_INF ? fmaxf(fmaf((float)n0, an.x, ff.z) - tau_e, 0.0f) : TVAM_INF;
        float Ty = ff.w < TVAM_INF ? fmaxf(fmaf((float)n1, an.y, ff.w) - tau_e, 0.0f) : TVAM_INF;
        const float rem = tau_x - tau_e, stop = rem - 1e-6f;
        const float nt0 = k.nsig2 * (ff.x + tau_e);
        const int sxb = stx * 4, syb = sty * tw * 4;
        char* pv = reinterpret_cast<char*>(tile) + (size_t)((vy - y0 + 1) * tw + (vx - x0 + 1)) * 4;
        float e0 = W2 ? k.sig_t * pl_exp2(nt0) : pl_exp2(nt0), tp = 0.0f;  // as in the planar adjoint
        const float mhs = -0.5f * k.sig_t, msig = -k.sig_t;
        for (;;) {
            const float tn = fminf(fminf(Tx, Ty), rem);
            const float dt = fmaxf(tn - tp, 0.0f);
            const float cw = W2 ? e0 * dt * fmaf(mhs, dt, 1.0f) : e0 * tvam_omexp(k.sig_t * dt);
            const float e1 = W2 ? fmaf(msig, cw, e0) : e0 - cw;
            tp = tn;
#pragma unroll
            for (int z = 0; z < Z; ++z) {
                if (FIXED)
                    __hip_atomic_fetch_add(reinterpret_cast<int*>(pv + z * pstride), pl_rint(cw * em[z]),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                else
                    __hip_atomic_fetch_add(reinterpret_cast<float*>(pv + z * pstride), cw * em[z], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            const bool mx = Tx <= Ty;
            Tx = mx ? Tx + an.x : Tx;
            Ty = mx ? Ty : Ty + an.y;
            pv += mx ? sxb : syb;
            e0 = e1;
            if (!(tn < stop)) break;
        }
    }
}

template <int Z, int NT>
__global__ __launch_bounds__(NT) void tvam_fwd_rays_planar_kernel(TvamConsts k, TvamPlanar pl, TvamTiles tp,
                                                                       const float* __restrict__ pat,
                                                                       const float* __restrict__ scale,
                                                                       float* __restrict__ dose) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tsx = tp.tsx, tsy = tp.tsy;
    const int tw = pl.rayfwd_pitch, th = tsy + 2;
    const int pw = tvam_ray_fwd_plane(tw, th);  // plane pitch in words
    int* itile = reinterpret_cast<int*>(smem);
    int* s_roff = itile + (size_t)pw * Z;
    int* s_rows = s_roff + Z + 1;

    const int tile_id = blockIdx.x, z0 = blockIdx.y * Z;
    const int x0 = (tile_id % tp.ntx) * tsx, y0 = (tile_id / tp.ntx) * tsy;
    const int x1 = min(x0 + tsx, k.res[0]), y1 = min(y0 + tsy, k.res[1]);
    const int wx = x1 - x0, wy = y1 - y0;
    const size_t plane = (size_t)k.res[0] * k.res[1];
    const float fscale = scale[0];
    const bool fixed = scale[1] != 0.0f;

    for (int i = threadIdx.x; i < pw * Z; i += (int)blockDim.x) itile[i] = 0;  // 0 == 0.0f
    if (threadIdx.x == 0) {
        int n = 0;
        for (int z = 0; z < Z; ++z) {
            s_roff[z] = n;
            if (z0 + z < k.nz)
                for (int q = pl.slice_off[z0 + z]; q < pl.slice_off[z0 + z + 1]; ++q) s_rows[n++] = pl.slice_rows[q];
        }
        s_roff[Z] = n;
    }
    __syncthreads();
    if (s_roff[Z] > 0) {
        const bool w2 = k.vox_chord < TVAM_W2_MAX;
        if (fixed && w2)
            fwd_rays_body<Z, true, true>(k, pl, tp, pat, fscale, smem, s_roff, s_rows, tile_id, tw, pw * 4, x0, x1, y0, y1);
        else if (fixed)
            fwd_rays_body<Z, true, false>(k, pl, tp, pat, fscale, smem, s_roff, s_rows, tile_id, tw, pw * 4, x0, x1, y0, y1);
        else
            fwd_rays_body<Z, false, false>(k, pl, tp, pat, fscale, smem, s_roff, s_rows, tile_id, tw, pw * 4, x0, x1, y0, y1);
    }
    __syncthreads();
    // dose = sum / voxel volume (volume.py:41-42, sensor.py:404)
    const float outscale = k.inv_vol / fscale;
    const float* ftile = reinterpret_cast<const float*>(smem);
    for (int z = 0; z < Z && z0 + z < k.nz; ++z)
        for (int i = threadIdx.x; i < wx * wy; i += (int)blockDim.x) {
            const int ly = i / wx, lx = i - ly * wx;
            const size_t li = (size_t)z * pw + (size_t)(ly + 1) * tw + (lx + 1);
            const float v = fixed ? (float)itile[li] * outscale : ftile[li] * k.inv_vol;
            dose[(size_t)(z0 + z) * plane + (size_t)(y0 + ly) * k.res[0] + (x0 + lx)] = v;
        }
}

hipError_t tvam_launch_fwd_rays_planar(const TvamConsts& k, const TvamPlanar& pl, const TvamTiles& t, int Z,
                                       const float* pat, unsigned* amax, float* scale, float* dose,
                                       hipStream_t stream) {
    const int64_t per_angle = (int64_t)k.crop_y * k.crop_x;
    hipError_t e = hipMemsetAsync(amax, 0, (size_t)pl.ns * sizeof(unsigned), stream);
    if (e != hipSuccess) return e;
    const unsigned chunks = (unsigned)std::min<int64_t>((per_angle + 4095) / 4096, 64);
    hipLaunchKernelGGL(tvam_pattern_amax_kernel, dim3(chunks, (unsigned)pl.ns), dim3(256), 0, stream, per_angle, pat,
                       amax);
    hipLaunchKernelGGL(tvam_fwd_scale_kernel, dim3(1), dim3(256), 0, stream, k, pl.ns, pl.max_rows_slice, amax, scale);
    dim3 grid((unsigned)(t.ntx * t.nty), (unsigned)((k.nz + Z - 1) / Z));
    const size_t lds = tvam_planar_rayfwd_lds(pl, t, Z);
#define TVAM_RAYFWD_LAUNCH(ZZ)                                                                                  \
    if (pl.rayfwd_nt == 1024)                                                                                   \
        hipLaunchKernelGGL((tvam_fwd_rays_planar_kernel<ZZ, 1024>), grid, dim3(1024), lds, stream, k, pl, t, pat, \
                           scale, dose);                                                                        \
    else                                                                                                        \
        hipLaunchKernelGGL((tvam_fwd_rays_planar_kernel<ZZ, 512>), grid, dim3(512), lds, stream, k, pl, t, pat,   \
                           scale, dose);
    switch (Z) {
        case 4: TVAM_RAYFWD_LAUNCH(4) break;
        case 8: TVAM_RAYFWD_LAUNCH(8) break;
        default: return hipErrorInvalidValue;
    }
#undef TVAM_RAYFWD_LAUNCH
    return hipGetLastError();
}
