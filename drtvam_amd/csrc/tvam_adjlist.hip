// tvam_adjlist.hip — planar adjoint over slice-invariant visit lists.
//
// Under regular sampling a ray (angle, DMD column) of a planar scene takes the same xy path
// through every z-slice (tvam_planar.hip), so the visits of its in-tile chord -- the voxel
// sequence and the weights e^{-st t} (1 - e^{-st dt}) of sensor.py:383-438 -- are the same for
// all 400 slices.  The tile adjoint of tvam_planar.hip re-derives them (closed-form resume,
// crossing times, weight recurrence: 21 VALU per visit) once per (ray, tile, chunk of 8 slices),
// i.e. 50 times per visit on a 400-slice film.  Here the plan marches every (ray, tile) once,
// with the same fp32 expressions, and stores the weights; the adjoint then streams them:
// per visit one weight (a quarter of a coalesced 16-byte load), four ds_read_b128 of the 16
// slices' gradient (two of 8 where a 16-slice tile does not fit in LDS) and eight v_pk_fma.
//
// Layout (TvamPlanar::adjl_*):
//   * group = (xy tile, part): the tile's crossing rays split into adj_split parts, as the
//     tile adjoint's gridDim.z; its rays in chunks of 64, one chunk per wave at a time;
//   * hdr[chunk][lane] = {LDS byte offset of the entry voxel's 16-byte chunk in plane 0, slot
//     (angle << 16 | column, 0xffffffff: empty lane), interface weight bits, x step | y step << 16
//     in LDS bytes};
//   * w[coff[chunk] + q][lane] = float4 of visits 4q .. 4q + 3 of the lane's ray, padded with 0 to
//     the chunk's longest ray; the lowest mantissa bit of a weight says which axis the march
//     steps after the visit (0: x, 1: y) -- a relative change of at most 2^-23 of that weight.
// A workgroup = (group, 16-slice chunk); the workgroups of one group are dispatched to one XCD
// back to back (blockIdx -> (group, chunk) below), so the group's weights (~2 MB on config 2)
// are read from HBM once and from that XCD's L2 by the other chunks.
#include "tvam_internal.h"

#include <algorithm>
#include <numeric>

__device__ __forceinline__ float al_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// The tile adjoint's per-(ray, tile) march (tvam_planar.hip, tvam_adj_planar_kernel), the
// same fp32 expressions in the same order: visit(index, cw, ystep) per visit.  Returns the visit
// count (0: the ray misses the vial or this tile); pv0 = byte offset of the entry voxel's 16-byte
// chunk in a plane of row pitch tw0 / tw1 (by the ray's step quadrant qd), dxy = the x and y steps
// in bytes.
template <bool W2, typename V>
__device__ __forceinline__ int adjl_march(const TvamConsts& k, const TvamPlanar& pl, const TvamTiles& tp, uint32_t e,
                                          int x0, int x1, int y0, int y1, int tw0, int tw1, int& pv0, float& wray,
                                          int& dxy, int& qd, V&& visit) {
    const int al = (int)(e >> 16), colc = (int)(e & 0xffffu);
    const int ri = pl.rec_i[(size_t)al * k.crop_x + colc];
    const float4 ff = pl.rec_f[(size_t)al * k.crop_x + colc];
    float4 an;
    wray = 1.0f;
    if (pl.rec_g) {  // refracted ray: its own direction (signed step times) and weight
        const float4 gg = pl.rec_g[(size_t)al * k.crop_x + colc];
        an = make_float4(fabsf(gg.x), fabsf(gg.y), gg.x < 0.0f ? -1.0f : 1.0f, gg.y < 0.0f ? -1.0f : 1.0f);
        wray = gg.z;
    } else {
        an = tp.ang[al];
    }
    const int stx = (int)an.z, sty = (int)an.w;
    qd = (stx < 0 ? 2 : 0) + (sty < 0 ? 1 : 0);  // step quadrant: row pitch tw0 (equal signs) or tw1
    const int tw = qd == 0 || qd == 3 ? tw0 : tw1;
    if (ri < 0) return 0;  // misses the vial / grid
    const int svx = ri & 0xffff, svy = ri >> 16;
    float tin0, tout0, tin1, tout1;
    int nin0, nout0, nin1, nout1;
    tvam_axis_window(svx, stx, ff.z, an.x, x0, x1, tin0, tout0, nin0, nout0);
    tvam_axis_window(svy, sty, ff.w, an.y, y0, y1, tin1, tout1, nin1, nout1);
    const float tau_e = fmaxf(fmaxf(tin0, tin1), 0.0f);
    const float tau_x = fminf(fminf(tout0, tout1), ff.y);
    if (!(tau_e < tau_x)) return 0;
    const int n0 = tvam_axis_steps(tau_e, ff.z, an.x, nin0, nout0);
    const int n1 = tvam_axis_steps(tau_e, ff.w, an.y, nin1, nout1);
    const int vx = svx + stx * n0, vy = svy + sty * n1;
    float Tx = ff.z < TVAM_INF ? fmaxf(fmaf((float)n0, an.x, ff.z) - tau_e, 0.0f) : TVAM_INF;
    float Ty = ff.w < TVAM_INF ? fmaxf(fmaf((float)n1, an.y, ff.w) - tau_e, 0.0f) : TVAM_INF;
    const float rem = tau_x - tau_e, stop = rem - 1e-6f;
    const float nt0 = k.nsig2 * (ff.x + tau_e);
    pv0 = ((vy - y0 + 1) * tw + (vx - x0 + 1)) * 16;
    dxy = (int)(((uint32_t)(stx * 16) & 0xffffu) | ((uint32_t)(sty * tw * 16) << 16));
    float e0 = W2 ? k.sig_t * al_exp2(nt0) : al_exp2(nt0), tp0 = 0.0f;
    const float mhs = -0.5f * k.sig_t, msig = -k.sig_t;
    int n = 0;
    for (;;) {
        const float tn = fminf(fminf(Tx, Ty), rem);
        const float dt = fmaxf(tn - tp0, 0.0f);
        const float cw = W2 ? e0 * dt * fmaf(mhs, dt, 1.0f) : e0 * tvam_omexp(k.sig_t * dt);
        const float e1 = W2 ? fmaf(msig, cw, e0) : e0 - cw;
        tp0 = tn;
        const bool mx = Tx <= Ty;
        Tx = mx ? Tx + an.x : Tx;
        Ty = mx ? Ty : Ty + an.y;
        visit(n, cw, !mx);
        ++n;
        e0 = e1;
        if (!(tn < stop)) break;
    }
    return n;
}


__device__ __forceinline__ void adjl_tile_bounds(const TvamConsts& k, const TvamTiles& tp, int tile, int& x0, int& x1,
                                                 int& y0, int& y1) {
    x0 = (tile % tp.ntx) * tp.tsx;
    y0 = (tile / tp.ntx) * tp.tsy;
    x1 = min(x0 + tp.tsx, k.res[0]);
    y1 = min(y0 + tp.tsy, k.res[1]);
}

// Visits, step quadrant and entry voxel of every (slot, tile): grid (slot blocks, tiles);
// ent = quadrant << 24 | entry voxel (plane chunk index).
template <bool W2>
__global__ __launch_bounds__(256) void tvam_adjl_count_kernel(TvamConsts k, TvamPlanar pl, TvamTiles tp,
                                                              uint32_t* __restrict__ cnt, uint32_t* __restrict__ ent) {
    const int tile = blockIdx.y;
    const int64_t j = tp.slot_off[tile] + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= tp.slot_off[tile + 1]) return;
    int x0, x1, y0, y1;
    adjl_tile_bounds(k, tp, tile, x0, x1, y0, y1);
    int pv0 = 0, dxy, qd = 0;
    float wray;
    cnt[j] = (uint32_t)adjl_march<W2>(k, pl, tp, tp.slots[j], x0, x1, y0, y1, pl.adjl_tw0, pl.adjl_tw1, pv0, wray,
                                      dxy, qd, [](int, float, bool) {});
    ent[j] = (uint32_t)qd << 24 | (uint32_t)(pv0 >> 4);
}

// Headers and weights of every chunk lane: grid (chunks * 64 / 256).  cslot: the lane's slot |
// start delay << 27 (the lane walks `delay` weight-0 x steps before its entry voxel, which sets its
// 16-byte chunk residue at every later step), or -1 - r for an empty lane (it walks from plane chunk
// r, a residue its lane group leaves free); cgrp: the chunk's (tile, quadrant) = tile * 4 + quadrant.
template <bool W2>
__global__ __launch_bounds__(256) void tvam_adjl_fill_kernel(TvamConsts k, TvamPlanar pl, TvamTiles tp, int64_t nchunks,
                                                             const int32_t* __restrict__ cslot,
                                                             const int32_t* __restrict__ cgrp, int4* __restrict__ hdr,
                                                             float4* __restrict__ w) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nchunks * 64) return;
    const int64_t c = i >> 6;
    const int lane = (int)(i & 63);
    const int64_t r0 = pl.adjl_coff[c], n4 = pl.adjl_coff[c + 1] - r0;
    float* wl = reinterpret_cast<float*>(w + r0 * 64 + lane);  // visit v at wl[(v / 4) * 256 + v % 4]
    const int32_t cs = cslot[i];
    const int tq = cgrp[c], qd = tq & 3;
    int n = 0, pv0, dxy, q2 = qd, dl = 0;
    float wray = 0.0f;
    uint32_t e = 0xffffffffu;
    if (cs >= 0) {
        const int32_t j = cs & ((1 << 27) - 1);
        dl = cs >> 27;
        int x0, x1, y0, y1;
        adjl_tile_bounds(k, tp, tq >> 2, x0, x1, y0, y1);
        e = tp.slots[j];
        n = adjl_march<W2>(k, pl, tp, e, x0, x1, y0, y1, pl.adjl_tw0, pl.adjl_tw1, pv0, wray, dxy, q2,
                           [&](int v, float cw, bool ys) {
                               uint32_t b = __float_as_uint(cw);
                               b = (b & ~1u) | (ys ? 1u : 0u);
                               v += dl;
                               if ((int64_t)(v >> 2) < n4) wl[(size_t)(v >> 2) * 256 + (v & 3)] = __uint_as_float(b);
                           });
        pv0 -= dl * (int)(short)(dxy & 0xffff);
    } else {  // empty lane: x steps (the quadrant's sign) from its free residue, weight 0
        pv0 = (-1 - cs) * 16;
        dxy = (qd & 2) ? 0xfff0 : 16;
    }
    // the delay's and the padding's visits: weight 0, x steps (the lane's chunk keeps moving with
    // its lane group's)
    for (int v = 0; v < dl; ++v) wl[(size_t)(v >> 2) * 256 + (v & 3)] = 0.0f;
    for (int v = dl + n; v < n4 * 4; ++v) wl[(size_t)(v >> 2) * 256 + (v & 3)] = 0.0f;
    hdr[i] = make_int4(pv0, (int)e, __float_as_int(wray), dxy);
}

// The adjoint: one workgroup per (group, chunk of Z slices), NT threads, waves take the group's
// chunks round robin.  The gradient tile is [z/4][voxel][4] (planes of 16-byte chunks, 1-voxel
// guard band) scaled by 1/voxel volume (volume.py:130), as in the tile adjoint, with the row pitch
// of the group's step quadrant: +1 (mod 16) where the x and y steps have equal signs, -1 (mod 16)
// where they differ, so that every visit -- an x or a y step -- moves a lane's 16-byte chunk by
// the same +-1 and the lanes of a ds_read_b128 lane group keep the distinct chunks (mod 16) they
// entered with: no bank conflicts.  Padding visits keep stepping in x through zeroed slack
// (adjl_slack bytes) before, between and after the two planes.
template <int Z, int NT, int MINW = 1, int PFD = 4>
__global__ __launch_bounds__(NT, MINW) void tvam_adjl_kernel(TvamConsts k, TvamPlanar pl, TvamTiles tp, int nzc,
                                                       const int32_t* __restrict__ idxmap,
                                                       const float* __restrict__ gin, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // blockIdx -> (group, slice chunk): workgroup b runs on XCD b % 8; XCD x takes the listed
    // groups x, x + 8, ..., each over all its slice chunks back to back (its weights stay in that
    // XCD's L2).  Only groups that hold chunks are listed: an angle shard's rays fall in one or two
    // step quadrants, and with every group in the grid the XCDs of the empty quadrants idled
    // (groups 4 t + q land on XCDs q and q + 4).
    const int b = (int)blockIdx.x, xcd = b & 7, ib = b >> 3;
    const int gq = ib / nzc, zc = ib - gq * nzc;
    const int gi = xcd + 8 * gq;
    if (gi >= pl.adjl_nlist) return;
    const int grp = pl.adjl_glist[gi];
    const int c0 = pl.adjl_gchunk[grp], c1 = pl.adjl_gchunk[grp + 1];
    if (c0 >= c1) return;
    const int tq = grp / pl.adjl_parts, tile_id = tq >> 2, qd = tq & 3;
    const int z0 = (zc + pl.adj_zc0) * Z;
    const int tw = qd == 0 || qd == 3 ? pl.adjl_tw0 : pl.adjl_tw1, th = tp.tsy + 2;
    const int nvox = tw * th, S = pl.adjl_slack;
    const int P = nvox * 16 + S;  // plane stride in bytes
    char* tb = reinterpret_cast<char*>(smem) + S;  // plane 0
    int* s_roff = reinterpret_cast<int*>(tb + (size_t)P * (Z / 4));
    int* s_rows = s_roff + Z + 1;
    int* s_next = s_rows + pl.max_rows_chunk * ((Z + 7) / 8);  // the group's next unclaimed chunk
    int x0, x1, y0, y1;
    adjl_tile_bounds(k, tp, tile_id, x0, x1, y0, y1);
    const int wx = x1 - x0, wy = y1 - y0;
    const size_t plane = (size_t)k.res[0] * k.res[1];
    // gradient tile: a thread per voxel, its Z loads issued together (clamped addresses, no
    // branches), Z / 4 ds_write_b128
    int nonzero = 0;
    for (int li = threadIdx.x; li < nvox; li += NT) {
        const int ly = li / tw - 1, lx = li - (ly + 1) * tw - 1;
        const bool in = lx >= 0 && ly >= 0 && lx < wx && ly < wy;
        const int gx = min(max(x0 + lx, 0), k.res[0] - 1), gy = min(max(y0 + ly, 0), k.res[1] - 1);
        const float* src = gin + (size_t)gy * k.res[0] + gx;
        float v[Z];
#pragma unroll
        for (int z = 0; z < Z; ++z) v[z] = src[(size_t)min(z0 + z, k.nz - 1) * plane];
#pragma unroll
        for (int z = 0; z < Z; ++z) v[z] = in && z0 + z < k.nz ? v[z] * k.inv_vol : 0.0f;
#pragma unroll
        for (int z = 0; z < Z; ++z) nonzero |= v[z] != 0.0f ? 1 : 0;
#pragma unroll
        for (int q = 0; q < Z / 4; ++q)
            *reinterpret_cast<float4*>(tb + (size_t)q * P + (size_t)li * 16) =
                make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    }
    // zeroed slack: [-S, 0) of every plane and S after the last
    for (int i = threadIdx.x; i < (Z / 4 + 1) * (S / 16); i += NT) {
        const int q = i / (S / 16), o = i - q * (S / 16);
        *reinterpret_cast<float4*>(tb + (size_t)q * P - S + (size_t)o * 16) = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    if (threadIdx.x == 0) {
        *s_next = c0 + NT / 64;  // wave w starts on chunk c0 + w
        int n = 0;
        for (int z = 0; z < Z; ++z) {
            s_roff[z] = n;
            if (z0 + z < k.nz)
                for (int q = pl.slice_off[z0 + z]; q < pl.slice_off[z0 + z + 1]; ++q) s_rows[n++] = pl.slice_rows[q];
        }
        s_roff[Z] = n;
    }
    // an all-zero gradient tile (the thresholded loss is flat wherever the dose meets its bounds)
    // makes every partial exactly 0, which adds nothing: no march
    const int any = __syncthreads_or(nonzero);
    if (s_roff[Z] == 0 || !any) return;  // (or no DMD row lies in these slices)

    const int lane = (int)threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform chunk loop
    // A wave claims the group's chunks one at a time from an LDS counter (the chunks differ in
    // length: a fixed round robin left a few waves marching while the workgroup held its CU; the
    // builder orders each group's chunks longest first).
    // Pipelined over the wave's chunks: a chunk's header and its first four weight rows are loaded
    // before the previous chunk's gradient atomics are issued.  A load's data waits for every older
    // vector-memory operation of the wave (atomics included, ~3000 cycles each under load), so the
    // march of the next chunk starts on rows that do not queue behind the atomics, and by the time
    // it needs row 4 (16 visits later) they have drained.
    int c = c0 + wv;
    if (c >= c1) return;
    int4 h;
    int n4;
    const float4* wp;
    float4 w[PFD];  // weight rows PFD ahead, a register ring
    auto load_chunk = [&](int cc) {
        h = pl.adjl_hdr[(size_t)cc * 64 + lane];
        const int64_t r0 = pl.adjl_coff[cc];
        n4 = (int)(pl.adjl_coff[cc + 1] - r0);  // >= 1: chunks hold crossing rays only
        wp = pl.adjl_w + r0 * 64 + lane;
        const int last = n4 - 1;
#pragma unroll
        for (int j = 0; j < PFD; ++j) w[j] = wp[(size_t)min(j, last) * 64];
    };
    load_chunk(c);
    for (;;) {
        int pv = h.x;
        const int dx = (int)(short)(h.w & 0xffff), ddy = (h.w >> 16) - dx;
        const uint32_t e = (uint32_t)h.y;
        const float wsc = k.wscale * __int_as_float(h.z);
        float acc[Z];
#pragma unroll
        for (int z = 0; z < Z; ++z) acc[z] = 0.0f;
        auto visits = [&](const float4 w4) {
            const float ws[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float cw = ws[u];
#pragma unroll
                for (int z4 = 0; z4 < Z / 4; ++z4) {
                    const float4 gv = *reinterpret_cast<const float4*>(tb + pv + z4 * P);
                    acc[4 * z4 + 0] = fmaf(cw, gv.x, acc[4 * z4 + 0]);
                    acc[4 * z4 + 1] = fmaf(cw, gv.y, acc[4 * z4 + 1]);
                    acc[4 * z4 + 2] = fmaf(cw, gv.z, acc[4 * z4 + 2]);
                    acc[4 * z4 + 3] = fmaf(cw, gv.w, acc[4 * z4 + 3]);
                }
                pv += dx + ((__float_as_int(cw) & 1) ? ddy : 0);
            }
        };
        const int last = n4 - 1;
        int q = 0;
#pragma unroll 1
        for (; q + PFD - 1 < n4; q += PFD) {
#pragma unroll
            for (int j = 0; j < PFD; ++j) {
                const float4 t = w[j];
                w[j] = wp[(size_t)min(q + PFD + j, last) * 64];
                visits(t);
            }
        }
#pragma unroll
        for (int j = 0; j < PFD - 1; ++j)
            if (q + j < n4) visits(w[j]);
#pragma unroll
        for (int z = 0; z < Z; ++z) acc[z] *= wsc;
        const int cn = __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(s_next, 1) : 0);
        if (cn < c1) load_chunk(cn);  // before this chunk's atomics
        if (e != 0xffffffffu) {  // (empty lanes add nothing)
            const int al = (int)(e >> 16), colc = (int)(e & 0xffffu);
            const int64_t base = (int64_t)(k.a0 + al) * k.crop_y * k.crop_x + colc - k.shard_base;
            // a partial of exactly 0 (every visited gradient voxel 0: the thresholded loss is flat
            // wherever the dose meets its bounds) adds nothing: no atomic for it
#pragma unroll
            for (int z = 0; z < Z; ++z) {
                if (acc[z] == 0.0f) continue;
                for (int q2 = s_roff[z]; q2 < s_roff[z + 1]; ++q2) {
                    int64_t act = base + (int64_t)s_rows[q2] * k.crop_x;
                    if (idxmap) {
                        act = idxmap[act];
                        if (act < 0) continue;
                    }
                    atomicAdd(&out[act], acc[z]);  // backward_from(Le * em_grad), volume.py:274-276
                }
            }
        }
        if (cn >= c1) break;
        c = cn;
    }
}

size_t tvam_adjl_lds(const TvamPlanar& pl, const TvamTiles& t, int Z) {
    const int tw = std::max(pl.adjl_tw0, pl.adjl_tw1);
    return (size_t)(Z / 4) * ((size_t)tw * (t.tsy + 2) * 16 + pl.adjl_slack) + pl.adjl_slack +
           (size_t)(Z + 2 + pl.max_rows_chunk * ((Z + 7) / 8)) * sizeof(int);
}

hipError_t tvam_launch_adj_lists(const TvamConsts& k, const TvamPlanar& pl, const TvamTiles& t, int Z,
                                 const int32_t* idxmap, const float* gin, float* out, hipStream_t stream) {
    // slice chunks of this launch in units of the plan's adjoint chunk Z (tvam_adjoint_slices)
    const int ZL = pl.adjl_z;
    if (ZL != 8 && ZL != 16) return hipErrorInvalidValue;
    TvamPlanar q = pl;
    if (pl.adj_nzc > 0) {
        const int z0 = pl.adj_zc0 * Z, z1 = std::min(k.nz, (pl.adj_zc0 + pl.adj_nzc) * Z);
        if (z0 % ZL) return hipErrorInvalidValue;
        q.adj_zc0 = z0 / ZL;
        q.adj_nzc = (z1 - z0 + ZL - 1) / ZL;
    }
    const int nzc = q.adj_nzc > 0 ? q.adj_nzc : (k.nz + ZL - 1) / ZL;
    const int64_t gpad = ((int64_t)pl.adjl_nlist + 7) / 8 * 8;
    const int64_t nb = gpad * nzc;
    if (nb <= 0) return hipSuccess;
    if (nb > 0x7fffffff) return hipErrorInvalidValue;
    const size_t lds = tvam_adjl_lds(pl, t, ZL);
    if (ZL == 16)  // one workgroup per CU: registers to spare for 8 weight rows in flight
        hipLaunchKernelGGL((tvam_adjl_kernel<16, 1024, 1, 8>), dim3((unsigned)nb), dim3(1024), lds, stream, k, q, t, nzc,
                           idxmap, gin, out);
    else  // two 768-thread workgroups (6 waves per SIMD) per CU at <= 80 VGPRs
        hipLaunchKernelGGL((tvam_adjl_kernel<8, 768, 6>), dim3((unsigned)nb), dim3(768), lds, stream, k, q, t, nzc, idxmap,
                           gin, out);
    return hipGetLastError();
}

// Plan creation.  Per (tile, step quadrant): the tile's crossing rays in slot order (angle, then
// column), in chunks of 64 consecutive rays (their gradient atomics stay coalesced); within a
// chunk each ds_read_b128 lane group ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, + 32) is dealt
// rays of distinct entry chunks mod 16 first, and its empty lanes the residues it leaves free.
// The (tile, quadrant) chunk lists are split into `parts` groups.  Owned buffers come back in
// `bufs` (freed with the plan); hipErrorOutOfMemory when the lists would exceed `max_bytes`
// (the plan then keeps the tile adjoint).
hipError_t tvam_build_adj_lists(const TvamConsts& k, TvamPlanar& pl, const TvamTiles& t, int parts, size_t max_bytes,
                                TvamAdjListBufs& bufs, hipStream_t stream) {
    const int ntiles = t.ntx * t.nty;
    const bool w2 = k.vox_chord < TVAM_W2_MAX;  // the tile adjoint's weight form (tvam_launch_adj_planar)
    const int w = t.tsx + 2;
    pl.adjl_tw0 = w + ((1 - w) % 16 + 16) % 16;   // = 1 (mod 16)
    pl.adjl_tw1 = w + ((15 - w) % 16 + 16) % 16;  // = 15 (mod 16)
    std::vector<int64_t> off((size_t)ntiles + 1);
    hipError_t e;
    if ((e = hipMemcpy(off.data(), t.slot_off, off.size() * sizeof(int64_t), hipMemcpyDeviceToHost)) != hipSuccess)
        return e;
    const int64_t nslots = off[(size_t)ntiles];
    uint32_t *d_cnt = nullptr, *d_ent = nullptr;
    if ((e = hipMalloc((void**)&d_cnt, (size_t)std::max<int64_t>(nslots, 1) * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc((void**)&d_ent, (size_t)std::max<int64_t>(nslots, 1) * sizeof(uint32_t))) != hipSuccess) {
        (void)hipFree(d_cnt);
        return e;
    }
    int64_t maxn = 0;
    for (int i = 0; i < ntiles; ++i) maxn = std::max(maxn, off[(size_t)i + 1] - off[(size_t)i]);
    if (maxn > 0) {
        dim3 grid((unsigned)((maxn + 255) / 256), (unsigned)ntiles);
        if (w2)
            hipLaunchKernelGGL((tvam_adjl_count_kernel<true>), grid, dim3(256), 0, stream, k, pl, t, d_cnt, d_ent);
        else
            hipLaunchKernelGGL((tvam_adjl_count_kernel<false>), grid, dim3(256), 0, stream, k, pl, t, d_cnt, d_ent);
    }
    std::vector<uint32_t> cnt((size_t)nslots), ent((size_t)nslots);
    if ((e = hipGetLastError()) == hipSuccess) e = hipStreamSynchronize(stream);
    if (e == hipSuccess && nslots > 0 &&
        ((e = hipMemcpy(cnt.data(), d_cnt, cnt.size() * sizeof(uint32_t), hipMemcpyDeviceToHost)) != hipSuccess ||
         (e = hipMemcpy(ent.data(), d_ent, ent.size() * sizeof(uint32_t), hipMemcpyDeviceToHost)) != hipSuccess)) {
    }
    (void)hipFree(d_cnt);
    (void)hipFree(d_ent);
    if (e != hipSuccess) return e;
    static const int LG[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                  {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                  {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                  {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
    std::vector<int32_t> gchunk, cslot, cgrp;
    std::vector<int64_t> coff(1, 0);
    std::vector<int64_t> q[4];
    int64_t maxlen = 0;
    for (int tile = 0; tile < ntiles; ++tile) {
        for (auto& v : q) v.clear();
        for (int64_t j = off[(size_t)tile]; j < off[(size_t)tile + 1]; ++j)
            if (cnt[(size_t)j] > 0) q[ent[(size_t)j] >> 24].push_back(j);
        for (int qd = 0; qd < 4; ++qd) {
            const std::vector<int64_t>& v = q[qd];
            const int64_t nch = ((int64_t)v.size() + 63) / 64;
            for (int part = 0; part < parts; ++part) {
                gchunk.push_back((int32_t)cgrp.size());
                const size_t g0 = cgrp.size();
                for (int64_t ch = nch * part / parts; ch < nch * (part + 1) / parts; ++ch) {
                    const size_t b0 = (size_t)ch * 64, b1 = std::min(v.size(), b0 + 64);
                    // lane group g takes rays 16 g .. 16 g + 15 of the chunk; in each group, longest first,
                    // a ray starts after the least delay d whose residue (entry - d s, s = the quadrant's
                    // x step) no earlier lane of the group holds; empty lanes take the free residues
                    const int sgn = (qd & 2) ? -1 : 1;
                    int32_t lanes[64];
                    uint32_t m = 0;
                    for (int g = 0; g < 4; ++g) {
                        int idx[16], nr = 0;
                        for (size_t i = b0 + 16 * g; i < std::min(b1, b0 + 16 * g + 16); ++i) idx[nr++] = (int)(i - b0);
                        std::stable_sort(idx, idx + nr, [&](int a1, int a2) {
                            return cnt[(size_t)v[b0 + a1]] > cnt[(size_t)v[b0 + a2]];
                        });
                        unsigned seen = 0;
                        for (int r = 0; r < nr; ++r) {
                            const int64_t j = v[b0 + idx[r]];
                            const int res = (int)(ent[(size_t)j] & 15u);
                            int dl = 0;
                            while (dl < 15 && (seen >> (((res - dl * sgn) % 16 + 16) % 16) & 1u)) ++dl;
                            seen |= 1u << (((res - dl * sgn) % 16 + 16) % 16);
                            lanes[LG[g][r]] = (int32_t)j | dl << 27;
                            m = std::max(m, cnt[(size_t)j] + (uint32_t)dl);
                        }
                        int rr = 0;
                        for (int r = nr; r < 16; ++r) {
                            while (rr < 15 && (seen >> rr & 1u)) ++rr;
                            seen |= 1u << rr;
                            lanes[LG[g][r]] = -1 - rr;
                        }
                    }
                    for (int l = 0; l < 64; ++l) cslot.push_back(lanes[l]);
                    cgrp.push_back(tile * 4 + qd);
                    coff.push_back(coff.back() + (int64_t)((m + 3) / 4));
                    maxlen = std::max<int64_t>(maxlen, (m + 3) / 4 * 4);
                }
                // the group's chunks longest first (the kernel's waves claim them in this order)
                const size_t nc = cgrp.size() - g0;
                if (nc > 1) {
                    std::vector<int64_t> len(nc);
                    for (size_t i = 0; i < nc; ++i) len[i] = coff[g0 + i + 1] - coff[g0 + i];
                    std::vector<size_t> ord(nc);
                    std::iota(ord.begin(), ord.end(), (size_t)0);
                    std::stable_sort(ord.begin(), ord.end(), [&](size_t a1, size_t a2) { return len[a1] > len[a2]; });
                    std::vector<int32_t> cs2(nc * 64);
                    for (size_t i = 0; i < nc; ++i)
                        std::copy(cslot.begin() + (g0 + ord[i]) * 64, cslot.begin() + (g0 + ord[i] + 1) * 64,
                                  cs2.begin() + i * 64);
                    std::copy(cs2.begin(), cs2.end(), cslot.begin() + g0 * 64);
                    for (size_t i = 0; i < nc; ++i) coff[g0 + i + 1] = coff[g0 + i] + len[ord[i]];
                }
            }
        }
    }
    gchunk.push_back((int32_t)cgrp.size());
    std::vector<int32_t> glist;  // the groups that hold chunks
    for (size_t g = 0; g + 1 < gchunk.size(); ++g)
        if (gchunk[g + 1] > gchunk[g]) glist.push_back((int32_t)g);
    const int64_t nchunks = (int64_t)cgrp.size();
    const size_t wbytes = (size_t)coff.back() * 64 * sizeof(float4);
    const size_t hbytes = (size_t)nchunks * 64 * sizeof(int4);
    if (wbytes + hbytes > max_bytes) return hipErrorOutOfMemory;
    // padding / empty lanes walk up to maxlen x steps (16 bytes each) from a plane position, delayed
    // lanes start up to 15 x steps before their entry voxel
    if (nslots >= (1 << 27)) return hipErrorOutOfMemory;  // slot | delay << 27
    pl.adjl_slack = (int32_t)(16 * (maxlen + 16));
    int32_t *d_cslot = nullptr, *d_cgrp = nullptr;
    auto up = [&](void** dst, const void* src, size_t bytes) -> hipError_t {
        hipError_t r = hipMalloc(dst, std::max<size_t>(bytes, 16));
        if (r == hipSuccess && bytes) r = hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
        return r;
    };
    if ((e = up((void**)&bufs.gchunk, gchunk.data(), gchunk.size() * sizeof(int32_t))) != hipSuccess ||
        (e = up((void**)&bufs.glist, glist.data(), glist.size() * sizeof(int32_t))) != hipSuccess ||
        (e = up((void**)&bufs.coff, coff.data(), coff.size() * sizeof(int64_t))) != hipSuccess ||
        (e = up((void**)&d_cslot, cslot.data(), cslot.size() * sizeof(int32_t))) != hipSuccess ||
        (e = up((void**)&d_cgrp, cgrp.data(), cgrp.size() * sizeof(int32_t))) != hipSuccess ||
        (e = hipMalloc((void**)&bufs.hdr, std::max<size_t>(hbytes, 16))) != hipSuccess ||
        (e = hipMalloc((void**)&bufs.w, std::max<size_t>(wbytes, 16))) != hipSuccess) {
        (void)hipFree(d_cslot);
        (void)hipFree(d_cgrp);
        return e;
    }
    pl.adjl_gchunk = bufs.gchunk;
    pl.adjl_glist = bufs.glist;
    pl.adjl_nlist = (int32_t)glist.size();
    pl.adjl_coff = bufs.coff;
    pl.adjl_hdr = bufs.hdr;
    pl.adjl_w = bufs.w;
    pl.adjl_ngroups = ntiles * 4 * parts;
    pl.adjl_parts = parts;
    if (nchunks > 0) {
        const unsigned nb = (unsigned)((nchunks * 64 + 255) / 256);
        if (w2)
            hipLaunchKernelGGL((tvam_adjl_fill_kernel<true>), dim3(nb), dim3(256), 0, stream, k, pl, t, nchunks, d_cslot,
                               d_cgrp, bufs.hdr, bufs.w);
        else
            hipLaunchKernelGGL((tvam_adjl_fill_kernel<false>), dim3(nb), dim3(256), 0, stream, k, pl, t, nchunks, d_cslot,
                               d_cgrp, bufs.hdr, bufs.w);
    }
    if ((e = hipGetLastError()) == hipSuccess) e = hipStreamSynchronize(stream);
    (void)hipFree(d_cslot);
    (void)hipFree(d_cgrp);
    bufs.bytes = wbytes + hbytes;
    bufs.visits_padded = coff.back() * 256;
    return e;
}
