// tvam_bricks.h -- a scattered segment's DDA state and the bricks it crosses (tvam_scatter.hip):
// the record writer's brick count and the bin fill's walk.  Host + device, so that
// tools/brick_count_check.hip checks the closed-form count against the walk on the CPU.
#pragma once
#include "tvam_internal.h"

namespace {

struct SegDda {
    float t_start, tau_end;
    float dtm0[3], ts[3];  // ts > 0; step sign separate
    int sv[3], step[3];
};

__host__ __device__ __forceinline__ bool sc_dda_init(const TvamConsts& k, const float o[3], const float d[3], float maxt,
                                            SegDda& q) {
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
    if (!(isfinite(t_start) && isfinite(t_end) && t_start < t_end)) return false;
    q.t_start = t_start;
    q.tau_end = t_end - t_start;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float gs = fmaf(d[a], t_start, o[a]);
        q.step[a] = d[a] > 0.0f ? 1 : -1;
        int sv = (int)((gs - k.bmin[a]) / k.h[a]);
        sv = sv < 0 ? 0 : (sv > k.res[a] - 1 ? k.res[a] - 1 : sv);
        q.sv[a] = sv;
        float next = k.bmin[a] + (float)(sv + q.step[a]) * k.h[a];
        if (d[a] < 0.0f) next = next + k.h[a];
        const bool valid = fabsf(d[a]) > 1e-8f;
        float dtm = valid ? (next - gs) / d[a] : TVAM_INF;
        if (dtm < 0.0f) dtm = TVAM_INF;
        q.dtm0[a] = dtm;
        q.ts[a] = valid ? (k.h[a] / d[a]) * (float)q.step[a] : TVAM_INF;
    }
    return true;
}

__host__ __device__ __forceinline__ int sc_nbr(const TvamConsts& k, int a) {
    const int B = a == 0 ? TVAM_BX : (a == 1 ? TVAM_BY : TVAM_BZ);
    return (k.res[a] + B - 1) / B;
}

// tvam_axis_window's exit time of one axis' window [lo, hi), without branches (the same values)
__host__ __device__ __forceinline__ float sc_axis_tout(int sv, int step, float dtm0, float ts, int lo, int hi) {
    const int nout = step > 0 ? hi - sv : sv - lo + 1;
    const float tm = nout > 0 ? fmaf((float)(nout - 1), ts, dtm0) : -TVAM_INF;
    const float tf = (sv >= lo && sv < hi) ? TVAM_INF : -TVAM_INF;  // an axis that never steps
    return dtm0 < TVAM_INF ? tm : tf;
}

// Bricks a segment's DDA visits, in time order: each axis' brick windows
// partition time exactly (tvam_axis_window on brick bounds), so stepping the
// axis whose window closes first walks the same sequence the brick kernel
// resumes from.  F(brick id, relative time the segment enters / leaves the
// brick) per brick; returns the count.  Branch-free steps (selects; only the
// stepped axis can leave the grid): the per-axis if / else chain compiled to ~50
// scalar exec-mask instructions per step on top of ~70 VALU, and the fill kernel
// and the record writer spend most of their time in this loop.
template <typename F>
__host__ __device__ __forceinline__ int sc_walk_bricks(const TvamConsts& k, const SegDda& q, F&& f) {
    const int nb0 = sc_nbr(k, 0), nb1 = sc_nbr(k, 1), nb2 = sc_nbr(k, 2);
    int b0 = q.sv[0] / TVAM_BX, b1 = q.sv[1] / TVAM_BY, b2 = q.sv[2] / TVAM_BZ;
    int cnt = 0;
    float tprev = 0.0f;
    // each axis' exit time from the current brick; a step changes one axis' brick, so only that
    // axis' exit is formed again (the same sc_axis_tout values as forming all three every step)
    float t0 = sc_axis_tout(q.sv[0], q.step[0], q.dtm0[0], q.ts[0], b0 * TVAM_BX, min(b0 * TVAM_BX + TVAM_BX, k.res[0]));
    float t1 = sc_axis_tout(q.sv[1], q.step[1], q.dtm0[1], q.ts[1], b1 * TVAM_BY, min(b1 * TVAM_BY + TVAM_BY, k.res[1]));
    float t2 = sc_axis_tout(q.sv[2], q.step[2], q.dtm0[2], q.ts[2], b2 * TVAM_BZ, min(b2 * TVAM_BZ + TVAM_BZ, k.res[2]));
    for (int guard = 0; guard < 4096; ++guard) {
        const int bid = (b2 * nb1 + b1) * nb0 + b0;
        ++cnt;
        const bool m0 = t0 <= t1 && t0 <= t2;
        const bool m1 = !m0 && t1 <= t2;
        const float tm = m0 ? t0 : (m1 ? t1 : t2);
        f(bid, tprev, fminf(tm, q.tau_end));
        tprev = tm;
        if (!(tm < q.tau_end)) break;
        // the stepped axis: its next brick and exit (selects: one exit formed per step)
        const int B = m0 ? TVAM_BX : (m1 ? TVAM_BY : TVAM_BZ);
        const int st = m0 ? q.step[0] : (m1 ? q.step[1] : q.step[2]);
        const int bn = (m0 ? b0 : (m1 ? b1 : b2)) + st;
        const int nb = m0 ? nb0 : (m1 ? nb1 : nb2);
        if ((unsigned)bn >= (unsigned)nb) break;
        const int sv = m0 ? q.sv[0] : (m1 ? q.sv[1] : q.sv[2]);
        const float dtm = m0 ? q.dtm0[0] : (m1 ? q.dtm0[1] : q.dtm0[2]);
        const float ts = m0 ? q.ts[0] : (m1 ? q.ts[1] : q.ts[2]);
        const int res = m0 ? k.res[0] : (m1 ? k.res[1] : k.res[2]);
        const float tn = sc_axis_tout(sv, st, dtm, ts, bn * B, min(bn * B + B, res));
        b0 = m0 ? bn : b0;
        b1 = m1 ? bn : b1;
        b2 = (m0 || m1) ? b2 : bn;
        t0 = m0 ? tn : t0;
        t1 = m1 ? tn : t1;
        t2 = (m0 || m1) ? t2 : tn;
    }
    return cnt;
}

// sc_walk_bricks' count in closed form, without the walk.  An axis' brick-face crossings are at
// T_j = fmaf(n_j, ts, dtm0), n_j = n0 + j B (j = 0, 1, ...): sc_axis_tout's exit times of the
// successive bricks, the same fp32 expressions, non-decreasing in j.  The walk takes the crossings
// in (time, axis x < y < z) order and stops at the first one at or after tau_end, or at the first
// one that leaves the grid (crossing J of its axis); it counts the bricks it enters.  So with E the
// earliest grid-leaving crossing before tau_end, an axis contributes its crossings j < J ordered
// before E (or before tau_end without E): a monotone count, taken from the division's estimate and
// corrected on the exact T_j (a step or two at most).  Returns 1 + the crossings (the start brick).
__host__ __device__ __forceinline__ int sc_brick_count(const TvamConsts& k, const SegDda& q) {
    int n0[3], J[3];
    float te = 0.0f;
    int ea = -1;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int B = a == 0 ? TVAM_BX : (a == 1 ? TVAM_BY : TVAM_BZ);
        const int sv = q.sv[a], b0 = sv / B;
        int nx;
        if (q.step[a] > 0) {
            n0[a] = (b0 + 1) * B - sv - 1;
            J[a] = sc_nbr(k, a) - 1 - b0;
            nx = k.res[a] - sv - 1;
        } else {
            n0[a] = sv - b0 * B;
            J[a] = b0;
            nx = sv;
        }
        if (q.dtm0[a] < TVAM_INF) {
            const float tx = fmaf((float)nx, q.ts[a], q.dtm0[a]);  // leaves the grid
            if (tx < q.tau_end && (ea < 0 || tx < te)) {
                te = tx;
                ea = a;
            }
        }
    }
    int cnt = 1;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (!(q.dtm0[a] < TVAM_INF) || J[a] == 0) continue;
        const int B = a == 0 ? TVAM_BX : (a == 1 ? TVAM_BY : TVAM_BZ);
        const float L = ea >= 0 ? te : q.tau_end;
        const bool incl = ea >= 0 && a <= ea;
        const float ts = q.ts[a], d0 = q.dtm0[a];
        auto taken = [&](int j) {
            const float t = fmaf((float)(n0[a] + j * B), ts, d0);
            return t < L || (incl && t == L);
        };
        const float jf = ((L - d0) / ts - (float)n0[a]) / (float)B;
        int j = jf > 0.0f ? (int)fminf(ceilf(jf), (float)J[a]) : 0;
        while (j > 0 && !taken(j - 1)) --j;
        while (j < J[a] && taken(j)) ++j;
        cnt += j;
    }
    return cnt < 4096 ? cnt : 4096;
}

}  // namespace
