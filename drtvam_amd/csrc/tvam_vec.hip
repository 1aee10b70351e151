// tvam_vec.hip — fused vector kernels of the linear L-BFGS step
// (lbfgs.py:146-275 of the reference, restated in drtvam_amd/lbfgs.py).
//
// The two-loop recursion only ever needs dot products between the current
// gradient g and the history pairs (s_i, y_i); written in terms of the Gram
// entries s_i.y_j, y_i.y_j, s_i.g, y_i.g, g.g it becomes scalar work, and the
// search direction is one linear combination of g, s_i, y_i.  So one step
// touches the n-vectors in three passes instead of ~4m + 10:
//   tvam_lbfgs_history   : s_new = p - p_old, y_new = g - g_old and every dot
//                          the recursion needs, in one read of p, p_old, g,
//                          g_old and the retained history;
//   tvam_lbfgs_direction : d = cg g + sum cs_j s_j + sum cy_j y_j;
//   tvam_axpy_clamp      : p_new = max(p + alpha d, lo) (update + clamp,
//                          optimize.py:316-318).
// Dot products accumulate in fp64 per thread, then per block, then over a
// fixed number of blocks in a fixed order (deterministic).
#include "tvam_internal.h"

#define TVAM_VB 256       // threads per block
#define TVAM_VGRID_MAX 2048  // most blocks of the reduction kernels (work[] holds grid * ndots doubles)
#define TVAM_HMAX 8
#define TVAM_VU 1  // grid-stride elements per loop trip (2 and 4: no faster, profiles/r06/vec/)

#include <algorithm>
#include <cstdlib>

// launch geometry knobs (read once): blocks of the history pass and of the direction pass
static int vec_knob(const char* name, int def) {
    const int x = tvam_knob(name, def);
    return x > 0 ? x : def;
}
static int hist_grid() {
    static const int g = std::min(vec_knob("TVAM_VEC_HGRID", 768), TVAM_VGRID_MAX);
    return g;
}
static int dir_grid() {
    static const int g = vec_knob("TVAM_VEC_DGRID", 1024);
    return g;
}

// a streamed float4, loaded non-temporal: every pass reads a history vector once, gigabytes before the
// next pass reads it again (direction pass 0.75 -> 0.65 ms at config 2's size, profiles/r06/vec/)
__device__ __forceinline__ float4 vld(const float* p, uint64_t i) {
    typedef float vf4 __attribute__((ext_vector_type(4)));
    const vf4 v = __builtin_nontemporal_load(reinterpret_cast<const vf4*>(p) + i);
    return make_float4(v.x, v.y, v.z, v.w);
}

struct VecPtrs {
    const float* s[TVAM_HMAX];
    const float* y[TVAM_HMAX];
};

// Segments of the vectors (tvam_lbfgs_history_rows / tvam_lbfgs_direction_rows): float4 index t
// of the part -> segment t / len4, float4 off4 + segment * stride4 + t % len4 (a band of DMD rows
// of every angle)
struct VecSeg {
    uint32_t len4;
    uint64_t stride4, off4;
};

__device__ __forceinline__ uint64_t vec_seg_index(const VecSeg& sg, uint64_t t) {
    const uint64_t a = t / sg.len4;
    return sg.off4 + a * sg.stride4 + (t - a * sg.len4);
}

__device__ __forceinline__ double warp_sum(double v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Block-reduce ND accumulators and write this block's partials.
template <int ND>
__device__ __forceinline__ void block_partials(double (&acc)[ND], double* __restrict__ work) {
    __shared__ double red[TVAM_VB / 64][ND > 0 ? ND : 1];
#pragma unroll
    for (int d = 0; d < ND; ++d) {
        const double v = warp_sum(acc[d]);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][d] = v;
    }
    __syncthreads();
    for (int d = threadIdx.x; d < ND; d += TVAM_VB) {
        double s = 0.0;
        for (int w = 0; w < TVAM_VB / 64; ++w) s += red[w][d];
        work[(size_t)blockIdx.x * ND + d] = s;
    }
}

// Dots written (H = retained pairs, NEW = a new pair is formed; index j runs
// over the retained pairs, then the new one):
//   [0, HT)        s_j . g          HT = H + NEW
//   [HT, 2HT)      y_j . g
//   if NEW:
//   [2HT, 3HT)     s_new . y_j
//   [3HT, 4HT)     s_j . y_new
//   [4HT, 5HT)     y_new . y_j
//   last           g . g
template <int H, bool NEW>
struct HistLayout {
    static constexpr int HT = H + (NEW ? 1 : 0);
    static constexpr int ND = (NEW ? 5 * HT : 2 * HT) + 1;
};

// SPRE: s_new already holds p - p_old (written by the previous step's update, tvam_axpy_clamp_dev's
// s_out): read instead of formed from p and p_old (two vector reads and a write fewer)
template <int H, bool NEW, bool SEG = false, bool SPRE = false>
__global__ __launch_bounds__(TVAM_VB) void tvam_lbfgs_hist_kernel(uint64_t n, const float* __restrict__ p,
                                                                   const float* __restrict__ p_old,
                                                                   const float* __restrict__ g,
                                                                   const float* __restrict__ g_old, VecPtrs hv,
                                                                   float* __restrict__ s_new,
                                                                   float* __restrict__ y_new,
                                                                   double* __restrict__ work, VecSeg sg) {
    using L = HistLayout<H, NEW>;
    constexpr int HT = L::HT, ND = L::ND;
    double acc[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) acc[d] = 0.0;

    auto visit = [&](float pv, float pov, float gv, float gov, const float (&sv)[TVAM_HMAX],
                     const float (&yv)[TVAM_HMAX], float& sn, float& yn) {
        sn = NEW ? pv - pov : 0.0f;
        yn = NEW ? gv - gov : 0.0f;
#pragma unroll
        for (int j = 0; j < HT; ++j) {
            const float sj = j < H ? sv[j] : sn, yj = j < H ? yv[j] : yn;
            acc[j] = fma((double)sj, (double)gv, acc[j]);
            acc[HT + j] = fma((double)yj, (double)gv, acc[HT + j]);
            if (NEW) {
                acc[2 * HT + j] = fma((double)sn, (double)yj, acc[2 * HT + j]);
                acc[3 * HT + j] = fma((double)sj, (double)yn, acc[3 * HT + j]);
                acc[4 * HT + j] = fma((double)yn, (double)yj, acc[4 * HT + j]);
            }
        }
        acc[ND - 1] = fma((double)gv, (double)gv, acc[ND - 1]);
    };

    const uint64_t n4 = n / 4, stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // VU grid-stride elements per trip, all their loads issued before the first is summed (more bytes
    // in flight per wave); each thread still sums its elements in grid-stride order (the same dots)
    struct El {
        float4 g4, p4, po4, go4, s4[H > 0 ? H : 1], y4[H > 0 ? H : 1];
    };
    for (uint64_t t0 = tid; t0 < n4; t0 += (uint64_t)TVAM_VU * stride) {
        El el[TVAM_VU];
#pragma unroll
        for (int u = 0; u < TVAM_VU; ++u) {
            const uint64_t t = t0 + (uint64_t)u * stride;
            if (t >= n4) break;
            const uint64_t i = SEG ? vec_seg_index(sg, t) : t;
            el[u].g4 = vld(g, i);
            el[u].p4 = el[u].po4 = el[u].go4 = make_float4(0, 0, 0, 0);
            if (NEW) {
                if (SPRE) {
                    el[u].p4 = vld(s_new, i);  // s_new = p - p_old, with p_old = 0 below
                } else {
                    el[u].p4 = vld(p, i);
                    el[u].po4 = vld(p_old, i);
                }
                el[u].go4 = vld(g_old, i);
            }
#pragma unroll
            for (int j = 0; j < H; ++j) {
                el[u].s4[j] = vld(hv.s[j], i);
                el[u].y4[j] = vld(hv.y[j], i);
            }
        }
#pragma unroll
        for (int u = 0; u < TVAM_VU; ++u) {
            const uint64_t t = t0 + (uint64_t)u * stride;
            if (t >= n4) break;
            const uint64_t i = SEG ? vec_seg_index(sg, t) : t;
            const El& e = el[u];
            float sv[TVAM_HMAX], yv[TVAM_HMAX];
            float4 sn4, yn4;
#define TVAM_LANE(c)                                                    \
            _Pragma("unroll") for (int j = 0; j < H; ++j) {             \
                sv[j] = e.s4[j].c;                                      \
                yv[j] = e.y4[j].c;                                      \
            }                                                           \
            visit(e.p4.c, e.po4.c, e.g4.c, e.go4.c, sv, yv, sn4.c, yn4.c);
            TVAM_LANE(x) TVAM_LANE(y) TVAM_LANE(z) TVAM_LANE(w)
#undef TVAM_LANE
            if (NEW) {
                if (!SPRE) reinterpret_cast<float4*>(s_new)[i] = sn4;
                reinterpret_cast<float4*>(y_new)[i] = yn4;
            }
        }
    }
    for (uint64_t i = 4 * n4 + tid; !SEG && i < n; i += stride) {  // tail
        float sv[TVAM_HMAX], yv[TVAM_HMAX];
#pragma unroll
        for (int j = 0; j < H; ++j) {
            sv[j] = hv.s[j][i];
            yv[j] = hv.y[j][i];
        }
        float sn, yn;
        visit(NEW ? (SPRE ? s_new[i] : p[i]) : 0.0f, NEW && !SPRE ? p_old[i] : 0.0f, g[i], NEW ? g_old[i] : 0.0f, sv,
              yv, sn, yn);
        if (NEW) {
            if (!SPRE) s_new[i] = sn;
            y_new[i] = yn;
        }
    }
    block_partials<ND>(acc, work);
}

// Sum the per-block partials of dot d over the blocks, in block order.
__global__ __launch_bounds__(TVAM_VB) void tvam_partials_kernel(int nd, int nblocks, const double* __restrict__ work,
                                                                double* __restrict__ dots) {
    __shared__ double red[TVAM_VB / 64];
    const int d = blockIdx.x;
    double s = 0.0;
    for (int b = threadIdx.x; b < nblocks; b += TVAM_VB) s += work[(size_t)b * nd + d];
    s = warp_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < TVAM_VB / 64; ++w) t += red[w];
        dots[d] = t;
    }
}

template <int H, bool NEW>
static hipError_t launch_hist(uint64_t n, const float* p, const float* p_old, const float* g, const float* g_old,
                              const VecPtrs& hv, float* s_new, float* y_new, double* work, double* dots,
                              hipStream_t stream, const VecSeg& sg) {
    // a band of rows (sg.len4 > 0): fewer blocks, the rest of the GPU keeps the neighbouring band's adjoint
    const int nb = sg.len4 ? std::max(64, (int)std::min<uint64_t>(hist_grid(), (n / 4 + TVAM_VB - 1) / TVAM_VB))
                           : hist_grid();
    if (sg.len4)
        hipLaunchKernelGGL((tvam_lbfgs_hist_kernel<H, NEW, true>), dim3(nb), dim3(TVAM_VB), 0, stream, n, p, p_old, g,
                           g_old, hv, s_new, y_new, work, sg);
    else if (NEW && !p_old)  // s_new precomputed (tvam_lbfgs_history: g_old given, p_old NULL)
        hipLaunchKernelGGL((tvam_lbfgs_hist_kernel<H, NEW, false, true>), dim3(nb), dim3(TVAM_VB), 0, stream, n, p,
                           p_old, g, g_old, hv, s_new, y_new, work, sg);
    else
        hipLaunchKernelGGL((tvam_lbfgs_hist_kernel<H, NEW>), dim3(nb), dim3(TVAM_VB), 0, stream, n, p, p_old, g,
                           g_old, hv, s_new, y_new, work, sg);
    hipLaunchKernelGGL(tvam_partials_kernel, dim3(HistLayout<H, NEW>::ND), dim3(TVAM_VB), 0, stream,
                       HistLayout<H, NEW>::ND, nb, work, dots);
    return hipGetLastError();
}

template <bool NEW>
static hipError_t dispatch_hist(int h, uint64_t n, const float* p, const float* p_old, const float* g,
                                const float* g_old, const VecPtrs& hv, float* s_new, float* y_new, double* work,
                                double* dots, hipStream_t stream, const VecSeg& sg) {
    switch (h) {
#define TVAM_H(H) \
    case H: return launch_hist<H, NEW>(n, p, p_old, g, g_old, hv, s_new, y_new, work, dots, stream, sg);
        TVAM_H(0) TVAM_H(1) TVAM_H(2) TVAM_H(3) TVAM_H(4) TVAM_H(5) TVAM_H(6) TVAM_H(7)
#undef TVAM_H
        default: return hipErrorInvalidValue;
    }
}

hipError_t tvam_launch_lbfgs_history(uint64_t n, const float* p, const float* p_old, const float* g,
                                     const float* g_old, int h, const float* const* S, const float* const* Y,
                                     float* s_new, float* y_new, double* work, double* dots, hipStream_t stream,
                                     uint64_t nseg, uint64_t seg_len, uint64_t seg_stride, uint64_t seg_off) {
    VecPtrs hv{};
    for (int j = 0; j < h; ++j) {
        hv.s[j] = S[j];
        hv.y[j] = Y[j];
    }
    VecSeg sg{};
    if (nseg > 0) {
        n = nseg * seg_len;
        sg.len4 = (uint32_t)(seg_len / 4);
        sg.stride4 = seg_stride / 4;
        sg.off4 = seg_off / 4;
    }
    if (p_old || g_old) return dispatch_hist<true>(h, n, p, p_old, g, g_old, hv, s_new, y_new, work, dots, stream, sg);
    return dispatch_hist<false>(h, n, p, p_old, g, g_old, hv, s_new, y_new, work, dots, stream, sg);
}

// ---------------------------------------------------------------------------
struct DirCoef {
    float cg;
    float cs[TVAM_HMAX], cy[TVAM_HMAX];
};

// DEV: the coefficients come from device memory (tvam_lbfgs_coef_kernel's output: cg, cs[8], cy[8]).
// SEG: n = the part's elements (segments x length), indices through VecSeg.
template <int H, bool DEV = false, bool SEG = false>
__global__ __launch_bounds__(TVAM_VB) void tvam_lbfgs_dir_kernel(uint64_t n, const float* __restrict__ g, VecPtrs hv,
                                                                  DirCoef c, const float* __restrict__ cdev,
                                                                  float* __restrict__ d, VecSeg sg = VecSeg{}) {
    if (DEV) {
        c.cg = cdev[0];
#pragma unroll
        for (int j = 0; j < H; ++j) {
            c.cs[j] = cdev[1 + j];
            c.cy[j] = cdev[1 + TVAM_HMAX + j];
        }
    }
    const uint64_t n4 = n / 4, stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t t0 = tid; t0 < n4; t0 += (uint64_t)TVAM_VU * stride) {
        float4 g4[TVAM_VU], s4[TVAM_VU][H > 0 ? H : 1], y4[TVAM_VU][H > 0 ? H : 1];
#pragma unroll
        for (int u = 0; u < TVAM_VU; ++u) {  // every load of the trip first (bytes in flight)
            const uint64_t t = t0 + (uint64_t)u * stride;
            if (t >= n4) break;
            const uint64_t i = SEG ? vec_seg_index(sg, t) : t;
            g4[u] = vld(g, i);
#pragma unroll
            for (int j = 0; j < H; ++j) {
                s4[u][j] = vld(hv.s[j], i);
                y4[u][j] = vld(hv.y[j], i);
            }
        }
#pragma unroll
        for (int u = 0; u < TVAM_VU; ++u) {
            const uint64_t t = t0 + (uint64_t)u * stride;
            if (t >= n4) break;
            const uint64_t i = SEG ? vec_seg_index(sg, t) : t;
            float4 r = make_float4(c.cg * g4[u].x, c.cg * g4[u].y, c.cg * g4[u].z, c.cg * g4[u].w);
#pragma unroll
            for (int j = 0; j < H; ++j) {
                r.x = fmaf(c.cs[j], s4[u][j].x, fmaf(c.cy[j], y4[u][j].x, r.x));
                r.y = fmaf(c.cs[j], s4[u][j].y, fmaf(c.cy[j], y4[u][j].y, r.y));
                r.z = fmaf(c.cs[j], s4[u][j].z, fmaf(c.cy[j], y4[u][j].z, r.z));
                r.w = fmaf(c.cs[j], s4[u][j].w, fmaf(c.cy[j], y4[u][j].w, r.w));
            }
            reinterpret_cast<float4*>(d)[i] = r;
        }
    }
    for (uint64_t i = 4 * n4 + tid; !SEG && i < n; i += stride) {
        float r = c.cg * g[i];
#pragma unroll
        for (int j = 0; j < H; ++j) r = fmaf(c.cs[j], hv.s[j][i], fmaf(c.cy[j], hv.y[j][i], r));
        d[i] = r;
    }
}

hipError_t tvam_launch_lbfgs_direction(uint64_t n, const float* g, int h, const float* const* S,
                                       const float* const* Y, float cg, const float* cs, const float* cy, float* d,
                                       hipStream_t stream) {
    VecPtrs hv{};
    DirCoef c{};
    c.cg = cg;
    for (int j = 0; j < h; ++j) {
        hv.s[j] = S[j];
        hv.y[j] = Y[j];
        c.cs[j] = cs[j];
        c.cy[j] = cy[j];
    }
    const dim3 grid(dir_grid()), block(TVAM_VB);
    switch (h) {
#define TVAM_H(H) \
    case H: hipLaunchKernelGGL(tvam_lbfgs_dir_kernel<H>, grid, block, 0, stream, n, g, hv, c, nullptr, d, VecSeg{}); break;
        TVAM_H(0) TVAM_H(1) TVAM_H(2) TVAM_H(3) TVAM_H(4) TVAM_H(5) TVAM_H(6) TVAM_H(7) TVAM_H(8)
#undef TVAM_H
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// The two-loop recursion on the device (lbfgs.py:221-243 in Gram form, as the host recursion of
// drtvam_amd/lbfgs.py evaluated it before): one lane, so the direction pass follows the history
// pass and its all-reduce on the stream without a host round trip.  gram[] keeps the retained
// pairs' entries between steps, indexed by ring slot: s_a.y_b at [a][b], y_a.y_b at 64 + [a][b];
// a new pair's entries come from the history pass's dots.  The same fp64 operations in the same
// order as that host code (no contraction), so the f32-rounded coefficients -- and the
// direction -- are bit-identical to it.  coef: cg | cs[8] | cy[8]; gdz: g.d (the Armijo slope).
struct LbfgsOrder {
    int slot[TVAM_HMAX];
};

__global__ void tvam_lbfgs_coef_kernel(int H, int is_new, int first, LbfgsOrder o, const double* __restrict__ dots,
                                       double* __restrict__ gram, float* __restrict__ coef,
                                       double* __restrict__ gdz) {
#pragma clang fp contract(off)
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double* SY = gram;
    double* YY = gram + TVAM_HMAX * TVAM_HMAX;
    const double* Sg = dots;
    const double* Yg = dots + H;
    const double gg = dots[(is_new ? 5 * H : 2 * H)];
    if (is_new) {
        const int sl = o.slot[H - 1];
        for (int j = 0; j < H; ++j) {
            const int sj = o.slot[j];
            SY[sl * TVAM_HMAX + sj] = dots[2 * H + j];  // s_new . y_j
            SY[sj * TVAM_HMAX + sl] = dots[3 * H + j];  // s_j . y_new
            YY[sl * TVAM_HMAX + sj] = dots[4 * H + j];
            YY[sj * TVAM_HMAX + sl] = dots[4 * H + j];
        }
    }
    double a[TVAM_HMAX], b[TVAM_HMAX];
    for (int i = H - 1; i >= 0; --i) {
        const int si = o.slot[i];
        double s = 0.0;
        for (int j = i + 1; j < H; ++j) s = s + a[j] * SY[si * TVAM_HMAX + o.slot[j]];
        a[i] = (Sg[i] - s) / SY[si * TVAM_HMAX + si];
    }
    const int last = H > 0 ? o.slot[H - 1] : 0;
    const double gamma = (first || H == 0) ? 1.0 : SY[last * TVAM_HMAX + last] / YY[last * TVAM_HMAX + last];
    for (int i = 0; i < H; ++i) {
        const int yi = o.slot[i];
        double s1 = 0.0;
        for (int j = 0; j < H; ++j) s1 = s1 + a[j] * YY[yi * TVAM_HMAX + o.slot[j]];
        double yz = gamma * (Yg[i] - s1);
        double s2 = 0.0;
        for (int j = 0; j < i; ++j) s2 = s2 + (a[j] - b[j]) * SY[o.slot[j] * TVAM_HMAX + yi];
        yz = yz + s2;
        b[i] = yz / SY[yi * TVAM_HMAX + yi];
    }
    // d = -z, z = gamma (g - sum a_j y_j) + sum (a_j - b_j) s_j
    const double cg = -gamma;
    double r = cg * gg, rs = 0.0, ry = 0.0;
    coef[0] = (float)cg;
    for (int j = 0; j < H; ++j) {
        const double cs = -(a[j] - b[j]), cy = gamma * a[j];
        coef[1 + j] = (float)cs;
        coef[1 + TVAM_HMAX + j] = (float)cy;
        rs = rs + cs * Sg[j];
        ry = ry + cy * Yg[j];
    }
    gdz[0] = r + rs + ry;
}

hipError_t tvam_launch_lbfgs_coef(int h, int is_new, int first, const int* order, const double* dots, double* gram,
                                  float* coef, double* gdz, hipStream_t stream) {
    LbfgsOrder o{};
    for (int j = 0; j < h; ++j) o.slot[j] = order[j];
    hipLaunchKernelGGL(tvam_lbfgs_coef_kernel, dim3(1), dim3(64), 0, stream, h, is_new, first, o, dots, gram, coef, gdz);
    return hipGetLastError();
}

hipError_t tvam_launch_lbfgs_direction_dev(uint64_t n, const float* g, int h, const float* const* S,
                                           const float* const* Y, const float* coef, float* d, hipStream_t stream,
                                           uint64_t nseg, uint64_t seg_len, uint64_t seg_stride, uint64_t seg_off) {
    VecPtrs hv{};
    for (int j = 0; j < h; ++j) {
        hv.s[j] = S[j];
        hv.y[j] = Y[j];
    }
    const DirCoef c{};
    VecSeg sg{};
    const bool seg = nseg > 0;
    if (seg) {
        n = nseg * seg_len;
        sg.len4 = (uint32_t)(seg_len / 4);
        sg.stride4 = seg_stride / 4;
        sg.off4 = seg_off / 4;
    }
    // a part of the vector: fewer blocks, so that the rest of the GPU keeps the forward of the
    // previous part (tvam_lbfgs_direction_rows)
    const int nb = seg ? std::max(64, (int)std::min<uint64_t>(dir_grid(), (n / 4 + TVAM_VB - 1) / TVAM_VB)) : dir_grid();
    const dim3 grid(nb), block(TVAM_VB);
    switch (h) {
#define TVAM_H(H)                                                                                                 \
    case H:                                                                                                       \
        if (seg)                                                                                                  \
            hipLaunchKernelGGL((tvam_lbfgs_dir_kernel<H, true, true>), grid, block, 0, stream, n, g, hv, c, coef, \
                               d, sg);                                                                            \
        else                                                                                                      \
            hipLaunchKernelGGL((tvam_lbfgs_dir_kernel<H, true>), grid, block, 0, stream, n, g, hv, c, coef, d,    \
                               sg);                                                                               \
        break;
        TVAM_H(0) TVAM_H(1) TVAM_H(2) TVAM_H(3) TVAM_H(4) TVAM_H(5) TVAM_H(6) TVAM_H(7) TVAM_H(8)
#undef TVAM_H
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// alpha_dev (tvam_axpy_clamp_dev): the step size read from device memory, tvam_armijo_kernel's pick
// s_out (optional): the next history pair's s = out - p (the fp32 difference tvam_lbfgs_history forms
// from p_new and p_old, so that pass reads it instead of both vectors)
__global__ __launch_bounds__(TVAM_VB) void tvam_axpy_clamp_kernel(uint64_t n, const float* __restrict__ p, float alpha,
                                                                  const float* __restrict__ d, float lo,
                                                                  float* __restrict__ out,
                                                                  const float* __restrict__ alpha_dev,
                                                                  float* __restrict__ s_out) {
    if (alpha_dev) alpha = alpha_dev[0];
    const uint64_t n4 = n / 4, stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t i = tid; i < n4; i += stride) {
        const float4 p4 = reinterpret_cast<const float4*>(p)[i];
        const float4 d4 = reinterpret_cast<const float4*>(d)[i];
        const float4 o = make_float4(fmaxf(fmaf(alpha, d4.x, p4.x), lo), fmaxf(fmaf(alpha, d4.y, p4.y), lo),
                                     fmaxf(fmaf(alpha, d4.z, p4.z), lo), fmaxf(fmaf(alpha, d4.w, p4.w), lo));
        reinterpret_cast<float4*>(out)[i] = o;
        if (s_out) reinterpret_cast<float4*>(s_out)[i] = make_float4(o.x - p4.x, o.y - p4.y, o.z - p4.z, o.w - p4.w);
    }
    for (uint64_t i = 4 * n4 + tid; i < n; i += stride) {
        const float o = fmaxf(fmaf(alpha, d[i], p[i]), lo);
        out[i] = o;
        if (s_out) s_out[i] = o - p[i];
    }
}

hipError_t tvam_launch_axpy_clamp(uint64_t n, const float* p, float alpha, const float* d, float lo, float* out,
                                  hipStream_t stream, const float* alpha_dev, float* s_out) {
    hipLaunchKernelGGL(tvam_axpy_clamp_kernel, dim3(2048), dim3(TVAM_VB), 0, stream, n, p, alpha, d, lo, out,
                       alpha_dev, s_out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// The first batch of Armijo probes decided on the device (FusedLinearLBFGS.step), so that the
// update p + alpha d can follow the probes on the stream while the host reads them: alpha[0] =
// a_j for the first probe j with f_j <= loss + c1 a_j g.d, a_j = a0 / 2^j (lbfgs.py:256-266), in
// the host loop's fp64 operations and order (no contraction); 0 when no probe passes (the host
// then discards the update launched behind it).  loss = loss_dev[0] / loss_div, or loss_host.
// report (optional, e.g. pinned host memory the host polls, no copy kernel and no event): the undivided
// loss, g.d, the probes and the chosen alpha, as f64, then 1.0 once they are visible system-wide.
__global__ void tvam_armijo_kernel(int nprobe, double a0, const double* __restrict__ probes,
                                   const double* __restrict__ loss_dev, double loss_host, double loss_div,
                                   const double* __restrict__ gdz, double c1, float* __restrict__ alpha,
                                   double* __restrict__ report) {
#pragma clang fp contract(off)
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const double l0 = loss_dev ? loss_dev[0] : loss_host;
    const double lv = loss_dev ? l0 / loss_div : loss_host;
    const double gd = 0.0 + gdz[0];
    float r = 0.0f;
    for (int j = 0; j < nprobe; ++j) {
        const double a = a0 * ldexp(1.0, -j);
        if (probes[j] <= lv + c1 * a * gd) {
            r = (float)a;
            break;
        }
    }
    alpha[0] = r;
    if (report) {
        report[0] = l0;
        report[1] = gdz[0];
        for (int j = 0; j < nprobe; ++j) report[2 + j] = probes[j];
        report[2 + nprobe] = (double)r;
        __threadfence_system();
        report[3 + nprobe] = 1.0;
        __threadfence_system();
    }
}

hipError_t tvam_launch_armijo(int nprobe, double a0, const double* probes, const double* loss_dev, double loss_host,
                              double loss_div, const double* gdz, double c1, float* alpha, double* report,
                              hipStream_t stream) {
    hipLaunchKernelGGL(tvam_armijo_kernel, dim3(1), dim3(64), 0, stream, nprobe, a0, probes, loss_dev, loss_host,
                       loss_div, gdz, c1, alpha, report);
    return hipGetLastError();
}
