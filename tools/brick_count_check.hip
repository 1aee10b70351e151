// CPU check of the record writer's closed-form brick count (sc_brick_count, tvam_bricks.h)
// against the bin fill's walk (sc_walk_bricks) on random segments: random origins inside and
// outside the grid, random / axis-aligned / near-axis directions, grids whose sizes are and are not
// multiples of the brick.  Host code only (no GPU).  Build and run: tools/brick_count_check.sh
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../drtvam_amd/csrc/tvam_bricks.h"

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 2000000;
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    const int grids[][3] = {{400, 400, 400}, {64, 64, 64}, {50, 70, 33}, {32, 32, 16}, {97, 13, 130}, {800, 800, 800}};
    long bad = 0, total = 0, maxc = 0;
    for (const auto& gr : grids) {
        TvamConsts k{};
        for (int a = 0; a < 3; ++a) {
            k.res[a] = gr[a];
            k.h[a] = 2.0f / (float)gr[0];
            k.bmin[a] = -0.5f * k.h[a] * (float)gr[a];
            k.bmax[a] = 0.5f * k.h[a] * (float)gr[a];
        }
        for (long i = 0; i < n; ++i) {
            float o[3], d[3];
            for (int a = 0; a < 3; ++a) o[a] = (k.bmin[a] - 0.2f) + (k.bmax[a] - k.bmin[a] + 0.4f) * U(rng);
            const int kind = (int)(U(rng) * 4.0f);
            for (int a = 0; a < 3; ++a) d[a] = 2.0f * U(rng) - 1.0f;
            if (kind == 1) d[(int)(U(rng) * 2.999f)] = 0.0f;                      // in an axis plane
            if (kind == 2) { d[0] *= 1e-7f; d[1] *= 1e-6f; }                         // near an axis
            if (kind == 3) for (int a = 0; a < 3; ++a) o[a] = k.bmin[a] + k.h[a] * (float)(int)(U(rng) * gr[a]);  // on faces
            float nn = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
            if (!(nn > 0.0f)) continue;
            for (int a = 0; a < 3; ++a) d[a] /= nn;
            const float maxt = U(rng) < 0.3f ? TVAM_INF : 4.0f * U(rng);
            SegDda q;
            if (!sc_dda_init(k, o, d, maxt, q)) continue;
            const int w = sc_walk_bricks(k, q, [](int, float, float) {});
            const int c = sc_brick_count(k, q);
            ++total;
            if (w > maxc) maxc = w;
            if (w != c && bad++ < 10)
                printf("mismatch grid %dx%dx%d walk %d count %d  o %.9g %.9g %.9g  d %.9g %.9g %.9g maxt %g\n", gr[0], gr[1],
                       gr[2], w, c, o[0], o[1], o[2], d[0], d[1], d[2], maxt);
        }
    }
    printf("segments %ld mismatches %ld longest walk %ld\n", total, bad, maxc);
    return bad == 0 ? 0 : 1;
}
