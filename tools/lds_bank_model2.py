"""Total LDS-cycle inefficiency of the planar adjoint's gathers (bank conflicts x idle lanes), per
slot order / layout, on the config-2 geometry of tools/lds_bank_model.py: LDS cycles of one
ds_read_b128 per lane-visit over all waves / (visits / 16), the conflict-free full-wave cost.
usage: python tools/lds_bank_model2.py [N] [tile] [window]"""
import sys

from lds_bank_model import GROUPS, pitch_of_quadrant, quadrant, tile_rays


def wave_cycles(lanes, f):
    L = max((len(r[2]) for r in lanes if r is not None), default=0)
    tot = 0
    for k in range(L):
        for g in GROUPS:
            seen = {}
            for l in g:
                r = lanes[l]
                if r is not None and k < len(r[2]):
                    ch = f(*r[2][k], r[0])
                    seen.setdefault(ch % 16, set()).add(ch)
            if seen:
                tot += max(len(s) for s in seen.values())
    return tot


def deal(pool_rays, f):
    """One wave from the front of pool_rays (a list, consumed): per 16-lane group the earliest rays
    of distinct entry residues, then the earliest remaining."""
    res = lambda r: f(*r[2][0], r[0]) % 16
    lanes = [None] * 64
    for g in GROUPS:
        used, pick = set(), []
        for i, r in enumerate(pool_rays):
            if len(pick) == 16:
                break
            if res(r) not in used:
                used.add(res(r))
                pick.append(i)
        for i in range(len(pool_rays)):
            if len(pick) == 16:
                break
            if i not in pick:
                pick.append(i)
        for l, i in zip(g, pick):
            lanes[l] = pool_rays[i]
        for i in sorted(pick, reverse=True):
            pool_rays.pop(i)
    return lanes


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    ts = int(sys.argv[2]) if len(sys.argv) > 2 else 45
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    rays = tile_rays(N, N, ts * 2, ts * 3, ts)
    visits = sum(len(r[2]) for r in rays)
    base = visits / 16
    # current: one pitch, slot order (angle-major, columns), waves of 64 consecutive slots
    f = lambda x, y, a: (y + 1) * 47 + x + 1
    cur = sum(wave_cycles(rays[w:w + 64] + [None] * max(0, 64 - len(rays[w:w + 64])), f)
              for w in range(0, len(rays), 64))
    print(f"current (pitch 47, slot order): {cur / base:.3f}")
    for sort_len in (False, True):
        tot = 0
        for q in range(4):
            fq = (lambda p: lambda x, y, a: (y + 1) * p + x + 1)(pitch_of_quadrant(q))
            rq = [r for r in rays if quadrant(r[0], N) == q]
            pos = 0
            while pos < len(rq):
                block = rq[pos:pos + W]
                pos += W
                if sort_len:
                    block.sort(key=lambda r: -len(r[2]))
                while block:
                    tot += wave_cycles(deal(block, fq), fq)
        print(f"quadrant pitches, blocks of {W}, length-sorted={sort_len}: {tot / base:.3f}")


if __name__ == "__main__":
    main()
