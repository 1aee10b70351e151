"""Benchmark: optimizer iterations/sec (fwd+adjoint), 400^3 voxels x 400 angles.

One step = one LinearLBFGS iteration of the drtvam optimize loop
(optimize.py:292-320, lbfgs.py:198-275): forward render -> thresholded loss +
dL/dD -> adjoint render -> L-BFGS two-loop -> forward render of the search
direction -> Armijo probes -> clamp.  Workload = BASELINE.json configs[1]:
index-matched scene, 400^3 voxels, 400 angles, 400x400 DMD, 1 ray/pixel,
synthetic patterns U[0, 0.1) (seed 0) and an analytic target (benchy.ply is
not available).  Every ray is marched (zero-pattern skipping disabled).

--config 3 runs BASELINE.json configs[2] instead: the same scene behind a
cylindrical glass vial (two refracting interfaces per ray); --config 4 runs
configs[3]: that vial around a scattering resin, 16 jittered rays per pixel;
--config 5 --n 800 runs configs[4]: a square vial with an occluder mesh.

Multi-GPU: one process per GPU (torch.distributed.run), angles sharded in
contiguous blocks, dose all-reduced over RCCL twice per iteration, L-BFGS
dots all-reduced.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def scene_config(config, N, A):
    from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction, cylindrical_scattering, square_occluded
    return {2: benchy_index_matched, 3: cylindrical_refraction, 4: cylindrical_scattering,
            5: square_occluded}[config](N=N, angles=A)


def cpu_baseline(config, N, seconds, threads):
    """Oracle (C/OpenMP port of the reference march) on a bounded angle subset of the same workload."""
    import numpy as np
    from oracle import oracle
    from drtvam_amd.configs import desc_from_config

    oracle.build()

    def run(na):
        cfg = scene_config(config, N, N)
        spp = cfg.get("spp", 1) if not cfg.get("regular_sampling") else 1
        d = desc_from_config(cfg)
        # the first na angles of the N-angle scene, as a sparse active set (dense order)
        pix = np.arange(na * N * N, dtype=np.uint32)
        pat = np.random.default_rng(0).uniform(0.0, 0.1, na * N * N).astype(np.float32)
        G = np.random.default_rng(1).uniform(-1.0, 1.0, (N, N, N)).astype(np.float32)
        t0 = time.perf_counter()
        _, v = oracle.forward(d, pat, active_pixels=pix, spp=spp, nthreads=threads)
        t1 = time.perf_counter()
        oracle.adjoint(d, G, active_pixels=pix, spp=spp, nthreads=threads)
        t2 = time.perf_counter()
        return t1 - t0, t2 - t1, v

    tf, ta, _ = run(2)
    per_angle = (2 * tf + ta) / 2
    na = int(max(2, min(N, seconds / max(per_angle, 1e-6))))
    tf, ta, v = run(na)
    t_iter = (2 * tf + ta) * (N / na)
    return {"value": 1.0 / t_iter, "unit": "it/s", "cores": threads, "kind": "port",
            "sample": f"oracle/tvam_oracle.c (C/OpenMP, {threads} threads, slice-private accumulation) on {na} of {N} "
                      f"angles of the {N}^3 config-{config} workload: fwd {tf:.2f}s + adj {ta:.2f}s, "
                      f"{v / tf / 1e6:.0f} M visits/s; iteration = 2 fwd + 1 adj scaled to {N} angles "
                      f"(loss/L-BFGS vector work not included)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, choices=[2, 3, 4, 5], default=2,
                    help="BASELINE.json configs[1] (2: index-matched, the metric's workload), configs[2] "
                         "(3: cylindrical vial, refraction) or configs[3] (4: cylindrical vial, scattering "
                         "resin, 16 jittered rays per pixel) or configs[4] (5: square vial + occluder mesh, 4 jittered rays per "
                         "pixel; use --n 800)")
    ap.add_argument("--n", type=int, default=400, help="voxels per axis = DMD pixels per axis = angles")
    ap.add_argument("--angles", type=int, default=None)
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--zero-skip", action="store_true", help="skip rays whose pattern value is 0 (exact)")
    ap.add_argument("--stats", action="store_true", help="report float-fallback tiles per forward (syncs)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--shard", choices=["auto", "angle", "slab"], default="auto",
                    help="multi-GPU partition: z-slabs of the film + DMD row bands (planar scenes, no dose "
                         "all-reduce; auto) or angle blocks + RCCL dose all-reduce")
    ap.add_argument("--emulate", type=str, default=None, metavar="RANK/WORLD",
                    help="time one rank's shard of a WORLD-rank run on this single GPU (no collectives; "
                         "scaling study only, never the bench line)")
    args = ap.parse_args()

    import torch
    from drtvam_amd import _abi
    from drtvam_amd.optimize import TvamProblem

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    N = args.n
    A = args.angles or N
    cfg = scene_config(args.config, N, A)
    cfg["tile"] = args.tile
    cfg["shard"] = args.shard
    cfg["flags"] = (0 if args.zero_skip else _abi.FLAG_NO_ZERO_SKIP) | (_abi.FLAG_FWD_STATS if args.stats else 0)
    t_setup = time.perf_counter()
    if args.emulate:
        er, ew = (int(v) for v in args.emulate.split("/"))
        prob = TvamProblem(cfg, device=dev, rank=er, world_size=ew)
        rank = er
    else:
        prob = TvamProblem(cfg, device=dev)
    g = torch.Generator().manual_seed(0)
    full = torch.rand(prob.n_global, generator=g) * 0.1
    prob.x0 = prob.local_from_global(full)
    del full
    visits = prob.proj.count_visits(prob.spp, 0)
    rays = prob.n_local * prob.spp
    log(f"[rank {rank}] setup {time.perf_counter() - t_setup:.1f}s, shard {prob.shard}: angles [{prob.a0},{prob.a1}), "
        f"slices [{prob.z0},{prob.z1}), rows [{prob.r0},{prob.r1}), "
        f"visits/pass {visits:.3e}, rays {rays:.3e}")

    # HIP-event timing of the dominant kernels (forward / adjoint projection) on their launch stream
    fwd_ms, adj_ms = [], []
    state = {"on": False}
    orig_fwd, orig_adj = prob.proj.forward, prob.proj.adjoint

    def timed(fn, acc):
        def wrap(*a, **k):
            if not state["on"]:
                return fn(*a, **k)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = fn(*a, **k)
            e.record()
            acc.append((s, e))
            if args.stats and acc is fwd_ms:
                log(f"  forward: {prob.proj.fallback_tiles()} float-fallback tiles, "
                    f"{s.elapsed_time(e):.2f} ms")
            return out
        return wrap

    prob.proj.forward = timed(orig_fwd, fwd_ms)
    prob.proj.adjoint = timed(orig_adj, adj_ms)

    for i in range(args.warmup):
        prob.iteration(i)
        log(f"[rank {rank}] warmup {i} loss {prob.loss_hist[-1]:.6e}")
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    state["on"] = True
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        prob.iteration(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    state["on"] = False
    elapsed = t1 - t0
    fwd = [s.elapsed_time(e) for s, e in fwd_ms]
    adj = [s.elapsed_time(e) for s, e in adj_ms]
    fwd_avg = sum(fwd) / len(fwd) / 1e3
    adj_avg = sum(adj) / len(adj) / 1e3 if adj else float("nan")
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    log(f"[rank {rank}] {args.steps} iterations in {elapsed:.3f}s; fwd {fwd_avg * 1e3:.2f} ms, adj {adj_avg * 1e3:.2f} ms, "
        f"last loss {prob.loss_hist[-1]:.6e}")

    if args.emulate:
        print(json.dumps({"emulate": args.emulate, "shard": prob.shard, "ms_per_step": elapsed / args.steps * 1e3,
                          "fwd_ms": fwd_avg * 1e3, "adj_ms": adj_avg * 1e3, "visits_per_pass": visits,
                          "slices": [prob.z0, prob.z1], "rows": [prob.r0, prob.r1],
                          "angles": [prob.a0, prob.a1]}), flush=True)
        return
    if rank != 0:
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    alg_bytes = 8.0 * visits + 4.0 * rays  # forward = 8 B per visit + 4 B per ray
    achieved = alg_bytes / fwd_avg / 1e9
    # HBM bytes per forward launch from the committed rocprofv3 PMC passes
    # (profiles/pmc_traffic.json, made by tools/profile_round.sh + tools/summarize_profile.py)
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if N == 400 and A == 400 and world == 1 and args.config == 2 and os.path.exists(tpath):
        traffic = json.load(open(tpath))["per_launch"]["forward"]["hbm_bytes"]
    cpu = None
    if args.cpu_baseline == "auto" and world == 1:
        threads = min(16, os.cpu_count() or 1)
        log(f"cpu baseline ({threads} threads, ~{args.cpu_seconds:.0f}s) ...")
        cpu = cpu_baseline(args.config, N, args.cpu_seconds, threads)
    result = {
        "metric": "optimizer iterations/sec (fwd+adjoint), 400³ voxels × 400 angles",
        "value": args.steps / elapsed,
        "unit": "it/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": (f"config2: index-matched, {N}^3 voxels, {A} angles, {N}x{N} DMD, 1 ray/px, regular sampling"
                         if args.config == 2 else
                         f"config3: cylindrical vial (glass r 8/9 mm, n 1.54 | resin n 1.40), {N}^3 voxels, {A} angles, "
                         f"{N}x{N} DMD, 1 ray/px, regular sampling" if args.config == 3 else
                         f"config4: cylindrical vial, scattering resin (sigma_t 0.1/mm, albedo 0.5, Rayleigh), "
                         f"{N}^3 voxels, {A} angles, {N}x{N} DMD, {prob.spp} jittered rays/px" if args.config == 4 else
                         f"config5: square vial + occluder mesh (box_hole_occlusion scene), {N}^3 voxels, {A} angles, "
                         f"{N}x{N} DMD, {prob.spp} jittered rays/px"),
            "voxels": N ** 3, "angles": A, "dmd": [N, N], "spp": prob.spp, "sigma_t": cfg["vial"]["medium"]["extinction"],
            "parallelism": ("single GPU" if world == 1 else
                            f"z-slab x{world} (film slabs + DMD row bands, scalar all-reduces only)"
                            if prob.shard == "slab" else f"angle-shard x{world} + RCCL dose all-reduce"),
            "zero_skip": bool(args.zero_skip), "tile": prob.proj.desc.tile,
            "fwd_ms": fwd_avg * 1e3, "adj_ms": adj_avg * 1e3, "visits_per_pass": visits, "rays_per_pass": rays,
            "final_loss": prob.loss_hist[-1],
        },
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "tvam_fwd_planar_kernel" if prob.proj.planar_forward else "tvam_tile_kernel<FWD>",
                     "alg_bytes_per_launch": alg_bytes,
                     "note": "SURVEY 8(d) algorithmic bytes (per-visit dose RMW); the LDS / register-resident "
                             "kernels move far fewer real bytes, so frac > 1 means past the naive HBM roofline "
                             "(the real limit is VALU / LDS issue, DESIGN.md)"},
        "cpu_baseline": cpu,
    }
    print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
