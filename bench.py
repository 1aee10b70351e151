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
dots all-reduced.  Rank 0 prints one JSON line.  `python bench.py --gpus N`
without a torch.distributed environment starts those N ranks itself (a child
torch.distributed.run, before this process touches the GPU) and passes rank
0's line through.
"""
import argparse
import gc
import glob
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)



def log(*a):
    print(*a, file=sys.stderr, flush=True)


def scene_config(config, N, A):
    from drtvam_amd.configs import benchy_index_matched, cylindrical_refraction, cylindrical_scattering, square_occluded
    return {2: benchy_index_matched, 3: cylindrical_refraction, 4: cylindrical_scattering,
            5: square_occluded}[config](N=N, angles=A)


def host_info():
    """CPU model, logical CPUs of the machine and of this process's affinity / OpenMP share."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = nproc
    omp = os.environ.get("OMP_NUM_THREADS")
    omp_threads = min(affinity, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else affinity
    # the reported baseline runs on every CPU of the process's affinity; the OMP_NUM_THREADS share
    # (16 per GPU on the box) is timed beside it
    return {"cpu_model": model, "nproc": nproc, "affinity": affinity, "omp_num_threads": omp, "threads": affinity,
            "omp_threads": omp_threads}


def cpu_baseline(config, N, seconds, threads, alt_threads=None):
    """Oracle (C/OpenMP port of the reference march) on a bounded angle subset of the same workload,
    plus the loss / L-BFGS vector work of an iteration (numpy, timed on one pass and scaled).
    `threads`: the OpenMP threads of the reported value (the process's affinity count); the same
    sample is also timed at `alt_threads` (the OMP_NUM_THREADS share) when that differs."""
    import numpy as np
    from oracle import oracle
    from drtvam_amd.configs import desc_from_config

    oracle.build()

    def run(na, nthreads=threads):
        cfg = scene_config(config, N, N)
        spp = cfg.get("spp", 1) if not cfg.get("regular_sampling") else 1
        d = desc_from_config(cfg)
        # the first na angles of the N-angle scene, as a sparse active set (dense order)
        pix = np.arange(na * N * N, dtype=np.uint32)
        pat = np.random.default_rng(0).uniform(0.0, 0.1, na * N * N).astype(np.float32)
        G = np.random.default_rng(1).uniform(-1.0, 1.0, (N, N, N)).astype(np.float32)
        t0 = time.perf_counter()
        _, v = oracle.forward(d, pat, active_pixels=pix, spp=spp, nthreads=nthreads)
        t1 = time.perf_counter()
        oracle.adjoint(d, G, active_pixels=pix, spp=spp, nthreads=nthreads)
        t2 = time.perf_counter()
        return t1 - t0, t2 - t1, v

    tf, ta, _ = run(2)
    per_angle = (2 * tf + ta) / 2
    na = int(max(2, min(N, seconds / max(per_angle, 1e-6))))
    tf, ta, v = run(na)
    t_march = (2 * tf + ta) * (N / na)
    # vector work of one iteration: ~3 loss passes (value + dL/dD, Armijo probes) over the film and
    # ~20 L-BFGS passes (history dots, direction, update) over the patterns (lbfgs.py:198-275), each
    # timed as one fused numpy pass a * x + y over N^3 floats
    x = np.random.default_rng(2).uniform(0, 1, N ** 3).astype(np.float32)
    y = np.empty_like(x)
    t0 = time.perf_counter()
    np.multiply(x, np.float32(0.5), out=y)
    np.add(y, x, out=y)
    t_pass = time.perf_counter() - t0
    t_vec = 23 * t_pass
    t_iter = t_march + t_vec
    alt = None
    if alt_threads and alt_threads != threads:
        tf2, ta2, _ = run(na, alt_threads)
        alt = {"threads": alt_threads, "value": 1.0 / ((2 * tf2 + ta2) * (N / na) + t_vec), "unit": "it/s",
               "sample": f"the same {na} angles: fwd {tf2:.2f}s + adj {ta2:.2f}s"}
    return {"value": 1.0 / t_iter, "unit": "it/s", "cores": threads, "kind": "port",
            "at_omp_num_threads": alt,
            "impl": "oracle/tvam_oracle.c: scalar C restatement (gcc -O3 -fopenmp, no SIMD intrinsics), "
                    "slice-private accumulation -- not Dr.Jit's LLVM backend (mitsuba/drjit are not installed)",
            "host": host_info(),
            "sample": f"{na} of {N} angles of the {N}^3 config-{config} workload: fwd {tf:.2f}s + adj {ta:.2f}s "
                      f"({v / tf / 1e6:.0f} M visits/s); iteration = (2 fwd + 1 adj) x {N}/{na} = {t_march:.1f}s "
                      f"+ 23 vector passes over {N}^3 floats (numpy, {t_pass * 1e3:.0f} ms each) = {t_vec:.2f}s"}


# Roofline of the dominant kernel, from the committed counter summary of the current build
# (tools/pmc_final.sh: tools/pmc_bench.sh + tools/roofline_summary.py -> profiles/r06/roofline_config<K>.json): the
# binding resource's bytes per launch (LDS-array cycles x 256 B, or HBM FETCH x 2 + WRITE) over
# the kernel's average launch time measured live in the timed iterations (HIP events around each
# launch on its stream, tvam_plan_kernel_time), against the 2.4 GHz spec peak (LDS 157.3 TB/s,
# HBM 8 TB/s; MI355X_MICROARCH.md).  The counter run's own launch time and fraction stay beside
# them, and every counter field can be recomputed from that one file.
ROOFLINE_DIR = os.path.join(ROOT, "profiles", "r06")


def csrc_digest():
    """sha256 (first 16 hex digits) of the kernel sources and the ABI header: the build a counter
    summary was collected on (tools/pmc_bench.sh writes it beside the counters).  A summary whose
    digest differs from the tree's describes other kernels and is reported as stale."""
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "drtvam_amd", "csrc", "*.hip"))
                   + glob.glob(os.path.join(ROOT, "drtvam_amd", "csrc", "*.h"))
                   + [os.path.join(ROOT, "drtvam_amd", "csrc", "build.sh"), os.path.join(ROOT, "include", "tvam.h")])
    for f in files:
        h.update(os.path.relpath(f, ROOT).encode())
        h.update(b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]
DOMINANT = {2: "forward: voxel-driven planar forward (two per iteration)",
            3: "forward: voxel-driven planar forward over refracted chords (two per iteration)",
            4: "forward brick march of the scattered segments (23 launches per forward, two forwards per iteration)",
            5: "forward: per-ray tile kernel of the jittered first segments (two per iteration)"}


def make_roofline(args, N, A, world, prob, visits, rays, fwd_s, adj_s, kt=None):
    """kt: (total ms, launches) of the dominant kernel over the timed iterations, from HIP events
    on its launch stream (Projection.kernel_time): `achieved` / `frac` are the counters' resource
    bytes (or instructions) per launch over that live average launch time; the counter run's own
    figures stay beside them."""
    alg_bytes = 8.0 * visits + 4.0 * rays  # forward = 8 B per visit + 4 B per ray
    info = {"fwd_call_ms": fwd_s * 1e3, "adj_call_ms": adj_s * 1e3,
            "survey_8d_model": {"alg_bytes_per_forward": alg_bytes, "rate_gbs": alg_bytes / fwd_s / 1e9,
                                "note": "per-visit dose read-modify-write model of SURVEY 8(d); the gather-form "
                                        "kernels keep the dose in registers / LDS, so this rate is no roofline"}}
    path = os.path.join(ROOFLINE_DIR, f"roofline_config{args.config}.json")
    full = N == (800 if args.config == 5 else 400) and A == N and world == 1 and not args.filter_radon
    if not (full and os.path.exists(path)):
        return {"bound": None, "achieved": None, "peak": None, "unit": "GB/s", "frac": None, "traffic": None,
                "note": "counter summaries are committed for the BASELINE sizes on one GPU", **info}
    summ = json.load(open(path))
    r = summ["roofline"]
    here = csrc_digest()
    if summ.get("csrc_sha16") != here:
        # counters of other kernel sources: no fraction is claimed for the kernels this run timed
        return {"bound": r["bound"], "achieved": None, "peak": r["peak"], "unit": r["unit"], "frac": None,
                "traffic": None, "stale": True, "kernel": summ["kernel"], "role": DOMINANT[args.config],
                "counters": os.path.relpath(path, ROOT), "counters_build": summ["build"],
                "counters_csrc_sha16": summ.get("csrc_sha16"), "csrc_sha16": here,
                "stale_frac": r["frac"], **info}
    achieved, frac, live = r["achieved"], r["frac"], None
    if kt is not None and kt[1] > 0:
        live_ns = kt[0] * 1e6 / kt[1]
        achieved = r["resource_bytes_per_launch"] / live_ns
        frac = achieved / r["peak"]
        live = {"launch_ns": live_ns, "launches": kt[1], "source": "HIP events around each launch on its stream "
                                                                   "(tvam_plan_kernel_time), timed iterations"}
    return {"bound": r["bound"], "achieved": achieved, "peak": r["peak"], "unit": r["unit"], "frac": frac,
            "live": live, "achieved_counter_run": r["achieved"], "frac_counter_run": r["frac"],
            "traffic": r["traffic"], "traffic_over_min": r["traffic_over_min"], "min_bytes": r["min_bytes"],
            "kernel": summ["kernel"], "role": DOMINANT[args.config], "launch_ns_counter_run": summ["avg_ns"],
            "clock_ghz_counter_run": summ["clock_ghz_measured"],
            "secondary": {"valu_issue_frac": r["valu_issue_frac"], "hbm_frac": r["hbm_frac"], "lds_frac": r["lds_frac"],
                          "lds_bank_conflict_frac": r["lds_bank_conflict_frac"],
                          "frac_at_measured_clock": r["frac_at_measured_clock"]},
            "counters": os.path.relpath(path, ROOT), "counters_build": summ["build"], "stale": False,
            "counters_csrc_sha16": summ["csrc_sha16"], "csrc_sha16": here, **info}


def launch_ranks(n):
    """`bench.py --gpus N` outside torch.distributed: run this same command as N ranks of a child
    torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous on a free port) and exit with
    its status.  Nothing here touches the GPU; rank 0's JSON line reaches stdout unchanged."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    log(f"bench.py --gpus {n}: launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); > 1 without WORLD_SIZE in the environment starts them itself; "
                         "under torch.distributed.run it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--prewarm", type=float, default=1.0,
                    help="seconds of untimed forward projections before the warmup iterations (GPU and host "
                         "clocks of a fresh box ramp up; the optimiser state is not touched)")
    ap.add_argument("--config", type=int, choices=[2, 3, 4, 5], default=2,
                    help="BASELINE.json configs[1] (2: index-matched, the metric's workload), configs[2] "
                         "(3: cylindrical vial, refraction) or configs[3] (4: cylindrical vial, scattering "
                         "resin, 16 jittered rays per pixel) or configs[4] (5: square vial + occluder mesh, 4 jittered rays per "
                         "pixel; use --n 800)")
    ap.add_argument("--res", "--n", dest="n", type=int, default=400,
                    help="voxels per axis = DMD pixels per axis = angles (--res under torch.distributed.run, "
                         "whose parser takes --n for its own --nnodes)")
    ap.add_argument("--angles", type=int, default=None)
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--zero-skip", action="store_true", help="skip rays whose pattern value is 0 (exact)")
    ap.add_argument("--stats", action="store_true", help="report float-fallback tiles per forward (syncs)")
    ap.add_argument("--breakdown", type=int, default=3,
                    help="iterations after the timed ones whose forward / adjoint calls are timed (fwd_ms, adj_ms)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--shard", choices=["auto", "angle", "slab"], default="auto",
                    help="multi-GPU partition: z-slabs of the film + DMD row bands (planar scenes, no dose "
                         "all-reduce; auto) or angle blocks + RCCL dose all-reduce")
    ap.add_argument("--emulate", type=str, default=None, metavar="RANK/WORLD",
                    help="time one rank's shard of a WORLD-rank run on this single GPU (no collectives; "
                         "scaling study only, never the bench line)")
    ap.add_argument("--ar-gbs", type=float, default=300.0,
                    help="--emulate with --shard angle: RCCL all-reduce bus bandwidth (GB/s) of the cost model")
    ap.add_argument("--filter-radon", action="store_true",
                    help="compact the active set to the pixels whose rays cross the target (optimize.py:143-163)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend for WORLD_SIZE > 1 (nccl = RCCL over xGMI; gloo: tests)")
    ap.add_argument("--slab-bands", type=int, default=None,
                    help="slab bands of a pipelined planar iteration (TvamProblem.direction_parts; 1: unbanded, the "
                         "full-film launches the committed counters describe)")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, form the process group, all-reduce one value and print the world "
                         "line without touching a GPU (tests of the launcher; use with --backend gloo)")
    args = ap.parse_args()

    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    import torch
    from drtvam_amd import _abi
    from drtvam_amd.optimize import TvamProblem

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}")
    if args.launch_check:
        import torch.distributed as dist
        if world > 1:
            dist.init_process_group(args.backend)
        ones = torch.ones(1, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(ones)
        if rank == 0:
            print(json.dumps({"launch_check": True, "n_gpus": world, "backend": args.backend if world > 1 else None,
                              "allreduce_ranks": int(ones.item())}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    ndev = torch.cuda.device_count()
    gpu = local % max(ndev, 1)  # one GPU per rank; ranks share a GPU only when there are fewer (tests)
    torch.cuda.set_device(gpu)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", gpu)

    N = args.n
    A = args.angles or N
    cfg = scene_config(args.config, N, A)
    cfg["tile"] = args.tile
    cfg["shard"] = args.shard
    cfg["flags"] = (0 if args.zero_skip else _abi.FLAG_NO_ZERO_SKIP) | (_abi.FLAG_FWD_STATS if args.stats else 0)
    if args.filter_radon:
        cfg["filter_radon"] = True
    if args.slab_bands is not None:
        cfg["direction_parts"] = args.slab_bands
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
    if prob.active_dense is not None:  # filter_radon: the compacted active set's entries
        prob.x0 = prob.x0[prob.active_dense].contiguous()
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
    # overlapped angle shards render a forward as slice ranges (ShardedLoop.forward): one forward =
    # the ranges from slice 0 on, timed together
    fwd_slices, orig_slices = [], getattr(prob.proj, "forward_slices", None)

    def timed_slices(*a, **k):
        if not state["on"]:
            return orig_slices(*a, **k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig_slices(*a, **k)
        e.record()
        fwd_slices.append((a[4] if len(a) > 4 else k.get("z0", 0), s, e))
        return out

    if orig_slices is not None:
        prob.proj.forward_slices = timed_slices

    t_pre = time.perf_counter()
    n_pre = 0
    while n_pre == 0 or time.perf_counter() - t_pre < args.prewarm:
        prob.forward_local(prob.x0, 0)  # this rank's projection only: no collective, state untouched
        torch.cuda.synchronize()
        n_pre += 1
        if args.prewarm <= 0:
            break
    for i in range(args.warmup):
        prob.iteration(i)
        log(f"[rank {rank}] warmup {i} loss {prob.loss_hist[-1]:.6e}")
    # as drtvam_amd.optimize.main's loop: long-lived setup objects out of the cyclic GC
    gc.collect()
    gc.freeze()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    prob.proj.kernel_time(True)  # (dominant-kernel launch events from here on; no GPU work)
    t0 = time.perf_counter()
    # step boundaries as events on the stream every launch goes to (the median of the steps)
    step_ev = [torch.cuda.Event(enable_timing=True)]
    step_ev[0].record()
    for i in range(args.warmup, args.warmup + args.steps):
        prob.iteration(i)
        step_ev.append(torch.cuda.Event(enable_timing=True))
        step_ev[-1].record()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    kt = prob.proj.kernel_time(False)
    elapsed = t1 - t0
    # the forward / adjoint call times of the line (fwd_ms / adj_ms): events around each call, taken in
    # --breakdown iterations after the timed ones (an event record between two kernels idles the GPU
    # for a few microseconds: none in the timed steps beyond the step boundaries and the dominant
    # kernel's launch events)
    state["on"] = True
    for i in range(args.warmup + args.steps, args.warmup + args.steps + args.breakdown):
        prob.iteration(i)
    torch.cuda.synchronize()
    state["on"] = False
    fwd = [s.elapsed_time(e) for s, e in fwd_ms]
    if fwd_slices:  # per forward: the sum of its slice ranges' times
        for z0, s, e in fwd_slices:
            if z0 == 0 or not fwd:
                fwd.append(0.0)
            fwd[-1] += s.elapsed_time(e)
    adj = [s.elapsed_time(e) for s, e in adj_ms]
    step_ms = sorted(a.elapsed_time(b) for a, b in zip(step_ev[:-1], step_ev[1:]))
    step_med = step_ms[len(step_ms) // 2] if len(step_ms) % 2 else 0.5 * (step_ms[len(step_ms) // 2 - 1] +
                                                                          step_ms[len(step_ms) // 2])
    fwd_avg = sum(fwd) / len(fwd) / 1e3 if fwd else float("nan")
    adj_avg = sum(adj) / len(adj) / 1e3 if adj else float("nan")
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    log(f"[rank {rank}] {args.steps} iterations in {elapsed:.3f}s; fwd {fwd_avg * 1e3:.2f} ms, adj {adj_avg * 1e3:.2f} ms, "
        f"last loss {prob.loss_hist[-1]:.6e}")

    if args.emulate:
        ew = int(args.emulate.split("/")[1])
        ms = elapsed / args.steps * 1e3
        rec = {"emulate": args.emulate, "shard": prob.shard, "config": args.config, "n": N,
               "ms_per_step": ms, "ms_per_step_median": step_med, "fwd_ms": fwd_avg * 1e3, "adj_ms": adj_avg * 1e3, "visits_per_pass": visits,
               "slices": [prob.z0, prob.z1], "rows": [prob.r0, prob.r1], "angles": [prob.a0, prob.a1],
               "device_mem_used_bytes": (lambda fr_tot: fr_tot[1] - fr_tot[0])(torch.cuda.mem_get_info(dev))}
        if prob.proj.desc.albedo != 0.0:  # scattering: the brick-bin chunking and its device memory
            rec["bins"] = prob.proj.bin_stats()
        if not prob.proj.desc.regular_sampling:
            rec["tiles"] = prob.proj.tile_stats()
        if prob.shard == "angle" and ew > 1:
            # two ring all-reduces of the full dose per iteration (main forward + line-search forward):
            # each moves 2 (W - 1) / W of the film per rank at the RCCL bus bandwidth --ar-gbs.  When the
            # projection renders slice ranges (ShardedLoop.forward_chunks), range k's all-reduce runs on
            # RCCL's stream under range k + 1's forward: only the last range's is exposed, unless the
            # all-reduce of a range outlasts the forward of the next
            fr = prob.proj.desc.film_res
            film = 4.0 * fr[0] * fr[1] * fr[2]
            ar_ms = 2 * (2.0 * (ew - 1) / ew) * film / (args.ar_gbs * 1e9) * 1e3
            zc = prob.proj.fwd_chunk
            chunks = prob.forward_chunks() or [(0, fr[2])]
            nchunk = len(chunks)
            per_fwd_ar, per_fwd_fwd = ar_ms / 2, fwd_avg * 1e3
            exposed = 2 * (per_fwd_ar / nchunk + max(0.0, (per_fwd_ar - per_fwd_fwd) * (nchunk - 1) / nchunk))
            rec.update({"allreduce_model": {"bytes_per_allreduce": film, "per_iteration": 2, "bus_gbs": args.ar_gbs,
                                            "ms_per_iteration": ar_ms, "slice_ranges": nchunk, "fwd_chunk": zc,
                                            "exposed_ms_per_iteration": exposed},
                        "ms_per_step_with_allreduce": ms + exposed,
                        "ms_per_step_without_overlap": ms + ar_ms})
        print(json.dumps(rec), flush=True)
        return
    if rank != 0:
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    # the adjoint on a dense gradient (U[-1, 1)): the timed iterations run near convergence,
    # where the thresholded loss's gradient is exactly 0 on most of the film and the adjoint skips those
    # partials and tiles (bit-identical); this is the same call with nothing to skip, untimed for `value`
    dense = None
    if world == 1 and adj:
        gd = torch.empty(tuple(prob.proj.film_shape), device=dev).uniform_(
            -1.0, 1.0, generator=torch.Generator(device=dev).manual_seed(1))
        n_act = prob.x0.numel()
        ga = orig_adj(gd, n_act, prob.active_pixels, prob.spp, 0)
        ts = []
        for _ in range(5):
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_.record()
            orig_adj(gd, n_act, prob.active_pixels, prob.spp, 0, out=ga)
            e_.record()
            torch.cuda.synchronize()
            ts.append(s_.elapsed_time(e_))
        adj_dense = sorted(ts)[len(ts) // 2]
        dense = {"adj_ms": adj_dense, "adj_ms_timed_iterations": adj_avg * 1e3,
                 "ms_per_step_model": step_med - adj_avg * 1e3 + adj_dense,
                 "note": "adjoint of a U[-1,1) gradient (no zero partials or tiles to skip), median of 5 calls; "
                         "ms_per_step_model = the median step with its adjoint replaced by this one"}
        del gd, ga
    roofline = make_roofline(args, N, A, world, prob, visits, rays, fwd_avg, adj_avg, kt)
    cpu = None
    if args.cpu_baseline == "auto" and world == 1:
        hi = host_info()
        log(f"cpu baseline ({hi['threads']} threads, and {hi['omp_threads']}; ~{args.cpu_seconds:.0f}s) ...")
        cpu = cpu_baseline(args.config, N, args.cpu_seconds, hi["threads"], hi["omp_threads"])
    result = {
        "metric": f"optimizer iterations/sec (fwd+adjoint), {N}³ voxels × {A} angles",
        "value": args.steps / elapsed,
        "unit": "it/s",
        "n_gpus": world,
        "world_size": dist.get_world_size() if dist else 1,
        "backend": (args.backend if dist else None),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        # the median of the timed steps (HIP events at the step boundaries) beside the mean
        "ms_per_step_median": step_med,
        "value_median": 1e3 / step_med,
        "ms_per_step_min_max": [step_ms[0], step_ms[-1]],
        "dense_gradient": dense,
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
                            if prob.shard == "slab" else
                            f"angle-shard x{world} + {'RCCL' if args.backend == 'nccl' else 'gloo'} dose all-reduce"),
            "shard": prob.shard if world > 1 else None,
            "zero_skip": bool(args.zero_skip), "prewarm_forwards": n_pre, "tile": prob.proj.desc.tile,
            # slab bands of the pipelined iteration (TvamProblem._iteration_pipelined; 1: unbanded)
            "slab_bands": (len(prob.opt.pipeline.parts) if getattr(prob.opt, "pipeline", None) is not None else 1),
            "filter_radon": ({"active": prob.n_filtered, "of": prob.n_global} if prob.active_pixels is not None
                             else None),
            "fwd_ms": fwd_avg * 1e3, "adj_ms": adj_avg * 1e3, "visits_per_pass": visits, "rays_per_pass": rays,
            "final_loss": prob.loss_hist[-1],
            # scattering: the last (line-search) forward's brick-bin chunks, how many the cache served
            "bins": prob.proj.bin_stats() if prob.proj.desc.albedo != 0.0 else None,
            # jittered sampling: the per-ray tile kernels' stray rays and the row walks they cost
            "tiles": prob.proj.tile_stats() if not prob.proj.desc.regular_sampling else None,
        },
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
