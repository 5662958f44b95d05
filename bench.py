"""Benchmark: batched 12-var contact-force QP solves/s on MI355X (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

Workload = BASELINE.json configs[1]: a batch of 1 024 identical-sparsity C1
contact-force QPs (12 vars / 20 ineq / 6 eq) per GPU.  One step =
one batched IPM solve (kkt_initialize + QP_SOLVE) of this rank's
resident batch followed by the device-side argmin; for N > 1 the per-rank
winners are exchanged with one RCCL all_gather (config 5's argmin gather:
qpb_argmin_allgather, the library's C ABI, on a second stream).
Shards are independent (weak scaling): rank r owns QP ids [r*B, (r+1)*B);
config 5 (65 536 QPs over 8 GPUs) is `--gpus 8 --batch 8192`.

At this batch size qpb_solve runs the row kernel (four QPs per wavefront).
Beside the headline, rank 0 of a 1-GPU run also measures a 2^20-QP batch
(working set ~2 GB, far above the 256 MB Infinity Cache) as `large_batch`, the
HBM-scale throughput figure; configs[2] (4 gait patterns, 4 streams) as
`mixed_patterns`; and under `shapes` configs[3] (MPC horizon, N = 380, tree
kernel) and the controller's own 30/68/18 stance QP, each next to the
reference qpSWIFT on the host cores.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1024, help="QPs per GPU per step (configs[1]: 1024)")
    ap.add_argument("--large-batch", type=int, default=1 << 20,
                    help="QPs of the secondary large-batch leg (1-GPU runs; 0 = skip)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "lane", "wave", "wave1", "auto1"])
    ap.add_argument("--no-mixed", dest="mixed", action="store_false",
                    help="skip the configs[2] leg (4 gait patterns x 1024 QPs)")
    ap.add_argument("--no-shapes", dest="shapes", action="store_false",
                    help="skip the configs[3] (MPC) and controller-shape legs")
    ap.add_argument("--tol", type=float, default=1e-6)
    ap.add_argument("--exact", action="store_true", help="bench the bit-faithful kernel")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-sample", type=int, default=65536)
    ap.add_argument("--cpu-passes", type=int, default=10)
    ap.add_argument("--dry-run", action="store_true",
                    help="launch the ranks, join a gloo group and report each rank's env and shard, "
                         "then stop before the first GPU call (CPU test of the --gpus N launcher)")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def count_gpus_in_child() -> int:
    """Visible GPUs, counted by a throwaway child process: whatever HIP (or amdsmi)
    initialisation the count needs happens there, so the launcher itself never loads
    the HIP runtime -- a parent that touched the GPU and then spawns ranks is the
    pattern this pool refuses.  -1 when the child fails."""
    import subprocess
    try:
        r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True, timeout=600)
        return int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else -1
    except Exception:
        return -1


def _parent_maps_report():
    """QPB_BENCH_PARENT_MAPS=<file>: the launcher writes the shared objects mapped into
    its own process (tests/test_multi.py checks that no HIP runtime is among them)."""
    out = os.environ.get("QPB_BENCH_PARENT_MAPS")
    if not out:
        return
    libs = set()
    with open("/proc/self/maps") as f:
        for ln in f:
            parts = ln.split()
            if len(parts) >= 6 and ".so" in parts[-1]:
                libs.add(os.path.basename(parts[-1]))
    with open(out, "w") as f:
        json.dump({"pid": os.getpid(), "libs": sorted(libs),
                   "torch_imported": "torch" in sys.modules}, f)


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes of this
    script (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT
    set as torch.distributed.run sets them) and return the worst exit code.  This
    process never touches the GPU and never imports torch: the device count comes from
    a throwaway child (count_gpus_in_child), and it refuses to run fewer ranks than
    asked.  Rank 0 prints the JSON line; every rank's stderr passes through."""
    import subprocess
    n = args.gpus
    if not args.dry_run:
        have = count_gpus_in_child()
        if have < n:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {have}", file=sys.stderr)
            return 2
    port = int(os.environ.get("MASTER_PORT", 0)) or _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    _parent_maps_report()
    bad = [c for c in codes if c != 0]
    if bad:
        print(f"bench.py: rank exit codes {codes}", file=sys.stderr)
        return bad[0] if bad[0] > 0 else 1
    return 0


def dry_run(args, rank, world, local) -> None:
    """The rank's view of the launch, exchanged over gloo: env, device index and the
    QP ids it would own.  Stops before any GPU call."""
    import torch
    import torch.distributed as dist
    from apf_quadruped_amd.shard import shard_range
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(rank, world, args.batch)
    mine = torch.tensor([rank, local, world, lo, hi], dtype=torch.int64)
    if world > 1:
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
    else:
        parts = [mine]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "gpus_arg": args.gpus,
                          "ranks": [dict(zip(("rank", "local_rank", "world", "lo", "hi"), p.tolist()))
                                    for p in parts],
                          "master": [os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")]}))
    if world > 1:
        dist.destroy_process_group()


def make_shard(plan, seed, q0, B, chunk=65536, gen=None):
    """Synthetic QPs [q0, q0+B) (C1 unless `gen(ids)` is given) packed in the
    plan's tiled layout (host)."""
    from apf_quadruped_amd import workloads as W
    parts = {k: [] for k in ("P", "A", "G", "c", "h", "b")}
    for s in range(0, B, chunk):
        ids = np.arange(q0 + s, q0 + min(B, s + chunk))
        d = gen(ids) if gen is not None else W.contact_force_qp(seed, ids)
        v = plan.pack(d["P"], d["A"], d["G"], d["c"], d["h"], d["b"])
        for k in parts:
            parts[k].append(v[k])
    return {k: np.concatenate(v) for k, v in parts.items()}


def flops_per_qp(info, iters):
    """Algorithmic FP64 flops of one solve (FMA = 2), SURVEY §8d accounting."""
    n, m, p, N, lnz = info.n, info.m, info.p, info.N, info.lnz
    fac = 2 * info.fac_updates + 3 * info.fac_divs
    solve = 4 * lnz + N
    resid = 2 * (2 * info.nnzP + 2 * info.nnzG + 2 * info.nnzA) + 2 * (n + m + p)
    vec = 30 * m + 10 * (n + p)
    per_it = fac + 2 * solve + resid + vec
    return (fac + solve + 2 * info.nnzG) + iters * per_it + resid


def host_cpus():
    """The host cores this process can run on: the affinity set, capped by the
    cgroup CPU quota when one is set (a GPU box shares its host: os.cpu_count()
    shows the whole machine, the quota is this job's share), plus the CPU model."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    use = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return dict(threads=use, affinity_cpus=aff, nproc=os.cpu_count(), cgroup_quota_cpus=quota, model=model)


def cpu_baseline(seed, sample, passes, tol, gen=None, label="C1"):
    """Reference qpSWIFT on ALL host cores this process may use (host_cpus):
    oracle/_ref (the reference's own C sources compiled by `make -C oracle ref`
    in the build container) when present, else the oracle restatement ("port").
    gen(ids) -> dense QP dict (default: C1 contact-force QPs)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from apf_quadruped_amd import workloads as W
    hc = host_cpus()
    threads = hc["threads"]
    d = gen(np.arange(sample)) if gen is not None else W.contact_force_qp(seed, np.arange(sample))
    n, m, p = int(d["n"]), int(d["m"]), int(d["p"])
    P, A, G = W.to_colmajor(d["P"]), W.to_colmajor(d["A"]), W.to_colmajor(d["G"])
    c, h, b = (np.ascontiguousarray(d[k]) for k in ("c", "h", "b"))
    x = np.zeros((sample, n)); flags = np.zeros(sample, np.int64); iters = np.zeros(sample, np.int64)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    lp = lambda a: a.ctypes.data_as(C.POINTER(C.c_long))
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libref_batch.so")
    if os.path.exists(ref_so):
        L = C.CDLL(ref_so)
        L.ref_solve_dense_batch.argtypes = [C.c_long] * 4 + [C.POINTER(C.c_double)] * 6 + \
            [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_long), C.POINTER(C.c_long), C.c_int]
        run = lambda: L.ref_solve_dense_batch(sample, n, m, p, dp(P), dp(A), dp(G), dp(c), dp(h), dp(b),
                                              tol, dp(x), lp(flags), lp(iters), threads)
        kind = "reference"
    else:
        from oracle_py import Oracle
        o = Oracle()
        run = lambda: o.lib.oracle_solve_dense_batch(sample, n, m, p, dp(P), dp(A), dp(G), dp(c), dp(h),
                                                     dp(b), None, tol, tol, 100, dp(x), lp(flags), lp(iters),
                                                     threads)
        kind = "port"
    run()                                   # warm caches / page in
    t0 = time.perf_counter()
    for _ in range(passes):
        run()
    dt = time.perf_counter() - t0
    return dict(value=sample * passes / dt, unit="QP solves/s", cores=threads, kind=kind,
                sample=f"{sample} {label} QPs x {passes} passes, setup+solve per QP (QP_SETUP_dense + QP_SOLVE "
                       f"+ QP_CLEANUP_dense, AMD ordering), tol {tol:g}, {threads} threads, {dt:.2f} s wall",
                build=("oracle/Makefile `ref`: reference qpSWIFT C sources, gcc -O2" if kind == "reference"
                       else "oracle/qpswift_oracle.c restatement, gcc -O2"),
                host={k: hc[k] for k in ("affinity_cpus", "nproc", "cgroup_quota_cpus", "model")},
                mean_iters=float(iters.mean()), optimal_frac=float((flags == 0).mean()))


def shape_leg(name, gen, B, tol, dev, steps=50, warmup=5, cpu=None):
    """One non-headline workload on one GPU: B QPs of `gen`'s shape per launch
    (solve + argmin per step), kernel duration from HIP events, algorithmic-byte
    roofline, and (cpu = (sample, passes)) the reference on the host cores."""
    from apf_quadruped_amd.batch import Plan
    d0 = gen(np.arange(1))
    plan = Plan.from_dense(d0["n"], d0["m"], d0["p"], d0["P"][0], d0["A"][0], d0["G"][0])
    plan.compile()
    el, km, out, _ = run_leg(plan, B, steps, warmup, tol, dev, 0, 1, 0, gather=False, gen=gen)
    bpq = plan.bytes_per_qp()
    ach = bpq * B / (km * 1e-3) / 1e9
    kn = plan.kernel_name(B)
    res = {"workload": name, "batch": B, "value": B * steps / el, "unit": "QP solves/s",
           "ms_per_step": el * 1e3 / steps, "kernel": kn, "kernel_ms": km, "kernel_qps": B / (km * 1e-3),
           "kkt_N": plan.info.N, "nnz_L": plan.info.lnz,
           "roofline": {"bound": measured_bound(kn, B), "roofline_ref": "hbm", "achieved": ach,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": ach / HBM_PEAK_GBS, "traffic": traffic_for(kn, B), "bytes_per_qp": bpq},
           "mean_iters": float(out["iters"].float().mean().item()),
           "optimal_frac": float((out["flag"] == 0).float().mean().item())}
    if cpu is not None:
        res["cpu_baseline"] = cpu_baseline(0, cpu[0], cpu[1], tol, gen=gen, label=name)
    return res


def run_leg(plan, B, steps, warmup, tol, dev, rank, world, seed, gather=True, gen=None, info=None):
    """Timed loop of `steps` steps (solve + argmin [+ all_gather]) on resident
    inputs.  Returns (wall seconds max over ranks, mean kernel ms max over
    ranks, outputs, gathered winners); `info` (a dict) receives the gather path."""
    import torch
    import torch.distributed as dist
    from apf_quadruped_amd.shard import make_argmin_gather, shard_range
    base = shard_range(rank, world, B)[0]
    host = make_shard(plan, seed, base, B, chunk=65536 if gen is None else 1024, gen=gen)
    vals = {k: torch.from_numpy(v).to(dev) for k, v in host.items()}
    del host
    coll = gather and world > 1
    nbuf = 2 if coll else 1
    # outputs and the rank's {fval, index} are double-buffered when the gather runs:
    # step i solves into set i % 2 while step i-1's gather may still read the other
    outs = [plan.alloc_outputs(B, device=dev) for _ in range(nbuf)]
    bests = [torch.zeros(2, dtype=torch.float64, device=dev) for _ in range(nbuf)]
    n = plan.n
    stream = torch.cuda.current_stream(dev)
    # one step = qpb_solve_best: the batched solve and the argmin {fval, index}
    # (inside the solve launch for the row kernel -- its last wave reduces the
    # per-wave partials -- else a separate single-block launch on the same stream)
    solves = [plan.launcher(vals, outs[k], B, reltol=tol, abstol=tol, stream=stream, best=bests[k])
              for k in range(nbuf)]
    if coll:
        # the argmin gather through the C ABI: qpb_argmin_allgather =
        # payload kernel + ncclAllGather of 16 + 8n B per rank (RCCL, xGMI) + device
        # reduce, on its own stream so it overlaps the next step's solve
        # (every rank takes the same path: the ranks agree on qpb_comm_init's outcome)
        ag, ginfo = make_argmin_gather(rank, world, dev)
        if ginfo["init_error"]:
            print(f"[rank {rank}] qpb_comm_init failed ({ginfo['init_error']}); torch all_gather fallback",
                  file=sys.stderr)
        if info is not None:
            info.update(ginfo)
        gs = torch.cuda.Stream(dev)
        winners = [torch.zeros(2 + n, dtype=torch.float64, device=dev) for _ in range(nbuf)]
        solved = [torch.cuda.Event() for _ in range(nbuf)]
        gathered_ev = [None] * nbuf

    def step(i):
        k = i % nbuf
        if not coll:
            solves[k]()
            return
        if gathered_ev[k] is not None:
            stream.wait_event(gathered_ev[k])     # step i-2's gather has read outs[k]
        solves[k]()
        solved[k].record(stream)
        gs.wait_event(solved[k])
        ag.gather(bests[k], outs[k]["x"], n, B, base, winners[k], gs)
        if gathered_ev[k] is None:
            gathered_ev[k] = torch.cuda.Event()
        gathered_ev[k].record(gs)

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # kernel duration: one HIP event pair on the launch stream around kev further
    # back-to-back launches (GPU-bound: a launch is queued faster than the kernel
    # runs), so the average is the kernel plus the ~1 us dispatch gap -- an upper
    # bound that rocprof's per-dispatch durations (profiles/) bracket from below.
    # Per-launch event pairs would add their own ~3 us; per-step events inside the
    # timed loop cost ~8 us of host time per step, so they stay out of it.
    kev = min(steps, 50)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(kev):
        solves[0]()
    e1.record(stream)
    torch.cuda.synchronize()
    kern_ms = e0.elapsed_time(e1) / kev
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    last = (steps - 1) % nbuf
    if coll:
        result = winners[last].clone()
        ag.close()
    else:
        result = bests[last].clone()
    return elapsed, kern_ms, outs[last], result


def mixed_patterns_leg(tol, dev, per_pattern=1024, steps=50, warmup=5):
    """configs[2]: 4 x 1024 QPs, one sparsity pattern per gait phase (stance4,
    trot BL+FR, trot BR+FL, crawl), bucketed into one plan each.  A step is ONE
    launch of the plans' group kernel (qpb_group_solve: every pattern's QPs in
    their own blocks + the argmin over all 4 096 in the same launch).  For
    comparison, `per_plan_streams` times the same work as four qpb_solve_best
    launches on four streams (joined by events)."""
    import torch
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import Plan, PlanGroup
    legs = []
    for k, name in enumerate(("stance4", "trot_blfr", "trot_brfl", "crawl_blflfr")):
        stance = W.STANCE_SETS[name]
        gen = lambda ids, st=stance: W.contact_force_qp(plans.SEED + 3, ids, stance=st, feasible_wrench=True)
        d0 = gen(np.arange(1))
        plan = Plan.from_dense(12, d0["m"], 6, d0["P"][0], d0["A"][0], d0["G"][0])
        plan.compile()
        host = make_shard(plan, plans.SEED + 3, k * per_pattern, per_pattern, gen=gen)
        vals = {kk: torch.from_numpy(v).to(dev) for kk, v in host.items()}
        out = plan.alloc_outputs(per_pattern, device=dev)
        best = torch.zeros(2, dtype=torch.float64, device=dev)
        st = torch.cuda.Stream(dev)
        legs.append(dict(name=name, plan=plan, out=out, stream=st, vals=vals,
                         solve=plan.launcher(vals, out, per_pattern, reltol=tol, abstol=tol, stream=st, best=best)))
    main = torch.cuda.current_stream(dev)
    group = PlanGroup([L["plan"] for L in legs])
    group.compile()
    gbest = torch.zeros(2, dtype=torch.float64, device=dev)
    gsolve = group.launcher([L["vals"] for L in legs], [L["out"] for L in legs], [per_pattern] * len(legs),
                            reltol=tol, abstol=tol, stream=main, best=gbest)

    def streams_step():
        ev = torch.cuda.Event()
        ev.record(main)
        for L in legs:
            L["stream"].wait_event(ev)
            L["solve"]()
        for L in legs:
            e = torch.cuda.Event()
            e.record(L["stream"])
            main.wait_event(e)

    def timed(step):
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    el_streams = timed(streams_step)
    el = timed(gsolve)
    # kernel duration of the group launch (events on its stream, outside the timed loop)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for _ in range(20):
        gsolve()
    e1.record(main)
    torch.cuda.synchronize()
    kms = e0.elapsed_time(e1) / 20
    B = per_pattern * len(legs)
    return {"batch": B, "patterns": [L["name"] for L in legs], "value": B * steps / el,
            "ms_per_step": el * 1e3 / steps, "kernel": group.kernel_name(), "kernel_ms": kms,
            "traffic": traffic_for(group.kernel_name()),
            "algorithmic_bytes_per_launch": sum(L["plan"].bytes_per_qp() * per_pattern for L in legs),
            "member_kernels": [L["plan"].kernel_name(per_pattern) for L in legs],
            "kkt_N": [L["plan"].info.N for L in legs],
            "per_plan_streams": {"value": B * steps / el_streams, "ms_per_step": el_streams * 1e3 / steps},
            "optimal_frac": float(np.mean([(L["out"]["flag"] == 0).float().mean().item() for L in legs]))}


def trace_leg(tol, dev, steps=20, warmup=3):
    """Recorded Gazebo traces (traces.py): every logged step of
    the reference's DogBot runs with >= 2 feet on the ground, as contact-force QPs
    assembled on the device from the recorded foot positions / CoM wrench
    (qpb_assemble_contact, outside the timed loop) and solved as ONE group launch
    (one member per stance set) + argmin.  Real gaits include infeasible
    two-foot phases: those QPs run to maxit (100 iterations), as in qpSWIFT."""
    import torch
    from apf_quadruped_amd import traces, workloads as W
    from apf_quadruped_amd.batch import PlanGroup, to_tiled
    batches = traces.stance_batches()
    plans_ = traces.stance_plans(batches)
    vals, outs, Bs = [], [], []
    for (mask, r, Wr), plan in zip(batches, plans_):
        B = len(r)
        feet = torch.from_numpy(to_tiled(r.reshape(B, 12))).to(dev)
        wrench = torch.from_numpy(to_tiled(Wr)).to(dev)
        vals.append(plan.assemble_contact(feet, wrench, stance=mask, mu=W.MU, B=B))
        outs.append(plan.alloc_outputs(B, device=dev))
        Bs.append(B)
    grp = PlanGroup(plans_)
    grp.compile()
    best = torch.zeros(2, dtype=torch.float64, device=dev)
    go = grp.launcher(vals, outs, Bs, reltol=tol, abstol=tol, best=best)
    for _ in range(warmup):
        go()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        go()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    flags = torch.cat([o["flag"][:B] for o, B in zip(outs, Bs)])
    iters = torch.cat([o["iters"][:B] for o, B in zip(outs, Bs)]).float()
    Bt = sum(Bs)
    maxit_frac = float((flags == 2).float().mean().item())
    return {"workload": f"recorded Gazebo traces: {Bt} logged steps of 5 DogBot runs, {len(Bs)} stance sets, one group launch",
            "label": f"maxit-dominated: {100 * maxit_frac:.0f} % of the QPs are infeasible two-foot phases that run to "
                     "maxit (100 iterations, QP_MAXIT) as in qpSWIFT; the rate measures that grinding, not the solver",
            "maxit_frac": maxit_frac,
            "batch": Bt, "value": Bt * steps / el, "unit": "QP solves/s", "ms_per_step": el * 1e3 / steps,
            "kernel": grp.kernel_name(), "traffic": traffic_for(grp.kernel_name()),
            "stance_sets": [int(b[0]) for b in batches],
            "optimal_frac": float((flags == 0).float().mean().item()), "mean_iters": float(iters.mean().item()),
            "max_iters": int(iters.max().item())}


def apf_leg(tol, dev, B=8192, steps=50, warmup=5):
    """Config 5's per-GPU share (8 192 APF-sampled contact-force QPs) end to end on
    the device: each step assembles the QPs from the robot terms
    (qpb_assemble_contact: 18 doubles per QP in) and solves them
    with the argmin (qpb_solve_best)."""
    import torch
    from apf_quadruped_amd import plans, workloads as W
    from apf_quadruped_amd.batch import to_tiled
    plan = plans.standard_plan("c1")
    plan.compile()
    ids = np.arange(B)
    r, Wr = W.contact_inputs(plans.SEED + 5, ids)
    feet = torch.from_numpy(to_tiled(r.reshape(B, 12))).to(dev)
    wrench = torch.from_numpy(to_tiled(Wr)).to(dev)
    vals = plan.assemble_contact(feet, wrench, stance=0xF, mu=W.MU, B=B)
    out = plan.alloc_outputs(B, device=dev)
    best = torch.zeros(2, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    solve = plan.launcher(vals, out, B, reltol=tol, abstol=tol, stream=stream, best=best)

    def step():
        plan.assemble_contact(feet, wrench, stance=0xF, mu=W.MU, B=B, out=vals, stream=stream)
        solve()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"workload": f"configs[4] per-GPU share: {B} APF-sampled C1 QPs assembled on the device + solved + argmin",
            "batch": B, "value": B * steps / el, "unit": "QP solves/s", "ms_per_step": el * 1e3 / steps,
            "input_bytes_per_qp": 18 * 8, "kernel": plan.kernel_name(B), "traffic": traffic_for(plan.kernel_name(B), B),
            "optimal_frac": float((out["flag"] == 0).float().mean().item())}


def _sq_record(kname, B):
    """The newest SQ-counter summary for this kernel at this batch (profiles/r0N_sq_*.json,
    scripts/gpu_sq*.sh + scripts/sq_summary.py): row-kernel files key "B=<B>", the tree
    and band files "B=<B>", the wave and wide-row files "<kernel> B=<B>"."""
    kind = next((k for k in ("rowx", "row", "tree", "wave", "band") if kname.startswith("qpb_" + k)), None)
    if kind is None:
        return None, None
    for rnd in ("r06", "r05", "r04", "r03"):
        name = f"{rnd}_sq_{kind}.json"
        f = os.path.join(ROOT, "profiles", name)
        if not os.path.exists(f):
            continue
        d = json.load(open(f))
        r = d.get(f"{kname} B={B}") or (d.get(f"B={B}") if kind not in ("wave", "rowx") else None)
        if r:
            return r, "profiles/" + name
    return None, None


def fp64_issued(kname, B):
    """FP64 actually issued (SQ_INSTS_VALU_FMA_F64 lane-ops, from the same SQ summary) next
    to the algorithmic fraction, so the lanes' redundant work is visible in the line."""
    r, src = _sq_record(kname, B)
    if not r or "fp64_issue_frac_of_peak" not in r:
        return {"issued_frac": None}
    return {"issued_frac": r["fp64_issue_frac_of_peak"],
            "issued_lane_fma_per_qp": r.get("per_qp", {}).get("fma_f64_lane_ops"), "issued_source": src}


def measured_bound(kname, B):
    """roofline.bound from the measured limiter, not from the roofline the fraction is
    quoted against: "valu_issue" when the SIMDs' VALU is busy >= 60 % of the launch,
    "latency" when it is not (a wave's dependency chain, few waves per SIMD),
    "unmeasured" without counters for this kernel and batch.  (HBM never binds here:
    traffic is <= 1.6x the algorithmic bytes at <= 10 % of peak.)"""
    r, _ = _sq_record(kname, B)
    if not r or r.get("simd_valu_busy") is None:
        return "unmeasured"
    return "valu_issue" if r["simd_valu_busy"] >= 0.6 else "latency"


def limiter_for(B):
    """What the SQ counters say bounds the row kernel at this batch
    (the newest profiles/r0N_sq_row.json; scripts/gpu_sq.sh + scripts/sq_summary.py)."""
    name = next((n for n in ("r06_sq_row.json", "r05_sq_row.json", "r04_sq_row.json", "r03_sq_row.json")
                 if os.path.exists(os.path.join(ROOT, "profiles", n))), None)
    if name is None:
        return None
    f = os.path.join(ROOT, "profiles", name)
    r = json.load(open(f)).get(f"B={B}")
    if not r:
        return None
    fr = r["frac_of_wave_cycles"]
    return {"kind": r.get("kind", "VALU issue + LDS/memory latency (neither HBM nor FP64 peak)"),
            "valu_active_frac": fr["valu_active"], "waitcnt_frac": fr["wait_any (s_waitcnt: LDS / memory)"],
            "waves_per_simd": r["waves_per_simd_avg"], "fp64_lane_fma_per_qp": r["per_qp"]["fma_f64_lane_ops"],
            "source": "profiles/" + name}


def controller_apf_leg(dev, K=8192, steps=20, warmup=3, order="amd"):
    """The controller's own call, batched: one tick of one robot,
    K APF-sampled candidate targets (main.cpp:1263-1422).  A step = the candidates'
    desired wrenches (qpb_apf_wrench) + their 30/68/18 stance QPs assembled from the
    robot terms (qpb_assemble_controller, shared terms, main.cpp:1471-1647) + one
    solve with the fused argmin (qpb_solve_best) at the controller's tol 1e-2.
    order "amd": the reference's AMD ordering (QPB_ORDER_AMD: the pivots of qpSWIFT's
    Permut = NULL, so the answers are the reference's to 1e-6; one QP per wavefront);
    "own": the plan's leaves-first ordering (the wide row kernel, four QPs per
    wavefront; the same QPs, the factor in another pivot order)."""
    import torch
    from apf_quadruped_amd import workloads as W
    from apf_quadruped_amd.batch import Plan, apf_state, apf_wrench, to_tiled
    d = W.controller_qp(0xD06B07 + 30, np.arange(1))
    plan = Plan.from_dense(30, 68, 18, d["P"][0], d["A"][0], d["G"][0], order=order)
    plan.compile()
    st = apf_state(**W.apf_tick_state())      # a plausible synthetic tick state
    rng = np.random.default_rng(11)
    targets = torch.from_numpy(to_tiled(np.asarray(st.com[:2])[None] + rng.uniform(-0.6, 0.6, (K, 2)))).to(dev)
    terms = torch.from_numpy(W.pack_terms(W.controller_terms(0xD06B07 + 43, np.arange(1)))[0].copy()).to(dev)
    stream = torch.cuda.current_stream(dev)
    wd = apf_wrench(st, targets, K=K, stream=stream)
    vals = plan.assemble_controller(terms, B=K, shared=True, wdes=wd, stream=stream)
    out = plan.alloc_outputs(K, device=dev)
    best = torch.zeros(2, dtype=torch.float64, device=dev)
    solve = plan.launcher(vals, out, K, reltol=1e-2, abstol=1e-2, stream=stream, best=best)

    def step():
        apf_wrench(st, targets, K=K, wrench=wd, stream=stream)
        plan.assemble_controller(terms, B=K, shared=True, wdes=wd, out=vals, stream=stream)
        solve()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"workload": f"controller call batched: {K} APF-sampled candidates of one tick, wrench + 30/68/18 "
                        f"assembly on the device + solve ({'AMD' if order == 'amd' else 'leaves-first'} order, "
                        "tol 1e-2) + argmin",
            "batch": K, "value": K * steps / el, "unit": "QP solves/s", "ms_per_step": el * 1e3 / steps,
            "kernel": plan.kernel_name(K), "traffic": traffic_for(plan.kernel_name(K), K),
            "algorithmic_bytes_per_launch": plan.bytes_per_qp() * K, "input_bytes_per_candidate": 16,
            "optimal_frac": float((out["flag"] == 0).float().mean().item()),
            "mean_iters": float(out["iters"].float().mean().item()), "best": best.cpu().tolist()}


def traffic_for(kname, B=None):
    """HBM bytes per launch of kernel `kname` at batch B from the PMC passes committed in
    profiles/traffic.json (scripts/traffic_all.py); a kernel profiled at one grid only
    (plan groups) matches by name."""
    tfile = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tfile):
        data = json.load(open(tfile))
        t = data.get(f"{kname}@{B}")
        if t is None:
            same = [v for v in data.values() if v.get("kernel") == kname]
            t = same[0] if len(same) == 1 else None
        if t:
            return float(t["hbm_bytes_per_launch"])
    return None


def main():
    args = parse()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))           # before anything touches the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to measure another rank count")
    if args.dry_run:
        dry_run(args, rank, world, local)
        return
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from apf_quadruped_amd.batch import Plan
    from apf_quadruped_amd import plans

    seed = plans.SEED + 1
    d0 = plans.standard_qp("c1")
    plan = Plan.from_dense(12, 20, 6, d0["P"][0], d0["A"][0], d0["G"][0], exact=args.exact, kernel=args.kernel)
    plan.compile()
    B = args.batch
    ginfo = {}
    elapsed, kern_ms, out, gathered = run_leg(plan, B, args.steps, args.warmup, args.tol, dev, rank, world, seed,
                                              info=ginfo)
    kname = plan.kernel_name(B)
    flags = out["flag"].cpu().numpy()
    iters = out["iters"].cpu().numpy()
    mean_it = float(iters.mean())
    ms_step = elapsed * 1e3 / args.steps
    value = world * B * args.steps / elapsed
    bpq = plan.bytes_per_qp()
    achieved = bpq * B / (kern_ms * 1e-3) / 1e9
    fpq = flops_per_qp(plan.info, mean_it)
    fp64_tf = fpq * B / (kern_ms * 1e-3) / 1e12

    # secondary leg: one large batch per launch (row kernel), HBM-scale numbers
    large = None
    if rank == 0 and world == 1 and args.large_batch > 0:
        BL = args.large_batch
        el, km, outl, _ = run_leg(plan, BL, 10, 2, args.tol, dev, 0, 1, seed, gather=False)
        kl = plan.kernel_name(BL)
        itl = float(outl["iters"].float().mean().item())
        achl = bpq * BL / (km * 1e-3) / 1e9
        large = {"batch": BL, "value": BL * 10 / el, "ms_per_step": el * 1e3 / 10, "kernel": kl,
                 "kernel_ms": km, "kernel_qps": BL / (km * 1e-3),
                 "roofline": {"bound": measured_bound(kl, BL), "roofline_ref": "hbm", "achieved": achl,
                              "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": achl / HBM_PEAK_GBS, "traffic": traffic_for(kl, BL),
                              "limiter": limiter_for(BL) if kl.startswith("qpb_row") else None},
                 "fp64_tflops": flops_per_qp(plan.info, itl) * BL / (km * 1e-3) / 1e12,
                 "mean_iters": itl, "optimal_frac": float((outl["flag"] == 0).float().mean().item())}
        del outl

    # configs[2]: 4 096 QPs across the 4 gait contact patterns (mixed KKT sparsity):
    # one plan per pattern, all four in one group launch
    mixed = None
    if rank == 0 and world == 1 and args.mixed:
        mixed = mixed_patterns_leg(args.tol, dev)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(seed, args.cpu_sample, args.cpu_passes, args.tol)

    # configs[3] (MPC horizon, N = 380, band kernel) and the controller's own
    # stance QP (30/68/18), each with its CPU reference
    shapes = None
    if rank == 0 and world == 1 and args.shapes:
        from apf_quadruped_amd import workloads as W
        shapes = [
            shape_leg("configs[3]: MPC horizon N=10 (120/200/60), batch 1024", lambda ids: W.mpc_qp(plans.SEED + 4, ids),
                      1024, args.tol, dev, cpu=None if args.no_cpu else (256, 16)),
            shape_leg("controller stance QP 30/68/18 (main.cpp:1649), batch 1024",
                      lambda ids: W.controller_qp(plans.SEED + 30, ids), 1024, args.tol, dev,
                      cpu=None if args.no_cpu else (512, 16)),
            shape_leg("controller trot QP 30/70/12 (main.cpp:2005), batch 1024",
                      lambda ids: W.controller_qp(plans.SEED + 31, ids, phase="trot"), 1024, args.tol, dev,
                      cpu=None if args.no_cpu else (512, 16)),
            shape_leg("controller crawl QP 30/69/15 (main.cpp:3232), batch 1024",
                      lambda ids: W.controller_qp(plans.SEED + 31, ids, phase="crawl"), 1024, args.tol, dev,
                      cpu=None if args.no_cpu else (512, 16)),
            apf_leg(args.tol, dev),
            controller_apf_leg(dev),
            controller_apf_leg(dev, order="own"),
            trace_leg(args.tol, dev),
        ]

    if rank == 0:
        line = {
            "metric": "QP solves/sec (batched 12-var contact-force QP)",
            "value": value,
            "unit": "QP solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (counter-based RNG, SURVEY §8d contact-force QPs, resident in HBM)",
            "config": {"workload": "configs[1]: batch of 1024 identical-sparsity C1 contact-force QPs per GPU"
                                   if B == 1024 else f"batch of {B} identical-sparsity C1 contact-force QPs per GPU",
                       "qps_per_gpu": B, "global_batch": B * world, "tol": args.tol,
                       "kernel": kname, "arith": "exact" if args.exact else "fast",
                       "kkt_N": plan.info.N, "nnz_L": plan.info.lnz, "parallelism": f"shard{world}"},
            "roofline": {"bound": measured_bound(kname, B), "roofline_ref": "hbm", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic_for(kname, B),
                         "algorithmic_bytes_per_launch": bpq * B, "bytes_per_qp": bpq,
                         "kernel_ms": kern_ms, "kernel": kname,
                         "limiter": limiter_for(B) if kname.startswith("qpb_row") else None},
            "fp64": dict({"achieved_tflops": fp64_tf, "peak_tflops": FP64_PEAK_TFLOPS,
                          "frac": fp64_tf / FP64_PEAK_TFLOPS, "flops_per_qp": fpq}, **fp64_issued(kname, B)),
            "mean_iters": mean_it,
            "optimal_frac": float((flags == 0).mean()),
            "large_batch": large,
            "mixed_patterns": mixed,
            "shapes": shapes,
            "cpu_baseline": cpu,
        }
        if world > 1:
            g = gathered.cpu().numpy()          # {fval, global index, x*} from qpb_argmin_allgather
            gi = int(g[1])
            line["argmin"] = {"fval": float(g[0]), "index": gi, "rank": gi // B if gi >= 0 else -1,
                              "x": g[2:].tolist() if gi >= 0 else None,
                              "gather": ginfo.get("gather"), "rccl_ranks": ginfo.get("rccl_ranks"),
                              "init_error": ginfo.get("init_error"),
                              "collective": ("qpb_argmin_allgather (RCCL ncclAllGather, 16 + 8n B per rank)"
                                             if ginfo.get("gather") == "qpb_argmin_allgather" else
                                             "torch all_gather_into_tensor (RCCL) + qpb_argmin_reduce")}
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
