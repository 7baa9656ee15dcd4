#!/usr/bin/env python3
"""Benchmark: pod x node Filter+Score evaluations/s and pods scheduled/s (BASELINE.json metric).

Workload (N=1 default): BASELINE config C2 — 5,000-node synthetic cluster, 10,000 pending
pods, default plugin profile, percentageOfNodesToScore=100, scheduled sequentially on
one MI355X (each pod sees the previous pods' bindings).  One "step" = the whole
10,000-pod batch from the same initial snapshot (node state is reset on the device
before each step; pod programs and the cluster are resident in HBM before timing).

Multi-GPU (`--gpus N`: under torchrun, or started without it, when this process launches the
N rank processes itself before touching any GPU; one process per GPU): every rank schedules
its own independent C2 cluster (a what-if scenario; seed + rank) — scenario sharding, no
data-path collective, "weak" scaling.  Control-plane barrier/max uses gloo.  Beside it, the
same line carries `c4_split`: BASELINE config C4 (100,000 nodes x 20,000 pods, zone PTS) as ONE
split grid over all N GPUs (kss/split.py; N = 1: the whole grid on one GPU), strong scaling —
the north_star "pods/s at 100k nodes at 1/2/4/8 GPUs" figure — and `c5_sweep`: BASELINE config
C5 (4,096 what-if scenarios x 1,000 nodes x 1,000 pods) spread over the N GPUs, 4,096 / N
scenarios per GPU in one resident sweep each.

Prints ONE JSON line on rank 0.  Other modes: --config 1..4, --scenarios S (C5), --split P,
--node-axis, --per-pod, --postfilter.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# Algorithmic bytes per (pod, node) evaluation, SURVEY §8(d) / BASELINE.md §2:
# default profile reads 92 B of node state and writes 17 B of verdict + raw scores.
B_EVAL = {1: 109, 2: 109, 3: 129, 4: 129, 5: 109}
# each config's pod recipe (SURVEY §8(d) synthetic inputs)
RECIPE = {1: "default profile", 2: "default profile", 3: "default profile + PodTopologySpread + InterPodAffinity",
          4: "default profile + zone PodTopologySpread (DoNotSchedule)", 5: "default profile"}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def cpu_threads():
    """Host threads for the CPU baseline: the process's CPU share (OMP_NUM_THREADS, which the
    GPU box sets to its per-GPU share, else the affinity mask), with nproc stated beside it."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    t = int(env) if env and env.isdigit() and int(env) > 0 else aff
    return max(1, min(t, aff)), {"nproc": os.cpu_count(), "affinity_cpus": aff, "omp_num_threads": env}


def cpu_baseline(config, n_nodes, n_pods, seconds, threads, seed=0, curve=True, pct=100):
    """The CPU oracle (plain-C restatement, OpenMP over nodes: the reference's
    parallelize.Until over nodes inside each pod) on the same workload: the whole
    sequential batch is scheduled from the initial snapshot, repeated until `seconds` of wall
    time have passed (a bounded sample; a smaller pod prefix when one batch alone is longer)."""
    import oracle_c
    from kss import abi, native

    s = native.Synth(config, seed, n_nodes, n_pods)
    prof = abi.default_profile()
    prof.pct_nodes_to_score = pct
    kw = dict(threads=threads, record=False, n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)
    # size the prefix so one batch takes at most ~seconds/3
    n = min(n_pods, 64)
    t0 = time.perf_counter()
    oracle_c.schedule(prof, s.cluster, s.pods, n, n_nodes, **kw)
    dt = time.perf_counter() - t0
    n = int(min(n_pods, max(n, n * (seconds / 3) / max(dt, 1e-4))))
    reps, t_used = 0, 0.0
    while t_used < seconds:
        t0 = time.perf_counter()
        oracle_c.schedule(prof, s.cluster, s.pods, n, n_nodes, **kw)
        t_used += time.perf_counter() - t0
        reps += 1
    evals = reps * n * num_feasible_nodes_to_find(n_nodes, pct)
    _, host = cpu_threads()
    out = {"value": evals / t_used, "unit": "pod-node evals/s", "cores": threads, "kind": "port", "host": host,
           "sample": f"{reps} x the first {n} of {n_pods} pods of config C{config} ({n_nodes} nodes), "
                     f"sequential from the initial snapshot, {t_used:.1f} s wall, "
                     f"oracle/kss_oracle.c OpenMP over nodes ({threads} threads)",
           "pods_per_s": reps * n / t_used}
    if curve and threads > 1:
        out["threads_curve"] = thread_curve(prof, s, n_nodes, n, threads, out["pods_per_s"], kw)
    return out


def thread_curve(prof, s, n_nodes, n, threads, pods_per_s_at_threads, kw, seconds=2.0):
    """The same oracle at 1 and threads/4 threads (short samples) beside the main figure, and
    the figure at Parallelism = nproc PROJECTED by an Amdahl fit to the 1- and
    `threads`-thread points: it is not measured, because a one-GPU box's CPU share is 16
    threads (OMP_NUM_THREADS) while nproc counts the whole machine's cores."""
    import oracle_c
    pts = {}
    for t in sorted({1, max(1, threads // 4)}):
        m = max(1, n // 8)
        k, used = 0, 0.0
        while used < seconds:
            t0 = time.perf_counter()
            oracle_c.schedule(prof, s.cluster, s.pods, m, n_nodes, **dict(kw, threads=t))
            used += time.perf_counter() - t0
            k += 1
        pts[t] = k * m / used
    pts[threads] = pods_per_s_at_threads
    s_meas = pts[threads] / pts[1]  # speedup at `threads`
    f = max(0.0, min(1.0, (threads / s_meas - 1.0) / (threads - 1.0)))  # serial fraction
    nproc = os.cpu_count() or threads
    s_nproc = 1.0 / (f + (1.0 - f) / nproc)
    return {"pods_per_s": {str(t): round(v, 2) for t, v in sorted(pts.items())}, "serial_fraction": round(f, 4),
            "nproc": nproc, "pods_per_s_at_nproc_projected": round(pts[1] * s_nproc, 2),
            "note": "1 and threads/4 from short samples of the same pod prefix; the nproc figure is an Amdahl "
                    "projection from the 1- and max-thread points (not measured: a one-GPU box's CPU share is "
                    "16 threads)"}


def gpu_over_cpu(gpu_pods_per_s, cpu):
    """The GPU line against the CPU restatement: at the measured thread count, and against the
    faster nproc projection (thread_curve) when there is one."""
    if not cpu or not cpu.get("pods_per_s"):
        return None
    out = {f"vs_{cpu['cores']}_threads": gpu_pods_per_s / cpu["pods_per_s"]}
    curve = cpu.get("threads_curve") or {}
    if curve:  # the fastest CPU figure: any measured thread count, or the nproc projection
        best = max([cpu["pods_per_s"], curve.get("pods_per_s_at_nproc_projected", 0.0)] +
                   list(curve.get("pods_per_s", {}).values()))
        out["vs_fastest_cpu"] = gpu_pods_per_s / best
    return out


def cpu_baseline_scenarios(n_nodes, n_pods, seconds, threads, seed_of):
    """C5 on the CPU: independent scenarios in parallel (one oracle call per scenario and
    thread, single-threaded inside; ctypes releases the GIL), as many scenarios as fit in
    about `seconds` of wall time."""
    import concurrent.futures as cf

    import oracle_c
    from kss import abi, native

    prof = abi.default_profile()

    def one(k):
        s = native.Synth(5, seed_of(k), n_nodes, n_pods)
        oracle_c.schedule(prof, s.cluster, s.pods, n_pods, n_nodes, threads=1, record=False,
                          n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)
        s.close()

    t0 = time.perf_counter()
    one(0)
    per = time.perf_counter() - t0
    n_scen = max(threads, int(seconds / max(per, 1e-4) * threads))
    n_scen = (n_scen + threads - 1) // threads * threads
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(max_workers=threads) as ex:
        list(ex.map(one, range(n_scen)))
    dt = time.perf_counter() - t0
    _, host = cpu_threads()
    return {"value": n_scen * n_pods * n_nodes / dt, "unit": "pod-node evals/s", "cores": threads, "kind": "port",
            "host": host, "pods_per_s": n_scen * n_pods / dt,
            "sample": f"{n_scen} C5 scenarios ({n_nodes} nodes x {n_pods} pods each, synthesis included), "
                      f"{threads} scenarios in parallel, {dt:.1f} s wall, oracle/kss_oracle.c single-threaded per scenario"}


def num_feasible_nodes_to_find(n: int, pct: int) -> int:
    """v1.26 schedule_one.go numFeasibleNodesToFind (the simulator's scheduler always has pct 0:
    simulator/scheduler/scheduler.go:163,258-275)."""
    if n < 100 or pct >= 100:
        return n
    if pct <= 0:
        pct = max(5, 50 - n // 125)
    return max(100, n * pct // 100)


def rank_seed(seed_base, cfg, rank):
    """Scenario sharding: rank r schedules its own independent cluster; rank 0 is the
    canonical BASELINE cluster of config cfg."""
    return seed_base + cfg + 7919 * rank


def reduce_over_ranks(elapsed, scheduled, dist):
    """Whole-job timing and work: the slowest rank's elapsed time (MAX) and the pods
    scheduled by all ranks (SUM), over the control-plane (gloo) group."""
    if dist is None:
        return elapsed, scheduled
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    sc = torch.tensor([scheduled], dtype=torch.float64)
    dist.all_reduce(sc, op=dist.ReduceOp.SUM)
    return float(t.item()), int(sc.item())


def measure_traffic(args, cfg, mode=(), match=("k_simple", "k_schedule", "k_spread"), mean=False, timeout=120):
    """HBM bytes per launch of the scheduling kernel from rocprofv3 PMC counters: one child
    process per counter (FETCH_SIZE, WRITE_SIZE), started before this process touches the
    GPU, running ONE step.  A step of several launches (C4: one k_spread launch per static
    chunk) reports the mean over its launches (`launches` in the detail).  FETCH_SIZE is
    doubled (gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md "HBM").  Returns
    (bytes, detail) or (None, reason)."""
    if not shutil.which("rocprofv3"):
        return None, "rocprofv3 not found"
    kb, launches = {}, 0
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="kss_pmc_")
        cmd = ["timeout", "-s", "KILL", str(timeout), "rocprofv3", "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "p",
               "--", sys.executable, os.path.abspath(__file__), "--inner", "--steps", "1", "--warmup", "0",
               "--config", str(cfg), "--nodes", str(args.nodes), "--pods", str(args.pods), *mode]
        subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd=ROOT)
        vals = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if r.get("Counter_Name") == ctr and any(m in r["Kernel_Name"] for m in match):
                    vals.append(float(r["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if not vals:
            return None, f"no {ctr} sample"
        kb[ctr] = sum(vals) / len(vals) if mean or len(vals) > 1 else vals[0]
        launches = len(vals)
    fetch = 2.0 * kb["FETCH_SIZE"] * 1024.0
    write = kb["WRITE_SIZE"] * 1024.0
    return fetch + write, {"fetch_bytes": fetch, "write_bytes": write, "fetch_size_kb_raw": kb["FETCH_SIZE"],
                           "launches": launches, "per": "launch (mean over the launches of one step)"}


# VALU issue peak of the chip: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD every
# 2 cycles (SIMD-32, MI355X_MICROARCH.md "Wave scheduling"), 2.4 GHz max clock.
VALU_PEAK_INSTS = 256 * 4 * 2.4e9 / 2
SQ_GROUP = ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
            "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU")


def measure_sq(args, cfg, mode=(), match=("k_simple", "k_schedule", "k_spread"), timeout=120):
    """Instruction-issue counters of the loop kernel: ONE rocprofv3 --pmc pass of eight SQ
    counters (one pass holds at most 8 SQ_ counters) over a one-step child run started before
    this process touches the GPU.  Counts are summed over the launches of the step.  Returns
    ({counter: value}, detail) or (None, reason)."""
    if not shutil.which("rocprofv3"):
        return None, "rocprofv3 not found"
    d = tempfile.mkdtemp(prefix="kss_sq_")
    cmd = ["timeout", "-s", "KILL", str(timeout), "rocprofv3", "--pmc", *SQ_GROUP, "--output-format", "csv", "-d", d,
           "-o", "p", "--", sys.executable, os.path.abspath(__file__), "--inner", "--steps", "1", "--warmup", "0",
           "--config", str(cfg), "--nodes", str(args.nodes), "--pods", str(args.pods), *mode]
    subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd=ROOT)
    vals, disp = {}, set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if any(m in r["Kernel_Name"] for m in match) and r.get("Counter_Name") in SQ_GROUP:
                vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                disp.add(r.get("Dispatch_Id"))
    shutil.rmtree(d, ignore_errors=True)
    if len(vals) < len(SQ_GROUP):
        return None, f"SQ counters missing: {sorted(set(SQ_GROUP) - set(vals))}"
    return vals, {"launches": len(disp), "counters": list(SQ_GROUP)}


def valu_roofline(sq, kern_s, evals):
    """roofline.valu: achieved VALU wave-instructions/s of the loop kernel (SQ_INSTS_VALU over
    its HIP-event time) against the chip's issue peak, with the issue / wait split."""
    if not sq:
        return None
    achieved = sq["SQ_INSTS_VALU"] / kern_s
    wc = max(sq["SQ_WAVE_CYCLES"], 1.0)
    return {"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_INSTS, "unit": "wave64 VALU insts/s",
            "frac": achieved / VALU_PEAK_INSTS, "valu_insts": sq["SQ_INSTS_VALU"],
            "valu_insts_per_eval": sq["SQ_INSTS_VALU"] / evals, "salu_insts_per_eval": sq["SQ_INSTS_SALU"] / evals,
            "lds_insts_per_eval": sq["SQ_INSTS_LDS"] / evals,
            "wave_cycles_active_valu_frac": sq["SQ_ACTIVE_INST_VALU"] / wc, "wave_cycles_wait_frac": sq["SQ_WAIT_ANY"] / wc,
            "counters": sq, "peak_note": "256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction"}


def run_scenarios(args):
    """What-if scenario sweep (SURVEY 8(e) scenario axis, C5 shape): each rank schedules
    `--scenarios` independent clusters (config-5 recipe, seed + global scenario index) in
    one kss_schedule_scenarios launch, one workgroup per scenario, no collective.  The
    timed figure is the launch's HIP-event time (inputs resident: the upload precedes the
    first event); the wall time including the host->device upload is reported beside it."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    traffic, traffic_detail = None, "not measured"
    sq, sq_detail = None, "not measured"
    if rank == 0 and world == 1 and not args.no_traffic:  # before this process touches the GPU
        traffic, traffic_detail = measure_traffic(args, 5, mode=("--scenarios", str(args.scenarios)))
        # k_static counted too: the sweep's device time covers reset + k_static + k_simple
        sq, sq_detail = measure_sq(args, 5, mode=("--scenarios", str(args.scenarios)), match=("k_simple", "k_static"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from kss import abi, native
    from kss.synth import SEED_BASE
    S = args.scenarios
    n_nodes = args.nodes or 1000
    n_pods = args.pods or 1000
    seed_of = lambda k: SEED_BASE + 5 + 7919 * (rank * S + k)  # noqa: E731
    synths = [native.Synth(5, seed_of(k), n_nodes, n_pods) for k in range(S)]
    prof = abi.default_profile()
    clusters = [x.cluster for x in synths]
    podsets = [x.pods for x in synths]
    # stage once (pack + one upload); every step then restores the snapshots on the device
    # and schedules all scenarios: inputs resident
    t0 = time.perf_counter()
    sweep = native.Sweep(prof, clusters, podsets, device=local)
    stage_s = time.perf_counter() - t0
    info = sweep.info()
    for _ in range(args.warmup):
        sweep.run()
    if dist:
        dist.barrier()
    dev_ms, t0 = [], time.perf_counter()
    for _ in range(args.steps):
        chosen, ms = sweep.run()
        dev_ms.append(ms)
    wall = time.perf_counter() - t0
    elapsed = wall
    scheduled = int((chosen >= 0).sum())
    elapsed, scheduled_total = reduce_over_ranks(elapsed, scheduled, dist)
    evals = world * S * n_pods * n_nodes * args.steps
    kern_s = sum(dev_ms) / len(dev_ms) / 1e3
    achieved = B_EVAL[5] * S * n_pods * n_nodes / kern_s / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        threads, _ = cpu_threads()
        cpu = cpu_baseline_scenarios(n_nodes, n_pods, args.cpu_seconds, threads, seed_of)
    if rank == 0:
        out = {
            "metric": "pod x node filter+score evals/sec (pods scheduled/sec in extra)",
            "value": evals / elapsed,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64/f64",
            "data": "synthetic (SplitMix64, config-5 recipe, seed per scenario)",
            "config": {"workload": f"C5 shape: {S * world} scenarios x {n_nodes} nodes x {n_pods} pods, default "
                                   f"profile, pct=100", "scenarios": S * world, "nodes": n_nodes, "pods": n_pods,
                       "parallelism": f"scenario batch x{world}"},
            "pods_per_s": scheduled_total * args.steps / elapsed,
            "device_ms_per_step": kern_s * 1e3,
            "stage_ms_once": stage_s * 1e3,
            "upload_bytes": info["upload_bytes"],
            "evals_per_s_incl_stage_one_step": S * n_pods * n_nodes / (stage_s + elapsed / args.steps),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": info["kernel"],
                         "bytes_per_eval": B_EVAL[5], "algorithmic_bytes_per_launch": B_EVAL[5] * S * n_pods * n_nodes,
                         "traffic_detail": traffic_detail,
                         "note": "achieved: ALGORITHMIC bytes (109 B per evaluation, most of which never leave LDS) "
                                 "over the device time of reset + k_static + k_simple per sweep; the binding limit "
                                 "of this throughput-mode config is instruction issue: see valu"},
            "valu": valu_roofline(sq, kern_s, S * n_pods * n_nodes), "valu_detail": sq_detail,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    sweep.close()
    for x in synths:
        x.close()
    if dist:
        dist.destroy_process_group()


def run_node_axis(args):
    """Node-axis bench line (SURVEY 8(e), C4 shape): the SAME cluster on every rank, rows
    split into contiguous blocks, two collectives per pod (all_gather of 32 B statistics,
    all_reduce MAX of the 8 B packed key) over RCCL when world > 1.  Pods use the default
    profile recipe (config 2): zone PodTopologySpread is not yet on the node axis.
    `value` = pod x node evals of the whole cluster / max-over-ranks step time (strong
    scaling: the total work is fixed as ranks are added)."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    traffic, traffic_detail = None, "not measured"
    if rank == 0 and world == 1 and not args.no_traffic:  # per k_axis_eval launch, mean over a 200-pod run
        a = argparse.Namespace(**vars(args))
        a.pods = 200
        traffic, traffic_detail = measure_traffic(a, 2, mode=("--node-axis",), match=("k_axis_eval",), mean=True)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    from kss import abi, native, nodeaxis
    from kss.synth import SEED_BASE
    n_nodes = args.nodes or 100000
    n_pods = args.pods or 20000
    s = native.Synth(2, SEED_BASE + 4, n_nodes, n_pods)
    sch = nodeaxis.NodeAxisScheduler(s.cluster, s.pods, abi.default_profile(), device=local)

    def step():
        sch.reset()
        out = sch.schedule()
        torch.cuda.synchronize()
        return out

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        chosen = step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    scheduled = int((chosen >= 0).sum().item())
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # live roofline of the dominant kernel (k_axis_eval): 200 launches on the scheduler's stream
    k = min(200, n_pods)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(sch.stream):
        e0.record(sch.stream)
        for i in range(k):
            sch.ctx.axis_eval(i, sch.stats[0].data_ptr(), 0, 0, 1, sch.key[0].data_ptr(), sch.chosen.data_ptr(),
                              sch.stream.cuda_stream)
        e1.record(sch.stream)
    e1.synchronize()
    eval_s = e0.elapsed_time(e1) / 1e3 / k
    rows = sch.hi - sch.lo
    achieved = B_EVAL[2] * rows / eval_s / 1e9
    if rank == 0:
        out = {
            "metric": "pod x node filter+score evals/sec (pods scheduled/sec in extra)",
            "value": n_pods * n_nodes * args.steps / elapsed,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64/f64",
            "data": "synthetic (SplitMix64 seed 0x5EED0004, config-2 pod recipe)",
            "config": {"workload": f"C4 shape: {n_nodes} nodes x {n_pods} pods, default profile, node-axis sharded, "
                                   f"pct=100", "nodes": n_nodes, "pods": n_pods, "parallelism": f"node-axis x{world}"},
            "pods_per_s": scheduled * args.steps / elapsed,
            "us_per_pod": elapsed / args.steps / n_pods * 1e6,
            "pods_scheduled_per_step": scheduled,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_detail": traffic_detail,
                         "kernel": "k_axis_eval",
                         "bytes_per_eval": B_EVAL[2], "algorithmic_bytes_per_launch": B_EVAL[2] * rows,
                         "kernel_us": eval_s * 1e6,
                         "note": "per pod the path is latency-bound: 2 launches + 2 collectives"},
            "cpu_baseline": None,
        }
        print(json.dumps(out), flush=True)
    sch.close()
    s.close()
    if dist:
        dist.destroy_process_group()


def run_split(args):
    """Node axis as a split grid (kss/split.py): ONE k_spread / k_simple grid
    whose shards are spread over the ranks' GPUs, the per-pod exchanges done by the kernels
    themselves with xGMI peer stores into every part's inbox (no launch, collective or host
    round trip per pod).  C4's recipe (config 4: default profile + zone DoNotSchedule spread),
    the SAME cluster on every rank, `value` = evals of the whole cluster / max-over-ranks time
    (strong scaling).  world 1 with --split P > 1 runs P parts on the one GPU (an emulation
    that measures the split exchange's cost, not a speed-up)."""
    import numpy as np
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    torch.zeros(1, device="cuda")  # torch's HIP runtime before libkss's
    dist = None
    if world > 1:
        import torch.distributed as dist  # control plane only: the IPC handles, barriers, max of timings
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from kss import abi, native, split
    from kss.synth import SEED_BASE
    cfg = args.split_recipe
    n_nodes = args.nodes or 100000
    n_pods = args.pods or 20000
    parts = world if world > 1 else max(1, args.split)
    # 256 shards in all for k_spread (~391 nodes per shard at 100k nodes); k_simple sweeps at most 128
    wl = max(1, (256 if cfg == 4 else 128) // parts)
    s = native.Synth(cfg, SEED_BASE + cfg, n_nodes, n_pods)
    if world > 1:
        runner = split.SplitRank(s.cluster, s.pods, wl, device=local)
        ctxs = [runner.ctx]
        run = lambda: [runner.run(n_pods)]  # noqa: E731
    elif parts > 1:
        runner = split.InProcessSplit(s.cluster, s.pods, parts, wl)
        ctxs = runner.ctxs
        run = lambda: runner.run(n_pods)  # noqa: E731
    else:
        c = native.Context(abi.default_profile(), device=local)
        c.load(s.cluster)
        c.stage(s.pods)
        ctxs = [c]
        run = lambda: [c.run_staged(n_pods)]  # noqa: E731

    handoff = {"reloads": 0, "shadow": 0, "final": 0}  # k_spread hand-off counters over every run

    def step():
        for c in ctxs:
            c.reset()
        outs = run()
        for c in ctxs:
            for k, v in c.last_handoff_status().items():
                handoff[k] += v
        return outs

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        outs = step()
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    chosen = outs[0]
    scheduled = int((chosen >= 0).sum())
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loop_s = ctxs[0].last_loop_ms() / 1e3
    rows = -(-n_nodes // parts)
    achieved = B_EVAL[cfg] * n_pods * rows / loop_s / 1e9
    if rank == 0:
        cpu = None
        if not args.no_cpu:  # the host restatement, the same figure at every world size
            threads, _ = cpu_threads()
            cpu = cpu_baseline(cfg, n_nodes, n_pods, args.cpu_seconds, threads, seed=SEED_BASE + cfg)
        out = {
            "metric": "pod x node filter+score evals/sec (pods scheduled/sec in extra)",
            "value": n_pods * n_nodes * args.steps / elapsed,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64/f64",
            "data": f"synthetic (SplitMix64 seed 0x5EED000{cfg}, config-{cfg} recipe)",
            "config": {"workload": f"C4: {n_nodes} nodes x {n_pods} pods, {RECIPE[cfg]}, "
                                   f"split grid {parts} part(s) x {wl} shards, pct=100",
                       "nodes": n_nodes, "pods": n_pods, "parallelism": f"node-axis split x{parts}"
                       + (" (one GPU)" if world == 1 and parts > 1 else "")},
            "pods_per_s": scheduled * args.steps / elapsed,
            "us_per_pod": elapsed / args.steps / n_pods * 1e6,
            "pods_scheduled_per_step": scheduled,
            "kernel": ctxs[0].last_kernel(),
            "geometry": ctxs[0].last_geometry(),
            "handoff": dict(handoff, note="k_spread node-state hand-off counters summed over every run of every "
                                          "part: prologue reloads, loads the shadow answered, last write-backs that "
                                          "failed the final check (all 0 = every hand-off clean)"),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None, "traffic_detail": "not measured",
                         "kernel": ctxs[0].last_kernel(), "bytes_per_eval": B_EVAL[cfg],
                         "algorithmic_bytes_per_launch": B_EVAL[cfg] * n_pods * rows,
                         "loop_kernel_ms": loop_s * 1e3,
                         "note": "latency-bound: per pod 3-4 granule exchanges across every part's shards"},
            "cpu_baseline": cpu,
            "gpu_over_cpu": gpu_over_cpu(scheduled * args.steps / elapsed, cpu),
        }
        print(json.dumps(out), flush=True)
    if world > 1 or parts > 1:
        runner.close()
    else:
        ctxs[0].close()
    s.close()
    if dist:
        dist.destroy_process_group()


def latency_profile(cfg, n_nodes, n_pods, seed, device, pct=100):
    """roofline.latency: the per-pod chain is latency-bound, so beside the HBM fraction the line
    carries the phase breakdown of one stamped run (KSS_STAMPS_FILE: s_memrealtime per phase,
    the first 128 pods, outside the timed region) and the measured exchange floor (per
    exchange, the median over pods of the fastest shard's wait from the last publish to
    completion).  bound_us_per_pod = exchanges per pod x floor."""
    import tempfile
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    import stamps
    from kss import abi, native
    path = os.path.join(tempfile.mkdtemp(prefix="kss_stamps_"), "stamps.bin")
    native.set_stamps_file(path)
    try:
        s = native.Synth(cfg, seed, n_nodes, min(n_pods, 1000))
        prof = abi.default_profile()
        prof.pct_nodes_to_score = pct
        ctx = native.Context(prof, device=device)
        ctx.load(s.cluster)
        ctx.stage(s.pods)
        ctx.run_staged(s.n_pods)
        ctx.close()
        s.close()
    finally:
        native.set_stamps_file(None)
    out = stamps.latency_summary(path)
    if not out.get("pods"):  # the stamp buffer did not fit in the shard's LDS (k_spread at large shards)
        return {"kernel": out.get("kernel"), "shards": out.get("shards"), "pods": 0, "bound_us_per_pod": None,
                "note": "no phase stamps: the stamp buffer does not fit beside this geometry's LDS"}
    floors = out.get("exchange_floor_us", {})
    out["bound_us_per_pod"] = round(sum(floors.values()), 3)
    out["source"] = "KSS_STAMPS_FILE phase stamps, shard 0 (floors: all shards), first 128 pods of a 1000-pod run"
    return out


def run_per_pod(args):
    """The drop-in per-pod path as the Go plugin drives it: PreFilter ->
    kss_eval_pod (the pod's program uploaded, every per-node record copied back in one
    transfer), Reserve -> kss_commit (AssumePod from the kernel arguments), pod after pod on
    the C2 cluster.  Reports the host-observed microseconds per call."""
    import numpy as np
    from kss import abi, native
    from kss.synth import SEED_BASE
    n_nodes = args.nodes or (100 if args.config == 1 else 5000)
    n_pods = args.pods or 500
    cfg = args.config if args.config in (1, 2, 3) else 2  # C3: spread + inter-pod programs (the general chain)
    s = native.Synth(cfg, SEED_BASE + cfg, n_nodes, n_pods)
    prof = abi.default_profile()
    prof.pct_nodes_to_score = args.pct  # --pct 0: the simulator's own setting (adaptive window)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    for j in range(min(args.warmup * 20, n_pods)):  # warm the kernels, then restore the snapshot
        r = ctx.eval_pod(s.pods, j)
        if r.chosen >= 0:
            ctx.commit(s.pods, j, r.chosen)
    ctx.reset()
    # result buffers reused across pods, as the plugin keeps them: the full record (every
    # per-node array, for per-plugin Filter / Score / NormalizeScore answers), or the slim one
    # (verdicts + weighted totals, for one plugin answering Filter and Score)
    full = native.PodResult(n_nodes)
    slim = native.PodResult(n_nodes, fields=("fail_plugin", "fail_detail", "total"))

    # the in-place variant: kss_eval_pod_view leaves the full record in the pinned staging
    # and hands back pointers (the Go plugin reads them through unsafe.Slice; here the
    # ctypes call alone, no numpy views)
    import ctypes
    view = abi.PodView()
    pods_ref = ctypes.byref(s.pods)

    class _ViewCall:
        def __call__(self, j):
            native.check(native.lib().kss_eval_pod_view(ctx.h, pods_ref, j, abi.KSS_FIELD_ALL, ctypes.byref(view)))
            return view

    def loop(res):
        t_eval, t_commit, ch = [], [], []
        call = res if isinstance(res, _ViewCall) else (lambda j: ctx.eval_pod(s.pods, j, out=res))
        t0 = time.perf_counter()
        for j in range(n_pods):
            a = time.perf_counter()
            r = call(j)
            b = time.perf_counter()
            if r.chosen >= 0:
                ctx.commit(s.pods, j, r.chosen)
            c = time.perf_counter()
            t_eval.append(b - a)
            t_commit.append(c - b)
            ch.append(r.chosen)
        return time.perf_counter() - t0, np.array(t_eval) * 1e6, np.array(t_commit) * 1e6, ch

    elapsed, ev, cm, chosen = loop(full)
    ctx.reset()
    elapsed_slim, ev_slim, _, chosen_slim = loop(slim)
    assert chosen_slim == chosen
    ctx.reset()
    elapsed_view, ev_view, _, chosen_view = loop(_ViewCall())
    assert chosen_view == chosen

    # the persistent service grid (kss_service_*): the staged pods by index, one command per
    # call through a pinned ring, no launch / upload / stream synchronisation per pod
    ctx.reset()
    ctx.stage(s.pods)
    sview = abi.PodView()
    cview = abi.PodCView()

    def svc_loop(fields, compact=False):
        t_eval, t_commit, ch = [], [], []
        ev_fn = native.lib().kss_service_eval_compact if compact else native.lib().kss_service_eval
        vp = ctypes.byref(cview if compact else sview)
        v = cview if compact else sview
        t0 = time.perf_counter()
        for j in range(n_pods):
            a = time.perf_counter()
            native.check(ev_fn(ctx.h, j, fields, vp))
            b = time.perf_counter()
            if v.chosen >= 0:
                native.check(native.lib().kss_service_commit(ctx.h, j, v.chosen))
            c = time.perf_counter()
            t_eval.append(b - a)
            t_commit.append(c - b)
            ch.append(v.chosen)
            assert not compact or not cview.is_wide
        el = time.perf_counter() - t0
        ctx.service_stop()
        return el, np.array(t_eval) * 1e6, np.array(t_commit) * 1e6, ch

    for j in range(min(args.warmup * 20, n_pods)):  # start the grid, warm it
        native.check(native.lib().kss_service_eval(ctx.h, j, abi.KSS_FIELD_ALL, ctypes.byref(sview)))
    ctx.service_stop()
    ctx.reset()
    elapsed_svc, ev_svc, cm_svc, chosen_svc = svc_loop(abi.KSS_FIELD_ALL)
    assert chosen_svc == chosen, "service choices differ from kss_eval_pod's"
    # one stamped pass (KSS_SERVICE_STAMPS): where shard 0 spends an evaluation
    native.set_option("service_stamps", 1)
    slim_fields = abi.KSS_FIELD_FAIL | abi.KSS_FIELD_DETAIL | abi.KSS_FIELD_TOTAL

    def stamped(fields):
        ctx.reset()
        phases = []
        for j in range(min(100, n_pods)):
            native.check(native.lib().kss_service_eval(ctx.h, j, fields, ctypes.byref(sview)))
            st = ctx.service_stamps()
            phases.append([(st[1] - st[0]) / 100.0, (st[2] - st[1]) / 100.0, (st[3] - st[2]) / 100.0,
                           (st[4] - st[2]) / 100.0, (st[3] - st[4]) / 100.0,
                           (st[5] - st[1]) / 100.0 if st[5] else 0.0, (st[6] - st[5]) / 100.0 if st[6] else 0.0,
                           (st[7] - st[6]) / 100.0 if st[7] else 0.0, (st[2] - st[7]) / 100.0 if st[7] else 0.0])
            if sview.chosen >= 0:
                native.check(native.lib().kss_service_commit(ctx.h, j, sview.chosen))
        ctx.service_stop()
        return np.median(np.array(phases), axis=0)

    ph = stamped(abi.KSS_FIELD_ALL)
    ph_slim = stamped(slim_fields)
    native.set_option("service_stamps", 0)
    ctx.reset()
    elapsed_svc_slim, ev_svc_slim, _, chosen_svc_slim = svc_loop(slim_fields)
    assert chosen_svc_slim == chosen
    ctx.reset()
    elapsed_svc_c, ev_svc_c, _, chosen_svc_c = svc_loop(abi.KSS_FIELD_ALL, compact=True)
    assert chosen_svc_c == chosen
    svc_mode = ctx.service_mode()
    # the same two loops on the general chain (schedule_pod + the record copy), for comparison
    native.set_option("service_general", 1)
    ctx.reset()
    el_g, ev_g, _, ch_g = svc_loop(abi.KSS_FIELD_ALL)
    ctx.reset()
    el_gs, ev_gs, _, ch_gs = svc_loop(slim_fields)
    native.set_option("service_general", 0)
    assert ch_g == chosen and ch_gs == chosen
    # A/B: the simple evaluation with every lane's system fence (the general chain's record fence),
    # and with the static words evaluated per call instead of the table k_static fills at the start
    ab = {}
    for env, opt in (("KSS_SVC_FULL_FENCE", "svc_full_fence"), ("KSS_SVC_NO_STATIC", "svc_no_static"),
                     ("KSS_SVC_INLINE_SWEEP", "svc_inline_sweep")):
        native.set_option(opt, 1)
        ctx.reset()
        el_ab, ev_ab, _, ch_ab = svc_loop(slim_fields)
        native.set_option(opt, 0)
        assert ch_ab == chosen
        ab[env] = float(np.median(ev_ab))
    out = {
        "metric": "per-pod API: kss_eval_pod + kss_commit latency (pods/sec in value)",
        "value": n_pods / elapsed,
        "unit": "pods/s",
        "n_gpus": 1,
        "steps": 1,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64/f64",
        "data": f"synthetic (SplitMix64 seed 0x5EED000{cfg})",
        "config": {"workload": f"C{cfg} cluster, per-pod API: {n_nodes} nodes, {n_pods} pods one call pair each, "
                               f"pct={args.pct}",
                   "nodes": n_nodes, "pods": n_pods, "parallelism": "none", "percentage_of_nodes_to_score": args.pct},
        "eval_us": {"median": float(np.median(ev)), "mean": float(ev.mean()), "p90": float(np.percentile(ev, 90))},
        "eval_slim_us": {"median": float(np.median(ev_slim)), "mean": float(ev_slim.mean()),
                         "p90": float(np.percentile(ev_slim, 90)), "fields": "fail_plugin, fail_detail, total",
                         "pods_per_s": n_pods / elapsed_slim},
        "eval_view_us": {"median": float(np.median(ev_view)), "mean": float(ev_view.mean()),
                         "p90": float(np.percentile(ev_view, 90)),
                         "fields": "all, in place (kss_eval_pod_view: no copy into caller arrays)",
                         "pods_per_s": n_pods / elapsed_view},
        "commit_us": {"median": float(np.median(cm)), "mean": float(cm.mean()), "p90": float(np.percentile(cm, 90))},
        "service": {"api": "kss_service_eval + kss_service_commit (resident grid, pinned command ring)",
                    "pods_per_s": n_pods / elapsed_svc,
                    "eval_us": {"median": float(np.median(ev_svc)), "mean": float(ev_svc.mean()),
                                "p90": float(np.percentile(ev_svc, 90)), "fields": "all, in place"},
                    "commit_us": {"median": float(np.median(cm_svc)), "mean": float(cm_svc.mean()),
                                  "p90": float(np.percentile(cm_svc, 90))},
                    "slim": {"pods_per_s": n_pods / elapsed_svc_slim, "fields": "fail_plugin, fail_detail, total",
                             "eval_us": {"median": float(np.median(ev_svc_slim)), "mean": float(ev_svc_slim.mean()),
                                         "p90": float(np.percentile(ev_svc_slim, 90))}},
                    "compact": {"pods_per_s": n_pods / elapsed_svc_c,
                                "api": "kss_service_eval_compact (every field; raw / total int32, norm uint8)",
                                "eval_us": {"median": float(np.median(ev_svc_c)), "mean": float(ev_svc_c.mean()),
                                            "p90": float(np.percentile(ev_svc_c, 90))}},
                    "mode": {2: "k_simple-shaped evaluation on an XCD-local grid, record stored from registers",
                             1: "k_simple-shaped evaluation, record stored from registers",
                             0: "general chain (schedule_pod + record copy)"}.get(svc_mode, "not started"),
                    "slim_ab_eval_us_median": {"KSS_SVC_FULL_FENCE=1 (every lane's system fence)": ab["KSS_SVC_FULL_FENCE"],
                                               "KSS_SVC_NO_STATIC=1 (static words per call)": ab["KSS_SVC_NO_STATIC"],
                                               "KSS_SVC_INLINE_SWEEP=1 (the exchange sweep inlined)": ab["KSS_SVC_INLINE_SWEEP"]},
                    "general_chain": {"eval_us_median": float(np.median(ev_g)), "slim_eval_us_median": float(np.median(ev_gs)),
                                      "pods_per_s": n_pods / el_g, "slim_pods_per_s": n_pods / el_gs,
                                      "note": "KSS_SERVICE_GENERAL=1: the chain every program shape takes"},
                    "shard0_phases_us_median": {"relay": float(ph[0]), "pod": float(ph[1]),
                                                "record_copy_and_fence": float(ph[2]), "record_stores": float(ph[3]),
                                                "system_fence": float(ph[4]),
                                                "note": "the k_simple-shaped evaluation stores the record from "
                                                        "registers inside 'pod'; the fence is the rest"},
                    "shard0_phases_us_median_slim": {"relay": float(ph_slim[0]), "pod": float(ph_slim[1]),
                                                     "system_fence": float(ph_slim[4]),
                                                     "pod_node_pass": float(ph_slim[5]),
                                                     "pod_stats_exchange": float(ph_slim[6]),
                                                     "pod_normalise_and_record": float(ph_slim[7]),
                                                     "pod_key_exchange": float(ph_slim[8])},
                    "geometry": ctx.last_geometry()},
        "eval_device_ms_last": ctx.last_timing()[0],
        "geometry": ctx.last_geometry(),
        "pods_scheduled": int(sum(1 for c in chosen if c >= 0)),
    }
    print(json.dumps(out), flush=True)
    ctx.close()
    s.close()


def run_snapshot(args):
    """The snapshot path the plugin takes: a C<config> cluster written as the simulator's
    ResourcesForSnap JSON, read back (kss/snapshot.py read_snapshot), compiled (kss/compile.py) and
    scheduled as one sequential batch with the profile the simulator's configuration yields --
    percentageOfNodesToScore 0, the adaptive window (profile_from_config) -- every step from the
    snapshot's state (a device reset).  Reports the kernel the batch took, pods/s and the window's
    evaluations per pod; the JSON read and the compile are timed beside it, once."""
    import json as _json
    from kss import native, snapshot, synth
    from kss.compile import compile_cluster
    cfg = args.config if args.config in (1, 2, 3) else 2
    n_nodes = args.nodes or 1000
    n_pods = args.pods or 2000
    nodes, bound, pods = synth.make_cluster(cfg, n_nodes=n_nodes, n_pods=n_pods)
    t0 = time.perf_counter()
    snap = snapshot.read_snapshot(_json.dumps(synth.to_resources_for_snap(nodes, bound, pods)))
    cc, cp, _ = compile_cluster(snap.nodes, snap.bound, snap.pending, snap.namespaces)
    prof = snapshot.profile_from_config(snap.scheduler_config, cc.scalars)
    compile_s = time.perf_counter() - t0
    ctx = native.Context(prof)
    ctx.load(cc.as_struct(), names=native.make_names(cc.node_names, cc.taints, cc.scalars))
    ps = cp.as_struct()
    ctx.stage(ps)
    for _ in range(args.warmup):
        ctx.reset()
        ctx.run_staged(cp.n)
    ts = []
    for _ in range(args.steps):
        ctx.reset()
        a = time.perf_counter()
        chosen = ctx.run_staged(cp.n)
        ts.append(time.perf_counter() - a)
    el = sum(ts)
    k = num_feasible_nodes_to_find(cc.n_nodes, prof.pct_nodes_to_score)
    out = {
        "metric": "pods scheduled/sec, simulator snapshot path (ResourcesForSnap -> compile -> batch)",
        "value": cp.n * args.steps / el,
        "unit": "pods/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64/f64",
        "data": f"synthetic (kss.synth config {cfg} objects as ResourcesForSnap JSON)",
        "config": {"workload": f"C{cfg} recipe snapshot: {cc.n_nodes} nodes, {cp.n} pending pods, pct="
                               f"{prof.pct_nodes_to_score} (the simulator's reset config)",
                   "nodes": cc.n_nodes, "pods": cp.n, "percentage_of_nodes_to_score": prof.pct_nodes_to_score},
        "kernel": ctx.last_kernel(),
        "geometry": ctx.last_geometry(),
        "evals_per_pod": k,
        "scheduled": int((chosen >= 0).sum()),
        "read_and_compile_s_once": compile_s,
    }
    print(json.dumps(out), flush=True)
    ctx.close()


def run_postfilter(args):
    """DefaultPreemption PostFilter dry run as the simulator's cycle runs it:
    kss_eval_pod, and for an unschedulable pod kss_postfilter_pod on the same snapshot, on a
    saturated cluster (every node nearly full of pods of mixed priority; pending pods of
    higher priority).  Reports dry runs per second (host-observed, one k_preempt launch each)
    and the k_preempt device time; the CPU baseline is the plain-C restatement
    (oracle/kss_oracle.c, OpenMP over nodes at the box's thread share) on the same pods."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import preempt_fixtures as pf
    from kss import abi, native
    from kss.compile import compile_cluster
    n_nodes = args.nodes or 5000
    n_pods = args.pods or 200
    t_gen = time.perf_counter()
    nodes, bound, pods = pf.saturated(11, n_nodes, n_pods)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    t_gen = time.perf_counter() - t_gen
    ps, bs = cp.as_struct(), cc.as_boundset()
    ctx = native.Context(abi.default_profile())
    ctx.load(cc.as_struct())
    ctx.load_bound(bs)
    unsched = []
    for j in range(n_pods):  # the snapshot stays saturated: nothing is committed
        if ctx.eval_pod(ps, j).chosen < 0:
            unsched.append(j)
    for j in unsched[:max(args.warmup, 1) * 3]:
        ctx.postfilter_pod(ps, j)
    host_us, dev_us, nominated, victims = [], [], 0, 0
    nominated_of = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for j in unsched:
            a = time.perf_counter()
            r = ctx.postfilter_pod(ps, j)
            nominated_of[j] = r["nominated"]
            host_us.append((time.perf_counter() - a) * 1e6)
            dev_us.append(ctx.last_timing()[0] * 1e3)
            nominated += r["status"] == abi.KSS_PREEMPT_NOMINATED
            victims += r["n_victims"]
    elapsed = time.perf_counter() - t0
    runs = len(host_us)
    cpu = None
    if not args.no_cpu and unsched:
        # the plain-C restatement (oracle/kss_oracle.c kss_oracle_postfilter: the filter pass, then
        # SelectVictimsOnNode node-parallel over OpenMP, as DryRunPreemption fans out with
        # parallelize.Until), the same pods on the same snapshot, checked against the device's
        # choices on the way
        import oracle_c
        threads, host = cpu_threads()
        prof = abi.default_profile()
        cl = cc.as_struct()
        done, agree, c0 = 0, 0, time.perf_counter()
        while time.perf_counter() - c0 < args.cpu_seconds:
            for j in unsched:
                r = oracle_c.postfilter(prof, cl, ps, j, bs, threads=threads)
                agree += r["nominated"] == nominated_of[j]
                done += 1
                if time.perf_counter() - c0 > args.cpu_seconds:
                    break
        cs = time.perf_counter() - c0
        cpu = {"value": done / cs, "unit": "dry runs/s", "cores": threads, "kind": "port", "host": host,
               "sample": f"{done} dry runs of the {len(unsched)} unschedulable pods of the same saturated "
                         f"{n_nodes}-node cluster (repeated), oracle/kss_oracle.c kss_oracle_postfilter, "
                         f"OpenMP over nodes ({threads} threads), {cs:.1f} s wall",
               "nominations_equal_device": agree == done}
    out = {
        "metric": "DefaultPreemption PostFilter dry runs/sec (unschedulable pods on a saturated cluster)",
        "value": runs / elapsed,
        "unit": "dry runs/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (tests/preempt_fixtures.saturated seed 11)",
        "config": {"workload": f"PostFilter: {n_nodes} saturated nodes, {len(bound)} bound pods, "
                               f"{len(unsched)} unschedulable of {n_pods} pending",
                   "nodes": n_nodes, "bound_pods": len(bound), "dry_runs_per_step": len(unsched)},
        "host_us": {"median": float(np.median(host_us)), "p90": float(np.percentile(host_us, 90))},
        "k_preempt_us": {"median": float(np.median(dev_us)), "mean": float(np.mean(dev_us)),
                         "max": float(np.max(dev_us))},
        "nominated_fraction": nominated / max(runs, 1),
        "victims_per_nomination": victims / max(nominated, 1),
        "compile_s": t_gen,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    ctx.close()


def visible_gpus() -> int:
    """GPUs this process could open, counted without initialising HIP (torch.cuda.device_count
    does not create a context on this image), so a launcher may still spawn rank processes."""
    import torch
    return torch.cuda.device_count()


def free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` started without torchrun: start N rank processes (torch.distributed.run,
    one per GPU, 127.0.0.1) from this process, which never touches the GPU, and return their
    exit code.  Fails clearly when fewer than N GPUs are visible."""
    vis = visible_gpus()
    if n > vis:
        print(f"bench.py: {n} GPUs requested, {vis} visible", file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__), *argv]
    return subprocess.call(cmd, cwd=ROOT)


def rank_env():
    """(world, rank, local_rank) from torchrun's environment (1, 0, 0 without it)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def c4_split_leg(args, world: int, rank: int, local: int, dist) -> dict:
    """The north_star node-axis figure beside the main line: C4 (100,000 nodes x 20,000 pods,
    default profile + zone PTS) scheduled as ONE split grid over all `world` GPUs (world 1:
    the unsplit grid on one GPU), strong scaling.  Each rank runs its part in a child process
    (`bench.py --split 1`, its own gloo group for the IPC handles), so a failing cross-GPU
    exchange is reported in the line instead of ending the bench.  Rank 0's child also times
    the CPU restatement on a bounded C4 prefix.  Returns rank 0's result (others: {})."""
    return child_leg(args, world, rank, local, dist, ["--split", "1", "--split-recipe", "4"], "C4 split",
                     args.c4_timeout, min(args.cpu_seconds, 8.0))


def c5_sweep_leg(args, world: int, rank: int, local: int, dist) -> dict:
    """BASELINE configs[4] beside the main line: 4,096 independent what-if scenarios (KEP-184) x
    1,000 nodes x 1,000 pods in all, 4,096 / world per rank in one resident sweep per GPU (no
    data-path collective), so every world size runs the same whole job (strong scaling; at world
    8 it is the 512-per-GPU shape BASELINE names).  Child processes as in the C4 leg."""
    res = child_leg(args, world, rank, local, dist, ["--scenarios", str(4096 // world)], "C5 sweep",
                    args.c4_timeout, min(args.cpu_seconds, 6.0), traffic=True)
    if res and "error" not in res:
        res["scaling"] = "strong"  # 4,096 scenarios in all at every world size
    return res


def c3_leg(args, world: int, rank: int, local: int, dist) -> dict:
    """BASELINE configs[2] beside the main line: C3 (5,000 nodes x 10,000 pods, default profile +
    PodTopologySpread + InterPodAffinity programs: k_static + k_spread), the same fields as the
    main line (roofline with PMC traffic, latency and VALU rooflines, CPU baseline) from a child
    `bench.py --config 3` run.  At world > 1 every rank schedules its own C3 cluster (weak)."""
    return child_leg(args, world, rank, local, dist, ["--config", "3", "--no-legs"], "C3", args.c4_timeout,
                     min(args.cpu_seconds, 8.0), traffic=True)


def c2_pct0_leg(args, world: int, rank: int, local: int, dist) -> dict:
    """The simulator's own setting beside the main line: C2 with percentageOfNodesToScore = 0,
    the adaptive numFeasibleNodesToFind the simulator's scheduler always runs with
    (simulator/scheduler/scheduler.go:163,258-275): max(5, 50 - 5000/125) = 10 % -> each pod
    filters nodes from nextStartNodeIndex until 500 feasible ones are found, and scores those.
    `evals` counts the filter evaluations the window actually made per pod (the line's
    evals_per_pod), not N."""
    return child_leg(args, world, rank, local, dist, ["--config", "2", "--pct", "0", "--no-legs", "--no-traffic"],
                     "C2 pct=0", args.c4_timeout, min(args.cpu_seconds, 6.0))


def c3_pct0_leg(args, world: int, rank: int, local: int, dist) -> dict:
    """C3 at the simulator's adaptive default (percentageOfNodesToScore = 0: K = 500 of 5,000
    nodes), on k_spread's window (kss_spread.cuh spread_schedule WIN): the PreFilter statistics
    over every node, the filter until the 501st feasible node from nextStartNodeIndex, the score
    over the 500 kept ones."""
    return child_leg(args, world, rank, local, dist, ["--config", "3", "--pct", "0", "--no-legs", "--no-traffic"],
                     "C3 pct=0", args.c4_timeout, min(args.cpu_seconds, 6.0))


def child_leg(args, world: int, rank: int, local: int, dist, mode, label, timeout, cpu_seconds,
              traffic=False) -> dict:
    """Run `bench.py <mode>` as one child process per rank (torchrun's environment passed on, a
    fresh gloo port), after the main timing.  Returns rank 0's JSON line (others: {}), or an
    error record when any rank's child failed."""
    import torch
    port = torch.tensor([free_port() if rank == 0 else 0], dtype=torch.int64)
    if dist:
        dist.broadcast(port, 0)
    env = dict(os.environ, WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(local),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(int(port.item())))
    cmd = [sys.executable, os.path.abspath(__file__), *mode,
           "--steps", str(max(args.steps, 3)), "--warmup", str(max(args.warmup, 1)),
           "--cpu-seconds", str(cpu_seconds)]
    if args.no_cpu:
        cmd.append("--no-cpu")
    if traffic and args.no_traffic:
        cmd.append("--no-traffic")
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
        rc, out, err = r.returncode, r.stdout, r.stderr
    except subprocess.TimeoutExpired as e:
        rc, out, err = "timeout", e.stdout or "", e.stderr or ""
        out = out if isinstance(out, str) else out.decode(errors="replace")
        err = err if isinstance(err, str) else err.decode(errors="replace")
    wall = time.perf_counter() - t0
    res = {}
    if rank == 0:
        lines = [ln for ln in out.splitlines() if ln.startswith("{")]
        if rc == 0 and lines:
            res = json.loads(lines[-1])
        else:
            res = {"error": f"{label} leg failed (rc {rc})", "stderr_tail": err[-600:]}
        res["leg_wall_s"] = wall
    ok = torch.tensor([1 if rc == 0 else 0], dtype=torch.int64)
    if dist:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if rank == 0 and not ok.item() and "error" not in res:
        res["error"] = f"a peer rank's {label} child failed"
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=0,
                    help="GPUs (rank processes); without torchrun, N > 1 starts the N ranks itself")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=0)
    ap.add_argument("--pods", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 FETCH/WRITE_SIZE passes")
    ap.add_argument("--inner", action="store_true", help="child run under the profiler: no CPU leg, no traffic")
    ap.add_argument("--scenarios", type=int, default=0,
                    help="C5 shape: this many independent what-if clusters per rank in one launch")
    ap.add_argument("--node-axis", action="store_true",
                    help="C4 shape: one cluster sharded along the node axis over the ranks (RCCL per pod)")
    ap.add_argument("--split", type=int, default=0,
                    help="C4 node axis as one split grid over the ranks' GPUs (world 1: this many parts on one GPU)")
    ap.add_argument("--split-recipe", type=int, default=4, choices=(2, 4),
                    help="--split pod recipe: 4 (C4: zone PTS, k_spread) or 2 (default profile, k_simple)")
    ap.add_argument("--per-pod", action="store_true", help="the drop-in per-pod API: kss_eval_pod + kss_commit")
    ap.add_argument("--no-latency", action="store_true", help="skip the stamped latency-profile run")
    ap.add_argument("--postfilter", action="store_true", help="DefaultPreemption PostFilter dry runs (kss_postfilter_pod)")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 split-grid leg of the main line")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 scenario-sweep leg of the main line")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 (PTS + IPA, k_spread) leg of the main line")
    ap.add_argument("--no-pct0", action="store_true", help="skip the C2 / C3 percentageOfNodesToScore=0 legs of the main line")
    ap.add_argument("--no-legs", action="store_true", help="no extra legs (the legs' own child runs)")
    ap.add_argument("--pct", type=int, default=100,
                    help="percentageOfNodesToScore of the profile (100: every node, the north_star setting; "
                         "0: the simulator's adaptive default)")
    ap.add_argument("--c4-timeout", type=float, default=420.0, help="seconds for the C4 split-grid leg")
    ap.add_argument("--snapshot", action="store_true",
                    help="the simulator's snapshot path: a ResourcesForSnap JSON read back, compiled, scheduled "
                         "with the profile the simulator's config gives (percentageOfNodesToScore 0)")
    args = ap.parse_args()
    if args.inner:
        args.no_cpu = args.no_traffic = args.no_latency = args.no_legs = True
    if args.no_legs:
        args.no_c3 = args.no_pct0 = args.no_c4 = args.no_c5 = True
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if world_env is not None and args.gpus and int(world_env) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}")
    if world_env is not None and int(os.environ.get("LOCAL_RANK", "0")) >= max(1, visible_gpus()):
        sys.exit(f"bench.py: LOCAL_RANK {os.environ.get('LOCAL_RANK')} but {visible_gpus()} GPU(s) visible")
    if args.per_pod:
        return run_per_pod(args)
    if args.snapshot:
        return run_snapshot(args)
    if args.postfilter:
        return run_postfilter(args)
    if args.split:
        return run_split(args)
    if args.node_axis:
        return run_node_axis(args)
    if args.scenarios:
        return run_scenarios(args)

    world, rank, local = rank_env()
    dist = None
    if world > 1:
        import torch.distributed as dist  # control plane only (barrier / max of timings)
        dist.init_process_group("gloo", rank=rank, world_size=world)

    cfg = args.config
    traffic, traffic_detail = None, "not measured"
    sq, sq_detail = None, "not measured"
    if rank == 0 and world == 1 and not args.no_traffic:
        traffic, traffic_detail = measure_traffic(args, cfg, timeout=300 if cfg == 4 else 120)
        sq, sq_detail = measure_sq(args, cfg, timeout=300 if cfg == 4 else 120)

    from kss import abi, native
    from kss.synth import DEFAULT_SIZES, SEED_BASE

    n_nodes = args.nodes or DEFAULT_SIZES[cfg][0]
    n_pods = args.pods or DEFAULT_SIZES[cfg][1]
    seed = rank_seed(SEED_BASE, cfg, rank)
    s = native.Synth(cfg, seed, n_nodes, n_pods)
    prof = abi.default_profile()
    prof.pct_nodes_to_score = args.pct
    ctx = native.Context(prof, device=local)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    import numpy as np
    chosen = np.zeros(n_pods, np.int32)
    xcd_fallbacks = []

    loop_ms = []

    def step():
        ctx.reset()
        ctx.run_staged(n_pods, out=chosen)
        loop_ms.append(ctx.last_loop_ms())
        xcd_fallbacks.append(ctx.last_xcd_local().get("fallbacks", 0))
        return ctx.last_timing()[0]

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    kern_ms = []
    for _ in range(args.steps):
        kern_ms.append(step())
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    scheduled = int((chosen >= 0).sum())
    elapsed, scheduled_total = reduce_over_ranks(elapsed, scheduled, dist)

    # filter + score evaluations per pod: every node at pct=100; below, the window's
    # numFeasibleNodesToFind (a lower bound of the nodes it filters, stated in the line)
    evals_per_pod = num_feasible_nodes_to_find(n_nodes, args.pct)
    evals = world * n_pods * evals_per_pod * args.steps
    value = evals / elapsed
    pods_per_s = scheduled_total * args.steps / elapsed
    kern_avg_s = sum(kern_ms) / len(kern_ms) / 1e3
    loop_s = sum(loop_ms[-args.steps:]) / args.steps / 1e3  # the dominant kernel (k_simple / k_schedule) alone
    achieved = B_EVAL[cfg] * n_pods * n_nodes / loop_s / 1e9  # = per-launch bytes / mean launch time
    # loop-kernel launches per step: one per static chunk (C4: several); from the PMC run when it
    # ran, else from the chunk size the library reports
    launches = traffic_detail.get("launches", 0) if isinstance(traffic_detail, dict) else 0
    launches = launches or max(1, ctx.last_timing()[1] // 2 if ctx.last_kernel() != "k_schedule" else 1)

    print(json.dumps({"rank": rank, "device": local, "world_size": world, "pods_scheduled": scheduled,
                      "elapsed_s": t1 - t0}), file=sys.stderr, flush=True)
    # the node-axis figure (C4 split grid over every rank's GPU) once the main timing is done
    main_shape = cfg == 2 and not args.nodes and not args.pods and args.pct == 100
    c4 = None if args.no_c4 or not main_shape else c4_split_leg(args, world, rank, local, dist)
    c5 = None if args.no_c5 or not main_shape else c5_sweep_leg(args, world, rank, local, dist)
    c3 = None if args.no_c3 or not main_shape else c3_leg(args, world, rank, local, dist)
    c2p0 = None if args.no_pct0 or not main_shape else c2_pct0_leg(args, world, rank, local, dist)
    c3p0 = None if args.no_pct0 or not main_shape else c3_pct0_leg(args, world, rank, local, dist)
    if rank == 0:
        cpu = None
        if not args.no_cpu and world == 1:
            threads, _ = cpu_threads()
            cpu = cpu_baseline(cfg, n_nodes, n_pods, args.cpu_seconds, threads, seed=seed, pct=args.pct)
        latency = None
        if not args.no_latency and world == 1:
            latency = latency_profile(cfg, n_nodes, n_pods, seed, local, pct=args.pct)
            latency["us_per_pod"] = elapsed / args.steps / n_pods * 1e6
            if latency.get("bound_us_per_pod"):
                latency["frac"] = latency["bound_us_per_pod"] / latency["us_per_pod"]
        out = {
            "metric": "pod x node filter+score evals/sec (pods scheduled/sec in extra)",
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64/f64",
            "data": "synthetic (SplitMix64 seed 0x5EED0000+config[+7919*rank])",
            "config": {"workload": f"C{cfg}: {n_nodes} nodes x {n_pods} pods, {RECIPE[cfg]}, sequential, "
                                   f"pct={args.pct}"
                                   + (f"; one independent cluster per GPU (seed + rank) x{world}" if world > 1 else ""),
                       "nodes": n_nodes, "pods": n_pods, "parallelism": f"scenario x{world}",
                       "percentage_of_nodes_to_score": args.pct},
            "evals_per_pod": evals_per_pod,
            "evals_note": ("every node filtered and scored" if evals_per_pod == n_nodes else
                           f"numFeasibleNodesToFind = {evals_per_pod} per pod: the window filters at least this many "
                           "nodes (more when some are infeasible) and scores at most this many"),
            "pods_per_s": pods_per_s,
            "pods_scheduled_per_step": scheduled,
            "kernel_ms_per_step": kern_avg_s * 1e3,
            "loop_kernel_ms_per_step": loop_s * 1e3,
            "us_per_pod": elapsed / args.steps / n_pods * 1e6,
            "geometry": ctx.last_geometry(),
            "xcd_fallbacks": int(sum(xcd_fallbacks[-args.steps:])),
            "xcd_local": ctx.last_xcd_local().get("used", 0),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": ctx.last_kernel(), "bytes_per_eval": B_EVAL[cfg],
                         "launches_per_step": launches,
                         "algorithmic_bytes_per_launch": B_EVAL[cfg] * n_pods * n_nodes / launches,
                         "traffic_detail": traffic_detail, "latency": latency,
                         "valu": valu_roofline(sq, loop_s, n_pods * n_nodes), "valu_detail": sq_detail},
            "cpu_baseline": cpu,
            "gpu_over_cpu": gpu_over_cpu(pods_per_s, cpu),
            "c4_split": c4,
            "c5_sweep": c5,
            "c3": c3,
            "c2_pct0": c2p0,
            "c3_pct0": c3p0,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    s.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
