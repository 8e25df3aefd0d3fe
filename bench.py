#!/usr/bin/env python3
"""Benchmark of the hot path: batched IFOPT eval_g + eval_jac_g of CentroidalPlanner instances.

One step = one pass of the hot path over one batch resident in HBM: the fused eval kernel (values
+ CSR Jacobian values of every instance + per-workgroup residual partials) and the one-workgroup
finish of the per-shard residual norms.  Steps run in buckets (--bucket, default 10): one HIP-graph
replay launches a bucket's steps, and with N > 1 ranks one RCCL all-gather (asynchronous, on the
collective stream) carries the bucket's per-step norms.  Instances shard
across ranks with no data-path exchange: per-rank batch is fixed -> weak scaling.

Default workload = the north-star point BASELINE.json's metric is quoted on: 4-contact Ground env,
batch 1,048,576 per GPU (1.95 GB of algorithmic traffic per step, far past the 256 MiB Infinity
Cache).  BASELINE.json configs[1] (65,536 instances) is reported beside it as a side field.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config ground4_1m|ground4|sq8|mixed16|none4|solve5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Rank 0 prints one JSON line.  Fields beyond the driver contract:
  roofline      dominant kernel (cpl_eval_*): algorithmic bytes per launch / mean launch
                duration from HIP events on the launch stream; traffic = HBM bytes per launch from
                rocprofv3 PMC passes (FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE)
  cpu_baseline  the oracle (CPU restatement, "port") on the host cores, bounded sample, plus a
                single-core figure, the CPU model and the affinity count
  check         checker leg (after timing): a strided sample of the TIMED g / jac against the oracle
  jac_folded    the same batch with values-only Jacobian records (CPL_EVAL_JAC_FOLDED: structural
                constants skipped), kernel time and bytes
  configs1_65k  BASELINE.json configs[1] (65,536 x 4 Ground) kernel time on the same GPU
  configs2_sq8  BASELINE.json configs[2] (262,144 x 8 Superquadric): kernel time, HBM fraction, VALU
                roofline (PMC), checker sample
  configs3_mixed16  BASELINE.json configs[3]'s 1,048,576 x 16 mixed batch on one GPU: kernel time, HBM
                fraction, per-kind checker sample
  configs3_mixed16_shard  one rank's shard of configs[3] sharded over 8 GPUs (131,072 x 16 mixed) through
                the same split launch: kernel time and predicted_strong_speedup_8 = t(1,048,576) / t(131,072)
  configs4_solve5_lbfgs  BASELINE.json configs[4] (8,192 concurrent solves) in the reference's Hessian
                mode (IPOPT's L-BFGS): solves/s, iterations, and the compiled restatement of the same
                iteration (oracle/cpl_solve_host.c) on all usable host cores (OpenMP over instances) and
                on one core;
                .single_solve: one instance solved alone (CentroidalPlanner::Solve()'s batch of one):
                GPU ms per solve beside that compiled restatement on one core
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "NLP eval_g+eval_jac_g throughput (rows/sec) at batch*contacts; HBM GB/s vs peak"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
KERNEL_NAME = "cpl_eval"  # matches cpl_eval_pipe_kernel / _entry_kernel (none/Ground), cpl_eval_tile_kernel, cpl_eval_kernel


def algorithmic_bytes(N, env, outputs=("g", "jac"), with_mass=True):
    """Per instance: read x (3+9N) [+ mass]; write g (m) + jac (nnz) [+ f + grad (n)]."""
    has_env = env != "none"
    n = 3 + 9 * N
    m = 6 + (6 if has_env else 2) * N
    nnz = 6 + 15 * N + (27 if has_env else 12) * N
    b = n + (1 if with_mass else 0)
    if "g" in outputs:
        b += m
    if "jac" in outputs:
        b += nnz
    if "f" in outputs:
        b += 1
    if "grad" in outputs:
        b += n
    return 8 * b, m


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment, N > 1 spawns N rank processes")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="ground4_1m", help="ground4_1m | ground4 | sq8 | mixed16 | none4 | solve5")
    ap.add_argument("--batch", type=int, default=0, help="override per-GPU batch")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-side", action="store_true", help="skip the configs[1] side measurement")
    ap.add_argument("--no-check", action="store_true", help="skip the checker leg")
    ap.add_argument("--check-sample", type=int, default=4096, help="instances in the checker leg's strided sample")
    ap.add_argument("--no-graph", action="store_true", help="launch each step from Python instead of a HIP graph")
    ap.add_argument("--collective-always", action="store_true",
                    help="tests: the RCCL process group and the bucketed norms all-gather even at one rank")
    ap.add_argument("--bucket", type=int, default=10,
                    help="steps per HIP-graph replay and per residual-norm all-gather (1 = per step)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--max-ls", type=int, default=40, help="solve5: backtracking trials per iteration at most")
    ap.add_argument("--max-soc", type=int, default=4, help="solve5: second-order corrections on the first trial")
    ap.add_argument("--ls-kernel", type=int, default=2, help="solve5: the engine's ls_kernel option (0 / 1 / 2)")
    ap.add_argument("--hessian", default="exact", choices=["exact", "limited-memory"],
                    help="solve5: exact Lagrangian Hessian (analytic kernel) or IFOPT's limited-memory default")
    ap.add_argument("--cpu-sample", type=int, default=512, help="solve5: instances in the CPU baseline's sample")
    ap.add_argument("--pmc-child", default="", help=argparse.SUPPRESS)
    # CPU rehearsal of the multi-rank launch (tests only: gloo, the shard's evaluation supplied by a
    # file the test names; never on a GPU run)
    ap.add_argument("--rehearse-cpu", default="", help=argparse.SUPPRESS)
    return ap.parse_args()


# ------------------------------------------------------------------------------------------
# multi-rank launch: one process per GPU
# ------------------------------------------------------------------------------------------
def resolve_world(args):
    """(world, rank, local_rank, spawn): WORLD_SIZE / RANK / LOCAL_RANK from the environment (the
    driver's torch.distributed.run launch); without them, --gpus N > 1 asks this process to spawn the
    N ranks itself.  A --gpus that disagrees with WORLD_SIZE is refused."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world}")
        return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")), False
    n = 1 if args.gpus is None else int(args.gpus)
    if n < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    return n, 0, 0, n > 1


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(world, argv=None, poll_s=0.5):
    """`python bench.py --gpus N` with no WORLD_SIZE: start N fresh rank processes of this script
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1, a free MASTER_PORT) — this parent
    makes no GPU call, so every rank (rank 0's PMC passes and CPU leg included) starts from a clean
    process.  Rank 0's stdout (the JSON line) is forwarded; the other ranks' stdout goes to stderr.
    If a rank fails, the others are stopped and the exit code is non-zero."""
    argv = sys.argv[1:] if argv is None else list(argv)
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (the only kind the host supports)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(),
                                      start_new_session=True))
    import threading

    lines = []

    def pump():  # rank 0's stdout, read as it comes (a full pipe would stall the rank)
        for raw in procs[0].stdout:
            lines.append(raw.decode(errors="replace"))

    th = threading.Thread(target=pump, daemon=True)
    th.start()
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            # a rank's failure usually takes its peers' collectives down with it: give them a moment to
            # exit on their own so that every rank that failed by itself is named, not just the lowest
            t_end = time.time() + 3.0
            while time.time() < t_end and any(p.poll() is None for p in procs):
                time.sleep(poll_s)
            failed = [(r, p.poll()) for r, p in enumerate(procs) if p.poll() not in (None, 0)]
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(poll_s)
    if failed is not None:
        import signal

        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
    th.join(timeout=30)
    for ln in lines:
        if ln.lstrip().startswith("{"):
            sys.stdout.write(ln)
        else:
            sys.stderr.write(ln)
    sys.stdout.flush()
    if failed is not None:
        for r, c in failed:
            print(f"bench.py: rank {r} exited with {c}", file=sys.stderr)
        return 1
    return 0


def rehearse_cpu(args, world, rank):
    """CPU rehearsal of the multi-rank bench (tests: gloo on CPU ranks).  The same shard, bucketed
    step loop (distributed.BucketedNormGather) and max-over-ranks timing as the GPU path; the shard's
    per-step residual norms come from ``norms(prob, x, mass, tag) -> [max, sumsq]`` defined in the
    file --rehearse-cpu names (a test file: the CPU stands in for the rank's GPU).  Prints the line
    with roofline = null."""
    import importlib.util

    import torch
    import torch.distributed as dist

    from centroidalplanner_amd.distributed import BucketedNormGather, shard
    from centroidalplanner_amd.workload import CONFIGS, generate, make_problem

    spec = importlib.util.spec_from_file_location("_bench_rehearsal", args.rehearse_cpu)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    cfg = CONFIGS[args.config]
    total = args.batch or cfg.batch
    start, batch = shard(total, rank, world) if cfg.config_id == 4 and not args.batch else (0, total)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    prob = make_problem(cfg.n_contacts, cfg.env)
    x, mass, tag = generate(cfg.n_contacts, cfg.env, batch, 0xC910 + cfg.config_id + 7919 * rank)
    local = torch.tensor(mod.norms(prob, x, mass, tag), dtype=torch.float64)

    def launch(rows, count):
        for s in range(count):
            rows[s].copy_(local)

    K, W = args.steps, args.warmup
    runner = BucketedNormGather(world, max(1, min(args.bucket, K)), torch.device("cpu"), launch)
    for w in runner.run(W):
        if w is not None:
            w.wait()
    runner.reset()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for w in runner.run(K):
        if w is not None:
            w.wait()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    gather = None
    totals = torch.tensor([dt, float(batch)], dtype=torch.float64)
    if world > 1:
        t = totals[:1].clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        b = totals[1:].clone()
        dist.all_reduce(b, op=dist.ReduceOp.SUM)
        dt, total_rows = float(t.item()), int(b.item())
        gather = runner.last_bucket_report(rank, K)
    else:
        total_rows = batch
    _, m = algorithmic_bytes(cfg.n_contacts, cfg.env)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": total_rows * m * K / dt, "unit": "rows/s", "n_gpus": world,
                          "steps": K, "warmup": W, "ms_per_step": dt / K * 1e3, "higher_is_better": True,
                          "scaling": scaling_of(cfg, args), "vs_baseline": None, "dtype": "f64",
                          "data": "synthetic (CPU rehearsal of the multi-rank launch)",
                          "config": {"workload": cfg.name, "batch_per_gpu": batch, "batch_total": total_rows,
                                     "parallelism": f"instance-sharded x{world} (gloo, CPU rehearsal)"},
                          "residual_gather": gather, "roofline": None, "cpu_baseline": None}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def scaling_of(cfg, args):
    """configs[3] is quoted as 1,048,576 instances over the node: sharded, its total is fixed (strong
    scaling); every other config keeps its per-GPU batch (weak scaling)."""
    return "strong" if cfg.config_id == 4 and not args.batch else "weak"


# ------------------------------------------------------------------------------------------
# PMC traffic (child processes under rocprofv3; run before this process touches the GPU)
# ------------------------------------------------------------------------------------------
def pmc_child(args):
    """Runs the eval kernel a few times; executed under rocprofv3 --pmc."""
    import torch
    from centroidalplanner_amd.workload import CONFIGS, config_inputs

    cfg = CONFIGS[args.config]
    prob, x, mass, tag = config_inputs(cfg, args.batch or cfg.batch)
    dev = torch.device("cuda:0")
    xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
    tt = None if tag is None else torch.tensor(tag, device=dev)
    out = prob.eval_batch(xt, mt, tt, outputs=("g", "jac"))
    for _ in range(PMC_LAUNCHES - 1):
        prob.eval_batch(xt, mt, tt, outputs=("g", "jac"), out=out)
    torch.cuda.synchronize()


PMC_LAUNCHES = 6  # eval launches of the pmc child


def _pmc_pass(args, counters, timeout=240):
    """One rocprofv3 --pmc pass over the pmc child; returns {counter: per eval LAUNCH} — the sum over
    the eval kernels' dispatches / the child's launches (a mixed batch's default launch is two
    kernels, the kind split's Ground and Superquadric halves)."""
    import csv

    rocprof = "/opt/rocm/bin/rocprofv3"
    d = tempfile.mkdtemp(prefix="cpl_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = [rocprof, "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--pmc-child", "1", "--config", args.config]
    if args.batch:
        cmd += ["--batch", str(args.batch)]
    subprocess.run(cmd, check=True, timeout=timeout, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd=ROOT)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise RuntimeError(f"no counter csv for {counters}")
    per = {}
    with open(files[0]) as fh:
        for row in csv.DictReader(fh):
            if KERNEL_NAME in row.get("Kernel_Name", ""):
                per.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
                per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    if not per:
        raise RuntimeError(f"no {counters} rows for {KERNEL_NAME}")
    return {k: sum(v.values()) / PMC_LAUNCHES for k, v in per.items()}


def collect_pmc(args, timeout=240):
    """HBM traffic of the eval kernel: FETCH_SIZE and WRITE_SIZE in separate passes."""
    if not os.path.exists("/opt/rocm/bin/rocprofv3"):
        return None, "rocprofv3 not found"
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        try:
            vals.update(_pmc_pass(args, [counter], timeout))  # KB per dispatch
        except Exception as e:  # noqa: BLE001
            return None, f"rocprofv3 {counter} pass failed: {e}"
    # gfx950: FETCH_SIZE reads 1/2 of a wide coalesced stream's bytes (MI355X_MICROARCH.md §HBM)
    traffic = (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
    return traffic, vals


# FP64 VALU of MI355X: 78.6 TFLOP/s = 256 CUs x 4 SIMDs x 16 FMA lanes x 2 x 2.4 GHz, i.e. one wave64
# FP64 instruction per SIMD per 4 cycles; f32 / integer VALU one per 2 cycles (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6
CLK_HZ = 2.4e9
SIMDS = 256 * 4
VALU_PASSES = (("SQ_INSTS_VALU", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_SALU"),
               ("SQ_INSTS_VALU_FLOPS_FP64", "SQ_INSTS_VALU_FLOPS_FP64_TRANS", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES",
                "SQ_WAIT_ANY"))


def collect_valu_counters(args, timeout=240):
    c = {}
    for counters in VALU_PASSES:
        c.update(_pmc_pass(args, counters, timeout))
    return c


def valu_roofline(c, kernel_ms):
    """The VALU roofline of a transcendental-heavy eval kernel (Superquadric / mixed) from PMC passes:
    issue_frac = the kernel's VALU issue cycles at full rate (4 cycles per wave64 FP64 instruction,
    2 otherwise, over 1024 SIMDs at 2.4 GHz) / its duration; fp64 TFLOP/s = 64 lanes x
    SQ_INSTS_VALU_FLOPS_FP64(+_TRANS) / duration against the 78.6 TFLOP/s FP64 vector peak.
    c: counters per eval launch (collect_valu_counters, run before this process touches the GPU)."""
    t = kernel_ms * 1e-3
    f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                       "SQ_INSTS_VALU_TRANS_F64"))
    issue_s = (4.0 * f64 + 2.0 * (c["SQ_INSTS_VALU"] - f64)) / (SIMDS * CLK_HZ)
    tflops = 64.0 * (c.get("SQ_INSTS_VALU_FLOPS_FP64", 0.0) + c.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0.0)) / t / 1e12
    return {
        "bound": "valu", "achieved": tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
        "frac": tflops / FP64_PEAK_TFLOPS, "issue_frac": issue_s / t, "issue_bound_ms": issue_s * 1e3,
        "wait_frac": c.get("SQ_WAIT_ANY", 0.0) / max(c.get("SQ_WAVE_CYCLES", 1.0), 1.0),
        "valu_active_frac": c.get("SQ_ACTIVE_INST_VALU", 0.0) / max(c.get("SQ_WAVE_CYCLES", 1.0), 1.0),
        "counters_per_launch": c,
    }


# ------------------------------------------------------------------------------------------
# CPU baseline: the oracle (CPU restatement of the reference path) on the host cores
# ------------------------------------------------------------------------------------------
def host_cpu_info():
    """CPU model, the affinity count of this process and the threads the CPU legs use.  Threads =
    the CPUs this process may run on (sched_getaffinity), capped by OMP_NUM_THREADS when the
    environment sets it (the GPU box sets it to the box's CPU share, 16 per GPU: its affinity mask
    shows the whole host)."""
    affinity = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(affinity, omp) if omp > 0 else affinity
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "affinity": affinity, "omp_num_threads": omp or None, "threads": threads}


def cpu_baseline(cfg, seconds):
    """The oracle on the host cores: a fixed sample of the workload evaluated `reps` times so that
    the timed CPU work lasts about `seconds` (10-30 s) on every usable core (host_cpu_info), then a
    smaller sample on one core for about a quarter of that."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from centroidalplanner_amd.workload import config_inputs

    info = host_cpu_info()
    threads = info["threads"]
    B = min(cfg.batch, 262144)
    prob, x, mass, tag = config_inputs(cfg, B)
    t1 = pyoracle.time_eval_batch(prob.desc(), x, mass, tag, outputs=("g", "jac"), nthreads=threads, reps=1)
    reps = max(1, int(round(seconds / max(t1, 1e-6))))
    t = pyoracle.time_eval_batch(prob.desc(), x, mass, tag, outputs=("g", "jac"), nthreads=threads, reps=reps)
    _, m = algorithmic_bytes(cfg.n_contacts, cfg.env)  # t: seconds per pass
    # single core: the first B1 instances of the same sample
    B1 = min(B, 16384)
    s1 = pyoracle.time_eval_batch(prob.desc(), x[:B1], None if mass is None else mass[:B1],
                                  None if tag is None else tag[:B1], outputs=("g", "jac"), nthreads=1, reps=1)
    reps1 = max(1, int(round(0.25 * seconds / max(s1, 1e-6))))
    s1 = pyoracle.time_eval_batch(prob.desc(), x[:B1], None if mass is None else mass[:B1],
                                  None if tag is None else tag[:B1], outputs=("g", "jac"), nthreads=1, reps=reps1)
    return {
        "value": B * m / t,
        "unit": "rows/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{B} instances of '{cfg.name}' x {reps} passes (g+jac, IFOPT-order assembly) in {t * reps:.1f} s "
                  f"on {threads} threads",
        "instances_per_s": B / t,
        "single_core": {"value": B1 * m / s1, "unit": "rows/s", "instances_per_s": B1 / s1,
                        "sample": f"{B1} instances x {reps1} passes in {s1 * reps1:.1f} s on 1 thread"},
        **{k: info[k] for k in ("cpu_model", "affinity", "omp_num_threads")},
    }


def single_instance_latency(prob, cfg, dev, reps=2000):
    """The single-instance TNLP path (one IPOPT callback pair per launch):
    microseconds per eval_g + eval_jac_g of ONE instance, host x in, host g / jac out — H2D copy of x
    from pinned memory, one cpl_eval_batch launch, D2H of g and jac, stream synchronise — against
    the oracle's single-instance time on one core (the CPU restatement, IFOPT-order assembly).  Tells
    integrators where batching starts to pay."""
    import ctypes

    import numpy as np
    import torch

    from centroidalplanner_amd import _abi
    from centroidalplanner_amd.workload import generate

    n, m, nnz = prob.get_nlp_info()
    x, mass, tag = generate(cfg.n_contacts, cfg.env, 1, 12345)
    hx = torch.tensor(x, dtype=torch.float64).pin_memory()
    hg = torch.empty(1, m, dtype=torch.float64).pin_memory()
    hj = torch.empty(1, nnz, dtype=torch.float64).pin_memory()
    dx = torch.empty(1, n, dtype=torch.float64, device=dev)
    dg = torch.empty(1, m, dtype=torch.float64, device=dev)
    dj = torch.empty(1, nnz, dtype=torch.float64, device=dev)
    dt = None if tag is None else torch.tensor(tag, device=dev)
    s = torch.cuda.Stream(dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    desc = prob.desc()
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731

    def once():
        with torch.cuda.stream(s):
            dx.copy_(hx, non_blocking=True)
            _abi.check(_abi.lib.cpl_eval_batch(ctypes.byref(desc), 1, p(dx), None, p(dt), p(dg), p(dj), None, None, sp))
            hg.copy_(dg, non_blocking=True)
            hj.copy_(dj, non_blocking=True)
        s.synchronize()

    for _ in range(50):
        once()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    staged_us = (time.perf_counter() - t0) / reps * 1e6

    # the product entry a TNLP adapter binds: cpl_eval_batch_host on ordinary (pageable) host arrays,
    # as IPOPT hands them over (zero-copy through the library's pinned staging at this size)
    ax = np.ascontiguousarray(x, dtype=np.float64)
    ag, aj = np.empty((1, m)), np.empty((1, nnz))
    at = None if tag is None else np.ascontiguousarray(tag, dtype=np.uint8)
    ptr = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731

    def host_once():
        _abi.check(_abi.lib.cpl_eval_batch_host(ctypes.byref(desc), 1, ptr(ax), None, ptr(at), ptr(ag), ptr(aj),
                                                None, None, None, 0))

    for _ in range(50):
        host_once()
    t0 = time.perf_counter()
    for _ in range(reps):
        host_once()
    gpu_us = (time.perf_counter() - t0) / reps * 1e6
    res = {"gpu_us_per_callback_pair": gpu_us,
           "path": "cpl_eval_batch_host(B=1) on pageable host arrays: memcpy into pinned staging, one launch reading x "
                   "and writing g, jac in host memory, stream sync, memcpy out",
           "staged_device_api_us": staged_us,
           "staged_device_api_path": "pinned H2D x + cpl_eval_batch(B=1) + D2H g, jac + stream sync"}
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle

        xs = np.repeat(x, 4096, axis=0)
        t = pyoracle.time_eval_batch(desc, xs, None, None if tag is None else np.repeat(tag, 4096), outputs=("g", "jac"),
                                     nthreads=1, reps=3)
        res["cpu_us_per_instance_one_core"] = t / xs.shape[0] * 1e6
        res["break_even_batch"] = gpu_us / res["cpu_us_per_instance_one_core"]
    except Exception as e:  # noqa: BLE001
        res["cpu_error"] = str(e)
    return res


def eigen_order_field(prob, env, x, mass, tag, got, ref):
    """The kernels' outputs against the oracle built in the other plausible Eigen reduction order
    (a0 b0 + (a1 b1 + a2 b2), tests/eigen_order.py): per output class that differs, the largest
    deviation in ulps (2^-52) of the un-cancelled terms (cone values, cone Jacobian row 1, normal rows)
    or of the value itself — DESIGN.md section 3's bounds, carried by every bench line."""
    from eigen_order import order_deviation

    r = order_deviation(prob, env, x, mass, tag, got={"g": got["g"], "jac": got["jac"]})
    eps = 2.0 ** -52
    cls = {}
    worst_unc, worst_plain = 0.0, 0.0
    for k, v in r.items():
        if not isinstance(v, dict) or not v.get("differ"):
            continue
        if "max_rel_uncancelled" in v:  # (cone values, cone Jacobian row 1, normal rows: cancelling terms)
            u = v["max_rel_uncancelled"] / eps
            worst_unc = max(worst_unc, u)
            cls[k] = {"differ": v["differ"], "entries": v["entries"], "max_ulps_uncancelled": u}
        else:  # every other class: relative to the value itself
            u = v["max_rel"] / eps
            worst_plain = max(worst_plain, u)
            cls[k] = {"differ": v["differ"], "entries": v["entries"], "max_ulps_plain": u}
    return {"max_ulps_uncancelled": worst_unc, "max_ulps_plain_other": worst_plain, "classes": cls}


def checker_leg(prob, env, xt, mt, tt, out, batch, sample):
    """Checker (outside every timed region): a strided sample of the instances whose g / jac the
    timed steps wrote, recomputed by the oracle from the same device inputs and compared with the
    parity policy of tests/parity_util.py (bit-identical for everything without a data-dependent
    pow).  Test infrastructure: the oracle is the checker here, never the thing measured."""
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import pyoracle
    from parity_util import check_outputs

    dev = xt.device
    if tt is None:  # one kind: a strided sample of the batch plus its tail
        stride = max(1, batch // max(1, sample))
        groups = {env: torch.unique(torch.cat([torch.arange(0, batch, stride, device=dev),
                                               torch.tensor([batch - 1], device=dev)]))}
    else:  # mixed batch: a strided sample of EACH environment kind (plus each kind's last instance)
        kinds = {1: "ground", 2: "superquadric"}
        groups = {}
        for code, name in kinds.items():
            members = torch.nonzero(tt == code).flatten()
            if members.numel() == 0:
                continue
            stride = max(1, members.numel() // max(1, sample // len(kinds)))
            pick = torch.unique(torch.cat([torch.arange(0, members.numel(), stride, device=dev),
                                           torch.tensor([members.numel() - 1], device=dev)]))
            groups[name] = members[pick]
    res = {"instances": 0, "policy": "tests/parity_util.py", "ok": True, "per_kind": {}}
    finite = True
    for kind, idx in groups.items():
        x = xt[idx].cpu().numpy()
        mass = mt[idx].cpu().numpy() if mt is not None else None
        tag = tt[idx].cpu().numpy() if tt is not None else None
        got = {k: out[k][idx].cpu().numpy() for k in ("g", "jac")}
        ref = pyoracle.eval_batch(prob.desc(), x, mass, tag, outputs=("g", "jac"))
        part = {"instances": int(idx.numel())}
        try:
            rep = check_outputs(prob, env, x, got, ref, tag)
            part["ok"] = True
            part["bitwise_frac"] = {k: v["bitwise_frac"] for k, v in rep.items()}
            # the entries outside the north-star bound read literally (plain relative 1e-10; the policy's
            # scaled bound is what `ok` asserts) and the largest plain relative error
            part["outside_plain_1e-10"] = {k: v["plain_rel_hist"]["ge1e-10"] for k, v in rep.items()}
            part["max_plain_rel_err"] = {k: v["max_plain_rel_err"] for k, v in rep.items()}
            part["eigen_order"] = eigen_order_field(prob, env, x, mass, tag, got, ref)
        except AssertionError as e:
            part["ok"] = False
            part["error"] = str(e)[:400]
        res["per_kind"][kind] = part
        res["instances"] += part["instances"]
        res["ok"] = res["ok"] and part["ok"]
        finite = finite and bool(np.isfinite(got["g"]).all() and np.isfinite(got["jac"]).all())
    if len(groups) == 1:  # (the single-kind line keeps its flat fields)
        only = next(iter(res["per_kind"].values()))
        res.update({k: v for k, v in only.items() if k != "instances"})
    res["finite"] = finite
    return res


# ------------------------------------------------------------------------------------------
# side fields of the default run: the other BASELINE.json configs on the driver's clock
# ------------------------------------------------------------------------------------------
def side_sq8(dev, stream, valu_counters, check_sample=1024):
    """BASELINE.json configs[2] (262,144 x 8 Superquadric) on the same GPU: the eval kernel's time
    (HIP events on the launch stream), its HBM fraction, its VALU roofline (PMC passes collected
    before this process touched the GPU) and a checker sample of every kernel output."""
    import ctypes

    import torch

    from centroidalplanner_amd import _abi
    from centroidalplanner_amd.workload import CONFIGS, generate, make_problem

    cfg = CONFIGS["sq8"]
    B = cfg.batch
    prob = make_problem(cfg.n_contacts, cfg.env)
    x, mass, tag = generate(cfg.n_contacts, cfg.env, B, 0xC910 + cfg.config_id)
    xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
    del x, mass
    out = prob.eval_batch(xt, mt, outputs=("g", "jac", "norms"))
    ms = ctypes.c_double()
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    rounds = []
    for _ in range(5):  # the median of five timed rounds of 20 launches (the first warms the clocks)
        _abi.check(_abi.lib.cpl_time_eval_batch(ctypes.byref(prob.desc()), B, p(xt), p(mt), None, p(out["g"]),
                                                p(out["jac"]), None, None, p(out["norms"]),
                                                ctypes.c_void_p(stream.cuda_stream), 20, ctypes.byref(ms)))
        rounds.append(ms.value)
    ms.value = sorted(rounds)[len(rounds) // 2]
    bytes_inst, m = algorithmic_bytes(cfg.n_contacts, cfg.env)
    res = {"workload": cfg.name, "kernel_ms": ms.value, "rows_per_s": B * m / (ms.value * 1e-3),
           "hbm_gbps": bytes_inst * B / (ms.value * 1e-3) / 1e9,
           "frac_of_peak": bytes_inst * B / (ms.value * 1e-3) / 1e9 / HBM_PEAK_GBPS,
           "bytes_per_instance": bytes_inst}
    if isinstance(valu_counters, dict):
        v = valu_roofline(valu_counters, ms.value)
        res["roofline_valu"] = {k: v[k] for k in ("achieved", "peak", "unit", "frac", "issue_frac", "wait_frac",
                                                  "valu_active_frac")}
    elif valu_counters:
        res["roofline_valu"] = {"error": valu_counters}
    try:
        res["check"] = checker_leg(prob, cfg.env, xt, mt, None, out, B, check_sample)
    except Exception as e:  # noqa: BLE001
        res["check"] = {"ok": False, "error": f"checker leg failed: {e}"}
    del out, xt, mt
    try:  # the stress box of tests/test_gpu_parity.py (contacts near the surface, large P terms): every
        # instance checked, the plain-1e-10 misses counted
        xs, ms_, _ = generate(cfg.n_contacts, cfg.env, 20000, 99, stress=True)
        xst, mst = torch.tensor(xs, device=dev), torch.tensor(ms_, device=dev)
        so = prob.eval_batch(xst, mst, outputs=("g", "jac"))
        torch.cuda.synchronize()
        res["stress_box"] = checker_leg(prob, cfg.env, xst, mst, None, so, xs.shape[0], xs.shape[0])
        del so, xst, mst
    except Exception as e:  # noqa: BLE001
        res["stress_box"] = {"ok": False, "error": f"stress-box leg failed: {e}"}
    torch.cuda.empty_cache()
    return res


def side_mixed16(dev, stream, check_sample=512):
    """BASELINE.json configs[3] (1,048,576 x 16 contacts, Ground / Superquadric tagged per instance) on
    ONE GPU: the eval kernel's time (median of timed rounds, HIP events), its HBM fraction and a
    per-kind checker sample (both environment kinds) of the outputs."""
    import ctypes

    import torch

    from centroidalplanner_amd import _abi
    from centroidalplanner_amd.workload import CONFIGS, config_inputs

    cfg = CONFIGS["mixed16"]
    prob, x, mass, tag = config_inputs(cfg)
    B = x.shape[0]
    xt, mt, tt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev), torch.tensor(tag, device=dev)
    del x, mass
    out = prob.eval_batch(xt, mt, tt, outputs=("g", "jac", "norms"))
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    ms = ctypes.c_double()
    rounds = []
    for _ in range(3):
        _abi.check(_abi.lib.cpl_time_eval_batch(ctypes.byref(prob.desc()), B, p(xt), p(mt), p(tt), p(out["g"]),
                                                p(out["jac"]), None, None, p(out["norms"]),
                                                ctypes.c_void_p(stream.cuda_stream), 5, ctypes.byref(ms)))
        rounds.append(ms.value)
    kms = sorted(rounds)[1]
    bytes_inst, m = algorithmic_bytes(cfg.n_contacts, cfg.env)
    res = {"workload": cfg.name + " (one GPU)", "kernel_ms": kms, "rows_per_s": B * m / (kms * 1e-3),
           "hbm_gbps": bytes_inst * B / (kms * 1e-3) / 1e9,
           "frac_of_peak": bytes_inst * B / (kms * 1e-3) / 1e9 / HBM_PEAK_GBPS, "bytes_per_instance": bytes_inst}
    # one rank's shard of the 8-GPU strong-scaled run (distributed.shard: the first B / 8 instances),
    # timed through the same split launch on this GPU: t(B) / t(B / 8) predicts the 8-GPU speedup
    # (north_star: >= 6x at 8) — the shard's fixed costs (partition, side-stream fork / join, the norms'
    # finish) grow relative to its work
    Bs = B // 8
    sout = {k: v[:Bs] for k, v in out.items() if k in ("g", "jac")}
    sn = torch.empty_like(out["norms"])
    srounds = []
    for _ in range(5):
        _abi.check(_abi.lib.cpl_time_eval_batch(ctypes.byref(prob.desc()), Bs, p(xt), p(mt), p(tt), p(sout["g"]),
                                                p(sout["jac"]), None, None, p(sn),
                                                ctypes.c_void_p(stream.cuda_stream), 10, ctypes.byref(ms)))
        srounds.append(ms.value)
    sms = sorted(srounds)[2]
    res["shard_of_8"] = {"batch": Bs, "kernel_ms": sms, "rows_per_s": Bs * m / (sms * 1e-3),
                         "frac_of_peak": bytes_inst * Bs / (sms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                         "predicted_strong_speedup_8": kms / sms}
    try:
        res["check"] = checker_leg(prob, cfg.env, xt, mt, tt, out, B, check_sample)
    except Exception as e:  # noqa: BLE001
        res["check"] = {"ok": False, "error": f"checker leg failed: {e}"}
    del out, xt, mt, tt
    torch.cuda.empty_cache()
    return res


def run_solve5(dev, batch, hessian, steps, warm, max_ls, max_soc, cpu_sample, rank=0, world=1, barrier=None,
               ls_kernel=2):
    """BASELINE.json configs[4]: `steps` complete batched solves of `batch` TestBasic ground instances
    (centroidalplanner_amd/batch_ipm.py -> the native engine), after `warm` untimed ones.  Returns
    (dt seconds for the timed solves, the last result, the CPU leg or None)."""
    import torch

    from centroidalplanner_amd.batch_ipm import KernelEvaluator, batch_ipm_solve
    from centroidalplanner_amd.workload import solve_inputs, solve_problem

    prob = solve_problem().GetCplProblem()
    X0, mass = solve_inputs(prob, batch, seed=0xC910 + 5 + 7919 * rank)
    X0t, mt = torch.tensor(X0, device=dev), torch.tensor(mass, device=dev)
    opts = dict(max_iter=300 if hessian == "exact" else 1000, max_ls=max_ls, max_soc=max_soc, hessian=hessian,
                ls_kernel=ls_kernel)
    for _ in range(warm):
        batch_ipm_solve(prob, X0t, mt, **opts)
    torch.cuda.synchronize()
    if barrier:
        barrier()
    ev = KernelEvaluator(prob)
    t0 = time.perf_counter()
    for _ in range(steps):
        r = batch_ipm_solve(prob, X0t, mt, evaluator=ev, **opts)
    torch.cuda.synchronize()
    if barrier:
        barrier()
    dt = time.perf_counter() - t0
    cpu = None
    if rank == 0 and world == 1 and cpu_sample > 0:
        try:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle

            info = host_cpu_info()
            threads = info["threads"]
            # all usable cores (min(affinity, OMP_NUM_THREADS), the eval leg's count): the whole batch
            # split over OpenMP threads, each instance solved by the single-thread restatement (per-thread
            # state) — 8 192 instances are ~1.5 s on 16 threads (~25 core-seconds)
            Bm = batch
            tm, stm, itm = pyoracle.time_solve_mt(prob.desc(), X0[:Bm], mass[:Bm], max_iter=opts["max_iter"],
                                                  hessian=hessian, threads=threads)
            # one core: the first cpu_sample instances one after another
            Bc = min(cpu_sample, batch)
            tc, stc, itc = pyoracle.time_solve(prob.desc(), X0[:Bc], mass[:Bc], max_iter=opts["max_iter"],
                                               hessian=hessian)
            okm, okc = int((stm <= 1).sum()), int((stc <= 1).sum())
            what = (f"the compiled restatement of the same method (oracle/cpl_solve_host.c, gcc -O2: IPOPT's method "
                    f"with dense QR / Cholesky KKT solves, hessian={hessian}; IPOPT itself is not in the image) over "
                    f"the oracle's callbacks; per-instance agreement with the GPU solves in `agreement`")
            # per instance: the GPU engine's outcome against the compiled restatement's on the same start
            # points (the two evaluate in different summation orders; DESIGN.md section 5 says where the
            # trajectories part)
            import numpy as np

            gst, git = r.status.cpu().numpy()[:Bm], r.iterations.cpu().numpy()[:Bm]
            dit = np.abs(git.astype(np.int64) - itm.astype(np.int64))
            agree = {"instances": int(Bm), "status_equal_frac": float((gst == stm).mean()),
                     "iterations_equal_frac": float((git == itm).mean()),
                     "iterations_within_2_frac": float((dit <= 2).mean()),
                     "iterations_absdiff_max": int(dit.max()), "iterations_absdiff_p99": float(np.percentile(dit, 99)),
                     "gpu_iterations_max": int(git.max()), "cpu_iterations_max": int(itm.max()),
                     "gpu_iterations_mean": float(git.mean()), "cpu_iterations_mean": float(itm.mean())}
            cpu = {"value": Bm / tm, "unit": "solves/s", "cores": threads, "kind": "port",
                   "sample": f"the first {Bm} of the {batch} instances over {threads} OpenMP threads (each instance "
                             f"solved on one thread) by {what} ({okm}/{Bm} solved, iterations mean "
                             f"{float(itm.mean()):.1f}, {tm:.2f} s)",
                   "single_core": {"value": Bc / tc, "unit": "solves/s", "cores": 1,
                                   "sample": f"the first {Bc} instances one after another on one core ({okc}/{Bc} "
                                             f"solved, {tc:.2f} s)"},
                   "agreement": agree,
                   **{k: info[k] for k in ("cpu_model", "affinity", "omp_num_threads")}}
        except Exception as e:  # noqa: BLE001
            cpu = {"error": str(e)}
    return dt, r, cpu


def side_solve5(dev, cpu_sample=64):
    """configs[4] in the reference's Hessian mode (IFOPT's limited-memory default) as a side field:
    one timed batched solve of 8,192 instances after one warm-up, and a small CPU sample."""
    from centroidalplanner_amd.workload import SOLVE_CONFIG

    B = SOLVE_CONFIG.batch
    dt, r, cpu = run_solve5(dev, B, "limited-memory", 1, 1, 40, 4, cpu_sample)
    its = r.iterations.double()
    return {"workload": SOLVE_CONFIG.name, "hessian": "limited-memory (IPOPT's L-BFGS, IFOPT's default)",
            "solves_per_s": B / dt, "ms_per_solve_batch": dt * 1e3, "batch": B,
            "solved": int((r.status <= 1).sum().item()), "iterations_max": int(its.max().item()),
            "iterations_mean": float(its.mean().item()), "lockstep_iterations": r.iterations_run,
            "cpu_baseline": cpu}


def side_single_solve(dev, reps=7):
    """The facade's primary call, CentroidalPlanner::Solve() (src/CentroidalPlanner.cpp:22-34): ONE
    instance of the solve workload solved in IFOPT's limited-memory mode by the native engine (B = 1:
    every kernel of an iteration is launch latency), median of `reps` solves after a warm-up, beside the
    compiled restatement of the same iteration over the oracle's callbacks on one CPU core
    (oracle/cpl_solve_host.c)."""
    import statistics

    import torch

    from centroidalplanner_amd.batch_ipm import batch_ipm_solve
    from centroidalplanner_amd.workload import solve_inputs, solve_problem

    prob = solve_problem().GetCplProblem()
    X0, mass = solve_inputs(prob, 1, seed=0xC910 + 5)
    X0t, mt = torch.tensor(X0, device=dev), torch.tensor(mass, device=dev)
    opts = dict(max_iter=1000, hessian="limited-memory")
    r = batch_ipm_solve(prob, X0t, mt, **opts)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = batch_ipm_solve(prob, X0t, mt, **opts)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ms = statistics.median(ts) * 1e3
    res = {"workload": "one instance of the solve workload (4-contact Ground), IFOPT's limited-memory Hessian",
           "gpu_ms_per_solve": ms, "iterations": int(r.iterations[0].item()), "status": int(r.status[0].item()),
           "us_per_iteration": ms * 1e3 / max(1, int(r.iterations_run))}
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle

        tcs = []
        for _ in range(reps):
            tc, stc, itc = pyoracle.time_solve(prob.desc(), X0, mass, max_iter=opts["max_iter"], hessian=opts["hessian"])
            tcs.append(tc)
        res["cpu_baseline"] = {"value": statistics.median(tcs) * 1e3, "unit": "ms per solve", "cores": 1, "kind": "port",
                               "sample": f"the same instance, median of {reps}: the compiled restatement of the same "
                                         f"method (oracle/cpl_solve_host.c, gcc -O2, dense QR / Cholesky KKT; "
                                         f"IPOPT itself is not in the image) over the oracle's callbacks, one core "
                                         f"({int(itc[0])} iterations, status {int(stc[0])})"}
    except Exception as e:  # noqa: BLE001
        res["cpu_baseline"] = {"error": str(e)}
    return res


# ------------------------------------------------------------------------------------------
def solve_bench(args):
    """BASELINE.json configs[4]: the full solve loop, 8,192 concurrent 4-contact Ground instances on
    one GPU (centroidalplanner_amd/batch_ipm.py).  One step = one complete batched solve from the
    starting points to termination of every instance; every callback of every iteration is one
    cpl_eval_batch launch.  cpu_baseline = the compiled restatement of the same iteration
    (oracle/cpl_solve_host.c) over the oracle's callbacks on one core, a bounded sample of the instances."""
    import torch

    from centroidalplanner_amd.workload import SOLVE_CONFIG

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch.distributed as dist

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    B = args.batch or SOLVE_CONFIG.batch
    steps = max(1, min(args.steps, 5))
    warm = 1 if args.warmup > 0 else 0
    dt, r, cpu = run_solve5(dev, B, args.hessian, steps, warm, args.max_ls, args.max_soc,
                            0 if args.no_cpu else args.cpu_sample, rank, world,
                            barrier=dist.barrier if world > 1 else None, ls_kernel=args.ls_kernel)
    if world > 1:
        tdt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tdt, op=dist.ReduceOp.MAX)
        dt = float(tdt.item())
    ok = int((r.status <= 1).sum().item())
    its = r.iterations.double()
    if rank == 0:
        print(json.dumps({
            "metric": "concurrent CentroidalPlanner solves per second (full interior-point solve loop, GPU callbacks)",
            "value": B * world * steps / dt, "unit": "solves/s", "n_gpus": world, "steps": steps, "warmup": warm,
            "ms_per_step": dt / steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (TestBasic ground scenario, per-instance mass U[80,150])",
            "config": {"workload": SOLVE_CONFIG.name, "contacts": 4, "environment": "ground", "batch_per_gpu": B,
                       "parallelism": f"instance-sharded x{world}",
                       "hessian": ("exact (analytic Lagrangian Hessian kernel)" if args.hessian == "exact"
                                   else "limited-memory (IPOPT's L-BFGS: 6 pairs, scalar1 initialisation; IFOPT's IpoptSolver default)"),
                       "max_ls": args.max_ls, "max_soc": args.max_soc},
            "solved": ok, "iterations_max": int(its.max().item()), "iterations_mean": float(its.mean().item()),
            "lockstep_iterations": r.iterations_run, "eval_launches_per_solve": r.evaluations,
            "compactions": r.compactions,
            "graph": r.graph,
            "cpu_baseline": cpu,
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.pmc_child:
        pmc_child(args)
        return 0
    world, rank, local_rank, spawn = resolve_world(args)
    if spawn:  # before anything touches the GPU
        return spawn_ranks(world)
    if args.rehearse_cpu:
        rehearse_cpu(args, world, rank)
        return 0
    if args.config == "solve5":
        solve_bench(args)
        return 0

    from centroidalplanner_amd.workload import CONFIGS

    cfg = CONFIGS[args.config]
    batch = args.batch or cfg.batch
    if cfg.config_id == 4 and not args.batch:
        from centroidalplanner_amd.distributed import shard

        batch = shard(cfg.batch, rank, world)[1]  # config 4 is quoted as 1,048,576 over the node

    # rank 0's legs that run before this process touches the GPU (the other ranks wait for it in the
    # process-group rendezvous): the PMC passes (child processes under rocprofv3, the per-rank batch)
    # and the CPU baseline
    traffic, pmc_info, valu_counters = None, None, None
    if rank == 0 and not args.no_pmc:
        pmc_args = argparse.Namespace(config=args.config, batch=batch if batch != cfg.batch else args.batch)
        traffic, pmc_info = collect_pmc(pmc_args)
        if cfg.env in ("superquadric", "mixed"):  # VALU-bound kernels: the VALU roofline too
            try:
                valu_counters = collect_valu_counters(pmc_args)
            except Exception as e:  # noqa: BLE001
                valu_counters = f"VALU PMC passes failed: {e}"
    sq8_counters = None
    if world == 1 and not args.no_side and args.config == "ground4_1m" and not args.no_pmc:
        try:  # configs[2]'s VALU counters for its side field (PMC passes run before the GPU is touched)
            sq8_counters = collect_valu_counters(argparse.Namespace(config="sq8", batch=0))
        except Exception as e:  # noqa: BLE001
            sq8_counters = f"VALU PMC passes failed: {e}"

    cpu = None
    if rank == 0 and not args.no_cpu:
        try:
            cpu = cpu_baseline(cfg, args.cpu_seconds)
        except Exception as e:  # noqa: BLE001
            cpu = {"error": str(e)}

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist_on = world > 1 or args.collective_always  # (the latter: the RCCL path exercised on one GPU)
    if dist_on:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from centroidalplanner_amd import _abi
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(cfg.n_contacts, cfg.env)
    x, mass, tag = generate(cfg.n_contacts, cfg.env, batch, 0xC910 + cfg.config_id + 7919 * rank)
    xt = torch.tensor(x, device=dev)
    mt = torch.tensor(mass, device=dev)
    tt = None if tag is None else torch.tensor(tag, device=dev)
    del x, mass, tag
    out = prob.eval_batch(xt, mt, tt, outputs=("g", "jac", "norms"))
    stream = torch.cuda.Stream(dev)  # launch stream: graph capture and replay
    K, W = args.steps, args.warmup
    # steps run in buckets of S: one HIP-graph replay launches the S steps' kernels and, with N > 1
    # ranks, one all-gather carries the S steps' per-shard norms (fewer, larger collectives: the
    # per-step host cost is neither a graph launch nor an RCCL enqueue).  Each step still evaluates
    # the whole batch and writes its own norms row.
    S = max(1, min(args.bucket, K))

    import ctypes

    from centroidalplanner_amd.distributed import BucketedNormGather

    def launch(nb, count):
        # `count` steps' device work: per step the fused eval (values + CSR Jacobian values +
        # per-workgroup residual partials) and the one-workgroup finish of the shard's norms, on
        # one stream (a side-stream finish overlapping the next eval measured slower: 33.5 vs
        # 30.0 us per step at 65 536 x 4 — the cross-stream graph edges cost more than the finish)
        for s in range(count):
            out["norms"] = nb[s]
            prob.eval_batch(xt, mt, tt, outputs=("g", "jac", "norms"), out=out, stream=torch.cuda.current_stream(dev))

    # the bucketed step loop with its asynchronous all-gather (distributed.BucketedNormGather: the
    # same code the gloo world-2 tests drive on the CPU)
    runner = BucketedNormGather(world, S, dev, launch, stream=stream, gather_always=dist_on)
    norms = runner.norms
    sizes = sorted(set(runner.sizes(K) + runner.sizes(W)))
    with torch.cuda.stream(stream):  # warm the launch path (per-stream workspaces) before capture
        for nb in norms:
            launch(nb, 1)
    torch.cuda.synchronize()
    graphs = {}
    if not args.no_graph:  # one HIP graph per (norms buffer, bucket size)
        for j, nb in enumerate(norms):
            for c in sizes:
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, stream=stream):
                    launch(nb, c)
                graphs[(j, c)] = gr
        torch.cuda.synchronize()
        runner.replay = {key: gr.replay for key, gr in graphs.items()}
    gather_info = None

    for w in runner.run(W):
        if w is not None:
            w.wait()
    torch.cuda.synchronize()
    runner.reset()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    works = runner.run(K)
    for w in works:
        if w is not None:
            w.wait()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    total_batch = batch
    if dist_on:
        tdt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tdt, op=dist.ReduceOp.MAX)
        dt = float(tdt.item())
        tb = torch.tensor([batch], dtype=torch.int64, device=dev)
        dist.all_reduce(tb, op=dist.ReduceOp.SUM)  # instances of the whole job (shards may differ by 1)
        total_batch = int(tb.item())
        # every timed step's norms reached every rank: the last bucket's gather holds one row per
        # (rank, step); combined over ranks it is the whole job's residual for that step, and this
        # rank's rows must be the norms it computed locally
        gather_info = runner.last_bucket_report(rank, K)

    # live kernel timing: HIP events on the launch stream around back-to-back eval launches only
    ms = ctypes.c_double()
    reps = max(K, 20)

    def p(t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else None

    # the step's launches (eval with fused norms + finish); events bracket each eval kernel alone
    _abi.check(_abi.lib.cpl_time_eval_batch(ctypes.byref(prob.desc()), batch, p(xt), p(mt), p(tt), p(out["g"]), p(out["jac"]),
                                            None, None, p(norms[0][0]), ctypes.c_void_p(stream.cuda_stream), reps,
                                            ctypes.byref(ms)))
    kernel_ms = ms.value

    bytes_inst, m = algorithmic_bytes(cfg.n_contacts, cfg.env)
    alg_bytes = bytes_inst * batch
    rows_total = total_batch * m * K
    value = rows_total / dt
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9

    valu = None
    if isinstance(valu_counters, dict):
        valu = valu_roofline(valu_counters, kernel_ms)
    elif valu_counters:
        valu = {"error": valu_counters}

    check = None
    if rank == 0 and not args.no_check:
        try:
            check = checker_leg(prob, cfg.env, xt, mt, tt, out, batch, args.check_sample)
        except Exception as e:  # noqa: BLE001
            check = {"ok": False, "error": f"checker leg failed: {e}"}

    folded = None
    if rank == 0 and world == 1 and not args.no_side:
        # the values-only Jacobian layout (CPL_EVAL_JAC_FOLDED) of the same batch: the structural
        # constants are not written (same g, the remaining Jacobian values bit-identical)
        fo = prob.eval_batch(xt, mt, tt, outputs=("g", "jac", "norms"), jac_folded=True)
        _abi.check(_abi.lib.cpl_time_eval_batch_ex(ctypes.byref(prob.desc()), batch, p(xt), p(mt), p(tt), p(fo["g"]),
                                                   p(fo["jac"]), None, None, p(fo["norms"]), _abi.EVAL_JAC_FOLDED,
                                                   ctypes.c_void_p(stream.cuda_stream), max(K, 20), ctypes.byref(ms)))
        var_k, _, _ = prob.jac_fold_info()
        same = None
        if not args.no_check:
            same = bool(torch.equal(out["jac"][:, torch.as_tensor(var_k.astype("int64"), device=dev)], fo["jac"])
                        and torch.equal(out["g"], fo["g"]))
        fbytes = 8 * (prob.n + 1 + prob.m + int(var_k.size))
        folded = {
            "kernel_ms": ms.value,
            "bytes_per_instance": fbytes,
            "rows_per_s": batch * m / (ms.value * 1e-3),
            "hbm_gbps": fbytes * batch / (ms.value * 1e-3) / 1e9,
            "frac_of_peak": fbytes * batch / (ms.value * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "speedup_vs_csr": kernel_ms / ms.value,
            "values_equal_csr": same,
        }
        del fo

    single = None
    if rank == 0 and world == 1 and not args.no_side:
        single = single_instance_latency(prob, cfg, dev)

    side = None
    if rank == 0 and world == 1 and not args.no_side and args.config == "ground4_1m":
        # BASELINE.json configs[1] (65,536 x 4 Ground) on the same GPU: kernel time only
        del out
        torch.cuda.empty_cache()
        scfg = CONFIGS["ground4"]
        sb = scfg.batch
        sp = make_problem(scfg.n_contacts, scfg.env)
        x1, m1, _ = generate(scfg.n_contacts, scfg.env, sb, 0xC910 + scfg.config_id)
        x1t, m1t = torch.tensor(x1, device=dev), torch.tensor(m1, device=dev)
        del x1, m1
        o1 = sp.eval_batch(x1t, m1t, outputs=("g", "jac", "norms"))
        _abi.check(_abi.lib.cpl_time_eval_batch(ctypes.byref(sp.desc()), sb, p(x1t), p(m1t), None, p(o1["g"]), p(o1["jac"]),
                                                None, None, p(o1["norms"]), ctypes.c_void_p(stream.cuda_stream), 50,
                                                ctypes.byref(ms)))
        sbytes, sm = algorithmic_bytes(4, "ground")
        side = {
            "workload": scfg.name,
            "kernel_ms": ms.value,
            "rows_per_s": sb * sm / (ms.value * 1e-3),
            "hbm_gbps": sbytes * sb / (ms.value * 1e-3) / 1e9,
            "frac_of_peak": sbytes * sb / (ms.value * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "note": "128 MB working set: fits the 256 MiB Infinity Cache",
        }

    sq8 = solve5 = mixed = None
    if rank == 0 and world == 1 and not args.no_side and args.config == "ground4_1m":
        try:
            sq8 = side_sq8(dev, stream, sq8_counters)
        except Exception as e:  # noqa: BLE001
            sq8 = {"error": str(e)}
        try:
            mixed = side_mixed16(dev, stream)
        except Exception as e:  # noqa: BLE001
            mixed = {"error": str(e)}
        try:
            solve5 = side_solve5(dev, 0 if args.no_cpu else 512)
        except Exception as e:  # noqa: BLE001
            solve5 = {"error": str(e)}
        try:
            solve5["single_solve"] = side_single_solve(dev)
        except Exception as e:  # noqa: BLE001
            solve5["single_solve"] = {"error": str(e)}

    if rank == 0:
        res = {
            "metric": METRIC,
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": dt / K * 1e3,
            "higher_is_better": True,
            "scaling": scaling_of(cfg, args),
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded SURVEY.md §8(d) instances; no published reference number)",
            "config": {
                "workload": cfg.name,
                "contacts": cfg.n_contacts,
                "environment": cfg.env,
                "batch_per_gpu": batch,
                "batch_total": total_batch,
                "outputs": "g + jac (IFOPT CSR values), per-shard residual norms",
                "parallelism": f"instance-sharded x{world}" + (" + RCCL all-gather of residual norms" if world > 1 else ""),
                "launch": (f"hip-graph, {S} steps per replay" if graphs else "eager")
                + (f", one all-gather per {S} steps" if world > 1 else ""),
                "rank_inputs": "distinct per rank (seed 0xC910 + config + 7919 * rank): weak scaling over "
                               "different instances, no data-path exchange",
            },
            "instances_per_s": total_batch * K / dt,
            "residual_gather": gather_info,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "kernel": KERNEL_NAME,
                "kernel_ms": kernel_ms,
                "algorithmic_bytes_per_launch": alg_bytes,
                "bytes_per_instance": bytes_inst,
                "pmc": pmc_info,
            },
            "cpu_baseline": cpu,
        }
        res["check"] = check
        if valu:
            res["roofline_valu"] = valu
        if folded:
            res["jac_folded"] = folded
        if side:
            res["configs1_65k"] = side
        if single:
            res["single_instance"] = single
        if sq8:
            res["configs2_sq8"] = sq8
        if mixed is not None:
            shard = mixed.pop("shard_of_8", None) if isinstance(mixed, dict) else None
            res["configs3_mixed16"] = mixed
            if shard:
                res["configs3_mixed16_shard"] = shard
        if solve5:
            res["configs4_solve5_lbfgs"] = solve5
        print(json.dumps(res), flush=True)

    if dist_on:
        dist.barrier()  # every rank leaves together (rank 0 ran the checker leg after the timing)
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
