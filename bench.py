"""Benchmark: DDP+IFT iterations/s of the batched Dubins+DBaS tube-MPC closed-loop step (T = 50).

One bench "step" = one Algorithm-2 closed-loop step for every trajectory (core/tube_mpc.py:803-1023):
nominal iLQR (10 fixed iterations, 7 line-search alphas) + ancillary iLQR (20 fixed iterations) + one
IFT pass (DDP sensitivity + DOC gradient) + cross-rank gradient all-reduce + theta update + plant step.
metric value = trajectories_all_ranks * (10 + 20 + 1) / seconds_per_step   

Every timed step of the headline `value` is the first closed-loop step of a fresh episode over the same
synthetic batch (reset: x0, b0 = B(h(x0)), zero warm starts, theta0 -- inside the timed region).  The
second field, `steady_state`, times the free-running loop instead: one episode start, then warm-started
steps t >= 1 with the shared theta updated every step.  In f32 a few trajectories' ancillary plans enter
an obstacle from step 1 on (b ~ 1e10, also in f64) and their IFT gradients are ill-conditioned
(|g| ~ 1e15-1e30 against ~1e2 typical); the f32 health policy (TubeMPC grad_bound, 1e6) drops such rows
from the batch mean as it drops flagged trajectories, which keeps theta finite.

Scaling: by default the GLOBAL batch (--batch, 65,536 = BASELINE config 5) is split over the N ranks by
shard_range ("scaling": "strong", 8,192 trajectories per GPU at N = 8); --weak keeps --batch per GPU.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--weak] [--no-cpu]
  N > 1 without a torch.distributed environment: bench.py launches its N ranks itself (a child
  `python -m torch.distributed.run --nproc-per-node N ...` started before any GPU call, one process per
  GPU over RCCL) and exits with the child's status; under torchrun it is one rank.
  --dry-run: the same launch / process group / sharding / timing arithmetic on CPU (gloo), with a
  placeholder step instead of the GPU kernels (tests/test_bench_launch.py).
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import re
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "differentiable-tube-mpc_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from diff_tube_mpc_strict_pt.core import TubeMPC, shard_range  # noqa: E402
from diff_tube_mpc_strict_pt.core.problem import paper_config, paper_setup_from_config  # noqa: E402

# SURVEY.md §8d algorithmic HBM bytes per trajectory per closed-loop step (phase-split tape traffic):
# 10 nominal iterations x 7,652 B + 20 ancillary iterations x 9,676 B + one IFT pass 4,284 B.
ALGO_BYTES_PER_TRAJ_STEP = 10 * 7652 + 20 * 9676 + 4284  # = 274,324
NOMINAL_ITER_BYTES = 7652  # one nominal iLQR iteration of one trajectory, f32; x 2 in f64
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)
VALU_ISSUE_CYCLES = 4.5  # cycles one wave64 VALU instruction costs its wave at one wave per SIMD (profiles/r02/issue_cost.txt)
ITERS_PER_STEP = 10 + 20 + 1


def bench_setup(dtype_name: str):
    cfg = paper_config()
    st = paper_setup_from_config(cfg)
    # benchmark mode: fixed iteration counts (tol = -1, no early exit), SURVEY.md §8d
    import dataclasses

    nom = dataclasses.replace(st.ilqr_nom, tol=-1.0)
    aux = dataclasses.replace(st.ilqr_aux, tol=-1.0)
    return dataclasses.replace(st, ilqr_nom=nom, ilqr_aux=aux)


def initial_states(lo: int, hi: int, device, dtype) -> torch.Tensor:
    """x0 per GLOBAL trajectory index: px, py ~ U[0,1], theta ~ U[0, pi/2]; generated
    in global order so every sharding sees the same inputs."""
    g = torch.Generator().manual_seed(0)
    n = hi
    u = torch.rand(n, 3, generator=g, dtype=torch.float64)[lo:hi]
    x0 = torch.stack([u[:, 0], u[:, 1], u[:, 2] * (np.pi / 2)], 1)
    return x0.to(device=device, dtype=dtype)


def lib_sha256() -> str:
    """sha256 of the libdtmpc.so this process loads (a PMC summary is only valid for the same library)."""
    import hashlib

    from diff_tube_mpc_strict_pt import _lib

    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_summary(batch: int, kernel: str = "tube"):
    """The newest committed rocprofv3 --pmc summary (profiles/rNN/pmc_*.json, scripts/pmc_summary.py) of this
    workload and batch for the SAME library build (sha256), or (None, reason)."""
    def newest_first(path):  # profiles/rNN/pmc_vMM.json: the highest round, then the highest version
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.relpath(path, REPO))]

    want = lib_sha256()
    best, why = None, "no PMC summary for this batch"
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", "**", "*pmc*.json"), recursive=True), key=newest_first):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if int(d.get("batch", -1)) != batch or d.get("workload", "tube") != kernel:
            continue
        if d.get("lib_sha256") != want:
            best, why = None, f"newest PMC summary for this batch ({os.path.relpath(p, REPO)}) is of another library build"
            continue
        best, why = d, os.path.relpath(p, REPO)
    return best, why


def issue_of(summary) -> dict | None:
    """The instruction-issue roofline of the kernel from its PMC summary: VALU instructions per wave x 4.5 cycles
    (what one wave64 VALU instruction costs its wave at one wave per SIMD, scripts/ubench/issue_cost.hip) over the
    kernel's shader cycles (GRBM_GUI_ACTIVE / 8 XCDs, MI355X_MICROARCH.md: effective clock), and the SQ's own VALU
    busy share of the wave cycles."""
    if not summary:
        return None
    c = summary.get("counters_per_dispatch", {})
    if not all(k in c for k in ("SQ_INSTS_VALU", "SQ_WAVES", "GRBM_GUI_ACTIVE")):
        return None
    per_wave = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
    cycles = c["GRBM_GUI_ACTIVE"] / 8.0
    out = {"valu_instr_per_wave": per_wave, "kernel_cycles": cycles,
           "valu_issue_frac": per_wave * VALU_ISSUE_CYCLES / cycles,
           "salu_instr_per_wave": c.get("SQ_INSTS_SALU", 0.0) / c["SQ_WAVES"]}
    if "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c:
        out["valu_active_frac"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
    ks = summary.get("kernel_trace") or {}
    if ks.get("avg_ns"):
        out["clock_ghz"] = cycles / ks["avg_ns"]
    return out


def pmc_traffic(batch: int, kernel: str = "tube"):
    """Per-launch HBM bytes of the dominant kernel from a committed rocprofv3 --pmc summary
    (profiles/rNN/pmc_*.json, written by scripts/pmc_summary.py) for the SAME library build (sha256) and
    batch, or (None, reason).  FETCH_SIZE / WRITE_SIZE are calibrated there on a known-byte launch
    (MI355X_MICROARCH.md §HBM: gfx950 under-reports wide coalesced reads)."""
    d, why = pmc_summary(batch, kernel)
    if d is None:
        return None, why
    b = d.get("kernel_bytes_per_launch", d.get("tube_step_bytes_per_launch"))
    return (float(b), why) if b is not None else (None, why + " has no HBM counters")


def cpu_baseline(setup, seconds_target: float = 15.0):
    """The C oracle (oracle/liboracle.so, a restatement of the reference) timed on host cores."""
    from diff_tube_mpc_strict_pt import _abi
    from oracle.oracle import Oracle, build

    build()
    threads = int(os.environ.get("DTMPC_CPU_THREADS", min(16, os.cpu_count() or 1)))
    o = Oracle(np.float32, nthreads=threads)
    N = setup.problem.horizon
    sp = setup.problem.to_c()
    tcfg = _abi.DtmpcTubeCfg()
    tcfg.nominal = setup.nominal_cost.to_c()
    tcfg.nom_ilqr = setup.ilqr_nom.to_c()
    tcfg.aux_ilqr = setup.ilqr_aux.to_c()
    tcfg.disturbance = 1
    for f in range(3):
        tcfg.w_low[f], tcfg.w_high[f] = setup.w_low[f], setup.w_high[f]

    def run(B):
        x0 = initial_states(0, B, "cpu", torch.float32).numpy().T.copy()
        h, _, _ = o.h_eval(sp, x0[0], x0[1])
        b0 = o.barrier(sp, h)[0]
        state = {"x": x0, "b": b0.copy(), "xbar": x0.copy(), "bbar": b0.copy(),
                 "Xnom": np.zeros((N + 1, 4, B), np.float32), "Unom": np.zeros((N, 2, B), np.float32),
                 "Xaux": np.zeros((N + 1, 4, B), np.float32), "Uaux": np.zeros((N, 2, B), np.float32)}
        t0 = time.perf_counter()
        o.tube_step(sp, tcfg, state, np.array(setup.theta0, np.float32), step=0, want_log=False)
        return time.perf_counter() - t0

    B = 4 * threads
    dt = run(B)
    B = int(min(262144, max(B, B * seconds_target / max(dt, 1e-3))))
    B -= B % threads
    dt = run(B)
    return {"value": B * ITERS_PER_STEP / dt, "unit": "DDP+IFT iters/s", "cores": threads, "kind": "port",
            "sample": f"C oracle (oracle/dtmpc_oracle.c) f32, one closed-loop step of {B} trajectories "
                      f"(10+20 fixed iLQR iterations, 7 alphas, + IFT), OpenMP {threads} threads, {dt:.1f} s"}


def nominal_ddp_leg(dev, dtype_name: str, B: int = 4096, steps: int = 20, warmup: int = 3, generic: bool = False):
    """BASELINE config 2: batched nominal DDP (Dubins n = 3, m = 2 + barrier state, T = 50) over B
    trajectories on one GPU -- dtmpc_ilqr_solve_ws (core.ddp.ilqr_solve's entry: the fused solver at the
    default lane count, f32 and f64) with the nominal target cost, 10 fixed iterations
    (tol = -1), 7 line-search alphas, zero warm start; generic=True times dtmpc_ilqr_solve (the generic
    kernel) instead.  One step = one solve of the whole batch from the same x0 / V_init (the control tape
    is re-seeded inside the timed region: it is the in/out buffer)."""
    import ctypes as C
    import dataclasses

    from diff_tube_mpc_strict_pt import _lib
    from diff_tube_mpc_strict_pt.core.ddp import _prep_x0, dbas_init

    dt = torch.float32 if dtype_name == "f32" else torch.float64
    st = bench_setup(dtype_name)
    cfg = dataclasses.replace(st.ilqr_nom, tol=-1.0)
    N = st.problem.horizon
    lib = _lib.load()
    spec, cc, ic = st.problem.to_c(), st.nominal_cost.to_c(), cfg.to_c()
    x3 = initial_states(0, B, dev, dt)
    x0 = _prep_x0(torch.cat([x3, dbas_init(st.problem, x3)[:, None]], 1))  # b0 = B(h(x0))
    kw = dict(dtype=dt, device=dev)
    U0 = torch.zeros(N, 2, B, **kw)
    Us, Xs = torch.empty_like(U0), torch.empty(N + 1, 4, B, **kw)
    Ks, ks = torch.empty(N, 8, B, **kw), torch.empty(N, 2, B, **kw)
    iters = torch.zeros(B, dtype=torch.int32, device=dev)
    status = torch.zeros(B, dtype=torch.int32, device=dev)
    code = 0 if dt == torch.float32 else 1
    lanes = int(lib.dtmpc_tube_lanes_dtype(B, code))
    wb = int(lib.dtmpc_ilqr_workspace_bytes(code, N, B, lanes))
    work = torch.empty(max(wb, 1), dtype=torch.uint8, device=dev)
    fused = bool(lib.dtmpc_ilqr_fused_eligible(code, C.byref(spec), C.byref(cc), C.byref(ic)))  # the path that runs

    def solve(e0=None, e1=None):
        Us.copy_(U0)
        if e0 is not None:
            e0.record()
        if generic:
            _lib.check(lib.dtmpc_ilqr_solve(code, C.byref(spec), C.byref(cc), C.byref(ic), B, x0.data_ptr(), None,
                                            None, Xs.data_ptr(), Us.data_ptr(), Ks.data_ptr(), ks.data_ptr(),
                                            iters.data_ptr(), status.data_ptr(), None, _lib.stream_of(x0)),
                       "dtmpc_ilqr_solve")
        else:
            _lib.check(lib.dtmpc_ilqr_solve_ws(code, C.byref(spec), C.byref(cc), C.byref(ic), B, x0.data_ptr(), None,
                                               None, Xs.data_ptr(), Us.data_ptr(), Ks.data_ptr(), ks.data_ptr(),
                                               iters.data_ptr(), status.data_ptr(), None, None, lanes, work.data_ptr(), wb,
                                               _lib.stream_of(x0)), "dtmpc_ilqr_solve_ws")
        if e1 is not None:
            e1.record()

    for _ in range(warmup):
        solve()
    torch.cuda.synchronize(dev)
    # HIP events on the launch stream around the solve alone (the warm-start re-seed copy is outside them)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for e0, e1 in ev:
        solve(e0, e1)
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t0) / steps
    kern = [a.elapsed_time(b) for a, b in ev]
    out = {"workload": f"BASELINE config 2: batched nominal DDP, {cfg.max_iter} fixed iterations (tol=-1), "
                       f"{len(cfg.line_search_alphas)} alphas, T={N}, zero warm start",
           "batch": B, "dtype": dtype_name, "ms_per_step": 1e3 * wall,
           "kernel": ("generic ilqr_kernel" if generic or not fused else f"fused ilqr_fast_kernel, {lanes} lanes"),
           "event_ms_median": float(np.median(kern)), "kernel_ms": float(np.mean(kern)),
           "value": B * cfg.max_iter / wall, "unit": "DDP iters/s",
           "nonzero_status": int((status != 0).sum())}
    if not generic and fused:
        # 7,652 algorithmic bytes per nominal iteration and trajectory (f32; f64 twice)
        algo = NOMINAL_ITER_BYTES * cfg.max_iter * B * (2 if dtype_name == "f64" else 1)
        wl = f"nominal_ddp_{dtype_name}"
        traffic, src = pmc_traffic(B, kernel=wl)
        out["roofline"] = roofline_of(algo, out["kernel_ms"], traffic, src, workload=wl, batch=B)
    return out


def warm_up(step, warmup: int, dev, min_launches: int = 8, max_launches: int = 40, rel: float = 0.01) -> int:
    """Untimed warm-up past the clock ramp (the first launches of a fresh box ramp from
    ~4.3 to ~4.05 ms): at least max(warmup, min_launches) steps, then more until two consecutive steps'
    HIP-event times agree within `rel`, at most max_launches.  Returns the number run."""
    n, last = 0, None
    while True:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        step()
        e1.record()
        torch.cuda.synchronize(dev)
        n += 1
        t = e0.elapsed_time(e1)
        if n >= max(warmup, min_launches) and last is not None and abs(t - last) <= rel * last:
            return n
        if n >= max_launches:
            return n
        last = t


def roofline_of(algo_bytes: float, kernel_ms: float, traffic=None, traffic_src=None, workload=None,
                batch=None) -> dict:
    """HBM roofline of one kernel: algorithmic bytes per launch over its mean HIP-event time, the calibrated
    PMC bytes beside them, and (from the same PMC summary) the instruction-issue roofline (issue_of)."""
    achieved = algo_bytes / (kernel_ms * 1e-3) / 1e9
    out = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
           "algo_bytes_per_launch": algo_bytes}
    if workload is not None:
        summ, _ = pmc_summary(batch, workload)
        out["issue"] = issue_of(summ)
        if out["issue"] is not None:
            out["issue"]["source"] = traffic_src
    return out


def tube_leg(dev, dtype_name: str, B: int, steps: int, warmup: int, adapt: bool = True, workload: str = ""):
    """The tube step (episode start) on one GPU, B trajectories, in f32 or f64: the headline's other
    precision, and BASELINE configs 3 (adapt=False: nominal + ancillary tube MPC, theta held) and 4 (the
    same step with the IFT adaptation update of Algorithm 2) at B = 4,096.  roofline: SURVEY §8d's 274,324
    algorithmic bytes per trajectory in f32 (x 2 in f64) over the fused kernel's HIP-event time."""
    dt = torch.float32 if dtype_name == "f32" else torch.float64
    setup = bench_setup(dtype_name)
    mpc = TubeMPC(setup, batch=B, device=dev, dtype=dt, disturbance="philox", seed=0, global_offset=0,
                  global_batch=B, process_group=None)
    x0 = initial_states(0, B, dev, dt)

    def one(k=None):
        mpc.reset(x0)
        mpc.step(kernel_events=k, adapt=adapt)

    nwarm = warm_up(one, warmup, dev)
    kev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for k in kev:
        one(k)
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t0) / steps
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in kev]))
    algo = ALGO_BYTES_PER_TRAJ_STEP * B * (2 if dtype_name == "f64" else 1)
    wl = "tube" if dtype_name == "f32" else "tube_f64"
    traffic, src = pmc_traffic(B, kernel=wl)
    out = {"batch": B, "dtype": dtype_name, "ms_per_step": 1e3 * wall, "warmup_run": nwarm,
           "kernel_ms": kern_ms, "adapt": adapt,
           "value": B * ITERS_PER_STEP / wall, "unit": "DDP+IFT iters/s",
           "roofline": roofline_of(algo, kern_ms, traffic, src, workload=wl, batch=B),
           "flagged_trajectories": int((mpc.status != 0).sum()), "lanes": mpc.lanes,
           # the fused kernel in this precision (f64: csrc/dtmpc_fast64.hip) unless switched off for A/B
           "kernel": ("generic tube_step_kernel"
                      if os.environ.get("DTMPC_FAST") == "0" or (dtype_name == "f64" and os.environ.get("DTMPC_FAST64") == "0")
                      else "fused tube_fast_kernel")}
    if workload:
        out["workload"] = workload
    del mpc
    torch.cuda.empty_cache()
    return out


def receding_leg(dev, dtype_name: str, B: int = 65536, H: int = 20, reps: int = 3):
    """The receding-horizon nominal MPC (run_nominal.py:204-415, BASELINE config 1's workload) batched over B
    starts x0 ~ U[0,1]^2 x U[0, pi/2] (paper configuration, tol = 1e-3, early exits): one dtmpc_nominal_receding
    launch runs every run's whole loop (the fused solver, csrc/dtmpc_fast.hip receding_fast_kernel).  Time per
    receding step = launch time / H; iLQR solves/s = the steps the runs actually took / launch time."""
    from diff_tube_mpc_strict_pt.core.problem import paper_config
    from diff_tube_mpc_strict_pt.core.receding import nominal_receding, receding_setup_from_config

    tdt = torch.float32 if dtype_name == "f32" else torch.float64
    problem, cost, icfg = receding_setup_from_config(paper_config())
    g = torch.Generator().manual_seed(0)
    u = torch.rand(B, 3, generator=g, dtype=torch.float64)
    x0 = torch.stack([u[:, 0], u[:, 1], u[:, 2] * (math.pi / 2)], 1).to(tdt).to(dev)
    nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=x0[:1024], H=2, check=False)
    ms, r = [], None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record()
        r = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=x0, H=H, check=False)
        e1.record()
        torch.cuda.synchronize(dev)
        ms.append(e0.elapsed_time(e1))
    t = float(np.median(ms))
    solves = int(r.h_ran.sum())
    iters = int(r.iters.sum())
    # algorithmic bytes: SURVEY.md §8d's 7,652 B per nominal iLQR iteration (f32; f64 twice) times the iterations
    # the runs actually took (each run's own tol exits and run exits: dtmpc_nominal_receding_it)
    algo = NOMINAL_ITER_BYTES * iters * (2 if dtype_name == "f64" else 1)
    wl = f"receding_{dtype_name}"
    traffic, src = pmc_traffic(B, kernel=wl)
    return {"workload": "receding-horizon nominal MPC (run_nominal.py), B runs x H steps, tol=1e-3, 7 alphas",
            "batch": B, "H": H, "dtype": dtype_name, "ms_per_receding_step": t / H, "launch_ms": t,
            "ilqr_solves_per_s": solves / (t * 1e-3), "solves": solves, "ilqr_iterations": iters,
            "failed": int((r.status != 0).sum()),
            "success": int((r.success_t >= 0).sum()), "collided": int(r.collided.sum()),
            "roofline": roofline_of(algo, t, traffic, src, workload=wl, batch=B)}


def _free_port() -> int:
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """Start the N ranks as ONE child process tree (torch.distributed.run, one process per GPU) and
    return its exit status.  Called before this process touches the GPU (no exec: a child, not a
    replacement)."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL over dmabuf IPC on this host driver
    return subprocess.run(cmd, env=env).returncode


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536,
                    help="GLOBAL trajectories split over the ranks (strong scaling); per GPU with --weak")
    ap.add_argument("--weak", action="store_true", help="--batch trajectories per GPU (weak scaling)")
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU-baseline leg")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo rehearsal of launch, sharding and timing with a placeholder step (no GPU)")
    ap.add_argument("--no-steady", action="store_true", help="skip the free-running (warm-started) loop field")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N > 1: all-reduce theta in line instead of beside the next step's nominal solve (TubeMPC overlap)")
    ap.add_argument("--no-weak-leg", action="store_true",
                    help="N > 1: skip the weak-scaling leg (65,536 trajectories per GPU) beside the strong-scaling line")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the secondary legs (f64 tube step, config-2 nominal DDP at B = 4096)")
    ap.add_argument("--workload", default="tube", choices=["tube", "nominal-ddp", "receding"],
                    help="nominal-ddp: print only the BASELINE config-2 line (one GPU); receding: only the receding "
                         "driver's leg (one GPU; profiling runs)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if env_world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={env_world}")
    if args.dry_run:
        dev = torch.device("cpu")
        if env_world > 1:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if env_world > 1:
            dist.init_process_group("nccl", device_id=dev)  # RCCL
    world = dist.get_world_size() if dist.is_initialized() else 1
    if dist.is_initialized():
        rank = dist.get_rank()
    if args.workload == "nominal-ddp":
        if world != 1 or args.dry_run:
            raise SystemExit("--workload nominal-ddp is a one-GPU leg")
        leg = nominal_ddp_leg(dev, args.dtype, B=args.batch if args.batch != 65536 else 4096, steps=args.steps,
                              warmup=args.warmup)
        print(json.dumps({"metric": "batched nominal DDP iters/sec, Dubins+DBaS T=50", "value": leg["value"],
                          "unit": leg["unit"], "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": leg["ms_per_step"], "higher_is_better": True, "scaling": "strong",
                          "vs_baseline": None, "dtype": args.dtype, "data": "synthetic x0 (bench.initial_states)",
                          "config": {"workload": leg["workload"], "global_batch": leg["batch"]}, "leg": leg}))
        return
    if args.workload == "receding":
        if world != 1 or args.dry_run:
            raise SystemExit("--workload receding is a one-GPU leg")
        leg = receding_leg(dev, args.dtype, B=args.batch)
        print(json.dumps({"metric": "receding-horizon iLQR solves/sec, Dubins+DBaS T=50", "value": leg["ilqr_solves_per_s"],
                          "unit": "iLQR solves/s", "n_gpus": 1, "ms_per_step": leg["ms_per_receding_step"],
                          "higher_is_better": True, "dtype": args.dtype, "leg": leg}))
        return
    dtype = torch.float32 if args.dtype == "f32" else torch.float64
    setup = bench_setup(args.dtype)
    Bg = args.batch * world if args.weak else args.batch
    if Bg < world:
        raise SystemExit(f"global batch {Bg} < {world} ranks")
    lo, hi = shard_range(Bg, rank, world)

    if args.dry_run:
        mpc = None

        def step(kernel_events=None):
            time.sleep(0.002)
    else:
        mpc = TubeMPC(setup, batch=hi - lo, device=dev, dtype=dtype, disturbance="philox", seed=0,
                      global_offset=lo, global_batch=Bg, process_group=None,
                      overlap=False if args.no_overlap else None)
        x0 = initial_states(lo, hi, dev, dtype)

        def step(kernel_events=None):
            mpc.reset(x0)
            mpc.step(kernel_events=kernel_events)

    def sync():
        if not args.dry_run:
            torch.cuda.synchronize(dev)

    def barrier():
        sync()
        if world > 1:
            dist.barrier()
            sync()

    if args.dry_run:
        for _ in range(args.warmup):
            step()
        nwarm = args.warmup
    else:
        nwarm = warm_up(step, args.warmup, dev)
    # every rank warms up at least as long as the slowest (the same count keeps the ranks in step)
    if world > 1:
        wt = torch.tensor([nwarm], dtype=torch.int64, device=dev)
        dist.all_reduce(wt, op=dist.ReduceOp.MAX)
        for _ in range(int(wt) - nwarm):
            step()
        nwarm = int(wt)
    barrier()
    if args.dry_run:
        ev = kev = None
    else:
        # HIP events on the launch stream: whole step, and the fused tube_step kernel alone -- in overlap mode around
        # each of its two launches (phase 1: nominal, phase 2: the rest), so the kernel time excludes the launch
        # stream's wait for the previous step's theta update (end of phase 1 -> start of phase 2), reported beside it
        nkev = 4 if mpc.overlap else 2
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        kev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(nkev)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s in range(args.steps):
        if ev is not None:
            ev[s][0].record()
            step(kernel_events=kev[s])
            ev[s][1].record()
        else:
            step()
    barrier()
    wall = time.perf_counter() - t0
    wait_ms = 0.0
    if ev is not None:
        step_ms = [e0.elapsed_time(e1) for e0, e1 in ev]
        if mpc.overlap:
            kern_ms = float(np.mean([k[0].elapsed_time(k[1]) + k[2].elapsed_time(k[3]) for k in kev]))
            wait_ms = float(np.mean([k[1].elapsed_time(k[2]) for k in kev]))
        else:
            kern_ms = float(np.mean([k[0].elapsed_time(k[1]) for k in kev]))
        # f32 can overflow on trajectories driven deep into an obstacle's relaxed barrier, exactly where
        # the reference raises FloatingPointError in f32; such trajectories are flagged and counted
        flagged_local = int((mpc.status != 0).sum())
    else:
        step_ms, kern_ms, flagged_local = [1e3 * wall / max(args.steps, 1)], 1e3 * wall / max(args.steps, 1), 0
    red = torch.tensor([wall, kern_ms], dtype=torch.float64, device=dev)
    cnt = torch.tensor([flagged_local], dtype=torch.int64, device=dev)
    # every rank's own figures (the first multi-GPU run must explain itself): its shard, kernel time,
    # the launch stream's wait for the theta update, the whole-step wall time and whether the overlap path ran
    mine = torch.tensor([rank, hi - lo, kern_ms, wait_ms, 1e3 * wall / max(args.steps, 1),
                         float(bool(mpc is not None and mpc.overlap)), float(mpc.lanes if mpc is not None else 0)],
                        dtype=torch.float64, device=dev)
    gathered = [torch.zeros_like(mine) for _ in range(world)]
    if world > 1:
        dist.all_reduce(red, op=dist.ReduceOp.MAX)  # the slowest rank sets the step time
        dist.all_reduce(cnt)
        dist.all_gather(gathered, mine)
    else:
        gathered = [mine]
    wall, kern_ms_max = float(red[0]), float(red[1])
    per_rank = [{"rank": int(g[0]), "batch": int(g[1]), "kernel_ms": float(g[2]), "theta_wait_ms": float(g[3]),
                 "wall_ms_per_step": float(g[4]), "overlap": bool(g[5]), "lanes": int(g[6])}
                for g in (t.cpu() for t in gathered)]

    # second field: the free-running Algorithm-2 loop -- one episode start, then warm-started steps t >= 1
    # (shifted warm starts, advanced plant, theta updated by the batch-mean gradient under the f32 health
    # policy of TubeMPC.grad_bound), K steps timed after W untimed ones
    steady = None
    if not args.dry_run and not args.no_steady:
        mpc.reset(x0)
        for _ in range(max(args.warmup, 1)):
            mpc.step()
        barrier()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            mpc.step()
        barrier()
        sw = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(sw, op=dist.ReduceOp.MAX)
        sw = float(sw)
        th = mpc.theta.double().cpu()
        steady = {"ms_per_step": 1e3 * sw / args.steps, "value": Bg * ITERS_PER_STEP / (sw / args.steps),
                  "steps": [max(args.warmup, 1), max(args.warmup, 1) + args.steps],
                  "theta": [float(v) for v in th], "theta_finite": bool(torch.isfinite(th).all()),
                  "healthy_fraction_last_step": mpc.healthy_count / Bg,
                  "grad_bound": float(mpc.cfg.grad_bound)}

    # N > 1, strong scaling (the default): the same step with BASELINE config 5's 65,536 trajectories PER GPU beside the
    # strong-scaling line (the per-GPU shard of the fixed global batch shrinks to 8,192 at N = 8, into the small-batch
    # regime) -- value = N x 65,536 x 31 / the slowest rank's step time
    weak = None
    if world > 1 and not args.weak and not args.no_weak_leg:
        Bw = 65536
        lo_w, hi_w = shard_range(Bw * world, rank, world)
        if args.dry_run:
            def wstep():
                time.sleep(0.002)
            ov = False
        else:
            del mpc
            torch.cuda.empty_cache()
            mpc = TubeMPC(setup, batch=hi_w - lo_w, device=dev, dtype=dtype, disturbance="philox", seed=0,
                          global_offset=lo_w, global_batch=Bw * world, process_group=None,
                          overlap=False if args.no_overlap else None)
            xw = initial_states(lo_w, hi_w, dev, dtype)
            ov = mpc.overlap

            def wstep():
                mpc.reset(xw)
                mpc.step()
        for _ in range(max(nwarm // 2, args.warmup)):
            wstep()
        barrier()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            wstep()
        barrier()
        tw = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
        dist.all_reduce(tw, op=dist.ReduceOp.MAX)
        tw = float(tw) / args.steps
        weak = {"scaling": "weak", "batch_per_gpu": hi_w - lo_w, "global_batch": Bw * world, "ms_per_step": 1e3 * tw,
                "value": Bw * world * ITERS_PER_STEP / tw, "overlap": ov}

    ms_per_step = 1e3 * wall / args.steps
    value = Bg * ITERS_PER_STEP / (wall / args.steps)
    algo_bytes = ALGO_BYTES_PER_TRAJ_STEP * (hi - lo) * (2 if args.dtype == "f64" else 1)
    traffic, traffic_src = ((None, "dry run") if args.dry_run
                            else pmc_traffic(hi - lo, kernel="tube" if args.dtype == "f32" else "tube_f64"))
    out = {
        "metric": "DDP+IFT iters/sec, batched Dubins+DBaS T=50",
        "value": value,
        "unit": "DDP+IFT iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic: x0 ~ U[0,1]^2 x U[0,pi/2] per global index, Philox disturbances, configs/dubins.yaml values",
        "config": {
            "workload": "Algorithm-2 tube step (episode start): nominal iLQR 10 it + ancillary iLQR 20 it "
                        "(7 alphas, tol=-1) + IFT + theta all-reduce/update + plant",
            "global_batch": Bg, "batch_per_gpu": hi - lo, "horizon": setup.problem.horizon, "obstacles": 5,
            "line_search_alphas": len(setup.ilqr_nom.line_search_alphas), "parallelism": f"dp{world}",
        },
        # N > 1: the step as two launches with the theta all-reduce + update on a side stream beside the next
        # step's nominal solve (TubeMPC overlap); one process has no collective
        "overlap": bool(mpc.overlap) if mpc is not None else False,
        "kernel_ms": kern_ms,
        "kernel_ms_max_over_ranks": kern_ms_max,
        # per rank: shard, fused-kernel time (overlap: the two launches' sum), the launch stream's wait for the
        # previous step's theta all-reduce + update (0 without overlap), wall time per step, overlap path, lanes.
        # RCCL unmeasured until the driver's multi-GPU run (one-GPU boxes only in this build's budget).
        "ranks": per_rank,
        "comm": {"backend": (dist.get_backend() if dist.is_initialized() else None),
                 "collective": "all_reduce(SUM) of 8 floats per step" if world > 1 else None,
                 "overlap": bool(mpc.overlap) if mpc is not None else False,
                 "theta_wait_ms_max_over_ranks": max(r["theta_wait_ms"] for r in per_rank)},
        "flagged_trajectories": int(cnt[0]),
        "event_ms_per_step_median": float(np.median(step_ms)),
        "warmup_run": nwarm,
        "roofline": roofline_of(algo_bytes, kern_ms, traffic, traffic_src,
                                workload=None if args.dry_run else ("tube" if args.dtype == "f32" else "tube_f64"),
                                batch=hi - lo),
    }
    out["steady_state"] = steady
    out["weak_scaling"] = weak
    if world == 1 and not args.dry_run and not args.no_extra:
        # secondary legs: the reference's configured precision (configs/dubins.yaml:8,
        # f64) on the same tube step, and BASELINE config 2 (batched nominal DDP, B = 4,096) in f32 / f64
        other = "f64" if args.dtype == "f32" else "f32"
        del mpc
        torch.cuda.empty_cache()
        out[f"tube_{other}"] = tube_leg(dev, other, Bg, steps=min(args.steps, 5), warmup=1)
        # BASELINE configs 3 and 4 (one GPU, B = 4,096, f32): the tube MPC with theta held, and the same step
        # with the IFT adaptation update
        out["config3_tube_b4096"] = tube_leg(dev, "f32", 4096, steps=args.steps, warmup=args.warmup, adapt=False,
                                             workload="BASELINE config 3: tube MPC (nominal 10 + ancillary 20 "
                                                      "fixed iterations, DBaS), theta held, B=4096, episode start")
        out["config4_adapt_b4096"] = tube_leg(dev, "f32", 4096, steps=args.steps, warmup=args.warmup, adapt=True,
                                              workload="BASELINE config 4: the config-3 step + IFT sensitivity, "
                                                       "DOC gradient and theta update (Algorithm 2), B=4096")
        out["nominal_ddp"] = {d: nominal_ddp_leg(dev, d, B=4096, steps=args.steps, warmup=args.warmup)
                              for d in ("f32", "f64")}
        out["nominal_ddp"]["f32_generic"] = nominal_ddp_leg(dev, "f32", B=4096, steps=args.steps,
                                                            warmup=args.warmup, generic=True)
        out["receding"] = {d: receding_leg(dev, d) for d in ("f32", "f64")}
    if args.dry_run:
        out["dry_run"] = True
    if rank == 0 and not args.no_cpu and world == 1 and not args.dry_run:
        out["cpu_baseline"] = cpu_baseline(setup)
    else:
        out["cpu_baseline"] = None
    # the reference's own PyTorch CPU path, measured in the build container (it cannot travel to the GPU
    # box): SURVEY.md §6 / BASELINE.md, 8 processes x 1 thread, fixed-iteration tube steps
    out["reference_cpu_container"] = {"f32": 18.3, "f64": 23.6, "unit": "DDP+IFT iters/s", "cores": 8,
                                      "where": "build container (8 Xeon cores), not this box: the reference "
                                               "itself (PyTorch, 8 processes x 1 thread)",
                                      "source": "SURVEY.md §6, BASELINE.md"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
