"""Batched differentiable tube MPC on MI355X (HIP), Algorithm 2 of the paper.

* :class:`TubeMPC` — NEW batched entry (the reference has no such class): B independent
  closed loops share the adaptive ancillary weights theta = (Qa, Ra, qba).  One call of
  :meth:`TubeMPC.step` = one closed-loop step for every trajectory (core/tube_mpc.py:803-1023):
  nominal iLQR -> ancillary iLQR -> upper loss -> DDP sensitivity -> DOC gradient -> plant step ->
  warm-start shift, all inside one fused HIP kernel; then a fixed-order reduction of the
  per-workgroup gradient sums, a cross-rank all-reduce (RCCL) when the batch is sharded, and the
  momentum/projection update of theta (core/tube_mpc.py:978-984) with the batch-mean gradient.
  With B = 1 this is exactly the reference's loop body.
* :class:`GeneralTubeMPC` — the same batched loop for the GENERAL path (core/tube_mpc.py:40-663):
  softplus / tanh parameterised weights and DBaS parameters, both MPCs adapting by the IFT gradient
  (the nominal one through the ancillary's reference-trajectory gradient).  One fused kernel for the
  solves + sensitivities + IFT, a 24-float reduction / all-reduce, the clipped / momentum / projected
  update, then the plant step with the updated parameters.
* :func:`run_closed_loop_experiment` — signature- and output-compatible with the reference
  (core/tube_mpc.py:40): the paper mode (core/tube_mpc.py:666-1048) or the general path.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch
from torch import Tensor

from .. import _abi, _lib
from .ddp import _dtype_code, raise_for_status
from .problem import GeneralSetup, PaperSetup, general_setup_from_config, paper_setup_from_config, softplus

__all__ = ["ExperimentTrajectories", "TubeMPC", "GeneralTubeMPC", "run_closed_loop_experiment", "shard_range",
           "allreduce_sums", "DEFAULT_GRAD_BOUND_F32"]

# f32 health bound on a trajectory's DOC gradient components (TubeMPC grad_bound, dtmpc_tube_cfg.grad_bound)
DEFAULT_GRAD_BOUND_F32 = 1e6


@dataclass
class ExperimentTrajectories:
    """core/tube_mpc.py:27-37"""

    x_real: list
    u_real: list
    x_bar: list
    u_bar: list
    loss: list
    b_real: list
    Qa_history: list
    Ra_history: list
    qba_history: list


def shard_range(global_batch: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous global-index slice [lo, hi) of trajectories owned by `rank`."""
    if world_size < 1 or not (0 <= rank < world_size):
        raise ValueError("bad rank / world_size")
    base, rem = divmod(global_batch, world_size)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def allreduce_sums(sums: Tensor, group=None) -> Tensor:
    """Sum the [L, gQ(3), gR(2), gqb, count] vector (or the general path's 25) over ranks (RCCL on HIP
    devices, gloo on CPU)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if sums.is_cuda and dist.get_backend(group) == "gloo":
            # gloo (ranks sharing one device, where RCCL refuses): through host memory
            host = sums.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            sums.copy_(host)
        else:
            dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
    return sums


class TubeMPC:
    """Device-resident batched closed loop.

    Args:
      setup: :class:`PaperSetup` (or a config dict for :func:`paper_setup_from_config`).
      batch: trajectories owned by this process.
      device: HIP device.
      dtype: torch.float32 (default, the benchmark precision) or torch.float64.
      disturbance: "philox" (device counter-based RNG keyed by global index and step) or "injected"
        (pass w to :meth:`step`).
      global_offset / global_batch: position of this shard in the global batch (multi-GPU).
      write_log: keep the per-step record (x, u, xbar, ubar, b, L, gQ, gR, gqb) on device.
      record_costs: keep the costs behind those decisions (``costs`` [I_nom + I_aux, 8, B]: every
        line-search candidate's cost by alpha position; fused kernels only).
      record_choices: keep the step's decision record (``choices`` [I_nom + I_aux, B] int8: the winning
        line-search alpha position of every nominal, then ancillary iteration, -1 not run).
      grad_bound: health policy of the shared update -- a trajectory whose DOC gradient row has a
        component above this magnitude drops out of the batch mean like a flagged one.  Default: 1e6 in
        f32 (the reference's own f32 path overflows on such trajectories: obstacle-grazing ancillary plans
        give |g| ~ 1e15-1e30 against ~1e2 typical), none in f64.  At B = 1 on the reference's closed loop
        the bound never triggers, so the update is the reference's exactly (tests/test_gpu_parity.py).
    """

    def __init__(self, setup, *, batch: int, device="cuda", dtype=torch.float32, disturbance: str = "philox",
                 seed: int = 0, global_offset: int = 0, global_batch: Optional[int] = None, process_group=None,
                 write_log: bool = False, record_choices: bool = False, grad_bound: Optional[float] = None,
                 record_costs: bool = False, overlap: Optional[bool] = None):
        if isinstance(setup, dict):
            setup = paper_setup_from_config(setup)
        self.setup: PaperSetup = setup
        self.B = int(batch)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("TubeMPC runs on a HIP device; there is no CPU fallback")
        self.dtype = dtype
        self.global_offset = int(global_offset)
        self.global_batch = int(global_batch) if global_batch is not None else self.B
        self.group = process_group
        self.lib = _lib.load()
        p = setup.problem
        self.N = N = p.horizon
        if setup.ilqr_nom.line_search_alphas != setup.ilqr_aux.line_search_alphas:
            raise ValueError("nominal and ancillary solves must share the line-search alphas")
        self._dt = _dtype_code(torch.empty(0, dtype=dtype))
        self.spec = p.to_c()
        cfg = _abi.DtmpcTubeCfg()
        cfg.nominal = setup.nominal_cost.to_c()
        cfg.nom_ilqr = setup.ilqr_nom.to_c()
        cfg.aux_ilqr = setup.ilqr_aux.to_c()
        if disturbance not in ("philox", "injected"):
            raise ValueError("disturbance must be 'philox' or 'injected'")
        cfg.disturbance = 1 if disturbance == "philox" else 0
        cfg.write_log = 1 if write_log else 0
        cfg.seed = int(seed) & ((1 << 64) - 1)
        for f in range(3):
            cfg.w_low[f] = float(setup.w_low[f])
            cfg.w_high[f] = float(setup.w_high[f])
        if grad_bound is None:
            grad_bound = DEFAULT_GRAD_BOUND_F32 if dtype == torch.float32 else 0.0
        cfg.grad_bound = float(grad_bound)
        self.cfg = cfg
        self.adapt = setup.adapt.to_c()
        kw = dict(dtype=dtype, device=self.device)
        B = self.B
        self.x = torch.zeros(3, B, **kw)
        self.b = torch.zeros(B, **kw)
        self.xbar = torch.zeros(3, B, **kw)
        self.bbar = torch.zeros(B, **kw)
        self.Xnom = torch.zeros(N + 1, 4, B, **kw)
        self.Unom = torch.zeros(N, 2, B, **kw)
        self.Xaux = torch.zeros(N + 1, 4, B, **kw)
        self.Uaux = torch.zeros(N, 2, B, **kw)
        # lanes per trajectory and the fast kernel's launch chunk: resolved once here (DTMPC_TUBE_LANES and
        # DTMPC_FAST_CHUNK are read by the library only now), and the workspace sized for exactly these
        self.lanes = int(self.lib.dtmpc_tube_lanes_dtype(B, self._dt))  # the precision's own rule (ABI 6)
        self.chunk = int(self.lib.dtmpc_tube_chunk(N, self.lanes))
        wbytes = int(self.lib.dtmpc_tube_workspace_bytes(self._dt, N, B, self.lanes, self.chunk))
        if wbytes <= 0:
            raise ValueError(f"no tube-step workspace for horizon {N}, batch {B}, lanes {self.lanes}")
        self.work = torch.empty(wbytes, dtype=torch.uint8, device=self.device)
        self.n_partials = int(self.lib.dtmpc_tube_partials_count(B, self.lanes))
        self.partials = torch.zeros(self.n_partials, _abi.TUBE_SUMS, **kw)
        # theta, vel and sums are written by the theta update, which overlap mode runs on a side stream after step()
        # returns: the public names are properties that join() first, the buffers live here
        self._sums = torch.zeros(_abi.TUBE_SUMS, **kw)
        self._theta0 = torch.tensor(setup.theta0, **kw)
        self._theta = self._theta0.clone()
        self._vel = torch.zeros(6, **kw)
        self._theta_ready = None  # event on the side stream: the last step's theta update is done
        self.status = torch.zeros(B, dtype=torch.int32, device=self.device)
        self.iters = torch.zeros(2, B, dtype=torch.int32, device=self.device)
        self.log = torch.zeros(_abi.LOG_FIELDS, B, **kw) if write_log else None
        nch = setup.ilqr_nom.max_iter + setup.ilqr_aux.max_iter
        self.choices = (torch.full((max(nch, 1), B), -1, dtype=torch.int8, device=self.device)
                        if record_choices else None)
        # the costs behind the decisions: [I_nom + I_aux, 8, B] every candidate's J by alpha position (fused
        # kernels only; NaN where not run)
        self.costs = (torch.full((max(nch, 1), 8, B), float("nan"), dtype=dtype, device=self.device)
                      if record_costs else None)
        self.t = 0
        st = _abi.DtmpcTubeState()
        st.x, st.b, st.xbar, st.bbar = (t.data_ptr() for t in (self.x, self.b, self.xbar, self.bbar))
        st.Xnom, st.Unom, st.Xaux, st.Uaux = (t.data_ptr() for t in (self.Xnom, self.Unom, self.Xaux, self.Uaux))
        st.work = self.work.data_ptr()
        st.theta = self._theta.data_ptr()
        st.partials = self.partials.data_ptr()
        st.log = self.log.data_ptr() if self.log is not None else None
        st.status = self.status.data_ptr()
        st.iters = self.iters.data_ptr()
        st.lanes = self.lanes
        st.n_partials = self.n_partials
        st.chunk = self.chunk
        st.work_bytes = wbytes
        st.choices = self.choices.data_ptr() if self.choices is not None else None
        st.costs = self.costs.data_ptr() if self.costs is not None else None
        st.phase = 0
        self.state = st
        # overlap (the nominal solve is theta-independent, core/tube_mpc.py:723-728): each step runs
        # as two launches (dtmpc_tube_state.phase 1: nominal, 2: the rest) and its theta all-reduce + update go to
        # a side stream, which the NEXT step's phase 2 waits on -- so the collective overlaps the next nominal
        # solve and never blocks the launch stream.  Default: on when the step has a cross-rank sum (a process
        # group of > 1 ranks) and the fused kernel runs it in one chunk of ITS precision (dtmpc_tube_split_ok: the f64
        # chunk is about half the f32 one); overlap=True forces it (tests).
        import torch.distributed as dist

        multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1
        can = bool(self.lib.dtmpc_tube_split_ok(self._dt, C.byref(self.spec), C.byref(self.cfg), self.B, self.lanes,
                                                self.chunk))
        if overlap and not can:
            raise ValueError("overlap needs the fused tube kernel and B within one launch chunk (dtmpc_tube_split_ok)")
        self.overlap = bool(can and (multi if overlap is None else overlap))
        self._side = torch.cuda.Stream(device=self.device) if self.overlap else None

    # -----------------------------------------------------------------------------------------
    def join(self) -> None:
        """Make the current stream wait for the side stream's theta update (overlap mode): after it, theta,
        vel and sums are the last step's on the current stream.  A no-op otherwise."""
        if self._theta_ready is not None:
            torch.cuda.current_stream(self.device).wait_event(self._theta_ready)

    # the adaptation state: every read (and in-place write) through these orders the current stream after the last
    # step's theta update, wherever overlap mode put it
    @property
    def theta(self) -> Tensor:
        """[6] shared ancillary weights Qa(3), Ra(2), qba after the last step's update."""
        self.join()
        return self._theta

    @property
    def vel(self) -> Tensor:
        """[6] momentum of the theta update."""
        self.join()
        return self._vel

    @property
    def sums(self) -> Tensor:
        """[8] the last step's global sums L, gQ(3), gR(2), gqb, healthy count."""
        self.join()
        return self._sums

    def reset(self, x0: Tensor, U_nom0: Optional[Tensor] = None, U_aux0: Optional[Tensor] = None) -> None:
        """x0 [B, 3]: plant and nominal start at x0, b0 = B(h(x0)) (core/tube_mpc.py:770-779);
        warm starts default to zero; theta and momentum restart from the setup."""
        if x0.shape != (self.B, 3):
            raise ValueError(f"x0 must be [{self.B}, 3]")
        self.join()
        if U_nom0 is None and U_aux0 is None:
            # the whole episode start in one launch (dtmpc_tube_reset)
            x0c = x0.to(device=self.device, dtype=self.dtype).contiguous()
            _lib.check(self.lib.dtmpc_tube_reset(self._dt, C.byref(self.spec), self.B, x0c.data_ptr(),
                                                 C.byref(self.state), self._theta0.data_ptr(),
                                                 self._theta.data_ptr(), self._vel.data_ptr(), self._stream()),
                       "dtmpc_tube_reset")
            self.t = 0
            return
        xs = x0.to(device=self.device, dtype=self.dtype).t().contiguous()
        self.x.copy_(xs)
        self.xbar.copy_(xs)
        _lib.check(self.lib.dtmpc_dbas_init(self._dt, C.byref(self.spec), self.B, self.x.data_ptr(),
                                            self.b.data_ptr(), self._stream()), "dtmpc_dbas_init")
        self.bbar.copy_(self.b)
        self.Unom.zero_()
        self.Uaux.zero_()
        if U_nom0 is not None:
            self.Unom.copy_(U_nom0.to(self.Unom).permute(1, 2, 0))
        if U_aux0 is not None:
            self.Uaux.copy_(U_aux0.to(self.Uaux).permute(1, 2, 0))
        self._theta.copy_(self._theta0)
        self._vel.zero_()
        self.status.zero_()
        self.t = 0

    def _stream(self) -> int:
        return int(torch.cuda.current_stream(self.device).cuda_stream)

    def step(self, w: Optional[Tensor] = None, kernel_events=None, adapt: bool = True) -> None:
        """One closed-loop step for the whole batch (asynchronous on the current stream).
        kernel_events: optional torch.cuda.Event pair (start, end) recorded around the fused kernel -- in overlap mode
        a 4-tuple (start1, end1, start2, end2) around its two launches, so that the kernel time (the sum of the two
        spans) excludes the launch stream's wait for the previous step's theta update, which is end1 -> start2
        (ADVICE r05); a pair is accepted there too and then spans both launches and the wait.
        adapt=False: theta is held (no partial-sum reduction, all-reduce or update) -- the tube MPC of
        BASELINE config 3 without the adaptation step of config 4; the IFT pass still runs in the fused
        kernel (its per-trajectory rows land in the log)."""
        wp = None
        if self.cfg.disturbance == 0:
            if w is None or w.shape != (self.B, 3):
                raise ValueError(f"injected disturbance w must be [{self.B}, 3]")
            self._w = w.to(device=self.device, dtype=self.dtype).t().contiguous()
            wp = self._w.data_ptr()
        s = self._stream()
        if self.costs is not None:  # the kernel writes the candidates that ran: NaN marks the rest
            self.costs.fill_(float("nan"))
        ev = tuple(kernel_events) if kernel_events is not None else ()
        if len(ev) not in (0, 2, 4):
            raise ValueError("kernel_events: a (start, end) pair or, in overlap mode, (start1, end1, start2, end2)")
        if ev:
            ev[0].record()
        if self.overlap:
            self._launch(1, wp, s)  # the nominal solve: no theta (the side stream may still be updating it)
            if len(ev) == 4:
                ev[1].record()
            self.join()
            if len(ev) == 4:
                ev[2].record()
            self._launch(2, wp, s)
        else:
            self._launch(0, wp, s)
        if ev:
            ev[-1].record()
        if not adapt:
            self.t += 1
            return
        if self.overlap:
            _lib.check(self.lib.dtmpc_partials_reduce(self._dt, self.n_partials, self.partials.data_ptr(),
                                                      self._sums.data_ptr(), s), "dtmpc_partials_reduce")
            ready = torch.cuda.Event()
            ready.record()
            side = self._side
            side.wait_event(ready)
            with torch.cuda.stream(side):
                allreduce_sums(self._sums, self.group)  # RCCL's stream waits on `side`, `side` on the collective
                _lib.check(self.lib.dtmpc_theta_update(self._dt, C.byref(self.adapt), 0.0, self._sums.data_ptr(),
                                                       self._theta.data_ptr(), self._vel.data_ptr(),
                                                       int(side.cuda_stream)), "dtmpc_theta_update")
                self._theta_ready = torch.cuda.Event()
                self._theta_ready.record(side)
            self.t += 1
            return
        _lib.check(self.lib.dtmpc_partials_reduce(self._dt, self.n_partials, self.partials.data_ptr(),
                                                  self._sums.data_ptr(), s), "dtmpc_partials_reduce")
        allreduce_sums(self._sums, self.group)
        # inv_batch 0: batch mean over the healthy trajectories (sums[7] counts them across ranks)
        _lib.check(self.lib.dtmpc_theta_update(self._dt, C.byref(self.adapt), 0.0,
                                               self._sums.data_ptr(), self._theta.data_ptr(), self._vel.data_ptr(), s),
                   "dtmpc_theta_update")
        self.t += 1

    def _launch(self, phase: int, wp, s: int) -> None:
        self.state.phase = phase
        _lib.check(self.lib.dtmpc_tube_step(self._dt, C.byref(self.spec), C.byref(self.cfg), self.B,
                                            self.global_offset, self.t, C.byref(self.state), wp, s),
                   "dtmpc_tube_step")

    def check(self) -> None:
        raise_for_status(self.status, "tube step")

    # convenience views (trajectory-major copies)
    @property
    def loss_mean(self) -> float:
        """Mean upper loss of the last step over the healthy trajectories of the global batch."""
        self.join()
        n = float(self.sums[_abi.TUBE_SUMS - 1])
        return float(self.sums[0]) / n if n > 0 else float("nan")

    @property
    def healthy_count(self) -> int:
        """Trajectories of the global batch that contributed to the last step's mean gradient."""
        self.join()
        return int(round(float(self.sums[_abi.TUBE_SUMS - 1])))

    @property
    def flagged_count(self) -> int:
        """Trajectories of the global batch with a status flag (OR-accumulated over the episode)."""
        n = torch.tensor([float((self.status != 0).sum())], dtype=torch.float64, device=self.status.device)
        return int(round(float(allreduce_sums(n, self.group))))

    @property
    def bound_dropped_count(self) -> int:
        """Trajectories of the global batch that the last step's mean gradient left out ONLY because of
        the health bound: a gradient component above ``grad_bound`` or non-finite -- non-finite
        rows are left out even with the bound disabled, since one NaN row would make the batch mean NaN --
        i.e. the global batch minus the healthy and the flagged trajectories."""
        return self.global_batch - self.healthy_count - self.flagged_count

    def nominal_tape(self):
        return self.Xnom.permute(2, 0, 1), self.Unom.permute(2, 0, 1)


# ---------------------------------------------------------------------------------------------
class GeneralTubeMPC:
    """Device-resident batched closed loop of the general path (core/tube_mpc.py:40-663).

    theta [2, 12] (raw, DTMPC_P_* layout; row 0 ancillary, row 1 nominal) is shared by the batch
    and updated with the batch-mean IFT gradient; at B = 1 every step is the reference's loop body.
    Arguments as :class:`TubeMPC`."""

    def __init__(self, setup, *, batch: int, device="cuda", dtype=torch.float32, disturbance: str = "philox",
                 seed: int = 0, global_offset: int = 0, global_batch: Optional[int] = None, process_group=None,
                 write_log: bool = False):
        if isinstance(setup, dict):
            setup = general_setup_from_config(setup)
        self.setup: GeneralSetup = setup
        if setup.adapt_steps != 1:
            raise NotImplementedError("adaptation.steps != 1 is not supported (core/tube_mpc.py:401)")
        self.B = int(batch)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("GeneralTubeMPC runs on a HIP device; there is no CPU fallback")
        self.dtype = dtype
        self.global_offset = int(global_offset)
        self.global_batch = int(global_batch) if global_batch is not None else self.B
        self.group = process_group
        self.lib = _lib.load()
        self.N = N = setup.problem.horizon
        if disturbance not in ("philox", "injected"):
            raise ValueError("disturbance must be 'philox' or 'injected'")
        self._dt = _dtype_code(torch.empty(0, dtype=dtype))
        self.spec = setup.problem.to_c()
        self.cfg = setup.to_c(disturbance=1 if disturbance == "philox" else 0, seed=seed, write_log=write_log)
        kw = dict(dtype=dtype, device=self.device)
        B = self.B
        self.x = torch.zeros(3, B, **kw)
        self.b = torch.zeros(B, **kw)
        self.xbar = torch.zeros(3, B, **kw)
        self.bbar = torch.zeros(B, **kw)
        self.Xnom = torch.zeros(N + 1, 4, B, **kw)
        self.Unom = torch.zeros(N, 2, B, **kw)
        self.Xaux = torch.zeros(N + 1, 4, B, **kw)
        self.Uaux = torch.zeros(N, 2, B, **kw)
        self.work = torch.empty(self.lib.dtmpc_general_workspace_bytes(self._dt, N, B), dtype=torch.uint8,
                                device=self.device)
        self.n_partials = int(self.lib.dtmpc_general_partials_count(B))
        self.partials = torch.zeros(self.n_partials, _abi.GEN_SUMS, **kw)
        self.sums = torch.zeros(_abi.GEN_SUMS, **kw)
        self._theta0 = torch.tensor(setup.theta0, **kw)
        self.theta = self._theta0.clone()
        self.vel = torch.zeros(2, _abi.P_COUNT, **kw)
        self.gout = torch.zeros(_abi.GEN_SUMS, B, **kw)
        self.status = torch.zeros(B, dtype=torch.int32, device=self.device)
        self.iters = torch.zeros(2, B, dtype=torch.int32, device=self.device)
        self.log = torch.zeros(_abi.GEN_LOG_FIELDS, B, **kw) if write_log else None
        self.t = 0
        st = _abi.DtmpcGeneralState()
        st.x, st.b, st.xbar, st.bbar = (t.data_ptr() for t in (self.x, self.b, self.xbar, self.bbar))
        st.Xnom, st.Unom, st.Xaux, st.Uaux = (t.data_ptr() for t in (self.Xnom, self.Unom, self.Xaux, self.Uaux))
        st.work = self.work.data_ptr()
        st.theta = self.theta.data_ptr()
        st.velocity = self.vel.data_ptr()
        st.partials = self.partials.data_ptr()
        st.sums = self.sums.data_ptr()
        st.gout = self.gout.data_ptr()
        st.log = self.log.data_ptr() if self.log is not None else None
        st.status = self.status.data_ptr()
        st.iters = self.iters.data_ptr()
        st.n_partials = self.n_partials
        self.state = st

    def _stream(self) -> int:
        return int(torch.cuda.current_stream(self.device).cuda_stream)

    def _spec_for(self, row, nominal: bool):
        """spec with the DBaS parameters of a raw row (core/tube_mpc.py:134-153)"""
        import dataclasses

        p = dataclasses.replace(self.setup.problem, dbas_alpha=softplus(float(row[9])) + 1e-6,
                                dbas_gamma=math.tanh(float(row[10])))
        sp = p.to_c()
        sp.h_offset = softplus(float(row[11])) if nominal else 0.0
        return sp

    def reset(self, x0: Tensor, U_nom0: Optional[Tensor] = None, U_aux0: Optional[Tensor] = None) -> None:
        """x0 [B, 3]: plant and nominal start at x0; b0 = B_theta(h(x0)), bbar0 = B_theta_bar(h(x0) - s)
        (core/tube_mpc.py:157-158); warm starts zero; theta / momentum restart from the setup."""
        if x0.shape != (self.B, 3):
            raise ValueError(f"x0 must be [{self.B}, 3]")
        xs = x0.to(device=self.device, dtype=self.dtype).t().contiguous()
        self.x.copy_(xs)
        self.xbar.copy_(xs)
        s = self._stream()
        for row, nominal, out in ((self.setup.theta0[0], False, self.b), (self.setup.theta0[1], True, self.bbar)):
            sp = self._spec_for(row, nominal)
            _lib.check(self.lib.dtmpc_dbas_init(self._dt, C.byref(sp), self.B, self.x.data_ptr(), out.data_ptr(), s),
                       "dtmpc_dbas_init")
        self.Unom.zero_()
        self.Uaux.zero_()
        if U_nom0 is not None:
            self.Unom.copy_(U_nom0.to(self.Unom).permute(1, 2, 0))
        if U_aux0 is not None:
            self.Uaux.copy_(U_aux0.to(self.Uaux).permute(1, 2, 0))
        self.theta.copy_(self._theta0)
        self.vel.zero_()
        self.status.zero_()
        self.t = 0

    def step(self, w: Optional[Tensor] = None, kernel_events=None) -> None:
        """One closed-loop step of the general path for the whole batch (asynchronous)."""
        wp = None
        if self.cfg.disturbance == 0:
            if w is None or w.shape != (self.B, 3):
                raise ValueError(f"injected disturbance w must be [{self.B}, 3]")
            self._w = w.to(device=self.device, dtype=self.dtype).t().contiguous()
            wp = self._w.data_ptr()
        s = self._stream()
        if kernel_events is not None:
            kernel_events[0].record()
        _lib.check(self.lib.dtmpc_general_step(self._dt, C.byref(self.spec), C.byref(self.cfg), self.B,
                                               C.byref(self.state), s), "dtmpc_general_step")
        if kernel_events is not None:
            kernel_events[1].record()
        _lib.check(self.lib.dtmpc_partials_reduce_n(self._dt, self.n_partials, _abi.GEN_SUMS,
                                                    self.partials.data_ptr(), self.sums.data_ptr(), s),
                   "dtmpc_partials_reduce_n")
        allreduce_sums(self.sums, self.group)
        # inv_batch 0: batch mean over the healthy trajectories (sums[24] counts them across ranks)
        _lib.check(self.lib.dtmpc_general_update(self._dt, C.byref(self.spec), C.byref(self.cfg),
                                                 0.0, C.byref(self.state), s),
                   "dtmpc_general_update")
        _lib.check(self.lib.dtmpc_general_plant(self._dt, C.byref(self.spec), C.byref(self.cfg), self.B,
                                                self.global_offset, self.t, C.byref(self.state), wp, s),
                   "dtmpc_general_plant")
        self.t += 1

    def check(self) -> None:
        raise_for_status(self.status, "general tube step")

    @property
    def loss_mean(self) -> float:
        """Mean upper loss of the last step over the healthy trajectories of the global batch."""
        n = float(self.sums[_abi.GEN_SUMS - 1])
        return float(self.sums[0]) / n if n > 0 else float("nan")


def _save_outputs(run_dir: str, traj: ExperimentTrajectories) -> None:
    """core/tube_mpc.py:626-636"""
    os.makedirs(run_dir, exist_ok=True)
    np.save(os.path.join(run_dir, "x_real.npy"), np.stack(traj.x_real, axis=0))
    np.save(os.path.join(run_dir, "u_real.npy"), np.stack(traj.u_real, axis=0))
    np.save(os.path.join(run_dir, "x_bar.npy"), np.stack(traj.x_bar, axis=0))
    np.save(os.path.join(run_dir, "u_bar.npy"), np.stack(traj.u_bar, axis=0))
    np.save(os.path.join(run_dir, "b_real.npy"), np.stack(traj.b_real, axis=0))
    np.save(os.path.join(run_dir, "loss.npy"), np.asarray(traj.loss, dtype=np.float64))
    if len(traj.Qa_history) > 0:
        np.save(os.path.join(run_dir, "Qa_history.npy"), np.stack(traj.Qa_history, axis=0))
        np.save(os.path.join(run_dir, "Ra_history.npy"), np.stack(traj.Ra_history, axis=0))
        np.save(os.path.join(run_dir, "qba_history.npy"), np.asarray(traj.qba_history, dtype=np.float64))


def _run_general(cfg: Dict[str, Any], *, device, run_dir: str) -> Dict[str, Any]:
    """General path of core/tube_mpc.py:40-663 for one trajectory on the HIP device."""
    setup = general_setup_from_config(cfg)
    dtype = torch.float64 if setup.use_float64 else torch.float32
    H = setup.task_horizon
    mpc = GeneralTubeMPC(setup, batch=1, device=device, dtype=dtype, disturbance="injected", write_log=True)
    mpc.reset(torch.tensor([list(setup.x0)], dtype=dtype, device=device))
    low = torch.tensor(setup.w_low, device=device, dtype=dtype)
    high = torch.tensor(setup.w_high, device=device, dtype=dtype)
    logs = torch.zeros(H, _abi.GEN_LOG_FIELDS, dtype=dtype, device=device)
    thetas = torch.zeros(H, 2, _abi.P_COUNT, dtype=dtype, device=device)
    probe = torch.empty(1, 3, device=device, dtype=dtype)
    for t in range(H):
        if (t % 25) == 0:
            print(f"[step {t}/{H}] running...", flush=True)
        w = low + (high - low) * torch.rand_like(probe)
        mpc.step(w)
        logs[t].copy_(mpc.log[:, 0])
        thetas[t].copy_(mpc.theta)
    mpc.check()
    lg = logs.cpu().numpy()
    th = torch.nn.functional.softplus(thetas[:, 0]).cpu().numpy()  # theta.Q() etc. (:611-614)
    traj = ExperimentTrajectories(
        x_real=list(lg[:, 0:3]), u_real=list(lg[:, 3:5]), x_bar=list(lg[:, 5:8]), u_bar=list(lg[:, 8:10]),
        loss=[float(v) for v in lg[:, 11]], b_real=list(lg[:, 10]),
        Qa_history=list(th[:, 0:3]) if setup.adapt_ancillary else [],
        Ra_history=list(th[:, 3:5]) if setup.adapt_ancillary else [],
        qba_history=[float(v) for v in th[:, 8]] if setup.adapt_ancillary else [])
    _save_outputs(run_dir, traj)
    summary = {
        "system": "dubins",
        "H": H,
        "N": setup.problem.horizon,
        "final_state": np.asarray(traj.x_real[-1]).tolist(),
        "final_barrier_state": float(np.array(traj.b_real[-1]).reshape(-1)[0]),
        "final_loss": float(traj.loss[-1]),
    }
    return {"summary": summary}


# ---------------------------------------------------------------------------------------------
def run_closed_loop_experiment(cfg: Dict[str, Any], *, device: torch.device, run_dir: str) -> Dict[str, Any]:
    """Drop-in for core/tube_mpc.py:40 in the configured paper mode (core/tube_mpc.py:666-1048).

    The disturbance is drawn exactly as the reference draws it (torch.rand_like on ``device`` with
    the global generator, core/systems/dubins.py:59-67), then injected into the fused HIP step, so a
    seeded run consumes the same random stream as the reference."""
    system_cfg = cfg["system"]
    if system_cfg["name"] != "dubins":
        raise NotImplementedError("Only dubins is wired in the skeleton; other systems are added next.")
    paper_mode = bool(cfg.get("paper_dubins_mode", True))
    adapt_nominal = bool(cfg.get("adaptation", {}).get("adapt_nominal", True))
    device = torch.device(device)
    if not (paper_mode and not adapt_nominal):  # core/tube_mpc.py:48-49
        return _run_general(cfg, device=device, run_dir=run_dir)
    setup = paper_setup_from_config(cfg)
    dtype = torch.float64 if setup.use_float64 else torch.float32
    H = setup.task_horizon
    mpc = TubeMPC(setup, batch=1, device=device, dtype=dtype, disturbance="injected", write_log=True)
    x0 = torch.tensor([list(setup.x0)], dtype=dtype, device=device)
    mpc.reset(x0)
    low = torch.tensor(setup.w_low, device=device, dtype=dtype)
    high = torch.tensor(setup.w_high, device=device, dtype=dtype)
    logs = torch.zeros(H, _abi.LOG_FIELDS, dtype=dtype, device=device)
    thetas = torch.zeros(H, 6, dtype=dtype, device=device)
    probe = torch.empty(1, 3, device=device, dtype=dtype)
    for t in range(H):
        if (t % 25) == 0:
            print(f"[step {t}/{H}] running...", flush=True)
        w = low + (high - low) * torch.rand_like(probe)
        mpc.step(w)
        logs[t].copy_(mpc.log[:, 0])
        thetas[t].copy_(mpc.theta)
    mpc.check()
    lg = logs.cpu().numpy()
    th = thetas.cpu().numpy()
    traj = ExperimentTrajectories(
        x_real=list(lg[:, 0:3]), u_real=list(lg[:, 3:5]), x_bar=list(lg[:, 5:8]), u_bar=list(lg[:, 8:10]),
        loss=[float(v) for v in lg[:, 11]], b_real=list(lg[:, 10]), Qa_history=list(th[:, 0:3]),
        Ra_history=list(th[:, 3:5]), qba_history=[float(v) for v in th[:, 5]])
    _save_outputs(run_dir, traj)
    summary = {
        "system": "dubins",
        "H": H,
        "N": setup.problem.horizon,
        "final_state": np.asarray(traj.x_real[-1]).tolist(),
        "final_barrier_state": float(np.array(traj.b_real[-1]).reshape(-1)[0]),
        "final_loss": float(traj.loss[-1]),
        "note": "Dubins run aligned to paper: nominal fixed, ancillary adapts, alpha=0, gamma=0.",
    }
    return {"summary": summary}
