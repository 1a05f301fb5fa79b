"""Multi-process (world_size 2, gloo, CPU) test of the sharded closed loop: contiguous global-index
shards (shard_range), Philox disturbances keyed by global index, the cross-rank sum of the
[L, gQ, gR, gqb] vector (allreduce_sums) and the identical theta update on every rank must reproduce
the single-process run over the whole batch.  The per-trajectory step is computed by the oracle
(CPU stand-in for the HIP kernel; the kernel itself is checked against the oracle in test_gpu_parity)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

B_GLOBAL = 48
STEPS = 2
SEED = 5


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_shard(lo, hi, allreduce):
    """Closed loop over global trajectories [lo, hi) with the oracle; returns (x per step, theta per step)."""
    from _common import paper_setup

    from diff_tube_mpc_strict_pt import _abi
    from diff_tube_mpc_strict_pt.core import allreduce_sums
    from oracle.oracle import Oracle

    st = paper_setup()
    o = Oracle(np.float64)
    sp = st.problem.to_c()
    N = st.problem.horizon
    rng = np.random.default_rng(0)
    xg = np.stack([rng.uniform(0, 1, B_GLOBAL), rng.uniform(0, 1, B_GLOBAL), rng.uniform(0, np.pi / 2, B_GLOBAL)], 1)
    x = xg[lo:hi]
    B = hi - lo
    b = o.barrier(sp, o.h_eval(sp, x[:, 0], x[:, 1])[0])[0]
    state = {"x": x.T.copy(), "b": b.copy(), "xbar": x.T.copy(), "bbar": b.copy(),
             "Xnom": np.zeros((N + 1, 4, B)), "Unom": np.zeros((N, 2, B)),
             "Xaux": np.zeros((N + 1, 4, B)), "Uaux": np.zeros((N, 2, B))}
    tcfg = _abi.DtmpcTubeCfg()
    tcfg.nominal, tcfg.nom_ilqr, tcfg.aux_ilqr = st.nominal_cost.to_c(), st.ilqr_nom.to_c(), st.ilqr_aux.to_c()
    tcfg.disturbance, tcfg.seed = 1, SEED
    for f in range(3):
        tcfg.w_low[f], tcfg.w_high[f] = st.w_low[f], st.w_high[f]
    theta, vel = np.array(st.theta0), np.zeros(6)
    xs, ths = [], []
    for t in range(STEPS):
        gout, _, so, _ = o.tube_step(sp, tcfg, state, theta, goff=lo, step=t)
        assert (so == 0).all()
        sums = torch.zeros(8, dtype=torch.float64)
        sums[:7] = torch.from_numpy(gout.sum(1))
        if allreduce:
            allreduce_sums(sums)
        theta, vel = o.theta_update(st.adapt.to_c(), 1.0 / B_GLOBAL, sums.numpy(), theta, vel)
        xs.append(state["x"].copy())
        ths.append(theta.copy())
    return xs, ths


def _worker(rank, world, port, outdir):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (repo, os.path.join(repo, "differentiable-tube-mpc_amd"), here):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from diff_tube_mpc_strict_pt.core import shard_range

    lo, hi = shard_range(B_GLOBAL, rank, world)
    xs, ths = _run_shard(lo, hi, allreduce=True)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), lo=lo, hi=hi, x=np.stack(xs), th=np.stack(ths))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharded_closed_loop_matches_single_process(tmp_path, oracle_lib):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    xs_full, ths_full = _run_shard(0, B_GLOBAL, allreduce=False)
    r = [np.load(os.path.join(tmp_path, f"rank{k}.npz")) for k in range(world)]
    assert int(r[0]["hi"]) == int(r[1]["lo"]) and int(r[1]["hi"]) == B_GLOBAL
    for t in range(STEPS):
        # identical theta on every rank, equal to the single-process batch-mean update
        assert np.array_equal(r[0]["th"][t], r[1]["th"][t])
        assert np.allclose(r[0]["th"][t], ths_full[t], rtol=1e-12, atol=1e-14)
        # per-trajectory states: shards concatenated == full batch (global-index keyed disturbances)
        x_sharded = np.concatenate([r[0]["x"][t], r[1]["x"][t]], axis=1)
        assert np.allclose(x_sharded, xs_full[t], rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("world", [3])
def test_allreduce_sums_is_identity_without_process_group(world):
    from diff_tube_mpc_strict_pt.core import allreduce_sums

    v = torch.arange(8, dtype=torch.float64)
    assert torch.equal(allreduce_sums(v.clone()), v)
