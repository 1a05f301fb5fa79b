"""Phase cycle breakdown of the fused tube step from a profiling build (libdtmpc_prof.so, built with
python differentiable-tube-mpc_amd/build.py --variant prof -D DTMPC_PROFILE).  Prints, per phase, the
mean s_memtime cycles per wave and the share of the wave lifetime.
usage: DTMPC_LIBRARY=.../libdtmpc_prof.so python scripts/phase_prof.py [--batch B]"""
import argparse
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import bench_setup, initial_states  # noqa: E402
from diff_tube_mpc_strict_pt import _lib  # noqa: E402
from diff_tube_mpc_strict_pt.core import TubeMPC  # noqa: E402

NAMES = ["nom.init", "nom.backward", "nom.linesearch", "nom.commit", "aux.init", "aux.backward",
         "aux.linesearch", "aux.commit", "misc", "sens+grad", "plant+shift"]
ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
a = ap.parse_args()
lib = _lib.load()
fast = os.environ.get("DTMPC_FAST", "1") != "0"  # the specialised kernel has its own accumulators
rd = lib.dtmpc_prof_read_fast if fast else lib.dtmpc_prof_read
rs = lib.dtmpc_prof_reset_fast if fast else lib.dtmpc_prof_reset
rd.argtypes = [C.c_void_p]
st = bench_setup("f32")
mpc = TubeMPC(st, batch=a.batch, device="cuda", dtype=torch.float32, disturbance="philox", seed=0)
x0 = initial_states(0, a.batch, "cuda", torch.float32)
mpc.reset(x0)
mpc.step()
torch.cuda.synchronize()
rs()
mpc.reset(x0)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
mpc.step(kernel_events=(e0, e1))
torch.cuda.synchronize()
buf = np.zeros(16, np.uint64)
assert rd(buf.ctypes.data) == 0
waves = a.batch * mpc.lanes // 64 if hasattr(mpc, "lanes") else a.batch // 64
cyc = buf[:11].astype(np.float64) / waves
tot = cyc.sum()
print(f"kernel {e0.elapsed_time(e1):.3f} ms; per-wave total {tot:.4g} cycles")
for n, c in zip(NAMES, cyc):
    print(f"{n:16s} {c:12.4g} cyc/wave {100 * c / tot:6.1f} %")
print("per step-pass (N=50): nom.backward/it %.0f, nom.ls/it %.0f, nom.commit/it %.0f cycles" %
      (cyc[1] / 10 / 50, cyc[2] / 10 / 50, cyc[3] / 10 / 50))

if fast and hasattr(lib, "dtmpc_prof_lsstat_fast"):
    st = np.zeros(64, np.uint64)
    lib.dtmpc_prof_lsstat_fast.argtypes = [C.c_void_p]
    assert lib.dtmpc_prof_lsstat_fast(st.ctypes.data) == 0
    for name, o in (("nominal", 0), ("ancillary", 32)):
        w = st[o:o + 8].astype(np.float64)
        n = max(float(st[o + 8]), 1.0)
        print(f"{name}: winners by alpha position {[int(x) for x in w]} (share {np.round(w / max(w.sum(), 1), 3).tolist()}); "
              f"wave-iterations {int(st[o + 8])}: all keep {st[o + 9] / n:.3f}, all first {st[o + 10] / n:.3f}, "
              f"all keep-or-first {st[o + 11] / n:.3f}")
