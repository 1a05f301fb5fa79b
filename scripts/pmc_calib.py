"""Known-byte calibration launch for the HBM counters (run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE).

dtmpc_dbas_rollout reads x0 [4][B] + U [N][2][B] and writes X [N+1][4][B], all with the tube kernel's
access pattern (one dword per lane, 256 B per wave per field plane).  At B = 262,144 the 319 MB it
touches exceeds the 256 MiB Infinity Cache, so every byte crosses the memory-side counters once.
scripts/pmc_summary.py divides the measured bytes by the known ones to get this pattern's correction."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd")]
import torch  # noqa: E402

from diff_tube_mpc_strict_pt import _abi, _lib  # noqa: E402
from diff_tube_mpc_strict_pt.core.problem import paper_config, paper_setup_from_config  # noqa: E402

B = 262144
st = paper_setup_from_config(paper_config())
N = st.problem.horizon
spec = st.problem.to_c()
lib = _lib.load()
dev = torch.device("cuda", 0)
x0 = torch.rand(4, B, device=dev)
U = torch.rand(N, 2, B, device=dev)
X = torch.empty(N + 1, 4, B, device=dev)
for _ in range(3):
    _lib.check(lib.dtmpc_dbas_rollout(_abi.F32, C.byref(spec), B, x0.data_ptr(), U.data_ptr(), X.data_ptr(),
                                      _lib.stream_of(x0)), "dtmpc_dbas_rollout")
torch.cuda.synchronize()
print({"kernel": "rollout_kernel", "batch": B, "read_bytes": 4 * B * (4 + 2 * N),
       "write_bytes": 4 * B * 4 * (N + 1)})
