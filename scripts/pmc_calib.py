"""Known-byte calibration launch for the HBM counters (run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE).

dtmpc_diag_record_stream copies per-lane 16-byte X records and 8-byte U records ([rows][B][W], one buffer
resource) -- the fast tube kernel's own access pattern -- from src to dst.  At B = 262,144, N = 50 each
side is 319 MB, past the 256 MiB Infinity Cache, so every byte crosses the memory-side counters once.
scripts/pmc_summary.py divides the measured bytes by the known ones to correct the tube step's figures
(MI355X_MICROARCH.md §HBM: calibrate on a known byte count in your own access pattern)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd")]
import torch  # noqa: E402

from diff_tube_mpc_strict_pt import _lib  # noqa: E402

B, N = 262144, 50
lib = _lib.load()
fn = lib.dtmpc_diag_record_stream
fn.restype = C.c_int
fn.argtypes = [C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
nbytes = B * ((N + 1) * 16 + N * 8)
dev = torch.device("cuda", 0)
src = torch.rand(nbytes // 4, device=dev)
dst = torch.empty_like(src)
for _ in range(3):
    _lib.check(fn(B, N, src.data_ptr(), dst.data_ptr(), _lib.stream_of(src)), "dtmpc_diag_record_stream")
torch.cuda.synchronize()
assert torch.equal(src, dst)
print({"kernel": "record_stream_kernel", "batch": B, "read_bytes": nbytes, "write_bytes": nbytes})
