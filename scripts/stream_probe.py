"""What the HBM delivers to the headline kernel's own record stream at its own occupancy (GPU).

stream_probe_kernel (csrc/dtmpc_fast.hip, dtmpc_diag_stream_probe) streams the tube kernel's records -- per step a
16-B X row, an 8-B U row and a 32-B gain record read, the other bank's X and U rows written (70 % read), buffer
accesses with the row base in soffset -- one lane per trajectory, loads D steps ahead, PASSES passes over a
horizon of 50 steps.  B = 65,536 is the headline's launch: 256 workgroups of 256 lanes, one wave per SIMD;
B = 131,072 two waves per SIMD.  Beside it the plain streams of scripts/bw_probe.py (full occupancy).
usage: python scripts/stream_probe.py [passes]"""
import ctypes as C
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "differentiable-tube-mpc_amd")]


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    from diff_tube_mpc_strict_pt import _lib

    lib = _lib.load()
    f = lib.dtmpc_diag_stream_probe
    f.restype = C.c_int
    f.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 68  # 68 x 80 B x 50 steps ~ the headline's 274 KB per trajectory
    N = 50
    s = torch.cuda.current_stream().cuda_stream
    print(f"record-stream probe: N = {N}, {passes} passes, 80 B per trajectory-step (56 read + 24 written)")
    for B in (65536, 131072, 32768, 8192):
        buf = torch.zeros(B * N * 20, dtype=torch.float32, device="cuda")
        for D in (0, 1, 2, 4):
            def run():
                rc = f(B, N, passes, D, buf.data_ptr(), s)
                assert rc == 0, lib.dtmpc_last_error()
            t = timed(run)
            nb = B * N * 80 * passes
            print(f"B = {B:6d} ({B * 1.0 / 65536:.3g} waves/SIMD)  depth {D}: {t * 1e3:7.3f} ms  {nb / t / 1e12:.2f} TB/s"
                  f"  ({nb / 1e9:.2f} GB per launch)", flush=True)
        del buf
    n = (1 << 31) // 4
    a = torch.rand(n, device="cuda")
    b = torch.rand(n, device="cuda")
    c = torch.empty_like(a)
    nb = n * 4
    print(f"float copy (torch, full occupancy)    {2 * nb / timed(lambda: c.copy_(a)) / 1e12:.2f} TB/s")
    print(f"add 2 read : 1 write (torch)          {3 * nb / timed(lambda: torch.add(a, b, out=c)) / 1e12:.2f} TB/s")


if __name__ == "__main__":
    main()
