"""Build libdtmpc.so (HIP, gfx950) in-tree: differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc.so.

Plain hipcc, no build system: one translation unit (csrc/dtmpc_kernels.hip).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "dtmpc_kernels.hip")
DEPS = [os.path.join(HERE, "csrc", f) for f in ("dtmpc_device.hpp", "dtmpc_solver.hpp")] + [
    os.path.join(os.path.dirname(HERE), "include", "dtmpc.h")
]
OUT = os.path.join(HERE, "diff_tube_mpc_strict_pt", "libdtmpc.so")
ARCH = os.environ.get("DTMPC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-std=c++17", "-Wall", "-Wno-unused-function"]


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(p) <= t for p in [SRC, *DEPS, __file__])


def build(force: bool = False) -> str:
    if not force and up_to_date():
        return OUT
    cmd = [HIPCC, *FLAGS, "-o", OUT + ".tmp", SRC]
    print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
