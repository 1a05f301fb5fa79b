"""MI355X-native batched differentiable tube MPC (drop-in package name of the reference).

Host Python over PyTorch-ROCm; the hot path runs in hand-written HIP kernels behind the C ABI of
include/dtmpc.h (libdtmpc.so, loaded by :mod:`._lib`).
"""
