"""Dubins system, obstacle safety functions and the DBaS-augmented Jacobian (counterpart of the
reference's core/systems/), evaluated by per-point HIP kernels (include/dtmpc_systems.h)."""
