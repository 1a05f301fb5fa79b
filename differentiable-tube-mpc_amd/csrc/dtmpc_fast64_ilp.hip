// dtmpc_fast64_ilp.hip — the f64 tube step's one-lane kernels (fk64::tube_fast_kernel<M, 1, G0>) in their own
// translation unit (dtmpc_fast_ilp.hip's f64 twin, launch_tube_fast_ilp64; the f64 two-lane form gained nothing from
// the iterative ILP schedule and stays in dtmpc_fast64.hip).
#define DTMPC_FAST_F64 1
#define DTMPC_FAST_ILP_TU 1
#include "dtmpc_fast.hip"
