// dtmpc_fast64_p1.hip — the f64 tube step's one-lane kernels (fk64::tube_fast_kernel<M, 1, G0>) in their own
// translation unit (dtmpc_fast_p1.hip's f64 twin; launch_tube_fast_p164).
#define DTMPC_FAST_F64 1
#define DTMPC_FAST_P1_TU 1
#include "dtmpc_fast.hip"
