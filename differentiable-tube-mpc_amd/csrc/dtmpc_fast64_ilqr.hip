// dtmpc_fast64_ilqr.hip — the standalone batched iLQR (dtmpc_ilqr_solve_ws) on the fused solver in f64 (the
// reference's configured precision): dtmpc_fast.hip with real = double, its iLQR host part (suffix 64).
#define DTMPC_FAST_F64 1
#define DTMPC_FAST_ILQR_TU 1
#include "dtmpc_fast.hip"
