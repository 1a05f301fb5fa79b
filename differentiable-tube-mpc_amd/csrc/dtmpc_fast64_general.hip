// dtmpc_fast64_general.hip — the general path's two solves (dtmpc_general_step) on the fused solver in f64:
// dtmpc_fast.hip with real = double, its general-solve host part (suffix 64).
#define DTMPC_FAST_F64 1
#define DTMPC_FAST_GENERAL_TU 1
#include "dtmpc_fast.hip"
