// dtmpc_fast_ilqr.hip — the standalone batched iLQR (dtmpc_ilqr_solve_ws) on dtmpc_fast.hip's solver:
// the same device code, instantiated in its own translation unit so that it compiles in parallel with
// the tube step's instantiations (the host part is the #else branch of DTMPC_FAST_ILQR_TU there).
#define DTMPC_FAST_ILQR_TU 1
#include "dtmpc_fast.hip"
