// dtmpc_fast_general.hip — the general IFT path's two solves (dtmpc_general_step) on dtmpc_fast.hip's
// solver: the same device code, instantiated in its own translation unit (compiled in parallel with the
// tube step's; the host part is the DTMPC_FAST_GENERAL_TU branch there).
#define DTMPC_FAST_GENERAL_TU 1
#include "dtmpc_fast.hip"
