// dtmpc_fast_p1.hip — the tube step's one-lane kernels (tube_fast_kernel<M, 1, G0>, the headline batch's form) in
// their own translation unit, so that build.py can compile them with the scheduler that suits one wave per SIMD
// (UNIT_FLAGS); dtmpc_fast.hip's launcher calls launch_tube_fast_p1 for lanes == 1.
#define DTMPC_FAST_P1_TU 1
#include "dtmpc_fast.hip"
