// dtmpc_fast_ilp.hip — the tube step's one- and two-lane kernels (tube_fast_kernel<M, 1 | 2, G0>: the headline batch's
// form and the 16,384-32,768 shards') in their own translation unit, so that build.py can compile them with the
// scheduler that suits one or two waves per SIMD (UNIT_FLAGS: iterative ILP); dtmpc_fast.hip's launcher calls
// launch_tube_fast_ilp for them.
#define DTMPC_FAST_ILP_TU 1
#include "dtmpc_fast.hip"
