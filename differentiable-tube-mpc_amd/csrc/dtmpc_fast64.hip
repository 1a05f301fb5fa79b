// dtmpc_fast64.hip — the fused tube step (dtmpc_fast.hip) instantiated in f64, the reference's configured
// precision (configs/dubins.yaml:8 use_float64: true): the same kernel source with `real` = double, in its
// own namespace (fk64) and translation unit; its host entry points carry the suffix 64 (dtmpc_host.hpp).
#define DTMPC_FAST_F64 1
#include "dtmpc_fast.hip"
