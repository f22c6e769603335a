// k_solve family 1 (see ks_solve.hip: launch_family)
#define KS_TU 1
#include "ks_solve.hip"
