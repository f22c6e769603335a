// k_solve family 3 (see ks_solve.hip: launch_family)
#define KS_TU 3
#include "ks_solve.hip"
