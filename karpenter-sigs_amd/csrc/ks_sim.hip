// k_solve family 2 (see ks_solve.hip: launch_family)
#define KS_TU 2
#include "ks_solve.hip"
