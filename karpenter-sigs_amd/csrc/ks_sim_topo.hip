// k_solve family 3 (see ks_solve.hip: launch_family)
#define KS_TU 3
// simulations with topology scan one node per lane per step past the register window: C5 + topology
// 10.91 ms against 11.35 ms (2 per lane) and 11.09 ms (3 per lane), DESIGN §8 round 4
#define KS_NODE_K 1
#include "ks_solve.hip"
