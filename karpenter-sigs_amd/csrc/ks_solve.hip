// ks_solve.hip — MI355X (gfx950) kernels for Scheduler.Solve.
//
// One Solve = one 64-lane wavefront (one workgroup).  The reference's Solve is a sequential commit
// chain (scheduler.go:140-189: every placement depends on all earlier ones), so the chain stays in
// one wave with wave-uniform control flow and no inter-wave synchronisation; the data-parallel
// parts of each step map onto the 64 lanes:
//   - existing-node first-fit (scheduler.go:240-244)   lane per node, ballot + ffs picks the first
//   - in-flight NodeClaim scan (scheduler.go:250-254)  lane per sorted position: a quick reject
//     (template taints, pod <= max Allocatable - requests, Compatible) from position-indexed
//     arrays, then a wave-cooperative NodeClaim.Add on candidates in order (nodeclaim.go:65-119)
//   - instance-type filter (nodeclaim.go:225-260)      lane per template IT position, ballots build
//     the remaining-options bitset and the six filterResults flags in one pass
//   - new NodeClaim per template (scheduler.go:258-283) incl. limits (filterByRemainingResources,
//     subtractMax)
// When a pod leaves a claim's requirements unchanged (resource-only pods), NodeClaim.Add's option
// filter reduces to Fits on growing requests, so the options it drops are a prefix of each
// resource's Allocatable-ascending order: a per-claim threshold per resource advances over that
// order and clears exactly the dropped options (no scan of the surviving ones).
// Latency is the bound (the chain is sequential), so everything a step touches lives in LDS or
// VGPRs: the 64-pod queue window (one lane per entry, read with readlane), the claim order, pod
// counts and quick-reject headroom per position, each claim's template / requests / max-Allocatable
// / options bitset / thresholds (for the first Plan::KL claims), the templates' Allocatable tables
// and the remaining NodePool limits.  Pointers carry explicit address spaces (ks_problem.h), so no
// access is a flat access.  Lanes never hand data to each other through HBM except at the window
// refill (behind one release fence, read with sc1 loads that bypass the L1).  HBM holds the cold
// state (requirement records, existing nodes, overflow claims) and the write-only commit log.
// Independent Solves (replicas, consolidation simulations) are independent workgroups, so a launch
// of thousands of them fills the 256 CUs.  Nothing here is a dense contraction: no MFMA.
#include <hip/hip_runtime.h>

#ifndef KS_FM_OFF
#define KS_FM_OFF 0
#endif
#ifndef KS_TU
#define KS_TU 0
#endif
#ifndef KS_RUN_MIN  // shortest run of identical pods the simulation fast path places in one step
#define KS_RUN_MIN 3
#endif
#ifndef KS_NODE_K  // existing nodes per lane per step of the first-fit scan beyond the register window
#define KS_NODE_K 2
#endif
#ifndef KS_SORT_LANE0  // 1: the claim re-sort's exact pdqsort on lane 0 (the round-2 form)
#define KS_SORT_LANE0 0
#endif
#ifndef KS_CLAIM_RUNS  // LEAN Solve: runs of identical pods placed on one NodeClaim in one step
#define KS_CLAIM_RUNS 1
#endif

#include "ks_gosort.h"
#include "ks_problem.h"
#include "ks_reqset.h"

namespace ks {

using LI32 = int32_t KS_L*;
using LI64 = int64_t KS_L*;
using LU32 = uint32_t KS_L*;
using LU64 = uint64_t KS_L*;
using GI32 = int32_t KS_G*;
using GI64 = int64_t KS_G*;
using GU32 = uint32_t KS_G*;
using DevLayout = ReqLayoutT<const KeyMeta KS_L*, const uint32_t KS_G*, const int64_t KS_G*>;
// Topology-group sets of the popped pod kept in LDS beyond word 0 (Solver::s_gw rows)
enum GroupSet : int { GS_MASK = 0, GS_SEL, GS_INV, GS_ACT, GS_N };

__device__ __forceinline__ int lane() { return (int)threadIdx.x & (kWave - 1); }
__device__ __forceinline__ uint64_t wballot(bool p) { return __ballot(p ? 1 : 0); }
__device__ __forceinline__ int ctz64(uint64_t m) { return __builtin_ctzll(m); }
__device__ __forceinline__ int popc64(uint64_t m) { return __popcll(m); }
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
// A wave-uniform branch condition.  The commit chain's control flow is uniform by construction, but
// the compiler cannot prove it for values that pass through LDS atomics or lane-indexed loads; a
// condition it believes divergent turns the whole Solve loop into exec-masked code (every loop-carried
// scalar in a VGPR, mask bookkeeping spilled to VGPR lanes).  readfirstlane makes the branch scalar.
__device__ __forceinline__ bool ub(bool x) { return __builtin_amdgcn_readfirstlane((int)x) != 0; }
__device__ __forceinline__ int64_t uni64(int64_t x) {
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
                   (uint32_t)__builtin_amdgcn_readfirstlane((int)x));
}
__device__ __forceinline__ int rdl(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ int64_t rdl64(int64_t x, int l) {
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), l) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)x, l));
}
// Ordering point for LDS traffic between the lanes of the (single) wave: the wave's LDS operations
// execute in order, so only the compiler must be kept from reordering; no s_waitcnt, no s_barrier.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
// HBM hand-off point (rare paths): every outstanding store of this wave completes first.
__device__ __forceinline__ void hbm_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); }
template <class T>
__device__ __forceinline__ T ld_sc1(const T KS_G* p) {  // L1-bypassing load of HBM state other lanes wrote
  return __hip_atomic_load((T*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t lds_and(LU32 p, uint32_t v) {  // ds_and_rtn_b32
  return __hip_atomic_fetch_and(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
// Wave-wide inclusive scans (sum / max) over the 64 lanes: DPP row_shr within each 16-lane row, then the
// rows' totals carried across by readlane.
__device__ __forceinline__ int wscan_add(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  const int r0 = __builtin_amdgcn_readlane(v, 15), r1 = r0 + __builtin_amdgcn_readlane(v, 31);
  const int r2 = r1 + __builtin_amdgcn_readlane(v, 47), l = lane();
  return v + (l >= 48 ? r2 : l >= 32 ? r1 : l >= 16 ? r0 : 0);
}
__device__ __forceinline__ int wscan_max(int v) {  // values >= -1
  auto mx = [](int a, int b) { return a > b ? a : b; };
  v = mx(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xf, 0xf, false));
  v = mx(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xf, 0xf, false));
  v = mx(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xf, 0xf, false));
  v = mx(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xf, 0xf, false));
  const int r0 = __builtin_amdgcn_readlane(v, 15), r1 = mx(r0, __builtin_amdgcn_readlane(v, 31));
  const int r2 = mx(r1, __builtin_amdgcn_readlane(v, 47)), l = lane();
  return mx(v, l >= 48 ? r2 : l >= 32 ? r1 : l >= 16 ? r0 : -1);
}
// Wave-wide reductions to a uniform value: DPP row_shr steps leave each 16-lane row's total in its lane 15,
// four readlanes combine the rows (no LDS round trip, unlike a __shfl_xor butterfly: ds_bpermute per step).
// Every lane must be active; `fill` is the operation's identity.
template <int CTRL>
__device__ __forceinline__ int dpp32(int old, int v) { return __builtin_amdgcn_update_dpp(old, v, CTRL, 0xf, 0xf, false); }
template <int CTRL>
__device__ __forceinline__ int64_t dpp64(int64_t old, int64_t v) {
  const int lo = dpp32<CTRL>((int)old, (int)v), hi = dpp32<CTRL>((int)(old >> 32), (int)(v >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int CTRL> __device__ __forceinline__ int dppT(int old, int v) { return dpp32<CTRL>(old, v); }
template <int CTRL> __device__ __forceinline__ uint32_t dppT(uint32_t old, uint32_t v) { return (uint32_t)dpp32<CTRL>((int)old, (int)v); }
template <int CTRL> __device__ __forceinline__ int64_t dppT(int64_t old, int64_t v) { return dpp64<CTRL>(old, v); }
template <int CTRL> __device__ __forceinline__ uint64_t dppT(uint64_t old, uint64_t v) { return (uint64_t)dpp64<CTRL>((int64_t)old, (int64_t)v); }
__device__ __forceinline__ int rdlT(int x, int l) { return rdl(x, l); }
__device__ __forceinline__ uint32_t rdlT(uint32_t x, int l) { return (uint32_t)rdl((int)x, l); }
__device__ __forceinline__ int64_t rdlT(int64_t x, int l) { return rdl64(x, l); }
__device__ __forceinline__ uint64_t rdlT(uint64_t x, int l) { return (uint64_t)rdl64((int64_t)x, l); }
template <class T, class F>
__device__ __forceinline__ T wred(T v, T fill, F op) {
  v = op(v, dppT<0x111>(fill, v));  // row_shr:1
  v = op(v, dppT<0x112>(fill, v));  // row_shr:2
  v = op(v, dppT<0x114>(fill, v));  // row_shr:4
  v = op(v, dppT<0x118>(fill, v));  // row_shr:8
  return op(op(rdlT(v, 15), rdlT(v, 31)), op(rdlT(v, 47), rdlT(v, 63)));
}
template <class T> __device__ __forceinline__ T wred_min(T v, T fill) { return wred(v, fill, [](T a, T b) { return b < a ? b : a; }); }
template <class T> __device__ __forceinline__ T wred_max(T v, T fill) { return wred(v, fill, [](T a, T b) { return b > a ? b : a; }); }
template <class T> __device__ __forceinline__ T wred_add(T v) { return wred(v, (T)0, [](T a, T b) { return a + b; }); }
// How many more pods requesting `req` of a resource fit a node with `free` of it, capped at m:
// floor(free / req) from a float estimate (rq ~ 1 / req from v_rcp_f32; relative error ~1e-7, so the
// estimate is within one of the quotient below m + 2 for any m < 10^6) corrected exactly by int64 multiplies.
// free < 0 (INT64_MIN marks a node that never fits) takes none.  req is wave-uniform (its branches are
// scalar); the per-lane part is branch-free: the estimate is clamped before the conversion and
// the correction and the bounds are selects.  req == 1 (the pods resource) needs no division.
__device__ __forceinline__ float run_rcp(int64_t req) { return req > 0 ? __builtin_amdgcn_rcpf((float)req) : 0.f; }
__device__ __forceinline__ int run_cap(int64_t free, int64_t req, float rq, int m) {
  if (req == 0) return free >= 0 ? m : 0;
  if (req == 1) return free <= 0 ? 0 : (free < (int64_t)m ? (int)free : m);
  const float q = fminf((float)free * rq, (float)(m + 2));
  int qi = q > 0.f ? (int)q : 0;
  qi -= (int64_t)qi * req > free ? 1 : 0;
  qi += (int64_t)(qi + 1) * req <= free ? 1 : 0;
  qi = qi < m ? qi : m;
  return free >= req ? qi : 0;
}

// Contiguous HBM -> LDS copy by the wave with U loads in flight per lane before their stores (a prologue's
// table staging is otherwise a chain of dependent round trips, one per 64 elements).
template <int U, class T>
__device__ __forceinline__ void lds_copy(T KS_L* dst, const T KS_G* src, int n) {
  int i = lane();
  for (; i + (U - 1) * kWave < n; i += U * kWave) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = src[i + u * kWave];
#pragma unroll
    for (int u = 0; u < U; u++) dst[i + u * kWave] = v[u];
  }
  for (; i < n; i += kWave) dst[i] = src[i];
}

#ifdef KS_PHASE_STATS
#define PH_BEGIN(v) uint64_t v = __builtin_amdgcn_s_memtime()
#define PH_END(v, slot) cyc[slot] += __builtin_amdgcn_s_memtime() - v
#define PHS_END(v, slot) scyc[slot] += __builtin_amdgcn_s_memtime() - v  // sub-phases (Solver member)
#define SPHS_END(o, v, slot) o.scyc[slot] += __builtin_amdgcn_s_memtime() - v  // (from k_solve)
#define FPH_END(v, slot) fcyc[slot] += __builtin_amdgcn_s_memtime() - v  // fine phases (k_solve, CT_FINE)
#else
#define PH_BEGIN(v)
#define PH_END(v, slot)
#define PHS_END(v, slot)
#define SPHS_END(o, v, slot)
#define FPH_END(v, slot)
#endif

// ------------------------------------------------------------------------------------------------
// Init: per-replica workspace state (copies of the resident initial state), one grid-stride pass.
// ------------------------------------------------------------------------------------------------
#if KS_TU == 0
__global__ void k_init(KsDev D, const KsWork* works, int nrep, const int32_t* qorder) {
  const KsDims d = D.d;
  const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t gsz = (int64_t)gridDim.x * blockDim.x;
  for (int r = 0; r < nrep; r++) {
    const KsWork W = works[r];
    for (int64_t i = gtid; i < (int64_t)d.N * d.R; i += gsz) W.n_req[i] = D.n_req0[i];
    for (int64_t i = gtid; i < (int64_t)d.N * d.RSW; i += gsz) W.n_rs[i] = D.n_rs0[i];
    for (int64_t i = gtid; i < d.N; i += gsz) W.n_hp[i] = D.n_hp0[i];
    if (d.volAny)
      for (int64_t i = gtid; i < (int64_t)d.N * d.VD; i += gsz) W.n_vc[i] = D.n_vc0[i];
    if (d.G) {
      for (int64_t i = gtid; i < d.tgCntWords; i += gsz) W.tg_cnt[i] = D.tg_cnt0[i];
      for (int64_t i = gtid; i < (int64_t)d.G * (d.Kcap + 1); i += gsz) W.tg_ccnt[i] = 0;
      for (int64_t i = gtid; i < d.G; i += gsz) W.tg_cpos[i] = 0;
      for (int64_t i = gtid; i < d.G; i += gsz) W.tg_act[i] = 0;
      for (int64_t i = gtid; i < (int64_t)d.P * d.GMW; i += gsz) W.log_hg[i] = 0;
    }
    for (int64_t i = gtid; i < d.P; i += gsz) {
      W.queue[i] = qorder[i];
      W.pod_state[i] = D.pod_state0[i];
      W.pod_status[i] = ST_PENDING;
      W.pod_fstate[i] = -1;
    }
    for (int64_t i = gtid; i < d.NU; i += gsz) W.last_len[i] = 0;
    for (int64_t i = gtid; i < CT_NCOUNTERS; i += gsz) W.counters[i] = 0;
  }
}

#endif  // KS_TU == 0

// ------------------------------------------------------------------------------------------------
// Solve
// ------------------------------------------------------------------------------------------------
template <bool INL> struct ClaimView;
template <> struct ClaimView<true> { LI32 tpl; LI64 req; LI64 max; LU32 rem; LI32 thr; LI32 cnt; };
template <> struct ClaimView<false> { GI32 tpl; GI64 req; GI64 max; GU32 rem; GI32 thr; GI32 cnt; };

// One queue entry per lane (the 64-pod window), read wave-uniformly with readlane.
template <int RT>
struct Window {
  int p, g, uid, s, flags, pf, st;
  int rl;  // LEAN, nothing pushed back yet: identical pods from this queue position to the end of their run
  uint64_t ll, tol0, tol1, toltpl, hpc, hpu, hpo;
  uint64_t tsel, tinv, town, trss;  // TOPO: word 0 of the pod's selecting / inverse / owned group sets, st_rss keys
  int64_t req[RT > 0 ? RT : kMaxR];
};

// RT > 0: resource count known at compile time (loops unrolled, requests in VGPRs).
// TL: the instance-type tables (Allocatable per template position, sorted Allocatable lists) are
// LDS-resident.  Compile-time, so the hot loops carry no HBM branch (a join of an LDS and an HBM
// path would wait on vmcnt, i.e. on every outstanding store).
// SIM: a consolidation simulation (helpers.go:73-127) over the shared cluster problem: pods are
// the simulation's local subset (W.pod_map), the candidates' nodes are masked out, and existing
// node state is copy-on-write (a node's HBM slot is initialised the first time a pod lands on it).
// Requirements.Add (requirements.go:118-125) of `in` into `out`, both in LDS: the rs_add of
// ks_reqset.h with each key's words spread over the lanes (headers are wave-uniform; one wave,
// so every lane's reads of a key precede lane 0's header stores).  Returns whether a key of
// `mask` changed (what rs_equal_keys against the old record would report).
// Every branch is wave-uniform (the key loop, the per-key case, the 64-word blocks); the per-lane work is
// branch-free -- a lane past the key's last word computes on a clamped index and stores nothing, `diff` is
// accumulated by select -- and every header and bound store is a wave-wide store of a uniform value (DESIGN §3:
// the AMDGPU backend of this toolchain miscompiled divergent per-lane updates in loops; round 2's out-of-line
// form of this function worked around that without removing the pattern).
__device__ __forceinline__ bool rs_add_wave(const DevLayout& L, LU32 out, LU32 in, uint64_t mask) {
  const uint64_t pi = rs_present(in), po = rs_present(out);
  uint64_t cm = rs_compl(out), hg = rs_hasgt(out), hl = rs_haslt(out);
  const uint64_t icm = rs_compl(in), ihg = rs_hasgt(in), ihl = rs_haslt(in);
  uint32_t diff = 0;
  for (uint64_t m = pi; m; m &= m - 1) {
    const int k = ctz64(m);
    const uint64_t one = 1ull << k;
    const KeyMeta km = L.keys[k];
    const bool watched = (mask & one) != 0;
    const int base = L.HDR + km.off;
    if (po & one) {
      const KeyIx x = key_ix_header(L, out, in, k);
      for (int i0 = 0; i0 < km.nw; i0 += kWave) {
        const int i = i0 + lane();
        const bool live = i < km.nw;
        const int ic = live ? i : i0;
        const uint32_t old = out[base + ic];
        const uint32_t nw = key_ix_word(L, out, in, k, ic, x);
        if (live) out[base + i] = nw;
        diff |= (live && watched && nw != old) ? 1u : 0u;
      }
      const bool keep = !x.dne && x.compl_;
      const uint64_t ncm = keep ? (cm | one) : (cm & ~one);
      const uint64_t nhg = (keep && x.hg) ? (hg | one) : (hg & ~one);
      const uint64_t nhl = (keep && x.hl) ? (hl | one) : (hl & ~one);
      diff |= (watched && (((ncm ^ cm) | (nhg ^ hg) | (nhl ^ hl)) & one) != 0) ? 1u : 0u;
      cm = ncm;
      hg = nhg;
      hl = nhl;
      if (km.bslot >= 0) {
        const int64_t ngt = keep && x.hg ? x.gt : 0, nlt = keep && x.hl ? x.lt : 0;
        diff |= (watched && (ngt != rs_gt(out, km.bslot) || nlt != rs_lt(out, km.bslot))) ? 1u : 0u;
        wsync();
        rs_set_gt(out, km.bslot, ngt);  // wave-wide store of uniform values (see commit_claim)
        rs_set_lt(out, km.bslot, nlt);
      }
    } else {  // rs_copy_key
      for (int i0 = 0; i0 < km.nw; i0 += kWave) {
        const int i = i0 + lane();
        const bool live = i < km.nw;
        const uint32_t v = in[base + (live ? i : i0)];
        if (live) out[base + i] = v;
      }
      diff |= watched ? 1u : 0u;  // the key appears
      cm = (cm & ~one) | (icm & one);
      hg = (hg & ~one) | (ihg & one);
      hl = (hl & ~one) | (ihl & one);
      if (km.bslot >= 0) {
        const int64_t g = rs_gt(in, km.bslot), l = rs_lt(in, km.bslot);
        wsync();
        rs_set_gt(out, km.bslot, g);  // wave-wide store of uniform values
        rs_set_lt(out, km.bslot, l);
      }
    }
  }
  wsync();
  wr64(out, 0, po | pi);  // wave-wide store of uniform values (see commit_claim)
  wr64(out, 2, cm);
  wr64(out, 4, hg);
  wr64(out, 6, hl);
  wsync();
  return wballot(diff != 0) != 0;
}

// Requirements.Intersects(IT, X) (requirements.go:241-258) on the keys `keys` of X, for word wc of template
// t's position bitset, from the host's per-(key, value) position tables (ks_host.cpp "feasibility tables"):
// per key, the positions whose IT lacks the key (only shared keys are checked), those holding a value X
// admits, and -- when X's operator is NotIn / DoesNotExist -- those whose IT says DoesNotExist (both
// negative).  Every lane of the wave calls it with the same X, t and keys (ballots over X's values).
// dnePass: pass the DoesNotExist positions unconditionally (k_feasibility's factorised rows: whether
// they pass depends on the operator of the whole record, which feas_masks tests per step).
template <class PX>
__device__ __forceinline__ uint32_t fk_intersects_word(const KsDev& D, const DevLayout& L, PX X, int t, int wc,
                                                       uint64_t keys, bool dnePass = false) {
  const uint32_t KS_G* F = D.fk_words;
  const KsDims& d = D.d;
  const int TW = d.TW;
  uint32_t ic = ~0u;
  for (uint64_t m = keys; m; m &= m - 1) {
    const int k = ctz64(m);
    const int base = D.fk_key_off[t * d.NK + k];
    const KeyMeta km = L.keys[k];
    uint32_t acc = F[base + wc];  // positions whose IT lacks the key
    const int op = rs_op(L, X, k);
    if (dnePass || op == OP_NOTIN || op == OP_DNE) acc |= F[base + TW + wc];
    if (!bit(rs_compl(X), k)) {  // X In: the positions holding one of its values
      for (int i = 0; i < km.nw; i++) {
        uint32_t x = X[L.HDR + km.off + i];
        while (x) {
          const int v = i * 32 + __builtin_ctz(x);
          x &= x - 1;
          acc |= F[base + (3 + v) * TW + wc];
        }
      }
    } else if (!bit(d.fkMulti, k)) {  // complement, one value per IT: In positions minus the values X excludes
      uint32_t sub = 0;
      for (int v0 = 0; v0 < km.nv; v0 += kWave) {
        uint64_t out = wballot(v0 + lane() < km.nv && !rs_member(L, X, k, v0 + lane()));
        for (; out; out &= out - 1) sub |= F[base + (3 + v0 + ctz64(out)) * TW + wc];
      }
      acc |= F[base + 2 * TW + wc] & ~sub;
    } else {  // complement over multi-valued ITs: the values X admits
      for (int v0 = 0; v0 < km.nv; v0 += kWave) {
        uint64_t in = wballot(v0 + lane() < km.nv && rs_member(L, X, k, v0 + lane()));
        for (; in; in &= in - 1) acc |= F[base + (3 + v0 + ctz64(in)) * TW + wc];
      }
    }
    ic &= acc;
  }
  return ic;
}

#if KS_TU == 0
// Requirements.Intersects(IT, X) for word wc, as fk_intersects_word, evaluated by a group of GW lanes (GW = 32:
// the two halves of the wave work on different rows, each with its own X, t and key set; the complement
// branches ballot over the group's lanes only).
template <int GW, class PX>
__device__ __forceinline__ uint32_t fk_intersects_word_g(const KsDev& D, const DevLayout& L, PX X, int t, int wc,
                                                         uint64_t keys) {
  const uint32_t KS_G* F = D.fk_words;
  const KsDims& d = D.d;
  const int TW = d.TW;
  const int sub = lane() & (GW - 1), sh = GW == 64 ? 0 : (lane() & 32);
  auto gballot = [&](bool p) -> uint64_t {
    const uint64_t b = wballot(p);
    return GW == 64 ? b : (uint64_t)(uint32_t)(b >> sh);
  };
  uint32_t ic = ~0u;
  for (uint64_t m = keys; m; m &= m - 1) {
    const int k = ctz64(m);
    const int base = D.fk_key_off[t * d.NK + k];
    const KeyMeta km = L.keys[k];
    uint32_t acc = F[base + wc] | F[base + TW + wc];  // lacks the key; DoesNotExist (passed, see feas_masks)
    if (!bit(rs_compl(X), k)) {  // X In: the positions holding one of its values
      for (int i = 0; i < km.nw; i++) {
        uint32_t x = X[L.HDR + km.off + i];
        while (x) {
          const int v = i * 32 + __builtin_ctz(x);
          x &= x - 1;
          acc |= F[base + (3 + v) * TW + wc];
        }
      }
    } else if (!bit(d.fkMulti, k)) {  // complement, one value per IT: In positions minus the values X excludes
      uint32_t sbt = 0;
      for (int v0 = 0; v0 < km.nv; v0 += GW) {
        uint64_t out = gballot(v0 + sub < km.nv && !rs_member(L, X, k, v0 + sub));
        for (; out; out &= out - 1) sbt |= F[base + (3 + v0 + ctz64(out)) * TW + wc];
      }
      acc |= F[base + 2 * TW + wc] & ~sbt;
    } else {  // complement over multi-valued ITs: the values X admits
      for (int v0 = 0; v0 < km.nv; v0 += GW) {
        uint64_t in = gballot(v0 + sub < km.nv && rs_member(L, X, k, v0 + sub));
        for (; in; in &= in - 1) acc |= F[base + (3 + v0 + ctz64(in)) * TW + wc];
      }
    }
    ic &= acc;
  }
  return ic;
}

// k_feasibility (north_star "feasibility matrix"): the static part of the pod x
// instance-type feasibility per (relaxation state, template) row, over the words of the template's position
// bitset.  Row = Tolerates(template taints) AND Intersects(IT, template) AND Intersects(IT, state) on the keys
// no instance type constrains with more than one value (nodeclaim.go:68-71,225-260; requirements.go:241-258).
// k_solve ANDs the row where it would otherwise re-evaluate those keys per step (feas_masks); it tests the
// template's taints before it reads a row (try_templates, claim_quick), so an intolerant row is all zero and
// costs no reads.  HBM-bound: reads the state's and template's records and the template's position tables,
// writes TW words per row.
// Persistent 256-lane blocks: the key table is staged once per block, and each wave walks rows with a
// grid stride.  A row of TW <= 32 words takes half a wave (two rows per wave step), so lanes are not idle
// for the narrow template lists (C3: TW = 25).
template <int GW>
__global__ __launch_bounds__(256) void k_feasibility(KsDev D) {
  const KsDims& d = D.d;
  __shared__ __attribute__((aligned(16))) uint32_t s_kraw[64 * sizeof(KeyMeta) / 4];
  for (int i = threadIdx.x; i < d.NK * (int)(sizeof(KeyMeta) / 4); i += blockDim.x) s_kraw[i] = ((const uint32_t KS_G*)D.keys)[i];
  __syncthreads();
  DevLayout L;
  L.nkeys = d.NK;
  L.W = d.W;
  L.NB = d.NB;
  L.HDR = d.HDR;
  L.RSW = d.RSW;
  L.keys = (const KeyMeta KS_L*)s_kraw;
  L.wordValid = D.wordValid;
  L.vIsInt = D.vIsInt;
  L.vInt = D.vInt;
  constexpr int RPW = 64 / GW;  // rows per wave step
  const int rows = d.S * d.NTPL;
  const int wave = (int)(threadIdx.x >> 6), half = GW == 64 ? 0 : (lane() >> 5), sub = lane() & (GW - 1);
  const uint64_t km = d.itKeys & ~d.fkMulti;
  for (int r0 = (blockIdx.x * 4 + wave) * RPW; r0 < rows; r0 += gridDim.x * 4 * RPW) {
    const int row = r0 + half;
    const bool live = row < rows;
    const int rr = live ? row : rows - 1;
    const int s = rr / d.NTPL, t = rr - s * d.NTPL;
    uint32_t KS_G* out = D.st_fm + (int64_t)rr * d.TW;
    if (!((D.st_toltpl[s] >> t) & 1ull)) {  // the state does not tolerate the template's taints
      for (int w = sub; w < d.TW; w += GW)
        if (live) out[w] = 0;
      continue;
    }
    const uint32_t KS_G* X = D.st_rs + (int64_t)s * d.RSW;
    const uint32_t KS_G* T = D.tpl_rs + (int64_t)t * d.RSW;
    const uint64_t kx = rs_present(X) & km, kt = rs_present(T) & km;
    for (int w0 = 0; w0 < d.TW; w0 += GW) {
      const int w = w0 + sub;
      const int wc = w < d.TW ? w : d.TW - 1;
      const uint32_t v = fk_intersects_word_g<GW>(D, L, X, t, wc, kx) & fk_intersects_word_g<GW>(D, L, T, t, wc, kt);
      if (live && w < d.TW) out[w] = v;
    }
  }
}
// k_feasibility_nodes (north_star "feasibility matrix", the existing-node side): per relaxation state with
// label requirements and per existing node, Taints.Tolerates AND the strict Requirements.Compatible of
// ExistingNode.Add (existingnode.go:64-124; taints.go:38-50; requirements.go:163-174) on the node's
// initial labels.  Both inputs are static for the whole Solve / pass, so k_solve's node scan reads one
// bit instead of re-running Compatible per (pod, node) step -- until a commit narrows a node's own
// requirements (existingnode.go:118), after which that node is tested exactly again.
// One thread per (row, node): a block of 256 nodes of one row; lanes evaluate their node against the same
// state record (uniform key loop), a ballot packs 64 node bits, lanes 0 and 32 store one word each.
__global__ __launch_bounds__(256) void k_feasibility_nodes(KsDev D, int nbx) {
  const KsDims& d = D.d;
  __shared__ __attribute__((aligned(16))) uint32_t s_kraw[64 * sizeof(KeyMeta) / 4];
  for (int i = threadIdx.x; i < d.NK * (int)(sizeof(KeyMeta) / 4); i += blockDim.x) s_kraw[i] = ((const uint32_t KS_G*)D.keys)[i];
  __syncthreads();
  DevLayout L;
  L.nkeys = d.NK;
  L.W = d.W;
  L.NB = d.NB;
  L.HDR = d.HDR;
  L.RSW = d.RSW;
  L.keys = (const KeyMeta KS_L*)s_kraw;
  L.wordValid = D.wordValid;
  L.vIsInt = D.vIsInt;
  L.vInt = D.vInt;
  const int row = blockIdx.x / nbx, bx = blockIdx.x - row * nbx;
  const int s = D.fn_state[row];
  const uint32_t KS_G* X = D.st_rs + (int64_t)s * d.RSW;
  const uint64_t t0 = D.st_tol[2 * s], t1 = D.st_tol[2 * s + 1];
  const int NWN = (d.N + 31) >> 5;
  const int n = bx * 256 + (int)threadIdx.x;  // a wave's 64 nodes start at a multiple of 64
  bool ok = false;
  if (n < d.N) {
    const uint64_t KS_G* tp = D.n_taint + 2 * (int64_t)n;
    ok = ((tp[0] & ~t0) | (tp[1] & ~t1)) == 0 && rs_compatible(L, D.n_rs0 + (int64_t)n * d.RSW, X, 0);
  }
  const uint64_t b = wballot(ok);
  const int w = (n - lane()) >> 5;  // this wave's first word
  uint32_t KS_G* out = D.st_fn + (int64_t)row * NWN;
  if (lane() == 0 && w < NWN) out[w] = (uint32_t)b;
  if (lane() == 32 && w + 1 < NWN) out[w + 1] = (uint32_t)(b >> 32);
}
#endif

// A topology simulation keeps its register window's node domains in LDS (Solver::s_tdw): the first kTdw nodes,
// the first kTdwKeys key slots (make_plan counts the bytes).
constexpr int kTdw = 256, kTdwKeys = 4;

template <int RT, bool TL, bool SIM, bool TOPO, bool LEAN>
struct Solver {
  static constexpr int RM = RT > 0 ? RT : kMaxR;
  // LEAN: the problem uses none of host ports, limited volumes, pod label requirements, shared UIDs,
  // negative requests or topology (KsDims::lean, set by the encoder).  Those paths compile out, which
  // frees the registers they pinned (SGPR spills) and the instructions they cost on every pop.
  static_assert(!(LEAN && TOPO), "LEAN excludes topology");
  __device__ __forceinline__ bool hpA() const { return !LEAN && d.hpAny; }
  __device__ __forceinline__ bool volA() const { return !LEAN && d.volAny; }
  __device__ __forceinline__ bool negR() const { return !LEAN && d.negReq; }
  __device__ __forceinline__ bool dupU() const { return !LEAN && d.dupUids; }
  __device__ __forceinline__ bool keys(int sflags) const { return !LEAN && (sflags & SF_HAS_KEYS); }
  // By value: a reference to a byval kernel argument forces a scratch copy of the whole struct
  // (every field access then becomes a scratch load); values scalarise into SGPRs.
  // Launch constants by reference, not by copy: the kernel arguments stay in the kernarg segment and
  // the work descriptor in constant memory, read with scalar loads where used.  (Copies of these
  // ~1 KB structs did not fit the SGPRs and lived in scratch memory: a private-memory round trip
  // on many hot-path reads.)
  const KsDev& D;
  const KsDims& d;
  const KsWork KS_C& W;
  const Plan& pl;
  DevLayout L;
  ClaimView<true> lc;   // claims [0, KL)
  ClaimView<false> gc;  // claims [KL, KO)
  LI32 s_order;         // [KO] s.newNodeClaims as claim ids
  LI32 s_okey;          // [KO] len(Pods) of the claim at each position
  LI32 s_ptpl;          // [KO] template of the claim at each position
  LI64 s_phead;         // [KO][R] max Allocatable - requests of the claim at each position
  LI64 s_talloc;        // [totalTplIts][R] Allocatable per template position (pl.talloc)
  LI64 s_tsa;           // tsort_alloc (pl.tsort)
  LI32 s_tsp;           // tsort_pos (pl.tsort)
  LI32 s_tbeg;          // [NTPL+1]
  LI64 s_pool;          // [NPOOL][R] remaining limits
  LU32 s_rs;            // [RSW] candidate requirements
  LU32 s_pin;           // [RSW] the popped pod's requirement record (its relaxation state), when it has keys
  LU32 s_rem;           // [TW+2] candidate options
  LU32 s_cand;          // [TW+2] limit-filtered template options
  LU32 s_fic;           // [TW+2] feas_masks: Intersects(IT, X) per position
  LU32 s_fof;           // [TW+2] feas_masks: hasOffering(IT, X) per position
  LU32 s_firr;          // [TW+2] feas_masks: irregular positions (exact per-position check)
  LU32 s_rmv;           // SIM: [ceil(N/32)] nodes removed by the simulation (the candidates)
  LU32 s_tch;           // SIM: [ceil(N/32)] nodes whose requests live in a W.n_req slot
  LU32 s_tchr;          // SIM: [ceil(N/32)] nodes whose requirements live in a W.n_rs slot; Solve (d.fnOn): nodes
                        // whose requirements a commit narrowed (k_feasibility_nodes's bits no longer apply)
  LU32 s_tvol;          // SIM: [ceil(N/32)] nodes whose volume counts live in a W.n_vc slot (W.n_vslot)
  LI32 s_tgm;           // [G][TGM_WORDS] topology group metadata
  LI32 s_tmin;          // [G] domainMinCount of the popped pod, per spread group
  LU32 s_trs0;          // [RSW] AddRequirements' nodeRequirements snapshot
  LU32 s_trs1;          // [RSW] one group's domains as a single-key record
  LI32 s_tdom;          // [pl.tdl] the node domain table (a Solve whose table fits)
  LI32 s_tdw;           // SIM + TOPO: the register window's node domains, [key slot < kTdwKeys][kTdw]
  LI32 s_live;          // [pl.livl] a Solve's live node list (ks_solve_body.inc)
  LI32 s_tcs;           // [pl.tcl] the count table's LDS-resident prefix: the small-key groups (a Solve: the
                        // whole table when it fits, make_plan)
  LU32 s_tcd;           // SIM: dirty bits over count words [tgSmall, tgCntWords): set once W.tg_cnt holds the word
  // Topology-group sets are GMW-word bitsets (ks_problem.h).  Word 0 lives in a register (it is the whole set
  // whenever a problem has <= 64 groups); words 1.. live in LDS, s_gw[set * GMW + w] (sets GS_*).
  LU64 s_gw;            // [GS_N][GMW] when GMW > 1
  uint64_t t_mask = 0;  // groups matching the popped pod (owned in its state | inverse groups selecting it), word 0
  uint64_t t_sel = 0;   // groups whose selector selects the popped pod, word 0
  uint64_t t_inv = 0;   // inverse groups the popped pod owns, word 0
  bool t_any = false;   // t_mask is not empty (any word)
  bool t_rec = false;   // t_sel | t_inv is not empty (any word): Topology.Record has groups to visit
  int t_s = 0;          // the popped pod's relaxation state
  uint64_t t_rss = 0;   // keys the state's strict pod requirements name (rs_present of its st_rss row)
  const uint32_t KS_G* fnp = nullptr;  // k_feasibility_nodes's row of the popped pod's state (null: none)
  bool t_nonode = false;  // some matching group admits no domain at all: no existing node can pass
  uint64_t t_active = ~0ull;  // groups in t.topologies so far (late groups join at their relaxation), word 0
  int64_t algbytes = 0;
  bool rem_same = false;  // the last claim_full left the claim's options unchanged (commit skips the copy back)
  uint64_t cur_hpc = 0, cur_hpu = 0;  // the popped pod's host-port conflict / reservation masks
  uint64_t cur_hpo = 0;               // its own initial entries on existing nodes (HostPortUsage.Add replaces them)
  // the popped pod's volumes (volA), in LDS (SGPRs are the scarce resource of the non-LEAN loop): driver
  // entries [VO_DB, VO_DE) of D.pod_vd, NewScheduler-time mounts of its PVCs [VO_SB, VO_SE) of D.pod_vs, this
  // Solve's earlier mounts of them [0, VO_NSP) of W.vspec (PF_VSHARED pods: its PVCs [VO_UB, VO_UE) of
  // D.pod_vu); VO_NLOG entries in W.vlog; SIM: VO_NSLOT W.n_vc slots in use
  enum : int { VO_DB = 0, VO_DE, VO_SB, VO_SE, VO_NSP, VO_UB, VO_UE, VO_NLOG, VO_NSLOT, VO_WORDS };
  LI32 s_vol;
#ifdef KS_PHASE_STATS
  mutable uint64_t scyc[4] = {0, 0, 0, 0};  // claim_full sub-phases: requirements, thresholds, masks, apply
#endif

  __device__ Solver(const KsDev& D_, const KsWork KS_C& W_, const Plan& p_) : D(D_), d(D_.d), W(W_), pl(p_) {}
  __device__ __forceinline__ int R() const { return RT > 0 ? RT : d.R; }

  template <bool INL>
  __device__ __forceinline__ const ClaimView<INL>& cv() const {
    if constexpr (INL) return lc;
    else return gc;
  }

  template <class P>
  __device__ __forceinline__ bool fits(const int64_t* req, P alloc) const {  // resources.go:162-175
    bool ok = true;
#pragma unroll
    for (int r = 0; r < RM; r++) {
      if (RT == 0 && r >= d.R) break;
      const int64_t a = alloc[r];
      ok &= (a >= 0) & (req[r] <= a);
    }
    return ok;
  }
  __device__ __forceinline__ bool fits_pos(const int64_t* req, int gpos) const {
    if constexpr (TL) return fits(req, s_talloc + (int64_t)gpos * R());
    else return fits(req, D.it_alloc + (int64_t)D.tpl_its[gpos] * R());
  }
  __device__ __forceinline__ int64_t alloc_pos(int gpos, int r) const {
    if constexpr (TL) return s_talloc[(int64_t)gpos * R() + r];
    else return D.it_alloc[(int64_t)D.tpl_its[gpos] * R() + r];
  }
  __device__ __forceinline__ int64_t tsort_a(int64_t i) const {
    if constexpr (TL) return s_tsa[i];
    else return D.tsort_alloc[i];
  }
  __device__ __forceinline__ int tsort_p(int64_t i) const {
    if constexpr (TL) return s_tsp[i];
    else return D.tsort_pos[i];
  }

  // Commit log (scheduler.go:253/274 placements in order): lane (i & 63) holds entry i until 64 are
  // buffered, then one coalesced store.  Per-pod global stores would make the next global load wait
  // for their write acknowledgements (vmcnt counts stores on gfx9).
  int lg_p = 0, lg_t = 0;
  // (A simulation's placements are never read back -- the host reads its record -- so SIM only counts them.)
  __device__ __forceinline__ void log_commit(int p, int tgt, int& nlog) {
    if constexpr (SIM) {
      nlog++;
      return;
    }
    if (lane() == (nlog & (kWave - 1))) {
      lg_p = p;
      lg_t = tgt;
    }
    nlog++;
    if ((nlog & (kWave - 1)) == 0) {
      W.log_pod[nlog - kWave + lane()] = lg_p;
      W.log_tgt[nlog - kWave + lane()] = lg_t;
    }
  }
  // Commit-log entries for `n` (<= 64) placements at once: lane t holds entry nlog + t (pod, target).
  __device__ __forceinline__ void log_batch(int n, int pod_t, int tgt_t, int& nlog) {
    if constexpr (SIM) {
      nlog += n;
      return;
    }
    const int b0 = nlog & (kWave - 1);
    const int src = (lane() - b0) & (kWave - 1);  // the entry this lane buffers: nlog + src
    const int pv = __shfl(pod_t, src), tv = __shfl(tgt_t, src);
    const bool mine = src < n;
    if (mine && lane() >= b0) {
      lg_p = pv;
      lg_t = tv;
    }
    if (b0 + n >= kWave) {  // the buffered block is complete: store it, then buffer the wrapped entries
      W.log_pod[nlog - b0 + lane()] = lg_p;
      W.log_tgt[nlog - b0 + lane()] = lg_t;
      if (mine && lane() < b0) {
        lg_p = pv;
        lg_t = tv;
      }
    }
    nlog += n;
  }
  __device__ __forceinline__ void log_flush(int nlog) {
    if constexpr (SIM) return;
    const int k = nlog & (kWave - 1);
    if (lane() < k) {
      W.log_pod[nlog - k + lane()] = lg_p;
      W.log_tgt[nlog - k + lane()] = lg_t;
    }
  }
  template <class PR>
  __device__ __forceinline__ bool has_offering(int it, PR rs) const {  // nodeclaim.go:270-278
    const int b = D.it_off_beg[it], e = D.it_off_beg[it + 1];
    for (int o = b; o < e; o++)
      if (rs_member(L, rs, d.zoneKey, D.off_zone[o]) && rs_member(L, rs, d.ctKey, D.off_ct[o])) return true;
    return false;
  }
  // filterInstanceTypesByRequirements' requirement and offering tests (nodeclaim.go:225-278) for every
  // position of template t at once, from the host's per-(key, value) position bitsets (ks_host.cpp
  // "feasibility tables"): for each key of X that instance types constrain, Requirements.Intersects
  // passes on the positions whose IT lacks the key (only shared keys are checked), on those holding a
  // value X admits, and -- when X's operator is NotIn / DoesNotExist -- on those whose IT says
  // DoesNotExist (both negative, requirements.go:248-252); the keys intersect.  hasOffering is the union
  // over the (zone, capacity-type) pairs X admits (a missing key admits all).  Lane w owns word w:
  // s_fic, s_fof; s_firr marks positions whose IT holds a complement requirement (checked exactly).
  // fmrow: k_feasibility's row for (the popped pod's state, t) -- the keys no instance type constrains
  // with more than one value, already intersected for the template and the state -- when X is the
  // template's or a claim's requirements plus that state's (Compatible with it) and nothing else: per
  // such key the test factorises for the value positions (an IT's single value is admitted by X = A + B
  // iff by A and by B), and the claim's options already satisfy A's part.  An IT's DoesNotExist does not
  // factorise (Exists + NotIn is NotIn, which it intersects, requirements.go:248-252): the row passes
  // those positions and they are tested here against X's operator.  Only the multi-valued keys are
  // evaluated in full then.
  __device__ __forceinline__ void feas_masks(LU32 X, int t, const uint32_t KS_G* fmrow = nullptr) {
    const uint32_t KS_G* F = D.fk_words;
    const int TW = d.TW;
    const int ball = D.fk_tpl[3 * t], birr = D.fk_tpl[3 * t + 1], boff = D.fk_tpl[3 * t + 2];
    const uint64_t keysX = rs_present(X) & d.itKeys & (fmrow ? d.fkMulti : ~0ull);
    uint64_t keysDne = 0;  // fmrow: X's single-valued IT keys whose operator is In / Exists
    if (fmrow)
      for (uint64_t m = rs_present(X) & d.itKeys & ~d.fkMulti; m; m &= m - 1) {
        const int op = rs_op(L, X, ctz64(m));
        if (op != OP_NOTIN && op != OP_DNE) keysDne |= m & (~m + 1);
      }
    const int nz = L.keys[d.zoneKey].nv, nc = L.keys[d.ctKey].nv;
    for (int w0 = 0; w0 < TW; w0 += kWave) {
      const int w = w0 + lane();
      const int wc = w < TW ? w : TW - 1;
      uint32_t ic = F[ball + wc] & fk_intersects_word(D, L, X, t, wc, keysX);
      if (fmrow) {
        ic &= fmrow[wc];
        // the row passes DoesNotExist positions; they intersect X iff X's operator is negative there
        for (uint64_t m = keysDne; m; m &= m - 1) ic &= ~F[D.fk_key_off[t * d.NK + ctz64(m)] + TW + wc];
      }
      uint32_t of = 0;
      for (int c0 = 0; c0 < nc; c0 += kWave) {
        const uint64_t cm0 = wballot(c0 + lane() < nc && rs_member(L, X, d.ctKey, c0 + lane()));
        if (!cm0) continue;
        for (int z0 = 0; z0 < nz; z0 += kWave) {
          for (uint64_t zm = wballot(z0 + lane() < nz && rs_member(L, X, d.zoneKey, z0 + lane())); zm; zm &= zm - 1) {
            const int z = z0 + ctz64(zm);
            for (uint64_t cm = cm0; cm; cm &= cm - 1) of |= F[boff + (z * nc + c0 + ctz64(cm)) * TW + wc];
          }
        }
      }
      const uint32_t irr = F[birr + wc];
      if (w < TW) {
        s_fic[w] = ic;
        s_fof[w] = of;
        s_firr[w] = irr;
      }
    }
    wsync();
  }
  // k_feasibility's row for (state s, template t), or null where it does not apply: not computed, or
  // topology requirements were added to the record (they are not part of the row).
  __device__ __forceinline__ const uint32_t KS_G* fm_row(int s, int t) const {
    if (KS_FM_OFF || !d.fmOn || (TOPO && t_any)) return nullptr;
    return D.st_fm + ((int64_t)s * d.NTPL + t) * d.TW;
  }
  __device__ __forceinline__ bool fbit(LU32 m, int pos) const { return (m[pos >> 5] >> (pos & 31)) & 1u; }

  template <class PD, class PS>
  __device__ __forceinline__ void copy_words(PD dst, PS src, int n) const {
    for (int i = lane(); i < n; i += kWave) dst[i] = src[i];
  }
  __device__ __forceinline__ void store_bits(LU32 dst, int base, uint64_t m) const {
    if (lane() == 0) {
      dst[base >> 5] = (uint32_t)m;
      if ((base >> 5) + 1 < d.TW) dst[(base >> 5) + 1] = (uint32_t)(m >> 32);
    }
  }
  __device__ __forceinline__ int popc_words(LU32 w, int n) const {
    int c = 0;
    for (int i = lane(); i < n; i += kWave) c += __popc(w[i]);
    return wred_add(c);
  }


  // --- existing nodes (ExistingNode.Add, existingnode.go:64-124) -------------------------------
  // Volumes (VolumeUsage, volumeusage.go:183-227; KsDev in ks_problem.h).  vol_pop loads the popped pod's
  // entries (wave-uniform); for a pod sharing a PVC with other pods being scheduled it also collects the
  // earlier placements' log entries of its PVCs (W.vlog -> W.vspec; every store here is a wave-wide store of
  // a uniform value, so each lane later reads what it wrote itself).
  __device__ __forceinline__ int vo(int f) const { return uni(s_vol[f]); }
  __device__ __forceinline__ void vo_set(int f, int v) const { s_vol[f] = v; }  // wave-wide store of a uniform value
  __device__ __forceinline__ void vol_pop(int g, int pf) {
    vo_set(VO_DB, D.pod_vdbeg[g]);
    vo_set(VO_DE, D.pod_vdbeg[g + 1]);
    vo_set(VO_SB, D.pod_vsbeg[g]);
    vo_set(VO_SE, D.pod_vsbeg[g + 1]);
    int ub = 0, ue = 0, nsp = 0;
    if (pf & PF_VSHARED) {
      ub = uni(D.pod_vubeg[g]);
      ue = uni(D.pod_vubeg[g + 1]);
      const int nlog = vo(VO_NLOG);
      for (int i0 = 0; i0 < nlog; i0 += kWave) {
        const int i = i0 + lane();
        const int ic = i < nlog ? i : i0;
        const int lu = W.vlog[2 * ic], ln = W.vlog[2 * ic + 1];
        bool hit = false;
        for (int k = ub; k < ue; k++) hit |= D.pod_vu[k] == lu;
        for (uint64_t m = wballot(hit && i < nlog); m; m &= m - 1) {
          const int l = ctz64(m);
          W.vspec[2 * nsp] = rdl(lu, l);  // wave-wide stores of uniform values
          W.vspec[2 * nsp + 1] = rdl(ln, l);
          nsp++;
        }
      }
    }
    vo_set(VO_UB, ub);
    vo_set(VO_UE, ue);
    vo_set(VO_NSP, nsp);
    wsync();
  }
  __device__ __forceinline__ bool vol_any() const { return vo(VO_DE) > vo(VO_DB); }
  // The pod's PVCs of driver v that node n mounts already (at NewScheduler time, or by an earlier placement).
  __device__ __forceinline__ int vol_mounted(int n, int v) const {
    int c = 0;
    for (int k = vo(VO_SB), e = vo(VO_SE); k < e; k++) c += (D.pod_vs[2 * k] == n && D.vol_udrv[D.pod_vs[2 * k + 1]] == v) ? 1 : 0;
    for (int k = 0, e = vo(VO_NSP); k < e; k++) c += (W.vspec[2 * k + 1] == n && D.vol_udrv[W.vspec[2 * k]] == v) ? 1 : 0;
    return c;
  }
  __device__ __forceinline__ const int32_t KS_G* vol_row(int n) const {
    if (!SIM) return W.n_vc + (int64_t)n * d.VD;
    return tbit(s_tvol, n) ? W.n_vc + (int64_t)W.n_vslot[n] * d.VD : D.n_vc0 + (int64_t)n * d.VD;
  }
  // VolumeUsage.ExceedsLimits (volumeusage.go:202-209) of the popped pod on node n (per lane): per limited
  // driver it mounts, the node's count plus its PVCs the node does not mount yet.
  __device__ __forceinline__ bool vol_ok(int n) const {
    const int32_t KS_G* vc = vol_row(n);
    bool ok = true;
    for (int j = vo(VO_DB), e = vo(VO_DE); j < e; j++) {
      const int v = D.pod_vd[2 * j], c = D.pod_vd[2 * j + 1];
      ok &= vc[v] + c - vol_mounted(n, v) <= D.n_vlim[(int64_t)n * d.VD + v];
    }
    return ok;
  }
  // VolumeUsage.Add (existingnode.go:122) of the popped pod on node n (wave-uniform n; wave-wide stores of
  // uniform values).  SIM: the node's counts move to a W.n_vc slot at its first such placement.
  __device__ __forceinline__ void vol_commit(int n) {
    int32_t KS_G* vc;
    if (SIM) {
      if (!tbit(s_tvol, n)) {
        const int slot = vo(VO_NSLOT);
        for (int v = 0; v < d.VD; v++) W.n_vc[(int64_t)slot * d.VD + v] = D.n_vc0[(int64_t)n * d.VD + v];
        W.n_vslot[n] = slot;
        vo_set(VO_NSLOT, slot + 1);
        __hip_atomic_fetch_or(s_tvol + (n >> 5), 1u << (n & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        wsync();
        vc = W.n_vc + (int64_t)slot * d.VD;
      } else {
        vc = W.n_vc + (int64_t)uni(W.n_vslot[n]) * d.VD;
      }
    } else {
      vc = W.n_vc + (int64_t)n * d.VD;
    }
    for (int j = vo(VO_DB), e = vo(VO_DE); j < e; j++) {
      const int v = D.pod_vd[2 * j], c = D.pod_vd[2 * j + 1];
      const int add = uni(c - vol_mounted(n, v));
      if (add) vc[v] = uni(vc[v]) + add;
    }
    // the shared pod's PVCs not yet on n join the log (each (PVC, node) pair once)
    int nlog = vo(VO_NLOG);
    for (int k = vo(VO_UB), e = vo(VO_UE); k < e; k++) {
      const int u = D.pod_vu[k];
      bool on = false;
      for (int q = vo(VO_SB), qe = vo(VO_SE); q < qe; q++) on |= D.pod_vs[2 * q] == n && D.pod_vs[2 * q + 1] == u;
      for (int q = 0, qe = vo(VO_NSP); q < qe; q++) on |= W.vspec[2 * q + 1] == n && W.vspec[2 * q] == u;
      if (!ub(on)) {
        W.vlog[2 * nlog] = u;
        W.vlog[2 * nlog + 1] = n;
        nlog++;
      }
    }
    vo_set(VO_NLOG, nlog);
    hbm_release();
    wsync();
  }
  // Lane (n & 63) is the only lane that ever reads or writes node n's mutable state.
  __device__ __forceinline__ bool tbit(LU32 m, int n) const { return (m[n >> 5] >> (n & 31)) & 1u; }
  // Existing-node check for KN nodes per lane (positions n, n + 64, ... of the first-fit order): every
  // load of all of them is issued before any test, so a (KN * 64)-node step of the scan costs one memory
  // round trip (two with topology: the nodes' domains, then their counts).  Out-of-range positions are
  // clamped for the loads and masked.  nf: NodeFlag bits.  sl[i]: the node passed every check but lacks
  // the label of a matching group's key, so only the wave-cooperative node_slow can decide it (ok is
  // false then).
  // LIST: lane l of block i tests node nl[i] (the Solve's live list; -1: none) instead of n0 + 64 i + l; stay[i]:
  // the node still passes Fits for these requests once the pod is committed to it (the list keeps it).
  template <int KN, bool LIST = false>
  __device__ __forceinline__ void node_okK(int n0, int sflags, const int64_t* pod, uint64_t tol0, uint64_t tol1,
                                           bool* ok, int* nf, int64_t (*q)[RM], bool* sl, bool* rk,
                                           const int* nl = nullptr, bool* stay = nullptr) const {
    int c[KN];
    uint64_t tx[KN], ty[KN], h[KN];
    int64_t a[KN][RM];
    PH_BEGIN(tok);
#pragma unroll
    for (int i = 0; i < KN; i++) {
      const int n = LIST ? nl[i] : n0 + i * kWave;
      c[i] = LIST ? (n >= 0 ? n : 0) : n < d.N ? n : d.N - 1;
      const bool own = !SIM || tbit(s_tch, c[i]);
      const uint64_t KS_G* tp = D.n_taint + 2 * c[i];
      const int64_t KS_G* ap = D.n_avail + (int64_t)c[i] * R();
      const int64_t KS_G* qp = (own ? W.n_req : D.n_req0) + (int64_t)c[i] * R();
      tx[i] = tp[0];
      ty[i] = tp[1];
#pragma unroll
      for (int r = 0; r < RM; r++) {
        if (RT == 0 && r >= d.R) break;
        a[i][r] = ap[r];
        q[i][r] = qp[r];
      }
      nf[i] = SIM ? D.n_flags[c[i]] : 0;
      h[i] = 0;
      if (hpA()) h[i] = own ? W.n_hp[c[i]] : D.n_hp0[c[i]];  // HostPortUsage.Conflicts (hostportusage.go:74-85)
    }
#pragma unroll
    for (int i = 0; i < KN; i++) {
      bool rr = LIST ? nl[i] >= 0 : n0 + i * kWave < d.N;
      if (SIM) rr &= !tbit(s_rmv, c[i]);  // the simulation removed these candidates
      bool st = true;
#pragma unroll
      for (int r = 0; r < RM; r++) {  // Fits(requests + pod, Available())
        if (RT == 0 && r >= d.R) break;
        rr &= (a[i][r] >= 0) & (q[i][r] + pod[r] <= a[i][r]);
        if (LIST) st &= q[i][r] + 2 * pod[r] <= a[i][r];
      }
      if (LIST) stay[i] = st;
      rk[i] = rr;  // (permanent for these requests: the caller's resource-failing prefix)
      ok[i] = rr & (((tx[i] & ~tol0) | (ty[i] & ~tol1)) == 0) & ((h[i] & cur_hpc) == 0);  // Taints.Tolerates
      if (volA() && vol_any() && ok[i]) ok[i] = vol_ok(c[i]);
      if (keys(sflags) && ok[i]) ok[i] = node_compat(c[i]);  // strict Compatible
      sl[i] = false;
    }
    PH_BEGIN(ttp);
    if (TOPO && t_any) topo_node_stateK<KN>(c, ok, sl);  // topology (existingnode.go:106-114)
    if (LIST) PHS_END(ttp, 1);  // stats build: its topology tests
  }
  __device__ __forceinline__ const uint32_t KS_G* node_rs(int n) const {
    if (!SIM) return W.n_rs + (int64_t)n * d.RSW;
    return tbit(s_tchr, n) ? W.n_rs + (int64_t)W.n_slot[n] * d.RSW : D.n_rs0 + (int64_t)n * d.RSW;
  }
  // ExistingNode.Add's strict Compatible(node requirements, pod requirements) (existingnode.go:97-104) for
  // node n: k_feasibility_nodes's bit while the node keeps its initial record (that bit also ANDs the
  // taint test the caller already applied), else the exact test on the node's current record.
  __device__ __forceinline__ bool node_compat(int n) const {
    if (fnp && !tbit(s_tchr, n)) return (fnp[n >> 5] >> (n & 31)) & 1u;
    return rs_compatible(L, node_rs(n), s_pin, 0);
  }
  // Solve (d.fnOn): node j's requirements were narrowed by a commit; its row bit no longer applies.
  __device__ __forceinline__ void node_rs_changed(int j) const {
    if (!SIM && d.fnOn)
      __hip_atomic_fetch_or(s_tchr + (j >> 5), 1u << (j & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  // Solve: commit of a pod to node j by its owner lane.
  __device__ __forceinline__ void node_commit(int j, int s, int sflags, const int64_t* pod) {
    for (int r = 0; r < R(); r++) W.n_req[(int64_t)j * R() + r] += pod[r];
    if (hpA()) W.n_hp[j] = (W.n_hp[j] & ~cur_hpo) | cur_hpu;  // HostPortUsage.Add (hostportusage.go:70-72)
    if (keys(sflags)) {
      rs_add(L, W.n_rs + (int64_t)j * d.RSW, s_pin);
      node_rs_changed(j);
    }
  }
  // SIM: copy-on-write commit (wave-uniform).  W.n_req is indexed by node but only the nodes a pod
  // landed on are ever written (s_tch marks them), so a fresh simulation needs no initialisation.
  // Requirements are copied only when a pod with label requirements lands, into the next compact
  // slot of W.n_rs (wave-cooperatively, through LDS).
  // `q`: the owner lane's requests of node j as node_okK loaded them (no reload before the store).
  // regReq: node j sits in the register window (its requests are updated there, not in HBM).
  __device__ __forceinline__ void sim_node_commit(int j, int s, int sflags, const int64_t* pod, const int64_t* q,
                                                  int& nrs, bool regReq) {
    const int owner = j & (kWave - 1);
    const bool fresh = !tbit(s_tch, j);
    wsync();
    if (!regReq && lane() == owner) {
#pragma unroll
      for (int r = 0; r < RM; r++) {
        if (RT == 0 && r >= d.R) break;
        W.n_req[(int64_t)j * R() + r] = q[r] + pod[r];
      }
      if (hpA()) W.n_hp[j] = ((fresh ? D.n_hp0[j] : W.n_hp[j]) & ~cur_hpo) | cur_hpu;
      if (fresh) s_tch[j >> 5] |= 1u << (j & 31);
    }
    if (keys(sflags)) {
      const bool rsfresh = !tbit(s_tchr, j);
      int slot;
      if (rsfresh) {
        slot = nrs++;
        copy_words(s_rs, D.n_rs0 + (int64_t)j * d.RSW, d.RSW);
      } else {
        int v = 0;
        if (lane() == owner) v = W.n_slot[j];
        slot = rdl(v, owner);
        copy_words(s_rs, W.n_rs + (int64_t)slot * d.RSW, d.RSW);
      }
      wsync();
      rs_add_wave(L, s_rs, s_pin, 0);
      copy_words(W.n_rs + (int64_t)slot * d.RSW, s_rs, d.RSW);
      if (lane() == owner && rsfresh) W.n_slot[j] = slot;
      if (lane() == 0) s_tchr[j >> 5] |= 1u << (j & 31);
      hbm_release();
    }
    wsync();
  }

  // --- Topology (topology.go, topologygroup.go) ------------------------------------------------
  // Counts and registered bits are written by one lane and read by others: loads bypass the L1.
  __device__ __forceinline__ int tg(int g, int f) const { return s_tgm[g * TGM_WORDS + f]; }
  // count of domain v, -1 while the domain is not registered (absent from TopologyGroup.domains)
  // Small-key groups read LDS.  The hostname groups (one word per node) live in HBM: a Solve's workspace
  // holds a full copy (k_init); a simulation reads the shared NewTopology counts until it first writes a
  // word (copy-on-write, s_tcd), so no simulation copies the table.
  __device__ __forceinline__ int tcnt_at(int off) const {
    if (off < pl.tcl) return s_tcs[off];
    if constexpr (SIM) {
      const int b = off - d.tgSmall;
      const int own = ld_sc1(W.tg_cnt + off), shared = D.tg_cnt0[off];
      return ((s_tcd[b >> 5] >> (b & 31)) & 1u) ? own : shared;
    }
    return ld_sc1(W.tg_cnt + off);
  }
  __device__ __forceinline__ int tcnt(int g, int v) const { return tcnt_at(tg(g, TGM_CNT) + v); }
  // node n's domain of group g's key (-1: the node lacks the label): LDS in a Solve whose table fits, and for
  // a topology simulation's register-window nodes (the first kTdw nodes: every scan starts there)
  __device__ __forceinline__ int tdom(int g, int n) const {
    if constexpr (SIM && TOPO)
      if (n < kTdw && tg(g, TGM_KSLOT) < kTdwKeys) return s_tdw[tg(g, TGM_KSLOT) * kTdw + n];
    const int off = tg(g, TGM_KSLOT) * d.N + n;
    return off < pl.tdl ? s_tdom[off] : D.n_tdom[off];
  }
  // Topology.Record's count increment of word `off` (recording registers the domain), by one lane;
  // concurrent callers touch distinct words.
  __device__ __forceinline__ void tcnt_inc(int off) const {
    const int c = tcnt_at(off);
    const int n = c < 0 ? 1 : c + 1;
    if (off < pl.tcl) {
      s_tcs[off] = n;
      return;
    }
    W.tg_cnt[off] = n;
    if constexpr (SIM) {
      const int b = off - d.tgSmall;
      __hip_atomic_fetch_or(s_tcd + (b >> 5), 1u << (b & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
  }
  __device__ __forceinline__ int tccnt(int g, int claim) const { return ld_sc1(W.tg_ccnt + (int64_t)g * W.ccs + claim); }  // claim <= Kcap (a fresh claim at the cap)
  // podDomains.Has (strict pod requirements).  A key the pod's strict requirements do not name admits every value
  // (Get() of a missing key is Exists), which is the common case: the row's presence mask (t_rss, read with the
  // pop's other group words) answers it without a load.
  __device__ __forceinline__ bool tpod_has(int g, int v) const {
    const int k = tg(g, TGM_KEY);
    if (!((t_rss >> k) & 1ull)) return true;
    return rs_member(L, D.st_rss + (int64_t)t_s * d.RSW, k, v);
  }
  // Per pop: the matching groups (getMatchingTopologies, topology.go:366-379: owned groups, then
  // inverse groups whose selector selects the pod), domainMinCount per spread group (:192-213) and,
  // per affinity group, whether some domain the pod allows already holds a selected pod (:215-221;
  // for hostname keys that includes NodeClaim placeholders, counted in tg_cpos).
  // Word w of the set {0, ..., n-1}.
  __device__ __forceinline__ static uint64_t bits_below(int n, int w) {
    const int k = n - 64 * w;
    return k >= 64 ? ~0ull : k <= 0 ? 0ull : ((1ull << k) - 1ull);
  }
  // Word w of group set `set` (GS_*); r0: the set's register word 0.
  __device__ __forceinline__ uint64_t gword(int set, int w, uint64_t r0) const {
    return w == 0 ? r0 : (uint64_t)uni64((int64_t)s_gw[set * d.GMW + w]);
  }
  __device__ __forceinline__ bool sel_has(int g) const {  // the popped pod is selected by group g
    return ((gword(GS_SEL, g >> 6, t_sel) >> (g & 63)) & 1ull) != 0;
  }
  // sel0 / inv0 / own0 / rss0: word 0 of the pod's group sets and its strict keys, gathered with the queue
  // window (refill), so a pop's group evaluation starts without a memory round trip
  __device__ __forceinline__ void topo_pop(int s, int gpod, uint64_t sel0, uint64_t inv0, uint64_t own0, uint64_t rss0) {
    t_s = s;
    const int GMW = d.GMW;
    const uint64_t KS_G* sel = D.pod_gsel + (int64_t)gpod * GMW;
    const uint64_t KS_G* inv = D.pod_ginv + (int64_t)gpod * GMW;
    const uint64_t KS_G* own = D.st_gown + (int64_t)s * GMW;
    t_sel = sel0;
    t_inv = inv0;
    t_rss = rss0;
    t_mask = own0 | (t_sel & bits_below(d.G, 0) & ~bits_below(d.G1, 0));
    if (SIM) t_mask &= ~W.tdead[0];
    bool anyM = t_mask != 0, anyR = (t_sel | t_inv) != 0;
    if (GMW > 1) {  // words 1.. (more than 64 groups), one lane each, into LDS
      bool m = false, r = false;
      for (int w = 1 + lane(); w < GMW; w += kWave) {
        const uint64_t sw = sel[w], iw = inv[w];
        uint64_t mw = own[w] | (sw & bits_below(d.G, w) & ~bits_below(d.G1, w));
        if (SIM) mw &= ~W.tdead[w];
        s_gw[GS_SEL * GMW + w] = sw;
        s_gw[GS_INV * GMW + w] = iw;
        s_gw[GS_MASK * GMW + w] = mw;
        m = m || mw != 0;
        r = r || (sw | iw) != 0;
      }
      anyM = anyM || wballot(m) != 0;
      anyR = anyR || wballot(r) != 0;
      wsync();
    }
    t_any = anyM;
    t_rec = anyR;
    t_nonode = false;
    for (int w = 0; w < GMW; w++)
      for (uint64_t m = gword(GS_MASK, w, t_mask); m; m &= m - 1) {
        const int g = 64 * w + ctz64(m);
        if (tg(g, TGM_TYPE) == TG_AFFINITY) {
          const int nv = tg(g, TGM_NV);
          bool pos = false, reg = false;
          for (int v = lane(); v < nv && !pos; v += kWave) {
            const int c = tcnt(g, v);
            const bool has = c >= 0 && tpod_has(g, v);
            pos = has && c > 0;
            reg = reg || has;
          }
          if (lane() == 0 && tg(g, TGM_HOST) && tpod_has(g, nv) && ld_sc1(W.tg_cpos + g) > 0) pos = true;
          const bool any = wballot(pos) != 0;
          s_tmin[g] = any ? 1 : 0;  // wave-wide store of a uniform value
          // topo_node_ok's test for this group over every domain: with a selected pod somewhere the
          // node's domain must hold one; otherwise only a self-selecting pod passes (a registered domain)
          if (!tg(g, TGM_HOST) && !any && !(sel_has(g) && wballot(reg))) t_nonode = true;
          continue;
        }
        if (tg(g, TGM_TYPE) == TG_ANTI) {  // topo_node_ok: the node's domain must hold no selected pod
          if (!tg(g, TGM_HOST)) {
            const int nv = tg(g, TGM_NV);
            bool ok = false;
            for (int v = lane(); v < nv && !ok; v += kWave) ok = tcnt(g, v) == 0 && tpod_has(g, v);
            if (!wballot(ok)) t_nonode = true;
          }
          continue;
        }
        if (tg(g, TGM_TYPE) != TG_SPREAD) continue;
        int mn = 0x7fffffff, num = 0;
        if (!tg(g, TGM_HOST)) {  // hostname groups always have a min of 0
          const int nv = tg(g, TGM_NV);
          int lo = 0x7fffffff;  // smallest registered count (any domain): topo_node_ok's best case
          for (int v = lane(); v < nv; v += kWave) {
            const int c = tcnt(g, v);
            if (c >= 0) lo = c < lo ? c : lo;
            if (c >= 0 && tpod_has(g, v)) {
              num++;
              mn = c < mn ? c : mn;
            }
          }
          mn = wred_min(mn, 0x7fffffff);
          lo = wred_min(lo, 0x7fffffff);
          num = wred_add(num);
          if (tg(g, TGM_MIND) >= 0 && num < tg(g, TGM_MIND)) mn = 0;
          const int self = sel_has(g) ? 1 : 0;
          if (lo == 0x7fffffff || (int64_t)lo + self - mn > tg(g, TGM_SKEW)) t_nonode = true;
        } else {
          mn = 0;
        }
        s_tmin[g] = mn;  // wave-wide store of a uniform value (mn is reduced over the wave)
      }
    wsync();
  }
  // ExistingNode.Add's topology step for node n (one lane each): a node's single domain of each matching group
  // must be the one TopologyGroup.Get returns (existingnode.go:106-114).  0 fails, 1 passes, 2: every labelled
  // group passes, but the node lacks the label of some group's key (its domain then comes from the
  // requirements it accumulated; node_slow decides).  The node scan's default, topo_node_stateK, applies these
  // tests group by group to a lane's KN nodes (their loads issued together); KS_TOPO_SEQ calls this per node.
  __device__ __forceinline__ int topo_node_state1(int n) const {
    int st = 1;
    for (int w = 0; w < d.GMW; w++)
      for (uint64_t m = gword(GS_MASK, w, t_mask); m; m &= m - 1) {
        const int g = 64 * w + ctz64(m);
        const int v = tdom(g, n);
        if (v < 0) {
          st = 2;
          continue;
        }
        const int c = tcnt(g, v);
        if (c < 0) return 0;  // unregistered: Get never returns it
        const int type = tg(g, TGM_TYPE);
        if (type == TG_SPREAD) {
          const int self = sel_has(g) ? 1 : 0;
          if ((int64_t)c + self - s_tmin[g] > tg(g, TGM_SKEW)) return 0;
        } else if (type == TG_AFFINITY) {  // a selected pod's domain, or the bootstrap for a self-selecting pod
          if (!tpod_has(g, v)) return 0;
          if (s_tmin[g] ? c == 0 : !sel_has(g)) return 0;
        } else if (c != 0 || !tpod_has(g, v)) {
          return 0;
        }
      }
    return st;
  }
  // KN nodes per lane, group by group: the KN domain and count loads of one group are issued together
  // (topo_node_state1's tests, state updated branch-free; KS_TOPO_SEQ: one node after the other).
  template <int KN>
  __device__ __forceinline__ void topo_node_stateK(const int* c, bool* ok, bool* sl) const {
#ifdef KS_TOPO_SEQ
#pragma unroll
    for (int i = 0; i < KN; i++) {
      const int st = ok[i] ? topo_node_state1(c[i]) : 0;
      ok[i] = st == 1;
      sl[i] = st == 2;
    }
#else
    int st[KN];
#pragma unroll
    for (int i = 0; i < KN; i++) st[i] = ok[i] ? 1 : 0;
    for (int w = 0; w < d.GMW; w++)
      for (uint64_t m = gword(GS_MASK, w, t_mask); m; m &= m - 1) {
        const int g = 64 * w + ctz64(m);
        int v[KN], cn[KN];
#pragma unroll
        for (int i = 0; i < KN; i++) v[i] = st[i] ? tdom(g, c[i]) : -1;
#pragma unroll
        for (int i = 0; i < KN; i++) cn[i] = v[i] >= 0 ? tcnt(g, v[i]) : 0;
        const int type = tg(g, TGM_TYPE), self = sel_has(g) ? 1 : 0, skew = tg(g, TGM_SKEW), mn = s_tmin[g];
#pragma unroll
        for (int i = 0; i < KN; i++) {
          const int vv = v[i] < 0 ? 0 : v[i];  // (v < 0 decides below; no out-of-range member test)
          bool pass;
          if (type == TG_SPREAD) pass = (int64_t)cn[i] + self - mn <= skew;
          else if (type == TG_AFFINITY) pass = tpod_has(g, vv) && (mn ? cn[i] != 0 : self != 0);
          else pass = cn[i] == 0 && tpod_has(g, vv);
          pass = pass && cn[i] >= 0;  // unregistered: Get never returns it
          const int nx = v[i] < 0 ? 2 : pass ? st[i] : 0;
          st[i] = st[i] == 0 ? 0 : nx;
        }
      }
#pragma unroll
    for (int i = 0; i < KN; i++) {
      ok[i] = st[i] == 1;
      sl[i] = st[i] == 2;
    }
#endif
  }
  // ExistingNode.Add's requirement and topology steps for node j, wave-wide, for a node lacking the
  // label of a matching group's key (existingnode.go:91-115): nodeRequirements = the node's requirements
  // + the pod's, then AddRequirements picks the domains over nodeRequirements.Get(key) exactly as for a
  // NodeClaim (a missing key reads as Exists, a pod's NotIn leaves the complement), and the strict
  // Compatible decides.  The other checks already passed.  On success s_rs holds the node's new
  // requirements (the pod's and the topology's added).
  __device__ __forceinline__ bool node_slow(int j, int s, int sflags) {
    wsync();
    copy_words(s_rs, node_rs(j), d.RSW);
    wsync();
    if (keys(sflags)) rs_add_wave(L, s_rs, s_pin, 0);
    return topo_apply(s_rs, -1, 0) == 0;
  }
  // The node's requirements after a node_slow commit (n.requirements = nodeRequirements): s_rs.
  // SIM: into the node's copy-on-write slot.
  __device__ __forceinline__ void node_store_rs(int j, int& nrs) {
    wsync();
    if (!SIM) {
      copy_words(W.n_rs + (int64_t)j * d.RSW, s_rs, d.RSW);
      if (lane() == 0) node_rs_changed(j);
    } else {
      const int owner = j & (kWave - 1);
      const bool rsfresh = !tbit(s_tchr, j);
      int slot;
      if (rsfresh) {
        slot = nrs++;
      } else {
        int v = 0;
        if (lane() == owner) v = W.n_slot[j];
        slot = rdl(v, owner);
      }
      copy_words(W.n_rs + (int64_t)slot * d.RSW, s_rs, d.RSW);
      if (lane() == owner && rsfresh) W.n_slot[j] = slot;
      if (lane() == 0) s_tchr[j >> 5] |= 1u << (j & 31);
    }
    hbm_release();
    wsync();
  }
  // Topology.AddRequirements + Compatible on a NodeClaim's candidate record `rs` (LDS), wave-wide.
  // Returns 0, FC_TOPO | group << 16, or FC_TOPO_COMPAT; on success rs holds the final requirements.
  // claim < 0: an existing node's record (node_slow; no hostname placeholder); allow: the final
  // Compatible's AllowUndefined keys (NodeClaim: well-known labels, nodeclaim.go:96; node: none).
  __device__ __forceinline__ uint32_t topo_apply(LU32 rs, int claim, uint64_t allow) {
    copy_words(s_trs0, rs, d.RSW);
    wsync();
    for (int w = 0; w < d.GMW; w++)
    for (uint64_t m = gword(GS_MASK, w, t_mask); m; m &= m - 1) {
      const int g = 64 * w + ctz64(m);
      const int k = tg(g, TGM_KEY), nv = tg(g, TGM_NV);
      const bool host = tg(g, TGM_HOST) != 0;
      const KeyMeta km = L.keys[k];
      const int nslot = nv + (host && claim >= 0 ? 1 : 0);  // + the claim's own hostname-placeholder (private bit)
      for (int i = lane(); i < d.RSW; i += kWave) s_trs1[i] = 0;
      wsync();
      // The values a domain scan visits.  When the record holds the key as an In set (a NodeClaim's
      // hostname: its own placeholder), Requirements.Add below keeps only values of that set (rs only
      // shrinks from the snapshot s_trs0), so the scan over the set's bits leaves rs exactly as the scan
      // over the whole universe would -- 5000 hostnames become one word per lane.
      const bool inSet = bit(rs_present(s_trs0), k) && !bit(rs_compl(s_trs0), k);
      auto scan = [&](bool restrict, auto&& body) {
        if (restrict && inSet) {
          for (int wd = lane(); wd < km.nw; wd += kWave)
            for (uint32_t x = s_trs0[L.HDR + km.off + wd]; x; x &= x - 1) {
              const int v = wd * 32 + __builtin_ctz(x);
              if (v < nslot) body(v);
            }
        } else {
          for (int v = lane(); v < nslot; v += kWave) body(v);
        }
      };
      if (tg(g, TGM_TYPE) == TG_SPREAD) {  // nextDomainTopologySpread: smallest count, then smallest name
        const int self = sel_has(g) ? 1 : 0, mn = s_tmin[g], skew = tg(g, TGM_SKEW);
        uint64_t best = ~0ull;
        scan(true, [&](int v) {
          const bool nodeHas = rs_member(L, s_trs0, k, v);
          int c = -1;
          if (nodeHas) c = v < nv ? tcnt(g, v) : tccnt(g, claim);  // placeholders are always registered
          const bool cand = c >= 0;
          c += self;
          if (cand && (int64_t)c - mn <= skew) {
            const uint64_t key = ((uint64_t)(uint32_t)c << 32) | (uint32_t)v;
            best = key < best ? key : best;
          }
        });
        best = wred_min(best, (uint64_t)~0ull);
        if (best == ~0ull) return FC_TOPO | ((uint32_t)g << 16);
        const int bv = (int)(uint32_t)best;
        if (lane() == 0) s_trs1[L.HDR + km.off + (bv >> 5)] = 1u << (bv & 31);
      } else if (tg(g, TGM_TYPE) == TG_AFFINITY) {  // nextDomainAffinity
        const bool self = sel_has(g);
        if (s_tmin[g]) {  // the domains already holding a selected pod (other placeholders drop out in Add)
          scan(true, [&](int v) {
            const int c = v < nv ? tcnt(g, v) : tccnt(g, claim);
            if (c > 0 && tpod_has(g, v))
              __hip_atomic_fetch_or(s_trs1 + L.HDR + km.off + (v >> 5), 1u << (v & 31), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_WAVEFRONT);
          });
        } else if (self) {  // bootstrap: first registered pod∩node domain, then first registered pod domain
          // (canonical map order = sorted names = value order; for hostname keys the claim's own
          // placeholder is its only node domain, and any other insert drops out in Add)
          uint32_t z1 = ~0u, z2 = ~0u;
          for (int v = lane(); v < nslot; v += kWave) {
            const int c = v < nv ? tcnt(g, v) : tccnt(g, claim);  // a placeholder: -1 if not registered
            if (c < 0 || !tpod_has(g, v)) continue;
            if (v < nv) z2 = (uint32_t)v < z2 ? (uint32_t)v : z2;
            if (rs_member(L, s_trs0, k, v)) z1 = (uint32_t)v < z1 ? (uint32_t)v : z1;
            if (v >= nv) z2 = z2 == ~0u ? (uint32_t)v : z2;  // registered, so the options are not empty
          }
          z1 = wred_min(z1, ~0u);
          z2 = wred_min(z2, ~0u);
          if (z1 == ~0u && z2 == ~0u) return FC_TOPO | ((uint32_t)g << 16);
          if (lane() == 0) {
            if (z1 != ~0u) s_trs1[L.HDR + km.off + (z1 >> 5)] |= 1u << (z1 & 31);
            if (z2 != ~0u) s_trs1[L.HDR + km.off + (z2 >> 5)] |= 1u << (z2 & 31);
          }
        } else {
          return FC_TOPO | ((uint32_t)g << 16);
        }
      } else {  // nextDomainAntiAffinity: registered zero-count domains the pod's domains allow
        // (a Solve renders which check failed -- no zero-count domain at all vs none the record allows --
        // so only simulations, which report success alone, restrict this scan)
        bool any = false;
        scan(SIM, [&](int v) {
          bool in;
          if (v < nv) {
            in = tcnt(g, v) == 0 && tpod_has(g, v);
          } else {
            const bool has = tpod_has(g, v);
            any = any || has;  // some registered placeholder has a zero count (the fresh claim's, at least)
            in = has && tccnt(g, claim) == 0;
          }
          if (in) {
            __hip_atomic_fetch_or(s_trs1 + L.HDR + km.off + (v >> 5), 1u << (v & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WAVEFRONT);
            any = true;
          }
        });
        if (wballot(any) == 0) return FC_TOPO | ((uint32_t)g << 16);
      }
      wsync();
      // requirements.Add(domains), run by every lane in lockstep on the same LDS words (wave-wide stores
      // of uniform values, see commit_claim)
      wr64(s_trs1, 0, 1ull << k);
      wsync();
      rs_add(L, rs, s_trs1);
      wsync();
    }
    // Compatible(nodeRequirements, topologyRequirements, AllowUndefinedWellKnownLabels)
    int ok = 1;
    if (lane() == 0) ok = rs_compatible(L, s_trs0, rs, allow) ? 1 : 0;
    ok = rdl(ok, 0);
    return ok ? 0u : (uint32_t)FC_TOPO_COMPAT;
  }
  // Topology.Record (topology.go:125-148) for the pod's final requirements F on NodeClaim `claim`,
  // or on existing node `node` (claim -1), wave-wide.  Only groups that count the pod are visited:
  // owned groups whose selector selects it, inverse groups it owns.  On an existing node F[key] is
  // the node's own label value (the strict Compatible admitted nothing else; ks_topo.cpp refuses
  // the one input where a pod's NotIn could stand in for a missing label), so the node's domain
  // table replaces the scan over F's value words.
  // Solve (not SIM): logAt >= 0 is the commit's log position; its log_hg entry gets the hostname groups Topology.Record
  // counted the pod in (the host replays them to print a hostname group's counts in an unsatisfiable-topology
  // message).
  template <class PR>
  __device__ __forceinline__ void topo_record(PR F, int claim, int node, uint64_t allow, int logAt) {
    hbm_release();
    const int GMW = d.GMW;
    if (node >= 0) {  // an existing node: one domain per group (its label); group 64 w + l in lane l
      for (int w = 0; w < GMW; w++) {
        const uint64_t sel = gword(GS_SEL, w, t_sel), inv = gword(GS_INV, w, t_inv), act = gword(GS_ACT, w, t_active);
        const uint64_t m = (sel & bits_below(d.G1, w) & act) | inv;
        if (!m) continue;
        bool mine = ((m >> lane()) & 1ull) != 0;
        const int g = mine ? 64 * w + lane() : 0;
        // a spread group over a filtered node set counts the pod only where the filter admits the node
        const bool filt = mine && g < d.G1 && tg(g, TGM_TYPE) == TG_SPREAD && tg(g, TGM_FEND) > tg(g, TGM_FBEG);
        for (uint64_t fm = wballot(filt); fm; fm &= fm - 1) {
          const int gf = 64 * w + ctz64(fm);
          int match = 0;
          if (lane() == 0)
            for (int f = tg(gf, TGM_FBEG); f < tg(gf, TGM_FEND) && !match; f++)
              match = rs_compatible(L, F, D.tg_frs + (int64_t)f * d.RSW, allow) ? 1 : 0;
          const bool keep = rdl(match, 0) != 0;
          mine = lane() == (gf & 63) ? (mine && keep) : mine;
        }
        const int v = mine ? tdom(g, node) : -1;
        if (v >= 0) tcnt_inc(tg(g, TGM_CNT) + v);  // recording registers the domain (distinct words per lane)
        const uint64_t hg = wballot(v >= 0 && tg(g, TGM_HOST) != 0);
        if (!SIM && logAt >= 0 && hg) W.log_hg[(int64_t)logAt * GMW + w] = hg;  // wave-wide store of a uniform value
      }
      hbm_release();
      wsync();
      return;
    }
    const uint64_t pres = rs_present(F), compl_ = rs_compl(F);
    for (int w = 0; w < GMW; w++) {
      uint64_t hg = 0;
      const uint64_t sel = gword(GS_SEL, w, t_sel), inv = gword(GS_INV, w, t_inv), act = gword(GS_ACT, w, t_active);
      for (uint64_t m = (sel & bits_below(d.G1, w) & act) | inv; m; m &= m - 1) {
        const int g = 64 * w + ctz64(m);
        const bool ownedGroup = g < d.G1;
        if (ownedGroup && tg(g, TGM_TYPE) == TG_SPREAD && tg(g, TGM_FEND) > tg(g, TGM_FBEG)) {  // nodeFilter
          int match = 0;
          if (lane() == 0)
            for (int f = tg(g, TGM_FBEG); f < tg(g, TGM_FEND) && !match; f++)
              match = rs_compatible(L, F, D.tg_frs + (int64_t)f * d.RSW, allow) ? 1 : 0;
          if (!rdl(match, 0)) continue;
        }
        if (node >= 0) {
          int rec = 0;
          if (lane() == 0) {
            const int v = tdom(g, node);
            if (v >= 0) tcnt_inc(tg(g, TGM_CNT) + v);  // recording registers the domain
            rec = v >= 0;
          }
          if (!SIM && tg(g, TGM_HOST) && rdl(rec, 0)) hg |= 1ull << (g & 63);
          continue;
        }
        const int k = tg(g, TGM_KEY), nv = tg(g, TGM_NV);
        if (!bit(pres, k)) continue;  // Get() of a missing key is Exists: no values
        const KeyMeta km = L.keys[k];
        if (ownedGroup && tg(g, TGM_TYPE) != TG_ANTI) {  // spread / affinity: only a collapsed domain
          int tot = 0;
          for (int wd = lane(); wd < km.nw; wd += kWave) tot += __popc(F[L.HDR + km.off + wd]);
          tot = wred_add(tot);
          if (bit(compl_, k) || tot != 1) continue;
        }
        bool any = false;
        for (int wd = lane(); wd < km.nw; wd += kWave) {  // anti-affinity: every domain of the requirement
          uint32_t x = F[L.HDR + km.off + wd];
          any = any || x != 0;
          while (x) {
            const int v = wd * 32 + __builtin_ctz(x);
            x &= x - 1;
            if (v >= nv) {
              if (claim >= 0) {  // -1: not registered in a late group (recording registers it)
                const int64_t at = (int64_t)g * W.ccs + claim;
                const int cc = W.tg_ccnt[at];
                W.tg_ccnt[at] = cc < 0 ? 1 : cc + 1;
                if (cc <= 0) W.tg_cpos[g] += 1;  // one more placeholder holding a counted pod
              }
            } else {
              tcnt_inc(tg(g, TGM_CNT) + v);
            }
          }
        }
        if (!SIM && tg(g, TGM_HOST) && wballot(any)) hg |= 1ull << (g & 63);
      }
      if (!SIM && logAt >= 0 && hg) W.log_hg[(int64_t)logAt * GMW + w] = hg;  // wave-wide store of a uniform value
    }
    hbm_release();
    wsync();
  }

  // Topology.Update for relaxation state s1 (topology.go:102-119), wave-wide: the late groups it owns that do not
  // exist yet are created now.  The NodeClaims made so far registered their placeholders before these groups
  // existed (NewNodeClaim's Register only reaches t.topologies), so their placeholder domains start unregistered.
  __device__ __forceinline__ void topo_activate_state(int s1, int nclaims, int hostCtr) {
    const int GMW = d.GMW;
    const uint64_t KS_G* own = D.st_gown + (int64_t)s1 * GMW;
    bool any = false;
    for (int w = 0; w < GMW; w++) {
      const uint64_t act = gword(GS_ACT, w, t_active), fresh = own[w] & ~act;
      if (!fresh) continue;
      any = true;
      for (uint64_t m = fresh; m; m &= m - 1) {
        const int g = 64 * w + ctz64(m);
        for (int c = lane(); c < nclaims; c += kWave) W.tg_ccnt[(int64_t)g * W.ccs + c] = -1;
        if (!SIM) W.tg_act[g] = hostCtr;  // placeholders up to this ordinal were never registered (uniform store)
      }
      if (w == 0) t_active = act | fresh;
      else s_gw[GS_ACT * GMW + w] = act | fresh;  // wave-wide store of a uniform value
    }
    if (any) hbm_release();
    wsync();
  }

  // --- NodeClaim quick reject at sorted position j: necessary conditions of NodeClaim.Add ------
  __device__ __forceinline__ bool claim_quick(int j, int s, int sflags, uint64_t toltpl, const int64_t* pod) const {
    if (!((toltpl >> s_ptpl[j]) & 1ull)) return false;  // Taints.Tolerates (nodeclaim.go:68-71)
    if (hpA() && (W.c_hp[s_order[j]] & cur_hpc)) return false;  // host port conflicts (:72-75)
    bool ok = true;
#pragma unroll
    for (int r = 0; r < RM; r++) {
      if (RT == 0 && r >= d.R) break;
      ok &= pod[r] <= s_phead[(int64_t)j * R() + r];
    }
    if (ok && keys(sflags))
      ok = rs_compatible(L, W.c_rs + (int64_t)s_order[j] * d.RSW, s_pin, d.allowWK);
    return ok;
  }

  // --- wave-cooperative NodeClaim.Add on claim c -------------------------------------------------
  // Builds s_rs / s_rem, the new requests, thresholds and option count.  Returns options left > 0.
  template <bool INL>
  __device__ __forceinline__ bool claim_full(int c, int s, int sflags, const int64_t* pod, int64_t* req, int* nthr,
                                             int& ncnt) {
    const ClaimView<INL>& v = cv<INL>();
    bool changed = false;
    PH_BEGIN(u0);
    if (keys(sflags) || (TOPO && t_any)) {
      const uint32_t KS_G* crs = W.c_rs + (int64_t)c * d.RSW;
      copy_words(s_rs, crs, d.RSW);
      wsync();
      if (keys(sflags))
        changed = rs_add_wave(L, s_rs, s_pin, (sflags & SF_TOUCHES_IT_KEYS) ? d.itKeys : 0);
      if (TOPO && t_any) {
        if (topo_apply(s_rs, c, d.allowWK) != 0) {  // topology requirements (nodeclaim.go:92-100)
          ncnt = 0;
          return false;
        }
        changed = !rs_equal_keys(L, s_rs, crs, d.itKeys);
      }
      algbytes += 8 * d.RSW;
    }
    const int t = uni(v.tpl[c]);
#pragma unroll
    for (int r = 0; r < RM; r++) {
      if (RT == 0 && r >= d.R) break;
      req[r] = v.req[(int64_t)c * R() + r] + pod[r];
      nthr[r] = uni(v.thr[(int64_t)c * R() + r]);
    }
    const int tb = s_tbeg[t], nIT = s_tbeg[t + 1] - tb;
    PHS_END(u0, 0);
    PH_BEGIN(u1);
    rem_same = false;
    if (!negR()) {
      // Requests only grow: the options a request no longer fits are a prefix of each resource's
      // Allocatable-ascending order beyond its threshold.
      int removed = 0, examined = 0;
      // the smallest Allocatable left beyond each resource's threshold, all read at once: a resource whose
      // request still fits it removes nothing and skips its ballot loop (the common step)
      int64_t nxt[RM];
      bool moves = false;
#pragma unroll
      for (int r = 0; r < RM; r++) {
        if (RT == 0 && r >= d.R) break;
        nxt[r] = nthr[r] < nIT ? tsort_a((int64_t)tb * R() + (int64_t)r * nIT + nthr[r]) : INT64_MAX;
        moves |= nxt[r] < req[r];
      }
      if (!changed && !moves) {  // the options stay as they are: no working copy, nothing to write back
        algbytes += 16 * R() + 4 * R();
        PHS_END(u1, 1);
        rem_same = true;
        ncnt = uni(v.cnt[c]);
        return ncnt > 0;
      }
      copy_words(s_rem, v.rem + (int64_t)c * d.TW, d.TW);
      wsync();
      for (int r = 0; r < R(); r++) {
        const int64_t base = (int64_t)tb * R() + (int64_t)r * nIT;
        int k = nthr[r];
        if (!(nxt[r] < req[r])) continue;
        while (k < nIT) {
          const int i = k + lane();
          const bool ex = i < nIT && tsort_a(base + i) < req[r];
          const uint64_t m = wballot(ex);
          if (m == 0) break;
          bool was = false;
          if (ex) {
            const int pos = tsort_p(base + i);
            const uint32_t bit = 1u << (pos & 31);
            was = (lds_and(s_rem + (pos >> 5), ~bit) & bit) != 0;
          }
          removed += __popcll(wballot(was));
          const int nm = __popcll(m);
          k += nm;
          examined += nm;
          if (nm < kWave) break;
        }
        nthr[r] = k;
      }
      algbytes += 8 * d.TW + 16 * R() + 4 * R() + (int64_t)examined * 12;
      wsync();
      PHS_END(u1, 1);
      if (!changed) {
        ncnt = uni(v.cnt[c]) - removed;
        return ncnt > 0;
      }
      // Requirements changed: the options left are those the new requirements still admit, from
      // the feasibility masks (one word per lane), exact per position only for irregular ones.
      PH_BEGIN(u2);
      feas_masks(s_rs, t, fm_row(s, t));
      PHS_END(u2, 2);
      PH_BEGIN(u3);
      for (int w0 = 0; w0 < d.TW; w0 += kWave) {
        const int w = w0 + lane();
        uint32_t keep = 0, irr = 0;
        if (w < d.TW) {
          const uint32_t rem = s_rem[w];
          irr = rem & s_firr[w];
          keep = rem & ~s_firr[w] & s_fic[w] & s_fof[w];
        }
        for (uint64_t any = wballot(irr != 0); any; any &= any - 1) {  // rare: complement IT requirements
          const int ow = w0 + ctz64(any);
          const uint32_t bits = (uint32_t)rdl((int)irr, ow - w0);
          const bool mine = lane() < 32 && ((bits >> lane()) & 1u);
          bool ok = false;
          if (mine) {
            const int it = D.tpl_its[tb + ow * 32 + lane()];
            ok = rs_intersects(L, D.it_rs + (int64_t)it * d.RSW, s_rs) && has_offering(it, s_rs);
          }
          const uint32_t okb = (uint32_t)wballot(ok);
          if (w == ow) keep |= okb;
        }
        if (w < d.TW) s_rem[w] = keep;
      }
      wsync();
      ncnt = popc_words(s_rem, d.TW);
      algbytes += 12 * (int64_t)d.TW;
      PHS_END(u3, 3);
      return ncnt > 0;
    }
    copy_words(s_rem, v.rem + (int64_t)c * d.TW, d.TW);
    wsync();
    int cnt = 0, scanned = 0;
    if (changed) feas_masks(s_rs, t, fm_row(s, t));
    for (int base = 0; base < nIT; base += kWave) {
      const int wi = base >> 5;
      const uint64_t bits = (uint64_t)s_rem[wi] | (wi + 1 < d.TW ? (uint64_t)s_rem[wi + 1] << 32 : 0ull);
      uint64_t m = 0;
      if (bits) {
        const int gpos = tb + base + lane();
        const int pos = base + lane();
        bool ok = (bits >> lane()) & 1ull;
        if (ok) ok = fits_pos(req, gpos);
        if (ok && changed) {
          if (fbit(s_firr, pos)) {
            const int it = D.tpl_its[gpos];
            ok = rs_intersects(L, D.it_rs + (int64_t)it * d.RSW, s_rs) && has_offering(it, s_rs);
          } else {
            ok = fbit(s_fic, pos) && fbit(s_fof, pos);
          }
        }
        m = wballot(ok);
        scanned += __popcll(bits);
      }
      wsync();
      store_bits(s_rem, base, m);
      cnt += __popcll(m);
    }
    ncnt = cnt;
    algbytes += 8 * d.TW + 16 * R() + (int64_t)scanned * 8 * R();
    wsync();
    return cnt > 0;
  }

  // exact max Allocatable per resource over the options (quick-reject bound); refreshes the
  // headroom of the claim's sorted position `pos` (-1: none yet)
  template <bool INL, class PB>
  __device__ __forceinline__ void recompute_max(int c, PB bits, int t, int pos) {
    const ClaimView<INL>& v = cv<INL>();
    const int tb = s_tbeg[t], nIT = s_tbeg[t + 1] - tb;
    for (int r = 0; r < R(); r++) {
      int64_t m = INT64_MIN;
      if (!negR()) {  // the first option from the top of the Allocatable-ascending order
        const int64_t base = (int64_t)tb * R() + (int64_t)r * nIT;
        for (int k = nIT - 1; k >= 0; k -= kWave) {
          const int i = k - lane();
          bool in = false;
          if (i >= 0) {
            const int q = tsort_p(base + i);
            in = (bits[q >> 5] >> (q & 31)) & 1u;
          }
          const uint64_t hit = wballot(in);
          if (hit) {
            m = tsort_a(base + k - ctz64(hit));
            break;
          }
        }
      } else {
        for (int q = lane(); q < nIT; q += kWave)
          if ((bits[q >> 5] >> (q & 31)) & 1u) {
            const int64_t a = alloc_pos(tb + q, r);
            m = a > m ? a : m;
          }
        m = wred_max(m, (int64_t)INT64_MIN);
      }
      m = rdl64(m, 0);  // lane 0's value, stored by every lane (claim state is written wave-wide, see commit_claim)
      v.max[(int64_t)c * R() + r] = m;
      if (pos >= 0) s_phead[(int64_t)pos * R() + r] = m - v.req[(int64_t)c * R() + r];
    }
    if (!INL) hbm_release();
    wsync();
  }

  // Returns whether s.newNodeClaims is still non-decreasing after the increment at `pos`.
  template <bool INL>
  __device__ __forceinline__ bool commit_claim(int c, int pos, int n, int p, int sflags, const int64_t* pod,
                                               const int64_t* req, const int* nthr, int ncnt, int& nlog) {
    const ClaimView<INL>& v = cv<INL>();
    const int okNew = uni(s_okey[pos]) + 1;
    const bool srt = pos + 1 >= n || okNew <= uni(s_okey[pos + 1]);
    // Claim state is written by every lane with the same (wave-uniform) values rather than under
    // `lane() == 0`: a lane-0-only LDS store was lost in some builds, a wave-wide one has no
    // exec-mask region to get wrong.  Same-address stores of one value are benign.
    int64_t heads[RM];  // (each lane reads before it writes the same words: program order keeps it)
#pragma unroll
    for (int r = 0; r < RM; r++) {
      if (RT == 0 && r >= d.R) break;
      heads[r] = s_phead[(int64_t)pos * R() + r];
    }
#pragma unroll
    for (int r = 0; r < RM; r++) {
      if (RT == 0 && r >= d.R) break;
      v.req[(int64_t)c * R() + r] = req[r];
      v.thr[(int64_t)c * R() + r] = nthr[r];
      s_phead[(int64_t)pos * R() + r] = heads[r] - pod[r];
    }
    v.cnt[c] = ncnt;
    s_okey[pos] = okNew;
    if (hpA()) W.c_hp[c] |= cur_hpu;  // hostPortUsage.Add (wave-wide store of a uniform value)
    if (keys(sflags) || (TOPO && t_any)) copy_words(W.c_rs + (int64_t)c * d.RSW, s_rs, d.RSW);
    if (!rem_same) copy_words(v.rem + (int64_t)c * d.TW, s_rem, d.TW);
    log_commit(p, c, nlog);
    // The max bound stays valid as the options only shrink; it is tightened lazily when a full check
    // fails.  HBM-resident claim state is re-read by other lanes: drain the stores first.
    if (keys(sflags) || !INL || hpA()) hbm_release();
    wsync();
    if (TOPO && t_rec) {  // Topology.Record on the claim's final requirements (nodeclaim.go:121)
      if (keys(sflags) || t_any) topo_record(s_rs, c, -1, d.allowWK, nlog - 1);
      else topo_record(W.c_rs + (int64_t)c * d.RSW, c, -1, d.allowWK, nlog - 1);
    }
    algbytes += 24 * R() + 4 * d.TW + 8;
    return srt;
  }

  // --- runs of identical resource-only pods on one NodeClaim (LEAN Solve) -------------------------
  // After a pod lands on the claim at sorted position `pos` and s.newNodeClaims stays non-decreasing, an
  // identical next pod meets the same sort (nothing to reorder), the same rejections before `pos` (those
  // claims and the existing nodes did not change) and lands on this claim again while it accepts -- as
  // long as the claim's count stays <= the next position's.  The pods one claim takes that way: at most
  // M (the run, and that count bound), and at most as many as its best remaining option still fits:
  // max over the options of min over resources of floor((Allocatable - requests) / pod).
  template <bool INL>
  __device__ __forceinline__ int claim_run_cap(int c, const int64_t* pod, int M) const {
    const ClaimView<INL>& v = cv<INL>();
    const int t = uni(v.tpl[c]);
    const int tb = s_tbeg[t], nIT = s_tbeg[t + 1] - tb;
    float rq[RM];
    int64_t rc[RM];
#pragma unroll
    for (int r = 0; r < RM; r++) {
      if (RT == 0 && r >= d.R) break;
      rq[r] = run_rcp(pod[r]);
      rc[r] = v.req[(int64_t)c * R() + r];
    }
    int best = 0;
    for (int q0 = 0; q0 < nIT; q0 += kWave) {
      const int q = q0 + lane();
      if (q < nIT && ((v.rem[(int64_t)c * d.TW + (q >> 5)] >> (q & 31)) & 1u)) {
        int cap = M;
#pragma unroll
        for (int r = 0; r < RM; r++) {
          if (RT == 0 && r >= d.R) break;
          const int x = run_cap(alloc_pos(tb + q, r) - rc[r], pod[r], rq[r], M);
          cap = x < cap ? x : cap;
        }
        best = cap > best ? cap : best;
      }
    }
    return wred_max(best, (int)0x80000000);
  }
  // Commit of k identical pods (podk = k x pod, claim_full already applied to it) to claim c at sorted
  // position pos: commit_claim's stores with the count advanced by k.  Returns whether s.newNodeClaims
  // is still non-decreasing.
  template <bool INL>
  __device__ __forceinline__ bool commit_bulk(int c, int pos, int n, int k, const int64_t* podk, const int64_t* req,
                                              const int* nthr, int ncnt) {
    const ClaimView<INL>& v = cv<INL>();
    const int okNew = uni(s_okey[pos]) + k;
    const bool srt = pos + 1 >= n || okNew <= uni(s_okey[pos + 1]);
    int64_t heads[RM];
#pragma unroll
    for (int r = 0; r < RM; r++) {
      if (RT == 0 && r >= d.R) break;
      heads[r] = s_phead[(int64_t)pos * R() + r];
    }
#pragma unroll
    for (int r = 0; r < RM; r++) {  // wave-wide stores of uniform values (see commit_claim)
      if (RT == 0 && r >= d.R) break;
      v.req[(int64_t)c * R() + r] = req[r];
      v.thr[(int64_t)c * R() + r] = nthr[r];
      s_phead[(int64_t)pos * R() + r] = heads[r] - podk[r];
    }
    v.cnt[c] = ncnt;
    s_okey[pos] = okNew;
    if (!rem_same) copy_words(v.rem + (int64_t)c * d.TW, s_rem, d.TW);
    if (!INL) hbm_release();
    wsync();
    return srt;
  }

  // --- new NodeClaim from each template in order (scheduler.go:258-283) -----------------------
  // Returns 1 placed, 0 failed (fail codes recorded), 2 no templates (add() returns nil), -1 cap.
  __device__ __forceinline__ int try_templates(int p, int s, int sflags, uint64_t toltpl, const int64_t* pod,
                                               int& nclaims, int& nlog, int& hostCtr, bool& srt) {
    if (d.NTPL == 0) return 2;
    for (int t = 0; t < d.NTPL; t++) {
      uint32_t code = FC_NONE;
      int hostid = -1;
      const int tb = s_tbeg[t], nIT = s_tbeg[t + 1] - tb;
      const int pool = D.tpl_pool[t];
      // filterByRemainingResources (scheduler.go:364-383)
      uint64_t anyCand = 0;
      for (int base = 0; base < nIT; base += kWave) {
        const int pos = base + lane();
        bool ok = pos < nIT;
        if (ok && pool >= 0) {
          const uint32_t mask = D.pool_mask[pool];
          const int64_t KS_G* cap = D.it_cap + (int64_t)D.tpl_its[tb + pos] * R();
          for (int r = 0; r < R(); r++)
            if (((mask >> r) & 1u) && cap[r] > s_pool[(int64_t)pool * R() + r]) ok = false;
        }
        const uint64_t m = wballot(ok);
        store_bits(s_cand, base, m);
        anyCand |= m;
      }
      wsync();
      if (pool >= 0 && anyCand == 0) {
        code = FC_LIMITS;
      } else {
        hostid = ++hostCtr;  // NewNodeClaim: atomic.AddInt64(&nodeID, 1) (nodeclaim.go:48)
        if (!((toltpl >> t) & 1ull)) {
          code = FC_TAINTS;
        } else {
          copy_words(s_rs, D.tpl_rs + (int64_t)t * d.RSW, d.RSW);
          wsync();
          bool ok = true;
          if (keys(sflags)) {
            ok = rs_compatible(L, s_rs, s_pin, d.allowWK);
            if (ok) rs_add_wave(L, s_rs, s_pin, 0);
          }
          if (TOPO && ok && t_any) {  // topology requirements of the fresh NodeClaim (nodeclaim.go:92-100)
            const uint32_t tc = topo_apply(s_rs, nclaims, d.allowWK);
            if (tc) {
              ok = false;
              code = tc;
              const int64_t slot = ((int64_t)p * d.NTPL + t) * d.FSW;
              if (SIM) {  // simulations render no messages
              } else if (tc == FC_TOPO_COMPAT) {
                copy_words(W.fail_rs + slot, s_rs, d.RSW);  // the topology requirements, for the message
              } else {
                const int g = (int)(tc >> 16) & 0xffff, nv = tg(g, TGM_NV);
                if (!tg(g, TGM_HOST))  // the counts (-1: unregistered), for the message (FSW fits them)
                  for (int v = lane(); v < nv; v += kWave) W.fail_rs[slot + v] = (uint32_t)tcnt(g, v);
                else if (lane() == 0)  // hostname: the commits so far; the host replays their log_hg entries
                  W.fail_rs[slot] = (uint32_t)nlog;
              }
            }
          }
          if (!ok) {
            if (code == FC_NONE) code = FC_COMPAT;
          } else {
            int64_t req[RM];
            for (int r = 0; r < R(); r++) req[r] = D.tpl_daemon[(int64_t)t * R() + r] + pod[r];
            uint32_t flags = 0;
            uint64_t any = 0;
            feas_masks(s_rs, t, fm_row(s, t));
            for (int base = 0; base < nIT; base += kWave) {
              const int pos = base + lane();
              const bool in = pos < nIT && ((s_cand[pos >> 5] >> (pos & 31)) & 1u);
              bool ic = false, fi = false, of = false;
              if (in) {
                if (fbit(s_firr, pos)) {
                  const int it = D.tpl_its[tb + pos];
                  ic = rs_intersects(L, D.it_rs + (int64_t)it * d.RSW, s_rs);
                  of = has_offering(it, s_rs);
                } else {
                  ic = fbit(s_fic, pos);
                  of = fbit(s_fof, pos);
                }
                fi = fits_pos(req, tb + pos);
              }
              if (wballot(ic)) flags |= FF_REQ;
              if (wballot(fi)) flags |= FF_FITS;
              if (wballot(of)) flags |= FF_OFF;
              if (wballot(ic && fi && !of)) flags |= FF_REQ_FITS;
              if (wballot(ic && of && !fi)) flags |= FF_REQ_OFF;
              if (wballot(fi && of && !ic)) flags |= FF_FITS_OFF;
              const uint64_t m = wballot(ic && fi && of);
              store_bits(s_rem, base, m);
              any |= m;
            }
            algbytes += 4 * d.RSW + (int64_t)nIT * (8 * R() + 4 * d.RSW + 16);
            wsync();
            if (any == 0) {
              code = FC_NO_IT | (flags << 8);
              if (!SIM && TOPO && t_any) {  // the message prints the requirements the topology narrowed
                copy_words(W.fail_rs + ((int64_t)p * d.NTPL + t) * d.FSW, s_rs, d.RSW);
                code |= FC_RS_SNAP;
              }
            } else {
              if (nclaims >= pl.KO) return -1;
              const int c = nclaims++;
              if (SIM && TOPO)  // the next fresh claim's placeholder counts (a simulation zeroes one column per claim)
                for (int g = lane(); g < d.G; g += kWave) W.tg_ccnt[(int64_t)g * W.ccs + nclaims] = 0;
              const bool inl = c < pl.KL;
              copy_words(W.c_rs + (int64_t)c * d.RSW, s_rs, d.RSW);
              if (inl) copy_words(lc.rem + (int64_t)c * d.TW, s_rem, d.TW);
              else copy_words(gc.rem + (int64_t)c * d.TW, s_rem, d.TW);
              // thresholds: how much of each resource's ascending Allocatable order req excludes
              int thr[RM];
              for (int r = 0; r < R(); r++) {
                const int64_t b = (int64_t)tb * R() + (int64_t)r * nIT;
                int k = 0;
                for (int q = 0; q < nIT; q += kWave)
                  k += __popcll(wballot(q + lane() < nIT && tsort_a(b + q + lane()) < req[r]));
                thr[r] = k;
              }
              const int cnt = popc_words(s_rem, d.TW);
              // wave-wide stores of uniform values (see commit_claim)
              for (int r = 0; r < R(); r++) {
                if (inl) {
                  lc.req[(int64_t)c * R() + r] = req[r];
                  lc.thr[(int64_t)c * R() + r] = thr[r];
                } else {
                  gc.req[(int64_t)c * R() + r] = req[r];
                  gc.thr[(int64_t)c * R() + r] = thr[r];
                }
              }
              if (inl) {
                lc.tpl[c] = t;
                lc.cnt[c] = cnt;
              } else {
                gc.cnt[c] = cnt;
              }
              W.c_tpl[c] = t;  // wave-wide stores of uniform values (see commit_claim)
              W.c_hp[c] = cur_hpu;
              W.c_host[c] = hostid;
              s_order[c] = c;
              s_okey[c] = 1;
              s_ptpl[c] = t;
              srt = c == 0 || uni(s_okey[c - 1]) <= 1;
              log_commit(p, c, nlog);
              hbm_release();  // c_rs / c_tpl / overflow state are read by other lanes later
              wsync();
              if (TOPO && t_rec) topo_record(s_rs, c, -1, d.allowWK, nlog - 1);
              if (inl) recompute_max<true>(c, s_rem, t, c);
              else recompute_max<false>(c, s_rem, t, c);
              if (pool >= 0) {  // subtractMax (scheduler.go:347-362)
                const uint32_t mask = D.pool_mask[pool];
                for (int r = 0; r < R(); r++) {
                  if (!((mask >> r) & 1u)) continue;
                  int64_t m = INT64_MIN;
                  for (int pos = lane(); pos < nIT; pos += kWave)
                    if ((s_rem[pos >> 5] >> (pos & 31)) & 1u) {
                      const int64_t v = D.it_cap[(int64_t)D.tpl_its[tb + pos] * R() + r];
                      m = v > m ? v : m;
                    }
                  m = wred_max(m, (int64_t)INT64_MIN);
                  s_pool[(int64_t)pool * R() + r] -= m;  // wave-wide (m is reduced over the wave)
                }
                wsync();
              }
              return 1;
            }
          }
        }
      }
      W.fail_code[(int64_t)p * d.NTPL + t] = code;  // wave-wide stores of uniform values
      W.fail_host[(int64_t)p * d.NTPL + t] = hostid;
    }
    return 0;
  }

  // try_templates' NewNodeClaim calls for a pod every template fails on topology (simNoClaim): a template whose
  // instance types all exceed its NodePool's remaining limits fails before NewNodeClaim (scheduler.go:262-268);
  // every other one increments the hostname counter (nodeclaim.go:44-48).  Returns 0 (the pod is not placed).
  __device__ __forceinline__ int sim_template_calls(int& hostCtr) const {
    for (int t = 0; t < d.NTPL; t++) {
      const int pool = D.tpl_pool[t];
      bool call = pool < 0;
      if (!call) {
        const int tb = s_tbeg[t], nIT = s_tbeg[t + 1] - tb;
        const uint32_t mask = D.pool_mask[pool];
        uint64_t anyCand = 0;
        for (int base = 0; base < nIT && !anyCand; base += kWave) {
          const int pos = base + lane();
          bool ok = pos < nIT;
          if (ok) {
            const int64_t KS_G* cap = D.it_cap + (int64_t)D.tpl_its[tb + pos] * R();
            for (int r = 0; r < R(); r++)
              ok = ok && !(((mask >> r) & 1u) && cap[r] > s_pool[(int64_t)pool * R() + r]);
          }
          anyCand = wballot(ok);
        }
        call = anyCand != 0;
      }
      if (call) hostCtr = uni(hostCtr + 1);
    }
    return 0;
  }

  // --- s.newNodeClaims re-sort (scheduler.go:247) --------------------------------------------------
  // Called only when the array is not non-decreasing (a non-decreasing array is provably left
  // untouched by pdqsort).  Lane 0 replays Go's pdqsort_func; the position-indexed quick-reject
  // arrays are then regathered from the claims.
  // Move the entry at position `from` to `to`, shifting the ones between by one (wave-parallel, in
  // 64-entry chunks ordered so every chunk is read before it is overwritten).  Equals the adjacent
  // swap chains of partialInsertionSort.
  __device__ __forceinline__ void pis_move(int from, int to) {
    if (from == to) return;
    const int k0 = uni(s_okey[from]), v0 = uni(s_order[from]);
    wsync();
    if (to < from) {  // [to, from) shifts right, high chunk first
      for (int hi = from; hi > to; hi -= kWave) {
        const int lo = hi - kWave > to ? hi - kWave : to, j = lo + lane();
        int k = 0, v = 0;
        if (j < hi) { k = s_okey[j]; v = s_order[j]; }
        wsync();
        if (j < hi) { s_okey[j + 1] = k; s_order[j + 1] = v; }
        wsync();
      }
    } else {  // (from, to] shifts left, low chunk first
      for (int lo = from + 1; lo <= to; lo += kWave) {
        const int hi = lo + kWave <= to + 1 ? lo + kWave : to + 1, j = lo + lane();
        int k = 0, v = 0;
        if (j < hi) { k = s_okey[j]; v = s_order[j]; }
        wsync();
        if (j < hi) { s_okey[j - 1] = k; s_order[j - 1] = v; }
        wsync();
      }
    }
    s_okey[to] = k0;  // wave-wide store of uniform values (see commit_claim)
    s_order[to] = v0;
    wsync();
  }
  // First i in [from, n) with key[i] < key[i-1] (a descent), or n.  Four chunks per round trip: the
  // scan usually runs to the end of the array (proving it sorted), so it is latency-bound.
  __device__ __forceinline__ int pis_descent(int from, int n) const {
    for (int base = from; base < n; base += 4 * kWave) {
      uint64_t m[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int i = base + u * kWave + lane();
        const int k1 = i < n ? s_okey[i] : 0, k0 = i < n ? s_okey[i - 1] : 0;
        m[u] = wballot(k1 < k0);
      }
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (m[u]) return base + u * kWave + ctz64(m[u]);
    }
    return n;
  }
  // choosePivot_func (zsortfunc.go): the wave reads the (up to) nine samples at once, lane t sample t,
  // and the medians run on scalars; same pivot and hint as GoSortT::choosePivot.
  __device__ __forceinline__ int w_choose_pivot(int a, int b, int& hint) const {
    const int l = b - a;
    int i = a + l / 4, j = a + l / 4 * 2, k = a + l / 4 * 3, swaps = 0;
    if (l >= 8) {
      const int t = lane() < 9 ? lane() : 0, g = t / 3;
      const int pos = (g == 0 ? i : g == 1 ? j : k) + (t % 3) - 1;
      const int key = s_okey[pos];
      int ik[9], kk[9];
#pragma unroll
      for (int u = 0; u < 9; u++) {
        ik[u] = (u / 3 == 0 ? i : u / 3 == 1 ? j : k) + (u % 3) - 1;
        kk[u] = rdl(key, u);
      }
      auto median = [&](int ia, int ka, int ib, int kb, int ic, int kc, int& km) {
        if (kb < ka) { swaps++; int t0 = ia; ia = ib; ib = t0; t0 = ka; ka = kb; kb = t0; }
        if (kc < kb) { swaps++; int t0 = ib; ib = ic; ic = t0; t0 = kb; kb = kc; kc = t0; }
        if (kb < ka) { swaps++; int t0 = ia; ia = ib; ib = t0; t0 = ka; ka = kb; kb = t0; }
        km = kb;
        return ib;
      };
      int ki = kk[1], kj = kk[4], kq = kk[7];
      if (l >= 50) {
        i = median(ik[0], kk[0], ik[1], kk[1], ik[2], kk[2], ki);
        j = median(ik[3], kk[3], ik[4], kk[4], ik[5], kk[5], kj);
        k = median(ik[6], kk[6], ik[7], kk[7], ik[8], kk[8], kq);
      }
      int km = 0;
      j = median(i, ki, j, kj, k, kq, km);
    }
    hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
    return j;
  }
  // partialInsertionSort_func(data, 0, n) of Go 1.21 (zsortfunc.go), wave-parallel: each of its <= 5
  // steps finds the next descent by ballot, swaps the pair, then moves the smaller entry left past
  // every greater one and the greater entry right past every smaller one.  Returns its result and
  // widens [tlo, thi] to the positions it moved.
  __device__ __forceinline__ bool pis_wave(int a, int b, int& tlo, int& thi) {
    int i = a + 1;
    for (int step = 0; step < 5; step++) {
      i = pis_descent(i, b);
      if (i == b) return true;
      if (b - a < 50) return false;
      const int x = uni(s_okey[i]), y = uni(s_okey[i - 1]);  // after the swap: x at i-1, y at i
      int p = i - 1;  // x passes the entries q < i-1 with x < key[q] (Go's loop runs down to index 1,
      if (i - a >= 2) {  // not to a, once the pair is at least two past a)
        for (int hi = i - 1; hi > 0; hi -= kWave) {
          const int q = hi - 1 - lane();
          const uint64_t m = wballot(q >= 0 && !(x < s_okey[q]));
          if (m) { p = hi - ctz64(m); break; }
          p = hi - kWave > 0 ? hi - kWave : 0;
        }
      }
      int r = i;  // y passes the entries q > i with key[q] < y
      for (int lo = i + 1; lo < b; lo += kWave) {
        const int q = lo + lane();
        const uint64_t m = wballot(q < b && !(s_okey[q] < y));
        if (m) { r = lo + ctz64(m) - 1; break; }
        r = lo + kWave - 1 < b - 1 ? lo + kWave - 1 : b - 1;
      }
      pis_move(i, p);  // x (at i before the swap) to p; y moves from i-1 to i with the shifted run
      pis_move(i, r);  // y to r
      tlo = p < tlo ? p : tlo;
      thi = r > thi ? r : thi;
    }
    return false;
  }

  // --- the rest of pdqsort_func, wave-parallel and swap-for-swap equal to Go's (ks_gosort.h) -------
  // Exchange of two uniform positions (wave-wide stores of uniform values).
  __device__ __forceinline__ void w_swap(int i, int j) {
    const int ki = uni(s_okey[i]), kj = uni(s_okey[j]), vi = uni(s_order[i]), vj = uni(s_order[j]);
    wsync();
    s_okey[i] = kj;
    s_order[i] = vj;
    wsync();
    s_okey[j] = ki;
    s_order[j] = vi;
    wsync();
  }
  // Entries of [a, b) whose key is below `pk` (below_or_eq: at most `pk`).
  __device__ __forceinline__ int w_count(int a, int b, int pk, bool below_or_eq) const {
    int c = 0;
    for (int base = a; base < b; base += kWave) {
      const int p = base + lane();
      const int k = p < b ? s_okey[p] : 0;
      c += __popcll(wballot(p < b && (below_or_eq ? k <= pk : k < pk)));
    }
    return c;
  }
  // A Hoare pass (partition_func / partitionEqual_func) whose boundary `m` is known up front: its i scan
  // stops on the left region's entries [l0, m) of the wrong side, its j scan on the right region's
  // [m, r1), and it exchanges the k-th from the left with the k-th from the right, for every k (the two
  // counts are equal, and the scans cross exactly at the boundary).  `eq` selects partitionEqual's
  // predicates (wrong on the left: key > pk) over partition's (key >= pk).  Returns the exchange count.
  __device__ int w_hoare(int l0, int m, int r1, int pk, bool eq) {
    int lb = l0, rb = r1, lbase = 0, rtop = 0, swaps = 0;
    uint64_t mL = 0, mR = 0;
    for (;;) {
      if (mL == 0) {
        if (lb >= m) break;
        const int p = lb + lane();
        const int k = p < m ? s_okey[p] : 0;
        mL = wballot(p < m && (eq ? k > pk : k >= pk));
        lbase = lb;
        lb += kWave;
        continue;
      }
      if (mR == 0) {
        if (rb <= m) break;
        const int p = rb - 1 - lane();  // bit t <-> position rtop - t: ascending bits walk down from r1
        const int k = p >= m ? s_okey[p] : 0;
        mR = wballot(p >= m && (eq ? k <= pk : k < pk));
        rtop = rb - 1;
        rb -= kWave;
        continue;
      }
      const int nL = __popcll(mL), nR = __popcll(mR), np = nL < nR ? nL : nR;
      const uint64_t below = (1ull << lane()) - 1ull;
      const bool inL = (mL >> lane()) & 1ull, inR = (mR >> lane()) & 1ull;
      const int rkL = __popcll(mL & below), rkR = __popcll(mR & below);
      // ds_permute pushes every lane's position to its rank (a bijection over the 64 lanes)
      const int dL = inL ? rkL : nL + (lane() - rkL), dR = inR ? rkR : nR + (lane() - rkR);
      const int posL = __builtin_amdgcn_ds_permute(dL * 4, lbase + lane());
      const int posR = __builtin_amdgcn_ds_permute(dR * 4, rtop - lane());
      if (lane() < np) {  // disjoint positions: the lanes' exchanges do not overlap
        const int kl = s_okey[posL], vl = s_order[posL], kr = s_okey[posR], vr = s_order[posR];
        s_okey[posL] = kr;
        s_order[posL] = vr;
        s_okey[posR] = kl;
        s_order[posR] = vl;
      }
      wsync();
      for (int t = 0; t < np; t++) {
        mL &= mL - 1;
        mR &= mR - 1;
      }
      swaps += np;
    }
    return swaps;
  }
  // partition_func: returns the new pivot position; `already` = no exchange was needed.
  __device__ __forceinline__ int w_partition(int a, int b, int pivot, bool& already) {
    w_swap(a, pivot);
    const int pk = uni(s_okey[a]);
    const int j = a + w_count(a + 1, b, pk, false);
    already = w_hoare(a + 1, j + 1, b, pk, false) == 0;
    w_swap(j, a);
    return j;
  }
  // partitionEqual_func: returns the first position past the entries equal to the pivot.
  __device__ __forceinline__ int w_partition_equal(int a, int b, int pivot) {
    w_swap(a, pivot);
    const int pk = uni(s_okey[a]);
    const int m = a + 1 + w_count(a + 1, b, pk, true);
    w_hoare(a + 1, m, b, pk, true);
    return m;
  }
  __device__ __forceinline__ void w_reverse(int a, int b) {
    const int h = (b - a) / 2;
    for (int base = 0; base < h; base += kWave) {
      const int t = base + lane();
      if (t < h) {
        const int i = a + t, j = b - 1 - t;
        const int ki = s_okey[i], vi = s_order[i], kj = s_okey[j], vj = s_order[j];
        s_okey[i] = kj;
        s_order[i] = vj;
        s_okey[j] = ki;
        s_order[j] = vi;
      }
    }
    wsync();
  }
  // GoSortExactT::run with the whole wave: frames live one per lane (lane k = stack slot k), the
  // partitions, reversals and partialInsertionSorts run wave-parallel; insertionSort (<= 12 entries),
  // heapSort (the depth limit), breakPatterns and choosePivot stay on lane 0.  resumePivot as in run().
  __device__ void w_pdqsort(int n, int resumePivot) {
    int fa = 0, fb = 0, fl = 0, ff = 0;  // this lane's stack slot: a, b, limit, flags (wb | wp << 1)
    int sp = 0;
    {
      const bool me = lane() == 0;
      fa = me ? 0 : fa;
      fb = me ? n : fb;
      fl = me ? GoSortT<LI32>::bitsLen((uint32_t)n) : fl;
      ff = me ? 3 : ff;
      sp = 1;
    }
    bool resume = resumePivot >= 0;
    int dummy_lo = 0, dummy_hi = 0;
    while (sp > 0) {
      sp--;
      int a = rdl(fa, sp), b = rdl(fb, sp), limit = rdl(fl, sp);
      const int flags = rdl(ff, sp);
      bool wasBalanced = flags & 1, wasPartitioned = (flags >> 1) & 1;
      for (;;) {
        const int length = b - a;
        int pivot;
        if (resume) {
          resume = false;
          pivot = resumePivot;
        } else {
          if (length <= 12 || limit == 0) {
            if (lane() == 0) {
              GoSortT<LI32> g{s_okey, s_order};
              if (length <= 12) g.insertionSort(a, b);
              else g.heapSort(a, b);
            }
            wsync();
            break;
          }
          if (!wasBalanced) {
            if (lane() == 0) {
              GoSortT<LI32> g{s_okey, s_order};
              g.breakPatterns(a, b);
            }
            wsync();
            limit--;
          }
          int hint = 0;
          pivot = w_choose_pivot(a, b, hint);
          if (hint == 2) {
            w_reverse(a, b);
            pivot = (b - 1) - (pivot - a);
            hint = 1;
          }
          if (wasBalanced && wasPartitioned && hint == 1 && pis_wave(a, b, dummy_lo, dummy_hi)) break;
        }
        if (a > 0 && ub(!(s_okey[a - 1] < s_okey[pivot]))) {
          a = w_partition_equal(a, b, pivot);
          continue;
        }
        bool already = false;
        const int mid = w_partition(a, b, pivot, already);
        wasPartitioned = already;
        const int leftLen = mid - a, rightLen = b - mid, thr = length / 8;
        if (sp + 2 > kWave) return;  // unreachable: depth <= 2*log2(n) + 2
        int c0a, c0b, c1a, c1b;
        if (leftLen < rightLen) {
          wasBalanced = leftLen >= thr;
          c0a = mid + 1; c0b = b; c1a = a; c1b = mid;  // continuation, then the recursive call
        } else {
          wasBalanced = rightLen >= thr;
          c0a = a; c0b = mid; c1a = mid + 1; c1b = b;
        }
        const bool m0 = lane() == sp, m1 = lane() == sp + 1;
        fa = m0 ? c0a : (m1 ? c1a : fa);
        fb = m0 ? c0b : (m1 ? c1b : fb);
        fl = (m0 || m1) ? limit : fl;
        ff = m0 ? ((int)wasBalanced | ((int)wasPartitioned << 1)) : (m1 ? 3 : ff);
        sp += 2;
        break;
      }
    }
  }
  // Returns true when lane 0 ran the exact pdqsort (the wave-parallel fast path did not finish it).
  __device__ __forceinline__ bool sort_claims(int n) {
    int tlo = n, thi = -1, pivot = -1;
    bool done = false;
    if (n > 12) {  // pdqsort_func's top-level frame: choosePivot (reads only), then partialInsertionSort
      int hint = 0;
      const int pv = w_choose_pivot(0, n, hint);
      if (hint == 1) {
        pivot = pv;
        done = pis_wave(0, n, tlo, thi);
      }
    }
    if (!done) {
#if KS_SORT_LANE0
      if (lane() == 0) {
        GoSortExactT<LI32> g{GoSortT<LI32>{s_okey, s_order}};
        g.run(n, pivot);
      }
#else
      w_pdqsort(n, pivot);
#endif
      tlo = 0;
      thi = n - 1;
    }
    wsync();
    for (int j = tlo + lane(); j <= thi; j += kWave) {
      const int c = s_order[j];
      const bool inl = c < pl.KL;
      s_ptpl[j] = inl ? lc.tpl[c] : W.c_tpl[c];
      for (int r = 0; r < R(); r++) {
        const int64_t i = (int64_t)c * R() + r;
        s_phead[(int64_t)j * R() + r] = inl ? lc.max[i] - lc.req[i] : gc.max[i] - gc.req[i];
      }
    }
    wsync();
    algbytes += (int64_t)(thi - tlo + 1) * (8 + 16 * R());
    return !done;
  }

  // --- consolidation decision for this simulation (SIM epilogue) -------------------------------
  // worstLaunchPrice (helpers.go:235-258): the max price over the available offerings of the
  // preferred capacity type (spot first) whose zone the requirements allow.
  template <class PR>
  __device__ __forceinline__ double worst_price(int it, PR rs, bool spot, bool od) const {
    const int b = D.it_off_beg[it], e = D.it_off_beg[it + 1];
    for (int pass = 0; pass < 2; pass++) {
      if (!(pass == 0 ? spot : od)) continue;
      const int want = pass == 0 ? d.spotBit : d.odBit;
      bool any = false;
      double w = 0;
      for (int o = b; o < e; o++)
        if (D.off_ct[o] == want && rs_member(L, rs, d.zoneKey, D.off_zone[o])) {
          const double pr = D.off_price[o];
          if (!any || pr > w) w = pr;
          any = true;
        }
      if (any) return w;
    }
    return __DBL_MAX__;
  }
  // filterByPrice (helpers.go:160-169) over the options bitset `in` of template t -> `out`
  template <class PI, class PO, class PR>
  __device__ __forceinline__ int price_filter(PI in, PO out, int t, PR rs, bool spot, bool od, double price) const {
    const int tb = s_tbeg[t], nIT = s_tbeg[t + 1] - tb;
    int cnt = 0;
    for (int base = 0; base < nIT; base += kWave) {
      const int pos = base + lane();
      bool keep = pos < nIT && ((in[pos >> 5] >> (pos & 31)) & 1u);
      if (keep) keep = worst_price(D.tpl_its[tb + pos], rs, spot, od) < price;
      const uint64_t m = wballot(keep);
      if (lane() == 0) {
        out[base >> 5] = (uint32_t)m;
        if ((base >> 5) + 1 < d.TW) out[(base >> 5) + 1] = (uint32_t)(m >> 32);
      }
      cnt += __popcll(m);
    }
    return cnt;
  }
  // simulateScheduling's post-check (helpers.go:115-124) + computeConsolidation (consolidation.go:
  // 113-194) + filterOutSameType (multinodeconsolidation.go:155-188), into the record W.rec
  // anyPushed: some pod failed an attempt (its status array exists, sim_queue_init); otherwise every pod was placed.
  __device__ __forceinline__ void sim_record(int P, int nclaims, int hostCtr, bool allSched, int err, bool anyPushed,
                                             bool anyRelaxed) {
    if (anyPushed) {
      hbm_release();  // pod statuses written by lane 0
      bool bad = false;
      for (int i = lane(); i < P; i += kWave)
        bad |= ld_sc1(W.pod_status + i) == ST_FAILED && !(D.pod_flags[W.pod_map[i]] & PF_PROVISIONABLE);
      allSched = allSched && wballot(bad) == 0;
    }
    int32_t KS_G* rec = W.rec;
    const int TW = d.TW;
    int32_t KS_G* o_opt = rec + RF_HDR;
    int32_t KS_G* o_price = o_opt + TW;
    int32_t KS_G* o_same = o_price + TW;
    for (int i = lane(); i < 3 * TW; i += kWave) o_opt[i] = 0;
    int flags = (allSched ? RB_ALL_SCHEDULED : 0) | (anyRelaxed ? RB_RELAXED : 0), tpl = -1, host = -1, nopt = 0,
        nprice = 0, nsame = 0;
    int action = CA_NOOP;
    if (nclaims > 0 && err == KE_OK) {
      const int c = uni(s_order[0]);
      const bool inl = c < pl.KL;
      tpl = inl ? uni(lc.tpl[c]) : uni(W.c_tpl[c]);
      host = W.c_host[c];
      const uint32_t KS_G* crs = W.c_rs + (int64_t)c * d.RSW;
      wsync();
      for (int i = lane(); i < TW; i += kWave) o_opt[i] = inl ? lc.rem[(int64_t)c * TW + i] : gc.rem[(int64_t)c * TW + i];
      rec[RF_CLAIM] = c;  // wave-wide store of a uniform value
      {
        int cc = 0;
        for (int i = lane(); i < TW; i += kWave) cc += __popc(inl ? lc.rem[(int64_t)c * TW + i] : gc.rem[(int64_t)c * TW + i]);
        nopt = wred_add(cc);
      }
      const bool spot = rs_member(L, crs, d.ctKey, d.spotBit), od = rs_member(L, crs, d.ctKey, d.odBit);
      flags |= (spot ? RB_HAS_SPOT : 0) | (od ? RB_HAS_OD : 0);
      if (allSched && nclaims == 1) {
        if (W.cflags & CF_PRICE_ERR) {
          action = CA_ERROR;
        } else {
          // filterByPrice into LDS scratch (s_cand), then filterOutSameType into s_rem
          nprice = inl ? price_filter(lc.rem + (int64_t)c * TW, s_cand, tpl, crs, spot, od, W.price)
                       : price_filter(gc.rem + (int64_t)c * TW, s_cand, tpl, crs, spot, od, W.price);
          wsync();
          for (int i = lane(); i < TW; i += kWave) o_price[i] = s_cand[i];
          if (nprice > 0 && !((W.cflags & CF_ALL_SPOT) && spot)) {
            action = CA_REPLACE;
            const bool narrowed = spot && od;  // [spot, on-demand] -> spot (consolidation.go:183-188)
            if (narrowed) flags |= RB_NARROWED;
            if (W.cflags & CF_MULTI) {
              const int tb = s_tbeg[tpl], nIT = s_tbeg[tpl + 1] - tb;
              double mx = __DBL_MAX__;
              for (int pos = lane(); pos < nIT; pos += kWave)
                if ((s_cand[pos >> 5] >> (pos & 31)) & 1u) {
                  const double v = W.st_price[D.tpl_its[tb + pos]];
                  if (v == v && v < mx) mx = v;
                }
              for (int off = 32; off >= 1; off >>= 1) {
                const double x = __shfl_xor(mx, off);
                mx = x < mx ? x : mx;
              }
              nsame = price_filter(s_cand, s_rem, tpl, crs, spot, od && !narrowed, mx);
              wsync();
              for (int i = lane(); i < TW; i += kWave) o_same[i] = s_rem[i];
            }
          }
        }
      }
    } else if (allSched && nclaims == 0 && err == KE_OK) {
      action = CA_DELETE;
    }
    {  // wave-wide stores of uniform values
      rec[RF_FLAGS] = flags;
      rec[RF_NCLAIMS] = nclaims;
      rec[RF_HOSTINCR] = hostCtr;
      rec[RF_TPL] = tpl;
      rec[RF_HOST] = host;
      rec[RF_ACTION] = action;
      rec[RF_NOPT] = nopt;
      rec[RF_NPRICE] = nprice;
      rec[RF_NSAME] = nsame;
      rec[RF_ERROR] = err;
      rec[RF_ALGB_LO] = (int32_t)(uint32_t)(uint64_t)algbytes;
      rec[RF_ALGB_HI] = (int32_t)(uint32_t)((uint64_t)algbytes >> 32);
    }
  }

  // A simulation's queue state (what k_init does for a Solve), written at its first push-back: until then the
  // queue is the NewQueue order itself and every pod is pending in its first relaxation state, which the window
  // reads directly (refill's `ident`) -- most simulations never push a pod back and skip this.
  __device__ __forceinline__ void sim_queue_init(int P) {
    for (int i = lane(); i < P; i += kWave) {
      W.queue[i] = i;
      W.pod_state[i] = W.sstart ? W.sstart[W.pod_map[i]] : D.pod_state0[W.pod_map[i]];
      W.pod_status[i] = ST_PENDING;
      W.pod_fstate[i] = -1;
      W.last_len[i] = 0;
    }
    hbm_release();
    wsync();
  }

  // --- 64-pod queue window: one gather per 64 pops, one entry per lane ------------------------
  // ident: no pod was pushed back yet in this Solve, so every pod is in its first relaxation state, its
  // staleness word is 0, a simulation's pending status is untouched and its queue is still the identity:
  // the window reads the pods' first-state copies (pod_s0) instead of going through W.pod_state and the
  // state tables (one dependent memory level fewer per refill).
  __device__ __forceinline__ void refill(Window<RT>& w, int qhead, int qlen, int P, bool pushed, bool ident) {
    if (pushed) hbm_release();  // queue pushes / relaxation states / staleness words have landed
    const int n = qlen < kWave ? qlen : kWave;
    if (lane() < n) {
      int pos = qhead + lane();
      if (pos >= P) pos -= P;
      w.p = SIM && ident ? pos : ld_sc1(W.queue + pos);
      w.g = SIM ? W.pod_map[w.p] : w.p;
      w.uid = SIM ? w.p : D.pod_uid[w.p];  // simulations reject duplicate UIDs: local index == UID
      if (ident) {
        w.s = D.pod_state0[w.g];
        w.ll = 0;
        const uint64_t KS_G* s0 = D.pod_s0 + 4 * (int64_t)w.g;
        w.tol0 = s0[0];
        w.tol1 = s0[1];
        w.toltpl = s0[2];
        w.flags = (int)(uint32_t)s0[3];
        w.st = ST_PENDING;
      } else {
        w.s = ld_sc1(W.pod_state + w.p);
        w.ll = ld_sc1(W.last_len + w.uid);
        w.flags = D.st_flags[w.s];
        w.st = SIM ? ld_sc1(W.pod_status + w.p) : 0;
        w.toltpl = D.st_toltpl[w.s];
        w.tol0 = D.st_tol[2 * w.s];
        w.tol1 = D.st_tol[2 * w.s + 1];
      }
      w.pf = SIM || (!LEAN && d.volAny) ? D.pod_flags[w.g] : 0;
      w.rl = LEAN && ident ? W.run_len[pos] : 1;
      w.hpc = D.pod_hpc[w.g];
      w.hpu = D.pod_hpu[w.g];
      w.hpo = D.pod_hpo[w.g];
      if (TOPO) {
        w.tsel = D.pod_gsel[(int64_t)w.g * d.GMW];
        w.tinv = D.pod_ginv[(int64_t)w.g * d.GMW];
        w.town = D.st_gown[(int64_t)w.s * d.GMW];
        w.trss = rs_present(D.st_rss + (int64_t)w.s * d.RSW);
      }
#pragma unroll
      for (int r = 0; r < RM; r++) {
        if (RT == 0 && r >= d.R) break;
        w.req[r] = D.pod_req[(int64_t)w.g * R() + r];
      }
    }
  }
};

// --- Multi-wave simulations (MW) ------------------------------------------------------------------
// A long simulation (a multi-node prefix re-schedules thousands of pods as one dependent chain) runs on a
// 4-wave workgroup: wave 0 runs the simulation as the single-wave kernel does, and the register window's
// 64-node blocks are spread over the waves (wave k holds nodes [64k, 64k + 64)).  The window steps of the
// resource-only fast path are split by block: a run of identical pods computes each block's per-node
// capacity and scan on its own wave, the blocks' totals meet in an LDS mailbox, and each wave commits its
// block's shares; a single pod's first fit is one ballot per block.  Two workgroup barriers per step
// (parameters posted / block results posted).  Everything else -- queue, node scan past the window,
// NodeClaims, templates, relaxation, the decision -- stays on wave 0.  The helpers keep their
// AllNonPendingPodsScheduled and algorithmic-byte contributions and hand them over at MW_EXIT.
enum MwCmd : int { MW_RUN = 1, MW_FIT = 2, MW_EXIT = 3 };
enum MwSlot : int {  // uint32 words of the mailbox (LDS, after the plan's dynamic LDS)
  MB_CMD = 0, MB_SEQ = 1, MB_M = 2, MB_FPF = 3, MB_FT0 = 4, MB_FT1 = 6, MB_FP = 8,  // FP: 2 words per resource
  MB_TOT = 40, MB_MASK = 48, MB_UMASK = 56, MB_ALL = 64, MB_AB = 72, MB_WORDS = 80
};
constexpr int kMwWaves = 4;
constexpr size_t kMwBytes = 4 * MB_WORDS;
__device__ __forceinline__ void mb_st64(LU32 mb, int i, uint64_t v) {
  mb[i] = (uint32_t)v;
  mb[i + 1] = (uint32_t)(v >> 32);
}
__device__ __forceinline__ uint64_t mb_ld64(LU32 mb, int i) { return (uint64_t)mb[i] | ((uint64_t)mb[i + 1] << 32); }
__device__ __forceinline__ void mw_barrier() { __syncthreads(); }

// One 64-node block of the register window, free capacity form (FREEW): as k_solve's window init.
template <int RM>
struct MwBlock {
  uint64_t tx, ty;
  int64_t av[RM];
  int nf;
};
template <int RM>
__device__ __forceinline__ void mw_block_init(MwBlock<RM>& b, const KsDev& D, LU32 s_rmv, int kb) {
  const KsDims& d = D.d;
  const int n = kb * kWave + lane(), c = n < d.N ? n : d.N - 1;
  b.tx = D.n_taint[2 * c];
  b.ty = D.n_taint[2 * c + 1];
  bool never = n >= d.N || ((s_rmv[c >> 5] >> (c & 31)) & 1u) != 0;
#pragma unroll
  for (int r = 0; r < RM; r++) {
    const int64_t a = D.n_avail[(int64_t)c * RM + r], q = D.n_req0[(int64_t)c * RM + r];
    never |= a < 0;
    b.av[r] = a - q;
  }
#pragma unroll
  for (int r = 0; r < RM; r++) b.av[r] = never ? INT64_MIN : b.av[r];
  b.nf = D.n_flags[c];
}
// A run of m identical pods: this lane's node capacity for it (as the single-wave run step).
template <int RM>
__device__ __forceinline__ int mw_run_cap(const MwBlock<RM>& b, int m, const int64_t* fp, const float* rq, uint64_t ft0,
                                          uint64_t ft1) {
  const bool tol = (((b.tx & ~ft0) | (b.ty & ~ft1)) == 0);
  int cap = tol ? m : 0;
#pragma unroll
  for (int r = 0; r < RM; r++) {
    const int c = run_cap(b.av[r], fp[r], rq[r], m);
    cap = c < cap ? c : cap;
  }
  return cap;
}
// The lane's share of the run given the pods the blocks before this one take (base); branch-free.
template <int RM>
__device__ __forceinline__ int mw_run_commit(MwBlock<RM>& b, int base, int cap, int incl, int m, const int64_t* fp) {
  const int p0 = base + incl - cap, room = m - p0;
  const int tk = room <= 0 ? 0 : (cap < room ? cap : room);
#pragma unroll
  for (int r = 0; r < RM; r++) b.av[r] -= (int64_t)tk * fp[r];
  return tk;
}
template <int RM>
__device__ __forceinline__ bool mw_fits(const MwBlock<RM>& b, const int64_t* fp, uint64_t ft0, uint64_t ft1) {
  bool ok = (((b.tx & ~ft0) | (b.ty & ~ft1)) == 0);
#pragma unroll
  for (int r = 0; r < RM; r++) ok &= fp[r] <= b.av[r];
  return ok;
}
// The first block (in node order) whose ballot holds a fit: (block, its ballot), uniform; -1 if none.
__device__ __forceinline__ int mw_first_fit(LU32 mb, uint64_t& mj) {
  int kj = -1;
  mj = 0;
#pragma unroll
  for (int q = 0; q < kMwWaves; q++) {
    const uint64_t mq = mb_ld64(mb, MB_MASK + 2 * q);
    const bool take = kj < 0 && mq != 0;
    kj = take ? q : kj;
    mj = take ? mq : mj;
  }
  mj = (uint64_t)uni64((int64_t)mj);
  return uni(kj);
}

// Waves 1..3 of an MW simulation: their window block, the mailbox loop, then their contributions.
template <int RM>
__device__ __forceinline__ void mw_helper(const KsDev& D, const KsWork& W, LU32 s_rmv, LU32 mb, int k) {
  const int R = D.d.R;
  mw_barrier();  // B0a: wave 0's prologue (the removed-node mask) is in LDS
  MwBlock<RM> b;
  mw_block_init<RM>(b, D, s_rmv, k);
  mb_st64(mb, MB_UMASK + 2 * k, wballot(b.nf & NF_UNUSABLE));  // wave-wide store of a uniform value
  mw_barrier();  // B0b
  bool winUnusable = false;
#pragma unroll
  for (int q = 0; q < kMwWaves; q++) winUnusable |= mb_ld64(mb, MB_UMASK + 2 * q) != 0;
  winUnusable = ub(winUnusable);
  bool all = true;
  int64_t ab = 0;
  int seen = 0;
  // every wave-0 step posts a new sequence number; a bound on the steps and a stale number (wave 0 gone
  // without MW_EXIT, which the kernel never does) both end the loop, so no helper can outlive wave 0
  const int maxOps = 4 * W.P + 64;
  for (int it = 0; it < maxOps; it++) {
    mw_barrier();  // B1: a step's parameters are posted
    const int seq = uni((int)mb[MB_SEQ]), cmd = uni((int)mb[MB_CMD]);
    if (seq == seen) return;
    seen = seq;
    if (cmd == MW_EXIT) {
      mb[MB_ALL + k] = all ? 1u : 0u;  // wave-wide stores of uniform values
      mb_st64(mb, MB_AB + 2 * k, (uint64_t)ab);
      mw_barrier();  // B2
      return;
    }
    const int m = uni((int)mb[MB_M]), fpf = uni((int)mb[MB_FPF]);
    const uint64_t ft0 = (uint64_t)uni64((int64_t)mb_ld64(mb, MB_FT0)), ft1 = (uint64_t)uni64((int64_t)mb_ld64(mb, MB_FT1));
    int64_t fp[RM];
#pragma unroll
    for (int r = 0; r < RM; r++) fp[r] = uni64((int64_t)mb_ld64(mb, MB_FP + 2 * r));
    if (cmd == MW_RUN) {
      float rq[RM];
#pragma unroll
      for (int r = 0; r < RM; r++) rq[r] = run_rcp(fp[r]);
      const int cap = mw_run_cap<RM>(b, m, fp, rq, ft0, ft1);
      const int incl = wscan_add(cap);
      mb[MB_TOT + k] = (uint32_t)rdl(incl, kWave - 1);  // wave-wide store of a uniform value
      mw_barrier();  // B2: every block's total is posted
      int base = 0;
#pragma unroll
      for (int q = 0; q < kMwWaves; q++) base += q < k ? (int)mb[MB_TOT + q] : 0;
      base = uni(base);
      const int tk = mw_run_commit<RM>(b, base, cap, incl, m, fp);
      const bool unusable = tk > 0 && (b.nf & NF_UNUSABLE);
      if (winUnusable && !(fpf & PF_PROVISIONABLE) && wballot(unusable)) all = false;
      ab += (int64_t)rdl(wscan_add(tk * (k * kWave + lane() + 1)), kWave - 1) * (16 * R + 16);
    } else {  // MW_FIT: a single pod's first fit over the window
      mb_st64(mb, MB_MASK + 2 * k, wballot(mw_fits<RM>(b, fp, ft0, ft1)));
      mw_barrier();  // B2: every block's ballot is posted
      uint64_t mj;
      const int kj = mw_first_fit(mb, mj);
      if (kj == k) {
        const bool own = lane() == ctz64(mj);
#pragma unroll
        for (int r = 0; r < RM; r++) b.av[r] -= own ? fp[r] : 0;
      }
    }
  }
}

template <int RT, bool TL, bool SIM, bool TOPO, bool LEAN, bool MW = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, MW ? 256 : 64))) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_solve(KsDev D, const KsWork* works, Plan pl) {
#define KS_BODY_WORK ((const KsWork KS_C*)works)[blockIdx.x]
#define KS_BODY_SMEM_DECL                                             \
  extern __shared__ __attribute__((aligned(16))) char smem_generic[]; \
  char KS_L* smem = (char KS_L*)smem_generic;
#include "ks_solve_body.inc"
#undef KS_BODY_WORK
#undef KS_BODY_SMEM_DECL
}

// The same body for one simulation of a mixed launch (k_sim_mixed): work item widx, LDS at smem_in.
template <int RT, bool TL, bool SIM, bool TOPO, bool LEAN, bool MW>
__device__ __forceinline__ void solve_body(const KsDev& D, const KsWork* works, const Plan& pl, int widx,
                                           char KS_L* smem_in) {
#define KS_BODY_WORK ((const KsWork KS_C*)works)[widx]
#define KS_BODY_SMEM_DECL char KS_L* smem = smem_in;
#include "ks_solve_body.inc"
#undef KS_BODY_WORK
#undef KS_BODY_SMEM_DECL
}

// One launch for a consolidation pass with long simulations (MW): workgroups [0, nmw) run the long ones on
// 4 waves, dispatched first; each later workgroup runs four short ones, one per wave, each in its own LDS
// slice (stride bytes).  The two kinds overlap on the chip, which two launches on two streams did not.
template <int RT>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 256))) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_sim_mixed(
    KsDev D, const KsWork* works, Plan pl, int nmw, int n, int stride) {
  extern __shared__ __attribute__((aligned(16))) char smem_mixed[];
  char KS_L* base = (char KS_L*)smem_mixed;
  if ((int)blockIdx.x < nmw) {
    solve_body<RT, true, true, false, true, true>(D, works, pl, (int)blockIdx.x, base);
  } else {
    const int wv = (int)(threadIdx.x >> 6);
    const int s = nmw + ((int)blockIdx.x - nmw) * kMwWaves + wv;
    if (s < n) solve_body<RT, true, true, false, true, false>(D, works, pl, s, base + (size_t)wv * stride);
  }
}

// Every translation unit instantiates one k_solve family (KS_TU 0: Solve, 1: Solve + topology,
// 2: simulations, 3: simulations + topology; ks_solve_topo.hip / ks_sim.hip / ks_sim_topo.hip
// include this file), so the four compile in parallel.
template <bool SIM, bool TOPO>
hipError_t launch_family(const KsDev& D, const KsWork* works_dev, int n, const Plan& pl, hipStream_t st) {
#define KS_LAUNCH(RT_, TL_, LEAN_) \
  hipLaunchKernelGGL((k_solve<RT_, TL_, SIM, TOPO, LEAN_>), dim3(n), dim3(kWave), pl.lds, st, D, works_dev, pl)
  if (n <= 0) return hipSuccess;  // e.g. a consolidation pass with no candidates: nothing to simulate
  const bool tl = pl.talloc != 0;
  // the lean instantiations exist for the common shapes only: 3 or 4 resources, LDS-resident tables
  const bool lean = !TOPO && D.d.lean && tl;
  switch (D.d.R) {
    case 3: if (lean) KS_LAUNCH(3, true, !TOPO); else if (tl) KS_LAUNCH(3, true, false); else KS_LAUNCH(3, false, false); break;
    case 4: if (lean) KS_LAUNCH(4, true, !TOPO); else if (tl) KS_LAUNCH(4, true, false); else KS_LAUNCH(4, false, false); break;
    default: if (tl) KS_LAUNCH(0, true, false); else KS_LAUNCH(0, false, false); break;
  }
#undef KS_LAUNCH
  return hipGetLastError();
}
using FamilyFn = hipError_t (*)(const KsDev&, const KsWork*, int, const Plan&, hipStream_t);
hipError_t launch_solve_plain(const KsDev& D, const KsWork* w, int n, const Plan& pl, hipStream_t st);
hipError_t launch_solve_topo(const KsDev& D, const KsWork* w, int n, const Plan& pl, hipStream_t st);
hipError_t launch_sims_plain(const KsDev& D, const KsWork* w, int n, const Plan& pl, hipStream_t st);
hipError_t launch_sims_topo(const KsDev& D, const KsWork* w, int n, const Plan& pl, hipStream_t st);
hipError_t launch_sims_mw(const KsDev& D, const KsWork* w, int n, const Plan& pl, hipStream_t st);
hipError_t launch_sims_mixed(const KsDev& D, const KsWork* w, int n, int nmw, const Plan& pl, hipStream_t st);

#if KS_TU == 1
hipError_t launch_solve_topo(const KsDev& D, const KsWork* w, int n, const Plan& pl, hipStream_t st) {
  return launch_family<false, true>(D, w, n, pl, st);
}
#elif KS_TU == 2
hipError_t launch_sims_plain(const KsDev& D, const KsWork* w, int n, const Plan& pl, hipStream_t st) {
  return launch_family<true, false>(D, w, n, pl, st);
}
// One mixed launch (k_sim_mixed): the first nmw simulations on 4-wave workgroups, the rest four to a workgroup.
// hipErrorNotSupported when four LDS slices do not fit a CU (the caller falls back to two launches).
hipError_t launch_sims_mixed(const KsDev& D, const KsWork* w, int n, int nmw, const Plan& pl, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const size_t stride = (pl.lds + 15) & ~(size_t)15;
  const size_t lds = std::max(pl.lds + kMwBytes, (size_t)kMwWaves * stride);
  if (D.d.G || !D.d.lean || !pl.talloc || D.d.N <= 0 || lds > 160 * 1024) return hipErrorNotSupported;
  const int grid = nmw + (n - nmw + kMwWaves - 1) / kMwWaves;
  const dim3 blk(kMwWaves * kWave);
  switch (D.d.R) {
    case 3: hipLaunchKernelGGL((k_sim_mixed<3>), dim3(grid), blk, lds, st, D, w, pl, nmw, n, (int)stride); break;
    case 4: hipLaunchKernelGGL((k_sim_mixed<4>), dim3(grid), blk, lds, st, D, w, pl, nmw, n, (int)stride); break;
    default: return hipErrorNotSupported;
  }
  return hipGetLastError();
}
// The long simulations on 4-wave workgroups (MW): resource-only pods with the window in free-capacity form
// (the LEAN instantiations); hipErrorNotSupported for other problems (the caller runs them single-wave).
hipError_t launch_sims_mw(const KsDev& D, const KsWork* w, int n, const Plan& pl, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (D.d.G || !D.d.lean || !pl.talloc || D.d.N <= 0 || pl.lds + kMwBytes > 160 * 1024) return hipErrorNotSupported;
  const dim3 blk(kMwWaves * kWave);
  switch (D.d.R) {
    case 3: hipLaunchKernelGGL((k_solve<3, true, true, false, true, true>), dim3(n), blk, pl.lds + kMwBytes, st, D, w, pl); break;
    case 4: hipLaunchKernelGGL((k_solve<4, true, true, false, true, true>), dim3(n), blk, pl.lds + kMwBytes, st, D, w, pl); break;
    default: return hipErrorNotSupported;
  }
  return hipGetLastError();
}
#elif KS_TU == 3
hipError_t launch_sims_topo(const KsDev& D, const KsWork* w, int n, const Plan& pl, hipStream_t st) {
  return launch_family<true, true>(D, w, n, pl, st);
}
#else
hipError_t launch_solve_plain(const KsDev& D, const KsWork* w, int n, const Plan& pl, hipStream_t st) {
  return launch_family<false, false>(D, w, n, pl, st);
}

// LDS plan.  Position-indexed state (order, pod count, template, headroom) bounds the NodeClaims
// per Solve (KO); claims [0, KL) also keep their template/requests/max/options/thresholds in LDS,
// the rest in HBM.  The instance-type tables go to LDS first when they leave room for 64 claims.
// One-Solve launches use the whole 160 KiB of a CU; batched simulations pass a smaller budget.
// wideKO: a Solve that created more NodeClaims than the default plan holds is re-planned with 64 LDS-resident
// claims and the rest of the LDS given to claim positions: level 1 keeps the instance-type tables in LDS, level 2
// (when 1 still holds too few) moves them to HBM.  C3 (844 NodeClaims): 56.0k -> 59.1k pods/s at level 1.
static Plan make_plan_live(const KsDims& d, size_t budget, bool sim, int wideKO, bool live);
Plan make_plan(const KsDims& d, size_t budget, bool sim, int wideKO) {
  // The live node list serves the non-LEAN Solve instantiations with a register window (RT 3 or 4, launch_family):
  // a lean problem runs LEAN whenever its instance-type tables fit in LDS (talloc), so its plan reserves the list
  // only when they do not.
  const bool rt = d.R == 3 || d.R == 4;
  if (sim || !rt) return make_plan_live(d, budget, sim, wideKO, false);
  if (d.lean) {
    const Plan lean = make_plan_live(d, budget, sim, wideKO, false);
    if (lean.talloc) return lean;
  }
  return make_plan_live(d, budget, sim, wideKO, true);
}

static Plan make_plan_live(const KsDims& d, size_t budget, bool sim, int wideKO, bool live) {
  auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
  Plan pl{};
  const size_t R = d.R, TW = d.TW, tot = d.totalTplIts;
  const size_t fixed = r16(sizeof(KeyMeta) * d.NK) + r16(4 * (size_t)(d.NTPL + 1)) + r16(8 * (size_t)(d.NPOOL + 1) * R) +
                       2 * r16(4 * (size_t)d.RSW) + 5 * r16(4 * TW + 8) + 16 * 16 + (d.volAny ? 48 : 0) +
                       (sim ? 4 * r16(4 * (size_t)((d.N + 31) / 32)) : d.fnOn ? r16(4 * (size_t)((d.N + 31) / 32)) : 0) +
                       (d.G ? r16(4 * (size_t)d.G * TGM_WORDS) + r16(4 * (size_t)d.G) + 2 * r16(4 * (size_t)d.RSW) +
                                  (d.GMW > 1 ? r16(8 * (size_t)GS_N * d.GMW) : 0) +
                                  (sim ? r16(4 * (size_t)((d.tgCntWords - d.tgSmall + 31) / 32)) + 4 * kTdwKeys * kTdw : 0)
                              : 0);
  const size_t posB = 16 + 8 * R;                        // order, okey, ptpl, phead (+ rounding)
  const size_t clmB = 16 + 16 * R + 4 * TW + 4 * R;      // tpl, cnt, req, max, rem, thr (+ rounding)
  const size_t slack = 10 * 16;                          // per-array 16-byte rounding
  const size_t tallocB = r16(8 * tot * R);
  const size_t tsortB = r16(8 * tot * R) + r16(4 * tot * R);
  size_t avail = budget > fixed + slack ? budget - fixed - slack : 0;
  // The topology count table's LDS-resident prefix: the small-key groups; a Solve also keeps the
  // hostname groups there when the whole table takes at most a quarter of what is left (a simulation's
  // hostname counts are copy-on-write over the shared HBM table instead).
  pl.tcl = d.G ? d.tgSmall : 0;
  if (d.G && !sim && 4 * (size_t)d.tgCntWords <= avail / 4) pl.tcl = d.tgCntWords;
  const size_t tclB = r16(4 * (size_t)pl.tcl);
  avail = avail > tclB ? avail - tclB : 0;
  // the node domain table likewise (a Solve's first-fit scan reads it for every node and matching group)
  const size_t tdWords = (size_t)d.TK * (size_t)d.N;
  pl.tdl = d.G && !sim && tdWords > 0 && 4 * tdWords <= avail / 4 ? (int32_t)tdWords : 0;
  const size_t tdlB = r16(4 * (size_t)pl.tdl);
  avail = avail > tdlB ? avail - tdlB : 0;
  // a Solve's live node list: the existing nodes past the register window passing Fits for the current
  // request vector (ks_solve_body.inc)
  pl.livl = live && d.N > 0 && !d.negReq && !d.tgUnlab && 4 * (size_t)d.N <= avail / 4 ? d.N : 0;
  const size_t livB = r16(4 * (size_t)pl.livl);
  avail = avail > livB ? avail - livB : 0;
  // The threshold filter needs the sorted lists only without negative requests.
  const size_t tablesB = tallocB + (d.negReq ? 0 : tsortB);
  pl.talloc = (wideKO < 2 && tablesB + 64 * (posB + clmB) <= avail) ? 1 : 0;
  pl.tsort = pl.talloc && !d.negReq;
  if (pl.talloc) avail -= tablesB;
  const size_t kAll = avail / (posB + clmB);
  size_t ko, kl;
  if (kAll >= (size_t)d.Kcap) {
    ko = kl = d.Kcap;
  } else if (wideKO) {  // 64 LDS-resident claims, the rest to positions (C3: 8-96 claims measured within 1.5 %)
    kl = std::min<size_t>(64, kAll);
    ko = std::min((size_t)d.Kcap, (avail - kl * clmB) / posB);
  } else {  // half the LDS to positions, half to claim state
    ko = std::min((size_t)d.Kcap, std::max(kAll, avail / 2 / posB));
    kl = std::min(ko, (avail - ko * posB) / clmB);
  }
  pl.KO = (int)ko;
  pl.KL = (int)kl;
  pl.lds = fixed + tclB + tdlB + livB + 3 * r16(4 * ko) + r16(8 * ko * R) + 2 * r16(4 * kl) + 2 * r16(8 * kl * R) + r16(4 * kl * TW) +
           r16(4 * kl * R) + (pl.tsort ? tsortB : 0) + (pl.talloc ? tallocB : 0);
  return pl;
}

void launch_feasibility(const KsDev& D, hipStream_t st) {
  const int rows = D.d.S * D.d.NTPL;
  if (D.d.TW <= 32) {  // two rows per wave step
    const int blocks = std::min(2048, (rows + 7) / 8);
    hipLaunchKernelGGL(k_feasibility<32>, dim3(blocks), dim3(256), 0, st, D);
  } else {
    const int blocks = std::min(2048, (rows + 3) / 4);
    hipLaunchKernelGGL(k_feasibility<64>, dim3(blocks), dim3(256), 0, st, D);
  }
}

void launch_feasibility_nodes(const KsDev& D, hipStream_t st) {
  const int nbx = (D.d.N + 255) / 256;
  hipLaunchKernelGGL(k_feasibility_nodes, dim3(D.d.FNR * nbx), dim3(256), 0, st, D, nbx);
}

hipError_t queue_sort(const KsDev& D, uint64_t* keys, int32_t* vals, void* temp, size_t tempBytes, int32_t* out,
                      hipStream_t st);
hipError_t sim_run_lengths(const int32_t* podmap, const int32_t* entry_sim, const int64_t* pod_req, const uint64_t* pod_s0,
                           const int32_t* pod_flags, int R, int n, uint64_t* words, int32_t* run_len, hipStream_t st,
                           bool strict);

// One ks_solve: queue sort -> workspace init -> [mid event] -> k_solve (all on one stream).
// Topology problems get their own instantiation: the group state would otherwise occupy SGPRs (and
// their spills) across the whole commit loop of every topology-free Solve.
// fixed_order: NewQueue's order computed on the host (pods tying on the whole sort key), no radix sort.
// run_len / run_words (LEAN problems): the identical pods left in each queue position's run, which the LEAN
// Solve's claim runs read while nothing has been pushed back (they may then reach past the queue window).
hipError_t launch_solve(const KsDev& D, const KsWork* works_dev, int nrep, const Plan& pl, int32_t* qorder,
                        uint64_t* skeys, int32_t* svals, void* stemp, size_t stempBytes, hipStream_t st,
                        hipEvent_t mid, const int32_t* fixed_order, hipEvent_t* feas, int32_t* run_len,
                        uint64_t* run_words) {
  if (pl.lds > 160 * 1024) return hipErrorInvalidValue;
  if (!fixed_order) {
    hipError_t e = queue_sort(D, skeys, svals, stemp, stempBytes, qorder, st);
    if (e != hipSuccess) return e;
  }
  if (D.d.lean && run_len && run_words) {
    hipError_t e = sim_run_lengths(fixed_order ? fixed_order : qorder, nullptr, D.pod_req, D.pod_s0, D.pod_flags, D.d.R,
                                   D.d.P, run_words, run_len, st, true);
    if (e != hipSuccess) return e;
  }
  if (D.d.fmOn) {
    if (feas) (void)hipEventRecord(feas[0], st);
    launch_feasibility(D, st);
    if (feas) (void)hipEventRecord(feas[1], st);
  }
  if (D.d.fnOn) {
    if (feas) (void)hipEventRecord(feas[2], st);
    launch_feasibility_nodes(D, st);
    if (feas) (void)hipEventRecord(feas[3], st);
  }
  hipLaunchKernelGGL(k_init, dim3(512), dim3(256), 0, st, D, works_dev, nrep,
                     fixed_order ? fixed_order : (const int32_t*)qorder);
  if (mid) (void)hipEventRecord(mid, st);
  return (D.d.G ? launch_solve_topo : launch_solve_plain)(D, works_dev, nrep, pl, st);
}

// A batch of consolidation simulations (one wavefront each); their pod_map lists must already be
// in NewQueue order (sim_queue_sort).
hipError_t launch_sims(const KsDev& D, const KsWork* works_dev, int nsims, const Plan& pl, hipStream_t st) {
  if (pl.lds > 160 * 1024) return hipErrorInvalidValue;
  if (nsims <= 0) return hipSuccess;
  if (D.d.fmOn) launch_feasibility(D, st);
  if (D.d.fnOn) launch_feasibility_nodes(D, st);
  return (D.d.G ? launch_sims_topo : launch_sims_plain)(D, works_dev, nsims, pl, st);
}
bool sims_mw_supported(const KsDev& D, const Plan& pl) {
  return !D.d.G && D.d.lean && pl.talloc && D.d.N > 0 && pl.lds + kMwBytes <= 160 * 1024 && (D.d.R == 3 || D.d.R == 4);
}
// The first nmw simulations (the long ones) on 4-wave workgroups on st2, the rest single-wave on st,
// concurrently: st2 waits for st's work so far (fork), st waits for st2 at the end (join).
hipError_t launch_sims_split(const KsDev& D, const KsWork* works_dev, int nsims, int nmw, const Plan& pl, hipStream_t st,
                             hipStream_t st2, hipEvent_t fork, hipEvent_t join) {
  if (nmw <= 0 || !sims_mw_supported(D, pl)) return launch_sims(D, works_dev, nsims, pl, st);
  if (pl.lds > 160 * 1024) return hipErrorInvalidValue;
  if (D.d.fmOn) launch_feasibility(D, st);
  if (D.d.fnOn) launch_feasibility_nodes(D, st);
  // one launch when four simulations' LDS fit a workgroup: the long ones are dispatched first
  const hipError_t em = launch_sims_mixed(D, works_dev, nsims, nmw, pl, st);
  if (em != hipErrorNotSupported) return em;
  hipError_t e = hipEventRecord(fork, st);
  if (e == hipSuccess) e = hipStreamWaitEvent(st2, fork, 0);
  if (e == hipSuccess) e = launch_sims_mw(D, works_dev, nmw, pl, st2);
  if (e == hipSuccess && nsims > nmw) e = launch_sims_plain(D, works_dev + nmw, nsims - nmw, pl, st);
  if (e == hipSuccess) e = hipEventRecord(join, st2);
  if (e == hipSuccess) e = hipStreamWaitEvent(st, join, 0);
  return e;
}
#endif

}  // namespace ks
