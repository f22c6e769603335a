// ks_solve.hip — MI355X (gfx950) kernels for Scheduler.Solve.
//
// One Solve = one 64-lane wavefront (one workgroup).  The reference's Solve is a sequential commit
// chain (scheduler.go:140-189: every placement depends on all earlier ones), so the chain stays in
// one wave with wave-uniform control flow and no inter-wave synchronisation; the data-parallel
// parts of each step map onto the 64 lanes:
//   - existing-node first-fit (scheduler.go:240-244)   lane per node, ballot + ffs picks the first
//   - in-flight NodeClaim scan (scheduler.go:250-254)  lane per sorted position: a quick reject
//     (template taints, requests + pod <= max Allocatable of the remaining options, Compatible)
//     then a wave-cooperative NodeClaim.Add on candidates in order (nodeclaim.go:65-119)
//   - instance-type filter (nodeclaim.go:225-260)      lane per template IT position, ballots build
//     the remaining-options bitset and the six filterResults flags in one pass
//   - new NodeClaim per template (scheduler.go:258-283) incl. limits (filterByRemainingResources,
//     subtractMax)
// Latency is the bound (the chain is sequential), so the state every step touches lives in LDS:
// the claim order and pod counts, each claim's template / requests / max-Allocatable / options
// bitset (for the first Plan::KL claims), the templates' instance-type Allocatable tables, and a
// 64-pod window of queue entries fetched with one coalesced gather per 64 pops.  HBM holds the
// cold state (requirement records, existing nodes, overflow claims) and the commit log.
// Independent Solves (replicas, consolidation simulations) are independent workgroups, so a launch
// of thousands of them fills the 256 CUs.  Nothing here is a dense contraction: no MFMA.
#include <hip/hip_runtime.h>

#include "ks_gosort.h"
#include "ks_problem.h"
#include "ks_reqset.h"

namespace ks {

__device__ __forceinline__ int lane() { return (int)threadIdx.x; }
__device__ __forceinline__ uint64_t wballot(bool p) { return __ballot(p ? 1 : 0); }
__device__ __forceinline__ int ctz64(uint64_t m) { return __builtin_ctzll(m); }
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
// One-wave workgroup: s_barrier is cheap and orders LDS traffic between lanes.
__device__ __forceinline__ void wsync() { __syncthreads(); }

#ifdef KS_PHASE_STATS
#define PH_BEGIN(v) uint64_t v = __builtin_amdgcn_s_memtime()
#define PH_END(v, slot) cyc[slot] += __builtin_amdgcn_s_memtime() - v
#else
#define PH_BEGIN(v)
#define PH_END(v, slot)
#endif

// ------------------------------------------------------------------------------------------------
// Init: per-replica workspace state (copies of the resident initial state), one grid-stride pass.
// ------------------------------------------------------------------------------------------------
__global__ void k_init(KsDev D, const KsWork* works, int nrep, const int32_t* qorder) {
  const KsDims d = D.d;
  const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t gsz = (int64_t)gridDim.x * blockDim.x;
  for (int r = 0; r < nrep; r++) {
    const KsWork W = works[r];
    for (int64_t i = gtid; i < (int64_t)d.N * d.R; i += gsz) W.n_req[i] = D.n_req0[i];
    for (int64_t i = gtid; i < (int64_t)d.N * d.RSW; i += gsz) W.n_rs[i] = D.n_rs0[i];
    for (int64_t i = gtid; i < d.P; i += gsz) {
      W.queue[i] = qorder[i];
      W.pod_state[i] = D.pod_state0[i];
      W.pod_status[i] = ST_PENDING;
      W.pod_fstate[i] = -1;
    }
    for (int64_t i = gtid; i < d.NU; i += gsz) W.last_len[i] = 0;
    for (int64_t i = gtid; i < (int64_t)d.NPOOL * d.R; i += gsz) W.pool_rem[i] = D.pool_rem0[i];
    for (int64_t i = gtid; i < CT_NCOUNTERS; i += gsz) W.counters[i] = 0;
  }
}

// ------------------------------------------------------------------------------------------------
// Solve
// ------------------------------------------------------------------------------------------------
struct Solver {
  const KsDev& D;
  const KsDims& d;
  const KsWork& W;
  const Plan& pl;
  ReqLayout L;
  // LDS-resident state
  int32_t* s_order;   // [KO] s.newNodeClaims as claim ids
  int32_t* s_okey;    // [KO] len(Pods) of the claim at each position
  int32_t* s_ctpl;    // [KL]
  int64_t* s_creq;    // [KL][R]
  int64_t* s_cmax;    // [KL][R]
  uint32_t* s_crem;   // [KL][TW]
  int64_t* s_talloc;  // [totalTplIts][R] (pl.talloc)
  int32_t* s_tbeg;    // [NTPL+1]
  uint32_t* s_rs;     // [RSW] candidate requirements
  uint32_t* s_rem;    // [TW+2] candidate options
  uint32_t* s_cand;   // [TW+2] limit-filtered template options
  int64_t* s_req;     // [kMaxR] candidate requests
  // 64-pod window
  int32_t *w_p, *w_uid, *w_s, *w_flags;
  uint64_t *w_ll, *w_tol;
  int64_t* w_req;
  int64_t algbytes = 0;

  __device__ Solver(const KsDev& D_, const KsWork& W_, const Plan& p_) : D(D_), d(D_.d), W(W_), pl(p_) {}

  // claim-state accessors: LDS for c < KL, HBM otherwise
  __device__ int ctpl(int c) const { return c < pl.KL ? s_ctpl[c] : W.c_tpl[c]; }
  __device__ int64_t* creq(int c) const { return c < pl.KL ? s_creq + (int64_t)c * d.R : W.c_req + (int64_t)c * d.R; }
  __device__ int64_t* cmax(int c) const { return c < pl.KL ? s_cmax + (int64_t)c * d.R : W.c_max + (int64_t)c * d.R; }
  __device__ uint32_t* crem(int c) const { return c < pl.KL ? s_crem + (int64_t)c * d.TW : W.c_rem + (int64_t)c * d.TW; }
  __device__ const int64_t* talloc(int gpos) const {  // Allocatable of template position gpos
    return pl.talloc ? s_talloc + (int64_t)gpos * d.R : D.it_alloc + (int64_t)D.tpl_its[gpos] * d.R;
  }

  __device__ bool fits(const int64_t* req, const int64_t* alloc) const {  // resources.go:162-175
    for (int r = 0; r < d.R; r++) {
      const int64_t a = alloc[r];
      if (a < 0 || req[r] > a) return false;
    }
    return true;
  }
  __device__ bool has_offering(int it, const uint32_t* rs) const {  // nodeclaim.go:270-278
    const int b = D.it_off_beg[it], e = D.it_off_beg[it + 1];
    for (int o = b; o < e; o++)
      if (rs_member(L, rs, d.zoneKey, D.off_zone[o]) && rs_member(L, rs, d.ctKey, D.off_ct[o])) return true;
    return false;
  }
  __device__ static bool tolerates(const uint64_t* taint, const uint64_t* tol) {
    return ((taint[0] & ~tol[0]) | (taint[1] & ~tol[1])) == 0;
  }
  __device__ void copy_words(uint32_t* dst, const uint32_t* src, int n) const {
    for (int i = lane(); i < n; i += kWave) dst[i] = src[i];
  }
  __device__ void store_bits(uint32_t* dst, int base, uint64_t m) const {
    if (lane() == 0) {
      dst[base >> 5] = (uint32_t)m;
      if ((base >> 5) + 1 < d.TW) dst[(base >> 5) + 1] = (uint32_t)(m >> 32);
    }
  }

  // --- existing nodes (ExistingNode.Add, existingnode.go:64-124) -------------------------------
  __device__ bool node_ok(int n, int s, int sflags, const int64_t* pod, const uint64_t* tol) const {
    if (!tolerates(D.n_taint + 2 * n, tol)) return false;
    const int64_t* av = D.n_avail + (int64_t)n * d.R;
    const int64_t* rq = W.n_req + (int64_t)n * d.R;
    for (int r = 0; r < d.R; r++) {
      const int64_t a = av[r];
      if (a < 0 || rq[r] + pod[r] > a) return false;
    }
    if (sflags & SF_HAS_KEYS)  // strict Compatible: no AllowUndefinedWellKnownLabels
      return rs_compatible(L, W.n_rs + (int64_t)n * d.RSW, D.st_rs + (int64_t)s * d.RSW, 0);
    return true;
  }

  // --- NodeClaim quick reject: necessary conditions of NodeClaim.Add ----------------------------
  __device__ bool claim_quick(int c, int s, int sflags, const int64_t* pod, const uint64_t* tol) const {
    const int t = ctpl(c);
    if (!tolerates(D.tpl_taint + 2 * t, tol)) return false;
    const int64_t* rq = creq(c);
    const int64_t* mx = cmax(c);
    for (int r = 0; r < d.R; r++)
      if (rq[r] + pod[r] > mx[r]) return false;
    if (sflags & SF_HAS_KEYS)
      return rs_compatible(L, W.c_rs + (int64_t)c * d.RSW, D.st_rs + (int64_t)s * d.RSW, d.allowWK);
    return true;
  }

  // --- wave-cooperative NodeClaim.Add on claim c: builds s_rs / s_req / s_rem; true if any IT remains
  __device__ bool claim_full(int c, int s, int sflags, const int64_t* pod) {
    bool changed = false;
    if (sflags & SF_HAS_KEYS) {
      const uint32_t* crs = W.c_rs + (int64_t)c * d.RSW;
      copy_words(s_rs, crs, d.RSW);
      wsync();
      if (lane() == 0) rs_add(L, s_rs, D.st_rs + (int64_t)s * d.RSW);
      wsync();
      changed = (sflags & SF_TOUCHES_IT_KEYS) && !rs_equal_keys(L, s_rs, crs, d.itKeys);
      algbytes += 8 * d.RSW;
    }
    const int t = ctpl(c);
    const int64_t* crq = creq(c);
    if (lane() < d.R) s_req[lane()] = crq[lane()] + pod[lane()];
    wsync();
    const int tb = s_tbeg[t], nIT = s_tbeg[t + 1] - tb;
    const uint32_t* rem = crem(c);
    uint64_t any = 0;
    int scanned = 0;
    for (int base = 0; base < nIT; base += kWave) {
      const int wi = base >> 5;
      const uint64_t bits = (uint64_t)rem[wi] | (wi + 1 < d.TW ? (uint64_t)rem[wi + 1] << 32 : 0ull);
      uint64_t m = 0;
      if (bits) {
        const int pos = base + lane();
        bool ok = (bits >> lane()) & 1ull;
        if (ok) {
          ok = fits(s_req, talloc(tb + pos));
          if (ok && changed) {
            const int it = D.tpl_its[tb + pos];
            ok = rs_intersects(L, D.it_rs + (int64_t)it * d.RSW, s_rs) && has_offering(it, s_rs);
          }
        }
        m = wballot(ok);
        scanned += __popcll(bits);
      }
      store_bits(s_rem, base, m);
      any |= m;
    }
    algbytes += 4 * d.TW + 16 * d.R + (int64_t)scanned * 8 * d.R;
    wsync();
    return any != 0;
  }

  // max Allocatable per resource over the options in `bits` (quick-reject bound)
  __device__ void update_max(int c, const uint32_t* bits, int t) {
    const int tb = s_tbeg[t], nIT = s_tbeg[t + 1] - tb;
    int64_t* mx = cmax(c);
    for (int r = 0; r < d.R; r++) {
      int64_t m = INT64_MIN;
      for (int pos = lane(); pos < nIT; pos += kWave)
        if ((bits[pos >> 5] >> (pos & 31)) & 1u) {
          const int64_t a = talloc(tb + pos)[r];
          m = a > m ? a : m;
        }
      for (int off = 32; off >= 1; off >>= 1) {
        const int64_t o = __shfl_xor(m, off);
        m = o > m ? o : m;
      }
      if (lane() == 0) mx[r] = m;
    }
    wsync();
  }

  __device__ void commit_claim(int c, int pos, int p, int sflags, int& nlog) {
    int64_t* crq = creq(c);
    if (lane() < d.R) crq[lane()] = s_req[lane()];
    if (sflags & SF_HAS_KEYS) copy_words(W.c_rs + (int64_t)c * d.RSW, s_rs, d.RSW);
    uint32_t* rem = crem(c);
    bool diff = false;
    for (int i = lane(); i < d.TW; i += kWave) {
      diff |= rem[i] != s_rem[i];
      rem[i] = s_rem[i];
    }
    if (lane() == 0) {
      s_okey[pos] += 1;
      W.log_pod[nlog] = p;
      W.log_tgt[nlog] = c;
      W.pod_status[p] = ST_SCHEDULED;
    }
    nlog++;
    // HBM-resident claim state (requirements, overflow claims) is re-read by other lanes
    if ((sflags & SF_HAS_KEYS) || c >= pl.KL) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    wsync();
    if (wballot(diff)) update_max(c, s_rem, ctpl(c));
    algbytes += 16 * d.R + 4 * d.TW;
  }

  // --- new NodeClaim from each template in order (scheduler.go:258-283) -----------------------
  // Returns 1 placed, 0 failed (fail codes recorded), 2 no templates (add() returns nil), -1 cap.
  __device__ int try_templates(int p, int s, int sflags, const int64_t* pod, const uint64_t* tol, int& nclaims,
                               int& nlog, int& hostCtr) {
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
          const int64_t* cap = D.it_cap + (int64_t)D.tpl_its[tb + pos] * d.R;
          const int64_t* rem = W.pool_rem + (int64_t)pool * d.R;
          for (int r = 0; r < d.R; r++)
            if (((mask >> r) & 1u) && cap[r] > rem[r]) ok = false;
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
        if (!tolerates(D.tpl_taint + 2 * t, tol)) {
          code = FC_TAINTS;
        } else {
          copy_words(s_rs, D.tpl_rs + (int64_t)t * d.RSW, d.RSW);
          wsync();
          bool ok = true;
          if (sflags & SF_HAS_KEYS) {
            ok = rs_compatible(L, s_rs, D.st_rs + (int64_t)s * d.RSW, d.allowWK);
            if (ok && lane() == 0) rs_add(L, s_rs, D.st_rs + (int64_t)s * d.RSW);
            wsync();
          }
          if (!ok) {
            code = FC_COMPAT;
          } else {
            if (lane() < d.R) s_req[lane()] = D.tpl_daemon[(int64_t)t * d.R + lane()] + pod[lane()];
            wsync();
            uint32_t flags = 0;
            uint64_t any = 0;
            for (int base = 0; base < nIT; base += kWave) {
              const int pos = base + lane();
              const bool in = pos < nIT && ((s_cand[pos >> 5] >> (pos & 31)) & 1u);
              bool ic = false, fi = false, of = false;
              if (in) {
                const int it = D.tpl_its[tb + pos];
                ic = rs_intersects(L, D.it_rs + (int64_t)it * d.RSW, s_rs);
                fi = fits(s_req, talloc(tb + pos));
                of = has_offering(it, s_rs);
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
            algbytes += 4 * d.RSW + (int64_t)nIT * (8 * d.R + 4 * d.RSW + 16);
            wsync();
            if (any == 0) {
              code = FC_NO_IT | (flags << 8);
            } else {
              if (nclaims >= pl.KO) return -1;
              const int c = nclaims++;
              copy_words(W.c_rs + (int64_t)c * d.RSW, s_rs, d.RSW);
              copy_words(crem(c), s_rem, d.TW);
              if (lane() < d.R) creq(c)[lane()] = s_req[lane()];
              if (lane() == 0) {
                if (c < pl.KL) s_ctpl[c] = t;
                W.c_tpl[c] = t;
                W.c_host[c] = hostid;
                s_order[c] = c;
                s_okey[c] = 1;
                W.log_pod[nlog] = p;
                W.log_tgt[nlog] = c;
                W.pod_status[p] = ST_SCHEDULED;
              }
              nlog++;
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
              wsync();
              update_max(c, s_rem, t);
              if (pool >= 0) {  // subtractMax (scheduler.go:347-362)
                const uint32_t mask = D.pool_mask[pool];
                for (int r = 0; r < d.R; r++) {
                  if (!((mask >> r) & 1u)) continue;
                  int64_t m = INT64_MIN;
                  for (int pos = lane(); pos < nIT; pos += kWave)
                    if ((s_rem[pos >> 5] >> (pos & 31)) & 1u) {
                      const int64_t v = D.it_cap[(int64_t)D.tpl_its[tb + pos] * d.R + r];
                      m = v > m ? v : m;
                    }
                  for (int off = 32; off >= 1; off >>= 1) {
                    const int64_t o = __shfl_xor(m, off);
                    m = o > m ? o : m;
                  }
                  if (lane() == 0) W.pool_rem[(int64_t)pool * d.R + r] -= m;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
              }
              wsync();
              return 1;
            }
          }
        }
      }
      if (lane() == 0) {
        W.fail_code[(int64_t)p * d.NTPL + t] = code;
        W.fail_host[(int64_t)p * d.NTPL + t] = hostid;
      }
    }
    return 0;
  }

  // --- s.newNodeClaims re-sort (scheduler.go:247) --------------------------------------------------
  __device__ void sort_claims(int n, int64_t& sorts, int64_t& slow) {
    bool desc = false;
    for (int base = 0; base < n; base += kWave) {
      const int j = base + lane();
      const bool dd = j > 0 && j < n && s_okey[j] < s_okey[j - 1];
      desc |= wballot(dd) != 0;
    }
    sorts++;
    if (!desc) return;  // non-decreasing: pdqsort performs no swap
    slow++;
    if (lane() == 0) {
      GoSortExact g{GoSort{s_okey, s_order}};
      g.run(n);
    }
    wsync();
  }

  // --- 64-pod queue window -------------------------------------------------------------------------
  __device__ void refill(int qhead, int qlen, int P) {
    const int n = qlen < kWave ? qlen : kWave;
    if (lane() < n) {
      int pos = qhead + lane();
      if (pos >= P) pos -= P;
      const int p = W.queue[pos];
      const int uid = D.pod_uid[p];
      const int s = W.pod_state[p];
      w_p[lane()] = p;
      w_uid[lane()] = uid;
      w_s[lane()] = s;
      w_ll[lane()] = W.last_len[uid];
      w_flags[lane()] = D.st_flags[s];
      w_tol[2 * lane()] = D.st_tol[2 * s];
      w_tol[2 * lane() + 1] = D.st_tol[2 * s + 1];
      for (int r = 0; r < d.R; r++) w_req[lane() * d.R + r] = D.pod_req[(int64_t)p * d.R + r];
    }
    wsync();
  }
};

__global__ __launch_bounds__(64) void k_solve(KsDev D, const KsWork* works, Plan pl) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const KsWork W = works[blockIdx.x];
  const KsDims& d = D.d;
  Solver S(D, W, pl);
  char* sp = smem;
  auto take = [&](size_t bytes) { char* r = sp; sp += (bytes + 15) & ~(size_t)15; return r; };
  KeyMeta* s_keys = (KeyMeta*)take(sizeof(KeyMeta) * d.NK);
  S.s_order = (int32_t*)take(4 * (size_t)pl.KO);
  S.s_okey = (int32_t*)take(4 * (size_t)pl.KO);
  S.s_ctpl = (int32_t*)take(4 * (size_t)pl.KL);
  S.s_creq = (int64_t*)take(8 * (size_t)pl.KL * d.R);
  S.s_cmax = (int64_t*)take(8 * (size_t)pl.KL * d.R);
  S.s_crem = (uint32_t*)take(4 * (size_t)pl.KL * d.TW);
  S.s_talloc = (int64_t*)take(pl.talloc ? 8 * (size_t)d.totalTplIts * d.R : 0);
  S.s_tbeg = (int32_t*)take(4 * (size_t)(d.NTPL + 1));
  S.s_rs = (uint32_t*)take(4 * (size_t)d.RSW);
  S.s_rem = (uint32_t*)take(4 * (size_t)d.TW + 8);
  S.s_cand = (uint32_t*)take(4 * (size_t)d.TW + 8);
  S.s_req = (int64_t*)take(8 * kMaxR);
  S.w_p = (int32_t*)take(4 * kWave);
  S.w_uid = (int32_t*)take(4 * kWave);
  S.w_s = (int32_t*)take(4 * kWave);
  S.w_flags = (int32_t*)take(4 * kWave);
  S.w_ll = (uint64_t*)take(8 * kWave);
  S.w_tol = (uint64_t*)take(16 * kWave);
  S.w_req = (int64_t*)take(8 * (size_t)kWave * d.R);
  for (int i = lane(); i < d.NK * (int)(sizeof(KeyMeta) / 4); i += kWave)
    ((uint32_t*)s_keys)[i] = ((const uint32_t*)D.keys)[i];
  for (int i = lane(); i <= d.NTPL; i += kWave) S.s_tbeg[i] = D.tpl_it_beg[i];
  if (pl.talloc)
    for (int i = lane(); i < d.totalTplIts * d.R; i += kWave)
      S.s_talloc[i] = D.it_alloc[(int64_t)D.tpl_its[i / d.R] * d.R + i % d.R];
  S.L.nkeys = d.NK;
  S.L.W = d.W;
  S.L.NB = d.NB;
  S.L.HDR = d.HDR;
  S.L.RSW = d.RSW;
  S.L.keys = s_keys;
  S.L.wordValid = D.wordValid;
  S.L.vIsInt = D.vIsInt;
  S.L.vInt = D.vInt;
  wsync();

  const int P = d.P;
  int nclaims = 0, nlog = 0, hostCtr = d.hostnameSeed;
  uint32_t epoch = 1;
  int qhead = 0, qlen = P;
  int wn = 0, wi = 0;  // window size / next index
  int64_t pops = 0, sorts = 0, slow = 0, windows = 0;
  // Every pop either places a pod, relaxes it, or marks it stale; the reference's queue can cycle
  // O(P^2) in adversarial inputs, far beyond any realistic batch.  Bound it so a logic error ends the
  // kernel with KE_ITER_CAP instead of hanging the device.
  const int64_t popCap = (int64_t)64 * (d.S + P) + 100000;
  int err = KE_OK;
#ifdef KS_PHASE_STATS
  uint64_t cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t tstart = __builtin_amdgcn_s_memtime();
#endif

  while (qlen > 0) {
    PH_BEGIN(t0);
    if (wi == wn) {
      S.refill(qhead, qlen, P);
      wn = qlen < kWave ? qlen : kWave;
      wi = 0;
      windows++;
    }
    // Queue.Pop (queue.go:46-61)
    const int p = uni(S.w_p[wi]);
    const int uid = uni(S.w_uid[wi]);
    const uint64_t ll = d.dupUids ? W.last_len[uid] : S.w_ll[wi];
    if ((uint32_t)(ll >> 32) == epoch && (uint32_t)ll == (uint32_t)qlen) break;
    qhead = qhead + 1 == P ? 0 : qhead + 1;
    qlen--;
    if (++pops > popCap) { err = KE_ITER_CAP; break; }
    const int s = uni(S.w_s[wi]);
    const int sflags = uni(S.w_flags[wi]);
    const int64_t* pod = S.w_req + wi * d.R;
    const uint64_t* tol = S.w_tol + 2 * wi;
    wi++;
    PH_END(t0, 0);
    bool placed = false;
    // 1) existing nodes in order
    PH_BEGIN(t1);
    for (int base = 0; base < d.N && !placed; base += kWave) {
      const int n = base + lane();
      const bool ok = n < d.N && S.node_ok(n, s, sflags, pod, tol);
      const uint64_t m = wballot(ok);
      S.algbytes += (int64_t)min(kWave, d.N - base) * (16 * d.R + 16);
      if (m) {
        const int j = base + ctz64(m);
        if (lane() < d.R) W.n_req[(int64_t)j * d.R + lane()] += pod[lane()];
        if ((sflags & SF_HAS_KEYS) && lane() == 0)
          rs_add(S.L, W.n_rs + (int64_t)j * d.RSW, D.st_rs + (int64_t)s * d.RSW);
        if (lane() == 0) {
          W.log_pod[nlog] = p;
          W.log_tgt[nlog] = -(j + 1);
          W.pod_status[p] = ST_SCHEDULED;
        }
        nlog++;
        placed = true;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // n_req / n_rs are re-read by other lanes
        wsync();
      }
    }
    PH_END(t1, 1);
    // 2) in-flight NodeClaims, sorted by pod count
    if (!placed && nclaims > 0) {
      PH_BEGIN(t2);
      S.sort_claims(nclaims, sorts, slow);
      PH_END(t2, 2);
      for (int base = 0; base < nclaims && !placed; base += kWave) {
        PH_BEGIN(t3);
        const int j = base + lane();
        const bool q = j < nclaims && S.claim_quick(S.s_order[j], s, sflags, pod, tol);
        uint64_t m = wballot(q);
        S.algbytes += (int64_t)min(kWave, nclaims - base) * (16 * d.R + 4);
        PH_END(t3, 3);
        while (m && !placed) {
          const int jj = base + ctz64(m);
          m &= m - 1;
          const int c = uni(S.s_order[jj]);
          PH_BEGIN(t4);
          const bool ok = S.claim_full(c, s, sflags, pod);
          PH_END(t4, 4);
          if (ok) {
            PH_BEGIN(t5);
            S.commit_claim(c, jj, p, sflags, nlog);
            PH_END(t5, 5);
            placed = true;
          }
        }
      }
    }
    // 3) new NodeClaim per template
    if (!placed) {
      PH_BEGIN(t6);
      const int r = S.try_templates(p, s, sflags, pod, tol, nclaims, nlog, hostCtr);
      PH_END(t6, 6);
      if (r < 0) { err = KE_CLAIM_CAP; break; }
      if (r == 1) placed = true;
      if (r == 2) {  // no templates: add() returns a nil error
        if (lane() == 0) W.pod_status[p] = ST_SCHEDULED;
        placed = true;
      }
    }
    if (placed) continue;
    // failure: Preferences.Relax (preferences.go:38) + Queue.Push (queue.go:64-71)
    const int s0 = D.pod_state0[p], ns = D.pod_nstate[p];
    const bool relaxed = s - s0 + 1 < ns;
    if (lane() == 0) {
      W.pod_status[p] = ST_FAILED;
      W.pod_fstate[p] = s;
      if (relaxed) W.pod_state[p] = s + 1;
    }
    if (relaxed) epoch++;
    int tail = qhead + qlen;
    if (tail >= P) tail -= P;
    if (lane() == 0) W.queue[tail] = p;
    qlen++;
    if (!relaxed && lane() == 0) W.last_len[uid] = ((uint64_t)epoch << 32) | (uint32_t)qlen;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // queue / pod_state are re-read by the window
    wsync();
  }
  // write back LDS-resident claim state for the host
  for (int i = lane(); i < nclaims; i += kWave) W.order[i] = S.s_order[i];
  const int kl = nclaims < pl.KL ? nclaims : pl.KL;
  for (int i = lane(); i < kl * d.R; i += kWave) W.c_req[i] = S.s_creq[i];
  for (int i = lane(); i < kl * d.TW; i += kWave) W.c_rem[i] = S.s_crem[i];
  if (lane() == 0) {
    W.counters[CT_NCLAIMS] = nclaims;
    W.counters[CT_NLOG] = nlog;
    W.counters[CT_HOSTCTR] = hostCtr;
    W.counters[CT_ERROR] = err;
    W.counters[CT_POPS] = pops;
    W.counters[CT_ALGBYTES] = S.algbytes;
    W.counters[CT_SORTS] = sorts;
    W.counters[CT_SORT_SLOW] = slow;
    W.counters[CT_WINDOWS] = windows;
#ifdef KS_PHASE_STATS
    for (int i = 0; i < 7; i++) W.counters[CT_CYC_POP + i] = (int64_t)cyc[i];
    W.counters[CT_CYC_TOTAL] = (int64_t)(__builtin_amdgcn_s_memtime() - tstart);
#endif
  }
}

// LDS plan: put as much claim state in LDS as `budget` allows (one-Solve launches use the whole
// 160 KiB of a CU; batched simulations pass a smaller budget to keep several waves per CU).
Plan make_plan(const KsDims& d, size_t budget) {
  auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
  Plan pl{};
  pl.KO = d.Kcap < 8192 ? d.Kcap : 8192;
  const size_t fixed = r16(sizeof(KeyMeta) * d.NK) + r16(4 * (size_t)(d.NTPL + 1)) + r16(4 * (size_t)d.RSW) +
                       2 * r16(4 * (size_t)d.TW + 8) + r16(8 * kMaxR) + 4 * r16(4 * kWave) + r16(8 * kWave) +
                       r16(16 * kWave) + r16(8 * (size_t)kWave * d.R) + 2 * r16(4 * (size_t)pl.KO) + 16 * 8;
  const size_t perClaim = 4 + 16 * (size_t)d.R + 4 * (size_t)d.TW;
  const size_t tallocB = r16(8 * (size_t)d.totalTplIts * d.R);
  size_t avail = budget > fixed ? budget - fixed : 0;
  pl.talloc = (tallocB + 64 * perClaim <= avail) ? 1 : 0;
  if (pl.talloc) avail -= tallocB;
  size_t kl = avail / (perClaim + 16);
  pl.KL = (int)(kl < (size_t)pl.KO ? kl : (size_t)pl.KO);
  pl.lds = fixed + (pl.talloc ? tallocB : 0) + r16(4 * (size_t)pl.KL) + 2 * r16(8 * (size_t)pl.KL * d.R) +
           r16(4 * (size_t)pl.KL * d.TW);
  return pl;
}

hipError_t queue_sort(const KsDev& D, uint64_t* keys, int32_t* vals, void* temp, size_t tempBytes, int32_t* out,
                      hipStream_t st);

// One ks_solve: queue sort -> workspace init -> [mid event] -> k_solve (all on one stream).
hipError_t launch_solve(const KsDev& D, const KsWork* works_dev, int nrep, const Plan& pl, int32_t* qorder,
                        uint64_t* skeys, int32_t* svals, void* stemp, size_t stempBytes, hipStream_t st,
                        hipEvent_t mid) {
  if (pl.lds > 160 * 1024) return hipErrorInvalidValue;
  hipError_t e = queue_sort(D, skeys, svals, stemp, stempBytes, qorder, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_init, dim3(512), dim3(256), 0, st, D, works_dev, nrep, (const int32_t*)qorder);
  if (mid) (void)hipEventRecord(mid, st);
  hipLaunchKernelGGL(k_solve, dim3(nrep), dim3(kWave), pl.lds, st, D, works_dev, pl);
  return hipGetLastError();
}

}  // namespace ks
