// ks_capi.cpp — the C-ABI (include/karpenter_amd.h): HBM upload of the encoded problem, per-solve
// workspace, kernel launch and reconstruction of scheduling.Results (scheduler.go:102-106).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/karpenter_amd.h"
#include "ks_archive.h"
#include "ks_host.h"
#include "ks_runtime.h"

using namespace ks;

static thread_local std::string g_err;
namespace ks {
void set_last_error(const std::string& m) { g_err = m; }
}  // namespace ks

namespace {

struct WorkLayout {
  size_t c_tpl, c_cnt, c_thr, c_host, c_req, c_max, c_rs, c_rem, order, n_req, n_rs, queue, qorder, pod_state, last_len,
      log_pod, log_tgt, pod_status, pod_fstate, fail_code, fail_host, pool_rem, counters, n_hp, c_hp, n_vc, vlog, vspec, tg_cnt,
      tg_ccnt, tg_cpos, fail_rs, log_hg, tg_act, run_len, run_words, total;
  int32_t ccs;  // tg_ccnt row stride
};

WorkLayout work_layout(const KsDims& d) {
  Arena a;
  WorkLayout w{};
  size_t K = d.Kcap, P = std::max(d.P, 1), N = std::max(d.N, 1);
  w.ccs = d.Kcap + 1;
  w.c_tpl = a.add(4 * K);
  w.c_cnt = a.add(4 * K);
  w.c_thr = a.add(4 * K * d.R);
  w.c_host = a.add(4 * K);
  w.c_req = a.add(8 * K * d.R);
  w.c_max = a.add(8 * K * d.R);
  w.c_rs = a.add(4 * K * d.RSW);
  w.c_rem = a.add(4 * K * d.TW);
  w.order = a.add(4 * K);
  w.n_req = a.add(8 * N * d.R);
  w.n_rs = a.add(4 * N * d.RSW);
  w.queue = a.add(4 * P);
  w.qorder = a.add(4 * P);
  w.pod_state = a.add(4 * P);
  w.last_len = a.add(8 * (size_t)d.NU);
  w.log_pod = a.add(4 * P);
  w.log_tgt = a.add(4 * P);
  w.pod_status = a.add(4 * P);
  w.pod_fstate = a.add(4 * P);
  w.fail_code = a.add(4 * P * std::max(d.NTPL, 1));
  w.fail_host = a.add(4 * P * std::max(d.NTPL, 1));
  w.pool_rem = a.add(8 * (size_t)std::max(d.NPOOL, 1) * d.R);
  w.counters = a.add(8 * CT_NCOUNTERS);
  w.n_hp = a.add(8 * N);
  w.c_hp = a.add(8 * K);
  w.n_vc = a.add(d.volAny ? 4 * N * std::max(d.VD, 1) : 4);
  w.vlog = a.add(8 * (size_t)std::max(d.vLogCap, 1));
  w.vspec = a.add(8 * (size_t)std::max(d.vLogCap, 1));
  w.tg_cnt = a.add(4 * std::max<size_t>(d.G ? (size_t)d.tgCntWords : 1, 1));
  w.tg_ccnt = a.add(4 * (size_t)std::max(d.G, 1) * (d.G ? K + 1 : 1));
  w.tg_cpos = a.add(4 * (size_t)std::max(d.G, 1));
  w.fail_rs = a.add(d.G ? 4 * (size_t)P * std::max(d.NTPL, 1) * d.FSW : 4);
  w.log_hg = a.add(d.G ? 8 * P * (size_t)d.GMW : 8);
  w.tg_act = a.add(4 * (size_t)std::max(d.G, 1));
  w.run_len = a.add(4 * P);
  w.run_words = a.add(8 * ((P + 63) / 64));
  w.total = a.total;
  return w;
}

KsWork work_ptrs(char* base, const WorkLayout& w) {
  KsWork k{};
  k.c_tpl = (int32_t*)(base + w.c_tpl);
  k.c_cnt = (int32_t*)(base + w.c_cnt);
  k.c_thr = (int32_t*)(base + w.c_thr);
  k.c_host = (int32_t*)(base + w.c_host);
  k.c_req = (int64_t*)(base + w.c_req);
  k.c_max = (int64_t*)(base + w.c_max);
  k.c_rs = (uint32_t*)(base + w.c_rs);
  k.c_rem = (uint32_t*)(base + w.c_rem);
  k.order = (int32_t*)(base + w.order);
  k.n_req = (int64_t*)(base + w.n_req);
  k.n_rs = (uint32_t*)(base + w.n_rs);
  k.queue = (int32_t*)(base + w.queue);
  k.qorder = (int32_t*)(base + w.qorder);
  k.pod_state = (int32_t*)(base + w.pod_state);
  k.last_len = (uint64_t*)(base + w.last_len);
  k.log_pod = (int32_t*)(base + w.log_pod);
  k.log_tgt = (int32_t*)(base + w.log_tgt);
  k.pod_status = (int32_t*)(base + w.pod_status);
  k.pod_fstate = (int32_t*)(base + w.pod_fstate);
  k.fail_code = (uint32_t*)(base + w.fail_code);
  k.fail_host = (int32_t*)(base + w.fail_host);
  k.pool_rem = (int64_t*)(base + w.pool_rem);
  k.counters = (int64_t*)(base + w.counters);
  k.n_hp = (uint64_t*)(base + w.n_hp);
  k.c_hp = (uint64_t*)(base + w.c_hp);
  k.n_vc = (int32_t*)(base + w.n_vc);
  k.n_vslot = nullptr;
  k.vlog = (int32_t*)(base + w.vlog);
  k.vspec = (int32_t*)(base + w.vspec);
  k.tg_cnt = (int32_t*)(base + w.tg_cnt);
  k.tg_ccnt = (int32_t*)(base + w.tg_ccnt);
  k.tg_cpos = (int32_t*)(base + w.tg_cpos);
  k.fail_rs = (uint32_t*)(base + w.fail_rs);
  k.log_hg = (uint64_t*)(base + w.log_hg);
  k.tg_act = (int32_t*)(base + w.tg_act);
  k.run_len = (const int32_t*)(base + w.run_len);
  k.ccs = w.ccs;
  return k;
}

template <class T>
void dl(std::vector<T>& v, const void* src, size_t n, hipStream_t st) {
  v.resize(n);
  if (n) HIPCHK(hipMemcpyAsync(v.data(), src, n * sizeof(T), hipMemcpyDeviceToHost, st));
}

}  // namespace

struct ks_results {
  struct Claim {
    int tpl;
    int64_t host;
    std::vector<int32_t> pods, its;
    std::vector<uint32_t> rec;  // the NodeClaim's requirement record (RSW words)
    // structured accessors (ks_results_nodeclaim_requests / _requirements); the pointer arrays point
    // into the string vectors, rebuilt by bind() after every move
    std::vector<std::string> reqNames, reqQty;
    std::vector<const char*> reqNameP, reqQtyP;
    struct Req {
      std::string key, op;
      std::vector<std::string> values;
      int hasGt = 0, hasLt = 0;
      int64_t gt = 0, lt = 0;
    };
    // Rendered on first use: the requirement list (finish_reqs) and the JSON text (finish_json:
    // requirementsString, the launch list) -- a caller reading only pods and options pays for neither
    mutable bool reqsDone = false, jsonDone = false;
    mutable std::string json;
    mutable std::vector<Req> reqs;
    mutable std::vector<std::vector<const char*>> reqValP;
    mutable std::vector<ks_requirement> reqC;
    void bind() {
      reqNameP.clear();
      reqQtyP.clear();
      for (auto& x : reqNames) reqNameP.push_back(x.c_str());
      for (auto& x : reqQty) reqQtyP.push_back(x.c_str());
    }
    void bind_reqs() const {
      reqValP.assign(reqs.size(), {});
      reqC.clear();
      for (size_t i = 0; i < reqs.size(); i++) {
        for (auto& v : reqs[i].values) reqValP[i].push_back(v.c_str());
        reqC.push_back(ks_requirement{reqs[i].key.c_str(), reqs[i].op.c_str(), (int)reqs[i].values.size(),
                                      reqValP[i].data(), reqs[i].hasGt, reqs[i].hasLt, reqs[i].gt, reqs[i].lt});
      }
    }
  };
  ks_problem* pb = nullptr;  // a reference on the problem the lazy rendering reads (ks_problem_free defers)
  // First-use rendering writes the claims' caches: serialised, so two threads reading one Results (ctypes
  // and cgo release the interpreter / scheduler around the call) render once; what a call hands out is
  // never rebuilt afterwards.
  mutable std::mutex render;
  ~ks_results() {
    if (pb && --pb->refs == 0) delete pb;
  }
  struct ENode {
    int index;
    std::string name;
    std::vector<int32_t> pods;
  };
  std::vector<Claim> claims;
  std::vector<ENode> nodes;
  std::vector<std::pair<int32_t, std::string>> errors;
  double kernel_ms = 0, solve_ms = 0, algbytes = 0, feas_ms = 0, feas_bytes = 0, feasn_ms = 0, feasn_bytes = 0;
  std::vector<int64_t> counters;
};

void ks_upload(ks_problem* pb) {
  Host& h = pb->host;
  auto& t = h.tab;
  Arena a;
  struct Item { size_t off; const void* src; size_t bytes; };
  std::vector<Item> items;
  auto put = [&](const void* src, size_t bytes) {
    size_t off = a.add(std::max<size_t>(bytes, 16));
    items.push_back({off, src, bytes});
    return off;
  };
  size_t o_keys = put(h.keys.data(), h.keys.size() * sizeof(KeyMeta));
  size_t o_wv = put(h.wordValid.data(), h.wordValid.size() * 4);
  size_t o_vi = put(h.vIsInt.data(), h.vIsInt.size() * 4);
  size_t o_vint = put(h.vInt.data(), h.vInt.size() * 8);
  size_t o_ita = put(t.it_alloc.data(), t.it_alloc.size() * 8);
  size_t o_itc = put(t.it_cap.data(), t.it_cap.size() * 8);
  size_t o_itr = put(t.it_rs.data(), t.it_rs.size() * 4);
  size_t o_ofb = put(t.it_off_beg.data(), t.it_off_beg.size() * 4);
  size_t o_ofz = put(t.off_zone.data(), t.off_zone.size() * 4);
  size_t o_ofc = put(t.off_ct.data(), t.off_ct.size() * 4);
  size_t o_tr = put(t.tpl_rs.data(), t.tpl_rs.size() * 4);
  size_t o_tt = put(t.tpl_taint.data(), t.tpl_taint.size() * 8);
  size_t o_td = put(t.tpl_daemon.data(), t.tpl_daemon.size() * 8);
  size_t o_tb = put(t.tpl_it_beg.data(), t.tpl_it_beg.size() * 4);
  size_t o_ti = put(t.tpl_its.data(), t.tpl_its.size() * 4);
  size_t o_tp = put(t.tpl_pool.data(), t.tpl_pool.size() * 4);
  size_t o_tsa = put(t.tsort_alloc.data(), t.tsort_alloc.size() * 8);
  // Allocatable per template position ([totalTplIts][R], position-major): what k_solve stages into LDS (TL)
  // with one contiguous copy instead of a gather through tpl_its (every simulation's prologue does it)
  std::vector<int64_t> tplAlloc((size_t)std::max(h.dims.totalTplIts, 1) * h.dims.R, 0);
  for (int i = 0; i < h.dims.totalTplIts; i++)
    for (int r = 0; r < h.dims.R; r++)
      tplAlloc[(size_t)i * h.dims.R + r] = t.it_alloc[(size_t)t.tpl_its[(size_t)i] * h.dims.R + r];
  size_t o_tpa = put(tplAlloc.data(), tplAlloc.size() * 8);
  size_t o_tsp = put(t.tsort_pos.data(), t.tsort_pos.size() * 4);
  size_t o_pr = put(t.pool_rem0.data(), t.pool_rem0.size() * 8);
  size_t o_pm = put(t.pool_mask.data(), t.pool_mask.size() * 4);
  size_t o_preq = put(t.pod_req.data(), t.pod_req.size() * 8);
  size_t o_ps0 = put(t.pod_state0.data(), t.pod_state0.size() * 4);
  size_t o_pns = put(t.pod_nstate.data(), t.pod_nstate.size() * 4);
  size_t o_pu = put(t.pod_uid.data(), t.pod_uid.size() * 4);
  size_t o_psk = put(t.pod_sortkey.data(), t.pod_sortkey.size() * 8);
  size_t o_sr = put(t.st_rs.data(), t.st_rs.size() * 4);
  size_t o_st = put(t.st_tol.data(), t.st_tol.size() * 8);
  size_t o_sf = put(t.st_flags.data(), t.st_flags.size() * 4);
  size_t o_stt = put(t.st_toltpl.data(), t.st_toltpl.size() * 8);
  std::vector<uint64_t> ps0((size_t)std::max(h.dims.P, 1) * 4, 0);
  for (int p = 0; p < h.dims.P; p++) {
    const int s0 = t.pod_state0[(size_t)p];
    ps0[(size_t)p * 4] = t.st_tol[(size_t)s0 * 2];
    ps0[(size_t)p * 4 + 1] = t.st_tol[(size_t)s0 * 2 + 1];
    ps0[(size_t)p * 4 + 2] = t.st_toltpl[(size_t)s0];
    ps0[(size_t)p * 4 + 3] = (uint32_t)t.st_flags[(size_t)s0];
  }
  size_t o_ps0i = put(ps0.data(), ps0.size() * 8);
  size_t o_na = put(t.n_avail.data(), t.n_avail.size() * 8);
  size_t o_nr = put(t.n_req0.data(), t.n_req0.size() * 8);
  size_t o_nrs = put(t.n_rs0.data(), t.n_rs0.size() * 4);
  size_t o_nt = put(t.n_taint.data(), t.n_taint.size() * 8);
  size_t o_nf = put(t.n_flags.data(), t.n_flags.size() * 4);
  size_t o_pf = put(t.pod_flags.data(), t.pod_flags.size() * 4);
  size_t o_op = put(t.off_price.data(), t.off_price.size() * 8);
  size_t o_phc = put(t.pod_hpc.data(), t.pod_hpc.size() * 8);
  size_t o_phu = put(t.pod_hpu.data(), t.pod_hpu.size() * 8);
  size_t o_pho = put(t.pod_hpo.data(), t.pod_hpo.size() * 8);
  size_t o_nhp = put(t.n_hp0.data(), t.n_hp0.size() * 8);
  size_t o_vdb = put(t.pod_vdbeg.data(), t.pod_vdbeg.size() * 4);
  size_t o_vd = put(t.pod_vd.data(), t.pod_vd.size() * 4);
  size_t o_vsb = put(t.pod_vsbeg.data(), t.pod_vsbeg.size() * 4);
  size_t o_vs = put(t.pod_vs.data(), t.pod_vs.size() * 4);
  size_t o_vub = put(t.pod_vubeg.data(), t.pod_vubeg.size() * 4);
  size_t o_vu = put(t.pod_vu.data(), t.pod_vu.size() * 4);
  size_t o_vud = put(t.vol_udrv.data(), t.vol_udrv.size() * 4);
  size_t o_nvc = put(t.n_vc0.data(), t.n_vc0.size() * 4);
  size_t o_nvl = put(t.n_vlim.data(), t.n_vlim.size() * 4);
  size_t o_tgm = put(t.tg_meta.data(), t.tg_meta.size() * 4);
  size_t o_tgc = put(t.tg_cnt0.data(), t.tg_cnt0.size() * 4);
  size_t o_tgf = put(t.tg_frs.data(), t.tg_frs.size() * 4);
  size_t o_sgo = put(t.st_gown.data(), t.st_gown.size() * 8);
  size_t o_pgs = put(t.pod_gsel.data(), t.pod_gsel.size() * 8);
  size_t o_pgi = put(t.pod_ginv.data(), t.pod_ginv.size() * 8);
  size_t o_tgl = put(t.tg_late.data(), t.tg_late.size() * 8);
  size_t o_srs = put(t.st_rss.data(), t.st_rss.size() * 4);
  size_t o_ntd = put(t.n_tdom.data(), t.n_tdom.size() * 4);
  size_t o_fkw = put(t.fk_words.data(), t.fk_words.size() * 4);
  size_t o_fkk = put(t.fk_key_off.data(), t.fk_key_off.size() * 4);
  size_t o_fkt = put(t.fk_tpl.data(), t.fk_tpl.size() * 4);
  // k_feasibility_nodes rows: one per relaxation state with label requirements (the others' strict
  // Compatible is trivially true, their node test is the taint mask alone)
  std::vector<int32_t> fnrow((size_t)std::max(h.dims.S, 1), -1), fnState;
  for (int s = 0; s < h.dims.S; s++)
    if (t.st_flags[(size_t)s] & SF_HAS_KEYS) {
      fnrow[(size_t)s] = (int32_t)fnState.size();
      fnState.push_back(s);
    }
  if (fnState.empty()) fnState.push_back(0);
  size_t o_fnr = put(fnrow.data(), fnrow.size() * 4);
  size_t o_fns = put(fnState.data(), fnState.size() * 4);
  // one allocation, zeroed on the device (padding and empty tables), each table copied from its host vector
  // (no host staging image of the whole problem)
  HIPCHK(hipMalloc(&pb->dbuf, a.total));
  HIPCHK(hipMemsetAsync(pb->dbuf, 0, a.total, pb->stream));
  for (auto& it : items)
    if (it.bytes) HIPCHK(hipMemcpyAsync((char*)pb->dbuf + it.off, it.src, it.bytes, hipMemcpyHostToDevice, pb->stream));
  HIPCHK(hipStreamSynchronize(pb->stream));
  char* b = (char*)pb->dbuf;
  KsDev& D = pb->dev;
  // k_feasibility's output: one row of TW words per (relaxation state, template), rewritten by every
  // Solve / pass; skipped (the kernel evaluates every key itself) if it would exceed 1 GiB
  const size_t fmBytes = 4 * (size_t)h.dims.S * h.dims.NTPL * h.dims.TW;
  // (only steps of pods with label requirements read a row)
  bool keys = false;
  for (int32_t f : t.st_flags) keys = keys || (f & SF_HAS_KEYS);
  h.dims.fmOn = fmBytes > 0 && fmBytes <= ((size_t)1 << 30) && h.dims.NK <= 64 && keys && !getenv("KS_NO_FEASIBILITY");
  // algorithmic bytes of one k_feasibility launch: per (state, template) row the TW words written, the
  // two records' headers and the key words read, and one position-table word per lane for every table
  // row the per-key test ORs (the lacks / DoesNotExist rows, plus one per admitted In value)
  pb->fmBytes = 0;
  if (h.dims.fmOn) {
    const uint64_t km = h.dims.itKeys & ~h.dims.fkMulti;
    auto tableWords = [&](const uint32_t* rec) {
      double w = 0;
      for (uint64_t m = rs_present(rec) & km; m; m &= m - 1) {
        const int k = __builtin_ctzll(m);
        const KeyMeta& kmeta = h.keys[(size_t)k];
        w += 2;
        if (!bit(rs_compl(rec), k))
          for (int i = 0; i < kmeta.nw; i++) w += __builtin_popcount(rec[h.dims.HDR + kmeta.off + i]);
        else
          w += kmeta.nv;
      }
      return w;
    };
    // (a row whose state does not tolerate the template's taints is written as zeros without reads)
    std::vector<double> tplW((size_t)h.dims.NTPL);
    for (int tt = 0; tt < h.dims.NTPL; tt++) tplW[(size_t)tt] = tableWords(&t.tpl_rs[(size_t)tt * h.dims.RSW]);
    for (int s = 0; s < h.dims.S; s++) {
      const double sw = tableWords(&t.st_rs[(size_t)s * h.dims.RSW]);
      for (int tt = 0; tt < h.dims.NTPL; tt++)
        pb->fmBytes += ((t.st_toltpl[(size_t)s] >> tt) & 1u)
                           ? 4.0 * h.dims.TW * (1 + sw + tplW[(size_t)tt]) + 4.0 * 2 * h.dims.HDR + 4.0
                           : 4.0 * h.dims.TW + 4.0;
    }
  }
  if (h.dims.fmOn) HIPCHK(hipMalloc(&pb->fmbuf, fmBytes));
  D.st_fm = (uint32_t*)pb->fmbuf;
  // k_feasibility_nodes: FNR rows of ceil(N/32) words (skipped above 512 MiB: the node scan then runs the
  // strict Compatible per step).  Algorithmic bytes per launch: per (row, node) the node's taints, record
  // header and the words of the keys the state's record holds; per row the state's record and tolerations;
  // the rows written.
  const int FNR = fnrow.empty() ? 0 : (int)std::count_if(fnrow.begin(), fnrow.end(), [](int32_t x) { return x >= 0; });
  const size_t NWN = ((size_t)h.dims.N + 31) / 32;
  const size_t fnBytes = 4 * (size_t)FNR * NWN;
  h.dims.FNR = FNR;
  h.dims.fnOn = FNR > 0 && h.dims.N > 0 && fnBytes <= ((size_t)1 << 29) && !getenv("KS_NO_NODE_ROWS");
  pb->fnBytes = 0;
  if (h.dims.fnOn) {
    for (int i = 0; i < FNR; i++) {
      const uint32_t* X = &t.st_rs[(size_t)fnState[(size_t)i] * h.dims.RSW];
      double kw = 0;
      for (uint64_t m = rs_present(X); m; m &= m - 1) kw += h.keys[(size_t)__builtin_ctzll(m)].nw;
      pb->fnBytes += (double)h.dims.N * (16.0 + 4.0 * (8 + kw)) + 4.0 * h.dims.RSW + 16.0 + 4.0 * NWN;
    }
    HIPCHK(hipMalloc(&pb->fnbuf, fnBytes));
  }
  D.st_fn = (uint32_t*)pb->fnbuf;
  D.st_fnrow = (const int32_t*)(b + o_fnr);
  D.fn_state = (const int32_t*)(b + o_fns);
  D.d = h.dims;
  D.keys = (const KeyMeta*)(b + o_keys);
  D.wordValid = (const uint32_t*)(b + o_wv);
  D.vIsInt = (const uint32_t*)(b + o_vi);
  D.vInt = (const int64_t*)(b + o_vint);
  D.it_alloc = (const int64_t*)(b + o_ita);
  D.it_cap = (const int64_t*)(b + o_itc);
  D.it_rs = (const uint32_t*)(b + o_itr);
  D.it_off_beg = (const int32_t*)(b + o_ofb);
  D.off_zone = (const int32_t*)(b + o_ofz);
  D.off_ct = (const int32_t*)(b + o_ofc);
  D.tpl_rs = (const uint32_t*)(b + o_tr);
  D.tpl_taint = (const uint64_t*)(b + o_tt);
  D.tpl_daemon = (const int64_t*)(b + o_td);
  D.tpl_it_beg = (const int32_t*)(b + o_tb);
  D.tpl_its = (const int32_t*)(b + o_ti);
  D.tpl_pool = (const int32_t*)(b + o_tp);
  D.tsort_alloc = (const int64_t*)(b + o_tsa);
  D.tpl_alloc = (const int64_t*)(b + o_tpa);
  D.tsort_pos = (const int32_t*)(b + o_tsp);
  D.pool_rem0 = (const int64_t*)(b + o_pr);
  D.pool_mask = (const uint32_t*)(b + o_pm);
  D.pod_req = (const int64_t*)(b + o_preq);
  D.pod_state0 = (const int32_t*)(b + o_ps0);
  D.pod_s0 = (const uint64_t*)(b + o_ps0i);
  D.pod_nstate = (const int32_t*)(b + o_pns);
  D.pod_uid = (const int32_t*)(b + o_pu);
  D.pod_sortkey = (const int64_t*)(b + o_psk);
  D.st_rs = (const uint32_t*)(b + o_sr);
  D.st_tol = (const uint64_t*)(b + o_st);
  D.st_flags = (const int32_t*)(b + o_sf);
  D.st_toltpl = (const uint64_t*)(b + o_stt);
  D.n_avail = (const int64_t*)(b + o_na);
  D.n_req0 = (const int64_t*)(b + o_nr);
  D.n_rs0 = (const uint32_t*)(b + o_nrs);
  D.n_taint = (const uint64_t*)(b + o_nt);
  D.n_flags = (const int32_t*)(b + o_nf);
  D.pod_flags = (const int32_t*)(b + o_pf);
  D.off_price = (const double*)(b + o_op);
  D.pod_hpc = (const uint64_t*)(b + o_phc);
  D.pod_hpu = (const uint64_t*)(b + o_phu);
  D.pod_hpo = (const uint64_t*)(b + o_pho);
  D.n_hp0 = (const uint64_t*)(b + o_nhp);
  D.pod_vdbeg = (const int32_t*)(b + o_vdb);
  D.pod_vd = (const int32_t*)(b + o_vd);
  D.pod_vsbeg = (const int32_t*)(b + o_vsb);
  D.pod_vs = (const int32_t*)(b + o_vs);
  D.pod_vubeg = (const int32_t*)(b + o_vub);
  D.pod_vu = (const int32_t*)(b + o_vu);
  D.vol_udrv = (const int32_t*)(b + o_vud);
  D.n_vc0 = (const int32_t*)(b + o_nvc);
  D.n_vlim = (const int32_t*)(b + o_nvl);
  D.tg_meta = (const int32_t*)(b + o_tgm);
  D.tg_cnt0 = (const int32_t*)(b + o_tgc);
  D.tg_frs = (const uint32_t*)(b + o_tgf);
  D.st_gown = (const uint64_t*)(b + o_sgo);
  D.pod_gsel = (const uint64_t*)(b + o_pgs);
  D.pod_ginv = (const uint64_t*)(b + o_pgi);
  D.tg_late = (const uint64_t*)(b + o_tgl);
  D.st_rss = (const uint32_t*)(b + o_srs);
  D.n_tdom = (const int32_t*)(b + o_ntd);
  D.fk_words = (const uint32_t*)(b + o_fkw);
  D.fk_key_off = (const int32_t*)(b + o_fkk);
  D.fk_tpl = (const int32_t*)(b + o_fkt);
}

// A hostname-keyed group's domains at an unsatisfiable-topology failure (topology.go:167), rebuilt from the
// Solve's commit log: NewTopology's counts (tg_cnt0: existing nodes registered by NewExistingNode,
// existingnode.go:60, and countDomains' cluster pods), plus one per commit the device logged as counted in
// the group (log_hg) before the failure (`seq` commits) -- on an existing node its hostname, on a NodeClaim
// its hostname-placeholder -- plus every placeholder NewNodeClaim registered (nodeclaim.go:48-50, one per
// ordinal up to the failing attempt's `ord`; a late group only sees those made after it was created,
// `act`).  Recording registers a domain.  Entries "name:count" in Go's sorted map-key order.
static std::string hostnameCounts(const Host& h, int g, int seq, int64_t ord, int32_t act,
                                  const std::vector<uint64_t>& loghg, const std::vector<int32_t>& logt,
                                  const std::vector<int32_t>& chost) {
  const KsDims& d = h.dims;
  const int32_t* gm = &h.tab.tg_meta[(size_t)g * TGM_WORDS];
  const int k = gm[TGM_KEY], nv = gm[TGM_NV];
  if (seq < 0 || seq > (int)logt.size() || (size_t)seq * d.GMW > loghg.size())
    throw KsError(KS_ERR_INTERNAL, "hostname topology failure outside the commit log");
  std::vector<int32_t> cnt(h.tab.tg_cnt0.begin() + gm[TGM_CNT], h.tab.tg_cnt0.begin() + gm[TGM_CNT] + nv);
  std::map<int64_t, int32_t> ph;  // placeholder ordinal -> count
  for (int64_t o = std::max<int64_t>(h.hostnameSeed, act) + 1; o <= ord; o++) ph[o] = 0;
  for (int i = 0; i < seq; i++) {
    if (!gtest(loghg, (size_t)i, d.GMW, g)) continue;
    if (logt[(size_t)i] >= 0) {
      ph[chost[(size_t)logt[(size_t)i]]] += 1;
    } else {
      const int v = h.tab.n_tdom[(size_t)gm[TGM_KSLOT] * d.N + (size_t)(-logt[(size_t)i] - 1)];
      if (v < 0 || v >= nv) throw KsError(KS_ERR_INTERNAL, "hostname record on a node without a hostname domain");
      cnt[(size_t)v] = cnt[(size_t)v] < 0 ? 1 : cnt[(size_t)v] + 1;
    }
  }
  std::vector<std::pair<std::string, int32_t>> e;
  for (int v = 0; v < nv; v++)
    if (cnt[(size_t)v] >= 0) e.push_back({h.values[(size_t)k][(size_t)v], cnt[(size_t)v]});
  for (auto& kv : ph) e.push_back({h.placeholder(kv.first), kv.second});
  std::sort(e.begin(), e.end());
  std::string o;
  for (size_t i = 0; i < e.size(); i++) o += (i ? " " : "") + e[i].first + ":" + std::to_string(e[i].second);
  return o;
}

// Host replay of the device's bookkeeping before any result is rendered (a lost or stale device store turns
// into a loud KS_ERR_INTERNAL, never a wrong Results): the commit log places each pod at most once (a Solve
// records ST_FAILED per failed attempt and nothing on success, so the status is not cross-checked here); the
// claim order is a permutation; every NodeClaim holds pods and options, its options are
// positions of its template's list whose Allocatable fits the claim's requests (the device's Fits,
// nodeclaim.go:225-260); every existing node's requests (its daemon remainder plus the pods placed there)
// fit its Available (existingnode.go:78-83).  The claims' requests are replayed against the Merge below.
static void replay_check(const Host& h, int nc, int nl, const std::vector<int32_t>& order,
                         const std::vector<int32_t>& ctpl, const std::vector<int64_t>& creq,
                         const std::vector<uint32_t>& crem, const std::vector<int32_t>& logp,
                         const std::vector<int32_t>& logt) {
  const KsDims& d = h.dims;
  auto fail = [](const std::string& m) { throw KsError(KS_ERR_INTERNAL, "device state check: " + m); };
  std::vector<char> placed((size_t)d.P, 0);
  std::vector<int32_t> claimCount((size_t)nc, 0);
  std::vector<int64_t> nodeReq(h.tab.n_req0);
  for (int i = 0; i < nl; i++) {
    const int p = logp[(size_t)i], t = logt[(size_t)i];
    if (p < 0 || p >= d.P) fail("commit log pod index " + std::to_string(p) + " out of range");
    if (placed[(size_t)p]++) fail("pod " + std::to_string(p) + " placed twice");
    if (t >= 0) {
      if (t >= nc) fail("commit log claim " + std::to_string(t) + " beyond " + std::to_string(nc));
      claimCount[(size_t)t]++;
    } else {
      const int n = -t - 1;
      if (n >= d.N) fail("commit log node " + std::to_string(n) + " out of range");
      for (int r = 0; r < d.R; r++) nodeReq[(size_t)n * d.R + r] += h.tab.pod_req[(size_t)p * d.R + r];
    }
  }
  for (int n = 0; n < d.N; n++)
    for (int r = 0; r < d.R; r++) {
      const int64_t q = nodeReq[(size_t)n * d.R + r], a = h.tab.n_avail[(size_t)n * d.R + r];
      if (q != h.tab.n_req0[(size_t)n * d.R + r] && !(a >= 0 && q <= a))
        fail("node " + std::to_string(n) + " over its Available for " + h.resNames[(size_t)r]);
    }
  // VolumeUsage: every existing node that took pods keeps each limited driver's PVC union within its limit
  // (ExceedsLimits held at each placement and the union only grows, volumeusage.go:202-219)
  if (d.volAny) {
    std::vector<std::map<std::string, std::set<std::string>>> use((size_t)d.N);
    std::vector<char> took((size_t)d.N, 0);
    for (int i = 0; i < nl; i++) {
      const int p = logp[(size_t)i], t = logt[(size_t)i];
      if (t >= 0) continue;
      const int n = -t - 1;
      if (!took[(size_t)n]) use[(size_t)n] = h.nodes[(size_t)n].volumes;
      took[(size_t)n] = 1;
      const PodH& ph = h.pods[(size_t)p];
      if (h.tab.pod_flags[(size_t)p] & PF_VOLERR) fail("pod " + std::to_string(p) + " whose GetVolumes fails placed on a node");
      for (auto& name : ph.pvcNames) {
        auto dv = h.volumeDrivers.find(ph.ns + "/" + name);
        if (dv != h.volumeDrivers.end() && !dv->second.empty()) use[(size_t)n][dv->second].insert(ph.ns + "/" + name);
      }
    }
    for (int n = 0; n < d.N; n++) {
      if (!took[(size_t)n]) continue;
      for (auto& kv : h.nodes[(size_t)n].volumeLimits) {
        auto u = use[(size_t)n].find(kv.first);
        if (u != use[(size_t)n].end() && (int64_t)u->second.size() > kv.second)
          fail("node " + std::to_string(n) + " over its volume limit for " + kv.first);
      }
    }
  }
  std::vector<char> seen((size_t)nc, 0);
  for (int k = 0; k < nc; k++) {
    const int c = order[(size_t)k];
    if (c < 0 || c >= nc || seen[(size_t)c]++) fail("NodeClaim order is not a permutation");
  }
  for (int c = 0; c < nc; c++) {
    const int t = ctpl[(size_t)c];
    if (t < 0 || t >= d.NTPL) fail("NodeClaim " + std::to_string(c) + " template out of range");
    if (claimCount[(size_t)c] == 0) fail("NodeClaim " + std::to_string(c) + " holds no pod");
    const int nIT = (int)h.tpls[(size_t)t].its.size();
    int opts = 0;
    for (int w = 0; w < d.TW; w++) {
      const int lo = w * 32;
      const uint32_t valid = nIT >= lo + 32 ? ~0u : nIT > lo ? (1u << (nIT - lo)) - 1u : 0u;
      if (crem[(size_t)c * d.TW + w] & ~valid) fail("NodeClaim " + std::to_string(c) + " has options beyond its template's list");
      for (uint32_t m = crem[(size_t)c * d.TW + w]; m; m &= m - 1) {
        const int pos = lo + __builtin_ctz(m);
        opts++;
        const int it = h.tab.tpl_its[(size_t)h.tab.tpl_it_beg[(size_t)t] + pos];
        for (int r = 0; r < d.R; r++) {
          const int64_t a = h.tab.it_alloc[(size_t)it * d.R + r];
          if (!(a >= 0 && creq[(size_t)c * d.R + r] <= a))
            fail("NodeClaim " + std::to_string(c) + " keeps option " + h.its[(size_t)it].name + " its requests exceed (" +
                 h.resNames[(size_t)r] + ")");
        }
      }
    }
    if (opts == 0) fail("NodeClaim " + std::to_string(c) + " has no instance type option");
  }
}

// The rendered halves of a NodeClaim result, each on first use: the structured Requirements after
// FinalizeScheduling (ks_results_nodeclaim_requirements), and the JSON text (ks_results_json: requirement
// strings, requirementsString, the launch list).
static void finish_reqs(const Host& h, const ks_results::Claim& cl) {
  if (cl.reqsDone) return;
  const KsDims& d = h.dims;
  const uint32_t* rec = cl.rec.data();
  const uint64_t pr = rs_present(rec);
  static const char* opn[] = {"In", "NotIn", "Exists", "DoesNotExist"};
  for (int kk = 0; kk < d.NK; kk++) {  // FinalizeScheduling drops the hostname requirement
    if (!bit(pr, kk) || kk == h.hostKey) continue;
    ks_results::Claim::Req q;
    q.key = h.keyNames[(size_t)kk];
    const int op = rs_op(h.L, rec, kk);
    q.op = opn[op];
    const KeyMeta& km = h.keys[(size_t)kk];
    if (op == OP_IN || op == OP_NOTIN) {
      for (int b = 0; b < km.nv; b++)
        if ((rec[h.L.HDR + km.off + (b >> 5)] >> (b & 31)) & 1u) q.values.push_back(h.values[(size_t)kk][(size_t)b]);
      std::sort(q.values.begin(), q.values.end());
    }
    if (km.bslot >= 0) {
      q.hasGt = bit(rs_hasgt(rec), kk) ? 1 : 0;
      q.hasLt = bit(rs_haslt(rec), kk) ? 1 : 0;
      if (q.hasGt) q.gt = rs_gt(rec, km.bslot);
      if (q.hasLt) q.lt = rs_lt(rec, km.bslot);
    }
    cl.reqs.push_back(std::move(q));
  }
  cl.bind_reqs();
  cl.reqsDone = true;
}
static void finish_json(const Host& h, const ks_results::Claim& cl) {
  if (cl.jsonDone) return;
  const KsDims& d = h.dims;
  const Host::Tpl& tp = h.tpls[(size_t)cl.tpl];
  const uint32_t* rec = cl.rec.data();
  std::string j = "{\"nodePoolName\":";
  ksjson::quote(j, tp.pool);
  j += ",\"hostname\":";
  ksjson::quote(j, h.placeholder(cl.host));
  j += ",\"pods\":[";
  for (size_t i = 0; i < cl.pods.size(); i++) j += (i ? "," : "") + std::to_string(cl.pods[i]);
  j += "],\"instanceTypeOptions\":[";
  for (size_t i = 0; i < cl.its.size(); i++) {
    if (i) j += ",";
    ksjson::quote(j, h.its[cl.its[i]].name);
  }
  j += "],\"requests\":{";
  for (size_t i = 0; i < cl.reqNames.size(); i++) {
    if (i) j += ",";
    ksjson::quote(j, cl.reqNames[i]);
    j += ":";
    ksjson::quote(j, cl.reqQty[i]);
  }
  j += "},\"requirements\":[";
  bool first = true;
  const uint64_t pr = rs_present(rec);
  for (int kk = 0; kk < d.NK; kk++) {  // FinalizeScheduling drops the hostname requirement
    if (!bit(pr, kk) || kk == h.hostKey) continue;
    if (!first) j += ",";
    first = false;
    ksjson::quote(j, h.reqString(rec, kk, true, cl.host));
  }
  j += "],\"requirementsString\":";
  ksjson::quote(j, h.reqsString(rec, cl.host));
  // NodeClaimTemplate.ToNodeClaim's launch list (nodeclaimtemplate.go:55-60): the options ordered by
  // (cheapest available offering the claim's zone / capacity-type requirements allow, name)
  // (OrderByPrice, types.go:62-79; Offerings.Requirements / Cheapest :147-166), first 100.
  auto allows = [&](int key, const std::string& v) {  // Requirements.Get(key).Has(v); missing key = Exists
    if (key < 0 || !bit(rs_present(rec), key)) return true;
    auto id = h.valueId[(size_t)key].find(v);
    if (id != h.valueId[(size_t)key].end()) return rs_member(h.L, rec, key, id->second);
    return bit(rs_compl(rec), key);  // a value outside the universe: only a complement set holds it
  };
  std::vector<std::pair<double, std::string>> launch;
  for (int it : cl.its) {
    double price = std::numeric_limits<double>::max();
    bool any = false;
    for (auto& of : h.its[(size_t)it].all) {
      if (!of.available || !allows(h.zoneKey, of.zone) || !allows(h.ctKey, of.ct)) continue;
      if (!any || of.price < price) price = of.price;
      any = true;
    }
    launch.push_back({price, h.its[(size_t)it].name});
  }
  std::sort(launch.begin(), launch.end());
  j += ",\"launchInstanceTypes\":[";
  for (size_t i = 0; i < launch.size() && i < 100; i++) {
    if (i) j += ",";
    ksjson::quote(j, launch[i].second);
  }
  j += "]}";
  cl.json = j;
  cl.jsonDone = true;
}

// Rebuild Results from the replica-0 workspace.
static ks_results* collect(ks_problem* pb, const KsWork& W) {
  PhaseTimer pt("collect");
  Host& h = pb->host;
  const KsDims& d = h.dims;
  hipStream_t st = pb->stream;
  std::vector<int64_t> ctr;
  dl(ctr, W.counters, CT_NCOUNTERS, st);
  HIPCHK(hipStreamSynchronize(st));
  if (ctr[CT_ERROR] != KE_OK)
    throw KsError(ctr[CT_ERROR] == KE_CLAIM_CAP ? KS_ERR_CAPACITY : KS_ERR_INTERNAL,
                  ctr[CT_ERROR] == KE_CLAIM_CAP ? "NodeClaim capacity (" + std::to_string(pb->lastKO) +
                                                      " per Solve at this LDS budget) exceeded"
                                                : "solve kernel iteration cap hit");
  int nc = (int)ctr[CT_NCLAIMS], nl = (int)ctr[CT_NLOG];
  std::vector<int32_t> order, ctpl, chost, logp, logt, status, fstate;
  std::vector<int64_t> creq;
  std::vector<uint32_t> crs, crem, fcode;
  std::vector<int32_t> fhost;
  dl(order, W.order, nc, st);
  dl(ctpl, W.c_tpl, nc, st);
  dl(chost, W.c_host, nc, st);
  dl(creq, W.c_req, (size_t)nc * d.R, st);
  dl(crs, W.c_rs, (size_t)nc * d.RSW, st);
  dl(crem, W.c_rem, (size_t)nc * d.TW, st);
  dl(logp, W.log_pod, nl, st);
  dl(logt, W.log_tgt, nl, st);
  dl(status, W.pod_status, d.P, st);
  HIPCHK(hipStreamSynchronize(st));
  bool anyFailed = false;  // (the failure tables are read only for pods whose last attempt failed)
  for (int p = 0; p < d.P && !anyFailed; p++) anyFailed = status[(size_t)p] == ST_FAILED;
  if (anyFailed) {
    dl(fstate, W.pod_fstate, d.P, st);
    dl(fcode, W.fail_code, (size_t)d.P * std::max(d.NTPL, 1), st);
    dl(fhost, W.fail_host, (size_t)d.P * std::max(d.NTPL, 1), st);
    HIPCHK(hipStreamSynchronize(st));
  }
  std::vector<uint32_t> frs;  // topology failure snapshots, only when some pod failed on one
  std::vector<uint64_t> loghg;
  std::vector<int32_t> tgact;
  if (d.G) {
    bool need = false;
    for (int p = 0; p < d.P && !need; p++) {
      if (status[p] != ST_FAILED) continue;
      for (int t = 0; t < d.NTPL; t++) {
        const uint32_t c = fcode[(size_t)p * d.NTPL + t] & 0xff;
        need = need || c == FC_TOPO || c == FC_TOPO_COMPAT || (fcode[(size_t)p * d.NTPL + t] & FC_RS_SNAP);
      }
    }
    if (need) {
      dl(frs, W.fail_rs, (size_t)d.P * d.NTPL * d.FSW, st);
      dl(loghg, W.log_hg, (size_t)nl * d.GMW, st);
      dl(tgact, W.tg_act, d.G, st);
      HIPCHK(hipStreamSynchronize(st));
    }
  }

  pt.mark("download");
  replay_check(h, nc, nl, order, ctpl, creq, crem, logp, logt);
  pt.mark("replay check");
  auto* res = new ks_results();
  res->pb = pb;
  pb->refs++;
  res->counters = ctr;
  res->algbytes = (double)ctr[CT_ALGBYTES];
  std::vector<std::vector<int32_t>> claimPods(nc), nodePods(d.N);
  for (int i = 0; i < nl; i++) {
    if (logt[i] >= 0) claimPods[logt[i]].push_back(logp[i]);
    else nodePods[-logt[i] - 1].push_back(logp[i]);
  }
  for (int k = 0; k < nc; k++) {
    int c = order[k];
    ks_results::Claim cl;
    cl.tpl = ctpl[c];
    cl.host = chost[c];
    cl.pods = claimPods[c];
    const Host::Tpl& tp = h.tpls[cl.tpl];
    for (int pos = 0; pos < (int)tp.its.size(); pos++)
      if ((crem[(size_t)c * d.TW + (pos >> 5)] >> (pos & 31)) & 1u) cl.its.push_back(tp.its[pos]);
    // requests = Merge(daemon, RequestsForPods(pod_1), ...) replayed in commit order (resources.go:53-63),
    // in the exact device units: Quantity.Add adopts the addend's format while the sum is zero
    int64_t sum[kMaxR];
    uint8_t fmt[kMaxR];
    uint32_t present = h.tab.tpl_rmask[(size_t)cl.tpl];
    for (int r = 0; r < d.R; r++) {
      sum[r] = h.tab.tpl_daemon[(size_t)cl.tpl * d.R + r];
      fmt[r] = h.tab.tpl_rfmt[(size_t)cl.tpl * d.R + r];
    }
    for (int p : cl.pods) {
      const uint32_t m = h.tab.pod_rmask[(size_t)p];
      present |= m;
      for (uint32_t b = m; b; b &= b - 1) {
        const int r = __builtin_ctz(b);
        if (sum[r] == 0) fmt[r] = h.tab.pod_rfmt[(size_t)p * d.R + r];
        sum[r] += h.tab.pod_req[(size_t)p * d.R + r];
      }
    }
    QList req;
    for (int r = 0; r < d.R; r++) {
      if (!((present >> r) & 1u)) continue;
      if (sum[r] != creq[(size_t)c * d.R + r])
        throw KsError(KS_ERR_INTERNAL, "device requests diverge from the replayed Merge for " + h.resNames[(size_t)r] +
                                           " (claim " + std::to_string(c) + " at position " + std::to_string(k) + " of " +
                                           std::to_string(nc) + ": device " + std::to_string(creq[(size_t)c * d.R + r]) +
                                           ", replay " + std::to_string(sum[r]) + " over " +
                                           std::to_string(cl.pods.size()) + " pods)");
      Qty q = h.fromDev(r, sum[r]);
      q.f = (QFmt)fmt[r];
      req.emplace_hint(req.end(), h.resNames[(size_t)r], q);  // resource ids are in name order
    }
    for (auto& kv : req) {
      cl.reqNames.push_back(kv.first);
      cl.reqQty.push_back(qty_str(kv.second));
    }
    cl.rec.assign(crs.begin() + (size_t)c * d.RSW, crs.begin() + (size_t)(c + 1) * d.RSW);
    res->claims.push_back(std::move(cl));
  }
  for (auto& c : res->claims) c.bind();  // after the last move of the claims vector
  pt.mark("claims");
  for (int n = 0; n < d.N; n++) res->nodes.push_back(ks_results::ENode{h.nodes[n].origIndex, h.nodes[n].name, nodePods[n]});
  // PodErrors (scheduler.go:179-183 keeps non-nil errors only)
  // k_solve records ST_FAILED at each failed attempt and nothing on success: a pod is an error iff
  // its last recorded attempt failed and it is not in the commit log.
  std::vector<char> inLog(d.P, 0);
  for (int i = 0; i < nl; i++) inLog[logp[i]] = 1;
  for (int p = 0; p < d.P; p++) {
    if (status[p] != ST_FAILED || inLog[p]) continue;
    int s = fstate[p];
    int s0 = h.tab.pod_state0[p];
    const PodState& ps = h.states[p][s - s0];
    std::vector<std::string> segs;
    for (int t = 0; t < d.NTPL; t++) {
      uint32_t code = fcode[(size_t)p * d.NTPL + t];
      int64_t host = fhost[(size_t)p * d.NTPL + t];
      const Host::Tpl& tp = h.tpls[t];
      std::string pre = "incompatible with nodepool " + go_quote(tp.pool) + ", daemonset overhead=" + qlist_json(tp.daemon) + ", ";
      switch (code & 0xff) {
        case FC_LIMITS:
          segs.push_back("all available instance types exceed limits for nodepool: " + go_quote(tp.pool));
          break;
        case FC_TAINTS: {
          std::string m;
          for (auto& x : tp.taints) {
            bool ok = false;
            for (auto& tol : ps.tols) {
              bool e = tol.effect.empty() || tol.effect == x.effect;
              bool k = tol.key.empty() || tol.key == x.key;
              bool v = (tol.op.empty() || tol.op == "Equal") ? tol.value == x.value : tol.op == "Exists";
              ok = ok || (e && k && v);
            }
            if (!ok) m += (m.empty() ? "" : "; ") + std::string("did not tolerate ") + x.key + "=" + x.value + ":" + x.effect;
          }
          segs.push_back(pre + m);
          break;
        }
        case FC_COMPAT: {
          std::vector<uint32_t> r(h.tab.tpl_rs.begin() + (size_t)t * d.RSW, h.tab.tpl_rs.begin() + (size_t)(t + 1) * d.RSW);
          auto errs = h.compatErrors(r.data(), ps.rsAll.data(), true, host);
          std::string m;
          for (size_t i = 0; i < errs.size(); i++) m += (i ? "; " : "") + errs[i];
          segs.push_back(pre + "incompatible requirements, " + m);
          break;
        }
        case FC_NO_IT: {
          uint32_t f = (code >> 8) & 0x3f;
          std::vector<uint32_t> r(h.tab.tpl_rs.begin() + (size_t)t * d.RSW, h.tab.tpl_rs.begin() + (size_t)(t + 1) * d.RSW);
          if (code & FC_RS_SNAP) {
            const uint32_t* snap = &frs[((size_t)p * d.NTPL + t) * d.FSW];
            r.assign(snap, snap + d.RSW);
          } else {
            rs_add(h.L, r.data(), ps.rsAll.data());
          }
          QList cum = tp.daemon;
          for (auto& kv : h.pods[p].requests) cum[kv.first].add(kv.second);
          bool rq = f & FF_REQ, fi = f & FF_FITS, of = f & FF_OFF;
          std::string why;  // filterResults.FailureReason (nodeclaim.go:165-221)
          if (!rq && !fi && !of) why = "no instance type met the scheduling requirements or had enough resources or had a required offering";
          else if (!rq && !fi) why = "no instance type met the scheduling requirements or had enough resources";
          else if (!rq && !of) why = "no instance type met the scheduling requirements or had a required offering";
          else if (!fi && !of) why = "no instance type had enough resources or had a required offering";
          else if (!rq) why = "no instance type met all requirements";
          else if (!fi) {
            why = "no instance type has enough resources";
            auto c = cum.find("cpu");
            if (c != cum.end() && c->second.n >= (__int128)1000000 * 1000000000) why += " (CPU request >= 1 Million, m vs M typo?)";
          } else if (!of) why = "no instance type has the required offering";
          else if (f & FF_REQ_FITS) why = "no instance type which met the scheduling requirements and had enough resources, had a required offering";
          else if (f & FF_FITS_OFF) why = "no instance type which had enough resources and the required offering met the scheduling requirements";
          else if (f & FF_REQ_OFF) why = "no instance type which met the scheduling requirements and the required offering had the required resources";
          else why = "no instance type met the requirements/resources/offering tuple";
          segs.push_back(pre + "no instance type satisfied resources " + qlist_json(cum) + " and requirements " +
                         h.reqsString(r.data(), host) + " (" + why + ")");
          break;
        }
        case FC_TOPO: {  // Topology.AddRequirements (topology.go:160-165)
          const int g = (int)(code >> 16) & 0xffff;
          const int32_t* gm = &h.tab.tg_meta[(size_t)g * TGM_WORDS];
          const int k = gm[TGM_KEY], nv = gm[TGM_NV];
          const uint32_t* fr = &frs[((size_t)p * d.NTPL + t) * d.FSW];
          // fmt %v of TopologyGroup.domains (map[string]int32): the registered domains in name order
          std::string counts = "map[";
          if (!gm[TGM_HOST]) {  // the device snapshot of the counts at the failure (-1: not registered)
            bool first = true;
            for (int v = 0; v < nv; v++)
              if ((int32_t)fr[v] >= 0) {
                counts += (first ? "" : " ") + h.values[(size_t)k][(size_t)v] + ":" + std::to_string((int32_t)fr[v]);
                first = false;
              }
          } else {
            counts += hostnameCounts(h, g, (int)fr[0], host, tgact[(size_t)g], loghg, logt, chost);
          }
          counts += "]";
          std::vector<uint32_t> nr(h.tab.tpl_rs.begin() + (size_t)t * d.RSW, h.tab.tpl_rs.begin() + (size_t)(t + 1) * d.RSW);
          rs_add(h.L, nr.data(), ps.rsAll.data());
          auto dom = [&](const uint32_t* rec) {
            return bit(rs_present(rec), k) ? h.reqString(rec, k, false, host) : h.keyNames[(size_t)k] + " Exists";
          };
          segs.push_back(pre + "unsatisfiable topology constraint for " +
                         (gm[TGM_TYPE] == TG_SPREAD ? "topology spread" : gm[TGM_TYPE] == TG_AFFINITY ? "pod affinity" : "pod anti-affinity") + ", key=" +
                         h.keyNames[(size_t)k] + " (counts = " + counts + ", podDomains = " + dom(ps.rsStrict.data()) +
                         ", nodeDomains = " + dom(nr.data()) + ")");
          break;
        }
        case FC_TOPO_COMPAT: {  // Compatible(nodeRequirements, topologyRequirements) (nodeclaim.go:96-98)
          std::vector<uint32_t> nr(h.tab.tpl_rs.begin() + (size_t)t * d.RSW, h.tab.tpl_rs.begin() + (size_t)(t + 1) * d.RSW);
          rs_add(h.L, nr.data(), ps.rsAll.data());
          auto errs = h.compatErrors(nr.data(), &frs[((size_t)p * d.NTPL + t) * d.FSW], true, host);
          std::string m;
          for (size_t i = 0; i < errs.size(); i++) m += (i ? "; " : "") + errs[i];
          segs.push_back(pre + m);
          break;
        }
        default:
          throw KsError(KS_ERR_INTERNAL, "failed pod without a failure code");
      }
    }
    std::string msg;
    for (size_t i = 0; i < segs.size(); i++) msg += (i ? "; " : "") + segs[i];
    res->errors.push_back({p, msg});
  }
  pt.mark("nodes + pod errors");
  return res;
}

extern "C" {

const char* ks_last_error(void) { return g_err.c_str(); }
void ks_free(void* p) { free(p); }
const char* ks_build_info(void) { return "karpenter_amd gfx950 one-wavefront-per-Solve v1"; }

int ks_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// The device half of NewScheduler for an encoded host model: upload, queue-sort workspaces, the host's
// NewQueue order when pods tie.
static void problem_device_init(ks_problem* pb) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) throw KsError(KS_ERR_HIP, "no HIP device visible");
  HIPCHK(hipGetDevice(&pb->device));
  HIPCHK(hipStreamCreateWithFlags(&pb->stream, hipStreamNonBlocking));
  ks_upload(pb);
  size_t np = std::max(pb->host.dims.P, 1);
  HIPCHK(hipMalloc(&pb->skeys, 2 * np * sizeof(uint64_t)));
  HIPCHK(hipMalloc(&pb->svals, 2 * np * sizeof(int32_t)));
  pb->stempBytes = std::max<size_t>(queue_sort_temp_bytes((int)np), 256);
  HIPCHK(hipMalloc(&pb->stemp, pb->stempBytes));
  if (!pb->host.hostQueue.empty()) {
    HIPCHK(hipMalloc(&pb->hqorder, 4 * np));
    HIPCHK(hipMemcpy(pb->hqorder, pb->host.hostQueue.data(), 4 * pb->host.hostQueue.size(), hipMemcpyHostToDevice));
  }
}

int ks_problem_create(const char* json, size_t len, ks_problem** out) {
  API_TRY
  if (!json || !out) throw KsError(KS_ERR_ARG, "null argument");
  ksjson::Value root = ksjson::Parser(json, len ? len : strlen(json)).parse();
  std::unique_ptr<ks_problem> pb(new ks_problem());
  pb->host.build(root);
  ksjson::release_async(std::move(root));
  problem_device_init(pb.get());
  *out = pb.release();
  return KS_OK;
  API_CATCH
}

// --- binary snapshot (ks_archive.h, ks_snapshot.cpp) ----------------------------------------------------
extern "C++" {
namespace {
// the format version: 05 = round 6 (per relaxation state, the minDomains its spread groups would be created
// with, PodState::gmd); 04 = round 5's final layout (taint and host-port classes, live resource names, sparse
// volume tables, injectFailed); 03 = round 5's first (sparse volume tables, injectFailed); 02 = round 4 (group
// sets); 01 = round 3.  A blob of another version is refused with a version error (snapshot_check_header).
constexpr char kProblemMagic[8] = {'K', 'S', 'P', 'R', 'O', 'B', '0', '5'};
}  // namespace

void snapshot_header(ArOut& a, const char magic[8]) {
  a.raw(magic, 8);
  uint32_t v[4] = {1u, (uint32_t)sizeof(KsDims), (uint32_t)sizeof(KeyMeta), (uint32_t)sizeof(Host)};
  a.raw(v, sizeof(v));
}
void snapshot_check_header(ArIn& a, const char magic[8]) {
  char m[8];
  uint32_t v[4];
  a.raw(m, 8);
  a.raw(v, sizeof(v));
  if (memcmp(m, magic, 6) == 0 && memcmp(m, magic, 8) != 0)  // the same kind, another format version
    throw KsError(KS_ERR_PARSE, "binary snapshot format version " + std::string(m + 6, 2) + ", this build reads version " +
                                    std::string(magic + 6, 2));
  if (memcmp(m, magic, 8) != 0) throw KsError(KS_ERR_PARSE, "not a binary snapshot of this kind");
  if (v[0] != 1u || v[1] != sizeof(KsDims) || v[2] != sizeof(KeyMeta) || v[3] != sizeof(Host))
    throw KsError(KS_ERR_PARSE, "binary snapshot from another build of the library");
}
char* snapshot_bytes(const std::string& s) {
  char* b = (char*)malloc(std::max<size_t>(s.size(), 1));
  if (!b) throw KsError(KS_ERR_CAPACITY, "out of host memory");
  memcpy(b, s.data(), s.size());
  return b;
}
}  // extern "C++"

int ks_problem_save(const ks_problem* p, void** buf, size_t* len) {
  API_TRY
  if (!p || !buf || !len) throw KsError(KS_ERR_ARG, "null argument");
  ArOut a;
  snapshot_header(a, kProblemMagic);
  host_save(a, const_cast<Host&>(p->host));
  *buf = snapshot_bytes(a.buf);
  *len = a.buf.size();
  return KS_OK;
  API_CATCH
}

int ks_problem_create_binary(const void* buf, size_t len, ks_problem** out) {
  API_TRY
  if (!buf || !out) throw KsError(KS_ERR_ARG, "null argument");
  std::unique_ptr<ks_problem> pb(new ks_problem());
  try {
    ArIn a{(const char*)buf, (const char*)buf + len};
    snapshot_check_header(a, kProblemMagic);
    host_load(a, pb->host);
    if (a.p != a.end) throw KsError(KS_ERR_PARSE, "binary snapshot has trailing bytes");
  } catch (const ArchiveError& e) {
    throw KsError(KS_ERR_PARSE, e.what());
  }
  problem_device_init(pb.get());
  *out = pb.release();
  return KS_OK;
  API_CATCH
}

// Host-only check of the snapshot format: encode the snapshot, save it, load the bytes into a fresh model and
// save that again; the two byte strings must be identical (*bytes: the snapshot size).
int ks_snapshot_check(const char* json, size_t len, size_t* bytes) {
  API_TRY
  if (!json) throw KsError(KS_ERR_ARG, "null argument");
  PhaseTimer pt("ks_snapshot_check");
  ksjson::Value root = ksjson::Parser(json, len ? len : strlen(json)).parse();
  Host h;
  h.build(root);
  pt.mark("parse + encode");
  ArOut a;
  host_save(a, h);
  pt.mark("save");
  Host g;
  try {
    ArIn in{a.buf.data(), a.buf.data() + a.buf.size()};
    host_load(in, g);
    pt.mark("load");
    if (in.p != in.end) throw KsError(KS_ERR_INTERNAL, "snapshot reload left bytes");
  } catch (const ArchiveError& e) {
    throw KsError(KS_ERR_INTERNAL, e.what());
  }
  ArOut b;
  host_save(b, g);
  if (bytes) *bytes = a.buf.size();
  if (a.buf != b.buf) throw KsError(KS_ERR_INTERNAL, "snapshot save -> load -> save is not the identity");
  return KS_OK;
  API_CATCH
}

// Host-only: the binary snapshot of a JSON problem without creating a handle (no device), e.g. to convert
// fixtures offline on a machine without a GPU; ks_problem_create_binary accepts the bytes.
int ks_problem_encode_binary(const char* json, size_t len, void** buf, size_t* blen) {
  API_TRY
  if (!json || !buf || !blen) throw KsError(KS_ERR_ARG, "null argument");
  ksjson::Value root = ksjson::Parser(json, len ? len : strlen(json)).parse();
  Host h;
  h.build(root);
  ArOut a;
  snapshot_header(a, kProblemMagic);
  host_save(a, h);
  *buf = snapshot_bytes(a.buf);
  *blen = a.buf.size();
  return KS_OK;
  API_CATCH
}

// Host-only: load and validate a problem snapshot (the checks ks_problem_create_binary runs before any upload):
// KS_OK, or KS_ERR_PARSE for a truncated, foreign or internally inconsistent blob.
int ks_problem_check_binary(const void* buf, size_t len) {
  API_TRY
  if (!buf) throw KsError(KS_ERR_ARG, "null argument");
  Host h;
  try {
    ArIn a{(const char*)buf, (const char*)buf + len};
    snapshot_check_header(a, kProblemMagic);
    host_load(a, h);
    if (a.p != a.end) throw KsError(KS_ERR_PARSE, "binary snapshot has trailing bytes");
  } catch (const ArchiveError& e) {
    throw KsError(KS_ERR_PARSE, e.what());
  }
  return KS_OK;
  API_CATCH
}

// Host-only encode (no device): layout sizes for diagnostics and CPU tests.
int ks_problem_inspect(const char* json, size_t len, char** out) {
  API_TRY
  if (!json || !out) throw KsError(KS_ERR_ARG, "null argument");
  ksjson::Value root = ksjson::Parser(json, len ? len : strlen(json)).parse();
  Host h;
  h.build(root);
  const KsDims& d = h.dims;
  std::string o = "{";
  auto kv = [&](const char* k, long long v) { o += std::string(o.size() > 1 ? "," : "") + "\"" + k + "\":" + std::to_string(v); };
  kv("R", d.R); kv("keys", d.NK); kv("W", d.W); kv("NB", d.NB); kv("RSW", d.RSW); kv("T", d.T); kv("templates", d.NTPL);
  kv("pools", d.NPOOL); kv("nodes", d.N); kv("pods", d.P); kv("states", d.S); kv("uids", d.NU); kv("TW", d.TW);
  kv("Kcap", d.Kcap); kv("taints", (long long)h.taints.size()); kv("G", d.G); kv("G1", d.G1);
  kv("hostQueue", h.hostQueue.empty() ? 0 : 1); kv("hostPorts", (long long)h.hostPortUniverse.size());
  long long nlate = 0;
  for (uint64_t x : h.tab.tg_late) nlate += __builtin_popcountll(x);
  kv("lateGroups", nlate); kv("groupWords", d.GMW); kv("unlabelledNodes", d.tgUnlab);
  long long nfail = 0, nshared = 0, nverr = 0;
  for (char x : h.injectFailed) nfail += x ? 1 : 0;
  for (int32_t f : h.tab.pod_flags) {
    nshared += (f & PF_VSHARED) ? 1 : 0;
    nverr += (f & PF_VOLERR) ? 1 : 0;
  }
  kv("volAny", d.volAny); kv("volDrivers", d.VD); kv("volPvcs", d.NVU); kv("volLogCap", d.vLogCap);
  kv("volSharedPods", nshared); kv("volErrorPods", nverr); kv("injectFailed", nfail);
  kv("volStaticMounts", (long long)(h.tab.pod_vsbeg.empty() ? 0 : h.tab.pod_vsbeg.back()));
  // LDS plans (ks_solve.hip make_plan) at the default and a few reduced budgets
  o += ",\"plans\":{";
  const size_t budgets[] = {160 * 1024 - 256, 6000, 9000, 14000, 24000, 40000};
  for (size_t i = 0; i < sizeof(budgets) / sizeof(budgets[0]); i++) {
    Plan pl = make_plan(d, budgets[i]);
    o += (i ? ",\"" : "\"") + std::to_string(budgets[i]) + "\":{\"KO\":" + std::to_string(pl.KO) +
         ",\"KL\":" + std::to_string(pl.KL) + ",\"talloc\":" + std::to_string(pl.talloc) +
         ",\"tsort\":" + std::to_string(pl.tsort) + ",\"lds\":" + std::to_string(pl.lds) + "}";
  }
  o += "}";
  o += ",\"keyNames\":[";
  for (size_t i = 0; i < h.keyNames.size(); i++) { if (i) o += ","; ksjson::quote(o, h.keyNames[i]); }
  o += "],\"resources\":[";
  for (size_t i = 0; i < h.resNames.size(); i++) { if (i) o += ","; ksjson::quote(o, h.resNames[i]); }
  o += "]}";
  *out = strdup(o.c_str());
  return KS_OK;
  API_CATCH
}

// A problem lives until its last Results is freed too (Results render lazily from it).
void ks_problem_free(ks_problem* p) {
  if (p && --p->refs == 0) delete p;
}
void ks_results_free(ks_results* r) { delete r; }

int ks_solve(ks_problem* pb, const ks_solve_opts* opts, ks_results** out) {
  API_TRY
  if (!pb || !out) throw KsError(KS_ERR_ARG, "null argument");
  int reps = opts && opts->replicas > 1 ? opts->replicas : 1;
  DeviceGuard guard(pb->device, opts);
  const KsDims& d = pb->host.dims;
  // one Solve per CU gets the whole 160 KiB; larger batches trade LDS for waves per CU
  size_t budget = 160 * 1024 - 256;
  if (reps > 256) budget = std::max<size_t>(24 * 1024, budget * 256 / reps);
  if (opts && opts->lds_budget > 0) budget = std::min<size_t>(budget, (size_t)opts->lds_budget);
  Plan pl = make_plan(d, budget, false, pb->wideKO);
  if (pl.lds > 160 * 1024 || pl.KO < 1)
    throw KsError(KS_ERR_CAPACITY, "solve state does not fit the LDS budget");
  pb->lastKO = pl.KO;
  WorkLayout wl = work_layout(d);
  size_t need = wl.total * reps;
  if (need > pb->wbytes || reps != pb->wreps) {
    if (pb->wbuf) HIPCHK(hipFree(pb->wbuf));
    if (pb->works_dev) HIPCHK(hipFree(pb->works_dev));
    pb->wbuf = nullptr;
    pb->works_dev = nullptr;
    HIPCHK(hipMalloc(&pb->wbuf, need));
    HIPCHK(hipMalloc(&pb->works_dev, sizeof(KsWork) * reps));
    std::vector<KsWork> ws;
    for (int r = 0; r < reps; r++) ws.push_back(work_ptrs((char*)pb->wbuf + wl.total * r, wl));
    for (auto& x : ws) x.run_len = ws[0].run_len;  // one queue order (k_init copies it to every replica)
    HIPCHK(hipMemcpy(pb->works_dev, ws.data(), sizeof(KsWork) * reps, hipMemcpyHostToDevice));
    pb->wbytes = need;
    pb->wreps = reps;
  }
  KsWork w0 = work_ptrs((char*)pb->wbuf, wl);
  hipEvent_t e0, em, e1, ef[4];
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&em));
  HIPCHK(hipEventCreate(&e1));
  for (auto& e : ef) HIPCHK(hipEventCreate(&e));
  // A Solve that outgrows the default plan's NodeClaim capacity runs again with the wide plan; the
  // caller pays both launches, so the reported times are their sums (the re-plan is remembered).
  float ms = 0, setup = 0, fms = 0, fnms = 0;
  int feasLaunches = 0, attempts = 0;
  for (int attempt = 0; attempt < 4; attempt++) {
    attempts++;
    HIPCHK(hipEventRecord(e0, pb->stream));
    HIPCHK(launch_solve(pb->dev, pb->works_dev, reps, pl, w0.qorder, pb->skeys, pb->svals, pb->stemp,
                        pb->stempBytes, pb->stream, em, pb->hqorder, ef, (int32_t*)w0.run_len,
                        (uint64_t*)((char*)pb->wbuf + wl.run_words)));
    HIPCHK(hipEventRecord(e1, pb->stream));
    HIPCHK(hipEventSynchronize(e1));
    float a = 0, b = 0, f = 0;
    HIPCHK(hipEventElapsedTime(&a, e0, e1));
    HIPCHK(hipEventElapsedTime(&b, e0, em));
    if (pb->dev.d.fmOn) {
      HIPCHK(hipEventElapsedTime(&f, ef[0], ef[1]));
      feasLaunches++;
    }
    if (pb->dev.d.fnOn) {
      float fn = 0;
      HIPCHK(hipEventElapsedTime(&fn, ef[2], ef[3]));
      fnms += fn;
    }
    ms += a;
    setup += b;
    fms += f;
    int64_t err = 0;
    HIPCHK(hipMemcpy(&err, w0.counters + CT_ERROR, 8, hipMemcpyDeviceToHost));
    if (err == KE_LEAN_EXIT && pb->dev.d.lean) {
      // shared UIDs and a push-back: the non-LEAN instantiation (remembered for later Solves of this problem)
      pb->dev.d.lean = 0;
      continue;
    }
    if (err != KE_CLAIM_CAP || pb->wideKO >= 2) break;
    // more NodeClaims than the plan holds: re-plan with claim positions filling the LDS (level 1 keeps the
    // instance-type tables in LDS, level 2 moves them to HBM; remembered for later Solves of this problem)
    // and solve again
    const int prevKO = pl.KO;
    pb->wideKO++;
    pl = make_plan(d, budget, false, pb->wideKO);
    if (pb->wideKO == 1 && pl.KO <= prevKO) pl = make_plan(d, budget, false, pb->wideKO = 2);
    if (pl.lds > 160 * 1024 || pl.KO < 1) break;
    pb->lastKO = pl.KO;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(em);
  (void)hipEventDestroy(e1);
  for (auto& e : ef) (void)hipEventDestroy(e);
  ks_results* r;
  if (opts && opts->timing_only) {
    r = new ks_results();
    dl(r->counters, w0.counters, CT_NCOUNTERS, pb->stream);
    HIPCHK(hipStreamSynchronize(pb->stream));
    if (r->counters[CT_ERROR] != KE_OK) {
      std::string msg = "solve kernel reported error " + std::to_string(r->counters[CT_ERROR]);
      delete r;
      throw KsError(KS_ERR_INTERNAL, msg);
    }
    r->algbytes = (double)r->counters[CT_ALGBYTES];
  } else {
    r = collect(pb, w0);
  }
  r->kernel_ms = ms;
  r->solve_ms = ms - setup;
  r->feas_ms = fms;
  r->feas_bytes = pb->dev.d.fmOn ? pb->fmBytes * feasLaunches : 0;  // bytes of every launch feas_ms sums
  r->feasn_ms = fnms;
  r->feasn_bytes = pb->dev.d.fnOn ? pb->fnBytes * attempts : 0;  // one k_feasibility_nodes per launch
  *out = r;
  return KS_OK;
  API_CATCH
}

int ks_results_json(const ks_results* r, char** json_out) {
  API_TRY
  std::string o = "{\"newNodeClaims\":[";
  std::lock_guard<std::mutex> lk(r->render);
  for (size_t i = 0; i < r->claims.size(); i++) {
    finish_json(r->pb->host, r->claims[i]);
    o += (i ? "," : "") + r->claims[i].json;
  }
  o += "],\"existingNodes\":[";
  // existing nodes are reported by name in calculateExistingNodeClaims order
  for (size_t i = 0; i < r->nodes.size(); i++) {
    o += i ? ",{\"name\":" : "{\"name\":";
    ksjson::quote(o, r->nodes[i].name);
    o += ",\"pods\":[";
    for (size_t k = 0; k < r->nodes[i].pods.size(); k++) o += (k ? "," : "") + std::to_string(r->nodes[i].pods[k]);
    o += "]}";
  }
  o += "],\"podErrors\":{";
  for (size_t i = 0; i < r->errors.size(); i++) {
    if (i) o += ",";
    ksjson::quote(o, std::to_string(r->errors[i].first));
    o += ":";
    ksjson::quote(o, r->errors[i].second);
  }
  o += "},\"stats\":{";
  static const char* names[] = {"nclaims", "ncommits", "hostnameCounter", "error", "pops", "algBytes",
                                "sorts", "sortsWithDescent", "claimFull", "claimQuickFail", "windows",
                                "cycPop", "cycNodes", "cycSort", "cycQuick", "cycFull", "cycCommit", "cycTemplates",
                                "cycTotal", "cycNodeCommit", "cycFullRs", "cycFullThr", "cycFullMasks", "cycFullApply",
                                "runs", "runPods", "sortsExact", "fineTopoPop", "fineState", "fineRefill",
                                "fineWindowTests", "fineWindowBlocks", "fineRecord", "fineNodeCommit", "fineWindowTopo"};
  for (int i = 0; i < CT_NCOUNTERS; i++) o += std::string(i ? "," : "") + "\"" + names[i] + "\":" + std::to_string(r->counters[i]);
  o += "}}";
  *json_out = strdup(o.c_str());
  return KS_OK;
  API_CATCH
}

int ks_results_num_new_nodeclaims(const ks_results* r) { return (int)r->claims.size(); }
int ks_results_nodeclaim(const ks_results* r, int i, int* tpl, const int32_t** pods, int* np, const int32_t** its, int* nit) {
  if (i < 0 || i >= (int)r->claims.size()) return KS_ERR_ARG;
  const auto& c = r->claims[i];
  if (tpl) *tpl = c.tpl;
  if (pods) *pods = c.pods.data();
  if (np) *np = (int)c.pods.size();
  if (its) *its = c.its.data();
  if (nit) *nit = (int)c.its.size();
  return KS_OK;
}
int ks_results_nodeclaim_requests(const ks_results* r, int i, int* n, const char* const** names,
                                  const char* const** quantities) {
  if (!r || i < 0 || i >= (int)r->claims.size()) return KS_ERR_ARG;
  const auto& c = r->claims[(size_t)i];
  if (n) *n = (int)c.reqNameP.size();
  if (names) *names = c.reqNameP.data();
  if (quantities) *quantities = c.reqQtyP.data();
  return KS_OK;
}
int ks_results_nodeclaim_requirements(const ks_results* r, int i, int* n, const ks_requirement** reqs) {
  if (!r || i < 0 || i >= (int)r->claims.size()) return KS_ERR_ARG;
  const auto& c = r->claims[(size_t)i];
  {
    std::lock_guard<std::mutex> lk(r->render);
    finish_reqs(r->pb->host, c);
  }
  if (n) *n = (int)c.reqC.size();
  if (reqs) *reqs = c.reqC.data();
  return KS_OK;
}
int ks_results_num_existing_nodes(const ks_results* r) { return (int)r->nodes.size(); }
int ks_results_existing_node(const ks_results* r, int i, int* idx, const int32_t** pods, int* np) {
  if (i < 0 || i >= (int)r->nodes.size()) return KS_ERR_ARG;
  if (idx) *idx = r->nodes[i].index;
  if (pods) *pods = r->nodes[i].pods.data();
  if (np) *np = (int)r->nodes[i].pods.size();
  return KS_OK;
}
int ks_results_num_pod_errors(const ks_results* r) { return (int)r->errors.size(); }
int ks_results_pod_error(const ks_results* r, int i, int* pod, const char** msg) {
  if (i < 0 || i >= (int)r->errors.size()) return KS_ERR_ARG;
  if (pod) *pod = r->errors[i].first;
  if (msg) *msg = r->errors[i].second.c_str();
  return KS_OK;
}
double ks_results_kernel_ms(const ks_results* r) { return r->kernel_ms; }
double ks_results_solve_kernel_ms(const ks_results* r) { return r->solve_ms; }
double ks_results_feasibility_ms(const ks_results* r) { return r->feas_ms; }
double ks_results_feasibility_bytes(const ks_results* r) { return r->feas_bytes; }
double ks_results_node_feasibility_ms(const ks_results* r) { return r->feasn_ms; }
double ks_results_node_feasibility_bytes(const ks_results* r) { return r->feasn_bytes; }
double ks_results_algorithmic_bytes(const ks_results* r) { return r->algbytes; }

}  // extern "C"
