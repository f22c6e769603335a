// ks_snapshot.cpp — binary snapshot of the host model (ks_archive.h): every member of Host and of the
// types it holds, listed once per type for both directions.  The static_asserts on the struct sizes make
// a member added later a compile error here until it is listed.
#include "ks_archive.h"
#include "ks_host.h"
#include "ks_parallel.h"

#include <algorithm>

namespace ks {

template <class A> void io(A& a, Qty& q) { io_all(a, q.n, q.f); }
template <class A> void io(A& a, NSR& x) { io_all(a, x.key, x.op, x.values); }
template <class A> void io(A& a, TaintH& x) { io_all(a, x.key, x.value, x.effect); }
template <class A> void io(A& a, TolH& x) { io_all(a, x.key, x.op, x.value, x.effect); }
template <class A> void io(A& a, PrefTerm& x) { io_all(a, x.weight, x.exprs); }
template <class A> void io(A& a, SelReq& x) { io_all(a, x.key, x.op, x.values); }
template <class A> void io(A& a, LabelSel& x) { io_all(a, x.present, x.reqs); }
template <class A> void io(A& a, AffTerm& x) { io_all(a, x.sel, x.namespaces, x.nsSelector, x.nsSel, x.key); }
template <class A> void io(A& a, SpreadC& x) { io_all(a, x.key, x.when, x.maxSkew, x.minDomains, x.sel); }
template <class A> void io(A& a, HostPortH& x) { io_all(a, x.ip, x.proto, x.port, x.ip16, x.ipValid); }
template <class A> void io(A& a, PodH& x) {
  io_all(a, x.name, x.ns, x.uid, x.created, x.labels, x.nodeSelector, x.hasAffinity, x.hasNodeAffinity, x.hasRequired,
         x.requiredTerms, x.preferred, x.hasPodAffinity, x.hasPodAnti, x.affRequired, x.antiRequired, x.affPreferred,
         x.antiPreferred, x.tsc, x.nodeName, x.phase, x.tols, x.requests, x.hostPorts, x.volumes, x.pvcNames, x.ports,
         x.provisionable, x.ownedByNode, x.ownedByDaemonSet, x.terminal, x.deleting, x.annotations, x.hasPriority,
         x.notReady, x.priority);
}
// (rsAll / rsStrict are the rows tab.st_rs / tab.st_rss already hold: restored from them after a load)
template <class A> void io(A& a, PodState& x) { io_all(a, x.hasPreferred, x.tols, x.gown, x.gmd, x.spec); }
template <class A> void io(A& a, TopoGroup& x) {
  io_all(a, x.type, x.key, x.hash, x.keyId, x.maxSkew, x.minDomains, x.namespaces, x.sel, x.filterNil, x.filter, x.domains,
         x.late);
}
template <class A> void io(A& a, Host::Offer& x) { io_all(a, x.zone, x.ct, x.price, x.available); }
template <class A> void io(A& a, Host::IT& x) { io_all(a, x.name, x.reqs, x.capacity, x.alloc, x.offers, x.prices, x.all); }
template <class A> void io(A& a, Host::Tpl& x) {
  io_all(a, x.pool, x.reqs, x.labels, x.poolLabels, x.taints, x.its, x.daemon, x.limitPool, x.rs);
}
template <class A> void io(A& a, Host::Pool& x) { io_all(a, x.name, x.remaining); }
template <class A> void io(A& a, Host::Node& x) {
  io_all(a, x.name, x.hostName, x.labels, x.taints, x.available, x.capacity, x.dsRequests, x.req0, x.initialized, x.ready,
         x.origIndex, x.hostPorts, x.volumes, x.volumeLimits);
}
// A table of fixed-width rows most of which are zero (the relaxation states' requirement records: a
// resource-only pod's record is empty): the row width, a bitmap of the non-zero rows and those rows only.
template <class A>
void io_rows(A& a, std::vector<uint32_t>& v, uint64_t width) {
  uint64_t n = v.size();
  io_len(a, n);
  io(a, width);
  if (width == 0 || n % width) throw ArchiveError("binary snapshot: row table width");
  const uint64_t rows = n / width;
  std::vector<uint64_t> nz((rows + 63) / 64, 0);
  if constexpr (A::reading) {
    a.need(8 * ((rows + 63) / 64));  // the bitmap must be there before the table is allocated
    io(a, nz);
    if (nz.size() != (rows + 63) / 64) throw ArchiveError("binary snapshot: row bitmap size");
    v.assign(n, 0);
    for (uint64_t r = 0; r < rows; r++)
      if ((nz[r >> 6] >> (r & 63)) & 1ull) a.raw(&v[r * width], 4 * width);
  } else {
    for (uint64_t r = 0; r < rows; r++)
      for (uint64_t k = 0; k < width; k++)
        if (v[r * width + k]) {
          nz[r >> 6] |= 1ull << (r & 63);
          break;
        }
    io(a, nz);
    for (uint64_t r = 0; r < rows; r++)
      if ((nz[r >> 6] >> (r & 63)) & 1ull) a.raw(&v[r * width], 4 * width);
  }
}

template <class A> void io_tables(A& a, Host::Tables& t, uint64_t rsw) {
  io_all(a, t.tsort_alloc, t.it_alloc, t.it_cap, t.tpl_daemon, t.pool_rem0, t.pod_req, t.pod_sortkey, t.n_avail, t.n_req0,
         t.off_price, t.n_flags, t.pod_flags, t.pod_hpc, t.pod_hpu, t.pod_hpo, t.n_hp0, t.pod_vdbeg, t.pod_vd, t.pod_vsbeg,
         t.pod_vs, t.pod_vubeg, t.pod_vu, t.vol_udrv, t.n_vc0, t.n_vlim, t.tg_meta, t.tg_cnt0, t.tg_frs, t.st_gown, t.pod_gsel, t.pod_ginv, t.n_tdom, t.it_rs, t.tpl_rs, t.n_rs0,
         t.pool_mask, t.st_toltpl, t.tpl_taint, t.st_tol, t.n_taint, t.tsort_pos, t.it_off_beg, t.off_zone, t.off_ct,
         t.tpl_it_beg, t.tpl_its, t.tpl_pool, t.pod_state0, t.pod_nstate, t.pod_uid, t.st_flags, t.pod_rmask, t.tpl_rmask,
         t.pod_rfmt, t.tpl_rfmt, t.fk_words, t.fk_key_off, t.fk_tpl, t.tg_late);
  // (st_rss is one word when the problem has no topology groups)
  io_rows(a, t.st_rs, rsw);
  io_rows(a, t.st_rss, t.st_rss.size() < rsw && !A::reading ? t.st_rss.size() : rsw);
}

// Large per-pod vectors (pods, their relaxation chains, the cluster's bound pods) go as an offset table plus
// one blob, so both directions run on the host worker threads (ks_parallel.h): each element is encoded into /
// decoded from its own byte range.
template <class A, class T>
void io_par(A& a, std::vector<T>& v) {
  uint64_t n = v.size();
  io_len(a, n);
  if constexpr (A::reading) {
    a.need(8 * (n + 1));  // the offset table itself
    if (n > (uint64_t)INT32_MAX) throw ArchiveError("binary snapshot: too many elements");
  }
  std::vector<uint64_t> off(n + 1, 0);
  if constexpr (A::reading) {
    io(a, off);
    if (off.size() != n + 1 || off[0] != 0 || off[n] > (uint64_t)(a.end - a.p))
      throw ArchiveError("binary snapshot offsets out of range");
    // the whole table is checked before any element is decoded: every element's byte range lies inside
    // [0, off[n]], so no decode (on a worker thread) can read past the caller's buffer
    for (uint64_t i = 0; i < n; i++)
      if (off[i] > off[i + 1]) throw ArchiveError("binary snapshot offsets out of order");
    v.resize(n);
    const char* base = a.p;
    parallel_for((int)n, 64, [&](int i) {
      ArIn sub{base + off[(size_t)i], base + off[(size_t)i + 1]};
      io(sub, v[(size_t)i]);
      if (sub.p != sub.end) throw ArchiveError("binary snapshot element size mismatch");
    });
    a.p = base + off[n];
  } else {
    std::vector<std::string> parts(n);
    parallel_for((int)n, 64, [&](int i) {
      ArOut sub;
      io(sub, v[(size_t)i]);
      parts[(size_t)i] = std::move(sub.buf);
    });
    for (uint64_t i = 0; i < n; i++) off[i + 1] = off[i] + parts[i].size();
    io(a, off);
    for (auto& p : parts) a.raw(p.data(), p.size());
  }
}

// A loaded model must be internally consistent before anything reads it by its dims: every table at
// least as long as the dims say the host and the kernels index it (ks_capi.cpp problem_device_init, the
// k_* kernels), every stored index inside the table it points into.  A blob that is complete but corrupt
// (a flipped dims field, a shortened table) is refused here as a parse error instead of being read out of
// bounds on the host or the device.
void host_check(const Host& h) {
  const KsDims& d = h.dims;
  auto bad = [](const char* what) { throw ArchiveError(std::string("binary snapshot: inconsistent ") + what); };
  auto need = [&](size_t have, int64_t want, const char* what) {
    if (want < 0 || (int64_t)have < want) bad(what);
  };
  if (d.R < 1 || d.R > kMaxR || d.NK < 0 || d.NK > 64 || d.NTPL < 0 || d.NTPL > kMaxTpl || d.T < 0 || d.N < 0 ||
      d.P < 0 || d.S < 1 || d.NU < 1 || d.NPOOL < 0 || d.VD < 0 || d.NVU < 0 || d.vLogCap < 0 || d.TW < 1 || d.G < 0 ||
      d.G1 < 0 || d.G1 > d.G || d.Kcap < 1)
    bad("dims");
  if (d.HDR != 8 + 4 * d.NB || d.RSW < d.HDR + d.W || d.W < 0 || d.NB < 0) bad("record layout");
  if ((int)h.keys.size() != d.NK || (int)h.keyNames.size() != d.NK || (int)h.values.size() != d.NK) bad("key tables");
  need(h.wordValid.size(), d.W, "wordValid");
  need(h.vIsInt.size(), d.W, "vIsInt");
  for (const KeyMeta& km : h.keys) {
    if (km.off < 0 || km.nw < 0 || km.off + km.nw > d.W || km.nv < 0 || km.nv > 32 * km.nw) bad("key layout");
    if (km.bslot >= d.NB) bad("key bound slot");
    if (km.vint >= 0 && (size_t)km.vint + (size_t)km.nv > h.vInt.size()) bad("key int table");
  }
  for (int k : {d.zoneKey, d.ctKey})
    if (k < 0 || k >= d.NK) bad("zone / capacity-type key");
  if ((int)h.tpls.size() != d.NTPL || (int)h.its.size() != d.T || (int)h.nodes.size() != d.N ||
      (int)h.pods.size() != d.P || (int)h.states.size() != d.P || (int)h.pools.size() != d.NPOOL ||
      (int)h.groups.size() != d.G)
    bad("object counts");
  const Host::Tables& t = h.tab;
  const int64_t R = d.R, RSW = d.RSW, T = d.T, N1 = std::max(d.N, 1), P1 = std::max(d.P, 1), S = d.S;
  const int64_t NT1 = std::max(d.NTPL, 1), NP1 = std::max(d.NPOOL, 1), VD1 = std::max(d.VD, 1);
  need(t.it_alloc.size(), T * R, "it_alloc");
  need(t.it_cap.size(), T * R, "it_cap");
  need(t.it_rs.size(), T * RSW, "it_rs");
  need(t.it_off_beg.size(), T + 1, "it_off_beg");
  need(t.tpl_rs.size(), NT1 * RSW, "tpl_rs");
  need(t.tpl_taint.size(), NT1 * 2, "tpl_taint");
  need(t.tpl_daemon.size(), NT1 * R, "tpl_daemon");
  need(t.tpl_rmask.size(), NT1, "tpl_rmask");
  need(t.tpl_rfmt.size(), NT1 * R, "tpl_rfmt");
  need(t.tpl_it_beg.size(), (int64_t)d.NTPL + 1, "tpl_it_beg");
  need(t.tpl_pool.size(), NT1, "tpl_pool");
  need(t.pool_rem0.size(), NP1 * R, "pool_rem0");
  need(t.pool_mask.size(), NP1, "pool_mask");
  need(t.pod_req.size(), P1 * R, "pod_req");
  need(t.pod_rfmt.size(), P1 * R, "pod_rfmt");
  need(t.pod_sortkey.size(), P1 * 4, "pod_sortkey");
  for (auto* v : {&t.pod_state0, &t.pod_nstate, &t.pod_uid, &t.pod_flags}) need(v->size(), P1, "per-pod table");
  for (auto* v : {&t.pod_hpc, &t.pod_hpu, &t.pod_hpo}) need(v->size(), P1, "per-pod mask");
  need(t.pod_rmask.size(), P1, "pod_rmask");
  need(t.st_rs.size(), S * RSW, "st_rs");
  need(t.st_tol.size(), S * 2, "st_tol");
  need(t.st_flags.size(), S, "st_flags");
  need(t.st_toltpl.size(), S, "st_toltpl");
  if (d.GMW < 1 || d.GMW < (d.G + 63) / 64) bad("group set width");
  need(t.st_gown.size(), S * d.GMW, "st_gown");
  need(t.tg_late.size(), d.GMW, "tg_late");
  need(t.n_avail.size(), N1 * R, "n_avail");
  need(t.n_req0.size(), N1 * R, "n_req0");
  need(t.n_rs0.size(), N1 * RSW, "n_rs0");
  need(t.n_taint.size(), N1 * 2, "n_taint");
  need(t.n_flags.size(), N1, "n_flags");
  need(t.n_hp0.size(), N1, "n_hp0");
  need(t.n_vc0.size(), N1 * VD1, "n_vc0");
  need(t.n_vlim.size(), N1 * VD1, "n_vlim");
  // the sparse volume tables: CSR offsets monotone and in range, every driver / node / PVC index inside its
  // table, the shared pods' PVC lists within the log capacity
  for (auto* b : {&t.pod_vdbeg, &t.pod_vsbeg, &t.pod_vubeg}) need(b->size(), (int64_t)d.P + 1, "volume CSR offsets");
  need(t.vol_udrv.size(), std::max<int64_t>(d.NVU, 1), "vol_udrv");
  auto csr = [&](const std::vector<int32_t>& beg, size_t entries, const char* what) {
    if (beg[0] != 0) bad(what);
    for (int64_t p = 0; p < d.P; p++)
      if (beg[(size_t)p] > beg[(size_t)p + 1]) bad(what);
    if ((size_t)beg[(size_t)d.P] > entries) bad(what);
  };
  csr(t.pod_vdbeg, t.pod_vd.size() / 2, "pod_vd");
  csr(t.pod_vsbeg, t.pod_vs.size() / 2, "pod_vs");
  csr(t.pod_vubeg, t.pod_vu.size(), "pod_vu");
  for (size_t i = 0; i + 1 < t.pod_vd.size(); i += 2)
    if (t.pod_vd[i] < 0 || (t.pod_vd[i] >= d.VD && d.P > 0 && t.pod_vdbeg[(size_t)d.P] > 0) || t.pod_vd[i + 1] < 0) bad("pod_vd entry");
  for (size_t i = 0; i + 1 < t.pod_vs.size() && t.pod_vsbeg[(size_t)d.P] > 0; i += 2)
    if (t.pod_vs[i] < 0 || t.pod_vs[i] >= d.N || t.pod_vs[i + 1] < 0 || t.pod_vs[i + 1] >= d.NVU) bad("pod_vs entry");
  for (size_t i = 0; i < (size_t)t.pod_vubeg[(size_t)d.P]; i++)
    if (t.pod_vu[i] < 0 || t.pod_vu[i] >= d.NVU) bad("pod_vu entry");
  for (int64_t u = 0; u < d.NVU; u++)
    if (t.vol_udrv[(size_t)u] < 0 || t.vol_udrv[(size_t)u] >= d.VD) bad("vol_udrv entry");
  if (t.pod_vubeg[(size_t)d.P] > d.vLogCap) bad("volume log capacity");
  need(t.pod_gsel.size(), P1 * d.GMW, "pod_gsel");
  need(t.pod_ginv.size(), P1 * d.GMW, "pod_ginv");
  // CSR tables and the indices the kernels follow
  auto mono = [&](const std::vector<int32_t>& v, size_t n, int64_t hi, const char* what) {
    if (v[0] != 0) bad(what);
    for (size_t i = 0; i < n; i++)
      if (v[i] > v[i + 1]) bad(what);
    if (v[n] > hi) bad(what);
  };
  mono(t.it_off_beg, (size_t)T, (int64_t)std::min({t.off_zone.size(), t.off_ct.size(), t.off_price.size()}), "offerings");
  mono(t.tpl_it_beg, (size_t)d.NTPL, (int64_t)t.tpl_its.size(), "template instance-type lists");
  if (t.tpl_it_beg[(size_t)d.NTPL] != d.totalTplIts) bad("totalTplIts");
  for (int i = 0; i < d.NTPL; i++) {
    const int n = t.tpl_it_beg[(size_t)i + 1] - t.tpl_it_beg[(size_t)i];
    if (n > d.maxTplIts || (d.maxTplIts + 31) / 32 > d.TW) bad("template list width");
    if (t.tpl_pool[(size_t)i] >= d.NPOOL) bad("template pool");
  }
  for (int32_t x : t.tpl_its)
    if (x < 0 || x >= d.T) bad("template instance type");
  need(t.tsort_alloc.size(), (int64_t)std::max(d.totalTplIts, 1) * R, "tsort_alloc");
  need(t.tsort_pos.size(), (int64_t)std::max(d.totalTplIts, 1) * R, "tsort_pos");
  for (int64_t p = 0; p < d.P; p++) {
    const int64_t s0 = t.pod_state0[(size_t)p], ns = t.pod_nstate[(size_t)p];
    if (s0 < 0 || ns < 1 || s0 + ns > S || ns != (int64_t)h.states[(size_t)p].size()) bad("relaxation states");
    if (t.pod_uid[(size_t)p] < 0 || t.pod_uid[(size_t)p] >= d.NU) bad("pod uid");
  }
  if (!h.hostQueue.empty()) {
    if ((int)h.hostQueue.size() != d.P) bad("host queue");
    for (int32_t x : h.hostQueue)
      if (x < 0 || x >= d.P) bad("host queue entry");
  }
  // topology
  if (d.G) {
    need(t.tg_meta.size(), (int64_t)d.G * TGM_WORDS, "tg_meta");
    need(t.n_tdom.size(), (int64_t)std::max(d.TK, 1) * N1, "n_tdom");
    need(t.st_rss.size(), S * RSW, "st_rss");
    if (d.tgCntWords != (int32_t)t.tg_cnt0.size() || d.tgSmall < 0 || d.tgSmall > d.tgCntWords) bad("count table");
    for (int g = 0; g < d.G; g++) {
      const int32_t* m = &t.tg_meta[(size_t)g * TGM_WORDS];
      if (m[TGM_KEY] < 0 || m[TGM_KEY] >= d.NK || m[TGM_NV] < 0 || m[TGM_NV] > h.keys[(size_t)m[TGM_KEY]].nv ||
          m[TGM_CNT] < 0 || (int64_t)m[TGM_CNT] + std::max(m[TGM_NV], 1) > d.tgCntWords || m[TGM_FBEG] < 0 ||
          m[TGM_FBEG] > m[TGM_FEND] || (int64_t)m[TGM_FEND] * RSW > (int64_t)t.tg_frs.size() || m[TGM_KSLOT] < 0 ||
          m[TGM_KSLOT] >= d.TK)
        bad("topology group");
    }
    for (int32_t v : t.n_tdom)
      if (v < -1 || v >= std::max(d.tgMaxNv, 1) + 1) bad("node domain");
  }
}

// The layout pointers (L) point into the vectors and are re-aimed after a load; the build-only members
// (topoExcluded, preParsedPods, the value-set scratch) are not part of the model a snapshot carries.
template <class A> void host_io(A& a, Host& h) {
  PhaseTimer pt(A::reading ? "host_load" : "host_save");
  io_all(a, h.keyNames, h.keyId, h.values, h.valueId, h.keys, h.wordValid, h.vIsInt, h.vInt, h.hostKey, h.zoneKey, h.ctKey,
         h.hostPrivBit, h.allowWK, h.itKeys, h.wellKnown, h.resNames, h.resId, h.resShift, h.taints, h.hostPortUniverse,
         h.hostPortOwner, h.volumeDrivers, h.volDrivers, h.volUniverse, h.injectFailed, h.its, h.tpls, h.pools, h.toleratePreferNoSchedule,
         h.nodes, h.daemons);
  pt.mark("universe, types, templates, nodes");
  io_par(a, h.pods);
  pt.mark("pods");
  io_par(a, h.states);
  pt.mark("relaxation states");
  io_par(a, h.clusterPods);
  io_all(a, h.groups, h.groupsOwned, h.nodeLabelsByName, h.namespaceList, h.podGsel, h.podGinv, h.topoContrib,
         h.topoInvOwner, h.topoInvOwners, h.topoUniverse, h.topoHostActive, h.hostnameSeed, h.hostQueue, h.emptyTopology);
  pt.mark("topology");
  io_all(a, h.dims);
  io_tables(a, h.tab, (uint64_t)std::max(h.dims.RSW, 1));
  pt.mark("tables");
  if constexpr (A::reading) {
    // each relaxation state's requirement records from the device tables (state s = pod_state0[p] + i)
    const size_t RSW = (size_t)h.dims.RSW;
    const bool strict = !h.groups.empty();
    if (h.tab.pod_state0.size() < h.states.size()) throw ArchiveError("binary snapshot: states without a first index");
    parallel_for((int)h.states.size(), 256, [&](int p) {
      auto& chain = h.states[(size_t)p];
      for (size_t i = 0; i < chain.size(); i++) {
        const size_t st = (size_t)h.tab.pod_state0[(size_t)p] + i;
        if ((st + 1) * RSW > h.tab.st_rs.size() || (strict && (st + 1) * RSW > h.tab.st_rss.size()))
          throw ArchiveError("binary snapshot: relaxation state outside the tables");
        chain[i].rsAll.assign(h.tab.st_rs.begin() + st * RSW, h.tab.st_rs.begin() + (st + 1) * RSW);
        if (strict) chain[i].rsStrict.assign(h.tab.st_rss.begin() + st * RSW, h.tab.st_rss.begin() + (st + 1) * RSW);
      }
    });
    h.L.nkeys = h.dims.NK;
    h.L.W = h.dims.W;
    h.L.NB = h.dims.NB;
    h.L.HDR = h.dims.HDR;
    h.L.RSW = h.dims.RSW;
    h.L.keys = h.keys.data();
    h.L.wordValid = h.wordValid.data();
    h.L.vIsInt = h.vIsInt.data();
    h.L.vInt = h.vInt.data();
    h.topoExcluded = nullptr;
    h.preParsedPods = nullptr;
    host_check(h);
  }
}

// Layout guards: adding a member to one of these types changes its size and stops the build here until the
// member is listed above (sizes of this toolchain's libstdc++, x86-64).
static_assert(sizeof(PodH) == 640, "PodH changed: update io(PodH) in ks_snapshot.cpp");
static_assert(sizeof(Host::Tables) == 1464, "Host::Tables changed: update io(Host::Tables)");
static_assert(sizeof(Host::Node) == 456, "Host::Node changed: update io(Host::Node)");
static_assert(sizeof(Host::Tpl) == 280, "Host::Tpl changed: update io(Host::Tpl)");
static_assert(sizeof(Host::IT) == 224, "Host::IT changed: update io(Host::IT)");
static_assert(sizeof(TopoGroup) == 256, "TopoGroup changed: update io(TopoGroup)");
static_assert(sizeof(PodState) == 144, "PodState changed: update io(PodState)");
static_assert(sizeof(Host) == 3000, "Host changed: update host_io");
static_assert(sizeof(HostPortH) == 88 && sizeof(AffTerm) == 128 && sizeof(SpreadC) == 104 && sizeof(LabelSel) == 32,
              "a pod-spec type changed: update its io()");

void host_save(ArOut& a, Host& h) { host_io(a, h); }
void host_load(ArIn& a, Host& h) { host_io(a, h); }

}  // namespace ks
