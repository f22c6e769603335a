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
template <class A> void io(A& a, PodState& x) { io_all(a, x.hasPreferred, x.tols, x.gown, x.spec); }
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
         t.off_price, t.n_flags, t.pod_flags, t.pod_hpc, t.pod_hpu, t.pod_hpo, t.n_hp0, t.pod_vm, t.vol_dm, t.n_vm0, t.n_vc0,
         t.n_vlim, t.tg_meta, t.tg_cnt0, t.tg_frs, t.st_gown, t.pod_gsel, t.pod_ginv, t.n_tdom, t.it_rs, t.tpl_rs, t.n_rs0,
         t.pool_mask, t.st_toltpl, t.tpl_taint, t.st_tol, t.n_taint, t.tsort_pos, t.it_off_beg, t.off_zone, t.off_ct,
         t.tpl_it_beg, t.tpl_its, t.tpl_pool, t.pod_state0, t.pod_nstate, t.pod_uid, t.st_flags, t.pod_rmask, t.tpl_rmask,
         t.pod_rfmt, t.tpl_rfmt, t.fk_words, t.fk_key_off, t.fk_tpl);
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
  std::vector<uint64_t> off(n + 1, 0);
  if constexpr (A::reading) {
    v.resize(n);
    io(a, off);
    if (off.size() != n + 1 || off[n] > (uint64_t)(a.end - a.p)) throw ArchiveError("binary snapshot offsets out of range");
    const char* base = a.p;
    parallel_for((int)n, 64, [&](int i) {
      if (off[(size_t)i] > off[(size_t)i + 1]) throw ArchiveError("binary snapshot offsets out of order");
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

// The layout pointers (L) point into the vectors and are re-aimed after a load; the build-only members
// (topoExcluded, preParsedPods, the value-set scratch) are not part of the model a snapshot carries.
template <class A> void host_io(A& a, Host& h) {
  PhaseTimer pt(A::reading ? "host_load" : "host_save");
  io_all(a, h.keyNames, h.keyId, h.values, h.valueId, h.keys, h.wordValid, h.vIsInt, h.vInt, h.hostKey, h.zoneKey, h.ctKey,
         h.hostPrivBit, h.allowWK, h.itKeys, h.wellKnown, h.resNames, h.resId, h.resShift, h.taints, h.hostPortUniverse,
         h.hostPortOwner, h.volumeDrivers, h.volDrivers, h.volUniverse, h.its, h.tpls, h.pools, h.toleratePreferNoSchedule,
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
  }
}

// Layout guards: adding a member to one of these types changes its size and stops the build here until the
// member is listed above (sizes of this toolchain's libstdc++, x86-64).
static_assert(sizeof(PodH) == 640, "PodH changed: update io(PodH) in ks_snapshot.cpp");
static_assert(sizeof(Host::Tables) == 1344, "Host::Tables changed: update io(Host::Tables)");
static_assert(sizeof(Host::Node) == 456, "Host::Node changed: update io(Host::Node)");
static_assert(sizeof(Host::Tpl) == 280, "Host::Tpl changed: update io(Host::Tpl)");
static_assert(sizeof(Host::IT) == 224, "Host::IT changed: update io(Host::IT)");
static_assert(sizeof(TopoGroup) == 256, "TopoGroup changed: update io(TopoGroup)");
static_assert(sizeof(PodState) == 104, "PodState changed: update io(PodState)");
static_assert(sizeof(Host) == 2848, "Host changed: update host_io");
static_assert(sizeof(HostPortH) == 88 && sizeof(AffTerm) == 128 && sizeof(SpreadC) == 104 && sizeof(LabelSel) == 32,
              "a pod-spec type changed: update its io()");

void host_save(ArOut& a, Host& h) { host_io(a, h); }
void host_load(ArIn& a, Host& h) { host_io(a, h); }

}  // namespace ks
