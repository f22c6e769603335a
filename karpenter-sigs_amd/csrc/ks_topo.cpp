// ks_topo.cpp — host half of the Topology (pkg/controllers/provisioning/scheduling/topology.go):
// the NewTopology construction the reference runs inside Provisioner.NewScheduler, encoded for the
// device.
//
//   domain universe     provisioner.go:229-283 (pool requirements + labels + instance types)
//   inverse groups      updateInverseAffinities / updateInverseAntiAffinity (topology.go:190-232)
//   owned groups        Update -> newForTopologies / newForAffinities, deduplicated by Hash
//                       (topology.go:91-122,293-337, topologygroup.go:70-91,142-158)
//   initial counts      countDomains over the cluster's bound pods (topology.go:238-291)
//   registration        NewExistingNode registers every node's hostname (existingnode.go:60)
//
// Device view: groups [0, G1) are t.topologies in creation order, [G1, G) t.inverseTopologies; the
// kernels iterate them in that order.  A relaxed state whose groups the initial Update pass did not
// create (a dropped required node-affinity term changes a spread group's node filter, so its hash)
// makes Topology.Update create them mid-Solve (topology.go:102-119): countDomains over the cluster's
// bound pods, the universe domains, and no hostname Register of the existing nodes or of the
// NodeClaims made so far.  Those "late" groups are built here too, after the initial ones (in pod and
// relaxation order), and k_solve activates each one at the relaxation that creates it: before that
// it records nothing, and NodeClaims created before it are not registered in it.
// namespaceSelector terms resolve against the snapshot's namespace list ("namespaces").
#include <algorithm>
#include <climits>
#include <unordered_map>

#include "ks_host.h"
#include "ks_parallel.h"

namespace ks {

namespace {

const char* kHostnameKey = "kubernetes.io/hostname";

bool sel_req_matches(const SelReq& r, const std::map<std::string, std::string>& labels) {
  auto it = labels.find(r.key);
  const bool has = it != labels.end();
  if (r.op == "In") return has && std::find(r.values.begin(), r.values.end(), it->second) != r.values.end();
  if (r.op == "NotIn") return !has || std::find(r.values.begin(), r.values.end(), it->second) == r.values.end();
  if (r.op == "Exists") return has;
  if (r.op == "DoesNotExist") return !has;
  return false;
}
bool sel_valid(const LabelSel& s) {  // LabelSelectorAsSelector: an invalid requirement -> error
  for (auto& r : s.reqs) {
    if ((r.op == "In" || r.op == "NotIn") && r.values.empty()) return false;
    if ((r.op == "Exists" || r.op == "DoesNotExist") && !r.values.empty()) return false;
    if (r.op != "In" && r.op != "NotIn" && r.op != "Exists" && r.op != "DoesNotExist") return false;
  }
  return true;
}
// TopologyGroup.selects (topologygroup.go:259-265): nil or invalid selector -> labels.Nothing()
bool sel_selects(const LabelSel& s, const std::map<std::string, std::string>& labels) {
  if (!s.present || !sel_valid(s)) return false;
  for (auto& r : s.reqs) if (!sel_req_matches(r, labels)) return false;
  return true;
}
// TopologyListOptions (topology.go:381-401): nil -> labels.Everything()
bool sel_lists(const LabelSel& s, const std::map<std::string, std::string>& labels) {
  if (!s.present) return true;
  if (!sel_valid(s)) return false;
  for (auto& r : s.reqs) if (!sel_req_matches(r, labels)) return false;
  return true;
}
std::string sel_key(const LabelSel& s) {  // Hash identity (hashstructure with SlicesAsSets)
  if (!s.present) return "nil";
  std::vector<std::string> parts;
  for (auto& r : s.reqs) {
    std::vector<std::string> v = r.values;
    std::sort(v.begin(), v.end());
    std::string x = r.key + "|" + r.op + "|";
    for (auto& y : v) x += y + ",";
    parts.push_back(x);
  }
  std::sort(parts.begin(), parts.end());
  std::string o;
  for (auto& p : parts) o += p + ";";
  return o;
}

// NewTopologyGroup (topologygroup.go:70-91) + its Hash (topologygroup.go:142-158)
TopoGroup make_group(const Host& h, int type, const std::string& key, const PodH& p, const std::set<std::string>& ns,
                     const LabelSel& sel, int32_t maxSkew, int32_t minDomains) {
  TopoGroup g;
  g.type = type;
  g.key = key;
  g.keyId = h.keyId.at(key);
  g.namespaces = ns;
  g.sel = sel;
  g.maxSkew = maxSkew;
  g.minDomains = minDomains;
  g.filterNil = type != TG_SPREAD;
  if (type == TG_SPREAD) {  // MakeTopologyNodeFilter (topologynodefilter.go:33-51)
    std::vector<uint32_t> sel0 = h.emptyRec();
    h.addLabels(sel0, p.nodeSelector);
    if (p.hasAffinity && p.hasNodeAffinity && p.hasRequired) {
      for (auto& term : p.requiredTerms) {
        std::vector<uint32_t> r = sel0;
        for (auto& n : term) h.addNSR(r, n.key, n.op, n.values);
        g.filter.push_back(r);
      }
    } else {
      g.filter.push_back(sel0);
    }
  }
  g.hash = key + "#" + std::to_string(type) + "#";
  for (auto& n : ns) g.hash += n + ",";
  g.hash += "#" + sel_key(sel) + "#" + std::to_string(maxSkew) + "#";
  if (g.filterNil) g.hash += "nil";
  for (auto& f : g.filter) {  // the filter records' words, as bytes (an exact key, not a printable one)
    g.hash.append(reinterpret_cast<const char*>(f.data()), f.size() * sizeof(uint32_t));
    g.hash += "|";
  }
  return g;
}

// buildNamespaceList (topology.go:339-362): the pod's namespace when neither is set, else the listed
// namespaces plus the namespaces whose labels the selector matches (empty selector: all of them)
std::set<std::string> term_ns(const Host& h, const PodH& p, const AffTerm& t) {
  if (t.namespaces.empty() && !t.nsSelector) return std::set<std::string>{p.ns};
  std::set<std::string> out(t.namespaces.begin(), t.namespaces.end());
  if (!t.nsSelector) return out;
  if (!sel_valid(t.nsSel))
    throw KsError(-1, "pod " + p.ns + "/" + p.name + ": tracking topology counts, parsing selector: invalid namespaceSelector");
  for (auto& ns : h.namespaceList) {
    bool ok = true;
    for (auto& r : t.nsSel.reqs) ok = ok && sel_req_matches(r, ns.second);
    if (ok) out.insert(ns.first);
  }
  return out;
}

std::vector<TopoGroup> anti_groups(const Host& h, const PodH& p) {
  std::vector<TopoGroup> gs;
  for (auto& t : p.antiRequired) gs.push_back(make_group(h, TG_ANTI, t.key, p, term_ns(h, p, t), t.sel, INT32_MAX, -1));
  return gs;
}

// TopologyNodeFilter.Matches (topologynodefilter.go:55-70) against a node's label record
template <class Rec>
bool filter_matches(const Host& h, const TopoGroup& g, Rec nodeRec) {
  if (g.filterNil || g.filter.empty()) return true;
  for (auto& f : g.filter)
    if (rs_present(f.data()) == 0) return true;  // an empty term is Compatible with every record
  const std::vector<uint32_t>& rec = nodeRec();
  for (auto& f : g.filter)
    if (rs_compatible(h.L, rec.data(), f.data(), 0)) return true;
  return false;
}

}  // namespace

void Host::buildTopology() {
  bool any = false;
  for (auto& chain : states)
    for (auto& st : chain) any = any || st.spec != nullptr;
  for (auto& cp : clusterPods) any = any || !cp.antiRequired.empty();
  if (emptyTopology) any = false;  // AddRequirements / Record see no groups; pod affinity terms are inert
  const int P = (int)pods.size(), N = (int)nodes.size(), S = dims.S;
  dims.GMW = 1;
  tab.pod_gsel.assign(std::max(P, 1), 0);
  tab.pod_ginv.assign(std::max(P, 1), 0);
  tab.tg_late.assign(1, 0);
  if (!any) {
    dims.G = dims.G1 = 0;
    dims.tgCntWords = 1;
    dims.tgSmall = 0;
    dims.FSW = dims.RSW;
    tab.tg_meta.assign(TGM_WORDS, 0);
    tab.tg_cnt0.assign(1, 0);
    tab.tg_frs.assign(dims.RSW, 0);
    tab.n_tdom.assign(1, -1);
    dims.TK = 0;
    return;
  }
  PhaseTimer pt("buildTopology");
  // A pod whose VolumeTopology.Inject failed is not in NewTopology's pod list (provisioner.go:432-442): its
  // UID is not excluded from the counts and Topology.Update never ran for it, so its state 0 owns no group;
  // a later relaxation's Update creates and owns its groups (the late groups below).  That Update would also
  // create inverse anti-affinity groups mid-Solve, which the device does not model: refused.
  auto injFailed = [&](int p) { return (size_t)p < injectFailed.size() && injectFailed[(size_t)p]; };
  for (int p = 0; p < P; p++)
    if (injFailed(p) && pods[(size_t)p].hasAffinity && pods[(size_t)p].hasPodAnti && !pods[(size_t)p].antiRequired.empty())
      throw KsError(-2, "pod " + pods[(size_t)p].ns + "/" + pods[(size_t)p].name +
                            ": volume topology injection failed and the pod has required pod anti-affinity (its "
                            "inverse groups would be created mid-Solve)");
  // --- domain universe (provisioner.go:229-283)
  std::map<std::string, std::set<std::string>> dom;
  auto valuesOf = [&](const std::vector<uint32_t>& rec, int k) {  // Requirement.Values(): the raw set
    std::vector<std::string> out;
    const KeyMeta& km = keys[(size_t)k];
    for (int b = 0; b < (int)values[(size_t)k].size(); b++)
      if ((rec[(size_t)(L.HDR + km.off + (b >> 5))] >> (b & 31)) & 1u) out.push_back(values[(size_t)k][(size_t)b]);
    return out;
  };
  for (auto& t : tpls) {
    if (t.its.empty()) continue;
    std::vector<uint32_t> base = emptyRec();
    for (auto& n : t.reqs) addNSR(base, n.key, n.op, n.values);
    addLabels(base, t.poolLabels);
    for (int i : t.its) {
      std::vector<uint32_t> r = base;
      rs_add(L, r.data(), &tab.it_rs[(size_t)i * dims.RSW]);
      const uint64_t pr = rs_present(r.data());
      for (int k = 0; k < dims.NK; k++)
        if (bit(pr, k)) for (auto& v : valuesOf(r, k)) dom[keyNames[(size_t)k]].insert(v);
    }
    const uint64_t pr = rs_present(base.data());
    for (int k = 0; k < dims.NK; k++)
      if (bit(pr, k) && rs_op(L, base.data(), k) == OP_IN) for (auto& v : valuesOf(base, k)) dom[keyNames[(size_t)k]].insert(v);
  }

  pt.mark("universe");
  // --- groups
  // NewTopology's excludedPods: the UIDs of the pods it receives, which leaves out those whose injection failed
  // (provisioner.go:432-442).  The consolidation view excludes only the pods every simulation schedules (pending,
  // deleting nodes'); each simulation then takes its candidates' counted pods out (ks_cons.cpp sim_topology).
  std::set<std::string> excluded;
  if (topoExcluded) {
    excluded = *topoExcluded;
    for (int p = 0; p < P; p++)
      if (injFailed(p)) excluded.erase(pods[(size_t)p].uid);
  } else {
    for (int p = 0; p < P; p++)
      if (!injFailed(p)) excluded.insert(pods[(size_t)p].uid);
  }
  topoContrib.clear();
  topoInvOwner.clear();
  // (group index, domain) per counted cluster pod, resolved to value ids once the groups are final
  std::unordered_map<std::string, std::vector<std::pair<int, std::string>>> contrib;  // uid -> contributions (per-uid order kept)
  std::vector<TopoGroup> own, inv;
  std::unordered_map<std::string, int> ownByHash, invByHash;  // lookups only (creation order is kept by the vectors)
  // every node's label record, built once (before the first node filter needs one; read-only after,
  // so countDomains' worker threads share it)
  std::map<std::string, std::vector<uint32_t>> nodeRecs;
  bool nodeRecsBuilt = false;
  auto buildNodeRecs = [&]() {
    if (nodeRecsBuilt) return;
    for (auto& n : nodeLabelsByName) {
      std::vector<uint32_t> r = emptyRec();
      addNodeLabels(r, n.second);  // (the filter terms name only universe keys)
      nodeRecs.emplace(n.first, std::move(r));
    }
    nodeRecsBuilt = true;
  };
  auto filterMatches = [&](const TopoGroup& g, const std::string& name) {
    return filter_matches(*this, g, [&]() -> const std::vector<uint32_t>& { return nodeRecs.at(name); });
  };
  // TopologyGroup.domains starts with the universe's values of the key (NewTopologyGroup); seeded only
  // for groups that are new (a pod whose group exists already shares it)
  auto seedDomains = [&](TopoGroup& g) {
    auto d = dom.find(g.key);
    if (d != dom.end()) for (auto& v : d->second) g.domains[v] = 0;
  };
  auto makeGroup = [&](int type, const std::string& key, const PodH& p, const std::set<std::string>& ns,
                       const LabelSel& sel, int32_t maxSkew, int32_t minDomains) {
    return make_group(*this, type, key, p, ns, sel, maxSkew, minDomains);
  };
  auto termNs = [&](const PodH& p, const AffTerm& t) { return term_ns(*this, p, t); };
  auto countDomains = [&](TopoGroup& g, int gidx) {  // topology.go:238-291
    if (!g.filterNil && !g.filter.empty()) buildNodeRecs();
    // each cluster pod's domain (or none), on worker threads; counted in pod order
    const int NC = (int)clusterPods.size();
    std::vector<const std::string*> dsel((size_t)NC, nullptr);
    parallel_for(NC, 1024, [&](int i) {
      const PodH& cp = clusterPods[(size_t)i];
      if (!g.namespaces.count(cp.ns) || !sel_lists(g.sel, cp.labels)) return;
      if (cp.nodeName.empty() || cp.phase == "Failed" || cp.phase == "Succeeded" || cp.deleting) return;
      if (excluded.count(cp.uid)) return;
      auto n = nodeLabelsByName.find(cp.nodeName);
      if (n == nodeLabelsByName.end()) return;
      auto l = n->second.find(g.key);
      const std::string* d;
      if (l != n->second.end()) d = &l->second;
      else if (g.key == kHostnameKey) d = &n->first;
      else return;
      if (!filterMatches(g, n->first)) return;
      dsel[(size_t)i] = d;
    });
    for (int i = 0; i < NC; i++) {
      if (!dsel[(size_t)i]) continue;
      g.domains[*dsel[(size_t)i]]++;
      if (topoExcluded) contrib[clusterPods[(size_t)i].uid].push_back({gidx, *dsel[(size_t)i]});
    }
  };
  auto antiGroups = [&](const PodH& p) { return anti_groups(*this, p); };
  // a state's first constraint of each group sets the minDomains its Update would create the group with; those
  // differing from the group's (the whole problem's first creator's) are kept per state (PodState::gmd)
  auto noteMd = [&](const std::vector<int32_t>& seen, std::vector<std::pair<int32_t, int32_t>>& gmd, int idx, int32_t md) {
    if (std::find(seen.begin(), seen.end(), idx) != seen.end()) return;
    if (md != own[(size_t)idx].minDomains) gmd.push_back({idx, md});
  };
  auto inverseAnti = [&](const PodH& p, std::vector<TopoGroup> gs, const std::map<std::string, std::string>* labels,
                         bool cluster) {
    std::vector<int32_t> owned;  // updateInverseAntiAffinity (topology.go:207-232): inverse group indices
    for (TopoGroup& g : gs) {
      auto it = invByHash.find(g.hash);
      int idx;
      if (it == invByHash.end()) {
        idx = (int)inv.size();
        invByHash[g.hash] = idx;
        seedDomains(g);
        inv.push_back(g);
      } else {
        idx = it->second;
      }
      if (labels) {
        auto d = labels->find(inv[(size_t)idx].key);
        if (d != labels->end()) {
          inv[(size_t)idx].domains[d->second]++;
          if (topoExcluded) contrib[p.uid].push_back({-1 - idx, d->second});
        }
      }
      if (cluster && topoExcluded) topoInvOwner[p.uid].push_back(idx);
      owned.push_back(idx);
    }
    return owned;
  };
  auto ownedSpecGroups = [&](const PodH& sp) {  // newForTopologies + newForAffinities
    std::vector<TopoGroup> fresh;
    for (auto& c : sp.tsc) fresh.push_back(makeGroup(TG_SPREAD, c.key, sp, {sp.ns}, c.sel, c.maxSkew, c.minDomains));
    if (sp.hasAffinity && sp.hasPodAffinity) {  // the type map's affinity entry first (canonical order)
      for (auto& t : sp.affRequired) fresh.push_back(makeGroup(TG_AFFINITY, t.key, sp, termNs(sp, t), t.sel, INT32_MAX, -1));
      for (auto& t : sp.affPreferred)
        fresh.push_back(makeGroup(TG_AFFINITY, t.second.key, sp, termNs(sp, t.second), t.second.sel, INT32_MAX, -1));
    }
    if (sp.hasAffinity && sp.hasPodAnti) {
      for (auto& t : sp.antiRequired) fresh.push_back(makeGroup(TG_ANTI, t.key, sp, termNs(sp, t), t.sel, INT32_MAX, -1));
      for (auto& t : sp.antiPreferred)
        fresh.push_back(makeGroup(TG_ANTI, t.second.key, sp, termNs(sp, t.second), t.second.sel, INT32_MAX, -1));
    }
    return fresh;
  };
  for (auto& cp : clusterPods) {  // ForPodsWithAntiAffinity: bound pods with required anti-affinity
    if (cp.antiRequired.empty() || cp.nodeName.empty() || excluded.count(cp.uid)) continue;
    auto n = nodeLabelsByName.find(cp.nodeName);
    if (n == nodeLabelsByName.end()) continue;
    inverseAnti(cp, antiGroups(cp), &n->second, true);
  }
  pt.mark("cluster inverse anti-affinity");
  // the groups each pod's spec implies, built on worker threads (independent per pod), then
  // deduplicated by hash in pod order exactly as the sequential Update calls would
  std::vector<std::vector<TopoGroup>> podAnti((size_t)P), podOwn((size_t)P);
  std::vector<char> podHasAnti((size_t)P, 0);
  parallel_for(P, 64, [&](int p) {
    const std::shared_ptr<PodH>& sp = states[(size_t)p][0].spec;
    if (!sp || injFailed(p)) return;
    if (sp->hasAffinity && sp->hasPodAnti && (!sp->antiRequired.empty() || !sp->antiPreferred.empty())) {
      podHasAnti[(size_t)p] = 1;
      podAnti[(size_t)p] = antiGroups(*sp);
    }
    podOwn[(size_t)p] = ownedSpecGroups(*sp);
  });
  pt.mark("pods' groups (workers)");
  std::vector<std::vector<int32_t>> invOwned(P);
  for (int p = 0; p < P; p++) {  // NewTopology: Update(pod) for every pod, in order
    const std::shared_ptr<PodH>& sp = states[(size_t)p][0].spec;
    if (!sp || injFailed(p)) continue;
    if (podHasAnti[(size_t)p]) invOwned[(size_t)p] = inverseAnti(*sp, std::move(podAnti[(size_t)p]), nullptr, false);
    std::vector<int32_t> gown;
    std::vector<std::pair<int32_t, int32_t>> gmd;
    for (auto& g : podOwn[(size_t)p]) {
      auto it = ownByHash.find(g.hash);
      int idx;
      if (it == ownByHash.end()) {
        idx = (int)own.size();
        seedDomains(g);
        countDomains(g, idx);
        ownByHash[g.hash] = idx;
        own.push_back(g);
      } else {
        idx = it->second;
      }
      noteMd(gown, gmd, idx, g.minDomains);
      gown.push_back(idx);
    }
    std::sort(gown.begin(), gown.end());
    gown.erase(std::unique(gown.begin(), gown.end()), gown.end());
    states[(size_t)p][0].gown = std::move(gown);
    states[(size_t)p][0].gmd = std::move(gmd);
  }
  pt.mark("pods' groups + countDomains");
  std::vector<int32_t> late;
  for (int p = 0; p < P; p++)
    for (size_t k = 1; k < states[(size_t)p].size(); k++) {
      PodState& st = states[(size_t)p][k];
      if (!st.spec) continue;
      std::vector<int32_t> gown;
      std::vector<std::pair<int32_t, int32_t>> gmd;
      for (auto& g : ownedSpecGroups(*st.spec)) {
        auto it = ownByHash.find(g.hash);
        int idx;
        if (it == ownByHash.end()) {  // created by this relaxation's Update (topology.go:102-119)
          idx = (int)own.size();
          seedDomains(g);
          countDomains(g, idx);
          g.late = true;
          ownByHash[g.hash] = idx;
          own.push_back(g);
          late.push_back(idx);
        } else {
          idx = it->second;
        }
        noteMd(gown, gmd, idx, g.minDomains);
        gown.push_back(idx);
      }
      std::sort(gown.begin(), gown.end());
      gown.erase(std::unique(gown.begin(), gown.end()), gown.end());
      st.gown = std::move(gown);
      st.gmd = std::move(gmd);
    }
  for (int p = 0; p < P; p++)
    for (size_t k = 1; k < states[(size_t)p].size(); k++)
      for (auto& gm : states[(size_t)p][k].gmd)
        if (own[(size_t)gm.first].late)
          throw KsError(-2, "topology group created by relaxations whose spread constraints differ in minDomains "
                            "(the group's minDomains would depend on which relaxation runs first)");
  pt.mark("relaxation states' groups");
  // Group sets are GMW-word bitsets on the device (no 64-group limit); the group index rides in bits 16..31
  // of a topology failure code (FC_TOPO), and the group table must fit the LDS plan (make_plan refuses it
  // with KS_ERR_CAPACITY long before this bound).
  if (own.size() + inv.size() > 65535) throw KsError(-3, "more than 65535 topology groups");
  const int G1 = (int)own.size(), G = G1 + (int)inv.size();
  const int GMW = std::max(1, (G + 63) / 64);
  dims.GMW = GMW;
  tab.tg_late.assign((size_t)GMW, 0);
  for (int g : late) gset(tab.tg_late, 0, GMW, g);
  groups = own;
  groups.insert(groups.end(), inv.begin(), inv.end());
  groupsOwned = G1;
  for (auto& g : groups)  // NewExistingNode registers every node's hostname (existingnode.go:60)
    if (g.key == kHostnameKey && !g.late)  // in the groups that exist by then
      for (auto& n : nodes) g.domains.emplace(n.hostName, 0);
  tab.pod_gsel.assign((size_t)std::max(P, 1) * GMW, 0);
  tab.pod_ginv.assign((size_t)std::max(P, 1) * GMW, 0);
  parallel_for(P, 256, [&](int p) {  // per pod, independent (each writes its own row)
    for (int i : invOwned[(size_t)p]) gset(tab.pod_ginv, (size_t)p, GMW, G1 + i);
    for (int g = 0; g < G; g++)
      if (groups[(size_t)g].namespaces.count(pods[(size_t)p].ns) && sel_selects(groups[(size_t)g].sel, pods[(size_t)p].labels))
        gset(tab.pod_gsel, (size_t)p, GMW, g);
  });

  pt.mark("hostnames + pod selectors");
  // --- device tables
  tab.tg_meta.assign((size_t)G * TGM_WORDS, 0);
  tab.tg_cnt0.clear();
  tab.tg_frs.clear();
  int maxNv = 0;
  // Count-table layout: the groups over small keys (zone, capacity type, ...) first, up to kTgSmallCap
  // words -- k_solve keeps that prefix in LDS -- then the hostname groups (one word per node), which stay
  // in HBM (copy-on-write per simulation).
  constexpr size_t kTgSmallCap = 2048;
  std::vector<int> order;
  std::vector<char> isSmall((size_t)G, 0);
  size_t smallWords = 0;
  for (int g = 0; g < G; g++) {
    const size_t nv = std::max<size_t>(values[(size_t)groups[(size_t)g].keyId].size(), 1);
    if (groups[(size_t)g].key != kHostnameKey && smallWords + nv <= kTgSmallCap) {
      isSmall[(size_t)g] = 1;
      smallWords += nv;
      order.push_back(g);
    }
  }
  for (int g = 0; g < G; g++)
    if (!isSmall[(size_t)g]) order.push_back(g);
  dims.tgSmall = 0;
  std::vector<std::vector<int32_t>> cnts((size_t)G);
  for (int g = 0; g < G; g++) {
    TopoGroup& tg = groups[(size_t)g];
    int32_t* m = &tab.tg_meta[(size_t)g * TGM_WORDS];
    const int nv = (int)values[(size_t)tg.keyId].size();  // universe values (the hostname private bit excluded)
    maxNv = std::max(maxNv, nv);
    m[TGM_TYPE] = tg.type;
    m[TGM_KEY] = tg.keyId;
    m[TGM_SKEW] = tg.maxSkew;
    m[TGM_MIND] = tg.minDomains;
    m[TGM_NV] = nv;
    m[TGM_FBEG] = (int32_t)(tab.tg_frs.size() / dims.RSW);
    m[TGM_HOST] = tg.key == kHostnameKey ? 1 : 0;
    std::vector<int32_t> cnt(std::max(nv, 1), -1);  // -1: domain not registered (absent from the map)
    for (auto& kv : tg.domains) {
      auto vi = valueId[(size_t)tg.keyId].find(kv.first);
      if (vi == valueId[(size_t)tg.keyId].end())
        throw KsError(-5, "topology domain " + kv.first + " outside the value universe of " + tg.key);
      cnt[(size_t)vi->second] = kv.second;
    }
    cnts[(size_t)g] = std::move(cnt);
    bool trivial = false;  // an empty term is Compatible with everything: the filter always matches
    for (auto& f : tg.filter) trivial = trivial || rs_present(f.data()) == 0;
    if (!trivial)
      for (auto& f : tg.filter) tab.tg_frs.insert(tab.tg_frs.end(), f.begin(), f.end());
    m[TGM_FEND] = (int32_t)(tab.tg_frs.size() / dims.RSW);
  }
  if (tab.tg_frs.empty()) tab.tg_frs.assign(dims.RSW, 0);
  for (size_t i = 0; i < order.size(); i++) {
    const int g = order[i];
    tab.tg_meta[(size_t)g * TGM_WORDS + TGM_CNT] = (int32_t)tab.tg_cnt0.size();
    tab.tg_cnt0.insert(tab.tg_cnt0.end(), cnts[(size_t)g].begin(), cnts[(size_t)g].end());
    if (isSmall[(size_t)g]) dims.tgSmall = (int32_t)tab.tg_cnt0.size();
  }
  // A node's domain depends on the key only: one row per distinct topology key ([TK][N]; a wave reads 64
  // nodes of one key), small enough for a Solve to keep in LDS.
  std::vector<int> slotKey, slotOf(keyNames.size(), -1);
  for (int g = 0; g < G; g++) {
    const int k = groups[(size_t)g].keyId;
    if (slotOf[(size_t)k] < 0) {
      slotOf[(size_t)k] = (int)slotKey.size();
      slotKey.push_back(k);
    }
    tab.tg_meta[(size_t)g * TGM_WORDS + TGM_KSLOT] = slotOf[(size_t)k];
  }
  dims.TK = (int32_t)slotKey.size();
  tab.n_tdom.assign((size_t)std::max(N, 1) * std::max(dims.TK, 1), -1);
  for (int n = 0; n < N; n++)
    for (int k = 0; k < dims.TK; k++) {
      const std::string& key = keyNames[(size_t)slotKey[(size_t)k]];
      std::string d;
      if (key == kHostnameKey) {
        d = nodes[(size_t)n].hostName;
      } else {
        auto l = nodes[(size_t)n].labels.find(key);
        if (l == nodes[(size_t)n].labels.end()) continue;
        d = l->second;
      }
      tab.n_tdom[(size_t)k * N + n] = valueId[(size_t)slotKey[(size_t)k]].at(d);
    }
  // A node without a group's label takes that key only from a pod's NotIn requirement
  // (existingnode.go:97-115: the strict Compatible admits nothing else), after which the topology
  // domain is chosen like a NodeClaim's; k_solve decides such nodes wave-wide (node_slow).
  dims.tgUnlab = 0;
  for (size_t i = 0; i < tab.n_tdom.size() && G > 0 && N > 0; i++) dims.tgUnlab |= tab.n_tdom[i] < 0;
  pt.mark("count tables + node domains");
  if (topoExcluded) {  // the consolidation view: what each simulation's exclusions take away
    for (auto& kv : contrib)
      for (auto& gd : kv.second) {
        const int g = gd.first >= 0 ? gd.first : G1 + (-1 - gd.first);
        topoContrib[kv.first].push_back({g, valueId[(size_t)groups[(size_t)g].keyId].at(gd.second)});
      }
    for (auto& kv : topoInvOwner) {  // (a pod owning one group twice owns it once)
      std::sort(kv.second.begin(), kv.second.end());
      kv.second.erase(std::unique(kv.second.begin(), kv.second.end()), kv.second.end());
      for (int32_t& i : kv.second) i += G1;
    }
    topoInvOwners.assign((size_t)G, 0);
    for (auto& kv : topoInvOwner)
      for (int32_t g : kv.second) topoInvOwners[(size_t)g]++;
    topoHostActive.clear();
    if (keyId.count(kHostnameKey))
      for (auto& n : nodes) {
        auto v = valueId[(size_t)keyId.at(kHostnameKey)].find(n.hostName);
        if (v != valueId[(size_t)keyId.at(kHostnameKey)].end()) topoHostActive.insert(v->second);
      }
    topoUniverse.assign((size_t)G, {});
    for (int g = 0; g < G; g++) {
      const TopoGroup& tg = groups[(size_t)g];
      topoUniverse[(size_t)g].assign(values[(size_t)tg.keyId].size(), 0);
      auto d = dom.find(tg.key);
      if (d != dom.end())
        for (auto& v : d->second) topoUniverse[(size_t)g][(size_t)valueId[(size_t)tg.keyId].at(v)] = 1;
    }
  }
  dims.G = G;
  dims.G1 = G1;
  dims.tgMaxNv = maxNv;
  dims.FSW = dims.RSW;
  for (auto& g : groups)
    if (g.key != kHostnameKey) {
      const int nv = (int)values[(size_t)g.keyId].size();
      dims.FSW = std::max(dims.FSW, nv);
    }
  dims.tgCntWords = (int32_t)tab.tg_cnt0.size();
  pt.mark("consolidation contributions");
}

// ks_cons_update's bindPods in a topology cluster: what countDomains (topology.go:238-291) and
// ForPodsWithAntiAffinity's inverse counts (topology.go:190-203) take from one more bound cluster pod under
// the groups the build made: (group, value) contributions and the inverse groups it owns.  False when a
// domain or an inverse group it needs is outside the build's universe (the caller refuses the update).
bool Host::topoClusterPod(const PodH& cp, std::vector<std::pair<int, int>>& contrib, std::vector<int32_t>& inv) const {
  contrib.clear();
  inv.clear();
  if (cp.nodeName.empty()) return true;
  auto n = nodeLabelsByName.find(cp.nodeName);
  if (n == nodeLabelsByName.end()) return true;
  std::vector<uint32_t> rec;
  auto nodeRec = [&]() -> const std::vector<uint32_t>& {
    if (rec.empty()) {
      rec = emptyRec();
      addNodeLabels(rec, n->second);
    }
    return rec;
  };
  auto domainOf = [&](const TopoGroup& g, int* v) {
    auto l = n->second.find(g.key);
    const std::string* d;
    if (l != n->second.end()) d = &l->second;
    else if (g.key == kHostnameKey) d = &n->first;
    else return 0;  // no domain: not counted
    auto it = valueId[(size_t)g.keyId].find(*d);
    if (it == valueId[(size_t)g.keyId].end()) return -1;
    *v = it->second;
    return 1;
  };
  const int G1 = dims.G1, G = dims.G;
  if (!(cp.phase == "Failed" || cp.phase == "Succeeded" || cp.deleting))
    for (int g = 0; g < G1; g++) {
      const TopoGroup& tg = groups[(size_t)g];
      if (!tg.namespaces.count(cp.ns) || !sel_lists(tg.sel, cp.labels)) continue;
      int v = 0;
      const int k = domainOf(tg, &v);
      if (k < 0) return false;
      if (k == 0 || !filter_matches(*this, tg, nodeRec)) continue;
      contrib.push_back({g, v});
    }
  if (!cp.antiRequired.empty())
    for (const TopoGroup& ag : anti_groups(*this, cp)) {
      int idx = -1;
      for (int g = G1; g < G && idx < 0; g++)
        if (groups[(size_t)g].hash == ag.hash) idx = g;
      if (idx < 0) return false;
      auto d = n->second.find(groups[(size_t)idx].key);  // (the inverse count reads the label only)
      if (d != n->second.end()) {
        auto it = valueId[(size_t)groups[(size_t)idx].keyId].find(d->second);
        if (it == valueId[(size_t)groups[(size_t)idx].keyId].end()) return false;
        contrib.push_back({idx, it->second});
      }
      inv.push_back(idx);
    }
  std::sort(inv.begin(), inv.end());
  inv.erase(std::unique(inv.begin(), inv.end()), inv.end());
  return true;
}

}  // namespace ks
