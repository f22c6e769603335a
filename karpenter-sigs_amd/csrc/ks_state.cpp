// ks_state.cpp — cluster-state accounting: StateNode accessor values from the API objects.
//
// The snapshot the Solve / consolidation entry points read carries, per StateNode, the values of its
// accessors (Name, HostName, Labels, Taints, Capacity, Available, DaemonSetRequests, Initialized,
// HostPortUsage, MarkedForDeletion).  In the reference those are maintained by the cluster-state
// informers.  ks_cluster_state derives the state they converge to from the object lists:
//   Cluster.UpdateNodeClaim / UpdateNode      pkg/controllers/state/cluster.go:220-263
//   newStateFromNode + populateResourceRequests cluster.go:415-490 (bound, non-terminal pods)
//   updateNodeUsageFromPod / updateForPod     cluster.go:492-512, statenode.go:314-333
//   StateNode accessors                       statenode.go:110-298 (Name, HostName, Labels, Taints,
//                                             Registered, Initialized, Capacity, Allocatable,
//                                             Available, DaemonSetRequests, PodRequests, MarkedForDeletion)
//   KnownEphemeralTaints / Taint.MatchTaint   pkg/scheduling/taints.go:28-32 (k8s.io/api v0.28.4)
//   resources.Merge / MergeInto / Subtract    pkg/utils/resources/resources.go:49-96
// Host-only (no device).  Pure function of its input; output order is canonical (NodeClaims with a
// providerID in input order, then Nodes not paired with one, in input order).
#include <algorithm>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "../../include/karpenter_amd.h"
#include "ks_host.h"
#include "ks_runtime.h"

namespace ks {
namespace {

using ksjson::Value;

const char* const kPoolLabel = "karpenter.sh/nodepool";
const char* const kInitLabel = "karpenter.sh/initialized";
const char* const kRegLabel = "karpenter.sh/registered";
const char* const kITLabel = "node.kubernetes.io/instance-type";
const char* const kHostLabel = "kubernetes.io/hostname";

std::string sget(const Value* v, const char* k) {
  const Value* x = v ? v->get(k) : nullptr;
  return x && x->is_str() ? x->s : std::string();
}
const Value* path(const Value* v, std::initializer_list<const char*> ks) {
  for (const char* k : ks) {
    if (!v || !v->is_obj()) return nullptr;
    v = v->get(k);
  }
  return v;
}
std::map<std::string, std::string> smap(const Value* v) {
  std::map<std::string, std::string> m;
  if (v && v->is_obj())
    for (auto& kv : v->obj()) m[kv.first] = kv.second.str();
  return m;
}
QList qlist(const Value* v) {
  QList q;
  if (v && v->is_obj())
    for (auto& kv : v->obj()) q[kv.first] = qty_parse(kv.second.str());
  return q;
}
std::vector<TaintH> taints(const Value* v) {
  std::vector<TaintH> out;
  if (v && v->is_arr())
    for (auto& e : v->arr()) out.push_back(TaintH{sget(&e, "key"), sget(&e, "value"), sget(&e, "effect")});
  return out;
}
bool deleting(const Value* obj) {
  const Value* d = path(obj, {"metadata", "deletionTimestamp"});
  return d && !d->is_null() && !(d->is_str() && d->s.empty());
}

struct Entry {
  const Value* node = nullptr;
  const Value* claim = nullptr;
  std::map<std::string, QList> podRequests, dsRequests;  // by pod key "ns/name" (sorted: canonical sums)
  std::map<std::string, std::vector<HostPortH>> ports;
  std::map<std::string, std::map<std::string, std::set<std::string>>> volumes;  // pod key -> driver -> PVC ids
  std::vector<const Value*> pods;  // bound pods (GetNodePods' listing, unfiltered)

  std::map<std::string, std::string> nodeLabels() const { return smap(path(node, {"metadata", "labels"})); }
  bool managed() const { return claim || (node && !nodeLabels()[kPoolLabel].empty()); }
  bool registered() const { return !managed() || (node && nodeLabels()[kRegLabel] == "true"); }
  bool initialized() const { return !managed() || (node && nodeLabels()[kInitLabel] == "true"); }
  // the NodeClaim's representation until the Node registers (statenode.go:110-181)
  const Value* face() const { return !node || (claim && !registered()) ? claim : node; }
  std::string name() const { return sget(path(face(), {"metadata"}), "name"); }
  std::map<std::string, std::string> labels() const { return smap(path(face(), {"metadata", "labels"})); }
  std::string hostName() const {
    auto l = labels();
    auto it = l.find(kHostLabel);
    return it == l.end() || it->second.empty() ? name() : it->second;
  }
  std::vector<TaintH> taintList() const {
    // Taints() (statenode.go:183-205): known ephemeral taints, plus the startup taints until initialized
    std::vector<TaintH> eph = {{"node.kubernetes.io/not-ready", "", "NoSchedule"},
                               {"node.kubernetes.io/unreachable", "", "NoSchedule"},
                               {"node.cloudprovider.kubernetes.io/uninitialized", "true", "NoSchedule"}};
    if (!initialized() && managed() && claim)
      for (auto& t : taints(path(claim, {"spec", "startupTaints"}))) eph.push_back(t);
    const bool fromClaim = (!registered() && claim) || !node;
    std::vector<TaintH> out;
    for (auto& t : taints(fromClaim ? path(claim, {"spec", "taints"}) : path(node, {"spec", "taints"}))) {
      bool eph_ = false;
      for (auto& e : eph) eph_ = eph_ || (e.key == t.key && e.effect == t.effect);  // Taint.MatchTaint
      if (!eph_) out.push_back(t);
    }
    return out;
  }
  // Capacity() / Allocatable() (statenode.go:225-259): zero Node values take the NodeClaim's until initialized
  QList resources(const char* field) const {
    if (!initialized() && claim) {
      QList fromClaim = qlist(path(claim, {"status", field}));
      if (!node) return fromClaim;
      QList ret = qlist(path(node, {"status", field}));
      for (auto& kv : fromClaim) {
        auto it = ret.find(kv.first);
        if (it == ret.end() || it->second.n == 0) ret[kv.first] = kv.second;
      }
      return ret;
    }
    return qlist(path(node, {"status", field}));
  }
};

void dump(std::string& o, const Value& v) {
  switch (v.kind) {
    case Value::Null: o += "null"; break;
    case Value::Bool: o += v.b ? "true" : "false"; break;
    case Value::Number: o += v.s; break;
    case Value::String: ksjson::quote(o, v.s); break;
    case Value::Arr: {
      o += "[";
      for (size_t i = 0; i < v.arr().size(); i++) {
        if (i) o += ",";
        dump(o, v.arr()[i]);
      }
      o += "]";
      break;
    }
    case Value::Obj: {
      o += "{";
      bool first = true;
      for (auto& kv : v.obj()) {
        if (!first) o += ",";
        first = false;
        ksjson::quote(o, kv.first);
        o += ":";
        dump(o, kv.second);
      }
      o += "}";
      break;
    }
  }
}

void put_qlist(std::string& o, const QList& q) {
  o += "{";
  bool first = true;
  for (auto& kv : q) {
    if (!first) o += ",";
    first = false;
    ksjson::quote(o, kv.first);
    o += ":";
    ksjson::quote(o, qty_str(kv.second));
  }
  o += "}";
}

}  // namespace

std::string cluster_state_json(const Value& root) {
  std::vector<std::string> order;  // providerIDs, canonical order
  std::map<std::string, Entry> byID;
  auto entry = [&](const std::string& id) -> Entry& {
    if (!byID.count(id)) order.push_back(id);
    return byID[id];
  };
  if (const Value* ncs = root.get("nodeClaims"))
    for (auto& nc : ncs->arr()) {
      const std::string id = sget(path(&nc, {"status"}), "providerID");
      if (id.empty()) continue;  // UpdateNodeClaim: no providerID yet (cluster.go:224-226)
      entry(id).claim = &nc;
    }
  std::map<std::string, std::string> nodeNameToID;
  if (const Value* ns = root.get("nodes"))
    for (auto& n : ns->arr()) {
      auto l = smap(path(&n, {"metadata", "labels"}));
      const bool managed = !l[kPoolLabel].empty(), initialized = !l[kInitLabel].empty();
      std::string id = sget(path(&n, {"spec"}), "providerID");
      if (id.empty()) {
        if (managed) continue;  // UpdateNode (cluster.go:243-249)
        id = sget(path(&n, {"metadata"}), "name");
      }
      if (managed && l[kITLabel].empty() && !initialized) continue;  // cluster.go:252-255
      entry(id).node = &n;
      nodeNameToID[sget(path(&n, {"metadata"}), "name")] = id;
    }
  const Value* drivers = root.get("volumeDrivers");
  if (const Value* ps = root.get("pods"))
    for (auto& pv : ps->arr()) {
      PodH p = parse_pod(pv);
      if (p.nodeName.empty()) continue;
      auto id = nodeNameToID.find(p.nodeName);
      if (id == nodeNameToID.end()) continue;  // NotFound: the node is not tracked (cluster.go:500-504)
      Entry& e = byID[id->second];
      e.pods.push_back(&pv);
      if (p.terminal) continue;  // UpdatePod: terminal pods release their usage (cluster.go:277-281)
      const std::string key = p.ns + "/" + p.name;
      e.podRequests[key] = p.requests;  // updateForPod (statenode.go:314-333)
      if (p.ownedByDaemonSet) e.dsRequests[key] = p.requests;
      else e.dsRequests.erase(key);
      e.ports[key] = p.ports;
      // GetVolumes (volumeusage.go:82-113): PVC id "ns/claim" -> CSI driver; unresolved ones are skipped
      auto& vol = e.volumes[key];
      vol.clear();
      for (auto& claim : p.pvcNames) {
        const std::string id = p.ns + "/" + claim;
        const Value* drv = drivers ? drivers->get(id) : nullptr;
        if (drv && drv->is_str() && !drv->s.empty()) vol[drv->s].insert(id);
      }
    }
  std::string o = "[";
  bool firstNode = true;
  for (const std::string& id : order) {
    const Entry& e = byID[id];
    QList podReq, dsReq;  // PodRequests() / DaemonSetRequests(): MergeInto over the pods
    for (auto& kv : e.podRequests)
      for (auto& r : kv.second) podReq[r.first].add(r.second);
    for (auto& kv : e.dsRequests)
      for (auto& r : kv.second) dsReq[r.first].add(r.second);
    QList avail = e.resources("allocatable");  // Available() = Subtract(Allocatable(), PodRequests())
    for (auto& kv : avail) {
      auto it = podReq.find(kv.first);
      if (it == podReq.end()) continue;
      if (kv.second.n == 0) kv.second.f = it->second.f;
      kv.second.n -= it->second.n;
    }
    bool ready = false;  // GetCondition(Node, Ready).Status == True (helpers.go:119)
    if (const Value* cs = path(e.node, {"status", "conditions"}))
      for (auto& c : cs->arr())
        if (sget(&c, "type") == "Ready") {
          ready = sget(&c, "status") == "True";
          break;
        }
    if (!firstNode) o += ",";
    firstNode = false;
    o += "{\"name\":";
    ksjson::quote(o, e.name());
    o += ",\"providerID\":";
    ksjson::quote(o, id);
    o += ",\"hostName\":";
    ksjson::quote(o, e.hostName());
    o += ",\"labels\":{";
    bool first = true;
    for (auto& kv : e.labels()) {
      if (!first) o += ",";
      first = false;
      ksjson::quote(o, kv.first);
      o += ":";
      ksjson::quote(o, kv.second);
    }
    o += "},\"annotations\":{";  // StateNode.Annotations() (statenode.go:148-161): the same object as Labels()
    first = true;
    for (auto& kv : smap(path(e.face(), {"metadata", "annotations"}))) {
      if (!first) o += ",";
      first = false;
      ksjson::quote(o, kv.first);
      o += ":";
      ksjson::quote(o, kv.second);
    }
    o += "},\"taints\":[";
    first = true;
    for (auto& t : e.taintList()) {
      if (!first) o += ",";
      first = false;
      o += "{\"key\":";
      ksjson::quote(o, t.key);
      o += ",\"value\":";
      ksjson::quote(o, t.value);
      o += ",\"effect\":";
      ksjson::quote(o, t.effect);
      o += "}";
    }
    o += "],\"capacity\":";
    put_qlist(o, e.resources("capacity"));
    o += ",\"allocatable\":";
    put_qlist(o, e.resources("allocatable"));
    o += ",\"available\":";
    put_qlist(o, avail);
    o += ",\"podRequests\":";
    put_qlist(o, podReq);
    o += ",\"daemonSetRequests\":";
    put_qlist(o, dsReq);
    o += std::string(",\"initialized\":") + (e.initialized() ? "true" : "false");
    o += std::string(",\"ready\":") + (ready ? "true" : "false");
    const bool marked = (e.claim && deleting(e.claim)) || (e.node && !e.claim && deleting(e.node));
    o += std::string(",\"markedForDeletion\":") + (marked ? "true" : "false");
    o += ",\"creationTimestamp\":";
    ksjson::quote(o, sget(path(e.node, {"metadata"}), "creationTimestamp"));
    o += ",\"hostPortUsage\":{";
    first = true;
    for (auto& kv : e.ports) {
      if (kv.second.empty()) continue;
      if (!first) o += ",";
      first = false;
      ksjson::quote(o, kv.first);
      o += ":[";
      for (size_t i = 0; i < kv.second.size(); i++) {
        if (i) o += ",";
        o += "{\"ip\":";
        ksjson::quote(o, kv.second[i].ip);
        o += ",\"port\":" + std::to_string(kv.second[i].port) + ",\"protocol\":";
        ksjson::quote(o, kv.second[i].proto);
        o += "}";
      }
      o += "]";
    }
    // VolumeUsage (union of the pods' volumes) and populateVolumeLimits (cluster.go:457-471: CSINode
    // drivers with an allocatable count)
    std::map<std::string, std::set<std::string>> vu;
    for (auto& kv : e.volumes)
      for (auto& dv : kv.second) vu[dv.first].insert(dv.second.begin(), dv.second.end());
    o += "},\"volumeUsage\":{";
    first = true;
    for (auto& kv : vu) {
      if (!first) o += ",";
      first = false;
      ksjson::quote(o, kv.first);
      o += ":[";
      bool f2 = true;
      for (auto& id : kv.second) {
        if (!f2) o += ",";
        f2 = false;
        ksjson::quote(o, id);
      }
      o += "]";
    }
    o += "},\"volumeLimits\":{";
    first = true;
    if (e.node)
      if (const Value* csis = root.get("csiNodes"))
        for (auto& cn : csis->arr()) {
          if (sget(path(&cn, {"metadata"}), "name") != sget(path(e.node, {"metadata"}), "name")) continue;
          if (const Value* ds = path(&cn, {"spec", "drivers"}))
            for (auto& dv : ds->arr()) {
              const Value* alloc = dv.get("allocatable");
              if (!alloc || alloc->is_null()) continue;
              const Value* cnt = alloc->get("count");
              if (!first) o += ",";
              first = false;
              ksjson::quote(o, sget(&dv, "name"));
              o += ":" + std::to_string(cnt ? cnt->i64() : 0);
            }
          break;
        }
    o += "},\"pods\":[";
    for (size_t i = 0; i < e.pods.size(); i++) {
      if (i) o += ",";
      dump(o, *e.pods[i]);
    }
    o += "]}";
  }
  return o + "]";
}

}  // namespace ks

extern "C" int ks_cluster_state(const char* json, size_t len, char** out_json) {
  API_TRY
  if (!json || !out_json) throw ks::KsError(KS_ERR_ARG, "null argument");
  ksjson::Value root = ksjson::Parser(json, len ? len : strlen(json)).parse();
  if (!root.is_obj()) throw ks::KsError(KS_ERR_PARSE, "cluster is not an object");
  *out_json = strdup(ks::cluster_state_json(root).c_str());
  return KS_OK;
  API_CATCH
}
