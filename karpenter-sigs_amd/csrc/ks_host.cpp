// ks_host.cpp — snapshot parsing, universe interning and encoding (the NewScheduler half of the
// boundary), plus the text renderers used to rebuild Results (Requirements.String, PodErrors).
//
// Reference behaviour encoded here (paths under /root/reference):
//   NewNodeClaimTemplate            pkg/controllers/provisioning/scheduling/nodeclaimtemplate.go:43-53
//   NewScheduler / getDaemonOverhead / calculateExistingNodeClaims     scheduler.go:49-83,287-341
//   NewExistingNode                 existingnode.go:40-62
//   NewPodRequirements / NewStrictPodRequirements / HasPreferredNodeAffinity  requirements.go:56-109
//   Preferences.Relax               preferences.go:38-147 (precomputed as a chain of pod states)
//   RequestsForPods / Ceiling       pkg/utils/resources/resources.go:27-35,99-115
//   InstanceType.Allocatable        pkg/cloudprovider/types.go:100-110
//   Taints.Tolerates / ToleratesTaint pkg/scheduling/taints.go:38-50 (k8s.io/api v0.28.4)
#include "ks_host.h"
#include "ks_volume.h"

#include <arpa/inet.h>
#include <cstring>

#include <algorithm>
#include <cstring>

#include "ks_gosort.h"

namespace ks {

static const char* kHostname = "kubernetes.io/hostname";
static const char* kZone = "topology.kubernetes.io/zone";
static const char* kCT = "karpenter.sh/capacity-type";
static const char* kNodePoolKey = "karpenter.sh/nodepool";

std::string normalize_key(const std::string& k) {  // v1beta1.NormalizedLabels (labels.go:94-100)
  if (k == "failure-domain.beta.kubernetes.io/zone") return kZone;
  if (k == "beta.kubernetes.io/arch") return "kubernetes.io/arch";
  if (k == "beta.kubernetes.io/os") return "kubernetes.io/os";
  if (k == "beta.kubernetes.io/instance-type") return "node.kubernetes.io/instance-type";
  if (k == "failure-domain.beta.kubernetes.io/region") return "topology.kubernetes.io/region";
  return k;
}

std::string go_quote(const std::string& s) {
  std::string o = "\"";
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
    else if (c == '\n') o += "\\n";
    else if (c == '\t') o += "\\t";
    else if (c < 0x20 || c == 0x7f) { char b[8]; snprintf(b, sizeof b, "\\x%02x", c); o += b; }
    else o += (char)c;
  }
  return o + "\"";
}

std::string qlist_json(const QList& l) {
  if (l.empty()) return "{}";
  std::string s = "{";
  bool first = true;
  for (auto& kv : l) {
    if (!first) s += ",";
    first = false;
    ksjson::quote(s, kv.first);
    s += ":";
    ksjson::quote(s, qty_str(kv.second));
  }
  return s + "}";
}

static bool go_atoi(const std::string& s, int64_t& out) {  // strconv.Atoi
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
  if (i == s.size()) return false;
  unsigned __int128 v = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (unsigned)(s[i] - '0');
    if (v > ((unsigned __int128)1 << 63)) return false;
  }
  if (!neg && v == ((unsigned __int128)1 << 63)) return false;
  out = neg ? (int64_t)(0 - (uint64_t)v) : (int64_t)v;
  return true;
}

// ---------------------------------------------------------------------------------------------
// JSON helpers
// ---------------------------------------------------------------------------------------------
using ksjson::Value;
static std::string jstr(const Value* v, const char* k, const std::string& d = "") {
  if (!v) return d;
  const Value* x = v->get(k);
  return x && x->is_str() ? x->s : d;
}
static std::map<std::string, std::string> jmap(const Value* v) {
  std::map<std::string, std::string> m;
  if (v) for (auto& kv : v->obj()) m[kv.first] = kv.second.str();
  return m;
}
static QList jqlist(const Value* v) {
  QList q;
  if (v)
    for (auto& kv : v->obj()) {
      try {
        q[kv.first] = qty_parse(kv.second.is_str() ? kv.second.s : kv.second.s);
      } catch (const std::exception& e) {
        throw KsError(-1, std::string("quantity ") + kv.first + ": " + e.what());
      }
    }
  return q;
}
static std::vector<NSR> jnsr(const Value* v) {
  std::vector<NSR> out;
  if (!v) return out;
  for (auto& e : v->arr()) {
    NSR n;
    n.key = jstr(&e, "key");
    n.op = jstr(&e, "operator");
    if (auto* vs = e.get("values")) for (auto& x : vs->arr()) n.values.push_back(x.str());
    out.push_back(n);
  }
  return out;
}
static std::vector<TaintH> jtaints(const Value* v) {
  std::vector<TaintH> out;
  if (!v) return out;
  for (auto& e : v->arr()) out.push_back(TaintH{jstr(&e, "key"), jstr(&e, "value"), jstr(&e, "effect")});
  return out;
}
static int64_t jtime(const std::string& s) {
  if (s.size() < 19) return 0;
  int Y = atoi(s.substr(0, 4).c_str()), M = atoi(s.substr(5, 2).c_str()), D = atoi(s.substr(8, 2).c_str());
  int h = atoi(s.substr(11, 2).c_str()), mi = atoi(s.substr(14, 2).c_str()), se = atoi(s.substr(17, 2).c_str());
  int y = Y - (M <= 2);
  int era = (y >= 0 ? y : y - 399) / 400;
  int yoe = y - era * 400;
  int doy = (153 * (M + (M > 2 ? -3 : 9)) + 2) / 5 + D - 1;
  int doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return ((int64_t)era * 146097 + doe - 719468) * 86400 + h * 3600 + mi * 60 + se;
}

static void mergeInto(QList& dst, const QList& src) {
  for (auto& kv : src) dst[kv.first].add(kv.second);
}

// Ceiling(pod).Requests + pods (resources.go:27-35,99-115,124-147)
bool HostPortH::unspecified() const {
  if (!ipValid) return false;
  for (int i = 0; i < 16; i++) {
    // IPv4 unspecified is ::ffff:0.0.0.0 in the 16-byte form
    if (i == 10 || i == 11) continue;
    if (ip16[i]) return false;
  }
  return (ip16[10] == 0 && ip16[11] == 0) || (ip16[10] == 0xff && ip16[11] == 0xff);
}

bool HostPortH::matches(const HostPortH& o) const {
  if (proto != o.proto || port != o.port) return false;
  const bool equal = ipValid && o.ipValid ? ip16 == o.ip16 : (!ipValid && !o.ipValid);  // net.IP.Equal
  return equal || unspecified() || o.unspecified();
}

HostPortH make_host_port(const std::string& ip, int32_t port, const std::string& proto) {
  HostPortH h;
  h.ip = ip;
  h.port = port;
  h.proto = proto;
  in6_addr a6;
  in_addr a4;
  if (inet_pton(AF_INET, ip.c_str(), &a4) == 1) {  // net.ParseIP: IPv4 -> v4-in-v6 form
    h.ip16[10] = h.ip16[11] = 0xff;
    memcpy(&h.ip16[12], &a4, 4);
    h.ipValid = true;
  } else if (inet_pton(AF_INET6, ip.c_str(), &a6) == 1) {
    memcpy(h.ip16.data(), &a6, 16);
    h.ipValid = true;
  }
  return h;
}

static QList podRequests(const Value& pod, bool& hostPorts, bool& volumes) {
  QList req;
  const Value* sp = pod.get("spec");
  auto limitsIntoRequests = [](const Value& c) {
    QList r, l;
    if (auto* res = c.get("resources")) {
      r = jqlist(res->get("requests"));
      l = jqlist(res->get("limits"));
    }
    for (auto& kv : l) if (!r.count(kv.first)) r[kv.first] = kv.second;
    return r;
  };
  if (sp) {
    if (auto* cs = sp->get("containers"))
      for (auto& c : cs->arr()) {
        mergeInto(req, limitsIntoRequests(c));
        if (auto* ps = c.get("ports"))
          for (auto& p : ps->arr())
            if (p.get("hostPort") && p.get("hostPort")->i64() != 0) hostPorts = true;
      }
    if (auto* cs = sp->get("initContainers"))
      for (auto& c : cs->arr()) {
        QList m = limitsIntoRequests(c);
        QList out = req;  // MaxResources(req, m): keep the earlier quantity unless strictly greater
        for (auto& kv : m) {
          auto it = out.find(kv.first);
          if (it == out.end() || kv.second.n > it->second.n) out[kv.first] = kv.second;
        }
        req = out;
      }
    if (auto* oh = sp->get("overhead"); oh && !oh->is_null()) mergeInto(req, jqlist(oh));
    if (auto* vs = sp->get("volumes"))
      for (auto& v : vs->arr())
        if (v.get("persistentVolumeClaim") || v.get("ephemeral")) volumes = true;
  }
  Qty one;
  one.n = 1000000000;
  one.f = QFmt::DecExp;
  req["pods"] = one;  // NewQuantity(1, DecimalExponent)
  return req;
}

static LabelSel jsel(const Value* v) {  // metav1.LabelSelector
  LabelSel s;
  if (!v || v->is_null()) return s;
  s.present = true;
  for (auto& kv : jmap(v->get("matchLabels"))) s.reqs.push_back({kv.first, "In", {kv.second}});
  if (auto* es = v->get("matchExpressions"))
    for (auto& e : es->arr()) {
      SelReq r{jstr(&e, "key"), jstr(&e, "operator"), {}};
      if (auto* vs = e.get("values")) for (auto& x : vs->arr()) r.values.push_back(x.str());
      s.reqs.push_back(r);
    }
  return s;
}

static AffTerm jaffterm(const Value* t) {  // v1.PodAffinityTerm
  AffTerm a;
  if (!t) return a;
  a.sel = jsel(t->get("labelSelector"));
  if (auto* ns = t->get("namespaces")) for (auto& x : ns->arr()) a.namespaces.push_back(x.str());
  if (auto* nss = t->get("namespaceSelector"); nss && !nss->is_null()) {
    a.nsSelector = true;
    a.nsSel = jsel(nss);
  }
  a.key = jstr(t, "topologyKey");
  return a;
}

PodH parse_pod(const Value& v) {
  PodH p;
  const Value* md = v.get("metadata");
  p.name = jstr(md, "name");
  p.ns = jstr(md, "namespace");
  p.uid = jstr(md, "uid");
  p.created = jtime(jstr(md, "creationTimestamp"));
  std::string nodeName, nominated;
  bool failedToSchedule = false;
  if (md) {
    p.labels = jmap(md->get("labels"));
    p.annotations = jmap(md->get("annotations"));
    if (auto* x = md->get("deletionTimestamp")) p.deleting = !x->is_null();
    if (auto* ors = md->get("ownerReferences"))
      for (auto& o : ors->arr()) {
        const std::string av = jstr(&o, "apiVersion"), kind = jstr(&o, "kind");
        if (av == "apps/v1" && kind == "DaemonSet") p.ownedByDaemonSet = true;
        if (av == "v1" && kind == "Node") p.ownedByNode = true;
      }
  }
  if (auto* st = v.get("status")) {
    const std::string ph = jstr(st, "phase");
    p.terminal = ph == "Failed" || ph == "Succeeded";
    nominated = jstr(st, "nominatedNodeName");
    p.phase = ph;
    if (auto* cs = st->get("conditions"))
      for (auto& c : cs->arr())
      {
        if (jstr(&c, "type") == "PodScheduled" && jstr(&c, "reason") == "Unschedulable") failedToSchedule = true;
        if (jstr(&c, "type") == "Ready" && jstr(&c, "status") == "False") p.notReady = true;
      }
  }
  const Value* sp = v.get("spec");
  if (sp) {
    nodeName = jstr(sp, "nodeName");
    p.nodeName = nodeName;
    if (auto* x = sp->get("priority"); x && !x->is_null()) {
      p.hasPriority = true;
      p.priority = (int32_t)x->i64();
    }
    p.nodeSelector = jmap(sp->get("nodeSelector"));
    if (auto* af = sp->get("affinity"); af && !af->is_null()) {
      p.hasAffinity = true;
      if (auto* na = af->get("nodeAffinity"); na && !na->is_null()) {
        p.hasNodeAffinity = true;
        if (auto* rq = na->get("requiredDuringSchedulingIgnoredDuringExecution"); rq && !rq->is_null()) {
          p.hasRequired = true;
          if (auto* ts = rq->get("nodeSelectorTerms"))
            for (auto& t : ts->arr()) p.requiredTerms.push_back(jnsr(t.get("matchExpressions")));
        }
        if (auto* pr = na->get("preferredDuringSchedulingIgnoredDuringExecution"))
          for (auto& t : pr->arr())
            p.preferred.push_back(PrefTerm{(int32_t)(t.get("weight") ? t.get("weight")->i64() : 0),
                                           t.get("preference") ? jnsr(t.get("preference")->get("matchExpressions"))
                                                               : std::vector<NSR>{}});
      }
      for (int anti = 0; anti < 2; anti++) {
        auto* pa = af->get(anti ? "podAntiAffinity" : "podAffinity");
        if (!pa || pa->is_null()) continue;
        (anti ? p.hasPodAnti : p.hasPodAffinity) = true;
        if (auto* r = pa->get("requiredDuringSchedulingIgnoredDuringExecution"))
          for (auto& t : r->arr()) (anti ? p.antiRequired : p.affRequired).push_back(jaffterm(&t));
        if (auto* r = pa->get("preferredDuringSchedulingIgnoredDuringExecution"))
          for (auto& t : r->arr())
            (anti ? p.antiPreferred : p.affPreferred)
                .push_back({(int32_t)(t.get("weight") ? t.get("weight")->i64() : 0), jaffterm(t.get("podAffinityTerm"))});
      }
    }
    if (auto* ts = sp->get("tolerations"))
      for (auto& t : ts->arr()) p.tols.push_back(TolH{jstr(&t, "key"), jstr(&t, "operator"), jstr(&t, "value"), jstr(&t, "effect")});
    if (auto* ts = sp->get("topologySpreadConstraints"))
      for (auto& t : ts->arr()) {
        SpreadC c;
        c.key = jstr(&t, "topologyKey");
        c.when = jstr(&t, "whenUnsatisfiable");
        c.maxSkew = t.get("maxSkew") ? (int32_t)t.get("maxSkew")->i64() : 0;
        if (auto* md = t.get("minDomains"); md && !md->is_null()) c.minDomains = (int32_t)md->i64();
        c.sel = jsel(t.get("labelSelector"));
        p.tsc.push_back(c);
      }
  }
  p.requests = podRequests(v, p.hostPorts, p.volumes);
  if (sp)
    if (auto* vs = sp->get("volumes"))  // volume.GetPersistentVolumeClaim (utils/volume/volume.go:29-38)
      for (auto& vol : vs->arr()) {
        if (auto* pvc = vol.get("persistentVolumeClaim"); pvc && !pvc->is_null())
          p.pvcNames.push_back(jstr(pvc, "claimName"));
        else if (auto* eph = vol.get("ephemeral"); eph && !eph->is_null())
          p.pvcNames.push_back(p.name + "-" + jstr(&vol, "name"));
      }
  if (sp)
    if (auto* cs = sp->get("containers"))
      for (auto& c : cs->arr())
        if (auto* ps = c.get("ports"))
          for (auto& x : ps->arr()) {
            const int64_t hp = x.get("hostPort") ? x.get("hostPort")->i64() : 0;
            if (hp == 0) continue;
            std::string ip = jstr(&x, "hostIP");
            if (ip.empty()) ip = "0.0.0.0";  // GetHostPorts defaults the IP, keeps the protocol as given
            p.ports.push_back(make_host_port(ip, (int32_t)hp, jstr(&x, "protocol")));
          }
  p.provisionable = nodeName.empty() && nominated.empty() && failedToSchedule && !p.ownedByDaemonSet && !p.ownedByNode;
  return p;
}

static bool toleratesTaint(const TolH& t, const TaintH& x) {  // v1.Toleration.ToleratesTaint
  if (!t.effect.empty() && t.effect != x.effect) return false;
  if (!t.key.empty() && t.key != x.key) return false;
  if (t.op.empty() || t.op == "Equal") return t.value == x.value;
  return t.op == "Exists";
}
static bool tolerates(const std::vector<TaintH>& taints, const std::vector<TolH>& tols) {
  for (auto& x : taints) {
    bool ok = false;
    for (auto& t : tols) ok = ok || toleratesTaint(t, x);
    if (!ok) return false;
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
// Universe
// ---------------------------------------------------------------------------------------------
void Host::internKey(const std::string& key) {
  if (!keyId.count(key)) { keyId[key] = -1; }
}
void Host::intern(const std::string& key, const std::string& val) {
  internKey(key);
  valueSet_[key].insert(val);
}

void Host::addNSR(std::vector<uint32_t>& rec, const std::string& key0, const std::string& op,
                  const std::vector<std::string>& vals) const {
  std::string key = normalize_key(key0);
  int k = keyId.at(key);
  std::vector<uint32_t> one = emptyRec();
  const KeyMeta& km = keys[k];
  uint64_t bitk = 1ull << k;
  wr64(one.data(), 0, bitk);
  auto setv = [&](const std::string& v) {
    int b = valueId[k].at(v);
    one[L.HDR + km.off + (b >> 5)] |= 1u << (b & 31);
  };
  if (op == "In") {
    for (auto& v : vals) setv(v);
  } else if (op == "NotIn") {
    wr64(one.data(), 2, bitk);
    for (auto& v : vals) setv(v);
  } else if (op == "Exists") {
    wr64(one.data(), 2, bitk);
  } else if (op == "DoesNotExist") {
  } else if (op == "Gt" || op == "Lt") {
    int64_t x = 0;
    go_atoi(vals.empty() ? "" : vals[0], x);  // prevalidated in Go; errors -> 0
    wr64(one.data(), 2, bitk);
    if (op == "Gt") { wr64(one.data(), 4, bitk); rs_set_gt(one.data(), km.bslot, x); }
    else { wr64(one.data(), 6, bitk); rs_set_lt(one.data(), km.bslot, x); }
  } else {
    throw KsError(-2, "unsupported node selector operator: " + op);
  }
  rs_add(L, rec.data(), one.data());
}

void Host::addLabels(std::vector<uint32_t>& rec, const std::map<std::string, std::string>& labels) const {
  for (auto& kv : labels) addNSR(rec, kv.first, "In", {kv.second});
}
void Host::addNodeLabels(std::vector<uint32_t>& rec, const std::map<std::string, std::string>& labels) const {
  for (auto& kv : labels)
    if (keyId.count(normalize_key(kv.first))) addNSR(rec, kv.first, "In", {kv.second});
}

// newPodRequirements (requirements.go:64-100).  Sorting the preferred terms mutates the pod, as
// the reference's sort.Slice does.
std::vector<uint32_t> Host::podRequirements(PodH& p, bool all) const {
  std::vector<uint32_t> r = emptyRec();
  addLabels(r, p.nodeSelector);
  if (!p.hasAffinity || !p.hasNodeAffinity) return r;
  if (all && !p.preferred.empty()) {
    int n = (int)p.preferred.size();
    std::vector<int32_t> key(n), idx(n);
    for (int i = 0; i < n; i++) { key[i] = -p.preferred[i].weight; idx[i] = i; }
    GoSortExact s{GoSort{key.data(), idx.data()}};
    s.run(n);
    std::vector<PrefTerm> sorted(n);
    for (int i = 0; i < n; i++) sorted[i] = p.preferred[idx[i]];
    p.preferred = sorted;
    for (auto& e : p.preferred[0].exprs) addNSR(r, e.key, e.op, e.values);
  }
  if (p.hasRequired && !p.requiredTerms.empty())
    for (auto& e : p.requiredTerms[0]) addNSR(r, e.key, e.op, e.values);
  return r;
}

void Host::tolMask(const std::vector<TolH>& tols, const std::vector<int>& cls, uint64_t out[2]) const {
  out[0] = out[1] = 0;
  for (size_t i = 0; i < taints.size(); i++) {
    bool ok = false;
    for (auto& t : tols) ok = ok || toleratesTaint(t, taints[i]);
    if (ok) out[cls[i] >> 6] |= 1ull << (cls[i] & 63);  // (every taint of a class is tolerated alike)
  }
}

int64_t Host::toDev(int r, const Qty& q) const {
  __int128 d = 1;
  for (int i = 0; i < resShift[r]; i++) d *= 10;
  return (int64_t)(q.n / d);
}
Qty Host::fromDev(int r, int64_t v) const {
  __int128 d = 1;
  for (int i = 0; i < resShift[r]; i++) d *= 10;
  Qty q;
  q.n = (__int128)v * d;
  return q;
}

std::string Host::placeholder(int64_t id) const {
  char b[64];
  snprintf(b, sizeof b, "hostname-placeholder-%04lld", (long long)id);
  return b;
}

// ---------------------------------------------------------------------------------------------
// build: the NewScheduler half of the boundary
// ---------------------------------------------------------------------------------------------
void Host::build(const Value& root) {
  PhaseTimer pt("Host::build");
  if (auto* t = root.get("topology"); t && !t->is_null())
    throw KsError(-2, "explicit topology groups are not accepted: pass the pods' topology spread / pod "
                      "(anti-)affinity terms and the cluster's bound pods (clusterPods, clusterNodes)");
  auto parsePods = [](const Value* v, std::vector<PodH>& out) {  // independent per pod: worker threads
    if (!v) return;
    const ksjson::Array& a = v->arr();
    out.resize(a.size());
    parallel_for((int)a.size(), 256, [&](int i) { out[(size_t)i] = parse_pod(a[(size_t)i]); });
  };
  parsePods(root.get("clusterPods"), clusterPods);
  if (auto* nss = root.get("namespaces"))  // the cluster's Namespace list, for namespaceSelector terms
    for (auto& v : nss->arr()) {
      const Value* md = v.get("metadata") ? v.get("metadata") : &v;
      std::map<std::string, std::string> labels;
      if (const Value* l = md->get("labels"))
        for (auto& kv : l->obj()) labels[kv.first] = kv.second.str();
      namespaceList.push_back({jstr(md, "name"), labels});
    }
  if (auto* cns = root.get("clusterNodes"))
    for (auto& v : cns->arr()) nodeLabelsByName[jstr(&v, "name")] = jmap(v.get("labels"));
  if (auto* wk = root.get("wellKnownLabels")) for (auto& x : wk->arr()) wellKnown.insert(x.str());
  else
    wellKnown = {kNodePoolKey, kZone, "topology.kubernetes.io/region", "node.kubernetes.io/instance-type",
                 "kubernetes.io/arch", "kubernetes.io/os", kCT, "node.kubernetes.io/windows-build"};
  if (auto* hs = root.get("hostnameSeed")) hostnameSeed = hs->i64();
  if (auto* et = root.get("emptyTopology")) emptyTopology = et->boolean();

  pt.mark("head");
  // --- instance types
  if (auto* v = root.get("instanceTypes"))
    for (auto& e : v->arr()) {
      IT it;
      it.name = jstr(&e, "name");
      it.reqs = jnsr(e.get("requirements"));
      it.capacity = jqlist(e.get("capacity"));
      QList total;
      if (auto* oh = e.get("overhead")) {
        mergeInto(total, jqlist(oh->get("kubeReserved")));
        mergeInto(total, jqlist(oh->get("systemReserved")));
        mergeInto(total, jqlist(oh->get("evictionThreshold")));
      }
      it.alloc = it.capacity;  // Subtract keeps the lhs keys only
      for (auto& kv : it.alloc) {
        auto o = total.find(kv.first);
        if (o != total.end()) {
          if (kv.second.n == 0) kv.second.f = o->second.f;
          kv.second.n -= o->second.n;
        }
      }
      if (auto* os = e.get("offerings"))
        for (auto& o : os->arr()) {
          bool avail = o.get("available") ? o.get("available")->boolean(true) : true;
          const double price = o.get("price") ? o.get("price")->f64() : 0.0;
          it.all.push_back(Offer{jstr(&o, "zone"), jstr(&o, "capacityType"), price, avail});
          if (avail) {
            it.offers.push_back({jstr(&o, "zone"), jstr(&o, "capacityType")});
            it.prices.push_back(price);
          }
        }
      its.push_back(std::move(it));
    }
  const Value* byPool = root.get("instanceTypesByNodePool");
  // --- templates
  if (auto* v = root.get("nodeClaimTemplates"))
    for (auto& np : v->arr()) {
      Tpl t;
      t.pool = jstr(np.get("metadata"), "name");
      const Value* tpl = np.get("spec") ? np.get("spec")->get("template") : nullptr;
      if (tpl) {
        if (auto* tm = tpl->get("metadata")) t.labels = jmap(tm->get("labels"));
        if (auto* ts = tpl->get("spec")) {
          t.reqs = jnsr(ts->get("requirements"));
          t.taints = jtaints(ts->get("taints"));
        }
      }
      t.poolLabels = t.labels;
      t.labels[kNodePoolKey] = t.pool;
      if (byPool && byPool->get(t.pool))
        for (auto& x : byPool->get(t.pool)->arr()) {
          int64_t i = x.i64();
          if (i < 0 || i >= (int64_t)its.size()) throw KsError(-1, "instanceTypesByNodePool index out of range");
          t.its.push_back((int)i);
        }
      tpls.push_back(std::move(t));
    }
  if ((int)tpls.size() > kMaxTpl) throw KsError(-3, "too many NodeClaimTemplates");
  // --- node pools (limits, PreferNoSchedule taints)
  if (auto* v = root.get("nodePools"))
    for (auto& np : v->arr()) {
      Pool p;
      p.name = jstr(np.get("metadata"), "name");
      const Value* spec = np.get("spec");
      if (spec && spec->get("limits") && !spec->get("limits")->is_null()) p.remaining = jqlist(spec->get("limits"));
      if (spec && spec->get("template") && spec->get("template")->get("spec"))
        for (auto& t : jtaints(spec->get("template")->get("spec")->get("taints")))
          if (t.effect == "PreferNoSchedule") toleratePreferNoSchedule = true;
      pools.push_back(p);
    }
  // --- existing nodes
  if (auto* v = root.get("stateNodes"))
    for (auto& e : v->arr()) {
      Node n;
      n.name = jstr(&e, "name");
      n.hostName = jstr(&e, "hostName", n.name);
      n.labels = jmap(e.get("labels"));
      n.taints = jtaints(e.get("taints"));
      n.available = jqlist(e.get("available"));
      n.capacity = jqlist(e.get("capacity"));
      n.dsRequests = jqlist(e.get("daemonSetRequests"));
      n.initialized = e.get("initialized") ? e.get("initialized")->boolean(true) : true;
      n.ready = e.get("ready") ? e.get("ready")->boolean(true) : true;
      if (auto* hu = e.get("hostPortUsage"))  // StateNode.HostPortUsage(): pod key -> ports
        for (auto& kv : hu->obj())
          for (auto& x : kv.second.arr())
            n.hostPorts.push_back({kv.first, make_host_port(x.get("ip") ? x.get("ip")->str() : "0.0.0.0",
                                                            (int32_t)(x.get("port") ? x.get("port")->i64() : 0),
                                                            x.get("protocol") ? x.get("protocol")->str() : "TCP")});
      if (auto* vu = e.get("volumeUsage"))  // StateNode.VolumeUsage(): driver -> PVC keys
        for (auto& kv : vu->obj())
          for (auto& x : kv.second.arr()) n.volumes[kv.first].insert(x.str());
      if (auto* vl = e.get("volumeLimits"))  // CSINode drivers' allocatable counts (cluster.go:468)
        for (auto& kv : vl->obj()) n.volumeLimits[kv.first] = kv.second.i64();
      n.origIndex = (int)nodes.size();
      nodes.push_back(std::move(n));
    }
  std::stable_sort(nodes.begin(), nodes.end(), [](const Node& a, const Node& b) {  // scheduler.go:313-321
    if (a.initialized != b.initialized) return a.initialized;
    return a.name < b.name;
  });
  pt.mark("its+templates+nodes");
  if (auto* v = root.get("daemonSetPods")) for (auto& e : v->arr()) daemons.push_back(parse_pod(e));
  if (preParsedPods) pods = std::move(*preParsedPods);
  else parsePods(root.get("pods"), pods);
  if (auto* v = root.get("volumeDrivers"))
    for (auto& kv : v->obj()) volumeDrivers[kv.first] = kv.second.str();
  // Provisioner.NewScheduler's injectTopology (provisioner.go:283-284,432-442) and, without an explicit
  // "volumeDrivers" map, GetVolumes' driver resolution, both from the snapshot's PVC / PV / StorageClass
  // objects (ks_volume.cpp)
  std::set<std::string> volErrKeys;
  {
    VolumeObjects vobj;
    vobj.parse(root);
    injectFailed.assign(pods.size(), 0);
    if (vobj.present) {
      parallel_for((int)pods.size(), 256, [&](int i) { injectFailed[(size_t)i] = vobj.inject(pods[(size_t)i], nullptr) ? 0 : 1; });
      if (!root.get("volumeDrivers"))
        for (auto& p : pods)
          for (auto& name : p.pvcNames) {
            const std::string key = p.ns + "/" + name;
            if (volumeDrivers.count(key) || volErrKeys.count(key)) continue;
            std::string drv;
            if (!vobj.driver(key, drv)) volErrKeys.insert(key);
            else if (vobj.pvcs.count(key)) volumeDrivers[key] = drv;
          }
    }
  }

  pt.mark("parse pods");
  // --- universe of keys and values
  internKey(kHostname);
  internKey(kZone);
  internKey(kCT);
  intern(kCT, "spot");  // worstLaunchPrice asks Has(spot) / Has(on-demand) of every requirement set
  intern(kCT, "on-demand");
  std::set<std::string> bounded;
  auto visitNSR = [&](const std::vector<NSR>& v) {
    for (auto& n : v) {
      std::string k = normalize_key(n.key);
      internKey(k);
      if (n.op == "In" || n.op == "NotIn") for (auto& x : n.values) intern(k, x);
      if (n.op == "Gt" || n.op == "Lt") bounded.insert(k);
    }
  };
  auto visitLabels = [&](const std::map<std::string, std::string>& m) {
    for (auto& kv : m) intern(normalize_key(kv.first), kv.second);
  };
  auto visitPod = [&](const PodH& p) {
    visitLabels(p.nodeSelector);
    for (auto& t : p.requiredTerms) visitNSR(t);
    for (auto& t : p.preferred) visitNSR(t.exprs);
  };
  for (auto& it : its) {
    visitNSR(it.reqs);
    for (auto& o : it.offers) { intern(kZone, o.first); intern(kCT, o.second); }
  }
  for (auto& t : tpls) { visitNSR(t.reqs); visitLabels(t.labels); }
  for (auto& n : nodes) intern(kHostname, n.hostName);  // (node labels below: only the keys something mentions)
  for (auto& p : pods) visitPod(p);
  for (auto& p : daemons) visitPod(p);
  // topology keys and the domains the cluster's nodes contribute (countDomains, updateInverseAffinities)
  {
    std::set<std::string> tkeys;
    auto visitTopo = [&](const PodH& p) {
      for (auto& c : p.tsc) tkeys.insert(c.key);
      for (auto& t : p.antiRequired) tkeys.insert(t.key);
      for (auto& t : p.antiPreferred) tkeys.insert(t.second.key);
      for (auto& t : p.affRequired) tkeys.insert(t.key);
      for (auto& t : p.affPreferred) tkeys.insert(t.second.key);
    };
    for (auto& p : pods) visitTopo(p);
    for (auto& p : clusterPods) visitTopo(p);
    for (auto& n : nodes) nodeLabelsByName[n.name] = n.labels;
    for (auto& k : tkeys) {
      internKey(k);  // topology keys are matched verbatim (not normalised) by the reference
      for (auto& kv : nodeLabelsByName) {
        auto l = kv.second.find(k);
        if (l != kv.second.end()) intern(k, l->second);
        else if (k == kHostname) intern(k, kv.first);
      }
    }
  }
  // An existing node's labels enter its requirement record only for keys some requirement, template label or
  // topology key mentions: ExistingNode.Add's strict Compatible(node, pod) (existingnode.go:97-104,
  // requirements.go:163-174) reads the node's value of a key only when the pod names it, the daemon overhead
  // test likewise, and a node's record is never rendered.  So the label keys only nodes carry (a production
  // node has dozens) do not count against the 64-key universe and cost no record words.
  for (auto& n : nodes)
    for (auto& kv : n.labels) {
      const std::string k = normalize_key(kv.first);
      if (keyId.count(k)) intern(k, kv.second);
    }
  for (auto& kv : valueSet_[kHostname])
    if (kv.rfind("hostname-placeholder-", 0) == 0)
      throw KsError(-2, "input names a hostname-placeholder value (reserved for new NodeClaims)");

  if (keyId.size() > 64) throw KsError(-3, "more than 64 distinct label keys");
  int k = 0, off = 0, nb = 0, vint = 0;
  for (auto& kv : keyId) {  // std::map: keys sorted by name -> id order == Go's sorted error order
    kv.second = k++;
    keyNames.push_back(kv.first);
    auto& vs = valueSet_[kv.first];
    values.emplace_back(vs.begin(), vs.end());
    std::map<std::string, int> ids;
    for (size_t i = 0; i < values.back().size(); i++) ids[values.back()[i]] = (int)i;
    valueId.push_back(ids);
    KeyMeta m{};
    m.nv = (int)values.back().size() + (kv.first == kHostname ? 1 : 0);
    m.nw = std::max(1, (m.nv + 31) / 32);
    m.off = off;
    off += m.nw;
    m.bslot = bounded.count(kv.first) ? nb++ : -1;
    m.vint = m.bslot >= 0 ? vint : -1;
    if (m.bslot >= 0) vint += m.nv;
    keys.push_back(m);
  }
  hostKey = keyId[kHostname];
  zoneKey = keyId[kZone];
  ctKey = keyId[kCT];
  hostPrivBit = keys[hostKey].nv - 1;
  int W = off;
  wordValid.assign(W, 0);
  vIsInt.assign(W, 0);
  vInt.assign(std::max(vint, 1), 0);
  for (size_t kk = 0; kk < keys.size(); kk++) {
    const KeyMeta& m = keys[kk];
    for (int b = 0; b < m.nv; b++) wordValid[m.off + b / 32] |= 1u << (b % 32);
    if (m.bslot >= 0)
      for (int b = 0; b < (int)values[kk].size(); b++) {
        int64_t x;
        if (go_atoi(values[kk][b], x)) {
          vIsInt[m.off + b / 32] |= 1u << (b % 32);
          vInt[m.vint + b] = x;
        }
      }
  }
  for (auto& w : wellKnown) {
    auto it = keyId.find(w);
    if (it != keyId.end()) allowWK |= 1ull << it->second;
  }
  dims.NK = (int)keys.size();
  dims.W = W;
  dims.NB = nb;
  dims.HDR = 8 + 4 * nb;
  dims.RSW = (dims.HDR + W + 1) & ~1;
  L.nkeys = dims.NK;
  L.W = W;
  L.NB = nb;
  L.HDR = dims.HDR;
  L.RSW = dims.RSW;
  L.keys = keys.data();
  L.wordValid = wordValid.data();
  L.vIsInt = vIsInt.data();
  L.vInt = vInt.data();

  pt.mark("universe");
  // --- resources
  // The resource universe is the names some request list (pods, daemons) or NodePool limit holds: Fits reads
  // the candidate's names only (resources.go:162-175), and the limits test the names the limits list.  Any
  // other name (an instance type's or node's extra capacity nobody requests) decides only through Fits'
  // negative-total rule, which the encoder folds into the entity (neverFits below).
  std::set<std::string> live = {"pods"};  // (every template's daemon overhead names it, getDaemonOverhead)
  for (auto& p : pods) for (auto& kv : p.requests) live.insert(kv.first);
  for (auto& p : daemons) for (auto& kv : p.requests) live.insert(kv.first);
  for (auto& p : pools) for (auto& kv : p.remaining) live.insert(kv.first);
  std::map<std::string, std::vector<__int128>> seen;
  auto visitQ = [&](const QList& q) {
    for (auto& kv : q) if (live.count(kv.first)) seen[kv.first].push_back(kv.second.n);
  };
  for (auto& it : its) { visitQ(it.capacity); visitQ(it.alloc); }
  for (auto& p : pods) visitQ(p.requests);
  for (auto& p : daemons) visitQ(p.requests);
  for (auto& n : nodes) { visitQ(n.available); visitQ(n.capacity); visitQ(n.dsRequests); }
  for (auto& p : pools) visitQ(p.remaining);
  if (seen.size() > (size_t)kMaxR)
    throw KsError(-3, "more than 16 resource names in the pods' / daemons' requests and the NodePool limits");
  for (auto& kv : seen) {
    int shift = 9;
    for (__int128 x : kv.second) {
      while (shift > 0) {
        __int128 d = 1;
        for (int i = 0; i < shift; i++) d *= 10;
        if (x % d == 0) break;
        shift--;
      }
    }
    __int128 d = 1;
    for (int i = 0; i < shift; i++) d *= 10;
    for (__int128 x : kv.second) {
      __int128 v = x / d;
      if (v > ((__int128)1 << 52) || v < -((__int128)1 << 52))
        throw KsError(-3, "quantity of " + kv.first + " exceeds the int64 fixed-point range");
    }
    resId[kv.first] = (int)resNames.size();
    resNames.push_back(kv.first);
    resShift.push_back(shift);
  }
  int R = (int)resNames.size();
  dims.R = R;
  auto vec = [&](const QList& q, int64_t* out) {
    for (int r = 0; r < R; r++) out[r] = 0;
    for (auto& kv : q) {
      auto id = resId.find(kv.first);
      if (id != resId.end()) out[id->second] = toDev(id->second, kv.second);
    }
  };
  // Fits fails on any negative total (resources.go:166-170), outside the universe too: such an entity never fits
  auto neverFits = [&](const QList& q, int64_t* out) {
    for (auto& kv : q)
      if (!resId.count(kv.first) && kv.second.n < 0) out[0] = -1;
  };
  auto qmeta = [&](const QList& q, uint32_t& mask, uint8_t* fmt) {  // names present + formats
    mask = 0;
    for (auto& kv : q) {
      const int r = resId.at(kv.first);
      mask |= 1u << r;
      fmt[r] = (uint8_t)kv.second.f;
    }
  };

  // --- taints universe
  auto internTaint = [&](const TaintH& t) {
    for (auto& x : taints) if (x.key == t.key && x.value == t.value && x.effect == t.effect) return;
    taints.push_back(t);
  };
  for (auto& t : tpls) for (auto& x : t.taints) internTaint(x);
  for (auto& n : nodes) for (auto& x : n.taints) internTaint(x);
  // The device's taint masks are two words over taint CLASSES: taints that exactly the same toleration lists
  // tolerate are interchangeable in every Taints.Tolerates test the device makes (a node's or a template's
  // taints against a relaxation state's tolerations, taints.go), so they share a bit.  The classes are formed
  // once the relaxation chains' toleration lists are final (below); the masks are filled there.
  std::vector<int> taintClass;
  auto taintMask = [&](const std::vector<TaintH>& ts, uint64_t* out) {
    out[0] = out[1] = 0;
    for (auto& t : ts)
      for (size_t i = 0; i < taints.size(); i++)
        if (taints[i].key == t.key && taints[i].value == t.value && taints[i].effect == t.effect)
          out[taintClass[i] >> 6] |= 1ull << (taintClass[i] & 63);
  };

  // --- instance types
  int T = (int)its.size();
  dims.T = T;
  tab.it_alloc.assign((size_t)T * R, 0);
  tab.it_cap.assign((size_t)T * R, 0);
  tab.it_rs.assign((size_t)T * dims.RSW, 0);
  tab.it_off_beg.assign(T + 1, 0);
  for (int i = 0; i < T; i++) {
    vec(its[i].alloc, &tab.it_alloc[(size_t)i * R]);
    neverFits(its[i].alloc, &tab.it_alloc[(size_t)i * R]);
    vec(its[i].capacity, &tab.it_cap[(size_t)i * R]);
    std::vector<uint32_t> rs = emptyRec();
    for (auto& n : its[i].reqs) addNSR(rs, n.key, n.op, n.values);
    std::copy(rs.begin(), rs.end(), tab.it_rs.begin() + (size_t)i * dims.RSW);
    itKeys |= rs_present(rs.data());
    for (size_t o = 0; o < its[i].offers.size(); o++) {
      tab.off_zone.push_back(valueId[zoneKey].at(its[i].offers[o].first));
      tab.off_ct.push_back(valueId[ctKey].at(its[i].offers[o].second));
      tab.off_price.push_back(its[i].prices[o]);
    }
    tab.it_off_beg[i + 1] = (int)tab.off_zone.size();
  }
  itKeys |= (1ull << zoneKey) | (1ull << ctKey);
  if (tab.off_zone.empty()) { tab.off_zone.push_back(0); tab.off_ct.push_back(0); tab.off_price.push_back(0); }

  // --- templates: requirements, daemon overhead (getDaemonOverhead scheduler.go:324-341)
  int NT = (int)tpls.size();
  dims.NTPL = NT;
  tab.tpl_rs.assign((size_t)std::max(NT, 1) * dims.RSW, 0);
  tab.tpl_taint.assign((size_t)std::max(NT, 1) * 2, 0);
  tab.tpl_daemon.assign((size_t)std::max(NT, 1) * R, 0);
  tab.tpl_rmask.assign((size_t)std::max(NT, 1), 0);
  tab.tpl_rfmt.assign((size_t)std::max(NT, 1) * R, 0);
  tab.tpl_it_beg.assign(NT + 1, 0);
  tab.tpl_pool.assign(std::max(NT, 1), -1);
  int maxIts = 0;
  std::vector<std::vector<uint32_t>> daemonAll;
  for (auto& d : daemons) {
    PodH c = d;
    daemonAll.push_back(podRequirements(c, true));
  }
  for (int t = 0; t < NT; t++) {
    Tpl& tp = tpls[t];
    tp.rs = emptyRec();
    for (auto& n : tp.reqs) addNSR(tp.rs, n.key, n.op, n.values);
    addLabels(tp.rs, tp.labels);
    std::vector<uint32_t> withHost = tp.rs;
    {
      std::vector<uint32_t> h = emptyRec();
      const KeyMeta& hm = keys[hostKey];
      wr64(h.data(), 0, 1ull << hostKey);
      h[L.HDR + hm.off + (hostPrivBit >> 5)] |= 1u << (hostPrivBit & 31);
      rs_add(L, withHost.data(), h.data());
    }
    std::copy(withHost.begin(), withHost.end(), tab.tpl_rs.begin() + (size_t)t * dims.RSW);
    QList overhead;
    int nd = 0;
    for (size_t i = 0; i < daemons.size(); i++) {
      if (!tolerates(tp.taints, daemons[i].tols)) continue;
      if (!rs_compatible(L, tp.rs.data(), daemonAll[i].data(), allowWK)) continue;
      QList r = daemons[i].requests;
      r.erase("pods");
      mergeInto(overhead, r);
      nd++;
    }
    Qty pods;
    pods.n = (__int128)nd * 1000000000;
    pods.f = QFmt::DecExp;
    overhead["pods"] = pods;
    tp.daemon = overhead;
    if (!resId.count("pods")) throw KsError(-5, "pods resource missing");
    vec(overhead, &tab.tpl_daemon[(size_t)t * R]);
    qmeta(overhead, tab.tpl_rmask[(size_t)t], &tab.tpl_rfmt[(size_t)t * R]);
    for (int i : tp.its) tab.tpl_its.push_back(i);
    tab.tpl_it_beg[t + 1] = (int)tab.tpl_its.size();
    maxIts = std::max(maxIts, (int)tp.its.size());
    for (size_t p = 0; p < pools.size(); p++)
      if (pools[p].name == tp.pool) tab.tpl_pool[t] = (int)p;
  }
  if (tab.tpl_its.empty()) tab.tpl_its.push_back(0);
  dims.maxTplIts = maxIts;
  dims.totalTplIts = (int)tab.tpl_it_beg[NT];
  dims.TW = std::max(1, (maxIts + 31) / 32);
  // Per template and resource, the template positions ordered by Allocatable ascending: the options a
  // growing request excludes (resources.go:162-175 Fits) are always a prefix of this order.
  tab.tsort_alloc.assign((size_t)std::max(dims.totalTplIts, 1) * R, 0);
  tab.tsort_pos.assign((size_t)std::max(dims.totalTplIts, 1) * R, 0);
  for (int t = 0; t < NT; t++) {
    const int tb = tab.tpl_it_beg[t], n = tab.tpl_it_beg[t + 1] - tb;
    std::vector<int> ord(n);
    for (int r = 0; r < R; r++) {
      for (int i = 0; i < n; i++) ord[i] = i;
      auto al = [&](int i) { return tab.it_alloc[(size_t)tab.tpl_its[tb + i] * R + r]; };
      std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return al(a) < al(b); });
      const size_t base = (size_t)tb * R + (size_t)r * n;
      for (int i = 0; i < n; i++) {
        tab.tsort_alloc[base + i] = al(ord[i]);
        tab.tsort_pos[base + i] = ord[i];
      }
    }
  }

  // --- feasibility tables (k_solve feas_masks): per template, the positions of its instance-type list as
  // bitsets per (key, value), so Requirements.Intersects(IT, X) and hasOffering(IT, X) of
  // filterInstanceTypesByRequirements (nodeclaim.go:225-278) evaluate for every position at once as
  // unions and intersections of bitsets.  Per template: [all positions][irregular] then per key of an
  // instance type: [lacks the key][DoesNotExist][In][has value 0][has value 1]..., then the available
  // offerings per (zone, capacity-type) value pair.  An IT requirement that is a complement (NotIn /
  // Exists / Gt / Lt) makes its position irregular: those keep the exact per-position check.
  {
    const int TW = dims.TW, NK = dims.NK;
    tab.fk_key_off.assign((size_t)std::max(NT, 1) * NK, -1);
    tab.fk_tpl.assign((size_t)std::max(NT, 1) * 3, 0);
    tab.fk_words.clear();
    uint64_t multi = 0;  // keys some instance type constrains with more than one value
    auto blk = [&](size_t words) {
      const size_t o = tab.fk_words.size();
      tab.fk_words.resize(o + words, 0);
      return o;
    };
    auto setb = [&](size_t off, int p) { tab.fk_words[off + (size_t)(p >> 5)] |= 1u << (p & 31); };
    for (int t = 0; t < NT; t++) {
      const int tb = tab.tpl_it_beg[t], n = tab.tpl_it_beg[t + 1] - tb;
      const size_t all = blk((size_t)TW), irr = blk((size_t)TW);
      for (int p = 0; p < n; p++) setb(all, p);
      for (uint64_t m = itKeys; m; m &= m - 1) {
        const int k = __builtin_ctzll(m);
        const KeyMeta& km = keys[(size_t)k];
        const size_t base = blk((size_t)(3 + km.nv) * TW);
        tab.fk_key_off[(size_t)t * NK + k] = (int32_t)base;
        for (int p = 0; p < n; p++) {
          const uint32_t* r = &tab.it_rs[(size_t)tab.tpl_its[(size_t)(tb + p)] * dims.RSW];
          if (!bit(rs_present(r), k)) {
            setb(base, p);
            continue;
          }
          if (bit(rs_compl(r), k)) {
            setb(irr, p);
            continue;
          }
          int cnt = 0;
          for (int v = 0; v < km.nv; v++)
            if ((r[L.HDR + km.off + (v >> 5)] >> (v & 31)) & 1u) {
              setb(base + (size_t)(3 + v) * TW, p);
              cnt++;
            }
          setb(base + (size_t)(cnt == 0 ? 1 : 2) * TW, p);
          if (cnt > 1) multi |= 1ull << k;
        }
      }
      const int nz = keys[(size_t)zoneKey].nv, nc = keys[(size_t)ctKey].nv;
      const size_t off = blk((size_t)nz * nc * TW);
      for (int p = 0; p < n; p++) {
        const int it = tab.tpl_its[(size_t)(tb + p)];
        for (int o = tab.it_off_beg[(size_t)it]; o < tab.it_off_beg[(size_t)it + 1]; o++)
          setb(off + ((size_t)tab.off_zone[(size_t)o] * nc + tab.off_ct[(size_t)o]) * TW, p);
      }
      tab.fk_tpl[(size_t)t * 3] = (int32_t)all;
      tab.fk_tpl[(size_t)t * 3 + 1] = (int32_t)irr;
      tab.fk_tpl[(size_t)t * 3 + 2] = (int32_t)off;
    }
    if (tab.fk_words.size() > (size_t)INT32_MAX) throw KsError(-3, "feasibility tables exceed 2^31 words");
    dims.fkMulti = multi;
    if (tab.fk_words.empty()) tab.fk_words.push_back(0);
  }

  pt.mark("resources+taints+its+templates");
  // --- existing nodes (NewExistingNode, calculateExistingNodeClaims)
  int N = (int)nodes.size();
  dims.N = N;
  tab.n_avail.assign((size_t)std::max(N, 1) * R, 0);
  tab.n_req0.assign((size_t)std::max(N, 1) * R, 0);
  tab.n_rs0.assign((size_t)std::max(N, 1) * dims.RSW, 0);
  tab.n_taint.assign((size_t)std::max(N, 1) * 2, 0);
  tab.n_flags.assign(std::max(N, 1), 0);
  tab.n_hp0.assign(std::max(N, 1), 0);
  // --- host ports: masks over a universe of (IP, port, protocol) triples (HostPort.Matches,
  // hostportusage.go:45-58).  HostPortUsage.reserved is keyed by pod (namespace/name): Conflicts skips
  // the entries of the pod being checked and Add replaces that pod's entries (hostportusage.go:70-85).
  // A node's initial entries whose pod key is also a pod being scheduled (e.g. a re-created StatefulSet
  // pod whose predecessor still holds the ports) get universe elements of their own, tagged with that
  // key: the pod's conflict mask leaves them out, and its commit clears them (pod_hpo).
  bool anyPorts = false;
  for (auto& p : pods) anyPorts = anyPorts || !p.ports.empty();
  for (auto& n : nodes) anyPorts = anyPorts || !n.hostPorts.empty();
  std::map<std::string, int> podKeyCount;
  if (anyPorts)
    for (auto& p : pods) podKeyCount[p.ns + "/" + p.name]++;
  hostPortOwner.clear();
  auto internHP = [&](const HostPortH& h, const std::string& owner) {
    for (size_t i = 0; i < hostPortUniverse.size(); i++)
      if (hostPortUniverse[i].ip == h.ip && hostPortUniverse[i].port == h.port && hostPortUniverse[i].proto == h.proto &&
          hostPortOwner[i] == owner)
        return (int)i;
    hostPortUniverse.push_back(h);
    hostPortOwner.push_back(owner);
    return (int)hostPortUniverse.size() - 1;
  };
  for (auto& p : pods) for (auto& h : p.ports) internHP(h, "");
  std::set<std::string> ownerKeys;  // pods being scheduled with entries on some existing node
  for (auto& n : nodes)
    for (auto& e : n.hostPorts) {
      const bool pending = podKeyCount.count(e.first) != 0;
      if (pending) ownerKeys.insert(e.first);
      internHP(e.second, pending ? e.first : "");
    }
  for (auto& p : pods) {  // Add on a NodeClaim replaces a same-key pod's entries: not modelled
    if (!anyPorts) break;
    const std::string key = p.ns + "/" + p.name;
    if (podKeyCount[key] > 1 && (!p.ports.empty() || ownerKeys.count(key)))
      throw KsError(-2, "pods being scheduled share the key " + key + " and host ports");
  }
  // The device masks are one word over element CLASSES: elements that every pod being scheduled treats alike
  // (in its conflict set, its reservations and its own initial entries, or in none of them) evolve alike
  // under Conflicts / Add on every node and NodeClaim, so they share a bit; a node's entries that no pod
  // matches collapse into one class.  Classes are formed with the pods' masks (below).
  std::vector<std::vector<int>> nodeHP((size_t)N);
  auto hpMask = [&](const std::vector<std::pair<std::string, HostPortH>>& v, std::vector<int>& out) {
    for (auto& e : v) out.push_back(internHP(e.second, podKeyCount.count(e.first) ? e.first : ""));
    return 0ull;
  };
  dims.hpAny = hostPortUniverse.empty() ? 0 : 1;
  // --- volume limits (ExistingNode.Add: GetVolumes + VolumeUsage.ExceedsLimits, existingnode.go:70-78).
  // GetVolumes skips PVCs the snapshot does not resolve (NotFound) and empty drivers; it fails for a claim
  // bound to a PV that does not exist (volErrKeys), and then ExistingNode.Add fails on every node
  // (PF_VOLERR).  Only drivers some node limits can fail the check; the pods' PVCs of those drivers form the
  // universe (ids u), any number of them.  Per node and driver: |usage ∪ pod| = count + |pod PVCs not yet
  // mounted|, where "mounted" is asked only of the pod's own PVCs (KsDev, ks_problem.h).  A node already over a
  // limit rejects every pod (the union always holds its own set), which the encoder folds into an
  // unsatisfiable Available().
  std::set<std::string> limited;
  for (auto& n : nodes)
    for (auto& kv : n.volumeLimits) {
      if (kv.second < 0 || kv.second > INT32_MAX)
        throw KsError(-2, "node " + n.name + ": volume limit out of range for driver " + kv.first);
      limited.insert(kv.first);
    }
  auto podVolumes = [&](const PodH& p) {  // GetVolumes (volumeusage.go:82-113): driver -> set of PVC keys
    std::map<std::string, std::set<std::string>> out;
    for (auto& name : p.pvcNames) {
      auto it = volumeDrivers.find(p.ns + "/" + name);
      if (it == volumeDrivers.end() || it->second.empty()) continue;
      out[it->second].insert(p.ns + "/" + name);
    }
    return out;
  };
  std::map<std::string, int> volBit, volDrv;  // PVC key -> u; driver -> v
  volDrivers.clear();
  volUniverse.clear();
  std::vector<int32_t> udrv;
  std::vector<std::vector<int>> podU(pods.size());  // per pod: its universe PVCs
  std::vector<std::vector<std::pair<int, int>>> podVD(pods.size());  // per pod: (v, count)
  std::vector<char> podVolErr(pods.size(), 0);
  for (size_t i = 0; i < pods.size(); i++) {
    for (auto& name : pods[i].pvcNames) podVolErr[i] |= volErrKeys.count(pods[i].ns + "/" + name) ? 1 : 0;
    for (auto& dv : podVolumes(pods[i])) {
      if (!limited.count(dv.first)) continue;
      auto d = volDrv.find(dv.first);
      if (d == volDrv.end()) {
        d = volDrv.emplace(dv.first, (int)volDrivers.size()).first;
        volDrivers.push_back(dv.first);
      }
      podVD[i].push_back({d->second, (int)dv.second.size()});
      for (auto& key : dv.second) {
        auto b = volBit.find(key);
        if (b == volBit.end()) {
          b = volBit.emplace(key, (int)volUniverse.size()).first;
          volUniverse.push_back(key);
          udrv.push_back(d->second);
        }
        podU[i].push_back(b->second);
      }
    }
  }
  const int VD = (int)volDrivers.size(), NVU = (int)volUniverse.size();
  if ((int64_t)std::max(N, 1) * std::max(VD, 1) > INT32_MAX / 2) throw KsError(-3, "volume count table exceeds 2^30 entries");
  dims.VD = VD;
  dims.NVU = NVU;
  // the nodes mounting each universe PVC at NewScheduler time
  std::vector<std::vector<int>> uNodes((size_t)NVU);
  tab.n_vc0.assign((size_t)std::max(N, 1) * std::max(VD, 1), 0);
  tab.n_vlim.assign((size_t)std::max(N, 1) * std::max(VD, 1), INT32_MAX);
  std::vector<char> volBlocked(std::max(N, 1), 0);
  for (int i = 0; i < N; i++) {
    Node& n = nodes[i];
    for (auto& kv : n.volumeLimits) {
      auto u = n.volumes.find(kv.first);
      if (u != n.volumes.end() && (int64_t)u->second.size() > kv.second) volBlocked[i] = 1;
    }
    for (int v = 0; v < VD; v++) {
      auto u = n.volumes.find(volDrivers[v]);
      if (u != n.volumes.end()) {
        tab.n_vc0[(size_t)i * VD + v] = (int32_t)u->second.size();
        for (auto& key : u->second) {
          auto b = volBit.find(key);
          if (b != volBit.end() && udrv[(size_t)b->second] == v) uNodes[(size_t)b->second].push_back(i);
        }
      }
      auto l = n.volumeLimits.find(volDrivers[v]);
      if (l != n.volumeLimits.end()) tab.n_vlim[(size_t)i * VD + v] = (int32_t)l->second;
    }
  }
  // pods sharing a PVC with another pod being scheduled: their placements log the PVCs they mount
  std::vector<int> uPods((size_t)NVU, 0);
  for (auto& us : podU) for (int u : us) uPods[(size_t)u]++;
  const int P0 = (int)pods.size();
  tab.pod_vdbeg.assign((size_t)P0 + 1, 0);
  tab.pod_vsbeg.assign((size_t)P0 + 1, 0);
  tab.pod_vubeg.assign((size_t)P0 + 1, 0);
  tab.pod_vd.clear();
  tab.pod_vs.clear();
  tab.pod_vu.clear();
  std::vector<char> podShared(pods.size(), 0);
  int64_t vlog = 0;
  bool anyVol = false;
  for (int i = 0; i < P0; i++) {
    for (auto& e : podVD[(size_t)i]) {
      tab.pod_vd.push_back(e.first);
      tab.pod_vd.push_back(e.second);
    }
    for (int u : podU[(size_t)i]) {
      for (int n : uNodes[(size_t)u]) {
        tab.pod_vs.push_back(n);
        tab.pod_vs.push_back(u);
      }
      podShared[(size_t)i] |= uPods[(size_t)u] > 1 ? 1 : 0;
    }
    if (podShared[(size_t)i]) {
      tab.pod_vu.insert(tab.pod_vu.end(), podU[(size_t)i].begin(), podU[(size_t)i].end());
      vlog += (int64_t)podU[(size_t)i].size();
    }
    anyVol = anyVol || !podVD[(size_t)i].empty() || podVolErr[(size_t)i];
    tab.pod_vdbeg[(size_t)i + 1] = (int32_t)(tab.pod_vd.size() / 2);
    tab.pod_vsbeg[(size_t)i + 1] = (int32_t)(tab.pod_vs.size() / 2);
    tab.pod_vubeg[(size_t)i + 1] = (int32_t)tab.pod_vu.size();
  }
  if (tab.pod_vs.size() > (size_t)INT32_MAX || vlog > INT32_MAX / 4) throw KsError(-3, "volume tables exceed 2^30 entries");
  for (auto* v : {&tab.pod_vd, &tab.pod_vs}) if (v->empty()) v->assign(2, 0);
  if (tab.pod_vu.empty()) tab.pod_vu.push_back(0);
  tab.vol_udrv = udrv;
  if (tab.vol_udrv.empty()) tab.vol_udrv.push_back(0);
  dims.vLogCap = (int32_t)vlog;
  dims.volAny = anyVol && N > 0 ? 1 : 0;
  for (int i = 0; i < N; i++) {
    Node& n = nodes[i];
    tab.n_flags[i] = (!n.initialized || !n.ready) ? NF_UNUSABLE : 0;
    tab.n_hp0[i] = hpMask(n.hostPorts, nodeHP[(size_t)i]);
    std::vector<uint32_t> lab = emptyRec();
    addNodeLabels(lab, n.labels);  // the keys of the universe only (see the universe build)
    QList dreq;
    int nd = 0;
    for (size_t d = 0; d < daemons.size(); d++) {
      if (!tolerates(n.taints, daemons[d].tols)) continue;
      if (!rs_compatible(L, lab.data(), daemonAll[d].data(), 0)) continue;
      QList r = daemons[d].requests;
      r.erase("pods");
      mergeInto(dreq, r);
      nd++;
    }
    Qty pq;
    pq.n = (__int128)nd * 1000000000;
    pq.f = QFmt::DecExp;
    dreq["pods"] = pq;
    n.req0 = dreq;  // Subtract(daemon, DaemonSetRequests) keeps lhs keys; negatives clamp to 0
    for (auto& kv : n.req0) {
      auto s = n.dsRequests.find(kv.first);
      if (s != n.dsRequests.end()) {
        if (kv.second.n == 0) kv.second.f = s->second.f;
        kv.second.n -= s->second.n;
      }
      if (kv.second.n < 0) kv.second.n = 0;
    }
    vec(n.available, &tab.n_avail[(size_t)i * R]);
    neverFits(n.available, &tab.n_avail[(size_t)i * R]);
    if (volBlocked[i]) tab.n_avail[(size_t)i * R] = -1;  // Fits fails on any negative total (resources.go:166-170)
    vec(n.req0, &tab.n_req0[(size_t)i * R]);
    addNSR(lab, kHostname, "In", {n.hostName});
    std::copy(lab.begin(), lab.end(), tab.n_rs0.begin() + (size_t)i * dims.RSW);
  }
  pt.mark("nodes+hostports+volumes");
  // --- limits: remaining = Limits - capacity of existing nodes in the pool
  int NP = (int)pools.size();
  dims.NPOOL = NP;
  tab.pool_rem0.assign((size_t)std::max(NP, 1) * R, 0);
  tab.pool_mask.assign(std::max(NP, 1), 0);
  for (int p = 0; p < NP; p++) {
    QList rem = pools[p].remaining;
    for (auto& n : nodes) {
      auto l = n.labels.find(kNodePoolKey);
      if (l == n.labels.end() || l->second != pools[p].name) continue;
      for (auto& kv : rem) {
        auto c = n.capacity.find(kv.first);
        if (c != n.capacity.end()) {
          if (kv.second.n == 0) kv.second.f = c->second.f;
          kv.second.n -= c->second.n;
        }
      }
    }
    pools[p].remaining = rem;
    for (auto& kv : rem) {
      auto it = resId.find(kv.first);
      if (it == resId.end()) continue;
      tab.pool_mask[p] |= 1u << it->second;
      tab.pool_rem0[(size_t)p * R + it->second] = toDev(it->second, kv.second);
    }
  }

  pt.mark("limits");
  // --- pods: requests, queue sort keys, relaxation chains
  int P = (int)pods.size();
  dims.P = P;
  tab.pod_req.assign((size_t)std::max(P, 1) * R, 0);
  tab.pod_rmask.assign((size_t)std::max(P, 1), 0);
  tab.pod_rfmt.assign((size_t)std::max(P, 1) * R, 0);
  tab.pod_sortkey.assign((size_t)std::max(P, 1) * 4, 0);
  tab.pod_state0.assign(std::max(P, 1), 0);
  tab.pod_nstate.assign(std::max(P, 1), 0);
  tab.pod_uid.assign(std::max(P, 1), 0);
  tab.pod_flags.assign(std::max(P, 1), 0);
  tab.pod_hpc.assign(std::max(P, 1), 0);
  tab.pod_hpu.assign(std::max(P, 1), 0);
  tab.pod_hpo.assign(std::max(P, 1), 0);
  const size_t NUH = hostPortUniverse.size();
  // per element, the pods that have it in their conflict / reservation / own-entry sets (pod order)
  std::vector<std::vector<int32_t>> hpSig(NUH);
  for (int i = 0; i < P; i++) {
    tab.pod_flags[i] = (pods[i].provisionable ? PF_PROVISIONABLE : 0) | (podShared[(size_t)i] ? PF_VSHARED : 0) |
                       (podVolErr[(size_t)i] ? PF_VOLERR : 0);
    if (NUH == 0 || (pods[i].ports.empty() && !ownerKeys.count(pods[i].ns + "/" + pods[i].name))) continue;
    const std::string key = pods[i].ns + "/" + pods[i].name;
    for (size_t u = 0; u < NUH; u++) {
      bool hpc = false, hpu = false;
      const bool hpo = hostPortOwner[u] == key;  // its own entries: never a conflict, replaced by Add
      for (auto& h : pods[i].ports) {
        hpu = hpu || (hostPortUniverse[u].ip == h.ip && hostPortUniverse[u].port == h.port &&
                      hostPortUniverse[u].proto == h.proto && hostPortOwner[u].empty());
        hpc = hpc || (h.matches(hostPortUniverse[u]) && hostPortOwner[u] != key);
      }
      const int code = (hpc ? 1 : 0) | (hpu ? 2 : 0) | (hpo ? 4 : 0);
      if (code) hpSig[u].push_back(i * 8 + code);
    }
  }
  if (NUH) {
    std::map<std::vector<int32_t>, int> cls;
    std::vector<int> hpClass(NUH);
    for (size_t u = 0; u < NUH; u++) hpClass[u] = cls.emplace(hpSig[u], (int)cls.size()).first->second;
    if (cls.size() > 64)
      throw KsError(-3, "more than 64 host-port classes (" + std::to_string(NUH) +
                            " (IP, port, protocol) entries that the pods being scheduled tell apart)");
    for (size_t u = 0; u < NUH; u++)
      for (int32_t e : hpSig[u]) {
        const int i = e >> 3, code = e & 7;
        const uint64_t b = 1ull << hpClass[u];
        if (code & 1) tab.pod_hpc[(size_t)i] |= b;
        if (code & 2) tab.pod_hpu[(size_t)i] |= b;
        if (code & 4) tab.pod_hpo[(size_t)i] |= b;
      }
    for (int i = 0; i < N; i++)
      for (int u : nodeHP[(size_t)i]) tab.n_hp0[(size_t)i] |= 1ull << hpClass[(size_t)u];
  }
  std::map<std::string, int> uids;
  for (auto& p : pods) uids[p.uid] = 0;
  int u = 0;
  for (auto& kv : uids) kv.second = u++;  // id == rank in Go string order
  dims.NU = std::max(u, 1);
  int cpuR = resId.count("cpu") ? resId["cpu"] : -1, memR = resId.count("memory") ? resId["memory"] : -1;
  std::vector<std::array<int64_t, 4>> sk(P);
  int S = 0;
  states.assign((size_t)P, {});
  // per pod (independent: worker threads): requests, queue key, relaxation chain
  parallel_for(P, 128, [&](int i) {
    PodH& p = pods[i];
    vec(p.requests, &tab.pod_req[(size_t)i * R]);
    qmeta(p.requests, tab.pod_rmask[(size_t)i], &tab.pod_rfmt[(size_t)i * R]);
    int64_t cpu = cpuR >= 0 ? tab.pod_req[(size_t)i * R + cpuR] : 0;
    int64_t mem = memR >= 0 ? tab.pod_req[(size_t)i * R + memR] : 0;
    int64_t* k4 = &tab.pod_sortkey[(size_t)i * 4];
    const int uidRank = uids.at(p.uid);
    k4[0] = -cpu;  // descending
    k4[1] = -mem;
    k4[2] = p.created;
    k4[3] = uidRank;
    sk[i] = {k4[0], k4[1], k4[2], k4[3]};
    tab.pod_uid[i] = uidRank;
    // relaxation chain
    PodH cur = p;
    std::vector<PodState> chain;
    for (int guard = 0; guard < 256; guard++) {
      PodState st;
      st.rsAll = podRequirements(cur, true);
      st.rsStrict = podRequirements(cur, false);
      st.hasPreferred = cur.hasAffinity && cur.hasNodeAffinity && !cur.preferred.empty();
      st.tols = cur.tols;
      if (!cur.tsc.empty() || !cur.antiRequired.empty() || !cur.antiPreferred.empty() || !cur.affRequired.empty() ||
          !cur.affPreferred.empty())
        st.spec = std::make_shared<PodH>(cur);
      chain.push_back(std::move(st));
      // Preferences.Relax (preferences.go:38-58)
      bool relaxed = false;
      if (cur.hasAffinity && cur.hasNodeAffinity && cur.hasRequired && cur.requiredTerms.size() > 1) {
        cur.requiredTerms.erase(cur.requiredTerms.begin());
        relaxed = true;
      } else if (cur.hasAffinity && cur.hasPodAffinity && !cur.affPreferred.empty()) {
        std::stable_sort(cur.affPreferred.begin(), cur.affPreferred.end(),
                         [](const std::pair<int32_t, AffTerm>& a, const std::pair<int32_t, AffTerm>& b) { return a.first > b.first; });
        cur.affPreferred.erase(cur.affPreferred.begin());
        relaxed = true;
      } else if (cur.hasAffinity && cur.hasPodAnti && !cur.antiPreferred.empty()) {
        std::stable_sort(cur.antiPreferred.begin(), cur.antiPreferred.end(),
                         [](const std::pair<int32_t, AffTerm>& a, const std::pair<int32_t, AffTerm>& b) { return a.first > b.first; });
        cur.antiPreferred.erase(cur.antiPreferred.begin());
        relaxed = true;
      } else if (cur.hasAffinity && cur.hasNodeAffinity && !cur.preferred.empty()) {
        std::stable_sort(cur.preferred.begin(), cur.preferred.end(),
                         [](const PrefTerm& a, const PrefTerm& b) { return a.weight > b.weight; });
        cur.preferred.erase(cur.preferred.begin());
        relaxed = true;
      } else {
        for (size_t j = 0; j < cur.tsc.size(); j++)
          if (cur.tsc[j].when == "ScheduleAnyway") {
            cur.tsc[j] = cur.tsc.back();
            cur.tsc.pop_back();
            relaxed = true;
            break;
          }
        if (!relaxed && toleratePreferNoSchedule) {
          bool have = false;
          for (auto& t : cur.tols)
            if (t.key.empty() && t.op == "Exists" && t.value.empty() && t.effect == "PreferNoSchedule") have = true;
          if (!have) {
            cur.tols.push_back(TolH{"", "Exists", "", "PreferNoSchedule"});
            relaxed = true;
          }
        }
      }
      if (!relaxed) break;
    }
    states[(size_t)i] = std::move(chain);
  });
  for (int i = 0; i < P; i++) {
    tab.pod_state0[i] = S;
    tab.pod_nstate[i] = (int)states[(size_t)i].size();
    S += (int)states[(size_t)i].size();
  }
  for (int c = 0; c < 4; c++) {
    int64_t mn = 0, mx = 0;
    for (int i = 0; i < P; i++) {
      mn = i ? std::min(mn, sk[i][c]) : sk[i][c];
      mx = i ? std::max(mx, sk[i][c]) : sk[i][c];
    }
    uint64_t span = (uint64_t)(mx - mn);
    int bits = 0;
    while (span) { bits++; span >>= 1; }
    dims.skMin[c] = mn;
    dims.skBits[c] = bits;
  }
  dims.dupUids = (int)uids.size() < P ? 1 : 0;
  // The threshold filter in k_solve assumes requests only grow (no negative quantities).
  dims.negReq = 0;
  for (int64_t v : tab.pod_req) dims.negReq |= v < 0;
  for (int64_t v : tab.tpl_daemon) dims.negReq |= v < 0;
  {
    // NewQueue: sort.Slice(pods, byCPUAndMemoryDescending) (queue.go:37-43,83-112).  Its less() is the
    // lexicographic order of (-cpu, -memory, creationTimestamp, uid); without ties every unstable sort
    // agrees and the device radix-sorts the keys.  With ties the order is pdqsort's swap sequence over
    // the input order: emulate sort.Slice on the keys' dense ranks (less() is all pdqsort observes).
    std::vector<int> idx(P);
    for (int i = 0; i < P; i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](int a, int b) { return sk[a] < sk[b]; });
    bool ties = false;
    for (int i = 1; i < P && !ties; i++) ties = sk[idx[i]] == sk[idx[i - 1]];
    hostQueue.clear();
    if (ties) {
      std::vector<int32_t> key(P), val(P);
      int rank = 0;
      for (int i = 0; i < P; i++) {
        if (i > 0 && sk[idx[i]] != sk[idx[i - 1]]) rank++;
        key[idx[i]] = rank;
      }
      for (int i = 0; i < P; i++) val[i] = i;
      GoSortExact g{GoSort{key.data(), val.data()}};
      g.run(P);
      hostQueue = val;
    }
  }
  pt.mark("pods encode");
  dims.S = std::max(S, 1);
  buildTopology();
  pt.mark("topology");
  // Topology ownership is keyed by UID (TopologyGroup.owners, topologygroup.go; Topology.Update removes
  // the UID from every group first, topology.go:91-122): pods sharing a UID share their groups, which
  // the per-pod relaxation states here do not model.
  if (dims.dupUids && !groups.empty())
    throw KsError(-2, "pods sharing a UID own topology groups (TopologyGroup owners are keyed by UID)");
  {  // taint classes: the distinct toleration lists of every relaxation state, then one class per distinct
     // "tolerated by which lists" signature
    std::map<std::vector<std::string>, int> lists;
    std::vector<const std::vector<TolH>*> tl;
    for (auto& chain : states)
      for (auto& st : chain) {
        std::vector<std::string> k;
        for (auto& t : st.tols) k.push_back(t.key + '\x1f' + t.op + '\x1f' + t.value + '\x1f' + t.effect);
        if (lists.emplace(std::move(k), (int)tl.size()).second) tl.push_back(&st.tols);
      }
    std::map<std::vector<uint64_t>, int> sig;
    taintClass.assign(taints.size(), 0);
    for (size_t i = 0; i < taints.size(); i++) {
      std::vector<uint64_t> b((tl.size() + 63) / 64, 0);
      for (size_t j = 0; j < tl.size(); j++) {
        bool ok = false;
        for (auto& t : *tl[j]) ok = ok || toleratesTaint(t, taints[i]);
        if (ok) b[j >> 6] |= 1ull << (j & 63);
      }
      taintClass[i] = sig.emplace(std::move(b), (int)sig.size()).first->second;
    }
    if (sig.size() > 128)
      throw KsError(-3, "more than 128 taint classes (" + std::to_string(taints.size()) +
                            " taints that the pods' toleration lists tell apart)");
    for (int t = 0; t < NT; t++) taintMask(tpls[(size_t)t].taints, &tab.tpl_taint[(size_t)t * 2]);
    for (int i = 0; i < N; i++) taintMask(nodes[(size_t)i].taints, &tab.n_taint[(size_t)i * 2]);
  }
  tab.st_rs.assign((size_t)dims.S * dims.RSW, 0);
  tab.st_tol.assign((size_t)dims.S * 2, 0);
  tab.st_flags.assign(dims.S, 0);
  tab.st_toltpl.assign(dims.S, 0);
  tab.st_gown.assign((size_t)dims.S * dims.GMW, 0);
  tab.st_rss.assign(groups.empty() ? 1 : (size_t)dims.S * dims.RSW, 0);
  int s = 0;
  for (auto& chain : states)
    for (auto& st : chain) {
      std::copy(st.rsAll.begin(), st.rsAll.end(), tab.st_rs.begin() + (size_t)s * dims.RSW);
      uint64_t m[2];
      tolMask(st.tols, taintClass, m);
      tab.st_tol[(size_t)s * 2] = m[0];
      tab.st_tol[(size_t)s * 2 + 1] = m[1];
      uint64_t pres = rs_present(st.rsAll.data());
      uint64_t tt = 0;
      for (int t = 0; t < dims.NTPL; t++)
        if (((tab.tpl_taint[(size_t)t * 2] & ~m[0]) | (tab.tpl_taint[(size_t)t * 2 + 1] & ~m[1])) == 0) tt |= 1ull << t;
      tab.st_toltpl[s] = tt;
      if (!groups.empty()) {
        for (int32_t g : st.gown) gset(tab.st_gown, (size_t)s, dims.GMW, g);
        std::copy(st.rsStrict.begin(), st.rsStrict.end(), tab.st_rss.begin() + (size_t)s * dims.RSW);
      }
      tab.st_flags[s] = (st.hasPreferred ? SF_HAS_PREFERRED : 0) | ((pres & itKeys) ? SF_TOUCHES_IT_KEYS : 0) |
                        (pres ? SF_HAS_KEYS : 0);
      s++;
    }
  dims.zoneKey = zoneKey;
  dims.ctKey = ctKey;
  dims.hostKey = hostKey;
  dims.spotBit = valueId[ctKey].at("spot");
  dims.odBit = valueId[ctKey].at("on-demand");
  dims.allowWK = allowWK;
  dims.itKeys = itKeys;
  dims.hostnameSeed = (int32_t)hostnameSeed;
  dims.Kcap = std::max(1, std::min(P, 16384));
  bool anyKeys = false;
  for (int32_t f : tab.st_flags) anyKeys |= (f & SF_HAS_KEYS) != 0;
  // Shared UIDs (BenchmarkScheduling's literal pods all have UID "") matter only once a pod is pushed back
  // (Queue.Pop's lastLen is keyed by UID, queue.go:54-69): the LEAN Solve takes them and leaves at the first
  // push-back (KE_LEAN_EXIT), after which the host re-runs the Solve non-LEAN.
  dims.lean = !dims.hpAny && !dims.volAny && !dims.negReq && groups.empty() && !anyKeys ? 1 : 0;
}

// ---------------------------------------------------------------------------------------------
// Renderers
// ---------------------------------------------------------------------------------------------
std::string Host::reqString(const uint32_t* rec, int k, bool full, int64_t privateHost) const {
  int op = rs_op(L, rec, k);
  static const char* opn[] = {"In", "NotIn", "Exists", "DoesNotExist"};
  std::string s = keyNames[k] + " " + opn[op];
  if (op == OP_IN || op == OP_NOTIN) {
    std::vector<std::string> vs;
    const KeyMeta& km = keys[k];
    for (int b = 0; b < km.nv; b++)
      if ((rec[L.HDR + km.off + (b >> 5)] >> (b & 31)) & 1u)
        vs.push_back(k == hostKey && b == hostPrivBit ? placeholder(privateHost) : values[k][b]);
    std::sort(vs.begin(), vs.end());
    if (!full && vs.size() > 5) {
      size_t n = vs.size();
      vs.resize(5);
      vs.push_back("and " + std::to_string(n - 5) + " others");
    }
    s += " [";
    for (size_t i = 0; i < vs.size(); i++) { if (i) s += " "; s += vs[i]; }
    s += "]";
  }
  const KeyMeta& km = keys[k];
  if (km.bslot >= 0) {
    if (bit(rs_hasgt(rec), k)) s += " >" + std::to_string(rs_gt(rec, km.bslot));
    if (bit(rs_haslt(rec), k)) s += " <" + std::to_string(rs_lt(rec, km.bslot));
  }
  return s;
}

std::string Host::reqsString(const uint32_t* rec, int64_t privateHost) const {
  std::vector<std::string> parts;
  uint64_t pr = rs_present(rec);
  for (int k = 0; k < dims.NK; k++)
    if (bit(pr, k) && k != hostKey) parts.push_back(reqString(rec, k, false, privateHost));
  std::sort(parts.begin(), parts.end());
  std::string s;
  for (size_t i = 0; i < parts.size(); i++) { if (i) s += ", "; s += parts[i]; }
  return s;
}

static int editDistance(const std::string& s, const std::string& t) {  // requirements.go:177-210
  int m = (int)s.size(), n = (int)t.size();
  if (m == 0) return n;
  if (n == 0) return m;
  std::vector<int> prev(n, 0), cur(n, 0);
  for (int j = 1; j < n; j++) prev[j] = j;
  for (int i = 1; i < m; i++) {
    for (int j = 1; j < n; j++)
      cur[j] = std::min(std::min(prev[j] + 1, cur[j - 1] + 1), prev[j - 1] + (s[i] != t[j] ? 1 : 0));
    std::swap(prev, cur);
  }
  return prev[n - 1];
}

std::vector<std::string> Host::compatErrors(const uint32_t* r, const uint32_t* in, bool loose,
                                            int64_t privateHost) const {
  std::vector<std::string> out;
  uint64_t uf = 0, xf = 0;
  rs_compatible(L, r, in, loose ? allowWK : 0, &uf, &xf);
  auto hint = [&](const std::string& key) -> std::string {  // labelHint requirements.go:220-238
    auto suffix = [](const std::string& k) {
      auto p = k.find('/');
      return p == std::string::npos ? k : k.substr(p + 1);
    };
    auto endsWith = [](const std::string& a, const std::string& b) {
      return a.size() >= b.size() && a.compare(a.size() - b.size(), b.size(), b) == 0;
    };
    std::vector<std::string> cands;
    if (loose) cands.assign(wellKnown.begin(), wellKnown.end());
    for (const auto& c : cands)
      if (c.find(key) != std::string::npos || editDistance(key, c) < (int)c.size() / 5 || endsWith(c, suffix(key)))
        return " (typo of " + go_quote(c) + "?)";
    uint64_t pr = rs_present(r);
    for (int k = 0; k < dims.NK; k++) {
      if (!bit(pr, k)) continue;
      const std::string& c = keyNames[k];
      if (c.find(key) != std::string::npos || editDistance(key, c) < (int)c.size() / 5 || endsWith(c, suffix(key)))
        return " (typo of " + go_quote(c) + "?)";
    }
    return "";
  };
  for (int k = 0; k < dims.NK; k++)
    if (bit(uf, k)) out.push_back("label " + go_quote(keyNames[k]) + " does not have known values" + hint(keyNames[k]));
  for (int k = 0; k < dims.NK; k++)
    if (bit(xf, k))
      out.push_back("key " + keyNames[k] + ", " + reqString(in, k, false, privateHost) + " not in " +
                    reqString(r, k, false, privateHost));
  return out;
}

}  // namespace ks
