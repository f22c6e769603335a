// cpu_ref.cpp — ORACLE (test infrastructure only; never linked into the product).
//
// A single-threaded CPU restatement of the Karpenter provisioning scheduler hot path, following the
// reference's own data structures (string-keyed maps and sets, k8s Quantities) so that it checks the
// MI355X product's bitset / fixed-point encoding independently.  Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may load it.
//
// Reference files restated (paths relative to /root/reference):
//   pkg/controllers/provisioning/scheduling/scheduler.go      (NewScheduler, Solve, add, limits)
//   pkg/controllers/provisioning/scheduling/queue.go          (Queue)
//   pkg/controllers/provisioning/scheduling/nodeclaim.go      (NodeClaim.Add, IT filter, FailureReason)
//   pkg/controllers/provisioning/scheduling/existingnode.go   (ExistingNode)
//   pkg/controllers/provisioning/scheduling/nodeclaimtemplate.go
//   pkg/controllers/provisioning/scheduling/preferences.go    (Relax)
//   pkg/scheduling/{requirement.go,requirements.go,taints.go,hostportusage.go}
//   pkg/utils/resources/resources.go, pkg/cloudprovider/types.go, pkg/apis/v1beta1/labels.go
//
// Go map-iteration-order choices are made canonically (sorted keys); see DESIGN.md §Parity.
#include <algorithm>
#include <cctype>
#include <chrono>
#include <atomic>
#include <thread>
#include <cmath>
#include <limits>
#include <memory>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "go_sort.h"
#include "json_min.h"
#include "quantity.h"

namespace oref {

using std::map;
using std::set;
using std::string;
using std::vector;
using oq::Quantity;
using ResourceList = map<string, Quantity>;

// ---------------------------------------------------------------------------------------------
// labels.go:57-100 (v1beta1) and k8s.io/api well-known label constants
// ---------------------------------------------------------------------------------------------
static const string kHostname = "kubernetes.io/hostname";
static const string kZone = "topology.kubernetes.io/zone";
static const string kCapacityType = "karpenter.sh/capacity-type";
static const string kNodePool = "karpenter.sh/nodepool";

static string normalizeKey(const string& key) {  // requirement.go:42-44, labels.go:94-100
  static const map<string, string> norm = {
      {"failure-domain.beta.kubernetes.io/zone", "topology.kubernetes.io/zone"},
      {"beta.kubernetes.io/arch", "kubernetes.io/arch"},
      {"beta.kubernetes.io/os", "kubernetes.io/os"},
      {"beta.kubernetes.io/instance-type", "node.kubernetes.io/instance-type"},
      {"failure-domain.beta.kubernetes.io/region", "topology.kubernetes.io/region"},
  };
  auto it = norm.find(key);
  return it == norm.end() ? key : it->second;
}

// strconv.Atoi (base 10, int64): optional sign, at least one digit, no other characters.
static bool goAtoi(const string& s, int64_t& out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
  if (i >= s.size()) return false;
  unsigned __int128 v = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
    if (v > (unsigned __int128)INT64_MAX + 1) return false;
  }
  if (!neg && v > (unsigned __int128)INT64_MAX) return false;
  out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
  return true;
}

static string goQuote(const string& s) {  // fmt %q for the ASCII keys used here
  string o = "\"";
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
    else if (c == '\n') o += "\\n";
    else if (c == '\t') o += "\\t";
    else if (c < 0x20 || c == 0x7f) { char b[8]; snprintf(b, sizeof b, "\\x%02x", c); o += b; }
    else o += (char)c;
  }
  return o + "\"";
}

// ---------------------------------------------------------------------------------------------
// requirement.go:33-280
// ---------------------------------------------------------------------------------------------
struct Requirement {
  string key;
  bool complement = false;
  set<string> values;
  bool hasGt = false, hasLt = false;
  int64_t gt = 0, lt = 0;
};

static bool withinIntPtrs(const string& v, bool hasGt, int64_t gt, bool hasLt, int64_t lt) {  // :238-254
  if (!hasGt && !hasLt) return true;
  int64_t x;
  if (!goAtoi(v, x)) return false;
  if (hasGt && gt >= x) return false;
  if (hasLt && lt <= x) return false;
  return true;
}

static Requirement NewRequirement(const string& key0, const string& op, const vector<string>& values) {  // :41-79
  Requirement r;
  r.key = normalizeKey(key0);
  if (op == "In") {
    r.values.insert(values.begin(), values.end());
    r.complement = false;
    return r;
  }
  r.complement = true;
  if (op == "In" || op == "DoesNotExist") r.complement = false;
  if (op == "In" || op == "NotIn") r.values.insert(values.begin(), values.end());
  if (op == "Gt") {
    int64_t v = 0;
    goAtoi(values.empty() ? "" : values[0], v);  // prevalidated; errors ignored -> 0
    r.hasGt = true; r.gt = v;
  }
  if (op == "Lt") {
    int64_t v = 0;
    goAtoi(values.empty() ? "" : values[0], v);
    r.hasLt = true; r.lt = v;
  }
  return r;
}

static int64_t Len(const Requirement& r) {  // :210-215
  if (r.complement) return INT64_MAX - (int64_t)r.values.size();
  return (int64_t)r.values.size();
}

static string Operator(const Requirement& r) {  // :197-208
  if (r.complement) return Len(r) < INT64_MAX ? "NotIn" : "Exists";
  return Len(r) > 0 ? "In" : "DoesNotExist";
}

static Requirement Intersection(const Requirement& r, const Requirement& q) {  // :128-161
  bool complement = r.complement && q.complement;
  bool hasGt = r.hasGt || q.hasGt;
  int64_t gt = r.hasGt && q.hasGt ? std::max(r.gt, q.gt) : (r.hasGt ? r.gt : q.gt);
  bool hasLt = r.hasLt || q.hasLt;
  int64_t lt = r.hasLt && q.hasLt ? std::min(r.lt, q.lt) : (r.hasLt ? r.lt : q.lt);
  if (hasGt && hasLt && gt >= lt) return NewRequirement(r.key, "DoesNotExist", {});
  set<string> values;
  if (r.complement && q.complement) {
    values = r.values;
    values.insert(q.values.begin(), q.values.end());
  } else if (r.complement && !q.complement) {
    for (auto& v : q.values) if (!r.values.count(v)) values.insert(v);
  } else if (!r.complement && q.complement) {
    for (auto& v : r.values) if (!q.values.count(v)) values.insert(v);
  } else {
    for (auto& v : r.values) if (q.values.count(v)) values.insert(v);
  }
  for (auto it = values.begin(); it != values.end();) {
    if (!withinIntPtrs(*it, hasGt, gt, hasLt, lt)) it = values.erase(it);
    else ++it;
  }
  if (!complement) { hasGt = hasLt = false; gt = lt = 0; }
  Requirement out;
  out.key = r.key;
  out.values = std::move(values);
  out.complement = complement;
  out.hasGt = hasGt; out.gt = gt;
  out.hasLt = hasLt; out.lt = lt;
  return out;
}

static bool Has(const Requirement& r, const string& v) {  // :182-187
  if (r.complement) return !r.values.count(v) && withinIntPtrs(v, r.hasGt, r.gt, r.hasLt, r.lt);
  return r.values.count(v) && withinIntPtrs(v, r.hasGt, r.gt, r.hasLt, r.lt);
}

static string joinVals(const vector<string>& v) {
  string s = "[";
  for (size_t i = 0; i < v.size(); i++) { if (i) s += " "; s += v[i]; }
  return s + "]";
}

static string String(const Requirement& r) {  // :217-236
  string op = Operator(r);
  string s;
  if (op == "Exists" || op == "DoesNotExist") {
    s = r.key + " " + op;
  } else {
    vector<string> values(r.values.begin(), r.values.end());  // sets.List: sorted
    if (values.size() > 5) {
      size_t n = values.size();
      values.resize(5);
      values.push_back("and " + std::to_string(n - 5) + " others");
    }
    s = r.key + " " + op + " " + joinVals(values);
  }
  if (r.hasGt) s += " >" + std::to_string(r.gt);
  if (r.hasLt) s += " <" + std::to_string(r.lt);
  return s;
}

// Untruncated canonical form used for result parity (String() truncates after 5 values).
static string FullString(const Requirement& r) {
  string op = Operator(r);
  string s = r.key + " " + op;
  if (op == "In" || op == "NotIn") s += " " + joinVals(vector<string>(r.values.begin(), r.values.end()));
  if (r.hasGt) s += " >" + std::to_string(r.gt);
  if (r.hasLt) s += " <" + std::to_string(r.lt);
  return s;
}

// ---------------------------------------------------------------------------------------------
// requirements.go:36-279
// ---------------------------------------------------------------------------------------------
using Errs = vector<string>;  // multierr: Error() joins with "; "
static string joinErrs(const Errs& e) {
  string s;
  for (size_t i = 0; i < e.size(); i++) { if (i) s += "; "; s += e[i]; }
  return s;
}

struct Requirements {
  map<string, Requirement> m;  // key -> requirement (iteration canonicalised to sorted key order)
  void Add(const Requirement& r) {  // :118-125
    auto it = m.find(r.key);
    if (it != m.end()) m[r.key] = Intersection(r, it->second);
    else m[r.key] = r;
  }
  void AddAll(const Requirements& o) { for (auto& kv : o.m) Add(kv.second); }
  bool Has(const string& k) const { return m.count(k) > 0; }
  Requirement Get(const string& k) const {  // :145-151
    auto it = m.find(k);
    if (it == m.end()) return NewRequirement(k, "Exists", {});
    return it->second;
  }
  string String() const {  // :272-279
    vector<string> parts;
    for (auto& kv : m) if (kv.first != kHostname) parts.push_back(oref::String(kv.second));
    std::sort(parts.begin(), parts.end());
    string s;
    for (size_t i = 0; i < parts.size(); i++) { if (i) s += ", "; s += parts[i]; }
    return s;
  }
};

static Requirements NewLabelRequirements(const map<string, string>& labels) {  // :56-62
  Requirements r;
  for (auto& kv : labels) r.Add(NewRequirement(kv.first, "In", {kv.second}));
  return r;
}

struct NSR { string key, op; vector<string> values; };
static Requirements NewNodeSelectorRequirements(const vector<NSR>& v) {  // :47-54
  Requirements r;
  for (auto& x : v) r.Add(NewRequirement(x.key, x.op, x.values));
  return r;
}

// editDistance (requirements.go:177-210), including its off-by-one loop bounds.
static int editDistance(const string& s, const string& t) {
  int m = (int)s.size(), n = (int)t.size();
  if (m == 0) return n;
  if (n == 0) return m;
  vector<int> prev(n, 0), cur(n, 0);
  for (int j = 1; j < n; j++) prev[j] = j;
  for (int i = 1; i < m; i++) {
    for (int j = 1; j < n; j++) {
      int diff = s[i] != t[j] ? 1 : 0;
      cur[j] = std::min(std::min(prev[j] + 1, cur[j - 1] + 1), prev[j - 1] + diff);
    }
    std::swap(prev, cur);
  }
  return prev[n - 1];
}

static string getSuffix(const string& key) {
  auto p = key.find('/');
  return p == string::npos ? key : key.substr(p + 1);
}
static bool hasSuffix(const string& s, const string& suf) {
  return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

static string labelHint(const Requirements& r, const string& key, const set<string>& allowed) {  // :220-238
  for (auto& wk : allowed) {
    if (wk.find(key) != string::npos || editDistance(key, wk) < (int)wk.size() / 5)
      return " (typo of " + goQuote(wk) + "?)";
    if (hasSuffix(wk, getSuffix(key))) return " (typo of " + goQuote(wk) + "?)";
  }
  for (auto& kv : r.m) {
    const string& ex = kv.first;
    if (ex.find(key) != string::npos || editDistance(key, ex) < (int)ex.size() / 5)
      return " (typo of " + goQuote(ex) + "?)";
    if (hasSuffix(ex, getSuffix(key))) return " (typo of " + goQuote(ex) + "?)";
  }
  return "";
}

static Errs Intersects(const Requirements& r, const Requirements& in) {  // :241-258
  Errs errs;
  for (auto& kv : r.m) {
    if (!in.Has(kv.first)) continue;
    const Requirement& existing = kv.second;
    Requirement incoming = in.Get(kv.first);
    if (Len(Intersection(existing, incoming)) == 0) {
      string io = Operator(incoming), eo = Operator(existing);
      if ((io == "NotIn" || io == "DoesNotExist") && (eo == "NotIn" || eo == "DoesNotExist")) continue;
      errs.push_back("key " + kv.first + ", " + String(incoming) + " not in " + String(existing));
    }
  }
  return errs;
}

static Errs Compatible(const Requirements& r, const Requirements& in, const set<string>* allowUndefined) {  // :163-174
  static const set<string> none;
  const set<string>& allowed = allowUndefined ? *allowUndefined : none;
  Errs errs;
  for (auto& kv : in.m) {
    if (allowed.count(kv.first)) continue;
    string op = Operator(kv.second);
    if (r.Has(kv.first) || op == "NotIn" || op == "DoesNotExist") continue;
    errs.push_back("label " + goQuote(kv.first) + " does not have known values" + labelHint(r, kv.first, allowed));
  }
  Errs e2 = Intersects(r, in);
  errs.insert(errs.end(), e2.begin(), e2.end());
  return errs;
}

// ---------------------------------------------------------------------------------------------
// k8s object model (subset of v1.Pod / v1.Taint / v1.Toleration fields on the path)
// ---------------------------------------------------------------------------------------------
struct Taint { string key, value, effect; };
struct Toleration { string key, op, value, effect; };

// k8s.io/api core/v1 toleration.go ToleratesTaint / MatchToleration (k8s.io/api v0.28.4, go.mod:24)
static bool ToleratesTaint(const Toleration& t, const Taint& taint) {
  if (!t.effect.empty() && t.effect != taint.effect) return false;
  if (!t.key.empty() && t.key != taint.key) return false;
  if (t.op.empty() || t.op == "Equal") return t.value == taint.value;
  if (t.op == "Exists") return true;
  return false;
}
static bool MatchToleration(const Toleration& a, const Toleration& b) {
  return a.key == b.key && a.effect == b.effect && a.op == b.op && a.value == b.value;
}

struct HostPort { string ip; int32_t port = 0; string proto; };
static bool ipUnspecified(const string& ip) { return ip == "0.0.0.0" || ip == "::" || ip == "0:0:0:0:0:0:0:0"; }
static bool HostPortMatches(const HostPort& p, const HostPort& q) {  // hostportusage.go:45-58
  if (p.proto != q.proto) return false;
  if (p.port != q.port) return false;
  if (p.ip != q.ip && !ipUnspecified(p.ip) && !ipUnspecified(q.ip)) return false;
  return true;
}

struct PreferredTerm { int32_t weight = 0; vector<NSR> exprs; };
struct Container { ResourceList requests, limits; vector<HostPort> ports; };

struct LabelSelectorReq { string key, op; vector<string> values; };
struct LabelSelector {
  bool present = false;           // nil selector: selects() matches nothing, TopologyListOptions lists everything
  vector<LabelSelectorReq> reqs;  // matchLabels (op "In", one value) then matchExpressions
};
struct PodAffinityTermS {
  LabelSelector selector;
  vector<string> namespaces;
  bool hasNamespaceSelector = false;
  LabelSelector namespaceSelector;
  string topologyKey;
};
struct TSCS {
  string key, when;
  int32_t maxSkew = 0;
  bool hasMinDomains = false;
  int32_t minDomains = 0;
  LabelSelector selector;
};

struct Pod {
  string name, ns, uid;
  map<string, string> labels;
  int64_t created = 0;
  string nodeName, phase, nominatedNodeName;
  bool failedToSchedule = false, ownedByDaemonSet = false, ownedByNode = false, deleting = false;
  bool notReady = false;  // a PodReady condition with status False (pdblimits.go:70-76)
  map<string, string> nodeSelector;
  bool hasAffinity = false, hasNodeAffinity = false, hasRequired = false;
  vector<vector<NSR>> requiredTerms;
  vector<PreferredTerm> preferred;
  bool hasPodAffinity = false, hasPodAnti = false;
  vector<PodAffinityTermS> affRequired, antiRequired;
  vector<std::pair<int32_t, PodAffinityTermS>> affPreferred, antiPreferred;
  vector<Toleration> tolerations;
  vector<Container> containers, initContainers;
  bool hasOverhead = false;
  ResourceList overhead;
  vector<TSCS> tsc;  // topologySpreadConstraints
  map<string, string> annotations;
  bool hasPriority = false;
  int32_t priority = 0;
  vector<string> pvcNames;  // spec.volumes: persistentVolumeClaim.claimName, or <pod>-<volume> for ephemeral
};

// pkg/utils/pod/scheduling.go:28-34
static bool IsProvisionable(const Pod& p) {
  return p.nodeName.empty() && p.nominatedNodeName.empty() && p.failedToSchedule && !p.ownedByDaemonSet &&
         !p.ownedByNode;
}

// ---------------------------------------------------------------------------------------------
// resources.go:27-175
// ---------------------------------------------------------------------------------------------
static void MergeInto(ResourceList& dest, const ResourceList& src) {
  for (auto& kv : src) {
    Quantity cur = dest.count(kv.first) ? dest[kv.first] : Quantity{};
    cur.add(kv.second);
    dest[kv.first] = cur;
  }
}
static ResourceList Merge(const vector<const ResourceList*>& lists) {
  ResourceList out;
  for (auto* l : lists) MergeInto(out, *l);
  return out;
}
static ResourceList MaxResources(const vector<const ResourceList*>& lists) {
  ResourceList out;
  for (auto* l : lists)
    for (auto& kv : *l) {
      auto it = out.find(kv.first);
      if (it == out.end() || kv.second.cmp(it->second) > 0) out[kv.first] = kv.second;
    }
  return out;
}
static ResourceList Subtract(const ResourceList& lhs, const ResourceList& rhs) {
  ResourceList out;
  for (auto& kv : lhs) {
    Quantity cur = kv.second;
    auto it = rhs.find(kv.first);
    if (it != rhs.end()) cur.sub(it->second);
    out[kv.first] = cur;
  }
  return out;
}
static ResourceList MergeLimitsIntoRequests(const Container& c) {
  ResourceList r = c.requests;
  for (auto& kv : c.limits) if (!r.count(kv.first)) r[kv.first] = kv.second;
  return r;
}
static ResourceList CeilingRequests(const Pod& p) {
  ResourceList req;
  for (auto& c : p.containers) MergeInto(req, MergeLimitsIntoRequests(c));
  for (auto& c : p.initContainers) {
    ResourceList m = MergeLimitsIntoRequests(c);
    req = MaxResources({&req, &m});
  }
  if (p.hasOverhead) MergeInto(req, p.overhead);
  return req;
}
static ResourceList RequestsForPods(const vector<const Pod*>& pods) {
  vector<ResourceList> each;
  for (auto* p : pods) each.push_back(CeilingRequests(*p));
  vector<const ResourceList*> ptrs;
  for (auto& e : each) ptrs.push_back(&e);
  ResourceList merged = Merge(ptrs);
  merged["pods"] = oq::make((int64_t)pods.size(), oq::Format::DecimalExponent);
  return merged;
}
static bool Fits(const ResourceList& cand, const ResourceList& total) {
  for (auto& kv : total) if (kv.second.sign() < 0) return false;
  for (auto& kv : cand) {
    auto it = total.find(kv.first);
    Quantity t = it == total.end() ? Quantity{} : it->second;
    if (kv.second.cmp(t) > 0) return false;
  }
  return true;
}
static string ResourcesString(const ResourceList& l) {  // resources.String -> pretty.Concise (json)
  if (l.empty()) return "{}";
  string s = "{";
  bool first = true;
  for (auto& kv : l) {
    if (!first) s += ",";
    first = false;
    ojson::quote(s, kv.first);
    s += ":";
    ojson::quote(s, kv.second.str());
  }
  return s + "}";
}

// ---------------------------------------------------------------------------------------------
// Pod requirements (requirements.go:56-109) — mutates preferred-term order like the reference.
// ---------------------------------------------------------------------------------------------
struct PrefSorter {
  vector<PreferredTerm>& v;
  bool less(int i, int j) { return v[i].weight > v[j].weight; }
  void swap(int i, int j) { std::swap(v[i], v[j]); }
};

static Requirements newPodRequirements(Pod& p, bool all) {
  Requirements r = NewLabelRequirements(p.nodeSelector);
  if (!p.hasAffinity || !p.hasNodeAffinity) return r;
  if (all && !p.preferred.empty()) {
    PrefSorter s{p.preferred};
    gosort::slice(s, (int)p.preferred.size());
    r.AddAll(NewNodeSelectorRequirements(p.preferred[0].exprs));
  }
  if (p.hasRequired && !p.requiredTerms.empty()) r.AddAll(NewNodeSelectorRequirements(p.requiredTerms[0]));
  return r;
}
static Requirements NewPodRequirements(Pod& p) { return newPodRequirements(p, true); }
static Requirements NewStrictPodRequirements(Pod& p) { return newPodRequirements(p, false); }
static bool HasPreferredNodeAffinity(const Pod& p) { return p.hasAffinity && p.hasNodeAffinity && !p.preferred.empty(); }

static Errs Tolerates(const vector<Taint>& taints, const Pod& p) {  // taints.go:38-50
  Errs errs;
  for (auto& t : taints) {
    bool ok = false;
    for (auto& tol : p.tolerations) ok = ok || ToleratesTaint(tol, t);
    if (!ok) errs.push_back("did not tolerate " + t.key + "=" + t.value + ":" + t.effect);
  }
  return errs;
}

static vector<HostPort> GetHostPorts(const Pod& p) {  // hostportusage.go:93-114
  vector<HostPort> out;
  for (auto& c : p.containers)
    for (auto& hp : c.ports) {
      if (hp.port == 0) continue;
      HostPort x = hp;
      if (x.ip.empty()) x.ip = "0.0.0.0";
      out.push_back(x);
    }
  return out;
}

static string HostPortString(const HostPort& p) {  // hostportusage.go:41-43
  return "IP=" + p.ip + " Port=" + std::to_string(p.port) + " Proto=" + p.proto;
}

struct HostPortUsage {
  map<string, vector<HostPort>> reserved;  // key: namespace/name
  bool Conflicts(const string& podKey, const vector<HostPort>& ports, string* msg = nullptr) const {
    for (auto& n : ports)
      for (auto& kv : reserved)
        for (auto& e : kv.second)
          if (HostPortMatches(n, e) && kv.first != podKey) {
            if (msg) *msg = HostPortString(n) + " conflicts with existing HostPort configuration " + HostPortString(e);
            return true;
          }
    return false;
  }
  void Add(const string& podKey, const vector<HostPort>& ports) { reserved[podKey] = ports; }
};

// ---------------------------------------------------------------------------------------------
// cloudprovider/types.go:83-166
// ---------------------------------------------------------------------------------------------
struct Offering { string capacityType, zone; double price = 0; bool available = true; };
struct InstanceType {
  string name;
  Requirements reqs;
  vector<Offering> offerings;
  ResourceList capacity, allocatable;
};

// ---------------------------------------------------------------------------------------------
// Problem snapshot (what NewScheduler receives)
// ---------------------------------------------------------------------------------------------
struct NodeClaimTemplate {  // nodeclaimtemplate.go:35-53
  string nodePoolName;
  Requirements reqs;
  vector<NSR> poolRequirements;       // NodePool spec.template.spec.requirements (topology domains)
  map<string, string> poolLabels;     // NodePool spec.template.metadata.labels (without karpenter.sh/nodepool)
  vector<Taint> taints;
  vector<int> instanceTypes;  // indices into Problem::its (the pool's GetInstanceTypes list)
};
struct NodePoolLimits { string name; bool hasLimits = false; ResourceList limits; bool preferNoSchedule = false; };
// VolumeUsage (volumeusage.go:183-227): driver -> unique PVC keys mounted, and per-driver limits
// (CSINode allocatable counts, cluster.go:468).
using Volumes = map<string, set<string>>;
struct VolumeUsage {
  Volumes volumes;
  map<string, int> limits;
  bool ExceedsLimits(const Volumes& add) const {  // volumeusage.go:202-209
    for (auto& kv : add) {
      auto l = limits.find(kv.first);
      if (l == limits.end()) continue;
      set<string> u = kv.second;
      auto e = volumes.find(kv.first);
      if (e != volumes.end()) u.insert(e->second.begin(), e->second.end());
      if ((int)u.size() > l->second) return true;
    }
    for (auto& kv : volumes) {  // drivers only the node mounts: the union is the node's own set
      if (add.count(kv.first)) continue;
      auto l = limits.find(kv.first);
      if (l != limits.end() && (int)kv.second.size() > l->second) return true;
    }
    return false;
  }
  void Add(const Volumes& v) {
    for (auto& kv : v) volumes[kv.first].insert(kv.second.begin(), kv.second.end());
  }
};
struct StateNodeSnap {
  string name, hostName;
  map<string, string> labels;
  vector<Taint> taints;
  ResourceList available, capacity, daemonSetRequests;
  bool initialized = true;
  HostPortUsage hostPorts;
  VolumeUsage volumes;
};
struct Problem {
  set<string> wellKnown;
  vector<InstanceType> its;
  vector<NodeClaimTemplate> templates;
  vector<NodePoolLimits> nodePools;
  vector<StateNodeSnap> nodes;
  vector<Pod> daemonSetPods;
  vector<Pod> pods;
  int64_t hostnameSeed = 0;
  bool emptyTopology = false;  // the benchmark's &scheduling.Topology{} (scheduling_benchmark_test.go:124)
  // cluster state the Topology counts (topology.go:190-291): bound pods and node labels by node name
  vector<Pod> clusterPods;
  map<string, map<string, string>> nodeLabels;
  vector<std::pair<string, map<string, string>>> namespaces;  // the cluster's Namespace list (name, labels)
  map<string, string> volumeDrivers;  // "ns/pvc" -> resolved CSI driver (resolveDriver, volumeusage.go:115-172)
  bool hasVolumeDrivers = false;      // the snapshot gave volumeDrivers (else resolved from the objects below)
  // the cluster's PersistentVolumeClaim / PersistentVolume / StorageClass objects (volumes.inc)
  bool volObjects = false;
  struct PVCObj { string volumeName, storageClass; };
  struct PVObj { string csiDriver; bool awsEBS = false, required = false; vector<vector<NSR>> terms; };
  struct SCObj { string provisioner; vector<vector<NSR>> allowedTopologies; };
  map<string, PVCObj> pvcs;  // "namespace/name"
  map<string, PVObj> pvs;
  map<string, SCObj> scs;
};

#include "volumes.inc"

// ---------------------------------------------------------------------------------------------
// JSON -> model
// ---------------------------------------------------------------------------------------------
static map<string, string> strMap(const ojson::Value* v) {
  map<string, string> m;
  if (v) for (auto& kv : v->obj()) m[kv.first] = kv.second.str();
  return m;
}
static ResourceList resList(const ojson::Value* v) {
  ResourceList r;
  if (v) for (auto& kv : v->obj()) r[kv.first] = oq::parse(kv.second.is_str() ? kv.second.s : kv.second.s);
  return r;
}
static vector<NSR> nsrList(const ojson::Value* v) {
  vector<NSR> out;
  if (!v) return out;
  for (auto& e : v->arr()) {
    NSR n;
    n.key = e.get("key") ? e.get("key")->str() : "";
    n.op = e.get("operator") ? e.get("operator")->str() : "";
    if (auto* vs = e.get("values")) for (auto& x : vs->arr()) n.values.push_back(x.str());
    out.push_back(n);
  }
  return out;
}
static vector<Taint> taintList(const ojson::Value* v) {
  vector<Taint> out;
  if (!v) return out;
  for (auto& e : v->arr()) {
    Taint t;
    if (auto* x = e.get("key")) t.key = x->str();
    if (auto* x = e.get("value")) t.value = x->str();
    if (auto* x = e.get("effect")) t.effect = x->str();
    out.push_back(t);
  }
  return out;
}
static int64_t parseTime(const string& s) {  // RFC3339 "YYYY-MM-DDTHH:MM:SSZ" -> unix seconds
  if (s.size() < 19) return 0;
  int Y = std::stoi(s.substr(0, 4)), M = std::stoi(s.substr(5, 2)), D = std::stoi(s.substr(8, 2));
  int h = std::stoi(s.substr(11, 2)), mi = std::stoi(s.substr(14, 2)), se = std::stoi(s.substr(17, 2));
  int y = Y - (M <= 2);
  int era = (y >= 0 ? y : y - 399) / 400;
  int yoe = y - era * 400;
  int doy = (153 * (M + (M > 2 ? -3 : 9)) + 2) / 5 + D - 1;
  int doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  int64_t days = (int64_t)era * 146097 + doe - 719468;
  return days * 86400 + h * 3600 + mi * 60 + se;
}
static Container parseContainer(const ojson::Value& c) {
  Container k;
  if (auto* r = c.get("resources")) {
    k.requests = resList(r->get("requests"));
    k.limits = resList(r->get("limits"));
  }
  if (auto* ps = c.get("ports"))
    for (auto& p : ps->arr()) {
      HostPort hp;
      hp.port = p.get("hostPort") ? (int32_t)p.get("hostPort")->i64() : 0;
      hp.ip = p.get("hostIP") ? p.get("hostIP")->str() : "";
      hp.proto = p.get("protocol") ? p.get("protocol")->str() : "";
      k.ports.push_back(hp);
    }
  return k;
}
static LabelSelector parseLabelSelector(const ojson::Value* v) {  // metav1.LabelSelector
  LabelSelector s;
  if (!v || v->is_null()) return s;
  s.present = true;
  for (auto& kv : strMap(v->get("matchLabels"))) s.reqs.push_back({kv.first, "In", {kv.second}});
  if (auto* es = v->get("matchExpressions"))
    for (auto& e : es->arr()) {
      LabelSelectorReq r;
      r.key = e.get("key") ? e.get("key")->str() : "";
      r.op = e.get("operator") ? e.get("operator")->str() : "";
      if (auto* vs = e.get("values")) for (auto& x : vs->arr()) r.values.push_back(x.str());
      s.reqs.push_back(r);
    }
  return s;
}

static PodAffinityTermS parseAffinityTerm(const ojson::Value& t) {
  PodAffinityTermS a;
  a.selector = parseLabelSelector(t.get("labelSelector"));
  if (auto* ns = t.get("namespaces")) for (auto& x : ns->arr()) a.namespaces.push_back(x.str());
  if (auto* nss = t.get("namespaceSelector"); nss && !nss->is_null()) {
    a.hasNamespaceSelector = true;
    a.namespaceSelector = parseLabelSelector(nss);
  }
  a.topologyKey = t.get("topologyKey") ? t.get("topologyKey")->str() : "";
  return a;
}

static Pod parsePod(const ojson::Value& v) {
  Pod p;
  const ojson::Value* md = v.get("metadata");
  if (md) {
    if (auto* x = md->get("name")) p.name = x->str();
    if (auto* x = md->get("namespace")) p.ns = x->str();
    if (auto* x = md->get("uid")) p.uid = x->str();
    p.labels = strMap(md->get("labels"));
    p.annotations = strMap(md->get("annotations"));
    if (auto* x = md->get("creationTimestamp")) p.created = parseTime(x->str());
    if (auto* x = md->get("deletionTimestamp")) p.deleting = !x->is_null();
    if (auto* ors = md->get("ownerReferences"))
      for (auto& o : ors->arr()) {
        string av = o.get("apiVersion") ? o.get("apiVersion")->str() : "";
        string kind = o.get("kind") ? o.get("kind")->str() : "";
        if (av == "apps/v1" && kind == "DaemonSet") p.ownedByDaemonSet = true;
        if (av == "v1" && kind == "Node") p.ownedByNode = true;
      }
  }
  const ojson::Value* sp = v.get("spec");
  if (sp) {
    if (auto* x = sp->get("nodeName")) p.nodeName = x->str();
    if (auto* x = sp->get("priority"); x && !x->is_null()) { p.hasPriority = true; p.priority = (int32_t)x->i64(); }
    p.nodeSelector = strMap(sp->get("nodeSelector"));
    if (auto* af = sp->get("affinity"); af && !af->is_null()) {
      p.hasAffinity = true;
      if (auto* na = af->get("nodeAffinity"); na && !na->is_null()) {
        p.hasNodeAffinity = true;
        if (auto* rq = na->get("requiredDuringSchedulingIgnoredDuringExecution"); rq && !rq->is_null()) {
          p.hasRequired = true;
          if (auto* ts = rq->get("nodeSelectorTerms"))
            for (auto& t : ts->arr()) p.requiredTerms.push_back(nsrList(t.get("matchExpressions")));
        }
        if (auto* pr = na->get("preferredDuringSchedulingIgnoredDuringExecution"))
          for (auto& t : pr->arr()) {
            PreferredTerm pt;
            pt.weight = t.get("weight") ? (int32_t)t.get("weight")->i64() : 0;
            if (auto* pf = t.get("preference")) pt.exprs = nsrList(pf->get("matchExpressions"));
            p.preferred.push_back(pt);
          }
      }
      for (int anti = 0; anti < 2; anti++) {
        auto* pa = af->get(anti ? "podAntiAffinity" : "podAffinity");
        if (!pa || pa->is_null()) continue;
        (anti ? p.hasPodAnti : p.hasPodAffinity) = true;
        if (auto* r = pa->get("requiredDuringSchedulingIgnoredDuringExecution"))
          for (auto& t : r->arr()) (anti ? p.antiRequired : p.affRequired).push_back(parseAffinityTerm(t));
        if (auto* r = pa->get("preferredDuringSchedulingIgnoredDuringExecution"))
          for (auto& t : r->arr())
            (anti ? p.antiPreferred : p.affPreferred)
                .push_back({t.get("weight") ? (int32_t)t.get("weight")->i64() : 0,
                            t.get("podAffinityTerm") ? parseAffinityTerm(*t.get("podAffinityTerm")) : PodAffinityTermS{}});
      }
    }
    if (auto* vs = sp->get("volumes"))  // volume.GetPersistentVolumeClaim (utils/volume/volume.go:29-38)
      for (auto& vol : vs->arr()) {
        const string vname = vol.get("name") ? vol.get("name")->str() : "";
        if (auto* pvc = vol.get("persistentVolumeClaim"); pvc && !pvc->is_null())
          p.pvcNames.push_back(pvc->get("claimName") ? pvc->get("claimName")->str() : "");
        else if (auto* eph = vol.get("ephemeral"); eph && !eph->is_null())
          p.pvcNames.push_back(p.name + "-" + vname);
      }
    if (auto* ts = sp->get("tolerations"))
      for (auto& t : ts->arr()) {
        Toleration tol;
        if (auto* x = t.get("key")) tol.key = x->str();
        if (auto* x = t.get("operator")) tol.op = x->str();
        if (auto* x = t.get("value")) tol.value = x->str();
        if (auto* x = t.get("effect")) tol.effect = x->str();
        p.tolerations.push_back(tol);
      }
    if (auto* cs = sp->get("containers")) for (auto& c : cs->arr()) p.containers.push_back(parseContainer(c));
    if (auto* cs = sp->get("initContainers")) for (auto& c : cs->arr()) p.initContainers.push_back(parseContainer(c));
    if (auto* oh = sp->get("overhead"); oh && !oh->is_null()) { p.hasOverhead = true; p.overhead = resList(oh); }
    if (auto* ts = sp->get("topologySpreadConstraints"))
      for (auto& t : ts->arr()) {
        TSCS c;
        c.key = t.get("topologyKey") ? t.get("topologyKey")->str() : "";
        c.when = t.get("whenUnsatisfiable") ? t.get("whenUnsatisfiable")->str() : "";
        c.maxSkew = t.get("maxSkew") ? (int32_t)t.get("maxSkew")->i64() : 0;
        if (auto* md = t.get("minDomains"); md && !md->is_null()) {
          c.hasMinDomains = true;
          c.minDomains = (int32_t)md->i64();
        }
        c.selector = parseLabelSelector(t.get("labelSelector"));
        p.tsc.push_back(c);
      }
  }
  if (auto* st = v.get("status")) {
    if (auto* x = st->get("phase")) p.phase = x->str();
    if (auto* x = st->get("nominatedNodeName")) p.nominatedNodeName = x->str();
    if (auto* cs = st->get("conditions"))
      for (auto& c : cs->arr())
      {
        if (c.get("type") && c.get("type")->str() == "PodScheduled" && c.get("reason") &&
            c.get("reason")->str() == "Unschedulable")
          p.failedToSchedule = true;
        if (c.get("type") && c.get("type")->str() == "Ready" && c.get("status") && c.get("status")->str() == "False")
          p.notReady = true;
      }
  }
  return p;
}

// NewNodeClaimTemplate (nodeclaimtemplate.go:43-53) from a NodePool object.
static NodeClaimTemplate templateFromNodePool(const ojson::Value& np) {
  NodeClaimTemplate t;
  const ojson::Value* md = np.get("metadata");
  t.nodePoolName = md && md->get("name") ? md->get("name")->str() : "";
  const ojson::Value* tpl = np.get("spec") ? np.get("spec")->get("template") : nullptr;
  map<string, string> labels;
  vector<NSR> reqs;
  if (tpl) {
    if (auto* tm = tpl->get("metadata")) labels = strMap(tm->get("labels"));
    if (auto* ts = tpl->get("spec")) {
      reqs = nsrList(ts->get("requirements"));
      t.taints = taintList(ts->get("taints"));
    }
  }
  t.poolRequirements = reqs;
  t.poolLabels = labels;
  labels[kNodePool] = t.nodePoolName;
  t.reqs = NewNodeSelectorRequirements(reqs);
  t.reqs.AddAll(NewLabelRequirements(labels));
  return t;
}

static Problem parseProblem(const ojson::Value& root) {
  Problem pb;
  if (auto* wk = root.get("wellKnownLabels")) for (auto& x : wk->arr()) pb.wellKnown.insert(x.str());
  else
    pb.wellKnown = {kNodePool, kZone, "topology.kubernetes.io/region", "node.kubernetes.io/instance-type",
                    "kubernetes.io/arch", "kubernetes.io/os", kCapacityType, "node.kubernetes.io/windows-build"};
  map<string, int> itIndex;
  if (auto* its = root.get("instanceTypes"))
    for (auto& v : its->arr()) {
      InstanceType it;
      it.name = v.get("name") ? v.get("name")->str() : "";
      it.reqs = NewNodeSelectorRequirements(nsrList(v.get("requirements")));
      if (auto* os = v.get("offerings"))
        for (auto& o : os->arr()) {
          Offering of;
          of.capacityType = o.get("capacityType") ? o.get("capacityType")->str() : "";
          of.zone = o.get("zone") ? o.get("zone")->str() : "";
          of.price = o.get("price") ? o.get("price")->f64() : 0;
          of.available = o.get("available") ? o.get("available")->boolean(true) : true;
          it.offerings.push_back(of);
        }
      it.capacity = resList(v.get("capacity"));
      ResourceList kr, sr, et;
      if (auto* oh = v.get("overhead")) {
        kr = resList(oh->get("kubeReserved"));
        sr = resList(oh->get("systemReserved"));
        et = resList(oh->get("evictionThreshold"));
      }
      ResourceList total = Merge({&kr, &sr, &et});
      it.allocatable = Subtract(it.capacity, total);  // types.go:100-110
      itIndex[it.name] = (int)pb.its.size();
      pb.its.push_back(std::move(it));
    }
  const ojson::Value* byPool = root.get("instanceTypesByNodePool");
  if (auto* ts = root.get("nodeClaimTemplates"))
    for (auto& v : ts->arr()) {
      NodeClaimTemplate t = templateFromNodePool(v);
      if (byPool && byPool->get(t.nodePoolName)) {
        for (auto& x : byPool->get(t.nodePoolName)->arr()) t.instanceTypes.push_back((int)x.i64());
      }
      pb.templates.push_back(std::move(t));
    }
  if (auto* ns = root.get("nodePools"))
    for (auto& v : ns->arr()) {
      NodePoolLimits l;
      l.name = v.get("metadata") && v.get("metadata")->get("name") ? v.get("metadata")->get("name")->str() : "";
      const ojson::Value* spec = v.get("spec");
      if (spec && spec->get("limits") && !spec->get("limits")->is_null()) {
        l.hasLimits = true;
        l.limits = resList(spec->get("limits"));
      }
      if (spec && spec->get("template") && spec->get("template")->get("spec"))
        for (auto& t : taintList(spec->get("template")->get("spec")->get("taints")))
          if (t.effect == "PreferNoSchedule") l.preferNoSchedule = true;
      pb.nodePools.push_back(l);
    }
  if (auto* ns = root.get("stateNodes"))
    for (auto& v : ns->arr()) {
      StateNodeSnap n;
      n.name = v.get("name") ? v.get("name")->str() : "";
      n.hostName = v.get("hostName") ? v.get("hostName")->str() : n.name;
      n.labels = strMap(v.get("labels"));
      n.taints = taintList(v.get("taints"));
      n.available = resList(v.get("available"));
      n.capacity = resList(v.get("capacity"));
      n.daemonSetRequests = resList(v.get("daemonSetRequests"));
      n.initialized = v.get("initialized") ? v.get("initialized")->boolean(true) : true;
      if (auto* vu = v.get("volumeUsage"))
        for (auto& kv : vu->obj())
          for (auto& x : kv.second.arr()) n.volumes.volumes[kv.first].insert(x.str());
      if (auto* vl = v.get("volumeLimits"))
        for (auto& kv : vl->obj()) n.volumes.limits[kv.first] = (int)kv.second.i64();
      if (auto* hp = v.get("hostPortUsage"))
        for (auto& kv : hp->obj()) {
          vector<HostPort> ports;
          for (auto& e : kv.second.arr()) {
            HostPort x;
            x.ip = e.get("ip") ? e.get("ip")->str() : "0.0.0.0";
            x.port = e.get("port") ? (int32_t)e.get("port")->i64() : 0;
            x.proto = e.get("protocol") ? e.get("protocol")->str() : "TCP";
            ports.push_back(x);
          }
          n.hostPorts.reserved[kv.first] = ports;
        }
      pb.nodes.push_back(std::move(n));
    }
  if (auto* ds = root.get("daemonSetPods")) for (auto& v : ds->arr()) pb.daemonSetPods.push_back(parsePod(v));
  if (auto* ps = root.get("pods")) for (auto& v : ps->arr()) pb.pods.push_back(parsePod(v));
  if (auto* hs = root.get("hostnameSeed")) pb.hostnameSeed = hs->i64();
  if (auto* et = root.get("emptyTopology")) pb.emptyTopology = et->boolean();
  if (auto* vd = root.get("volumeDrivers")) {
    pb.hasVolumeDrivers = true;
    for (auto& kv : vd->obj()) pb.volumeDrivers[kv.first] = kv.second.str();
  }
  parseVolumeObjects(root, pb);
  if (auto* cps = root.get("clusterPods")) for (auto& v : cps->arr()) pb.clusterPods.push_back(parsePod(v));
  if (auto* nss = root.get("namespaces"))
    for (auto& v : nss->arr()) {
      const ojson::Value* md = v.get("metadata") ? v.get("metadata") : &v;
      pb.namespaces.push_back({md->get("name") ? md->get("name")->str() : "", strMap(md->get("labels"))});
    }
  for (auto& n : pb.nodes) pb.nodeLabels[n.name] = n.labels;
  if (auto* cns = root.get("clusterNodes"))
    for (auto& v : cns->arr()) pb.nodeLabels[v.get("name") ? v.get("name")->str() : ""] = strMap(v.get("labels"));
  (void)itIndex;
  return pb;
}

#include "topology.inc"

// ---------------------------------------------------------------------------------------------
// Scheduler (scheduler.go, nodeclaim.go, existingnode.go, queue.go, preferences.go)
// ---------------------------------------------------------------------------------------------
struct NodeClaim {
  int tpl = -1;
  string hostname;
  Requirements reqs;
  vector<int> itOptions;  // indices into Problem::its, in InstanceTypeOptions order
  ResourceList requests, daemonResources;
  vector<int> pods;
  HostPortUsage hostPorts;
};

struct ExistingNode {
  int node = -1;
  vector<int> pods;
  ResourceList requests;
  Requirements reqs;
  HostPortUsage hostPorts;
  VolumeUsage volumes;
};

struct FilterResults {  // nodeclaim.go:144-160
  vector<int> remaining;
  bool requirementsMet = false, fits = false, hasOffering = false;
  bool requirementsAndFits = false, requirementsAndOffering = false, fitsAndOffering = false;
  ResourceList requests;
  string FailureReason() const {  // nodeclaim.go:165-221
    if (!remaining.empty()) return "";
    if (!requirementsMet && !fits && !hasOffering)
      return "no instance type met the scheduling requirements or had enough resources or had a required offering";
    if (!requirementsMet && !fits) return "no instance type met the scheduling requirements or had enough resources";
    if (!requirementsMet && !hasOffering) return "no instance type met the scheduling requirements or had a required offering";
    if (!fits && !hasOffering) return "no instance type had enough resources or had a required offering";
    if (!requirementsMet) return "no instance type met all requirements";
    if (!fits) {
      string msg = "no instance type has enough resources";
      auto it = requests.find("cpu");
      Quantity cpu = it == requests.end() ? Quantity{} : it->second;
      if (cpu.cmp(oq::parse("1M")) >= 0) msg += " (CPU request >= 1 Million, m vs M typo?)";
      return msg;
    }
    if (!hasOffering) return "no instance type has the required offering";
    if (requirementsAndFits)
      return "no instance type which met the scheduling requirements and had enough resources, had a required offering";
    if (fitsAndOffering)
      return "no instance type which had enough resources and the required offering met the scheduling requirements";
    if (requirementsAndOffering)
      return "no instance type which met the scheduling requirements and the required offering had the required resources";
    return "no instance type met the requirements/resources/offering tuple";
  }
};

struct Result {
  bool ok = true;
  Errs errs;
};

class Scheduler {
 public:
  explicit Scheduler(Problem& pb) : pb_(pb) {
    nodeID_ = pb.hostnameSeed;
    // Provisioner.NewScheduler: injectTopology before NewTopology (provisioner.go:283-287, 432-442)
    injectFailed_.assign(pb.pods.size(), false);
    for (size_t i = 0; i < pb.pods.size(); i++) injectFailed_[i] = !VolumeTopologyInject(pb, pb.pods[i]);
    buildTopology();
    initAlgBytes();
    // NewScheduler (scheduler.go:49-83)
    for (auto& np : pb.nodePools) if (np.preferNoSchedule) toleratePreferNoSchedule_ = true;
    for (size_t t = 0; t < pb.templates.size(); t++) {  // getDaemonOverhead :324-341
      vector<const Pod*> daemons;
      for (auto& d : pb.daemonSetPods) {
        Pod dp = d;
        if (!Tolerates(pb.templates[t].taints, dp).empty()) continue;
        if (!Compatible(pb.templates[t].reqs, NewPodRequirements(dp), &pb.wellKnown).empty()) continue;
        daemons.push_back(&d);
      }
      daemonOverhead_.push_back(RequestsForPods(daemons));
    }
    for (auto& np : pb.nodePools) remaining_[np.name] = np.hasLimits ? np.limits : ResourceList{};
    // calculateExistingNodeClaims :287-322
    for (size_t i = 0; i < pb.nodes.size(); i++) {
      auto& n = pb.nodes[i];
      vector<const Pod*> daemons;
      for (auto& d : pb.daemonSetPods) {
        Pod dp = d;
        if (!Tolerates(n.taints, dp).empty()) continue;
        if (!Compatible(NewLabelRequirements(n.labels), NewPodRequirements(dp), nullptr).empty()) continue;
        daemons.push_back(&d);
      }
      ResourceList dr = RequestsForPods(daemons);
      ExistingNode en;  // NewExistingNode existingnode.go:40-62
      en.node = (int)i;
      en.requests = Subtract(dr, n.daemonSetRequests);
      for (auto& kv : en.requests)
        if (kv.second.sign() < 0) kv.second.nano = 0;  // v.Set(0): value 0, format kept
      en.reqs = NewLabelRequirements(n.labels);
      en.reqs.Add(NewRequirement(kHostname, "In", {n.hostName}));
      en.hostPorts = n.hostPorts;
      en.volumes = n.volumes;
      topo_.Register(kHostname, n.hostName);  // NewExistingNode (existingnode.go:60)
      existing_.push_back(std::move(en));
      auto lp = n.labels.find(kNodePool);
      string pool = lp == n.labels.end() ? "" : lp->second;
      if (remaining_.count(pool)) remaining_[pool] = Subtract(remaining_[pool], n.capacity);
    }
    std::stable_sort(existing_.begin(), existing_.end(), [&](const ExistingNode& a, const ExistingNode& b) {
      bool ia = pb_.nodes[a.node].initialized, ib = pb_.nodes[b.node].initialized;
      if (ia && !ib) return true;
      if (!ia && ib) return false;
      return pb_.nodes[a.node].name < pb_.nodes[b.node].name;
    });
  }

  // Solve (scheduler.go:140-189)
  void Solve() {
    vector<int> q(pb_.pods.size());
    for (size_t i = 0; i < q.size(); i++) q[i] = (int)i;
    reqsCache_.resize(pb_.pods.size());
    for (size_t i = 0; i < q.size(); i++) reqsCache_[i] = CeilingRequestsFor((int)i);
    // NewQueue: sort.Slice(pods, byCPUAndMemoryDescending) (queue.go:37-43,83-112)
    struct QS {
      Scheduler* s;
      vector<int>& q;
      bool less(int i, int j) { return s->byCPUAndMemoryDescending(q[i], q[j]); }
      void swap(int i, int j) { std::swap(q[i], q[j]); }
    } qs{this, q};
    gosort::slice(qs, (int)q.size());
    queue_ = q;
    head_ = 0;
    errors_.assign(pb_.pods.size(), Result{});
    attempted_.assign(pb_.pods.size(), false);
    relaxCount_.assign(pb_.pods.size(), 0);
    for (;;) {
      int p;
      if (!Pop(p)) break;
      attempted_[p] = true;
      errors_[p] = add(p);
      if (errors_[p].ok) continue;
      bool relaxed = Relax(pb_.pods[p]);
      if (relaxed) relaxCount_[p]++;
      Push(p, relaxed);
      if (relaxed && !pb_.emptyTopology) topo_.Update(pb_.pods[p]);
    }
    for (auto& nc : claims_) nc.reqs.m.erase(kHostname);  // FinalizeScheduling nodeclaim.go:123-128
  }

  string ResultsJSON() const;

  // Results accessors for the consolidation restatement (read after Solve)
  int numNewNodeClaims() const { return (int)order_.size(); }
  const NodeClaim& newNodeClaim(int k) const { return claims_[order_[k]]; }
  const vector<ExistingNode>& existingNodes() const { return existing_; }
  bool podError(int p) const { return attempted_[p] && !errors_[p].ok; }
  int64_t nodeIDCounter() const { return nodeID_; }
  // Relax calls that changed pod p's spec in this Solve (Preferences.Relax mutates the *v1.Pod in place,
  // preferences.go:38-147; the consolidation restatement carries such pods into the next probe)
  int relaxCount(int p) const { return relaxCount_[p]; }

  long long attempts = 0;  // statistics: NodeClaim.Add calls
  int64_t algBytes() const { return algBytes_; }

 private:
  Problem& pb_;
  Topology topo_;

  // Provisioner.NewScheduler -> NewTopology (provisioner.go:229-287, topology.go:61-85)
  void buildTopology() {
    if (pb_.emptyTopology) return;  // no groups: AddRequirements / Record are no-ops
    topo_.domains = topologyDomains(pb_);
    topo_.clusterPods = &pb_.clusterPods;
    topo_.nodes = &pb_.nodeLabels;
    topo_.namespaceList = &pb_.namespaces;
    // the pods NewTopology receives: those whose volume topology injection succeeded
    for (size_t i = 0; i < pb_.pods.size(); i++)
      if (!injectFailed_[i]) topo_.excluded.insert(pb_.pods[i].uid);
    for (auto& cp : pb_.clusterPods) {  // updateInverseAffinities via ForPodsWithAntiAffinity
      if (!(cp.hasAffinity && cp.hasPodAnti && !cp.antiRequired.empty())) continue;
      if (cp.nodeName.empty()) continue;
      auto n = pb_.nodeLabels.find(cp.nodeName);
      if (n == pb_.nodeLabels.end()) continue;
      if (topo_.excluded.count(cp.uid)) continue;
      topo_.inverseAnti(cp, &n->second);
    }
    for (size_t i = 0; i < pb_.pods.size(); i++)
      if (!injectFailed_[i]) topo_.Update(pb_.pods[i]);
  }
  vector<bool> injectFailed_;
  int64_t nodeID_ = 0;
  bool toleratePreferNoSchedule_ = false;
  vector<ResourceList> daemonOverhead_;
  map<string, ResourceList> remaining_;
  vector<ExistingNode> existing_;
  vector<NodeClaim> claims_;
  vector<int> order_;  // s.newNodeClaims as indices into claims_
  vector<int> queue_;
  size_t head_ = 0;
  map<string, int> lastLen_;
  vector<Result> errors_;
  vector<bool> attempted_;
  vector<int> relaxCount_;
  vector<ResourceList> reqsCache_;

  ResourceList CeilingRequestsFor(int p) { return RequestsForPods({&pb_.pods[p]}); }

  // SURVEY.md §8d algorithmic bytes: the bytes of every candidate the reference scans per pod step, in a
  // fixed-width encoding (R int64 resource vectors, W 32-bit requirement words per object with
  // W = sum over its keys of ceil((|V_key| + 1) / 32) + 1, a T-bit instance-type set):
  //   existing node tried   16R + 4W_node + 8 per topology group evaluated
  //   NodeClaim tried       16R + 4W_claim + T/8 (+ per remaining instance type scanned 8R + 4W_it + 4)
  //   commit                 8R + 4W + T/8
  // A measurement of this restatement (test infrastructure), not part of the reference.
  int64_t algBytes_ = 0;
  int64_t R_ = 0, T8_ = 0;
  map<string, int64_t> keyWords_;
  vector<int64_t> itW_;
  void initAlgBytes() {
    map<string, set<string>> uni;
    set<string> res;
    auto addReqs = [&](const Requirements& r) {
      for (auto& kv : r.m) for (auto& v : kv.second.values) uni[kv.first].insert(v);
      for (auto& kv : r.m) uni[kv.first];
    };
    for (auto& it : pb_.its) {
      addReqs(it.reqs);
      for (auto& kv : it.allocatable) res.insert(kv.first);
    }
    for (auto& t : pb_.templates) addReqs(t.reqs);
    for (auto& n : pb_.nodes) for (auto& kv : n.labels) uni[kv.first].insert(kv.second);
    for (auto& p : pb_.pods) {
      Pod cp = p;
      addReqs(NewPodRequirements(cp));
      for (auto& kv : RequestsForPods({&p})) res.insert(kv.first);
    }
    for (auto& kv : uni) keyWords_[kv.first] = ((int64_t)kv.second.size() + 1 + 31) / 32 + 1;
    R_ = (int64_t)res.size();
    T8_ = ((int64_t)pb_.its.size() + 7) / 8;
    for (auto& it : pb_.its) itW_.push_back(W(it.reqs));
  }
  int64_t W(const Requirements& r) const {
    int64_t w = 0;
    for (auto& kv : r.m) {
      auto k = keyWords_.find(kv.first);
      w += k == keyWords_.end() ? 2 : k->second;
    }
    return w;
  }

  bool byCPUAndMemoryDescending(int a, int b) {  // queue.go:83-112
    const ResourceList& l = reqsCache_[a];
    const ResourceList& r = reqsCache_[b];
    auto get = [](const ResourceList& x, const char* k) {
      auto it = x.find(k);
      return it == x.end() ? Quantity{} : it->second;
    };
    int c = get(l, "cpu").cmp(get(r, "cpu"));
    if (c < 0) return false;
    if (c > 0) return true;
    int m = get(l, "memory").cmp(get(r, "memory"));
    if (m < 0) return false;
    if (m > 0) return true;
    const Pod& lp = pb_.pods[a];
    const Pod& rp = pb_.pods[b];
    if (lp.created != rp.created) return lp.created < rp.created;
    return lp.uid < rp.uid;
  }

  bool Pop(int& p) {  // queue.go:46-61
    size_t len = queue_.size() - head_;
    if (len == 0) return false;
    p = queue_[head_];
    auto it = lastLen_.find(pb_.pods[p].uid);
    if (it != lastLen_.end() && it->second == (int)len) return false;
    head_++;
    return true;
  }
  void Push(int p, bool relaxed) {  // queue.go:64-71
    queue_.push_back(p);
    if (relaxed) lastLen_.clear();
    else lastLen_[pb_.pods[p].uid] = (int)(queue_.size() - head_);
  }

  // Preferences.Relax (preferences.go:38-147)
  bool Relax(Pod& pod) {
    // removeRequiredNodeAffinityTerm
    if (pod.hasAffinity && pod.hasNodeAffinity && pod.hasRequired && pod.requiredTerms.size() > 1) {
      pod.requiredTerms.erase(pod.requiredTerms.begin());
      return true;
    }
    // removePreferredPodAffinityTerm (SliceStable by weight desc, drop first)
    auto byWeight = [](const std::pair<int32_t, PodAffinityTermS>& a, const std::pair<int32_t, PodAffinityTermS>& b) {
      return a.first > b.first;
    };
    if (pod.hasAffinity && pod.hasPodAffinity && !pod.affPreferred.empty()) {
      std::stable_sort(pod.affPreferred.begin(), pod.affPreferred.end(), byWeight);
      pod.affPreferred.erase(pod.affPreferred.begin());
      return true;
    }
    if (pod.hasAffinity && pod.hasPodAnti && !pod.antiPreferred.empty()) {
      std::stable_sort(pod.antiPreferred.begin(), pod.antiPreferred.end(), byWeight);
      pod.antiPreferred.erase(pod.antiPreferred.begin());
      return true;
    }
    // removePreferredNodeAffinityTerm
    if (pod.hasAffinity && pod.hasNodeAffinity && !pod.preferred.empty()) {
      std::stable_sort(pod.preferred.begin(), pod.preferred.end(),
                       [](const PreferredTerm& a, const PreferredTerm& b) { return a.weight > b.weight; });
      pod.preferred.erase(pod.preferred.begin());
      return true;
    }
    // removeTopologySpreadScheduleAnyway: swap-with-last then truncate
    for (size_t i = 0; i < pod.tsc.size(); i++) {
      if (pod.tsc[i].when == "ScheduleAnyway") {
        pod.tsc[i] = pod.tsc.back();
        pod.tsc.pop_back();
        return true;
      }
    }
    if (toleratePreferNoSchedule_) {
      Toleration t{"", "Exists", "", "PreferNoSchedule"};
      for (auto& x : pod.tolerations) if (MatchToleration(x, t)) return false;
      pod.tolerations.push_back(t);
      return true;
    }
    return false;
  }

  // ExistingNode.Add (existingnode.go:64-124); returns true on success (errors are discarded by add()).
  bool existingAdd(ExistingNode& n, int p) {
    Pod& pod = pb_.pods[p];
    const StateNodeSnap& sn = pb_.nodes[n.node];
    algBytes_ += 16 * R_ + 4 * W(n.reqs);
    const int64_t applied0 = topo_.applied;
    struct Touch {  // the topology groups AddRequirements evaluated, however the attempt ends
      Scheduler* s;
      int64_t a0;
      ~Touch() { s->algBytes_ += 8 * (s->topo_.applied - a0); }
    } touch{this, applied0};
    if (!Tolerates(sn.taints, pod).empty()) return false;
    vector<HostPort> hp = GetHostPorts(pod);
    string key = pod.ns + "/" + pod.name;
    bool volErr = false;
    Volumes vols = GetVolumes(pb_, pod, &volErr);
    if (volErr) return false;                         // existingnode.go:70-73
    if (n.volumes.ExceedsLimits(vols)) return false;  // existingnode.go:76-78
    if (n.hostPorts.Conflicts(key, hp)) return false;
    ResourceList podReq = RequestsForPods({&pod});
    ResourceList requests = Merge({&n.requests, &podReq});
    if (!Fits(requests, sn.available)) return false;
    Requirements nodeReqs = n.reqs;
    Requirements podReqs = NewPodRequirements(pod);
    if (!Compatible(nodeReqs, podReqs, nullptr).empty()) return false;
    nodeReqs.AddAll(podReqs);
    Requirements strict = HasPreferredNodeAffinity(pod) ? NewStrictPodRequirements(pod) : podReqs;
    Requirements topoReqs;
    string terr;
    if (!topo_.AddRequirements(strict, nodeReqs, pod, nullptr, topoReqs, terr)) return false;
    if (!Compatible(nodeReqs, topoReqs, nullptr).empty()) return false;
    nodeReqs.AddAll(topoReqs);
    n.pods.push_back(p);
    n.requests = requests;
    n.reqs = nodeReqs;
    algBytes_ += 8 * R_ + 4 * W(nodeReqs) + T8_;
    topo_.Record(pod, nodeReqs, nullptr);
    n.hostPorts.Add(key, hp);
    n.volumes.Add(vols);  // existingnode.go:122
    return true;
  }

  FilterResults filterInstanceTypes(const vector<int>& its, const Requirements& reqs, const ResourceList& requests) {
    FilterResults r;  // nodeclaim.go:225-260
    r.requests = requests;
    for (int i : its) {
      const InstanceType& it = pb_.its[i];
      bool itCompat = Intersects(it.reqs, reqs).empty();
      bool itFits = Fits(requests, it.allocatable);
      bool itOff = false;
      for (auto& o : it.offerings) {  // hasOffering :270-278
        if (!o.available) continue;
        if ((!reqs.Has(kZone) || Has(reqs.Get(kZone), o.zone)) &&
            (!reqs.Has(kCapacityType) || Has(reqs.Get(kCapacityType), o.capacityType))) {
          itOff = true;
          break;
        }
      }
      r.requirementsMet = r.requirementsMet || itCompat;
      r.fits = r.fits || itFits;
      r.hasOffering = r.hasOffering || itOff;
      r.requirementsAndFits = r.requirementsAndFits || (itCompat && itFits && !itOff);
      r.requirementsAndOffering = r.requirementsAndOffering || (itCompat && itOff && !itFits);
      r.fitsAndOffering = r.fitsAndOffering || (itFits && itOff && !itCompat);
      if (itCompat && itFits && itOff) r.remaining.push_back(i);
    }
    return r;
  }

  // NodeClaim.Add (nodeclaim.go:65-119)
  Result claimAdd(NodeClaim& n, int p) {
    attempts++;
    Pod& pod = pb_.pods[p];
    Result res;
    algBytes_ += 16 * R_ + 4 * W(n.reqs) + T8_;
    struct Touch {
      Scheduler* s;
      int64_t a0;
      ~Touch() { s->algBytes_ += 8 * (s->topo_.applied - a0); }
    } touch{this, topo_.applied};
    Errs te = Tolerates(pb_.templates[n.tpl].taints, pod);
    if (!te.empty()) { res.ok = false; res.errs = {joinErrs(te)}; return res; }
    vector<HostPort> hp = GetHostPorts(pod);
    string key = pod.ns + "/" + pod.name;
    string conflict;
    if (n.hostPorts.Conflicts(key, hp, &conflict)) {
      res.ok = false;
      res.errs = {"checking host port usage, " + conflict};
      return res;
    }
    Requirements ncReqs = n.reqs;
    Requirements podReqs = NewPodRequirements(pod);
    Errs ce = Compatible(ncReqs, podReqs, &pb_.wellKnown);
    if (!ce.empty()) { res.ok = false; res.errs = {"incompatible requirements, " + joinErrs(ce)}; return res; }
    ncReqs.AddAll(podReqs);
    Requirements strict = HasPreferredNodeAffinity(pod) ? NewStrictPodRequirements(pod) : podReqs;
    Requirements topoReqs;
    string terr;
    if (!topo_.AddRequirements(strict, ncReqs, pod, &pb_.wellKnown, topoReqs, terr)) {
      res.ok = false;
      res.errs = {terr};
      return res;
    }
    Errs te2 = Compatible(ncReqs, topoReqs, &pb_.wellKnown);
    if (!te2.empty()) { res.ok = false; res.errs = te2; return res; }
    ncReqs.AddAll(topoReqs);
    ResourceList podReq = RequestsForPods({&pod});
    ResourceList requests = Merge({&n.requests, &podReq});
    FilterResults f = filterInstanceTypes(n.itOptions, ncReqs, requests);
    for (int i : n.itOptions) algBytes_ += 8 * R_ + 4 * itW_[(size_t)i] + 4;
    if (f.remaining.empty()) {
      ResourceList cum = Merge({&n.daemonResources, &podReq});
      res.ok = false;
      res.errs = {"no instance type satisfied resources " + ResourcesString(cum) + " and requirements " +
                  ncReqs.String() + " (" + f.FailureReason() + ")"};
      return res;
    }
    n.pods.push_back(p);
    n.itOptions = f.remaining;
    n.requests = requests;
    n.reqs = ncReqs;
    algBytes_ += 8 * R_ + 4 * W(ncReqs) + T8_;
    topo_.Record(pod, ncReqs, &pb_.wellKnown);
    n.hostPorts.Add(key, hp);
    return res;
  }

  // Scheduler.add (scheduler.go:238-285)
  Result add(int p) {
    for (auto& n : existing_)
      if (existingAdd(n, p)) return Result{};
    struct CS {
      Scheduler* s;
      bool less(int i, int j) { return s->claims_[s->order_[i]].pods.size() < s->claims_[s->order_[j]].pods.size(); }
      void swap(int i, int j) { std::swap(s->order_[i], s->order_[j]); }
    } cs{this};
    gosort::slice(cs, (int)order_.size());
    for (int c : order_)
      if (claimAdd(claims_[c], p).ok) return Result{};
    Result res;
    res.ok = true;
    for (size_t t = 0; t < pb_.templates.size(); t++) {
      const NodeClaimTemplate& tpl = pb_.templates[t];
      vector<int> its = tpl.instanceTypes;
      auto rit = remaining_.find(tpl.nodePoolName);
      if (rit != remaining_.end()) {  // filterByRemainingResources :364-383
        vector<int> filtered;
        for (int i : its) {
          bool viable = true;
          for (auto& kv : rit->second) {
            auto c = pb_.its[i].capacity.find(kv.first);
            Quantity cq = c == pb_.its[i].capacity.end() ? Quantity{} : c->second;
            if (cq.cmp(kv.second) > 0) viable = false;
          }
          if (viable) filtered.push_back(i);
        }
        if (filtered.empty()) {
          res.ok = false;
          res.errs.push_back("all available instance types exceed limits for nodepool: " + goQuote(tpl.nodePoolName));
          continue;
        }
        its = filtered;
      }
      // NewNodeClaim (nodeclaim.go:46-63)
      NodeClaim nc;
      nc.tpl = (int)t;
      char hb[64];
      snprintf(hb, sizeof hb, "hostname-placeholder-%04lld", (long long)(++nodeID_));
      nc.hostname = hb;
      topo_.Register(kHostname, nc.hostname);
      nc.reqs = tpl.reqs;
      nc.reqs.Add(NewRequirement(kHostname, "In", {nc.hostname}));
      nc.itOptions = its;
      nc.requests = daemonOverhead_[t];
      nc.daemonResources = daemonOverhead_[t];
      Result r = claimAdd(nc, p);
      if (!r.ok) {
        res.ok = false;
        res.errs.push_back("incompatible with nodepool " + goQuote(tpl.nodePoolName) +
                           ", daemonset overhead=" + ResourcesString(daemonOverhead_[t]) + ", " + joinErrs(r.errs));
        continue;
      }
      claims_.push_back(std::move(nc));
      order_.push_back((int)claims_.size() - 1);
      if (rit != remaining_.end()) {  // subtractMax :347-362
        NodeClaim& c = claims_.back();
        vector<const ResourceList*> caps;
        for (int i : c.itOptions) caps.push_back(&pb_.its[i].capacity);
        ResourceList mx = MaxResources(caps);
        ResourceList out;
        for (auto& kv : rit->second) {
          Quantity cp = kv.second;
          auto m = mx.find(kv.first);
          cp.sub(m == mx.end() ? Quantity{} : m->second);
          out[kv.first] = cp;
        }
        rit->second = out;
      }
      return Result{};
    }
    return res;
  }
};

string Scheduler::ResultsJSON() const {
  string o = "{\"newNodeClaims\":[";
  for (size_t k = 0; k < order_.size(); k++) {
    const NodeClaim& c = claims_[order_[k]];
    if (k) o += ",";
    o += "{\"nodePoolName\":";
    ojson::quote(o, pb_.templates[c.tpl].nodePoolName);
    o += ",\"hostname\":";
    ojson::quote(o, c.hostname);
    o += ",\"pods\":[";
    for (size_t i = 0; i < c.pods.size(); i++) o += (i ? "," : "") + std::to_string(c.pods[i]);
    o += "],\"instanceTypeOptions\":[";
    for (size_t i = 0; i < c.itOptions.size(); i++) {
      if (i) o += ",";
      ojson::quote(o, pb_.its[c.itOptions[i]].name);
    }
    o += "],\"requests\":{";
    bool first = true;
    for (auto& kv : c.requests) {
      if (!first) o += ",";
      first = false;
      ojson::quote(o, kv.first);
      o += ":";
      ojson::quote(o, kv.second.str());
    }
    o += "},\"requirements\":[";
    first = true;
    for (auto& kv : c.reqs.m) {
      if (!first) o += ",";
      first = false;
      ojson::quote(o, FullString(kv.second));
    }
    o += "],\"requirementsString\":";
    ojson::quote(o, c.reqs.String());
    // NodeClaimTemplate.ToNodeClaim (nodeclaimtemplate.go:55-60): the launch list is
    // InstanceTypeOptions.OrderByPrice(Requirements) (types.go:62-79) cut to its first 100 entries;
    // an option's price is its cheapest available offering the zone / capacity-type requirements
    // allow (Offerings.Available().Requirements(reqs).Cheapest(), types.go:147-166), else MaxFloat64.
    vector<std::pair<double, string>> launch;
    const Requirement zone = c.reqs.Get(kZone), ct = c.reqs.Get(kCapacityType);
    for (int it : c.itOptions) {
      double price = std::numeric_limits<double>::max();
      bool any = false;
      for (auto& of : pb_.its[it].offerings) {
        if (!of.available || !Has(zone, of.zone) || !Has(ct, of.capacityType)) continue;
        if (!any || of.price < price) price = of.price;
        any = true;
      }
      launch.push_back({price, pb_.its[it].name});
    }
    std::sort(launch.begin(), launch.end());  // price, then name (names are unique)
    o += ",\"launchInstanceTypes\":[";
    for (size_t i = 0; i < launch.size() && i < 100; i++) {
      if (i) o += ",";
      ojson::quote(o, launch[i].second);
    }
    o += "]}";
  }
  o += "],\"existingNodes\":[";
  for (size_t k = 0; k < existing_.size(); k++) {
    const ExistingNode& n = existing_[k];
    if (k) o += ",";
    o += "{\"name\":";
    ojson::quote(o, pb_.nodes[n.node].name);
    o += ",\"pods\":[";
    for (size_t i = 0; i < n.pods.size(); i++) o += (i ? "," : "") + std::to_string(n.pods[i]);
    o += "]}";
  }
  o += "],\"podErrors\":{";
  bool first = true;
  for (size_t p = 0; p < errors_.size(); p++) {
    if (!attempted_[p] || errors_[p].ok) continue;
    if (!first) o += ",";
    first = false;
    ojson::quote(o, std::to_string(p));
    o += ":";
    ojson::quote(o, joinErrs(errors_[p].errs));
  }
  o += "},\"stats\":{\"claimAddCalls\":" + std::to_string(attempts) + ",\"algBytesRef\":" + std::to_string(algBytes_) + "}}";
  return o;
}

#include "consolidation.inc"
#include "cluster_state.inc"

// ---------------------------------------------------------------------------------------------
// Requirement-algebra evaluator for the reference's golden vectors (requirement_test.go,
// requirements_test.go).  Input: {"ops":[{"op":..., ...}]}; output {"results":[...]}.
// ---------------------------------------------------------------------------------------------
static Requirement reqFromJson(const ojson::Value& v) {
  vector<string> vals;
  if (auto* vs = v.get("values")) for (auto& x : vs->arr()) vals.push_back(x.str());
  return NewRequirement(v.get("key") ? v.get("key")->str() : "key", v.get("operator")->str(), vals);
}
static Requirements reqsFromJson(const ojson::Value& v) {
  Requirements r;
  for (auto& e : v.arr()) r.Add(reqFromJson(e));
  return r;
}
static string reqStructJson(const Requirement& r) {
  string o = "{\"key\":";
  ojson::quote(o, r.key);
  o += ",\"complement\":" + string(r.complement ? "true" : "false") + ",\"values\":[";
  bool first = true;
  for (auto& v : r.values) { if (!first) o += ","; first = false; ojson::quote(o, v); }
  o += "]";
  if (r.hasGt) o += ",\"gt\":" + std::to_string(r.gt);
  if (r.hasLt) o += ",\"lt\":" + std::to_string(r.lt);
  return o + "}";
}

static string evalOps(const ojson::Value& root, const set<string>& wellKnown) {
  string o = "{\"results\":[";
  bool first = true;
  for (auto& op : root.get("ops")->arr()) {
    if (!first) o += ",";
    first = false;
    string kind = op.get("op")->str();
    if (kind == "intersection") {
      o += reqStructJson(Intersection(reqFromJson(*op.get("a")), reqFromJson(*op.get("b"))));
    } else if (kind == "has") {
      o += Has(reqFromJson(*op.get("a")), op.get("value")->str()) ? "true" : "false";
    } else if (kind == "operator") {
      ojson::quote(o, Operator(reqFromJson(*op.get("a"))));
    } else if (kind == "len") {
      o += std::to_string(Len(reqFromJson(*op.get("a"))));
    } else if (kind == "string") {
      ojson::quote(o, String(reqFromJson(*op.get("a"))));
    } else if (kind == "intersection_string") {
      ojson::quote(o, String(Intersection(reqFromJson(*op.get("a")), reqFromJson(*op.get("b")))));
    } else if (kind == "compatible") {
      bool loose = op.get("allowUndefinedWellKnown") && op.get("allowUndefinedWellKnown")->boolean();
      Errs e = Compatible(reqsFromJson(*op.get("a")), reqsFromJson(*op.get("b")), loose ? &wellKnown : nullptr);
      o += "{\"ok\":" + string(e.empty() ? "true" : "false") + ",\"error\":";
      ojson::quote(o, joinErrs(e));
      o += "}";
    } else if (kind == "reqs_string") {
      ojson::quote(o, reqsFromJson(*op.get("a")).String());
    } else if (kind == "quantity") {
      ojson::quote(o, oq::parse(op.get("value")->str()).str());
    } else if (kind == "quantity_add") {
      Quantity a = oq::parse(op.get("a")->str());
      a.add(oq::parse(op.get("b")->str()));
      ojson::quote(o, a.str());
    } else {
      o += "null";
    }
  }
  return o + "]}";
}

}  // namespace oref

// ---------------------------------------------------------------------------------------------
// C entry points (ctypes from tests / bench cpu_baseline)
// ---------------------------------------------------------------------------------------------
static thread_local std::string g_err;

static char* dupstr(const std::string& s) {
  char* p = (char*)malloc(s.size() + 1);
  memcpy(p, s.c_str(), s.size() + 1);
  return p;
}

extern "C" {

const char* oref_last_error() { return g_err.c_str(); }
void oref_free(char* p) { free(p); }

// Solve one snapshot.  *out receives the results JSON; *seconds the time spent in Solve only.
int oref_solve_json(const char* snapshot, char** out, double* seconds) {
  try {
    ojson::Value root = ojson::parse(snapshot);
    oref::Problem pb = oref::parseProblem(root);
    auto t0 = std::chrono::steady_clock::now();
    oref::Scheduler s(pb);
    s.Solve();
    auto t1 = std::chrono::steady_clock::now();
    if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
    if (out) *out = dupstr(s.ResultsJSON());
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// Solve the same snapshot `reps` times (fresh Scheduler each time, as Provisioner does), parsing
// once; returns total Solve seconds.  Used for the bounded CPU-baseline sample.
int oref_time_solve(const char* snapshot, int reps, double* seconds) {
  try {
    ojson::Value root = ojson::parse(snapshot);
    double total = 0;
    for (int r = 0; r < reps; r++) {
      oref::Problem pb = oref::parseProblem(root);
      auto t0 = std::chrono::steady_clock::now();
      oref::Scheduler s(pb);
      s.Solve();
      total += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    *seconds = total;
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// Consolidation (single- and multi-node) over a cluster snapshot.  all_sims=1 simulates every
// candidate and every multi-node prefix and reports each outcome.
int oref_consolidate_json(const char* snapshot, int all_sims, char** out, double* seconds) {
  try {
    ojson::Value root = ojson::parse(snapshot);
    oref::ConsProblem cp = oref::parseConsProblem(root);
    auto t0 = std::chrono::steady_clock::now();
    std::string r = oref::consolidateJSON(cp, all_sims != 0);
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (out) *out = dupstr(r);
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// consolidate_json(all_sims=1) with the simulations precomputed on `threads` host threads (checker speed-up
// for the full-size digests; consolidation.inc precompute).
int oref_consolidate_json_threads(const char* snapshot, int threads, char** out, double* seconds) {
  try {
    ojson::Value root = ojson::parse(snapshot);
    oref::ConsProblem cp = oref::parseConsProblem(root);
    auto t0 = std::chrono::steady_clock::now();
    std::string r = oref::consolidateJSON(cp, true, nullptr, threads);
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (out) *out = dupstr(r);
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// consolidate_json with the methods' timeouts on a virtual clock (ConsClock).
int oref_consolidate_clock_json(const char* snapshot, int all_sims, double multi_timeout_s, double single_timeout_s,
                                double sim_seconds, char** out) {
  try {
    ojson::Value root = ojson::parse(snapshot);
    oref::ConsProblem cp = oref::parseConsProblem(root);
    oref::ConsClock clk;
    clk.multiTimeout = multi_timeout_s;
    clk.singleTimeout = single_timeout_s;
    clk.simSeconds = sim_seconds;
    if (out) *out = dupstr(oref::consolidateJSON(cp, all_sims != 0, &clk));
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// Tie-enumeration mode for Go map-order choice points (topology.inc TieBreak): 0 canonical, 1 largest
// domain name, 2 seeded pseudo-random.
int oref_set_tie_mode(int mode, unsigned long long seed) {
  oref::TieBreak::mode() = mode;
  oref::TieBreak::state() = seed ? seed : 0x9E3779B97F4A7C15ull;
  return 0;
}

// Cluster-state accounting: StateNode accessor values from Node / NodeClaim / Pod lists.
int oref_cluster_state(const char* cluster, char** out) {
  try {
    ojson::Value root = ojson::parse(cluster);
    if (out) *out = dupstr(oref::clusterStateJSON(root));
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// Validation of a consolidation command against the current cluster snapshot (validation.go:68-180).
int oref_validate_json(const char* snapshot, const char* command, char** out) {
  try {
    ojson::Value root = ojson::parse(snapshot);
    ojson::Value cmd = ojson::parse(command);
    oref::ConsProblem cp = oref::parseConsProblem(root);
    std::string r = oref::validateJSON(cp, cmd);
    if (out) *out = dupstr(r);
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// CPU baseline sample: the first `count` single-node consolidation simulations (simulateScheduling +
// computeConsolidation per candidate, as SingleNodeConsolidation runs them), timed after parsing.
// `threads` > 1 splits the (independent) simulations over that many host threads.
int oref_time_cons_sims(const char* snapshot, int count, int threads, double* seconds) {
  try {
    ojson::Value root = ojson::parse(snapshot);
    oref::ConsProblem cp = oref::parseConsProblem(root);
    const int n = std::min<int>(count, cp.nPass);
    const int nt = std::max(1, std::min(threads, n));
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; t++)
      pool.emplace_back([&cp, n, nt, t] {
        int64_t counter = cp.base.hostnameSeed;
        for (int i = t; i < n; i += nt) oref::computeConsolidation(cp, {i}, counter);
      });
    for (auto& th : pool) th.join();
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return n;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

int oref_eval_ops(const char* ops, char** out) {
  try {
    ojson::Value root = ojson::parse(ops);
    std::set<std::string> wk;
    if (auto* w = root.get("wellKnownLabels")) for (auto& x : w->arr()) wk.insert(x.str());
    else
      wk = {"karpenter.sh/nodepool", "topology.kubernetes.io/zone", "topology.kubernetes.io/region",
            "node.kubernetes.io/instance-type", "kubernetes.io/arch", "kubernetes.io/os",
            "karpenter.sh/capacity-type", "node.kubernetes.io/windows-build"};
    *out = dupstr(oref::evalOps(root, wk));
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

}  // extern "C"

#ifdef OREF_MAIN
#include <fstream>
#include <sstream>
int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: cpu_ref snapshot.json [reps]\n"); return 2; }
  std::ifstream f(argv[1]);
  std::stringstream ss;
  ss << f.rdbuf();
  std::string s = ss.str();
  if (argc > 2) {
    double secs = 0;
    if (oref_time_solve(s.c_str(), atoi(argv[2]), &secs)) { fprintf(stderr, "%s\n", oref_last_error()); return 1; }
    printf("%.6f\n", secs);
    return 0;
  }
  char* out = nullptr;
  double secs = 0;
  if (oref_solve_json(s.c_str(), &out, &secs)) { fprintf(stderr, "%s\n", oref_last_error()); return 1; }
  printf("%s\n", out);
  fprintf(stderr, "solve %.6f s\n", secs);
  oref_free(out);
  return 0;
}
#endif
