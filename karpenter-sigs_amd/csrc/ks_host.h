// ks_host.h — host-side problem model, encoder and renderer (declarations).
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <array>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "ks_json.h"
#include "ks_problem.h"
#include "ks_quantity.h"
#include "ks_reqset.h"

namespace ks {

struct KsError : std::runtime_error {
  int code;
  KsError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

using QList = std::map<std::string, Qty>;  // v1.ResourceList
struct NSR { std::string key, op; std::vector<std::string> values; };
struct TaintH { std::string key, value, effect; };
struct TolH { std::string key, op, value, effect; };
struct PrefTerm { int32_t weight; std::vector<NSR> exprs; };
// metav1.LabelSelector: matchLabels (as In with one value) then matchExpressions; nil = !present
struct SelReq { std::string key, op; std::vector<std::string> values; };
struct LabelSel { bool present = false; std::vector<SelReq> reqs; };
struct AffTerm { LabelSel sel; std::vector<std::string> namespaces; bool nsSelector = false; LabelSel nsSel; std::string key; };
struct SpreadC { std::string key, when; int32_t maxSkew = 0; int32_t minDomains = -1; LabelSel sel; };
// HostPort (hostportusage.go:38-43): IP (net.ParseIP, 16-byte form), port, protocol
struct HostPortH {
  std::string ip, proto;
  int32_t port = 0;
  std::array<uint8_t, 16> ip16{};
  bool ipValid = false;
  bool unspecified() const;
  bool matches(const HostPortH& o) const;  // HostPort.Matches (hostportusage.go:49-61)
};
HostPortH make_host_port(const std::string& ip, int32_t port, const std::string& proto);

// The pod fields the Solve path reads (pod spec subset; pkg/utils/pod, requirements.go:64-100,
// preferences.go, resources.go Ceiling).
struct PodH {
  std::string name, ns, uid;
  int64_t created = 0;
  std::map<std::string, std::string> labels, nodeSelector;
  bool hasAffinity = false, hasNodeAffinity = false, hasRequired = false;
  std::vector<std::vector<NSR>> requiredTerms;
  std::vector<PrefTerm> preferred;
  bool hasPodAffinity = false, hasPodAnti = false;
  std::vector<AffTerm> affRequired, antiRequired;
  std::vector<std::pair<int32_t, AffTerm>> affPreferred, antiPreferred;
  std::vector<SpreadC> tsc;  // topologySpreadConstraints
  std::string nodeName, phase;  // cluster pods (topology counting)
  std::vector<TolH> tols;
  QList requests;  // RequestsForPods(pod) incl. pods=1
  bool hostPorts = false, volumes = false;
  std::vector<std::string> pvcNames;  // volume.GetPersistentVolumeClaim names (claimName / <pod>-<volume>)
  std::vector<HostPortH> ports;  // GetHostPorts (hostportusage.go:92-114)
  bool provisionable = true;  // IsProvisionable (pkg/utils/pod/scheduling.go:28-34)
  // fields the disruption path reads (node.go:32-53 GetNodePods, helpers.go:137-159, scheduling.go:85-92)
  bool ownedByNode = false, ownedByDaemonSet = false, terminal = false, deleting = false;
  std::map<std::string, std::string> annotations;
  bool hasPriority = false;
  bool notReady = false;  // a Ready condition with status False (PDBLimits.CanEvictPods, pdblimits.go:70-76)
  int32_t priority = 0;
};
PodH parse_pod(const ksjson::Value& v);
// Cluster-state accounting (ks_state.cpp): StateNode accessor values from {nodeClaims, nodes, pods}
std::string cluster_state_json(const ksjson::Value& cluster);

struct PodState {  // one point of the relaxation chain
  std::vector<uint32_t> rsAll, rsStrict;
  bool hasPreferred = false;
  std::vector<TolH> tols;
  std::vector<int32_t> gown;  // topology groups the pod owns in this state (Topology.Update, topology.go:91-122)
  // (group, minDomains) of this state's spread constraints whose minDomains differs from the group's: a group's
  // Hash leaves minDomains out (topologygroup.go:142-158), so a group takes the minDomains of the pod whose
  // Update creates it (topology.go:108-118), which depends on which pods a Solve / simulation holds
  std::vector<std::pair<int32_t, int32_t>> gmd;
  std::shared_ptr<PodH> spec;  // the (relaxed) pod spec of this state, kept for topology pods only
};

// One topology group (topologygroup.go:56-68) as the device sees it.  Groups [0, G1) are
// t.topologies (creation order), [G1, G) t.inverseTopologies.
struct TopoGroup {
  int type = 0;  // TG_SPREAD / TG_ANTI
  std::string key, hash;
  int keyId = -1;
  int32_t maxSkew = 0, minDomains = -1;
  std::set<std::string> namespaces;
  LabelSel sel;
  bool filterNil = true;
  std::vector<std::vector<uint32_t>> filter;  // OR of requirement records (TopologyNodeFilter)
  std::map<std::string, int32_t> domains;    // registered domain -> count (initial state)
  bool late = false;  // created by a relaxed state's Topology.Update mid-Solve (topology.go:102-119)
};

struct Host {
  // universe
  std::vector<std::string> keyNames;             // sorted; id = index
  std::map<std::string, int> keyId;
  std::vector<std::vector<std::string>> values;  // per key, sorted
  std::vector<std::map<std::string, int>> valueId;
  std::vector<KeyMeta> keys;
  std::vector<uint32_t> wordValid, vIsInt;
  std::vector<int64_t> vInt;
  ReqLayout L{};
  int hostKey = -1, zoneKey = -1, ctKey = -1, hostPrivBit = -1;
  uint64_t allowWK = 0, itKeys = 0;
  std::set<std::string> wellKnown;
  // resources
  std::vector<std::string> resNames;
  std::map<std::string, int> resId;
  std::vector<int> resShift;  // device value = nano / 10^shift
  // taints
  std::vector<TaintH> taints;
  std::vector<HostPortH> hostPortUniverse;  // distinct (IP, port, protocol), bit i of the host-port masks
  std::vector<std::string> hostPortOwner;   // per element: "" or the key of the pod being scheduled whose initial entry it is
  std::map<std::string, std::string> volumeDrivers;  // "ns/pvc" -> resolved CSI driver (resolveDriver, volumeusage.go:115-172)
  std::vector<std::string> volDrivers, volUniverse;  // limited drivers (id v); the pods' PVC keys of those drivers (id u)
  // per pod: VolumeTopology.Inject failed (provisioner.go:432-442: the pod is left out of NewTopology's pod
  // list -- not excluded from the counts, no Topology.Update -- and still scheduled, uninjected)
  std::vector<char> injectFailed;
  // instance types
  struct Offer { std::string zone, ct; double price = 0; bool available = true; };
  struct IT { std::string name; std::vector<NSR> reqs; QList capacity, alloc; std::vector<std::pair<std::string, std::string>> offers;
              std::vector<double> prices; std::vector<Offer> all; };
  std::vector<IT> its;
  // templates
  struct Tpl {
    std::string pool;
    std::vector<NSR> reqs;
    std::map<std::string, std::string> labels;
    std::map<std::string, std::string> poolLabels;  // spec.template.metadata.labels (no karpenter.sh/nodepool)
    std::vector<TaintH> taints;
    std::vector<int> its;
    QList daemon;
    int limitPool = -1;
    std::vector<uint32_t> rs;  // without hostname
  };
  std::vector<Tpl> tpls;
  struct Pool { std::string name; QList remaining; };
  std::vector<Pool> pools;
  bool toleratePreferNoSchedule = false;
  // existing nodes (sorted)
  struct Node { std::string name, hostName; std::map<std::string, std::string> labels; std::vector<TaintH> taints;
                QList available, capacity, dsRequests, req0; bool initialized = true, ready = true; int origIndex = 0;
                std::vector<std::pair<std::string, HostPortH>> hostPorts;  // HostPortUsage: (pod key, port)
                std::map<std::string, std::set<std::string>> volumes;      // VolumeUsage: driver -> PVC keys
                std::map<std::string, int64_t> volumeLimits; };            // driver -> CSINode allocatable count
  std::vector<Node> nodes;
  std::vector<PodH> daemons;
  std::vector<PodH> pods;
  std::vector<std::vector<PodState>> states;  // per pod relaxation chain
  // topology (topology.go): groups, the cluster's bound pods and node labels it counts
  std::vector<TopoGroup> groups;
  int groupsOwned = 0;  // G1
  std::vector<PodH> clusterPods;
  std::map<std::string, std::map<std::string, std::string>> nodeLabelsByName;
  std::vector<std::pair<std::string, std::map<std::string, std::string>>> namespaceList;  // (name, labels)
  std::vector<uint64_t> podGsel, podGinv;  // per pod: groups that select it / inverse groups it owns
  // Consolidation view (ks_cons.cpp): NewTopology excludes only these UIDs (the pods every simulation
  // schedules); each simulation then subtracts its candidates' pods from the counts it records below.
  const std::set<std::string>* topoExcluded = nullptr;
  std::vector<PodH>* preParsedPods = nullptr;  // set: the snapshot's "pods" already parsed (moved in by build)
  std::map<std::string, std::vector<std::pair<int, int>>> topoContrib;  // cluster pod UID -> (group, value) counted
  std::map<std::string, std::vector<int32_t>> topoInvOwner;             // cluster pod UID -> inverse groups it owns
  std::vector<int> topoInvOwners;                                       // per group: owning cluster pods
  std::vector<std::vector<char>> topoUniverse;                          // per group, per value: in the domain universe
  std::set<int> topoHostActive;                                         // hostname value ids of the nodes (Register)
  bool activeHost(int v) const { return topoHostActive.count(v) != 0; }
  int64_t hostnameSeed = 0;
  // NewQueue order computed on the host (set only when some pods tie on the whole sort key, i.e. share
  // cpu, memory, creation time and UID, as the benchmark's un-applied pods do): sort.Slice's order of
  // tied pods is its swap sequence over the input order (ks_gosort.h), not a key order the radix sort
  // on the device can reproduce.
  std::vector<int32_t> hostQueue;
  bool emptyTopology = false;  // the benchmark's &scheduling.Topology{}: no groups (scheduling_benchmark_test.go:124)
  KsDims dims{};

  // host images of the device tables
  struct Tables {
    std::vector<int64_t> tsort_alloc, it_alloc, it_cap, tpl_daemon, pool_rem0, pod_req, pod_sortkey, n_avail, n_req0;
    std::vector<double> off_price;
    std::vector<int32_t> n_flags, pod_flags;
    std::vector<uint64_t> pod_hpc, pod_hpu, pod_hpo, n_hp0;
    // volume limits (volumeusage.go:183-227), sparse over the pods' PVC universe (ks_problem.h KsDev)
    std::vector<int32_t> pod_vdbeg, pod_vd, pod_vsbeg, pod_vs, pod_vubeg, pod_vu, vol_udrv;
    std::vector<int32_t> n_vc0, n_vlim;
    // topology groups (ks_topo.cpp)
    std::vector<int32_t> tg_meta;   // [G][TGM_WORDS]
    std::vector<int32_t> tg_cnt0;   // counts per (group, value) at NewScheduler time
    std::vector<uint32_t> tg_frs;   // node-filter requirement records
    std::vector<uint64_t> st_gown, pod_gsel, pod_ginv;  // [S][GMW], [P][GMW], [P][GMW] group sets
    std::vector<uint64_t> tg_late;                      // [GMW] groups a relaxation creates mid-Solve
    std::vector<uint32_t> st_rss;   // [S][RSW] strict pod requirements (NewStrictPodRequirements)
    std::vector<int32_t> n_tdom;    // [TK][N] value index of the node's label for each topology key (-1: none)
    std::vector<uint32_t> it_rs, tpl_rs, st_rs, n_rs0, pool_mask;
    std::vector<uint64_t> st_toltpl;
    std::vector<uint64_t> tpl_taint, st_tol, n_taint;
    std::vector<int32_t> tsort_pos, it_off_beg, off_zone, off_ct, tpl_it_beg, tpl_its, tpl_pool, pod_state0, pod_nstate, pod_uid,
        st_flags;
    // the Quantity side of each request list (results replay of Merge, resources.go:53-63, in integers):
    // which resources the list names and each entry's format ([P][R] / [NTPL][R])
    std::vector<uint32_t> pod_rmask, tpl_rmask;
    std::vector<uint8_t> pod_rfmt, tpl_rfmt;
    // feasibility tables (k_solve feas_masks)
    std::vector<uint32_t> fk_words;
    std::vector<int32_t> fk_key_off;  // [NTPL][NK] block of key k in template t, -1: no table
    std::vector<int32_t> fk_tpl;      // [NTPL][3]: all positions, irregular positions, offerings
  } tab;

  void build(const ksjson::Value& root);
  void buildTopology();  // ks_topo.cpp: after the pods' relaxation chains
  bool topoClusterPod(const PodH& cp, std::vector<std::pair<int, int>>& contrib, std::vector<int32_t>& inv) const;

  // encoded algebra helpers
  std::vector<uint32_t> emptyRec() const { return std::vector<uint32_t>(dims.RSW, 0); }
  void addNSR(std::vector<uint32_t>& rec, const std::string& key, const std::string& op,
              const std::vector<std::string>& vals) const;
  void addLabels(std::vector<uint32_t>& rec, const std::map<std::string, std::string>& labels) const;
  // an existing node's labels, restricted to the universe's keys (node-only keys are not interned: build)
  void addNodeLabels(std::vector<uint32_t>& rec, const std::map<std::string, std::string>& labels) const;
  std::vector<uint32_t> podRequirements(PodH& p, bool all) const;
  void tolMask(const std::vector<TolH>& tols, const std::vector<int>& cls, uint64_t out[2]) const;
  int64_t toDev(int r, const Qty& q) const;
  Qty fromDev(int r, int64_t v) const;

  // rendering
  std::string reqString(const uint32_t* rec, int k, bool full, int64_t privateHost) const;
  std::string reqsString(const uint32_t* rec, int64_t privateHost) const;  // Requirements.String()
  std::vector<std::string> compatErrors(const uint32_t* r, const uint32_t* in, bool loose, int64_t privateHost) const;
  std::string placeholder(int64_t id) const;

 private:
  void intern(const std::string& key, const std::string& val);
  void internKey(const std::string& key);
  std::map<std::string, std::set<std::string>> valueSet_;
};

// Host-side phase timing for diagnostics: KS_HOST_TIMING=1 prints each mark's milliseconds to stderr.
struct PhaseTimer {
  const char* what;
  bool on;
  std::chrono::steady_clock::time_point t;
  explicit PhaseTimer(const char* w) : what(w), on(std::getenv("KS_HOST_TIMING") != nullptr), t(std::chrono::steady_clock::now()) {}
  void mark(const char* phase) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[%s] %-34s %8.2f ms\n", what, phase, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};

// Binary snapshot of the host model (ks_snapshot.cpp, ks_archive.h)
// Topology-group sets as GMW-word bitsets (ks_problem.h): set bit g of row `row`; test it.
inline void gset(std::vector<uint64_t>& v, size_t row, int gmw, int g) { v[row * (size_t)gmw + (size_t)(g >> 6)] |= 1ull << (g & 63); }
inline bool gtest(const std::vector<uint64_t>& v, size_t row, int gmw, int g) {
  return (v[row * (size_t)gmw + (size_t)(g >> 6)] >> (g & 63)) & 1ull;
}

struct ArOut;
struct ArIn;
void host_save(ArOut& a, Host& h);
void host_load(ArIn& a, Host& h);

std::string qlist_json(const QList& l);  // resources.String (pretty.Concise)
std::string go_quote(const std::string& s);
std::string normalize_key(const std::string& k);

}  // namespace ks
