// ks_cons.cpp — consolidation (pkg/controllers/disruption) on the GPU.
//
//   host   : the cluster snapshot -> one resident scheduling problem holding every pod any simulation
//            schedules (pending pods, the candidates' reschedulable pods, the deleting nodes' pods)
//            and every active node; candidate construction and ordering; per-simulation views
//   device : every candidate-deletion simulation (simulateScheduling helpers.go:73-127 + the
//            computeConsolidation decision consolidation.go:113-194) as one wavefront of k_solve<SIM>,
//            a whole batch per launch, sharded across GPUs by simulation index
//   host   : the reference's sequential selection replayed over the gathered records
//            (MultiNodeConsolidation.firstNConsolidationOption multinodeconsolidation.go:87-137,
//            SingleNodeConsolidation.ComputeCommand singlenodeconsolidation.go:42-88)
//
// Candidate construction follows NewCandidate (types.go:54-113) for the listed nodes, disruptionCost /
// GetPodEvictionCost / lifetimeRemaining (helpers.go:137-177, types.go:136-145), filterCandidates'
// do-not-disrupt rule (helpers.go:47-71; PDBs are the caller's filter) and the cost sort of
// sortAndFilterCandidates (consolidation.go:73-83, Go sort.Slice emulated exactly).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <exception>
#include <ctime>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/karpenter_amd.h"
#include "ks_gosort.h"
#include "ks_archive.h"
#include "ks_host.h"
#include "ks_parallel.h"
#include "ks_runtime.h"

using namespace ks;
using ksjson::Value;

namespace {

const char* kCTKey = "karpenter.sh/capacity-type";
const char* kZoneKey = "topology.kubernetes.io/zone";
const char* kPoolKey = "karpenter.sh/nodepool";
const char* kITKey = "node.kubernetes.io/instance-type";

std::string jstr(const Value* v, const char* k, const std::string& d = "") {
  if (!v) return d;
  const Value* x = v->get(k);
  return x && x->is_str() ? x->str() : d;
}

// PDBLimits (pdblimits.go:36-110): the snapshot's PodDisruptionBudgets
struct Pdb {
  std::string ns;
  bool present = false;  // LabelSelectorAsSelector(nil) = Nothing; {} = Everything
  std::vector<std::pair<std::string, std::pair<std::string, std::vector<std::string>>>> reqs;  // key, (op, values)
  int64_t allowed = 0;
  bool unhealthyAlways = false;
};
std::vector<Pdb> parse_pdbs(const Value& root) {
  std::vector<Pdb> out;
  const Value* ps = root.get("podDisruptionBudgets");
  if (!ps) return out;
  for (auto& v : ps->arr()) {
    Pdb b;
    b.ns = jstr(v.get("metadata"), "namespace");
    const Value* sp = v.get("spec");
    const Value* sel = sp ? sp->get("selector") : nullptr;
    if (sel && !sel->is_null()) {
      b.present = true;
      if (const Value* ml = sel->get("matchLabels"))
        for (auto& kv : ml->obj()) b.reqs.push_back({kv.first, {"In", {kv.second.str()}}});
      if (const Value* me = sel->get("matchExpressions"))
        for (auto& e : me->arr()) {
          std::vector<std::string> vals;
          if (const Value* vs = e.get("values")) for (auto& x : vs->arr()) vals.push_back(x.str());
          const std::string op = jstr(&e, "operator");
          const bool setOp = op == "In" || op == "NotIn", exOp = op == "Exists" || op == "DoesNotExist";
          if (!(setOp || exOp) || (setOp && vals.empty()) || (exOp && !vals.empty()))
            throw KsError(KS_ERR_PARSE, "tracking PodDisruptionBudgets: invalid selector");
          b.reqs.push_back({jstr(&e, "key"), {op, vals}});
        }
    }
    b.unhealthyAlways = sp && jstr(sp, "unhealthyPodEvictionPolicy") == "AlwaysAllow";
    const Value* st = v.get("status");
    if (st && st->get("disruptionsAllowed")) b.allowed = st->get("disruptionsAllowed")->i64();
    out.push_back(std::move(b));
  }
  return out;
}
// CanEvictPods (pdblimits.go:58-84)
bool can_evict(const std::vector<Pdb>& pdbs, const PodH& p) {
  for (auto& b : pdbs) {
    if (b.ns != p.ns || !b.present) continue;
    bool match = true;
    for (auto& r : b.reqs) {
      auto it = p.labels.find(r.first);
      const bool has = it != p.labels.end();
      const std::string& op = r.second.first;
      const auto& vals = r.second.second;
      const bool in = has && std::find(vals.begin(), vals.end(), it->second) != vals.end();
      if (op == "In") match = match && in;
      else if (op == "NotIn") match = match && !in;
      else if (op == "Exists") match = match && has;
      else match = match && !has;
    }
    if (!match) continue;
    if (!(b.unhealthyAlways && p.notReady) && b.allowed == 0) return false;
  }
  return true;
}

int64_t parse_rfc3339(const std::string& s) {  // seconds; the snapshot uses "YYYY-MM-DDTHH:MM:SSZ"
  if (s.size() < 19) return 0;
  struct tm t{};
  t.tm_year = std::atoi(s.substr(0, 4).c_str()) - 1900;
  t.tm_mon = std::atoi(s.substr(5, 2).c_str()) - 1;
  t.tm_mday = std::atoi(s.substr(8, 2).c_str());
  t.tm_hour = std::atoi(s.substr(11, 2).c_str());
  t.tm_min = std::atoi(s.substr(14, 2).c_str());
  t.tm_sec = std::atoi(s.substr(17, 2).c_str());
  return (int64_t)timegm(&t);
}

// time.ParseDuration for the forms NodePool durations take ("720h", "1h30m", "90s", "1.5h")
bool go_duration(const std::string& s, int64_t& ns) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '-' || s[0] == '+') neg = s[i++] == '-';
  if (s.substr(i) == "0") { ns = 0; return true; }
  long double total = 0;
  while (i < s.size()) {
    size_t j = i;
    while (j < s.size() && (std::isdigit((unsigned char)s[j]) || s[j] == '.')) j++;
    if (j == i) return false;
    const long double v = std::stold(s.substr(i, j - i));
    size_t k = j;
    while (k < s.size() && !std::isdigit((unsigned char)s[k]) && s[k] != '.') k++;
    const std::string u = s.substr(j, k - j);
    long double mul;
    if (u == "ns") mul = 1;
    else if (u == "us" || u == "\xC2\xB5s" || u == "\xCE\xBCs") mul = 1e3;
    else if (u == "ms") mul = 1e6;
    else if (u == "s") mul = 1e9;
    else if (u == "m") mul = 60e9;
    else if (u == "h") mul = 3600e9;
    else return false;
    total += v * mul;
    i = k;
  }
  ns = (int64_t)(neg ? -total : total);
  return true;
}

double dur_seconds(int64_t d) { return (double)(d / 1000000000) + (double)(d % 1000000000) / 1e9; }
double clampf(double lo, double v, double hi) { return v < lo ? lo : (v > hi ? hi : v); }

double eviction_cost(const PodH& p) {  // GetPodEvictionCost helpers.go:137-159
  double cost = 1.0;
  auto a = p.annotations.find("controller.kubernetes.io/pod-deletion-cost");
  if (a != p.annotations.end() && !a->second.empty() && !std::isspace((unsigned char)a->second[0])) {
    char* end = nullptr;
    const double c = std::strtod(a->second.c_str(), &end);
    if (end && *end == 0) cost += c / std::pow(2.0, 27.0);  // a ParseFloat error is logged and ignored
  }
  if (p.hasPriority) cost += (double)p.priority / std::pow(2.0, 25.0);
  return clampf(-10.0, cost, 10.0);
}

bool do_not_disrupt(const PodH& p) {  // pkg/utils/pod/scheduling.go:85-92
  auto a = p.annotations.find("karpenter.sh/do-not-evict");
  auto b = p.annotations.find("karpenter.sh/do-not-disrupt");
  return (a != p.annotations.end() && a->second == "true") || (b != p.annotations.end() && b->second == "true");
}

}  // namespace

struct ks_cons {
  struct Cand {
    int node = -1;  // index into host.nodes (calculateExistingNodeClaims order)
    std::string name, pool, ct, zone;
    int it = -1;
    double cost = 0;
    std::vector<int> pods;  // global pod indices (GetNodePods)
  };
  struct Sim {
    std::vector<int> cands;  // indices into cands
    bool multi = false;
  };
  std::unique_ptr<ks_problem> pb;
  // An update that failed after it started editing the host model (an internal inconsistency, or the device
  // upload) left it half-applied or ahead of HBM: the handle refuses every later call (KS_ERR_HIP) instead of
  // simulating a mix (rebuild it with ks_cons_create).
  std::string broken;
  void check_usable() const {
    if (!broken.empty()) throw KsError(KS_ERR_HIP, "consolidation handle unusable after a failed update (" + broken + ")");
  }
  // [0, nPass): the pass's candidates in disruption-cost order; [nPass, size): nodes only
  // Validation.ShouldDisrupt admits (their pool has consolidateAfter Never), for validation's mapping
  std::vector<Cand> cands;
  int nPass = 0;
  std::vector<Sim> sims;  // multi-node prefixes first (largest first), then one per candidate
  int multiHi = 0;        // multi-node prefix lengths mid+1 for mid in [1, multiHi]
  std::vector<int> pending, deleting;
  std::set<std::string> nominated;  // Cluster.IsNodeNominated (validation.go:99-103)
  int64_t hostnameSeed = 0;
  int recWords = 0;

  // What the candidates are re-derived from after ks_cons_update (pod and node deltas between passes):
  // every node that passed NewCandidate's node tests, in the snapshot's "candidates" order, blocked or not;
  // the pods of every active node (GetNodePods order); and per pod its cost and filterCandidates verdict.
  struct CandIn {
    Cand k;                // pods and cost filled in by order_candidates
    double remaining = 1;  // lifetimeRemaining (types.go:136-145)
    bool passOk = true;    // ShouldDisrupt for the pass (consolidateAfter is not Never)
  };
  enum : int32_t { PN_PENDING = -1, PN_DELETING = -2, PN_GONE = -3 };
  std::vector<CandIn> candIn;
  std::vector<std::vector<int>> nodePods;  // [host node] GetNodePods
  std::vector<int32_t> podNode;            // [pod] host node index or PN_*
  std::vector<uint8_t> podBlock;           // [pod] bit 0: blocks its node; bit 1: would block once bound and Running
  std::vector<double> podCost;             // [pod] GetPodEvictionCost
  std::vector<uint8_t> nodeGone;           // [host node] removed by an update
  std::unordered_map<std::string, int> uidIndex, nodeIndex;  // built at the first update
  // topology clusters, built at the first update (from the host state, so also after a binary load):
  // clusterPods position per UID and UIDs per node name; per owned group, the remaining pods owning it in
  // their first state / only in later states (a pod counted once per group)
  std::unordered_map<std::string, int> cpIndex;
  std::unordered_map<std::string, std::vector<std::string>> cpByNode;
  std::vector<int> gOwn0, gOwnLate;
  bool topoIndexed = false;
  // per pod: its topoContrib / topoInvOwner entry (resolved once, kept current by ks_cons_update)
  std::vector<const std::vector<std::pair<int, int>>*> podContrib;
  std::vector<const std::vector<int32_t>*> podInv;
  // the groups some relaxation state creates with another minDomains (PodState::gmd), built on first use: the
  // states are fixed at create (an update only removes or binds pods, so the list stays a superset)
  std::vector<int> altGroups;
  bool altBuilt = false;
  int64_t updates = 0;
  // per host node, for the per-simulation limits (prepare_launch): the NodePools it counts against and its
  // capacity in device units (static for the handle; built on first use)
  std::vector<std::vector<int>> nodePoolIdx;
  std::vector<int64_t> nodeCapDev;

  // A launch of one rank's simulations, cached per (rank, world).  Validation runs its one
  // re-simulation in a launch of its own, so the pass's launch (records, requirement records,
  // counters) survives it.
  struct Launch {
    int lrank = -1, lworld = -1;
    std::vector<int> lsims;  // simulation ids of this rank, launch order
    void* lbuf = nullptr;    // workspaces + pod maps + views
    KsWork* lworks = nullptr;
    int32_t* lrec = nullptr;
    int32_t* hrec = nullptr;  // pinned host staging of the records (one DMA per pass, no pageable bounce)
    // A world-1 pass whose records stay in the handle (ks_cons_run with records NULL) downloads only their
    // headers (k_rec_headers: RF_HDR words per simulation, + 2 status words the device's record checks fill);
    // the decision fetches the option words of the few records it renders from lrec (RecView)
    int32_t* lhdr = nullptr;
    int32_t* hhdr = nullptr;  // host-mapped pinned: k_rec_headers writes it directly (dhdr: its device address)
    int32_t* dhdr = nullptr;
    unsigned long long* lst = nullptr;  // device: the two status words + the block counter (persist, see k_rec_headers)
    bool hdrOnly = false;
    bool keptFull = false;  // a world-1 run kept the records with KS_CONS_FULL_RECORDS set (full download)
    int32_t* lentries = nullptr;
    int32_t* lentrySim = nullptr;
    int32_t* lpodmap = nullptr;
    int32_t* lrunlen = nullptr;   // identical pods left in the run at each sorted entry (sim_run_lengths)
    uint64_t* lrunw = nullptr;    // run-start bits, 64 entries per word
    uint64_t* lkeys = nullptr;
    int32_t* lvals = nullptr;
    void* ltemp = nullptr;
    size_t ltempBytes = 0;
    int lnent = 0, lrbits = 0, lsbits = 0;
    int lnmw = 0;  // the plan's first lnmw simulations (the long multi-node prefixes) run on 4-wave workgroups
    bool lsorted = false;  // lpodmap holds every simulation's NewQueue order (a plan's pods never change)
    Plan lplan{};
    std::vector<KsWork> lhost;  // host copy of the launch's workspace views (diagnostics)
    // A topology plan is built in two phases: the multi-node prefixes (the long simulations, first in the plan)
    // get their NewTopology deltas in prepare_launch and are launched at once; the single-node simulations'
    // deltas are built while those run (pipeB: still to do, finish_topology) and launched behind them.
    bool pipeB = false;
    int nA = 0;                              // simulations [0, nA) launched first
    std::vector<std::vector<int>> podsB;     // pod lists of simulations [nA, ns)
    void* ltopoB = nullptr;                  // device: their topology inputs
    char* htopoB = nullptr;                  // pinned staging of those
    KsWork* hworksB = nullptr;               // pinned staging of their workspace views
    size_t capTopoB = 0, capHtopoB = 0, capHworksB = 0;
    // allocation capacities: a new plan (another rank / world, an update) reuses the buffers that fit
    size_t capBuf = 0, capWorks = 0, capRec = 0, capHrec = 0, capEnt = 0, capRunw = 0, capTemp = 0, capHdr = 0, capHhdr = 0;
    void release() {
      for (void* p : {(void*)lbuf, (void*)lworks, (void*)lrec, (void*)lentries, (void*)lentrySim, (void*)lpodmap,
                      (void*)lrunlen, (void*)lrunw, (void*)lkeys, (void*)lvals, ltemp, (void*)lhdr, (void*)lst, ltopoB})
        if (p) (void)hipFree(p);
      if (hrec) (void)hipHostFree(hrec);
      if (hhdr) (void)hipHostFree(hhdr);
      if (htopoB) (void)hipHostFree(htopoB);
      if (hworksB) (void)hipHostFree(hworksB);
      *this = Launch{};  // stale lookups (claim requirements, counters) now fail cleanly
    }
    // drop the plan, keep the allocations
    void invalidate() {
      lrank = lworld = -1;
      lsims.clear();
      lhost.clear();
      lnent = lrbits = lsbits = lnmw = 0;
      lsorted = false;
      hdrOnly = keptFull = false;
      lplan = Plan{};
      pipeB = false;
      nA = 0;
      podsB.clear();
    }
  };
  Launch L;
  hipEvent_t ev[2] = {nullptr, nullptr};  // run_sims' timing events
  hipStream_t st2 = nullptr;               // the multi-wave launch's stream (launch_sims_split)
  hipEvent_t evFork = nullptr, evJoin = nullptr;
  int32_t* rank = nullptr;  // global NewQueue rank of every pod
  // carry_walk: a probe re-run's starting relaxation state per pod (prepare_launch uploads it with the plan)
  const std::vector<int32_t>* carryStart = nullptr;
  // firstNConsolidationOption's binary search (multinodeconsolidation.go:101-135) as carry_walk resolved it for
  // the last decision: the probes in search order, each the pass's simulation of its prefix or a re-run from
  // the pod objects earlier probes relaxed
  struct Probe {
    int mid = 0;
    bool carried = false;       // re-run from carried relaxation states
    int sim = -1;               // the pass's simulation of the prefix
    std::vector<int32_t> rec;   // carried: the re-run's record
    std::vector<uint32_t> rs;   // carried: its NewNodeClaims[0] requirements (when it has a NodeClaim)
  };
  struct Walk {
    bool valid = false;
    uint64_t pass = 0;
    int world = 0;
    bool hasClock = false;
    double clock[3] = {0, 0, 0};
    std::vector<Probe> probes;
    int chosen = -1;   // the probe whose command is lastSavedCommand (-1: none)
    bool err = false;  // a probe's getCandidatePrices failed (ComputeCommand returns the error)
    int reruns = 0;    // launches on this GPU: carried probes, and probes whose relaxed states another rank holds
  };
  Walk walk;
  uint64_t passId = 0;  // ks_cons_run calls (a walk is valid for the pass it was computed on)
  Launch LR;            // the re-runs' launch (its buffers are kept between re-runs)

  int sim_of_multi(int mid) const { return multiHi - mid; }  // mid in [1, multiHi]
  int sim_of_single(int i) const { return multiHi + i; }
  int per_rank(int world) const { return ((int)sims.size() + world - 1) / world; }

  void free_launch() { L.release(); }
  void invalidate_launch() { L.invalidate(); }
  ~ks_cons() {
    int prev = -1;
    // (a handle whose load failed before device init has device -1: nothing to select, and hipSetDevice(-1)
    // would leave a sticky error for the caller's next launch)
    if (pb && pb->device >= 0 && hipGetDevice(&prev) == hipSuccess) (void)hipSetDevice(pb->device);
    free_launch();
    LR.release();
    if (rank) (void)hipFree(rank);
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {evFork, evJoin})
      if (e) (void)hipEventDestroy(e);
    if (st2) (void)hipStreamDestroy(st2);
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

namespace {

// The pass's candidates and simulations from candIn and the current pods: disruptionCost (helpers.go:170-176,
// summed in GetNodePods order) x lifetimeRemaining, filterCandidates, sort.Slice by cost, then the multi-node
// prefixes and the singles.  Run by build_cons and after every ks_cons_update.
void order_candidates(ks_cons& c) {
  // (the candidate and simulation vectors are rewritten in place: an update re-orders every pass, and
  // freeing / re-allocating 5000 candidates' and simulations' storage cost more than the rest)
  PhaseTimer pt("order_candidates");
  std::vector<int> pass, valOnly;  // candIn indices
  std::vector<double> cost(c.candIn.size(), 0.0);
  pass.reserve(c.candIn.size());
  for (size_t i = 0; i < c.candIn.size(); i++) {
    const ks_cons::CandIn& ci = c.candIn[i];
    if (c.nodeGone[(size_t)ci.k.node]) continue;
    double sum = 0;
    bool blocked = false;
    for (int p : c.nodePods[(size_t)ci.k.node]) {
      sum += c.podCost[(size_t)p];
      blocked = blocked || (c.podBlock[(size_t)p] & 1);
    }
    if (blocked) continue;
    cost[i] = sum * ci.remaining;
    (ci.passOk ? pass : valOnly).push_back((int)i);
  }
  pt.mark("costs");
  // sort.Slice(candidates, disruptionCost <): pdqsort only observes less(), so the costs' dense ranks
  // reproduce its swap sequence exactly.
  const int n = (int)pass.size();
  std::vector<int32_t> idx(n);
  {
    std::vector<double> vals(n);
    for (int i = 0; i < n; i++) vals[(size_t)i] = cost[(size_t)pass[(size_t)i]];
    std::sort(vals.begin(), vals.end());
    std::vector<int32_t> key(n);
    for (int i = 0; i < n; i++) {
      key[i] = (int32_t)(std::lower_bound(vals.begin(), vals.end(), cost[(size_t)pass[(size_t)i]]) - vals.begin());
      idx[i] = i;
    }
    GoSortExact g{GoSort{key.data(), idx.data()}};
    g.run(n);
  }
  pt.mark("sort");
  c.cands.resize((size_t)n + valOnly.size());
  auto put = [&](size_t at, int ii) {
    const ks_cons::CandIn& ci = c.candIn[(size_t)ii];
    ks_cons::Cand& k = c.cands[at];
    k.node = ci.k.node;
    k.name = ci.k.name;
    k.pool = ci.k.pool;
    k.ct = ci.k.ct;
    k.zone = ci.k.zone;
    k.it = ci.k.it;
    k.cost = cost[(size_t)ii];
    k.pods = c.nodePods[(size_t)ci.k.node];
  };
  for (int i = 0; i < n; i++) put((size_t)i, pass[(size_t)idx[i]]);
  for (size_t i = 0; i < valOnly.size(); i++) put((size_t)n + i, valOnly[i]);
  c.nPass = n;
  pt.mark("candidates");
  // the simulations: multi-node prefixes (firstNConsolidationOption's search space) and single nodes
  c.multiHi = 0;
  if (n >= 2) {
    int hi = std::min(n, 100);
    if (n <= hi) hi = n - 1;
    c.multiHi = hi;
  }
  c.sims.resize((size_t)c.multiHi + (size_t)n);
  size_t at = 0;
  for (int mid = c.multiHi; mid >= 1; mid--, at++) {
    ks_cons::Sim& s = c.sims[at];
    s.multi = true;
    s.cands.resize((size_t)mid + 1);
    for (int i = 0; i <= mid; i++) s.cands[(size_t)i] = i;
  }
  for (int i = 0; i < n; i++, at++) {
    ks_cons::Sim& s = c.sims[at];
    s.multi = false;
    s.cands.assign(1, i);
  }
}

// Parse the cluster snapshot into the resident problem + candidates + sims.
void build_cons(ks_cons& c, const Value& rootIn) {
  PhaseTimer pt("build_cons");
  if (!rootIn.is_obj()) throw KsError(KS_ERR_PARSE, "snapshot is not an object");
  // "cluster": {nodeClaims, nodes, pods} listings instead of "stateNodes": derive the StateNodes the
  // cluster-state informers would hold (ks_cluster_state)
  Value root = rootIn;
  if (const Value* cl = rootIn.get("cluster"); cl && !rootIn.get("stateNodes")) {
    const std::string sn = cluster_state_json(*cl);
    root.o = std::make_shared<ksjson::Object>(rootIn.obj());
    (*root.o)["stateNodes"] = ksjson::Parser(sn.data(), sn.size()).parse();
  }
  const Value* nodesV = root.get("stateNodes");
  // Active nodes (nodes.Active(): not marked for deletion) enter the problem; the deleting ones only
  // contribute their pods (deletingNodes.Pods, helpers.go:91-95).
  auto sub = std::make_shared<ksjson::Array>();
  auto pods = std::make_shared<ksjson::Array>();
  std::vector<std::vector<int>> nodePods;  // per snapshot node: global pod indices (GetNodePods)
  std::vector<PodH> podMeta;
  // every pod of the snapshot, parsed by worker threads (pods are independent)
  // (arr() of a null pointer's absence is the shared empty array: references stay into the DOM)
  static const Value kNone;
  std::vector<const Value*> allPodV;
  const Value* pendV = root.get("pendingPods");
  for (const Value& v : (pendV ? *pendV : kNone).arr()) allPodV.push_back(&v);
  for (const Value& nv : (nodesV ? *nodesV : kNone).arr())
    if (const Value* ps = nv.get("pods"))
      for (const Value& pv : ps->arr()) allPodV.push_back(&pv);
  std::vector<PodH> allPods(allPodV.size());
  parallel_for((int)allPodV.size(), 256, [&](int i) { allPods[(size_t)i] = parse_pod(*allPodV[(size_t)i]); });
  size_t next = 0;
  if (pendV)
    for (auto& v : pendV->arr()) {
      c.pending.push_back((int)pods->size());
      pods->push_back(v);
      podMeta.push_back(std::move(allPods[next++]));
    }
  std::map<std::string, int> nodeByName;
  std::vector<char> deletingNode;
  int ni = 0;
  for (const Value& nv : (nodesV ? *nodesV : kNone).arr()) {
    const std::string name = jstr(&nv, "name");
    const bool del = nv.get("markedForDeletion") ? nv.get("markedForDeletion")->boolean(false) : false;
    nodeByName[name] = ni++;
    deletingNode.push_back(del);
    if (nv.get("nominated") && nv.get("nominated")->boolean(false)) c.nominated.insert(name);
    if (!del) sub->push_back(nv);
    std::vector<int> mine;
    if (const Value* ps = nv.get("pods"))
      for (auto& pv : ps->arr()) {
        PodH& p = allPods[next++];
        if (p.ownedByNode || p.ownedByDaemonSet || p.terminal || p.deleting) continue;  // node.go:32-53
        mine.push_back((int)pods->size());
        pods->push_back(pv);
        podMeta.push_back(std::move(p));
      }
    nodePods.push_back(mine);
  }
  for (size_t i = 0; i < nodePods.size(); i++)
    if (deletingNode[i]) for (int p : nodePods[i]) c.deleting.push_back(p);

  pt.mark("parse pods + nodes");
  // the Solve snapshot the problem is encoded from
  Value solveRoot;
  solveRoot.kind = Value::Obj;
  solveRoot.o = std::make_shared<ksjson::Object>(root.obj());
  Value a1, a2;
  a1.kind = a2.kind = Value::Arr;
  a1.a = sub;
  a2.a = pods;
  (*solveRoot.o)["stateNodes"] = a1;
  (*solveRoot.o)["pods"] = a2;
  c.pb.reset(new ks_problem());
  Host& h = c.pb->host;
  // NewTopology excludes the pods a simulation schedules (topology.go:72-75).  The pending and the
  // deleting nodes' pods are in every simulation; the candidates' pods are taken out per simulation
  // (prepare_launch), from the contributions the build records.
  std::set<std::string> always;
  for (int p : c.pending) always.insert(podMeta[(size_t)p].uid);
  for (int p : c.deleting) always.insert(podMeta[(size_t)p].uid);
  h.topoExcluded = &always;
  h.preParsedPods = &podMeta;  // the Solve snapshot's "pods", already parsed above (moved into h.pods)
  h.build(solveRoot);
  h.topoExcluded = nullptr;
  h.preParsedPods = nullptr;
  const std::vector<PodH>& podH = h.pods;
  pt.mark("Host::build");
  if (h.dims.dupUids) throw KsError(KS_ERR_UNSUPPORTED, "consolidation snapshot has duplicate pod UIDs");
  // (a pod whose VolumeTopology.Inject fails stays out of every simulation's NewTopology pod list,
  // provisioner.go:432-442: it is not excluded from the counts, ks_topo.cpp, and sim_topology leaves its
  // contributions in place when its node is a candidate)
  c.hostnameSeed = h.hostnameSeed;
  std::map<std::string, int> hostNode;  // node name -> host.nodes index (sorted order)
  for (size_t i = 0; i < h.nodes.size(); i++) hostNode[h.nodes[i].name] = (int)i;

  // NodePools: expireAfter for lifetimeRemaining; consolidationPolicy (CRD default WhenUnderutilized) and
  // consolidateAfter ("Never": a NillableDuration with a nil Duration) for ShouldDisrupt
  std::map<std::string, int64_t> expire;
  std::set<std::string> poolNames, policyOff, afterNever;
  if (const Value* ps = root.get("nodePools"))
    for (auto& v : ps->arr()) {
      const std::string name = jstr(v.get("metadata"), "name");
      poolNames.insert(name);
      const Value* d = v.get("spec") ? v.get("spec")->get("disruption") : nullptr;
      int64_t ns = 0;
      if (d && d->get("expireAfter") && d->get("expireAfter")->is_str() && go_duration(d->get("expireAfter")->str(), ns))
        expire[name] = ns;
      if (d && d->get("consolidationPolicy") && d->get("consolidationPolicy")->is_str() &&
          d->get("consolidationPolicy")->str() != "WhenUnderutilized")
        policyOff.insert(name);
      if (d && d->get("consolidateAfter") && d->get("consolidateAfter")->is_str() && d->get("consolidateAfter")->str() == "Never")
        afterNever.insert(name);
    }
  std::map<std::string, std::map<std::string, int>> poolTypes;
  if (const Value* bp = root.get("instanceTypesByNodePool"))
    for (auto& kv : bp->obj())
      for (auto& x : kv.second.arr()) {
        const int64_t i = x.i64();
        if (i < 0 || i >= (int64_t)h.its.size()) throw KsError(KS_ERR_PARSE, "instanceTypesByNodePool index out of range");
        poolTypes[kv.first][h.its[(size_t)i].name] = (int)i;
      }
  const int64_t nowNs = parse_rfc3339(jstr(&root, "now")) * 1000000000;
  const std::vector<Pdb> pdbs = parse_pdbs(root);

  // per pod: where it is, its eviction cost and whether it blocks its node (filterCandidates, helpers.go:47-71:
  // a PDB allowing no eviction or a do-not-disrupt pod); bit 1 is the verdict for a pending pod once bound
  // and Running (ks_cons_update), when a Ready=False condition no longer applies
  const int P = (int)podH.size();
  c.podNode.assign((size_t)P, ks_cons::PN_GONE);
  c.podBlock.assign((size_t)P, 0);
  c.podCost.assign((size_t)P, 0.0);
  c.nodePods.assign(h.nodes.size(), {});
  c.nodeGone.assign(h.nodes.size(), 0);
  for (int p : c.pending) c.podNode[(size_t)p] = ks_cons::PN_PENDING;
  for (int p : c.deleting) c.podNode[(size_t)p] = ks_cons::PN_DELETING;
  for (const auto& kv : nodeByName) {
    if (deletingNode[(size_t)kv.second]) continue;
    auto hn = hostNode.find(kv.first);
    if (hn == hostNode.end()) continue;
    c.nodePods[(size_t)hn->second] = nodePods[(size_t)kv.second];
    for (int p : nodePods[(size_t)kv.second]) c.podNode[(size_t)p] = hn->second;
  }
  parallel_for(P, 1024, [&](int p) {
    const PodH& ph = podH[(size_t)p];
    c.podCost[(size_t)p] = eviction_cost(ph);
    const bool dnd = do_not_disrupt(ph);
    uint8_t b = (!can_evict(pdbs, ph) || dnd) ? 1 : 0;
    if (ph.notReady) {
      PodH ready = ph;
      ready.notReady = false;
      b |= (!can_evict(pdbs, ready) || dnd) ? 2 : 0;
    } else {
      b |= b << 1;
    }
    c.podBlock[(size_t)p] = b;
  });

  // NewCandidate for the listed nodes; nodes that would fail it are not candidates
  if (const Value* cs = root.get("candidates"))
    for (auto& v : cs->arr()) {
      const std::string name = v.str();
      auto it = nodeByName.find(name);
      if (it == nodeByName.end()) continue;
      const Value& nv = nodesV->arr()[(size_t)it->second];
      if (deletingNode[(size_t)it->second]) continue;
      auto hn = hostNode.find(name);
      if (hn == hostNode.end()) continue;
      const Host::Node& n = h.nodes[(size_t)hn->second];
      if (!n.initialized) continue;
      const Value* ann = nv.get("annotations");
      if (ann && ann->is_obj() && ann->get("karpenter.sh/do-not-disrupt")) continue;  // types.go:78-81 (key presence)
      auto lct = n.labels.find(kCTKey), lz = n.labels.find(kZoneKey), lp = n.labels.find(kPoolKey);
      if (lct == n.labels.end() || lz == n.labels.end() || lp == n.labels.end()) continue;
      auto pt = poolTypes.find(lp->second);
      if (!poolNames.count(lp->second) || pt == poolTypes.end()) continue;
      auto lit = n.labels.find(kITKey);
      if (lit == n.labels.end() || !pt->second.count(lit->second)) continue;
      if (c.nominated.count(name)) continue;  // types.go:110-113
      // ShouldDisrupt: consolidation.go:96-108 for the pass; validation.go:112-118 (no consolidateAfter
      // test) admits the rest for mapCandidates after the wait
      if (ann && ann->is_obj() && jstr(ann, "karpenter.sh/do-not-consolidate") == "true") continue;
      if (policyOff.count(lp->second)) continue;
      ks_cons::CandIn ci;
      ci.passOk = !afterNever.count(lp->second);
      ks_cons::Cand& k = ci.k;
      k.node = hn->second;
      k.name = name;
      k.pool = lp->second;
      k.ct = lct->second;
      k.zone = lz->second;
      k.it = pt->second.at(lit->second);
      auto ex = expire.find(k.pool);  // lifetimeRemaining types.go:136-145
      if (ex != expire.end()) {
        const int64_t created = parse_rfc3339(jstr(&nv, "creationTimestamp")) * 1000000000;
        const double age = dur_seconds(nowNs - created), total = dur_seconds(ex->second);
        ci.remaining = clampf(0.0, (total - age) / total, 1.0);
      }
      c.candIn.push_back(std::move(ci));
    }
  pt.mark("candidates");
  order_candidates(c);
  c.recWords = rec_words(h.dims.TW);
  pt.mark("sort + sims");
}

// Offerings.Get(capacityType, zone) (all offerings, available or not): first match
bool offering_price(const Host::IT& it, const std::string& ct, const std::string& zone, double& price) {
  for (auto& o : it.all)
    if (o.ct == ct && o.zone == zone) {
      price = o.price;
      return true;
    }
  return false;
}

// One simulation's NewTopology (topology.go:61-85) relative to the shared counts: the candidates'
// pods are excluded from countDomains and from the inverse anti-affinities (topology.go:190-203,
// 262-265), and the candidates' hostnames are no longer registered by NewExistingNode
// (existingnode.go:60).  Returns (tg_cnt offset, (pods removed << 1) | unregister-if-zero) pairs,
// one per touched domain; `dead` gets the inverse groups none of whose owners is in the simulation.
void late_only_groups(const Host& h, int p, std::vector<int32_t>& out);
void topo_index(ks_cons& c);

// Per pod of the handle: its cluster contributions and owned inverse groups (the UID-keyed maps resolved once
// per launch plan, so the simulations' sim_topology calls -- run in parallel -- do no string lookups).
struct PodTopo {
  std::vector<const std::vector<std::pair<int, int>>*> contrib;
  std::vector<const std::vector<int32_t>*> inv;
};
PodTopo pod_topo(const Host& h) {
  PodTopo t;
  const int P = (int)h.pods.size();
  t.contrib.assign((size_t)P, nullptr);
  t.inv.assign((size_t)P, nullptr);
  parallel_for(P, 1024, [&](int p) {
    const std::string& uid = h.pods[(size_t)p].uid;
    auto ct = h.topoContrib.find(uid);
    if (ct != h.topoContrib.end()) t.contrib[(size_t)p] = &ct->second;
    auto io = h.topoInvOwner.find(uid);
    if (io != h.topoInvOwner.end()) t.inv[(size_t)p] = &io->second;
  });
  return t;
}

// `start` (null: every pod's first state): the relaxation state each pod starts the simulation in (a probe re-run
// from carried pod objects, carry_walk).  `act` gets the groups in t.topologies when the simulation starts: those
// Topology.Update creates for its pods' starting states (topology.go:91-122), every inverse group.  The others
// join when a relaxation's Update creates them (k_solve topo_activate_state), with a late group's NewTopology
// state: the existing nodes' hostnames not registered (NewExistingNode ran before it existed, existingnode.go:60).
// The shared count table holds each group in the form the whole problem's build gave it (ks_topo.cpp: late = no
// pod's first state creates it); a hostname group this simulation creates in the other form gets per-node
// entries that register (or unregister) those hostnames -- only for groups some relaxation in the simulation can
// still create, the others are never read.
// `md` gets this simulation's minDomains overrides (group, value): a spread group takes the minDomains of the
// pod whose Update creates it (its Hash leaves minDomains out, topologygroup.go:142-158), the first simulation
// pod, in NewTopology's Update order (the pods list: pending, the candidates', the deleting nodes'), whose
// starting state owns it; a group only a relaxation creates takes its relaxing pod's (refused when those differ).
// `altGroups`: the groups some state gives another minDomains (PodState::gmd; empty: nothing to do);
// `anyInjFailed`: some pod's volume injection failed (Host::injectFailed) -- both once per launch plan.
std::vector<int32_t> sim_topology(const ks_cons& c, const ks_cons::Sim& sm, const std::vector<int>& simPods,
                                  const PodTopo& pt, std::vector<uint64_t>& dead, std::vector<uint64_t>& act,
                                  const std::vector<int32_t>* start, const std::vector<int>& altGroups,
                                  bool anyInjFailed, std::vector<int32_t>& md) {
  const Host& h = c.pb->host;
  const KsDims& d = h.dims;
  const int GMW = d.GMW;
  const int hostKey = h.keyId.count("kubernetes.io/hostname") ? h.keyId.at("kubernetes.io/hostname") : -1;
  // the owned groups at the start (act) and those a later relaxation state of a simulation pod owns (later)
  std::vector<uint64_t> later((size_t)GMW, 0);
  act.assign((size_t)GMW, 0);
  for (int p : simPods) {
    const int s0 = h.tab.pod_state0[(size_t)p], sEnd = s0 + h.tab.pod_nstate[(size_t)p];
    const int s = start ? (*start)[(size_t)p] : s0;
    for (int w = 0; w < GMW; w++) act[(size_t)w] |= h.tab.st_gown[(size_t)s * GMW + w];
    for (int k = s + 1; k < sEnd; k++)
      for (int w = 0; w < GMW; w++) later[(size_t)w] |= h.tab.st_gown[(size_t)k * GMW + w];
  }
  for (int g = d.G1; g < 64 * GMW; g++) act[(size_t)(g >> 6)] |= 1ull << (g & 63);  // inverse groups (and unused bits)
  auto simLate = [&](int g) { return g < d.G1 && !((act[(size_t)(g >> 6)] >> (g & 63)) & 1ull); };
  md.clear();
  for (int g : altGroups) {
    auto owns = [&](int s) { return ((h.tab.st_gown[(size_t)s * GMW + (size_t)(g >> 6)] >> (g & 63)) & 1ull) != 0; };
    auto mdOf = [&](int p, int s) {  // the minDomains state s of pod p creates group g with
      for (auto& e : h.states[(size_t)p][(size_t)(s - h.tab.pod_state0[(size_t)p])].gmd)
        if (e.first == g) return e.second;
      return h.groups[(size_t)g].minDomains;
    };
    int32_t v = INT32_MIN;
    bool found = false;
    for (int p : simPods) {  // the creator at NewTopology time
      const int s = start ? (*start)[(size_t)p] : h.tab.pod_state0[(size_t)p];
      if (owns(s)) {
        v = mdOf(p, s);
        found = true;
        break;
      }
    }
    if (!found) {  // created by a relaxation, if at all: every possible creator must agree
      for (int p : simPods) {
        const int s0 = h.tab.pod_state0[(size_t)p], sEnd = s0 + h.tab.pod_nstate[(size_t)p];
        for (int k = (start ? (*start)[(size_t)p] : s0) + 1; k < sEnd; k++) {
          if (!owns(k)) continue;
          const int32_t x = mdOf(p, k);
          if (found && x != v)
            throw KsError(KS_ERR_UNSUPPORTED, "a simulation's topology group is created by relaxations whose spread "
                                              "constraints differ in minDomains");
          v = x;
          found = true;
        }
      }
    }
    if (found && v != h.groups[(size_t)g].minDomains) {
      md.push_back(g);
      md.push_back(v);
    }
  }
  std::vector<std::pair<int, int>> touched;  // (group, value) per removed pod's contribution (sorted below)
  std::vector<int> ownersGone((size_t)d.G, 0);
  std::set<int> goneHosts;  // hostname value ids of the removed candidates
  for (int ci : sm.cands) {
    const ks_cons::Cand& k = c.cands[(size_t)ci];
    for (int p : k.pods) {
      // NewTopology excludes the pods it receives: not one whose volume injection failed (provisioner.go:432-442),
      // which stays counted where it is bound
      if (anyInjFailed && (size_t)p < h.injectFailed.size() && h.injectFailed[(size_t)p]) continue;
      if (const auto* ct = pt.contrib[(size_t)p]) touched.insert(touched.end(), ct->begin(), ct->end());
      if (const auto* io = pt.inv[(size_t)p])
        for (int32_t g : *io) ownersGone[(size_t)g]++;
    }
    auto hv = hostKey >= 0 ? h.valueId[(size_t)hostKey].find(h.nodes[(size_t)k.node].hostName)
                           : h.valueId[0].end();
    if (hostKey >= 0 && hv != h.valueId[(size_t)hostKey].end()) goneHosts.insert(hv->second);
  }
  std::sort(touched.begin(), touched.end());
  std::vector<std::pair<std::pair<int, int>, int>> dec;  // (group, value) -> pods removed, in (group, value) order
  for (size_t i = 0; i < touched.size();) {
    size_t j = i;
    while (j < touched.size() && touched[j] == touched[i]) j++;
    dec.push_back({touched[i], (int)(j - i)});
    i = j;
  }
  // hostname groups this simulation holds in the other late / initial form than the shared table's: created at
  // its start but late in the table, or late here but not in the table and creatable by one of its relaxations
  std::vector<int> flip;
  if (hostKey >= 0)
    for (int g = 0; g < d.G1; g++) {
      if (h.groups[(size_t)g].keyId != hostKey || simLate(g) == h.groups[(size_t)g].late) continue;
      if (!simLate(g) || ((later[(size_t)(g >> 6)] >> (g & 63)) & 1ull)) flip.push_back(g);
    }
  if (!goneHosts.empty() || !flip.empty()) {  // the removed candidates' hostname domains, touched or not (0 pods removed)
    std::vector<std::pair<std::pair<int, int>, int>> hostOnly;
    auto has = [&](int g, int v) {
      auto it = std::lower_bound(dec.begin(), dec.end(), std::make_pair(std::make_pair(g, v), INT_MIN));
      return it != dec.end() && it->first == std::make_pair(g, v);
    };
    for (int g = 0; g < d.G; g++)
      if (h.groups[(size_t)g].keyId == hostKey)
        for (int v : goneHosts)
          if (!has(g, v)) hostOnly.push_back({{g, v}, 0});
    // (INT_MIN marks a flip entry: its value is derived below)
    for (int g : flip)
      for (const Host::Node& n : h.nodes) {
        auto hv = h.valueId[(size_t)hostKey].find(n.hostName);
        if (hv == h.valueId[(size_t)hostKey].end() || goneHosts.count(hv->second) || has(g, hv->second)) continue;
        hostOnly.push_back({{g, hv->second}, INT_MIN});
      }
    if (!hostOnly.empty()) {
      dec.insert(dec.end(), hostOnly.begin(), hostOnly.end());
      std::sort(dec.begin(), dec.end());
      dec.erase(std::unique(dec.begin(), dec.end(), [](const auto& x, const auto& y) { return x.first == y.first; }),
                dec.end());
    }
  }
  std::vector<int32_t> out;
  for (auto& e : dec) {
    const int g = e.first.first, v = e.first.second;
    const bool host = h.groups[(size_t)g].keyId == hostKey;
    if (v < 0 || v >= h.tab.tg_meta[(size_t)g * TGM_WORDS + TGM_NV])
      throw KsError(KS_ERR_CAPACITY, "topology domain outside its group's value range");
    const int32_t off = h.tab.tg_meta[(size_t)g * TGM_WORDS + TGM_CNT] + v;
    if (e.second == INT_MIN) {  // a node's hostname in a flipped group: registered (0) unless the group is late here
      const int32_t c0 = h.tab.tg_cnt0[(size_t)off];
      const bool uni = h.topoUniverse[(size_t)g][(size_t)v];
      const int32_t want = c0 > 0 ? c0 : (simLate(g) && !uni ? -1 : 0);
      if (want == c0) continue;
      // the prologue stores c0 - (x >> 1), or -1 for a zero with bit 0 set
      out.push_back(off);
      out.push_back(want < 0 ? (c0 << 1) | 1 : (c0 - want) * 2);
      continue;
    }
    // still registered with no pod: a universe domain, or the hostname of a node the simulation keeps
    // (a late group never registered the nodes' hostnames: it was created after NewExistingNode)
    const bool keep = h.topoUniverse[(size_t)g][(size_t)v] || (host && !simLate(g) && h.activeHost(v) && !goneHosts.count(v));
    out.push_back(off);
    out.push_back((e.second << 1) | (keep ? 0 : 1));
  }
  // inverse groups a simulation pod owns (Topology.Update, topology.go:91-122)
  std::vector<uint64_t> simOwn((size_t)GMW, 0);
  for (int p : simPods)
    for (int w = 0; w < GMW; w++) simOwn[(size_t)w] |= h.tab.pod_ginv[(size_t)p * GMW + w];
  dead.assign((size_t)GMW, 0);
  for (int g = d.G1; g < d.G; g++)
    if (h.topoInvOwners[(size_t)g] - ownersGone[(size_t)g] <= 0 && !gtest(simOwn, 0, GMW, g)) gset(dead, 0, GMW, g);
  return out;
}

// Build and upload the launch of this rank's simulations (cached per (rank, world)).
void prepare_launch(ks_cons& c, int rank, int world) {
  if (c.L.lrank == rank && c.L.lworld == world) return;
  PhaseTimer pt("prepare_launch");
  c.invalidate_launch();
  ks_problem& pb = *c.pb;
  Host& h = pb.host;
  const KsDims& d = h.dims;
  const int R = d.R, N = std::max(d.N, 1), NT = std::max(d.NTPL, 1), NP = std::max(d.NPOOL, 1);
  std::vector<int> mine;
  for (int s = rank; s < (int)c.sims.size(); s += world) mine.push_back(s);
  const int ns = (int)mine.size();
  c.L.lsims = mine;
  // per-node capacity in device units (limits are restored for the removed candidates)
  auto nodeCap = [&](int node, int r) -> int64_t {
    auto it = h.nodes[(size_t)node].capacity.find(h.resNames[(size_t)r]);
    return it == h.nodes[(size_t)node].capacity.end() ? 0 : h.toDev(r, it->second);
  };
  Arena a;   // device workspaces (zeroed on the device, never staged on the host)
  Arena ai;  // per-simulation inputs (staged and uploaded): removed nodes, limits, prices, topology deltas
  struct Off {
    size_t c_tpl, c_cnt, c_thr, c_host, c_req, c_max, c_rs, c_rem, order, n_req, n_rs, n_slot, queue, pod_state,
        last_len, log_pod, log_tgt, pod_status, pod_fstate, fail_code, fail_host, counters, rm, pool0, st_price, n_hp,
        c_hp, tg_cnt, tg_ccnt, tg_cpos, tdel, tdead, tact, tmd, sstart, n_vslot, n_vc, vlog, vspec;
  };
  std::vector<Off> offs(ns);
  std::vector<int> simP(ns), entBeg(ns + 1, 0);
  std::vector<int32_t> entries, entrySim;
  std::vector<std::vector<int32_t>> tdel(ns);
  std::vector<std::vector<uint64_t>> tdead(ns), tact(ns);
  std::vector<std::vector<int32_t>> tmd(ns);
  std::vector<std::vector<int>> simPods(ns);
  // the leading multi-node prefixes (the long simulations): a topology plan builds the others' deltas while these
  // run (Launch::pipeB; KS_NO_PIPE=1: all before the launch)
  int nA = 0;
  while (nA < ns && c.sims[(size_t)mine[(size_t)nA]].multi) nA++;
  const bool pipe = d.G && nA > 0 && nA < ns && !std::getenv("KS_NO_PIPE");
  const int nTopo = pipe ? nA : ns;
  parallel_for(ns, 16, [&](int k) {
    const ks_cons::Sim& sm = c.sims[(size_t)mine[(size_t)k]];
    std::vector<int>& pods = simPods[k];
    pods = c.pending;
    for (int ci : sm.cands) pods.insert(pods.end(), c.cands[(size_t)ci].pods.begin(), c.cands[(size_t)ci].pods.end());
    pods.insert(pods.end(), c.deleting.begin(), c.deleting.end());
  });
  if (d.G) {  // every simulation's NewTopology deltas, independent per simulation
    if (c.podContrib.size() != h.pods.size()) {
      PodTopo t = pod_topo(h);
      c.podContrib.swap(t.contrib);
      c.podInv.swap(t.inv);
    }
    PodTopo ptopo;
    ptopo.contrib.swap(c.podContrib);
    ptopo.inv.swap(c.podInv);
    if (!c.altBuilt) {
      std::vector<char> alt((size_t)d.G, 0);
      for (auto& chain : h.states)
        for (auto& st : chain)
          for (auto& e : st.gmd) alt[(size_t)e.first] = 1;
      c.altGroups.clear();
      for (int g = 0; g < d.G; g++)
        if (alt[(size_t)g]) c.altGroups.push_back(g);
      c.altBuilt = true;
    }
    const std::vector<int>& altGroups = c.altGroups;
    const bool anyInjFailed = std::find(h.injectFailed.begin(), h.injectFailed.end(), 1) != h.injectFailed.end();
    pt.mark("minDomains groups");
    std::vector<std::exception_ptr> err((size_t)ns);
    parallel_for(nTopo, 4, [&](int k) {
      try {
        tdel[k] = sim_topology(c, c.sims[(size_t)mine[(size_t)k]], simPods[k], ptopo, tdead[k], tact[k], c.carryStart,
                               altGroups, anyInjFailed, tmd[k]);
      } catch (...) {
        err[(size_t)k] = std::current_exception();
      }
    });
    for (auto& e : err)
      if (e) {
        c.podContrib.swap(ptopo.contrib);
        c.podInv.swap(ptopo.inv);
        std::rethrow_exception(e);
      }
    c.podContrib.swap(ptopo.contrib);
    c.podInv.swap(ptopo.inv);
  }
  pt.mark("simulation pod lists + topology deltas");
  int maxP = 1;
  for (int k = 0; k < ns; k++) {
    const ks_cons::Sim& sm = c.sims[(size_t)mine[(size_t)k]];
    std::vector<int>& pods = simPods[k];
    simP[k] = (int)pods.size();
    maxP = std::max(maxP, simP[k]);
    for (int p : pods) {
      entries.push_back(p);
      entrySim.push_back(k);
    }
    entBeg[k + 1] = (int)entries.size();
    const size_t P = std::max(simP[k], 1), K = P;
    Off& o = offs[k];
    o.c_tpl = a.add(4 * K);
    o.c_cnt = a.add(4 * K);
    o.c_thr = a.add(4 * K * R);
    o.c_host = a.add(4 * K);
    o.c_req = a.add(8 * K * R);
    o.c_max = a.add(8 * K * R);
    o.c_rs = a.add(4 * K * d.RSW);
    o.c_rem = a.add(4 * K * d.TW);
    o.order = a.add(4 * K);
    o.n_req = a.add(8 * (size_t)N * R);  // indexed by node; written only where a pod lands
    o.n_rs = a.add(4 * P * d.RSW);
    o.n_slot = a.add(4 * (size_t)N);
    o.queue = a.add(4 * P);
    o.pod_state = a.add(4 * P);
    o.last_len = a.add(8 * P);
    o.log_pod = a.add(4 * P);
    o.log_tgt = a.add(4 * P);
    o.pod_status = a.add(4 * P);
    o.pod_fstate = a.add(4 * P);
    o.fail_code = a.add(4 * P * NT);
    o.fail_host = a.add(4 * P * NT);
    o.counters = a.add(8 * CT_NCOUNTERS);
    o.n_hp = a.add(d.hpAny ? 8 * (size_t)N : 8);
    o.c_hp = a.add(8 * K);
    o.rm = ai.add(4 * std::max<size_t>(sm.cands.size(), 1));
    o.pool0 = ai.add(8 * (size_t)NP * R);
    o.st_price = sm.multi ? ai.add(8 * (size_t)std::max(d.T, 1)) : 0;
    if (d.volAny) {  // copy-on-write rows: a node's slot is taken the first time a pod with PVCs lands there
      int64_t vcap = 0;  // the log: every PVC of the simulation's PF_VSHARED pods, at most once per placement
      for (int p : pods)
        if (h.tab.pod_flags[(size_t)p] & PF_VSHARED) vcap += h.tab.pod_vubeg[(size_t)p + 1] - h.tab.pod_vubeg[(size_t)p];
      o.n_vslot = a.add(4 * (size_t)N);
      o.n_vc = a.add(4 * P * std::max(d.VD, 1));
      o.vlog = a.add(8 * (size_t)std::max<int64_t>(vcap, 1));
      o.vspec = a.add(8 * (size_t)std::max<int64_t>(vcap, 1));
    }
    if (d.G) {
      o.tg_cnt = a.add(4 * (size_t)d.tgCntWords);
      o.tg_ccnt = a.add(4 * (size_t)d.G * (P + 1));
      o.tg_cpos = a.add(4 * (size_t)d.G);
      if (k < nTopo) {
        o.tdel = ai.add(8 * std::max<size_t>(tdel[k].size() / 2, 1));
        o.tdead = ai.add(8 * (size_t)d.GMW);
        o.tact = ai.add(8 * (size_t)d.GMW);
        o.tmd = ai.add(4 * std::max<size_t>(tmd[k].size(), 1));
      }
    }
    if (c.carryStart) o.sstart = ai.add(4 * c.carryStart->size());
  }
  c.L.lnent = (int)entries.size();
  const size_t inBase = a.total;
  pt.mark("pod lists + layout");
  // device buffers grow to the largest plan seen and are reused (a plan per update must not pay hipMalloc)
  auto grow = [](auto*& p, size_t& cap, size_t bytes) {
    if (bytes <= cap && p) return;
    if (p) HIPCHK(hipFree((void*)p));
    p = nullptr;
    HIPCHK(hipMalloc((void**)&p, bytes));
    cap = bytes;
  };
  const size_t ne = (size_t)std::max(c.L.lnent, 1), nsz = (size_t)std::max(ns, 1);
  grow(c.L.lbuf, c.L.capBuf, std::max<size_t>(inBase + ai.total, 256));
  char* base = (char*)c.L.lbuf;
  char* ibase = base + inBase;
  grow(c.L.lworks, c.L.capWorks, sizeof(KsWork) * nsz);
  grow(c.L.lrec, c.L.capRec, 4 * (size_t)c.recWords * nsz);
  const size_t hdrBytes = 4 * (size_t)RF_HDR * nsz + 16;  // headers + the two u64 status words
  grow(c.L.lhdr, c.L.capHdr, hdrBytes);
  if (!c.L.hhdr || hdrBytes > c.L.capHhdr) {
    if (c.L.hhdr) HIPCHK(hipHostFree(c.L.hhdr));
    c.L.hhdr = nullptr;
    HIPCHK(hipHostMalloc((void**)&c.L.hhdr, hdrBytes, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void**)&c.L.dhdr, c.L.hhdr, 0));
    c.L.capHhdr = hdrBytes;
  }
  if (!c.L.lst) {  // status words ~0, block counter 0: k_rec_headers leaves them so after every pass
    HIPCHK(hipMalloc((void**)&c.L.lst, 32));
    HIPCHK(hipMemset(c.L.lst, 0xff, 16));
    HIPCHK(hipMemset(c.L.lst + 2, 0, 16));
  }
  if (!c.L.hrec || 4 * (size_t)c.recWords * nsz > c.L.capHrec) {
    if (c.L.hrec) HIPCHK(hipHostFree(c.L.hrec));
    c.L.hrec = nullptr;
    HIPCHK(hipHostMalloc((void**)&c.L.hrec, 4 * (size_t)c.recWords * nsz, hipHostMallocDefault));
    c.L.capHrec = 4 * (size_t)c.recWords * nsz;
  }
  if (ne > c.L.capEnt || !c.L.lentries) {
    size_t cap = 0;  // the per-entry buffers share one capacity
    for (int32_t** q : {&c.L.lentries, &c.L.lentrySim, &c.L.lpodmap, &c.L.lrunlen}) {
      cap = 0;
      grow(*q, cap, 4 * ne);
    }
    cap = 0;
    grow(c.L.lkeys, cap, 16 * ne);
    cap = 0;
    grow(c.L.lvals, cap, 8 * ne);
    c.L.capEnt = ne;
  }
  grow(c.L.lrunw, c.L.capRunw, 8 * (size_t)std::max((c.L.lnent + 63) / 64, 1));
  c.L.ltempBytes = std::max<size_t>(queue_sort_temp_bytes(std::max(c.L.lnent, 1)), 256);
  grow(c.L.ltemp, c.L.capTemp, c.L.ltempBytes);
  pt.mark("device buffers");
  if (c.L.lnent) {
    HIPCHK(hipMemcpy(c.L.lentries, entries.data(), 4 * entries.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c.L.lentrySim, entrySim.data(), 4 * entrySim.size(), hipMemcpyHostToDevice));
  }
  c.L.lrbits = 1;
  while ((1ll << c.L.lrbits) < std::max(d.P, 2)) c.L.lrbits++;
  c.L.lsbits = 1;
  while ((1ll << c.L.lsbits) < std::max(ns, 2)) c.L.lsbits++;

  // per-simulation inputs: removed nodes, limits, prices
  pt.mark("entries upload");
  std::vector<char> stage(ai.total, 0);
  std::vector<int> itName((size_t)std::max(d.T, 1), 0);  // instance type -> dense id of its name
  {
    std::map<std::string, int> ids;
    for (int t = 0; t < d.T; t++) itName[(size_t)t] = ids.emplace(h.its[(size_t)t].name, (int)ids.size()).first->second;
  }
  // per candidate: its offering's price (Offerings.Get(ct, zone), first match) and capacity type
  std::vector<double> candPrice(c.cands.size(), 0.0);
  std::vector<char> candPriceOk(c.cands.size(), 0), candSpot(c.cands.size(), 0);
  for (size_t i = 0; i < c.cands.size(); i++) {
    const ks_cons::Cand& k = c.cands[i];
    candPriceOk[i] = offering_price(h.its[(size_t)k.it], k.ct, k.zone, candPrice[i]) ? 1 : 0;
    candSpot[i] = k.ct == "spot" ? 1 : 0;
  }
  if (c.nodePoolIdx.size() != h.nodes.size()) {
    c.nodePoolIdx.assign(h.nodes.size(), {});
    c.nodeCapDev.assign(h.nodes.size() * (size_t)R, 0);
    for (size_t n = 0; n < h.nodes.size(); n++) {
      auto l = h.nodes[n].labels.find(kPoolKey);
      for (int p = 0; l != h.nodes[n].labels.end() && p < d.NPOOL; p++)
        if (l->second == h.pools[(size_t)p].name) c.nodePoolIdx[n].push_back(p);
      for (int r = 0; r < R; r++) c.nodeCapDev[n * (size_t)R + r] = nodeCap((int)n, r);
    }
  }
  std::vector<KsWork> works(ns);
  const bool noTact = std::getenv("KS_NO_TACT") != nullptr;
  parallel_for(ns, 64, [&](int k) {  // independent per simulation (each writes its own stage slices and work)
    const ks_cons::Sim& sm = c.sims[(size_t)mine[(size_t)k]];
    const Off& o = offs[k];
    std::vector<int32_t> rm;
    for (int ci : sm.cands) rm.push_back(c.cands[(size_t)ci].node);
    std::sort(rm.begin(), rm.end());
    memcpy(stage.data() + o.rm, rm.data(), 4 * rm.size());
    int64_t* pool0 = (int64_t*)(stage.data() + o.pool0);
    std::copy(h.tab.pool_rem0.begin(), h.tab.pool_rem0.begin() + (size_t)NP * R, pool0);
    for (int node : rm)
      for (int p : c.nodePoolIdx[(size_t)node])
        for (int r = 0; r < R; r++)
          if ((h.tab.pool_mask[(size_t)p] >> r) & 1u) pool0[(size_t)p * R + r] += c.nodeCapDev[(size_t)node * R + r];
    KsWork w{};
    // getCandidatePrices (consolidation.go:197-207): float64 sum in candidate order
    double price = 0;
    int cflags = 0;
    bool allSpot = true;
    for (int ci : sm.cands) {
      if (!candPriceOk[(size_t)ci]) {
        cflags |= CF_PRICE_ERR;
        break;
      }
      price += candPrice[(size_t)ci];
    }
    for (int ci : sm.cands) allSpot = allSpot && candSpot[(size_t)ci];
    if (allSpot) cflags |= CF_ALL_SPOT;
    if (sm.multi) {
      cflags |= CF_MULTI;
      // filterOutSameType: the cheapest candidate offering per candidate instance type (by name); names as
      // dense ids (itName)
      std::vector<char> nameSeen(itName.size(), 0), nameHas(itName.size(), 0);
      std::vector<double> nameBest(itName.size(), 0.0);
      std::vector<int> touched;
      for (int ci : sm.cands) {
        const ks_cons::Cand& k = c.cands[(size_t)ci];
        const int id = itName[(size_t)k.it];
        if (!nameSeen[(size_t)id]) {
          nameSeen[(size_t)id] = 1;
          touched.push_back(id);
        }
        if (!candPriceOk[(size_t)ci]) continue;
        const double pr = candPrice[(size_t)ci];
        const double cur = nameHas[(size_t)id] ? nameBest[(size_t)id] : std::numeric_limits<double>::max();
        if (pr < cur) {
          nameBest[(size_t)id] = pr;
          nameHas[(size_t)id] = 1;
        }
      }
      double* st = (double*)(stage.data() + o.st_price);
      for (int t = 0; t < std::max(d.T, 1); t++) {
        const int id = t < d.T ? itName[(size_t)t] : -1;
        // a missing map entry reads as 0; types that are no candidate's are NaN (not filtered)
        st[t] = id >= 0 && nameSeen[(size_t)id] ? (nameHas[(size_t)id] ? nameBest[(size_t)id] : 0.0)
                                               : std::numeric_limits<double>::quiet_NaN();
      }
      w.st_price = (const double*)(ibase + o.st_price);
    }
    w.c_tpl = (int32_t*)(base + o.c_tpl);
    w.c_cnt = (int32_t*)(base + o.c_cnt);
    w.c_thr = (int32_t*)(base + o.c_thr);
    w.c_host = (int32_t*)(base + o.c_host);
    w.c_req = (int64_t*)(base + o.c_req);
    w.c_max = (int64_t*)(base + o.c_max);
    w.c_rs = (uint32_t*)(base + o.c_rs);
    w.c_rem = (uint32_t*)(base + o.c_rem);
    w.order = (int32_t*)(base + o.order);
    w.n_req = (int64_t*)(base + o.n_req);
    w.n_rs = (uint32_t*)(base + o.n_rs);
    w.n_slot = (int32_t*)(base + o.n_slot);
    w.queue = (int32_t*)(base + o.queue);
    w.qorder = nullptr;
    w.pod_state = (int32_t*)(base + o.pod_state);
    w.last_len = (uint64_t*)(base + o.last_len);
    w.log_pod = (int32_t*)(base + o.log_pod);
    w.log_tgt = (int32_t*)(base + o.log_tgt);
    w.pod_status = (int32_t*)(base + o.pod_status);
    w.pod_fstate = (int32_t*)(base + o.pod_fstate);
    w.fail_code = (uint32_t*)(base + o.fail_code);
    w.fail_host = (int32_t*)(base + o.fail_host);
    w.pool_rem = nullptr;
    w.counters = (int64_t*)(base + o.counters);
    w.n_hp = (uint64_t*)(base + o.n_hp);
    w.c_hp = (uint64_t*)(base + o.c_hp);
    w.pod_map = c.L.lpodmap + entBeg[k];
    w.run_len = c.L.lrunlen + entBeg[k];
    w.P = simP[k];
    w.nrm = (int32_t)rm.size();
    w.rm = (const int32_t*)(ibase + o.rm);
    w.pool0 = (const int64_t*)(ibase + o.pool0);
    w.rec = c.L.lrec + (size_t)k * c.recWords;
    w.price = price;
    w.cflags = cflags;
    w.ccs = simP[k] + 1;
    if (d.volAny) {
      w.n_vslot = (int32_t*)(base + o.n_vslot);
      w.n_vc = (int32_t*)(base + o.n_vc);
      w.vlog = (int32_t*)(base + o.vlog);
      w.vspec = (int32_t*)(base + o.vspec);
    }
    if (d.G) {
      w.tg_cnt = (int32_t*)(base + o.tg_cnt);
      w.tg_ccnt = (int32_t*)(base + o.tg_ccnt);
      w.tg_cpos = (int32_t*)(base + o.tg_cpos);
    }
    if (d.G && k < nTopo) {  // (the others' topology inputs: finish_topology)
      memcpy(stage.data() + o.tdel, tdel[k].data(), 4 * tdel[k].size());
      w.tdel = (const int32_t*)(ibase + o.tdel);
      w.ntdel = (int32_t)(tdel[k].size() / 2);
      memcpy(stage.data() + o.tdead, tdead[k].data(), 8 * tdead[k].size());
      w.tdead = (const uint64_t*)(ibase + o.tdead);
      memcpy(stage.data() + o.tact, tact[k].data(), 8 * tact[k].size());
      // (KS_NO_TACT: every group but the problem's late ones active at the start, round 5's form; diagnostics)
      w.tact = noTact ? nullptr : (const uint64_t*)(ibase + o.tact);
      if (!tmd[k].empty()) memcpy(stage.data() + o.tmd, tmd[k].data(), 4 * tmd[k].size());
      w.tmd = (const int32_t*)(ibase + o.tmd);
      w.ntmd = (int32_t)(tmd[k].size() / 2);
    }
    if (c.carryStart) {
      memcpy(stage.data() + o.sstart, c.carryStart->data(), 4 * c.carryStart->size());
      w.sstart = (const int32_t*)(ibase + o.sstart);
    }
    works[k] = w;
  });
  // The workspaces (~120 KB per simulation on C5, mostly the node-indexed copy-on-write request slots)
  // are zeroed on the device; only the inputs cross PCIe.
  pt.mark("per-simulation inputs");
  HIPCHK(hipMemset(c.L.lbuf, 0, inBase));
  if (ai.total) HIPCHK(hipMemcpy(ibase, stage.data(), ai.total, hipMemcpyHostToDevice));
  if (ns) HIPCHK(hipMemcpy(c.L.lworks, works.data(), sizeof(KsWork) * ns, hipMemcpyHostToDevice));
  c.L.lhost = works;
  // LDS plan: a small budget per simulation so several simulations share a CU.  A pass with topology is bound by
  // its longest simulation (a multi-node prefix), not by throughput: its simulations get room for the
  // instance-type tables in LDS (TL) at the price of fewer resident per CU.
  KsDims dd = d;
  dd.Kcap = std::max(1, std::min(maxP, 16384));
  c.L.lplan = make_plan(dd, d.G ? 64 * 1024 : 40 * 1024, true);
  if (c.L.lplan.lds > 80 * 1024 || c.L.lplan.KO < 1) c.L.lplan = make_plan(dd, 160 * 1024 - 256, true);
  if (c.L.lplan.lds > 160 * 1024 || c.L.lplan.KO < 1) throw KsError(KS_ERR_CAPACITY, "simulation state does not fit in LDS");
  // Simulations of at least 256 pods (the multi-node prefixes lead the plan) get 4-wave workgroups in one
  // mixed launch when the plan is chain-bound: its pods number at most kMwChainRatio times its longest
  // simulation's (C5: a rank of world >= 4).  A throughput-bound plan (world 1 or 2) runs single-wave, which is
  // faster there.  KS_SIM_MW=0 / 1 turns this off / on for every plan; KS_SIM_MW_MIN sets the pod
  // threshold (tests).
  constexpr int kMwChainRatio = 30;
  const char* mwEnv = std::getenv("KS_SIM_MW");
  const char* mwMinEnv = std::getenv("KS_SIM_MW_MIN");
  const int mwMin = mwMinEnv ? std::max(1, std::atoi(mwMinEnv)) : 256;
  const bool mwAuto = ns > 0 && (int64_t)c.L.lnent <= (int64_t)kMwChainRatio * simP[0];
  const bool mwWanted = mwEnv ? mwEnv[0] == '1' : mwAuto;
  c.L.lnmw = 0;
  if (mwWanted && sims_mw_supported(pb.dev, c.L.lplan))
    while (c.L.lnmw < ns && simP[(size_t)c.L.lnmw] >= mwMin) c.L.lnmw++;
  c.L.pipeB = pipe;
  c.L.nA = pipe ? nA : 0;
  if (pipe) c.L.podsB.assign(std::make_move_iterator(simPods.begin() + nA), std::make_move_iterator(simPods.end()));
  c.L.lrank = rank;
  c.L.lworld = world;
  pt.mark("zero + upload + LDS plan");
}

// The second phase of a topology plan (Launch::pipeB): the NewTopology deltas of simulations [nA, ns), built on
// the host while [0, nA) run, then their inputs and workspace views copied on stream `st` once `ready` (the plan's
// queue sort and feasibility rows) has passed -- pinned staging, so nothing waits for the running launch.
void finish_topology(ks_cons& c, hipStream_t st, hipEvent_t ready) {
  PhaseTimer pt("finish_topology");
  ks_problem& pb = *c.pb;
  Host& h = pb.host;
  const KsDims& d = h.dims;
  const int nA = c.L.nA, ns = (int)c.L.lsims.size(), nB = ns - nA;
  std::vector<std::vector<int32_t>> tdel((size_t)nB), tmd((size_t)nB);
  std::vector<std::vector<uint64_t>> tdead((size_t)nB), tact((size_t)nB);
  PodTopo ptopo;
  ptopo.contrib.swap(c.podContrib);
  ptopo.inv.swap(c.podInv);
  const bool anyInjFailed = std::find(h.injectFailed.begin(), h.injectFailed.end(), 1) != h.injectFailed.end();
  std::vector<std::exception_ptr> err((size_t)nB);
  parallel_for(nB, 4, [&](int k) {
    try {
      tdel[(size_t)k] = sim_topology(c, c.sims[(size_t)c.L.lsims[(size_t)(nA + k)]], c.L.podsB[(size_t)k], ptopo,
                                     tdead[(size_t)k], tact[(size_t)k], c.carryStart, c.altGroups, anyInjFailed,
                                     tmd[(size_t)k]);
    } catch (...) {
      err[(size_t)k] = std::current_exception();
    }
  });
  c.podContrib.swap(ptopo.contrib);
  c.podInv.swap(ptopo.inv);
  for (auto& e : err)
    if (e) {
      // the first phase's launch is in flight: let it finish before the next call's plan re-zeroes its buffers
      (void)hipStreamSynchronize(pb.stream);
      c.invalidate_launch();
      std::rethrow_exception(e);
    }
  pt.mark("topology deltas");
  Arena at;
  std::vector<size_t> o((size_t)nB * 4);
  for (int k = 0; k < nB; k++) {
    o[(size_t)k * 4 + 0] = at.add(8 * std::max<size_t>(tdel[(size_t)k].size() / 2, 1));
    o[(size_t)k * 4 + 1] = at.add(8 * (size_t)d.GMW);
    o[(size_t)k * 4 + 2] = at.add(8 * (size_t)d.GMW);
    o[(size_t)k * 4 + 3] = at.add(4 * std::max<size_t>(tmd[(size_t)k].size(), 1));
  }
  const size_t bytes = std::max<size_t>(at.total, 256), wbytes = sizeof(KsWork) * (size_t)std::max(nB, 1);
  if (!c.L.ltopoB || bytes > c.L.capTopoB) {
    if (c.L.ltopoB) HIPCHK(hipFree(c.L.ltopoB));
    c.L.ltopoB = nullptr;
    HIPCHK(hipMalloc(&c.L.ltopoB, bytes));
    c.L.capTopoB = bytes;
  }
  if (!c.L.htopoB || bytes > c.L.capHtopoB) {
    if (c.L.htopoB) HIPCHK(hipHostFree(c.L.htopoB));
    c.L.htopoB = nullptr;
    HIPCHK(hipHostMalloc((void**)&c.L.htopoB, bytes, hipHostMallocDefault));
    c.L.capHtopoB = bytes;
  }
  if (!c.L.hworksB || wbytes > c.L.capHworksB) {
    if (c.L.hworksB) HIPCHK(hipHostFree(c.L.hworksB));
    c.L.hworksB = nullptr;
    HIPCHK(hipHostMalloc((void**)&c.L.hworksB, wbytes, hipHostMallocDefault));
    c.L.capHworksB = wbytes;
  }
  char* stage = c.L.htopoB;
  const char* dev = (const char*)c.L.ltopoB;
  parallel_for(nB, 64, [&](int k) {
    const size_t* ok = &o[(size_t)k * 4];
    KsWork& w = c.L.lhost[(size_t)(nA + k)];
    memcpy(stage + ok[0], tdel[(size_t)k].data(), 4 * tdel[(size_t)k].size());
    w.tdel = (const int32_t*)(dev + ok[0]);
    w.ntdel = (int32_t)(tdel[(size_t)k].size() / 2);
    memcpy(stage + ok[1], tdead[(size_t)k].data(), 8 * tdead[(size_t)k].size());
    w.tdead = (const uint64_t*)(dev + ok[1]);
    memcpy(stage + ok[2], tact[(size_t)k].data(), 8 * tact[(size_t)k].size());
    w.tact = std::getenv("KS_NO_TACT") ? nullptr : (const uint64_t*)(dev + ok[2]);
    if (!tmd[(size_t)k].empty()) memcpy(stage + ok[3], tmd[(size_t)k].data(), 4 * tmd[(size_t)k].size());
    w.tmd = (const int32_t*)(dev + ok[3]);
    w.ntmd = (int32_t)(tmd[(size_t)k].size() / 2);
    c.L.hworksB[k] = w;
  });
  HIPCHK(hipStreamWaitEvent(st, ready, 0));  // the plan's queue sort and feasibility rows
  HIPCHK(hipMemcpyAsync(c.L.ltopoB, c.L.htopoB, at.total ? at.total : 8, hipMemcpyHostToDevice, st));
  if (nB) HIPCHK(hipMemcpyAsync(c.L.lworks + nA, c.L.hworksB, sizeof(KsWork) * (size_t)nB, hipMemcpyHostToDevice, st));
  c.L.pipeB = false;
  c.L.podsB.clear();
  pt.mark("inputs staged");
}

std::string names_json(const Host& h, const std::vector<int>& its) {
  std::string o = "[";
  for (size_t i = 0; i < its.size(); i++) {
    if (i) o += ",";
    ksjson::quote(o, h.its[(size_t)its[i]].name);
  }
  return o + "]";
}

std::vector<int> bits_to_its(const Host& h, int tpl, const int32_t* bits) {
  std::vector<int> out;
  const Host::Tpl& t = h.tpls[(size_t)tpl];
  for (int pos = 0; pos < (int)t.its.size(); pos++)
    if (((uint32_t)bits[pos >> 5] >> (pos & 31)) & 1u) out.push_back(t.its[(size_t)pos]);
  return out;
}

// The reference's sequential selection over the simulation records.
// rsOf(sim): NewNodeClaims[0]'s requirement record of simulation `sim` (kept in the workspace of the
// GPU that ran it; ks_cons_needed_sims lists the simulations whose record the output needs).
using RsFn = std::function<const uint32_t*(int)>;
// clk: the methods' timeouts on a virtual clock that advances clk->sim_seconds per simulation the replay
// consults (MultiNodeConsolidation's 1 min, multinodeconsolidation.go:34,99-110; SingleNodeConsolidation's
// 3 min, singlenodeconsolidation.go:29,58-65); null or sim_seconds 0: the clock never passes a timeout.
// The simulation records a decision reads: the gathered records ([rank][slot] layout), or -- after a world-1
// ks_cons_run that kept them in the handle -- their headers (k_rec_headers, already checked on the device),
// the option words of the few records the output renders fetched from the device on first use.
struct RecView {
  const ks_cons& c;
  int world = 1;
  const int32_t* full_ = nullptr;
  const int32_t* hdr_ = nullptr;
  mutable std::map<int, std::vector<int32_t>> fetched;
  const int32_t* head(int sim) const {
    if (full_) return full_ + ((size_t)(sim % world) * c.per_rank(world) + (size_t)(sim / world)) * c.recWords;
    return hdr_ + (size_t)sim * RF_HDR;
  }
  const int32_t* full(int sim) const {
    if (full_) return head(sim);
    std::vector<int32_t>& v = fetched[sim];
    if (v.empty()) {
      v.resize((size_t)c.recWords);
      HIPCHK(hipMemcpy(v.data(), c.L.lrec + (size_t)sim * c.recWords, 4 * (size_t)c.recWords, hipMemcpyDeviceToHost));
    }
    return v.data();
  }
};

// Record invariants (a lost or stale device store becomes a loud error, not a wrong decision): the action
// agrees with the NodeClaim count (computeConsolidation, consolidation.go:113-194: Delete = none, Replace =
// exactly one); NewNodeClaims[0]'s options lie in its template's list and number RF_NOPT; filterByPrice's
// and filterOutSameType's outputs are subsets of their inputs.
void check_record(const Host& h, const int32_t* r, const std::string& what) {
  const KsDims& d = h.dims;
  if (r[RF_ERROR] != KE_OK)
    throw KsError(r[RF_ERROR] == KE_CLAIM_CAP ? KS_ERR_CAPACITY : KS_ERR_INTERNAL,
                  what + " reported kernel error " + std::to_string(r[RF_ERROR]));
  auto bad = [&](const char* m) { throw KsError(KS_ERR_INTERNAL, what + " record check: " + m); };
  if (r[RF_ACTION] < CA_NOOP || r[RF_ACTION] > CA_ERROR) bad("action out of range");
  if (r[RF_NCLAIMS] < 0 || r[RF_HOSTINCR] < r[RF_NCLAIMS]) bad("NodeClaim counts");
  if (r[RF_ACTION] == CA_DELETE && r[RF_NCLAIMS] != 0) bad("Delete with NodeClaims");
  if (r[RF_ACTION] == CA_REPLACE && r[RF_NCLAIMS] != 1) bad("Replace without exactly one NodeClaim");
  if (r[RF_NCLAIMS] == 0) return;
  if (r[RF_TPL] < 0 || r[RF_TPL] >= d.NTPL) bad("template out of range");
  const int nIT = (int)h.tpls[(size_t)r[RF_TPL]].its.size();
  const uint32_t* o = (const uint32_t*)r + RF_HDR;
  int nopt = 0, nprice = 0, nsame = 0;
  for (int w = 0; w < d.TW; w++) {
    const int lo = w * 32;
    const uint32_t valid = nIT >= lo + 32 ? ~0u : nIT > lo ? (1u << (nIT - lo)) - 1u : 0u;
    if (o[w] & ~valid) bad("options beyond the template's list");
    if (o[d.TW + w] & ~o[w]) bad("filterByPrice output not a subset of the options");
    if (o[2 * d.TW + w] & ~o[d.TW + w]) bad("filterOutSameType output not a subset of filterByPrice's");
    nopt += __builtin_popcount(o[w]);
    nprice += __builtin_popcount(o[d.TW + w]);
    nsame += __builtin_popcount(o[2 * d.TW + w]);
  }
  if (nopt != r[RF_NOPT] || nopt == 0) bad("option count");
  if (nprice != r[RF_NPRICE] || nsame != r[RF_NSAME]) bad("price-filter counts");
}

// Every gathered record (full records: checked here; headers: k_rec_headers checked them on the device and left
// its verdict in the two status words).
void check_records(const ks_cons& c, const RecView& rv) {
  static const char* checkName[] = {"", "action out of range", "NodeClaim counts", "Delete with NodeClaims",
                                    "Replace without exactly one NodeClaim", "template out of range",
                                    "options beyond the template's list", "price filter output not a subset of its input",
                                    "option count", "price-filter counts"};
  if (!rv.full_) {
    const uint64_t* status = (const uint64_t*)(rv.hdr_ + (size_t)RF_HDR * c.sims.size());
    if (status[1] != ~0ull) {
      const int s = (int)(status[1] >> 32), e = (int)(uint32_t)status[1];
      throw KsError(e == KE_CLAIM_CAP ? KS_ERR_CAPACITY : KS_ERR_INTERNAL,
                    "simulation " + std::to_string(s) + " reported kernel error " + std::to_string(e));
    }
    if (status[0] != ~0ull) {
      const unsigned k = (unsigned)(uint32_t)status[0];
      throw KsError(KS_ERR_INTERNAL, "simulation " + std::to_string(status[0] >> 32) + " record check (device): " +
                                         (k < 10 ? checkName[k] : "?"));
    }
    return;
  }
  for (size_t s = 0; s < c.sims.size(); s++) check_record(c.pb->host, rv.head((int)s), "simulation " + std::to_string(s));
}

// Decode one relaxation-state readback of a simulation (its workspace's pod_map / pod_state, P entries): the
// states the candidates' pods of prefix [0, mid] were left in become their carried states.
void carry_states(const ks_cons& c, int mid, const std::vector<int32_t>& podmap, const std::vector<int32_t>& state,
                  std::vector<int32_t>& cur, std::vector<char>& moved) {
  const Host& h = c.pb->host;
  std::vector<char> cand(h.pods.size(), 0);
  for (int i = 0; i <= mid; i++)
    for (int p : c.cands[(size_t)i].pods) cand[(size_t)p] = 1;
  for (size_t i = 0; i < podmap.size(); i++) {
    const int g = podmap[i];
    if (g < 0 || (size_t)g >= cand.size() || !cand[(size_t)g]) continue;  // pending / deleting pods: fresh per probe
    const int s0 = h.tab.pod_state0[(size_t)g];
    if (state[i] < s0 || state[i] >= s0 + h.tab.pod_nstate[(size_t)g])
      throw KsError(KS_ERR_INTERNAL, "carried relaxation state outside the pod's chain");
    cur[(size_t)g] = state[i];
    moved[(size_t)g] = state[i] != s0;
  }
}

// One multi-node probe (candidates [0, mid]) in a launch of its own on this GPU, from the relaxation states
// `start` (null: every pod's first state): its record, NewNodeClaims[0]'s requirements and the states its Solve
// left the pods in.  The pass's plan and launch come back afterwards (the re-runs keep their own buffers, c.LR).
void rerun_probe(ks_cons& c, int mid, const std::vector<int32_t>* start, ks_cons::Probe& out,
                 std::vector<int32_t>& podmap, std::vector<int32_t>& state);

std::string decide_json(const ks_cons& c, const RecView& rv, int world, bool allSims, const RsFn& rsOf,
                        bool withCandidates = true, const ks_cons_clock* clk = nullptr, bool withSims = true) {
  const double simS = clk ? clk->sim_seconds : 0.0;
  const Host& h = c.pb->host;
  const KsDims& d = h.dims;
  const ks_cons::Walk& wk = c.walk;
  // a decision key: a simulation of the pass (>= 0), or -(2 + i) for carry_walk's re-run probe i
  auto rec = [&](int key) -> const int32_t* { return key >= 0 ? rv.head(key) : wk.probes[(size_t)(-2 - key)].rec.data(); };
  auto fullOf = [&](int key) -> const int32_t* {
    return key >= 0 ? rv.full(key) : wk.probes[(size_t)(-2 - key)].rec.data();
  };
  auto rsK = [&](int key) -> const uint32_t* { return key >= 0 ? rsOf(key) : wk.probes[(size_t)(-2 - key)].rs.data(); };
  auto candsOf = [&](int key) {
    if (key >= 0) return c.sims[(size_t)key].cands;
    std::vector<int> cs((size_t)wk.probes[(size_t)(-2 - key)].mid + 1);
    for (size_t i = 0; i < cs.size(); i++) cs[i] = (int)i;
    return cs;
  };
  auto multiOf = [&](int key) { return key < 0 || c.sims[(size_t)key].multi; };
  check_records(c, rv);
  if (!wk.valid) throw KsError(KS_ERR_INTERNAL, "decide without the multi-node search (carry_walk)");
  const int n = c.nPass;
  int64_t counter = c.hostnameSeed;
  std::map<int, int64_t> before;  // sim -> hostname counter before it ran
  auto run = [&](int sim) {
    if (before.count(sim)) return;
    before[sim] = counter;
    counter += rec(sim)[RF_HOSTINCR];
  };
  auto candNames = [&](const std::vector<int>& cs) {
    std::string o = "[";
    for (size_t i = 0; i < cs.size(); i++) {
      if (i) o += ",";
      ksjson::quote(o, c.cands[(size_t)cs[i]].name);
    }
    return o + "]";
  };
  auto simJSON = [&](int sim) {
    const int32_t* r = rec(sim);
    std::string o = "{\"candidates\":" + candNames(candsOf(sim)) + ",\"allNonPendingScheduled\":" +
                    ((r[RF_FLAGS] & RB_ALL_SCHEDULED) ? "true" : "false") +
                    ",\"newNodeClaims\":" + std::to_string(r[RF_NCLAIMS]);
    if (r[RF_NCLAIMS] > 0) {
      o += ",\"claim0\":{\"nodePoolName\":";
      ksjson::quote(o, h.tpls[(size_t)r[RF_TPL]].pool);
      o += ",\"instanceTypeOptions\":" + names_json(h, bits_to_its(h, r[RF_TPL], fullOf(sim) + RF_HDR));
      o += ",\"requirementsString\":";
      ksjson::quote(o, h.reqsString(rsK(sim), before.at(sim) + r[RF_HOST]));
      o += "}";
    }
    // the simulation's own computeConsolidation outcome: action, the replacement's options after
    // filterByPrice and (multi-node) after filterOutSameType
    static const char* sact[] = {"no-op", "delete", "replace", "error"};
    o += std::string(",\"action\":\"") + sact[r[RF_ACTION]] + "\"";
    if (r[RF_ACTION] == CA_REPLACE) {
      o += ",\"priceOptions\":" + names_json(h, bits_to_its(h, r[RF_TPL], fullOf(sim) + RF_HDR + d.TW));
      if (multiOf(sim))
        o += ",\"sameTypeOptions\":" + names_json(h, bits_to_its(h, r[RF_TPL], fullOf(sim) + RF_HDR + 2 * d.TW));
    }
    return o + "}";
  };
  // commandJSON: action, candidates, replacement (multi: filterOutSameType's options)
  constexpr int kNone = -1;
  auto cmdJSON = [&](int sim, bool err) {
    if (sim == kNone) return std::string("{\"action\":\"no-op\",\"candidates\":[]") + (err ? ",\"error\":true}" : "}");
    const int32_t* r = rec(sim);
    static const char* act[] = {"no-op", "delete", "replace", "no-op"};
    std::string o = std::string("{\"action\":\"") + act[r[RF_ACTION]] + "\",\"candidates\":" +
                    (r[RF_ACTION] == CA_NOOP || r[RF_ACTION] == CA_ERROR ? std::string("[]") : candNames(candsOf(sim)));
    if (r[RF_ACTION] == CA_REPLACE) {
      const bool multi = multiOf(sim);
      const uint32_t* r0 = rsK(sim);
      std::vector<uint32_t> rs(r0, r0 + d.RSW);
      if (r[RF_FLAGS] & RB_NARROWED) {
        std::vector<uint32_t> spot = h.emptyRec();
        h.addNSR(spot, kCTKey, "In", {"spot"});
        rs_add(h.L, rs.data(), spot.data());
      }
      o += ",\"replacement\":{\"nodePoolName\":";
      ksjson::quote(o, h.tpls[(size_t)r[RF_TPL]].pool);
      o += ",\"instanceTypeOptions\":" + names_json(h, bits_to_its(h, r[RF_TPL], fullOf(sim) + RF_HDR + (multi ? 2 : 1) * d.TW));
      o += ",\"requirements\":[";
      const uint64_t pr = rs_present(rs.data());
      bool first = true;
      for (int k = 0; k < d.NK; k++) {  // FinalizeScheduling dropped the hostname requirement
        if (!bit(pr, k) || k == h.hostKey) continue;
        if (!first) o += ",";
        first = false;
        ksjson::quote(o, h.reqString(rs.data(), k, true, before.at(sim) + r[RF_HOST]));
      }
      o += "]}";
    }
    if (err) o += ",\"error\":true";
    return o + "}";
  };

  std::string o = "{\"candidates\":[";
  if (withCandidates)
    for (int i = 0; i < n; i++) {
      if (i) o += ",";
      o += "{\"name\":";
      ksjson::quote(o, c.cands[(size_t)i].name);
      char buf[64];
      snprintf(buf, sizeof buf, ",\"disruptionCost\":%.17g}", c.cands[(size_t)i].cost);
      o += buf;
    }
  // MultiNodeConsolidation.firstNConsolidationOption: the binary search over the prefix length as carry_walk
  // resolved it (the pass's simulations, and the probes re-run from carried pod objects)
  if (allSims)
    for (int mid = 1; mid <= c.multiHi; mid++) run(c.sim_of_multi(mid));
  auto keyOf = [&](size_t i) { return wk.probes[i].carried ? -2 - (int)i : wk.probes[i].sim; };
  for (size_t i = 0; i < wk.probes.size(); i++) run(keyOf(i));
  const int multiSim = wk.chosen >= 0 ? keyOf((size_t)wk.chosen) : kNone;
  const bool multiErr = wk.err;
  std::string multiSims, multiPath;
  if (withSims) {
    if (allSims) {  // every prefix's simulation from the pass's (pristine) pods
      for (int mid = 1; mid <= c.multiHi; mid++) multiSims += (multiSims.empty() ? "" : ",") + simJSON(c.sim_of_multi(mid));
    } else {  // the probes the reference runs
      for (size_t i = 0; i < wk.probes.size(); i++) multiSims += (i ? "," : "") + simJSON(keyOf(i));
    }
  }
  for (size_t i = 0; i < wk.probes.size(); i++) {
    multiPath += (i ? "," : "") + std::string("{\"mid\":") + std::to_string(wk.probes[i].mid) + ",\"carried\":" +
                 (wk.probes[i].carried ? "true" : "false");
    if (withSims) {
      multiPath += "," + simJSON(keyOf(i)).substr(1);
    } else {
      static const char* sact[] = {"no-op", "delete", "replace", "error"};
      multiPath += std::string(",\"action\":\"") + sact[rec(keyOf(i))[RF_ACTION]] + "\"}";
    }
  }
  // SingleNodeConsolidation.ComputeCommand: the first candidate whose simulation yields an action
  int singleSim = -1;
  std::string singleSims;
  double now = 0;  // ComputeCommand's clock; timeout = start + SingleNodeConsolidationTimeoutDuration
  bool timedOut = false;
  for (int i = 0; i < n; i++) {
    if (singleSim >= 0 && !allSims) break;
    if (clk && singleSim < 0 && !timedOut && now > clk->single_timeout_s) {
      timedOut = true;  // s.clock.Now().After(timeout): abandon with no command
      if (!allSims) break;
    }
    if (!timedOut) now += simS;
    const int sim = c.sim_of_single(i);
    run(sim);
    if (withSims) singleSims += (i ? "," : "") + simJSON(sim);
    const int a = rec(sim)[RF_ACTION];
    if (singleSim >= 0 || timedOut || a == CA_ERROR || a == CA_NOOP) continue;
    singleSim = sim;
  }
  o += "],\"multi\":{\"command\":" + cmdJSON(multiSim, multiErr) + ",\"sims\":[" + multiSims + "],\"path\":[" +
       multiPath + "]}";
  o += ",\"single\":{\"command\":" + cmdJSON(singleSim, false) + ",\"sims\":[" + singleSims + "]}}";
  return o;
}

}  // namespace

namespace {

// The queue sort + simulation kernel over this rank's simulations; records to host or device memory.
// Returns the HIP-event time of both launches on the stream they ran on.
double run_sims(ks_cons& c, int rank, int world, void* records, bool onDevice) {
  PhaseTimer pt("run_sims");
  prepare_launch(c, rank, world);
  ks_problem& pb = *c.pb;
  const int ns = (int)c.L.lsims.size();
  if (!c.ev[0]) {  // the pass's timing events, created once per handle
    HIPCHK(hipEventCreate(&c.ev[0]));
    HIPCHK(hipEventCreate(&c.ev[1]));
  }
  HIPCHK(hipEventRecord(c.ev[0], pb.stream));
  // NewQueue per simulation (queue.go:37-44): the plan's pod lists and the global rank are fixed for the
  // handle, and the kernel only reads pod_map, so one sort per plan serves every pass
  if (!c.L.lsorted) {
    HIPCHK(sim_queue_sort(c.rank, c.L.lentries, c.L.lentrySim, c.L.lnent, c.L.lrbits, c.L.lsbits, c.L.lkeys, c.L.lvals,
                          c.L.ltemp, c.L.ltempBytes, c.L.lpodmap, pb.stream));
    HIPCHK(sim_run_lengths(c.L.lpodmap, c.L.lentrySim, pb.dev.pod_req, pb.dev.pod_s0, pb.dev.pod_flags, pb.host.dims.R,
                           c.L.lnent, c.L.lrunw, c.L.lrunlen, pb.stream));
    c.L.lsorted = true;
    pt.mark("queue sort + run lengths enqueued");
  }
  if (c.L.lnmw > 0 && !c.st2) {
    // the long simulations' stream at the highest priority: their workgroups must be dispatched before the
    // 5000 short ones fill the chip, or the pass becomes short ones + long chain instead of their max
    int least = 0, greatest = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIPCHK(hipStreamCreateWithPriority(&c.st2, hipStreamNonBlocking, greatest));
    HIPCHK(hipEventCreateWithFlags(&c.evFork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c.evJoin, hipEventDisableTiming));
  }
  if (c.L.pipeB) {
    // a new topology plan: the multi-node prefixes start at once, the single-node simulations' inputs are built
    // while they run and launched on the second stream (they fill the CUs the long prefixes leave idle)
    if (!c.st2) {
      int least = 0, greatest = 0;
      HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      HIPCHK(hipStreamCreateWithPriority(&c.st2, hipStreamNonBlocking, greatest));
      HIPCHK(hipEventCreateWithFlags(&c.evFork, hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&c.evJoin, hipEventDisableTiming));
    }
    if (pb.dev.d.fmOn) launch_feasibility(pb.dev, pb.stream);
    if (pb.dev.d.fnOn) launch_feasibility_nodes(pb.dev, pb.stream);
    HIPCHK(hipEventRecord(c.evFork, pb.stream));
    HIPCHK(launch_sims_topo(pb.dev, c.L.lworks, c.L.nA, c.L.lplan, pb.stream));
    pt.mark("first phase launched");
    finish_topology(c, c.st2, c.evFork);
    HIPCHK(launch_sims_topo(pb.dev, c.L.lworks + c.L.nA, ns - c.L.nA, c.L.lplan, c.st2));
    HIPCHK(hipEventRecord(c.evJoin, c.st2));
    HIPCHK(hipStreamWaitEvent(pb.stream, c.evJoin, 0));
  } else {
    HIPCHK(launch_sims_split(pb.dev, c.L.lworks, ns, c.L.lnmw, c.L.lplan, pb.stream, c.st2, c.evFork, c.evJoin));
  }
  HIPCHK(hipEventRecord(c.ev[1], pb.stream));
  pt.mark("launches enqueued");
  // the records follow on the same stream; one synchronisation covers both
  const size_t bytes = 4 * (size_t)c.recWords * ns, all = 4 * (size_t)c.recWords * c.per_rank(world);
  if (onDevice) {
    if (all > bytes) HIPCHK(hipMemsetAsync((char*)records + bytes, 0, all - bytes, pb.stream));
    if (bytes) HIPCHK(hipMemcpyAsync(records, c.L.lrec, bytes, hipMemcpyDeviceToDevice, pb.stream));
  } else if (!records && world == 1 && !std::getenv("KS_CONS_FULL_RECORDS")) {  // records stay in the handle: headers only
    // the headers and status go straight to the host-mapped buffer (no copy); KS_CONS_HDR_COPY stages them in
    // device memory and copies (A/B)
    const bool copy = std::getenv("KS_CONS_HDR_COPY") != nullptr;
    int32_t* out = copy ? c.L.lhdr : c.L.dhdr;
    unsigned long long* sout = (unsigned long long*)(out + (size_t)RF_HDR * ns);
    if (ns == 0) {
      unsigned long long* hs = (unsigned long long*)(c.L.hhdr + (size_t)RF_HDR * ns);
      hs[0] = hs[1] = ~0ull;
    } else {
      HIPCHK(rec_headers(c.L.lrec, ns, c.recWords, pb.host.dims.TW, pb.dev.tpl_it_beg, pb.host.dims.NTPL, out, c.L.lst,
                         (unsigned*)(c.L.lst + 2), sout, pb.stream));
      if (copy)
        HIPCHK(hipMemcpyAsync(c.L.hhdr, c.L.lhdr, 4 * (size_t)RF_HDR * ns + 16, hipMemcpyDeviceToHost, pb.stream));
    }
  } else if (bytes) {
    HIPCHK(hipMemcpyAsync(c.L.hrec, c.L.lrec, bytes, hipMemcpyDeviceToHost, pb.stream));
  }
  pt.mark("record copies enqueued");
  HIPCHK(hipStreamSynchronize(pb.stream));
  pt.mark("synchronized");
  c.L.hdrOnly = !onDevice && !records && world == 1 && !std::getenv("KS_CONS_FULL_RECORDS");
  c.L.keptFull = !onDevice && !records && world == 1 && !c.L.hdrOnly;
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, c.ev[0], c.ev[1]));
  if (!onDevice && records) {  // (records == NULL: they stay in the handle's pinned buffer, host_records)
    memcpy(records, c.L.hrec, bytes);
    if (all > bytes) memset((char*)records + bytes, 0, all - bytes);
  }
  return ms;
}

void rerun_probe(ks_cons& c, int mid, const std::vector<int32_t>* start, ks_cons::Probe& out,
                 std::vector<int32_t>& podmap, std::vector<int32_t>& state) {
  PhaseTimer pt("rerun_probe");
  std::vector<ks_cons::Sim> one(1);
  one[0].multi = true;
  one[0].cands.resize((size_t)mid + 1);
  for (int i = 0; i <= mid; i++) one[0].cands[(size_t)i] = i;
  one.swap(c.sims);
  std::swap(c.L, c.LR);
  c.L.invalidate();  // a new plan every time (the prefix and the starting states change), the buffers stay
  c.carryStart = start;
  auto restore = [&]() {
    c.carryStart = nullptr;
    c.L.invalidate();
    std::swap(c.L, c.LR);
    c.sims.swap(one);
  };
  try {
    out.rec.assign((size_t)c.recWords, 0);
    (void)run_sims(c, 0, 1, out.rec.data(), false);
    check_record(c.pb->host, out.rec.data(), "multi-node probe " + std::to_string(mid) + " (carried)");
    const KsWork& w = c.L.lhost[0];
    const int RSW = c.pb->host.dims.RSW;
    out.rs.clear();
    if (out.rec[RF_NCLAIMS] > 0) {
      out.rs.resize((size_t)RSW);
      HIPCHK(hipMemcpy(out.rs.data(), w.c_rs + (size_t)out.rec[RF_CLAIM] * RSW, 4 * (size_t)RSW, hipMemcpyDeviceToHost));
    }
    podmap.resize((size_t)w.P);
    state.resize((size_t)w.P);
    if (w.P) {
      HIPCHK(hipMemcpy(podmap.data(), w.pod_map, 4 * (size_t)w.P, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(state.data(), w.pod_state, 4 * (size_t)w.P, hipMemcpyDeviceToHost));
    }
    pt.mark("launch + readback");
  } catch (...) {
    restore();
    throw;
  }
  restore();
}

// firstNConsolidationOption (multinodeconsolidation.go:87-137) over the pass's records, with the reference's pod
// objects: NewCandidate lists each candidate's pods once per pass (types.go:114-126) and every probe appends
// those same *v1.Pod pointers to its simulation (helpers.go:102-104); a probe's Solve relaxes them in place
// (Preferences.Relax, preferences.go:60-147) and nothing deep-copies them, so a pod one probe relaxed starts the
// next probe in that relaxation state.  (The in-place sort of preferred node-affinity terms, requirements.go:
// 89-91, and VolumeTopology.Inject's re-appended requirements, volumetopology.go:68-71, leave every requirement
// set as it was.)  A probe none of whose candidates' pods an earlier probe relaxed is the pass's own simulation
// of its prefix; one that holds such a pod runs again on this GPU from the carried states (rerun_probe).  A probe
// whose record says it relaxed a pod (RB_RELAXED) hands its final states on: read back from this handle's
// workspace when this rank ran it, else from a re-run of it here.  Most passes relax nothing on the search path
// and launch nothing.
void carry_walk(ks_cons& c, const RecView& rv, int world, const ks_cons_clock* clk) {
  ks_cons::Walk& wk = c.walk;
  if (wk.valid && wk.pass == c.passId && wk.world == world && wk.hasClock == (clk != nullptr) &&
      (!clk || (wk.clock[0] == clk->multi_timeout_s && wk.clock[1] == clk->single_timeout_s &&
                wk.clock[2] == clk->sim_seconds)))
    return;
  PhaseTimer pt("carry_walk");
  check_records(c, rv);
  wk = ks_cons::Walk{};
  const Host& h = c.pb->host;
  const int P = (int)h.pods.size();
  // the carried relaxation state per pod and whether an earlier probe relaxed it; built at the first relaxation
  // on the path (most passes have none: no per-pass work proportional to the pods)
  std::vector<int32_t> cur;
  std::vector<char> moved;
  auto carrying = [&]() {
    if (cur.empty()) {
      cur.assign(h.tab.pod_state0.begin(), h.tab.pod_state0.begin() + P);
      moved.assign((size_t)P, 0);
    }
  };
  std::vector<int32_t> podmap, state;
  const double simS = clk ? clk->sim_seconds : 0.0;
  double now = 0;  // the search's clock; timeout = start + MultiNodeConsolidationTimeoutDuration
  int lo = 1, hi = c.multiHi;
  while (c.multiHi >= 1 && lo <= hi) {
    if (clk && now > clk->multi_timeout_s) break;  // m.clock.Now().After(timeout): lastSavedCommand
    now += simS;
    ks_cons::Probe pr;
    pr.mid = (lo + hi) / 2;
    pr.sim = c.sim_of_multi(pr.mid);
    for (int i = 0; i <= pr.mid && !pr.carried && !moved.empty(); i++)
      for (int p : c.cands[(size_t)i].pods)
        if (moved[(size_t)p]) {
          pr.carried = true;
          break;
        }
    const int32_t* r = nullptr;
    if (pr.carried) {
      rerun_probe(c, pr.mid, &cur, pr, podmap, state);
      wk.reruns++;
      r = pr.rec.data();
      carry_states(c, pr.mid, podmap, state, cur, moved);
    } else {
      r = rv.head(pr.sim);
      if (r[RF_FLAGS] & RB_RELAXED) {  // the states its Solve left the candidates' pods in
        int slot = -1;
        if (c.L.lworld == world && world >= 1 && pr.sim % world == c.L.lrank)
          for (size_t k = 0; k < c.L.lsims.size() && slot < 0; k++)
            if (c.L.lsims[k] == pr.sim) slot = (int)k;
        if (slot >= 0) {
          const KsWork& w = c.L.lhost[(size_t)slot];
          podmap.resize((size_t)w.P);
          state.resize((size_t)w.P);
          if (w.P) {
            HIPCHK(hipMemcpy(podmap.data(), w.pod_map, 4 * (size_t)w.P, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(state.data(), w.pod_state, 4 * (size_t)w.P, hipMemcpyDeviceToHost));
          }
        } else {  // another rank ran it: the same simulation here
          ks_cons::Probe tmp;
          rerun_probe(c, pr.mid, nullptr, tmp, podmap, state);
          wk.reruns++;
        }
        carrying();
        carry_states(c, pr.mid, podmap, state, cur, moved);
      }
    }
    wk.probes.push_back(std::move(pr));
    if (r[RF_ACTION] == CA_ERROR) {  // getCandidatePrices failed: ComputeCommand returns the error
      wk.err = true;
      wk.chosen = -1;
      break;
    }
    const bool validReplace = r[RF_ACTION] == CA_REPLACE && r[RF_NSAME] > 0;
    if (validReplace || r[RF_ACTION] == CA_DELETE) {  // filterOutSameType left options, or a Delete
      wk.chosen = (int)wk.probes.size() - 1;
      lo = wk.probes.back().mid + 1;
    } else {
      hi = wk.probes.back().mid - 1;
    }
  }
  wk.valid = true;
  wk.pass = c.passId;
  wk.world = world;
  wk.hasClock = clk != nullptr;
  if (clk) {
    wk.clock[0] = clk->multi_timeout_s;
    wk.clock[1] = clk->single_timeout_s;
    wk.clock[2] = clk->sim_seconds;
  }
  pt.mark("walk");
}

// Validation.IsValid after its wait (validation.go:68-107) + ValidateCommand (:120-180): the handle
// holds the *current* cluster snapshot, `cmd` a command (ks_cons_decide's shape) computed on an
// earlier one.  mapCandidates keeps GetCandidates order while c.cands is in disruption-cost order;
// the simulation cannot observe the difference (its pods follow NewQueue's total order and prices are
// not used).  The one re-simulation runs on the GPU through the same launch path as a pass.
std::string validate_json(ks_cons& c, const Value& cmd) {
  const Host& h = c.pb->host;
  std::vector<std::string> names;
  if (const Value* cs = cmd.get("candidates"))
    for (auto& v : cs->arr()) names.push_back(v.str());
  const std::set<std::string> proposed(names.begin(), names.end());
  const Value* rv = cmd.get("replacement");
  const bool hasReplacement = rv && rv->is_obj();
  std::set<std::string> replacement;  // cmd.replacements[0].InstanceTypeOptions names
  if (hasReplacement)
    if (const Value* its = rv->get("instanceTypeOptions"))
      for (auto& v : its->arr()) replacement.insert(v.str());
  auto out = [](bool valid, const char* reason, const std::string& sim) {
    std::string o = std::string("{\"valid\":") + (valid ? "true" : "false") + ",\"reason\":";
    ksjson::quote(o, reason);
    return o + ",\"sim\":" + (sim.empty() ? std::string("null") : sim) + "}";
  };
  std::vector<int> mapped;  // mapCandidates + filterCandidates (already applied to c.cands by build_cons)
  for (int i = 0; i < (int)c.cands.size(); i++)
    if (proposed.count(c.cands[(size_t)i].name)) mapped.push_back(i);
  if (mapped.size() != names.size()) return out(false, "candidates-changed", "");
  for (int i : mapped)
    if (c.nominated.count(c.cands[(size_t)i].name)) return out(false, "candidate-nominated", "");
  if (mapped.empty()) return out(false, "no-candidates", "");
  // a plan holding only this simulation in a launch of its own; the pass's plan and launch come back
  std::vector<ks_cons::Sim> saved(1);
  saved[0].cands = mapped;
  saved.swap(c.sims);
  ks_cons::Launch pass;
  std::swap(pass, c.L);
  auto restore = [&]() {
    c.free_launch();
    std::swap(pass, c.L);
    c.sims.swap(saved);
  };
  std::vector<int32_t> r((size_t)c.recWords, 0);
  try {
    (void)run_sims(c, 0, 1, r.data(), false);
  } catch (...) {
    restore();
    throw;
  }
  restore();
  if (r[RF_ERROR] != KE_OK)
    throw KsError(r[RF_ERROR] == KE_CLAIM_CAP ? KS_ERR_CAPACITY : KS_ERR_INTERNAL,
                  "validation simulation reported kernel error " + std::to_string(r[RF_ERROR]));
  const bool allSched = (r[RF_FLAGS] & RB_ALL_SCHEDULED) != 0;
  const int nclaims = r[RF_NCLAIMS];
  std::string sim = std::string("{\"allNonPendingScheduled\":") + (allSched ? "true" : "false") +
                    ",\"newNodeClaims\":" + std::to_string(nclaims);
  std::set<std::string> simTypes;
  if (nclaims > 0) {
    const std::vector<int> its = bits_to_its(h, r[RF_TPL], r.data() + RF_HDR);
    sim += ",\"claim0\":{\"nodePoolName\":";
    ksjson::quote(sim, h.tpls[(size_t)r[RF_TPL]].pool);
    sim += ",\"instanceTypeOptions\":" + names_json(h, its) + "}";
    for (int t : its) simTypes.insert(h.its[(size_t)t].name);
  }
  sim += "}";
  if (!allSched) return out(false, "pods-unschedulable", sim);
  if (nclaims == 0) return hasReplacement ? out(false, "replacement-not-needed", sim) : out(true, "", sim);
  if (nclaims > 1) return out(false, "multiple-nodeclaims", sim);
  if (!hasReplacement) return out(false, "replacement-needed", sim);
  // instanceTypesAreSubset (validation.go:183-187) over name sets
  for (auto& n : replacement)
    if (!simTypes.count(n)) return out(false, "instance-types-not-subset", sim);
  return out(true, "", sim);
}

// A node's initial HostPortUsage mask (KsDev::n_hp0) over the host-port element classes of the build
// (ks_host.cpp): the classes are re-derived from the persisted pods' ports and universe exactly as the build formed
// them (same signatures, same numbering; checked against the pods' masks), then node n's remaining entries are
// OR-ed in.  ks_cons_update after deleting a pod that holds host ports on n (HostPortUsage.DeletePod,
// hostportusage.go:87-90).
uint64_t node_host_port_mask(const Host& h, int n) {
  const size_t NUH = h.hostPortUniverse.size();
  if (NUH == 0) return 0;
  std::set<std::string> podKeys, ownerKeys;
  for (const PodH& p : h.pods) podKeys.insert(p.ns + "/" + p.name);
  for (const std::string& o : h.hostPortOwner)
    if (!o.empty()) ownerKeys.insert(o);
  std::vector<std::vector<int32_t>> sig(NUH);
  for (size_t i = 0; i < h.pods.size(); i++) {
    const PodH& p = h.pods[i];
    const std::string key = p.ns + "/" + p.name;
    if (p.ports.empty() && !ownerKeys.count(key)) continue;
    for (size_t u = 0; u < NUH; u++) {
      const HostPortH& e = h.hostPortUniverse[u];
      bool hpc = false, hpu = false;
      for (const HostPortH& x : p.ports) {
        hpu = hpu || (e.ip == x.ip && e.port == x.port && e.proto == x.proto && h.hostPortOwner[u].empty());
        hpc = hpc || (x.matches(e) && h.hostPortOwner[u] != key);
      }
      const int code = (hpc ? 1 : 0) | (hpu ? 2 : 0) | (h.hostPortOwner[u] == key ? 4 : 0);
      if (code) sig[u].push_back((int32_t)i * 8 + code);
    }
  }
  std::map<std::vector<int32_t>, int> cls;
  std::vector<int> cl(NUH);
  for (size_t u = 0; u < NUH; u++) cl[u] = cls.emplace(sig[u], (int)cls.size()).first->second;
  std::vector<uint64_t> hpc(h.pods.size(), 0), hpu(h.pods.size(), 0), hpo(h.pods.size(), 0);
  for (size_t u = 0; u < NUH; u++)
    for (int32_t e : sig[u]) {
      if (e & 1) hpc[(size_t)(e >> 3)] |= 1ull << cl[u];
      if (e & 2) hpu[(size_t)(e >> 3)] |= 1ull << cl[u];
      if (e & 4) hpo[(size_t)(e >> 3)] |= 1ull << cl[u];
    }
  for (size_t i = 0; i < h.pods.size(); i++)
    if (hpc[i] != h.tab.pod_hpc[i] || hpu[i] != h.tab.pod_hpu[i] || hpo[i] != h.tab.pod_hpo[i])
      throw KsError(KS_ERR_INTERNAL, "update: host-port classes differ from the build's");
  uint64_t m = 0;
  for (const auto& e : h.nodes[(size_t)n].hostPorts) {
    const std::string owner = podKeys.count(e.first) ? e.first : "";
    size_t u = 0;
    while (u < NUH && !(h.hostPortUniverse[u].ip == e.second.ip && h.hostPortUniverse[u].port == e.second.port &&
                        h.hostPortUniverse[u].proto == e.second.proto && h.hostPortOwner[u] == owner))
      u++;
    if (u == NUH) throw KsError(KS_ERR_INTERNAL, "update: a node's host-port entry is outside the universe");
    m |= 1ull << cl[u];
  }
  return m;
}

// ks_cons_update: the cluster-state events between two passes (state/cluster.go:220-512 UpdatePod /
// DeletePod / DeleteNode) applied to the resident handle, so the next pass needs no re-parse, no
// re-encode and no re-upload of the problem.  Applied in order: deletePods, bindPods (a pending pod now
// bound to an active node, Running and scheduled), removeNodes (with the pods still on them).  The node
// rows move with StateNode.Available() (allocatable minus pod requests, lhs keys only, resources.go
// Subtract), a removed node's capacity returns to its pool's limits (provisioner.go:204-296 re-reads them
// per pass) and the node can take no pod in any simulation.  The candidates and simulations are re-derived
// (order_candidates).  Topology clusters move the shared NewTopology counts with the pods (round 5).  Refused
// (KS_ERR_UNSUPPORTED, nothing applied): in clusters with volume limits, deleting or binding a pod that mounts
// volumes (a snapshot reports a node's VolumeUsage as one union, so a pod's share of it is not known; pods without
// volumes and node removals leave every node's usage as it is), and binding a pod with host ports (its entries
// would need universe elements and classes of their own).  Deleting a pod with host ports drops its node's entries
// (HostPortUsage.DeletePod, node_host_port_mask).
void apply_update(ks_cons& c, const Value& delta, bool device) {
  PhaseTimer pt("ks_cons_update");
  ks_problem& pb = *c.pb;
  Host& h = pb.host;
  const KsDims& d = h.dims;
  const int R = d.R;
  if (!delta.is_obj()) throw KsError(KS_ERR_PARSE, "update is not an object");
  for (const auto& kv : delta.obj())
    if (kv.first != "deletePods" && kv.first != "bindPods" && kv.first != "removeNodes")
      throw KsError(KS_ERR_PARSE, "update: unknown field " + kv.first);
  if (c.uidIndex.empty()) {
    c.uidIndex.reserve(h.pods.size());
    for (size_t i = 0; i < h.pods.size(); i++) c.uidIndex.emplace(h.pods[i].uid, (int)i);
  }
  if (c.nodeIndex.empty()) {
    c.nodeIndex.reserve(h.nodes.size());
    for (size_t i = 0; i < h.nodes.size(); i++) c.nodeIndex.emplace(h.nodes[i].name, (int)i);
  }
  auto podOf = [&](const Value& v) {
    if (!v.is_str()) throw KsError(KS_ERR_PARSE, "update: pod uid is not a string");
    auto it = c.uidIndex.find(v.str());
    if (it == c.uidIndex.end()) throw KsError(KS_ERR_ARG, "update: unknown pod " + v.str());
    return it->second;
  };
  auto nodeOf = [&](const Value* v) {
    if (!v || !v->is_str()) throw KsError(KS_ERR_PARSE, "update: node name is not a string");
    auto it = c.nodeIndex.find(v->str());
    if (it == c.nodeIndex.end() || c.nodeGone[(size_t)it->second])
      throw KsError(KS_ERR_ARG, "update: no active node " + v->str());
    return it->second;
  };
  static const Value kNone;
  const Value* dv = delta.get("deletePods");
  const Value* bv = delta.get("bindPods");
  const Value* rv = delta.get("removeNodes");
  // validate the whole update against the state it will meet, then apply it
  std::vector<int> del, bind, bindNode, rm;
  std::set<int> seenPod, seenNode;
  for (const Value& v : (dv ? *dv : kNone).arr()) {
    const int p = podOf(v);
    if (c.podNode[(size_t)p] == ks_cons::PN_GONE || !seenPod.insert(p).second)
      throw KsError(KS_ERR_ARG, "update: pod " + v.str() + " is already deleted");
    if (d.volAny && h.pods[(size_t)p].volumes)
      throw KsError(KS_ERR_UNSUPPORTED, "update: pod " + v.str() + " mounts volumes in a cluster with volume limits");
    del.push_back(p);
  }
  for (const Value& v : (bv ? *bv : kNone).arr()) {
    if (!v.is_obj() || !v.get("uid")) throw KsError(KS_ERR_PARSE, "update: bindPods entries are {uid, node}");
    const int p = podOf(*v.get("uid")), n = nodeOf(v.get("node"));
    if (c.podNode[(size_t)p] != ks_cons::PN_PENDING || !seenPod.insert(p).second)
      throw KsError(KS_ERR_ARG, "update: pod " + v.get("uid")->str() + " is not pending");
    if (h.pods[(size_t)p].hostPorts) throw KsError(KS_ERR_UNSUPPORTED, "update: pod has host ports");
    if (d.volAny && h.pods[(size_t)p].volumes)
      throw KsError(KS_ERR_UNSUPPORTED, "update: pod mounts volumes in a cluster with volume limits");
    bind.push_back(p);
    bindNode.push_back(n);
  }
  for (const Value& v : (rv ? *rv : kNone).arr()) {
    const int n = nodeOf(&v);
    if (!seenNode.insert(n).second) throw KsError(KS_ERR_ARG, "update: node " + v.str() + " removed twice");
    rm.push_back(n);
  }

  // Topology clusters: the shared NewTopology counts (tg_cnt0, topology.go:61-85) follow the events -- a
  // deleted cluster pod's countDomains and inverse anti-affinity contributions leave, a bound pod's join (it
  // is no longer one every simulation schedules), a removed node's pods leave and its hostname is no longer
  // registered by NewExistingNode.  Groups stay: one no remaining pod owns is never evaluated (only owned
  // groups are checked; an inverse group without owners is dead in every simulation, sim_topology).
  std::vector<std::vector<std::pair<int, int>>> bindContrib(bind.size());
  std::vector<std::vector<int32_t>> bindInv(bind.size());
  std::map<int32_t, int> topoLeave, topoLeaveLate;  // owner counts to take away once the update applies
  std::vector<int> toLate;                          // groups only relaxations create from now on
  if (d.G) {
    for (size_t i = 0; i < bind.size(); i++) {
      PodH cp = h.pods[(size_t)bind[i]];
      cp.nodeName = h.nodes[(size_t)bindNode[i]].name;
      cp.phase = "Running";
      if (!h.topoClusterPod(cp, bindContrib[i], bindInv[i]))
        throw KsError(KS_ERR_UNSUPPORTED, "update: bound pod " + cp.uid +
                                              " counts in a topology domain or inverse group the handle does not hold");
    }
    // A group that a leaving pod's first state creates and that remaining pods own only in later relaxation
    // states is a late group (created mid-Solve, ks_topo.cpp) in a fresh build: it becomes one here (toLate,
    // applied below).  (The simulations do not depend on it: each starts with the groups its own pods' starting
    // states create, sim_topology.)  Per-group owner counts over the remaining pods (built once) make the test
    // proportional to the leaving pods.
    auto lateOnly = [&](int p, std::vector<int32_t>& out) { late_only_groups(h, p, out); };
    if (!c.topoIndexed) topo_index(c);
    std::set<int> rmSet(rm.begin(), rm.end());
    std::set<int> leaving(del.begin(), del.end());
    for (size_t i = 0; i < bind.size(); i++)
      if (rmSet.count(bindNode[i])) leaving.insert(bind[i]);
    for (int n : rm)
      for (int p : c.nodePods[(size_t)n]) leaving.insert(p);
    for (size_t p = 0; p < c.podNode.size() && !rm.empty(); p++)  // (bound pods GetNodePods leaves out)
      if (c.podNode[p] >= 0 && rmSet.count(c.podNode[p])) leaving.insert((int)p);
    std::map<int32_t, int> d0, dl;  // owner counts the leaving pods take away
    std::vector<int32_t> tmp;
    for (int p : leaving) {
      if (c.podNode[(size_t)p] == ks_cons::PN_GONE) continue;
      std::vector<int32_t> s0 = h.states[(size_t)p][0].gown;
      std::sort(s0.begin(), s0.end());
      s0.erase(std::unique(s0.begin(), s0.end()), s0.end());
      for (int32_t g : s0) d0[g]++;
      lateOnly(p, tmp);
      for (int32_t g : tmp) dl[g]++;
    }
    for (auto& e : d0) {
      const int g = e.first;
      const int own0 = c.gOwn0[(size_t)g] - e.second, late = c.gOwnLate[(size_t)g] - (dl.count(g) ? dl[g] : 0);
      if (own0 <= 0 && late > 0 && !h.groups[(size_t)g].late) toLate.push_back(g);
    }
    topoLeave.swap(d0);
    topoLeaveLate.swap(dl);
  }

  pt.mark("validate");
  // From here on the host model is edited in place: any failure (a count that would go below zero, a device
  // upload) leaves it ahead of HBM or half-applied, so the handle refuses every later call (c.broken) instead of
  // simulating a mix.
  try {
  std::set<int> rows;  // node rows to re-derive
  auto move = [&](int n, const PodH& p, int sign) {  // StateNode.Available() after a pod leaves / lands
    Host::Node& hn = h.nodes[(size_t)n];
    for (const auto& kv : p.requests) {
      auto a = hn.available.find(kv.first);
      if (a == hn.available.end()) continue;
      a->second.n += sign * kv.second.n;
    }
    rows.insert(n);
  };
  auto erase = [](std::vector<int>& v, int x) {
    auto it = std::find(v.begin(), v.end(), x);
    if (it != v.end()) v.erase(it);
  };
  std::set<int> hpNodes;  // nodes whose HostPortUsage lost a pod's entries
  for (int p : del) {
    const int32_t where = c.podNode[(size_t)p];
    if (where >= 0) {
      erase(c.nodePods[(size_t)where], p);
      move(where, h.pods[(size_t)p], +1);
      auto& hp = h.nodes[(size_t)where].hostPorts;  // StateNode.hostPortUsage.DeletePod (statenode.go:314-339)
      const std::string key = h.pods[(size_t)p].ns + "/" + h.pods[(size_t)p].name;
      const size_t before = hp.size();
      hp.erase(std::remove_if(hp.begin(), hp.end(), [&](const auto& e) { return e.first == key; }), hp.end());
      if (hp.size() != before) hpNodes.insert(where);
    } else if (where == ks_cons::PN_PENDING) {
      erase(c.pending, p);
    } else if (where == ks_cons::PN_DELETING) {
      erase(c.deleting, p);
    }
    c.podNode[(size_t)p] = ks_cons::PN_GONE;
  }
  for (size_t i = 0; i < bind.size(); i++) {
    const int p = bind[i], n = bindNode[i];
    PodH& ph = h.pods[(size_t)p];
    erase(c.pending, p);
    ph.nodeName = h.nodes[(size_t)n].name;
    ph.phase = "Running";
    ph.provisionable = false;  // IsProvisionable: a bound pod (pkg/utils/pod/scheduling.go:28-34)
    ph.notReady = false;
    c.podBlock[(size_t)p] = (uint8_t)(((c.podBlock[(size_t)p] >> 1) & 1) * 3);
    h.tab.pod_flags[(size_t)p] &= ~PF_PROVISIONABLE;
    c.podNode[(size_t)p] = n;
    if (!(ph.ownedByNode || ph.ownedByDaemonSet || ph.terminal || ph.deleting))  // node.go:32-53
      c.nodePods[(size_t)n].push_back(p);
    move(n, ph, -1);
  }
  bool pools = false;
  for (int n : rm) {
    Host::Node& hn = h.nodes[(size_t)n];
    for (int p : c.nodePods[(size_t)n]) c.podNode[(size_t)p] = ks_cons::PN_GONE;
    for (size_t p = 0; p < c.podNode.size(); p++)  // bound pods GetNodePods leaves out
      if (c.podNode[p] == n) c.podNode[p] = ks_cons::PN_GONE;
    c.nodePods[(size_t)n].clear();
    c.nodeGone[(size_t)n] = 1;
    rows.erase(n);
    // the NodePool's remaining limits: its nodes' capacity is no longer subtracted (ks_host.cpp limits)
    auto l = hn.labels.find(kPoolKey);
    for (size_t q = 0; l != hn.labels.end() && q < h.pools.size(); q++) {
      if (h.pools[q].name != l->second) continue;
      for (auto& kv : h.pools[q].remaining) {
        auto cap = hn.capacity.find(kv.first);
        if (cap == hn.capacity.end()) continue;
        kv.second.n += cap->second.n;
        auto id = h.resId.find(kv.first);
        if (id != h.resId.end()) h.tab.pool_rem0[q * (size_t)R + (size_t)id->second] = h.toDev(id->second, kv.second);
      }
      pools = true;
    }
    int64_t* row = &h.tab.n_avail[(size_t)n * R];
    row[0] = -1;  // Fits fails on any negative total: no pod lands on a removed node
  }
  if (d.G) {
    const int hostKey = h.keyId.count("kubernetes.io/hostname") ? h.keyId.at("kubernetes.io/hostname") : -1;
    auto cnt = [&](int g, int v) -> int32_t& {
      return h.tab.tg_cnt0[(size_t)h.tab.tg_meta[(size_t)g * TGM_WORDS + TGM_CNT] + (size_t)v];
    };
    auto keep = [&](int g, int v) {  // registered with no pod: as sim_topology
      return h.topoUniverse[(size_t)g][(size_t)v] ||
             (h.groups[(size_t)g].keyId == hostKey && !h.groups[(size_t)g].late && h.activeHost(v));
    };
    for (auto& e : topoLeave) c.gOwn0[(size_t)e.first] -= e.second;
    for (auto& e : topoLeaveLate) c.gOwnLate[(size_t)e.first] -= e.second;
    auto leave = [&](const std::string& uid) {
      if (!c.podContrib.empty()) {  // the per-pod cache must not point at erased entries
        auto pi = c.uidIndex.find(uid);
        if (pi != c.uidIndex.end()) {
          c.podContrib[(size_t)pi->second] = nullptr;
          c.podInv[(size_t)pi->second] = nullptr;
        }
      }
      auto ct = h.topoContrib.find(uid);
      if (ct != h.topoContrib.end()) {
        for (auto& gv : ct->second) {
          int32_t& x = cnt(gv.first, gv.second);
          if (x <= 0) throw KsError(KS_ERR_INTERNAL, "update: topology count below zero");
          if (--x == 0 && !keep(gv.first, gv.second)) x = -1;
        }
        h.topoContrib.erase(ct);
      }
      auto io = h.topoInvOwner.find(uid);
      if (io != h.topoInvOwner.end()) {
        for (int32_t g : io->second) h.topoInvOwners[(size_t)g]--;
        h.topoInvOwner.erase(io);
      }
    };
    auto unlist = [&](const std::string& uid) {  // the cluster pod listing loses this pod (swap-remove)
      leave(uid);
      auto it = c.cpIndex.find(uid);
      if (it == c.cpIndex.end()) return;
      const size_t i = (size_t)it->second, last = h.clusterPods.size() - 1;
      const std::string node = h.clusterPods[i].nodeName;
      if (!node.empty()) {
        auto bn = c.cpByNode.find(node);
        if (bn != c.cpByNode.end()) {
          auto& v = bn->second;
          auto f = std::find(v.begin(), v.end(), uid);
          if (f != v.end()) {
            *f = v.back();
            v.pop_back();
          }
        }
      }
      c.cpIndex.erase(it);
      if (i != last) {
        h.clusterPods[i] = std::move(h.clusterPods[last]);
        c.cpIndex[h.clusterPods[i].uid] = (int)i;
      }
      h.clusterPods.pop_back();
    };
    for (int p : del) unlist(h.pods[(size_t)p].uid);  // (leave is idempotent for unlisted UIDs)
    for (size_t i = 0; i < bind.size(); i++) {
      const PodH& ph = h.pods[(size_t)bind[i]];
      unlist(ph.uid);
      for (auto& gv : bindContrib[i]) {
        int32_t& x = cnt(gv.first, gv.second);
        x = x < 0 ? 1 : x + 1;
      }
      if (!bindContrib[i].empty()) h.topoContrib[ph.uid] = bindContrib[i];
      if (!bindInv[i].empty()) {
        for (int32_t g : bindInv[i]) h.topoInvOwners[(size_t)g]++;
        h.topoInvOwner[ph.uid] = bindInv[i];
      }
      if (!c.podContrib.empty()) {
        auto ct = h.topoContrib.find(ph.uid);
        auto io = h.topoInvOwner.find(ph.uid);
        c.podContrib[(size_t)bind[i]] = ct != h.topoContrib.end() ? &ct->second : nullptr;
        c.podInv[(size_t)bind[i]] = io != h.topoInvOwner.end() ? &io->second : nullptr;
      }
      c.cpIndex[ph.uid] = (int)h.clusterPods.size();
      c.cpByNode[ph.nodeName].push_back(ph.uid);
      h.clusterPods.push_back(ph);
    }
    for (int n : rm) {
      const Host::Node& hn = h.nodes[(size_t)n];
      auto bn = c.cpByNode.find(hn.name);
      if (bn != c.cpByNode.end()) {
        const std::vector<std::string> uids = bn->second;
        for (const std::string& u : uids) unlist(u);
        c.cpByNode.erase(hn.name);
      }
      if (hostKey < 0) continue;
      auto hv = h.valueId[(size_t)hostKey].find(hn.hostName);
      if (hv == h.valueId[(size_t)hostKey].end()) continue;
      h.topoHostActive.erase(hv->second);
      for (int g = 0; g < d.G; g++)
        if (h.groups[(size_t)g].keyId == hostKey && cnt(g, hv->second) == 0 && !keep(g, hv->second))
          cnt(g, hv->second) = -1;
    }
    // a group now late: as a fresh build makes it, its domains are the universe's and the counted ones (no
    // NewExistingNode hostname registration, existingnode.go:60, ran after it)
    for (int g : toLate) {
      h.groups[(size_t)g].late = true;
      gset(h.tab.tg_late, 0, d.GMW, g);
      if (h.groups[(size_t)g].keyId != hostKey) continue;
      for (const Host::Node& hn : h.nodes) {
        auto hv = h.valueId[(size_t)hostKey].find(hn.hostName);
        if (hv != h.valueId[(size_t)hostKey].end() && cnt(g, hv->second) == 0 && !keep(g, hv->second))
          cnt(g, hv->second) = -1;
      }
    }
  }
  for (int n : hpNodes) h.tab.n_hp0[(size_t)n] = node_host_port_mask(h, n);
  for (int n : rows) {
    int64_t* row = &h.tab.n_avail[(size_t)n * R];
    for (int r = 0; r < R; r++) row[r] = 0;
    bool never = false;  // a negative total outside the resource universe (ks_host.cpp neverFits)
    for (const auto& kv : h.nodes[(size_t)n].available) {
      auto id = h.resId.find(kv.first);
      if (id != h.resId.end()) row[id->second] = h.toDev(id->second, kv.second);
      else never = never || kv.second.n < 0;
    }
    if (never) row[0] = -1;
  }
  pt.mark("apply");
  order_candidates(c);
  pt.mark("order candidates + plan");
  c.updates++;
  if (!device) return;
  // the changed device tables (a few hundred KB at most; the problem itself stays resident); the next pass
  // builds its plan into the previous plan's buffers
  c.invalidate_launch();
  KsDev& D = pb.dev;
  if (!rows.empty() || !rm.empty())
    HIPCHK(hipMemcpyAsync((void*)D.n_avail, h.tab.n_avail.data(), 8 * h.tab.n_avail.size(), hipMemcpyHostToDevice,
                          pb.stream));
  if (!hpNodes.empty())
    HIPCHK(hipMemcpyAsync((void*)D.n_hp0, h.tab.n_hp0.data(), 8 * h.tab.n_hp0.size(), hipMemcpyHostToDevice,
                          pb.stream));
  if (!bind.empty())
    HIPCHK(hipMemcpyAsync((void*)D.pod_flags, h.tab.pod_flags.data(), 4 * h.tab.pod_flags.size(),
                          hipMemcpyHostToDevice, pb.stream));
  if (d.G && (!del.empty() || !bind.empty() || !rm.empty()))
    HIPCHK(hipMemcpyAsync((void*)D.tg_cnt0, h.tab.tg_cnt0.data(), 4 * h.tab.tg_cnt0.size(), hipMemcpyHostToDevice,
                          pb.stream));
  if (!toLate.empty())
    HIPCHK(hipMemcpyAsync((void*)D.tg_late, h.tab.tg_late.data(), 8 * h.tab.tg_late.size(), hipMemcpyHostToDevice,
                          pb.stream));
  if (pools)
    HIPCHK(hipMemcpyAsync((void*)D.pool_rem0, h.tab.pool_rem0.data(), 8 * h.tab.pool_rem0.size(),
                          hipMemcpyHostToDevice, pb.stream));
  HIPCHK(hipStreamSynchronize(pb.stream));
  pt.mark("upload rows");
  } catch (const std::exception& e) {
    c.broken = e.what();
    throw;
  }
}

// The shared NewTopology state of a topology cluster, keyed by group identity (an FNV-1a digest of the
// group's Hash): per group the registered domains' counts, whether it is late, and whether any pod in the
// simulations' union or any cluster pod owns it (an unowned group is never evaluated).  ks_cons_update
// tests compare the owned groups with a from-scratch build.
std::string topology_json(const ks_cons& c) {
  const Host& h = c.pb->host;
  const KsDims& d = h.dims;
  std::vector<char> owned((size_t)d.G, 0);
  for (size_t p = 0; p < h.pods.size(); p++) {
    if (c.podNode[p] == ks_cons::PN_GONE) continue;
    for (auto& st : h.states[p])
      for (int32_t g : st.gown) owned[(size_t)g] = 1;
    for (int g = d.G1; g < d.G; g++)
      if (gtest(h.tab.pod_ginv, p, d.GMW, g)) owned[(size_t)g] = 1;
  }
  for (int g = d.G1; g < d.G; g++)
    if (h.topoInvOwners[(size_t)g] > 0) owned[(size_t)g] = 1;
  std::string o = "{";
  for (int g = 0; g < d.G; g++) {
    const TopoGroup& tg = h.groups[(size_t)g];
    uint64_t f = 1469598103934665603ull;
    for (unsigned char ch : tg.hash) f = (f ^ ch) * 1099511628211ull;
    f = (f ^ (unsigned)(g >= d.G1)) * 1099511628211ull;  // (an inverse group and an owned one may share a Hash)
    char buf[40];
    snprintf(buf, sizeof buf, "%s\"%016llx\":{", g ? "," : "", (unsigned long long)f);
    o += buf;
    o += std::string("\"late\":") + (tg.late ? "true" : "false") + ",\"owned\":" + (owned[(size_t)g] ? "true" : "false") +
         ",\"counts\":{";
    const int32_t* cnt = &h.tab.tg_cnt0[(size_t)h.tab.tg_meta[(size_t)g * TGM_WORDS + TGM_CNT]];
    bool first = true;
    for (int v = 0; v < h.tab.tg_meta[(size_t)g * TGM_WORDS + TGM_NV]; v++) {
      if (cnt[v] < 0) continue;
      o += first ? "" : ",";
      first = false;
      ksjson::quote(o, h.values[(size_t)tg.keyId][(size_t)v]);
      o += ":" + std::to_string(cnt[v]);
    }
    o += "}}";
  }
  return o + "}";
}

// Groups pod p owns in later relaxation states only (once each; ks_cons_update's late-group test).
void late_only_groups(const Host& h, int p, std::vector<int32_t>& out) {
  out.clear();
  const auto& st = h.states[(size_t)p];
  if (st.size() < 2) return;
  for (size_t k = 1; k < st.size(); k++)
    for (int32_t g : st[k].gown) out.push_back(g);
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  std::vector<int32_t> s0 = st[0].gown;
  std::sort(s0.begin(), s0.end());
  std::vector<int32_t> o2;
  std::set_difference(out.begin(), out.end(), s0.begin(), s0.end(), std::back_inserter(o2));
  out.swap(o2);
}

// The topology update indexes (ks_cons::cpIndex / cpByNode / gOwn0 / gOwnLate), from the host state: at the end
// of build_cons, or at the first update after a binary load.
void topo_index(ks_cons& c) {
  const Host& h = c.pb->host;
  const int G = h.dims.G;
  c.gOwn0.assign((size_t)G, 0);
  c.gOwnLate.assign((size_t)G, 0);
  std::vector<int32_t> tmp, s0;
  for (size_t p = 0; p < h.pods.size(); p++) {
    if (c.podNode[p] == ks_cons::PN_GONE) continue;
    s0 = h.states[p][0].gown;
    if (s0.size() > 1) {
      std::sort(s0.begin(), s0.end());
      s0.erase(std::unique(s0.begin(), s0.end()), s0.end());
    }
    for (int32_t g : s0) c.gOwn0[(size_t)g]++;
    late_only_groups(h, (int)p, tmp);
    for (int32_t g : tmp) c.gOwnLate[(size_t)g]++;
  }
  c.cpIndex.clear();
  c.cpByNode.clear();
  c.cpIndex.reserve(h.clusterPods.size());
  for (size_t i = 0; i < h.clusterPods.size(); i++) {
    c.cpIndex.emplace(h.clusterPods[i].uid, (int)i);
    if (!h.clusterPods[i].nodeName.empty()) c.cpByNode[h.clusterPods[i].nodeName].push_back(h.clusterPods[i].uid);
  }
  c.topoIndexed = true;
}

// Host-only description of a handle: the pass's candidates, the pending pods, the simulation plan and the
// active nodes' encoded rows (ks_cons_inspect, ks_cons_inspect_update).
std::string inspect_json(const ks_cons& c, bool nodes) {
  std::string o = "{\"candidates\":[";
  for (size_t i = 0; i < (size_t)c.nPass; i++) {
    if (i) o += ",";
    o += "{\"name\":";
    ksjson::quote(o, c.cands[i].name);
    char buf[96];
    snprintf(buf, sizeof buf, ",\"disruptionCost\":%.17g,\"pods\":%zu}", c.cands[i].cost, c.cands[i].pods.size());
    o += buf;
  }
  // the pending pods every simulation schedules, as encoded (name + device request vector)
  const Host& h = c.pb->host;
  o += "],\"pendingPods\":[";
  for (size_t i = 0; i < c.pending.size(); i++) {
    const int p = c.pending[i];
    o += i ? ",{\"name\":" : "{\"name\":";
    ksjson::quote(o, h.pods[(size_t)p].name);
    o += ",\"requests\":[";
    for (int r = 0; r < h.dims.R; r++)
      o += (r ? "," : "") + std::to_string(h.tab.pod_req[(size_t)p * h.dims.R + r]);
    o += "]}";
  }
  o += "],\"resources\":[";
  for (int r = 0; r < h.dims.R; r++) {
    if (r) o += ",";
    ksjson::quote(o, h.resNames[(size_t)r]);
  }
  o += "]";
  if (nodes) {
    // per active node: available and the pods GetNodePods yields (by name, in order); per pool: limits left
    o += ",\"nodeRows\":{";
    bool first = true;
    for (size_t n = 0; n < h.nodes.size(); n++) {
      if (c.nodeGone[n]) continue;
      o += first ? "" : ",";
      first = false;
      ksjson::quote(o, h.nodes[n].name);
      o += ":{\"available\":[";
      for (int r = 0; r < h.dims.R; r++) o += (r ? "," : "") + std::to_string(h.tab.n_avail[n * (size_t)h.dims.R + r]);
      o += "],\"pods\":[";
      for (size_t i = 0; i < c.nodePods[n].size(); i++) {
        o += i ? "," : "";
        ksjson::quote(o, h.pods[(size_t)c.nodePods[n][i]].name);
      }
      o += "]}";
    }
    o += "},\"poolRemaining\":[";
    for (size_t i = 0; i < h.tab.pool_rem0.size(); i++) o += (i ? "," : "") + std::to_string(h.tab.pool_rem0[i]);
    o += "]";
    if (h.dims.G) o += ",\"topology\":" + topology_json(c);
  }
  o += ",\"sims\":" + std::to_string(c.sims.size()) + ",\"multiPrefixes\":" + std::to_string(c.multiHi) +
       ",\"recordBytes\":" + std::to_string(4 * c.recWords) + ",\"pods\":" + std::to_string(h.dims.P) +
       ",\"nodes\":" + std::to_string(h.dims.N) + ",\"groups\":" + std::to_string(h.dims.G) +
       ",\"groupsOwned\":" + std::to_string(h.dims.G1) + "}";
  return o;
}

}  // namespace

extern "C" {

// The device half of a consolidation handle: upload + every pod's global NewQueue rank.
static void cons_device_init(ks_cons* c, PhaseTimer& pt) {
  ks_problem& pb = *c->pb;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) throw KsError(KS_ERR_HIP, "no HIP device visible");
  HIPCHK(hipGetDevice(&pb.device));
  HIPCHK(hipStreamCreateWithFlags(&pb.stream, hipStreamNonBlocking));
  pt.mark("device + stream");
  ks_upload(&pb);
  pt.mark("upload");
  // global NewQueue rank of every pod (each simulation's queue is this order restricted to its pods)
  const int P = pb.host.dims.P;
  const size_t np = std::max(P, 1);
  HIPCHK(hipMalloc(&pb.skeys, 2 * np * sizeof(uint64_t)));
  HIPCHK(hipMalloc(&pb.svals, 2 * np * sizeof(int32_t)));
  pb.stempBytes = std::max<size_t>(queue_sort_temp_bytes((int)np), 256);
  HIPCHK(hipMalloc(&pb.stemp, pb.stempBytes));
  int32_t* order = nullptr;
  HIPCHK(hipMalloc(&order, 4 * np));
  HIPCHK(hipMalloc(&c->rank, 4 * np));
  HIPCHK(queue_sort(pb.dev, pb.skeys, pb.svals, pb.stemp, pb.stempBytes, order, pb.stream));
  HIPCHK(rank_from_order(order, c->rank, P, pb.stream));
  HIPCHK(hipStreamSynchronize(pb.stream));
  (void)hipFree(order);
  pt.mark("queue rank");
}

int ks_cons_create(const char* json, size_t len, ks_cons** out) {
  API_TRY
  if (!json || !out) throw KsError(KS_ERR_ARG, "null argument");
  PhaseTimer pt("ks_cons_create");
  ksjson::Value root = ksjson::Parser(json, len ? len : strlen(json)).parse();
  pt.mark("json parse");
  std::unique_ptr<ks_cons> c(new ks_cons());
  build_cons(*c, root);
  ksjson::release_async(std::move(root));
  pt.mark("build_cons");
  cons_device_init(c.get(), pt);
  *out = c.release();
  return KS_OK;
  API_CATCH
}

// --- binary snapshot of a consolidation handle: the host model + candidates + simulation plan ----------
extern "C++" {
namespace ks {
template <class A> void io(A& a, ks_cons::Cand& x) { io_all(a, x.node, x.name, x.pool, x.ct, x.zone, x.it, x.cost, x.pods); }
template <class A> void io(A& a, ks_cons::Sim& x) { io_all(a, x.cands, x.multi); }
template <class A> void io(A& a, ks_cons::CandIn& x) { io_all(a, x.k, x.remaining, x.passOk); }
}  // namespace ks
namespace {
// the format version, with the embedded problem's (KSPROBnn): 05 = round 6 (KSPROB05); 04 = round 5's final
// layout (KSPROB04);
// 03 = round 5's first (KSPROB03); 02 = round 4; 01 = round 3.  Another version is refused (snapshot_check_header).
constexpr char kConsMagic[8] = {'K', 'S', 'C', 'O', 'N', 'S', '0', '5'};
template <class A> void cons_io(A& a, ks_cons& c) {
  io_all(a, c.cands, c.nPass, c.sims, c.multiHi, c.pending, c.deleting, c.nominated, c.hostnameSeed, c.recWords,
         c.candIn, c.nodePods, c.podNode, c.podBlock, c.podCost, c.nodeGone, c.updates);
}
// The loaded plan's indices must lie inside the loaded model (host_check covers the model itself).
void cons_check(const ks_cons& c) {
  const Host& h = c.pb->host;
  auto bad = [](const char* what) { throw ArchiveError(std::string("binary snapshot: inconsistent ") + what); };
  const int P = h.dims.P, N = h.dims.N, NC = (int)c.cands.size();
  if (c.nPass < 0 || c.nPass > NC || c.multiHi < 0 || c.multiHi > c.nPass) bad("candidate counts");
  if (c.recWords != rec_words(h.dims.TW)) bad("record width");
  if ((int)c.sims.size() != c.multiHi + c.nPass) bad("simulation plan");
  for (auto& cd : c.cands) {
    if (cd.node < 0 || cd.node >= N || cd.it < 0 || cd.it >= h.dims.T) bad("candidate node");
    for (int p : cd.pods)
      if (p < 0 || p >= P) bad("candidate pod");
  }
  for (auto& s : c.sims)
    for (int ci : s.cands)
      if (ci < 0 || ci >= c.nPass) bad("simulation candidate");
  for (const std::vector<int>* v : {&c.pending, &c.deleting})
    for (int p : *v)
      if (p < 0 || p >= P) bad("pending / deleting pod");
  if ((int)c.nodePods.size() != N || (int)c.nodeGone.size() != N || (int)c.podNode.size() != P ||
      (int)c.podBlock.size() != P || (int)c.podCost.size() != P)
    bad("update state sizes");
  for (auto& ci : c.candIn)
    if (ci.k.node < 0 || ci.k.node >= N || ci.k.it < 0 || ci.k.it >= h.dims.T) bad("candidate input node");
  for (auto& v : c.nodePods)
    for (int p : v)
      if (p < 0 || p >= P) bad("node pod");
  for (int32_t w : c.podNode)
    if (w < ks_cons::PN_GONE || w >= N) bad("pod placement");
}
}  // namespace
}  // extern "C++"

int ks_cons_save(const ks_cons* c, void** buf, size_t* len) {
  API_TRY
  if (!c || !buf || !len) throw KsError(KS_ERR_ARG, "null argument");
  ArOut a;
  snapshot_header(a, kConsMagic);
  host_save(a, c->pb->host);
  cons_io(a, const_cast<ks_cons&>(*c));
  *buf = snapshot_bytes(a.buf);
  *len = a.buf.size();
  return KS_OK;
  API_CATCH
}

int ks_cons_create_binary(const void* buf, size_t len, ks_cons** out) {
  API_TRY
  if (!buf || !out) throw KsError(KS_ERR_ARG, "null argument");
  PhaseTimer pt("ks_cons_create_binary");
  std::unique_ptr<ks_cons> c(new ks_cons());
  c->pb.reset(new ks_problem());
  try {
    ArIn a{(const char*)buf, (const char*)buf + len};
    snapshot_check_header(a, kConsMagic);
    host_load(a, c->pb->host);
    cons_io(a, *c);
    if (a.p != a.end) throw KsError(KS_ERR_PARSE, "binary snapshot has trailing bytes");
    cons_check(*c);
  } catch (const ArchiveError& e) {
    throw KsError(KS_ERR_PARSE, e.what());
  }
  pt.mark("load");
  cons_device_init(c.get(), pt);
  *out = c.release();
  return KS_OK;
  API_CATCH
}

// Host-only: candidates (NewCandidate + disruption-cost order) and the simulation plan, no device.
int ks_cons_inspect(const char* json, size_t len, char** out) {
  API_TRY
  if (!json || !out) throw KsError(KS_ERR_ARG, "null argument");
  PhaseTimer pt("ks_cons_inspect");
  ksjson::Value root = ksjson::Parser(json, len ? len : strlen(json)).parse();
  pt.mark("json parse");
  ks_cons c;
  build_cons(c, root);
  pt.mark("build_cons");
  root = ksjson::Value();
  pt.mark("json free");
  *out = strdup(inspect_json(c, false).c_str());
  return KS_OK;
  API_CATCH
}

// Host-only: a snapshot with an update applied (ks_cons_update's host half), described with the active
// nodes' rows, to compare against the snapshot the update leads to.
int ks_cons_inspect_update(const char* json, size_t len, const char* update_json, size_t ulen, char** out) {
  API_TRY
  if (!json || !update_json || !out) throw KsError(KS_ERR_ARG, "null argument");
  ksjson::Value root = ksjson::Parser(json, len ? len : strlen(json)).parse();
  ks_cons c;
  build_cons(c, root);
  root = ksjson::Value();
  const ksjson::Value delta = ksjson::Parser(update_json, ulen ? ulen : strlen(update_json)).parse();
  if (delta.kind == ksjson::Value::Arr) {  // a sequence of updates
    for (const ksjson::Value& u : delta.arr()) apply_update(c, u, false);
  } else if (!(delta.is_obj() && delta.obj().empty())) {
    apply_update(c, delta, false);
  }
  *out = strdup(inspect_json(c, true).c_str());
  return KS_OK;
  API_CATCH
}

int ks_cons_update(ks_cons* c, const char* update_json, size_t len) {
  API_TRY
  if (!c || !update_json) throw KsError(KS_ERR_ARG, "null argument");
  c->check_usable();
  DeviceGuard guard(c->pb->device, nullptr);
  const ksjson::Value delta = ksjson::Parser(update_json, len ? len : strlen(update_json)).parse();
  apply_update(*c, delta, true);
  return KS_OK;
  API_CATCH
}

void ks_cons_free(ks_cons* c) { delete c; }

int ks_cons_num_candidates(const ks_cons* c) { return c ? c->nPass : 0; }
int ks_cons_num_sims(const ks_cons* c) { return c ? (int)c->sims.size() : 0; }
int ks_cons_record_bytes(const ks_cons* c) { return c ? 4 * c->recWords : 0; }
int ks_cons_records_per_rank(const ks_cons* c, int world) { return c && world > 0 ? c->per_rank(world) : 0; }

// The gathered records: the caller's, or (NULL) those a world-1 ks_cons_run left in the handle (their headers in
// its pinned buffer).
static RecView host_records(const ks_cons* c, const void* records, int world) {
  RecView v{*c, world};
  if (records) {
    v.full_ = (const int32_t*)records;
    return v;
  }
  if (world != 1 || c->L.lworld != 1 || !(c->L.hdrOnly || c->L.keptFull) || c->L.lsims.size() != c->sims.size())
    throw KsError(KS_ERR_ARG, "records NULL without a world-1 run of every simulation on this handle");
  if (c->L.keptFull) v.full_ = c->L.hrec;  // (KS_CONS_FULL_RECORDS: the whole records were downloaded)
  else v.hdr_ = c->L.hhdr;
  return v;
}

int ks_cons_run(ks_cons* c, int rank, int world, const ks_solve_opts* opts, void* records, int records_on_device,
                double* kernel_ms) {
  API_TRY
  if (!c || (!records && (records_on_device || world != 1)) || world < 1 || rank < 0 || rank >= world)
    throw KsError(KS_ERR_ARG, "bad argument");
  c->check_usable();
  DeviceGuard guard(c->pb->device, opts);
  c->passId++;  // (a decision's multi-node search is re-resolved for the new records)
  const double ms = run_sims(*c, rank, world, records, records_on_device != 0);
  if (kernel_ms) *kernel_ms = ms;
  return KS_OK;
  API_CATCH
}

int ks_cons_validate(ks_cons* c, const char* command_json, size_t len, const ks_solve_opts* opts, char** json_out) {
  API_TRY
  if (!c || !command_json || !json_out) throw KsError(KS_ERR_ARG, "null argument");
  c->check_usable();
  DeviceGuard guard(c->pb->device, opts);
  ksjson::Value cmd = ksjson::Parser(command_json, len ? len : strlen(command_json)).parse();
  if (!cmd.is_obj()) throw KsError(KS_ERR_PARSE, "command is not an object");
  *json_out = strdup(validate_json(*c, cmd).c_str());
  return KS_OK;
  API_CATCH
}

// The simulations whose NewNodeClaims[0] requirement record the decision output needs, in the order
// ks_cons_decide consumes them (a dry run of the replay that records every lookup).
static std::vector<int> needed_sims(const ks_cons& c, const RecView& recs, int world, bool allSims,
                                    const ks_cons_clock* clk = nullptr) {
  std::vector<int> need;
  std::set<int> seen;
  std::vector<uint32_t> zero(std::max(c.pb->host.dims.RSW, 1), 0);
  decide_json(
      c, recs, world, allSims,
      [&](int sim) -> const uint32_t* {
        if (seen.insert(sim).second) need.push_back(sim);
        return zero.data();
      },
      false, clk);
  return need;
}

int ks_cons_requirement_words(const ks_cons* c) { return c ? c->pb->host.dims.RSW : 0; }

int ks_cons_needed_sims(ks_cons* c, const void* records, int world, int flags, int32_t* out, int cap) {
  API_TRY
  if (!c || world < 1) throw KsError(KS_ERR_ARG, "bad argument");
  c->check_usable();
  DeviceGuard guard(c->pb->device, nullptr);
  const RecView recs = host_records(c, records, world);
  carry_walk(*c, recs, world, nullptr);
  std::vector<int> need = needed_sims(*c, recs, world, (flags & KS_CONS_ALL_SIMS) != 0);
  for (int i = 0; i < (int)need.size() && i < cap; i++) out[i] = need[(size_t)i];
  return (int)need.size();
  API_CATCH
}

// NewNodeClaims[0]'s requirement record of simulation `sim` from this handle's last run (the rank
// that ran it).
int ks_cons_claim_requirements(ks_cons* c, int sim, uint32_t* out) {
  API_TRY
  if (!c || !out) throw KsError(KS_ERR_ARG, "bad argument");
  const int RSW = c->pb->host.dims.RSW;
  for (size_t k = 0; k < c->L.lsims.size(); k++)
    if (c->L.lsims[k] == sim) {
      int32_t claim = -1;
      HIPCHK(hipMemcpy(&claim, c->L.lrec + k * c->recWords + RF_CLAIM, 4, hipMemcpyDeviceToHost));
      if (claim < 0) throw KsError(KS_ERR_ARG, "simulation has no NodeClaim");
      HIPCHK(hipMemcpy(out, c->L.lhost[k].c_rs + (size_t)claim * RSW, 4 * (size_t)RSW, hipMemcpyDeviceToHost));
      return KS_OK;
    }
  throw KsError(KS_ERR_ARG, "simulation not in this rank's launch");
  API_CATCH
}

int ks_cons_decide(ks_cons* c, const void* records, int world, int flags, const uint32_t* rs_table,
                   char** json_out) {
  return ks_cons_decide_clock(c, records, world, flags, rs_table, nullptr, json_out);
}

int ks_cons_decide_clock(ks_cons* c, const void* records, int world, int flags, const uint32_t* rs_table,
                         const ks_cons_clock* clock, char** json_out) {
  API_TRY
  if (!c || !json_out || world < 1) throw KsError(KS_ERR_ARG, "bad argument");
  c->check_usable();
  DeviceGuard guard(c->pb->device, nullptr);  // (carried probes run on the handle's GPU)
  const RecView recs = host_records(c, records, world);
  carry_walk(*c, recs, world, clock);
  const bool all_sims = (flags & KS_CONS_ALL_SIMS) != 0;
  if (!rs_table && world == 1 && c->L.lworld == 1) {
    // One rank ran every simulation: the requirement records the output needs are read from this handle's
    // launch as the replay reaches them (one pass over the records, no needed_sims dry run).
    const int RSW = c->pb->host.dims.RSW;
    std::map<int, std::vector<uint32_t>> cache;
    auto fetch = [&](int sim) -> const uint32_t* {
      std::vector<uint32_t>& v = cache[sim];
      if (v.empty()) {
        const int32_t claim = recs.head(sim)[RF_CLAIM];
        if (sim < 0 || sim >= (int)c->L.lhost.size() || claim < 0)
          throw KsError(KS_ERR_INTERNAL, "simulation " + std::to_string(sim) + " has no NodeClaim record");
        v.resize((size_t)RSW);
        HIPCHK(hipMemcpy(v.data(), c->L.lhost[(size_t)sim].c_rs + (size_t)claim * RSW, 4 * (size_t)RSW,
                         hipMemcpyDeviceToHost));
      }
      return v.data();
    };
    *json_out = strdup(decide_json(*c, recs, world, all_sims, fetch, (flags & KS_CONS_CANDIDATES) != 0, clock,
                                   (flags & KS_CONS_NO_SIMS) == 0)
                           .c_str());
    return KS_OK;
  }
  std::vector<int> need = needed_sims(*c, recs, world, all_sims, clock);
  if (!need.empty() && !rs_table) throw KsError(KS_ERR_ARG, "requirement records of the needed simulations missing");
  std::map<int, const uint32_t*> table;
  for (size_t i = 0; i < need.size(); i++) table[need[i]] = rs_table + i * c->pb->host.dims.RSW;
  *json_out = strdup(decide_json(*c, recs, world, all_sims, [&](int sim) { return table.at(sim); },
                                 (flags & KS_CONS_CANDIDATES) != 0, clock, (flags & KS_CONS_NO_SIMS) == 0)
                         .c_str());
  return KS_OK;
  API_CATCH
}

// Diagnostics: the solve counters (ks_problem.h Counter) of the last run's simulation `sim` (this
// rank's launch; with the KS_PHASE_STATS build they include per-phase cycles).
int ks_cons_sim_counters(ks_cons* c, int sim, int64_t* out) {
  const int r = ks_cons_sim_counters_n(c, sim, out, CT_ABI);
  return r < 0 ? r : KS_OK;  // the specific KS_ERR_* code (ARG / HIP / ...), as every entry point returns it
}

int ks_cons_sim_counters_n(ks_cons* c, int sim, int64_t* out, int n) {
  API_TRY
  if (!c || !out || n < 0) throw KsError(KS_ERR_ARG, "bad argument");
  n = std::min(n, (int)CT_NCOUNTERS);
  for (size_t k = 0; k < c->L.lsims.size(); k++)
    if (c->L.lsims[k] == sim) {
      HIPCHK(hipMemcpy(out, c->L.lhost[k].counters, 8 * (size_t)n, hipMemcpyDeviceToHost));
      return n;
    }
  throw KsError(KS_ERR_ARG, "simulation not in this rank's launch");
  API_CATCH
}

int ks_cons_last_reruns(const ks_cons* c) { return c && c->walk.valid ? c->walk.reruns : -1; }

double ks_cons_records_alg_bytes(const ks_cons* c, const void* records, int world) {
  if (!c || world < 1 || (!records && !(world == 1 && c->L.lworld == 1 && (c->L.hdrOnly || c->L.keptFull)))) return 0;
  // (headers: RF_HDR words per simulation, the algorithmic-byte words among them)
  if (!records && c->L.keptFull) records = c->L.hrec;
  const int32_t* r = records ? (const int32_t*)records : c->L.hhdr;
  const size_t stride = records ? (size_t)c->recWords : (size_t)RF_HDR;
  const size_t n = records ? (size_t)c->per_rank(world) * world : c->sims.size();
  double sum = 0;
  for (size_t i = 0; i < n; i++) {
    const int32_t* x = r + i * stride;
    sum += (double)(((uint64_t)(uint32_t)x[RF_ALGB_HI] << 32) | (uint32_t)x[RF_ALGB_LO]);
  }
  return sum;
}

}  // extern "C"
