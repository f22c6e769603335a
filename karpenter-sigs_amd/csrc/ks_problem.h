// ks_problem.h — HBM layout of an encoded scheduling problem and of the per-solve workspace.
//
// Everything the reference's Scheduler reads during Solve (scheduler.go:140-285) is flattened into
// structure-of-arrays tables: int64 fixed-point resource vectors (one decimal scale per resource
// name, chosen so every quantity in the problem is an exact integer), ReqSet records
// (ks_reqset.h), taint bitmasks and CSR instance-type lists.  The tables are written once by
// ks_problem_create and stay resident; each ks_solve gets a fresh workspace.
#pragma once
#include <stdint.h>

#include "ks_reqset.h"

// Explicit address spaces for device code: HBM tables are global (1), solver state is LDS (3).
// Generic (flat) accesses would wait on both the vector-memory and LDS counters, i.e. on every
// outstanding commit-log store.  Host compilation sees plain pointers (identical layout).
#if defined(__HIP_DEVICE_COMPILE__)
#define KS_G __attribute__((address_space(1)))
#define KS_L __attribute__((address_space(3)))
#define KS_C __attribute__((address_space(4)))  // read-only for the whole launch: scalar loads
#else
#define KS_G
#define KS_L
#define KS_C
#endif

namespace ks {

constexpr int kMaxR = 16;         // resource names per problem
constexpr int kMaxTpl = 64;       // NodeClaimTemplates (NodePools) per problem (st_toltpl is one 64-bit mask)
constexpr int kWave = 64;

enum PodStatus : int32_t { ST_PENDING = 0, ST_SCHEDULED = 1, ST_FAILED = 2 };
enum FailCode : uint32_t {
  FC_NONE = 0,
  FC_LIMITS = 1,    // all available instance types exceed limits for nodepool
  FC_TAINTS = 2,    // Taints.Tolerates failed
  FC_HOSTPORT = 3,  // checking host port usage
  FC_COMPAT = 4,    // incompatible requirements
  FC_NO_IT = 5,     // no instance type satisfied resources ... (flags in bits 8..13)
  FC_TOPO = 6,      // unsatisfiable topology constraint (group in bits 16..31)
  FC_TOPO_COMPAT = 7,  // the topology requirements are incompatible with the NodeClaim's (record in fail_rs)
  FC_RS_SNAP = 1u << 15,  // FC_NO_IT: the claim's requirements (topology included) are in fail_rs
};
enum FilterFlag : uint32_t {  // filterResults booleans (nodeclaim.go:144-160)
  FF_REQ = 1, FF_FITS = 2, FF_OFF = 4, FF_REQ_FITS = 8, FF_REQ_OFF = 16, FF_FITS_OFF = 32,
};
enum StateFlag : int32_t { SF_HAS_PREFERRED = 1, SF_TOUCHES_IT_KEYS = 2, SF_HAS_KEYS = 4 };

struct KsDims {
  int32_t R, NK, W, NB, HDR, RSW;
  int32_t T, NTPL, NPOOL, N, P, S, NU;
  int32_t TW;          // words of the largest template instance-type bitset
  int32_t maxTplIts;   // longest template instance-type list
  int32_t zoneKey, ctKey, hostKey;
  int32_t Kcap;        // claim capacity per solve
  int32_t hostnameSeed;
  uint64_t allowWK;    // WellKnownLabels key mask (AllowUndefinedWellKnownLabels)
  uint64_t itKeys;     // keys any instance type constrains, plus zone and capacity-type
  int64_t skMin[4];    // queue sort key components: minimum and bit width of (value - min)
  int32_t skBits[4];
  int32_t dupUids;     // 1 if two pods share a UID (queue staleness then re-reads last_len)
  int32_t totalTplIts; // sum of template instance-type list lengths
  int32_t negReq;      // 1 if any pod or daemon request is negative (disables the threshold filter)
  int32_t spotBit, odBit;  // capacity-type value bits of "spot" / "on-demand" (always interned)
  int32_t hpAny;           // some pod or node uses host ports
  int32_t G, G1;           // topology groups (ks_topo.cpp): [0, G1) t.topologies, [G1, G) inverse
  int32_t tgMaxNv;         // largest value universe of a topology key
  int32_t tgCntWords;      // size of the count table
  int32_t tgSmall;         // count words [0, tgSmall): the non-hostname groups, LDS-resident in k_solve
  int32_t FSW;             // fail_rs words per (pod, template): RSW, or counts + registered bits if larger
  int32_t volAny;          // some pod mounts a PVC of a driver an existing node limits, or GetVolumes fails for it
  int32_t VD;              // limited drivers the pods mount (n_vc0 / n_vlim columns)
  int32_t NVU;             // the pods' PVCs of those drivers (universe ids u)
  int32_t vLogCap;         // placements that can log a shared PVC: sum over PF_VSHARED pods of their PVC count
  int32_t tgUnlab;         // some existing node lacks the label of a topology group's key (k_solve node_slow)
  int32_t GMW;             // 64-bit words of a topology-group set (st_gown, pod_gsel, pod_ginv, tg_late, log_hg):
                           // ceil(G / 64), at least 1
  uint64_t fkMulti;        // keys some instance type constrains with more than one value (feas_masks)
  int32_t fmOn;            // st_fm is computed (k_feasibility) and k_solve reads it
  int32_t lean;            // none of host ports, limited volumes, pod label requirements, negative requests,
                           // topology: k_solve's LEAN instantiation applies (with shared UIDs until a push-back)
  int32_t fnOn;            // st_fn is computed (k_feasibility_nodes) and k_solve reads it
  int32_t FNR;             // rows of st_fn: the relaxation states with label requirements
  int32_t TK;              // distinct topology keys (rows of n_tdom)
};

// Per-launch LDS plan (ks_solve.hip): capacities of the LDS-resident claim state.
struct Plan {
  int32_t KO;      // order/okey capacity = max NodeClaims per solve
  int32_t KL;      // claims [0, KL) keep template/requests/max/options in LDS, the rest in HBM
  int32_t talloc;  // 1: template instance-type Allocatable tables are LDS-resident
  int32_t tsort;   // 1: the sorted Allocatable lists (tsort_*) are LDS-resident
  int32_t tcl;     // topology count words [0, tcl) are LDS-resident (>= KsDims::tgSmall)
  int32_t tdl;     // node domain words [0, tdl) of n_tdom are LDS-resident (0 or TK * N)
  int32_t livl;    // a Solve's live node list (LDS words; 0: the scan walks every node)
  uint64_t lds;    // dynamic LDS bytes
};

// Device view (all pointers into one HBM allocation).
struct KsDev {
  KsDims d;
  const KeyMeta KS_G* keys;
  const uint32_t KS_G* wordValid;
  const uint32_t KS_G* vIsInt;
  const int64_t KS_G* vInt;
  // instance types
  const int64_t KS_G* it_alloc;    // [T][R]  Allocatable() = Capacity - Overhead (types.go:100-110)
  const int64_t KS_G* it_cap;      // [T][R]
  const uint32_t KS_G* it_rs;      // [T][RSW]
  const int32_t KS_G* it_off_beg;  // [T+1] available offerings
  const int32_t KS_G* off_zone;    // zone value bit
  const int32_t KS_G* off_ct;      // capacity-type value bit
  // templates (NodeClaimTemplates in caller order)
  const uint32_t KS_G* tpl_rs;     // [NTPL][RSW] template requirements + hostname (private bit)
  const uint64_t KS_G* tpl_taint;  // [NTPL][2]
  const int64_t KS_G* tpl_daemon;  // [NTPL][R] getDaemonOverhead (scheduler.go:324-341)
  const int32_t KS_G* tpl_it_beg;  // [NTPL+1]
  const int32_t KS_G* tpl_its;     // IT index per template position
  const int32_t KS_G* tpl_pool;    // [NTPL] limit pool or -1
  const int64_t KS_G* tsort_alloc; // [totalTplIts][R] per template, per resource: Allocatable ascending
  const int32_t KS_G* tsort_pos;   //   ... and the template position it belongs to (tb*R + r*nIT + i)
  const int64_t KS_G* tpl_alloc;   // [totalTplIts][R] Allocatable per template position (it_alloc of tpl_its)
  // NodePool limits (remainingResources, scheduler.go:76-78,306-308)
  const int64_t KS_G* pool_rem0;   // [NPOOL][R]
  const uint32_t KS_G* pool_mask;  // [NPOOL] resource names present in the remaining ResourceList
  // pods
  const int64_t KS_G* pod_req;     // [P][R] RequestsForPods(pod) (resources.go:27-35)
  const int32_t KS_G* pod_state0;  // [P] first relaxation state
  const int32_t KS_G* pod_nstate;  // [P]
  const int32_t KS_G* pod_uid;     // [P] interned UID (queue staleness key, queue.go:54-69)
  const int64_t KS_G* pod_sortkey; // [P][4] cpu, memory, creation second, uid rank (queue.go:83-112)
  const uint64_t KS_G* pod_s0;     // [P][4] the pod's first relaxation state: st_tol[0..1], st_toltpl, st_flags
                                   // (queue window refills before any Queue.Push read these, one level fewer)
  // relaxation states (preferences.go:38-147 applied 0..n times)
  const uint32_t KS_G* st_rs;      // [S][RSW] NewPodRequirements
  const uint64_t KS_G* st_tol;     // [S][2] tolerated-taint masks
  const int32_t KS_G* st_flags;    // [S]
  const uint64_t KS_G* st_toltpl;  // [S] bit t: the state tolerates template t's taints
  // existing nodes, in calculateExistingNodeClaims order (scheduler.go:313-321)
  const int64_t KS_G* n_avail;     // [N][R] StateNode.Available()
  const int64_t KS_G* n_req0;      // [N][R] remaining daemon requests (existingnode.go:43-52)
  const uint32_t KS_G* n_rs0;      // [N][RSW] node labels + hostname
  const uint64_t KS_G* n_taint;    // [N][2]
  const int32_t KS_G* n_flags;     // [N] NF_UNUSABLE: not initialized or not Ready (helpers.go:118-124)
  const int32_t KS_G* pod_flags;   // [P] PF_PROVISIONABLE (pkg/utils/pod/scheduling.go IsProvisionable)
  const double KS_G* off_price;    // available offerings' prices (worstLaunchPrice, helpers.go:235-258)
  const uint64_t KS_G* pod_hpc;    // [P] host-port triples a pod's ports Match (conflict mask)
  const uint64_t KS_G* pod_hpu;    // [P] host-port triples a pod reserves
  const uint64_t KS_G* pod_hpo;    // [P] elements of the pod's own initial entries on existing nodes
  const uint64_t KS_G* n_hp0;      // [N] host-port triples reserved on an existing node
  // topology (topology.go; ks_topo.cpp)
  const int32_t KS_G* tg_meta;     // [G][TGM_WORDS]
  const int32_t KS_G* tg_cnt0;     // per group: domain counts over its key's values, -1 = not registered (NewTopology state)
  const uint32_t KS_G* tg_frs;     // node-filter requirement records (spread groups)
  // group sets are GMW-word bitsets (bit g of word g / 64); one word covers every problem with <= 64 groups
  const uint64_t KS_G* st_gown;    // [S][GMW] groups the pod owns in the state
  const uint64_t KS_G* pod_gsel;   // [P][GMW] groups whose selector selects the pod
  const uint64_t KS_G* pod_ginv;   // [P][GMW] inverse groups the pod owns
  const uint64_t KS_G* tg_late;    // [GMW] groups a relaxed state creates mid-Solve: inactive until that relaxation
  const uint32_t KS_G* st_rss;     // [S][RSW] strict pod requirements (podDomains)
  const int32_t KS_G* n_tdom;      // [TK][N] value of the node's label for each topology key (TGM_KSLOT), -1 none
  // feasibility tables (ks_host.cpp; k_solve feas_masks): per template, position bitsets per (key, value)
  const uint32_t KS_G* fk_words;
  const int32_t KS_G* fk_key_off;  // [NTPL][NK]
  const int32_t KS_G* fk_tpl;      // [NTPL][3]
  // k_feasibility's output: per (relaxation state, template), the template positions whose instance type
  // Intersects both the template's and the state's requirements on every key no instance type constrains
  // with more than one value (fkMulti excluded); [S][NTPL][TW]
  uint32_t KS_G* st_fm;
  // k_feasibility_nodes's output: per relaxation state with label requirements (st_fnrow[s] = its row, -1
  // for the others; fn_state[row] = s), one bit per existing node: Taints.Tolerates(node taints) AND the
  // strict Requirements.Compatible(node labels, pod requirements) of ExistingNode.Add (existingnode.go:
  // 64-124), on the nodes' initial records; [FNR][ceil(N/32)]
  const int32_t KS_G* st_fnrow;
  const int32_t KS_G* fn_state;
  uint32_t KS_G* st_fn;
  // volume limits (volumeusage.go:183-227), sparse: any number of PVCs and drivers.  VolumeUsage.ExceedsLimits
  // of a pod on node n is, per limited driver v the pod mounts, count(n, v) + (the pod's PVCs of v that n does
  // not mount yet) <= limit(n, v); the other drivers cannot fail (a node over a limit before the Solve is
  // folded into an unsatisfiable Available by the encoder, and commits keep every count within its limit).
  // "Not mounted yet" needs membership only for the pod's own PVCs: those some node mounts at NewScheduler
  // time (pod_vs), and -- for a pod sharing a PVC with another pod being scheduled (PF_VSHARED) -- those an
  // earlier placement of this Solve mounted (the workspace log, KsWork::vlog).
  const int32_t KS_G* pod_vdbeg;   // [P+1] CSR into pod_vd
  const int32_t KS_G* pod_vd;      // [][2] (driver v, number of the pod's PVCs of v)
  const int32_t KS_G* pod_vsbeg;   // [P+1] CSR into pod_vs
  const int32_t KS_G* pod_vs;      // [][2] (node, PVC u): the pod's PVC u is mounted on the node at NewScheduler time
  const int32_t KS_G* pod_vubeg;   // [P+1] CSR into pod_vu (PF_VSHARED pods only)
  const int32_t KS_G* pod_vu;      // [] the pod's PVCs (universe ids)
  const int32_t KS_G* vol_udrv;    // [NVU] driver of PVC u
  const int32_t KS_G* n_vc0;       // [N][VD] PVCs of driver v mounted on the node (|VolumeUsage.volumes[v]|)
  const int32_t KS_G* n_vlim;      // [N][VD] the node's limit for driver v (INT32_MAX: none)
};

enum NodeFlag : int32_t { NF_UNUSABLE = 1 };
enum TopoGroupType : int32_t { TG_SPREAD = 0, TG_AFFINITY = 1, TG_ANTI = 2 };
enum TgMeta : int32_t {  // per topology group, int32 words
  TGM_TYPE = 0, TGM_KEY, TGM_SKEW, TGM_MIND, TGM_CNT, TGM_NV, TGM_FBEG, TGM_FEND, TGM_HOST,
  TGM_KSLOT,  // the group's key among the topology keys: its row of n_tdom
  TGM_WORDS = 12
};
enum PodFlag : int32_t {
  PF_PROVISIONABLE = 1,
  PF_VSHARED = 2,  // shares a PVC of a limited driver with another pod being scheduled (KsWork::vlog)
  PF_VOLERR = 4,   // GetVolumes fails (a bound PV that does not exist): ExistingNode.Add always errors
};
enum ConsFlag : int32_t { CF_PRICE_ERR = 1, CF_ALL_SPOT = 2, CF_MULTI = 4 };
enum ConsAction : int32_t { CA_NOOP = 0, CA_DELETE = 1, CA_REPLACE = 2, CA_ERROR = 3 };

// Consolidation simulation record (one per simulateScheduling + computeConsolidation, written by the
// SIM epilogue of k_solve), int32 words; gathered across GPUs as fixed-size records.
enum RecField {
  RF_FLAGS = 0,     // RB_* bits
  RF_NCLAIMS,       // len(results.NewNodeClaims)
  RF_HOSTINCR,      // NewNodeClaim calls (global nodeID counter increments, nodeclaim.go:44-48)
  RF_TPL,           // NewNodeClaims[0] template
  RF_HOST,          // NewNodeClaims[0] hostname ordinal (relative to the simulation's first)
  RF_ACTION,        // ConsAction of computeConsolidation (consolidation.go:113-194)
  RF_NOPT,          // len(NewNodeClaims[0].InstanceTypeOptions)
  RF_NPRICE,        // options left by filterByPrice
  RF_NSAME,         // options left by filterOutSameType (multi-node only)
  RF_ERROR,         // KernelError of the simulation's Solve
  RF_ALGB_LO,       // algorithmic bytes the simulation scanned, low / high word
  RF_ALGB_HI,
  RF_CLAIM,         // claim id of NewNodeClaims[0] in the simulation's workspace (its requirements stay there)
  RF_HDR = 16,      // then: [TW] options, [TW] after filterByPrice, [TW] after filterOutSameType
};
// RB_RELAXED: Preferences.Relax changed some pod of the simulation (the pod objects a multi-node probe relaxes
// carry into the next probe, multinodeconsolidation.go:111-114; ks_cons.cpp carry_walk)
enum RecBit { RB_ALL_SCHEDULED = 1, RB_NARROWED = 2, RB_HAS_SPOT = 4, RB_HAS_OD = 8, RB_RELAXED = 16 };
KS_HD int rec_words(int TW) { return RF_HDR + 3 * TW; }

// Per-solve workspace (one slice per replica / simulation).
struct KsWork {
  int32_t KS_G* c_tpl;      // [Kcap]
  int32_t KS_G* c_cnt;      // [Kcap] number of remaining options
  int32_t KS_G* c_thr;      // [Kcap][R] per resource: prefix of tsort already excluded by Fits
  int32_t KS_G* c_host;     // [Kcap] hostname-placeholder ordinal
  int64_t KS_G* c_req;      // [Kcap][R]
  int64_t KS_G* c_max;      // [Kcap][R] per-resource max Allocatable over the remaining options
  uint32_t KS_G* c_rs;      // [Kcap][RSW]
  uint32_t KS_G* c_rem;     // [Kcap][TW] InstanceTypeOptions as a bitset over the template list
  int32_t KS_G* order;      // [Kcap] final s.newNodeClaims order
  int64_t KS_G* n_req;      // [N][R]
  uint32_t KS_G* n_rs;      // [N][RSW]
  int32_t KS_G* queue;      // [P] ring
  int32_t KS_G* qorder;     // [P] NewQueue order
  int32_t KS_G* pod_state;  // [P] current relaxation state
  uint64_t KS_G* last_len;  // [NU] (epoch << 32) | len
  int32_t KS_G* log_pod;    // [P] commit log
  int32_t KS_G* log_tgt;    // [P] >=0 claim id, <0 -(node+1)
  int32_t KS_G* pod_status; // [P]
  int32_t KS_G* pod_fstate; // [P] relaxation state of the final failed attempt
  uint32_t KS_G* fail_code; // [P][NTPL]
  int32_t KS_G* fail_host;  // [P][NTPL]
  int64_t KS_G* pool_rem;   // [NPOOL][R]
  int64_t KS_G* counters;   // [16]
  uint64_t KS_G* n_hp;      // [N] host ports reserved per existing node (SIM: valid where s_tch is set)
  uint64_t KS_G* c_hp;      // [Kcap] host ports reserved per NodeClaim
  int32_t KS_G* n_vc;       // [N][VD] volume counts per existing node (copy of n_vc0); SIM: [P][VD] slots (n_vslot)
  int32_t KS_G* tg_cnt;     // topology domain counts (copy of tg_cnt0)
  int32_t KS_G* tg_cpos;    // [G] NodeClaims whose placeholder domain has a positive count
  int32_t KS_G* tg_ccnt;    // [G][Kcap] counts of the NodeClaims' hostname-placeholder domains
  uint32_t KS_G* fail_rs;   // [P][NTPL][FSW] FC_TOPO_COMPAT: requirements; FC_TOPO: the group's counts (-1: unregistered),
                            // or for a hostname group the commit-log length at the failure (the host replays log_hg)
  uint64_t KS_G* log_hg;    // [P][GMW] TOPO Solve: per commit, the hostname groups Topology.Record counted it in
  int32_t KS_G* tg_act;     // [G] TOPO Solve: NewNodeClaim ordinal counter when a late group was created
  // consolidation simulations only (k_solve<.., SIM=true>): this simulation's view of the shared
  // cluster problem (helpers.go:73-127 — candidates removed, their pods added to the pending ones)
  const int32_t KS_G* pod_map;  // [P] local -> global pod, in NewQueue order (k_sim_keys + sort)
  const int32_t KS_G* run_len;  // [P] identical pods (requests, tolerations, provisionable) from each queue position
                                // to the end of their run in this simulation's NewQueue order (k_sim_runs)
  int32_t P;                    // pods in this simulation
  int32_t nrm;                  // removed (candidate) nodes
  const int32_t KS_G* rm;       // [nrm] their indices in calculateExistingNodeClaims order
  const int64_t KS_G* pool0;    // [NPOOL][R] remaining limits with the candidates' capacity not subtracted
  const double KS_G* st_price;  // [T] filterOutSameType price per instance type, NaN: not a candidate type
  int32_t KS_G* rec;            // [rec_words] output record
  int32_t KS_G* n_slot;         // [N] W.n_rs slot of a node whose requirements changed (valid where s_tchr is set)
  double price;                 // getCandidatePrices (consolidation.go:197-207), summed in candidate order
  int32_t cflags;               // ConsFlag
  int32_t ccs;                  // tg_ccnt row stride (NodeClaims + 1)
  // SIM topology: NewTopology's counts with this simulation's pods excluded (topology.go:61-85)
  const int32_t KS_G* tdel;     // [ntdel][2]: tg_cnt offset, (pods removed << 1) | unregister-if-zero
  int32_t ntdel;
  const uint64_t KS_G* tdead;   // [GMW] inverse groups none of whose owners exist in this simulation
  const uint64_t KS_G* tact;    // [GMW] groups in t.topologies at this simulation's start (those its pods' starting
                                // states own, and the inverse groups); null: all but tg_late
  // a multi-node probe re-run from carried pods (ks_cons.cpp carry_walk): per global pod, the relaxation state it
  // starts in (the state the previous probe left it in); null: every pod starts in pod_state0
  const int32_t KS_G* sstart;
  // (group, minDomains) pairs: this simulation's spread groups whose creating pod (its first pod, in NewTopology's
  // Update order, whose starting state owns the group) gives another minDomains than the shared meta row's
  const int32_t KS_G* tmd;
  int32_t ntmd;
  // volumes (volA)
  int32_t KS_G* n_vslot;    // SIM: [N] n_vc row of a node whose volume usage changed (valid where s_tvol is set)
  int32_t KS_G* vlog;       // [vLogCap][2] (PVC u, node): PF_VSHARED pods' PVCs a placement mounted on a node
  int32_t KS_G* vspec;      // [vLogCap][2] the popped pod's entries of vlog
};

enum Counter {
  CT_NCLAIMS = 0, CT_NLOG, CT_HOSTCTR, CT_ERROR, CT_POPS, CT_ALGBYTES, CT_SORTS, CT_SORT_SLOW,
  CT_CLAIM_FULL, CT_CLAIM_QUICK_FAIL, CT_WINDOWS,
  // diagnostic build (-DKS_PHASE_STATS): s_memtime cycles per phase
  CT_CYC_POP, CT_CYC_NODES, CT_CYC_SORT, CT_CYC_QUICK, CT_CYC_FULL, CT_CYC_COMMIT, CT_CYC_TPL, CT_CYC_TOTAL,
  CT_CYC_NCOMMIT,  // existing-node commit (inside CT_CYC_NODES)
  CT_CYC_SUB,      // [4] claim_full sub-phases (inside CT_CYC_FULL): requirements, thresholds, masks, apply
  CT_ABI = 24,     // counters ks_cons_sim_counters hands out (include/karpenter_amd.h)
  CT_RUNS = 24,    // runs of identical pods placed in one step (simulation fast path; Solve NodeClaim runs)
  CT_RUN_PODS,     // pods those runs placed
  CT_SORT_EXACT,   // claim re-sorts that ran the lane-0 pdqsort (not the wave-parallel partialInsertionSort)
  CT_FINE,         // [8] diagnostic build: topo_pop, state record, window refill, window-block tests, window blocks
                   // tested (count), Topology.Record, simulation node commit, window-block tests' topology share
  CT_NCOUNTERS = 35
};
// KE_LEAN_EXIT: a LEAN Solve of pods sharing a UID met its first push-back (the host re-runs it non-LEAN)
enum KernelError { KE_OK = 0, KE_CLAIM_CAP = 1, KE_ITER_CAP = 2, KE_STACK = 3, KE_LEAN_EXIT = 4 };

}  // namespace ks
