/* karpenter_amd.h — C-ABI of the MI355X Karpenter scheduler hot path (libkarpenter_amd.so).
 *
 * Drop-in boundary for pkg/controllers/provisioning/scheduling in the reference
 * (/root/reference, paths relative to it).  A Go cgo shim marshals the arguments of
 *   NewScheduler(ctx, kubeClient, nodeClaimTemplates, nodePools, cluster, stateNodes, topology,
 *                instanceTypes, daemonSetPods, recorder, opts)        scheduler.go:49-83
 * plus the `pods` argument of
 *   (*Scheduler).Solve(ctx, pods) *Results                             scheduler.go:140-189
 * into one JSON snapshot (see INTEGRATION.md for the schema and the shim), and rebuilds
 *   Results{NewNodeClaims, ExistingNodes, PodErrors}                  scheduler.go:102-106
 * from the result, mapping pod indices back to the caller's *v1.Pod pointers.
 *
 * Plain C types only; no torch or HIP types cross this boundary.  Every call returns 0 on success
 * or a negative KS_ERR_* code; ks_last_error() then holds thread-local text.  A ks_problem is not
 * re-entrant (mirrors the single-goroutine Scheduler); use one per thread.
 */
#ifndef KARPENTER_AMD_H_
#define KARPENTER_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KS_OK 0
#define KS_ERR_PARSE -1       /* malformed snapshot JSON / quantity */
#define KS_ERR_UNSUPPORTED -2 /* input uses a feature this build does not encode (message says which) */
#define KS_ERR_CAPACITY -3    /* encoding limits exceeded (keys > 64, taints > 128, claims > cap) */
#define KS_ERR_HIP -4         /* HIP runtime error (no device, launch failure, fault) */
#define KS_ERR_INTERNAL -5    /* kernel reported an inconsistent state (iteration cap, overflow) */
#define KS_ERR_ARG -6

typedef struct ks_problem ks_problem;
typedef struct ks_results ks_results;

typedef struct ks_solve_opts {
  int device;          /* HIP device ordinal; -1 = current device */
  int simulation_mode; /* SchedulerOptions.SimulationMode (scheduler.go:44-47); decisions identical */
  int replicas;        /* >1: solve `replicas` independent copies in one launch (one wavefront each) */
  int timing_only;     /* 1: do not copy results back (counters and timings only); benchmarks */
  int lds_budget;      /* bytes of LDS per Solve; 0 = automatic (tests use small budgets to force the
                          HBM-resident claim path) */
  int reserved[3];
} ks_solve_opts;

/* NewScheduler equivalent: parse + encode the snapshot and upload it to HBM.  Replaces the Go
 * allocation-heavy construction at scheduler.go:49-83 + nodeclaimtemplate.go:43-53 +
 * existingnode.go:40-62; the caller keeps ownership of `snapshot_json`. */
int ks_problem_create(const char* snapshot_json, size_t len, ks_problem** out);
void ks_problem_free(ks_problem* p);

/* Binary snapshot of an encoded problem (the whole host model NewScheduler built: universes, tables, pods,
 * relaxation chains, topology): ks_problem_save writes it (free with ks_free); ks_problem_create_binary
 * rebuilds the problem from it and uploads it, skipping the JSON parse and the encode.  A snapshot is tied to
 * the library build that wrote it (a blob from another build is refused with KS_ERR_PARSE). */
int ks_problem_save(const ks_problem* p, void** buf, size_t* len);
int ks_problem_create_binary(const void* buf, size_t len, ks_problem** out);
/* Host-only (no device): encode snapshot_json, save it, load the bytes and save again; KS_OK when the two
 * byte strings are identical.  *bytes: the snapshot size. */
int ks_snapshot_check(const char* snapshot_json, size_t len, size_t* bytes);
/* Host-only (no device): the binary snapshot of snapshot_json, as ks_problem_save would write it for a
 * problem created from that JSON (free with ks_free), e.g. to convert fixtures offline. */
int ks_problem_encode_binary(const char* snapshot_json, size_t len, void** buf, size_t* blen);
/* Host-only (no device): the load-time checks of ks_problem_create_binary (header, lengths backed by bytes,
 * offset tables, every table against the dims and every stored index against its table): KS_OK, or
 * KS_ERR_PARSE for a truncated, foreign or internally inconsistent blob. */
int ks_problem_check_binary(const void* buf, size_t len);

/* Host-only encode of a snapshot (no device needed): returns JSON with the universe sizes (keys,
 * value words, resources, instance types, relaxation states).  Diagnostics / CPU tests. */
int ks_problem_inspect(const char* snapshot_json, size_t len, char** dims_json);

/* Solve (scheduler.go:140-189) on the GPU.  Fresh scheduler state every call (a Scheduler is
 * single-use in production, scheduler.go:49 is called per Schedule / per simulation). */
int ks_solve(ks_problem* p, const ks_solve_opts* opts, ks_results** out);
void ks_results_free(ks_results* r);

/* Results as canonical JSON: {"newNodeClaims":[{nodePoolName, hostname, pods[], instanceTypeOptions[],
 * requests{}, requirements[], requirementsString}], "existingNodes":[{name, pods[]}],
 * "podErrors":{"<pod index>": "<error text>"}}.  Free with ks_free. */
int ks_results_json(const ks_results* r, char** json_out);

/* Structured accessors for a cgo shim (no JSON on the hot return path). */
int ks_results_num_new_nodeclaims(const ks_results* r);
int ks_results_nodeclaim(const ks_results* r, int i, int* template_index, const int32_t** pods, int* n_pods,
                         const int32_t** instance_types, int* n_instance_types);
int ks_results_num_existing_nodes(const ks_results* r);
int ks_results_existing_node(const ks_results* r, int i, int* state_node_index, const int32_t** pods, int* n_pods);
int ks_results_num_pod_errors(const ks_results* r);
int ks_results_pod_error(const ks_results* r, int i, int* pod_index, const char** message);

/* One key of a NodeClaim's Requirements (pkg/scheduling/requirement.go:33-280), as a cgo shim rebuilds
 * it: Operator() ("In", "NotIn", "Exists", "DoesNotExist"; Gt/Lt read as "Exists" with bounds,
 * requirement.go:197-208), the value set in sorted order, and the Gt / Lt bounds. */
typedef struct ks_requirement {
  const char* key;
  const char* op;
  int n_values;
  const char* const* values;
  int has_gt, has_lt;
  int64_t gt, lt;
} ks_requirement;
/* NodeClaim i's Spec.Resources.Requests (nodeclaim.go:35-42, scheduler.go:102-106): resource names in
 * name order with canonical resource.Quantity.String() text.  Arrays live as long as r. */
int ks_results_nodeclaim_requests(const ks_results* r, int i, int* n, const char* const** names,
                                  const char* const** quantities);
/* NodeClaim i's Requirements after FinalizeScheduling (hostname removed, nodeclaim.go:123-128), one entry
 * per key in key order (what consolidation.go:134-188 reads from NewNodeClaims[0]). */
int ks_results_nodeclaim_requirements(const ks_results* r, int i, int* n, const ks_requirement** reqs);

/* Device time of the solve kernel(s) of the last ks_solve, measured with HIP events on the
 * stream the kernel ran on (milliseconds). */
double ks_results_kernel_ms(const ks_results* r);
/* The k_solve launch alone (the dominant kernel; excludes workspace init and the queue sort). */
double ks_results_solve_kernel_ms(const ks_results* r);
/* k_feasibility (the static pod-state x instance-type rows) inside this Solve: HIP-event time and its
 * algorithmic bytes; 0 when the problem has no pod label requirements (the kernel is not launched). */
double ks_results_feasibility_ms(const ks_results* r);
double ks_results_feasibility_bytes(const ks_results* r);
/* k_feasibility_nodes (the static pod-state x existing-node rows: taints + strict Compatible,
 * existingnode.go:64-124) inside this Solve: HIP-event time and algorithmic bytes; 0 when not launched
 * (no pod label requirements or no existing nodes). */
double ks_results_node_feasibility_ms(const ks_results* r);
double ks_results_node_feasibility_bytes(const ks_results* r);
/* Algorithmic bytes the solve scanned (SURVEY.md §8d formula, counted by the kernel). */
double ks_results_algorithmic_bytes(const ks_results* r);

/* ---- Consolidation (pkg/controllers/disruption) ------------------------------------------------
 * ks_cons_create replaces the per-simulation NewScheduler calls of simulateScheduling
 * (helpers.go:73-127) for one disruption pass: the cluster snapshot (state nodes
 * with their pods, pending pods, candidate node names, NodePools, instance types) is encoded once.
 * Candidates are built and ordered like NewCandidate + sortAndFilterCandidates (types.go:54-113,
 * consolidation.go:73-83).  The simulations are every multi-node prefix firstNConsolidationOption
 * can probe (multinodeconsolidation.go:87-137) and one per candidate (singlenodeconsolidation.go:
 * 42-88); each ends in the computeConsolidation decision (consolidation.go:113-194) on the GPU. */
typedef struct ks_cons ks_cons;
int ks_cons_create(const char* snapshot_json, size_t len, ks_cons** out);
/* Binary snapshot of a consolidation handle (host model + candidates in disruption-cost order + the
 * simulation plan), as for ks_problem_save / ks_problem_create_binary. */
int ks_cons_save(const ks_cons* c, void** buf, size_t* len);
int ks_cons_create_binary(const void* buf, size_t len, ks_cons** out);
/* Host-only (no device): JSON {candidates:[{name, disruptionCost, pods}], sims, multiPrefixes, recordBytes}. */
int ks_cons_inspect(const char* snapshot_json, size_t len, char** out_json);
/* Cluster-state events between two passes against the resident handle (replaces re-reading the cluster
 * and rebuilding the scheduler per pass: state/cluster.go:220-512 UpdatePod/DeletePod/DeleteNode,
 * provisioner.go:204-296).  update_json: {"deletePods":[uid], "bindPods":[{"uid","node"}],
 * "removeNodes":[name]}, applied in that order: a deleted pod frees its node's requests; a bound pod
 * (pending until now) is Running on an active node and takes its requests; a removed node takes its pods
 * with it and returns its capacity to its NodePool's limits.  In a topology cluster the shared NewTopology
 * counts follow (topology.go:61-85,190-230; the snapshot's clusterPods lose deleted / removed-node pods and
 * gain bound ones).  Candidates, their costs and order, and the simulations are re-derived; the next
 * ks_cons_run sees the new state.  All or nothing: KS_ERR_ARG for unknown / already-deleted / not-pending
 * pods or unknown nodes, KS_ERR_UNSUPPORTED for clusters with volume limits, pods with host ports, and a
 * topology update that would turn a group into one only a relaxation creates (rebuild with ks_cons_create
 * there). */
int ks_cons_update(ks_cons* c, const char* update_json, size_t len);
/* Host-only: the snapshot with update_json applied ("{}" for none, an array for a sequence), as ks_cons_inspect plus
 * "nodeRows" {name: {available (device units), pods}} for every active node and "poolRemaining". */
int ks_cons_inspect_update(const char* snapshot_json, size_t len, const char* update_json, size_t ulen,
                           char** out_json);
void ks_cons_free(ks_cons* c);
int ks_cons_num_candidates(const ks_cons* c);
int ks_cons_num_sims(const ks_cons* c);
int ks_cons_record_bytes(const ks_cons* c);           /* fixed size of one simulation record */
int ks_cons_records_per_rank(const ks_cons* c, int world);
/* Run the simulations s with s % world == rank on the current (or opts->device) GPU and write their
 * records, in order of s, to `records` (records_per_rank * record_bytes bytes; a device pointer when
 * records_on_device, so an all-gather over RCCL can collect them).  kernel_ms: HIP-event time of the
 * queue sort + simulation kernel on the stream they ran on. */
int ks_cons_run(ks_cons* c, int rank, int world, const ks_solve_opts* opts, void* records, int records_on_device,
                double* kernel_ms);
/* records may be NULL at world 1 (records_on_device 0): the records stay in the handle's pinned host buffer
 * until its next run, and ks_cons_decide / ks_cons_needed_sims / ks_cons_records_alg_bytes take records NULL
 * to read them there (no copy of the pass's records). */
/* Replay the reference's sequential choice over the gathered records ([rank][slot] layout):
 * JSON {"candidates":[{name, disruptionCost}], "multi":{"command", "sims", "path"}, "single":{"command", "sims"}}
 * ("path": the binary search's probes {mid, carried, action}: carried = re-run from pod objects an earlier probe relaxed).
 * flags: KS_CONS_ALL_SIMS reports every simulation (otherwise only those the reference would have
 * run); KS_CONS_CANDIDATES includes the candidate list (otherwise "candidates" is empty).
 * Requirement records (NewNodeClaims[0].Requirements) stay on the GPU that ran a simulation:
 * ks_cons_needed_sims lists (returns the count; writes up to cap) the simulations the output needs,
 * their owners (rank = sim % world) read them with ks_cons_claim_requirements (requirement_words
 * uint32 each), and rs_table passes them to ks_cons_decide in that order.  rs_table may be NULL when world is 1
 * and this handle's last ks_cons_run covered every simulation: the records are then read from that run. */
#define KS_CONS_ALL_SIMS 1   /* flags: report every simulation */
#define KS_CONS_CANDIDATES 2 /* flags: include the ordered candidate list */
#define KS_CONS_NO_SIMS 4    /* flags: leave out the per-simulation "sims" lists (the commands are unchanged) */
int ks_cons_requirement_words(const ks_cons* c);
int ks_cons_needed_sims(ks_cons* c, const void* records, int world, int flags, int32_t* out, int cap);
int ks_cons_claim_requirements(ks_cons* c, int sim, uint32_t* out);
int ks_cons_decide(ks_cons* c, const void* records, int world, int flags, const uint32_t* rs_table,
                   char** json_out);
/* The methods' timeouts (MultiNodeConsolidationTimeoutDuration = 1 min, multinodeconsolidation.go:34,99-110;
 * SingleNodeConsolidationTimeoutDuration = 3 min, singlenodeconsolidation.go:29,58-65) on a virtual clock
 * that advances sim_seconds per simulation the sequential replay consults: the multi-node search returns
 * its last saved command once the clock passes its timeout, the single-node scan abandons with no command.
 * The GPU has already run every simulation, so sim_seconds models the reference's per-simulation cost
 * (0: no timeout ever fires, which is ks_cons_decide). */
typedef struct ks_cons_clock {
  double multi_timeout_s;
  double single_timeout_s;
  double sim_seconds;
} ks_cons_clock;
int ks_cons_decide_clock(ks_cons* c, const void* records, int world, int flags, const uint32_t* rs_table,
                         const ks_cons_clock* clock, char** json_out);
/* Validation.IsValid after its wait + ValidateCommand (disruption/validation.go:68-180): the handle
 * holds the current cluster snapshot (stateNodes may carry "nominated": Cluster.IsNodeNominated);
 * command_json is a command as ks_cons_decide reports it ({"candidates": [names], "replacement":
 * {"instanceTypeOptions": [...]}} or no "replacement"), computed on an earlier snapshot.  The command's
 * candidates are re-filtered (NewCandidate, PDBs, do-not-disrupt), then re-simulated on the GPU.
 * Writes JSON {"valid": bool, "reason": "" | "candidates-changed" | "candidate-nominated" |
 * "no-candidates" | "pods-unschedulable" | "replacement-not-needed" | "multiple-nodeclaims" |
 * "replacement-needed" | "instance-types-not-subset", "sim": null | {allNonPendingScheduled,
 * newNodeClaims, claim0: {nodePoolName, instanceTypeOptions}}}.  Leaves the pass's plan unchanged. */
int ks_cons_validate(ks_cons* c, const char* command_json, size_t len, const ks_solve_opts* opts, char** json_out);
/* Diagnostics: the 24 solve counters of simulation `sim` in the last ks_cons_run of this handle. */
int ks_cons_sim_counters(ks_cons* c, int sim, int64_t* out24);
/* The same for up to n counters (27 in this build: + runs of identical pods, pods they placed, exact claim
 * re-sorts); n larger than the build's count copies that count. Returns the number copied or a negative
 * KS_ERR_* code. */
int ks_cons_sim_counters_n(ks_cons* c, int sim, int64_t* out, int n);
/* Multi-node probes the last ks_cons_decide / ks_cons_needed_sims ran on this handle's GPU (-1: none resolved).
 * The reference's binary search hands each probe the pod objects the earlier probes relaxed in place
 * (multinodeconsolidation.go:111-114, helpers.go:102-104, preferences.go:60-147): a probe holding such a pod is
 * re-simulated from the carried relaxation states, one launch per probe (typically none). */
int ks_cons_last_reruns(const ks_cons* c);
/* Algorithmic bytes the gathered simulations scanned, summed from their records. */
double ks_cons_records_alg_bytes(const ks_cons* c, const void* records, int world);

/* Cluster-state accounting (pkg/controllers/state: Cluster.UpdateNodeClaim / UpdateNode / UpdatePod,
 * cluster.go:220-512, and the StateNode accessors, statenode.go:110-333): from {"nodeClaims":
 * [v1beta1.NodeClaim], "nodes": [v1.Node], "pods": [v1.Pod], "volumeDrivers": {"ns/pvc": driver},
 * "csiNodes": [storagev1.CSINode]} derive the state the informers converge to, as the snapshot's
 * "stateNodes" array: {name, providerID, hostName, labels, taints, capacity, allocatable, available,
 * podRequests, daemonSetRequests, initialized, ready, markedForDeletion, creationTimestamp,
 * hostPortUsage, volumeUsage, volumeLimits, pods}.  Host-only (no device).  Free with ks_free. */
int ks_cluster_state(const char* cluster_json, size_t len, char** state_nodes_json);

void ks_free(void* p);
const char* ks_last_error(void);
int ks_device_count(void);
const char* ks_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* KARPENTER_AMD_H_ */
