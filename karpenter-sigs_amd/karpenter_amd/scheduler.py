"""ctypes binding of include/karpenter_amd.h, shaped like the reference's scheduling package.

Reference surface (pkg/controllers/provisioning/scheduling/scheduler.go):
    NewScheduler(ctx, kubeClient, nodeClaimTemplates, nodePools, cluster, stateNodes, topology,
                 instanceTypes, daemonSetPods, recorder, opts) *Scheduler        :49-83
    (*Scheduler).Solve(ctx, pods) *Results                                     :140-189
    Results{NewNodeClaims, ExistingNodes, PodErrors}                           :102-106
Here the NewScheduler arguments and the pods travel as one JSON snapshot.
"""
import ctypes
import json
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# KS_LIB_VARIANT=stats loads the diagnostic build with per-phase cycle counters; =asan the ASan + UBSan
# build of the host translation units (make -C karpenter-sigs_amd asan; scripts/asan_cpu_suite.sh); =tsan
# their ThreadSanitizer build (scripts/tsan_cpu_suite.sh).
_VARIANTS = {"stats": "libkarpenter_amd_stats.so", "asan": "libkarpenter_amd_asan.so", "tsan": "libkarpenter_amd_tsan.so"}
_VARIANT = os.environ.get("KS_LIB_VARIANT", "")
_LIB_PATH = os.path.join(_HERE, _VARIANTS.get(_VARIANT, "libkarpenter_amd_%s.so" % _VARIANT if _VARIANT else "libkarpenter_amd.so"))
_lib = None

KS_ERRORS = {-1: "KS_ERR_PARSE", -2: "KS_ERR_UNSUPPORTED", -3: "KS_ERR_CAPACITY", -4: "KS_ERR_HIP",
             -5: "KS_ERR_INTERNAL", -6: "KS_ERR_ARG"}


class KsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s: %s" % (KS_ERRORS.get(code, code), msg))
        self.code = code


class _Opts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("simulation_mode", ctypes.c_int), ("replicas", ctypes.c_int),
                ("timing_only", ctypes.c_int), ("lds_budget", ctypes.c_int),
                ("reserved", ctypes.c_int * 3)]


class _Clock(ctypes.Structure):  # ks_cons_clock
    _fields_ = [("multi_timeout_s", ctypes.c_double), ("single_timeout_s", ctypes.c_double),
                ("sim_seconds", ctypes.c_double)]


def library_path():
    return _LIB_PATH


def lib():
    """Load libkarpenter_amd.so (built in-tree by `make -C karpenter-sigs_amd`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise KsError(-4, "libkarpenter_amd.so not built (%s); run __graft_entry__.build()" % _LIB_PATH)
    l = ctypes.CDLL(_LIB_PATH)
    vp = ctypes.c_void_p
    l.ks_problem_create.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(vp)]
    l.ks_problem_inspect.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(vp)]
    l.ks_problem_free.argtypes = [vp]
    l.ks_solve.argtypes = [vp, ctypes.POINTER(_Opts), ctypes.POINTER(vp)]
    l.ks_results_free.argtypes = [vp]
    l.ks_results_json.argtypes = [vp, ctypes.POINTER(vp)]
    l.ks_results_kernel_ms.argtypes = [vp]
    l.ks_results_kernel_ms.restype = ctypes.c_double
    l.ks_results_solve_kernel_ms.argtypes = [vp]
    l.ks_results_solve_kernel_ms.restype = ctypes.c_double
    l.ks_results_algorithmic_bytes.argtypes = [vp]
    l.ks_results_algorithmic_bytes.restype = ctypes.c_double
    l.ks_results_feasibility_ms.argtypes = [vp]
    l.ks_results_feasibility_ms.restype = ctypes.c_double
    l.ks_results_feasibility_bytes.argtypes = [vp]
    l.ks_results_feasibility_bytes.restype = ctypes.c_double
    l.ks_results_node_feasibility_ms.argtypes = [vp]
    l.ks_results_node_feasibility_ms.restype = ctypes.c_double
    l.ks_results_node_feasibility_bytes.argtypes = [vp]
    l.ks_results_node_feasibility_bytes.restype = ctypes.c_double
    l.ks_cluster_state.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(vp)]
    l.ks_free.argtypes = [vp]
    l.ks_problem_save.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_size_t)]
    l.ks_problem_create_binary.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(vp)]
    l.ks_snapshot_check.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    l.ks_problem_encode_binary.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(vp),
                                           ctypes.POINTER(ctypes.c_size_t)]
    l.ks_problem_check_binary.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    l.ks_cons_save.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_size_t)]
    l.ks_cons_create_binary.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(vp)]
    l.ks_last_error.restype = ctypes.c_char_p
    l.ks_build_info.restype = ctypes.c_char_p
    _lib = l
    return l


def _check(rc):
    if rc != 0:
        raise KsError(rc, lib().ks_last_error().decode())


def _take_str(ptr):
    s = ctypes.cast(ptr, ctypes.c_char_p).value.decode()
    lib().ks_free(ptr)
    return s


def _encode(snapshot):
    return (snapshot if isinstance(snapshot, str) else json.dumps(snapshot)).encode()


def _records_buffer(records):
    """A ctypes buffer over gathered records: a run's own buffer (the memoryview run() returns) as is,
    anything else bytes-like copied once."""
    if (isinstance(records, memoryview) and isinstance(records.obj, ctypes.Array)
            and records.nbytes == ctypes.sizeof(records.obj)):  # the whole buffer, not a slice of it
        return records.obj
    return ctypes.create_string_buffer(bytes(records), len(records))


def inspect(snapshot):
    """Encode a snapshot on the host only (no device): universe sizes and layout, for diagnostics."""
    b = _encode(snapshot)
    out = ctypes.c_void_p()
    _check(lib().ks_problem_inspect(b, len(b), ctypes.byref(out)))
    return json.loads(_take_str(out))


def cluster_state(cluster):
    """Cluster-state accounting (pkg/controllers/state, cluster.go:220-512 + statenode.go:110-333):
    the StateNode accessor values the informers converge to for {"nodeClaims", "nodes", "pods"}, as a
    snapshot "stateNodes" list (host-only; no device)."""
    b = _encode(cluster)
    out = ctypes.c_void_p()
    _check(lib().ks_cluster_state(b, len(b), ctypes.byref(out)))
    return json.loads(_take_str(out))


class Results:
    """scheduling.Results: new_nodeclaims, existing_nodes, pod_errors (keys = input pod index)."""

    def __init__(self, doc, kernel_ms, alg_bytes, solve_kernel_ms=0.0):
        self.doc = doc
        self.new_nodeclaims = doc["newNodeClaims"]
        self.existing_nodes = doc["existingNodes"]
        self.pod_errors = {int(k): v for k, v in doc["podErrors"].items()}
        self.stats = doc.get("stats", {})
        self.kernel_ms = kernel_ms
        self.solve_kernel_ms = solve_kernel_ms
        self.algorithmic_bytes = alg_bytes
        self.feasibility_ms = 0.0     # k_feasibility inside this Solve (0: not launched)
        self.feasibility_bytes = 0.0  # its algorithmic bytes
        self.node_feasibility_ms = 0.0     # k_feasibility_nodes inside this Solve (0: not launched)
        self.node_feasibility_bytes = 0.0  # its algorithmic bytes

    def canonical(self):
        d = dict(self.doc)
        d.pop("stats", None)
        return d


class _Requirement(ctypes.Structure):  # ks_requirement
    _fields_ = [("key", ctypes.c_char_p), ("op", ctypes.c_char_p), ("n_values", ctypes.c_int),
                ("values", ctypes.POINTER(ctypes.c_char_p)), ("has_gt", ctypes.c_int), ("has_lt", ctypes.c_int),
                ("gt", ctypes.c_int64), ("lt", ctypes.c_int64)]


_accessors_bound = False


def _bind_accessors(l):
    global _accessors_bound
    if _accessors_bound:
        return
    vp, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)
    i32pp = ctypes.POINTER(ctypes.POINTER(ctypes.c_int32))
    strpp = ctypes.POINTER(ctypes.POINTER(ctypes.c_char_p))
    l.ks_results_num_new_nodeclaims.argtypes = [vp]
    l.ks_results_nodeclaim.argtypes = [vp, ctypes.c_int, ip, i32pp, ip, i32pp, ip]
    l.ks_results_nodeclaim_requests.argtypes = [vp, ctypes.c_int, ip, strpp, strpp]
    l.ks_results_nodeclaim_requirements.argtypes = [vp, ctypes.c_int, ip, ctypes.POINTER(ctypes.POINTER(_Requirement))]
    l.ks_results_num_existing_nodes.argtypes = [vp]
    l.ks_results_existing_node.argtypes = [vp, ctypes.c_int, ip, i32pp, ip]
    l.ks_results_num_pod_errors.argtypes = [vp]
    l.ks_results_pod_error.argtypes = [vp, ctypes.c_int, ip, ctypes.POINTER(ctypes.c_char_p)]
    _accessors_bound = True


class StructuredResults:
    """Results read through the C-ABI's structured accessors (what the cgo shim in INTEGRATION.md does):
    new_nodeclaims = [{template, pods, instance_types (indices), requests {name: quantity},
    requirements [(key, op, values, gt, lt)]}], existing_nodes = [(state node index, pods)],
    pod_errors = {pod index: message}."""

    def __init__(self, claims, nodes, errors, kernel_ms, solve_kernel_ms):
        self.new_nodeclaims = claims
        self.existing_nodes = nodes
        self.pod_errors = errors
        self.kernel_ms = kernel_ms
        self.solve_kernel_ms = solve_kernel_ms


def _read_structured(l, r):
    import numpy as np

    _bind_accessors(l)
    tpl, n1, n2 = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    a1, a2 = ctypes.POINTER(ctypes.c_int32)(), ctypes.POINTER(ctypes.c_int32)()
    claims = []
    for i in range(l.ks_results_num_new_nodeclaims(r)):
        _check(l.ks_results_nodeclaim(r, i, ctypes.byref(tpl), ctypes.byref(a1), ctypes.byref(n1), ctypes.byref(a2),
                                      ctypes.byref(n2)))
        pods = np.ctypeslib.as_array(a1, (n1.value,)).copy() if n1.value else np.zeros(0, np.int32)
        its = np.ctypeslib.as_array(a2, (n2.value,)).copy() if n2.value else np.zeros(0, np.int32)
        names, qtys = ctypes.POINTER(ctypes.c_char_p)(), ctypes.POINTER(ctypes.c_char_p)()
        _check(l.ks_results_nodeclaim_requests(r, i, ctypes.byref(n1), ctypes.byref(names), ctypes.byref(qtys)))
        requests = {names[k].decode(): qtys[k].decode() for k in range(n1.value)}
        rq = ctypes.POINTER(_Requirement)()
        _check(l.ks_results_nodeclaim_requirements(r, i, ctypes.byref(n1), ctypes.byref(rq)))
        reqs = []
        for k in range(n1.value):
            x = rq[k]
            reqs.append((x.key.decode(), x.op.decode(), [x.values[v].decode() for v in range(x.n_values)],
                         x.gt if x.has_gt else None, x.lt if x.has_lt else None))
        claims.append({"template": tpl.value, "pods": pods, "instance_types": its, "requests": requests,
                       "requirements": reqs})
    nodes = []
    for i in range(l.ks_results_num_existing_nodes(r)):
        _check(l.ks_results_existing_node(r, i, ctypes.byref(n2), ctypes.byref(a1), ctypes.byref(n1)))
        pods = np.ctypeslib.as_array(a1, (n1.value,)).copy() if n1.value else np.zeros(0, np.int32)
        nodes.append((n2.value, pods))
    errors = {}
    msg = ctypes.c_char_p()
    for i in range(l.ks_results_num_pod_errors(r)):
        _check(l.ks_results_pod_error(r, i, ctypes.byref(n1), ctypes.byref(msg)))
        errors[n1.value] = msg.value.decode()
    return claims, nodes, errors


def _take_bytes(fn, handle):
    buf, n = ctypes.c_void_p(), ctypes.c_size_t()
    _check(fn(handle, ctypes.byref(buf), ctypes.byref(n)))
    try:
        return ctypes.string_at(buf, n.value)
    finally:
        lib().ks_free(buf)


def snapshot_check(snapshot):
    """Host-only: encode, save, load, save again; raises unless the two snapshots are byte-identical.
    Returns the snapshot size in bytes."""
    b = _encode(snapshot)
    n = ctypes.c_size_t()
    _check(lib().ks_snapshot_check(b, len(b), ctypes.byref(n)))
    return n.value


def encode_binary(snapshot):
    """Host-only: the binary snapshot of a JSON problem (what Scheduler(snapshot).save() returns), no device."""
    b = _encode(snapshot)
    buf, n = ctypes.c_void_p(), ctypes.c_size_t()
    _check(lib().ks_problem_encode_binary(b, len(b), ctypes.byref(buf), ctypes.byref(n)))
    try:
        return ctypes.string_at(buf, n.value)
    finally:
        lib().ks_free(buf)


def check_binary(blob):
    """Host-only: ks_problem_create_binary's load-time checks; raises KsError (KS_ERR_PARSE) on a bad blob."""
    blob = bytes(blob)
    _check(lib().ks_problem_check_binary(blob, len(blob)))


class Scheduler:
    """NewScheduler(...) on the GPU: the snapshot is encoded once and stays resident in HBM.
    Scheduler.from_binary(blob) rebuilds one from save()'s binary snapshot (no JSON parse, no encode)."""

    def __init__(self, snapshot, _binary=None):
        h = ctypes.c_void_p()
        if _binary is not None:
            _check(lib().ks_problem_create_binary(_binary, len(_binary), ctypes.byref(h)))
        else:
            b = _encode(snapshot)
            _check(lib().ks_problem_create(b, len(b), ctypes.byref(h)))
        self._h = h

    @classmethod
    def from_binary(cls, blob):
        return cls(None, _binary=bytes(blob))

    def save(self):
        """The binary snapshot of the encoded problem (bytes)."""
        return _take_bytes(lib().ks_problem_save, self._h)

    def solve(self, replicas=1, device=-1, simulation_mode=True, timing_only=False, lds_budget=0):
        """Solve(ctx, pods) with fresh scheduler state; replicas>1 runs that many independent copies
        of the same Solve in one launch (one wavefront each) and returns replica 0's results."""
        o = _Opts(device, 1 if simulation_mode else 0, replicas, 1 if timing_only else 0, lds_budget)
        r = ctypes.c_void_p()
        _check(lib().ks_solve(self._h, ctypes.byref(o), ctypes.byref(r)))
        try:
            if timing_only:
                out = Results({"newNodeClaims": [], "existingNodes": [], "podErrors": {}},
                              lib().ks_results_kernel_ms(r), lib().ks_results_algorithmic_bytes(r),
                              lib().ks_results_solve_kernel_ms(r))
            else:
                js = ctypes.c_void_p()
                _check(lib().ks_results_json(r, ctypes.byref(js)))
                doc = json.loads(_take_str(js))
                out = Results(doc, lib().ks_results_kernel_ms(r), lib().ks_results_algorithmic_bytes(r),
                              lib().ks_results_solve_kernel_ms(r))
            out.feasibility_ms = lib().ks_results_feasibility_ms(r)
            out.feasibility_bytes = lib().ks_results_feasibility_bytes(r)
            out.node_feasibility_ms = lib().ks_results_node_feasibility_ms(r)
            out.node_feasibility_bytes = lib().ks_results_node_feasibility_bytes(r)
            return out
        finally:
            lib().ks_results_free(r)

    def solve_structured(self, device=-1, simulation_mode=True):
        """Solve(ctx, pods) with the Results read through the structured accessors (no JSON): the drop-in
        caller's full return path (INTEGRATION.md's cgo shim)."""
        l = lib()
        o = _Opts(device, 1 if simulation_mode else 0, 1, 0, 0)
        r = ctypes.c_void_p()
        _check(l.ks_solve(self._h, ctypes.byref(o), ctypes.byref(r)))
        try:
            claims, nodes, errors = _read_structured(l, r)
            return StructuredResults(claims, nodes, errors, l.ks_results_kernel_ms(r), l.ks_results_solve_kernel_ms(r))
        finally:
            l.ks_results_free(r)

    def timed_collect(self, steps, device=-1, simulation_mode=True):
        """Mean ms of `steps` ks_solve calls with the Results collected (no accessor walk) + ks_results_free:
        the C-ABI cost of the drop-in return path, without Python's per-field ctypes overhead."""
        import time
        l = lib()
        o = _Opts(device, 1 if simulation_mode else 0, 1, 0, 0)
        r = ctypes.c_void_p()
        t = time.perf_counter()
        for _ in range(steps):
            _check(l.ks_solve(self._h, ctypes.byref(o), ctypes.byref(r)))
            l.ks_results_free(r)
        return (time.perf_counter() - t) * 1000.0 / steps

    def close(self):
        if self._h:
            lib().ks_problem_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _cons_lib():
    l = lib()
    if not getattr(l, "_cons_ready", False):
        vp = ctypes.c_void_p
        l.ks_cons_create.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(vp)]
        l.ks_cons_free.argtypes = [vp]
        l.ks_cons_inspect.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(vp)]
        l.ks_cons_inspect_update.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                             ctypes.POINTER(vp)]
        l.ks_cons_update.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t]
        for f in ("ks_cons_num_candidates", "ks_cons_num_sims", "ks_cons_record_bytes"):
            getattr(l, f).argtypes = [vp]
        l.ks_cons_records_per_rank.argtypes = [vp, ctypes.c_int]
        l.ks_cons_run.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_Opts), vp, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_double)]
        l.ks_cons_decide.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(vp)]
        l.ks_cons_decide_clock.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(_Clock), ctypes.POINTER(vp)]
        l.ks_cons_requirement_words.argtypes = [vp]
        l.ks_cons_needed_sims.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
        l.ks_cons_claim_requirements.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]
        l.ks_cons_validate.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_Opts), ctypes.POINTER(vp)]
        l.ks_cons_sim_counters.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
        l.ks_cons_sim_counters_n.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
        l.ks_cons_records_alg_bytes.argtypes = [vp, vp, ctypes.c_int]
        l.ks_cons_records_alg_bytes.restype = ctypes.c_double
        l.ks_cons_last_reruns.argtypes = [vp]
        l.ks_cons_last_reruns.restype = ctypes.c_int
        l._cons_ready = True
    return l


def inspect_consolidation(snapshot):
    """Host-only: the ordered candidates and the simulation plan of a cluster snapshot."""
    b = _encode(snapshot)
    out = ctypes.c_void_p()
    _check(_cons_lib().ks_cons_inspect(b, len(b), ctypes.byref(out)))
    return json.loads(_take_str(out))


def inspect_consolidation_update(snapshot, update=None):
    """Host-only: the snapshot with a ks_cons_update delta applied (None: as it is), with every active
    node's encoded available row and pods and the pools' remaining limits ("nodeRows", "poolRemaining")."""
    b = _encode(snapshot)
    u = _encode(update if update is not None else {})
    out = ctypes.c_void_p()
    _check(_cons_lib().ks_cons_inspect_update(b, len(b), u, len(u), ctypes.byref(out)))
    return json.loads(_take_str(out))


def shard_slot(sim, world):
    """Where simulation `sim` lands in the [rank][slot] gather (ks_cons_run / ks_cons_decide)."""
    return sim % world, sim // world


class Consolidator:
    """One disruption pass of consolidation on the GPU (pkg/controllers/disruption).

    Mirrors MultiNodeConsolidation / SingleNodeConsolidation.ComputeCommand over a cluster snapshot
    (INTEGRATION.md §5): every candidate-deletion simulation (simulateScheduling, helpers.go:73-127)
    runs on the GPU with its computeConsolidation decision; `decide` replays the reference's
    sequential choice.  Sharding: rank r of `world` runs simulations s with s % world == r."""

    def __init__(self, snapshot, _binary=None):
        l = _cons_lib()
        h = ctypes.c_void_p()
        if _binary is not None:
            _check(l.ks_cons_create_binary(_binary, len(_binary), ctypes.byref(h)))
        else:
            b = _encode(snapshot)
            _check(l.ks_cons_create(b, len(b), ctypes.byref(h)))
        self._h = h
        self.num_candidates = l.ks_cons_num_candidates(h)
        self.num_sims = l.ks_cons_num_sims(h)
        self.record_bytes = l.ks_cons_record_bytes(h)
        self.requirement_words = l.ks_cons_requirement_words(h)

    @classmethod
    def from_binary(cls, blob):
        """A handle from save()'s binary snapshot (host model + candidates + simulation plan)."""
        return cls(None, _binary=bytes(blob))

    def save(self):
        return _take_bytes(_cons_lib().ks_cons_save, self._h)

    def records_per_rank(self, world=1):
        return _cons_lib().ks_cons_records_per_rank(self._h, world)

    def update(self, delta):
        """Cluster-state events since the snapshot or the last update (ks_cons_update):
        {"deletePods": [uid], "bindPods": [{"uid", "node"}], "removeNodes": [name]}.  The next run()
        simulates the updated cluster; the candidate and simulation counts are refreshed."""
        l = _cons_lib()
        b = _encode(delta)
        _check(l.ks_cons_update(self._h, b, len(b)))
        self.num_candidates = l.ks_cons_num_candidates(self._h)
        self.num_sims = l.ks_cons_num_sims(self._h)
        self._recbuf = None

    def run(self, rank=0, world=1, device=-1, out_ptr=None, keep=False):
        """Run this rank's simulations.  out_ptr: device pointer for records_per_rank*record_bytes
        bytes (e.g. a torch tensor's data_ptr()); None returns the records in host memory.
        Returns (records or None, kernel ms).

        The host records are a memoryview over one buffer per handle that every run() of the handle
        overwrites (no copy per pass): a caller keeping one pass's records across the next run() must copy
        them (bytes(records))."""
        l = _cons_lib()
        o = _Opts(device, 1, 1, 0, 0)
        ms = ctypes.c_double()
        if keep:  # world 1: the records stay in the handle's pinned buffer; pass records=None to decide()
            _check(l.ks_cons_run(self._h, rank, world, ctypes.byref(o), None, 0, ctypes.byref(ms)))
            return None, ms.value
        if out_ptr is None:
            # one host buffer per handle, reused by every pass and handed on without copies (a memoryview,
            # valid until the handle's next run; bytes(view) keeps a copy)
            n = self.records_per_rank(world) * self.record_bytes
            if getattr(self, "_recbuf", None) is None or len(self._recbuf) != n:
                self._recbuf = ctypes.create_string_buffer(n)
            _check(l.ks_cons_run(self._h, rank, world, ctypes.byref(o), ctypes.cast(self._recbuf, ctypes.c_void_p), 0,
                                 ctypes.byref(ms)))
            return memoryview(self._recbuf), ms.value
        _check(l.ks_cons_run(self._h, rank, world, ctypes.byref(o), ctypes.c_void_p(out_ptr), 1, ctypes.byref(ms)))
        return None, ms.value

    def needed_sims(self, records, world=1, all_sims=False):  # noqa: D401
        """Simulations whose NewNodeClaims[0] requirements the decision output needs (in order)."""
        l = _cons_lib()
        buf = _records_buffer(records)
        cap = 64
        while True:
            out = (ctypes.c_int32 * cap)()
            n = l.ks_cons_needed_sims(self._h, ctypes.cast(buf, ctypes.c_void_p), world, 1 if all_sims else 0, out, cap)
            if n < 0:
                _check(n)
            if n <= cap:
                return list(out[:n])
            cap = n

    def claim_requirements(self, sim):
        """NewNodeClaims[0]'s requirement record of `sim` (this rank must have run it)."""
        l = _cons_lib()
        out = (ctypes.c_uint32 * max(l.ks_cons_requirement_words(self._h), 1))()
        _check(l.ks_cons_claim_requirements(self._h, sim, out))
        return bytes(out)

    def decide(self, records, world=1, all_sims=False, fetch=None, candidates=True, clock=None, sims=True):
        """Sequential selection over the gathered records ([rank][slot] layout, bytes).  fetch(sim)
        returns the requirement record bytes of a needed simulation (default: this handle's run);
        candidates=False leaves out the ordered candidate list and sims=False the per-simulation lists (the
        commands are unchanged);
        clock=(multi_timeout_s, single_timeout_s, sim_seconds): the methods' timeouts on a virtual clock."""
        l = _cons_lib()
        if fetch is None and world == 1:
            tbuf = None  # this handle ran every simulation: the library reads the requirement records it needs
        else:
            need = self.needed_sims(records, world, all_sims)
            fetch = fetch or self.claim_requirements
            table = b"".join(fetch(s) for s in need)
            tbuf = ctypes.create_string_buffer(table, max(len(table), 4))
        buf = None if records is None else _records_buffer(records)  # None: the handle's own records (run(keep=True))
        js = ctypes.c_void_p()
        flags = (1 if all_sims else 0) | (2 if candidates else 0) | (0 if sims else 4)
        if clock is None:
            _check(l.ks_cons_decide(self._h, ctypes.cast(buf, ctypes.c_void_p), world, flags,
                                    None if tbuf is None else ctypes.cast(tbuf, ctypes.c_void_p), ctypes.byref(js)))
        else:
            clk = _Clock(*clock)
            _check(l.ks_cons_decide_clock(self._h, ctypes.cast(buf, ctypes.c_void_p), world, flags,
                                          None if tbuf is None else ctypes.cast(tbuf, ctypes.c_void_p), ctypes.byref(clk),
                                          ctypes.byref(js)))
        return json.loads(_take_str(js))

    def validate(self, command, device=-1):
        """Validation.IsValid after its wait + ValidateCommand (validation.go:68-180): `command` (a
        decide() command, computed on an earlier snapshot) re-checked against this handle's snapshot,
        its re-simulation run on the GPU.  Returns {"valid", "reason", "sim"}."""
        b = (command if isinstance(command, str) else json.dumps(command)).encode()
        js = ctypes.c_void_p()
        o = _Opts(device, 1, 1, 0, 0)
        _check(_cons_lib().ks_cons_validate(self._h, b, len(b), ctypes.byref(o), ctypes.byref(js)))
        return json.loads(_take_str(js))

    def sim_counters(self, sim):
        """Solve counters of simulation `sim` from the last run (ks_problem.h Counter order)."""
        out = (ctypes.c_int64 * 64)()  # the library copies min(64, its counter count) and returns that count
        n = _cons_lib().ks_cons_sim_counters_n(self._h, sim, out, 64)
        if n < 0:
            _check(n)
        return list(out)[:n]

    @property
    def last_reruns(self):
        """Multi-node probes the last decide() / needed_sims() re-simulated on this GPU from the pod objects
        earlier probes relaxed (ks_cons_last_reruns; -1: no decision yet)."""
        return _cons_lib().ks_cons_last_reruns(self._h)

    def alg_bytes(self, records, world=1):
        if records is None:
            return _cons_lib().ks_cons_records_alg_bytes(self._h, None, world)
        buf = _records_buffer(records)
        return _cons_lib().ks_cons_records_alg_bytes(self._h, ctypes.cast(buf, ctypes.c_void_p), world)

    def consolidate(self, all_sims=False, device=-1, clock=None):
        recs, ms = self.run(0, 1, device)
        doc = self.decide(recs, 1, all_sims, clock=clock)
        doc["kernel_ms"] = ms
        return doc

    def close(self):
        if self._h:
            _cons_lib().ks_cons_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
