"""ctypes bridge to oracle/_build/liboracle.so (test infrastructure only)."""
import ctypes
import json
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "liboracle_asan.so" if os.environ.get("KS_ORACLE_VARIANT") == "asan"
                    else "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        l = ctypes.CDLL(_LIB)
        l.oref_solve_json.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_double)]
        l.oref_solve_json.restype = ctypes.c_int
        l.oref_time_solve.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        l.oref_time_solve.restype = ctypes.c_int
        l.oref_eval_ops.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
        l.oref_eval_ops.restype = ctypes.c_int
        l.oref_consolidate_json.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                            ctypes.POINTER(ctypes.c_double)]
        l.oref_consolidate_json.restype = ctypes.c_int
        l.oref_consolidate_json_threads.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                                    ctypes.POINTER(ctypes.c_double)]
        l.oref_consolidate_json_threads.restype = ctypes.c_int
        l.oref_consolidate_clock_json.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                                  ctypes.c_double, ctypes.POINTER(ctypes.c_void_p)]
        l.oref_consolidate_clock_json.restype = ctypes.c_int
        l.oref_set_tie_mode.argtypes = [ctypes.c_int, ctypes.c_ulonglong]
        l.oref_set_tie_mode.restype = ctypes.c_int
        l.oref_cluster_state.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
        l.oref_cluster_state.restype = ctypes.c_int
        l.oref_validate_json.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
        l.oref_validate_json.restype = ctypes.c_int
        l.oref_time_cons_sims.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        l.oref_time_cons_sims.restype = ctypes.c_int
        l.oref_last_error.restype = ctypes.c_char_p
        l.oref_free.argtypes = [ctypes.c_void_p]
        _lib = l
    return _lib


def _take(ptr):
    l = lib()
    s = ctypes.cast(ptr, ctypes.c_char_p).value.decode()
    l.oref_free(ptr)
    return s


def solve(snapshot):
    """Run the oracle Solve on a snapshot dict (or JSON string); returns (results dict, seconds)."""
    l = lib()
    s = snapshot if isinstance(snapshot, str) else json.dumps(snapshot)
    out = ctypes.c_void_p()
    secs = ctypes.c_double()
    if l.oref_solve_json(s.encode(), ctypes.byref(out), ctypes.byref(secs)) != 0:
        raise RuntimeError("oracle: " + l.oref_last_error().decode())
    return json.loads(_take(out)), secs.value


def time_solve(snapshot, reps):
    l = lib()
    s = snapshot if isinstance(snapshot, str) else json.dumps(snapshot)
    secs = ctypes.c_double()
    if l.oref_time_solve(s.encode(), reps, ctypes.byref(secs)) != 0:
        raise RuntimeError("oracle: " + l.oref_last_error().decode())
    return secs.value


def consolidate(snapshot, all_sims=False, with_stats=False, threads=1):
    """Oracle multi-node then single-node consolidation over a cluster snapshot; returns (doc, seconds)
    (with_stats: (doc, seconds, stats), stats = {"algBytesRef": SURVEY §8d bytes over the simulations run}).
    all_sims: simulate every candidate / prefix (what the GPU computes) and report each outcome.
    threads > 1 (with all_sims): the simulations are precomputed on that many host threads."""
    l = lib()
    s = snapshot if isinstance(snapshot, str) else json.dumps(snapshot)
    out = ctypes.c_void_p()
    secs = ctypes.c_double()
    if all_sims and threads > 1:
        rc = l.oref_consolidate_json_threads(s.encode(), int(threads), ctypes.byref(out), ctypes.byref(secs))
    else:
        rc = l.oref_consolidate_json(s.encode(), 1 if all_sims else 0, ctypes.byref(out), ctypes.byref(secs))
    if rc != 0:
        raise RuntimeError("oracle: " + l.oref_last_error().decode())
    doc = json.loads(_take(out))
    stats = doc.pop("stats", {})
    return (doc, secs.value, stats) if with_stats else (doc, secs.value)


def consolidate_clock(snapshot, multi_timeout_s, single_timeout_s, sim_seconds, all_sims=False):
    """consolidate() with the methods' timeouts on a virtual clock advancing sim_seconds per simulation."""
    l = lib()
    s = snapshot if isinstance(snapshot, str) else json.dumps(snapshot)
    out = ctypes.c_void_p()
    if l.oref_consolidate_clock_json(s.encode(), 1 if all_sims else 0, multi_timeout_s, single_timeout_s, sim_seconds,
                                     ctypes.byref(out)) != 0:
        raise RuntimeError("oracle: " + l.oref_last_error().decode())
    doc = json.loads(_take(out))
    doc.pop("stats", None)
    return doc


def set_tie_mode(mode, seed=0):
    """Go map-order choice points in the oracle's topology: 0 = canonical (smallest domain name, what the
    GPU reproduces), 1 = largest name, 2 = seeded pseudo-random; 1 and 2 are other outcomes the
    reference's random map iteration can produce."""
    lib().oref_set_tie_mode(mode, seed)


def cluster_state(cluster):
    """Oracle cluster-state accounting (pkg/controllers/state): StateNode accessors from
    {"nodeClaims", "nodes", "pods"}; each node reports `podCount` (its bound pods) instead of the pods."""
    l = lib()
    s = cluster if isinstance(cluster, str) else json.dumps(cluster)
    out = ctypes.c_void_p()
    if l.oref_cluster_state(s.encode(), ctypes.byref(out)) != 0:
        raise RuntimeError("oracle: " + l.oref_last_error().decode())
    return json.loads(_take(out))


def validate(snapshot, command):
    """Oracle Validation.IsValid (after the wait) + ValidateCommand (validation.go:68-180): `command`
    (consolidate()'s command shape) proposed earlier, checked against the current `snapshot`."""
    l = lib()
    s = snapshot if isinstance(snapshot, str) else json.dumps(snapshot)
    c = command if isinstance(command, str) else json.dumps(command)
    out = ctypes.c_void_p()
    if l.oref_validate_json(s.encode(), c.encode(), ctypes.byref(out)) != 0:
        raise RuntimeError("oracle: " + l.oref_last_error().decode())
    return json.loads(_take(out))


def time_cons_sims(snapshot, count, threads=1):
    """Time the oracle's first `count` single-node consolidation simulations over `threads` host
    threads; returns (n, seconds)."""
    l = lib()
    s = snapshot if isinstance(snapshot, str) else json.dumps(snapshot)
    secs = ctypes.c_double()
    n = l.oref_time_cons_sims(s.encode(), count, threads, ctypes.byref(secs))
    if n < 0:
        raise RuntimeError("oracle: " + l.oref_last_error().decode())
    return n, secs.value


def eval_ops(ops, well_known=None):
    l = lib()
    doc = {"ops": ops}
    if well_known is not None:
        doc["wellKnownLabels"] = list(well_known)
    out = ctypes.c_void_p()
    if l.oref_eval_ops(json.dumps(doc).encode(), ctypes.byref(out)) != 0:
        raise RuntimeError("oracle: " + l.oref_last_error().decode())
    return json.loads(_take(out))["results"]
