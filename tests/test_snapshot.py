"""Binary snapshots of an encoded problem (ks_problem_save / ks_problem_create_binary, ks_cons_save /
ks_cons_create_binary; SURVEY.md §5 "binary problem file").

CPU: the format is the identity through save -> load -> save (ks_snapshot_check) on every shape the suite
encodes (topology, host ports, volumes, limits, taints, the consolidation cluster), and a truncated or
foreign blob is refused.  GPU: a problem / handle rebuilt from its snapshot gives the Results / decisions of
the one built from JSON, and both equal the oracle."""
import json
import struct

import pytest

import problems

KS_ERR_PARSE = -1
from karpenter_amd import (Consolidator, KsError, Scheduler, check_binary, encode_binary, inspect, snapshot_check,
                           synth)
from oracle import bridge

CPU_CASES = ([("random", s) for s in range(6)] + [("topology", s) for s in range(40, 44)] +
             [("hostports", s) for s in range(60, 62)] + [("c1", 0), ("c3", 300), ("c4", 400), ("cluster", 3),
                                                           ("cluster_topo", 4)])


def _snap(kind, arg):
    if kind == "random":
        return problems.random_problem(arg)
    if kind == "topology":
        return problems.random_problem(arg, n_nodes=12, topology=True, affinity=True)
    if kind == "hostports":
        return problems.random_problem(arg, host_ports=True)
    if kind == "c1":
        return synth.config1(literal=True)
    if kind == "c3":
        return synth.config3(arg)
    if kind == "c4":
        return synth.config4(arg, 80)
    if kind == "cluster":
        return synth.cluster_snapshot(n_nodes=20, pods_per_node=8, n_its=40, seed=arg, n_pending=3)
    return synth.cluster_snapshot(n_nodes=30, pods_per_node=6, n_its=40, seed=arg, n_pending=3, topology=8)


@pytest.mark.parametrize("kind,arg", CPU_CASES, ids=["%s-%s" % c for c in CPU_CASES])
def test_snapshot_roundtrip_is_identity(kind, arg):
    n = snapshot_check(json.dumps(_snap(kind, arg)))
    assert n > 0


GPU_SOLVE_CASES = [("random", s) for s in range(4)] + [("topology", 40), ("topology", 41), ("c1", 0), ("c3", 300)]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,arg", GPU_SOLVE_CASES, ids=["%s-%s" % c for c in GPU_SOLVE_CASES])
def test_solve_from_binary_snapshot(kind, arg):
    s = json.dumps(_snap(kind, arg))
    a = Scheduler(s)
    blob = a.save()
    b = Scheduler.from_binary(blob)
    ra, rb = a.solve(), b.solve()
    assert rb.canonical() == ra.canonical()
    want, _ = bridge.solve(s)
    want.pop("stats", None)
    assert problems.canonical(want) == rb.canonical()
    assert b.save() == blob  # the reloaded model saves to the same bytes
    with pytest.raises(KsError):
        Scheduler.from_binary(blob[: len(blob) // 2])
    a.close()
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,topo", [(3, 0), (4, 8), (5, 0)])
def test_consolidation_from_binary_snapshot(seed, topo):
    snap = synth.cluster_snapshot(n_nodes=24, pods_per_node=8, n_its=40, seed=seed, n_pending=3, topology=topo,
                                  spot_frac=0.5)
    s = json.dumps(snap)
    a = Consolidator(s)
    blob = a.save()
    b = Consolidator.from_binary(blob)
    ga, gb = a.consolidate(all_sims=True), b.consolidate(all_sims=True)
    ga.pop("kernel_ms")
    gb.pop("kernel_ms")
    assert gb == ga
    want, _ = bridge.consolidate(s, all_sims=True)
    assert gb == want
    with pytest.raises(KsError):
        Consolidator.from_binary(b"KSPROB01" + blob[8:])  # a problem's magic on a handle's bytes


def _u64s(blob, at, n):
    return list(struct.unpack_from("<%dQ" % n, blob, at))


def _pods_offsets(blob, n_pods, first_name):
    """Byte position of the pods' io_par offsets: element count n_pods, the offset vector (its length n_pods + 1,
    then the offsets from 0), then the elements, the first of which starts with the first pod's name (a
    length-prefixed string)."""
    pat = struct.pack("<QQQ", n_pods, n_pods + 1, 0)
    name = struct.pack("<Q", len(first_name)) + first_name.encode()
    at = blob.find(pat)
    while at >= 0:
        data = at + 8 * (n_pods + 3)
        off = _u64s(blob, at + 16, n_pods + 1)
        if (all(off[i] <= off[i + 1] for i in range(n_pods)) and off[-1] <= len(blob) - data and
                blob[data:data + len(name)] == name):
            return at + 16
        at = blob.find(pat, at + 1)
    raise AssertionError("pods offset table not found")


def _dims_at(blob, info):
    """Byte position of the serialized KsDims (its leading int32 fields are known from inspect())."""
    nb = info["NB"]
    pre = struct.pack("<13i", info["R"], info["keys"], info["W"], nb, 8 + 4 * nb, info["RSW"], info["T"],
                      info["templates"], info["pools"], info["nodes"], info["pods"], info["states"], info["uids"])
    at = blob.find(pre)
    assert at >= 0 and blob.find(pre, at + 1) < 0
    return at


@pytest.mark.parametrize("kind,arg", [("random", 1), ("topology", 41), ("c3", 300)])
def test_binary_snapshot_rejects_corrupt_blobs(kind, arg):
    """a complete but corrupt blob is a parse error, never an out-of-bounds read: an offset table
    whose element ends past the table's end, dims fields that disagree with the tables, oversized lengths."""
    snap = _snap(kind, arg)
    blob = encode_binary(json.dumps(snap))
    check_binary(blob)  # the untouched blob loads
    info = inspect(json.dumps(snap))
    P = info["pods"]
    # element 0's end offset far past the table's end (off[n] itself unchanged): rejected before any decode
    at = _pods_offsets(blob, P, snap["pods"][0]["metadata"]["name"])
    bad = bytearray(blob)
    struct.pack_into("<Q", bad, at + 8, _u64s(blob, at, P + 1)[-1] + 4096)
    with pytest.raises(KsError) as e:
        check_binary(bad)
    assert e.value.code == KS_ERR_PARSE
    # dims fields flipped: more pods / instance types / resources than the tables hold
    d = _dims_at(blob, info)
    for field, delta in ((10, 1000), (6, 64), (0, 1), (5, 2)):
        bad = bytearray(blob)
        v = struct.unpack_from("<i", bad, d + 4 * field)[0]
        struct.pack_into("<i", bad, d + 4 * field, v + delta)
        with pytest.raises(KsError) as e:
            check_binary(bad)
        assert e.value.code == KS_ERR_PARSE, field
    # a length field claiming 2^33 elements is refused without allocating them
    bad = bytearray(blob)
    struct.pack_into("<Q", bad, at - 16, 1 << 33)
    with pytest.raises(KsError) as e:
        check_binary(bad)
    assert e.value.code == KS_ERR_PARSE
    # truncation anywhere past the header
    for cut in (30, len(blob) // 3, len(blob) - 1):
        with pytest.raises(KsError):
            check_binary(blob[:cut])


@pytest.mark.gpu
def test_create_binary_rejects_flipped_dims():
    snap = problems.random_problem(2)
    s = json.dumps(snap)
    blob = Scheduler(s).save()
    d = _dims_at(blob, inspect(s))
    bad = bytearray(blob)
    struct.pack_into("<i", bad, d + 40, struct.unpack_from("<i", bad, d + 40)[0] + 1000)  # P
    with pytest.raises(KsError) as e:
        Scheduler.from_binary(bytes(bad))
    assert e.value.code == KS_ERR_PARSE


def test_binary_snapshot_version_mismatch_is_named():
    """a blob of an older format version (KSPROB01 / 02 / 03 / 04) is refused as a version mismatch,
    not as an inconsistent table."""
    blob = encode_binary(json.dumps(problems.random_problem(3)))
    assert blob[:8] == b"KSPROB05"
    for old in (b"KSPROB01", b"KSPROB02", b"KSPROB03", b"KSPROB04"):
        with pytest.raises(KsError) as e:
            check_binary(old + blob[8:])
        assert e.value.code == KS_ERR_PARSE and "format version" in str(e.value), str(e.value)


def test_corrupt_element_count_does_not_allocate():
    """a vector of non-trivial elements (pods, nodes) whose count is corrupt grows only with the
    elements actually decoded, so the blob runs out of input (a parse error) instead of forcing a huge
    allocation; here the node list's count is raised to 2^28 in a small blob."""
    snap = problems.random_problem(5, n_nodes=6)
    blob = encode_binary(json.dumps(snap))
    name = snap["stateNodes"][0]["name"]
    enc = struct.pack("<Q", len(name)) + name.encode()
    at = blob.find(struct.pack("<Q", 6) + enc)
    assert at >= 0
    bad = bytearray(blob)
    struct.pack_into("<Q", bad, at, 1 << 28)
    with pytest.raises(KsError) as e:
        check_binary(bytes(bad))
    assert e.value.code == KS_ERR_PARSE
