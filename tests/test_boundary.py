"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every declared symbol,
the host encoder accepts the reference-shaped snapshots and rejects unsupported inputs loudly."""
import ctypes
import os
import re

import pytest

import problems
from karpenter_amd import KsError, inspect, lib, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "karpenter_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ks_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    l = lib()
    syms = declared_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(l, s)]
    assert not missing, missing


def test_build_info_and_device_count_without_gpu():
    l = lib()
    l.ks_build_info.restype = ctypes.c_char_p
    assert b"gfx950" in l.ks_build_info()
    assert l.ks_device_count() >= 0


def test_inspect_config2_layout():
    d = inspect(synth.config2(1000))
    assert d["T"] == 400 and d["R"] == 3 and d["templates"] == 1 and d["pods"] == 1000
    assert "kubernetes.io/hostname" in d["keyNames"]
    assert d["TW"] == 13  # 400 instance types -> 13 bitset words


@pytest.mark.parametrize("seed", range(10))
def test_inspect_random_problems(seed):
    d = inspect(problems.random_problem(seed))
    assert d["keys"] <= 64 and d["states"] >= d["pods"]


def test_unsupported_topology_is_loud():
    snap = synth.config2(10)
    snap["topology"] = {"groups": []}
    with pytest.raises(KsError) as e:
        inspect(snap)
    assert e.value.code == -2


def test_host_ports_are_encoded():
    snap = synth.config2(10)
    snap["pods"][0]["spec"]["containers"][0]["ports"] = [{"hostPort": 80, "containerPort": 80}]
    snap["stateNodes"] = []
    assert inspect(snap)["pods"] == 10


def test_pod_holding_its_own_host_ports_encodes():
    """Conflicts' same-pod exception (hostportusage.go:78): a pod being scheduled whose key already holds
    ports on an existing node is encoded (its own entries are left out of its conflict mask)."""
    snap = problems.random_problem(3, n_nodes=2)
    snap["pods"][0]["spec"]["containers"][0]["ports"] = [{"hostPort": 80, "containerPort": 80}]
    p0 = snap["pods"][0]["metadata"]
    snap["stateNodes"][0]["hostPortUsage"] = {"%s/%s" % (p0["namespace"], p0["name"]): [{"port": 80}]}
    assert inspect(snap)["pods"] == len(snap["pods"])


def test_same_key_pods_with_host_ports_are_loud():
    """Two pods being scheduled under one namespace/name with host ports: HostPortUsage.Add on a NodeClaim
    would replace one's entries with the other's, which is not encoded."""
    snap = problems.random_problem(3, n_nodes=2)
    snap["pods"][0]["spec"]["containers"][0]["ports"] = [{"hostPort": 80, "containerPort": 80}]
    snap["pods"][1]["metadata"]["name"] = snap["pods"][0]["metadata"]["name"]
    with pytest.raises(KsError) as e:
        inspect(snap)
    assert e.value.code == -2


def test_queue_key_ties_encode():
    """Pods tying on the whole NewQueue key (cpu, memory, creation time, UID — BenchmarkScheduling's
    un-applied pods) get their order from the host's sort.Slice emulation (queue.go:38)."""
    snap = synth.config2(10)
    snap["pods"][1] = dict(snap["pods"][0])
    d = inspect(snap)
    assert d["hostQueue"] == 1 and d["uids"] == 9
    assert inspect(synth.config1(literal=True))["hostQueue"] == 1
    assert inspect(synth.config1())["hostQueue"] == 0


def test_groups_created_mid_solve_encode():
    """A relaxed state whose spread group re-hashes (OR'd required terms, topology.go:102-119) gets a
    late group, activated by the kernel at that relaxation."""
    snap = problems.random_problem(460, n_pods=150, topology=True, or_terms=True)
    assert inspect(snap)["lateGroups"] > 0


def test_shared_uids_with_topology_are_loud():
    """TopologyGroup owners are keyed by UID: pods sharing one with topology groups are refused."""
    snap = problems.random_problem(5, topology=True)
    for p in snap["pods"]:
        p["metadata"]["uid"] = ""
    with pytest.raises(KsError) as e:
        inspect(snap)
    assert e.value.code == -2


def test_bad_quantity_is_parse_error():
    snap = synth.config2(10)
    snap["pods"][0]["spec"]["containers"][0]["resources"]["requests"]["cpu"] = "12q"
    with pytest.raises(KsError) as e:
        inspect(snap)
    assert e.value.code == -1


def test_more_than_64_label_keys_is_capacity_error():
    """The requirement encoding holds at most 64 label keys; beyond that the library
    refuses with KS_ERR_CAPACITY instead of approximating."""
    snap = synth.config2(70)
    for i, p in enumerate(snap["pods"]):
        p["spec"]["nodeSelector"] = {"example.com/key-%03d" % i: "v"}
    with pytest.raises(KsError) as e:
        inspect(snap)
    assert e.value.code == -3, e.value


def test_64_label_keys_or_fewer_encode():
    snap = synth.config2(40)
    for i, p in enumerate(snap["pods"]):
        p["spec"]["nodeSelector"] = {"example.com/key-%03d" % i: "v"}
    assert inspect(snap)["keys"] <= 64


def test_cluster_state_rejects_bad_input_loudly():
    from karpenter_amd import cluster_state
    with pytest.raises(KsError) as e:
        cluster_state("[1, 2]")
    assert e.value.code == -1
    with pytest.raises(KsError):
        cluster_state('{"nodes": [{"metadata": {"name": "n"}, "spec": {"providerID": "p"}, '
                      '"status": {"allocatable": {"cpu": "12q"}}}]}')
