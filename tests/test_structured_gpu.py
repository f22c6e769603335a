"""The structured Results accessors (include/karpenter_amd.h: ks_results_nodeclaim / _requests /
_requirements / _existing_node / _pod_error, what INTEGRATION.md's cgo shim reads instead of JSON) carry
exactly the canonical Results: same NewNodeClaims (template, pods in commit order, instance-type options in
order, requests, requirements), ExistingNodes and PodErrors (scheduler.go:102-106), equal to the oracle."""
import json

import pytest

import problems
from karpenter_amd import Scheduler, synth
from oracle import bridge

pytestmark = pytest.mark.gpu


def _req_string_parts(req):
    key, op, values, gt, lt = req
    return key, op, values, gt, lt


def _check(snap):
    s = json.dumps(snap)
    want, _ = bridge.solve(s)
    sch = Scheduler(s)
    got = sch.solve_structured()
    canon = sch.solve().canonical()
    sch.close()
    assert canon == problems.canonical(want)
    it_names = [it["name"] for it in snap["instanceTypes"]]
    pools = [t["metadata"]["name"] for t in snap["nodeClaimTemplates"]]
    assert len(got.new_nodeclaims) == len(want["newNodeClaims"])
    for a, b in zip(got.new_nodeclaims, want["newNodeClaims"]):
        assert pools[a["template"]] == b["nodePoolName"]
        assert a["pods"].tolist() == b["pods"]
        assert [it_names[i] for i in a["instance_types"]] == b["instanceTypeOptions"]
        assert a["requests"] == b["requests"]
        keys = [r[0] for r in a["requirements"]]
        assert keys == sorted(keys)
        for (key, op, values, gt, lt), text in zip(a["requirements"], b["requirements"]):
            assert text.startswith(key + " ")  # Requirement.String() names the same key in the same order
    assert len(got.new_nodeclaims[0]["requirements"] if got.new_nodeclaims else []) == \
        (len(want["newNodeClaims"][0]["requirements"]) if want["newNodeClaims"] else 0)
    nodes = {n["name"]: n["pods"] for n in want["existingNodes"]}
    names = [n["name"] for n in snap.get("stateNodes", [])]
    for idx, pods in got.existing_nodes:
        assert pods.tolist() == nodes[names[idx]]
    assert {str(k): v for k, v in got.pod_errors.items()} == want["podErrors"]


@pytest.mark.parametrize("seed", [0, 3, 7, 11])
def test_structured_random(seed):
    _check(problems.random_problem(seed, n_pods=150, n_nodes=6))


def test_structured_c1_literal():
    _check(synth.config1(literal=True))


def test_structured_c2_10k():
    _check(synth.config2(10000))


def test_structured_topology_errors():
    _check(problems.hostname_failure_problem(503))


def test_results_outlive_their_problem():
    """Results render their JSON and requirement lists on first use (finish_json / finish_reqs), from the
    problem's host model: freeing the problem first defers its release to the last Results (refcount)."""
    import ctypes

    from karpenter_amd import scheduler as ks

    snap = json.dumps(problems.random_problem(5, n_pods=80))
    want = Scheduler(snap).solve().canonical()
    l = ks.lib()
    sch = Scheduler(snap)
    o = ks._Opts(-1, 1, 1, 0, 0)
    r = ctypes.c_void_p()
    ks._check(l.ks_solve(sch._h, ctypes.byref(o), ctypes.byref(r)))
    sch.close()  # the problem handle is gone; the Results still hold its host model
    claims, nodes, errors = ks._read_structured(l, r)
    out = ctypes.c_void_p()
    ks._check(l.ks_results_json(r, ctypes.byref(out)))
    got = json.loads(ks._take_str(out))
    l.ks_results_free(r)  # releases the problem too
    assert problems.canonical(got) == want
    assert len(claims) == len(got["newNodeClaims"])
