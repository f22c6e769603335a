"""The C-ABI from plain C: tests/c/abi_check.c is compiled with gcc against include/karpenter_amd.h only
(what a cgo shim binds) and linked to libkarpenter_amd.so.  CPU: it builds and the
host-only entry point answers like the Python binding.  GPU: a Solve read back through every
structured accessor (NodeClaims with pods / instance types / requests / requirements, existing nodes,
pod errors) equals the canonical JSON document of the same Solve."""
import json
import os
import subprocess

import pytest

import problems
from karpenter_amd import Scheduler, inspect, synth

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
EXE = os.path.join(HERE, "c", "abi_check")


def build():
    import __graft_entry__

    __graft_entry__.build_abi_check()
    return EXE


def _run(mode, snap, tmp_path):
    path = tmp_path / "snap.json"
    path.write_text(json.dumps(snap))
    out = subprocess.run([EXE, mode, str(path)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return json.loads(out.stdout)


def test_c_client_builds_and_inspects(tmp_path):
    build()
    snap = problems.random_problem(5)
    assert _run("inspect", snap, tmp_path) == inspect(snap)


def _req_string(q):  # Requirement.String() without truncation (the JSON's requirements entries)
    s = q["key"] + " " + q["op"]
    if q["op"] in ("In", "NotIn"):
        s += " [" + " ".join(q["values"]) + "]"
    if "gt" in q:
        s += " >%d" % q["gt"]
    if "lt" in q:
        s += " <%d" % q["lt"]
    return s


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 11, 27, 42])
def test_c_client_accessors_match_json(seed, tmp_path):
    if not os.path.exists(EXE):
        build()
    snap = problems.random_problem(seed, n_pods=200, n_nodes=6)
    got = _run("solve", snap, tmp_path)
    want = Scheduler(json.dumps(snap)).solve().canonical()
    its = [it["name"] for it in snap["instanceTypes"]]
    assert len(got["newNodeClaims"]) == len(want["newNodeClaims"])
    for c, w in zip(got["newNodeClaims"], want["newNodeClaims"]):
        assert snap["nodeClaimTemplates"][c["template"]]["metadata"]["name"] == w["nodePoolName"]
        assert c["pods"] == w["pods"]
        assert [its[i] for i in c["instanceTypes"]] == w["instanceTypeOptions"]
        assert c["requests"] == w["requests"]
        assert [_req_string(q) for q in c["requirements"]] == w["requirements"]
    names = [n["name"] for n in snap["stateNodes"]]
    assert sorted((names[n["stateNode"]], n["pods"]) for n in got["existingNodes"]) == \
        sorted((n["name"], n["pods"]) for n in want["existingNodes"])
    assert got["podErrors"] == want["podErrors"]


@pytest.mark.gpu
def test_c_client_bounds_requirements(tmp_path):
    """Gt / Lt bounds reach the structured requirement (C3's integer-label affinity)."""
    if not os.path.exists(EXE):
        build()
    snap = synth.config3(600)
    got = _run("solve", snap, tmp_path)
    want = Scheduler(json.dumps(snap)).solve().canonical()
    for c, w in zip(got["newNodeClaims"], want["newNodeClaims"]):
        assert [_req_string(q) for q in c["requirements"]] == w["requirements"]
