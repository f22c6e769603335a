"""Full-size parity at the BASELINE.json configs: the HIP path's canonical results against sha256 digests
of the oracle's results at the same sizes (tests/golden/full_size_digests.json, written in the build
container by tests/golden/make_full_size_digests.py, where the oracle needs minutes per config).

  C1  BenchmarkScheduling2000 with the benchmark's literal pods (empty UIDs, zero timestamps)
  C2  Scheduler.Solve, 50k pods x 400 instance types                       (scheduler.go:140-189)
  C3  20k pods, 800 instance types x 8 offerings, selectors / affinity / taints
  C4  10k pods onto 2k existing nodes, zonal + hostname spread, anti-affinity
  C5  consolidation over the 5k-node / 100k-pod cluster: every multi-node prefix and single-node
      simulation with its outcome and its own computeConsolidation command, and both commands
      (multinodeconsolidation.go:87-137, singlenodeconsolidation.go:42-88)
Decision-exercising variants (make_full_size_digests.py): C4X (NodeClaims under topology and
unsatisfiable hostname affinity PodErrors), C5R (Replace / NoOp: filterByPrice, spot rules,
filterOutSameType on a 5k-node cluster), C5T (the bench's consolidation-with-topology cluster).

A digest mismatch names the first differing NewNodeClaim / simulation."""
import hashlib
import json
import os

import pytest

from karpenter_amd import Consolidator, Scheduler

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
DIGESTS = json.load(open(os.path.join(HERE, "golden", "full_size_digests.json")))


def _mfd():
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_full_size_digests as m
    return m


def _snapshot(name):
    m = _mfd()
    snap = json.dumps(m.CONFIGS[name]())
    assert hashlib.sha256(snap.encode()).hexdigest() == DIGESTS[name]["snapshot"], \
        "synthetic %s input changed since the digests were made: re-run make_full_size_digests.py" % name
    return snap


def _check_solve(name):
    m = _mfd()
    want = DIGESTS[name]
    got = m.solve_digest(Scheduler(_snapshot(name)).solve().canonical())
    assert got["counts"] == want["counts"], (got["counts"], want["counts"])
    for i, (a, b) in enumerate(zip(got["newNodeClaims"], want["newNodeClaims"])):
        assert a == b, "%s: NewNodeClaims[%d] differs from the oracle" % (name, i)
    for k in ("existingNodes", "podErrors"):
        assert got[k] == want[k], "%s: %s differ from the oracle" % (name, k)
    assert got["all"] == want["all"]


def test_c1_literal_benchmark_scheduling_2000():
    _check_solve("C1")


def test_c2_50k_pods_400_instance_types():
    _check_solve("C2")


def test_c3_20k_pods_800_instance_types():
    _check_solve("C3")


def test_c4_10k_pods_onto_2k_nodes_topology():
    _check_solve("C4")


def test_c4x_overflow_to_nodeclaims_and_hostname_errors():
    want = DIGESTS["C4X"]["counts"]
    assert want["newNodeClaims"] > 0 and want["podErrors"] > 0
    _check_solve("C4X")


@pytest.mark.parametrize("name", ["C5", "C5R", "C5T"])
def test_c5_every_consolidation_simulation(name):
    m = _mfd()
    want = DIGESTS[name]
    if name == "C5R":  # the decisions this variant exists for
        acts = want["summary"]["singleActions"]
        assert acts["replace"] > 0 and acts["no-op"] > 0 and acts["delete"] > 0
    doc = Consolidator(_snapshot(name)).consolidate(all_sims=True)
    doc.pop("kernel_ms")
    got = m.cons_digest(doc)
    assert got["summary"] == want["summary"], (got["summary"], want["summary"])
    assert got["candidates"] == want["candidates"], "candidate order / disruption costs differ"
    for kind in ("multi", "single"):
        assert len(got[kind]["sims"]) == len(want[kind]["sims"])
        for i, (a, b) in enumerate(zip(got[kind]["sims"], want[kind]["sims"])):
            assert a == b, "%s simulation %d (%s) differs from the oracle" % (kind, i, doc[kind]["sims"][i]["candidates"][:3])
        assert got[kind]["command"] == want[kind]["command"], "%s command differs" % kind
    assert got["multi"]["path"] == want["multi"]["path"], "multi-node search path differs"
    assert got["all"] == want["all"]
