"""Empty and ragged inputs (the edge cases the reference tests exercise): snapshots shared by
the CPU checks (oracle + host encoder) and the GPU parity tests."""
import copy

from karpenter_amd import synth


def solve_cases():
    base = synth.benchmark_snapshot(40, n_its=30, seed=3)
    out = {}
    s = copy.deepcopy(base)
    s["pods"] = []
    out["no-pods"] = s
    s = copy.deepcopy(base)
    s["instanceTypes"] = []
    s["instanceTypesByNodePool"] = {k: [] for k in s["instanceTypesByNodePool"]}
    out["no-instance-types"] = s
    s = copy.deepcopy(base)
    s["nodeClaimTemplates"] = []
    s["nodePools"] = []
    out["no-templates-no-nodes"] = s
    s = copy.deepcopy(base)
    s["pods"] = [synth.pod(i) for i in range(7)]  # no requests at all: only pods=1 each
    out["requestless-pods"] = s
    s = copy.deepcopy(base)
    s["pods"] = s["pods"][:1]
    out["single-pod"] = s
    s = copy.deepcopy(base)
    big = synth.pod(999, cpu="100000", mem="1Ti")
    s["pods"] = [big] + s["pods"][:5]
    out["one-unschedulable"] = s
    return out


def cons_cases():
    out = {}
    snap = synth.cluster_snapshot(8, 4, n_its=30, it_range=(4, 20), seed=9)
    s = copy.deepcopy(snap)
    s["candidates"] = []
    out["no-candidates"] = s
    s = copy.deepcopy(snap)
    s["candidates"] = s["candidates"][:1]
    out["one-candidate"] = s
    s = copy.deepcopy(snap)
    s["candidates"] = ["no-such-node"] + s["candidates"][:2]
    out["unknown-candidate"] = s
    s = copy.deepcopy(snap)
    for n in s["stateNodes"]:
        n["pods"] = []
    out["empty-nodes"] = s
    return out
