"""Multi-wave simulations (MW, ks_solve.hip mw_helper): a long simulation's register window spread over a
4-wave workgroup (intra-simulation parallelism for the multi-node prefixes).

The 4-wave kernel is opt-in (KS_SIM_MW=1; measured slower end to end); here KS_SIM_MW_MIN=1
sends every simulation of small clusters through it, so runs that cross
window blocks, first fits in each block, pods that fall past the window to the general step, removed and
unusable nodes (AllNonPendingPodsScheduled) and pending pods are all compared with the oracle, simulation by
simulation, and with the single-wave kernel (KS_SIM_MW=0)."""
import json
import os

import pytest

from karpenter_amd import Consolidator, synth
from oracle import bridge

CASES = [  # (seed, nodes, pods per node, pending, not-ready fraction, uninitialized fraction)
    (1, 40, 8, 0, 0.0, 0.0),
    (2, 90, 12, 6, 0.1, 0.0),
    (3, 150, 6, 20, 0.05, 0.05),
    (4, 260, 4, 3, 0.2, 0.0),
    (5, 300, 10, 0, 0.0, 0.1),
]


def _run(snap, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        got = Consolidator(json.dumps(snap)).consolidate(all_sims=True)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    got.pop("kernel_ms")
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("seed,nodes,ppn,pending,nr,un", CASES)
def test_multi_wave_simulations_parity(seed, nodes, ppn, pending, nr, un):
    snap = synth.cluster_snapshot(nodes, ppn, n_its=60, seed=seed, n_pending=pending, not_ready_frac=nr,
                                  uninitialized_frac=un, spot_frac=0.3, it_range=(4, 40))
    want, _ = bridge.consolidate(json.dumps(snap), all_sims=True)
    mw = _run(snap, {"KS_SIM_MW": "1", "KS_SIM_MW_MIN": "1"})
    assert mw == want
    single = _run(snap, {"KS_SIM_MW": "0"})
    assert single == want
