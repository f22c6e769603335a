"""Multi-process sharded consolidation on the GPU: the exact exchange bench.py's consolidation_bench runs at
--gpus N (karpenter_amd.sharded.sharded_pass, which the bench's world > 1 branch calls and nothing else).  Two
(three) processes, each its own handle on the one GPU of the box, run the simulations s % world == rank with the
records written to device memory (ks_cons_run's records_on_device path), all-gather them, list the simulations
whose NewNodeClaim requirements the decision needs (ks_cons_needed_sims, which also resolves the multi-node
search with the pod objects earlier probes relaxed, re-running carried probes on each rank's GPU), build that
table with one all_reduce, and rank 0 decides.  The transport is gloo staged through host tensors (a one-GPU box
cannot host two RCCL ranks); the calls are the bench's.  Decision == the single-process pass, field for field."""
import json
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _snapshot(kind):
    if kind == "replace":
        from karpenter_amd import synth

        # spot/on-demand mix and small instance types: replacements (NodeClaim requirements needed) and deletes
        return json.dumps(synth.cluster_snapshot(40, 8, n_its=60, it_range=(6, 30), seed=11, spot_frac=0.5))
    import carry_scenarios as cs  # probes holding pods an earlier probe relaxed (re-run per rank)

    return json.dumps(cs.random_cluster(4, topology=False) if kind == "carry" else cs.make("late-carry", 0))


def _worker(rank, world, port, kind, q):
    import sys

    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from karpenter_amd import Consolidator
    from karpenter_amd.sharded import ShardBuffers, sharded_pass

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        snap = _snapshot(kind)
        c = Consolidator(snap)
        bufs = ShardBuffers(c, world, "cuda:0")
        _, recs, got = sharded_pass(c, rank, world, 0, bufs, all_sims=True, candidates=True, sims=True)
        need = c.needed_sims(recs, world, all_sims=True)
        if rank == 0:
            ref = Consolidator(snap)
            want = ref.decide(ref.run(0, 1)[0], 1, all_sims=True)
            q.put((json.dumps(got, sort_keys=True), json.dumps(want, sort_keys=True), len(need)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["replace", "carry", "late-carry"])
@pytest.mark.parametrize("world", [2, 3])
def test_multiprocess_sharded_pass_decides_like_one_process(world, kind):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, want, nneed = q.get(timeout=150)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == want
    doc = json.loads(want)
    assert doc["multi"]["sims"] or doc["single"]["sims"]
    if kind == "replace":
        assert nneed > 0  # the decision renders replacement requirements another rank's GPU holds
    else:
        assert any(p["carried"] for p in doc["multi"]["path"])
