"""Multi-process sharded consolidation on the GPU: the exchange bench.py's consolidation_bench runs at
--gpus N, with real simulation records instead of stand-ins (tests/test_dist_gloo.py rehearses only the
layout).  Two (three) processes, each its own handle on the one GPU of the box, run the simulations
s % world == rank; the records are all-gathered, every rank derives the simulations whose NewNodeClaim
requirements the decision needs (ks_cons_needed_sims), the owner of each broadcasts its record, and rank 0
replays the reference's selection.  The transport here is gloo over host memory (a one-GPU box cannot host
two RCCL ranks); the data flow is the bench's.  Decision == the single-process pass, field for field."""
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


def _snapshot():
    from karpenter_amd import synth

    # spot/on-demand mix and small instance types: replacements (NodeClaim requirements needed) and deletes
    return json.dumps(synth.cluster_snapshot(40, 8, n_its=60, it_range=(6, 30), seed=11, spot_frac=0.5))


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from karpenter_amd import Consolidator

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        snap = _snapshot()
        c = Consolidator(snap)
        mine, _ = c.run(rank, world)
        out = torch.frombuffer(bytearray(bytes(mine)), dtype=torch.uint8)
        parts = [torch.empty_like(out) for _ in range(world)]
        dist.all_gather(parts, out)
        recs = b"".join(bytes(p.numpy()) for p in parts)
        need = c.needed_sims(recs, world, all_sims=True)
        table = {}
        for s in need:
            t = torch.zeros(c.requirement_words, dtype=torch.int32)
            if rank == s % world:
                t.copy_(torch.frombuffer(bytearray(c.claim_requirements(s)), dtype=torch.int32))
            dist.broadcast(t, src=s % world)
            table[s] = bytes(t.numpy())
        if rank == 0:
            got = c.decide(recs, world, all_sims=True, fetch=table.__getitem__)
            ref = Consolidator(snap)
            want = ref.decide(ref.run(0, 1)[0], 1, all_sims=True)
            q.put((json.dumps(got, sort_keys=True), json.dumps(want, sort_keys=True), len(need)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_multiprocess_sharded_pass_decides_like_one_process(world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, want, nneed = q.get(timeout=150)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == want
    assert json.loads(want)["multi"]["sims"] or json.loads(want)["single"]["sims"]
