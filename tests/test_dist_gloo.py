"""world_size-2 gloo rehearsal of the multi-GPU consolidation gather (bench.py consolidation_bench):
rank r runs simulations s % world == r and writes them in order of s; an all-gather concatenates
the ranks' record blocks, and ks_cons_decide reads simulation s at [s % world][s // world]
(karpenter_amd.shard_slot).  The records here are stand-ins carrying their simulation id."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from karpenter_amd import shard_slot

NSIMS, WORDS = 23, 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    per = (NSIMS + world - 1) // world
    mine = torch.zeros(per, WORDS, dtype=torch.int32)
    for k, s in enumerate(range(rank, NSIMS, world)):
        mine[k, 0] = s
        mine[k, 1] = 1
    parts = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    if rank == 0:
        g = torch.stack(parts).reshape(world * per, WORDS)
        seen = []
        for s in range(NSIMS):
            r, k = shard_slot(s, world)
            row = g[r * per + k]
            seen.append((int(row[0]), int(row[1])))
        q.put(seen)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_layout_matches_decide_indexing(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    seen = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert seen == [(s, 1) for s in range(NSIMS)]
