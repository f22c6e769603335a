"""One consolidation pass sharded over the ranks of a torch.distributed group (bench.py --gpus N, and the
multi-process GPU tests call exactly this).

Every simulation reads the same immutable cluster problem, so rank r runs the simulations s with
s % world == r (Consolidator.run with a device output pointer: ks_cons_run's records_on_device path) and there
is no collective inside the pass.  The exchange after it:
  1. all_gather_into_tensor of the fixed-size records ([rank][slot] layout, shard_slot);
  2. every rank lists the simulations whose NewNodeClaims[0] requirements the decision renders
     (ks_cons_needed_sims; it also resolves firstNConsolidationOption's search with the carried pod objects,
     multinodeconsolidation.go:101-135, re-running carried probes on the rank's own GPU);
  3. one all_reduce builds that requirement table: each owner (sim % world) fills its rows, zeros elsewhere;
  4. rank 0 replays the sequential selection (ks_cons_decide).
On RCCL ("nccl") the records and the table stay in device memory; on gloo (the one-GPU box's multi-process
tests, CPU rehearsals) they are staged through host tensors, the data flow is the same."""
import torch
import torch.distributed as dist


class ShardBuffers:
    """The pass's device buffers for one rank: its records (records_per_rank x record_bytes) and the gather."""

    def __init__(self, c, world, device):
        per, rb = c.records_per_rank(world), c.record_bytes
        self.out = torch.empty(per * rb, dtype=torch.uint8, device=device)
        self.gathered = torch.empty(world * per * rb, dtype=torch.uint8, device=device)


def _host_staged():
    return dist.get_backend() == "gloo"


def sharded_pass(c, rank, world, device, bufs, all_sims=False, candidates=False, sims=False):
    """Run rank `rank`'s simulations, exchange the records and the needed requirement records, decide on rank 0
    (all_sims / candidates / sims: Consolidator.decide's flags).  Returns (kernel ms, gathered records as bytes,
    decision or None on the other ranks)."""
    _, ms = c.run(rank, world, device=device, out_ptr=bufs.out.data_ptr())
    if _host_staged():
        out = bufs.out.cpu()
        gathered = torch.empty(bufs.gathered.numel(), dtype=torch.uint8)
        dist.all_gather_into_tensor(gathered, out)
        recs = gathered.numpy().tobytes()
    else:
        dist.all_gather_into_tensor(bufs.gathered, bufs.out)
        recs = bufs.gathered.cpu().numpy().tobytes()
    need = c.needed_sims(recs, world, all_sims=all_sims)
    rsw = c.requirement_words
    table = {}
    if need:  # one collective: each owner fills its rows, zeros elsewhere, summed over the ranks
        t = torch.zeros(len(need) * rsw, dtype=torch.int32, device="cpu" if _host_staged() else bufs.out.device)
        for i, s in enumerate(need):
            if s % world == rank:
                t[i * rsw:(i + 1) * rsw].copy_(torch.frombuffer(bytearray(c.claim_requirements(s)), dtype=torch.int32))
        dist.all_reduce(t)
        host = t.cpu().numpy()
        table = {s: host[i * rsw:(i + 1) * rsw].tobytes() for i, s in enumerate(need)}
    doc = None
    if rank == 0:
        doc = c.decide(recs, world, all_sims=all_sims, fetch=table.__getitem__, candidates=candidates, sims=sims)
    return ms, recs, doc
