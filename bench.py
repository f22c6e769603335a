#!/usr/bin/env python3
"""Benchmark: pods/sec in Scheduler.Solve at 50k pods x 400 instance types (BASELINE.json configs[1]).

One step = one complete Solve (scheduler.go:140-189) of the C2 problem with fresh scheduler state,
inputs already resident in HBM (the snapshot is encoded and uploaded once, like NewScheduler).
Solve does not shard (every placement depends on all earlier ones), so N GPUs run N independent
replicas, one per rank ("replicas only"); value = pods solved by all ranks / max-rank time.

Prints ONE JSON line on rank 0 (the driver's contract), including:
  create_ms / e2e_*  what a drop-in caller pays: ks_problem_create (parse + encode + upload, the
                     NewScheduler-time work) and the rate including it and the results copy-back
  roofline     : dominant kernel k_solve, HIP-event duration vs the 8 TB/s HBM peak, for two byte
                 counts: the kernel's own scan (algorithmic_bytes_per_launch) and SURVEY.md §8d's
                 reference scan (algorithmic_bytes_ref, counted by the oracle); traffic = PMC HBM bytes
                 from the committed profile named in traffic_source
  cpu_baseline : the oracle (C++ restatement of the reference Solve) timed on this host on the same
                 workload, with the host's nproc / CPU model and the threads used
  solve_c1/c3/c4, consolidation(_topology): the other BASELINE.json configs, each with the same fields
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "karpenter-sigs_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
DIGESTS = os.path.join(ROOT, "tests", "golden", "full_size_digests.json")


def _host():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "cpu_model": model}


def _baseline(value, unit, threads, sample, secs):
    d = {"value": round(value, 2), "unit": unit, "cores": threads, "threads": threads, "kind": "port",
         "sample": sample + " (oracle/cpu_ref.cpp, %d host thread%s, %.1f s)" % (threads, "" if threads == 1 else "s", secs),
         "gomaxprocs": "n/a (no Go reference on this host)"}
    d.update(_host())
    return d


def _ref_bytes(name, snap_json):
    """SURVEY.md §8d algorithmic bytes of the reference's scan for a BASELINE config, as the oracle counted
    them when tests/golden/full_size_digests.json was made (the oracle needs minutes at these sizes);
    None if the workload is not the committed one."""
    try:
        d = json.load(open(DIGESTS)).get(name)
    except OSError:
        return None
    if not d or hashlib.sha256(snap_json.encode()).hexdigest() != d.get("snapshot"):
        return None
    return d.get("algBytesRef")


def _oracle_full(name, snap_json, units, unit):
    """The oracle on the whole workload (not a sample), as timed when tests/golden/full_size_digests.json was
    made: single-threaded for Solve, the threaded precompute for consolidation, in the build container (not
    on this host).  None if the workload is not the committed one."""
    try:
        d = json.load(open(DIGESTS)).get(name)
    except OSError:
        return None
    if not d or not d.get("oracle_seconds") or hashlib.sha256(snap_json.encode()).hexdigest() != d.get("snapshot"):
        return None
    return {"seconds": d["oracle_seconds"], "value": round(units / d["oracle_seconds"], 2), "unit": unit,
            "where": "build container, when the full-size digests were made (tests/golden/full_size_digests.json)"}


_LIB_SHA = None


def _lib_sha():
    """sha256 of the libkarpenter_amd build this process loaded."""
    global _LIB_SHA
    if _LIB_SHA is None:
        from karpenter_amd.scheduler import library_path

        with open(library_path(), "rb") as f:
            _LIB_SHA = hashlib.sha256(f.read()).hexdigest()
    return _LIB_SHA


def _traffic(tag):
    """(HBM bytes per launch, source, build match) of the committed PMC profile for `tag`.  build match: the
    profile was taken on the library this process loaded (False: a different build -- the figure is stale;
    None: the profile predates the build record)."""
    tpath = os.path.join(ROOT, "profiles", "traffic_%s.json" % tag)
    if os.path.exists(tpath):
        with open(tpath) as f:
            t = json.load(f)
        match = None if not t.get("lib_sha256") else t["lib_sha256"] == _lib_sha()
        src = "profiles/traffic_%s.json (rocprofv3 PMC, profile tag %s%s)" % (
            tag, t.get("tag"), "" if match else ", STALE: profiled on another build" if match is False
            else ", build unrecorded")
        return t.get("hbm_bytes_per_launch"), src, match
    return None, None, None


def _roofline(kernel, k_ms, kernel_bytes, ref_bytes, traffic_tag, per_gpu_div=1, extra=None):
    """The dominant kernel's roofline.  `frac` is always a physical fraction of the 8 TB/s HBM peak (<= 1):
    achieved / frac: SURVEY.md §8d algorithmic bytes -- the reference's scan, counted by the oracle on this exact
    workload (tests/golden/full_size_digests.json) -- per launch, over the HIP-event launch duration, when that
    rate is one HBM could deliver (the Solve lines).  Where it is not (the consolidation passes: the kernel
    skips scans the reference makes -- identical-pod runs placed in one step, the infeasible-topology
    shortcut -- so the reference-scan bytes it stands for exceed what HBM could move in that time), achieved /
    frac are the rocprofv3 PMC bytes per launch (FETCH_SIZE + WRITE_SIZE of the committed profile in
    traffic_source) over the same duration, i.e. what the kernel really moves, and `frac_basis` says so.
    reference_scan_achieved / reference_scan_frac: the §8d ratio itself, kept beside it on every line.
    hbm_achieved / hbm_frac: the PMC rate on every line that has a committed profile.
    kernel_scan_bytes / kernel_scan_frac: the kernel's own scan count (each pod of an identical-pod run
    credited with the first pod's scan), a bookkeeping figure."""
    traffic, src, match = _traffic(traffic_tag)
    sec = k_ms / 1000.0
    alg, asrc = (ref_bytes, "SURVEY 8d reference scan, oracle count (tests/golden/full_size_digests.json)") if ref_bytes \
        else (kernel_bytes, "kernel-counted scan (no oracle count for this workload)")
    ref_achieved = alg / sec / 1e9 / per_gpu_div
    r = {"bound": "hbm", "kernel": kernel, "achieved": round(ref_achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": ref_achieved / HBM_PEAK_GBS, "frac_basis": "algorithmic bytes (%s)" % asrc, "traffic": traffic,
         "traffic_source": src, "traffic_build_match": match, "algorithmic_bytes_per_launch": alg, "algorithmic_bytes_source": asrc,
         "kernel_ms": round(k_ms, 3), "reference_scan_achieved": round(ref_achieved, 3),
         "reference_scan_frac": ref_achieved / HBM_PEAK_GBS, "hbm_achieved": None, "hbm_frac": None,
         "kernel_scan_bytes": kernel_bytes,
         "kernel_scan_frac": kernel_bytes / sec / 1e9 / per_gpu_div / HBM_PEAK_GBS}
    if traffic:
        ha = traffic / sec / 1e9 / per_gpu_div
        r["hbm_achieved"] = round(ha, 3)
        r["hbm_frac"] = ha / HBM_PEAK_GBS
    if r["reference_scan_frac"] > 1:
        # not a bandwidth: report the physical PMC rate as the roofline (null without a committed profile)
        r["achieved"] = r["hbm_achieved"]
        r["frac"] = r["hbm_frac"]
        r["frac_basis"] = ("rocprofv3 PMC HBM bytes per launch (%s): the §8d reference-scan rate (reference_scan_frac) "
                           "exceeds the HBM peak because the kernel skips scans the reference makes" % src)
    if extra:
        r.update(extra)
    return r


def _pct(xs, q):
    """Nearest-rank percentile."""
    ys = sorted(xs)
    return ys[min(len(ys) - 1, max(0, -(-q * len(ys) // 100) - 1))]


def _create(cls, snap_json):
    """(handle, create_ms): the second of two constructions (the first pays the process's HIP init)."""
    cls(snap_json).close()
    t = time.perf_counter()
    h = cls(snap_json)
    return h, (time.perf_counter() - t) * 1000.0


def _create_binary(h, cls):
    """(save_ms, create_binary_ms, snapshot bytes): the handle rebuilt from its binary snapshot (the second of
    two loads, like _create), i.e. what a caller that keeps the encoded problem pays instead of create_ms."""
    t = time.perf_counter()
    blob = h.save()
    save_ms = (time.perf_counter() - t) * 1000.0
    cls.from_binary(blob).close()
    t = time.perf_counter()
    x = cls.from_binary(blob)
    load_ms = (time.perf_counter() - t) * 1000.0
    x.close()
    return save_ms, load_ms, len(blob)


def consolidation_bench(args, rank, world, local, dist, barrier_sync, topology=0):
    """C5 (BASELINE.json configs[4]): one consolidation pass = every candidate-deletion simulation of
    a 5k-node / 100k-pod cluster (5000 single-node + 100 multi-node prefix sims), sharded over the
    ranks by simulation index (s % world == rank), records all-gathered over RCCL, then the
    reference's sequential selection on rank 0.  value = simulations completed per second.
    topology=A: the same cluster with its pods in A apps carrying zonal / hostname spread, pod
    affinity and anti-affinity (synth.cluster_snapshot), every bound pod listed in clusterPods."""
    import torch

    from karpenter_amd import Consolidator, synth
    from karpenter_amd.sharded import ShardBuffers, sharded_pass

    snap = json.dumps(synth.config5(args.cons_nodes) if not topology else
                      synth.cluster_snapshot(args.cons_nodes, 20, 400, seed=4205, topology=topology))
    c, create_ms = _create(Consolidator, snap)
    save_ms, create_bin_ms, snap_bytes = _create_binary(c, Consolidator)
    dev = "cuda:%d" % local
    bufs = ShardBuffers(c, world, dev) if world > 1 else None

    def one_pass():
        if world == 1:  # the records stay in the handle's pinned buffer (decide reads them there)
            recs, ms = c.run(0, 1, device=local, keep=True)
            return ms, recs, c.decide(recs, 1, candidates=False, sims=False)
        # records on the device, all-gathered over RCCL; the needed requirement records in one all_reduce; rank 0
        # decides (karpenter_amd.sharded: the same function the multi-process GPU tests run)
        return sharded_pass(c, rank, world, local, bufs)

    t0 = time.perf_counter()
    one_pass()  # first pass: includes the launch plan's build and upload (prepare_launch)
    first_ms = (time.perf_counter() - t0) * 1000.0
    for _ in range(args.warmup):
        one_pass()
    barrier_sync()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.cons_steps):
        ms, recs, doc = one_pass()
        kms.append(ms)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed, max(kms)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kmax = float(t[0]), float(t[1])
    else:
        kmax = max(kms)
    if rank != 0:
        return None
    k_ms = sum(kms) / len(kms)
    algb = c.alg_bytes(recs, world)
    ref = _ref_bytes("C5T" if topology else "C5", snap)
    cpu = cpu1 = None
    if not args.no_cpu_baseline and world == 1:
        from oracle import bridge

        n_sims = args.cpu_sims if not topology else args.cpu_topo_sims
        n, secs = bridge.time_cons_sims(snap, n_sims, args.cpu_threads)
        cpu = _baseline(n / secs, "cands/s", args.cpu_threads,
                        "first %d single-node simulations of the same cluster (simulateScheduling + "
                        "computeConsolidation)" % n, secs)
        n1, secs1 = bridge.time_cons_sims(snap, max(n_sims // (4 * args.cpu_threads), 8), 1)
        cpu1 = _baseline(n1 / secs1, "cands/s", 1, "first %d single-node simulations of the same cluster "
                         "(sequential, as the reference's single goroutine runs them)" % n1, secs1)
    # Strong-scaling evidence on one GPU: the pass sharded as `world` ranks would run it (s % world == rank),
    # each shard's launch timed alone; a world-rank pass is bounded below by its slowest shard's kernel.
    shards = None
    if world == 1 and not args.no_shards:
        shards = {}
        for w in (2, 4, 8):
            per = []
            for r in range(w):
                c.run(r, w, device=local)  # the shard's launch plan
                per.append(min(c.run(r, w, device=local)[1] for _ in range(3)))
            shards[str(w)] = {"max_kernel_ms": round(max(per), 4), "mean_kernel_ms": round(sum(per) / w, 4),
                              "max_over_world1_kernel": round(max(per) / k_ms, 3)}
        c.run(0, 1, device=local)  # restore the whole-pass plan
    # Validation.IsValid + ValidateCommand (validation.go:68-180) of the command the controller would run
    # (multi-node first): one re-simulation on the GPU, timed after the passes (its own launch)
    final = doc["multi"]["command"] if doc["multi"]["command"]["action"] != "no-op" else doc["single"]["command"]
    vms = []
    for _ in range(3):
        tv = time.perf_counter()
        v = c.validate(final, device=local)
        vms.append((time.perf_counter() - tv) * 1000.0)
    validation = {"command": [final["action"], len(final["candidates"])], "valid": v["valid"], "reason": v["reason"],
                  "ms": round(sorted(vms)[1], 3)}
    name = "C5" if not topology else "C5 + topology (%d apps: spread, pod affinity, anti-affinity)" % topology
    pass_ms = elapsed * 1000.0 / args.cons_steps
    # Incremental update between passes (ks_cons_update): 10 pods deleted on one node and one node removed,
    # then the next pass (new plan: pod lists, queue sort, run lengths; simulations; decide), 5 times.  On a
    # topology cluster the update also moves the shared NewTopology counts and the pass re-derives every
    # simulation's count offsets.
    update = None
    if world == 1:
        nodes = json.loads(snap)["stateNodes"]
        ums, pms = [], []
        for i in range(5):
            a, b = nodes[200 + 2 * i], nodes[201 + 2 * i]
            delta = {"deletePods": [p["metadata"]["uid"] for p in a.get("pods", [])[:10]], "removeNodes": [b["name"]]}
            t0 = time.perf_counter()  # (the previous pass ended with its stream synchronized)
            c.update(delta)
            t1 = time.perf_counter()
            one_pass()
            t2 = time.perf_counter()
            ums.append((t1 - t0) * 1000.0)
            pms.append((t2 - t1) * 1000.0)
        tot = sorted(u + p for u, p in zip(ums, pms))
        update = {"events": "10 pod deletions + 1 node removal per update", "updates": len(ums),
                  "update_ms": round(sorted(ums)[len(ums) // 2], 3),
                  "pass_after_update_ms": round(sorted(pms)[len(pms) // 2], 3),
                  "update_plus_pass_ms": round(tot[len(tot) // 2], 3),
                  "update_plus_pass_ms_max": round(tot[-1], 3),
                  "vs_create_plus_first_pass_ms": round(create_ms + first_ms, 3)}
    return {
        "metric": "consolidation cands/sec (%s: %d nodes x 20 pods, 400 instance types)" % (name, args.cons_nodes),
        "value": round(c.num_sims * args.cons_steps / elapsed, 1),
        "unit": "cands/s",
        "n_gpus": world,
        "steps": args.cons_steps,
        "ms_per_pass": round(pass_ms, 3),
        "scaling": "strong",
        "simulations_per_pass": c.num_sims,
        "candidates": c.num_candidates,
        # ks_cons_create: parse + NewCandidate + encode + upload of the cluster snapshot (once per pass in
        # the reference's terms); e2e = a fresh snapshot every pass: create + first pass (plan + run + decide)
        "create_ms": round(create_ms, 3),
        # the same handle from its binary snapshot (ks_cons_create_binary: no JSON parse, no NewCandidate,
        # no encode; upload + queue ranks), and what writing that snapshot cost (ks_cons_save)
        "create_binary_ms": round(create_bin_ms, 3),
        "save_ms": round(save_ms, 3),
        "snapshot_bytes": snap_bytes,
        "first_pass_ms": round(first_ms, 3),
        "e2e_cands_per_s": round(c.num_sims / ((create_ms + first_ms) / 1000.0), 1),
        "decision": {"multi": [doc["multi"]["command"]["action"], len(doc["multi"]["command"]["candidates"])],
                     "single": [doc["single"]["command"]["action"], doc["single"]["command"]["candidates"]]},
        "roofline": _roofline("k_solve<SIM%s>" % (", TOPO" if topology else ""), k_ms, algb, ref,
                              "c5" if not topology else "c5t", per_gpu_div=world,
                              extra={"kernel_ms_max_rank": round(kmax, 3)}),
        "cpu_baseline": cpu,
        "cpu_baseline_1thread": cpu1,
        "oracle_full_size": _oracle_full("C5T" if topology else "C5", snap, c.num_sims, "cands/s"),
        "validation": validation,
        **({"incremental_update": update} if update else {}),
        **({"shards_on_one_gpu": shards} if shards else {}),
    }


def solve_line(args, local, name, snap, metric, reps, cpu_sample=None, extra=None, traffic_tag=None):
    """A Solve workload beside the C2 line: GPU time of `reps` Solves, create / e2e cost, the kernel's
    roofline against both byte counts, and the oracle on `cpu_sample` = (snapshot, pods, description)."""
    from karpenter_amd import Scheduler

    snap_json = json.dumps(snap)
    npods = len(snap["pods"])
    sch, create_ms = _create(Scheduler, snap_json)
    t = time.perf_counter()
    r = sch.solve(device=local)
    full_ms = (time.perf_counter() - t) * 1000.0
    for _ in range(max(args.warmup - 1, reps // 20)):  # (sub-ms Solves: a warm-up proportional to the reps)
        sch.solve(device=local, timing_only=True)
    t0 = time.perf_counter()
    ks, algb, fms, fbytes = [], [], [], 0.0
    for _ in range(reps):
        x = sch.solve(device=local, timing_only=True)
        ks.append(x.solve_kernel_ms)
        algb.append(x.algorithmic_bytes)
        fms.append(x.feasibility_ms)
        fbytes = x.feasibility_bytes
    el = (time.perf_counter() - t0) / reps
    k_ms = sum(ks) / len(ks)
    out = {"metric": metric, "value": round(npods / el, 1), "unit": "pods/s", "ms_per_step": round(el * 1000, 3),
           "kernel_ms": round(k_ms, 3), "create_ms": round(create_ms, 3),
           "e2e_pods_per_s": round(npods / ((create_ms + full_ms) / 1000.0), 1),
           "new_nodeclaims": len(r.new_nodeclaims), "pods_on_existing_nodes": sum(len(n["pods"]) for n in r.existing_nodes),
           "pod_errors": len(r.pod_errors),
           "roofline": _roofline("k_solve", k_ms, sum(algb) / len(algb), _ref_bytes(name, snap_json), traffic_tag),
           "cpu_baseline": None, "oracle_full_size": _oracle_full(name, snap_json, npods, "pods/s")}
    if fbytes > 0:  # k_feasibility (pod-state x instance-type rows) launched inside each Solve: its own roofline
        f_ms = sum(fms) / len(fms)
        out["feasibility"] = _roofline("k_feasibility", f_ms, fbytes, None, (traffic_tag or name.lower()) + "_feasibility"
                                       if traffic_tag else None)
    if extra:
        out.update(extra)
    if cpu_sample and not args.no_cpu_baseline:
        from oracle import bridge

        csnap, cpods, desc, creps = cpu_sample
        secs = bridge.time_solve(json.dumps(csnap), creps)
        out["cpu_baseline"] = _baseline(cpods * creps / secs, "pods/s", 1, desc, secs)
    sch.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pods", type=int, default=50000)
    ap.add_argument("--its", type=int, default=400)
    ap.add_argument("--cpu-pods", type=int, default=50000, help="oracle sample size (same workload shape)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-consolidation", action="store_true")
    ap.add_argument("--no-c1", action="store_true")
    ap.add_argument("--no-c3", action="store_true")
    ap.add_argument("--c3-pods", type=int, default=20000)
    ap.add_argument("--no-c4", action="store_true")
    ap.add_argument("--c4-pods", type=int, default=10000)
    ap.add_argument("--c4-nodes", type=int, default=2000)
    ap.add_argument("--only-consolidation", action="store_true", help="profiling: skip the Solve section")
    ap.add_argument("--only-solve", default="", help="profiling: run only this Solve line (c1, c2, c3, c4)")
    ap.add_argument("--no-c5", action="store_true", help="with --only-consolidation: skip the plain C5 pass (C5T only)")
    ap.add_argument("--cons-nodes", type=int, default=5000, help="C5 cluster size (20 pods per node)")
    ap.add_argument("--cons-steps", type=int, default=20)
    ap.add_argument("--no-shards", action="store_true", help="skip the per-shard kernel timing (world 2/4/8 on one GPU)")
    ap.add_argument("--cpu-sims", type=int, default=2400, help="oracle consolidation sample (simulations)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--c3-cpu-pods", type=int, default=2000, help="oracle C3 sample (pods)")
    ap.add_argument("--cons-topo-apps", type=int, default=20, help="topology consolidation line: apps (0: skip)")
    ap.add_argument("--cpu-topo-sims", type=int, default=100, help="oracle sample for the topology consolidation line")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist  # noqa: F811

        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    from karpenter_amd import Scheduler, synth

    def barrier_sync():
        if dist is not None:
            import torch

            dist.barrier()
            torch.cuda.synchronize()

    if args.only_consolidation:
        cons = None if args.no_c5 else consolidation_bench(args, rank, world, local, dist, barrier_sync)
        ctopo = (consolidation_bench(args, rank, world, local, dist, barrier_sync, args.cons_topo_apps)
                 if args.cons_topo_apps else None)
        if rank == 0:
            print(json.dumps({"consolidation": cons, "consolidation_topology": ctopo}))
        if dist is not None:
            dist.destroy_process_group()
        return
    if args.only_solve in ("c1", "c2", "c3", "c4"):
        if args.only_solve == "c1":
            line = solve_line(args, local, "C1", synth.config1(literal=True), "C1 profile", 200, traffic_tag="c1")
        elif args.only_solve == "c2":
            line = solve_line(args, local, "C2", synth.config2(args.pods), "C2 profile", args.steps, traffic_tag="c2")
        elif args.only_solve == "c3":
            line = solve_line(args, local, "C3", synth.config3(args.c3_pods), "C3 profile", 2, traffic_tag="c3")
        else:
            line = solve_line(args, local, "C4", synth.config4(args.c4_pods, args.c4_nodes), "C4 profile", 3,
                              traffic_tag="c4")
        print(json.dumps(line))
        return

    snap = synth.config2(args.pods) if args.its == 400 else synth.benchmark_snapshot(args.pods, args.its, 42, False)
    snap_json = json.dumps(snap)
    sch, create_ms = _create(Scheduler, snap_json)
    save_ms, create_bin_ms, snap_bytes = _create_binary(sch, Scheduler)

    # one full solve (results copied back and rendered) to verify the result shape outside the timed region
    t = time.perf_counter()
    check = sch.solve(device=local)
    full_ms = (time.perf_counter() - t) * 1000.0
    placed = sum(len(c["pods"]) for c in check.new_nodeclaims)
    assert placed + len(check.pod_errors) == args.pods, "solve lost pods"
    nclaims = len(check.new_nodeclaims)

    for _ in range(args.warmup):
        sch.solve(device=local, timing_only=True)
    barrier_sync()
    t0 = time.perf_counter()
    solve_ms, total_ms, algb = [], [], []
    for _ in range(args.steps):
        r = sch.solve(device=local, timing_only=True)
        solve_ms.append(r.solve_kernel_ms)
        total_ms.append(r.kernel_ms)
        algb.append(r.algorithmic_bytes)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    # the same Solves with the Results copied back and read through the structured accessors (what the
    # drop-in caller does: ks_solve + ks_results_* in INTEGRATION.md's cgo shim, no JSON)
    barrier_sync()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        sch.solve_structured(device=local)
    barrier_sync()
    structured_ms = (time.perf_counter() - t1) * 1000.0 / args.steps
    # the C-ABI part of that return path alone: ks_solve with the Results collected (the copy-back, the
    # replayed checks and the claim/node/error tables the accessors hand out) and ks_results_free -- what a cgo
    # caller pays before its own (C-speed) accessor walk; the Python walk above adds ctypes per field
    collected_ms = sch.timed_collect(args.steps, device=local)
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1000.0 / args.steps
    value = args.pods * world * args.steps / elapsed
    k_ms = sum(solve_ms) / len(solve_ms)
    bytes_per_launch = sum(algb) / len(algb)
    ref = _ref_bytes("C2", snap_json)
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        from oracle import bridge

        csnap = json.dumps(synth.config2(args.cpu_pods)) if args.cpu_pods != args.pods else snap_json
        res, secs = bridge.solve(csnap)
        if ref is None and args.cpu_pods == args.pods:
            ref = res.get("stats", {}).get("algBytesRef")
        cpu = _baseline(args.cpu_pods / secs, "pods/s", 1, "1 Solve of C2 with %d pods x %d instance types" %
                        (args.cpu_pods, args.its), secs)
    lines = {}
    if world == 1:
        if not args.no_c1:
            c1 = synth.config1(literal=True)
            lines["solve_c1"] = solve_line(
                args, local, "C1", c1, "pods/sec in Scheduler.Solve (C1: BenchmarkScheduling2000, the benchmark's "
                "literal pods: empty UIDs, zero timestamps; 400 fake instance types, empty topology)", 200,
                cpu_sample=(c1, 2000, "20 Solves of C1", 20), traffic_tag="c1")
        if not args.no_c3:
            sp = min(args.c3_cpu_pods, args.c3_pods)
            lines["solve_c3"] = solve_line(
                args, local, "C3", synth.config3(args.c3_pods),
                "pods/sec in Scheduler.Solve (C3: %d pods, 800 instance types x 8 offerings, 3 tainted NodePools, "
                "selectors/affinity/tolerations)" % args.c3_pods, 2,
                cpu_sample=(synth.config3(sp), sp, "1 Solve of C3 with %d pods (the oracle's per-pod cost grows with "
                            "the pod count: at 20k it takes ~460 s)" % sp, 1), traffic_tag="c3")
        if not args.no_c4:
            sp, sn = max(args.c4_pods // 4, 1), max(args.c4_nodes // 4, 1)
            lines["solve_c4"] = solve_line(
                args, local, "C4", synth.config4(args.c4_pods, args.c4_nodes),
                "pods/sec in Scheduler.Solve (C4: %d pods onto %d existing nodes, zonal + hostname spread, hostname "
                "anti-affinity, 20 apps)" % (args.c4_pods, args.c4_nodes), 3,
                cpu_sample=(synth.config4(sp, sn), sp, "1 Solve of C4 with %d pods onto %d nodes" % (sp, sn), 1),
                traffic_tag="c4")
    cons = None if args.no_consolidation else consolidation_bench(args, rank, world, local, dist, barrier_sync)
    ctopo = None
    if not args.no_consolidation and args.cons_topo_apps:
        ctopo = consolidation_bench(args, rank, world, local, dist, barrier_sync, args.cons_topo_apps)
    if rank != 0:
        dist.destroy_process_group()
        return
    out = {
        "metric": "pods/sec in Scheduler.Solve @50k pods x 400 types",
        "value": round(value, 1),
        "unit": "pods/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic",
        "config": {"workload": "C2: %d resource-only pods x %d fake.InstanceTypes, 1 NodeClaimTemplate, no limits, "
                               "empty topology (BenchmarkScheduling shape)" % (args.pods, args.its),
                   "pods": args.pods, "instance_types": args.its, "parallelism": "replicas%d" % world,
                   "new_nodeclaims": nclaims},
        # the drop-in caller's cost (never `value`): ks_problem_create = parse + encode + upload of the
        # snapshot; e2e = create + one Solve with its results copied back and rendered
        "create_ms": round(create_ms, 3),
        "create_binary_ms": round(create_bin_ms, 3),  # Scheduler.from_binary(save()): upload only
        "full_solve_ms": round(full_ms, 3),
        # a Solve with its Results read through the structured accessors, per step, and that rate
        "structured_solve_ms": round(structured_ms, 3),
        "structured_pods_per_s": round(args.pods * world / (structured_ms / 1000.0), 1),
        "collected_solve_ms": round(collected_ms, 3),
        "collected_over_kernel_only": round(collected_ms / (elapsed * 1000.0 / args.steps), 3) if elapsed else None,
        "e2e_pods_per_s": round(args.pods / ((create_ms + full_ms) / 1000.0), 1),
        "roofline": _roofline("k_solve", k_ms, bytes_per_launch, ref, "c2", extra={
            "setup_kernels_ms": round(sum(total_ms) / len(total_ms) - k_ms, 3),
            # SURVEY §8d timing protocol: median and p90 (nearest rank) of the timed Solves
            "kernel_ms_p50": round(_pct(solve_ms, 50), 3), "kernel_ms_p90": round(_pct(solve_ms, 90), 3)}),
        "cpu_baseline": cpu,
        "oracle_full_size": _oracle_full("C2", snap_json, args.pods, "pods/s"),
    }
    out.update(lines)
    out["consolidation"] = cons
    out["consolidation_topology"] = ctopo
    print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
