#!/usr/bin/env python3
"""bench.py — koord-scheduler sweep on MI355X: pods scheduled/sec + node-evals/sec.

Headline (``value``): BASELINE.json configs[1] = "C2": 10k pods onto a 5k-node synthetic cluster with
NodeResourcesFit + LoadAwareScheduling + ElasticQuota admission, percentageOfNodesToScore=100, lowest-index
tie-break.  One "step" = schedule the whole 10k-pod queue, one pod at a time semantically: restore the
snapshot (``ks_restore`` of a device-side checkpoint), the pods' PreFilter / EstimatePod work
(``prep_pods_kernel``), then the sweep -> select -> commit passes.  The raw pod columns are staged in HBM
before the timed region (host -> HBM copies are not timed; everything computed from them is).

The metric names 5k AND 100k nodes, so the same line carries ``c5``: configs[4] (1M pods x 100k nodes,
Fit + LoadAware) timed the same way — on one GPU at N=1, node-sharded over the N ranks at N>1 (strong
scaling: every rank sweeps its node range, one RCCL allgather of per-shard candidates per pass).
At N=1 it also carries ``c3`` (configs[2]: NUMA + DeviceShare joint allocation, 5k nodes), ``c4`` (configs[3]:
20k nodes with 50k Reservations), ``c2d`` (C2 under the complete v1beta2 default profile's upstream plugins as well:
NodeResourcesBalancedAllocation, TaintToleration, NodeAffinity, NodePorts, PodTopologySpread with the system default
constraints, InterPodAffinity), ``c2s`` (c2d without the last two: the round-4 c2d) and ``c3r`` (the shipped profile's
Reservation + NodeNUMAResource + DeviceShare together: C3's nodes with 12.5k reservations) and ``c3rd`` (c3r where
31.6 % of the reservations hold GPUs / RDMA: DeviceShare's reservation restore state), each with its own CPU baseline,
sample parity and roofline.

Multi-GPU (``--gpus N`` under torch.distributed.run): one process per GPU.  ``value`` at N>1 is C2 node-sharded
over the N ranks (strong scaling: one cluster, one queue, every rank sweeps its node range and the per-shard
candidates are exchanged by one RCCL allgather per pass); the ``c5`` record is the sharded 100k-node
cluster.  ``c2_replicas`` keeps the old replica line: N independent C2 clusters (seed + rank, weak scaling), which
the single-leader reference has no analogue of.  ``--replicas`` makes the replicas ``value`` again.

rank 0 prints ONE JSON line.  Timed steps run with the library's per-kernel HIP events off (they add a
dispatch gap between the pass kernels); the same number of steps is then re-run with the events on
(``profiled_steps``) for the kernel split, ``roofline`` (the sweep kernel, HBM bound) and
``roofline.commit`` (the sequential commit kernel).  ``cpu_baseline``: the CPU oracle (oracle/koord_oracle.c,
the reference's 16-worker Parallelizer shape) on a bounded sample of the same workload at 16 threads, with
1 and all-usable-host-core runs next to it (``by_threads``); ``parity`` = GPU results == oracle results on
that sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
GPU_CLOCK_GHZ = 2.4    # MI355X peak engine clock (MI355X_MICROARCH.md): commit cycles/pod are quoted at it
METRIC = "pods scheduled/sec + node-evals/sec (% HBM roofline) at 5k and 100k nodes"


def build_workload(name: str, seed: int, n_pods: int = 0):
    from koordinator_amd import synth

    if name not in ("c1", "c2", "c3", "c4", "c5", "c2d", "c2s", "c3r", "c3rd", "c3f"):
        raise SystemExit(f"unknown config {name}")
    if name == "c2d":
        # the complete v1beta2 default profile: c2s's plugins + PodTopologySpread (system default constraints for the
        # pods owned by a ReplicaSet, own constraints) and InterPodAffinity (synth.topology_specs)
        w = synth.c2_default(seed=seed, n_pods=n_pods) if n_pods else synth.c2_default(seed=seed)
        w = synth.with_topology(w, seed=seed + 9)
        w.name = "C2-default"
        return w
    # c3rd: c3r where 70 % of the reservations on non-policy device nodes hold GPUs / RDMA (about a third of all of them)
    c3rd = lambda **kw: synth.c3_rsv(dev_rsv_frac=0.7, **kw)  # noqa: E731
    fn = {"c2s": synth.c2_default, "c3r": synth.c3_rsv, "c3rd": c3rd, "c3f": synth.c3_full}.get(name) or getattr(synth, name)
    return fn(seed=seed, n_pods=n_pods) if n_pods else fn(seed=seed)


def lib_sha256() -> str:
    import hashlib

    from koordinator_amd import runtime

    with open(runtime.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def newest_profile(pattern: str):
    """The newest committed profile summary matching `pattern` that was measured with the library this process
    loaded (its lib_sha256 stamp, tools/traffic.py / valu.py); summaries of another build are skipped, so a number
    in the bench line always comes from this build."""
    import glob

    want = lib_sha256()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), reverse=True):
        with open(path) as f:
            t = json.load(f)
        if t.get("lib_sha256") == want:
            return t, os.path.relpath(path, ROOT)
    return None, None


def pmc_traffic(config: str, kernel: str):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary for this config measured with this
    library (profiles/rNN_<config>_traffic.json, written by tools/pmc_traffic.sh + tools/traffic.py from
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this same bench command); None when absent."""
    t, src = newest_profile(f"r*_{config}_traffic.json")
    if t is None:
        return None, None
    n = b = 0
    for k, v in t.get("kernels", {}).items():
        if kernel in k:
            n += v["launches"]
            b += v["hbm_bytes_per_launch"] * v["launches"]
    if not n:
        return None, None
    return round(b / n), src


def pmc_valu(config: str, kernel: str):
    """VALU-issue floor per launch of `kernel` (us) from the newest committed PMC summary for this config measured
    with this library (profiles/rNN_<config>_valu.json, tools/pmc_valu.sh + tools/valu.py: SQ_INSTS_VALU x 2 cycles
    over 1024 SIMDs at 2.4 GHz); None when absent."""
    t, src = newest_profile(f"r*_{config}_valu.json")
    if t is None:
        return None, None
    n = us = 0.0
    for k, v in t.get("kernels", {}).items():
        if kernel in k and "valu_issue_floor_us" in v:
            n += v["launches"]
            us += v["valu_issue_floor_us"] * v["launches"]
    if not n:
        return None, None
    return us / n, src


def host_cpus():
    """(CPU model, CPUs this process may run on): the affinity mask, capped by a cgroup-v2 cpu.max quota."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return model, n


def time_oracle(w, threads: int, n_pods: int):
    from oracle.oracle import Oracle

    cs = w.cpus
    o = Oracle(w.cfg, w.nodes.copy(), nthreads=threads, **w.tables())
    try:
        t = time.perf_counter()
        r = o.schedule(w.pods.rows(range(n_pods)))
        dt = time.perf_counter() - t
        if cs is not None:
            r["cpusets"] = o.fetch_cpusets(n_pods)
    finally:
        o.close()
    return r, dt


def sample_size(w, threads: int, budget_s: float) -> int:
    """Pods of a bounded prefix sized from a short probe so the timed oracle run takes about budget_s."""
    probe = min(w.pods.n, 300)
    _, dt = time_oracle(w, threads, probe)
    if dt * w.pods.n / probe <= budget_s:
        return w.pods.n
    return max(probe, int(budget_s * probe / max(dt, 1e-9)))


def cpu_baseline(w, gpu_res, budget_s: float, extra_budget_s: float):
    """The CPU oracle (port of the reference loop) on bounded prefixes of the workload: 16 threads (the
    reference Parallelizer's default, the headline baseline) plus 1 thread and every usable host core."""
    model, ncpu = host_cpus()
    n16 = sample_size(w, 16, budget_s)
    r, dt = time_oracle(w, 16, n16)
    keys = ("node", "status", "score", "reservation", "gpu_minors", "rdma_minors")
    parity = all(np.array_equal(r[k], gpu_res[k][:n16]) for k in keys)
    if "cpusets" in r:
        parity = parity and np.array_equal(r["cpusets"], gpu_res["cpusets"][:n16])
    by_threads = {"16": {"pods_per_s": round(n16 / dt, 1), "sample_pods": n16}}
    for th in sorted({1, ncpu} - {16}):
        if extra_budget_s <= 0:
            break
        n = sample_size(w, th, extra_budget_s)
        _, d = time_oracle(w, th, n)
        by_threads[str(th)] = {"pods_per_s": round(n / d, 1), "sample_pods": n}
    return {
        "value": round(n16 / dt, 1),
        "unit": "pods/s",
        "cores": 16,
        "kind": "port",
        "sample_short": f"first {n16} of {w.pods.n} pods, same inputs; C restatement, 16-worker Parallelizer",
        "sample": f"first {n16} of {w.pods.n} pods of {w.name} ({w.nodes.n} nodes), same inputs as the GPU run; "
                  f"CPU restatement with the reference Parallelizer shape (16 workers, chunk=min(sqrt(n),n/16+1)); "
                  f"omits Go map/Quantity/lister overheads, so it is a faster-than-reference baseline",
        "node_evals_per_s": round(n16 * w.nodes.n / dt, 1),
        "by_threads": by_threads,
        "host_cpu": model,
        "host_usable_cpus": ncpu,
        "host_nproc": os.cpu_count(),
        "parity_with_gpu_on_sample": bool(parity),
    }


def sweep_algo_bytes(w, prof, local_nodes: int) -> int:
    """Algorithmic bytes per sweep launch: SURVEY §8(d)'s B_node (LoadAware + Fit columns, each read once
    per pass: 106 B, +16 B with the prod-usage score term, +32 B for the batch-cpu / batch-memory scalar
    columns) x the nodes one launch sweeps, + the pass's pod records + the chunk-maxima output."""
    b_node = 106 + (16 if prof.loadaware is not None and prof.loadaware.score_according_prod_usage else 0) + 32
    algo = local_nodes * b_node + 64 * 128 + ((local_nodes + 63) // 64) * 64 * 4
    if w.devices is not None:
        # + NUMA amplification columns (16 B) and the device table (flags + 34 total / topology words +
        # 32 used words, int64; ks_dev.h)
        algo += local_nodes * (16 + 4 + (34 + 32) * 8)
    if prof.taint_toleration or prof.node_affinity or prof.node_ports:
        # + the TaintToleration / NodeAffinity / NodePorts dictionary words (4 x u64) and the pods' PodStat records
        algo += local_nodes * 32 + 64 * 112
    if w.reservations is not None:
        # + the owner-class column and the reservation table (CSR offsets, classes, meta, order rank,
        # allocatable/allocated x7, assigned, reserve-pod non-zero x2) read once
        algo += local_nodes * (8 + 4) + w.reservations.r * (8 + 4 + 4 + 7 * 8 * 2 + 4 + 16)
    return algo


def run_config(w, args, dist, world: int, rank: int, local_rank: int, shard: bool, steps: int, warmup: int,
               cfg_key: str, profile: bool):
    """Time `steps` scheduling steps of workload w on this rank (max over ranks); then the same steps with
    the per-kernel events on for the split.  Returns (record fields, gpu results)."""
    from koordinator_amd import abi, runtime

    prof = w.profile
    prof.device = local_rank if world > 1 else 0
    prof.batch_pods = args.batch_pods
    prof.candidates = args.candidates
    cfg = prof.to_ks_config()
    cfg.profile = 0
    ev = runtime.Evaluator(cfg, w.nodes, **w.tables(copy=False))
    try:
        nshards = 1
        if shard and world > 1:
            box = [runtime.shard_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            ev.shard(world, rank, box[0], args.vshards)
            nshards = world
        elif args.vshards > 1:
            ev.shard(1, 0, None, args.vshards)
        ev.stage(w.pods)
        ev.checkpoint()

        def sync():
            if dist is not None:
                import torch

                torch.cuda.synchronize()
                dist.barrier()

        ev.set_profile(False)
        for _ in range(warmup):
            ev.restore()
            ev.schedule_staged()
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            ev.restore()
            ev.schedule_staged()
        sync()
        elapsed = time.perf_counter() - t0
        st_last = ev.stats()
        agg = {"sweep_ms": 0.0, "select_ms": 0.0, "commit_ms": 0.0, "fixup_ms": 0.0, "sweep_launches": 0, "passes": 0,
               "cut_passes": 0, "rescans": 0, "bubble_passes": 0, "pre_reserves": 0}
        prof_elapsed = 0.0
        sweep_bytes = 0
        if profile:
            ev.set_profile(True)
            for _ in range(steps):
                ev.restore()
                tp = time.perf_counter()
                ev.schedule_staged()
                prof_elapsed += time.perf_counter() - tp
                st = ev.stats()
                for k in agg:
                    agg[k] += st[k]
                sweep_bytes = st["sweep_bytes"]
            ev.set_profile(False)
        else:
            for k in ("passes", "cut_passes", "rescans", "bubble_passes", "pre_reserves"):
                agg[k] = st_last[k] * steps
        if dist is not None:
            import torch

            t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        res = ev.fetch()
        if w.cpus is not None:
            res["cpusets"] = ev.fetch_cpusets(w.pods.n)
    finally:
        ev.close()

    n_pods, n_nodes = w.pods.n, w.nodes.n
    units = n_pods * steps * (1 if shard else world)  # replicas each schedule their own queue
    value = units / elapsed
    rec = {
        "value": round(value, 1),
        "unit": "pods/s",
        "ms_per_step": round(elapsed * 1000.0 / steps, 3),
        "steps": steps,
        "warmup": warmup,
        "node_evals_per_s": round(value * n_nodes, 1),
        "pods_per_step": n_pods,
        "nodes": n_nodes,
        "placed_per_step": int((res["status"] == 0).sum()),
        "into_reservations_per_step": int((res["reservation"] >= 0).sum()),
        "gpu_pods_placed_per_step": int((res["gpu_minors"] != 0).sum()),
        "rdma_pods_placed_per_step": int((res["rdma_minors"] != 0).sum()),
        "cpuset_pods_placed_per_step": int(((res["status"] == 0) & ((w.pods.flags & abi.KS_POD_CPU_BIND) != 0)).sum()),
        "profiled_steps": steps if profile else 0,
        "ms_per_profiled_step": round(prof_elapsed * 1000.0 / steps, 3) if profile else None,
        "passes_per_step": agg["passes"] / steps,
        "cut_passes_per_step": agg["cut_passes"] / steps,
        "rescans_per_step": agg["rescans"] / steps,
        # pipelined passes: each pass's sweep runs on a second stream while the previous pass
        # commits, so the kernel times below overlap and add up to more than ms_per_step
        "pipelined": int(st_last["pipelined"]),  # 0 off, 1 re-swept, 2 patched lists
        "bubble_passes_per_step": agg["bubble_passes"] / steps,
        # NUMA / device Reserves computed ahead of the commit (reserve_pre_kernel)
        "pre_reserves_per_step": agg["pre_reserves"] / steps,
        "kernel_ms_per_step": {"sweep": round(agg["sweep_ms"] / steps, 3), "select": round(agg["select_ms"] / steps, 3),
                               "commit": round(agg["commit_ms"] / steps, 3),
                               "dirty_resweep": round(agg["fixup_ms"] / steps, 3)},
        "roofline": None,
    }
    if profile and agg["sweep_launches"]:
        rec["roofline"] = pass_roofline(w, prof, cfg_key, agg, steps, n_pods, n_nodes // nshards, sweep_bytes,
                                        args.candidates or 32, world)
    return rec, res


def pass_roofline(w, prof, cfg_key: str, agg: dict, steps: int, n_pods: int, local_nodes: int, sweep_bytes: int,
                  cands: int, world: int) -> dict:
    """achieved = B_pass_total / t_kernels over one scheduling pass (a batch of <= 64 pods):
    B_pass_total = the sweep's algorithmic bytes (N x B_node + the pass's pod records + the chunk maxima) + the
    select's candidate lists (P x K x 16 B) + the commit's P x B_node (138 B: SURVEY's 106 B + the two batch scalar
    columns); t_kernels = (sweep + select + commit kernel time) / passes, from per-kernel HIP events of the profiled
    steps.  The same figure reproduces from rocprofv3's kernel statistics (profiles/rNN_<config>_kernel_stats.csv):
    B_pass_total / (avg sweep x sweep launches/pass + avg select + avg commit).  `sweep_*` is the sweep kernel alone,
    `commit_*` the sequential commit (the kernel that bounds the step)."""
    passes = max(agg["passes"], 1)
    sweep_s = agg["sweep_ms"] / agg["sweep_launches"] / 1000.0
    sweep_algo = sweep_algo_bytes(w, prof, local_nodes)
    pods_per_pass = n_pods * steps / passes
    commit_algo = int(round(pods_per_pass * 138))
    select_algo = int(round(pods_per_pass * cands * 16))
    launches_per_pass = agg["sweep_launches"] / passes  # two-phase sweeps (DeviceShare, normalizing plugins): 2
    b_pass = int(round(sweep_algo * launches_per_pass)) + select_algo + commit_algo
    # (+ the pipelined passes' list re-evaluation, a sweep_kernel launch in list mode on the commit stream)
    t_pass = (agg["sweep_ms"] + agg["select_ms"] + agg["commit_ms"] + agg["fixup_ms"]) / 1000.0 / passes
    achieved = b_pass / t_pass / 1e9
    mono = all(x is None for x in (w.quotas, w.reservations, w.devices, w.cpus, w.numa_nodes))
    c_kernel = "commit_mono_kernel" if mono else "commit_kernel"
    tr_sweep, src = pmc_traffic(cfg_key, "sweep_kernel")
    tr_sel, _ = pmc_traffic(cfg_key, "select_kernel")
    tr_com, _ = pmc_traffic(cfg_key, c_kernel)
    traffic = (int(round(tr_sweep * launches_per_pass)) + tr_sel + tr_com
               if None not in (tr_sweep, tr_sel, tr_com) else None)
    commit_s = agg["commit_ms"] / 1000.0 / passes
    roof = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 7), "traffic": traffic,
            "kernel": "pass (sweep+select+commit)", "bytes_per_pass": b_pass, "us_per_pass": round(t_pass * 1e6, 2),
            "sweep_frac": round(sweep_algo / sweep_s / 1e9 / HBM_PEAK_GBS, 5), "sweep_us": round(sweep_s * 1e6, 2),
            "sweep_bytes": sweep_algo, "sweep_traffic": tr_sweep,
            "commit_us": round(commit_s * 1e6, 2), "commit_kernel": c_kernel,
            "commit_share": round(agg["commit_ms"] / (agg["sweep_ms"] + agg["select_ms"] + agg["commit_ms"]), 4),
            "commit_cycles_per_pod": round(agg["commit_ms"] / 1000.0 * GPU_CLOCK_GHZ * 1e9 / (n_pods * steps), 1),
            "commit_traffic": tr_com, "traffic_source": src}
    floor_us, _ = pmc_valu(cfg_key, "sweep_kernel")
    if floor_us is not None and world == 1:
        # the sweep's instruction-issue bound next to the HBM one
        roof["sweep_valu_issue_frac"] = round(floor_us / (sweep_s * 1e6), 4)
    return roof


def run_preempt(args, steps: int, warmup: int, profile: bool, cpu: bool):
    """The ElasticQuota PostFilter (f4) on C2's cluster with NodeInfo.Pods on every node (synth.c2_preempt: 5k nodes,
    ~110k running pods, quotas at their limits): one step = the PostFilter of every preemptor in turn (ks_preempt:
    every node's dry run on the device + the candidate selection; nothing is deleted, so steps repeat exactly)."""
    from koordinator_amd import runtime
    from koordinator_amd.cluster import PodTable  # noqa: F401

    w = __import__("koordinator_amd.synth", fromlist=["c2_preempt"]).c2_preempt(n_nodes=5000, n_preemptors=args.preempt_pods)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), w.quotas.copy())
    rows = [w.preemptors.rows([i]) for i in range(w.preemptors.n)]
    pods = [r.ks() for r in rows]  # the ks_pod_cols pointer structs built once (as a Go shim keeps its C structs)
    res = []
    try:
        ev.load_node_pods(w.node_pods)
        ev.set_profile(False)
        for _ in range(warmup):
            for i, p in enumerate(pods):
                ev.preempt(p, int(w.priority[i]))
        t0 = time.perf_counter()
        for _ in range(steps):
            res = [ev.preempt(p, int(w.priority[i])) for i, p in enumerate(pods)]
        elapsed = time.perf_counter() - t0
        dry_ms = sel_ms = 0.0
        algo = 0
        if profile:
            ev.set_profile(True)
            for i, p in enumerate(pods):
                ev.preempt(p, int(w.priority[i]))
                st = ev.stats()
                dry_ms += st["sweep_ms"]
                sel_ms += st["select_ms"]
                algo = st["sweep_bytes"]
            ev.set_profile(False)
    finally:
        ev.close()
    calls = steps * len(pods)
    rec = {"value": round(calls / elapsed, 1), "unit": "preemptions/s", "ms_per_step": round(elapsed * 1000 / steps, 3),
           "steps": steps, "warmup": warmup, "preemptors_per_step": len(pods), "nodes": w.nodes.n,
           "running_pods": w.node_pods.m, "node_dry_runs_per_s": round(calls * w.nodes.n / elapsed, 1),
           "us_per_preemption": round(elapsed * 1e6 / calls, 2),
           "nominated_per_step": sum(1 for r in res if r["status"] == 0),
           "victims_per_step": int(sum(len(r["victims"]) for r in res)),
           "workload": f"C2-preempt: {w.nodes.n} nodes, {w.node_pods.m} running pods (NodeInfo.Pods), 32 quotas at their "
                       f"limits, {len(pods)} preemptors; ElasticQuota PostFilter (SelectVictimsOnNode on every node, "
                       f"pickOneNodeForPreemption) with Fit + LoadAware filters; timed per call (host staging + 2 kernels "
                       f"+ read-back)",
           "roofline": None}
    if profile and dry_ms:
        avg = dry_ms / len(pods) / 1000.0
        achieved = algo / avg / 1e9
        rec["roofline"] = {"bound": "hbm", "kernel": "preempt_dry_run_kernel", "achieved": round(achieved, 2),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                           "avg_launch_us": round(avg * 1e6, 3), "algorithmic_bytes_per_launch": algo,
                           "select_us": round(sel_ms / len(pods) * 1000, 3),
                           "traffic": pmc_traffic("preempt", "preempt_dry_run_kernel")[0]}
    if cpu:
        from oracle.oracle import Oracle

        model, ncpu = host_cpus()
        o = Oracle(w.cfg, w.nodes.copy(), w.quotas.copy(), nthreads=16)
        try:
            o.load_node_pods(w.node_pods)
            t0 = time.perf_counter()
            k = 0
            want = []
            while k < len(pods) and (k < 4 or time.perf_counter() - t0 < args.cpu_budget_s):
                want.append(o.preempt(rows[k], int(w.priority[k])))
                k += 1
            dt = time.perf_counter() - t0
        finally:
            o.close()
        keys = ("status", "node", "num_pdb_violations", "candidates", "potential_nodes")
        parity = all(all(res[i][kk] == want[i][kk] for kk in keys) and np.array_equal(res[i]["victims"], want[i]["victims"])
                     for i in range(k))
        rec["cpu_baseline"] = {"value": round(k / dt, 1), "unit": "preemptions/s", "cores": 16, "kind": "port",
                               "sample": f"first {k} of {len(pods)} preemptors, same cluster; the CPU restatement of "
                                         f"DryRunPreemption on the Parallelizer (16 workers)",
                               "host_cpu": model, "host_usable_cpus": ncpu}
        rec["parity"] = bool(parity)
        rec["speedup_vs_cpu_baseline"] = round(rec["value"] / rec["cpu_baseline"]["value"], 2)
    return rec


def workload_desc(w):
    return (f"{w.name}: {w.pods.n} pods x {w.nodes.n} nodes, NodeResourcesFit(LeastAllocated cpu/mem/batch-cpu/batch-mem)"
            f" + LoadAwareScheduling(defaults)" + (" + ElasticQuota(32 leaf quotas)" if w.quotas is not None else "")
            + (f" + Reservation(weight 5000, {w.reservations.r} reservations)" if w.reservations is not None else "")
            + (" + NodeNUMAResource(amplified CPUs, cpuset pods, NUMA topology policies) + DeviceShare(8 GPUs x 80GiB + 4 RDMA on"
               " 4 PCIe/2 NUMA per node, joint GPU+RDMA)" if w.devices is not None else "")
            + (" + upstream NodeResourcesBalancedAllocation + TaintToleration + NodeAffinity + NodePorts (v1beta2 default"
               " plugins)" if w.profile.balanced is not None and w.profile.taint_toleration else "")
            + (" + upstream PodTopologySpread(weight 2, system default constraints) + InterPodAffinity(weight 1)"
               f" ({int((w.pods.topo_flags & 1).sum())} topology pods)" if w.profile.topology else ""))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "c2d", "c2s", "c3r", "c3rd", "c3f"])
    ap.add_argument("--pods", type=int, default=0, help="pods per step (default: the config's own count)")
    ap.add_argument("--batch-pods", type=int, default=0)
    ap.add_argument("--candidates", type=int, default=0)
    ap.add_argument("--no-profile", action="store_true", help="do not bracket kernels with HIP events")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=15.0, help="16-thread oracle sample (per config)")
    ap.add_argument("--cpu-extra-budget-s", type=float, default=6.0, help="1-thread / all-core oracle samples")
    ap.add_argument("--replicas", action="store_true",
                    help="at N>1: N independent replicas of the main config as `value` (default: node-sharded)")
    ap.add_argument("--shard", action="store_true", help="(default at N>1; kept for old command lines)")
    ap.add_argument("--vshards", type=int, default=1, help="virtual shards per GPU (exercises the merge on one GPU)")
    ap.add_argument("--no-c5", action="store_true", help="skip the 100k-node c5 record")
    ap.add_argument("--c5-pods", type=int, default=1_000_000)
    ap.add_argument("--c5-steps", type=int, default=3)
    ap.add_argument("--c5-warmup", type=int, default=1)
    ap.add_argument("--no-sub", action="store_true", help="skip the c3 / c4 / c2d / c2s / c3r / c3rd sub-records")
    ap.add_argument("--sub-steps", type=int, default=3)
    ap.add_argument("--sub-warmup", type=int, default=1)
    ap.add_argument("--no-preempt", action="store_true", help="skip the preempt (ElasticQuota PostFilter) record")
    ap.add_argument("--preempt-pods", type=int, default=128)
    ap.add_argument("--detail", default="", help="also write every record in full (kernel split, per-thread CPU "
                    "baselines, roofline parts) to this JSON file; the printed line is the compact form")
    ap.add_argument("--preempt-only", action="store_true",
                    help="print only the preempt record (profiling runs of the PostFilter kernels, tools/pmc_traffic.sh)")
    args = ap.parse_args()
    if args.preempt_only:
        rec = run_preempt(args, args.steps, args.warmup, not args.no_profile, not args.no_cpu_baseline)
        print(json.dumps({"preempt": rec}), flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    args.shard = world > 1 and not args.replicas
    if world > 1:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    # replicas schedule their own cluster (seed + rank); shards split one shared cluster
    w = build_workload(args.config, seed=20261015 + (0 if args.shard else rank), n_pods=args.pods)
    rec, res = run_config(w, args, dist, world, rank, local_rank, args.shard, args.steps, args.warmup, args.config,
                          not args.no_profile)
    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": rec["value"],
            "unit": "pods/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": rec["ms_per_step"],
            "higher_is_better": True,
            "scaling": "strong" if args.shard else "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {"workload": workload_desc(w), "pods_per_step": w.pods.n, "nodes": w.nodes.n,
                       "percentage_of_nodes_to_score": 100,
                       "parallelism": (f"node-shards{world}x{args.vshards}" if args.shard or args.vshards > 1
                                       else (f"replicas{world}" if world > 1 else "single-gpu")),
                       "batch_pods": args.batch_pods or 64, "candidates": args.candidates or 32,
                       "timed_region": "restore snapshot + PreFilter/EstimatePod (prep_pods_kernel) + sweep/select/commit "
                                       "passes; raw pod columns staged in HBM beforehand"},
        }
        out.update({k: v for k, v in rec.items() if k not in ("value", "unit", "ms_per_step", "steps", "warmup")})
        out["cpu_baseline"] = None
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(w, res, args.cpu_budget_s, args.cpu_extra_budget_s)
            out["cpu_baseline"] = cb
            out["parity"] = cb["parity_with_gpu_on_sample"]
            out["speedup_vs_cpu_baseline"] = round(rec["value"] / cb["value"], 2)
    del w, res

    if world > 1 and args.shard and not args.no_sub:
        # the replica line: N independent clusters of the main config (seed + rank), weak scaling
        wr = build_workload(args.config, seed=20261015 + rank, n_pods=args.pods)
        rr, _ = run_config(wr, args, dist, world, rank, local_rank, False, args.steps, args.warmup, args.config, False)
        if rank == 0:
            rr["scaling"] = "weak"
            rr["parallelism"] = f"replicas{world}"
            out["c2_replicas" if args.config == "c2" else f"{args.config}_replicas"] = rr
        del wr

    if not args.no_c5 and args.config != "c5":
        # the metric's 100k-node configuration: one GPU at N=1, node-sharded over the ranks at N>1
        w5 = build_workload("c5", seed=20261015, n_pods=args.c5_pods)
        r5, res5 = run_config(w5, args, dist, world, rank, local_rank, True, args.c5_steps, args.c5_warmup, "c5",
                              not args.no_profile)
        if rank == 0:
            r5["workload"] = workload_desc(w5)
            r5["scaling"] = "strong"
            r5["parallelism"] = f"node-shards{world}" if world > 1 else "single-gpu"
            if world == 1 and not args.no_cpu_baseline:
                cb5 = cpu_baseline(w5, res5, args.cpu_budget_s, args.cpu_extra_budget_s)
                r5["cpu_baseline"] = cb5
                r5["parity"] = cb5["parity_with_gpu_on_sample"]
                r5["speedup_vs_cpu_baseline"] = round(r5["value"] / cb5["value"], 2)
            out["c5"] = r5
    if not args.no_sub and world == 1 and args.config == "c2":
        # SURVEY's C3 (NUMA + DeviceShare) and C4 (Reservation) workloads, each timed like the headline with its own
        # CPU baseline, sample parity and commit roofline (single GPU: neither is node-sharded)
        # c3r: the shipped profile's plugin set (Reservation + NodeNUMAResource + DeviceShare) on C3's nodes with C4-style
        # reservations (synth.c3_rsv); c3rd: c3r with reservations holding GPUs / RDMA (DeviceShare's restore state)
        # c2d: C2 under the complete v1beta2 default profile (c2s + PodTopologySpread + InterPodAffinity); c2s: without
        # those two (the round-4 c2d)
        for sub in ("c3", "c4", "c2d", "c2s", "c3r", "c3rd"):
            ws = build_workload(sub, seed=20261015)
            rs, ress = run_config(ws, args, None, 1, 0, 0, False, args.sub_steps, args.sub_warmup, sub,
                                  not args.no_profile)
            rs["workload"] = workload_desc(ws)
            rs["parallelism"] = "single-gpu"
            if not args.no_cpu_baseline:
                cbs = cpu_baseline(ws, ress, args.cpu_budget_s, args.cpu_extra_budget_s)
                rs["cpu_baseline"] = cbs
                rs["parity"] = cbs["parity_with_gpu_on_sample"]
                rs["speedup_vs_cpu_baseline"] = round(rs["value"] / cbs["value"], 2)
            out[sub] = rs
            del ws, ress
    if not args.no_sub and not args.no_preempt and world == 1 and args.config == "c2":
        out["preempt"] = run_preempt(args, args.sub_steps, args.sub_warmup, not args.no_profile, not args.no_cpu_baseline)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if out is not None:
        if args.detail:
            with open(args.detail, "w") as f:
                json.dump(out, f, indent=1)
        print(json.dumps(compact_line(out), separators=(",", ":")), flush=True)


SUB_KEYS = ("value", "unit", "ms_per_step", "steps", "warmup", "nodes", "pods_per_step", "node_evals_per_s", "scaling",
            "parallelism", "passes_per_step", "pipelined", "parity", "speedup_vs_cpu_baseline", "preemptors_per_step",
            "us_per_preemption")
ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "sweep_frac", "commit_us", "commit_share", "kernel",
             "avg_launch_us")


def compact_roof(r):
    return {k: r[k] for k in ROOF_KEYS if k in r} if r else None


def compact_cpu(cb):
    if not cb:
        return cb
    return {"value": cb["value"], "unit": cb["unit"], "cores": cb["cores"], "kind": cb["kind"],
            "sample": cb.get("sample_short", cb.get("sample", ""))[:90]}


def compact_line(out: dict) -> dict:
    """The printed line: the contract's keys, a flat roofline (SURVEY §8(d) pass figure + the sweep / commit parts), a
    short cpu_baseline, one short record per sub-workload, and c5 (the metric's 100k-node half) LAST, so a reader
    holding only the line's tail (the driver keeps ~2 KB) still sees its value, roofline, CPU baseline and parity."""
    head = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data")
    line = {k: out[k] for k in head}
    cfg = dict(out["config"])
    cfg["workload"] = cfg["workload"][:160]
    line["config"] = cfg
    line["roofline"] = compact_roof(out.get("roofline"))
    line["cpu_baseline"] = compact_cpu(out.get("cpu_baseline"))
    for k in ("parity", "speedup_vs_cpu_baseline", "node_evals_per_s", "passes_per_step", "pipelined"):
        if k in out:
            line[k] = out[k]
    subs = [k for k in out if isinstance(out[k], dict) and k not in head + ("config", "roofline", "cpu_baseline",
                                                                                 "kernel_ms_per_step", "c5")]
    for k in subs + (["c5"] if "c5" in out else []):
        r = out[k]
        c = {kk: r[kk] for kk in SUB_KEYS if kk in r}
        c["roofline"] = compact_roof(r.get("roofline"))
        c["cpu_baseline"] = compact_cpu(r.get("cpu_baseline"))
        line[k] = c
    return line


if __name__ == "__main__":
    main()
