#!/usr/bin/env python3
"""bench.py — koord-scheduler sweep on MI355X: pods scheduled/sec + node-evals/sec.

Default workload (N=1): BASELINE.json configs[1] = "C2": 10k pods onto a 5k-node
synthetic cluster with NodeResourcesFit + LoadAwareScheduling + ElasticQuota
admission, percentageOfNodesToScore=100, lowest-index tie-break.  One "step" =
schedule the whole 10k-pod queue, one pod at a time semantically (sweep ->
select -> commit passes on the device), starting from the same snapshot
(``ks_restore`` of a device-side checkpoint, included in the timed region).
Inputs are staged in HBM before the timed region.

Multi-GPU (``--gpus N`` under torch.distributed.run): one process per GPU, each
rank schedules its own C2 replica (seed + rank): replicas only, weak scaling —
the 5k-node C2 cluster does not warrant node sharding.

rank 0 prints ONE JSON line.  The timed steps run with the library's per-kernel HIP
events off (they add a dispatch gap between the pass kernels, ~19 % at C2); the same
number of steps is then re-run with the events on (``profiled_steps``) for the
kernel split.  Extra fields: ``roofline`` for the sweep (scoring) kernel from those
per-launch HIP events, ``cpu_baseline`` from the CPU
oracle (oracle/koord_oracle.c, the reference's 16-worker Parallelizer shape)
on the same workload, and ``parity`` = GPU placements == oracle placements.
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


def build_workload(name: str, seed: int, n_pods: int = 0):
    from koordinator_amd import synth

    if n_pods:
        return getattr(synth, name)(seed=seed, n_pods=n_pods)

    if name == "c2":
        return synth.c2(seed=seed)
    if name == "c1":
        return synth.c1(seed=seed)
    if name == "c3":
        return synth.c3(seed=seed)
    if name == "c4":
        return synth.c4(seed=seed)
    if name == "c5":
        return synth.c5(seed=seed)  # BASELINE configs[4]: 1M pods x 100k nodes
    raise SystemExit(f"unknown config {name}")


def pmc_traffic(config: str, kernel: str):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary for this config
    (profiles/rNN_<config>_traffic.json, written by tools/pmc_traffic.sh + tools/traffic.py from
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this same bench command); None when absent."""
    import glob

    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", f"r*_{config}_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        t = json.load(f)
    n = b = 0
    for k, v in t.get("kernels", {}).items():
        if kernel in k:
            n += v["launches"]
            b += v["hbm_bytes_per_launch"] * v["launches"]
    if not n:
        return None, None
    return round(b / n), os.path.relpath(files[-1], os.path.dirname(os.path.abspath(__file__)))


def pmc_valu(config: str, kernel: str):
    """VALU-issue floor per launch of `kernel` (us) from the newest committed PMC summary for this
    config (profiles/rNN_<config>_valu.json, tools/pmc_valu.sh + tools/valu.py: SQ_INSTS_VALU x 2 cycles
    over 1024 SIMDs at 2.4 GHz); None when absent."""
    import glob

    here = os.path.dirname(os.path.abspath(__file__))
    files = sorted(glob.glob(os.path.join(here, "profiles", f"r*_{config}_valu.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        t = json.load(f)
    n = us = 0.0
    for k, v in t.get("kernels", {}).items():
        if kernel in k and "valu_issue_floor_us" in v:
            n += v["launches"]
            us += v["valu_issue_floor_us"] * v["launches"]
    if not n:
        return None, None
    return us / n, os.path.relpath(files[-1], here)


def cpu_baseline(w, gpu_res, budget_s: float):
    """Time the CPU oracle (port of the reference loop) on a bounded prefix of the workload."""
    from oracle.oracle import Oracle

    threads = int(os.environ.get("KS_CPU_THREADS", "16"))
    threads = max(1, min(threads, os.cpu_count() or 1))
    # estimate the prefix that fits the budget from a short probe
    probe = min(w.pods.n, 500)
    rs = w.reservations
    dv = w.devices
    o = Oracle(w.cfg, w.nodes.copy(), w.quotas.copy() if w.quotas is not None else None, nthreads=threads,
               reservations=rs.copy() if rs is not None else None, devices=dv.copy() if dv is not None else None,
               cpu_state=w.cpus.copy() if w.cpus is not None else None)
    t = time.perf_counter()
    r_probe = o.schedule(w.pods.rows(range(probe)))
    dt = time.perf_counter() - t
    o.close()
    n_sample = w.pods.n if dt * w.pods.n / probe <= budget_s else max(probe, int(budget_s * probe / dt))
    o = Oracle(w.cfg, w.nodes.copy(), w.quotas.copy() if w.quotas is not None else None, nthreads=threads,
               reservations=rs.copy() if rs is not None else None, devices=dv.copy() if dv is not None else None,
               cpu_state=w.cpus.copy() if w.cpus is not None else None)
    t = time.perf_counter()
    r = o.schedule(w.pods.rows(range(n_sample)))
    dt = time.perf_counter() - t
    cs = o.fetch_cpusets(n_sample) if w.cpus is not None else None
    o.close()
    parity = bool(np.array_equal(r["node"], gpu_res["node"][:n_sample])
                  and np.array_equal(r["status"], gpu_res["status"][:n_sample])
                  and np.array_equal(r["score"], gpu_res["score"][:n_sample])
                  and np.array_equal(r["reservation"], gpu_res["reservation"][:n_sample])
                  and np.array_equal(r["gpu_minors"], gpu_res["gpu_minors"][:n_sample])
                  and np.array_equal(r["rdma_minors"], gpu_res["rdma_minors"][:n_sample])
                  and (cs is None or np.array_equal(cs, gpu_res["cpusets"][:n_sample])))
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": round(n_sample / dt, 1),
        "unit": "pods/s",
        "cores": threads,
        "kind": "port",
        "sample": f"first {n_sample} of {w.pods.n} pods of {w.name} ({w.nodes.n} nodes), same inputs as the GPU run; "
                  f"CPU restatement with the reference Parallelizer shape (16 workers, chunk=min(sqrt(n),n/16+1)); "
                  f"omits Go map/Quantity/lister overheads, so it is a faster-than-reference baseline",
        "node_evals_per_s": round(n_sample * w.nodes.n / dt, 1),
        "host_cpu": cpu_model,
        "host_nproc": os.cpu_count(),
        "parity_with_gpu_on_sample": parity,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5"])
    ap.add_argument("--pods", type=int, default=0, help="pods per step (default: the config's own count)")
    ap.add_argument("--batch-pods", type=int, default=0)
    ap.add_argument("--candidates", type=int, default=0)
    ap.add_argument("--no-profile", action="store_true", help="do not bracket kernels with HIP events")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=20.0)
    ap.add_argument("--shard", action="store_true",
                    help="shard the nodes over the ranks (RCCL allgather of per-shard candidates, SURVEY §8e); "
                         "default for --gpus N is N independent replicas")
    ap.add_argument("--vshards", type=int, default=1, help="virtual shards per GPU (exercises the merge on one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from koordinator_amd import abi, runtime

    # replicas schedule their own cluster (seed + rank); shards split one shared cluster
    w = build_workload(args.config, seed=20261015 + (0 if args.shard else rank), n_pods=args.pods)
    prof = w.profile
    prof.device = local_rank if world > 1 else 0
    prof.batch_pods = args.batch_pods
    prof.candidates = args.candidates
    cfg = prof.to_ks_config()
    cfg.profile = 0
    ev = runtime.Evaluator(cfg, w.nodes, w.quotas, w.reservations, w.devices, w.cpus)
    if args.shard or args.vshards > 1:
        uid = None
        if world > 1:
            box = [runtime.shard_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            uid = box[0]
        ev.shard(world if args.shard else 1, rank if args.shard else 0, uid, args.vshards)
    ev.stage(w.pods)
    ev.checkpoint()

    def sync():
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    # the timed steps run without the per-kernel HIP events (they add a dispatch gap between the pass
    # kernels); the kernel split and the roofline come from the same number of profiled steps afterwards
    ev.set_profile(False)
    for _ in range(args.warmup):
        ev.restore()
        ev.schedule_staged()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ev.restore()
        ev.schedule_staged()
    sync()
    elapsed = time.perf_counter() - t0
    st_last = ev.stats()
    agg = {"sweep_ms": 0.0, "select_ms": 0.0, "commit_ms": 0.0, "sweep_launches": 0, "passes": 0, "cut_passes": 0,
           "rescans": 0}
    sweep_bytes = 0
    prof_elapsed = 0.0
    if not args.no_profile:
        ev.set_profile(True)
        for _ in range(args.steps):
            ev.restore()
            tp = time.perf_counter()
            ev.schedule_staged()
            prof_elapsed += time.perf_counter() - tp
            st = ev.stats()
            for k in agg:
                agg[k] += st[k]
            sweep_bytes = st["sweep_bytes"]
    else:
        for k in ("passes", "cut_passes", "rescans"):
            agg[k] = st_last[k] * args.steps
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    res = ev.fetch()
    if w.cpus is not None:
        res["cpusets"] = ev.fetch_cpusets(w.pods.n)

    n_pods, n_nodes = w.pods.n, w.nodes.n
    total_pods = n_pods * args.steps * (1 if args.shard else world)
    value = total_pods / elapsed
    ms_per_step = elapsed * 1000.0 / args.steps
    out = None
    if rank == 0:
        roofline = None
        if agg["sweep_launches"]:
            avg_s = agg["sweep_ms"] / agg["sweep_launches"] / 1000.0
            # algorithmic bytes per sweep launch: SURVEY §8(d)'s B_node (LoadAware + Fit columns, each read
            # once per pass: 106 B, +16 B with the prod-usage score term, +32 B for the batch-cpu / batch-memory
            # scalar columns) x the nodes one launch sweeps, + the pass's pod records + the chunk-maxima output
            b_node = 106 + (16 if prof.loadaware is not None and prof.loadaware.score_according_prod_usage else 0) + 32
            local_nodes = n_nodes // (world if args.shard else 1)  # one rank sweeps its shard
            algo = local_nodes * b_node + 64 * 128 + ((local_nodes + 63) // 64) * 64 * 4
            if w.devices is not None:
                # + NUMA amplification columns (16 B) and the device table (flags + 34 total / topology words +
                # 32 used words, int64; ks_dev.h)
                algo += local_nodes * (16 + 4 + (34 + 32) * 8)
            if w.reservations is not None:
                # + the owner-class column and the reservation table (CSR offsets, classes, meta, order rank,
                # allocatable/allocated x7, assigned, reserve-pod non-zero x2) read once
                algo += local_nodes * (8 + 4) + w.reservations.r * (8 + 4 + 4 + 7 * 8 * 2 + 4 + 16)
            achieved = algo / avg_s / 1e9
            traffic, traffic_src = pmc_traffic(args.config, "sweep_kernel")
            roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "traffic_source": traffic_src,
                        "kernel": "sweep_kernel", "avg_launch_us": round(avg_s * 1e6, 3),
                        "algorithmic_bytes_per_launch": algo, "bytes_incl_pod_group_rereads": sweep_bytes}
            floor_us, valu_src = pmc_valu(args.config, "sweep_kernel")
            if floor_us is not None and world == 1:
                # the sweep's instruction-issue bound next to the HBM one
                roofline["valu_issue"] = {"floor_us": round(floor_us, 3),
                                          "frac": round(floor_us / (avg_s * 1e6), 4), "source": valu_src}
        out = {
            "metric": "pods scheduled/sec + node-evals/sec (% HBM roofline) at 5k and 100k nodes",
            "value": round(value, 1),
            "unit": "pods/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if args.shard else "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {"workload": f"{w.name}: {n_pods} pods x {n_nodes} nodes, NodeResourcesFit(LeastAllocated cpu/mem/batch-cpu/batch-mem)"
                                   f" + LoadAwareScheduling(defaults)" + (" + ElasticQuota(32 leaf quotas)" if w.quotas is not None else "")
                                   + (f" + Reservation(weight 5000, {w.reservations.r} reservations)" if w.reservations is not None else "")
                                   + (" + NodeNUMAResource(amplified CPUs, cpuset pods) + DeviceShare(8 GPUs x 80GiB + 4 RDMA on 4 PCIe/2 NUMA per node, joint GPU+RDMA)" if w.devices is not None else ""),
                       "pods_per_step": n_pods, "nodes": n_nodes, "percentage_of_nodes_to_score": 100,
                       "parallelism": (f"node-shards{world}x{args.vshards}" if args.shard or args.vshards > 1
                                       else (f"replicas{world}" if world > 1 else "single-gpu")),
                       "batch_pods": cfg.batch_pods or 64, "candidates": cfg.candidates or 32},
            "node_evals_per_s": round(value * n_nodes, 1),
            "placed_per_step": int((res["status"] == 0).sum()),
            "into_reservations_per_step": int((res["reservation"] >= 0).sum()),
            "gpu_pods_placed_per_step": int((res["gpu_minors"] != 0).sum()),
            "rdma_pods_placed_per_step": int((res["rdma_minors"] != 0).sum()),
            "cpuset_pods_placed_per_step": int(((res["status"] == 0) & ((w.pods.flags & abi.KS_POD_CPU_BIND) != 0)).sum()),
            "profiled_steps": 0 if args.no_profile else args.steps,
            "ms_per_profiled_step": round(prof_elapsed * 1000.0 / args.steps, 3) if not args.no_profile else None,
            "passes_per_step": agg["passes"] / args.steps,
            "cut_passes_per_step": agg["cut_passes"] / args.steps,
            "rescans_per_step": agg["rescans"] / args.steps,
            "kernel_ms_per_step": {"sweep": round(agg["sweep_ms"] / args.steps, 3),
                                   "select": round(agg["select_ms"] / args.steps, 3),
                                   "commit": round(agg["commit_ms"] / args.steps, 3)},
            "roofline": roofline,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(w, res, args.cpu_budget_s)
            out["cpu_baseline"] = cb
            out["parity"] = cb["parity_with_gpu_on_sample"]
            out["speedup_vs_cpu_baseline"] = round(value / cb["value"], 2)
    ev.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
