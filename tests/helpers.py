"""Shared workload builders for the parity tests (host-side only)."""
from __future__ import annotations

import numpy as np

from koordinator_amd import abi, synth
from koordinator_amd.cluster import NodeTable, PodTable, QuotaTable
from koordinator_amd.config import (BATCH_CPU, BATCH_MEMORY, CPU, EPHEMERAL, MEMORY, ElasticQuotaArgs,
                                    NodeResourcesBalancedAllocationArgs,
                                    LoadAwareSchedulingArgs, NodeResourcesFitArgs, SchedulerProfile)


def stress_nodes(n: int, rng: np.random.Generator, tight: bool = False) -> NodeTable:
    """synth nodes plus randomised LoadAware flags / thresholds / edge values."""
    t = synth.make_nodes(n, rng)
    flags = rng.integers(0, 256, n).astype(np.uint32)
    # mostly realistic: keep HAS_METRIC in 85 % of nodes
    flags = np.where(rng.random(n) < 0.85, flags | abi.KS_LA_HAS_METRIC, flags & ~np.uint32(abi.KS_LA_HAS_METRIC))
    t.la_flags[:] = flags
    t.la_thr_cpu[:] = rng.choice(np.array([0, 30, 50, 65, 100]), n)
    t.la_thr_memory[:] = rng.choice(np.array([0, 60, 95, 100]), n)
    t.la_prod_thr_cpu[:] = rng.choice(np.array([0, 20, 40, 100]), n)
    t.la_prod_thr_memory[:] = rng.choice(np.array([0, 50, 100]), n)
    # some nodes with raw-allocatable overrides and zero capacities
    over = rng.random(n) < 0.1
    t.la_alloc_milli_cpu[over] = t.la_alloc_milli_cpu[over] * 7 // 8
    t.la_alloc_memory[rng.random(n) < 0.02] = 0
    t.alloc_ephemeral[rng.random(n) < 0.05] = 0
    t.alloc_scalar[synth.SLOT_BATCH_CPU][rng.random(n) < 0.1] = 0
    if tight:
        t.pod_count[:] = rng.integers(100, 111, n)
        t.req_milli_cpu[:] = t.alloc_milli_cpu - rng.integers(0, 8000, n)
        t.req_milli_cpu[:] = np.maximum(t.req_milli_cpu, 0)
    # exact-boundary cases for the division: requested == capacity, capacity 1
    edge = rng.random(n) < 0.03
    t.nonzero_milli_cpu[edge] = t.alloc_milli_cpu[edge]
    t.la_term_memory[rng.random(n) < 0.03] = t.la_alloc_memory[rng.random(n) < 0.03].max(initial=0)
    return t


def stress_pods(p: int, rng: np.random.Generator, n_quotas: int = 0) -> PodTable:
    t = synth.make_pods(p, rng, n_quotas)
    ds = rng.random(p) < 0.05
    t.flags[ds] |= abi.KS_POD_DAEMONSET
    zero = rng.random(p) < 0.05
    t.req_milli_cpu[zero] = 0
    t.req_memory[zero] = 0
    t.req_scalar[:, zero] = 0
    t.flags[zero] &= ~np.uint32(abi.KS_POD_SCALAR_KEYS)
    t.la_req_cpu[zero] = 0
    t.la_lim_cpu[zero] = 0
    t.la_req_memory[zero] = 0
    t.la_lim_memory[zero] = 0
    mid = rng.random(p) < 0.05  # koord-mid pods: translated mid-cpu is absent -> estimate 0
    t.la_req_cpu[mid] = 0
    t.la_lim_cpu[mid] = 0
    t.la_dflt_cpu[mid] = 0
    t.la_dflt_memory[mid] = 0
    t.la_req_memory[mid] = 0
    t.la_lim_memory[mid] = 0
    t.req_ephemeral[rng.random(p) < 0.1] = 10 << 30
    if n_quotas:
        t.flags[rng.random(p) < 0.1] |= abi.KS_POD_NONPREEMPTIBLE
        t.quota[rng.random(p) < 0.05] = -1
    return t


def profile(strategy: str = "LeastAllocated", quota: bool = False, prod_usage: bool = False,
            batch_pods: int = 0, candidates: int = 0, fit_weight: int = 1, la_weight: int = 1,
            eph_weight: int = 0, check_parent: bool = False, filter_expired: bool = True,
            balanced: int = 0) -> SchedulerProfile:
    res = {CPU: 1, MEMORY: 1, BATCH_CPU: 1, BATCH_MEMORY: 1}
    if eph_weight:
        res[EPHEMERAL] = eph_weight
    la = LoadAwareSchedulingArgs(score_according_prod_usage=prod_usage, filter_expired_node_metrics=filter_expired)
    return SchedulerProfile(fit=NodeResourcesFitArgs(strategy=strategy, resources=res), fit_weight=fit_weight,
                            loadaware=la, loadaware_weight=la_weight,
                            quota=ElasticQuotaArgs(enable_check_parent_quota=check_parent) if quota else None,
                            batch_pods=batch_pods, candidates=candidates,
                            balanced=NodeResourcesBalancedAllocationArgs() if balanced else None,
                            balanced_weight=balanced or 1)


def nested_quotas(pods: PodTable, rng: np.random.Generator, n_leaf: int) -> QuotaTable:
    """leaf quotas under 4 parent groups (rows n_leaf..n_leaf+3)."""
    q = synth.make_quotas(pods, n_leaf, rng, admit_frac=0.85)
    full = QuotaTable(n_leaf + 4)
    for name in ("limit_mask", "min_mask"):
        getattr(full, name)[:n_leaf] = getattr(q, name)
        getattr(full, name)[n_leaf:] = getattr(q, name)[0]
    for name in ("limit", "used", "min", "nonpreemptible_used"):
        getattr(full, name)[:, :n_leaf] = getattr(q, name)
    full.parent[:n_leaf] = n_leaf + (np.arange(n_leaf) % 4)
    for g in range(4):
        kids = np.arange(n_leaf) % 4 == g
        full.limit[:, n_leaf + g] = (q.limit[:, kids].sum(axis=1) * 0.8).astype(np.int64)
        full.min[:, n_leaf + g] = full.limit[:, n_leaf + g] // 2
    return full


def homogeneous_pods(p: int, cpu: int = 1000, mem: int = 1 << 30) -> PodTable:
    t = PodTable(p)
    t.req_milli_cpu[:] = cpu
    t.req_memory[:] = mem
    t.nonzero_milli_cpu[:] = cpu
    t.nonzero_memory[:] = mem
    t.flags[:] = abi.KS_POD_PROD
    t.la_req_cpu[:] = cpu
    t.la_req_memory[:] = mem
    t.la_dflt_cpu[:] = 250
    t.la_dflt_memory[:] = 200 << 20
    return t


def assert_same_results(got: dict, want: dict, label: str = ""):
    for k in ("node", "status", "score"):
        g, w = np.asarray(got[k]), np.asarray(want[k])
        if not np.array_equal(g, w):
            bad = np.nonzero(g != w)[0]
            i = int(bad[0])
            raise AssertionError(
                f"{label}: {k} differs at {len(bad)} pods; first pod {i}: got "
                f"node={got['node'][i]} status={got['status'][i]} score={got['score'][i]}, want "
                f"node={want['node'][i]} status={want['status'][i]} score={want['score'][i]}")


def assert_same_state(got, want, label: str = ""):
    g, w = got.as_dict(), want.as_dict()
    for k in w:
        if not np.array_equal(g[k], w[k]):
            bad = np.argwhere(np.asarray(g[k]) != np.asarray(w[k]))
            raise AssertionError(f"{label}: node state {k} differs at {len(bad)} entries, first {bad[0].tolist()}")
