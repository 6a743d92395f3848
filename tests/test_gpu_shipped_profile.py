"""GPU parity of the shipped koord-scheduler profile's plugin set (config/manager/scheduler-config.yaml:58-96):
Reservation + NodeNUMAResource + DeviceShare together, next to NodeResourcesFit + LoadAware -- C3's nodes (NUMA
topology policies, cpuset pods, GPU / RDMA devices) with C4-style reservations (synth.c3_rsv).  The Reservation
BeforePreFilter restore feeds the NUMA plugin's amplified-CPU filter and, on policy nodes, the score over the
allocated NUMA nodes (calculateAllocatableAndRequested falls back to the restored NodeInfo); NodeNUMAResource's and
DeviceShare's own RestoreReservation hooks (nodenumaresource/reservation.go:68-115, deviceshare/reservation.go) give
nothing back for reservations that hold no cpuset and no device, which is what these reservations are.  Whole queues
against the oracle: placements, scores, statuses, nominated reservations, GPU / RDMA minors, cpusets, and the node,
reservation, device, CPU and NUMA-node state after every commit; single-pod Filter / Score parity.  A pod with device
requests is never nominated into (nor assumed into) one of these reservations: DeviceShare's FilterReservation rejects
a reservation that holds no device."""
import numpy as np
import pytest

from helpers import assert_same_results, assert_same_state
from koordinator_amd import abi, synth
from koordinator_amd.cluster import mask_cpus

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


def check(runtime, oracle_lib, w, label, pipeline=None, vshards=0):
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    if pipeline is not None:
        ev.set_pipeline(pipeline)
    if vshards:
        ev.shard(1, 0, None, virtual_shards=vshards)
    got = ev.schedule(w.pods)
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), nthreads=8, **w.tables())
    want = orc.schedule(w.pods)
    try:
        assert_same_results(got, want, label)
        for k in ("reservation", "gpu_minors", "rdma_minors"):
            assert np.array_equal(got[k], want[k]), f"{label}: {k} differ at pods {np.nonzero(got[k] != want[k])[0][:8]}"
        cs_g, cs_o = ev.fetch_cpusets(w.pods.n), orc.fetch_cpusets(w.pods.n)
        bad = np.nonzero((cs_g != cs_o).any(axis=1))[0]
        assert bad.size == 0, f"{label}: cpusets differ for pods {bad[:8]}: {[mask_cpus(cs_g[i]) for i in bad[:2]]}"
        for a, b in zip(ev.read_reservations(), orc.read_reservations()):
            assert np.array_equal(a, b), f"{label}: reservations differ"
        if w.reservations.dev_allocatable is not None:
            rg, ro = ev.read_reservation_devices(), orc.read_reservation_devices()
            bad = np.nonzero((rg != ro).any(axis=1))[0]
            assert bad.size == 0, f"{label}: reservation device allocations differ at rows {bad[:8]}"
        for a, b in zip(ev.read_cpu_state(), orc.read_cpu_state()):
            assert np.array_equal(a, b), f"{label}: CPU state differs"
        for g, o in zip(ev.read_devices(), orc.read_devices()):
            assert np.array_equal(g, o), f"{label}: device state differs"
        for g, o in zip(ev.read_numa_nodes(), orc.read_numa_nodes()):
            assert np.array_equal(g, o), f"{label}: NUMA-node state differs"
        assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
    finally:
        ev.close()
        orc.close()
    return got


def coverage(w, got):
    pol = (w.nodes.numa_flags >> abi.KS_NUMA_POLICY_SHIFT) & 3
    ok = got["status"] == abi.KS_S_SCHEDULED
    onpol = ok & (pol[np.maximum(got["node"], 0)] > 0)
    into = got["reservation"] >= 0
    dev = (w.pods.gpu_core + w.pods.gpu_memory + w.pods.gpu_memory_ratio + w.pods.rdma) > 0
    bind = (w.pods.flags & abi.KS_POD_CPU_BIND) != 0
    return {"placed": int(ok.sum()), "on_policy": int(onpol.sum()), "into_rsv": int(into.sum()),
            "into_rsv_on_policy": int((into & onpol).sum()), "dev_into_rsv": int((into & dev).sum()),
            "bind_into_rsv": int((into & bind).sum()),
            "dev_matched_placed": int((ok & dev & (w.pods.rsv_class >= 0)).sum())}


def test_shipped_profile_5k_nodes(runtime, oracle_lib):
    """5k C3 nodes (half SingleNUMANode) with 12.5k reservations, 10k pods"""
    w = synth.c3_rsv()
    c = coverage(w, check(runtime, oracle_lib, w, "c3rsv-5k"))
    # a device pod is never assumed into a reservation holding no device (DeviceShare's FilterReservation,
    # deviceshare/plugin.go:322-358), though the restore still frees the matched reservations' resources for it
    # (these reservations hold none: test_shipped_profile_device_reservations has ones that do)
    assert c["into_rsv_on_policy"] > 300 and c["bind_into_rsv"] > 300 and c["dev_matched_placed"] > 300, c
    assert c["dev_into_rsv"] == 0, c


@pytest.mark.parametrize("seed,policy", [
    (81, abi.KS_NUMA_POLICY_SINGLE_NUMA_NODE), (82, abi.KS_NUMA_POLICY_BEST_EFFORT), (83, abi.KS_NUMA_POLICY_RESTRICTED)])
def test_shipped_profile_policies(runtime, oracle_lib, seed, policy):
    w = synth.c3_rsv(seed=seed, n_nodes=700, n_pods=1500, policy=policy, policy_frac=0.7, rsv_per_node=3.0)
    c = coverage(w, check(runtime, oracle_lib, w, f"c3rsv-policy{policy}"))
    assert c["into_rsv_on_policy"] > 100, c


@pytest.mark.parametrize("seed", [87, 88])
def test_shipped_profile_device_reservations(runtime, oracle_lib, seed):
    """Reservations holding GPUs / RDMA (deviceshare/reservation.go): on non-policy device nodes 70 % of the
    reservations hold one or two GPU instances (whole or half) and half of those an RDMA share; the matched ones are
    allocated from first (Default / Aligned prefer their minors, Restricted requires them), the unmatched ones' assigned
    use is given back, device pods are nominated into them by FilterReservation / ScoreReservation"""
    w = synth.c3_rsv(seed=seed, n_nodes=600, n_pods=1500, policy_frac=0.3, dev_rsv_frac=0.7)
    held = (w.reservations.dev_allocatable != 0).any(axis=1)
    assert held.mean() > 0.3
    got = check(runtime, oracle_lib, w, f"c3rsv-devrsv{seed}")
    c = coverage(w, got)
    into = got["reservation"]
    assert c["dev_into_rsv"] > 50 and held[into[into >= 0]].sum() > 50, c


def test_shipped_profile_device_reservations_full_size(runtime, oracle_lib):
    """the bench's c3rd record itself (bench.py build_workload, sub-record seed): 10k pods x 5k nodes, about a third of
    the reservations holding GPUs / RDMA, every result and the final reservation / device / CPU state vs the oracle"""
    w = synth.c3_rsv(seed=20261015, dev_rsv_frac=0.7)
    assert w.nodes.n == 5000 and w.pods.n == 10_000
    held = (w.reservations.dev_allocatable != 0).any(axis=1)
    assert held.mean() > 0.3
    got = check(runtime, oracle_lib, w, "c3rd")
    into = got["reservation"]
    assert held[into[into >= 0]].sum() > 200


def test_shipped_profile_device_reservations_eval_pod(runtime, oracle_lib):
    w = synth.c3_rsv(seed=89, n_nodes=300, n_pods=300, policy_frac=0.3, dev_rsv_frac=0.7)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), **w.tables())
    try:
        for i in range(0, 300, 3):
            one = w.pods.rows([i])
            r_g, s_g, t_g = ev.eval_pod(one)
            r_o, s_o, t_o = orc.eval_pod(one)
            assert np.array_equal(r_g, r_o), f"pod {i}: reasons at nodes {np.nonzero(r_g != r_o)[0][:5]}"
            assert np.array_equal(s_g, s_o), f"pod {i}: scores at nodes {np.nonzero((s_g != s_o).any(axis=1))[0][:5]}"
            assert np.array_equal(t_g, t_o), f"pod {i}: totals"
    finally:
        ev.close()
        orc.close()


def test_shipped_profile_tight(runtime, oracle_lib):
    """few nodes, many pods: reservations, NUMA nodes and devices fill up"""
    w = synth.c3_rsv(seed=84, n_nodes=120, n_pods=1500, policy_frac=0.8, rsv_per_node=4.0)
    got = check(runtime, oracle_lib, w, "c3rsv-tight")
    assert (got["status"] != abi.KS_S_SCHEDULED).sum() > 100


def test_shipped_profile_pipelined_and_virtual_shards(runtime, oracle_lib):
    w = synth.c3_rsv(seed=85, n_nodes=900, n_pods=1200)
    check(runtime, oracle_lib, w, "c3rsv-pipe", pipeline=1)
    check(runtime, oracle_lib, w, "c3rsv-vshards", vshards=3)


def test_shipped_profile_eval_pod(runtime, oracle_lib):
    """single-pod Filter reasons, per-plugin scores (Reservation normalized included) and totals on every node"""
    w = synth.c3_rsv(seed=86, n_nodes=400, n_pods=400)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), **w.tables())
    try:
        for i in range(0, 400, 5):
            one = w.pods.rows([i])
            r_g, s_g, t_g = ev.eval_pod(one)
            r_o, s_o, t_o = orc.eval_pod(one)
            assert np.array_equal(r_g, r_o), f"pod {i}: reasons at nodes {np.nonzero(r_g != r_o)[0][:5]}"
            assert np.array_equal(s_g, s_o), f"pod {i}: scores at nodes {np.nonzero((s_g != s_o).any(axis=1))[0][:5]}"
            assert np.array_equal(t_g, t_o), f"pod {i}: totals"
    finally:
        ev.close()
        orc.close()


def test_c3_full_5k_nodes_quota_and_default_plugins(runtime, oracle_lib):
    """SURVEY C3 at full size under the rest of the shipped profile too: NUMA policies + DeviceShare + ElasticQuota +
    TaintToleration / NodeAffinity / NodePorts (synth.c3_full).  The commit kernel then holds the NUMA and device slot
    caches, the dictionary-plugin words, the PodStat records and the quota rows in one workgroup's LDS; the stats say
    how much of the CU's 160 KB that is and whether the helper waves' region still fit."""
    w = synth.c3_full()
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    try:
        got = ev.schedule(w.pods)
        st = ev.stats()
        cs_g = ev.fetch_cpusets(w.pods.n)
        dev_g = ev.read_devices()
        numa_g = ev.read_numa_nodes()
        nodes_g = ev.read_nodes()
        q_g = ev.read_quota_used()
    finally:
        ev.close()
    print(f"c3-full: commit LDS {st['commit_lds_bytes']} B of 163840, helper waves {st['commit_helpers']}, "
          f"passes {st['passes']}, cuts {st['cut_passes']}, pre-reserves {st['pre_reserves']}")
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), nthreads=8, **w.tables())
    try:
        want = orc.schedule(w.pods)
        assert_same_results(got, want, "c3-full")
        for k in ("gpu_minors", "rdma_minors"):
            assert np.array_equal(got[k], want[k]), f"c3-full: {k} differ"
        assert np.array_equal(cs_g, orc.fetch_cpusets(w.pods.n)), "c3-full: cpusets differ"
        for g, o in zip(dev_g, orc.read_devices()):
            assert np.array_equal(g, o), "c3-full: device state differs"
        for g, o in zip(numa_g, orc.read_numa_nodes()):
            assert np.array_equal(g, o), "c3-full: NUMA-node state differs"
        assert np.array_equal(q_g, orc.read_quota_used()), "c3-full: quota used differs"
        assert_same_state(nodes_g, orc.read_nodes(), "c3-full")
    finally:
        orc.close()
    assert st["commit_lds_bytes"] <= 160 * 1024
    rejected = int(((got["status"] & (abi.KS_S_QUOTA | abi.KS_S_QUOTA_NONPREEMPTIBLE)) != 0).sum())
    assert rejected > 100 and int((got["gpu_minors"] != 0).sum()) > 1000, rejected
