"""GPU parity for SURVEY's C3 as the reference runs it: half of the nodes carry a NUMA topology policy
(SingleNUMANode by default) with two NUMA nodes, where NodeNUMAResource and DeviceShare are both topology hint
providers (frameworkext/topologymanager; deviceshare/topology_hint.go) and cpuset pods take their CPUs per
allocated NUMA node (resource_manager.go allocateCPUSet).  Whole queues against the oracle: placements, scores,
statuses, GPU / RDMA minors, per-pod cpusets, the CPU state, the device table, Requested and the NUMA nodes'
allocatedResources after every commit; single-pod Filter/Score parity on device and cpuset pods; checkpoint /
restore of the per-NUMA cpuset counts; virtual shards."""
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


def check(runtime, oracle_lib, w, label, cfg=None, vshards=0):
    cfg = cfg or w.cfg
    ev = runtime.Evaluator(cfg, w.nodes.copy(), **w.tables())
    if vshards:
        ev.shard(1, 0, None, virtual_shards=vshards)
    got = ev.schedule(w.pods)
    orc = oracle_lib.Oracle(cfg, w.nodes.copy(), nthreads=8, **w.tables())
    want = orc.schedule(w.pods)
    assert_same_results(got, want, label)
    for k in ("gpu_minors", "rdma_minors"):
        assert np.array_equal(got[k], want[k]), f"{label}: {k} differ"
    cs_g, cs_o = ev.fetch_cpusets(w.pods.n), orc.fetch_cpusets(w.pods.n)
    bad = np.nonzero((cs_g != cs_o).any(axis=1))[0]
    assert bad.size == 0, (f"{label}: cpusets differ for pods {bad[:8]}: "
                           f"{[mask_cpus(cs_g[i]) for i in bad[:2]]} vs {[mask_cpus(cs_o[i]) for i in bad[:2]]}")
    for a, b in zip(ev.read_cpu_state(), orc.read_cpu_state()):
        assert np.array_equal(a, b), f"{label}: CPU state differs"
    for g, o, name in zip(ev.read_devices(), orc.read_devices(), ("core", "memory", "ratio", "rdma")):
        assert np.array_equal(g, o), f"{label}: device used {name} differs"
    for g, o, name in zip(ev.read_numa_nodes(), orc.read_numa_nodes(), ("cpu", "memory")):
        assert np.array_equal(g, o), f"{label}: NUMA used {name} differs"
    assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
    ev.close()
    orc.close()
    return got


def policy_stats(w, got):
    pol = (w.nodes.numa_flags >> abi.KS_NUMA_POLICY_SHIFT) & 3
    ok = got["status"] == abi.KS_S_SCHEDULED
    onpol = ok & (pol[np.maximum(got["node"], 0)] > 0)
    bind = (w.pods.flags & abi.KS_POD_CPU_BIND) != 0
    dev = (w.pods.gpu_core + w.pods.gpu_memory + w.pods.gpu_memory_ratio + w.pods.rdma) > 0
    return int(onpol.sum()), int((onpol & bind).sum()), int((onpol & dev).sum())


def test_c3_full_5k_nodes(runtime, oracle_lib):
    """5k nodes (half SingleNUMANode), 10k pods"""
    w = synth.c3()
    got = check(runtime, oracle_lib, w, "c3-5k")
    on, bind, dev = policy_stats(w, got)
    assert on > 2000 and bind > 300 and dev > 500, (on, bind, dev)


@pytest.mark.parametrize("seed,policy,numa_strategy", [
    (71, abi.KS_NUMA_POLICY_SINGLE_NUMA_NODE, "MostAllocated"),
    (72, abi.KS_NUMA_POLICY_BEST_EFFORT, "LeastAllocated"),
    (73, abi.KS_NUMA_POLICY_RESTRICTED, "LeastAllocated"),
    (74, abi.KS_NUMA_POLICY_RESTRICTED, "MostAllocated"),
])
def test_c3_policies(runtime, oracle_lib, seed, policy, numa_strategy):
    w = synth.c3(seed=seed, n_nodes=600, n_pods=1500, policy=policy, policy_frac=0.7)
    w.profile.numa.numa_scoring_strategy = numa_strategy
    got = check(runtime, oracle_lib, w, f"c3-policy{policy}-{numa_strategy}")
    assert policy_stats(w, got)[0] > 300


def test_c3_tight_nodes(runtime, oracle_lib):
    """few nodes, many pods: NUMA nodes and devices fill up, cpuset pods hit per-NUMA shortages"""
    w = synth.c3(seed=75, n_nodes=80, n_pods=1200, policy_frac=0.8)
    got = check(runtime, oracle_lib, w, "c3-tight")
    assert (got["status"] != abi.KS_S_SCHEDULED).sum() > 100


def test_c3_virtual_shards(runtime, oracle_lib):
    w = synth.c3(seed=76, n_nodes=900, n_pods=1200)
    check(runtime, oracle_lib, w, "c3-vshards", vshards=3)


def test_c3_eval_pod_parity(runtime, oracle_lib):
    """single-pod Filter reasons, per-plugin scores and totals on every node (the debug path), for device pods,
    cpuset pods and cpuset device pods"""
    w = synth.c3(seed=77, n_nodes=400, n_pods=400)
    bind = (w.pods.flags & abi.KS_POD_CPU_BIND) != 0
    dev = (w.pods.gpu_core + w.pods.gpu_memory + w.pods.gpu_memory_ratio + w.pods.rdma) > 0
    idx = np.concatenate([np.nonzero(dev & ~bind)[0][:25], np.nonzero(bind & ~dev)[0][:25], np.nonzero(bind & dev)[0][:25],
                          np.nonzero(~bind & ~dev)[0][:10]])
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), **w.tables())
    for i in idx:
        one = w.pods.rows([int(i)])
        r_g, s_g, t_g = ev.eval_pod(one)
        r_o, s_o, t_o = orc.eval_pod(one)
        assert np.array_equal(r_g, r_o), f"pod {i}: reasons {np.nonzero(r_g != r_o)[0][:5]}"
        assert np.array_equal(s_g, s_o), f"pod {i}: scores"
        assert np.array_equal(t_g, t_o), f"pod {i}: totals"
    ev.close()
    orc.close()


def test_c3_checkpoint_restore(runtime):
    """restore brings back the NUMA nodes' allocatedResources, cpuset counts, offsets and free CPUs"""
    w = synth.c3(seed=78, n_nodes=200, n_pods=600, policy_frac=0.9)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    ev.stage(w.pods)
    ev.checkpoint()
    outs = []
    for _ in range(2):
        ev.restore()
        ev.schedule_staged()
        outs.append((ev.fetch(), ev.fetch_cpusets(w.pods.n), ev.read_cpu_state()[0], ev.read_numa_nodes()))
    for k in ("node", "status", "score", "gpu_minors"):
        assert np.array_equal(outs[0][0][k], outs[1][0][k]), k
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][2], outs[1][2])
    for a, b in zip(outs[0][3], outs[1][3]):
        assert np.array_equal(a, b)
    ev.close()
