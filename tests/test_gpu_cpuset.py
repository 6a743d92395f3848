"""GPU parity for NodeNUMAResource cpusets (SURVEY a21/a22 cpu-bind pods, a24 CPU accumulator on
topology-policy-None nodes): the reference's accumulator tables through the HIP library, and whole-queue
scheduling against the oracle with cpu-bind pods mixed into Fit + LoadAware + NUMA (+ DeviceShare)
queues: placements, statuses, scores, the CPU sets of every pod, the nodes' CPU allocation and Requested."""
import json
import os

import numpy as np
import pytest

from cpuset_util import golden_cluster, supported_on_device
from helpers import assert_same_results, assert_same_state
from koordinator_amd import abi, synth
from koordinator_amd.cluster import mask_cpus

pytestmark = pytest.mark.gpu

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "cpuset.json")))
CASES = [c for c in G["cases"] if supported_on_device(c)]


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


@pytest.mark.parametrize("case", CASES, ids=[f"{c['test']}:{c['name']}" for c in CASES])
def test_golden_cpusets(runtime, case):
    cfg, nodes, st, pod = golden_cluster(case)
    ev = runtime.Evaluator(cfg, nodes, cpu_state=st)
    r = ev.schedule(pod)
    assert r["status"][0] == abi.KS_S_SCHEDULED and r["node"][0] == 0
    assert mask_cpus(ev.fetch_cpusets(1)[0]) == case["want"]
    alloc, xp, xn = ev.read_cpu_state()
    assert mask_cpus(alloc[0]) == sorted(case["allocated"] + case["want"])
    ev.close()


def run_pair(runtime, oracle_lib, w, label, devices=True):
    cfg = w.cfg
    tabs = w.tables()
    if not devices:
        tabs.pop("devices", None)
    ev = runtime.Evaluator(cfg, w.nodes.copy(), **tabs)
    got = ev.schedule(w.pods)
    orc = oracle_lib.Oracle(cfg, w.nodes.copy(), nthreads=8, **{k: v.copy() for k, v in tabs.items()})
    want = orc.schedule(w.pods)
    assert_same_results(got, want, label)
    assert np.array_equal(got["gpu_minors"], want["gpu_minors"]), label
    cs_g, cs_o = ev.fetch_cpusets(w.pods.n), orc.fetch_cpusets(w.pods.n)
    bad = np.nonzero((cs_g != cs_o).any(axis=1))[0]
    assert bad.size == 0, f"{label}: cpusets differ for pods {bad[:8]}: {[mask_cpus(cs_g[i]) for i in bad[:2]]} vs {[mask_cpus(cs_o[i]) for i in bad[:2]]}"
    for a, b in zip(ev.read_cpu_state(), orc.read_cpu_state()):
        assert np.array_equal(a, b), label
    assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
    ev.close()
    orc.close()
    return got, cs_g


@pytest.mark.parametrize("seed", [41, 42])
def test_schedule_cpuset_small(runtime, oracle_lib, seed):
    w = synth.c3(seed=seed, n_nodes=300, n_pods=800)
    got, cs = run_pair(runtime, oracle_lib, w, f"c3-small-{seed}")
    bind = (w.pods.flags & abi.KS_POD_CPU_BIND) != 0
    assert ((got["status"] == 0) & bind).sum() > 100


def test_schedule_cpuset_tight_reserve_failures(runtime, oracle_lib):
    """few free CPUs: Reserve failures (not enough cpus) leave no trace; later pods see unchanged nodes"""
    w = synth.c3(seed=43, n_nodes=120, n_pods=900)
    w.nodes.numa_cpu_amplification[:] = 3.0
    w.nodes.alloc_milli_cpu[:] = w.nodes.alloc_milli_cpu * 3
    got, _ = run_pair(runtime, oracle_lib, w, "c3-tight", devices=False)
    assert (got["status"] == abi.KS_S_RESERVE_FAILED).sum() > 0


@pytest.mark.parametrize("most", [False, True])
def test_schedule_cpuset_strategies_no_devices(runtime, oracle_lib, most):
    w = synth.c3(seed=44, n_nodes=400, n_pods=1200)
    w.profile.numa.numa_scoring_strategy = "MostAllocated" if most else "LeastAllocated"
    w.profile.deviceshare = None
    w.nodes.numa_flags[:] &= ~np.uint32(abi.KS_NUMA_ALLOC_MOST | abi.KS_NUMA_ALLOC_LEAST)
    run_pair(runtime, oracle_lib, w, f"c3-strategy-{most}", devices=False)


def test_schedule_cpuset_c3_prefix(runtime, oracle_lib):
    w = synth.c3(n_pods=1500)
    got, _ = run_pair(runtime, oracle_lib, w, "c3-prefix")
    assert (got["status"] == 0).sum() > 1200


def test_cpuset_checkpoint_restore(runtime):
    w = synth.c3(seed=45, n_nodes=200, n_pods=500)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    ev.stage(w.pods)
    ev.checkpoint()
    outs = []
    for _ in range(2):
        ev.restore()
        ev.schedule_staged()
        outs.append((ev.fetch(), ev.fetch_cpusets(w.pods.n), ev.read_cpu_state()[0]))
    for k in ("node", "status", "score"):
        assert np.array_equal(outs[0][0][k], outs[1][0][k])
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][2], outs[1][2])
    ev.close()


def test_eval_debug_cpu_bind(runtime, oracle_lib):
    w = synth.c3(seed=46, n_nodes=300, n_pods=60)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), **w.tables())
    seen = 0
    for i in range(w.pods.n):
        one = w.pods.rows([i])
        r_g, s_g, t_g = ev.eval_pod(one)
        r_o, s_o, t_o = orc.eval_pod(one)
        assert np.array_equal(r_g, r_o), f"pod {i}: reasons"
        assert np.array_equal(s_g, s_o), f"pod {i}: scores"
        assert np.array_equal(t_g, t_o), f"pod {i}: totals"
        seen += int((r_g & abi.KS_R_NUMA_INVALID_TOPOLOGY).any())
    assert seen > 0
    ev.close()
    orc.close()


@pytest.mark.parametrize("seed", range(4))
def test_full_pcpus_split_cores(runtime, oracle_lib, seed):
    """A preferred FullPCPUs request that is not a whole number of cores (takeCPUs takes a core's first CPUs in
    freeCoresInNode / freeCoresInSocket prefixes, whole cores then single cores in the fallback, then spread CPUs):
    the HIP accumulator against the oracle's restatement on the golden tables' topologies with random allocations,
    exclusive policies and strategies.  (The reference's tables hold no such request: parity against the oracle
    only.)"""
    rng = np.random.default_rng(100 + seed)
    n_checked = 0
    for case in G["cases"]:
        if case["max_ref"] != 1 or case["topo"][3] < 2:
            continue
        core_count = case["topo"][0] * case["topo"][1] * case["topo"][2]
        ncpu = core_count * case["topo"][3]
        c = dict(case)
        c["allocated"] = sorted(rng.choice(ncpu, int(rng.integers(0, ncpu // 2)), replace=False).tolist())
        c["allocated_excl"] = str(rng.choice(["None", "PCPULevel", "NUMANodeLevel"]))
        free = ncpu - len(c["allocated"])
        c["needed"] = int(rng.integers(1, max(2, free)))
        if c["needed"] % case["topo"][3] == 0:
            c["needed"] = max(1, c["needed"] - 1)
        c["bind"] = "FullPCPUs"
        c["excl"] = str(rng.choice(["None", "PCPULevel", "NUMANodeLevel"]))
        c["strategy"] = str(rng.choice(["Most", "Least"]))
        cfg, nodes, st, pod = golden_cluster(c)
        ev = runtime.Evaluator(cfg, nodes.copy(), cpu_state=st.copy() if hasattr(st, "copy") else st)
        got = ev.schedule(pod)
        cs_g = mask_cpus(ev.fetch_cpusets(1)[0])
        state_g = ev.read_cpu_state()
        ev.close()
        cfg, nodes, st, pod = golden_cluster(c)
        orc = oracle_lib.Oracle(cfg, nodes, cpu_state=st)
        want = orc.schedule(pod)
        cs_o = mask_cpus(orc.fetch_cpusets(1)[0])
        state_o = orc.read_cpu_state()
        orc.close()
        label = f"{case['name']} needed {c['needed']} excl {c['excl']}/{c['allocated_excl']} {c['strategy']}"
        assert got["status"][0] == want["status"][0] and got["node"][0] == want["node"][0], label
        assert cs_g == cs_o, f"{label}: {cs_g} (GPU) vs {cs_o} (oracle)"
        for a, b in zip(state_g, state_o):
            assert np.array_equal(a, b), label
        n_checked += int(want["status"][0] == abi.KS_S_SCHEDULED)
    assert n_checked > 10


def test_full_pcpus_split_cores_hand_traced(runtime):
    """the hand-traced split-core cases of tests/test_cpuset_golden.py on the device's accumulator"""
    from test_cpuset_golden import SPLIT_CORE_CASES

    for name, topo, alloc, needed, strategy, want in SPLIT_CORE_CASES:
        c = {"topo": list(topo), "allocated": alloc, "allocated_excl": "None", "needed": needed, "bind": "FullPCPUs",
             "excl": "None", "strategy": strategy}
        cfg, nodes, st, pod = golden_cluster(c)
        ev = runtime.Evaluator(cfg, nodes.copy(), cpu_state=st)
        got = ev.schedule(pod)
        cs = mask_cpus(ev.fetch_cpusets(1)[0])
        ev.close()
        assert got["status"][0] == abi.KS_S_SCHEDULED, name
        assert cs == want, f"{name}: {cs} vs {want}"
