"""NodeNUMAResource cpusets on the CPU oracle's scheduling path: the reference's accumulator tables
through ko_schedule (one node, one cpu-bind pod), Reserve failure, topology checks, and the
amplified request of cpu-bind pods."""
import json
import os

import numpy as np
import pytest

from cpuset_util import golden_cluster
from koordinator_amd import abi, synth
from koordinator_amd.cluster import mask_cpus
from oracle.oracle import Oracle

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "cpuset.json")))
CASES = [c for c in G["cases"] if c["max_ref"] == 1]


@pytest.mark.parametrize("case", CASES, ids=[f"{c['test']}:{c['name']}" for c in CASES])
def test_golden_through_oracle_schedule(case):
    cfg, nodes, st, pod = golden_cluster(case)
    o = Oracle(cfg, nodes, cpu_state=st)
    r = o.schedule(pod)
    assert r["status"][0] == abi.KS_S_SCHEDULED and r["node"][0] == 0
    assert mask_cpus(o.fetch_cpusets(1)[0]) == case["want"]
    alloc, _, _ = o.read_cpu_state()
    assert mask_cpus(alloc[0]) == sorted(case["allocated"] + case["want"])


def test_reserve_failed_leaves_state():
    case = dict(G["cases"][0])
    case["allocated"] = list(range(6))  # 2 of 8 CPUs free, the pod needs 4
    case["needed"] = 4
    cfg, nodes, st, pod = golden_cluster(case)
    nodes.alloc_milli_cpu[:] = 32000  # Fit passes (an amplified node): only the CPU count is short
    o = Oracle(cfg, nodes.copy(), cpu_state=st)
    r = o.schedule(pod)
    assert r["status"][0] == abi.KS_S_RESERVE_FAILED and r["node"][0] == 0
    assert o.read_nodes().req_milli_cpu[0] == nodes.req_milli_cpu[0]
    assert mask_cpus(o.read_cpu_state()[0][0]) == list(range(6))


def test_no_topology_filters_cpu_bind_pods():
    case = dict(G["cases"][0])
    cfg, nodes, st, pod = golden_cluster(case)
    st.topology[0] = -1
    st.allocated[0] = 0
    o = Oracle(cfg, nodes, cpu_state=st)
    reasons, _, _ = o.eval_pod(pod)
    assert reasons[0] == abi.KS_R_NUMA_INVALID_TOPOLOGY
    assert o.schedule(pod)["status"][0] == abi.KS_S_UNSCHEDULABLE


def test_cpu_bind_request_amplified():
    """ratio 2: a 4-CPU bind pod counts 8000m against amplified headroom (plugin.go:357-359)"""
    case = dict(G["cases"][0])
    cfg, nodes, st, pod = golden_cluster(case)
    nodes.numa_cpu_amplification[:] = 2.0
    nodes.alloc_milli_cpu[:] = 16000
    nodes.req_milli_cpu[:] = 9000
    pod.req_milli_cpu[:] = 4000
    o = Oracle(cfg, nodes, cpu_state=st)
    assert o.eval_pod(pod)[0][0] == abi.KS_R_NUMA_AMPLIFIED_CPU  # 16000 - 9000 = 7000 < 8000
    pod.flags[:] = abi.KS_POD_PROD  # the same request without cpu bind fits
    assert o.eval_pod(pod)[0][0] == 0


def test_c3_small_oracle_runs():
    w = synth.c3(n_nodes=200, n_pods=300)
    o = Oracle(w.cfg, w.nodes.copy(), **w.tables())
    r = o.schedule(w.pods)
    bind = (w.pods.flags & abi.KS_POD_CPU_BIND) != 0
    cs = o.fetch_cpusets(w.pods.n)
    placed = (r["status"] == 0) & bind
    assert placed.sum() > 50
    for i in np.nonzero(placed)[0]:
        assert len(mask_cpus(cs[i])) == w.pods.req_milli_cpu[i] // 1000
    assert all(not cs[i].any() for i in np.nonzero(~placed)[0])
