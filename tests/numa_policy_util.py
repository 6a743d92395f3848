"""Builders for the NUMA topology policy cases (tests/golden/numa_policy.json)."""
import json
import os

import numpy as np

from koordinator_amd import abi
from koordinator_amd.cluster import NodeTable, NumaNodes, PodTable
from koordinator_amd.config import CPU, MEMORY, NodeNUMAResourceArgs, SchedulerProfile

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "numa_policy.json")))
GI = 1 << 30
POLICY = {"BestEffort": abi.KS_NUMA_POLICY_BEST_EFFORT, "Restricted": abi.KS_NUMA_POLICY_RESTRICTED,
          "SingleNUMANode": abi.KS_NUMA_POLICY_SINGLE_NUMA_NODE}


def numa_profile(strategy="MostAllocated", numa_strategy="LeastAllocated"):
    return SchedulerProfile(fit=None, loadaware=None,
                            numa=NodeNUMAResourceArgs(strategy=strategy, resources={CPU: 1, MEMORY: 1},
                                                      numa_scoring_strategy=numa_strategy)).to_ks_config()


def score_case(c):
    """the plugin test harness: NUMA resources = node allocatable / count, existing pods allocated on NUMA 0"""
    n = len(c["nodes"])
    nodes = NodeTable(n)
    nn = NumaNodes(n)
    for i, nd in enumerate(c["nodes"]):
        nodes.alloc_milli_cpu[i] = nd["cpu"] * 1000
        nodes.alloc_memory[i] = nd["memory_gi"] * GI
        nodes.allowed_pods[i] = 110
        nodes.numa_flags[i] = POLICY[c["policy"]] << abi.KS_NUMA_POLICY_SHIFT
        k = nd["numa"]
        nn.count[i] = k
        nn.alloc_cpu[i, :k] = nd["cpu"] * 1000 // k
        nn.alloc_memory[i, :k] = nd["memory_gi"] * GI // k
    for e in c["existing"]:
        i = e["node"]
        nodes.req_milli_cpu[i] += e["cpu"] * 1000
        nodes.req_memory[i] += e["memory_gi"] * GI
        nn.used_cpu[i, 0] += e["cpu"] * 1000
        nn.used_memory[i, 0] += e["memory_gi"] * GI
        nn.used_present[i, 0] = 1
    nodes.nonzero_milli_cpu[:] = nodes.req_milli_cpu
    nodes.nonzero_memory[:] = nodes.req_memory
    pod = PodTable(1)
    pod.req_milli_cpu[:] = c["pod"]["cpu"] * 1000
    pod.req_memory[:] = c["pod"]["memory_gi"] * GI
    pod.nonzero_milli_cpu[:] = pod.req_milli_cpu
    pod.nonzero_memory[:] = pod.req_memory
    return nodes, nn, pod


def distribute_case(c):
    """resource_manager_test.go harness: 2 NUMA nodes of 52 CPUs / 128Gi, node allocatable 104 / 256Gi"""
    nodes = NodeTable(1)
    ratio = c["ratio"]
    nodes.alloc_milli_cpu[:] = int(np.ceil(104000 * ratio)) if ratio > 1 else 104000
    nodes.alloc_memory[:] = 256 * GI
    nodes.allowed_pods[:] = 110
    nodes.numa_cpu_amplification[:] = ratio
    nodes.numa_flags[:] = abi.KS_NUMA_POLICY_BEST_EFFORT << abi.KS_NUMA_POLICY_SHIFT
    nn = NumaNodes(1)
    nn.count[:] = 2
    nn.alloc_cpu[0, :2] = 52000
    nn.alloc_memory[0, :2] = 128 * GI
    nn.used_cpu[0, :2] = c["used_cpu_milli"]
    nn.used_present[0, :2] = c["present"]
    nn.cpuset_cpus[0, :2] = c["cpuset"]
    pod = PodTable(1)
    pod.req_milli_cpu[:] = c["pod_cpu_milli"]
    pod.nonzero_milli_cpu[:] = c["pod_cpu_milli"]
    return nodes, nn, pod
