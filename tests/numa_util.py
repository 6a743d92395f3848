"""Builders for the NodeNUMAResource golden cases (tests/golden/numa.json)."""
import json
import os

import numpy as np

from koordinator_amd import abi
from koordinator_amd.cluster import NodeTable, PodTable
from koordinator_amd.config import CPU, MEMORY, NodeNUMAResourceArgs, SchedulerProfile

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "numa.json")))


def nodes_of(specs):
    t = NodeTable(len(specs))
    for i, s in enumerate(specs):
        t.alloc_milli_cpu[i] = s["alloc_milli_cpu"]
        t.alloc_memory[i] = s["alloc_memory"]
        t.req_milli_cpu[i] = s["req_milli_cpu"]
        t.req_memory[i] = s["req_memory"]
        t.nonzero_milli_cpu[i] = s["req_milli_cpu"]
        t.nonzero_memory[i] = s["req_memory"]
        t.numa_cpu_amplification[i] = s["ratio"]
        t.numa_cpuset_cpus[i] = s["cpuset_cpus"]
    t.allowed_pods[:] = 110
    return t


def pod_of(spec):
    p = PodTable(1)
    p.req_milli_cpu[:] = spec["cpu"]
    p.req_memory[:] = spec["memory"]
    p.nonzero_milli_cpu[:] = spec["cpu"] or 100
    p.nonzero_memory[:] = spec["memory"] or 200 << 20
    return p


def numa_only(strategy="LeastAllocated"):
    """a profile with NodeNUMAResource alone (Fit and LoadAware off), as the plugin tests run it"""
    cfg = SchedulerProfile(fit=None, loadaware=None,
                           numa=NodeNUMAResourceArgs(strategy=strategy, resources={CPU: 1, MEMORY: 1})).to_ks_config()
    return cfg
