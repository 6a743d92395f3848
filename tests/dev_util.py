"""Builders for the DeviceShare golden cases (tests/golden/deviceshare.json)."""
import json
import os

from koordinator_amd import abi
from koordinator_amd.cluster import DeviceTable, NodeTable, PodTable
from koordinator_amd.config import GPU_MEMORY_RATIO, DeviceShareArgs, SchedulerProfile

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "deviceshare.json")))["cases"]


def plain_nodes(n):
    t = NodeTable(n)
    t.alloc_milli_cpu[:] = 64000
    t.alloc_memory[:] = 256 << 30
    t.allowed_pods[:] = 110
    return t


def devices_of(nodes_spec):
    d = DeviceTable(len(nodes_spec))
    d.flags[:] = abi.KS_DEV_PRESENT
    for i, ns in enumerate(nodes_spec):
        for k, tot in enumerate(ns["total"]):
            d.total_core[k, i], d.total_memory[k, i], d.total_ratio[k, i] = tot["core"], tot["memory"], tot["ratio"]
            u = ns["used"][k]
            if u:
                d.used_core[k, i], d.used_memory[k, i], d.used_ratio[k, i] = u["core"], u["memory"], u["ratio"]
    return d


def alloc_devices(c):
    d = DeviceTable(1)
    d.flags[:] = abi.KS_DEV_PRESENT
    for k in c["minors"]:
        t = c["total"]
        d.total_core[k, 0], d.total_memory[k, 0], d.total_ratio[k, 0] = t["core"], t["memory"], t["ratio"]
        u = c["used"].get(str(k))
        if u:
            d.used_core[k, 0], d.used_memory[k, 0], d.used_ratio[k, 0] = u["core"], u["memory"], u["ratio"]
    return d


def gpu_pod(core, ratio=0, memory=0):
    p = PodTable(1)
    p.gpu_core[:] = core
    p.gpu_memory_ratio[:] = ratio
    p.gpu_memory[:] = memory
    p.flags[:] = (abi.KS_POD_GPU_CORE if core else 0) | (abi.KS_POD_GPU_MEMORY if memory else 0)
    p.nonzero_milli_cpu[:] = 100
    p.nonzero_memory[:] = 200 << 20
    return p


def dev_only(strategy="LeastAllocated"):
    return SchedulerProfile(fit=None, loadaware=None,
                            deviceshare=DeviceShareArgs(strategy=strategy, resources={GPU_MEMORY_RATIO: 1})).to_ks_config()
