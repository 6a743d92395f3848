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


J = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "deviceshare_joint.json")))


def joint_devices(c, n=1):
    """The TestAutopilotAllocator device CR of case c on n identical nodes (ks_device_cols incl. RDMA and
    the PCIe / NUMA topology), with the case's assigned devices as used amounts."""
    t = J["topologies"][c["topology"]]
    gpu = J["gpu"]
    d = DeviceTable(n)
    d.flags[:] = abi.KS_DEV_PRESENT
    for k in range(8):
        d.total_core[k], d.total_memory[k], d.total_ratio[k] = gpu["core"], gpu["memory"], gpu["ratio"]
        d.gpu_pcie[k] = t["gpu_pcie"][k]
    for m, pc in zip(t["rdma_minors"], t["rdma_pcie"]):
        d.total_rdma[m] = J["rdma_total"]
        d.rdma_pcie[m] = pc
    for p, (nu, so) in enumerate(zip(t["pcie_numa"], t["pcie_socket"])):
        d.pcie_numa[p], d.pcie_socket[p] = nu, so
    a = c.get("assigned") or {}
    for k in a.get("gpu", []):
        d.used_core[k], d.used_memory[k], d.used_ratio[k] = gpu["core"], gpu["memory"], gpu["ratio"]
    for m, v in a.get("rdma", {}).items():
        d.used_rdma[int(m)] = v
    return d


def joint_pod(gpus, rdma=1, joint=abi.KS_JOINT_GPU_RDMA):
    p = gpu_pod(100 * gpus, 100 * gpus) if gpus else gpu_pod(0)
    p.rdma[:] = rdma
    p.joint[:] = joint if gpus else abi.KS_JOINT_NONE
    return p


def dev_default():
    """DeviceShareArgs after the v1beta2 defaults: LeastAllocated over gpu-memory-ratio, rdma, fpga (weight 1)"""
    return SchedulerProfile(fit=None, loadaware=None, deviceshare=DeviceShareArgs()).to_ks_config()


def dev_zero_weights():
    """allocator.scorer == nil in TestAutopilotAllocator: every device score is 0"""
    return SchedulerProfile(fit=None, loadaware=None,
                            deviceshare=DeviceShareArgs(resources={GPU_MEMORY_RATIO: 0})).to_ks_config()


def minors(mask, k=8):
    return [i for i in range(k) if (int(mask) >> i) & 1]
