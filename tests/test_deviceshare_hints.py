"""DeviceShare as a topology-manager hint provider (deviceshare/topology_hint.go:33-227): the C oracle's
generateTopologyHints and NUMA-restricted Allocate against the reference's TestPlugin_GetPodTopologyHints /
TestPlugin_Allocate tables (tests/golden/deviceshare_hints.json)."""
import json
import os

import pytest

from dev_util import J, dev_default, gpu_pod, plain_nodes
from koordinator_amd import abi
from koordinator_amd.cluster import DeviceTable
from oracle.oracle import Oracle

H = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "deviceshare_hints.json")))


def fake_device_cr(assigned=None):
    t = J["topologies"][H["topology"]]
    gpu = J["gpu"]
    d = DeviceTable(1)
    d.flags[:] = abi.KS_DEV_PRESENT
    for k in range(8):
        d.total_core[k], d.total_memory[k], d.total_ratio[k] = gpu["core"], gpu["memory"], gpu["ratio"]
        d.gpu_pcie[k] = t["gpu_pcie"][k]
    for m, pc in zip(t["rdma_minors"], t["rdma_pcie"]):
        d.total_rdma[m] = J["rdma_total"]
        d.rdma_pcie[m] = pc
    for p, (nu, so) in enumerate(zip(t["pcie_numa"], t["pcie_socket"])):
        d.pcie_numa[p], d.pcie_socket[p] = nu, so
    for k, u in (assigned or {}).items():
        d.used_core[int(k)], d.used_memory[int(k)], d.used_ratio[int(k)] = u["core"], u["memory"], u["ratio"]
    return d


def pod_of(c):
    p = gpu_pod(c.get("gpu_core", 0), c.get("gpu_ratio", 0), c.get("gpu_memory", 0))
    p.rdma[:] = c.get("rdma", 0)
    p.joint[:] = abi.KS_JOINT_GPU_RDMA if c.get("joint") else abi.KS_JOINT_NONE
    return p


def bits(b):
    return sum(1 << i for i in b)


@pytest.mark.parametrize("c", H["cases"], ids=[c["name"] for c in H["cases"]])
def test_topology_hints_table(c):
    o = Oracle(dev_default(), plain_nodes(1), devices=fake_device_cr(c.get("assigned_gpu")))
    lists, hints = o.dev_hints(pod_of(c), 0)
    if "hints" in c:
        assert lists == c["lists"]
        assert hints == [(bits(m), p) for m, p in c["hints"]]
    for m in c.get("allocates_on", []):
        # Allocate(affinity) succeeds exactly when the mask is a hint
        assert bits(m) in [h for h, _ in hints]


def test_no_device_info_is_no_preference():
    d = fake_device_cr()
    d.flags[:] = 0
    o = Oracle(dev_default(), plain_nodes(1), devices=d)
    assert o.dev_hints(pod_of(H["cases"][0]), 0) == (0, [])


def test_no_mask_with_enough_devices_is_no_preference():
    # 16 GPUs wanted: no NUMA mask holds them, minAffinitySize stays nil -> an empty map (no preference)
    c = dict(H["cases"][0], gpu_core=1600, gpu_ratio=1600, rdma=0)
    o = Oracle(dev_default(), plain_nodes(1), devices=fake_device_cr())
    assert o.dev_hints(pod_of(c), 0) == (0, [])


def test_enough_devices_but_none_free_gives_empty_lists():
    # every GPU fully used: the masks pass the device count but no allocation succeeds -> empty lists
    used = {str(k): {"core": 100, "memory": 0, "ratio": 100} for k in range(8)}
    o = Oracle(dev_default(), plain_nodes(1), devices=fake_device_cr(used))
    assert o.dev_hints(pod_of(dict(H["cases"][0], rdma=0)), 0) == (3, [])
