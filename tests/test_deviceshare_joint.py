"""DeviceShare RDMA devices and joint GPU + RDMA allocation (device_allocator.go:94-462,
numa_topology.go:98-240): the C oracle against the reference's TestAutopilotAllocator table
(tests/golden/deviceshare_joint.json) and hand-derived SamePCIe / RDMA-only cases."""
import numpy as np
import pytest

from dev_util import J, dev_default, dev_zero_weights, joint_devices, joint_pod, minors, plain_nodes
from koordinator_amd import abi
from oracle.oracle import Oracle

CASES = J["cases"]


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_autopilot_allocator_table(c):
    o = Oracle(dev_zero_weights(), plain_nodes(1), devices=joint_devices(c))
    res = o.schedule(joint_pod(c["gpu_wanted"]))
    assert res["status"][0] == 0 and res["node"][0] == 0
    assert minors(res["gpu_minors"][0]) == c["want_gpu"]
    assert minors(res["rdma_minors"][0]) == c["want_rdma"]
    # Reserve adds the request per instance (100 core / 100 ratio per GPU, 1 rdma per device)
    uc, um, ur, urd = o.read_devices()
    before = joint_devices(c)
    for k in c["want_gpu"]:
        assert uc[k, 0] - before.used_core[k, 0] == 100 and ur[k, 0] - before.used_ratio[k, 0] == 100
    for m in c["want_rdma"]:
        assert urd[m, 0] - before.used_rdma[m, 0] == 1


def _case(name):
    return next(c for c in CASES if c["name"] == name)


def test_same_pcie_scope():
    # SamePCIe with 3 GPUs: allocateByTopology ends on the NUMA-node group (GPUs 0,1,2 on switches 0,1);
    # the RDMA count is |switches| = 2 (RDMA 1, 2): the switch sets agree, validateJointAllocation passes
    c = _case("allocate 3 GPU and 2 VF")
    o = Oracle(dev_zero_weights(), plain_nodes(1), devices=joint_devices(c))
    res = o.schedule(joint_pod(3, joint=abi.KS_JOINT_GPU_RDMA_SAME_PCIE))
    assert minors(res["gpu_minors"][0]) == [0, 1, 2] and minors(res["rdma_minors"][0]) == [1, 2]
    # no RDMA left on switch 1 (RDMA 2 fully used): SamePCIe with 2 GPUs still finds switch 0
    d = joint_devices(c)
    d.used_rdma[2] = 100
    o = Oracle(dev_zero_weights(), plain_nodes(1), devices=d)
    res = o.schedule(joint_pod(2, joint=abi.KS_JOINT_GPU_RDMA_SAME_PCIE))
    assert minors(res["gpu_minors"][0]) == [0, 1] and minors(res["rdma_minors"][0]) == [1]
    # every RDMA device full: the joint allocation fails; best effort falls back to ... nothing either
    d = joint_devices(c)
    d.used_rdma[1:5] = 100
    o = Oracle(dev_zero_weights(), plain_nodes(1), devices=d)
    reasons, _, _ = o.eval_pod(joint_pod(1, joint=abi.KS_JOINT_GPU_RDMA_SAME_PCIE))
    assert reasons.tolist() == [abi.KS_R_DEV_JOINT]
    reasons, _, _ = o.eval_pod(joint_pod(1))
    assert reasons.tolist() == [abi.KS_R_DEV_INSUFFICIENT]


def test_same_pcie_violation():
    # GPUs free only on switch 0 (one) and switch 2 (one), RDMA free only on switch 1 and 3: no switch has
    # both, each NUMA group has 1 GPU < 2, the whole node allocates GPUs 1, 4 and RDMA 2, 4 (preferred
    # switches first) -> the switch sets differ -> "Device Joint-Allocate rules violation"
    c = _case("allocate 3 GPU and 2 VF")
    d = joint_devices(c)
    for k in (0, 2, 3, 5, 6, 7):
        d.used_core[k], d.used_memory[k], d.used_ratio[k] = 100, J["gpu"]["memory"], 100
    d.used_rdma[1] = 100
    d.used_rdma[3] = 100
    o = Oracle(dev_zero_weights(), plain_nodes(1), devices=d)
    reasons, _, _ = o.eval_pod(joint_pod(2, joint=abi.KS_JOINT_GPU_RDMA_SAME_PCIE))
    assert reasons.tolist() == [abi.KS_R_DEV_JOINT]
    res = o.schedule(joint_pod(2))  # best effort: the whole-node joint result stands
    assert minors(res["gpu_minors"][0]) == [1, 4] and minors(res["rdma_minors"][0]) == [2, 4]


def test_rdma_only_and_scores():
    c = _case("allocate 1 GPU and 1 VF")
    d = joint_devices(c, n=3)
    d.used_rdma[1:5, 1] = 40          # node 1: RDMA 40 % used
    d.total_rdma[:, 2] = 0            # node 2: no RDMA
    o = Oracle(dev_default(), plain_nodes(3), devices=d)
    reasons, scores, _ = o.eval_pod(joint_pod(0, rdma=50))
    assert reasons.tolist() == [0, 0, abi.KS_R_DEV_NO_RDMA]
    # scoreNode over rdma: node 0 (400 - 400 + 50) -> (400-50)*100/400 = 87; node 1 (400 - 240 + 50) -> 47;
    # normalized by the max 87
    assert scores[:2, abi.KS_SCORE_DEVICESHARE].tolist() == [100, 100 * 47 // 87]
    # multi-device RDMA request: 200 -> two whole devices, per-device score desc, minor asc
    res = o.schedule(joint_pod(0, rdma=200))
    assert res["node"][0] == 0 and minors(res["rdma_minors"][0]) == [1, 2]
    # the GPU + RDMA score is the sum of the per-type scoreNode values (can exceed 100 before normalize)
    reasons, scores, _ = o.eval_pod(joint_pod(1))
    assert reasons.tolist()[:2] == [0, 0]


def test_joint_without_rdma_request():
    """A [gpu, rdma] joint pod that requests no RDMA: jointAllocate still takes an RDMA device next to the GPUs, with a
    nil request (device_allocator.go:308-330): any device with free resources fits, none is used up, none scores the
    node; no switch is `preferred` (newDeviceTopologyGuide splits free devices only for requested types)."""
    c = _case("allocate 3 GPU and 2 VF")
    o = Oracle(dev_zero_weights(), plain_nodes(1), devices=joint_devices(c))
    res = o.schedule(joint_pod(2, rdma=0))
    assert minors(res["gpu_minors"][0]) == [0, 1] and minors(res["rdma_minors"][0]) == [1]
    _, _, _, urd = o.read_devices()
    assert np.array_equal(urd, joint_devices(c).used_rdma)  # nothing added to the RDMA devices
    # RDMA 1 (switch 0) fully used: switch 0 cannot complete the joint allocation, switch 1 does
    d = joint_devices(c)
    d.used_rdma[1] = 100
    o = Oracle(dev_zero_weights(), plain_nodes(1), devices=d)
    res = o.schedule(joint_pod(2, rdma=0))
    assert minors(res["gpu_minors"][0]) == [2, 3] and minors(res["rdma_minors"][0]) == [2]
    # every RDMA device full: best effort falls back to the GPUs alone (no RDMA type in the request); SamePCIe fails
    d = joint_devices(c)
    d.used_rdma[1:5] = 100
    o = Oracle(dev_zero_weights(), plain_nodes(1), devices=d)
    res = o.schedule(joint_pod(2, rdma=0))
    assert res["status"][0] == 0 and minors(res["gpu_minors"][0]) == [0, 1] and res["rdma_minors"][0] == 0
    reasons, _, _ = o.eval_pod(joint_pod(2, rdma=0, joint=abi.KS_JOINT_GPU_RDMA_SAME_PCIE))
    assert reasons.tolist() == [abi.KS_R_DEV_JOINT]
    # a node without RDMA devices is no KS_R_DEV_NO_RDMA for it (the pod requests none)
    d = joint_devices(c, n=2)
    d.total_rdma[:, 1] = 0
    o = Oracle(dev_default(), plain_nodes(2), devices=d)
    reasons, _, _ = o.eval_pod(joint_pod(1, rdma=0))
    assert reasons.tolist() == [0, 0]
