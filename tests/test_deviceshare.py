"""DeviceShare (GPU devices): the C oracle against the reference's DeviceShare score
and allocator tables (tests/golden/deviceshare.json)."""
import pytest

from dev_util import G, alloc_devices, dev_only, devices_of, gpu_pod, plain_nodes
from koordinator_amd import abi
from oracle.oracle import Oracle


@pytest.mark.parametrize("c", G["score"], ids=[c["name"] for c in G["score"]])
def test_score_and_normalize(c):
    o = Oracle(dev_only(c["strategy"]), plain_nodes(len(c["nodes"])), devices=devices_of(c["nodes"]))
    reasons, scores, total = o.eval_pod(gpu_pod(c["pod"]["core"], c["pod"]["ratio"]))
    assert reasons.tolist() == [0] * len(c["nodes"])
    assert scores[:, abi.KS_SCORE_DEVICESHARE].tolist() == c["want_normalized"]


@pytest.mark.parametrize("c", G["allocate"], ids=[c["name"] for c in G["allocate"]])
def test_allocate_minor(c):
    o = Oracle(dev_only(c["strategy"]), plain_nodes(1), devices=alloc_devices(c))
    res = o.schedule(gpu_pod(c["pod"]["core"], c["pod"]["ratio"]))
    assert res["node"][0] == 0
    assert [k for k in range(abi.KS_MAX_GPUS) if (int(res["gpu_minors"][0]) >> k) & 1] == c["want_minors"]
    uc, um, ur, _ = o.read_devices()
    k = c["want_minors"][0]
    before = alloc_devices(c)
    assert uc[k, 0] - before.used_core[k, 0] == 50 and ur[k, 0] - before.used_ratio[k, 0] == 50
    assert um[k, 0] - before.used_memory[k, 0] == 4 << 30  # memoryRatioToBytes(50, 8Gi)


def test_no_gpu_and_insufficient():
    nodes = [{"total": [], "used": []}, {"total": [{"core": 100, "memory": 16 << 30, "ratio": 100}],
                                         "used": [{"core": 100, "memory": 16 << 30, "ratio": 100}]}]
    o = Oracle(dev_only(), plain_nodes(2), devices=devices_of(nodes))
    reasons, _, _ = o.eval_pod(gpu_pod(100, 100))
    assert reasons.tolist() == [abi.KS_R_DEV_NO_GPU, abi.KS_R_DEV_INSUFFICIENT]
    # multi-device request: 200 ratio = 2 whole GPUs
    nodes = [{"total": [{"core": 100, "memory": 16 << 30, "ratio": 100}] * 3, "used": [None, {"core": 10, "memory": 0, "ratio": 10}, None]}]
    o = Oracle(dev_only(), plain_nodes(1), devices=devices_of(nodes))
    res = o.schedule(gpu_pod(200, 200))
    assert res["gpu_minors"][0] == 0b101
