"""PreBind write-back (koordinator_amd/prebind.py) against the annotation strings the reference's own PreBind tests
expect, and Kubernetes Quantity / CPUSet string forms.  CPU only."""
import json

import numpy as np
import pytest

from koordinator_amd import prebind as pb

GI = 1 << 30


def test_device_allocated_matches_reference_prebind_case():
    # deviceshare/plugin_test.go:3476-3517 ("pre-bind successfully"): two GPUs, minors 0 and 1, each with
    # gpu-core 100, gpu-memory-ratio 100, gpu-memory 16Gi
    want = ('{"gpu":[{"minor":0,"resources":{"koordinator.sh/gpu-core":"100","koordinator.sh/gpu-memory":"16Gi",'
            '"koordinator.sh/gpu-memory-ratio":"100"}},{"minor":1,"resources":{"koordinator.sh/gpu-core":"100",'
            '"koordinator.sh/gpu-memory":"16Gi","koordinator.sh/gpu-memory-ratio":"100"}}]}')
    assert pb.device_allocated(gpu_minors=0b11, gpu_core=100, gpu_memory=16 * GI, gpu_memory_ratio=100) == want


def test_device_allocated_multi_gpu_core_order_and_format():
    # devicehandler_gpu.go:55-63: a multi-GPU request rebuilds the per-instance list with gpu-core even when the
    # pod asked for none (0); a single GPU keeps the pod's own list (no gpu-core) and the pod's gpu-memory format
    multi = json.loads(pb.device_allocated(gpu_minors=0b110, gpu_core=None, gpu_memory=8 * GI, gpu_memory_ratio=100))
    assert [a["minor"] for a in multi["gpu"]] == [1, 2]
    assert multi["gpu"][0]["resources"] == {"koordinator.sh/gpu-core": "0", "koordinator.sh/gpu-memory": "8Gi",
                                            "koordinator.sh/gpu-memory-ratio": "100"}
    one = json.loads(pb.device_allocated(gpu_minors=0b1000, gpu_core=None, gpu_memory=8_000_000_000,
                                         gpu_memory_ratio=9, gpu_memory_format="DecimalSI"))
    assert one["gpu"][0]["resources"] == {"koordinator.sh/gpu-memory": "8G", "koordinator.sh/gpu-memory-ratio": "9"}
    # sortDeviceResourcesByMinor's order (score desc, then minor) when the caller has it
    o = json.loads(pb.device_allocated(gpu_minors=0b1011, gpu_core=50, gpu_memory=4 * GI, gpu_memory_ratio=50,
                                       gpu_order=[3, 0, 1], rdma_minors=0b101, rdma=100, rdma_order=[2, 0]))
    assert [a["minor"] for a in o["gpu"]] == [3, 0, 1] and [a["minor"] for a in o["rdma"]] == [2, 0]
    with pytest.raises(ValueError):
        pb.device_allocated(gpu_minors=0b11, gpu_core=1, gpu_memory=GI, gpu_memory_ratio=1, gpu_order=[0, 2])


def test_resource_status_matches_reference_prebind_case():
    # nodenumaresource/plugin_test.go:1281-1326: allocation CPUSet {0,1,2,3} -> ResourceStatus{CPUSet: "0-3"}
    got = pb.resource_status(cpus=[0, 1, 2, 3])
    assert got == '{"cpuset":"0-3"}'
    assert json.loads(got) == {"cpuset": "0-3"}


def test_reservation_allocated_matches_reference():
    # reservation/plugin_test.go:2042
    assert pb.reservation_allocated("assumed-reservation", "1234567890") == \
        '{"name":"assumed-reservation","uid":"1234567890"}'


def test_quantity_strings():
    # canonical Quantity.String forms (k8s.io/apimachinery resource.Quantity)
    q = pb.quantity_string
    assert q(4000, milli=True) == "4"
    assert q(2500, milli=True) == "2500m"
    assert q(500, milli=True) == "500m"
    assert q(1000) == "1k"
    assert q(1500) == "1500"
    assert q(100) == "100"
    assert q(0) == "0"
    assert q(16 * GI, "BinarySI") == "16Gi"
    assert q(3 * GI // 2, "BinarySI") == "1536Mi"
    assert q(1536, "BinarySI") == "1536"
    assert q(512, "BinarySI") == "512"
    assert q(1 << 20, "BinarySI") == "1Mi"
    # 10^6 = 2^6 * 15625: no power of 1024 divides it, so BinarySI prints the plain integer
    assert q(1000 * 1000, "BinarySI") == "1000000"


def test_cpuset_string():
    assert pb.cpuset_string([3, 1, 2, 0, 8, 10, 9, 12]) == "0-3,8-10,12"
    assert pb.cpuset_string([]) == ""
    assert pb.cpuset_string([5]) == "5"


def test_resource_status_with_numa_nodes():
    got = pb.resource_status(cpus=[0, 1, 2, 3], numa_nodes=[(0, 4000, 8 * GI), (1, 0, 0)])
    assert got == '{"cpuset":"0-3","numaNodeResources":[{"node":0,"resources":{"cpu":"4","memory":"8Gi"}}]}'


def test_prebind_annotations_from_result_rows():
    res = np.zeros(1, dtype=[("node", "i4"), ("gpu_minors", "u4"), ("rdma_minors", "u4")])[0]
    res["gpu_minors"], res["rdma_minors"] = 0b100, 0b10
    ann = pb.prebind_annotations(res, gpu_request=(None, 8 * GI, 50), rdma_request=1,
                                 reservation=("r-1", "uid-1"))
    assert json.loads(ann[pb.ANNOTATION_DEVICE_ALLOCATED]) == {
        "gpu": [{"minor": 2, "resources": {"koordinator.sh/gpu-memory": "8Gi", "koordinator.sh/gpu-memory-ratio": "50"}}],
        "rdma": [{"minor": 1, "resources": {"koordinator.sh/rdma": "1"}}]}
    assert ann[pb.ANNOTATION_RESERVATION_ALLOCATED] == '{"name":"r-1","uid":"uid-1"}'
    assert pb.ANNOTATION_RESOURCE_STATUS not in ann


# Test_appendResourceSpecIfMissed (nodenumaresource/plugin_test.go:1537-1645): (pod resource-spec, node CPU bind
# policy label, PreFilter state (required, preferred)) -> the pod's resource-spec afterwards
APPEND_RESOURCE_SPEC_CASES = [
    ("declared preferred cpu bind policy", {"preferredCPUBindPolicy": "SpreadByPCPUs"}, "", ("", "SpreadByPCPUs"),
     {"preferredCPUBindPolicy": "SpreadByPCPUs"}),
    ("declared default preferred cpu bind policy", {"preferredCPUBindPolicy": "Default"}, "", ("", "SpreadByPCPUs"),
     {"preferredCPUBindPolicy": "SpreadByPCPUs"}),
    ("declared required cpu bind policy", {"requiredCPUBindPolicy": "SpreadByPCPUs"}, "",
     ("SpreadByPCPUs", "SpreadByPCPUs"), {"requiredCPUBindPolicy": "SpreadByPCPUs"}),
    ("declared required and default preferred", {"requiredCPUBindPolicy": "SpreadByPCPUs", "preferredCPUBindPolicy": "Default"},
     "", ("SpreadByPCPUs", "SpreadByPCPUs"),
     {"requiredCPUBindPolicy": "SpreadByPCPUs", "preferredCPUBindPolicy": "SpreadByPCPUs"}),
    ("declared required, default preferred and exclusive policy",
     {"requiredCPUBindPolicy": "SpreadByPCPUs", "preferredCPUBindPolicy": "Default", "preferredCPUExclusivePolicy": "PCPULevel"},
     "", ("SpreadByPCPUs", "SpreadByPCPUs"),
     {"requiredCPUBindPolicy": "SpreadByPCPUs", "preferredCPUBindPolicy": "SpreadByPCPUs",
      "preferredCPUExclusivePolicy": "PCPULevel"}),
    ("LS Pod assigned on node with FullPCPUsOnly", None, "FullPCPUsOnly", ("", ""), {"requiredCPUBindPolicy": "FullPCPUs"}),
]


@pytest.mark.parametrize("name,spec,node_policy,state,want", APPEND_RESOURCE_SPEC_CASES, ids=[c[0] for c in APPEND_RESOURCE_SPEC_CASES])
def test_append_resource_spec_if_missed(name, spec, node_policy, state, want):
    got = pb.resource_spec_writeback(spec, state[0], state[1], node_policy)
    final = got if got is not None else (spec or {})
    assert final == want


def test_prebind_writes_resource_spec_for_defaulted_preferred_policy():
    # TestPlugin_PreBindWithCPUBindPolicyNone (plugin_test.go:1328-1381): a pod without a resource-spec whose
    # PreFilter state carries the default FullPCPUs preferred policy gets {"preferredCPUBindPolicy":"FullPCPUs"}
    # next to its resource-status {"cpuset":"0-3"}
    r = {"gpu_minors": 0, "rdma_minors": 0}
    out = pb.prebind_annotations(r, cpus=[0, 1, 2, 3], cpu_bind=(None, "", "FullPCPUs", ""))
    assert out[pb.ANNOTATION_RESOURCE_SPEC] == '{"preferredCPUBindPolicy":"FullPCPUs"}'
    assert out[pb.ANNOTATION_RESOURCE_STATUS] == '{"cpuset":"0-3"}'
    # a pod that already states the policy: no write-back (only the status)
    out = pb.prebind_annotations(r, cpus=[0, 1], cpu_bind=({"requiredCPUBindPolicy": "FullPCPUs"}, "FullPCPUs", "FullPCPUs", ""))
    assert pb.ANNOTATION_RESOURCE_SPEC not in out
    # a node label overrides the preferred policy and makes it required
    out = pb.prebind_annotations(r, cpus=[0, 1], cpu_bind=(None, "", "FullPCPUs", "SpreadByPCPUs"))
    assert out[pb.ANNOTATION_RESOURCE_SPEC] == '{"requiredCPUBindPolicy":"SpreadByPCPUs"}'
