"""GPU parity for DeviceShare RDMA devices and joint [gpu, rdma] allocation (SURVEY a26-a28;
device_allocator.go:188-339, numa_topology.go:98-240): the reference's TestAutopilotAllocator table and the
SamePCIe cases through the HIP library, per-node Filter reasons / scores of joint pods, and whole-queue
scheduling on C3-shaped clusters vs the oracle (placements, scores, GPU and RDMA minors, device state)."""
import numpy as np
import pytest

from dev_util import J, dev_default, dev_zero_weights, joint_devices, joint_pod, minors, plain_nodes
from helpers import assert_same_results, assert_same_state
from koordinator_amd import abi, synth
from koordinator_amd.config import DeviceShareArgs

pytestmark = pytest.mark.gpu
CASES = J["cases"]


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_golden_autopilot_allocator(runtime, c):
    ev = runtime.Evaluator(dev_zero_weights(), plain_nodes(1), devices=joint_devices(c))
    res = ev.schedule(joint_pod(c["gpu_wanted"]))
    assert res["status"][0] == 0 and res["node"][0] == 0
    assert minors(res["gpu_minors"][0]) == c["want_gpu"]
    assert minors(res["rdma_minors"][0]) == c["want_rdma"]
    _, _, _, urd = ev.read_devices()
    before = joint_devices(c)
    assert [m for m in range(abi.KS_MAX_RDMA) if urd[m, 0] != before.used_rdma[m, 0]] == c["want_rdma"]
    ev.close()


def _same_pcie_devices():
    c = next(x for x in CASES if x["name"] == "allocate 3 GPU and 2 VF")
    out = []
    out.append(("plain", joint_devices(c)))
    d = joint_devices(c)
    d.used_rdma[2] = 100
    out.append(("rdma2-full", d))
    d = joint_devices(c)
    d.used_rdma[1:5] = 100
    out.append(("rdma-full", d))
    d = joint_devices(c)
    for k in (0, 2, 3, 5, 6, 7):
        d.used_core[k], d.used_memory[k], d.used_ratio[k] = 100, J["gpu"]["memory"], 100
    d.used_rdma[1] = 100
    d.used_rdma[3] = 100
    out.append(("violation", d))
    return out


@pytest.mark.parametrize("gpus", [1, 2, 3, 4])
@pytest.mark.parametrize("joint", [abi.KS_JOINT_GPU_RDMA, abi.KS_JOINT_GPU_RDMA_SAME_PCIE])
@pytest.mark.parametrize("rdma", [1, 0])
def test_same_pcie_cases(runtime, oracle_lib, gpus, joint, rdma):
    """(rdma 0: the joint spec without an RDMA request -- jointAllocate takes RDMA devices with a nil request)"""
    for name, d in _same_pcie_devices():
        for cfg in (dev_zero_weights(), dev_default()):
            pod = joint_pod(gpus, rdma=rdma, joint=joint)
            ev = runtime.Evaluator(cfg, plain_nodes(1), devices=d.copy())
            orc = oracle_lib.Oracle(cfg, plain_nodes(1), devices=d.copy())
            r_g, s_g, _ = ev.eval_pod(pod)
            r_o, s_o, _ = orc.eval_pod(pod)
            assert r_g.tolist() == r_o.tolist(), name
            assert np.array_equal(s_g, s_o), name
            got, want = ev.schedule(pod), orc.schedule(pod)
            for k in ("node", "status", "score", "gpu_minors", "rdma_minors"):
                assert np.array_equal(got[k], want[k]), f"{name}: {k}"
            ev.close()
            orc.close()


def c3_small(seed, n=500, p=700):
    w = synth.c3(seed=seed, n_nodes=n, n_pods=p)
    return w


def check(runtime, oracle_lib, w, label, cfg=None):
    cfg = cfg or w.cfg
    ev = runtime.Evaluator(cfg, w.nodes.copy(), **w.tables())
    got = ev.schedule(w.pods)
    orc = oracle_lib.Oracle(cfg, w.nodes.copy(), nthreads=8, **w.tables())
    want = orc.schedule(w.pods)
    assert_same_results(got, want, label)
    for k in ("gpu_minors", "rdma_minors"):
        assert np.array_equal(got[k], want[k]), f"{label}: {k} differ"
    assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
    for g, o, name in zip(ev.read_devices(), orc.read_devices(), ("core", "memory", "ratio", "rdma")):
        assert np.array_equal(g, o), f"{label}: device used {name} differs"
    assert np.array_equal(ev.fetch_cpusets(w.pods.n), orc.fetch_cpusets(w.pods.n)), label
    ev.close()
    orc.close()
    return got


def test_eval_debug_joint_pods(runtime, oracle_lib):
    w = c3_small(51, n=300, p=400)
    idx = np.nonzero((w.pods.rdma > 0))[0][:40]
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), **w.tables())
    for i in idx:
        one = w.pods.rows([i])
        r_g, s_g, t_g = ev.eval_pod(one)
        r_o, s_o, t_o = orc.eval_pod(one)
        assert np.array_equal(r_g, r_o), f"pod {i}: reasons"
        assert np.array_equal(s_g, s_o), f"pod {i}: scores"
        assert np.array_equal(t_g, t_o), f"pod {i}: totals"
    ev.close()
    orc.close()


@pytest.mark.parametrize("seed,batch,cand", [(52, 64, 32), (53, 1, 1), (54, 17, 4)])
def test_schedule_c3_joint(runtime, oracle_lib, seed, batch, cand):
    w = c3_small(seed)
    w.profile.batch_pods = batch
    w.profile.candidates = cand
    got = check(runtime, oracle_lib, w, f"c3-joint-{seed}")
    joint = w.pods.joint != 0
    assert ((got["rdma_minors"] != 0) & joint).sum() > 20
    assert ((got["rdma_minors"] != 0) & ~joint).sum() > 0  # RDMA-only pods


def test_schedule_tight_rdma_most_allocated(runtime, oracle_lib):
    # few nodes, many joint pods: RDMA devices run out, SamePCIe pods fail with the joint reason
    w = c3_small(55, n=60, p=700)
    w.pods.joint[w.pods.rdma > 0] = abi.KS_JOINT_GPU_RDMA_SAME_PCIE
    w.profile.deviceshare = DeviceShareArgs(strategy="MostAllocated")
    check(runtime, oracle_lib, w, "tight-most")


@pytest.mark.parametrize("seed", [56, 57])
def test_schedule_c3_joint_without_rdma_request(runtime, oracle_lib, seed):
    """C3-shaped queues where a third of the joint pods keep the joint spec without the RDMA request"""
    w = c3_small(seed)
    rng = np.random.Generator(np.random.PCG64(seed))
    jr = (w.pods.joint != 0) & (rng.random(w.pods.n) < 0.35)
    w.pods.rdma[jr] = 0
    got = check(runtime, oracle_lib, w, f"c3-joint-nordma-{seed}")
    assert ((got["rdma_minors"] != 0) & jr).sum() > 5
