"""GPU parity for DeviceShare (GPU devices): the golden tables through the HIP library,
and whole-queue scheduling vs the oracle — placements, scores (normalized over the feasible nodes),
allocated minors and the device cache after every commit — alone and with NUMA + Reservation."""
import numpy as np
import pytest

from dev_util import G, alloc_devices, dev_only, devices_of, gpu_pod, plain_nodes
from helpers import assert_same_results, assert_same_state
from koordinator_amd import abi, synth
from koordinator_amd.config import GPU_MEMORY_RATIO, DeviceShareArgs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


@pytest.mark.parametrize("c", G["score"], ids=[c["name"] for c in G["score"]])
def test_golden_score(runtime, c):
    ev = runtime.Evaluator(dev_only(c["strategy"]), plain_nodes(len(c["nodes"])), devices=devices_of(c["nodes"]))
    reasons, scores, _ = ev.eval_pod(gpu_pod(c["pod"]["core"], c["pod"]["ratio"]))
    assert reasons.tolist() == [0] * len(c["nodes"])
    assert scores[:, abi.KS_SCORE_DEVICESHARE].tolist() == c["want_normalized"]
    ev.close()


@pytest.mark.parametrize("c", G["allocate"], ids=[c["name"] for c in G["allocate"]])
def test_golden_allocate(runtime, c):
    ev = runtime.Evaluator(dev_only(c["strategy"]), plain_nodes(1), devices=alloc_devices(c))
    res = ev.schedule(gpu_pod(c["pod"]["core"], c["pod"]["ratio"]))
    assert [k for k in range(abi.KS_MAX_GPUS) if (int(res["gpu_minors"][0]) >> k) & 1] == c["want_minors"]
    ev.close()


def dev_profile(p, strategy="LeastAllocated"):
    p.deviceshare = DeviceShareArgs(strategy=strategy, resources={GPU_MEMORY_RATIO: 1})
    return p


def check(runtime, oracle_lib, p, nodes, pods, devs, rs=None, label=""):
    cfg = p.to_ks_config()
    ev = runtime.Evaluator(cfg, nodes.copy(), reservations=rs.copy() if rs is not None else None, devices=devs.copy())
    got = ev.schedule(pods)
    orc = oracle_lib.Oracle(cfg, nodes.copy(), nthreads=8, reservations=rs.copy() if rs is not None else None,
                            devices=devs.copy())
    want = orc.schedule(pods)
    assert_same_results(got, want, label)
    assert np.array_equal(got["gpu_minors"], want["gpu_minors"]), f"{label}: allocated minors differ"
    assert np.array_equal(got["reservation"], want["reservation"]), label
    assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
    assert np.array_equal(got["rdma_minors"], want["rdma_minors"]), f"{label}: allocated RDMA minors differ"
    for g, w, name in zip(ev.read_devices(), orc.read_devices(), ("core", "memory", "ratio", "rdma")):
        assert np.array_equal(g, w), f"{label}: device used {name} differs"
    st = ev.stats()
    ev.close()
    orc.close()
    return got, st


def cluster(seed, n=600, p=800):
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = synth.make_nodes(n, rng)
    devs = synth.make_devices(nodes, rng)
    pods = synth.gpu_pods(synth.make_pods(p, rng), rng)
    return nodes, pods, devs


def test_eval_debug(runtime, oracle_lib):
    nodes, pods, devs = cluster(41, n=400, p=40)
    for strat in ("LeastAllocated", "MostAllocated"):
        cfg = dev_profile(synth.koord_profile(), strat).to_ks_config()
        ev = runtime.Evaluator(cfg, nodes, devices=devs)
        orc = oracle_lib.Oracle(cfg, nodes, devices=devs)
        for i in range(pods.n):
            one = pods.rows([i])
            r_g, s_g, t_g = ev.eval_pod(one)
            r_o, s_o, t_o = orc.eval_pod(one)
            assert np.array_equal(r_g, r_o), f"pod {i}: reasons"
            assert np.array_equal(s_g, s_o), f"pod {i}: scores"
            assert np.array_equal(t_g, t_o), f"pod {i}: totals"
        ev.close()
        orc.close()


@pytest.mark.parametrize("strategy,batch,cand", [("LeastAllocated", 64, 32), ("MostAllocated", 64, 32),
                                                 ("LeastAllocated", 1, 1), ("LeastAllocated", 17, 2)])
def test_schedule(runtime, oracle_lib, strategy, batch, cand):
    nodes, pods, devs = cluster(42)
    got, st = check(runtime, oracle_lib, dev_profile(synth.koord_profile(batch_pods=batch, candidates=cand), strategy),
                    nodes, pods, devs, label=f"dev-{strategy}-{batch}-{cand}")
    assert (got["gpu_minors"] != 0).sum() > 100


def test_schedule_tight_gpus(runtime, oracle_lib):
    # few GPU nodes: pods run out of devices, forcing Insufficient / cuts on the normalization max
    nodes, pods, devs = cluster(43, n=120, p=700)
    check(runtime, oracle_lib, dev_profile(synth.koord_profile()), nodes, pods, devs, label="tight")


def test_schedule_with_numa_and_reservations(runtime, oracle_lib):
    from test_gpu_numa import numa_nodes, prof_with_numa

    rng = np.random.Generator(np.random.PCG64(44))
    w = synth.c4(n_nodes=800, n_reservations=1800, n_pods=900)
    numa_nodes(w.nodes.n, rng, base=w.nodes)
    devs = synth.make_devices(w.nodes, rng)
    synth.gpu_pods(w.pods, rng)
    p = dev_profile(prof_with_numa(w.profile))
    got, _ = check(runtime, oracle_lib, p, w.nodes, w.pods, devs, w.reservations, "dev+numa+rsv")
    assert (got["reservation"] >= 0).sum() > 50 and (got["gpu_minors"] != 0).sum() > 50


def test_virtual_shards(runtime, oracle_lib):
    nodes, pods, devs = cluster(45, n=900, p=300)
    cfg = dev_profile(synth.koord_profile()).to_ks_config()
    ev = runtime.Evaluator(cfg, nodes.copy(), devices=devs.copy())
    ev.shard(1, 0, None, virtual_shards=3)
    got = ev.schedule(pods)
    orc = oracle_lib.Oracle(cfg, nodes.copy(), nthreads=8, devices=devs.copy())
    want = orc.schedule(pods)
    assert_same_results(got, want, "dev-vshards")
    assert np.array_equal(got["gpu_minors"], want["gpu_minors"])
    ev.close()
    orc.close()
