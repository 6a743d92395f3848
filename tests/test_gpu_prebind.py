"""PreBind write-back from a GPU schedule: the resource-status, device-allocated and
reservation-allocated annotations koordinator_amd/prebind.py builds from libkoordgpu.so's results (placements,
GPU / RDMA minors, CPU sets, NUMA allocations, nominated reservations) equal the ones built from the CPU oracle's
results for the same queue, pod by pod, on C3-shaped (devices, cpusets, SingleNUMANode nodes) and C4-shaped
(reservations) clusters."""
import numpy as np
import pytest

from koordinator_amd import abi, prebind, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()  # the in-tree HIP library; no fallback
    return rt


def mask_cpus(words):
    return [w * 64 + b for w, v in enumerate(words) for b in range(64) if (int(v) >> b) & 1]


def gpu_request(w, i, node):
    """CalcDesiredRequestsAndCount (devicehandler_gpu.go:40-64) per instance: (core or None, memory, ratio)"""
    dv, pods = w.devices, w.pods
    tm = next((int(dv.total_memory[k, node]) for k in range(abi.KS_MAX_GPUS)
               if dv.total_core[k, node] or dv.total_memory[k, node] or dv.total_ratio[k, node]), 0)
    core = int(pods.gpu_core[i]) if pods.flags[i] & abi.KS_POD_GPU_CORE else None
    if pods.gpu_memory[i] > 0:
        mem = int(pods.gpu_memory[i])
        ratio = int(float(mem) / float(tm) * 100) if tm else 0
    else:
        ratio = int(pods.gpu_memory_ratio[i])
        mem = ratio * tm // 100
    if ratio > 100 and ratio % 100 == 0:
        d = ratio // 100
        return (core or 0) // d, mem // d, ratio // d
    return core, mem, ratio


def annotations(w, res, cpus, numa):
    out = []
    for i in range(w.pods.n):
        if res["status"][i] != abi.KS_S_SCHEDULED:
            out.append(None)
            continue
        node = int(res["node"][i])
        r = {"gpu_minors": int(res["gpu_minors"][i]), "rdma_minors": int(res["rdma_minors"][i])}
        gr = gpu_request(w, i, node) if r["gpu_minors"] else None
        rd = int(w.pods.rdma[i])
        rdma = rd // (rd // 100) if rd > 100 and rd % 100 == 0 else rd
        nn = [(k, int(numa[i, k, 0]), int(numa[i, k, 1])) for k in range(abi.KS_MAX_NUMA) if numa[i, k].any()]
        rsv = int(res["reservation"][i])
        out.append(prebind.prebind_annotations(r, cpus=mask_cpus(cpus[i]) if cpus is not None else (), numa_nodes=nn,
                                               gpu_request=gr, rdma_request=rdma,
                                               reservation=(f"rsv-{rsv}", f"uid-{rsv}") if rsv >= 0 else None))
    return out


@pytest.mark.parametrize("wl", ["c3", "c4"])
def test_prebind_annotations_match_oracle(runtime, oracle_lib, wl):
    w = synth.c3(seed=81, n_nodes=300, n_pods=500) if wl == "c3" else synth.c4(n_nodes=800, n_reservations=2000, n_pods=500)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), nthreads=8, **w.tables())
    got, want = ev.schedule(w.pods), orc.schedule(w.pods)
    n = w.pods.n
    zeros = np.zeros((n, abi.KS_MAX_NUMA, 2), np.int64)
    if w.cpus is not None:
        ag = annotations(w, got, ev.fetch_cpusets(n), ev.fetch_numa_alloc(n))
        ao = annotations(w, want, orc.fetch_cpusets(n), orc.fetch_numa_alloc(n))
    else:
        ag = annotations(w, got, None, zeros)
        ao = annotations(w, want, None, zeros)
    bad = [i for i in range(n) if ag[i] != ao[i]]
    assert not bad, f"{wl}: annotations differ for pods {bad[:5]}: {ag[bad[0]]} vs {ao[bad[0]]}"
    placed = [ag[i] for i in range(n) if got["status"][i] == abi.KS_S_SCHEDULED]
    assert len(placed) > n // 2
    if wl == "c3":
        assert any(prebind.ANNOTATION_DEVICE_ALLOCATED in a for a in placed)
        assert any(prebind.ANNOTATION_RESOURCE_STATUS in a for a in placed)
    else:
        assert any(prebind.ANNOTATION_RESERVATION_ALLOCATED in a for a in placed)
    ev.close()
    orc.close()
