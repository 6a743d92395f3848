"""GPU parity of the nranks > 1 sharded path on one GPU (ks_shard_init_loopback).

Two or three contexts in this process are ranks of one node-sharded group.  Each sweeps and selects over its own chunk
range ([rank * V + v] shards), writes its candidate slots at its rank offset of the gather buffer, and receives the
peers' slots by device copies ordered by host barriers (the test transport standing in for ncclAllGather /
ncclAllReduce).  merge_kernel and the replicated commits are the RCCL path's code, so every rank's placements and
post-commit state must equal the oracle's, including pipelined passes with patched lists (the merged list is the one a
single select over every chunk gives, so patching it after the commit is exact).
"""
import numpy as np
import pytest

from helpers import assert_same_results, assert_same_state, profile, stress_nodes, stress_pods
from koordinator_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


def run_ranks(runtime, oracle_lib, cfg, nodes, pods, label, nranks=2, vshards=1, pipeline=0, **tables):
    evs = [runtime.Evaluator(cfg, nodes.copy(), **{k: v.copy() for k, v in tables.items()}) for _ in range(nranks)]
    try:
        for ev in evs:
            ev.set_pipeline(pipeline)
        runtime.shard_loopback(evs, vshards)

        def body(ev):
            got = ev.schedule(pods)
            out = {"got": got, "stats": ev.stats(), "state": ev.read_nodes()}
            if "quotas" in tables:
                out["quota"] = ev.read_quota_used()
            if "reservations" in tables:
                out["rsv"] = ev.read_reservations()
            if "devices" in tables:
                out["dev"] = ev.read_devices()
            if "cpu_state" in tables:
                out["cpusets"] = ev.fetch_cpusets(pods.n)
            return out

        outs = runtime.run_ranks(body, evs)
    finally:
        for ev in evs:
            ev.close()
    orc = oracle_lib.Oracle(cfg, nodes.copy(), nthreads=8, **{k: v.copy() for k, v in tables.items()})
    want = orc.schedule(pods)
    for r, o in enumerate(outs):
        tag = f"{label} rank {r}/{nranks}x{vshards}"
        assert_same_results(o["got"], want, tag)
        assert_same_state(o["state"], orc.read_nodes(), tag)
        if "quota" in o:
            assert np.array_equal(o["quota"], orc.read_quota_used()), f"{tag}: quota used differs"
        if "rsv" in o:
            oa, os_ = orc.read_reservations()
            assert np.array_equal(o["rsv"][0], oa) and np.array_equal(o["rsv"][1], os_), f"{tag}: reservations differ"
        if "dev" in o:
            for a, b in zip(o["dev"], orc.read_devices()):
                assert np.array_equal(a, b), f"{tag}: GPU state differs"
        if "cpusets" in o:
            assert np.array_equal(o["cpusets"], orc.fetch_cpusets(pods.n)), f"{tag}: cpusets differ"
        # every rank ran the same passes (the commits are replicated)
        for k in ("passes", "cut_passes", "rescans", "pipelined"):
            assert o["stats"][k] == outs[0]["stats"][k], f"{tag}: {k} differs between ranks"
    orc.close()
    return outs[0]["stats"]


def test_c5_shape_20k_pipelined_patched(runtime, oracle_lib):
    # the VERDICT's acceptance case: a 20k-node C5-shaped queue, pipelined with patched lists over 2 ranks
    w = synth.c5(n_nodes=20_000, n_pods=3000)
    st = run_ranks(runtime, oracle_lib, profile(candidates=3).to_ks_config(), w.nodes, w.pods, "c5-20k", pipeline=2)
    assert st["pipelined"] == 2


def test_c5_shape_20k_two_virtual_shards_per_rank(runtime, oracle_lib):
    w = synth.c5(n_nodes=20_000, n_pods=2000, seed=5)
    st = run_ranks(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "c5-20k-v2", vshards=2, pipeline=2)
    assert st["pipelined"] == 2


def test_c5_full_100k_nodes_two_ranks_two_vshards(runtime, oracle_lib):
    """the bench's C5 node count (100k) over 2 ranks x 2 virtual shards (4 shards, the N = 4 layout of the bench's
    sharded C5 on one GPU), pipelined with patched lists, 4,096 pods (64 passes)"""
    w = synth.c5(n_pods=4096, seed=11)
    st = run_ranks(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "c5-100k-2x2", vshards=2, pipeline=2)
    assert st["pipelined"] == 2 and st["passes"] >= 64


def test_c5_shape_not_pipelined(runtime, oracle_lib):
    w = synth.c5(n_nodes=20_000, n_pods=1500, seed=9)
    st = run_ranks(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "c5-20k-serial", pipeline=0)
    assert st["pipelined"] == 0


def test_c2_with_quotas(runtime, oracle_lib):
    w = synth.c2(n_pods=3000)
    run_ranks(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "C2", quotas=w.quotas)


def test_c2_with_quotas_pipelined(runtime, oracle_lib):
    w = synth.c2(n_pods=2000)
    st = run_ranks(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "C2-pipe", quotas=w.quotas, pipeline=2)
    assert st["pipelined"] == 2


def test_three_ranks_cut_heavy(runtime, oracle_lib):
    # an odd rank count (uneven chunk ranges) and 2 candidates: many cuts, rescans and bubbles on every rank
    rng = np.random.Generator(np.random.PCG64(23))
    nodes = stress_nodes(2500, rng)
    pods = stress_pods(900, rng)
    for pipe in (0, 2):
        run_ranks(runtime, oracle_lib, profile(candidates=2).to_ks_config(), nodes, pods, f"3ranks-p{pipe}", nranks=3,
                  pipeline=pipe)


def test_reservations_pipelined(runtime, oracle_lib):
    # Reservation (re-swept pipelined passes, not patched)
    w = synth.c4(n_nodes=1500, n_reservations=3500, n_pods=700)
    st = run_ranks(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "C4-small", reservations=w.reservations, pipeline=2)
    assert st["pipelined"] == 1


def test_deviceshare_numa_allreduce(runtime, oracle_lib):
    # DeviceShare's normalization maxima: the loopback max all-reduce across the ranks (ncclAllReduce's stand-in)
    w = synth.c3(n_nodes=600, n_pods=700)
    run_ranks(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "C3-small", **w.tables())


def test_default_profile_plugins(runtime, oracle_lib):
    # TaintToleration / NodeAffinity maxima (three normalization rows exchanged) + BalancedAllocation + ElasticQuota
    w = synth.c2_default(n_nodes=1500, n_pods=1200)
    run_ranks(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "C2d-small", **w.tables())
