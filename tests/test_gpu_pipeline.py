"""GPU parity of pipelined passes: each pass's sweep runs on a second stream while the previous
pass commits, then the chunks that commit wrote are re-swept before the select (or, for monotone plugin sets, the
select also runs during the commit and the lists are patched from the re-swept chunks, patch_kernel).  The candidate lists are then
exactly those of a sweep after the commit, so placements, statuses, scores, node / quota / reservation state and
even the pass / cut / rescan counts must equal both the oracle's results and the non-pipelined GPU run's.

ks_set_pipeline(2) forces the mode on clusters below the automatic size threshold, so the small, cut-heavy and
odd-shaped cases of test_gpu_parity.py / test_gpu_reservation.py run through it too.
"""
import numpy as np
import pytest

from helpers import assert_same_results, assert_same_state, homogeneous_pods, nested_quotas, profile, stress_nodes, stress_pods
from koordinator_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()  # the in-tree HIP library; no fallback
    return rt


def run_modes(runtime, oracle_lib, cfg, nodes, pods, label, vshards=1, **tables):
    """GPU with the pipeline forced on and off, and the oracle; every result and state compared."""
    out = {}
    for mode in (2, 0):
        ev = runtime.Evaluator(cfg, nodes.copy(), **{k: v.copy() for k, v in tables.items()})
        ev.set_pipeline(mode)
        if vshards > 1:
            ev.shard(1, 0, None, virtual_shards=vshards)
        got = ev.schedule(pods)
        st = ev.stats()
        state = ev.read_nodes()
        extra = {}
        if "quotas" in tables:
            extra["quota"] = ev.read_quota_used()
        if "reservations" in tables:
            extra["rsv"] = ev.read_reservations()
        ev.close()
        out[mode] = (got, st, state, extra)
    orc = oracle_lib.Oracle(cfg, nodes.copy(), nthreads=8, **{k: v.copy() for k, v in tables.items()})
    want = orc.schedule(pods)
    got, st, state, extra = out[2]
    assert st["pipelined"] in (1, 2), f"{label}: the pipelined mode did not run"
    assert out[0][1]["pipelined"] == 0
    assert_same_results(got, want, f"{label} pipelined")
    assert_same_state(state, orc.read_nodes(), f"{label} pipelined")
    assert_same_results(got, out[0][0], f"{label} pipelined vs not")
    if "quota" in extra:
        assert np.array_equal(extra["quota"], orc.read_quota_used()), f"{label}: quota used differs"
    if "rsv" in extra:
        assert np.array_equal(got["reservation"], want["reservation"]), f"{label}: nominated reservations differ"
        oa, os_ = orc.read_reservations()
        assert np.array_equal(extra["rsv"][0], oa) and np.array_equal(extra["rsv"][1], os_), f"{label}: reservations differ"
    # re-swept before the select (mode 1): the same passes, the candidate lists are the non-pipelined ones, only
    # bubbles are added after cuts; patched lists (mode 2, monotone plugin sets) may differ at the bound's ties and
    # leave a pod without a known top (a cut), so only the results are the same
    if st["pipelined"] == 1:
        for k in ("passes", "cut_passes", "rescans"):
            assert st[k] == out[0][1][k], f"{label}: {k} {st[k]} (pipelined) vs {out[0][1][k]}"
    assert st["bubble_passes"] <= st["cut_passes"] + 1, f"{label}: {st['bubble_passes']} bubbles"
    orc.close()
    return got, st


def test_c1_pipelined(runtime, oracle_lib):
    w = synth.c1()
    run_modes(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "C1")


def test_c2_prefix_with_quotas_pipelined(runtime, oracle_lib):
    w = synth.c2(n_pods=2500)
    run_modes(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "C2", quotas=w.quotas)


def test_cuts_and_rescans_make_bubbles(runtime, oracle_lib):
    # identical pods and two candidate chunks: passes are cut often, each cut leaves one bubble pass behind
    rng = np.random.Generator(np.random.PCG64(11))
    nodes = synth.make_nodes(300, rng)
    pods = homogeneous_pods(1500)
    _, st = run_modes(runtime, oracle_lib, profile(candidates=2).to_ks_config(), nodes, pods, "homogeneous")
    assert st["cut_passes"] > 0 and st["bubble_passes"] > 0 and st["rescans"] > 0


@pytest.mark.parametrize("batch,cand", [(1, 1), (7, 2), (33, 5), (64, 64)])
def test_batch_and_candidate_sizes_pipelined(runtime, oracle_lib, batch, cand):
    rng = np.random.Generator(np.random.PCG64(300 + batch * 3 + cand))
    nodes = stress_nodes(1000, rng)
    pods = stress_pods(350, rng)
    run_modes(runtime, oracle_lib, profile(batch_pods=batch, candidates=cand).to_ks_config(), nodes, pods, f"b{batch}k{cand}")


def test_quota_chain_pipelined(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(13))
    nodes = stress_nodes(1500, rng, tight=True)
    pods = stress_pods(900, rng, n_quotas=24)
    quotas = nested_quotas(pods, rng, 24)
    run_modes(runtime, oracle_lib, profile(quota=True, check_parent=True, candidates=3).to_ks_config(), nodes, pods,
              "quota-chain", quotas=quotas)


def test_virtual_shards_pipelined(runtime, oracle_lib):
    # three shards on one GPU: the re-sweep keeps to each shard's chunk range, the merge reads the pass's first pod
    rng = np.random.Generator(np.random.PCG64(17))
    nodes = stress_nodes(2000, rng)
    pods = stress_pods(600, rng)
    run_modes(runtime, oracle_lib, profile(candidates=4).to_ks_config(), nodes, pods, "vshards", vshards=3)


def test_most_allocated_pipelined_not_patched(runtime, oracle_lib):
    # MostAllocated is not monotone (a commit can raise a node's key): the select must follow the re-sweep
    rng = np.random.Generator(np.random.PCG64(19))
    nodes = stress_nodes(900, rng)
    pods = stress_pods(400, rng)
    _, st = run_modes(runtime, oracle_lib, profile(strategy="MostAllocated", candidates=4).to_ks_config(), nodes, pods,
                      "most")
    assert st["pipelined"] == 1


def test_patched_lists_c5_shape(runtime, oracle_lib):
    # 20k nodes of the C5 distribution with few candidates: patched lists lose their top often (cuts) and refill
    w = synth.c5(n_nodes=20_000, n_pods=3000)
    _, st = run_modes(runtime, oracle_lib, profile(candidates=3).to_ks_config(), w.nodes, w.pods, "c5-20k-k3")
    assert st["pipelined"] == 2


def test_reservations_pipelined(runtime, oracle_lib):
    # Reservation (kernel variant FEAT 1): the commit writes reservation rows of the nodes it touched
    w = synth.c4(n_nodes=1500, n_reservations=3500, n_pods=700)
    _, st = run_modes(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "C4-small", reservations=w.reservations)


def test_c5_prefix_automatic_mode(runtime, oracle_lib):
    """100k nodes: the automatic mode pipelines (no ks_set_pipeline call), bit-exact on a 1.5k-pod prefix."""
    w = synth.c5(n_pods=1500)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy())
    got = ev.schedule(w.pods)
    st = ev.stats()
    state = ev.read_nodes()
    ev.close()
    assert st["pipelined"] == 2  # monotone Fit + LoadAware: the select overlaps the commit, lists patched after it
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), nthreads=8)
    assert_same_results(got, orc.schedule(w.pods), "C5 prefix")
    assert_same_state(state, orc.read_nodes(), "C5 prefix")
    orc.close()


def test_c5_16k_pods_automatic_mode(runtime, oracle_lib):
    """100k nodes, 16,384 pods (256 pipelined passes with patched candidate lists, each pass's speculative sweep
    checked against the commit it overlapped): bit-exact placements and node state against the oracle (16 threads,
    ~10 s)."""
    w = synth.c5(n_pods=16_384, seed=77)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy())
    got = ev.schedule(w.pods)
    st = ev.stats()
    state = ev.read_nodes()
    ev.close()
    assert st["pipelined"] == 2 and st["passes"] >= 256
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), nthreads=16)
    assert_same_results(got, orc.schedule(w.pods), "C5 16k")
    assert_same_state(state, orc.read_nodes(), "C5 16k")
    orc.close()


def test_c5_64k_pods_automatic_mode(runtime, oracle_lib):
    """100k nodes, 65,536 pods (1,024 pipelined passes, patched lists): bit-exact placements and node state against
    the 16-thread oracle (~40 s of oracle time) -- four times the 16k sample, 6.6 % of the bench's 1M-pod queue."""
    w = synth.c5(n_pods=65_536, seed=78)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy())
    got = ev.schedule(w.pods)
    st = ev.stats()
    state = ev.read_nodes()
    ev.close()
    assert st["pipelined"] == 2 and st["passes"] >= 1024
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), nthreads=16)
    assert_same_results(got, orc.schedule(w.pods), "C5 64k")
    assert_same_state(state, orc.read_nodes(), "C5 64k")
    orc.close()
