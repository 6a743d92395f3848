"""The production RCCL exchange on one GPU: a one-rank communicator (ks_shard_init(1, 0, id, V) with V virtual shards)
sends every pass's candidate slots through ncclAllGather and the normalization maxima through ncclAllReduce(max) --
the calls the loopback transport stands in for -- and the placements / post-commit state must equal the CPU oracle's.
Afterwards every context is destroyed (ncclCommDestroy) and the process exits normally, so the communicator's
teardown runs against the process-wide CU-masked streams' atexit release (koordgpu.hip release_pipe_streams).

Run as its own process by tests/test_gpu_rccl.py (exit status 0 = every case matched and teardown was clean)."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

from helpers import assert_same_results, assert_same_state, profile  # noqa: E402
from koordinator_amd import runtime, synth  # noqa: E402
from oracle import oracle  # noqa: E402


def case(label, cfg, w_nodes, pods, vshards, pipeline, tables):
    uid = runtime.shard_unique_id()
    ev = runtime.Evaluator(cfg, w_nodes.copy(), **{k: v.copy() for k, v in tables.items()})
    t0 = time.time()
    try:
        ev.set_pipeline(pipeline)
        ev.shard(1, 0, uid, vshards)
        got = ev.schedule(pods)
        st = ev.stats()
        state = ev.read_nodes()
        dev = ev.read_devices() if "devices" in tables else None
        cps = ev.fetch_cpusets(pods.n) if "cpu_state" in tables else None
        quota = ev.read_quota_used() if "quotas" in tables else None
    finally:
        ev.close()  # ncclCommDestroy
    orc = oracle.Oracle(cfg, w_nodes.copy(), nthreads=8, **{k: v.copy() for k, v in tables.items()})
    try:
        want = orc.schedule(pods)
        assert_same_results(got, want, label)
        assert_same_state(state, orc.read_nodes(), label)
        if dev is not None:
            for a, b in zip(dev, orc.read_devices()):
                assert np.array_equal(a, b), f"{label}: GPU state differs"
        if cps is not None:
            assert np.array_equal(cps, orc.fetch_cpusets(pods.n)), f"{label}: cpusets differ"
        if quota is not None:
            assert np.array_equal(quota, orc.read_quota_used()), f"{label}: quota used differs"
    finally:
        orc.close()
    print(f"{label}: ok ({int((got['status'] == 0).sum())}/{pods.n} placed, passes {st['passes']}, pipelined "
          f"{st['pipelined']}, {time.time() - t0:.1f} s)", flush=True)
    return st


def main():
    oracle.build()
    w = synth.c5(n_nodes=20_000, n_pods=3000)
    st = case("c5-20k patched, RCCL 1 rank x 2 shards", profile(candidates=3).to_ks_config(), w.nodes, w.pods, 2, 2, {})
    assert st["pipelined"] == 2, st
    st = case("c5-20k unpipelined, RCCL 1 rank x 3 shards", w.cfg, w.nodes, w.pods, 3, 0, {})
    assert st["pipelined"] == 0, st
    w = synth.c2(n_pods=2000)
    case("C2 quotas re-swept pipeline, RCCL 1 rank x 2 shards", w.cfg, w.nodes, w.pods, 2, 1, w.tables())
    w = synth.c3(n_nodes=600, n_pods=700)
    case("C3-small DeviceShare maxima (ncclAllReduce), RCCL 1 rank x 2 shards", w.cfg, w.nodes, w.pods, 2, 0,
         w.tables())
    w = synth.c2_default(n_nodes=1500, n_pods=900)
    case("C2d-small three normalization rows, RCCL 1 rank x 2 shards", w.cfg, w.nodes, w.pods, 2, 0, w.tables())
    print("rccl one-rank: all cases match the oracle", flush=True)


if __name__ == "__main__":
    main()
