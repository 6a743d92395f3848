"""Node sharding.

CPU: two gloo ranks each select over their node-chunk shard, exchange the lists with an allgather
and merge; the merged list must equal one select over every chunk (the exactness argument the
merge kernel relies on), for random, tie-heavy and sparse score rows.
GPU: virtual shards on one MI355X (the same select -> slot -> merge path the RCCL allgather feeds)
must give placements identical to one shard and to the CPU oracle.
"""
import os

import numpy as np
import pytest

from shard_ref import merge_lists, select_chunks, shard_ranges


def _rows(seed, nrows=48, nchunks=157):
    rng = np.random.default_rng(seed)
    rows = []
    for r in range(nrows):
        kind = r % 4
        if kind == 0:
            h = rng.integers(0, 300, nchunks)
        elif kind == 1:
            h = rng.choice(np.array([0, 7, 8, 9]), nchunks)  # heavy ties
        elif kind == 2:
            h = np.where(rng.random(nchunks) < 0.05, rng.integers(1, 50, nchunks), 0)  # sparse
        else:
            h = np.full(nchunks, 5)
        rows.append(h)
    return rows


def _worker(rank, world, port, out_path):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bad = 0
    for K in (1, 4, 32, 64):
        for h in _rows(K):
            lo, hi = shard_ranges(len(h), world)[rank]
            mine, total, _ = select_chunks(h[lo:hi], K, c0=lo)
            gathered = [None] * world
            dist.all_gather_object(gathered, (mine, total))
            merged, ex_m = merge_lists([g[0] for g in gathered], [g[1] for g in gathered], dict(enumerate(h)), K)
            want, _, ex_w = select_chunks(h, K)
            bad += int(merged != want or ex_m != ex_w)
    with open(f"{out_path}.{rank}", "w") as f:
        f.write(str(bad))
    dist.destroy_process_group()


def test_shard_merge_equals_single_select_gloo_world2(tmp_path):
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "bad")
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    for r in range(2):
        assert open(f"{out}.{r}").read() == "0"


@pytest.mark.parametrize("world", [2, 3, 8])
def test_shard_merge_in_process(world):
    for K in (1, 3, 32):
        for h in _rows(100 + K, nrows=24, nchunks=61):
            lists, totals = [], []
            for lo, hi in shard_ranges(len(h), world):
                m, t, _ = select_chunks(h[lo:hi], K, c0=lo)
                lists.append(m)
                totals.append(t)
            assert merge_lists(lists, totals, dict(enumerate(h)), K)[0] == select_chunks(h, K)[0]


@pytest.mark.gpu
@pytest.mark.parametrize("vshards,cands", [(2, 0), (3, 0), (8, 0), (5, 4), (16, 1)])
def test_gpu_virtual_shards_match_single_and_oracle(vshards, cands):
    from helpers import assert_same_results, assert_same_state
    from koordinator_amd import runtime, synth
    from oracle.oracle import Oracle

    w = synth.c2(n_nodes=3000, n_pods=1200, n_quotas=16, candidates=cands)
    cfg = w.cfg
    one = runtime.Evaluator(cfg, w.nodes.copy(), w.quotas.copy())
    r1 = one.schedule(w.pods)
    ev = runtime.Evaluator(cfg, w.nodes.copy(), w.quotas.copy())
    ev.shard(1, 0, None, vshards)
    rs = ev.schedule(w.pods)
    assert_same_results(rs, r1, f"vshards={vshards}")
    orc = Oracle(cfg, w.nodes.copy(), w.quotas.copy(), nthreads=4)
    want = orc.schedule(w.pods)
    assert_same_results(rs, want, f"vshards={vshards} vs oracle")
    assert_same_state(ev.read_nodes(), orc.read_nodes(), "state")
    for e in (one, ev):
        e.close()
    orc.close()
