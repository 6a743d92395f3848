"""GPU parity under forced launch shapes and commit-kernel choices.

The sweep's grid-stride loop over (chunk, pod group) items must give the same candidates for any
pods-per-wave and block count, and both commit kernels (the monotone one, ks_mono.h, the default for Fit +
LoadAware without ElasticQuota; the general one, the default with ElasticQuota; KS_COMMIT_GENERAL=1 forces the
general one, =2 the monotone one with ElasticQuota too) must commit the same placements.  The overrides are read once per process, so each
shape runs in a child process: C2-shaped (ElasticQuota), C4-shaped (Reservation) and C3-shaped
(DeviceShare with hints, cpuset pods, NUMA-policy nodes: the phase-1 DeviceShare cache has its own
pods-per-wave output mapping) clusters, checked bit-exact against the CPU oracle.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os
import numpy as np
from koordinator_amd import runtime, synth
from oracle.oracle import Oracle

which = os.environ["SHAPE_WORKLOADS"].split(",")
make = {"c2": lambda: synth.c2(n_nodes=900, n_pods=384),
        "c1": lambda: synth.c1(n_pods=384),
        "c4": lambda: synth.c4(n_nodes=700, n_reservations=1500, n_pods=256),
        "c3": lambda: synth.c3(n_nodes=400, n_pods=320)}
for name in which:
    w = make[name]()
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    got = ev.schedule(w.pods)
    orc = Oracle(w.cfg, w.nodes.copy(), nthreads=4, **w.tables())
    want = orc.schedule(w.pods)
    for k in ("node", "status", "score", "reservation", "gpu_minors", "rdma_minors"):
        assert np.array_equal(got[k], want[k]), (w.name, k)
    gs, ws = ev.read_nodes().as_dict(), orc.read_nodes().as_dict()
    for k in ws:
        assert np.array_equal(gs[k], ws[k]), (w.name, "node state", k)
    if w.cpus is not None:
        assert np.array_equal(ev.fetch_cpusets(w.pods.n), orc.fetch_cpusets(w.pods.n)), (w.name, "cpusets")
    if w.devices is not None:
        for a, b in zip(ev.read_devices(), orc.read_devices()):
            assert np.array_equal(a, b), (w.name, "devices")
    ev.close()
    orc.close()
print("SHAPE OK")
"""


def _run(env_extra, workloads):
    env = dict(os.environ, SHAPE_WORKLOADS=",".join(workloads), **env_extra)
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "SHAPE OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


@pytest.mark.parametrize("ppw,cap", [(1, 8), (3, 24), (4, 16), (64, 8)])
def test_sweep_shape_invariant(ppw, cap):
    _run({"KS_SWEEP_PPW": str(ppw), "KS_SWEEP_BLOCK_CAP": str(cap)}, ["c2", "c4"])


@pytest.mark.parametrize("ppw,cap", [(3, 16), (5, 8), (64, 24)])
def test_sweep_shape_invariant_deviceshare(ppw, cap):
    _run({"KS_SWEEP_PPW": str(ppw), "KS_SWEEP_BLOCK_CAP": str(cap)}, ["c3"])


@pytest.mark.parametrize("ppw", [0, 3])
def test_general_commit_kernel_matches(ppw):
    # the monotone plugin set without quota (C1, ks_mono.h by default) through the general commit kernel
    extra = {"KS_COMMIT_GENERAL": "1"}
    if ppw:
        extra["KS_SWEEP_PPW"] = str(ppw)
    _run(extra, ["c1"])


@pytest.mark.parametrize("ppw", [0, 3])
def test_mono_commit_kernel_with_quota_matches(ppw):
    # the monotone plugin set with ElasticQuota (C2, the general kernel by default) through ks_mono.h
    extra = {"KS_COMMIT_GENERAL": "2"}
    if ppw:
        extra["KS_SWEEP_PPW"] = str(ppw)
    _run(extra, ["c2"])
