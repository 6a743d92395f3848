"""bench.py's sub-record workloads (CPU only): the c3r / c3rd records are the shipped plugin set without and with
reservations holding devices, and the full-size GPU parity test checks the c3rd record's own workload."""
import numpy as np

import bench
from koordinator_amd import synth


def test_c3r_holds_no_devices():
    w = bench.build_workload("c3r", seed=20261015, n_pods=500)
    assert w.reservations is not None and w.reservations.dev_allocatable is None


def test_c3rd_is_the_parity_tests_workload():
    w = bench.build_workload("c3rd", seed=20261015)
    ref = synth.c3_rsv(seed=20261015, dev_rsv_frac=0.7)  # tests/test_gpu_shipped_profile.py (full size)
    assert (w.nodes.n, w.pods.n) == (5000, 10_000)
    assert np.array_equal(w.reservations.dev_allocatable, ref.reservations.dev_allocatable)
    held = (w.reservations.dev_allocatable != 0).any(axis=1)
    assert 0.3 < held.mean() < 0.35
