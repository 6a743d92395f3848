"""Shared helpers for the per-pod framework mode tests (ks_assume / ks_unreserve and the oracle's ko_*)."""
import numpy as np

from koordinator_amd import abi, synth


def state(ev, w):
    """Every mutable table the Reserve / Unreserve paths touch, as plain arrays."""
    out = {}
    out.update({f"node.{k}": v for k, v in ev.read_nodes().as_dict().items()})
    if w.quotas is not None:
        out["quota.used"] = np.asarray(ev.read_quota_used())
    if w.reservations is not None:
        for i, a in enumerate(ev.read_reservations()):
            out[f"rsv.{i}"] = np.asarray(a)
    if w.devices is not None:
        for i, a in enumerate(ev.read_devices()):
            out[f"dev.{i}"] = np.asarray(a)
    if w.cpus is not None:
        for i, a in enumerate(ev.read_cpu_state()):
            out[f"cpu.{i}"] = np.asarray(a)
    if w.numa_nodes is not None:
        for i, a in enumerate(ev.read_numa_nodes()):
            out[f"numa.{i}"] = np.asarray(a)
    return out


def assert_states_equal(a, b, label):
    assert a.keys() == b.keys(), label
    for k in a:
        assert np.array_equal(a[k], b[k]), f"{label}: {k} differs"


def workloads(small=True):
    """C2 (quota), C3 (devices, cpusets, SingleNUMANode nodes), C4 (reservations) and C3-rsv (the shipped profile's
    Reservation + NodeNUMAResource + DeviceShare together), small sizes."""
    return [synth.c2(n_nodes=300, n_pods=200, n_quotas=8), synth.c3(n_nodes=200, n_pods=200),
            synth.c4(n_nodes=300, n_reservations=700, n_pods=200), synth.c3_rsv(n_nodes=200, n_pods=200)]
