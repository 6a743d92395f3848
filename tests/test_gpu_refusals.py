"""Inputs the library does not model are refused with KS_EUNSUPPORTED at the ABI, never computed
silently: the shim's KS_POD_UNMODELLED pods (FPGA, allocate hints, reserve pods), KS_DEV_UNMODELLED nodes (preemptible
device capacity, device-holding reservations), KS_NUMA_MAX_REF_COUNT nodes (CPU sharing), and ks_preempt outside the
ElasticQuota PostFilter's modelled plugin set."""
import numpy as np
import pytest

from helpers import profile
from koordinator_amd import abi, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


def refused(fn):
    from koordinator_amd.runtime import KsError

    with pytest.raises(KsError) as ei:
        fn()
    assert ei.value.rc == abi.KS_EUNSUPPORTED, ei.value


def test_unmodelled_pod(runtime):
    w = synth.c2(n_nodes=200, n_pods=10)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), w.quotas.copy())
    pods = w.pods.copy() if hasattr(w.pods, "copy") else w.pods.rows(np.arange(w.pods.n))
    pods.flags[3] |= abi.KS_POD_UNMODELLED
    refused(lambda: ev.schedule(pods))
    refused(lambda: ev.eval_pod(pods.rows([3])))
    refused(lambda: ev.assume(pods.rows([3]), 0))
    got = ev.schedule(pods.rows([0, 1, 2]))  # the others still run (placed or quota-rejected, as the oracle says)
    from oracle.oracle import Oracle

    orc = Oracle(w.cfg, w.nodes.copy(), w.quotas.copy())
    want = orc.schedule(pods.rows([0, 1, 2]))
    orc.close()
    assert np.array_equal(got["status"], want["status"]) and np.array_equal(got["node"], want["node"])
    ev.close()


def test_unmodelled_devices_and_cpu_sharing(runtime):
    w = synth.c3(n_nodes=120, n_pods=10)
    dev = w.devices.copy()
    dev.flags[5] |= abi.KS_DEV_UNMODELLED
    ev = runtime.Evaluator(w.cfg, w.nodes.copy())
    refused(lambda: ev.load_devices(dev))
    ev.close()
    nodes = w.nodes.copy()
    nodes.numa_flags[7] |= abi.KS_NUMA_MAX_REF_COUNT
    refused(lambda: runtime.Evaluator(w.cfg, nodes))


def test_preempt_outside_the_modelled_set(runtime):
    w = synth.c2_preempt(n_nodes=100, n_preemptors=2)
    # no quota row: the reference's cloned PostFilterState has no QuotaInfo
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), w.quotas.copy())
    ev.load_node_pods(w.node_pods)
    p = w.preemptors.rows([0])
    p.quota[0] = -1
    refused(lambda: ev.preempt(p, 5000))
    ev.close()
    # Reservation's PreFilter extensions are not modelled
    cfg = synth.koord_profile(with_quota=True, with_reservation=True).to_ks_config()
    ev = runtime.Evaluator(cfg, w.nodes.copy(), w.quotas.copy())
    ev.load_node_pods(w.node_pods)
    refused(lambda: ev.preempt(w.preemptors.rows([0]), 5000))
    ev.close()
    # ElasticQuota off
    ev = runtime.Evaluator(profile().to_ks_config(), w.nodes.copy())
    ev.load_node_pods(w.node_pods)
    refused(lambda: ev.preempt(w.preemptors.rows([0]), 5000))
    ev.close()
