"""The --debug-scores table (frameworkext/debug.go:61-108) built from the device's ks_eval_pod equals the one built
from the CPU oracle's, for pods of a cluster under the complete v1beta2 plugin set (PodTopologySpread, InterPodAffinity,
TaintToleration, NodeAffinity, BalancedAllocation, Fit, LoadAware)."""
import pytest

from koordinator_amd import synth
from koordinator_amd.debug_scores import eval_debug_table

pytestmark = pytest.mark.gpu


def test_debug_table_device_vs_oracle(oracle_lib):
    from koordinator_amd import runtime as rt

    rt.lib()
    w = synth.with_topology(synth.with_static_plugins(synth.c1(n_nodes=700, n_pods=40), seed=31), seed=32)
    cfg = w.cfg
    ev = rt.Evaluator(cfg, w.nodes.copy())
    orc = oracle_lib.Oracle(cfg, w.nodes.copy())
    names = [f"node-{i}" for i in range(w.nodes.n)]
    shown = 0
    try:
        for i in range(w.pods.n):
            pod = w.pods.rows([i])
            got = eval_debug_table(ev, cfg, pod, names, 10, f"default/pod-{i}")
            want = eval_debug_table(orc, cfg, pod, names, 10, f"default/pod-{i}")
            assert got == want, f"pod {i}"
            shown += got is not None
    finally:
        ev.close()
        orc.close()
    assert shown > 0
