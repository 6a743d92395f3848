"""The oracle's CPU accumulator against the reference's cpu_accumulator_test.go tables
(tests/golden/cpuset.json)."""
import json
import os

import pytest

from oracle import oracle as O
from tests.cpuset_util import build_topology as topology

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "cpuset.json")))


@pytest.mark.parametrize("case", G["cases"], ids=[f"{c['test']}:{c['name']}" for c in G["cases"]])
def test_take_cpus_golden(case):
    t = O.topo_from_ids(*topology(*case["topo"]))
    avail = [0 if c in case["allocated"] else 1 for c in range(t.ncpus)]
    excl = [O.EXCL[case["allocated_excl"]] if c in case["allocated"] else -1 for c in range(t.ncpus)]
    refc = [1 if c in case["allocated"] else 0 for c in range(t.ncpus)]
    got = O.take_cpus(t, avail, case["needed"], case["bind"], case["excl"], case["strategy"], case["max_ref"], refc, excl)
    assert got == case["want"]


@pytest.mark.parametrize("seq", G["sequences"], ids=[s["test"] for s in G["sequences"]])
def test_take_cpus_refcount_sequences(seq):
    """getAvailableCPUs (node_allocation.go:128-145) + takeCPUs + addCPUs, maxRefCount 2."""
    t = O.topo_from_ids(*topology(*seq["topo"], socket_shift_core=True))
    ref = [0] * t.ncpus
    excl = [-1] * t.ncpus
    for st in seq["steps"]:
        avail = [1 if ref[c] < seq["max_ref"] else 0 for c in range(t.ncpus)]
        got = O.take_cpus(t, avail, st["needed"], st["bind"], seq["excl"], seq["strategy"], seq["max_ref"], ref, excl)
        assert got == st["want"]
        for c in got:
            ref[c] += 1
            excl[c] = O.EXCL[seq["added_excl"]]
    if "final_available" in seq:
        assert [c for c in range(t.ncpus) if ref[c] < seq["max_ref"]] == seq["final_available"]


@pytest.mark.parametrize("sp", G["spread_order"], ids=[s["test"] for s in G["spread_order"]])
def test_spread_order(sp):
    t = O.topo_from_ids(*topology(*sp["topo"]))
    assert O.spread_order(t, sp["strategy"]) == sp["order"]


def test_take_cpus_not_enough():
    t = O.topo_from_ids(*topology(1, 1, 4, 2))
    assert O.take_cpus(t, [1] * 4 + [0] * 4, 5, "FullPCPUs") is None
    assert O.take_cpus(t, [1] * 8, 0, "FullPCPUs") == []
