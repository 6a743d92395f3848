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


# Preferred FullPCPUs requests that are not a whole number of cores, traced by hand through cpu_accumulator.go's
# takeCPUs (:86-232).  The reference's tables hold no such request, so these pin the split-core branches.
#  A: 1 socket / 1 node / 4 cores x 2 threads (core k = CPUs 2k, 2k+1), CPU 1 allocated, 5 CPUs: 5 <= CPUsPerNode, so
#     freeCoresInNode(true, true) lists node 0's full free cores in sortCores order (all 2 free: core id asc) --
#     [2 3 4 5 6 7] -- and takes its first 5.
#  B: 2 sockets x 1 node x 2 cores x 2 threads, CPU 7 allocated, 5 CPUs: 5 > CPUsPerNode = CPUsPerSocket = 4, so the
#     fallback: freeCoresInSocket(true) = [[0 1 2 3] [4 5]] sorted by length desc; needs(4) takes socket 0, needs(2)
#     fails for [4 5] (1 CPU left) and needs(CPUsPerCore) fails; freeCPUs orders the remaining cores by free CPUs on
#     the core ascending -- core 3 {6} before core 2 {4 5} -- and spreadCPUs keeps [6 4 5]: CPU 6.
#  C: the same topology, CPUs 1 and 7 allocated: the fallback takes the full cores {2 3} and {4 5} (insertion-sorted
#     equal lengths keep socket order), then freeCPUs over {0, 6}: equal colocation (2 and 2), socket, node and core
#     scores, so socket 0 first: CPU 0.
SPLIT_CORE_CASES = [
    ("A", (1, 1, 4, 2), [1], 5, "Least", [2, 3, 4, 5, 6]),
    ("B", (2, 1, 2, 2), [7], 5, "Least", [0, 1, 2, 3, 6]),
    ("B-most", (2, 1, 2, 2), [7], 5, "Most", [0, 1, 2, 3, 6]),
    ("C", (2, 1, 2, 2), [1, 7], 5, "Least", [0, 2, 3, 4, 5]),
]


@pytest.mark.parametrize("name,topo,alloc,needed,strategy,want", SPLIT_CORE_CASES, ids=[c[0] for c in SPLIT_CORE_CASES])
def test_full_pcpus_split_cores_hand_traced(name, topo, alloc, needed, strategy, want):
    t = O.topo_from_ids(*topology(*topo))
    avail = [0 if c in alloc else 1 for c in range(t.ncpus)]
    refc = [1 if c in alloc else 0 for c in range(t.ncpus)]
    excl = [O.EXCL["None"] if c in alloc else -1 for c in range(t.ncpus)]
    assert O.take_cpus(t, avail, needed, "FullPCPUs", "None", strategy, 1, refc, excl) == want
