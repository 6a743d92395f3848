"""Writes tests/golden/cpuset.json: the CPU accumulator tables of the reference's
pkg/scheduler/plugins/nodenumaresource/cpu_accumulator_test.go, transcribed as data
(topology shape for buildCPUTopologyForTest(sockets, nodesPerSocket, coresPerNode, cpusPerCore),
allocated CPUs, request, policies, expected CPU set).  Run: python tests/golden/make_cpuset_golden.py"""
import json
import os


def cs(s):
    out = []
    for part in str(s).split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(out)


def case(test, name, topo, needed, want, allocated="", bind="FullPCPUs", excl="None", strategy="Most",
         allocated_excl="None", max_ref=1):
    return {"test": test, "name": name, "topo": topo, "max_ref": max_ref, "allocated": cs(allocated),
            "allocated_excl": allocated_excl, "needed": needed, "bind": bind, "excl": excl, "strategy": strategy,
            "want": cs(want)}


C = []
# TestTakeFullPCPUs (cpu_accumulator_test.go:59-173), NUMAMostAllocated
T = "TestTakeFullPCPUs"
C += [case(T, "allocate on non-NUMA node", [1, 1, 4, 2], 2, "0,1"),
      case(T, "with allocated cpus", [1, 1, 4, 2], 2, "2,3", allocated="0,1"),
      case(T, "allocate whole socket", [2, 1, 4, 2], 8, "0-7"),
      case(T, "allocate across socket", [2, 1, 4, 2], 12, "0-11"),
      case(T, "allocate whole socket with partially-allocated socket", [2, 1, 4, 2], 8, "8-15", allocated="0,1"),
      case(T, "allocate in the smallest idle socket", [2, 2, 4, 2], 6, "24-29", allocated="0-5,16-23"),
      case(T, "allocate the most of CPUs on the same socket", [2, 2, 4, 2], 12, "6-15,24-25", allocated="0-5,16-23"),
      case(T, "allocate from first socket", [2, 2, 4, 2], 4, "4-7", allocated="0-3,8-11"),
      case(T, "allocate with less spread cpus", [2, 2, 2, 2], 4, "10,11,14,15", allocated="0,2,4,8,12"),
      case(T, "allocate with the most spread cpus", [2, 2, 2, 2], 6, "5,6,7,13,14,15", allocated="0,2,4,8,10,12"),
      case(T, "allocate with the most spread cpus on the smallest idle cpus socket", [2, 2, 2, 2], 6,
           "6,7,11,13,14,15", allocated="0,2,4,8,9,10,12")]
# TestTakeFullPCPUsWithNUMALeastAllocated (:175-289)
T = "TestTakeFullPCPUsWithNUMALeastAllocated"
L = dict(strategy="Least")
C += [case(T, "allocate on non-NUMA node", [1, 1, 4, 2], 2, "0,1", **L),
      case(T, "with allocated cpus", [1, 1, 4, 2], 2, "2,3", allocated="0,1", **L),
      case(T, "allocate whole socket", [2, 1, 4, 2], 8, "0-7", **L),
      case(T, "allocate across socket", [2, 1, 4, 2], 12, "0-11", **L),
      case(T, "allocate whole socket with partially-allocated socket", [2, 1, 4, 2], 8, "8-15", allocated="0,1", **L),
      case(T, "allocate in the most idle socket", [2, 2, 4, 2], 6, "8-13", allocated="0-5,16-23", **L),
      case(T, "allocate the most of CPUs on the same socket", [2, 2, 4, 2], 12, "6-15,24-25", allocated="0-5,16-23", **L),
      case(T, "allocate from second socket", [2, 2, 4, 2], 4, "16-19", allocated="0-3,8-11", **L),
      case(T, "allocate with less spread cpus", [2, 2, 2, 2], 4, "10,11,14,15", allocated="0,2,4,8,12", **L),
      case(T, "allocate with the less spread cpus 2", [2, 2, 2, 2], 6, "1,3,6,7,14,15", allocated="0,2,4,8,10,12", **L),
      case(T, "allocate with the most spread cpus on the most idle cpus socket 3", [2, 2, 4, 2], 6, "16-21",
           allocated="0,2,4,8,9,10,12", **L)]
# TestTakeSpreadByPCPUs (:301-361) and WithNUMALeastAllocated (:373-433)
for T, strat, wants in (("TestTakeSpreadByPCPUs", "Most", ["0,2,4,6", "1,3,4,6", "8,10,12,14", "1,3-7"]),
                        ("TestTakeSpreadByPCPUsWithNUMALeastAllocated", "Least",
                         ["0,2,4,6", "8,10,12,14", "8,10,12,14", "8,10,12,14,9,11"])):
    S = dict(bind="SpreadByPCPUs", strategy=strat)
    C += [case(T, "allocate on non-NUMA node", [1, 1, 4, 2], 4, wants[0], **S),
          case(T, "allocate satisfied the partially-allocated socket", [2, 1, 4, 2], 4, wants[1], allocated="0,2", **S),
          case(T, "allocate cpus on full-free socket", [2, 1, 4, 2], 4, wants[2], allocated="0,1,2,3", **S),
          case(T, "allocate most of CPUs in the same socket and overlapped-cores", [2, 1, 4, 2], 6, wants[3],
               allocated="0,2", **S)]
# TestTakeCPUsWithExclusivePolicy (:435-558): default allocated policy PCPULevel, request PCPULevel, SpreadByPCPUs
T = "TestTakeCPUsWithExclusivePolicy"
E = dict(bind="SpreadByPCPUs", excl="PCPULevel", allocated_excl="PCPULevel")
C += [case(T, "allocate cpus on full-free socket with PCPULevel", [2, 1, 4, 2], 4, "8,10,12,14", allocated="0,2", **E),
      case(T, "allocate overlapped cpus with PCPULevel", [2, 1, 4, 2], 10, "0,1,2,3,4,6,8,10,12,14", **E),
      case(T, "allocate cpus on large-size partially-allocated socket with PCPULevel", [2, 1, 8, 2], 4, "4,6,8,10",
           allocated="0,2", **E),
      case(T, "allocate cpus with none exclusive policy", [2, 1, 8, 2], 4, "1,3,4,6", allocated="0,2",
           bind="SpreadByPCPUs", excl="None", allocated_excl="PCPULevel"),
      case(T, "allocate cpus on full-free socket with NUMANodeLevel", [2, 1, 4, 2], 4, "8,10,12,14", allocated="0,2",
           bind="SpreadByPCPUs", excl="NUMANodeLevel", allocated_excl="NUMANodeLevel"),
      case(T, "allocate cpus on partially-allocated socket without NUMANodeLevel", [2, 1, 4, 2], 4, "1,3,4,6",
           allocated="0,2", bind="SpreadByPCPUs", excl="None", allocated_excl="NUMANodeLevel"),
      case(T, "allocate cpus on full-free socket with NUMANodeLevel with PCPUs", [2, 1, 4, 2], 4, "8,9,10,11",
           allocated="0,2", bind="FullPCPUs", excl="NUMANodeLevel", allocated_excl="NUMANodeLevel"),
      case(T, "allocate cpus on partially-allocated socket without NUMANodeLevel with PCPUs", [2, 1, 4, 2], 4, "4,5,6,7",
           allocated="0,2", bind="FullPCPUs", excl="None", allocated_excl="NUMANodeLevel")]
# TestTakePreferredCPUs first call (:758-763): plain takeCPUs
C += [case("TestTakePreferredCPUs", "takeCPUs spread 2", [2, 1, 16, 2], 2, "0,2", bind="SpreadByPCPUs")]

# sequences with maxRefCount 2: each step allocates with exclusive policy PCPULevel (addCPUs) on top of the previous
SEQ = [
    {"test": "TestTakeCPUsWithMaxRefCount", "topo": [1, 1, 4, 2], "max_ref": 2, "strategy": "Most", "excl": "None",
     "added_excl": "PCPULevel",
     "steps": [{"needed": 4, "bind": "FullPCPUs", "want": cs("0-3")},
               {"needed": 5, "bind": "FullPCPUs", "want": cs("0,4-7")},
               {"needed": 4, "bind": "FullPCPUs", "want": cs("2-5")}]},
    {"test": "TestTakeCPUsSortByRefCount", "topo": [1, 1, 16, 2], "max_ref": 2, "strategy": "Most", "excl": "None",
     "added_excl": "PCPULevel",
     "steps": [{"needed": 16, "bind": "SpreadByPCPUs", "want": cs("0,2,4,6,8,10,12,14,16,18,20,22,24,26,28,30")},
               {"needed": 16, "bind": "FullPCPUs", "want": cs("0-15")},
               {"needed": 16, "bind": "SpreadByPCPUs", "want": cs("1,3,5,7,9,11,13,15,17,19,21,23,25,27,29,31")},
               {"needed": 16, "bind": "FullPCPUs", "want": cs("16-31")}],
     "final_available": []},
]
# spread order of freeCPUs(false) on (2,2,4,2) (TestCPUSpreadByPCPUs :291-299, WithNUMALeastAllocated :363-371)
ORDER = list(range(0, 32, 2)) + list(range(1, 32, 2))
SPREAD = [{"test": "TestCPUSpreadByPCPUs", "topo": [2, 2, 4, 2], "strategy": "Most", "order": ORDER},
          {"test": "TestCPUSpreadByPCPUsWithNUMALeastAllocated", "topo": [2, 2, 4, 2], "strategy": "Least", "order": ORDER}]

out = {"source": "koordinator pkg/scheduler/plugins/nodenumaresource/cpu_accumulator_test.go",
       "cases": C, "sequences": SEQ, "spread_order": SPREAD}
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpuset.json"), "w") as f:
    json.dump(out, f, indent=1)
print(len(C), "cases,", len(SEQ), "sequences")
