"""CPU topology helpers shared by the cpuset tests."""


def build_topology(sockets, nodes_per_socket, cores_per_node, cpus_per_core, socket_shift_core=False):
    """buildCPUTopologyForTest (cpu_accumulator_test.go:30-57): CPU ids in (socket, node, core, thread) order."""
    core, node, socket = [], [], []
    nid = cid = 0
    for s in range(sockets):
        for _ in range(nodes_per_socket):
            for _ in range(cores_per_node):
                for _ in range(cpus_per_core):
                    core.append((s << 16 | cid) if socket_shift_core else cid)
                    node.append(nid)
                    socket.append(s)
                cid += 1
            nid += 1
    return core, node, socket


def golden_cluster(case):
    """One node holding a golden case's topology and allocation, one cpu-bind pod needing case["needed"]
    CPUs (preferred policy case["bind"], exclusive case["excl"]), NUMA allocate strategy by node label."""
    import numpy as np

    from koordinator_amd import abi
    from koordinator_amd.cluster import CpuState, NodeTable, PodTable, cpu_mask, cpu_topology
    from koordinator_amd.config import CPU, MEMORY, NodeNUMAResourceArgs, SchedulerProfile

    core, node, sock = build_topology(*case["topo"])
    ncpu = len(core)
    st = CpuState(1, [cpu_topology(core, node, sock)])
    st.topology[0] = 0
    alloc = case["allocated"]
    st.allocated[0] = cpu_mask(alloc)
    if case["allocated_excl"] == "PCPULevel":
        st.excl_pcpu[0] = cpu_mask(alloc)
    elif case["allocated_excl"] == "NUMANodeLevel":
        st.excl_numa[0] = cpu_mask(alloc)
    nodes = NodeTable(1)
    nodes.alloc_milli_cpu[:] = ncpu * 1000
    nodes.alloc_memory[:] = 1 << 40
    nodes.req_milli_cpu[:] = len(alloc) * 1000
    nodes.nonzero_milli_cpu[:] = len(alloc) * 1000
    nodes.allowed_pods[:] = 110
    nodes.numa_cpuset_cpus[:] = len(alloc)
    nodes.numa_flags[:] = abi.KS_NUMA_ALLOC_MOST if case["strategy"] == "Most" else abi.KS_NUMA_ALLOC_LEAST
    pod = PodTable(1)
    pod.req_milli_cpu[:] = case["needed"] * 1000
    pod.nonzero_milli_cpu[:] = case["needed"] * 1000
    pod.req_memory[:] = 1 << 30
    pod.nonzero_memory[:] = 1 << 30
    pod.flags[:] = abi.KS_POD_PROD | abi.KS_POD_CPU_BIND
    bind = abi.KS_CPU_BIND_FULL_PCPUS if case["bind"] == "FullPCPUs" else abi.KS_CPU_BIND_SPREAD_BY_PCPUS
    excl = {"None": 0, "PCPULevel": 1, "NUMANodeLevel": 2}[case["excl"]]
    pod.cpu_bind[:] = bind | (excl << abi.KS_CPU_EXCL_SHIFT)
    cfg = SchedulerProfile(loadaware=None, numa=NodeNUMAResourceArgs(resources={CPU: 1, MEMORY: 1})).to_ks_config()
    return cfg, nodes, st, pod


def supported_on_device(case):
    """maxRefCount 1, and FullPCPUs requests in whole cores (the evaluator refuses the rest)"""
    cpc = case["topo"][3]
    return case["max_ref"] == 1 and not (case["bind"] == "FullPCPUs" and case["needed"] % cpc)
