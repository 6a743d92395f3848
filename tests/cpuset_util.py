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
    """maxRefCount 1 (the evaluator refuses CPU sharing)"""
    return case["max_ref"] == 1


def bind_policy_cluster(topo, allocated=(), label=0, cpu_milli=4000, bind=None, required=False, excl=0,
                        strategy="Least"):
    """One node with CPU topology `topo` (buildCPUTopologyForTest), `allocated` CPUs, node CPU bind policy
    `label` (KS_NODE_CPU_BIND_*), and one pod requesting cpu_milli: cpu-bind with policy `bind` (required or
    preferred) or, for bind=None, a plain pod (cpu-bind only through the node's policy)."""
    import numpy as np

    from koordinator_amd import abi
    from koordinator_amd.cluster import CpuState, NodeTable, PodTable, cpu_mask, cpu_topology
    from koordinator_amd.config import CPU, MEMORY, NodeNUMAResourceArgs, SchedulerProfile

    core, node, sock = build_topology(*topo)
    ncpu = len(core)
    st = CpuState(1, [cpu_topology(core, node, sock)])
    st.topology[0] = 0
    st.allocated[0] = cpu_mask(list(allocated))
    nodes = NodeTable(1)
    nodes.alloc_milli_cpu[:] = ncpu * 1000
    nodes.alloc_memory[:] = 1 << 40
    nodes.req_milli_cpu[:] = len(allocated) * 1000
    nodes.nonzero_milli_cpu[:] = len(allocated) * 1000
    nodes.allowed_pods[:] = 110
    nodes.numa_cpuset_cpus[:] = len(allocated)
    nodes.numa_flags[:] = ((abi.KS_NUMA_ALLOC_MOST if strategy == "Most" else abi.KS_NUMA_ALLOC_LEAST) |
                           (label << abi.KS_NUMA_CPU_BIND_SHIFT))
    pod = PodTable(1)
    pod.req_milli_cpu[:] = cpu_milli
    pod.nonzero_milli_cpu[:] = cpu_milli
    pod.req_memory[:] = 1 << 30
    pod.nonzero_memory[:] = 1 << 30
    pod.flags[:] = abi.KS_POD_PROD
    if bind is not None:
        pod.flags[:] |= abi.KS_POD_CPU_BIND
        pod.cpu_bind[:] = bind | (excl << abi.KS_CPU_EXCL_SHIFT) | (abi.KS_CPU_BIND_REQUIRED if required else 0)
    cfg = SchedulerProfile(loadaware=None, numa=NodeNUMAResourceArgs(resources={CPU: 1, MEMORY: 1})).to_ks_config()
    return cfg, nodes, st, pod


# Filter of NodeNUMAResource with node CPU bind policies and required pod policies: the reference's
# TestPlugin_Filter cases (nodenumaresource/plugin_test.go:592-760) on buildCPUTopologyForTest(2, 1, 4, 2), no
# allocation.  (name, label, bind, required, cpu milli, expected reason bits)
def filter_cases():
    from koordinator_amd import abi
    F, S = abi.KS_CPU_BIND_FULL_PCPUS, abi.KS_CPU_BIND_SPREAD_BY_PCPUS
    LF, LS = abi.KS_NODE_CPU_BIND_FULL_PCPUS_ONLY, abi.KS_NODE_CPU_BIND_SPREAD_BY_PCPUS
    return [
        ("node FullPCPUsOnly, preferred FullPCPUs 5: SMTAlignmentError", LF, F, False, 5000, abi.KS_R_NUMA_SMT),
        ("LS pod on node FullPCPUsOnly, 5 CPUs: SMTAlignmentError", LF, None, False, 5000, abi.KS_R_NUMA_SMT),
        ("LS pod on node FullPCPUsOnly, 5200m: InvalidRequestedCPUs", LF, None, False, 5200, abi.KS_R_NUMA_INVALID_CPUS),
        ("node FullPCPUsOnly, preferred FullPCPUs 4", LF, F, False, 4000, 0),
        ("required FullPCPUs 5: SMTAlignmentError", 0, F, True, 5000, abi.KS_R_NUMA_SMT),
        ("required FullPCPUs 4", 0, F, True, 4000, 0),
        ("node FullPCPUsOnly, preferred SpreadByPCPUs 4", LF, S, False, 4000, 0),
        ("node SpreadByPCPUs, required FullPCPUs: CPUBindPolicyConflict", LS, F, True, 4000, abi.KS_R_NUMA_BIND_CONFLICT),
        ("node FullPCPUsOnly, required FullPCPUs 4", LF, F, True, 4000, 0),
        ("kubelet FullPCPUsOnly, required SpreadByPCPUs: CPUBindPolicyConflict", LF, S, True, 4000,
         abi.KS_R_NUMA_BIND_CONFLICT),
        ("required FullPCPUs 4 with no NUMA topology policy", 0, F, True, 4000, 0),
    ]


# allocateCPUSet with a required policy: TestResourceManagerAllocate (resource_manager_test.go:95-330) on
# buildCPUTopologyForTest(2, 1, 26, 2), NUMALeastAllocated, 4 CPUs.  (name, bind, allocated, want cpus or None)
def allocate_cases():
    from koordinator_amd import abi
    F, S = abi.KS_CPU_BIND_FULL_PCPUS, abi.KS_CPU_BIND_SPREAD_BY_PCPUS
    holes = [1, 3, 5] + list(range(7, 104))
    return [
        ("required FullPCPUs", F, [], [0, 1, 2, 3]),
        ("required FullPCPUs and allocated", F, list(range(4, 104)), [0, 1, 2, 3]),
        ("required FullPCPUs and allocated: no whole core", F, holes, None),
        ("required SpreadByPCPUs", S, [], [0, 2, 4, 6]),
        ("required SpreadByPCPUs and allocated", S, holes, [0, 2, 4, 6]),
        ("required SpreadByPCPUs and allocated: two cores", S, list(range(4, 104)), None),
    ]


def policy_bind_cluster(topo, allocated=(), label=0, cpu_milli=4000, bind=None, required=False,
                        policy=None):
    """bind_policy_cluster's node with a NUMA topology policy (default SingleNUMANode) and its NodeResourceTopology
    zones: one NUMA node per topology NUMA id, cpu = its CPUs x 1000, memory 2^39 each, allocatedResources cpu = the
    allocated CPUs there.  Returns (cfg, nodes, cpu_state, pod, numa_nodes)."""
    import numpy as np

    from koordinator_amd import abi
    from koordinator_amd.cluster import NumaNodes

    cfg, nodes, st, pod = bind_policy_cluster(topo, allocated=allocated, label=label, cpu_milli=cpu_milli, bind=bind,
                                              required=required)
    pol = abi.KS_NUMA_POLICY_SINGLE_NUMA_NODE if policy is None else policy
    nodes.numa_flags[:] |= np.uint32(pol << abi.KS_NUMA_POLICY_SHIFT)
    _, node, _ = build_topology(*topo)
    K = max(node) + 1
    nn = NumaNodes(1)
    nn.count[0] = K
    for k in range(K):
        cpus = [i for i, v in enumerate(node) if v == k]
        held = len([c for c in allocated if c in cpus])
        nn.alloc_cpu[0, k] = len(cpus) * 1000
        nn.alloc_memory[0, k] = 1 << 39
        nn.cpuset_cpus[0, k] = held
        nn.used_cpu[0, k] = held * 1000
        nn.used_present[0, k] = 1 if held else 0
    return cfg, nodes, st, pod, nn
