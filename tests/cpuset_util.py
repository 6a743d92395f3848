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
