"""The RCCL transport itself on one GPU: tests/rccl_one_rank.py in a child process -- a one-rank
communicator takes the ncclAllGather / ncclAllReduce branches of the candidate exchange on pipelined (patched and
re-swept) and unpipelined passes, C5-shaped at 20k nodes, C2 with quotas, C3-small with DeviceShare maxima and the
default-profile plugins, each bit-exact against the oracle; then ks_destroy's ncclCommDestroy and a normal process
exit (the atexit release of the shared CU-masked streams).  A non-zero exit status, a signal or a hang fails."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_rccl_one_rank_communicator_matches_oracle_and_exits_cleanly():
    env = dict(os.environ)
    env.setdefault("NCCL_SOCKET_IFNAME", "lo")  # the bootstrap socket of ncclGetUniqueId (no network on the box)
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_one_rank.py")], env=env, capture_output=True,
                       text=True, timeout=300)
    print(p.stdout)
    print(p.stderr[-4000:], file=sys.stderr)
    assert p.returncode == 0, f"rccl_one_rank.py exited with {p.returncode}:\n{p.stdout[-2000:]}\n{p.stderr[-3000:]}"
    assert "all cases match the oracle" in p.stdout
