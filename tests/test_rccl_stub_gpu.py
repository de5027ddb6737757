"""The native RCCL transport (ic_session_create_rccl; csrc/ic_comm.hip RcclComm)
with several ranks, one process each, on the one GPU of the test box.  Real
RCCL refuses two ranks of a communicator on one device, so the library is
pointed (ic_rccl_set_library) at the test stub tests/stub_rccl/libstubrccl.so,
which implements the same nccl* entry points over host shared memory.  What is
exercised is the library's own code: RcclComm's non-blocking creation polled
under the init timeout, its all-gathers, grouped sends / receives and the
counter all-reduce issued from C++, and the error paths (abort, a dead or
missing peer).  tools/rccl_stub_check.py runs the ranks and checks them:
  * world 2 and 4: the shards' weights, test values, amplitudes, templates,
    loop counts and per-iteration counters equal one unsharded session's and
    the C oracle's, bit for bit;
  * a rank that exits after creating its session, or whose ic_run fails
    (aborting its communicator): every other rank's ic_run fails with IC_ECOMM
    instead of hanging;
  * a rank that never creates its session: every other rank's creation fails
    with IC_ECOMM after the init timeout (CommInitRank blocked)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(REPO, "tools", "rccl_stub_check.py")


def _check(tmp_path, world, scenario, shape=(8, 1024, 256)):
    if not os.path.exists(os.path.join(REPO, "tests", "stub_rccl", "libstubrccl.so")):
        pytest.fail("tests/stub_rccl/libstubrccl.so missing (build(): make -C tests/stub_rccl)")
    cmd = [sys.executable, TOOL, "--world", str(world), "--scenario", scenario, "--out", str(tmp_path),
           "--timeout", "100", "--shape"] + [str(x) for x in shape]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=110)
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert line, p.stdout[-2000:] + p.stderr[-2000:]
    rec = json.loads(line[-1])
    assert rec["ok"], json.dumps(rec, indent=1)
    return rec


@pytest.mark.parametrize("world", [2, 4])
def test_native_rccl_ranks_equal_one_session_and_oracle(tmp_path, world):
    rec = _check(tmp_path, world, "ok")
    assert rec["zapped"] > 0
    assert all(rec["checks"].values())


@pytest.mark.parametrize("world,scenario", [(2, "exit"), (2, "fail"), (4, "fail"), (2, "nojoin")])
def test_native_rccl_failing_rank_unblocks_peers(tmp_path, world, scenario):
    rec = _check(tmp_path, world, scenario)
    for r, v in rec["ranks"].items():
        if int(r) != 1:
            assert v["rc"] == -5, v          # IC_ECOMM
            assert v["seconds"] < 60, v      # an error, not a hang
