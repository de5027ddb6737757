"""Channel shards as separate processes (one rank per process, SURVEY.md
§8(e)), several ranks sharing the box's one GPU over gloo (RCCL refuses two
ranks on one device; the driver's 8-GPU run exercises RCCL itself).  Every
rank runs its shard session through dist.TorchComm (tools/shard_check.py):

* bit-identity of the merged result with one unsharded session and with the C
  oracle's loop, at worlds 2 and 4, for both fit modes;
* failure handling: a rank whose transport fails mid-iteration returns
  IC_ECOMM, tears its process group down, and its peers' collectives fail
  instead of blocking (well inside the process-group timeout)."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(world, extra, out_dir, timeout=240, pg_timeout=120):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), IC_PG_TIMEOUT=str(pg_timeout), PYTHONUNBUFFERED="1")
        cmd = [sys.executable, os.path.join(REPO, "tools", "shard_check.py"), "--backend", "gloo",
               "--out", str(out_dir), *extra]
        procs.append(subprocess.Popen(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    t0 = time.time()
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=max(1.0, timeout - (time.time() - t0)))[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    recs = {}
    for r in range(world):
        path = os.path.join(str(out_dir), "rank%d.json" % r)
        if os.path.exists(path):
            with open(path) as f:
                recs[r] = json.loads(f.read())
    return [p.returncode for p in procs], recs, logs, time.time() - t0


@pytest.mark.parametrize("fit_mode", [0, 1])
@pytest.mark.parametrize("world", [2, 4])
def test_process_shards_match_one_session_and_oracle(world, fit_mode, tmp_path):
    rcs, recs, logs, _ = _run_ranks(world, ["--shape", "12", "1100", "256", "--oracle",
                                            "--fit-mode", str(fit_mode)], tmp_path)
    assert rcs == [0] * world, "\n".join(logs)
    assert sorted(recs) == list(range(world))
    r0 = recs[0]
    assert r0["bit_identical"] and r0["oracle_weights_equal"] and r0["oracle_loops_equal"], r0
    assert all(recs[r]["loops"] == r0["loops"] and recs[r]["zapped"] == r0["zapped"] for r in recs)


def test_failing_rank_unblocks_its_peers(tmp_path):
    world, pg_timeout = 2, 120
    rcs, recs, logs, elapsed = _run_ranks(world, ["--shape", "8", "600", "128", "--fail-rank", "1",
                                                  "--fail-at", "4"], tmp_path, pg_timeout=pg_timeout)
    assert sorted(recs) == [0, 1], "\n".join(logs)
    assert recs[1]["failed"] and "injected transport failure" in recs[1]["error"]
    assert "rc=-5" in recs[1]["error"]                       # IC_ECOMM from ic_run
    assert recs[0]["failed"] and "rc=-5" in recs[0]["error"], recs[0]   # the peer got an error, not a hang
    assert recs[0]["seconds"] < pg_timeout / 2
    assert all(rc == 3 for rc in rcs), rcs
    assert elapsed < pg_timeout


@pytest.mark.parametrize("suffix", [".ar", ".sf"])
def test_channel_sharded_cli_matches_single_process(suffix, tmp_path):
    """IC_CHANNEL_SHARDS=1 CLI at world 2: every rank reads only its channel
    slice of the file; rank 0's stdout, cleaned archive (weights and samples)
    and residual archive equal a one-process run's."""
    rcs, recs, logs, _ = _run_ranks(2, ["--cli", "--cli-suffix", suffix, "--shape", "10", "600", "128"], tmp_path)
    assert rcs == [0, 0], "\n".join(logs)
    r0 = recs[0]
    assert r0["stdout_equal"] and r0["weights_equal"] and r0["data_equal"] and r0["residual_equal"], r0
    assert "Total number of profiles: 6000" in r0["stdout"]
