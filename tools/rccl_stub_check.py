#!/usr/bin/env python
"""Multi-process check of libicgpu's NATIVE RCCL transport (ic_session_create_rccl,
csrc/ic_comm.hip RcclComm) on one GPU, through the test stub librccl
(tests/stub_rccl: the same nccl* entry points over host shared memory; real
RCCL refuses two ranks of a communicator on one device).

    python tools/rccl_stub_check.py --world 4 --scenario ok --out DIR

The parent spawns `world` rank processes.  Each points the library at the stub
(ic_rccl_set_library), rank 0 makes the unique id (ic_rccl_unique_id) and hands
it to the others through a file, every rank creates its channel shard over the
native transport, uploads its slice and runs.  Scenarios:
  ok      every rank runs; the parent assembles the shards' weights / test
          values / amplitudes and checks them against one unsharded session
          and the C oracle (bit for bit; loops and per-iteration counters too)
  exit    rank 1 exits after creating its session: the others' ic_run must fail
          with IC_ECOMM (the transport notices the dead peer), not hang
  fail    rank 1's ic_run fails (run before upload: IC_ESTATE) and aborts its
          communicator: the others' ic_run must fail with IC_ECOMM
  nojoin  rank 1 exits before ic_session_create_rccl: the others' creation must
          fail with IC_ECOMM after the init timeout (ic_rccl_set_init_timeout)
Prints one JSON line; exit status 0 when the scenario's expectation holds.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
STUB = os.path.join(REPO, "tests", "stub_rccl", "libstubrccl.so")
IC_ECOMM = -5


def child(a):
    import numpy as np

    from iterative_cleaner_amd import _native, synth
    rank, world = a.rank, a.world
    rec = {"rank": rank}
    out = os.path.join(a.out, "rank%d" % rank)
    _native.rccl_set_library(STUB)
    _native.rccl_set_init_timeout(a.init_timeout_ms)
    idf = os.path.join(a.out, "rccl_id.bin")
    if rank == 0:
        rid = _native.rccl_unique_id()
        with open(idf + ".tmp", "wb") as f:
            f.write(rid)
        os.replace(idf + ".tmp", idf)
    else:
        t0 = time.time()
        while not os.path.exists(idf):
            if time.time() - t0 > 60:
                raise SystemExit("rank %d: no unique id" % rank)
            time.sleep(0.01)
        with open(idf, "rb") as f:
            rid = f.read()
    if a.scenario == "nojoin" and rank == 1:
        os._exit(0)
    nsub, nchan, nbin = a.shape
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, a.seed, 0.2)
    raw = np.ascontiguousarray(data[:, 0])
    t0 = time.time()
    try:
        s = _native.ShardSession(nsub, nchan, nbin, rank, world, rccl_id=rid, device=0)
    except _native.NativeError as e:
        rec.update(stage="create", error=str(e), rc=_rc(str(e)), seconds=round(time.time() - t0, 3))
        _write(out, rec)
        return
    c0, c1 = s.chan_range
    if a.scenario == "exit" and rank == 1:
        os._exit(0)
    try:
        if not (a.scenario == "fail" and rank == 1):
            s.upload(raw[:, c0:c1], w0[:, c0:c1], shift[c0:c1])
        t1 = time.time()
        res = s.run()
        amp, info = s.fit()
        np.savez(out + ".npz", weights=res["weights"], test=res["test"], amp=amp, info=info,
                 changed=np.asarray(res["changed"]), T=s.template())
        rec.update(stage="run", loops=int(res["loops"]), c0=c0, c1=c1, seconds=round(time.time() - t1, 3))
    except _native.NativeError as e:
        rec.update(stage="run", error=str(e), rc=_rc(str(e)), seconds=round(time.time() - t0, 3))
    finally:
        s.close()
    _write(out, rec)


def _rc(msg):
    i = msg.rfind("(rc=")
    return int(msg[i + 4:msg.index(")", i)]) if i >= 0 else None


def _write(path, rec):
    with open(path + ".json", "w") as f:
        f.write(json.dumps(rec) + "\n")


def parent(a):
    import numpy as np

    os.makedirs(a.out, exist_ok=True)
    for f in os.listdir(a.out):
        if f.startswith("rank") or f.startswith("rccl_id"):
            os.remove(os.path.join(a.out, f))
    if not os.path.exists(STUB):
        raise SystemExit("build the stub first: make -C tests/stub_rccl")
    cmd = [sys.executable, "-u", os.path.abspath(__file__), "--world", str(a.world), "--scenario", a.scenario,
           "--out", a.out, "--seed", str(a.seed), "--init-timeout-ms", str(a.init_timeout_ms),
           "--shape"] + [str(x) for x in a.shape]
    t0 = time.time()
    procs = [subprocess.Popen(cmd + ["--rank", str(r)]) for r in range(a.world)]
    # reap every rank as it exits (an unreaped rank would look alive to its peers)
    codes = [None] * len(procs)
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        if time.time() - t0 > a.timeout:
            for i, p in enumerate(procs):
                if codes[i] is None:
                    p.kill()
                    p.wait()
                    codes[i] = "timeout"
        time.sleep(0.02)
    recs = {}
    for r in range(a.world):
        path = os.path.join(a.out, "rank%d.json" % r)
        if os.path.exists(path):
            with open(path) as f:
                recs[r] = json.loads(f.read())
    summary = {"world": a.world, "scenario": a.scenario, "shape": a.shape, "exit_codes": codes,
               "seconds": round(time.time() - t0, 2), "ranks": recs}
    ok = "timeout" not in codes
    if a.scenario == "ok":
        ok = ok and all(recs.get(r, {}).get("stage") == "run" and "error" not in recs[r] for r in range(a.world))
        if ok:
            from iterative_cleaner_amd import _native, synth
            from oracle import lib as oracle
            nsub, nchan, nbin = a.shape
            data, w0, shift = synth.make_cube(nsub, nchan, nbin, a.seed, 0.2)
            raw = np.ascontiguousarray(data[:, 0])
            parts = [np.load(os.path.join(a.out, "rank%d.npz" % r)) for r in range(a.world)]
            W = np.concatenate([p["weights"] for p in parts], axis=1)
            test = np.concatenate([p["test"] for p in parts], axis=1)
            amp = np.concatenate([p["amp"] for p in parts], axis=1)
            with _native.GpuSession(nsub, nchan, nbin, device=0) as s:
                s.upload(raw, w0, shift)
                one = s.run()
                amp1, _ = s.fit()
                T1 = s.template()
            ref = oracle.clean_loop(raw, w0, shift, want_details=True)
            checks = {
                "weights_eq_one_session": W.tobytes() == one["weights"].tobytes(),
                "test_eq_one_session": test.tobytes() == one["test"].tobytes(),
                "amp_eq_one_session": amp.tobytes() == amp1.tobytes(),
                "template_eq_one_session": all(p["T"].tobytes() == T1.tobytes() for p in parts),
                "changed_eq_one_session": all(list(p["changed"]) == list(one["changed"]) for p in parts),
                "loops_eq_one_session": all(recs[r]["loops"] == one["loops"] for r in range(a.world)),
                "weights_eq_oracle": W.tobytes() == ref["weights"].tobytes(),
                "amp_eq_oracle": amp.tobytes() == ref["amp"].tobytes(),
                "loops_eq_oracle": one["loops"] == ref["loops"],
            }
            summary["checks"] = checks
            summary["zapped"] = int((W == 0).sum())
            ok = all(checks.values())
    else:
        survivors = [r for r in range(a.world) if r != 1]
        stage = "create" if a.scenario == "nojoin" else "run"
        ok = ok and all(recs.get(r, {}).get("stage") == stage and recs[r].get("rc") == IC_ECOMM for r in survivors)
        if a.scenario == "fail":
            ok = ok and recs.get(1, {}).get("rc") == -4   # IC_ESTATE: run before upload
    summary["ok"] = bool(ok)
    print(json.dumps(summary))
    return 0 if ok else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--rank", type=int, default=-1, help="(internal) run as this rank")
    ap.add_argument("--scenario", default="ok", choices=("ok", "exit", "fail", "nojoin"))
    ap.add_argument("--shape", type=int, nargs=3, default=[8, 1024, 256])
    ap.add_argument("--seed", type=int, default=21)
    ap.add_argument("--init-timeout-ms", type=int, default=4000)
    ap.add_argument("--timeout", type=float, default=240.0, help="parent: seconds to wait for every rank")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    if a.rank >= 0:
        child(a)
        return 0
    return parent(a)


if __name__ == "__main__":
    sys.exit(main())
