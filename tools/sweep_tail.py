"""Sweep the k_fit_tail hand-over threshold on a bench workload (one GPU; C2 by default).

Prints one line per threshold: ms per clean (mean of --steps runs after one
warm-up) and the per-kernel times of the fit kernels.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
from iterative_cleaner_amd import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--thresholds", default="0,4096,8192,16384,32768,65536")
    ap.add_argument("--workload", default="C2", choices=sorted(bench.WORKLOADS))
    a = ap.parse_args()
    _native.load_library()
    dev = torch.device("cuda:0")
    nsub, nchan, nbin, seed, rfi = bench.WORKLOADS[a.workload]
    cube, w0, shift = bench.make_cube_device(nsub, nchan, nbin, seed, rfi, dev)
    sess = _native.GpuSession(nsub, nchan, nbin, max_iter=5, device=0)
    torch.cuda.synchronize()
    sess.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
    ref = None
    for th in [int(x) for x in a.thresholds.split(",")]:
        sess.set_fit_tail(th)
        sess.run(fetch=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            out = sess.run(fetch=True)
        torch.cuda.synchronize()
        ms = 1000 * (time.perf_counter() - t0) / a.steps
        w = out["weights"].tobytes()
        same = ref is None or w == ref
        ref = ref or w
        print("tail %6d: %.2f ms/clean (incl. weight fetch) loops=%d same_weights=%s"
              % (th, ms, out["loops"], same), flush=True)
    sess.close()


if __name__ == "__main__":
    main()
