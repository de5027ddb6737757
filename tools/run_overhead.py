"""Host overhead of one clean: the Python wrapper's sess.run() against a bare
ctypes ic_run loop on the same resident C1 archive (A/B probe, prints JSON)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from iterative_cleaner_amd import _native  # noqa: E402

nsub, nchan, nbin, seed, rfi = bench.WORKLOADS["C1"]
dev = torch.device("cuda", 0)
cube, w0, shift = bench.make_cube_device(nsub, nchan, nbin, seed, rfi, dev)
res = {}
with _native.GpuSession(nsub, nchan, nbin, max_iter=5, device=0) as s:
    s.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
    for _ in range(3):
        s.run(fetch=False)
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        s.run(fetch=False)
    res["wrapper_ms"] = 1000 * (time.perf_counter() - t0) / n
    loops = np.zeros(1, np.int32)
    ch = np.zeros(8, np.int32)
    nz = np.zeros(8, np.int32)
    ni = np.zeros(1, np.int32)
    cv = np.zeros(1, np.int32)
    args = [s.h, None, None, loops.ctypes.data, ch.ctypes.data, nz.ctypes.data, ni.ctypes.data, cv.ctypes.data]
    t0 = time.perf_counter()
    for _ in range(n):
        s.lib.ic_run(*args)
    res["bare_ic_run_ms"] = 1000 * (time.perf_counter() - t0) / n
print(json.dumps(res))
