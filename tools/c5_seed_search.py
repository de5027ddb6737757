#!/usr/bin/env python
"""Find seeds of the C5 heavy-RFI workload (256 x 1024 x 4096, 30 % RFI) whose
exact cleaning loop runs to max_iter = 5 ("pick the seed so the
loop reaches max_iter").  Prints one line per seed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    from iterative_cleaner_amd import _native
    nsub, nchan, nbin, _, rfi = bench.WORKLOADS["C5"]
    dev = torch.device("cuda", 0)
    with _native.GpuSession(nsub, nchan, nbin, max_iter=5, device=0) as s:
        for seed in range(int(sys.argv[1]), int(sys.argv[2])):
            cube, w0, shift = bench.make_cube_device(nsub, nchan, nbin, seed, rfi, dev)
            torch.cuda.synchronize()
            s.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
            out = s.run()
            print(seed, out["loops"], out["n_iter"], out["converged"], list(out["changed"]), flush=True)
            del cube, w0, shift


if __name__ == "__main__":
    main()
