"""Print the run statistics of the fit schedules on one small archive
(a probe for option fit_late_lanes; GPU)."""
import sys

import numpy as np

sys.path.insert(0, ".")
from iterative_cleaner_amd import _native, synth  # noqa: E402

shape = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "16x256x1024").split("x"))
data, w0, shift = synth.make_cube(*shape, 5, 0.1)
raw = np.ascontiguousarray(data[:, 0])
for opts, tail in (({}, None), ({"fit_late_lanes": 1 << 40}, 0), ({"fit_late_lanes": 1 << 40}, None),
                   ({"fit_late_lanes": 3000}, 0), ({"fit_schedule": 1}, None)):
    with _native.GpuSession(*shape, max_iter=5, device=0, options=opts) as s:
        if tail is not None:
            s.set_fit_tail(tail)
        s.upload(raw, w0, shift)
        out = s.run()
        amp, _ = s.fit()
        print(opts, tail, out["loops"], s.run_stats(), float(np.nansum(amp)), flush=True)
