"""ctypes binding of libicgpu.so (include/iterative_cleaner.h).

The product path has no CPU fallback: if the HIP library is missing, cannot
be loaded, or no GPU is visible, the calls below raise ``NativeError``.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# IC_LIBRARY: an alternative build of the same library (A/B measurements)
LIB_PATH = os.environ.get("IC_LIBRARY") or os.path.join(HERE, "libicgpu.so")
ABI_VERSION = 8

# symbols exported by libicgpu.so, as declared in include/iterative_cleaner.h
EXPORTS = ("ic_abi_version", "ic_device_count", "ic_session_create", "ic_session_destroy",
           "ic_upload", "ic_upload_device", "ic_run", "ic_get_residual", "ic_get_template",
           "ic_get_fit", "ic_get_diagnostics", "ic_get_kernel_times", "ic_kernel_name",
           "ic_set_timing", "ic_get_run_stats", "ic_set_fit_tail", "ic_last_error",
           "ic_shard_layout", "ic_session_create_shard", "ic_group_create", "ic_group_destroy",
           "ic_session_create_grouped", "ic_upload_async", "ic_host_alloc", "ic_host_free",
           "ic_upload_pols", "ic_comprehensive_stats", "ic_get_bad_fits",
           "ic_fit_profiles", "ic_get_diagnostics_f64", "ic_set_delays", "ic_rotate_profiles",
           "ic_set_timing_kernel", "ic_set_option", "ic_get_option", "ic_comprehensive_stats_rowstat",
           "ic_rccl_unique_id", "ic_session_create_rccl", "ic_rccl_set_library", "ic_rccl_set_init_timeout",
           "ic_set_delays2", "ic_rotate_profiles2")

# session schedule options (ic_set_option; include/iterative_cleaner.h): they
# choose how the loop is scheduled, never its arithmetic
OPTIONS = {"fit_tail": 1, "diag_fork": 2, "fork_delay": 3, "template_incr": 4, "fit_tiled": 5,
           "rowstat_waves": 6, "rowstat_minlen": 7, "diag_chain": 8, "sync_timeout_ms": 9,
           "fit_schedule": 10, "tail_split": 13, "rot_stats": 14}
FIT_ROUNDS = 0   # IC_FIT_ROUNDS: sweep / state rounds (k_fit_pass, k_fit_state, k_fit_tail); the only schedule

FIT_EXACT = 0    # IC_FIT_EXACT: scipy leastsq emulated bit for bit (the reference's arithmetic)
FIT_CLOSED = 1   # IC_FIT_CLOSED: closed-form amplitude fused with the diagnostics (fast mode)
DEDISP_SHIFT = 0  # IC_DEDISP_SHIFT: integer dedispersion shifts
DEDISP_FFT = 1    # IC_DEDISP_FFT: fractional delays, FFT phase rotation (phase_rotation.py)


class NativeError(RuntimeError):
    pass


class Params(C.Structure):
    _fields_ = [("nsub", C.c_int32), ("nchan", C.c_int32), ("nbin", C.c_int32),
                ("max_iter", C.c_int32), ("chanthresh", C.c_double),
                ("subintthresh", C.c_double), ("pr_on", C.c_int32), ("pr_factor", C.c_double),
                ("pr_start", C.c_int32), ("pr_end", C.c_int32), ("baseline_duty", C.c_double),
                ("fit_mode", C.c_int32), ("data_f64", C.c_int32), ("dedisp_mode", C.c_int32),
                ("input_dedispersed", C.c_int32)]


class RunStats(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("fit_rounds", C.c_int32),
                ("fit_profile_sweeps", C.c_int64), ("fit_tail_sweeps", C.c_int64),
                ("window_moves", C.c_int32), ("near_threshold", C.c_int32), ("reserved0", C.c_int64),
                ("reserved1", C.c_int64)]


class KernelTime(C.Structure):
    _fields_ = [("kernel", C.c_int32), ("launches", C.c_int32), ("ms", C.c_double)]


# ic_comm_ops callbacks (include/iterative_cleaner.h)
ALLOC_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p))
RELEASE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t), C.c_void_p,
                           C.POINTER(C.c_size_t), C.c_void_p)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)


class CommOps(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("alloc", ALLOC_FN), ("release", RELEASE_FN),
                ("allgather", ALLGATHER_FN), ("alltoallv", ALLTOALLV_FN),
                ("allreduce_sum_i32", ALLREDUCE_FN)]


_lib = None


def _init_torch_hip():
    """torch-ROCm bundles its own HIP runtime (torch/lib/libamdhip64.so) next to
    the one libicgpu.so links (/opt/rocm/lib/libamdhip64.so.7); both share the
    process's GPU address space, which is what lets torch tensors be passed to
    the C-ABI by pointer.  torch's runtime only finds the GPUs when it
    initialises first, so when torch is installed it is initialised before
    libicgpu is loaded (torch owns exchange buffers and streams in sharded and
    benchmark runs)."""
    try:
        import torch
    except ImportError:  # pragma: no cover - torch is part of the image
        return
    try:
        torch.cuda.is_available()
    except Exception:  # pragma: no cover
        pass


def load_library(path: str = LIB_PATH):
    """Load libicgpu.so (raises NativeError when absent — no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NativeError("libicgpu.so not built at %s (run __graft_entry__.build() or make -C "
                          "iterative_cleaner_amd/csrc)" % path)
    _init_torch_hip()
    try:
        lib = C.CDLL(path)
    except OSError as e:  # pragma: no cover - environment dependent
        raise NativeError("cannot load %s: %s" % (path, e))
    vp = C.c_void_p
    lib.ic_abi_version.restype = C.c_int
    lib.ic_device_count.restype = C.c_int
    lib.ic_last_error.restype = C.c_char_p
    lib.ic_kernel_name.restype = C.c_char_p
    lib.ic_kernel_name.argtypes = [C.c_int]
    lib.ic_session_create.argtypes = [C.POINTER(Params), C.c_int, C.POINTER(vp)]
    lib.ic_session_destroy.argtypes = [vp]
    lib.ic_session_destroy.restype = None
    lib.ic_upload.argtypes = [vp, vp, vp, vp]
    lib.ic_upload_device.argtypes = [vp, vp, vp, vp]
    lib.ic_run.argtypes = [vp] * 8
    lib.ic_get_residual.argtypes = [vp, vp]
    lib.ic_get_template.argtypes = [vp, vp]
    lib.ic_get_fit.argtypes = [vp, vp, vp]
    lib.ic_get_diagnostics.argtypes = [vp, vp, vp, vp, vp]
    lib.ic_get_diagnostics_f64.argtypes = [vp, vp, vp, vp, vp]
    lib.ic_get_kernel_times.argtypes = [vp, C.POINTER(KernelTime), C.c_int]
    lib.ic_set_timing.argtypes = [vp, C.c_int]
    lib.ic_set_timing_kernel.argtypes = [vp, C.c_int]
    lib.ic_get_run_stats.argtypes = [vp, C.POINTER(RunStats)]
    lib.ic_set_fit_tail.argtypes = [vp, C.c_int64]
    lib.ic_set_option.argtypes = [vp, C.c_int, C.c_int64]
    lib.ic_get_option.argtypes = [vp, C.c_int, C.POINTER(C.c_int64)]
    lib.ic_upload_async.argtypes = [vp, vp, vp, vp]
    lib.ic_upload_pols.argtypes = [vp, vp, C.c_int, vp, vp]
    lib.ic_host_alloc.argtypes = [C.c_size_t, C.POINTER(vp)]
    lib.ic_host_free.argtypes = [vp]
    lib.ic_host_free.restype = None
    lib.ic_shard_layout.argtypes = [C.c_int, C.c_int, C.c_int, vp, vp]
    lib.ic_session_create_shard.argtypes = [C.POINTER(Params), C.c_int, C.c_int, C.c_int,
                                            C.POINTER(CommOps), C.POINTER(vp)]
    lib.ic_group_create.argtypes = [C.c_int, C.POINTER(vp)]
    lib.ic_group_destroy.argtypes = [vp]
    lib.ic_group_destroy.restype = None
    lib.ic_session_create_grouped.argtypes = [C.POINTER(Params), C.c_int, vp, C.c_int, C.POINTER(vp)]
    lib.ic_rccl_unique_id.argtypes = [vp]
    lib.ic_session_create_rccl.argtypes = [C.POINTER(Params), C.c_int, C.c_int, C.c_int, vp, C.POINTER(vp)]
    lib.ic_rccl_set_library.argtypes = [C.c_char_p]
    lib.ic_rccl_set_init_timeout.argtypes = [C.c_int64]
    lib.ic_get_bad_fits.argtypes = [vp, vp, C.c_int]
    lib.ic_fit_profiles.argtypes = [C.c_int, C.c_int, C.c_int, vp, vp, C.c_int, vp, vp, vp]
    lib.ic_set_delays.argtypes = [vp, vp]
    lib.ic_set_delays2.argtypes = [vp, vp]
    lib.ic_rotate_profiles.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, C.c_int, vp]
    lib.ic_rotate_profiles2.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, C.c_int, vp]
    lib.ic_comprehensive_stats.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, C.c_double, C.c_double,
                                           vp, vp, vp, vp, vp]
    lib.ic_comprehensive_stats_rowstat.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, C.c_double,
                                                   C.c_double, vp, vp, vp, vp, vp, C.c_int, C.c_int]
    if lib.ic_abi_version() != ABI_VERSION:
        raise NativeError("libicgpu ABI %d != expected %d" % (lib.ic_abi_version(), ABI_VERSION))
    _lib = lib
    return lib


def _err(lib) -> str:
    m = lib.ic_last_error()
    return m.decode() if m else ""


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


def device_count() -> int:
    return int(load_library().ic_device_count())


def normalise_pulse_region(pulse_region, nbin):
    """Reference K6 (iterative_cleaner.py:280-283): active iff != [0, 0, 1];
    (factor, start, end) with Python slice semantics on nbin."""
    if list(pulse_region) == [0, 0, 1]:
        return 0, 1.0, 0, 0
    start, stop, _ = slice(int(pulse_region[1]), int(pulse_region[2])).indices(nbin)
    if stop < start:
        stop = start
    return 1, float(pulse_region[0]), start, stop


class GpuSession:
    """One cleaning session on one GPU (wraps ic_session_*)."""

    def __init__(self, nsub, nchan, nbin, max_iter=5, chanthresh=5.0, subintthresh=5.0,
                 pulse_region=(0, 0, 1), baseline_duty=0.15, device=0, fit_mode=FIT_EXACT, data_f64=False,
                 delay=None, options=None, input_dedispersed=False):
        self.lib = load_library()
        self.shape = (int(nsub), int(nchan), int(nbin))
        self.max_iter = int(max_iter)
        self.fit_mode = int(fit_mode)
        on, fac, a, b = normalise_pulse_region(list(pulse_region), int(nbin))
        self.params = Params(int(nsub), int(nchan), int(nbin), int(max_iter), float(chanthresh),
                             float(subintthresh), on, fac, a, b, float(baseline_duty), self.fit_mode,
                             1 if data_f64 else 0, DEDISP_SHIFT if delay is None else DEDISP_FFT,
                             1 if input_dedispersed else 0)
        self.data_f64 = bool(data_f64)
        h = C.c_void_p()
        rc = self._create(int(device), h)
        if rc != 0:
            raise NativeError("%s: %s (rc=%d)" % (self._create_name, _err(self.lib), rc))
        self.h = h
        for name, value in (options or {}).items():
            self.set_option(name, value)
        if delay is not None:
            self._initial_delays(delay)

    def _initial_delays(self, delay):
        self.set_delays(delay)

    def set_delays(self, delay):
        """Fractional delays in bins of a session created with `delay`
        (dedisp_mode IC_DEDISP_FFT), for this session's channels: (nchan,) per
        channel (ic_set_delays) or (nsub, nchan) per profile (ic_set_delays2)."""
        nsub, nchan = self.shape[0], self.shape[1]
        if np.ndim(delay) == 2:
            d = np.ascontiguousarray(delay, dtype=np.float64).reshape(nsub, nchan)
            self._check(self.lib.ic_set_delays2(self.h, _ptr(d)), "ic_set_delays2")
        else:
            d = np.ascontiguousarray(delay, dtype=np.float64).reshape(nchan)
            self._check(self.lib.ic_set_delays(self.h, _ptr(d)), "ic_set_delays")

    _create_name = "ic_session_create"

    def _create(self, device, h):
        return self.lib.ic_session_create(C.byref(self.params), device, C.byref(h))

    # context manager -----------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.ic_session_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc < 0:
            raise NativeError("%s: %s (rc=%d)" % (what, _err(self.lib), rc))
        return rc

    # data ----------------------------------------------------------------
    def upload(self, cube, w0, shift):
        nsub, nchan, nbin = self.shape
        cube = np.ascontiguousarray(cube, dtype=np.float32).reshape(nsub, nchan, nbin)
        w0 = np.ascontiguousarray(w0, dtype=np.float32).reshape(nsub, nchan)
        shift = np.ascontiguousarray(np.mod(shift, nbin), dtype=np.int32).reshape(nchan)
        self._check(self.lib.ic_upload(self.h, _ptr(cube), _ptr(w0), _ptr(shift)), "ic_upload")

    def upload_pols(self, data, w0, shift):
        """Full-polarisation data (nsub, npol, nchan, nbin): pscrunched on the GPU."""
        nsub, nchan, nbin = self.shape
        data = np.ascontiguousarray(data, dtype=np.float32)
        if data.ndim != 4 or data.shape[0] != nsub or data.shape[2:] != (nchan, nbin):
            raise ValueError("upload_pols: data shape %s != (%d, npol, %d, %d)" % (data.shape, nsub, nchan, nbin))
        w0 = np.ascontiguousarray(w0, dtype=np.float32).reshape(nsub, nchan)
        shift = np.ascontiguousarray(np.mod(shift, nbin), dtype=np.int32).reshape(nchan)
        self._check(self.lib.ic_upload_pols(self.h, _ptr(data), int(data.shape[1]), _ptr(w0), _ptr(shift)),
                    "ic_upload_pols")

    def upload_async(self, cube, w0, shift):
        """Queue the copy of the next archive (see ic_upload_async); the arrays
        must stay alive and unmodified until the run() that consumes them returns."""
        nsub, nchan, nbin = self.shape
        for a, shape, dt in ((cube, (nsub, nchan, nbin), np.float32), (w0, (nsub, nchan), np.float32),
                             (shift, (nchan,), np.int32)):
            if a.dtype != dt or a.shape != shape or not a.flags.c_contiguous:
                raise ValueError("upload_async needs C-contiguous %s %s arrays" % (dt.__name__, shape))
        self._check(self.lib.ic_upload_async(self.h, _ptr(cube), _ptr(w0), _ptr(shift)), "ic_upload_async")

    def upload_device(self, cube_ptr: int, w0_ptr: int, shift_ptr: int):
        """Device pointers (e.g. torch tensor .data_ptr()) on this session's GPU."""
        self._check(self.lib.ic_upload_device(self.h, C.c_void_p(cube_ptr), C.c_void_p(w0_ptr),
                                              C.c_void_p(shift_ptr)), "ic_upload_device")

    def run(self, fetch=True):
        nsub, nchan, _ = self.shape
        m = max(self.max_iter, 1)
        test = np.empty((nsub, nchan), np.float64) if fetch else None
        weights = np.empty((nsub, nchan), np.float32) if fetch else None
        loops = np.zeros(1, np.int32)
        changed = np.zeros(m, np.int32)
        nzero = np.zeros(m, np.int32)
        n_iter = np.zeros(1, np.int32)
        conv = np.zeros(1, np.int32)
        self._check(self.lib.ic_run(self.h, _ptr(test), _ptr(weights), _ptr(loops), _ptr(changed),
                                    _ptr(nzero), _ptr(n_iter), _ptr(conv)), "ic_run")
        k = int(n_iter[0])
        bad = np.zeros(m, np.int32)
        self._check(self.lib.ic_get_bad_fits(self.h, _ptr(bad), m), "ic_get_bad_fits")
        return dict(test=test, weights=weights, loops=int(loops[0]), n_iter=k,
                    converged=bool(conv[0]), changed=changed[:k].copy(), nzero=nzero[:k].copy(),
                    bad_fits=bad[:k].copy())

    def residual(self):
        out = np.empty(self.shape, np.float32)
        self._check(self.lib.ic_get_residual(self.h, _ptr(out)), "ic_get_residual")
        return out

    def template(self):
        out = np.empty(self.shape[2], np.float32)
        self._check(self.lib.ic_get_template(self.h, _ptr(out)), "ic_get_template")
        return out

    def fit(self):
        nsub, nchan, _ = self.shape
        amp = np.empty((nsub, nchan), np.float64)
        info = np.empty((nsub, nchan), np.int32)
        self._check(self.lib.ic_get_fit(self.h, _ptr(amp), _ptr(info)), "ic_get_fit")
        return amp, info

    def diagnostics(self):
        """(std, mean, ptp, fftmax) of the last iteration; ptp is f32 for f32 data
        (numpy.ma's dtype), f64 with data_f64."""
        nsub, nchan, _ = self.shape
        sd, mn, ff = (np.empty((nsub, nchan), np.float64) for _ in range(3))
        if self.data_f64:
            pt = np.empty((nsub, nchan), np.float64)
            self._check(self.lib.ic_get_diagnostics_f64(self.h, _ptr(sd), _ptr(mn), _ptr(pt), _ptr(ff)),
                        "ic_get_diagnostics_f64")
        else:
            pt = np.empty((nsub, nchan), np.float32)
            self._check(self.lib.ic_get_diagnostics(self.h, _ptr(sd), _ptr(mn), _ptr(pt), _ptr(ff)),
                        "ic_get_diagnostics")
        return sd, mn, pt, ff

    def set_timing(self, on: bool, only: str | None = None):
        """Per-kernel HIP-event timing of the following runs; `only`: one kernel
        name (the others run without events)."""
        kid = -1
        if only is not None:
            names = [self.lib.ic_kernel_name(q).decode() for q in range(64)]
            if only not in names:
                raise ValueError("unknown kernel %r" % only)
            kid = names.index(only)
        self._check(self.lib.ic_set_timing_kernel(self.h, kid), "ic_set_timing_kernel")
        self._check(self.lib.ic_set_timing(self.h, 1 if on else 0), "ic_set_timing")

    def set_fit_tail(self, threshold: int):
        """Profiles left at which k_fit_tail takes over the fit (0 = never)."""
        self._check(self.lib.ic_set_fit_tail(self.h, int(threshold)), "ic_set_fit_tail")

    def set_option(self, name: str, value: int):
        """A schedule option (OPTIONS; ic_set_option validates the value)."""
        if name not in OPTIONS:
            raise ValueError("unknown option %r (one of %s)" % (name, ", ".join(sorted(OPTIONS))))
        self._check(self.lib.ic_set_option(self.h, OPTIONS[name], int(value)), "ic_set_option(%s)" % name)

    def get_option(self, name: str) -> int:
        v = C.c_int64()
        self._check(self.lib.ic_get_option(self.h, OPTIONS[name], C.byref(v)), "ic_get_option(%s)" % name)
        return int(v.value)

    def run_stats(self):
        st = RunStats()
        self._check(self.lib.ic_get_run_stats(self.h, C.byref(st)), "ic_get_run_stats")
        return dict(iterations=st.iterations, fit_rounds=st.fit_rounds,
                    fit_profile_sweeps=int(st.fit_profile_sweeps),
                    fit_tail_sweeps=int(st.fit_tail_sweeps),
                    window_moves=int(st.window_moves), near_threshold=int(st.near_threshold))

    def kernel_times(self):
        buf = (KernelTime * 32)()
        n = self._check(self.lib.ic_get_kernel_times(self.h, buf, 32), "ic_get_kernel_times")
        out = {}
        for q in range(n):
            name = self.lib.ic_kernel_name(buf[q].kernel).decode()
            out[name] = dict(ms=buf[q].ms, launches=buf[q].launches)
        return out


def fit_profiles(profiles, template, fit_mode=FIT_EXACT, device=0):
    """remove_profile1d (iterative_cleaner.py:275-288) on the GPU for the
    (nprof, nbin) profiles: (amp f64, info i32, residual f32 a*T - p)."""
    lib = load_library()
    P = np.ascontiguousarray(profiles, dtype=np.float32)
    if P.ndim != 2:
        raise ValueError("fit_profiles: profiles must be (nprof, nbin)")
    T = np.ascontiguousarray(template, dtype=np.float32).reshape(P.shape[1])
    amp = np.empty(P.shape[0], np.float64)
    info = np.empty(P.shape[0], np.int32)
    R = np.empty(P.shape, np.float32)
    rc = lib.ic_fit_profiles(int(device), P.shape[0], P.shape[1], _ptr(T), _ptr(P), int(fit_mode), _ptr(amp),
                             _ptr(info), _ptr(R))
    if rc != 0:
        raise NativeError("ic_fit_profiles: %s (rc=%d)" % (_err(lib), rc))
    return amp, info, R


def rotate_profiles(cube, delay, sign=1, device=0):
    """Fractional dedispersion of a (nsub, nchan, nbin) cube on the GPU: the FFT
    phase rotation by +delay (sign 1, dedisperse) or -delay (sign -1); delay
    (nchan,) per channel (ic_rotate_profiles) or (nsub, nchan) per profile
    (ic_rotate_profiles2)."""
    lib = load_library()
    cube = np.ascontiguousarray(cube, dtype=np.float32)
    if cube.ndim != 3:
        raise ValueError("rotate_profiles: cube must be (nsub, nchan, nbin)")
    nsub, nchan, nbin = cube.shape
    out = np.empty_like(cube)
    if np.ndim(delay) == 2:
        d = np.ascontiguousarray(delay, dtype=np.float64).reshape(nsub, nchan)
        fn, name = lib.ic_rotate_profiles2, "ic_rotate_profiles2"
    else:
        d = np.ascontiguousarray(delay, dtype=np.float64).reshape(nchan)
        fn, name = lib.ic_rotate_profiles, "ic_rotate_profiles"
    rc = fn(int(device), nsub, nchan, nbin, _ptr(cube), _ptr(d), int(sign), _ptr(out))
    if rc != 0:
        raise NativeError("%s: %s (rc=%d)" % (name, _err(lib), rc))
    return out


def comprehensive_stats(data, weights, chanthresh=5.0, subintthresh=5.0, device=0, diagnostics=False,
                        rowstat_waves=8, rowstat_minlen=1024):
    """comprehensive_stats (iterative_cleaner.py:181-226) on the GPU for the
    (nsub, nchan, nbin) data and (nsub, nchan) weights the reference masks and
    weights at :111-117; returns test [, (std, mean, ptp, fftmax)].
    rowstat_*: the row-median form (IC_OPT_ROWSTAT_WAVES / _MINLEN)."""
    lib = load_library()
    data = np.ascontiguousarray(data, dtype=np.float32)
    if data.ndim != 3:
        raise ValueError("comprehensive_stats: data must be (nsub, nchan, nbin)")
    nsub, nchan, nbin = data.shape
    w = np.ascontiguousarray(weights, dtype=np.float32).reshape(nsub, nchan)
    test = np.empty((nsub, nchan), np.float64)
    sd, mn, ff = (np.empty((nsub, nchan), np.float64) for _ in range(3)) if diagnostics else (None,) * 3
    pt = np.empty((nsub, nchan), np.float32) if diagnostics else None
    rc = lib.ic_comprehensive_stats_rowstat(int(device), nsub, nchan, nbin, _ptr(data), _ptr(w),
                                            float(chanthresh), float(subintthresh), _ptr(test), _ptr(sd),
                                            _ptr(mn), _ptr(pt), _ptr(ff), int(rowstat_waves), int(rowstat_minlen))
    if rc != 0:
        raise NativeError("ic_comprehensive_stats: %s (rc=%d)" % (_err(lib), rc))
    return (test, (sd, mn, pt, ff)) if diagnostics else test


class PinnedArray:
    """Page-locked host memory (ic_host_alloc) viewed as a numpy array, so that
    ic_upload_async copies overlap the cleaning of the previous archive."""

    def __init__(self, shape, dtype=np.float32):
        self.lib = load_library()
        dt = np.dtype(dtype)
        n = int(np.prod(shape)) * dt.itemsize
        p = C.c_void_p()
        if self.lib.ic_host_alloc(n, C.byref(p)) != 0:
            raise NativeError("ic_host_alloc: %s" % _err(self.lib))
        self.ptr = p
        buf = (C.c_char * max(n, 1)).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=dt, count=int(np.prod(shape))).reshape(shape)

    def close(self):
        if getattr(self, "ptr", None):
            self.array = None
            self.lib.ic_host_free(self.ptr)
            self.ptr = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- channel shards

def shard_layout(nsub, nchan, world):
    """([(c0, c1)] per rank, [(s0, s1)] per rank) from ic_shard_layout (C++),
    the rule of iterative_cleaner_amd/shards.py."""
    lib = load_library()
    cr = np.zeros(2 * world, np.int32)
    rr = np.zeros(2 * world, np.int32)
    rc = lib.ic_shard_layout(int(nsub), int(nchan), int(world), _ptr(cr), _ptr(rr))
    if rc != 0:
        raise NativeError("ic_shard_layout: %s (rc=%d)" % (_err(lib), rc))
    return ([(int(cr[2 * r]), int(cr[2 * r + 1])) for r in range(world)],
            [(int(rr[2 * r]), int(rr[2 * r + 1])) for r in range(world)])


def rccl_unique_id() -> bytes:
    """128-byte RCCL unique id (ncclGetUniqueId through ic_rccl_unique_id), made
    by rank 0 and handed once to every rank of a native-RCCL shard group."""
    lib = load_library()
    buf = (C.c_char * 128)()
    rc = lib.ic_rccl_unique_id(C.cast(buf, C.c_void_p))
    if rc != 0:
        raise NativeError("ic_rccl_unique_id: %s (rc=%d)" % (_err(lib), rc))
    return bytes(buf.raw)


def rccl_set_library(path):
    """Load `path` instead of the ROCm install's librccl (ic_rccl_set_library;
    None = the default).  Process-wide, before the first RCCL use."""
    lib = load_library()
    rc = lib.ic_rccl_set_library(None if path is None else os.fsencode(path))
    if rc != 0:
        raise NativeError("ic_rccl_set_library: %s (rc=%d)" % (_err(lib), rc))


def rccl_set_init_timeout(ms):
    """How long ic_session_create_rccl waits for every rank to join (ms)."""
    lib = load_library()
    rc = lib.ic_rccl_set_init_timeout(int(ms))
    if rc != 0:
        raise NativeError("ic_rccl_set_init_timeout: %s (rc=%d)" % (_err(lib), rc))


class ShardGroup:
    """In-process shard group (ic_group_create): `world` shard sessions driven
    by `world` host threads of this process, exchanging by device copies."""

    def __init__(self, world):
        self.lib = load_library()
        self.world = int(world)
        h = C.c_void_p()
        if self.lib.ic_group_create(self.world, C.byref(h)) != 0:
            raise NativeError("ic_group_create: %s" % _err(self.lib))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.ic_group_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


class ShardSession(GpuSession):
    """Channel shard `rank` of `world` of one archive (global shape in the
    arguments; uploads and per-profile outputs are the shard's channel slice).
    Exchanges go through `group` (a ShardGroup: in-process), `comm` (an object
    with ``ops()`` returning a CommOps, e.g. dist.TorchComm: host callbacks) or
    `rccl_id` (rank 0's rccl_unique_id(): the library's own RCCL communicator,
    every collective issued from C++ on the session stream)."""

    _create_name = "ic_session_create_shard"

    def __init__(self, nsub, nchan, nbin, rank, world, group=None, comm=None, rccl_id=None, **kw):
        if sum(x is not None for x in (group, comm, rccl_id)) != 1:
            raise ValueError("ShardSession needs exactly one of group / comm / rccl_id")
        if rccl_id is not None and len(rccl_id) != 128:
            raise ValueError("rccl_id must be the 128 bytes of rccl_unique_id()")
        self.rank, self.world = int(rank), int(world)
        self.group, self.comm, self.rccl_id = group, comm, rccl_id
        chans, rows = shard_layout(nsub, nchan, world)
        self.chan_range = chans[self.rank]
        self.row_range = rows[self.rank]
        self.global_shape = (int(nsub), int(nchan), int(nbin))
        self._delay = None
        super().__init__(nsub, nchan, nbin, **kw)
        c0, c1 = self.chan_range
        self.shape = (int(nsub), c1 - c0, int(nbin))
        if self._delay is not None:   # the shard's own channels
            self.set_delays(self._delay)

    def _initial_delays(self, delay):
        self._delay = delay

    def _create(self, device, h):
        if self.group is not None:
            self._create_name = "ic_session_create_grouped"
            return self.lib.ic_session_create_grouped(C.byref(self.params), device, self.group.h,
                                                      self.rank, C.byref(h))
        if self.rccl_id is not None:
            self._create_name = "ic_session_create_rccl"
            self._id_buf = C.create_string_buffer(self.rccl_id, 128)
            return self.lib.ic_session_create_rccl(C.byref(self.params), device, self.rank, self.world,
                                                   C.cast(self._id_buf, C.c_void_p), C.byref(h))
        self._ops = self.comm.ops()
        return self.lib.ic_session_create_shard(C.byref(self.params), device, self.rank,
                                                self.world, C.byref(self._ops), C.byref(h))

    def _check(self, rc, what):
        if rc < 0 and self.comm is not None and getattr(self.comm, "error", None):
            raise NativeError("%s: %s (rc=%d); transport: %s"
                              % (what, _err(self.lib), rc, self.comm.error))
        return super()._check(rc, what)
