"""ctypes binding of libicgpu.so (include/iterative_cleaner.h).

The product path has no CPU fallback: if the HIP library is missing, cannot
be loaded, or no GPU is visible, the calls below raise ``NativeError``.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libicgpu.so")
ABI_VERSION = 2

# symbols exported by libicgpu.so, as declared in include/iterative_cleaner.h
EXPORTS = ("ic_abi_version", "ic_device_count", "ic_session_create", "ic_session_destroy",
           "ic_upload", "ic_upload_device", "ic_run", "ic_get_residual", "ic_get_template",
           "ic_get_fit", "ic_get_diagnostics", "ic_get_kernel_times", "ic_kernel_name",
           "ic_set_timing", "ic_get_run_stats", "ic_set_fit_tail", "ic_last_error")


class NativeError(RuntimeError):
    pass


class Params(C.Structure):
    _fields_ = [("nsub", C.c_int32), ("nchan", C.c_int32), ("nbin", C.c_int32),
                ("max_iter", C.c_int32), ("chanthresh", C.c_double),
                ("subintthresh", C.c_double), ("pr_on", C.c_int32), ("pr_factor", C.c_double),
                ("pr_start", C.c_int32), ("pr_end", C.c_int32), ("baseline_duty", C.c_double),
                ("fit_mode", C.c_int32)]


class RunStats(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("fit_rounds", C.c_int32),
                ("fit_profile_sweeps", C.c_int64), ("fit_tail_sweeps", C.c_int64),
                ("window_moves", C.c_int32), ("reserved", C.c_int32)]


class KernelTime(C.Structure):
    _fields_ = [("kernel", C.c_int32), ("launches", C.c_int32), ("ms", C.c_double)]


_lib = None


def load_library(path: str = LIB_PATH):
    """Load libicgpu.so (raises NativeError when absent — no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NativeError("libicgpu.so not built at %s (run __graft_entry__.build() or make -C "
                          "iterative_cleaner_amd/csrc)" % path)
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
    lib.ic_get_kernel_times.argtypes = [vp, C.POINTER(KernelTime), C.c_int]
    lib.ic_set_timing.argtypes = [vp, C.c_int]
    lib.ic_get_run_stats.argtypes = [vp, C.POINTER(RunStats)]
    lib.ic_set_fit_tail.argtypes = [vp, C.c_int64]
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
                 pulse_region=(0, 0, 1), baseline_duty=0.15, device=0):
        self.lib = load_library()
        self.shape = (int(nsub), int(nchan), int(nbin))
        self.max_iter = int(max_iter)
        on, fac, a, b = normalise_pulse_region(list(pulse_region), int(nbin))
        self.params = Params(int(nsub), int(nchan), int(nbin), int(max_iter), float(chanthresh),
                             float(subintthresh), on, fac, a, b, float(baseline_duty), 0)
        h = C.c_void_p()
        rc = self.lib.ic_session_create(C.byref(self.params), int(device), C.byref(h))
        if rc != 0:
            raise NativeError("ic_session_create: %s (rc=%d)" % (_err(self.lib), rc))
        self.h = h

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
        return dict(test=test, weights=weights, loops=int(loops[0]), n_iter=k,
                    converged=bool(conv[0]), changed=changed[:k].copy(), nzero=nzero[:k].copy())

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
        nsub, nchan, _ = self.shape
        sd, mn, ff = (np.empty((nsub, nchan), np.float64) for _ in range(3))
        pt = np.empty((nsub, nchan), np.float32)
        self._check(self.lib.ic_get_diagnostics(self.h, _ptr(sd), _ptr(mn), _ptr(pt), _ptr(ff)),
                    "ic_get_diagnostics")
        return sd, mn, pt, ff

    def set_timing(self, on: bool):
        self._check(self.lib.ic_set_timing(self.h, 1 if on else 0), "ic_set_timing")

    def set_fit_tail(self, threshold: int):
        """Profiles left at which k_fit_tail takes over the fit (0 = never)."""
        self._check(self.lib.ic_set_fit_tail(self.h, int(threshold)), "ic_set_fit_tail")

    def run_stats(self):
        st = RunStats()
        self._check(self.lib.ic_get_run_stats(self.h, C.byref(st)), "ic_get_run_stats")
        return dict(iterations=st.iterations, fit_rounds=st.fit_rounds,
                    fit_profile_sweeps=int(st.fit_profile_sweeps),
                    fit_tail_sweeps=int(st.fit_tail_sweeps),
                    window_moves=int(st.window_moves))

    def kernel_times(self):
        buf = (KernelTime * 32)()
        n = self._check(self.lib.ic_get_kernel_times(self.h, buf, 32), "ic_get_kernel_times")
        out = {}
        for q in range(n):
            name = self.lib.ic_kernel_name(buf[q].kernel).decode()
            out[name] = dict(ms=buf[q].ms, launches=buf[q].launches)
        return out
