"""CPU tests of the archive stand-in, the host-side cleaner logic and the C-ABI
library surface (no GPU compute calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

from helpers import GOLDEN

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ------------------------------------------------------------ archive stand-in
def test_dedisperse_roundtrip():
    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import synth
    data, w, shift = synth.make_cube(3, 20, 32, 1, 0.0)
    ar = ica.Archive(data, w, shift)
    ar.dedisperse()
    ded = ar.get_data()
    for c in range(20):
        assert np.array_equal(ded[:, 0, c], np.roll(data[:, 0, c], -shift[c], axis=-1))
    ar.dededisperse()
    assert np.array_equal(ar.get_data(), data)


def test_chan_sum_order_is_superblock_tree():
    """Sequential inside 256-channel super-blocks, partials by the halving tree:
    7 super-blocks -> (p0 + (p1 + p2)) + ((p3 + p4) + (p5 + p6))."""
    from iterative_cleaner_amd.archive import SUPER_BLOCK, chan_sum
    rng = np.random.default_rng(0)
    n = 7 * SUPER_BLOCK - 100
    t = rng.standard_normal(n) * 10.0 ** rng.uniform(-8, 8, n)
    p = []
    for b0 in range(0, n, SUPER_BLOCK):
        part = 0.0
        for c in range(b0, min(n, b0 + SUPER_BLOCK)):
            part = part + t[c]
        p.append(part)
    assert len(p) == 7
    want = (p[0] + (p[1] + p[2])) + ((p[3] + p[4]) + (p[5] + p[6]))
    assert chan_sum(t, 0) == want
    assert chan_sum(t[:SUPER_BLOCK], 0) == p[0]


@pytest.mark.parametrize("nsb", [1, 2, 3, 5, 8, 13, 32, 64])
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_sb_tree_shards_reproduce_single(nsb, world):
    """2^d shards each own one depth-d node of the tree; combining their roots
    with the same tree over `world` leaves gives the single-device bits."""
    from iterative_cleaner_amd.archive import sb_tree
    from iterative_cleaner_amd.shards import channel_shards
    if nsb < world:
        with pytest.raises(ValueError):
            channel_shards(nsb * 256, world)
        return
    rng = np.random.default_rng(nsb * 10 + world)
    parts = list(rng.standard_normal(nsb) * 10.0 ** rng.uniform(-12, 12, nsb))
    ranges = channel_shards(nsb * 256 - 17, world)
    roots = [sb_tree(parts[c0 // 256:(c1 + 255) // 256]) for c0, c1 in ranges]
    assert sb_tree(roots) == sb_tree(parts)
    assert ranges[0][0] == 0 and ranges[-1][1] == nsb * 256 - 17
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))


def test_window_argmin_nan_and_ties():
    from iterative_cleaner_amd.archive import window_argmin
    tot = np.array([3.0, 1.0, 1.0, 3.0, 5.0])
    assert window_argmin(tot, 1) == 1              # first of tied minima
    tot2 = np.array([3.0, 1.0, np.nan, 3.0])
    assert window_argmin(tot2, 1) == 2             # numpy: first NaN wins


def test_unload_load_roundtrip(tmp_path):
    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import synth
    ar = synth.make_archive(4, 8, 16, seed=2, npol=2, filename=str(tmp_path / "a.ar"))
    p = str(tmp_path / "b.ar")
    ar.unload(p)
    br = ica.Archive_load(p)
    assert np.array_equal(ar.get_data(), br.get_data())
    assert np.array_equal(ar.get_weights(), br.get_weights())
    assert np.array_equal(ar.get_dm_shift(), br.get_dm_shift())


def test_pscrunch_is_f32_sum():
    from iterative_cleaner_amd import synth
    ar = synth.make_archive(3, 5, 16, seed=3, npol=4)
    d = ar.get_data()
    ar.pscrunch()
    assert ar.get_npol() == 1
    assert np.array_equal(ar.get_data()[:, 0], (d[:, 0] + d[:, 1]).astype(np.float32))


# ------------------------------------------------------------ host logic
def test_cli_defaults_match_reference():
    """Namespace (and its repr, written to clean.log) equals the reference's
    parse_arguments defaults (iterative_cleaner.py:16-42)."""
    from iterative_cleaner_amd import cleaner
    ns = cleaner.parse_arguments(["a.ar"])
    assert repr(ns) == ("Namespace(archive=['a.ar'], chanthresh=5, subintthresh=5, max_iter=5, "
                        "print_zap=False, unload_res=False, pscrunch=False, quiet=False, "
                        "no_log=False, pulse_region=[0, 0, 1], output='', memory=False, "
                        "bad_chan=1, bad_subint=1)")
    ns = cleaner.parse_arguments(["-c", "3", "-r", "0.5", "30", "50", "a.ar", "b.ar"])
    assert ns.chanthresh == 3.0 and ns.pulse_region == [0.5, 30.0, 50.0]
    assert ns.archive == ["a.ar", "b.ar"]


def test_pulse_region_normalisation():
    from iterative_cleaner_amd._native import normalise_pulse_region
    assert normalise_pulse_region([0, 0, 1], 128) == (0, 1.0, 0, 0)
    assert normalise_pulse_region([0.0, 0.0, 1.0], 128) == (0, 1.0, 0, 0)
    assert normalise_pulse_region([0.5, 30.0, 50.0], 128) == (1, 0.5, 30, 50)
    assert normalise_pulse_region([2.0, -10, 300], 128) == (1, 2.0, 118, 128)
    assert normalise_pulse_region([2.0, 60, 10], 128) == (1, 2.0, 60, 60)


def test_output_names():
    from iterative_cleaner_amd import cleaner, synth
    ar = synth.make_archive(2, 4, 8, filename="/x/y/J1234.ar")
    ns = cleaner.parse_arguments(["a.ar"])
    assert cleaner._output_name(ar, ns) == "/x/y/J1234_cleaned.ar"
    ns = cleaner.parse_arguments(["-o", "std", "a.ar"])
    assert cleaner._output_name(ar, ns) == "J0000+0000.1400.000.60000.005000.ar"
    ns = cleaner.parse_arguments(["-o", "out.ar", "a.ar"])
    assert cleaner._output_name(ar, ns) == "out.ar"


def _bad_parts_expected(weights, bad_chan, bad_subint):
    w = weights.copy()
    nsub, nchan = w.shape
    zs = [i for i in range(nsub) if 1 - np.count_nonzero(weights[i]) / float(nchan) > bad_subint]
    zc = [j for j in range(nchan) if 1 - np.count_nonzero(weights[:, j]) / float(nsub) > bad_chan]
    w[zs, :] = 0
    w[:, zc] = 0
    return w, len(zs), len(zc)


def test_find_bad_parts(capsys):
    """K11: both passes use the entry weights; strict '>'."""
    from iterative_cleaner_amd import cleaner, synth
    rng = np.random.default_rng(5)
    ar = synth.make_archive(10, 20, 8, seed=5)
    w = (rng.random((10, 20)) > 0.3).astype(np.float32)
    w[2, :15] = 0
    w[:6, 4] = 0
    for i in range(10):
        for j in range(20):
            ar.get_Integration(i).set_weight(j, float(w[i, j]))
    ns = cleaner.parse_arguments(["--bad_chan", "0.5", "--bad_subint", "0.5", "a.ar"])
    want, nsb, ncb = _bad_parts_expected(w, 0.5, 0.5)
    cleaner.find_bad_parts(ar, ns)
    assert np.array_equal(ar.get_weights(), want)
    assert capsys.readouterr().out == "Removed %d bad subintegrations and %d bad channels.\n" % (nsb, ncb)


def test_set_weights_archive_nan_never_zaps():
    """K5: test >= 1 zaps; NaN never does; inf does."""
    from iterative_cleaner_amd import cleaner, synth
    ar = synth.make_archive(2, 3, 8)
    test = np.array([[0.5, 1.0, np.nan], [np.inf, 0.999, 7.0]])
    cleaner.set_weights_archive(ar, test)
    w = ar.get_weights()
    assert np.array_equal(w == 0, np.array([[False, True, False], [True, False, True]]))


# ------------------------------------------------------------ C-ABI surface
def _declared_symbols():
    hdr = open(os.path.join(REPO, "include", "iterative_cleaner.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(ic_[a-z0-9_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    from iterative_cleaner_amd import _native
    lib = ctypes.CDLL(_native.LIB_PATH)
    syms = _declared_symbols()
    assert len(syms) >= 14
    for name in syms:
        assert hasattr(lib, name), name
    assert set(syms) == set(_native.EXPORTS)


def test_library_abi_version_and_error_path():
    """Loads through the product binding; argument errors need no GPU."""
    from iterative_cleaner_amd import _native
    lib = _native.load_library()
    assert lib.ic_abi_version() == _native.ABI_VERSION
    h = ctypes.c_void_p()
    bad = _native.Params(0, 4, 8, 5, 5.0, 5.0, 0, 1.0, 0, 0, 0.15, 0)
    assert lib.ic_session_create(ctypes.byref(bad), 0, ctypes.byref(h)) == -1
    assert b"bad shape" in lib.ic_last_error()


def test_library_is_gfx950_code_object():
    from iterative_cleaner_amd import _native
    blob = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_product_has_no_oracle_or_cpu_fallback():
    """The product package never imports the oracle."""
    pkg = os.path.join(REPO, "iterative_cleaner_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(root, f)).read()
                assert "oracle" not in src.replace("oracle/", ""), f


def test_schedule_options_match_header_and_no_environment_knobs():
    """Every IC_OPT_* of the header is bound under the same number, the library
    sources read no environment variable (schedules are session options,
    validated when set), and a null session is refused without a GPU."""
    from iterative_cleaner_amd import _native
    hdr = open(os.path.join(REPO, "include", "iterative_cleaner.h")).read()
    declared = {m.group(1).lower(): int(m.group(2))
                for m in re.finditer(r"#define IC_OPT_([A-Z0-9_]+) (\d+)", hdr)}
    assert declared == _native.OPTIONS
    csrc = os.path.join(REPO, "iterative_cleaner_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".h")):
            assert "getenv" not in open(os.path.join(csrc, f)).read(), f
    lib = _native.load_library()
    assert lib.ic_set_option(None, 1, 0) == -1
    v = ctypes.c_int64()
    assert lib.ic_get_option(None, 1, ctypes.byref(v)) == -1


def test_rccl_missing_library_is_an_error_code_not_a_crash():
    """ic_rccl_set_library on a file that does not exist: ic_rccl_unique_id
    returns IC_ECOMM with the failing path in the message (the
    dlerror() message used to be read twice, the second read a null
    std::string, an exception through the C-ABI).  A fresh process, because
    the library load is process-wide."""
    code = (
        "import ctypes, sys\n"
        "sys.path.insert(0, %r)\n"
        "from iterative_cleaner_amd import _native\n"
        "lib = _native.load_library()\n"
        "assert lib.ic_rccl_set_library(b'/nonexistent/dir/librccl_missing.so') == 0\n"
        "buf = ctypes.create_string_buffer(128)\n"
        "rc = lib.ic_rccl_unique_id(ctypes.cast(buf, ctypes.c_void_p))\n"
        "msg = lib.ic_last_error()\n"
        "assert rc == -5, rc\n"
        "assert b'/nonexistent/dir/librccl_missing.so' in msg, msg\n"
        "rc2 = lib.ic_rccl_unique_id(ctypes.cast(buf, ctypes.c_void_p))\n"
        "assert rc2 == -5, rc2\n"
        "print('ok')\n" % REPO)
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.returncode, r.stdout, r.stderr)
