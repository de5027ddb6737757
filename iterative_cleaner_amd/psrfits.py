"""Minimal fold-mode PSRFITS reader/writer for the archive stand-in
(reference load/unload sites iterative_cleaner.py:47,
:60, :150, :162).  astropy and fitsio are not available, so the FITS layer is
hand-rolled: 2880-byte blocks, 80-character header cards, a primary HDU and
one big-endian BINTABLE extension EXTNAME = 'SUBINT' with the PSRFITS fold-mode
columns

    TSUBINT, OFFS_SUB, PERIOD (1D)   DAT_FREQ (nchan D)   DAT_WTS (nchan E)
    DAT_OFFS, DAT_SCL (npol*nchan E)  DATA (nbin*nchan*npol I, TDIM (nbin,nchan,npol))

Samples are int16 with a per-(subint, pol, channel) scale and offset:
value = f32(f32(DATA) * DAT_SCL + DAT_OFFS), the decoding psrchive applies.
The stand-in's own metadata rides in extra keywords / one extra column that
other PSRFITS readers ignore: IC_SHIFT (nchan J, integer dedispersion delays in
bins), IC_DELAY (nchan D per row, fractional delays in bins of an archive
dedispersed by FFT phase rotation; rows that differ are per-profile delays),
IC_DEDSP (dedispersed flag), IC_DUTY (baseline duty), IC_MJDE (end MJD).  Files
without IC_SHIFT (a foreign writer's) are dedispersed as psrchive would:
delays from DM, DAT_FREQ, OBSFREQ and each row's PERIOD (dedispersion.py),
integer shifts when every delay is integral, else the fractional FFT rotation
(an error at an nbin it cannot serve, never a silent rounding).
"""
from __future__ import annotations

import numpy as np

BLOCK = 2880
CARD = 80
MAGIC = b"SIMPLE  ="
_CODES = {"L": ("u1", 1), "B": ("u1", 1), "I": (">i2", 2), "J": (">i4", 4), "K": (">i8", 8),
          "E": (">f4", 4), "D": (">f8", 8), "A": ("S1", 1)}


def is_psrfits(path: str) -> bool:
    with open(path, "rb") as fh:
        return fh.read(len(MAGIC)) == MAGIC


# ------------------------------------------------------------------ header cards
def _fmt_value(v) -> str:
    if isinstance(v, bool):
        return "%20s" % ("T" if v else "F")
    if isinstance(v, (int, np.integer)):
        return "%20d" % int(v)
    if isinstance(v, (float, np.floating)):
        s = repr(float(v)).upper()
        if "E" not in s and "." not in s and "N" not in s:
            s += ".0"
        return "%20s" % s
    s = str(v).replace("'", "''")
    return "'%-8s'" % s


def _card(key: str, value=None, comment: str = "") -> bytes:
    if key == "END":
        return b"END".ljust(CARD)
    text = "%-8s= %s" % (key, _fmt_value(value))
    if comment:
        text += " / " + comment
    if len(text) > CARD:
        raise ValueError("FITS card too long: %r" % text)
    return text.ljust(CARD).encode("ascii")


def _header(cards) -> bytes:
    raw = b"".join(_card(*c) for c in cards) + _card("END")
    return raw + b" " * (-len(raw) % BLOCK)


def _parse_value(s: str):
    s = s.strip()
    if s.startswith("'"):
        out, i = [], 1
        while i < len(s):
            if s[i] == "'":
                if i + 1 < len(s) and s[i + 1] == "'":
                    out.append("'")
                    i += 2
                    continue
                break
            out.append(s[i])
            i += 1
        return "".join(out).rstrip()
    v = s.split("/")[0].strip()
    if v in ("T", "F"):
        return v == "T"
    try:
        return int(v)
    except ValueError:
        pass
    try:
        return float(v.replace("D", "E"))
    except ValueError:
        return v


def _read_header(fh) -> dict | None:
    hdr = {}
    while True:
        block = fh.read(BLOCK)
        if len(block) < BLOCK:
            return None if not hdr else hdr
        for i in range(0, BLOCK, CARD):
            card = block[i:i + CARD].decode("ascii", "replace")
            key = card[:8].strip()
            if key == "END":
                return hdr
            if card[8:10] == "= ":
                hdr[key] = _parse_value(card[10:])


def _data_bytes(hdr: dict) -> int:
    naxis = int(hdr.get("NAXIS", 0))
    if naxis == 0:
        return 0
    n = abs(int(hdr.get("BITPIX", 8))) // 8
    for i in range(1, naxis + 1):
        n *= int(hdr["NAXIS%d" % i])
    return n * int(hdr.get("GCOUNT", 1)) + int(hdr.get("PCOUNT", 0))


# ------------------------------------------------------------------ quantisation
def quantise(data: np.ndarray):
    """(nsub, npol, nchan, nbin) f32 -> (DATA i16, SCL f32, OFFS f32) per
    (subint, pol, chan); decode() of the result is within SCL/2 of data."""
    d = np.asarray(data, np.float32)
    mn = d.min(axis=3)
    mx = d.max(axis=3)
    offs = (0.5 * (mx.astype(np.float64) + mn)).astype(np.float32)
    scl = ((mx.astype(np.float64) - mn) / 65534.0).astype(np.float32)
    scl = np.where((scl > 0) & np.isfinite(scl), scl, np.float32(1.0)).astype(np.float32)
    q = np.rint((d.astype(np.float64) - offs[..., None]) / scl[..., None])
    q = np.clip(np.nan_to_num(q), -32767, 32767).astype(np.int16)
    return q, scl, offs


# psrchive state <-> PSRFITS POL_TYPE (fold-mode SUBINT keyword)
STATE_POL_TYPE = {"Intensity": "AA+BB", "PPQQ": "AABB", "Coherence": "AABBCRCI", "Stokes": "IQUV"}
POL_TYPE_STATE = {"AA+BB": "Intensity", "INTEN": "Intensity", "I": "Intensity", "AABB": "PPQQ",
                  "AABBCRCI": "Coherence", "IQUV": "Stokes"}


def decode(q: np.ndarray, scl: np.ndarray, offs: np.ndarray) -> np.ndarray:
    return (q.astype(np.float32) * scl[..., None] + offs[..., None]).astype(np.float32)


# ------------------------------------------------------------------ write
def save(ar, path: str, stand_in_meta: bool = True) -> None:
    """Write `ar` as fold-mode PSRFITS (stand_in_meta=False: standard columns
    and keywords only, as a foreign writer would produce)."""
    data = ar._data
    nsub, npol, nchan, nbin = data.shape
    q = getattr(ar, "_psrfits_q", None)
    if q is None or q[0].shape != data.shape or not np.array_equal(decode(*q), data):
        q = quantise(data)
    qd, scl, offs = q
    cfreq = float(ar.get_centre_frequency())
    freqs = getattr(ar, "_chan_freqs", None)
    if freqs is None or len(freqs) != nchan:
        freqs = cfreq + (np.arange(nchan) - (nchan - 1) / 2.0) * 1.0
    period = np.broadcast_to(np.asarray(getattr(ar, "_period", 1.0), np.float64), (nsub,))
    tsub = float(getattr(ar, "_tsubint", 10.0))
    cols = [("TSUBINT", "1D", None, (nsub,), np.full(nsub, tsub)),
            ("OFFS_SUB", "1D", None, (nsub,), (np.arange(nsub) + 0.5) * tsub),
            ("PERIOD", "1D", None, (nsub,), period),
            ("DAT_FREQ", "%dD" % nchan, None, (nsub, nchan), np.broadcast_to(freqs, (nsub, nchan))),
            ("DAT_WTS", "%dE" % nchan, None, (nsub, nchan), ar._weights),
            ("DAT_OFFS", "%dE" % (nchan * npol), None, (nsub, npol * nchan), offs.reshape(nsub, -1)),
            ("DAT_SCL", "%dE" % (nchan * npol), None, (nsub, npol * nchan), scl.reshape(nsub, -1)),
            ("DATA", "%dI" % (nbin * nchan * npol), "(%d,%d,%d)" % (nbin, nchan, npol),
             (nsub, npol * nchan * nbin), qd.reshape(nsub, -1)),
            ("IC_SHIFT", "%dJ" % nchan, None, (nsub, nchan), np.broadcast_to(ar._shift, (nsub, nchan)))]
    if getattr(ar, "_delay", None) is not None:
        cols.append(("IC_DELAY", "%dD" % nchan, None, (nsub, nchan), np.broadcast_to(ar._delay, (nsub, nchan))))
    if not stand_in_meta:
        cols = cols[:8]
    fields = []
    for name, form, _, _, _ in cols:
        rep = int(form[:-1] or 1)
        code = _CODES[form[-1]][0]
        fields.append((name, code, (rep,)) if rep > 1 else (name, code))
    dt = np.dtype(fields)
    rows = np.zeros(nsub, dtype=dt)
    for name, form, _, shape, val in cols:
        rows[name] = np.asarray(val).reshape(shape)
    mjd0 = float(ar.start_time().in_days())
    imjd = int(np.floor(mjd0))
    smjd = (mjd0 - imjd) * 86400.0
    pol_type = STATE_POL_TYPE.get(ar.get_state(), "AABB")
    primary = [("SIMPLE", True), ("BITPIX", 8), ("NAXIS", 0), ("EXTEND", True),
               ("FITSTYPE", "PSRFITS"), ("HDRVER", "6.1"), ("OBS_MODE", "PSR"),
               ("TELESCOP", "SYNTH"), ("SRC_NAME", ar.get_source()), ("OBSFREQ", cfreq),
               ("OBSBW", float(nchan)), ("OBSNCHAN", nchan), ("STT_IMJD", imjd),
               ("STT_SMJD", int(smjd)), ("STT_OFFS", smjd - int(smjd))]
    sub = [("XTENSION", "BINTABLE"), ("BITPIX", 8), ("NAXIS", 2), ("NAXIS1", dt.itemsize),
           ("NAXIS2", nsub), ("PCOUNT", 0), ("GCOUNT", 1), ("TFIELDS", len(cols))]
    for i, (name, form, tdim, _, _) in enumerate(cols, 1):
        sub.append(("TTYPE%d" % i, name))
        sub.append(("TFORM%d" % i, form))
        if tdim:
            sub.append(("TDIM%d" % i, tdim))
    sub += [("EXTNAME", "SUBINT"), ("INT_TYPE", "TIME"), ("INT_UNIT", "SEC"), ("NPOL", npol),
            ("POL_TYPE", pol_type), ("NBIN", nbin), ("NCHAN", nchan), ("CHAN_BW", 1.0),
            ("DM", float(getattr(ar, "_dm", 0.0))), ("RM", 0.0), ("NCHNOFFS", 0), ("NSBLK", 1)]
    if stand_in_meta:
        sub += [("IC_DEDSP", bool(ar.get_dedispersed())), ("IC_DUTY", float(ar.get_baseline_duty())),
                ("IC_MJDE", float(ar.end_time().in_days()))]
    body = rows.tobytes()
    with open(path, "wb") as fh:
        fh.write(_header(primary))
        fh.write(_header(sub))
        fh.write(body)
        fh.write(b"\0" * (-len(body) % BLOCK))


# ------------------------------------------------------------------ read
def _columns(hdr: dict):
    fields, tdims = [], {}
    for i in range(1, int(hdr["TFIELDS"]) + 1):
        name = hdr["TTYPE%d" % i]
        form = str(hdr["TFORM%d" % i]).strip()
        rep = int(form[:-1]) if form[:-1] else 1
        code = form[-1]
        if code not in _CODES:
            raise ValueError("unsupported TFORM %r" % form)
        base = _CODES[code][0]
        if code == "A":
            fields.append((name, "S%d" % rep))
        else:
            fields.append((name, base, (rep,)) if rep > 1 else (name, base))
        if "TDIM%d" % i in hdr:
            tdims[name] = tuple(int(x) for x in str(hdr["TDIM%d" % i]).strip("() ").split(","))
    return np.dtype(fields), tdims


def probe_shape(path: str):
    """(nsub, npol, nchan, nbin) from the SUBINT header alone."""
    with open(path, "rb") as fh:
        primary = _read_header(fh)
        if not primary or primary.get("SIMPLE") is not True:
            raise ValueError("%s: not a FITS file" % path)
        fh.seek(_data_bytes(primary) + (-_data_bytes(primary) % BLOCK), 1)
        while True:
            hdr = _read_header(fh)
            if hdr is None:
                raise ValueError("%s: no SUBINT table" % path)
            if hdr.get("EXTNAME") == "SUBINT":
                return int(hdr["NAXIS2"]), int(hdr["NPOL"]), int(hdr["NCHAN"]), int(hdr["NBIN"])
            n = _data_bytes(hdr)
            fh.seek(n + (-n % BLOCK), 1)


def load(path: str, channels=None):
    """Read a fold-mode PSRFITS archive.  channels = (c0, c1): only those
    channels; the SUBINT table is memory-mapped, so the other channels' samples
    are never read (channel-sharded cleaning)."""
    from .archive import Archive
    with open(path, "rb") as fh:
        primary = _read_header(fh)
        if not primary or primary.get("SIMPLE") is not True:
            raise ValueError("%s: not a FITS file" % path)
        fh.seek(_data_bytes(primary) + (-_data_bytes(primary) % BLOCK), 1)
        while True:
            hdr = _read_header(fh)
            if hdr is None:
                raise ValueError("%s: no SUBINT table" % path)
            n = _data_bytes(hdr)
            if hdr.get("EXTNAME") == "SUBINT":
                table_offset = fh.tell()
                break
            fh.seek(n + (-n % BLOCK), 1)
    dt, tdims = _columns(hdr)
    if dt.itemsize != int(hdr["NAXIS1"]):
        raise ValueError("%s: row size %d != NAXIS1 %d" % (path, dt.itemsize, hdr["NAXIS1"]))
    nsub = int(hdr["NAXIS2"])
    rows = np.memmap(path, dtype=dt, mode="r", offset=table_offset, shape=(nsub,))
    npol, nchan_total, nbin = int(hdr["NPOL"]), int(hdr["NCHAN"]), int(hdr["NBIN"])
    c0, c1 = (0, nchan_total) if channels is None else (int(channels[0]), int(channels[1]))
    if not 0 <= c0 < c1 <= nchan_total:
        raise ValueError("%s: channel range %s outside [0, %d)" % (path, (c0, c1), nchan_total))
    nchan = c1 - c0
    q = np.array(rows["DATA"].reshape(nsub, npol, nchan_total, nbin)[:, :, c0:c1], np.int16)
    scl = np.array(rows["DAT_SCL"].reshape(nsub, npol, nchan_total)[:, :, c0:c1], np.float32)
    offs = np.array(rows["DAT_OFFS"].reshape(nsub, npol, nchan_total)[:, :, c0:c1], np.float32)
    weights = np.array(rows["DAT_WTS"].reshape(nsub, nchan_total)[:, c0:c1], np.float32)
    freqs = np.array(rows["DAT_FREQ"].reshape(nsub, nchan_total)[0, c0:c1], np.float64) \
        if "DAT_FREQ" in dt.names else None
    period = np.array(rows["PERIOD"], np.float64).reshape(nsub) if "PERIOD" in dt.names \
        else np.ones(nsub, np.float64)
    cfreq = float(primary.get("OBSFREQ", 1400.0))
    dm = float(hdr.get("DM", 0.0))
    frac = None
    if "IC_DELAY" in dt.names:
        frac = np.array(rows["IC_DELAY"].reshape(nsub, nchan_total)[:, c0:c1], np.float64)
        if np.all(frac == frac[:1]):
            frac = np.ascontiguousarray(frac[0])
    if "IC_SHIFT" in dt.names:
        shift = np.array(rows["IC_SHIFT"].reshape(nsub, nchan_total)[0, c0:c1], np.int64)
    elif freqs is not None:
        # a foreign writer's file: psrchive's delays (DM, channel frequency, each
        # row's folding period) over the WHOLE band, then this slice's channels
        from . import dedispersion
        allf = np.array(rows["DAT_FREQ"].reshape(nsub, nchan_total)[0], np.float64)
        delay = dedispersion.delays_from_dm(dm, allf, cfreq, period, nbin)[:, c0:c1]
        shift, frac = dedispersion.plan(delay, nbin, path)
    else:
        shift = np.zeros(nchan, np.int64)
    mjd0 = float(primary.get("STT_IMJD", 60000)) + (float(primary.get("STT_SMJD", 0))
                                                     + float(primary.get("STT_OFFS", 0.0))) / 86400.0
    pol_type = str(hdr.get("POL_TYPE", "")).strip().upper()
    state = POL_TYPE_STATE.get(pol_type) if pol_type else None
    if state is not None and (state == "Intensity") != (npol == 1):
        state = None          # inconsistent header: fall back on the npol default
    del rows
    ar = Archive(decode(q, scl, offs), weights, shift, dedispersed=bool(hdr.get("IC_DEDSP", False)),
                 filename=path, source=str(primary.get("SRC_NAME", "J0000+0000")),
                 centre_frequency=cfreq, mjd_start=mjd0,
                 mjd_end=float(hdr.get("IC_MJDE", mjd0 + 0.01)),
                 baseline_duty=float(hdr.get("IC_DUTY", 0.15)), state=state, dm_delay=frac)
    if channels is not None:
        ar._chan_range = (c0, c1)
        ar._nchan_total = nchan_total
    ar._psrfits_q = (q, scl, offs)
    ar._format = "PSRFITS"
    ar._chan_freqs = freqs
    ar._period = period if np.any(period != period[:1]) else float(period[0])
    ar._dm = dm
    return ar
