"""Seeded synthetic archives.

p[s,c,:] = g[s,c] * pulse + n, float32, in the DISPERSED frame:
  pulse   Gaussian at phase 0.3, sigma 0.02 phase (dedispersed frame),
          delayed by dm_shift[c] = c mod 7 bins in channel c
  g       Gamma(shape 2, scale 0.5) scintillation gain per profile
  n       N(0, 1)
  narrowband RFI in a fraction f of channels: 5*N(0,1)*sin(2 pi nu phi),
          nu ~ U(1, 20) per channel, amplitude per (subint, channel)
  impulsive RFI in a fraction f of subints: +20 spikes, 1 % of samples
  2 % of channels carry w0 = 0
"""
from __future__ import annotations

import numpy as np

from .archive import Archive

CONFIGS = {
    # name: (nsub, nchan, nbin, seed, rfi_frac)
    "C1": (64, 256, 256, 0, 0.05),
    "C2": (360, 3200, 1024, 1, 0.05),
    "C3": (1024, 8192, 1024, 2, 0.05),
    "C4": (128, 1024, 512, 1000, 0.05),
    "C5": (256, 1024, 4096, 58, 0.30),   # seed 58: the loop runs to max_iter (tools/c5_seed_search.py)
}


def make_cube(nsub, nchan, nbin, seed=0, rfi_frac=0.05, npol=1, dead_frac=0.02):
    """Return (data f32 (nsub,npol,nchan,nbin), weights f32, dm_shift i64)."""
    rng = np.random.default_rng(seed)
    phase = (np.arange(nbin, dtype=np.float64) + 0.5) / nbin
    pulse = np.exp(-0.5 * ((phase - 0.3) / 0.02) ** 2)
    shift = (np.arange(nchan) % 7).astype(np.int64)
    g = rng.gamma(2.0, 0.5, size=(nsub, nchan))
    data = rng.standard_normal((nsub, nchan, nbin), dtype=np.float32)
    idx = (np.arange(nbin)[None, :] - shift[:, None]) % nbin   # dispersed = roll(ded, +shift)
    data += (g[:, :, None] * pulse[idx][None, :, :]).astype(np.float32)
    n_nb = int(round(rfi_frac * nchan))
    if n_nb:
        chans = rng.choice(nchan, size=n_nb, replace=False)
        nu = rng.uniform(1.0, 20.0, size=n_nb)
        amp = 5.0 * rng.standard_normal((nsub, n_nb))
        wave = np.sin(2.0 * np.pi * nu[:, None] * phase[None, :])
        data[:, chans, :] += (amp[:, :, None] * wave[None, :, :]).astype(np.float32)
    n_imp = int(round(rfi_frac * nsub))
    if n_imp:
        subs = rng.choice(nsub, size=n_imp, replace=False)
        hits = rng.random((n_imp, nchan, nbin)) < 0.01
        data[subs] += np.where(hits, np.float32(20.0), np.float32(0.0))
    weights = np.ones((nsub, nchan), dtype=np.float32)
    n_dead = int(round(dead_frac * nchan))
    if n_dead:
        weights[:, rng.choice(nchan, size=n_dead, replace=False)] = 0.0
    if npol > 1:
        # split into AA, BB (+ cross terms) so pscrunch (AA+BB) sums back close to the cube
        half = (data * np.float32(0.5)).astype(np.float32)
        pols = [half, (data - half).astype(np.float32)]
        for _ in range(npol - 2):
            pols.append(rng.standard_normal(data.shape, dtype=np.float32))
        data4 = np.stack(pols, axis=1)
    else:
        data4 = data[:, None]
    return np.ascontiguousarray(data4), weights, shift


def fractional_weights(w):
    """A deterministic edit putting non-dyadic fractional weights (0.3, 0.7) and
    0.5 on some live profiles (apply_weights multiplies by them, ic.py:296)."""
    w = np.array(w, dtype=np.float32, copy=True)
    nsub, nchan = w.shape
    for s in range(nsub):
        for c in range((s * 7) % 5, nchan, 5):
            if w[s, c] != 0:
                w[s, c] = (0.3, 0.7, 0.5)[(s + c) % 3]
    return w


def fractional_delays(shift, nbin):
    """Deterministic fractional per-channel delays in bins near the integer
    shifts (dedispersion by FFT phase rotation, phase_rotation.py): shift[c]
    + 0.45 sin(1.3 c), plus whole turns on every 5th channel (the rotation
    depends on the delay modulo nbin only)."""
    c = np.arange(len(shift))
    return (np.asarray(shift, dtype=np.float64) + 0.45 * np.sin(1.3 * c)
            + np.where(c % 5 == 4, 3.0 * nbin, 0.0))


def per_profile_delays(shift, nbin, nsub):
    """Deterministic per-(subint, channel) delays: :func:`fractional_delays`
    scaled by P_0 / P_s for a folding period that drifts by up to 2e-4 across
    the subints, as psrchive's per-Integration dedispersion sees it
    (delay[s, c] = dm_delay_c / P_s * nbin)."""
    s = np.arange(nsub)
    scale = 1.0 + 2e-4 * np.sin(0.7 * s + 0.3)
    return fractional_delays(shift, nbin)[None, :] * scale[:, None]


def make_archive(nsub, nchan, nbin, seed=0, rfi_frac=0.05, npol=1,
                 filename="synthetic.ar", **kw) -> Archive:
    data, weights, shift = make_cube(nsub, nchan, nbin, seed, rfi_frac, npol, **kw)
    return Archive(data, weights, shift, dedispersed=False, filename=filename)


def make_config(name: str, npol=1, filename=None) -> Archive:
    nsub, nchan, nbin, seed, f = CONFIGS[name]
    return make_archive(nsub, nchan, nbin, seed, f, npol,
                        filename=filename or ("%s.ar" % name))
