"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

This package restates the reference algorithm (iterative_cleaner.py:65-146,
:181-305) on the CPU so that the HIP path can be checked against it.  It is
imported only by ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` — never by the product package
``iterative_cleaner_amd`` (which fails loudly when its HIP library is
missing instead of falling back to anything here).

Contents
  restated.py        numpy restatement of the statistics (numpy.ma semantics
                     written out explicitly) and of numpy's pairwise sums
  reference_like.py  the reference's loop with its own library calls
                     (scipy.optimize.leastsq per profile, numpy.ma) — the
                     CPU baseline ("port") timed by bench.py
  ic_oracle.c        C restatement: exact n=1 MINPACK lmdif, the stand-in
                     template, residual, diagnostics, scalers, the loop
  lib.py             ctypes binding of ic_oracle.c (libic_oracle.so)

Pinning: every piece is checked against golden fixtures produced by running
the reference itself in the build container (tests/golden/make_golden.py)
and, for lmdif, against scipy 1.15.3 directly.
"""
