"""TEST INFRASTRUCTURE ONLY -- the parity oracle for warpcore's checksum.

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  It is the checker, never the thing measured or shipped.

* :mod:`oracle.c_oracle` -- ctypes binding of the C restatement
  (wc_oracle.c; -Ofast -march=native, pthreads) used at full sizes and as the
  timed CPU baseline.
* :mod:`oracle.py_oracle` -- an independent pure-Python restatement (loops,
  small cases only) used to cross-check the C restatement.

Reference restated: /root/reference/lib/src/in_cksum.c:74-167.
Parity status: see wc_oracle.h and DESIGN.md section 3 ("parity unpinned"
against the reference except for the known answers in tests/golden/kat.json;
the standard arithmetic is also pinned by Linux-kernel-computed checksums in
tests/golden/linux_vectors.npz).
"""
