"""CPU oracle for the multilinear hot path -- TEST INFRASTRUCTURE ONLY.

This package is the *checker*, never the thing measured or shipped.  Only
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import it.  The product path (``multilinear_amd``) never
imports or calls anything under ``oracle/`` and fails loudly when its HIP
library is missing.

Contents
--------
* ``field`` / ``transcript`` / ``ntt`` / ``merkle`` / ``fri`` /
  ``polynomials`` / ``sumcheck`` / ``pcs``: an exact pure-Python restatement
  of the reference algorithm (fr34za/multilinear @ 2025-06-20), each function
  citing the reference ``file:line`` it follows.  Python ints mod M and
  ``hashlib.sha256``; use it at sizes that finish in seconds.
* ``c/oracle.c`` -> ``liboracle.so``: a single-threaded C restatement of the
  same loops (``unsigned __int128`` arithmetic, its own SHA-256) used for the
  full-size on-box checks and as the ``cpu_baseline`` ("port").

Pinning status -- "parity unpinned" by reference-produced vectors
-----------------------------------------------------------------
The reference is Rust; ``cargo``/``rustc`` are absent and its crates
(winter-math 0.12.0, sha2 0.10.8) are not vendored, so it cannot be built or
run here, and its own tests hold **no** golden vectors (every test is a
round trip or prover->verifier self-consistency check).
The oracle is therefore pinned by:
  1. the reference's own self-consistency tests restated and passing
     (``intt(ntt(x)) == x``, Merkle open/verify, FRI prove->verify,
     PCS prove->verify, multilinear conversion round trip);
  2. published known answers of the third-party algorithms it depends on:
     FIPS 180-4 SHA-256 vectors, winter-math f128's published modulus and
     2^40-th root of unity;
  3. agreement of two independent restatements (this Python one and the C one).
No absolute field value or digest produced by the reference itself exists to
compare against: parity is unpinned in that sense.
"""
