"""CPU oracle for the decoding hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package; it is the checker, never the product.  The product
path (``exp_ldpc_amd``) does not import it and fails loudly without its HIP
library.

Contents:
* ``libqdec_oracle.so`` (built by ``oracle/Makefile``): a plain-C restatement of
  ldpc v1's BP loops (min-sum-log and product-sum, fp64 = ldpc, fp32 = this
  build's single-precision variant), the build-defined SSF (brute force), the
  final-correction fold, the logical check and the Philox storage sampler.
* ``ldpc_py``: a pure-Python line-by-line restatement of the same BP loops used to
  cross-check the C oracle on small cases.

Parity status (also in DESIGN.md): BP is pinned to the *published algorithm* of
ldpc v1 only -- ``ldpc`` itself is absent, so BP parity against ldpc is
UNPINNED; SSF has no reference implementation (build-defined, known-answer
tests); code construction, I/O, spacetime matrices, syndrome differencing, the
fold and the storage-circuit structure are pinned to fixtures generated from the
reference (tests/golden/make_golden.py).
"""
from .cpu import OracleLib, load, build  # noqa: F401
