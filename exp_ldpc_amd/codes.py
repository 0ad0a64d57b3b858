"""Core code types and the ``qecc`` text format (host side).

Mirrors the reference's input API so callers of the decoding path see the same
objects:

* ``QuantumCodeChecks`` / ``QuantumCodeLogicals`` / ``QuantumCode``
  (``python/qldpc/qecc_util.py:19-118``): canonical, read-only CSR X/Z checks and
  dense logicals.
* ``read_quantum_code`` / ``write_quantum_code``
  (``python/qldpc/quantum_code_io.py:6-71``): the DIMACS-like ``qecc`` format the
  p-sweep loads (``misc/_experiment.py:231-235``).
* ``make_check_matrix`` (``qecc_util.py:146-149``).

Any ``scipy.sparse`` flavour (``*_matrix`` or ``*_array``) is accepted (SURVEY
Appendix B: modern scipy yields ``csr_array``).  Error behaviour (exception types
and when they are raised) follows the reference.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable
from warnings import warn

import numpy as np
import scipy.sparse as sp

__all__ = [
    "QuantumCodeChecks", "QuantumCodeLogicals", "QuantumCode", "CircuitTargets",
    "make_check_matrix", "read_quantum_code", "write_quantum_code", "num_rows", "num_cols",
]


def _require_integral(a) -> None:
    dt = a.dtype
    if not np.issubdtype(dt, np.integer):
        raise TypeError("Got numpy object with non-integral dtype")
    if np.issubdtype(dt, np.signedinteger):
        warn("Got numpy object with signed integer datatype. This could cause problems due when overflowing")


def _canonical_csr(m):
    m = m.tocsr(copy=True)
    m.sum_duplicates()
    m.sort_indices()
    m.eliminate_zeros()
    m.data.flags.writeable = False
    return m


def num_rows(a) -> int:
    assert len(a.shape) == 2
    return a.shape[0]


def num_cols(a) -> int:
    assert len(a.shape) == 2
    return a.shape[1]


@dataclass(frozen=True, init=False)
class QuantumCodeChecks:
    """X and Z check matrices (qecc_util.py:19-51): CSR, sorted, deduplicated,
    explicit zeros dropped, data read-only."""
    x: sp.spmatrix
    z: sp.spmatrix

    def __init__(self, x, z):
        x = _canonical_csr(sp.csr_matrix(x) if not sp.issparse(x) else x)
        z = _canonical_csr(sp.csr_matrix(z) if not sp.issparse(z) else z)
        _require_integral(x)
        _require_integral(z)
        if x.shape[1] != z.shape[1]:
            raise ValueError("x and z checks act on an inconsistent number of qubits")
        object.__setattr__(self, "x", x)
        object.__setattr__(self, "z", z)

    @property
    def num_qubits(self) -> int:
        return self.x.shape[1]


@dataclass(frozen=True)
class QuantumCodeLogicals:
    """Logical operators, one per row (qecc_util.py:53-91): dense arrays as in
    the reference, or scipy sparse matrices (an extension for codes with
    thousands of sparse logicals, e.g. config 5's k = 4080 of weight 3, whose
    dense form is 866 MB; stored as a private CSR copy)."""
    x: np.ndarray
    z: np.ndarray

    def __post_init__(self):
        for name in ("x", "z"):
            a = getattr(self, name)
            if sp.issparse(a):
                object.__setattr__(self, name, sp.csr_matrix(a, copy=True))
        _require_integral(self.x)
        _require_integral(self.z)
        if self.x.shape[1] != self.z.shape[1]:
            raise ValueError("x and z logicals act on an inconsistent number of qubits")
        if self.x.shape[0] != self.z.shape[0]:
            raise ValueError("Number of provided X and Z logical operators mismatch")
        for a in (self.x, self.z):
            if not sp.issparse(a):
                a.flags.writeable = False

    @property
    def num_qubits(self) -> int:
        return self.x.shape[1]

    @property
    def num_logicals(self) -> int:
        return self.x.shape[0]

    @staticmethod
    def empty(num_qubits: int) -> "QuantumCodeLogicals":
        return QuantumCodeLogicals(np.zeros((0, num_qubits), dtype=np.uint32),
                                   np.zeros((0, num_qubits), dtype=np.uint32))


@dataclass(frozen=True, init=False)
class QuantumCode:
    checks: QuantumCodeChecks
    logicals: QuantumCodeLogicals

    def __init__(self, checks: QuantumCodeChecks, logicals: QuantumCodeLogicals | None = None):
        if logicals is None:
            logicals = QuantumCodeLogicals.empty(checks.num_qubits)
        if checks.num_qubits != logicals.num_qubits:
            raise ValueError("Number of qubits for checks and logicals is inconsistent")
        object.__setattr__(self, "checks", checks)
        object.__setattr__(self, "logicals", logicals)

    @property
    def num_qubits(self) -> int:
        return self.checks.num_qubits

    @property
    def num_logicals(self) -> int:
        return self.logicals.num_logicals


@dataclass(frozen=True, init=False)
class CircuitTargets:
    """Qubit index groups of the storage experiment (qecc_util.py:120-131)."""
    data: list
    x_checks: list
    z_checks: list
    ancillas: list

    def __init__(self, data, x_checks, z_checks):
        object.__setattr__(self, "data", list(data))
        object.__setattr__(self, "x_checks", list(x_checks))
        object.__setattr__(self, "z_checks", list(z_checks))
        object.__setattr__(self, "ancillas", list(x_checks) + list(z_checks))


def make_check_matrix(checks: Iterable[Iterable[int]], num_qubits: int) -> sp.csr_matrix:
    """Sparse 0/1 matrix whose row i has ones at ``checks[i]`` (qecc_util.py:146-149)."""
    checks = [list(r) for r in checks]
    rows = np.fromiter((i for i, r in enumerate(checks) for _ in r), dtype=np.int64)
    cols = np.fromiter((c for r in checks for c in r), dtype=np.int64)
    data = np.ones(rows.size, dtype=np.uint32)
    return sp.csr_matrix((data, (rows, cols)), shape=(len(checks), num_qubits), dtype=np.uint32)


_KINDS = ("X", "Z", "LX", "LZ")


def read_quantum_code(stream, validate_stabilizer_code=None) -> QuantumCode:
    """Parse the ``qecc`` format (quantum_code_io.py:6-62).

    Header ``qecc <qubits> <#X> <#Z> <#logicals>``; then one line per support
    ending with its kind (X, Z, LX, LZ); lines starting with ``c`` are comments.
    """
    if validate_stabilizer_code is None:
        validate_stabilizer_code = True
    raw = stream.readlines()
    lines = [l.split() for l in raw if not l.startswith("c")]
    lines = [l for l in lines if l]
    if not lines or lines[0][0] != "qecc" or len(lines[0]) != 5:
        raise RuntimeError("Invalid header. Expected qecc <# qubits> <# X checks> <# Z checks> <# logicals>")
    nq, nx, nz, nl = (int(v) for v in lines[0][1:])
    if nx + nz > nq:
        raise RuntimeError(f"Code overconstrained. Got {nx + nz} checks on {nq} qubits")
    rows = {k: [] for k in _KINDS}
    for l in lines[1:]:
        kind = l[-1]
        if kind not in rows:
            raise RuntimeError(f"Invalid check/logical type in line: \n {l}")
        support = [int(v) for v in l[:-1]]
        if any(v >= nq for v in support):
            raise RuntimeError(f"Out of bounds check support: \n {l}")
        rows[kind].append(support)
    if len(rows["X"]) + len(rows["Z"]) != nx + nz:
        raise RuntimeError(f"Number of checks does not match header. Expected {nx} + {nz}. "
                           f"Got {len(rows['X'])} + {len(rows['Z'])}")
    if len(rows["LZ"]) != len(rows["LX"]):
        raise RuntimeError(f"Number of X and Z logicals does not match: {len(rows['LX'])} X logicals "
                           f"and {len(rows['LZ'])} Z logicals")
    if len(rows["LZ"]) != nl:
        raise RuntimeError(f"Parsed number of logicals does not match header. Expected {nl}. Got {len(rows['LZ'])}")

    checks = QuantumCodeChecks(make_check_matrix(rows["X"], nq), make_check_matrix(rows["Z"], nq))
    logicals = QuantumCodeLogicals(make_check_matrix(rows["LX"], nq).toarray(),
                                   make_check_matrix(rows["LZ"], nq).toarray())
    if validate_stabilizer_code:
        if np.any((checks.x @ checks.z.T).toarray() % 2):
            raise RuntimeError("X and Z checks do not generate an abelian group")
        if logicals.num_logicals > 0:
            if np.any((checks.x @ logicals.z.T) % 2):
                raise RuntimeError("Z logicals do not commute with X checks")
            if np.any((checks.z @ logicals.x.T) % 2):
                raise RuntimeError("X logicals do not commute with Z checks")
    return QuantumCode(checks, logicals)


def write_quantum_code(stream, code: QuantumCode) -> None:
    """Write the ``qecc`` format (quantum_code_io.py:64-71): X, Z, LZ, LX sections,
    supports in ascending column order."""
    stream.write(f"qecc {code.num_qubits} {num_rows(code.checks.x)} {num_rows(code.checks.z)} "
                 f"{code.num_logicals}\n")
    for kind, mat in (("X", code.checks.x), ("Z", code.checks.z),
                      ("LZ", code.logicals.z), ("LX", code.logicals.x)):
        csr = sp.csr_matrix(mat, copy=True)
        csr.sum_duplicates()
        csr.sort_indices()
        csr.eliminate_zeros()
        for i in range(csr.shape[0]):
            cols = csr.indices[csr.indptr[i]:csr.indptr[i + 1]]
            stream.write(" ".join(str(int(c)) for c in cols) + f" {kind}\n")
