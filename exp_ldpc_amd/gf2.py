"""GF(2) linear algebra on bit-packed numpy rows (host-side, offline only).

Replaces the reference's use of the third-party ``galois`` package (v0.3.5, absent
from this image) for the two jobs the decoding path needs:

* the logical operators of a CSS code (reference ``get_logicals``,
  ``python/qldpc/homological_product_code.py:37-60``, which uses galois
  ``null_space`` / ``column_space`` / ``row_reduce``), and
* ranks for test assertions (reference ``get_rank``, ``python/qldpc/linalg.py:98-99``).

Rows are packed little-endian into uint64 words.  The elimination itself runs in
the host library (``qd_gf2_rref`` / ``qd_gf2_extend_basis``,
``csrc/qdec_gf2.cpp``, threaded over rows) when ``libqdec_hip.so`` is built --
it loads without a GPU -- so the 10^4..5*10^4-qubit codes of BASELINE configs 4
and 5 get their logicals in seconds; a numpy loop is kept for environments
without the library (code construction is offline tooling, not the decode
path).  Nothing here runs on the GPU: it produces fixtures and the dense ``Lz``
table that the logical-check kernel consumes.
"""
from __future__ import annotations

import numpy as np

__all__ = [
    "pack_rows", "unpack_rows", "row_reduce", "rank", "null_space",
    "homology_representatives", "pair_logicals", "css_logicals",
]


def pack_rows(a) -> np.ndarray:
    """Pack a dense 0/1 (r, n) array into (r, ceil(n/64)) uint64, bit j of row i at
    word j//64, bit j%64."""
    a = np.asarray(a)
    if a.ndim != 2:
        raise ValueError("expected a 2-d array")
    r, n = a.shape
    words = (n + 63) // 64
    bits = (a % 2).astype(np.uint8)
    padded = np.zeros((r, words * 64), dtype=np.uint8)
    padded[:, :n] = bits
    by = np.packbits(padded.reshape(r, words * 8, 8), axis=2, bitorder="little").reshape(r, words * 8)
    return by.view(np.uint64).reshape(r, words).copy()


def unpack_rows(p: np.ndarray, n: int) -> np.ndarray:
    """Inverse of :func:`pack_rows`."""
    r, words = p.shape
    by = np.ascontiguousarray(p).view(np.uint8).reshape(r, words * 8)
    bits = np.unpackbits(by, axis=1, bitorder="little")
    return bits[:, :n].astype(np.uint8)


def _bit(p: np.ndarray, col: int) -> np.ndarray:
    return (p[:, col >> 6] >> np.uint64(col & 63)) & np.uint64(1)


def _native():
    try:
        from . import _abi
        return _abi.load()
    except Exception:
        return None


def _rref_packed(p: np.ndarray, n: int, limit: int):
    """In-place RREF of packed rows over columns [0, limit); returns (rank, pivots)."""
    lib = _native()
    r = p.shape[0]
    if lib is not None and r and p.shape[1]:
        p = np.ascontiguousarray(p)
        piv = np.zeros(max(r, 1), dtype=np.int64)
        rank = int(lib.qd_gf2_rref(p.ctypes.data, r, p.shape[1], limit, piv.ctypes.data, 0))
        if rank < 0:
            raise ValueError("qd_gf2_rref: bad arguments")
        return p, rank, piv[:rank].copy()
    pivots = []
    row = 0
    for col in range(limit):
        if row >= r:
            break
        colbits = _bit(p[row:], col)
        hits = np.nonzero(colbits)[0]
        if hits.size == 0:
            continue
        piv = row + hits[0]
        if piv != row:
            p[[row, piv]] = p[[piv, row]]
        mask = _bit(p, col).astype(bool)
        mask[row] = False
        if mask.any():
            p[mask] ^= p[row]
        pivots.append(col)
        row += 1
    return p, row, np.array(pivots, dtype=np.int64)


def row_reduce(a, ncols: int | None = None):
    """Reduced row echelon form over GF(2).

    Pivots are searched in columns ``0 .. ncols-1`` (all columns by default).
    Returns ``(rref_dense, pivot_columns)`` with zero rows dropped.
    """
    a = np.asarray(a) % 2
    r, n = a.shape
    limit = n if ncols is None else ncols
    p, rank, piv = _rref_packed(pack_rows(a), n, limit)
    return unpack_rows(p[:rank], n), piv


def rank(a) -> int:
    a = np.asarray(a)
    if a.size == 0:
        return 0
    return int(row_reduce(a)[0].shape[0])


def null_space(a) -> np.ndarray:
    """Basis (rows) of ``{x : a x = 0}`` over GF(2)."""
    a = np.asarray(a) % 2
    n = a.shape[1]
    rref, piv = row_reduce(a)
    free = np.setdiff1d(np.arange(n), piv)
    basis = np.zeros((free.size, n), dtype=np.uint8)
    for t, f in enumerate(free):
        basis[t, f] = 1
        if piv.size:
            basis[t, piv] = rref[:, f]
    return basis


def homology_representatives(image_rows, kernel_rows) -> np.ndarray:
    """Rows of ``kernel_rows`` that extend a basis of span(image_rows) to a basis of
    span(kernel_rows) (same construction as the reference's
    ``compute_homology_reps``, homological_product_code.py:10-25: reduce
    [image; kernel] and keep the kernel rows that add a pivot)."""
    image_rows = np.asarray(image_rows) % 2
    kernel_rows = np.asarray(kernel_rows) % 2
    img, img_piv = row_reduce(image_rows)
    lib = _native()
    if lib is not None and kernel_rows.shape[0]:
        # reduce each kernel vector against rref(image) + the vectors kept so far
        n = kernel_rows.shape[1]
        pb, pk = pack_rows(img) if img.shape[0] else np.zeros((0, (n + 63) // 64), np.uint64), pack_rows(kernel_rows)
        acc = np.zeros(kernel_rows.shape[0], dtype=np.uint8)
        lead = np.ascontiguousarray(img_piv, dtype=np.int64)
        got = lib.qd_gf2_extend_basis(pb.ctypes.data, pb.shape[0], lead.ctypes.data, pk.ctypes.data, pk.shape[0],
                                      pk.shape[1], n, acc.ctypes.data, -1)
        if got < 0:
            raise ValueError("qd_gf2_extend_basis: bad arguments")
        return kernel_rows[acc.astype(bool)]
    # Columns of the augmented matrix [img^T | ker^T]: pivots beyond img's rank
    # pick the kernel vectors outside span(img).
    aug = np.hstack([img.T, kernel_rows.T])
    _, piv = row_reduce(aug)
    picks = piv[piv >= img.shape[0]] - img.shape[0]
    return kernel_rows[picks]


def pair_logicals(z_logicals, x_logicals) -> np.ndarray:
    """Re-combine Z logicals so that Lz Lx^T = I (reference ``compute_logical_pairs``,
    homological_product_code.py:27-39)."""
    z = np.asarray(z_logicals) % 2
    x = np.asarray(x_logicals) % 2
    k = x.shape[0]
    # BLAS float32 product: exact, every partial sum is an integer <= n < 2^24
    assert z.shape[1] < (1 << 24)
    inner = (z.astype(np.float32) @ x.T.astype(np.float32)).astype(np.int64) % 2
    aug = np.hstack([inner, z]).astype(np.uint8)
    red, _ = row_reduce(aug, ncols=k)
    return red[:, k:]


def css_logicals(hx, hz):
    """Return (Lx, Lz) uint8 dense for the CSS code with check matrices hx, hz
    (scipy sparse or dense).  Lx spans ker(Hz)/row(Hx); Lz spans ker(Hx)/row(Hz);
    Lz is paired with Lx."""
    hx = np.asarray(hx.todense() if hasattr(hx, "todense") else hx) % 2
    hz = np.asarray(hz.todense() if hasattr(hz, "todense") else hz) % 2
    lx = homology_representatives(hx, null_space(hz))
    lz = homology_representatives(hz, null_space(hx))
    lz = pair_logicals(lz, lx)
    return lx.astype(np.uint8), lz.astype(np.uint8)
