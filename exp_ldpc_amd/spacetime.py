"""Spacetime (multi-round) decoding matrices and syndrome bookkeeping (host side).

Mirrors ``python/qldpc/spacetime_code.py``:

* ``SpacetimeCode`` (:39-92): ``H_st = [blockdiag(H x (R+1)) | M]`` where
  measurement column ``t*r + j`` touches rows ``t*r + j`` and ``(t+1)*r + j``.
  The reference builds the block diagonal from ``itertools.repeat`` (:52), which
  scipy >= 1.11 consumes before use; here the intended R+1
  copies are built directly.  ``data_bits`` / ``measurement_bits`` keep the
  reference's slicing boundary (``_datablock_size`` = R*r, :75) for API fidelity;
  ``true_data_slice`` gives the real (R+1)*n data range.
* ``SpacetimeCodeSingleShot`` (:10-37): ``[H | I]``.
* ``spacetime_syndrome`` (reference ``_spacetime_syndrome``, :98-119): stacked
  per-round syndromes + final ``H @ readout``, differenced between rounds.

``fold_map`` exposes the column -> data-qubit map that the GPU kernels use to
apply ``final_correction`` in-kernel.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

__all__ = ["SpacetimeCode", "SpacetimeCodeSingleShot", "spacetime_syndrome", "spacetime_syndrome_batch"]


class SpacetimeCodeSingleShot:
    """``[H | I]``: one measurement-error column per check (spacetime_code.py:10-37)."""

    def __init__(self, check_matrix):
        h = sp.csr_matrix(check_matrix)
        r = h.shape[0]
        self.spacetime_check_matrix = sp.hstack([h, sp.identity(r, dtype=h.dtype, format="csr")], format="csr")
        self._datablock_size = h.shape[1]

    def final_correction(self, x):
        return self.data_bits(x)

    def data_bits(self, x):
        return x[: self._datablock_size]

    def measurement_bits(self, x):
        return x[self._datablock_size:]

    @property
    def fold_blocks(self) -> int:
        return 1

    @property
    def num_data(self) -> int:
        return self._datablock_size


class SpacetimeCode:
    """Difference-syndrome spacetime code over ``num_rounds`` noisy rounds plus the
    transversal readout (spacetime_code.py:39-92)."""

    def __init__(self, check_matrix, num_rounds: int):
        if num_rounds < 0:
            raise ValueError("num_rounds must be non-negative")
        h = sp.csr_matrix(check_matrix)
        r, n = h.shape
        R = int(num_rounds)
        diag = sp.block_diag([h] * (R + 1), format="csr") if R > 0 else h
        # measurement column c = t*r + j has ones at rows c and c + r
        c = np.arange(R * r, dtype=np.int64)
        meas = sp.csr_matrix((np.ones(2 * c.size, dtype=np.uint32),
                              (np.concatenate([c, c + r]), np.concatenate([c, c]))),
                             shape=((R + 1) * r, R * r))
        self.spacetime_check_matrix = sp.hstack([diag, meas], format="csr").astype(np.uint32)
        self._check_matrix = h
        self._num_rounds = R
        # reference quirk (spacetime_code.py:75): boundary at R*r, not (R+1)*n
        self._datablock_size = meas.shape[1]

    @property
    def num_rounds(self) -> int:
        return self._num_rounds

    @property
    def num_data(self) -> int:
        return self._check_matrix.shape[1]

    @property
    def fold_blocks(self) -> int:
        return self._num_rounds + 1

    def true_data_slice(self) -> slice:
        return slice(0, (self._num_rounds + 1) * self.num_data)

    def syndrome_from_history(self, history, readout):
        return spacetime_syndrome(self._num_rounds, self._check_matrix, history, readout)

    def final_correction(self, spacetime_correction):
        n = self.num_data
        x = np.asarray(spacetime_correction)
        acc = sum(x[i * n:(i + 1) * n] for i in range(self._num_rounds + 1))
        return acc % 2

    def data_bits(self, x):
        return x[: self._datablock_size]

    def measurement_bits(self, x):
        return x[self._datablock_size:]


def spacetime_syndrome(rounds: int, check_matrix, syndrome_history, readout) -> np.ndarray:
    """float64[(R+1)*r] difference syndrome (spacetime_code.py:98-119)."""
    h = sp.csr_matrix(check_matrix)
    r = h.shape[0]
    rows = np.zeros((rounds + 1, r))
    for t in range(rounds):
        rows[t] = np.asarray(syndrome_history(t))
    rows[rounds] = (h @ np.asarray(readout)) % 2
    out = rows.copy()
    out[1:] = (rows[1:] + rows[:-1]) % 2
    return out.reshape(-1)


def spacetime_syndrome_batch(rounds: int, check_matrix, history: np.ndarray, readout: np.ndarray) -> np.ndarray:
    """Batched form: ``history`` uint8[B, R, r], ``readout`` uint8[B, n] ->
    uint8[B, (R+1)*r]."""
    h = sp.csr_matrix(check_matrix)
    B = readout.shape[0]
    r = h.shape[0]
    rows = np.zeros((B, rounds + 1, r), dtype=np.uint8)
    if rounds:
        rows[:, :rounds] = history
    rows[:, rounds] = (h @ readout.T).T % 2
    out = rows.copy()
    out[:, 1:] ^= rows[:, :-1]
    return out.reshape(B, -1)
