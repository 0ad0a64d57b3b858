"""Storage experiment: measurement-record views and the on-device sampler.

Mirrors ``build_storage_simulation`` (``python/qldpc/storage_sim.py:110-199``) for
what the decoding path consumes:

* the record layout -- per round ``[X-check outcomes (mx), Z-check outcomes (mz)]``
  then the transversal data readout (n) -- and its views ``measurement_view``
  (:187-192) and ``data_view`` (:194-196);
* the noise: instead of writing a Stim circuit and sampling it, shots are drawn
  by the Philox sampler in csrc/qdec_sample.hip, which restates the noise the
  reference's ``depolarizing_noise`` rewrite places on that circuit (schedule
  pinned against the reference's circuit text, tests/test_storage_schedule.py).

The circuit text itself (gate scheduling by edge colouring) is out of scope:
under ``depolarizing_noise`` gates are noiseless and the schedule does not change
what the decoder sees.  ``StorageSim.circuit`` is therefore
None.  X-check outcomes in host records are zero: they are random in the first
round and never read by the Z-basis decoders (get_x_checks=False).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import numpy as np

__all__ = ["StorageSim", "build_storage_simulation"]


@dataclass(frozen=True)
class StorageSim:
    circuit: object
    measurement_view: Callable
    data_view: Callable
    rounds: int = 0
    noise_model: object = None
    code: object = None
    use_x_logicals: bool = False

    # ---- sampler (device) ----
    def check_matrix(self):
        return self.code.checks.x if self.use_x_logicals else self.code.checks.z

    def sample_device(self, decoder, B: int, seed: int, stream_id: int = 0, shot0: int = 0, out=None):
        """Sample B shots on `decoder`'s device (decoder must be built on the
        decoding check matrix).  Returns (spacetime syndrome uint8[B, (R+1)m],
        readout uint8[B, n]) as torch tensors."""
        import torch
        nm = self.noise_model
        if nm is None or getattr(nm, "kind", None) not in ("depolarizing", "trivial"):
            raise NotImplementedError("the device sampler implements depolarizing_noise / trivial_noise only")
        H = self.check_matrix()
        m, n = H.shape
        dev = torch.device("cuda", decoder.device)
        if out is None:
            syn = torch.empty((B, (self.rounds + 1) * m), dtype=torch.uint8, device=dev)
            rd = torch.empty((B, n), dtype=torch.uint8, device=dev)
        else:
            syn, rd = out
        decoder.sample_storage_device(self.rounds, nm.p, nm.pm, seed, stream_id, shot0, B, syn, rd)
        return syn, rd

    def records_from_samples(self, syn: np.ndarray, readout: np.ndarray) -> np.ndarray:
        """Host measurement records (reference layout) from sampler output:
        undo the round differencing; X-check outcomes are 0."""
        checks = self.code.checks
        mx, mz = checks.x.shape[0], checks.z.shape[0]
        R = self.rounds
        B = syn.shape[0]
        m = mx if self.use_x_logicals else mz
        diff = syn.reshape(B, R + 1, m)
        raw = np.bitwise_xor.accumulate(diff[:, :R], axis=1) if R else np.zeros((B, 0, m), np.uint8)
        rec = np.zeros((B, (mx + mz) * R + readout.shape[1]), dtype=np.uint8)
        for t in range(R):
            off = (mx + mz) * t + (0 if self.use_x_logicals else mx)
            rec[:, off:off + m] = raw[:, t]
        rec[:, (mx + mz) * R:] = readout
        return rec


def build_storage_simulation(rounds: int, noise_model, code, use_x_logicals=None) -> StorageSim:
    """Record views of the storage experiment with `rounds` noisy rounds
    (storage_sim.py:110-199; circuit text not generated, see module doc)."""
    if use_x_logicals is None:
        use_x_logicals = False
    mx, mz = code.checks.x.shape[0], code.checks.z.shape[0]
    n = code.num_qubits

    def meas_result(round_index, get_x_checks, measurement_vector, *_, mx=mx, mz=mz):
        off = (mx + mz) * round_index + (0 if get_x_checks else mx)
        cnt = mx if get_x_checks else mz
        return measurement_vector[off:off + cnt]

    def data_result(measurement_vector, *_, mx=mx, mz=mz, rounds=rounds, n=n):
        off = (mx + mz) * rounds
        return measurement_vector[off:off + n]

    return StorageSim(None, meas_result, data_result, rounds=int(rounds), noise_model=noise_model, code=code,
                      use_x_logicals=bool(use_x_logicals))
