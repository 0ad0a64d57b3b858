"""Noise models of the storage experiment (host side).

Mirrors ``python/qldpc/noise_model.py``: ``depolarizing_noise(p, pm)`` (:117-123),
``trivial_noise()`` (:10-12) and ``circuit_noise(p, pm)`` (:125-151) return
rewriter objects whose ``rewrite(targets, circuit)`` inserts noise into a
Stim-style circuit listing exactly where the reference does (the rewrite rules
are pinned by the reference's golden tests, tests/test_storage_sim.py:13-77,
restated in tests/test_noise_model.py).  The objects also carry their
parameters (``kind``, ``p``, ``pm``) so the on-device sampler
(csrc/qdec_sample.hip) can reproduce the noise without a circuit simulator:
under ``depolarizing_noise`` every data qubit gets DEPOLARIZE1(p) at the start
of each timestep holding a measurement, and every measurement flips with
probability pm.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Callable, Iterable, List

__all__ = ["NoiseRewriter", "depolarizing_noise", "trivial_noise", "circuit_noise", "circuit_ticks",
           "tokenize_line", "get_two_qubit_targets"]

_MEASUREMENT_GATES = ["M", "MZ", "MX", "MY", "MPP", "MR", "MRZ", "MRX", "MRY"]
_MEAS_RE = re.compile(r"^(?:\s*)(" + "|".join(_MEASUREMENT_GATES) + r")((?:\s*\d+\s*)+)$")
_TWO_QUBIT_GATES = {
    "CNOT", "CX", "CY", "CZ", "ISWAP", "ISWAP_DAG", "SQRT_XX", "SQRT_XX_DAG", "SQRT_YY", "SQRT_YY_DAG",
    "SQRT_ZZ", "SQRT_ZZ_DAG", "SWAP", "XCX", "XCY", "XCZ", "YCX", "YCY", "YCZ", "ZCX", "ZCY", "ZCZ",
}


def tokenize_line(line: str) -> List[str]:
    """Upper-cased whitespace tokens of a circuit line, comments dropped."""
    return [t.upper() for t in line.split("#")[0].split()]


def circuit_ticks(circuit: Iterable[str]) -> List[List[str]]:
    """Split a circuit listing into timesteps; a TICK line opens the next one
    (reference circuit_ticks, noise_model.py:19-50)."""
    steps: List[List[str]] = [[]]
    for line in circuit:
        toks = tokenize_line(line)
        if toks and toks[0] == "TICK":
            steps.append([])
        steps[-1].append(line)
    return steps


def get_two_qubit_targets(line: str):
    toks = tokenize_line(line)
    if len(toks) > 1 and toks[0] in _TWO_QUBIT_GATES:
        qs = [int(t) for t in toks[1:]]
        if len(qs) % 2:
            raise ValueError(f"Found an odd number of targets for a two qubit gate directive: \n f{line}")
        return list(zip(qs[::2], qs[1::2]))
    return []


def _noisy_measurement(line: str, p) -> str:
    m = _MEAS_RE.search(line)
    if m is None:
        return line
    return f"{m.group(1)}({p}){m.group(2)}"


@dataclass(frozen=True)
class NoiseRewriter:
    """A circuit rewriter plus the parameters the device sampler needs."""
    rewrite: Callable
    kind: str = "custom"
    p: float = 0.0
    pm: float = 0.0
    params: dict = field(default_factory=dict)


def _measurement_step_rewriter(p_data, p_meas, noisy: bool):
    def rewrite(targets, circuit):
        out = []
        for step in circuit_ticks(circuit):
            has_meas = any(_MEAS_RE.search(l) is not None for l in step)
            if not (noisy and step and has_meas):
                out.extend(step)
                continue
            body = step
            if tokenize_line(step[0])[:1] == ["TICK"]:
                out.append(step[0])
                body = step[1:]
            out.append(f"DEPOLARIZE1({p_data}) " + " ".join(str(q) for q in targets.data))
            out.extend(_noisy_measurement(l, p_meas) for l in body)
        return out
    return rewrite


def depolarizing_noise(p: float, pm: float) -> NoiseRewriter:
    """DEPOLARIZE1(p) on the data qubits at the start of every timestep containing
    a measurement; measurements flip with probability pm (noise_model.py:117-123)."""
    return NoiseRewriter(_measurement_step_rewriter(p, pm, True), kind="depolarizing", p=float(p), pm=float(pm))


def trivial_noise() -> NoiseRewriter:
    return NoiseRewriter(_measurement_step_rewriter(0, 0, False), kind="trivial", p=0.0, pm=0.0)


def circuit_noise(p: float, pm: float | None = None) -> NoiseRewriter:
    """Gate-level noise (noise_model.py:125-151).  The circuit rewrite is provided;
    the device sampler does not implement this model (it depends on the gate
    schedule), so storage sampling with it raises NotImplementedError."""
    if pm is None:
        pm = p

    def rewrite(targets, circuit):
        support = set(targets.data) | set(targets.ancillas)
        out = []
        for step in circuit_ticks(circuit):
            pairs = [pq for l in step for pq in get_two_qubit_targets(l)]
            ones = support - {q for pq in pairs for q in pq}
            out.extend(_noisy_measurement(l, pm) for l in step)
            if pairs:
                out.append(f"DEPOLARIZE2({p}) " + " ".join(f"{a} {b}" for a, b in pairs))
            out.append(f"DEPOLARIZE1({p}) " + " ".join(str(q) for q in sorted(ones)))
        return out
    return NoiseRewriter(rewrite, kind="circuit", p=float(p), pm=float(pm))
