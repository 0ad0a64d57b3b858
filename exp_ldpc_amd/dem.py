"""Detector-error-model (DEM) input for the detector decoding mode (host side).

Reference: ``DetectorSpacetimeCode`` (``python/qldpc/spacetime_code.py:122-183``)
turns a Stim ``DetectorErrorModel`` into a fault check matrix (detectors x
faults), a fault map (observables x faults) and fault priors; ``BPDetectorCorrect``
(``python/qldpc/misc/_experiment.py:128-151``) decodes detector samples with BP on
that matrix and corrects the observables.  Stim (1.13.0, absent here) produced
the DEM via ``circuit.detector_error_model()`` (``_experiment.py:174``).

This module supplies the two pieces without Stim:

* ``parse_dem`` reads the DEM text format (Stim's wire format:
  ``error(p) D.. L.. [^ ...]``, ``detector(...) D..``, ``logical_observable L..``,
  ``shift_detectors[(...)] k``, ``repeat N { ... }``, ``detector_separator``),
  flattening repeat blocks and detector shifts as ``DetectorErrorModel.flattened()``
  does.  Decomposition separators ``^`` are dropped: the reference keeps the
  union of an error's targets (``spacetime_code.py:157-158``).
* ``storage_experiment_dem`` writes the DEM of the storage experiment's Z
  sector for any R under ``depolarizing_noise(p, pm)`` from the circuit's
  noise semantics: X components of data DEPOLARIZE1 (2p/3 per
  event, the rate the reference's priors use, ``scripts/p_sweep.py:4-5``) and
  measurement / readout flips (pm).  Detectors are those of
  ``storage_sim.py:146-182`` (first-round Z detectors, then final-round Z
  detectors); observables are the Z logicals.  Faults with identical symptoms
  are kept as separate columns (Stim would merge them); the decoding problem is
  the spacetime code of ``spacetime_code.py:46-75``.  Agreement of this
  generator with Stim's output is **unpinned** (Stim absent).

``sample_dem`` draws detector samples by sampling every fault independently
from its prior -- for independent fault mechanisms the distribution Stim's
detector sampler produces.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Tuple

import numpy as np
import scipy.sparse as sp

__all__ = ["DemInstruction", "DetectorErrorModel", "parse_dem", "DetectorSpacetimeCode", "storage_experiment_dem",
           "sample_dem"]


@dataclass
class DemInstruction:
    type: str                       # 'error' | 'detector' | 'logical_observable'
    args: List[float] = field(default_factory=list)
    detectors: List[int] = field(default_factory=list)   # absolute detector ids
    observables: List[int] = field(default_factory=list)


@dataclass
class DetectorErrorModel:
    """A flattened DEM: instructions with absolute detector ids."""
    instructions: List[DemInstruction]

    def flattened(self) -> "DetectorErrorModel":
        return self

    def __iter__(self):
        return iter(self.instructions)

    @property
    def num_detectors(self) -> int:
        ids = [d for ins in self.instructions for d in ins.detectors]
        return 1 + max(ids) if ids else 0

    @property
    def num_observables(self) -> int:
        ids = [o for ins in self.instructions for o in ins.observables]
        return 1 + max(ids) if ids else 0

    @property
    def num_errors(self) -> int:
        return sum(1 for ins in self.instructions if ins.type == "error")


_HEAD = re.compile(r"^([a-z_]+)\s*(?:\(([^)]*)\))?\s*(.*)$")


def parse_dem(text: str) -> DetectorErrorModel:
    """Parse DEM text into a flattened model (repeat blocks unrolled,
    ``shift_detectors`` applied)."""
    lines = [l.split("#", 1)[0].strip() for l in text.splitlines()]
    lines = [l for l in lines if l]
    out: List[DemInstruction] = []

    def block_end(i: int) -> int:
        """Index after the '}' closing the block opened on line i."""
        depth, j = 1, i + 1
        while depth:
            if j >= len(lines):
                raise ValueError("unterminated repeat block in DEM")
            depth += lines[j].endswith("{") - (lines[j] == "}")
            j += 1
        return j

    def run(i: int, stop: int, offset: int) -> int:
        while i < stop:
            line = lines[i]
            if line == "}":
                raise ValueError("unbalanced '}' in DEM")
            m = _HEAD.match(line)
            if not m:
                raise ValueError(f"cannot parse DEM line: {line!r}")
            name, args, rest = m.group(1), m.group(2), m.group(3)
            if name == "repeat":
                if not line.endswith("{"):
                    raise ValueError("repeat block must open with '{'")
                count = int(rest.rstrip("{").strip())
                end = block_end(i)
                for _ in range(count):
                    offset = run(i + 1, end - 1, offset)
                i = end
                continue
            argv = [float(v) for v in args.split(",")] if args else []
            toks = rest.split()
            if name == "shift_detectors":
                offset += int(toks[0]) if toks else 0
            elif name in ("error", "detector", "logical_observable"):
                ins = DemInstruction(name, argv)
                for t in toks:
                    if t == "^":
                        continue
                    if t[0] == "D":
                        ins.detectors.append(int(t[1:]) + offset)
                    elif t[0] == "L":
                        ins.observables.append(int(t[1:]))
                    else:
                        raise ValueError(f"bad DEM target {t!r}")
                if name == "error" and len(argv) != 1:
                    raise ValueError("error instruction takes one probability")
                out.append(ins)
            elif name != "detector_separator":
                raise ValueError(f"unknown DEM instruction {name!r}")
            i += 1
        return offset

    run(0, len(lines), 0)
    return DetectorErrorModel(out)


def _from_columns(cols, nrows) -> sp.csr_matrix:
    r = np.fromiter((i for c in cols for i in c), dtype=np.int64)
    c = np.fromiter((j for j, col in enumerate(cols) for _ in col), dtype=np.int64)
    m = sp.coo_matrix((np.ones(r.size, dtype=np.uint32), (r, c)), shape=(nrows, len(cols))).tocsr()
    m.data %= 2  # a target listed twice in one error cancels
    m.eliminate_zeros()
    return m


class DetectorSpacetimeCode:
    """Fault check matrix (detectors x faults), fault map (observables x faults)
    and fault priors of a DEM (reference ``spacetime_code.py:122-183``).  Accepts
    DEM text or a parsed model."""

    def __init__(self, detector_model):
        dem = parse_dem(detector_model) if isinstance(detector_model, str) else detector_model.flattened()
        det_cols, obs_cols, priors = [], [], []
        for ins in dem:
            if ins.type not in ("error", "detector", "logical_observable"):
                raise AssertionError("requires a flattened model")
            if ins.type == "error":
                det_cols.append(ins.detectors)
                obs_cols.append(ins.observables)
                priors.append(ins.args[0])
        self.fault_check_matrix = _from_columns(det_cols, dem.num_detectors)
        self.fault_map = _from_columns(obs_cols, dem.num_observables)
        self.fault_priors = np.array(priors, dtype=np.float64)


def storage_experiment_dem(hz, lz, rounds: int, p: float, pm: float | None = None) -> str:
    """DEM text of the storage experiment's Z sector for any R >= 0 (module
    docstring).  Detector block t (rows t*m ..) is the differenced Z syndrome of
    round t (storage_sim.py:146-179: first-round detectors, then s_t ^ s_{t-1}),
    block R the final readout's Hz parities against the last round; observable i
    is LZ row i (:180-182).

    Fault columns follow the circuit's noise events in time order (the
    schedule the sampler restates: noise_model.py:163-193 on storage_sim.py:110-199,
    including the REPEAT-body DEPOLARIZE1 of rounds t >= 1):
      for t < R: the data error before round t's Z readout (flips block t),
                 round t's Z measurement flips (blocks t and t+1),
                 the data error after the readout (block t+1), and for t >= 1 the
                 one the rewriter places at the end of the REPEAT body (block t+1);
      then the readout flips (block R).  R = 0 has one data event and the readout.
    A data X error in slot t flips every later syndrome and the readout, so it
    fires only detector block t and the observables.

    Deviation from the reference at R >= 2 (unpinned: Stim is absent): the
    reference's bpd_detector decodes Stim's full circuit DEM
    (_experiment.py:174,186), which also holds the X-check detectors of the
    REPEAT body (storage_sim.py:156-157) and keeps X, Y and Z faults as separate
    columns, so Y errors couple the two sectors there.  This DEM is the Z sector
    only, with X and Y merged into one column of prior 2p/3 per event; for
    R <= 1 the two sectors do not interact on the Z detectors the decoder sees.
    At R >= 2 the GPU bpd_detector therefore solves this Z-sector BP problem,
    not Stim's two-sector one."""
    if rounds < 0:
        raise ValueError("rounds must be >= 0")
    pm = p if pm is None else pm
    hz = sp.csc_matrix(hz)
    lz = sp.csc_matrix(np.asarray(lz.todense() if sp.issparse(lz) else lz) % 2)
    m, n = hz.shape
    px = 2 * p / 3
    R = rounds
    col = lambda M, j: M.indices[M.indptr[j]:M.indptr[j + 1]].tolist()
    lines = []

    def err(prob, dets, obs):
        lines.append(("error(%r) " % float(prob) + " ".join([f"D{d}" for d in dets] + [f"L{o}" for o in obs])).rstrip())

    def data_slot(t):
        for j in range(n):
            err(px, [t * m + d for d in col(hz, j)], col(lz, j))

    for t in range(R):
        data_slot(t)                      # before round t's Z readout
        for i in range(m):                # Z-check measurement flip of round t
            err(pm, [t * m + i, (t + 1) * m + i], [])
        data_slot(t + 1)                  # after the readout
        if t >= 1:
            data_slot(t + 1)              # end of the REPEAT body (noise_model.py:183-189)
    if R == 0:
        data_slot(0)                      # single timestep: noise, then the final MZ
    for j in range(n):                    # readout flip of data qubit j
        err(pm, [R * m + d for d in col(hz, j)], col(lz, j))
    lines += [f"detector D{i}" for i in range(m * (R + 1))]
    lines += [f"logical_observable L{o}" for o in range(lz.shape[0])]
    return "\n".join(lines) + "\n"


def sample_dem(code: DetectorSpacetimeCode, shots: int, seed: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """(detectors uint8[B, D], observables uint8[B, K]): every fault drawn
    independently from its prior."""
    rng = np.random.default_rng(seed)
    f = (rng.random((shots, code.fault_priors.size)) < code.fault_priors).astype(np.int64)
    det = (code.fault_check_matrix.astype(np.int64) @ f.T).T % 2
    obs = (code.fault_map.astype(np.int64) @ f.T).T % 2
    return np.asarray(det, dtype=np.uint8), np.asarray(obs, dtype=np.uint8)
