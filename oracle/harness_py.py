"""CPU restatements of the reference's per-shot decoder wrappers (test
infrastructure only: tests/ import this as the checker, the product never does).

Each function follows one wrapper of /root/reference/python/qldpc/misc/_experiment.py
loop for loop, with the decoder object it constructs replaced by this build's
checkers: the C oracle's ldpc-v1 BP restatement (oracle/qdec_oracle.c via
oracle/cpu.py) and the numpy OSD restatement (oracle/osd_py.py).  ldpc's
``bposd_decoder.decode`` returns the BP hard decision when BP converged and the
OSD solution otherwise; ``bposd`` below does exactly that.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

from .osd_py import osd_decode


def bposd(orc, H, probs, syn, *, bp_method, precision, max_iter, ms_scaling, osd_method, osd_order):
    """ldpc v1 bposd_decoder(H, channel_probs=probs, ...).decode(s) for every row
    of syn; returns uint8[B, n]."""
    syn = np.ascontiguousarray(syn, dtype=np.uint8)
    out = orc.decode(H, probs, syn, method=bp_method, precision=precision, max_iter=max_iter,
                     ms_scaling=ms_scaling, want_llr=True)
    x = out["x"].copy()
    for b in np.nonzero((out["status"] & 1) == 0)[0]:
        _, osdw = osd_decode(H, syn[b], out["llr"][b], osd_method, osd_order)
        x[b] = osdw
    return x


def _opts(bp_osd_options, precision):
    o = bp_osd_options
    return dict(bp_method=o.get("bp_method", "ps"), precision=precision, max_iter=int(o.get("max_iter", 0) or 0),
                ms_scaling=float(o.get("ms_scaling_factor", 0.0)), osd_method=o.get("osd_method", "osd_cs"),
                osd_order=int(o.get("osd_order", 0)))


def single_shot_corrections(orc, Hz, rounds, raw_history, readout, bp_osd_options, priors, precision="f32"):
    """BPOSDCorrectSingleShot.readout_correction (_experiment.py:43-60) for a batch.

    raw_history: uint8[B, R, m], the Z-check outcomes history(t) of every round
    (not differenced); readout: uint8[B, n].  Returns uint8[B, n] corrections."""
    data_prior, meas_prior = priors
    Hz = sp.csr_matrix(Hz)
    m, n = Hz.shape
    # SpacetimeCodeSingleShot (spacetime_code.py:15-25): [Hz | I], priors by range (_experiment.py:33-35)
    Hss = sp.hstack([Hz, sp.identity(m, dtype=Hz.dtype)]).tocsr()
    pss = np.empty(n + m)
    pss[:n] = data_prior
    pss[n:] = meas_prior
    kw = _opts(bp_osd_options, precision)
    B = readout.shape[0]
    acc = np.zeros((B, n), np.uint8)
    for t in range(rounds):  # _experiment.py:45-52
        corr_syn = (Hz @ acc.T).T % 2
        syndrome = (corr_syn + raw_history[:, t]) % 2
        x = bposd(orc, Hss, pss, syndrome.astype(np.uint8), **kw)
        acc = (acc + x[:, :n]) % 2  # final_correction = data bits (spacetime_code.py:27-33)
    rd = (acc + readout) % 2  # :55
    syndrome = (Hz @ rd.T).T % 2  # :58
    final = bposd(orc, Hz, np.full(n, data_prior), syndrome.astype(np.uint8), **kw)  # :59, error_rate=data_prior
    return ((final + acc) % 2).astype(np.uint8)  # :60


def _spacetime_matrix(Hz, R, data_prior, meas_prior):
    """SpacetimeCode (spacetime_code.py:46-75, the intended (R+1)-copy block
    diagonal) and its channel prior with data / measurement columns set by their
    true ranges (_experiment.py:74-76 / :105-107)."""
    Hz = sp.csr_matrix(Hz)
    m, n = Hz.shape
    blocks = sp.block_diag([Hz] * (R + 1), format="csr")
    if R > 0:
        M = sp.lil_matrix(((R + 1) * m, R * m), dtype=np.uint8)
        for t in range(R):
            for j in range(m):
                M[t * m + j, t * m + j] = 1
                M[(t + 1) * m + j, t * m + j] = 1
        Hst = sp.hstack([blocks, M.tocsr()]).tocsr()
    else:
        Hst = blocks
    prior = np.empty(Hst.shape[1])
    prior[:(R + 1) * n] = data_prior
    prior[(R + 1) * n:] = meas_prior
    return Hst, prior


def _fold(x, n, R):
    """SpacetimeCode.final_correction (spacetime_code.py:81-84): XOR of the R+1
    data blocks."""
    fold = np.zeros((x.shape[0], n), np.uint8)
    for t in range(R + 1):
        fold ^= x[:, t * n:(t + 1) * n]
    return fold


def spacetime_bposd_corrections(orc, Hz, rounds, spacetime_syndrome, bp_osd_options, priors, precision="f32"):
    """BPOSDCorrect.readout_correction (_experiment.py:62-83) for a batch:
    bposd on H_st (SpacetimeCode, spacetime_code.py:46-75, intended (R+1)-copy
    block diagonal) with data/measurement priors, then final_correction = XOR
    of the R+1 data blocks (spacetime_code.py:81-84).  spacetime_syndrome is the
    differenced syndrome of spacetime_code.py:98-119, uint8[B, (R+1) m]."""
    data_prior, meas_prior = priors
    n = Hz.shape[1]
    Hst, prior = _spacetime_matrix(Hz, rounds, data_prior, meas_prior)
    x = bposd(orc, Hst, prior, spacetime_syndrome, **_opts(bp_osd_options, precision))
    return _fold(x, n, rounds)


def hybrid_corrections(orc, Hz, rounds, spacetime_syndrome, readout, bp_osd_options, priors, precision="f32"):
    """BPOSDHybridCorrect.readout_correction (_experiment.py:115-126) for a batch.

    Stage 1 is ldpc's bp_decoder on H_st (:110-113): BP only, its hard decision
    whether or not BP converged (.decode returns bp_decoding), folded onto the
    data qubits (:117-118).  The readout is corrected with it (:121), re-syndromed
    on Hz (:124), and stage 2 is bposd_decoder(Hz, error_rate=data_prior) (:96-100,
    :125).  Returns uint8[B, n]: stage-2 correction + stage-1 fold (:126)."""
    data_prior, meas_prior = priors
    Hz = sp.csr_matrix(Hz)
    n = Hz.shape[1]
    Hst, prior = _spacetime_matrix(Hz, rounds, data_prior, meas_prior)
    kw = _opts(bp_osd_options, precision)
    out = orc.decode(Hst, prior, np.ascontiguousarray(spacetime_syndrome, dtype=np.uint8), method=kw["bp_method"],
                     precision=precision, max_iter=kw["max_iter"], ms_scaling=kw["ms_scaling"], want_llr=False)
    stage1 = _fold(out["x"], n, rounds)  # :117-118
    rd = (stage1 + readout) % 2  # :121
    syndrome = (Hz @ rd.T).T % 2  # :124
    final = bposd(orc, Hz, np.full(n, data_prior), syndrome.astype(np.uint8), **kw)  # :125, error_rate=data_prior
    return ((final + stage1) % 2).astype(np.uint8)  # :126


def logical_failures(Lz, readout, corr):
    """any(Lz (readout + corr)) per shot (_experiment.py:205-209)."""
    v = (readout.astype(np.int64) + corr) % 2
    return ((v @ (np.asarray(Lz) % 2).T.astype(np.int64)) % 2).any(axis=1)
