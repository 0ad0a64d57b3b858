"""Compatibility package: the reference's import surface (``import qldpc``) for
the decoding path, backed by exp_ldpc_amd (MI355X).  With this repository on
PYTHONPATH the reference's ``scripts/p_sweep.py`` runs unchanged: it needs
``qldpc.noise_model.depolarizing_noise`` and ``qldpc.misc.p_sweep_main``
(reference python/qldpc/__init__.py, misc/__init__.py).  Code constructions
(HGP / lifted products) are not part of this build's scope."""
from exp_ldpc_amd.codes import (CircuitTargets, QuantumCode, QuantumCodeChecks, QuantumCodeLogicals,  # noqa: F401
                                read_quantum_code, write_quantum_code)
from exp_ldpc_amd.spacetime import SpacetimeCode, SpacetimeCodeSingleShot  # noqa: F401
from exp_ldpc_amd.storage_sim import StorageSim, build_storage_simulation  # noqa: F401

from . import noise_model  # noqa: F401
from . import misc  # noqa: F401
