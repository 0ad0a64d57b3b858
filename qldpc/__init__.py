"""Compatibility package: the reference's import surface (``import qldpc``,
reference python/qldpc/__init__.py) backed by exp_ldpc_amd (MI355X).  With this
repository on PYTHONPATH the reference's ``scripts/p_sweep.py`` and
``scripts/generate_hgp_code.py``-style code sources run unchanged: decoding path
(``qldpc.misc.p_sweep_main``, ``qldpc.noise_model``), code I/O, spacetime codes,
the DEM-based detector code, and the HGP / lifted-product constructions.
Edge colouring and swap routing (circuit scheduling) are out of scope
(DESIGN.md §7)."""
from exp_ldpc_amd.codes import (CircuitTargets, QuantumCode, QuantumCodeChecks, QuantumCodeLogicals,  # noqa: F401
                                read_quantum_code, write_quantum_code)
from exp_ldpc_amd.spacetime import SpacetimeCode, SpacetimeCodeSingleShot  # noqa: F401
from exp_ldpc_amd.dem import DetectorSpacetimeCode  # noqa: F401
from exp_ldpc_amd.storage_sim import StorageSim, build_storage_simulation  # noqa: F401
from exp_ldpc_amd.hgp import biregular_hgp, random_biregular_graph, remove_short_cycles  # noqa: F401
from exp_ldpc_amd.lifted import (lifted_product_code_cyclic, lifted_product_code_pgl2,  # noqa: F401
                                 qc_lifted_product_code)
from exp_ldpc_amd import lifted as lifted_product_code  # noqa: F401
from exp_ldpc_amd import lifted as matrix_lifted_product_code  # noqa: F401

from . import noise_model  # noqa: F401
from . import misc  # noqa: F401
