"""qldpc.misc compatibility module (reference python/qldpc/misc/__init__.py)."""
from exp_ldpc_amd.experiment import (BPDetectorCorrect, BPOSDCorrect, BPOSDCorrectSingleShot,  # noqa: F401
                                     BPOSDHybridCorrect, p_sweep, p_sweep_main, run_simulation)
