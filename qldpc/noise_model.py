"""qldpc.noise_model compatibility module (reference python/qldpc/noise_model.py)."""
from exp_ldpc_amd.noise_model import *  # noqa: F401,F403
from exp_ldpc_amd.noise_model import NoiseRewriter, circuit_noise, depolarizing_noise, trivial_noise  # noqa: F401
