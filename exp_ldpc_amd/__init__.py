"""exp_ldpc_amd: MI355X-native BP + small-set-flip syndrome decoding for qLDPC
storage experiments (the decoding hot path of qldpc/exp_ldpc).

Layers:
  csrc/ + libqdec_hip.so   HIP kernels (gfx950) and the C ABI (include/qdec.h)
  _abi                     ctypes binding; no CPU fallback
  decoder                  Decoder: one graph on one GPU, batched decode
  ldpc_compat              ldpc-v1 bp_decoder / bposd_decoder drop-ins
  osd                      OSD stage for BP failures (host C++)
  codes, spacetime         the reference's code types, qecc I/O, spacetime matrices
  noise_model, storage_sim noise semantics + on-device storage-experiment sampler
  experiment               decoder modes, run_simulation, p_sweep, p_sweep_main
"""
__version__ = "0.1.0"
