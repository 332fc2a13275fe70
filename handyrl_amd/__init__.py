"""handyrl_amd — MI355X-native learner hot path for HandyRL.

The reference's learner step (handyrl/train.py:357-401) re-designed for one
process per MI355X: return-target scans and the fused IS-ratio/loss as
hand-written gfx950 HIP kernels behind a C ABI (include/*.h, libhrl.so), the
env network on PyTorch-ROCm, and data parallelism over RCCL.
"""

__version__ = '0.1.0'
