"""hhfm_amd — MI355X-native scoring backend for the FM family of
context-aware recommenders in data-man-34/HHFM (FM, HHFM/OurModel7, AFM,
DeepFM).  Hand-written gfx950 HIP kernels behind a C ABI (include/hhfm.h),
bound by a thin pybind11 module; PyTorch-ROCm supplies device memory, streams
and torch.distributed (RCCL) only.
"""
__version__ = "0.1.0"
