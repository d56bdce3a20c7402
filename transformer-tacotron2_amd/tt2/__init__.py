"""tt2 -- MI355X-native Transformer-TTS mel engine (host side).

Python host code on PyTorch-ROCm (device memory, streams, torch.distributed)
driving hand-written gfx950 HIP kernels in libtt2.so through a C ABI.
"""
from . import _lib  # noqa: F401
