"""tt2_gemm_plan's kernel choice (host logic, CPU: the plan reads only sizes, flags and pointer
alignment): v10 (16) takes the NT products whose 256 x 256 tiles' rounds of the chip cost
less than v7's (the decoder FFN1 forward, the memory K/V projection), v11 (17) the other NT
forward products up to K = 1024, v7 (13) the long-K, dgrad / residual / split products, v8 (15)
the small ones; explicit variants win."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "transformer-tacotron2_amd"))
from tt2 import _lib  # noqa: E402
from tt2._lib import ACT_RELU, ACT_TANH, DT_BF16  # noqa: E402

_A = torch.empty(64, dtype=torch.bfloat16)
_C = torch.empty(64, dtype=torch.bfloat16)
_BIAS = torch.empty(16, dtype=torch.float32)
_L = C.CDLL(_lib.LIB_PATH)   # the plan is host code: no HIP device needed
_L.tt2_gemm_plan.argtypes = [C.POINTER(_lib.GemmArgs)]
_L.tt2_gemm_plan.restype = C.c_int


def plan(m, n, k, trans_a=False, trans_b=False, bias=None, res=None, ldr=0, act=0, beta=0.0, splits=1,
         variant=0):
    g = _lib.GemmArgs()
    g.a, g.b, g.c = _A.data_ptr(), _A.data_ptr(), _C.data_ptr()
    g.bias = bias.data_ptr() if bias is not None else None
    g.res, g.ldr, g.res_dtype = (res.data_ptr(), ldr, DT_BF16) if res is not None else (None, 0, 0)
    g.m, g.n, g.k = m, n, k
    g.lda, g.ldb, g.ldc = m if trans_a else k, n if trans_b else k, n
    g.dtype_in = g.dtype_out = DT_BF16
    g.trans_a, g.trans_b = int(trans_a), int(trans_b)
    g.act, g.alpha, g.beta = act, 1.0, beta
    g.splits, g.kernel_variant = splits, variant
    return _L.tt2_gemm_plan(C.byref(g))


def test_v10_takes_the_wide_forward_products():
    assert plan(12800, 2048, 512, bias=_BIAS, act=ACT_RELU) == 16   # FFN1 forward: 2 rounds vs 4
    assert plan(2048, 6144, 512, bias=_BIAS) == 16                  # memory K/V: 1 round vs 2
    assert plan(8192, 8192, 8192) == 16


def test_v11_takes_the_forward_k512_products():
    assert plan(12800, 512, 512, bias=_BIAS) == 17                  # 200 v7 tiles; v11 is v7's tile, 8 loaders
    assert plan(12800, 1536, 512, bias=_BIAS) == 17                 # QKV: 2 v10 rounds cost more than 3 of v7's
    assert plan(12800, 512, 1024, bias=_BIAS) == 17
    assert plan(12800, 512, 2048) == 13                             # long K: v7 (two MFMA waves per SIMD)
    assert plan(12800, 512, 512, trans_b=True) == 13                # activation gradients stay on v7 ...
    assert plan(12800, 512, 512, trans_b=True, variant=17) == 17    # ... unless forced
    assert plan(12800, 512, 512, res=_C, ldr=512) == 13             # a forward residual: v7


def test_v7_and_v8_keep_the_rest():
    assert plan(12800, 512, 2048) == 13
    assert plan(12800, 2048, 512, trans_b=True) == 13               # dgrad (N-contiguous B)
    assert plan(12800, 2048, 512, res=_C, ldr=2048) == 13           # residual epilogue
    assert plan(12800, 2048, 512, act=ACT_TANH) == 13
    assert plan(12800, 2048, 512, beta=1.0) == 13
    assert plan(512, 2048, 12800, trans_a=True, splits=2) == 13     # weight gradient
    assert plan(12800, 2040, 512) == 13                             # N % 256 != 0
    assert plan(2048, 512, 512) == 15                               # <= 64 v7 tiles: v8


def test_explicit_variants():
    assert plan(12800, 2048, 512, variant=13) == 13
    assert plan(12800, 512, 512, variant=16) == 16
    assert plan(12800, 2048, 512, trans_b=True, variant=16) != 16   # v10 is NT only


_L.tt2_gemm_stats_rows.argtypes = [C.POINTER(_lib.GemmArgs)]
_L.tt2_gemm_stats_rows.restype = C.c_int32


def stats_rows(m, n, k, trans_a=False, trans_b=False, splits=1, dtype_out=DT_BF16, conv=None):
    """tt2_gemm_stats_rows: the chunk height of a fused BatchNorm statistics request (host code)"""
    g = _lib.GemmArgs()
    g.a, g.b, g.c = _A.data_ptr(), _A.data_ptr(), _C.data_ptr()
    g.m, g.n, g.k = m, n, k
    g.lda, g.ldb, g.ldc = m if trans_a else k, n if trans_b else k, n
    if conv is not None:
        g.a_conv_t, g.a_conv_c, g.a_conv_pad = conv
        g.lda = conv[1]
    g.dtype_in, g.dtype_out = DT_BF16, dtype_out
    g.trans_a, g.trans_b = int(trans_a), int(trans_b)
    g.alpha = 1.0
    g.splits = splits
    return _L.tt2_gemm_stats_rows(C.byref(g))


def test_fused_statistics_chunk_height():
    # the post-net conv (v7: 256-row chunks) and the encoder pre-net conv (v8: 64-row chunks)
    assert stats_rows(12800, 512, 2560, conv=(800, 512, 2)) == 256
    assert stats_rows(2048, 512, 2560, conv=(128, 512, 2)) == 64
    assert stats_rows(2048, 512, 512, trans_b=True) == 64        # the pre-net projection's dgrad (v8)
    # a request that plans v10 falls back to v7's image epilogue; split-K, f32 C, n % 128 on v7
    # and a transposed v7 operand cannot carry the statistics
    assert stats_rows(12800, 2048, 512) == 256
    assert stats_rows(12800, 512, 2560, conv=(800, 512, 2), splits=2) == 0
    assert stats_rows(12800, 512, 512, dtype_out=0) == 0
    assert stats_rows(12800, 576, 512) == 0
    assert stats_rows(12800, 512, 512, trans_b=True) == 0


def test_algorithmic_bytes_count_epilogue_inputs_and_unique_conv_rows():
    """bench.py's roofline bytes per GEMM (tt2.ops.gemm_algo_bytes): operands and C once, each
    epilogue input once, an implicit-im2col operand as its unique rows."""
    from tt2.ops import gemm_algo_bytes
    g = _lib.GemmArgs()
    g.m, g.n, g.k = 12800, 512, 2048
    g.dtype_in = g.dtype_out = DT_BF16
    g.alpha, g.beta = 1.0, 0.0
    base = 2 * (12800 * 2048 + 512 * 2048) + 2 * 12800 * 512
    assert gemm_algo_bytes(g) == base
    g.res, g.res_dtype = _A.data_ptr(), DT_BF16
    g.gate, g.gate_dtype = _A.data_ptr(), DT_BF16
    g.bias = _BIAS.data_ptr()
    assert gemm_algo_bytes(g) == base + 2 * (2 * 12800 * 512) + 4 * 512
    c = _lib.GemmArgs()   # post-net conv: k = 5 taps x 512 channels, A read as 12800 x 512
    c.m, c.n, c.k = 12800, 512, 2560
    c.dtype_in = c.dtype_out = DT_BF16
    c.a_conv_t, c.a_conv_c, c.a_conv_pad = 800, 512, 2
    assert gemm_algo_bytes(c) == 2 * (12800 * 512 + 512 * 2560) + 2 * 12800 * 512
