"""ctypes binding of libtt2.so (include/tt2_capi.h).

``import torch`` happens first so libtt2 binds to the HIP runtime torch already
loaded (one runtime per process).  There is no fallback: if the library or a
GPU is missing, ``lib()`` raises.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede CDLL: one HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TT2_LIB") or os.path.join(_HERE, "libtt2.so")   # TT2_LIB: dev ablation builds

DT_F32 = 0
DT_BF16 = 1
DT_F16 = 2
ACT_NONE, ACT_RELU, ACT_TANH = 0, 1, 2

vp = C.c_void_p
i32, i64, u32, f32, sz = C.c_int32, C.c_int64, C.c_uint32, C.c_float, C.c_size_t


class GemmArgs(C.Structure):
    _fields_ = [
        ("a", vp), ("b", vp), ("c", vp),
        ("bias", vp), ("res", vp), ("gate", vp),
        ("drop_seed", vp),
        ("workspace", vp), ("ws_bytes", sz),
        ("lda", i64), ("ldb", i64), ("ldc", i64), ("ldr", i64), ("ldg", i64),
        ("m", i32), ("n", i32), ("k", i32),
        ("dtype_in", i32), ("dtype_out", i32), ("res_dtype", i32), ("gate_dtype", i32),
        ("trans_a", i32), ("trans_b", i32),
        ("act", i32), ("splits", i32),
        ("alpha", f32), ("beta", f32), ("gate_scale", f32),
        ("drop_site", u32), ("drop_thr", u32), ("drop_scale", f32),
        ("a_conv_t", i32), ("a_conv_c", i32), ("a_conv_pad", i32),
        ("b_conv_t", i32), ("b_conv_c", i32), ("b_conv_pad", i32),
        ("kernel_variant", i32),
        ("a_ksum", vp), ("a_ksum_beta", f32),
        ("a_ln_branch", vp), ("a_ln_gamma", vp), ("a_ln_beta", vp), ("a_ln_out", vp), ("a_ln_eps", f32),
        ("kv_cache", vp), ("kv_t", vp), ("kv_col0", i32), ("kv_bstride", i64), ("kv_ld", i64),
        ("main_only", i32),
        ("pe_table", vp), ("pe_alpha", vp), ("pe_t", vp),
        ("emit_mel", vp), ("emit_stop", vp), ("emit_prev", vp), ("emit_t", vp), ("emit_seed", vp),
        ("emit_done", vp), ("emit_nmels", i32), ("emit_tmax", i32),
        ("emit_stop_bias", vp), ("emit_stop_len", vp), ("emit_stop_thr", f32),
        ("col_stats", vp), ("bn_bwd", vp),
    ]


# (name, argtypes) for every exported entry point; tests check these exist.
class WflipJob(C.Structure):
    """tt2_wflip_job: one conv weight of a batched dgrad-weight flip (include/tt2_capi.h)."""
    _fields_ = [("w", vp), ("wd", vp), ("cout", i32), ("cin", i32), ("k", i32), ("pad_", i32)]


SIGNATURES: dict[str, tuple[list, object]] = {
    "tt2_last_error": ([], C.c_char_p),
    "tt2_version": ([], C.c_int),
    "tt2_init": ([C.c_int], C.c_int),
    "tt2_gemm_workspace_size": ([C.POINTER(GemmArgs)], sz),
    "tt2_gemm": ([C.POINTER(GemmArgs), vp], C.c_int),
    "tt2_gemm_plan": ([C.POINTER(GemmArgs)], C.c_int),
    "tt2_gemm_stats_rows": ([C.POINTER(GemmArgs)], C.c_int32),
    "tt2_gemm_grouped": ([C.POINTER(GemmArgs), C.c_int32, vp], C.c_int),
    "tt2_gemm_grouped_fin": ([C.POINTER(GemmArgs), C.c_int32, vp, vp], C.c_int),
    "tt2_gemm_grouped_ex": ([C.POINTER(GemmArgs), C.c_int32, vp, C.c_int32, vp], C.c_int),
    "tt2_probe_arm": ([], C.c_int),
    "tt2_probe_ms": ([C.c_int], C.c_float),
    "tt2_probe_span_ms": ([C.c_int], C.c_float),
    "tt2_probe_span_records": ([C.c_int, C.POINTER(C.c_uint64), C.c_int], C.c_int),
    "tt2_probe_span_width": ([], C.c_int),
    "tt2_probe_reset": ([], None),
}

_lib = None


class TT2Error(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libtt2.so and bind signatures (no device calls)."""
    global _lib
    if _lib is None:
        if not os.path.exists(path):
            raise TT2Error(f"libtt2.so not built ({path}); run transformer-tacotron2_amd/build_lib.py")
        L = C.CDLL(path)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


_inited = set()


def lib():
    """The library, initialised on the current device (raises without a GPU)."""
    L = load()
    if not torch.cuda.is_available():
        raise TT2Error("tt2: no HIP device available (libtt2 has no CPU fallback)")
    dev = torch.cuda.current_device()
    if dev not in _inited:
        check(L.tt2_init(dev), "tt2_init")
        _inited.add(dev)
    return L


def check(rc: int, what: str = "tt2"):
    if rc != 0:
        msg = load().tt2_last_error()
        raise TT2Error(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def dt(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return DT_BF16
    if t.dtype == torch.float32:
        return DT_F32
    if t.dtype == torch.float16:
        return DT_F16
    raise TT2Error(f"unsupported dtype {t.dtype}")


class AttnArgs(C.Structure):
    _fields_ = [
        ("q", vp), ("k", vp), ("v", vp), ("o", vp), ("dout", vp),
        ("o_out", vp), ("dq", vp), ("dk", vp), ("dv", vp),
        ("lse", vp), ("delta", vp),
        ("q_ld", i64), ("k_ld", i64), ("v_ld", i64), ("o_ld", i64), ("do_ld", i64),
        ("dq_ld", i64), ("dk_ld", i64), ("dv_ld", i64),
        ("key_len", vp),
        ("batch", i32), ("heads", i32), ("head_dim", i32), ("tq", i32), ("tk", i32), ("causal", i32),
        ("dtype", i32),
        ("scale", f32),
        ("variant", i32), ("parts", i32),
    ]


SIGNATURES.update({
    "tt2_attn_probs": ([C.POINTER(AttnArgs), vp, vp], C.c_int),
    "tt2_attn_fwd": ([C.POINTER(AttnArgs), vp], C.c_int),
    "tt2_attn_bwd": ([C.POINTER(AttnArgs), vp], C.c_int),
})


class ReduceArgs(C.Structure):
    _fields_ = [("src", vp), ("dst", vp), ("ld", i64), ("rows", i32), ("cols", i32), ("beta", f32)]


class LnArgs(C.Structure):
    _fields_ = [
        ("x", vp), ("branch", vp), ("dy", vp), ("y", vp), ("dx", vp), ("dbranch", vp),
        ("gamma", vp), ("beta", vp), ("mean", vp), ("rstd", vp), ("dgamma", vp), ("dbeta", vp),
        ("workspace", vp), ("ws_bytes", sz), ("drop_seed", vp),
        ("m", i32), ("c", i32), ("dtype", i32), ("eps", f32), ("grad_beta", f32),
        ("drop_site", u32), ("drop_thr", u32), ("drop_scale", f32), ("dbias", vp),
        ("defer_finalize", i32), ("finalize_prev", vp),
    ]


GEMM_STATS_ROWS = 256   # TT2_GEMM_STATS_ROWS: rows per chunk of tt2_gemm's fused column moments


class BnArgs(C.Structure):
    _fields_ = [
        ("y", vp), ("dout", vp), ("res", vp), ("out", vp), ("dy", vp),
        ("gamma", vp), ("beta", vp), ("mean", vp), ("rstd", vp), ("run_mean", vp), ("run_var", vp),
        ("dgamma", vp), ("dbeta", vp), ("workspace", vp), ("ws_bytes", sz), ("drop_seed", vp),
        ("res_ld", i64),
        ("m", i32), ("c", i32), ("act", i32), ("dtype", i32), ("out_dtype", i32), ("res_dtype", i32),
        ("dout_dtype", i32), ("training", i32), ("eps", f32), ("momentum", f32),
        ("drop_site", u32), ("drop_thr", u32), ("drop_scale", f32),
        ("sync_buf", vp), ("sync_world", i32), ("sync_rank", i32), ("stats_rows", i32),
    ]


class PeArgs(C.Structure):
    _fields_ = [
        ("x", vp), ("dout", vp), ("out", vp), ("dx", vp), ("alpha", vp), ("pe", vp), ("dalpha", vp),
        ("workspace", vp), ("ws_bytes", sz), ("drop_seed", vp), ("t_ptr", vp),
        ("m", i32), ("c", i32), ("t", i32), ("t_offset", i32), ("dtype", i32),
        ("drop_site", u32), ("drop_thr", u32), ("drop_scale", f32),
    ]


class LossArgs(C.Structure):
    _fields_ = [
        ("heads", vp), ("mel_after", vp), ("target", vp), ("mel_len", vp), ("loss_out", vp), ("g_heads", vp),
        ("g_after", vp), ("workspace", vp), ("ws_bytes", sz), ("heads_ld", i64),
        ("batch", i32), ("t", i32), ("n_mels", i32), ("grad_dtype", i32), ("pos_weight", f32), ("grad_scale", f32),
        ("separate_grads", i32),
    ]


class AdamArgs(C.Structure):
    _fields_ = [
        ("params", vp), ("grads", vp), ("exp_avg", vp), ("exp_avg_sq", vp), ("shadow_bf16", vp), ("step", vp),
        ("workspace", vp), ("ws_bytes", sz), ("n", i64),
        ("lr", f32), ("beta1", f32), ("beta2", f32), ("eps", f32), ("weight_decay", f32), ("clip_norm", f32),
        ("warmup", f32), ("noam", i32), ("d_model", i32), ("norm_parts", vp), ("norm_nparts", i32), ("gate", vp),
    ]


P_ = C.POINTER
SIGNATURES.update({
    "tt2_reduce_rows": ([P_(ReduceArgs), vp], C.c_int),
    "tt2_sumsq_parts": ([vp, i64, vp, C.c_int32, vp], C.c_int),
    "tt2_colsum_workspace_size": ([C.c_int, C.c_int], sz),
    "tt2_colsum": ([vp, C.c_int, i64, C.c_int, C.c_int, vp, f32, vp, sz, vp], C.c_int),
    "tt2_layernorm_fwd": ([P_(LnArgs), vp], C.c_int),
    "tt2_layernorm_bwd_workspace_size": ([P_(LnArgs)], sz),
    "tt2_layernorm_bwd": ([P_(LnArgs), vp], C.c_int),
    "tt2_layernorm_bwd_finalize": ([P_(LnArgs), vp], C.c_int),
    "tt2_reflect_pad": ([vp, i64, vp, C.c_int32, C.c_int32, vp, i64, C.c_int32, vp], C.c_int),
    "tt2_spec_magnitude": ([vp, i64, C.c_int32, C.c_int32, vp, i64, vp], C.c_int),
    "tt2_spec_rephase": ([vp, i64, vp, i64, C.c_int32, C.c_int32, vp, i64, vp], C.c_int),
    "tt2_overlap_add": ([vp, i64, vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, vp, i64, vp], C.c_int),
    "tt2_mel_rows": ([vp, i64, vp, vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_float, C.c_int32, vp],
                     C.c_int),
    "tt2_ln_combine": ([vp, vp, C.c_int32, vp, vp, vp, vp, C.c_int32, C.c_int32, C.c_float, C.c_int32, vp], C.c_int),
    "tt2_batchnorm_workspace_size": ([P_(BnArgs)], sz),
    "tt2_batchnorm_fwd": ([P_(BnArgs), vp], C.c_int),
    "tt2_batchnorm_bwd": ([P_(BnArgs), vp], C.c_int),
    "tt2_batchnorm_sync_size": ([P_(BnArgs)], sz),
    "tt2_batchnorm_fwd_stats": ([P_(BnArgs), vp], C.c_int),
    "tt2_batchnorm_fwd_apply": ([P_(BnArgs), vp], C.c_int),
    "tt2_batchnorm_bwd_stats": ([P_(BnArgs), vp], C.c_int),
    "tt2_batchnorm_bwd_apply": ([P_(BnArgs), vp], C.c_int),
    "tt2_embedding_fwd": ([vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp], C.c_int),
    "tt2_embedding_bwd": ([vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp], C.c_int),
    "tt2_posenc_fwd": ([P_(PeArgs), vp], C.c_int),
    "tt2_posenc_bwd_workspace_size": ([], sz),
    "tt2_posenc_bwd": ([P_(PeArgs), vp], C.c_int),
    "tt2_shift_right": ([vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp], C.c_int),
    "tt2_cast2d": ([vp, C.c_int, i64, vp, C.c_int, i64, C.c_int, C.c_int, vp], C.c_int),
    "tt2_loss_workspace_size": ([], sz),
    "tt2_tts_loss": ([P_(LossArgs), vp], C.c_int),
    "tt2_conv_weight_flip": ([vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp], C.c_int),
    "tt2_conv_weight_flip_batch": ([C.POINTER(WflipJob), i32, i32, vp], C.c_int),
    "tt2_adam_workspace_size": ([], sz),
    "tt2_adam_step": ([P_(AdamArgs), vp], C.c_int),
    "tt2_step_bump": ([vp, vp, vp], C.c_int),
    "tt2_adam_gate": ([vp, vp, C.c_int32, vp], C.c_int),
    "tt2_capture_joined": ([vp, C.POINTER(vp), C.c_int32, C.POINTER(C.c_int32)], C.c_int),
})


class AttnDecodeArgs(C.Structure):
    _fields_ = [
        ("q", vp), ("k", vp), ("v", vp), ("out", vp),
        ("q_ld", i64), ("k_bstride", i64), ("k_ld", i64), ("v_bstride", i64), ("v_ld", i64), ("o_ld", i64),
        ("key_len", vp), ("t_ptr", vp),
        ("batch", i32), ("heads", i32), ("head_dim", i32), ("tk", i32), ("dtype", i32),
        ("scale", f32),
        ("stop_len", vp), ("step", vp),
        ("wo", vp), ("wo_ld", i64), ("slab", vp),
        ("wq", vp), ("wq_ld", i64), ("bq", vp),
        ("ln_part", vp), ("ln_bias", vp), ("ln_gamma", vp), ("ln_beta", vp), ("ln_out", vp), ("ln_eps", f32),
    ]


MAX_DEC_LAYERS = 16


class DecLayer(C.Structure):
    _fields_ = [(n, vp) for n in (
        "qkv_w", "qkv_b", "o_w", "o_b", "ln1_g", "ln1_b", "cq_w", "cq_b", "co_w", "co_b", "ln2_g", "ln2_b",
        "ffn1_w", "ffn1_b", "ffn2_w", "ffn2_b", "ln3_g", "ln3_b")]


class DecodeDesc(C.Structure):
    _fields_ = [
        ("batch", i32), ("text_len", i32), ("t_max", i32), ("n_layers", i32), ("d_model", i32), ("n_heads", i32),
        ("d_ffn", i32), ("n_mels", i32), ("prenet_dim", i32), ("dtype", i32), ("schedule", i32),
        ("ln_eps", f32), ("prenet_dropout", f32), ("stop_logit", f32),
        ("fc1_w", vp), ("fc1_b", vp), ("fc2_w", vp), ("fc2_b", vp), ("proj_w", vp), ("proj_b", vp),
        ("alpha", vp), ("pe_table", vp),
        ("layers", DecLayer * MAX_DEC_LAYERS),
        ("heads_w", vp), ("heads_b", vp),
        ("mem_kv", vp), ("text_lens", vp),
        ("mel_seq", vp), ("stop_seq", vp), ("stop_len", vp), ("stop_bias", vp), ("step", vp), ("seed", vp),
        ("workspace", vp), ("ws_bytes", sz),
    ]


class FfnDecodeArgs(C.Structure):
    _fields_ = [
        ("x", vp), ("w1", vp), ("b1", vp), ("w2", vp), ("b2", vp), ("gamma", vp), ("beta", vp),
        ("hidden", vp), ("slab", vp), ("sync", vp), ("y", vp),
        ("m", i32), ("d_model", i32), ("d_ffn", i32), ("dtype", i32), ("eps", f32),
    ]


SIGNATURES.update({
    "tt2_attn_decode": ([C.POINTER(AttnDecodeArgs), vp], C.c_int),
    "tt2_ffn_decode": ([C.POINTER(FfnDecodeArgs), vp], C.c_int),
    "tt2_ffn_decode_stamps": ([C.POINTER(FfnDecodeArgs), vp, vp], C.c_int),
    "tt2_kv_append": ([vp, i64, vp, i64, i64, C.c_int, C.c_int, vp, C.c_int, vp], C.c_int),
    "tt2_decode_emit": ([vp, i64, C.c_int, C.c_int, C.c_int, vp, vp, vp, C.c_int, vp, vp, vp, vp, f32, vp], C.c_int),
    "tt2_decode_workspace_size": ([C.POINTER(DecodeDesc)], sz),
    "tt2_decode_reset": ([C.POINTER(DecodeDesc), u32, vp], C.c_int),
    "tt2_decode_step": ([C.POINTER(DecodeDesc), vp], C.c_int),
    "tt2_decode_graph_create": ([C.POINTER(DecodeDesc), vp, C.POINTER(vp)], C.c_int),
    "tt2_decode_graph_create_n": ([C.POINTER(DecodeDesc), i32, vp, C.POINTER(vp)], C.c_int),
    "tt2_decode_graph_launch": ([vp, i32, vp], C.c_int),
    "tt2_decode_graph_destroy": ([vp], C.c_int),
})


class Desc(C.Structure):
    """tt2_desc: shape and options of one block-level call (include/tt2_capi.h)."""
    _fields_ = [
        ("batch", i32), ("tq", i32), ("tk", i32), ("d_model", i32), ("n_heads", i32), ("d_ffn", i32),
        ("c_in", i32), ("c_out", i32), ("kernel", i32), ("dtype", i32), ("causal", i32), ("cross", i32),
        ("act", i32), ("training", i32), ("eps", f32), ("momentum", f32), ("dropout", f32),
        ("seed", vp), ("site", u32), ("k_len", vp), ("mel_len", vp), ("n_mels", i32), ("heads_ld", i32),
        ("pos_weight", f32), ("grad_scale", f32),
    ]


_PD = C.POINTER(Desc)
SIGNATURES.update({
    "tt2_attn_block_saved_size": ([_PD], sz),
    "tt2_attn_block_workspace_size": ([_PD], sz),
    "tt2_attn_block_fwd": ([_PD] + [vp] * 11 + [sz, vp], C.c_int),
    "tt2_attn_block_bwd": ([_PD] + [vp] * 17 + [sz, vp], C.c_int),
    "tt2_ffn_saved_size": ([_PD], sz),
    "tt2_ffn_workspace_size": ([_PD], sz),
    "tt2_ffn_fwd": ([_PD] + [vp] * 10 + [sz, vp], C.c_int),
    "tt2_ffn_bwd": ([_PD] + [vp] * 15 + [sz, vp], C.c_int),
    "tt2_linear_workspace_size": ([_PD], sz),
    "tt2_linear_fwd": ([_PD] + [vp] * 5 + [sz, vp], C.c_int),
    "tt2_linear_bwd": ([_PD] + [vp] * 7 + [sz, vp], C.c_int),
    "tt2_add_ln_saved_size": ([_PD], sz),
    "tt2_add_ln_workspace_size": ([_PD], sz),
    "tt2_add_ln_fwd": ([_PD] + [vp] * 6 + [vp], C.c_int),
    "tt2_add_ln_bwd": ([_PD] + [vp] * 10 + [sz, vp], C.c_int),
    "tt2_conv1d_bn_act_saved_size": ([_PD], sz),
    "tt2_conv1d_bn_act_workspace_size": ([_PD], sz),
    "tt2_conv1d_bn_act_fwd": ([_PD] + [vp] * 8 + [i32, vp, vp, vp, sz, vp], C.c_int),
    "tt2_conv1d_bn_act_bwd": ([_PD] + [vp] * 12 + [sz, vp], C.c_int),
    "tt2_conv_weight_pack": ([vp, vp, i32, i32, i32, i32, vp], C.c_int),
    "tt2_heads_workspace_size": ([_PD], sz),
    "tt2_heads_fwd": ([_PD] + [vp] * 5 + [sz, vp], C.c_int),
    "tt2_heads_bwd": ([_PD] + [vp] * 7 + [sz, vp], C.c_int),
    "tt2_loss_block_workspace_size": ([_PD], sz),
    "tt2_loss_fwd": ([_PD] + [vp] * 5 + [sz, vp], C.c_int),
    "tt2_loss_bwd": ([_PD] + [vp] * 7 + [sz, vp], C.c_int),
    "tt2_allreduce_bucket": ([vp, sz, i32, vp, vp], C.c_int),
    "tt2_comm_unique_id": ([vp], C.c_int),
    "tt2_comm_init": ([C.POINTER(vp), i32, vp, i32], C.c_int),
    "tt2_comm_destroy": ([vp], C.c_int),
    "tt2_comm_standin": ([vp, vp, sz, C.c_double, i32, vp, vp], C.c_int),
})
