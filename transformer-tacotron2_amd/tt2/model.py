"""TransformerTTS -- the drop-in model API of SURVEY 8(b) on the MI355X engine.

A reference-shaped training script works unchanged (torch.nn.Module + autograd):

    model = TransformerTTS(cfg, dtype=torch.bfloat16)
    model.load_state_dict(sd)                      # SURVEY 8(b) checkpoint layout
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    out = model(text, text_len, mel, mel_len)      # (mel_before, mel_after, stop_logits, None)
    total, parts = model.loss(out, mel, mel_len)   # honours its arguments
    opt.zero_grad(); total.backward(); opt.step()

and so does the engine's own fused fast path (no autograd, one hipGraph per step):

    model.train_step(text, text_len, mel, mel_len) # fwd + loss + bwd + fused Adam/clip/Noam
    model.loss(); model.backward()                 # loss / grads of the last forward

Every compute step runs in libtt2's gfx950 kernels; there is no CPU or
PyTorch-op fallback (a missing library or GPU raises).  The autograd boundary is two
torch.autograd.Functions: the whole forward (its backward is the engine's hand-written
backward, which writes the flat gradient buffer) and the fused loss kernel.

parameters() are views of the engine's flat f32 master buffer in the INTERNAL layout
(conv weights [Cout][tap][Cin], the six cross-attention K/V projections as one slot, mel +
stop heads as one [81, 512] slot; names ``slots.<slot>``); state_dict() stays in the
checkpoint layout.  An external optimizer updates the master weights in place; the bf16
shadow the kernels read is refreshed at the next forward (version-counter check).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
from torch.autograd.function import once_differentiable

from . import ops
from .capture import StepCapture
from .config import TTSConfig
from .engine import Arena, TTSEngine
from .params import from_state_dict, grads_to_state_dict_names, to_state_dict


class _TTSForward(torch.autograd.Function):
    """Teacher-forced forward as one autograd node; backward = the engine's backward from
    the output gradients (it rewrites the flat gradient buffer; a copy is handed to
    autograd, which accumulates it into each parameter's .grad)."""

    @staticmethod
    def forward(ctx, model, text, text_len, mel, mel_len, *params):
        A = model._run_forward(text, text_len, mel, mel_len)
        ctx.model, ctx.A, ctx.gen = model, A, A.gen
        return model.outputs(A)[:3]

    @staticmethod
    @once_differentiable
    def backward(ctx, g_before, g_after, g_stop):
        model, A = ctx.model, ctx.A
        if A.gen != ctx.gen:
            raise RuntimeError("TransformerTTS: another forward of the same (B, Tx, Ty) shape overwrote the "
                               "activations this backward needs; call backward before the next forward")
        model._stage_output_grads(A, g_before, g_after, g_stop)
        e = model.engine
        e.backward(A)
        if e.training:   # fresh dropout masks for the next step (the fused path bumps in its optimizer)
            ops.step_bump(model._seed_steps, e.seed)
        flat = e.grads.clone()
        return (None,) * 5 + tuple(e.lay.view(flat, n) for n in model._slot_names)


class _TTSLoss(torch.autograd.Function):
    """The fused loss kernel (masked MSE x 2 + BCE(pos_weight)) on the GIVEN outputs and
    targets; it writes d(total)/d(outputs) alongside the loss, backward scales them."""

    @staticmethod
    def forward(ctx, model, mel_before, mel_after, stop, mel, mel_len):
        L, gb, ga, gs = model._run_loss(mel_before, mel_after, stop, mel, mel_len)
        ctx.save_for_backward(gb, ga, gs)
        parts = (L[1].clone(), L[2].clone(), L[3].clone())
        ctx.mark_non_differentiable(*parts)
        return (L[0].clone(),) + parts

    @staticmethod
    @once_differentiable
    def backward(ctx, g_total, *_):
        gb, ga, gs = ctx.saved_tensors
        return None, gb * g_total, ga * g_total, gs * g_total, None, None


class TransformerTTS(nn.Module):
    def __init__(self, cfg: TTSConfig | None = None, dtype: torch.dtype = torch.bfloat16, device="cuda",
                 seed: int = 0):
        super().__init__()
        self.cfg = cfg or TTSConfig()
        self.engine = e = TTSEngine(self.cfg, dtype, device, seed)
        self._last: Arena | None = None
        self._graphs: dict = {}
        self._loss_bufs: dict = {}
        self._slot_names = list(e.lay.slots)
        self.metrics = None   # StepMetrics (enable_metrics / TT2_METRICS): one JSONL line per step
        if os.environ.get("TT2_METRICS"):
            self.enable_metrics(os.environ["TT2_METRICS"])
        # parameters alias the flat master buffer (in-place optimizer updates land in it)
        self.slots = nn.ParameterDict({n.replace(".", "__"): nn.Parameter(e.P(n)) for n in self._slot_names})
        # the autograd Function's inputs and returned gradients follow the ParameterDict's order
        key2slot = {n.replace(".", "__"): n for n in self._slot_names}
        self._slot_names = [key2slot[k] for k in self.slots.keys()]
        self._shadow_version = e.params._version
        self._seed_steps = torch.zeros(1, dtype=torch.int32, device=e.dev)

    def _apply(self, fn, recurse=True):
        raise NotImplementedError("TransformerTTS parameters live in libtt2's flat buffers: choose device and "
                                  "dtype at construction (TransformerTTS(cfg, dtype=..., device=...))")

    # ------------------------------------------------------------ modes
    def train(self, mode: bool = True):
        super().train(mode)
        self.engine.training = mode
        return self

    def _sync_shadow(self):
        """Refresh the bf16 weight shadow after an in-place update of the master weights
        from outside the engine (an external optimizer, load, manual edits)."""
        e = self.engine
        if e.params._version != self._shadow_version:
            e.sync_shadow()
            self._shadow_version = e.params._version

    def set_seed(self, seed: int):
        """Per-step dropout seed (uint32), same meaning as the oracle's set_seed."""
        self.engine.seed.fill_(seed)

    def pipeline_optimizer(self, on: bool = True):
        """Pipelined optimizer (opt-in): each train step's Adam is deferred to the start of the
        next step's forward, where it runs beside the encoder's forward (the encoder's share on
        the side stream ahead of the encoder, the rest ahead of the decoder).  Every update is
        the same as without it, in the same order, so the trajectory is identical; the
        parameters lag one Adam behind until flush_optimizer() (which state_dict(),
        save_checkpoint() and infer() call).  A captured step must be taken after at least one
        pipelined eager step (its graph then holds the deferred Adam).  Whether an update is
        pending is a device flag the deferred Adam checks, so flushing between replays (a
        checkpoint, an eval) never applies an update twice."""
        if not on:
            self.engine.flush_optimizer()
        self.engine.pipeline_opt = on

    def flush_optimizer(self):
        """Run a pipelined step's pending Adam now."""
        self.engine.flush_optimizer()

    # ------------------------------------------------------------ checkpoint
    def state_dict(self):
        e = self.engine
        e.flush_optimizer()
        return to_state_dict(self.cfg, e.lay, e.params, e.slay, e.stats, e.nbt)

    def load_state_dict(self, sd, strict: bool = True):
        P, S, nbt = from_state_dict(self.cfg, sd)
        self.engine.drop_pending_update()   # a pending pipelined Adam belongs to the replaced weights
        self.engine.load_slots(P, S, nbt)
        self._shadow_version = self.engine.params._version

    def save_checkpoint(self, path: str):
        """Training checkpoint: the SURVEY 8(b) state_dict, the Adam
        moments in the same checkpoint naming (so the file does not depend on the internal
        flat layout), the optimizer step, its hyper-parameters and the dropout-seed RNG state.
        Written with torch.save; load_checkpoint resumes bit for bit."""
        e = self.engine
        e.flush_optimizer()
        ck = {"format": "tt2-train-1", "cfg": self.cfg.to_dict(), "model": self.state_dict(),
              "rng": {"dropout_seed": int(e.seed.item()) & 0xFFFFFFFF}}
        if e.exp_avg is not None:
            zs = torch.zeros_like(e.stats)
            mom = lambda buf: {k: v for k, v in to_state_dict(self.cfg, e.lay, buf, e.slay, zs, {}).items()  # noqa: E731
                               if "running_" not in k and "num_batches" not in k}
            ck["optimizer"] = {"exp_avg": mom(e.exp_avg), "exp_avg_sq": mom(e.exp_avg_sq),
                               "step": int(e.step_t.item()), "hparams": dict(e.opt)}
        torch.save(ck, path)

    def load_checkpoint(self, path: str):
        """Resume from save_checkpoint (tensors only: torch.load(weights_only=True))."""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        if ck.get("format") != "tt2-train-1":
            raise ValueError(f"{path}: not a tt2 training checkpoint")
        if ck["cfg"] != self.cfg.to_dict():
            raise ValueError(f"{path}: config mismatch")
        self.load_state_dict(ck["model"])
        e = self.engine
        opt = ck.get("optimizer")
        if opt is not None:
            e.init_optimizer(**opt["hparams"])
            model_sd = ck["model"]
            for buf, key in ((e.exp_avg, "exp_avg"), (e.exp_avg_sq, "exp_avg_sq")):
                full = {k: opt[key].get(k, v) for k, v in model_sd.items()}   # stats keys: placeholders
                P, _, _ = from_state_dict(self.cfg, full)
                with torch.no_grad():
                    for k, v in P.items():
                        e.lay.view(buf, k).copy_(v.reshape(e.lay.view(buf, k).shape))
            e.step_t.fill_(opt["step"])
        seed = ck["rng"]["dropout_seed"]
        e.seed.fill_(seed - (1 << 32) if seed >= (1 << 31) else seed)

    def grads_state_dict(self):
        e = self.engine
        return grads_to_state_dict_names(self.cfg, e.lay, e.grads)

    def n_params(self) -> int:
        return self.engine.lay.n_params()

    # ------------------------------------------------------------ forward / loss / backward
    def input_buffers(self, B: int, Tx: int, Ty: int):
        """The step's own input tensors for shape (B, Tx, Ty): text [B, Tx] int64, text_len [B]
        int32, mel [B, Ty, 80] f32, mel_len [B] int32 (the arena's, which the kernels read).  A
        train_step / captured run handed exactly these tensors reads them in place, with no staging
        copies in front of the step (the static-input pattern of graph replay: a data loader
        writes the next batch into them, e.g. by non_blocking copies on a side stream)."""
        A = self.engine.arena(B, Tx, Ty)
        return A["text"].view(B, Tx), A["text_len"], A["mel"], A["mel_len"]

    @staticmethod
    def _is_arena_input(A: Arena, text, text_len, mel, mel_len) -> bool:
        return (text.data_ptr() == A["text"].data_ptr() and text_len.data_ptr() == A["text_len"].data_ptr()
                and mel.data_ptr() == A["mel"].data_ptr() and mel_len.data_ptr() == A["mel_len"].data_ptr()
                and text.dtype == torch.int64 and text_len.dtype == mel_len.dtype == torch.int32
                and mel.dtype == torch.float32)

    def _stage_into(self, A: Arena, text, text_len, mel, mel_len):
        if not self._is_arena_input(A, text, text_len, mel, mel_len):
            dev = self.engine.dev
            self.engine.stage_inputs(A, text.to(dev), text_len.to(dev, torch.int32), mel.to(dev, torch.float32),
                                     mel_len.to(dev, torch.int32))

    def _stage(self, text, text_len, mel, mel_len) -> Arena:
        B, Tx = text.shape
        Ty = mel.shape[1]
        A = self.engine.arena(B, Tx, Ty)
        self._stage_into(A, text, text_len, mel, mel_len)
        return A

    def _run_forward(self, text, text_len, mel, mel_len) -> Arena:
        self._sync_shadow()
        A = self._stage(text, text_len, mel, mel_len)
        A.gen += 1
        self.engine.forward(A)
        self._last = A
        return A

    def forward(self, text, text_len, mel, mel_len):
        """Teacher-forced forward (shift-right with a zero go frame).  Returns
        (mel_before [B,Ty,80], mel_after [B,Ty,80], stop_logits [B,Ty], None), f32.
        With grad mode on, the outputs carry an autograd node whose backward runs the
        engine's backward (so loss.backward() fills every parameter's .grad)."""
        params = list(self.slots.values())
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            mb, ma, st = _TTSForward.apply(self, text, text_len, mel, mel_len, *params)
            return mb, ma, st, None
        return self.outputs(self._run_forward(text, text_len, mel, mel_len))

    def _stage_output_grads(self, A: Arena, g_before, g_after, g_stop):
        """d(loss)/d(outputs) -> the engine's backward inputs: g_heads (f32 [Md, 96]: mel
        columns = d/d(mel_before) + d/d(mel_after), the post-net's residual path; column 80 =
        d/d(stop)) and g_after (the post-net output gradient)."""
        c = self.cfg
        Md = A.Md
        gh = A["g_heads"]
        z = lambda: torch.zeros(Md, c.n_mels, device=gh.device)  # noqa: E731
        gb = z() if g_before is None else g_before.reshape(Md, c.n_mels).float()
        ga = z() if g_after is None else g_after.reshape(Md, c.n_mels).float()
        gh[:, :c.n_mels].copy_(gb + ga)
        gh[:, c.n_mels].copy_(torch.zeros(Md, device=gh.device) if g_stop is None else g_stop.reshape(Md))
        A["g_after"].copy_(ga)

    def _run_loss(self, mel_before, mel_after, stop, mel, mel_len):
        """Loss kernel over the given tensors (staged into per-shape buffers); returns the
        loss vector and d(total)/d(mel_before, mel_after, stop)."""
        c, e = self.cfg, self.engine
        B, Ty = mel.shape[0], mel.shape[1]
        key = (B, Ty)
        S = self._loss_bufs.get(key)
        if S is None:
            f = lambda *sh: torch.zeros(*sh, dtype=torch.float32, device=e.dev)  # noqa: E731
            S = self._loss_bufs[key] = dict(heads=f(B * Ty, 96), after=f(B * Ty, c.n_mels), mel=f(B, Ty, c.n_mels),
                                            mel_len=torch.zeros(B, dtype=torch.int32, device=e.dev), loss=f(4),
                                            g_heads=f(B * Ty, 96), g_after=f(B * Ty, c.n_mels))
        Md = B * Ty
        S["heads"][:, :c.n_mels].copy_(mel_before.detach().reshape(Md, c.n_mels))
        S["heads"][:, c.n_mels].copy_(stop.detach().reshape(Md))
        S["after"].copy_(mel_after.detach().reshape(Md, c.n_mels))
        S["mel"].copy_(mel)
        S["mel_len"].copy_(mel_len)
        ops.tts_loss(S["heads"], 96, S["after"], S["mel"], S["mel_len"], S["loss"], S["g_heads"], S["g_after"], B,
                     Ty, c.n_mels, c.stop_pos_weight, 1.0, ws=e.ws, separate_grads=True)
        gb = S["g_heads"][:, :c.n_mels].reshape(B, Ty, c.n_mels).clone()
        gs = S["g_heads"][:, c.n_mels].reshape(B, Ty).clone()
        ga = S["g_after"].reshape(B, Ty, c.n_mels).clone()
        return S["loss"], gb, ga, gs

    def outputs(self, A: Arena):
        c = self.cfg
        B, Ty = A.B, A.Ty
        heads = A["heads"]
        mel_before = heads[:, :c.n_mels].reshape(B, Ty, c.n_mels).clone()
        stop = heads[:, c.n_mels].reshape(B, Ty).clone()
        mel_after = A["mel_after"].view(B, Ty, c.n_mels).clone()
        return mel_before, mel_after, stop, None

    def loss(self, outputs=None, mel=None, mel_len=None):
        """loss(outputs, mel, mel_len): the TTS loss of the given outputs (mel_before,
        mel_after, stop_logits, ...) against mel / mel_len, differentiable w.r.t. the outputs.
        loss() with no outputs: the engine fast path -- the loss of the last forward against
        the mel it was given (or mel / mel_len if passed), feeding backward().
        Returns (total, {"mel_before", "mel_after", "stop"}) as device scalars."""
        if outputs is not None:
            if mel is None or mel_len is None:
                raise ValueError("loss(outputs, mel, mel_len): mel and mel_len are required with outputs")
            dev = self.engine.dev
            total, lb, la, ls = _TTSLoss.apply(self, outputs[0], outputs[1], outputs[2],
                                               mel.to(dev, torch.float32), mel_len.to(dev, torch.int32))
            return total, {"mel_before": lb, "mel_after": la, "stop": ls}
        A = self._last
        if A is None:
            raise RuntimeError("loss() needs a forward() first")
        if mel is not None:
            A["mel"].copy_(mel)
        if mel_len is not None:
            A["mel_len"].copy_(mel_len)
        self.engine.loss(A)
        L = A["loss"]
        return L[0], {"mel_before": L[1], "mel_after": L[2], "stop": L[3]}

    def backward(self):
        if self._last is None:
            raise RuntimeError("backward() needs forward() + loss() first")
        self.engine.backward(self._last)

    # ------------------------------------------------------------ inference
    def infer(self, text, text_len, max_len: int, stop_threshold: float | None = 0.5, use_graph: bool = True,
              prenet_dropout: bool = True):
        """Greedy AR synthesis (hipGraph-replayed decode step, KV cache, cached
        cross K/V).  Returns (mel_after [B, T, 80] f32, out_len [B]).
        stop_threshold=None forces max_len frames.  prenet_dropout: Tacotron2's pre-net
        dropout stays on at inference; False switches it off (parity runs)."""
        self.engine.flush_optimizer()
        from .infer import Decoder
        self._sync_shadow()
        B, Tx = text.shape
        key = (B, Tx, max_len, prenet_dropout)
        dec = self._decoders.get(key) if hasattr(self, "_decoders") else None
        if dec is None:
            self._decoders = getattr(self, "_decoders", {})
            dec = Decoder(self.engine, B, Tx, max_len, prenet_dropout=prenet_dropout)
            self._decoders[key] = dec
        dev = self.engine.dev
        return dec.run(text.to(dev), text_len.to(dev), max_len, stop_threshold, use_graph)

    # ------------------------------------------------------------ diagnostics
    def alignments(self, layer: int = -1) -> torch.Tensor:
        """Encoder-decoder attention of decoder layer `layer` from the last forward:
        [B, H, Ty, Tx] f32 (rows sum to 1 over the valid phonemes).
        Recomputed on the GPU from the saved query, memory keys and log-sum-exp."""
        if self._last is None:
            raise RuntimeError("alignments() needs a forward first")
        e, A, c = self.engine, self._last, self.cfg
        l = layer % c.n_dec
        d, H = c.d_model, c.n_heads
        kvld = c.n_dec * 2 * d
        probs = torch.empty(A.B, H, A.Ty, A.Tx, dtype=torch.float32, device=e.dev)
        from . import ops
        ops.attn_probs(A[f"dcq{l}"], A["mkv"][:, 2 * d * l:], A[f"dclse{l}"], probs, d, kvld, A.B, H, A.Ty, A.Tx,
                       key_len=A["text_len"], scale=1.0 / math.sqrt(c.head_dim))
        return probs

    @staticmethod
    def diagonal_focus(align: torch.Tensor, text_len: torch.Tensor, mel_len: torch.Tensor) -> torch.Tensor:
        """Per-utterance focus rate: mean over valid frames of the max attention weight
        (averaged over heads) -- near 1 for a sharp monotonic alignment."""
        a = align.mean(1)
        B, Ty, _ = a.shape
        valid = torch.arange(Ty, device=a.device)[None, :] < mel_len.to(a.device)[:, None]
        mx = a.amax(-1)
        return (mx * valid).sum(1) / valid.sum(1).clamp_min(1)

    # ------------------------------------------------------------ training
    def configure_optimizer(self, **kw):
        self.engine.init_optimizer(**kw)

    def _step_body(self, A: Arena, sync_grads=None):
        e = self.engine
        e.forward(A)
        e.loss(A)
        e.backward(A)
        if sync_grads is not None:
            sync_grads()
        e.optimizer_step()

    def enable_metrics(self, path: str | None, world: int | None = None):
        """Per-step JSONL metrics (tt2/metrics.py) appended to `path`; None turns them off.
        world: ranks whose frames count in frames/s (default: torch.distributed's world size,
        looked up when the first line is written, so a model built before
        init_process_group still reports the whole job)."""
        from .metrics import StepMetrics
        if self.metrics is not None:
            self.metrics.close()
            self.metrics = None
        if path:
            self.metrics = StepMetrics(path, self.cfg, world)

    def _metrics_end(self, A: Arena, sync_grads):
        self.metrics.end(A["loss"], A.B, A.Tx, A.Ty, sync=getattr(sync_grads, "__self__", None), mel_len=A["mel_len"])

    def train_step(self, text, text_len, mel, mel_len, sync_grads=None):
        """One optimisation step, eagerly.  Returns the device loss vector
        [total, mse_before, mse_after, bce_stop] (no host sync)."""
        if self.engine.exp_avg is None:
            self.engine.init_optimizer()
        if self.metrics is not None:
            self.metrics.begin()
        self._sync_shadow()
        A = self._stage(text, text_len, mel, mel_len)
        self._step_body(A, sync_grads)
        self._last = A
        if self.metrics is not None:
            self._metrics_end(A, sync_grads)
        return A["loss"]

    def capture_train_step(self, B: int, Tx: int, Ty: int, sync_grads=None):
        """Capture fwd + loss + bwd + Adam for one shape into a hipGraph (via
        torch.cuda.CUDAGraph, which records our kernels on its capture stream).
        Returns a callable run(text, text_len, mel, mel_len) -> loss vector."""
        e = self.engine
        if e.bn_sync is not None and not e.bn_sync.in_graph:
            raise RuntimeError("capture_train_step: SyncBatchNorm over torch.distributed (gloo) exchanges "
                               "inside the forward and backward and cannot be captured; use train_step, or "
                               "the nccl backend (RCCL, captured)")
        if e.exp_avg is None:
            e.init_optimizer()
        if e.pipeline_opt and e._adam_parts is None:
            raise RuntimeError("capture_train_step: with the pipelined optimizer, capture after an eager step "
                               "(the graph holds that step's deferred Adam)")
        A = e.arena(B, Tx, Ty)
        # the caller's warm-up eager steps size every workspace; capture must not allocate.
        # Every arena buffer exists before capture (the warm-ups may have run the overlapped
        # backward, which uses per-layer copies in place of some shared scratch buffers)
        A.materialize()
        nbt_saved = dict(e.nbt)
        hook, e.grad_ready_hook = e.grad_ready_hook, None
        sync = getattr(sync_grads, "__self__", None)   # a GradSync's bound finish(): overlap buckets
        if sync is not None and getattr(sync, "in_graph", False):
            return self._capture_in_graph(A, sync, hook, nbt_saved)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g2 = torch.cuda.CUDAGraph() if sync_grads is not None else None
        # the segmented capture ends graphs inside the backward, where the overlapped weight
        # gradients' side stream (engine.wgrad_overlap) would still be forked: off for it
        # (only the gloo / TT2_DP_SYNC=segmented path takes this branch;
        # the nccl path at N > 1 is the one-graph capture below, with the side stream)
        ov_saved = e.wgrad_overlap
        if sync is not None and hasattr(sync, "take_ready"):
            e.wgrad_overlap = False
        segs = []   # [(graph, bucket indices launched right after its replay)]
        streams = lambda: self._capture_streams(sync)   # noqa: E731
        # captures are thread-local: RCCL's watchdog thread polls its work events during
        # capture, which a global-mode capture treats as a prohibited call (capture invalidated)
        torch.cuda.synchronize()
        cur = [StepCapture(torch.cuda.CUDAGraph(), s, streams, ops.CAPTURE_MODE)]
        try:
            with torch.cuda.stream(s):
                cur[0].begin()
                if sync is not None and hasattr(sync, "take_ready"):
                    # cut the forward+backward graph wherever a gradient bucket becomes final,
                    # so the replay can start that bucket's all-reduce while the rest of the
                    # backward runs (RCCL stays outside the graphs, on its own stream)
                    sync.reset()

                    def cut(offset):
                        if offset <= 0:       # the last buckets go to finish(): no empty tail graph
                            return
                        idx = sync.take_ready(offset)
                        if idx:
                            c, cur[0] = cur[0], None
                            c.end()
                            segs.append((c.graph, idx))
                            cur[0] = StepCapture(torch.cuda.CUDAGraph(), s, streams, ops.CAPTURE_MODE)
                            cur[0].begin()
                    e.grad_ready_hook = cut
                e.forward(A)
                e.loss(A)
                e.backward(A)
                e.grad_ready_hook = None
                if g2 is None:
                    e.optimizer_step()
                c, cur[0] = cur[0], None
                c.end()
                segs.append((c.graph, []))
                if sync is not None and hasattr(sync, "take_ready"):
                    sync.reset()
                if g2 is not None:
                    with StepCapture(g2, s, streams, ops.CAPTURE_MODE):
                        e.optimizer_step()
        except BaseException:
            # a capture left open aborts the process at teardown (~CUDAGraph): end it, drop the
            # graphs, restore the engine, re-raise
            if cur[0] is not None:
                cur[0].abort()
            e.grad_ready_hook = hook
            e.wgrad_overlap = ov_saved
            e.nbt = nbt_saved
            if sync is not None and hasattr(sync, "reset"):
                sync.reset()
            torch.cuda.current_stream().wait_stream(s)
            raise
        torch.cuda.current_stream().wait_stream(s)
        e.grad_ready_hook = hook
        e.wgrad_overlap = ov_saved
        e.nbt = nbt_saved  # capture records kernels only; each replay counts one batch
        self._graphs[(B, Tx, Ty)] = (segs, g2)

        def run(text, text_len, mel, mel_len):
            if self.metrics is not None:
                self.metrics.begin()
            self._stage_into(A, text, text_len, mel, mel_len)
            for g, idx in segs:
                g.replay()
                if idx:
                    sync.launch(idx)  # these buckets' all-reduce overlaps the next segment
            if g2 is not None:
                sync_grads()          # remaining buckets, then wait for all of them
                g2.replay()
            for k in e.nbt:
                e.nbt[k] += 1
            self._last = A
            if self.metrics is not None:
                self._metrics_end(A, sync_grads)
            return A["loss"]

        return run

    def _capture_streams(self, sync=None) -> dict:
        """The streams a captured step may fork into the capture, by role."""
        e = self.engine
        out = {"side": e._side}
        if sync is not None and getattr(sync, "stream", None) is not None:
            out["comm"] = sync.stream
        bn = e.bn_sync
        if bn is not None and getattr(bn, "grad_sync", None) is not None:
            out["bn_comm"] = bn.grad_sync.stream
        return out

    def _capture_in_graph(self, A: Arena, sync, hook, nbt_saved):
        """The data-parallel step as ONE hipGraph: the bucket all-reduces (RcclGradSync)
        fork onto the comm stream inside the capture as each bucket's gradients become
        final, overlap the rest of the backward, and join before Adam."""
        e = self.engine
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        sync.reset()
        try:
            # every stream the step forks (side, comm) is checked joined before the capture
            # ends; an exception ends the capture and re-raises (tt2/capture.py)
            with StepCapture(g, s, lambda: self._capture_streams(sync), ops.CAPTURE_MODE):
                e.grad_ready_hook = sync.ready
                e.forward(A)
                e.loss(A)
                e.backward(A)
                sync.finish()
                e.optimizer_step()
        except BaseException:
            e.nbt = nbt_saved
            torch.cuda.current_stream().wait_stream(s)
            raise
        finally:
            e.grad_ready_hook = hook
            sync.reset()
        torch.cuda.current_stream().wait_stream(s)
        e.nbt = nbt_saved
        self._graphs[(A.B, A.Tx, A.Ty)] = ([(g, [])], None)

        def run(text, text_len, mel, mel_len):
            if self.metrics is not None:
                self.metrics.begin()
            self._stage_into(A, text, text_len, mel, mel_len)
            g.replay()
            for k in e.nbt:
                e.nbt[k] += 1
            self._last = A
            if self.metrics is not None:
                self.metrics.end(A["loss"], A.B, A.Tx, A.Ty, mel_len=A["mel_len"])   # all-reduce span: inside the graph
            return A["loss"]

        return run
