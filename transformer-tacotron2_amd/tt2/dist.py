"""Data parallelism: utterance sharding + bucketed gradient all-reduce.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
Rank r trains on its own B utterances; the loss kernel pre-scales every
gradient by 1/world_size, so a SUM all-reduce of the flat f32 gradient buffer
yields the data-parallel mean.  The buffer is cut into ~25 MB buckets from the
END of the flat layout, because the backward produces gradients roughly in
reverse layout order (post-net, heads, decoder 5..0, ..., encoder embedding):
``ready(offset)`` is called by the engine whenever every gradient at flat index
>= offset is final and launches the buckets that became complete, so the
all-reduce of late layers overlaps the backward of early ones (RCCL runs on its
own stream, ordered after the producing kernels).  ``finish()`` launches the
rest and makes the current stream wait for all of them before the optimizer.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


class GradSync:
    def __init__(self, flat_grads: torch.Tensor, bucket_bytes: int = 25 << 20, group=None):
        self.flat = flat_grads
        self.group = group
        n = flat_grads.numel()
        per = max(1, bucket_bytes // flat_grads.element_size())
        self.buckets = []
        hi = n
        while hi > 0:
            lo = max(0, hi - per)
            self.buckets.append((lo, hi))
            hi = lo
        self.reset()

    @property
    def world(self) -> int:
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    def reset(self):
        self.next = 0
        self.works = []

    def _launch(self, lo, hi):
        w = dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self.works.append(w)

    def ready(self, offset: int):
        """Every gradient at flat index >= offset is final."""
        for i in self.take_ready(offset):
            self._launch(*self.buckets[i])

    def take_ready(self, offset: int) -> list[int]:
        """Indices of the buckets that became complete at offset (advances the cursor
        without launching: a captured step records where its buckets can go)."""
        out = []
        while self.next < len(self.buckets) and self.buckets[self.next][0] >= offset:
            out.append(self.next)
            self.next += 1
        return out

    def launch(self, idx: list[int]):
        """Launch the given buckets (in order) and advance the cursor past them."""
        for i in idx:
            self._launch(*self.buckets[i])
            self.next = max(self.next, i + 1)

    def finish(self):
        while self.next < len(self.buckets):
            self._launch(*self.buckets[self.next])
            self.next += 1
        for w in self.works:
            w.wait()
        self.reset()


def init_from_env(backend: str | None = None):
    """Initialise torch.distributed from torchrun's env (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT).  Returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            # TT2_DIST_BACKEND=gloo: rehearse the multi-rank control flow on one GPU
            backend = os.environ.get("TT2_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return rank, world, local


def attach(model, group=None, bucket_bytes: int = 25 << 20) -> GradSync:
    """Wire a TransformerTTS for data parallelism: gradient pre-scaling and the
    bucket hook.  Returns the GradSync whose finish() goes between backward and
    the optimizer step (pass it as train_step(..., sync_grads=sync.finish))."""
    eng = model.engine
    sync = GradSync(eng.grads, bucket_bytes, group)
    eng.grad_scale = 1.0 / sync.world
    eng.grad_ready_hook = sync.ready
    return sync


def broadcast_params(model, src: int = 0, group=None):
    """Make every replica start from rank src's weights and BN statistics."""
    eng = model.engine
    dist.broadcast(eng.params, src, group=group)
    dist.broadcast(eng.stats, src, group=group)
    eng.sync_shadow()
