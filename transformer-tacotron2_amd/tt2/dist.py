"""Data parallelism: utterance sharding + bucketed gradient all-reduce.

One process per GPU (torch.distributed for rendezvous, barriers and timing; the gradient
exchange itself is RCCL over xGMI).  Rank r trains on its own B utterances; the loss
kernel pre-scales every gradient by 1/world_size, so a SUM all-reduce of the flat f32
gradient buffer yields the data-parallel mean.  The buffer is cut into ~25 MB buckets
from the END of the flat layout, because the backward produces gradients roughly in
reverse layout order (post-net, heads, decoder 5..0, ..., encoder embedding):
``ready(offset)`` is called by the engine whenever every gradient at flat index
>= offset is final and launches the buckets that became complete, so the all-reduce of
late layers overlaps the backward of early ones.  ``finish()`` launches the rest and
makes the current stream wait for all of them before the optimizer.

Two implementations of that contract:

* ``RcclGradSync`` (the default with the ``nccl`` backend): libtt2's own RCCL
  communicator (``tt2_comm_init`` / ``tt2_allreduce_bucket``, include/tt2_capi.h).  Each
  bucket's all-reduce is issued on a dedicated comm stream that waits for an event on
  the compute stream, and ``finish()`` joins the comm stream back.  Nothing touches the
  host, so the whole step -- forward, backward, the bucket all-reduces overlapped with
  it, Adam -- is captured as ONE hipGraph (``in_graph``): no graph split per bucket.
* ``GradSync`` (gloo, or ``TT2_DP_SYNC=segmented``): torch.distributed async
  all-reduces; a captured step is cut into graph segments at bucket boundaries and the
  all-reduces run between segment replays (gloo work cannot be captured).
"""
from __future__ import annotations

import ctypes as C
import os
from datetime import timedelta

import torch
import torch.distributed as dist

from .capture import check_join_target

# RCCL channel floor for the bucket all-reduce (read by RCCL at communicator init).  A
# ring is bound by one xGMI link (~153 GB/s); more channels spread the ring traffic over
# the 7 links of an MI355X.  Only a floor: an explicit NCCL_MIN_NCHANNELS wins.
RCCL_MIN_CHANNELS = 32
RCCL_ENV_KEYS = ("NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_ALGO", "NCCL_PROTO", "RCCL_MSCCL_ENABLE",
                 "NCCL_P2P_LEVEL")


def rccl_env() -> dict:
    """The RCCL environment in effect (recorded in bench.py's JSON line)."""
    return {k: os.environ[k] for k in RCCL_ENV_KEYS if k in os.environ}


def _buckets(n: int, per: int, cuts=None) -> list[tuple[int, int]]:
    """Buckets [lo, hi) from the end of the flat buffer down.  Without cuts: `per` elements each.
    With cuts (the offsets at which the backward reports gradients final, engine.ready_offsets):
    layer-aligned buckets, one per reported range, a range smaller than per / 4 merged into the
    one below it -- a bucket is then complete as soon as its layer is, where fixed-size buckets
    straddling two layers wait for the lower one."""
    if not cuts:
        out, hi = [], n
        while hi > 0:
            lo = max(0, hi - per)
            out.append((lo, hi))
            hi = lo
        return out
    pts = sorted({c for c in cuts if 0 < c < n} | {0}, reverse=True)
    out, hi = [], n
    for lo in pts:
        if hi - lo < per // 4 and lo > 0:
            continue   # too small: extend down to the next cut
        out.append((lo, hi))
        hi = lo
    return out


class GradSync:
    in_graph = False

    def __init__(self, flat_grads: torch.Tensor, bucket_bytes: int = 25 << 20, group=None, cuts=None):
        self.flat = flat_grads
        self.group = group
        self.buckets = _buckets(flat_grads.numel(), max(1, bucket_bytes // flat_grads.element_size()), cuts)
        self.reset()

    @property
    def world(self) -> int:
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    def reset(self):
        self.next = 0
        self.works = []

    accepts_after = False   # ready(offset, after=event): see RcclGradSync

    def _launch(self, lo, hi, after=None):
        if after is not None:
            torch.cuda.current_stream().wait_event(after)
        w = dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self.works.append(w)

    def ready(self, offset: int, after=None):
        """Every gradient at flat index >= offset is final (on the current stream, or once the
        event `after` has completed)."""
        for i in self.take_ready(offset):
            self._launch(*self.buckets[i], after=after)

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

    def close(self):
        pass

    def bench_allreduce(self, reps: int = 5) -> dict:
        """Times the bucketed all-reduce of the whole gradient buffer on its own (a copy,
        outside any training step): algorithm and bus bandwidth of the exchange."""
        buf = self.flat.clone()
        saved, self.flat = self.flat, buf
        try:
            self.reset()
            self.finish()                      # warm
            torch.cuda.synchronize()
            if dist.is_initialized():
                dist.barrier(group=self.group)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(reps):
                self.finish()
            ev[1].record()
            torch.cuda.synchronize()
            t = ev[0].elapsed_time(ev[1]) / 1e3 / reps
        finally:
            self.flat = saved
            self.reset()
        nbytes = buf.numel() * buf.element_size()
        w = self.world
        return {"bytes": nbytes, "buckets": len(self.buckets), "ms": round(t * 1e3, 3),
                "algbw_GBps": round(nbytes / t / 1e9, 1),
                "busbw_GBps": round(2 * (w - 1) / w * nbytes / t / 1e9, 1) if w > 1 else None}


class RcclGradSync(GradSync):
    """Bucketed SUM all-reduce over libtt2's RCCL communicator on a comm stream, ordered
    after the producing kernels by stream waits only (capturable: ``in_graph``).
    ready(offset, after=event): the comm stream waits for that event instead of the current
    stream (the overlapped backward hands a bucket over after issuing its next side job)."""
    in_graph = True
    accepts_after = True

    def __init__(self, flat_grads: torch.Tensor, bucket_bytes: int = 25 << 20, group=None, cuts=None):
        from . import _lib
        self._lib = _lib
        super().__init__(flat_grads, bucket_bytes, group, cuts)
        os.environ.setdefault("NCCL_MIN_NCHANNELS", str(RCCL_MIN_CHANNELS))
        L = _lib.lib()
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        uid = (C.c_ubyte * 128)()   # ncclUniqueId
        if rank == 0:
            _lib.check(L.tt2_comm_unique_id(uid), "tt2_comm_unique_id")
        if dist.is_initialized() and self.world > 1:
            obj = [bytes(uid)]
            dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                       group=group)
            C.memmove(uid, obj[0], 128)
        self.comm = C.c_void_p()
        _lib.check(L.tt2_comm_init(C.byref(self.comm), self.world, uid, rank), "tt2_comm_init")
        self.stream = torch.cuda.Stream()
        self.pending = False
        # test hook: snap_hook(lo, hi) runs with the comm stream current right after each
        # bucket's all-reduce is issued (captured with it), e.g. to copy what RCCL produced
        self.snap_hook = None

    def _launch(self, lo, hi, after=None):
        if not (self.comm and self.comm.value):
            raise RuntimeError("RcclGradSync: the communicator was closed")
        cur = torch.cuda.current_stream()
        if after is not None:
            self.stream.wait_event(after)     # the bucket's gradients are final at `after`
        else:
            self.stream.wait_stream(cur)      # the bucket's gradients are final on `cur`
        if self._span is None and not torch.cuda.is_current_stream_capturing():
            # eager step: the exchange's span on the comm stream, from the first bucket's start
            # to finish() (StepMetrics' allreduce_ms; a captured step records no events)
            self._span = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
            self._span[0].record(self.stream)
        L = self._lib.lib()
        base = self.flat.data_ptr() + lo * self.flat.element_size()
        self._lib.check(L.tt2_allreduce_bucket(C.c_void_p(base), hi - lo, self._lib.dt(self.flat), self.comm,
                                               C.c_void_p(self.stream.cuda_stream)), "tt2_allreduce_bucket")
        if self.snap_hook is not None:
            with torch.cuda.stream(self.stream):
                self.snap_hook(lo, hi)
        self.pending = True

    def finish(self):
        while self.next < len(self.buckets):
            self._launch(*self.buckets[self.next])
            self.next += 1
        if self._span is not None and len(self._span) == 2:
            self._span[1].record(self.stream)
            self._done_span, self._span = tuple(self._span), None
        if self.pending:
            cur = torch.cuda.current_stream()
            check_join_target(cur, "RcclGradSync.finish")   # the comm stream joins the capture origin only
            cur.wait_stream(self.stream)
        self.reset()

    def reset(self):
        super().reset()
        self.pending = False
        if not hasattr(self, "_span"):
            self._span, self._done_span = None, None

    def pop_span(self):
        """(start, end) events of the last eager step's all-reduces on the comm stream."""
        s, self._done_span = self._done_span, None
        return s

    def close(self):
        """Destroy the communicator.  A BnSync sharing it (attach(sync_bn=True)) is detached
        from the engine first, so no later step can issue a collective on a freed handle."""
        eng = getattr(self, "engine", None)
        if eng is not None and getattr(eng, "bn_sync", None) is not None and eng.bn_sync.grad_sync is self:
            eng.bn_sync = None
        if eng is not None and getattr(eng, "grad_ready_hook", None) == self.ready:
            eng.grad_ready_hook = None
        if getattr(self, "comm", None) and self.comm.value:
            torch.cuda.synchronize()
            self._lib.check(self._lib.lib().tt2_comm_destroy(self.comm), "tt2_comm_destroy")
            self.comm = C.c_void_p()


class StandinGradSync(RcclGradSync):
    """RcclGradSync's schedule with a stand-in transport: the DP step of an N-rank job rehearsed on
    one GPU (bench.py --dp-standin).  Every bucket is handed to the comm stream exactly as in the
    production N-rank step (from the overlapped backward's side stream, inside the one captured
    graph), but instead of the 1-rank all-reduce the comm stream runs tt2_comm_standin with the
    footprint of this rank's share of an N-rank ring all-reduce: `wgs` work groups (RCCL's
    channels, NCCL_MIN_NCHANNELS), 2 (N-1)/N x bucket bytes of HBM copy traffic (read + write), and
    those CUs held for 2 (N-1)/N x bucket / busbw seconds (the ring's time on the xGMI links).  The
    gradients are not changed (at world 1 the sum is the identity), so the step's numerics are the
    plain ones.  Knobs: TT2_DP_STANDIN_N (8), TT2_DP_STANDIN_GBPS (bus bandwidth, 300),
    TT2_DP_STANDIN_WG (32)."""

    def __init__(self, flat_grads: torch.Tensor, bucket_bytes: int = 25 << 20, group=None, cuts=None):
        super().__init__(flat_grads, bucket_bytes, group, cuts)
        self.ranks = int(os.environ.get("TT2_DP_STANDIN_N", "8"))
        self.busbw = float(os.environ.get("TT2_DP_STANDIN_GBPS", "300")) * 1e9
        self.wgs = int(os.environ.get("TT2_DP_STANDIN_WG", str(RCCL_MIN_CHANNELS)))
        per = max(hi - lo for lo, hi in self.buckets) * flat_grads.element_size()
        self._scratch = torch.empty(per // 4 + 4, dtype=torch.float32, device=flat_grads.device)
        # per bucket, each work group's {start, end} (device wall clock) when recording (tools)
        self.rec = None   # torch.int64 [len(buckets), 2 * wgs] or None

    def params(self) -> dict:
        return {"ranks_modelled": self.ranks, "busbw_GBps": self.busbw / 1e9, "work_groups": self.wgs}

    def _launch(self, lo, hi, after=None):
        if not (self.comm and self.comm.value):
            raise RuntimeError("StandinGradSync: closed")
        if after is not None:
            self.stream.wait_event(after)
        else:
            self.stream.wait_stream(torch.cuda.current_stream())
        esz = self.flat.element_size()
        nbytes = (hi - lo) * esz
        f = 2.0 * (self.ranks - 1) / self.ranks
        src = self.flat.data_ptr() + lo * esz
        pad = (-src) % 16                     # buckets start at any element: copy from the next 16-B boundary
        copy = max(0, int(f / 2 * nbytes) - pad) // 16 * 16   # read + write = f x bucket bytes
        rec = None
        if self.rec is not None:
            bi = next(i for i, (a, b) in enumerate(self.buckets) if a == lo and b == hi)
            rec = C.c_void_p(self.rec[bi].data_ptr())
        self._lib.check(self._lib.lib().tt2_comm_standin(C.c_void_p(src + pad), C.c_void_p(self._scratch.data_ptr()),
                                                         copy, f * nbytes / self.busbw, self.wgs, rec,
                                                         C.c_void_p(self.stream.cuda_stream)), "tt2_comm_standin")
        self.pending = True


class BnSync:
    """SyncBatchNorm exchange (SURVEY.md:219, optional; per-replica statistics stay the
    default).  Each BatchNorm's forward moments and backward column sums leave the kernels as
    [world][3][C] rank slots (this rank's values and its row count, zeros elsewhere: exact and
    rank-ordered once summed, and ranks may hold different row counts), and ``exchange``
    SUM-all-reduces them between the two kernel phases (ops.batchnorm_fwd / _bwd with
    ``sync=``).

    With libtt2's RCCL communicator (``grad_sync``: the RcclGradSync that owns it) the
    all-reduce runs on the SAME comm stream as the gradient buckets, forked from and joined
    back to the compute stream by stream waits: every collective on the communicator is then
    issued from one stream in one program order on every rank (two streams sharing one
    communicator may interleave differently per rank and deadlock), and it is captured with
    the step (``in_graph``).  The exchange runs at world size 1 too (the identity), so a
    one-GPU test executes the captured path itself.  With gloo it is a blocking
    torch.distributed all-reduce, for eager steps only."""
    C_MAX = 2048   # tt2_batchnorm's channel limit

    def __init__(self, world: int, rank: int, group=None, grad_sync=None, device="cuda"):
        self.world, self.rank, self.group, self.grad_sync = world, rank, group, grad_sync
        self.in_graph = grad_sync is not None
        self.snap_hook = None   # test hook: called with the slots after each in-graph exchange
        # one buffer serves every BatchNorm: stats -> exchange -> apply run in stream order
        self._buf = torch.zeros((3 * world + 2) * self.C_MAX + 4, dtype=torch.float32, device=device)

    @property
    def comm(self):
        gs = self.grad_sync
        return gs.comm if gs is not None and gs.comm.value else None

    def buffer(self, nbytes: int) -> torch.Tensor:
        n = (nbytes + 3) // 4
        if n > self._buf.numel():
            raise ValueError(f"BnSync: {nbytes} B exchange buffer requested, {self._buf.numel() * 4} B held")
        return self._buf[:n]

    def exchange(self, slots: torch.Tensor):
        if self.grad_sync is not None:
            comm = self.comm
            if comm is None:
                raise RuntimeError("BnSync: the RCCL communicator was closed (RcclGradSync.close())")
            from . import _lib
            L = _lib.lib()
            cur, cs = torch.cuda.current_stream(), self.grad_sync.stream
            # the exchange joins the comm stream back into `cur`: under capture that must be the
            # capture's origin (raise here rather than segfault in hipStreamEndCapture)
            check_join_target(cur, "BnSync.exchange")
            cs.wait_stream(cur)              # the stats kernel's slots are written on `cur`
            _lib.check(L.tt2_allreduce_bucket(C.c_void_p(slots.data_ptr()), slots.numel(), _lib.dt(slots), comm,
                                              C.c_void_p(cs.cuda_stream)), "tt2_allreduce_bucket")
            if self.snap_hook is not None:
                with torch.cuda.stream(cs):
                    self.snap_hook(slots)
            cur.wait_stream(cs)              # the apply kernel reads the reduced slots
        elif self.world > 1:
            dist.all_reduce(slots, op=dist.ReduceOp.SUM, group=self.group)


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
            # before any communicator exists: RCCL caches its parameters at first use
            os.environ.setdefault("NCCL_MIN_NCHANNELS", str(RCCL_MIN_CHANNELS))
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend,
                                timeout=timedelta(seconds=int(os.environ.get("TT2_DIST_TIMEOUT_S", "600"))))
    return rank, world, local


def sync_kind(group=None) -> str:
    """'rccl' (in-graph, libtt2's communicator) with the nccl backend, else 'segmented'
    (torch.distributed work between graph segments); TT2_DP_SYNC overrides."""
    env = os.environ.get("TT2_DP_SYNC")
    if env in ("rccl", "segmented"):
        return env
    if dist.is_initialized() and dist.get_backend(group) == "nccl":
        return "rccl"
    return "segmented"


def attach(model, group=None, bucket_bytes: int = 25 << 20, kind: str | None = None,
           sync_bn: bool = False, sync_cls=None, bn_cls=None, layer_buckets: bool | None = None) -> GradSync:
    """Wire a TransformerTTS for data parallelism: gradient pre-scaling and the
    bucket hook.  Returns the sync object whose finish() goes between backward and
    the optimizer step (pass it as train_step(..., sync_grads=sync.finish)).
    sync_bn: SyncBatchNorm (the encoder pre-net's and post-net's BatchNorms take their
    training statistics over every rank's rows; BnSync).
    sync_cls / bn_cls: the exchange classes (default RcclGradSync or GradSync by `kind`, and
    BnSync); a subclass may swap the transport, as the issue-order test's recording syncs do.
    layer_buckets: buckets cut where the backward reports layers final (default: TT2_BUCKET_MODE,
    "layers" unless it says "fixed"), else fixed bucket_bytes slices from the end."""
    eng = model.engine
    kind = kind or sync_kind(group)
    cls = sync_cls or (RcclGradSync if kind == "rccl" else GradSync)
    if layer_buckets is None:
        layer_buckets = os.environ.get("TT2_BUCKET_MODE", "layers") != "fixed"
    sync = cls(eng.grads, bucket_bytes, group, cuts=eng.ready_offsets() if layer_buckets else None)
    eng.grad_scale = 1.0 / sync.world
    eng.grad_ready_hook = sync.ready
    sync.engine = eng
    if sync_bn:
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        eng.bn_sync = (bn_cls or BnSync)(sync.world, rank, group, grad_sync=sync if sync.in_graph else None,
                                         device=eng.dev)
    return sync


def compare_issue_logs(logs: list) -> list:
    """Every rank must issue the same collectives on a communicator in the same order (one
    stream per communicator; a rank that issues bucket k+1 before bucket k, or a BatchNorm
    exchange between other buckets, deadlocks an N-rank replay).  logs[r] is rank r's
    sequence of (kind, ...) records; returns [(rank, index, rank-0 record, this rank's
    record)] for every rank whose sequence differs from rank 0's (first difference only;
    None past the end of the shorter sequence)."""
    out = []
    ref = logs[0]
    for r, lg in enumerate(logs[1:], 1):
        n = max(len(ref), len(lg))
        for i in range(n):
            a = tuple(ref[i]) if i < len(ref) else None
            b = tuple(lg[i]) if i < len(lg) else None
            if a != b:
                out.append((r, i, a, b))
                break
    return out


def broadcast_params(model, src: int = 0, group=None):
    """Make every replica start from rank src's weights and BN statistics."""
    eng = model.engine
    dist.broadcast(eng.params, src, group=group)
    dist.broadcast(eng.stats, src, group=group)
    eng.sync_shadow()
