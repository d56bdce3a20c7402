"""Recording stand-ins for the RCCL exchange (test infrastructure, imported by GPU tests).

``RecordingSync`` is an ``RcclGradSync`` (in-graph semantics: the captured one-graph step,
bucket hooks from the overlapped backward's side stream, the comm stream forked and joined
by stream waits) that never touches a communicator.  Each bucket hand-off and each
SyncBatchNorm exchange (``RecordingBn``) is appended to ``log`` as it is ISSUED on the host --
(kind, offsets / size, role of the issuing stream) -- which is the order the comm stream (one
per communicator) would receive the collectives in.  Outside a capture, with world > 1, the
comm stream then really exchanges the bytes: it waits for the issuing stream, the buffer goes
to the host, a gloo all-reduce sums it and it comes back on the comm stream, so an eager step
has the production schedule's numerics.  Inside a capture (gloo cannot be captured) the comm
stream gets one tiny kernel instead, so the captured graph has the same fork/join topology.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.distributed as dist

from tt2.capture import check_join_target
from tt2.dist import BnSync, GradSync, RcclGradSync


def _role_of(sync, stream) -> str:
    eng = getattr(sync, "engine", None)
    if eng is not None and eng._side is not None and stream == eng._side:
        return "side"
    if stream == sync.stream:
        return "comm"
    return "main"


def _exchange(buf: torch.Tensor, issuing: torch.cuda.Stream, comm: torch.cuda.Stream, tick: torch.Tensor,
              group, world: int, after=None):
    if after is not None:
        comm.wait_event(after)
    else:
        comm.wait_stream(issuing)
    with torch.cuda.stream(comm):
        if torch.cuda.is_current_stream_capturing() or world == 1:
            tick.add_(1)
        else:
            comm.synchronize()
            host = buf.detach().cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            buf.copy_(host.to(buf.device))


class RecordingSync(RcclGradSync):
    in_graph = True

    def __init__(self, flat_grads: torch.Tensor, bucket_bytes: int = 25 << 20, group=None, cuts=None):
        GradSync.__init__(self, flat_grads, bucket_bytes, group, cuts)
        self.comm = C.c_void_p(1)      # truthy, never handed to RCCL
        self.stream = torch.cuda.Stream()
        self.pending = False
        self.snap_hook = None
        self.log = []
        self._tick = torch.zeros(1, device=flat_grads.device)
        self.hold = None               # negative control: a bucket index whose hand-off is held back

    def _launch(self, lo, hi, after=None):
        cur = torch.cuda.current_stream()
        self.log.append(("bucket", lo, hi, _role_of(self, cur)))
        _exchange(self.flat[lo:hi], cur, self.stream, self._tick, self.group, self.world, after)
        self.pending = True

    def ready(self, offset: int, after=None):
        idx = self.take_ready(offset)
        if self.hold is not None:
            held = [i for i in idx if i == self.hold]
            idx = [i for i in idx if i != self.hold]
            if held:
                self._held = held
            elif getattr(self, "_held", None) and idx:
                idx = idx + self._held      # the held bucket goes after the next one
                self._held = None
        for i in idx:
            self._launch(*self.buckets[i], after=after)

    def finish(self):
        if getattr(self, "_held", None):
            for i in self._held:
                self._launch(*self.buckets[i])
            self._held = None
        super().finish()

    def close(self):
        eng = getattr(self, "engine", None)
        if eng is not None and getattr(eng, "bn_sync", None) is not None and eng.bn_sync.grad_sync is self:
            eng.bn_sync = None
        if eng is not None and getattr(eng, "grad_ready_hook", None) == self.ready:
            eng.grad_ready_hook = None
        self.comm = C.c_void_p()


class RecordingBn(BnSync):
    def exchange(self, slots: torch.Tensor):
        gs = self.grad_sync
        cur = torch.cuda.current_stream()
        check_join_target(cur, "BnSync.exchange")   # as the RCCL exchange: joins into the origin only
        gs.log.append(("bn", slots.numel(), _role_of(gs, cur)))
        _exchange(slots, cur, gs.stream, gs._tick, self.group, self.world)
        if self.snap_hook is not None:
            with torch.cuda.stream(gs.stream):
                self.snap_hook(slots)
        cur.wait_stream(gs.stream)
