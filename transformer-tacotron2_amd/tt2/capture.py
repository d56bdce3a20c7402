"""hipGraph capture of a training step, with the fork/join discipline checked.

A captured step forks work onto other streams (the overlapped backward's side stream, the
RCCL comm stream, the encoder's stream) by stream waits; every such stream must be joined
back into the capture's origin stream before the capture ends.  ``StepCapture`` wraps
``torch.cuda.CUDAGraph.capture_begin`` / ``capture_end``:

* before ending a capture it asks libtt2 (``tt2_capture_joined``: the streams' current capture
  dependencies against the origin's ancestors in the graph being captured) whether every
  registered stream is joined, and raises ``CaptureError`` naming the stream that is not,
  instead of letting ``hipStreamEndCapture`` meet an unjoined fork;
* on any exception inside the captured region it joins every registered stream that takes part
  in the capture, ends the capture and drops the graph, then re-raises: the process survives
  and no stream is left in capture mode (a capture left open made ``~CUDAGraph`` abort the
  process);
* while it is open it is the thread's active capture (``active_origin()``), so code that joins a
  forked stream back (the RCCL comm stream in ``RcclGradSync.finish`` / ``BnSync.exchange``) can
  check, before it issues the join, that the join goes into the capture's origin stream
  (``check_join_target``).  A join into any other stream is the topology on which
  ``hipStreamEndCapture`` (the ROCm 7.0 runtime torch loads) segfaults even though the graph's
  dependencies show every stream joined (``tools/capture_topo.py nested2s``; DESIGN.md section
  6), so it is refused with ``CaptureError`` at the call instead of crashing the process at the
  capture's end.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import threading

import torch

from . import _lib

JOIN_NAMES = {0: "not captured", 1: "joined", 2: "UNJOINED", 3: "invalidated"}
_TRACE = os.environ.get("TT2_CAPTURE_TRACE") == "1"   # dev: print each stage of a capture's end


def _trace(*a):
    if _TRACE:
        print("[capture]", *a, file=sys.stderr, flush=True)


class CaptureError(RuntimeError):
    pass


_active = threading.local()   # the open StepCaptures of this thread (captures are thread-local)


def active_origin():
    """The origin stream of this thread's innermost open StepCapture, or None."""
    st = getattr(_active, "stack", None)
    return st[-1].origin if st else None


def check_join_target(stream: torch.cuda.Stream, what: str):
    """Raise CaptureError if `stream` is capturing inside an open StepCapture and is not that
    capture's origin: joining a forked stream into it would leave a join into a non-origin
    stream in the graph (the hipStreamEndCapture segfault).  Outside a capture: no-op."""
    origin = active_origin()
    if origin is None or stream == origin:
        return
    with torch.cuda.stream(stream):
        capturing = torch.cuda.is_current_stream_capturing()
    if capturing:
        raise CaptureError(f"{what}: joining into stream {stream.cuda_stream:#x}, which is not the capture's "
                           f"origin {origin.cuda_stream:#x}; every forked stream must be joined into the origin "
                           f"(DESIGN.md section 6, capture rule)")


def _push(cap):
    st = getattr(_active, "stack", None)
    if st is None:
        st = _active.stack = []
    st.append(cap)


def _pop(cap):
    st = getattr(_active, "stack", None)
    if st and cap in st:
        st.remove(cap)


def joined_status(origin: torch.cuda.Stream, streams: dict) -> dict:
    """{name: 0 not in the capture / 1 joined / 2 unjoined / 3 invalidated} for each stream,
    relative to the capturing origin stream (tt2_capture_joined)."""
    names = list(streams)
    if not names:
        return {}
    arr = (C.c_void_p * len(names))(*[streams[k].cuda_stream for k in names])
    st = (C.c_int32 * len(names))()
    _lib.check(_lib.lib().tt2_capture_joined(C.c_void_p(origin.cuda_stream), arr, len(names), st),
               "tt2_capture_joined")
    return {k: int(st[i]) for i, k in enumerate(names)}


class StepCapture:
    """``with StepCapture(graph, origin, streams_fn):`` captures the body into `graph` on
    `origin` (made current).  streams_fn() -> {name: stream} lists the streams the body may
    fork into the capture (evaluated at the end, so streams created lazily inside count)."""

    def __init__(self, graph, origin: torch.cuda.Stream, streams_fn=None, capture_error_mode: str = "global"):
        self.graph, self.origin = graph, origin
        self.streams_fn = streams_fn or (lambda: {})
        self.mode = capture_error_mode
        self._ctx = None

    def begin(self):
        self.graph.capture_begin(capture_error_mode=self.mode)
        _push(self)

    def _streams(self) -> dict:
        return {k: s for k, s in self.streams_fn().items() if s is not None and s != self.origin}

    def end(self):
        """End the capture after checking every registered stream is joined."""
        _trace("join check", {k: str(v) for k, v in self._streams().items()})
        st = joined_status(self.origin, self._streams())
        _trace("join status", st)
        bad = {k: JOIN_NAMES[v] for k, v in st.items() if v >= 2}
        if bad:
            self.abort()
            raise CaptureError(f"graph capture: streams not joined into the origin before capture end: {bad}")
        _trace("capture_end")
        with torch.cuda.stream(self.origin):
            self.graph.capture_end()
        _pop(self)
        _trace("capture ended")

    def abort(self):
        """Join whatever takes part in the capture, end it and discard the graph (errors of the
        teardown itself are swallowed: the caller re-raises the original one)."""
        # torch ends a capture only on the stream it began on: make the origin current (the
        # caller may already have left its stream context)
        _pop(self)
        with torch.cuda.stream(self.origin):
            try:
                st = joined_status(self.origin, self._streams())
                for k, s in self._streams().items():
                    if st.get(k) in (1, 2):
                        self.origin.wait_stream(s)
            except Exception:   # noqa: BLE001 - best effort: the capture must still be ended
                pass
            try:
                self.graph.capture_end()
            except Exception:   # noqa: BLE001
                pass
            try:
                self.graph.reset()
            except Exception:   # noqa: BLE001
                pass

    def __enter__(self):
        self._ctx = torch.cuda.stream(self.origin)
        self._ctx.__enter__()
        try:
            self.begin()
        except BaseException:
            self._ctx.__exit__(None, None, None)
            raise
        return self

    def __exit__(self, et, ev, tb):
        try:
            if et is None:
                self.end()
            else:
                self.abort()
        finally:
            self._ctx.__exit__(None, None, None)
        return False
