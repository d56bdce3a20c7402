"""Capture hygiene of the captured training step (tt2/capture.py, tt2_capture_joined):
* a stream forked into a capture and not joined back is reported by name (CaptureError)
  before the capture ends, a joined one passes, a stream outside the capture is ignored;
* an exception raised inside the captured region -- the segmented capture and the one-graph
  (in_graph) capture -- ends the capture and re-raises: the process survives, no stream is
  left capturing, and the same model then captures and replays normally."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from tt2.capture import CaptureError, StepCapture, joined_status  # noqa: E402
from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402


def test_join_check():
    x = torch.zeros(1 << 16, device="cuda")
    side, other, origin = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    origin.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    # joined fork: passes, graph replays
    g = torch.cuda.CUDAGraph()
    seen = {}
    with StepCapture(g, origin, lambda: {"side": side, "other": other}):
        x.add_(1)
        side.wait_stream(origin)
        with torch.cuda.stream(side):
            x.mul_(2)
        origin.wait_stream(side)
        seen.update(joined_status(origin, {"side": side, "other": other}))
    assert seen == {"side": 1, "other": 0}
    g.replay()
    torch.cuda.synchronize()
    assert x[0].item() == 2.0
    # unjoined fork: CaptureError naming it, and nothing is left capturing
    g2 = torch.cuda.CUDAGraph()
    with pytest.raises(CaptureError, match="side"):
        with StepCapture(g2, origin, lambda: {"side": side}):
            x.add_(1)
            side.wait_stream(origin)
            with torch.cuda.stream(side):
                x.mul_(3)
    assert not torch.cuda.is_current_stream_capturing()
    torch.cuda.synchronize()
    x.add_(1)     # the device and the streams still work
    torch.cuda.synchronize()
    assert x[0].item() == 3.0


def _batch():
    g = torch.Generator().manual_seed(7)
    B, Tx, Ty = 2, 24, 48
    text = torch.randint(1, 80, (B, Tx), generator=g).cuda()
    tl = torch.tensor([24, 15]).cuda()
    mel = torch.randn(B, Ty, 80, generator=g).cuda()
    ml = torch.tensor([48, 29]).cuda()
    return text, tl, mel, ml


def _model():
    torch.manual_seed(0)
    m = TransformerTTS(TTSConfig(), dtype=torch.bfloat16, seed=3)
    m.configure_optimizer(lr=1e-3, warmup=10.0)
    return m.train()


class _Boom(RuntimeError):
    pass


@pytest.fixture(scope="module")
def gloo1():
    import socket
    import torch.distributed as dist
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        yield
    finally:
        torch.cuda.synchronize()
        dist.destroy_process_group()


@pytest.mark.parametrize("path", ["single", "segmented", "in_graph", "in_graph_hook"])
def test_exception_inside_capture_is_raised_cleanly(gloo1, path):
    from _dp_recording import RecordingSync
    from tt2.dist import GradSync, attach
    b = _batch()
    B, Tx, Ty = b[0].shape[0], b[0].shape[1], b[2].shape[1]
    m, ref = _model(), _model()
    sync = None
    if path == "segmented":
        sync = attach(m, kind="segmented", bucket_bytes=4 << 20)
        assert type(sync) is GradSync
    elif path.startswith("in_graph"):
        sync = attach(m, bucket_bytes=4 << 20, sync_cls=RecordingSync)
        assert sync.in_graph
    fin = sync.finish if sync is not None else None
    for mm in (m, ref):
        mm.train_step(*b, sync_grads=fin if mm is m else None)
    e = m.engine
    real_backward = e.backward

    def exploding_backward(A):
        if torch.cuda.is_current_stream_capturing():
            real_backward(A)   # the side stream is forked and joined inside: raise after it
            raise _Boom("mid-capture failure")
        return real_backward(A)
    real_ready = sync.ready if sync is not None else None
    if path == "in_graph_hook":
        # raise from the second bucket hook: it runs on the side stream in the middle of the
        # overlapped backward, with the side and comm streams forked and not yet joined
        calls = [0]

        def exploding_ready(off):
            calls[0] += 1
            if torch.cuda.is_current_stream_capturing() and calls[0] == 2:
                raise _Boom("hook failure")
            return real_ready(off)
        sync.ready = exploding_ready
    else:
        e.backward = exploding_backward
    with pytest.raises(_Boom):
        m.capture_train_step(B, Tx, Ty, sync_grads=fin)
    assert not torch.cuda.is_current_stream_capturing()
    e.backward = real_backward
    if sync is not None:
        sync.ready = real_ready
    torch.cuda.synchronize()
    # the model recovers: capture again and replay in step with an eager reference
    run = m.capture_train_step(B, Tx, Ty, sync_grads=fin)
    for _ in range(2):
        la = ref.train_step(*b).clone()
        lb = run(*b).clone()
        assert torch.equal(la, lb)
    torch.cuda.synchronize()
    assert torch.equal(ref.engine.params, m.engine.params)
    if sync is not None:
        sync.close()


def test_syncbn_exchange_from_side_stream_is_refused(gloo1):
    """The capture rule as a guard: a SyncBatchNorm exchange issued from the
    encoder's side stream under capture would join the comm stream into that non-origin stream,
    the topology on which hipStreamEndCapture segfaults.  BnSync.exchange (here its recording
    stand-in, which shares the check) raises CaptureError at the call instead; the capture is
    ended cleanly, the process survives, and with the pre-net back on the main stream the same
    model captures and replays in step with its eager twin."""
    from _dp_recording import RecordingBn, RecordingSync
    from tt2.dist import attach
    b = _batch()
    B, Tx, Ty = b[0].shape[0], b[0].shape[1], b[2].shape[1]
    m, ref = _model(), _model()
    syncs = [attach(x, bucket_bytes=4 << 20, sync_bn=True, sync_cls=RecordingSync, bn_cls=RecordingBn)
             for x in (m, ref)]
    e = m.engine
    assert e.enc_overlap and e.bn_sync is not None
    e.syncbn_prenet_on_main = False       # the pre-net's exchanges now come from the side stream
    la = ref.train_step(*b, sync_grads=syncs[1].finish).clone()
    lb = m.train_step(*b, sync_grads=syncs[0].finish).clone()   # eager: no capture, no guard
    assert torch.equal(la, lb)
    assert any(r[0] == "bn" and r[2] == "side" for r in syncs[0].log)
    with pytest.raises(CaptureError, match="BnSync.exchange"):
        m.capture_train_step(B, Tx, Ty, sync_grads=syncs[0].finish)
    assert not torch.cuda.is_current_stream_capturing()
    torch.cuda.synchronize()
    e.syncbn_prenet_on_main = True
    run = m.capture_train_step(B, Tx, Ty, sync_grads=syncs[0].finish)
    for _ in range(2):
        la = ref.train_step(*b, sync_grads=syncs[1].finish).clone()
        lb = run(*b).clone()
        assert torch.equal(la, lb)
    torch.cuda.synchronize()
    assert torch.equal(ref.engine.params, m.engine.params)
    for s in syncs:
        s.close()


def test_check_join_target_outside_capture_is_noop():
    from tt2.capture import active_origin, check_join_target
    assert active_origin() is None
    check_join_target(torch.cuda.Stream(), "test")   # no open capture: nothing to check
