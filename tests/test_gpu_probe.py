"""libtt2's launch probe (bench.py's live roofline timing, GPU): the eager dispatch events and
the kernel's own wall-clock span both time the probed launch, and under stream capture the
span alone re-times it on every replay of the graph without adding anything to it."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2 import ops  # noqa: E402

M, N, K = 4096, 2048, 512


def _gemm():
    g = torch.Generator(device="cuda").manual_seed(3)
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    B = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    return A, B, C, (lambda: ops.gemm(A, B, C, M, N, K, K, K, N))


def test_probe_eager_events_and_span():
    A, B, C, run = _gemm()
    run()
    torch.cuda.synchronize()
    ops.PROBE = probe = ops.LaunchProbe()
    try:
        run()
        ev = probe.summary()
        sp = probe.summary(span=True)
    finally:
        ops.PROBE = None
        probe.close()
    (key, e), = ev.items()
    s = sp[key]
    assert e[0] == s[0] == 1
    # the span lies inside the dispatch: positive, not longer than the events' interval
    assert 0 < s[2] <= e[2] * 1.05, (s, e)
    ref = A.float() @ B.float().t()
    assert ((C.float() - ref).norm() / ref.norm()).item() < 1e-2   # the probed launch computed


def test_probe_span_under_capture_every_replay():
    A, B, C, run = _gemm()
    run()
    torch.cuda.synchronize()
    probe = ops.LaunchProbe()
    g, s = torch.cuda.CUDAGraph(), torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    ops.PROBE = probe
    try:
        with torch.cuda.graph(g, stream=s, capture_error_mode=ops.CAPTURE_MODE):
            run()
            run()
    finally:
        ops.PROBE = None
    torch.cuda.current_stream().wait_stream(s)
    try:
        spans = []
        for _ in range(3):
            C.zero_()
            g.replay()
            (key, v), = probe.summary(span=True).items()
            assert v[0] == 2 and v[2] > 0
            spans.append(v[2] / 2)
            assert C.abs().sum().item() > 0          # the replay ran the GEMM
        # each read re-armed the record: a replay never reports an accumulated span
        assert max(spans) < 3 * min(spans), spans
        flops = 2.0 * M * N * K
        assert flops / min(spans) < 2.6e15               # not faster than the chip's dense bf16 peak
    finally:
        probe.close()
        del g
