"""AR decode path vs the CPU oracle (GPU): forced length, prenet dropout switched off for
parity (it is on by default at inference, as Tacotron2 decodes).
fp32 mode must match within 1e-3; the hipGraph replay must equal eager launches."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2.config import TTSConfig  # noqa: E402
from tt2.infer import SCHEDULE_AUTO, SCHEDULE_PLAIN, SCHEDULE_SPLIT, SCHEDULE_SPLIT_FFN1, Decoder  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402
from tt2 import ops  # noqa: E402
from tt2_oracle import OracleConfig, TransformerTTSOracle, init_deterministic  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def setup(dtype):
    oracle = init_deterministic(TransformerTTSOracle(OracleConfig()), 3).eval()
    model = TransformerTTS(TTSConfig(), dtype=dtype).eval()
    model.load_state_dict(oracle.state_dict())
    g = torch.Generator().manual_seed(5)
    B, Tx = 3, 17
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl = torch.tensor([17, 12, 6])
    for b in range(B):
        text[b, tl[b]:] = 0
    return oracle, model, text, tl


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-3), (torch.bfloat16, 6e-2)])
def test_decode_matches_oracle(dtype, tol):
    oracle, model, text, tl = setup(dtype)
    T = 14
    ref_after, _, ref_before, ref_stop = oracle.infer(text, tl, T, force_len=True)
    after, out_len = model.infer(text, tl, T, stop_threshold=None, prenet_dropout=False)
    assert after.shape == ref_after.shape
    assert rel(after, ref_after) < tol
    dec = model._decoders[(3, 17, T, False)]
    assert rel(dec.mel_seq[:, :T], ref_before) < tol
    assert rel(dec.stop_seq[:, :T], ref_stop) < tol
    assert (out_len.cpu() == T).all()


def test_graph_replay_equals_eager():
    _, model, text, tl = setup(torch.bfloat16)
    T = 10
    a1, _ = model.infer(text, tl, T, stop_threshold=None, use_graph=True, prenet_dropout=False)
    a2, _ = model.infer(text, tl, T, stop_threshold=None, use_graph=False, prenet_dropout=False)
    assert torch.equal(a1, a2)


def test_decode_schedules_match():
    """bf16 decode, libtt2's split-K schedule (KV scatter, PE and emit epilogues, slabs folded
    by tt2_ln_combine) vs the plain one-launch-per-op schedule: same frames within bf16
    rounding of the LayerNorm inputs; both emits advanced the device step counter per frame."""
    _, model, text, tl = setup(torch.bfloat16)
    T = 10
    model.eval()
    ref = Decoder(model.engine, 3, 17, T, schedule=SCHEDULE_PLAIN, prenet_dropout=False)
    out = Decoder(model.engine, 3, 17, T, schedule=SCHEDULE_SPLIT, prenet_dropout=False)
    a, _ = ref.run(text.cuda(), tl.cuda(), T, stop_threshold=None)
    b, _ = out.run(text.cuda(), tl.cuda(), T, stop_threshold=None)
    assert rel(b, a) < 2e-2
    assert out.t.item() == T and ref.t.item() == T


@pytest.mark.parametrize("cd", [torch.bfloat16, torch.float16])
def test_one_launch_ffn_schedule_bitwise(cd):
    """The split schedule with each layer's FFN sublayer in one tt2_ffn_decode launch
    (SCHEDULE_SPLIT_FFN1) decodes the same frames, stop logits, stop positions and device
    counters bit for bit as the default (the FFN as three launches), with prenet dropout and a
    stop threshold, through the captured graph; bf16 and the fp16 step."""
    _, model, text, tl = setup(torch.bfloat16)
    T = 19
    outs = []
    for sched in (SCHEDULE_AUTO, SCHEDULE_SPLIT_FFN1):
        dec = Decoder(model.engine, 3, 17, T, seed=7, dtype=cd, schedule=sched)
        after, out_len = dec.run(text.cuda(), tl.cuda(), T, stop_threshold=0.5)
        torch.cuda.synchronize()
        outs.append((after.clone(), out_len.clone(), dec.mel_seq.clone(), dec.stop_seq.clone(), dec.t.item(),
                     dec.seed.item()))
    (a0, l0, m0, s0, t0, e0), (a1, l1, m1, s1, t1, e1) = outs
    assert torch.equal(m0, m1) and torch.equal(s0, s1)
    assert torch.equal(a0, a1) and torch.equal(l0, l1)
    assert (t0, e0) == (t1, e1)


def test_stop_token_early_exit():
    _, model, text, tl = setup(torch.bfloat16)
    e = model.engine
    with torch.no_grad():   # push the stop logit up so every utterance stops immediately
        e.P("heads.b")[80] = 50.0
        e.sync_shadow()
    after, out_len = model.infer(text, tl, 64, stop_threshold=0.5, prenet_dropout=False)
    assert (out_len.cpu() == 1).all()
    assert after.shape[1] < 64


@pytest.mark.parametrize("m", [1, 5, 32])
def test_skinny_gemm(m):
    g = torch.Generator().manual_seed(m)
    n, k = 200, 520
    A = torch.randn(m, k, generator=g).bfloat16().cuda()
    B = torch.randn(n, k, generator=g).bfloat16().cuda()
    bias = torch.randn(n, generator=g).cuda()
    C = torch.empty(m, n, dtype=torch.float32, device="cuda")
    ops.gemm(A, B, C, m, n, k, k, k, n, bias=bias, act=1, variant=3)
    ref = (A.double() @ B.double().t() + bias.double()).relu()
    assert rel(C, ref) < 1e-5


def test_decode_wide_batch_matches_oracle():
    """A 40-utterance batch takes the 64-row skinny kernels (4 row blocks per MFMA column
    tile): bf16 frames match the fp32 CPU oracle at the bf16 tolerance."""
    oracle = init_deterministic(TransformerTTSOracle(OracleConfig()), 4).eval()
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16).eval()
    model.load_state_dict(oracle.state_dict())
    g = torch.Generator().manual_seed(8)
    B, Tx, T = 40, 11, 6
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl = torch.randint(3, Tx + 1, (B,), generator=g)
    for b in range(B):
        text[b, tl[b]:] = 0
    ref_after, _, ref_before, ref_stop = oracle.infer(text, tl, T, force_len=True)
    after, out_len = model.infer(text, tl, T, stop_threshold=None, prenet_dropout=False)
    assert rel(after, ref_after) < 6e-2
    dec = model._decoders[(B, Tx, T, False)]
    assert rel(dec.mel_seq[:, :T], ref_before) < 6e-2


def test_long_form_limits_early_exit():
    """cfg5 shape (B=64, T_max=2000): per-utterance frame caps end the loop at the last
    cap (polled every 32 frames), out_len = caps, frames stay finite, and the first frames
    equal a short run of the same batch."""
    torch.manual_seed(0)
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16).eval()
    g = torch.Generator().manual_seed(2)
    B, Tx, Tm = 64, 128, 2000
    text = torch.randint(1, 80, (B, Tx), generator=g).cuda()
    tl = torch.full((B,), Tx, dtype=torch.long, device="cuda")
    caps = torch.randint(300, 700, (B,), generator=g)
    dec = Decoder(model.engine, B, Tx, Tm, prenet_dropout=False)
    after, out_len = dec.run(text, tl, Tm, stop_threshold=None, limits=caps)
    n = after.shape[1]
    assert int(caps.max()) <= n < int(caps.max()) + 32
    assert torch.equal(out_len.cpu(), caps)
    assert torch.isfinite(dec.mel_seq[:, :n]).all()
    short = Decoder(model.engine, B, Tx, 8, prenet_dropout=False)
    short.run(text, tl, 8, stop_threshold=None)
    assert rel(short.mel_seq[:, :8], dec.mel_seq[:, :8]) < 1e-6


def test_decode_fp16_matches_oracle():
    """cfg5's fp16 decode step (f16 weights copy, f16 KV cache, f16 cross K/V) on a bf16
    engine: frames match the fp32 oracle within the fp16 tolerance, and the fp16 frames sit
    at least as close to the oracle as the bf16 ones (more mantissa bits)."""
    oracle, model, text, tl = setup(torch.bfloat16)
    T = 12
    ref_after, _, ref_before, ref_stop = oracle.infer(text, tl, T, force_len=True)
    errs = {}
    for dt in (torch.float16, torch.bfloat16):
        dec = Decoder(model.engine, 3, 17, T, dtype=dt, prenet_dropout=False)
        after, out_len = dec.run(text.cuda(), tl.cuda(), T, stop_threshold=None)
        errs[dt] = rel(dec.mel_seq[:, :T], ref_before)
        assert rel(after, ref_after) < 6e-2
        assert (out_len.cpu() == T).all()
    assert errs[torch.float16] < 3e-2
    assert errs[torch.float16] <= errs[torch.bfloat16] * 1.5


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-3), (torch.bfloat16, 6e-2)])
def test_prenet_dropout_decode_matches_oracle(dtype, tol):
    """Tacotron2's always-on pre-net dropout at inference (sites 128 / 129):
    step j draws its masks with seed seed0 + j; the oracle's infer_prenet draws the same
    hash masks, so the frames agree like the dropout-free decode."""
    oracle, model, text, tl = setup(dtype)
    T, seed = 12, 77
    ref_after, _, ref_before, ref_stop = oracle.infer(text, tl, T, force_len=True, prenet_dropout_seed=seed)
    nodrop = oracle.infer(text, tl, T, force_len=True)[2]
    assert rel(nodrop, ref_before) > 1e-2          # the masks change the frames
    dec = Decoder(model.engine, 3, 17, T, prenet_dropout=True, seed=seed)
    after, out_len = dec.run(text.cuda(), tl.cuda(), T, stop_threshold=None)
    assert rel(dec.mel_seq[:, :T], ref_before) < tol
    assert rel(dec.stop_seq[:, :T], ref_stop) < tol
    assert rel(after, ref_after) < tol


@pytest.mark.parametrize("use_graph", [True, False])
def test_injected_stop_matches_oracle(use_graph):
    """Stop-token early exit through injected stop logits (f32 mode): stop_len and out_len
    are the injected lengths, frames up to each stop match the oracle's greedy decode with
    the same stop bias, frames after a stop are zero, and the finished utterances' skipped
    attention leaves the still-running ones unchanged (vs a forced-length run)."""
    oracle, model, text, tl = setup(torch.float32)
    T = 16
    lens = torch.tensor([5, 9, 12])
    dec = Decoder(model.engine, 3, 17, T, prenet_dropout=False)
    dec.inject_stop(lens)
    bias = dec.stop_bias.cpu()
    ref_after, ref_len, ref_before, _ = oracle.infer(text, tl, T, stop_bias=bias)
    assert torch.equal(ref_len, lens)
    after, out_len = dec.run(text.cuda(), tl.cuda(), T, stop_threshold=0.5, use_graph=use_graph)
    assert torch.equal(out_len.cpu(), lens)
    assert torch.equal(dec.stop_len.cpu().long(), lens)
    for b in range(3):
        n = int(lens[b])
        assert rel(dec.mel_seq[b, :n], ref_before[b, :n]) < 1e-3
        if n < after.shape[1]:
            assert float(dec.mel_seq[b, n:after.shape[1]].abs().max()) == 0.0
        # the batched post-net sees this utterance's frames followed by zero frames up to the
        # batch length (as a zero-padded batch in the reference would)
        padded = torch.cat([ref_before[b:b + 1, :n], torch.zeros(1, after.shape[1] - n, 80)], 1)
        assert rel(after[b, :n], oracle.postnet(padded)[0, :n]) < 1e-3
    forced = Decoder(model.engine, 3, 17, T, prenet_dropout=False)
    forced.run(text.cuda(), tl.cuda(), T, stop_threshold=None)
    assert rel(dec.mel_seq[2, :12], forced.mel_seq[2, :12]) < 1e-6


def teacher_forced_errors(oracle, text, tl, frames, lens, rows, n_run):
    """Per-utterance check of decoded frames without an O(T^2) CPU decode: the oracle's
    teacher-forced forward (eval) on the decoded frames must reproduce each frame t from
    frames 0..t-1 (its mel_before[:, t]).  Returns [(rel L2 of the frames, the oracle's
    post-net of the utterance's n_run emitted frames -- zeros after its stop, as the GPU
    batch's post-net sees them)] for the given utterance rows."""
    out = []
    with torch.no_grad():
        for b in rows:
            n = int(lens[b])
            mel = frames[b:b + 1, :n].float().cpu()
            mb, _, _, _ = oracle(text[b:b + 1].cpu(), tl[b:b + 1].cpu(), mel, torch.tensor([n]))
            ma = oracle.postnet(frames[b:b + 1, :n_run].float().cpu())
            out.append((rel(mel, mb), ma))
    return out


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-3), (torch.bfloat16, 5e-2)])
def test_cfg3_full_workload(dtype, tol):
    """SURVEY 8(d) cfg3 at its workload: B = 32, 128 phonemes, 800 forced frames, hipGraph
    step.  Pinned to the oracle by (i) a teacher-forced oracle forward over the decoded
    frames of 4 utterances (every frame t vs the oracle's prediction from frames < t) and
    (ii) the first 16 frames of all 32 utterances vs the oracle's greedy decode."""
    oracle = init_deterministic(TransformerTTSOracle(OracleConfig()), 6).eval()
    model = TransformerTTS(TTSConfig(), dtype=dtype).eval()
    model.load_state_dict(oracle.state_dict())
    g = torch.Generator().manual_seed(1)
    B, Tx, T = 32, 128, 800
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl = torch.full((B,), Tx, dtype=torch.long)
    dec = Decoder(model.engine, B, Tx, T, prenet_dropout=False)
    after, out_len = dec.run(text.cuda(), tl.cuda(), T, stop_threshold=None)
    assert after.shape == (B, T, 80) and (out_len.cpu() == T).all()
    frames = dec.mel_seq.cpu()
    assert torch.isfinite(frames).all()
    errs = teacher_forced_errors(oracle, text, tl, frames, out_len.cpu(), [0, 11, 22, 31], T)
    worst = max(e for e, _ in errs)
    print(f"cfg3 {dtype}: teacher-forced worst rel L2 {worst:.2e}")
    assert worst < tol
    for (e, ma), b in zip(errs, [0, 11, 22, 31]):
        assert rel(after[b], ma[0]) < (1e-3 if dtype == torch.float32 else 2e-2)
    _, _, ref_before, _ = oracle.infer(text, tl, 16, force_len=True)
    assert rel(frames[:, :16], ref_before) < (1e-3 if dtype == torch.float32 else 6e-2)


def test_cfg5_full_workload():
    """SURVEY 8(d) cfg5 at its workload: B = 64, 128 phonemes, T_max = 2000, fp16 decode step,
    stop-token early exit driven by injected stop logits at seeded lengths U[1000, 2000].
    Every utterance stops exactly at its injected length, the loop ends within one poll of the
    longest, and the shortest / longest / a middle utterance match the oracle's teacher-forced
    forward (frames and post-net) at the fp16 tolerance."""
    oracle = init_deterministic(TransformerTTSOracle(OracleConfig()), 7).eval()
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16).eval()
    model.load_state_dict(oracle.state_dict())
    g = torch.Generator().manual_seed(5)
    B, Tx, Tm = 64, 128, 2000
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl = torch.full((B,), Tx, dtype=torch.long)
    lens = torch.randint(1000, Tm + 1, (B,), generator=g)
    dec = Decoder(model.engine, B, Tx, Tm, dtype=torch.float16, prenet_dropout=False)
    dec.inject_stop(lens)
    after, out_len = dec.run(text.cuda(), tl.cuda(), Tm, stop_threshold=0.5)
    n = after.shape[1]
    assert int(lens.max()) <= n < int(lens.max()) + 32
    assert torch.equal(out_len.cpu(), lens)
    frames = dec.mel_seq.cpu()
    assert torch.isfinite(frames[:, :n]).all()
    rows = [int(lens.argmin()), int(lens.argmax()), int(lens.argsort()[B // 2])]
    errs = teacher_forced_errors(oracle, text, tl, frames, lens, rows, n)
    worst = max(e for e, _ in errs)
    print(f"cfg5 fp16: teacher-forced worst rel L2 {worst:.2e} over lengths {[int(lens[b]) for b in rows]}")
    assert worst < 3e-2
    for (e, ma), b in zip(errs, rows):
        k = int(lens[b])
        assert rel(after[b, :k], ma[0, :k]) < 3e-2
        if k < n:
            assert float(frames[b, k:n].abs().max()) == 0.0


def test_replay_past_t_max_leaves_buffers_unchanged():
    """The device step counter saturates at t_max: graph replays beyond it (through the C
    ABI directly, past the host-side clamp) write no KV-cache row -- the next utterance's
    cache rows and the row past the last layer stay as they were -- emit no frame and do
    not advance the counter or the dropout seed."""
    import ctypes as C
    from tt2._lib import check, lib, stream_ptr
    _, model, text, tl = setup(torch.bfloat16)
    T = 6
    for sched in (SCHEDULE_SPLIT, SCHEDULE_PLAIN):
        dec = Decoder(model.engine, 3, 17, T, schedule=sched)
        dec.run(text.cuda(), tl.cuda(), T + 5, stop_threshold=None)    # host clamp: T frames
        assert dec.t.item() == T
        ws0, mel0, stop0, seed0 = dec.ws.clone(), dec.mel_seq.clone(), dec.stop_seq.clone(), dec.seed.clone()
        g = dec.capture(None)
        check(lib().tt2_decode_graph_launch(C.c_void_p(g), 4, C.c_void_p(stream_ptr())), "launch")
        torch.cuda.synchronize()
        assert dec.t.item() == T and torch.equal(dec.seed, seed0)
        assert torch.equal(dec.mel_seq, mel0) and torch.equal(dec.stop_seq, stop0)
        # the KV cache [layer][b][t][K|V] is the workspace's tail: bit-identical (only scratch
        # before it differs); a row-t_max write would land in the next utterance's rows
        c = model.engine.cfg
        cache_bytes = c.n_dec * 3 * T * 2 * c.d_model * 2
        assert cache_bytes % 256 == 0
        assert torch.equal(dec.ws[-cache_bytes:], ws0[-cache_bytes:])


@pytest.mark.parametrize("steps", [4, 8])
def test_multi_step_graph_equals_one_step(steps, monkeypatch):
    """tt2_decode_graph_create_n: `steps` frames per graph launch (the rest by the one-step
    graph) decode the same frames, stop positions and device counters bit for bit as one
    frame per launch, with prenet dropout and a stop threshold (23 frames: not a multiple)."""
    _, model, text, tl = setup(torch.bfloat16)
    T = 23
    outs = []
    for gs in (1, steps):
        monkeypatch.setenv("TT2_DEC_GRAPH_STEPS", str(gs))
        dec = Decoder(model.engine, 3, 17, T, seed=11)
        assert dec.graph_steps == gs
        after, out_len = dec.run(text.cuda(), tl.cuda(), T, stop_threshold=0.5)
        torch.cuda.synchronize()
        outs.append((after.clone(), out_len.clone(), dec.mel_seq.clone(), dec.stop_seq.clone(), dec.t.clone(),
                     dec.seed.clone(), dec.stop_len.clone()))
        dec.close()
    for x, y in zip(*outs):
        assert torch.equal(x, y)
