"""Run-to-run determinism of the training step's pieces (dev tool, GPU): each kernel on fixed
inputs several times, compared bit for bit, and the in-place engine backward twice at the cfg2
shape with every parameter gradient and the encoder input gradient compared.

    python tools/det_check.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from tt2 import ops  # noqa: E402
from tt2._lib import lib  # noqa: E402
from tt2.config import TTSConfig  # noqa: E402
from tt2.engine import act_splits  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402


def same(name, outs):
    bad = [i for i in range(1, len(outs)) if not torch.equal(outs[0], outs[i])]
    print(f"{name:40s} {'deterministic' if not bad else 'DIFFERS in runs ' + str(bad)}", flush=True)


def main():
    torch.manual_seed(0)
    ws = ops.Workspace()
    M, C, K, T = 2048, 512, 5, 128
    dy = (torch.randn(M, C, device="cuda") * 0.1).bfloat16()
    wf = (torch.randn(C, K * C, device="cuda") * 0.02).bfloat16()
    import ctypes as Cc
    g = ops.gemm_args(dy, wf, torch.empty(M, C, device="cuda", dtype=torch.bfloat16), M, C, K * C, C, K * C, C,
                      a_conv=(T, C, 2), splits=act_splits(M, C, K * C), ws=ws)
    print("conv dgrad plan", lib().tt2_gemm_plan(Cc.byref(g)), "splits", act_splits(M, C, K * C), flush=True)
    outs = []
    for _ in range(5):
        out = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
        ops.gemm(dy, wf, out, M, C, K * C, C, K * C, C, a_conv=(T, C, 2), ws=ws, splits=act_splits(M, C, K * C))
        outs.append(out)
    torch.cuda.synchronize()
    same("enc conv dgrad 2048x512x2560 (conv)", outs)
    ids = torch.randint(0, 80, (M,), device="cuda")
    outs = []
    for _ in range(5):
        tab = torch.full((80, C), float("nan"), device="cuda")
        ops.embedding_bwd(ids, dy, tab, M, 80, pad_idx=0)
        outs.append(tab)
    torch.cuda.synchronize()
    same("embedding bwd", outs)
    ref = torch.zeros(80, C, dtype=torch.float64)
    idc, dyc = ids.cpu(), dy.double().cpu()
    for m in range(M):
        if idc[m] != 0:
            ref[idc[m]] += dyc[m]
    print("embedding bwd vs float64 max abs err", (outs[0].double().cpu() - ref).abs().max().item(), flush=True)
    # the engine's in-place backward twice (cfg2, ragged, dropout on)
    gen = torch.Generator().manual_seed(12)
    B, Tx, Ty = 16, 128, 800
    text = torch.randint(1, 80, (B, Tx), generator=gen)
    tl = torch.randint(Tx // 2, Tx + 1, (B,), generator=gen)
    mel = torch.randn(B, Ty, 80, generator=gen)
    ml = torch.randint(Ty // 2, Ty + 1, (B,), generator=gen)
    for i in range(B):
        text[i, tl[i]:] = 0
        mel[i, ml[i]:] = 0
    b = [t.cuda() for t in (text, tl, mel, ml)]
    m = TransformerTTS(TTSConfig(), dtype=torch.bfloat16, seed=5).train()
    with torch.no_grad():
        for name, (off, shape, n) in m.engine.lay.slots.items():
            if len(shape) >= 2:
                m.engine.P(name).normal_(0, 0.02)
        m.engine.sync_shadow()
    e = m.engine
    e.wgrad_overlap, e.enc_overlap = False, 0
    grads, inputs = [], []
    for _ in range(3):
        e.seed.fill_(5)
        A = m._stage(*b)
        e.forward(A)
        e.loss(A)
        e.backward(A)
        torch.cuda.synchronize()
        grads.append(e.grads.clone())
        inputs.append(torch.cat([A["g_xa"].view(-1)[:A.Me * 512], A["g_xb"].view(-1)[:A.Me * 512]]).clone())
    lay = e.lay
    for i in (1, 2):
        d = [n for n in lay.slots if not torch.equal(lay.view(grads[0], n), lay.view(grads[i], n))]
        print(f"engine backward run {i}: differing gradient slots {d[:10]}", flush=True)
    same("engine: encoder input-gradient scratch (g_xa | g_xb)", inputs)
    # the overlapped schedules on the same (warm) model, against the in-place run 0
    for ov, enc in ((True, 0), (True, 0), (True, 1), (True, 1), (False, 0)):
        e.wgrad_overlap, e.enc_overlap = ov, enc
        e.seed.fill_(5)
        A = m._stage(*b)
        e.forward(A)
        e.loss(A)
        e.backward(A)
        torch.cuda.synchronize()
        d = [(n, float((lay.view(grads[0], n) - lay.view(e.grads, n)).abs().max())) for n in lay.slots
             if not torch.equal(lay.view(grads[0], n), lay.view(e.grads, n))]
        print(f"overlap={ov} enc_overlap={enc}: {len(d)} differing slots {d[:12]}", flush=True)


if __name__ == "__main__":
    main()
