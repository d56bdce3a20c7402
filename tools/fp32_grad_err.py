"""fp32-mode gradient parity diagnostics (dev tool, GPU): engine and f32 oracle against a
float64 oracle on test_gpu_model's batch, per parameter (worst first).
    python tools/fp32_grad_err.py [seed ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("transformer-tacotron2_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import torch  # noqa: E402

from test_gpu_model import build, make_batch, rel  # noqa: E402


def run(seed, show=8):
    oracle, model = build(torch.float32)
    o64 = build(torch.float32)[0].double()
    text, tl, mel, ml = make_batch()
    for o in (oracle, o64):
        o.train(True)
        o.set_seed(seed)
    model.train(True)
    model.engine.dropout_enabled = True
    model.set_seed(seed)
    for o, m in ((oracle, mel), (o64, mel.double())):
        ob, oa, os_, _ = o(text, tl, m, ml)
        lo, _ = o.loss((ob, oa, os_), m, ml)
        lo.backward()
    model(text, tl.int(), mel, ml.int())
    model.loss()
    model.backward()
    gm = model.grads_state_dict()
    g32 = dict(oracle.named_parameters())
    gnorm = torch.sqrt(sum((p.grad.double() ** 2).sum() for p in o64.parameters() if p.grad is not None))
    rows = []
    for k, p in o64.named_parameters():
        if p.grad is None or p.grad.norm() < 1e-6 * gnorm:
            continue
        rows.append((rel(gm[k], p.grad), rel(g32[k].grad, p.grad), k))
    rows.sort(reverse=True)
    print(f"seed {seed}: engine-vs-f64 | f32 oracle-vs-f64 | param", flush=True)
    for r in rows[:show]:
        print(f"  {r[0]:.2e} {r[1]:.2e} {r[2]}", flush=True)


for s in [int(a) for a in sys.argv[1:]] or [1234]:
    run(s)
