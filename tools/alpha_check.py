"""pos.alpha gradient conditioning at full length (dev tool, GPU): the f32 engine and the f32
oracle, each against a float64 oracle, on test_gpu_fullsize's exact-f32 batch.
    python tools/alpha_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("transformer-tacotron2_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import torch  # noqa: E402

from test_gpu_fullsize import batch, rel  # noqa: E402
from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402
from tt2_oracle import OracleConfig, TransformerTTSOracle, init_deterministic  # noqa: E402


def main():
    torch.set_num_threads(16)
    text, tl, mel, ml = batch(2, (128, 97), (800, 611), seed=1)
    grads = {}
    for name, dt in (("f32", torch.float32), ("f64", torch.float64)):
        o = init_deterministic(TransformerTTSOracle(OracleConfig()), 21).train().to(dt)
        o.set_seed(99)
        m = mel.to(dt)
        ob, oa, os_, _ = o(text, tl, m, ml)
        lo, _ = o.loss((ob, oa, os_), m, ml)
        lo.backward()
        grads[name] = {k: p.grad.detach().clone() for k, p in o.named_parameters() if p.grad is not None}
        sd = o.float().state_dict() if name == "f32" else None
        if sd is not None:
            model = TransformerTTS(TTSConfig(), dtype=torch.float32).train()
            model.load_state_dict(sd)
    model.set_seed(99)
    model(text, tl.int(), mel, ml.int())
    model.loss()
    model.backward()
    gm = model.grads_state_dict()
    rows = []
    for k, g64 in grads["f64"].items():
        rows.append((rel(gm[k], g64), rel(grads["f32"][k], g64), rel(gm[k], grads["f32"][k]), k))
    rows.sort(reverse=True)
    print("engine-vs-f64  oracle32-vs-f64  engine-vs-oracle32  param", flush=True)
    for r in rows[:12]:
        print(f"{r[0]:.3e}  {r[1]:.3e}  {r[2]:.3e}  {r[3]}", flush=True)


if __name__ == "__main__":
    main()
