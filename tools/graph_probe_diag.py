"""Dev check (GPU): bench.graph_probe on the cfg2 step -- per-variant GEMM launch times inside
graph-replayed steps next to the eager-step probe."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from tt2 import ops  # noqa: E402
from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402

torch.manual_seed(0)
model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16)
model.configure_optimizer(lr=1.0, warmup=4000.0, clip_norm=1.0)
model.train()
batch = bench.synth_batch(0)
for _ in range(2):
    model.train_step(*batch)
torch.cuda.synchronize()
g = bench.graph_probe(model, *batch)
ops.PROBE = p = ops.LaunchProbe()
model.train_step(*batch)
e = p.summary()
ops.PROBE = None
for k in sorted(e, key=lambda k: -e[k][2]):
    gk = (g or {}).get(k)
    print(k, f"eager {e[k][2] / e[k][0] * 1e6:.2f} us x {e[k][0]}",
          f"graph {gk[2] / gk[0] * 1e6:.2f} us x {gk[0]:.0f}" if gk else "graph -")
