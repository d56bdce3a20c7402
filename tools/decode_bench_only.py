"""cfg3 + cfg5 decode timing alone (dev tool, GPU): bench.py's decode legs on a random-init model."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402

torch.manual_seed(0)
model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16)
eng = model.engine
with torch.no_grad():
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, (off, shape, n) in eng.lay.slots.items():
        if len(shape) >= 2:
            eng.P(name).copy_(torch.randn(shape, generator=g, device="cuda") / (n // shape[0]) ** 0.5)
    eng.sync_shadow()
out = {"decode": bench.decode_bench(model)}
if "--no-longform" not in sys.argv:
    out["longform"] = bench.longform_bench(model)
print(json.dumps(out))
