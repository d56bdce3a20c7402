"""AR decode run for kernel-trace profiling (dev tool, GPU): bench's cfg3 decoder (B=32,
128 phonemes), 800 graph-replayed steps (tools/summarize_decode_step.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from tt2.config import TTSConfig  # noqa: E402
from tt2.infer import Decoder  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402

torch.manual_seed(0)
model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16)
model.eval()
g = torch.Generator().manual_seed(1)
text = torch.randint(1, 80, (bench.DEC_B, bench.TX), generator=g).cuda()
tl = torch.full((bench.DEC_B,), bench.TX, dtype=torch.int32, device="cuda")
dec = Decoder(model.engine, bench.DEC_B, bench.TX, bench.DEC_T)
dec.encode(text, tl)
dec.capture(None)
dec.reset()
dec.decode_loop(bench.DEC_T, stop_threshold=None)
torch.cuda.synchronize()
print("ok")
