"""One cfg3 decode run for the PMC traffic passes (dev tool, GPU): bench's decoder (B=32,
128 phonemes, bf16), encoder + 800 forced hipGraph decode steps + post-net, exactly the
work bench.py's decode leg times, with no warm-up run (the counters cover one run).  The
steps are launched eagerly (tt2_decode_step, the same kernels the captured graph holds):
rocprofv3 --pmc over the libtt2-owned decode graph crashed the profiler (SIGSEGV) here.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/dtr/fetch -o run --output-format csv -- python3 tools/decode_traffic.py
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/dtr/write -o run --output-format csv -- python3 tools/decode_traffic.py
    python tools/summarize_decode_traffic.py gpurun_out/dtr r02
"""
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
dec.reset()
dec.decode_loop(bench.DEC_T, use_graph=False, stop_threshold=None)
mel, _ = dec.postnet(bench.DEC_T, None)
torch.cuda.synchronize()
print("decode run ok", tuple(mel.shape))
