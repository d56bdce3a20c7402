"""One decode run for the PMC traffic passes (dev tool, GPU), exactly the work bench.py's
decode legs time, with no warm-up run (the counters cover one run):

* default, cfg3: bench's decoder (B=32, 128 phonemes, bf16), encoder + 800 forced decode
  steps + post-net;
* ``--longform``, cfg5: B=64, fp16 decode step, T_max=2000, stop logits injected at bench's
  seeded lengths U[1000, 2000], steps until every utterance has stopped + post-net.

The steps are launched eagerly (tt2_decode_step, the same kernels the captured graph holds):
rocprofv3 --pmc over the libtt2-owned decode graph crashed the profiler (SIGSEGV) here.
The run's step count and algorithmic bytes go to <outdir>/decode_run.json for the summary.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/dtr/fetch -o run --output-format csv -- python3 tools/decode_traffic.py
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/dtr/write -o run --output-format csv -- python3 tools/decode_traffic.py
    python tools/summarize_decode_traffic.py gpurun_out/dtr r04
"""
import json
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

longform = "--longform" in sys.argv
outdir = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--out=")), None)
torch.manual_seed(0)
model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16)
model.eval()
if longform:
    g = torch.Generator().manual_seed(5)         # bench.longform_bench's draws, in its order
    B, T = bench.LF_B, bench.LF_T
    text = torch.randint(1, 80, (B, bench.TX), generator=g).cuda()
    lens = torch.randint(1000, T + 1, (B,), generator=g)
    dec = Decoder(model.engine, B, bench.TX, T, dtype=torch.float16)
    dec.inject_stop(lens)
    thr = 0.5
else:
    g = torch.Generator().manual_seed(1)
    B, T = bench.DEC_B, bench.DEC_T
    text = torch.randint(1, 80, (B, bench.TX), generator=g).cuda()
    dec = Decoder(model.engine, B, bench.TX, T)
    thr = None
tl = torch.full((B,), bench.TX, dtype=torch.int32, device="cuda")
dec.encode(text, tl)
dec.reset()
n = dec.decode_loop(T, use_graph=False, stop_threshold=thr)
mel, out_len = dec.postnet(n, thr)
torch.cuda.synchronize()
if longform and not torch.equal(out_len.cpu(), lens):
    raise SystemExit("long-form: the injected stops did not end the utterances")
algo = bench.longform_algo_bytes(lens, n) if longform else bench.DEC_BYTES
info = {"kind": "longform" if longform else "decode", "steps": n, "algorithmic_bytes_per_run": algo,
        "frames": int(out_len.sum()) if longform else B * T}
if outdir:
    os.makedirs(outdir, exist_ok=True)
    json.dump(info, open(os.path.join(outdir, "decode_run.json"), "w"))
print("decode run ok", tuple(mel.shape), json.dumps(info))
