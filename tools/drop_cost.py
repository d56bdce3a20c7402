"""What the dropout hash costs the training step (dev tool, GPU): the cfg2 step captured with
dropout on and with it off (same kernels, thr = 0 skips the hash), each timed as graph
replays, interleaved; per-kernel times of both under rocprofv3 if wanted.

    python tools/drop_cost.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402


def main():
    torch.manual_seed(0)
    text, tl, mel, ml = bench.synth_batch(0)
    runs = {}
    for on in (True, False):
        model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16)
        model.configure_optimizer(lr=1e-4, warmup=4000.0, clip_norm=1.0)
        model.train()
        model.engine.dropout_enabled = on
        for _ in range(3):
            model.train_step(text, tl, mel, ml)
        runs[on] = model.capture_train_step(text.shape[0], text.shape[1], mel.shape[1])
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    res = {True: [], False: []}
    for _ in range(3):
        for on in (True, False):
            for _ in range(3):
                runs[on](text, tl, mel, ml)
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(20):
                runs[on](text, tl, mel, ml)
            ev[1].record()
            torch.cuda.synchronize()
            res[on].append(ev[0].elapsed_time(ev[1]) / 20)
    print({("dropout on" if k else "dropout off"): [round(v, 3) for v in vs] for k, vs in res.items()})


if __name__ == "__main__":
    main()
