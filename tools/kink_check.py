import os, sys
ROOT = "/root/repo"
for p in ("transformer-tacotron2_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import torch
from test_gpu_model import build, make_batch
from tt2_oracle import dropout_keep
seed = 1234
oracle, model = build(torch.float32)
o64 = oracle.double()
text, tl, mel, ml = make_batch()
o64.train(True); o64.set_seed(seed)
model.train(True); model.engine.dropout_enabled = True; model.set_seed(seed)
pre = {}
for l, layer in enumerate(o64.encoder.layers):
    layer.ffn.w1.register_forward_hook(lambda m, i, o, l=l: pre.__setitem__(l, o.detach()))
o64(text, tl, mel.double(), ml)
model(text, tl.int(), mel, ml.int())
A = list(model.engine.arenas.values())[0]
for l in range(len(o64.encoder.layers)):
    e = A[f"ef1{l}"].float().cpu().reshape(-1)
    x = pre[l].reshape(-1)
    ez = e == 0
    oz = x <= 0
    # engine zero from dropout too: compare only where engine nonzero vs oracle nonpositive, and where engine zero but oracle positive and kept
    flips = ((~ez) & oz)
    near = x.abs().sort().values[:3]
    print(l, "engine nonzero where oracle relu-zero:", int(flips.sum()), "smallest |pre|:", near.tolist(),
          "vals at flips:", x[flips][:5].tolist(), e[flips][:5].tolist())
    i = x.abs().argmin()
    print("   smallest-|pre| element", int(i), "oracle pre", x[i].item(), "engine ef1", e[i].item())
dm = o64.encoder.layers[3].ffn.drop
keep = dropout_keep(seed, dm.site, pre[3].numel(), dm.p)
print("layer 3 element 53258 kept by the dropout mask:", bool(keep[53258]))
