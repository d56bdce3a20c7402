import sys, os, torch
sys.path.insert(0, "tests"); sys.path.insert(0, "transformer-tacotron2_amd"); sys.path.insert(0, "oracle")
from test_gpu_model import build, make_batch
oracle, model = build(torch.bfloat16, seed=3)
text, tl, mel, ml = make_batch(B=2, Tx=17, Ty=40, mel_len=(40, 27))
model.train(); model.engine.dropout_enabled = False
def run(pad):
    model.engine.pad_heads = pad
    model(text, tl.int(), mel, ml.int()); model.loss(); model.backward()
    return {k: v.clone() for k, v in model.grads_state_dict().items()}
a, b, c = run(True), run(True), run(False)
rel = lambda x, y: ((x.double() - y.double()).norm() / y.double().norm()).item()
k = "encoder.embed.weight"
print(os.environ.get("TT2_LIB", "new"), "same-config bitwise:", all(torch.equal(a[n], b[n]) for n in a), "pad vs unpad", k, rel(a[k], c[k]), "dec5 w2", rel(a["decoder.layers.5.ffn.w2.weight"], c["decoder.layers.5.ffn.w2.weight"]))
