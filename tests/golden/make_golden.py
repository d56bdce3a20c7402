"""Generate the golden fixtures under tests/golden/ (run in the dev container).

The reference (keonlee9420/Transformer-tacotron2) ships no code or fixtures,
so the oracle's sub-blocks are pinned against third-party implementations
present in this container:

* transformers 5.x SpeechT5 blocks, built from a local SpeechT5Config (no
  download): scaled positional encoding (modeling_speecht5.py:399-422),
  decoder pre-net (:648-697, dropout 0 so it is deterministic), post-net
  conv+BN layer and residual post-net (:700-762), BCE stop loss with
  pos_weight 5 (:1786-1844);
* torch stock nn.MultiheadAttention (same in_proj layout as SURVEY 8(b)).

Each fixture stores the INPUTS, the WEIGHTS actually used and the third-party
OUTPUT, so tests/test_oracle.py can re-run the oracle block on the same data
without transformers.  A final fixture stores end-to-end oracle outputs for
seeded weights (init_deterministic) as a drift guard.

    python tests/golden/make_golden.py            (all fixtures)
    python tests/golden/make_golden.py --drift    (only the oracle-only fixtures 6 and 7)
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from tt2_oracle import (OracleConfig, TransformerTTSOracle, dropout_keep, init_deterministic)  # noqa: E402


def save(name, **arrs):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in arrs.items()})
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def main():
    from transformers import SpeechT5Config
    from transformers.models.speecht5 import modeling_speecht5 as st5

    torch.manual_seed(0)
    # small widths keep the fixtures tiny; the oracle blocks are width-generic
    cfg = SpeechT5Config(hidden_size=64, num_mel_bins=80, speech_decoder_prenet_units=32,
                         speech_decoder_prenet_layers=2, speech_decoder_prenet_dropout=0.0, positional_dropout=0.0,
                         speech_decoder_postnet_layers=5, speech_decoder_postnet_units=48,
                         speech_decoder_postnet_kernel=5, speech_decoder_postnet_dropout=0.0, reduction_factor=1,
                         max_speech_positions=4000)

    # 1. scaled positional encoding
    pe = st5.SpeechT5ScaledPositionalEncoding(0.0, 512, 4000).eval()
    with torch.no_grad():
        pe.alpha.fill_(0.7)
        x = torch.randn(2, 9, 512)
        save("pe", x=x, alpha=pe.alpha.detach(), out=pe(x))

    # 2. decoder prenet (no speaker embedding, dropout 0) + scaled PE
    pre = st5.SpeechT5SpeechDecoderPrenet(cfg).eval()
    # SpeechT5's _consistent_dropout (:677-680) keeps with probability p (so p = 0 zeroes
    # everything); bypass it to pin the deterministic part of the block
    pre._consistent_dropout = lambda x, p: x
    with torch.no_grad():
        pre.encode_positions.alpha.fill_(1.3)
        x = torch.randn(2, 19, 80)
        out = pre(x)
        save("dec_prenet", x=x, fc1_w=pre.layers[0].weight, fc1_b=pre.layers[0].bias, fc2_w=pre.layers[1].weight,
             fc2_b=pre.layers[1].bias, proj_w=pre.final_layer.weight, proj_b=pre.final_layer.bias,
             alpha=pre.encode_positions.alpha, out=out)

    # 3. post-net (conv k5 no bias + BN eval + tanh, residual) and the heads
    post = st5.SpeechT5SpeechDecoderPostnet(cfg).eval()
    with torch.no_grad():
        for layer in post.layers:
            bn = layer.batch_norm
            bn.running_mean.normal_(0, 0.1)
            bn.running_var.uniform_(0.5, 1.5)
            bn.weight.normal_(1, 0.1)
            bn.bias.normal_(0, 0.1)
        h = torch.randn(2, 21, 64)
        before, after, logits = post(h)
        arrs = dict(h=h, feat_w=post.feat_out.weight, feat_b=post.feat_out.bias, prob_w=post.prob_out.weight,
                    prob_b=post.prob_out.bias, before=before, after=after, logits=logits)
        for i, layer in enumerate(post.layers):
            arrs[f"conv{i}_w"] = layer.conv.weight
            arrs[f"bn{i}_g"] = layer.batch_norm.weight
            arrs[f"bn{i}_b"] = layer.batch_norm.bias
            arrs[f"bn{i}_rm"] = layer.batch_norm.running_mean
            arrs[f"bn{i}_rv"] = layer.batch_norm.running_var
        save("postnet", **arrs)

    # 4. stop-token BCE (pos_weight 5) exactly as SpeechT5SpectrogramLoss builds it
    lossmod = st5.SpeechT5SpectrogramLoss(cfg)
    with torch.no_grad():
        B, T = 3, 29
        mel_len = torch.tensor([29, 20, 7])
        labels = torch.randn(B, T, 80)
        for b in range(B):
            labels[b, mel_len[b]:] = -100.0
        logits = torch.randn(B, T) * 3
        padding_mask = labels != -100.0
        masks = padding_mask[:, :, 0]
        stop_labels = torch.cat([~masks * 1.0, torch.ones(masks.size(0), 1)], dim=1)[:, 1:].masked_select(masks)
        bce = lossmod.bce_criterion(logits.masked_select(masks), stop_labels)
        save("stop_bce", logits=logits, mel_len=mel_len, bce=bce)

    # 5. nn.MultiheadAttention with key padding
    mha = torch.nn.MultiheadAttention(64, 4, batch_first=True).eval()
    with torch.no_grad():
        q = torch.randn(2, 13, 64)
        kv = torch.randn(2, 11, 64)
        kl = torch.tensor([11, 6])
        kpm = torch.arange(11)[None, :] >= kl[:, None]
        out, _ = mha(q, kv, kv, key_padding_mask=kpm, need_weights=False)
        save("mha", q=q, kv=kv, key_len=kl, in_w=mha.in_proj_weight, in_b=mha.in_proj_bias,
             out_w=mha.out_proj.weight, out_b=mha.out_proj.bias, out=out)

    drift_fixtures()


def drift_fixtures():
    """Fixtures of the oracle alone (no third-party code): regenerate with --drift after a
    deliberate change of the oracle's dropout hash or initialisation."""
    # 6. dropout hash known answers
    save("dropout_hash", keep_a=dropout_keep(1234, 77, 4096, 0.3), keep_b=dropout_keep(0xFFFFFFFF, 129, 4096, 0.5,
                                                                                      offset=1 << 20))

    # 7. end-to-end oracle drift guard (seeded weights, ragged batch, dropout on)
    model = init_deterministic(TransformerTTSOracle(OracleConfig()), 0)
    g = torch.Generator().manual_seed(0)
    B, Tx, Ty = 2, 17, 23
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl, ml = torch.tensor([17, 11]), torch.tensor([23, 15])
    for b in range(B):
        text[b, tl[b]:] = 0
    mel = torch.randn(B, Ty, 80, generator=g)
    for b in range(B):
        mel[b, ml[b]:] = 0
    model.train()
    model.set_seed(1234)
    before, after, stop, _ = model(text, tl, mel, ml)
    total, parts = model.loss((before, after, stop), mel, ml)
    save("e2e_oracle", text=text, text_len=tl, mel=mel, mel_len=ml, before=before, after=after, stop=stop,
         loss=torch.stack([total, parts["mel_before"], parts["mel_after"], parts["stop"]]))


if __name__ == "__main__":
    drift_fixtures() if "--drift" in sys.argv[1:] else main()
