"""CPU: pin the oracle against the golden fixtures (SpeechT5 blocks, torch
nn.MultiheadAttention, dropout-hash known answers) and check the spec counts."""
import os

import numpy as np
import pytest
import torch

from tt2_oracle import (MHA, OracleConfig, Postnet, ScaledPositionalEncoding, DecoderPrenet, TransformerTTSOracle,
                        count_params, dropout_keep, init_deterministic, tts_loss)

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with np.load(os.path.join(GOLD, name + ".npz")) as z:
        return {k: torch.from_numpy(z[k]) for k in z.files}


def close(a, b, tol=1e-5):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item() < tol


def test_param_count_and_keys():
    m = TransformerTTSOracle(OracleConfig())
    assert count_params(m) == 52986691   # 52.99M
    keys = list(m.state_dict().keys())
    assert "decoder.layers.5.cross_attn.in_proj_weight" in keys
    assert "postnet.convs.4.bn.running_var" in keys
    assert m.state_dict()["postnet.convs.0.conv.weight"].shape == (512, 80, 5)


def test_pe_matches_speecht5():
    z = load("pe")
    pe = ScaledPositionalEncoding(512, 4000)
    with torch.no_grad():
        pe.alpha.copy_(z["alpha"])
    assert close(pe(z["x"]), z["out"], 1e-6)


def test_decoder_prenet_matches_speecht5():
    z = load("dec_prenet")
    c = OracleConfig(d_model=64, dec_prenet=32, prenet_dropout=0.0)
    pre = DecoderPrenet(c)
    pos = ScaledPositionalEncoding(64, 4000)
    with torch.no_grad():
        for n in ("fc1", "fc2", "proj"):
            getattr(pre, n).weight.copy_(z[n + "_w"])
            getattr(pre, n).bias.copy_(z[n + "_b"])
        pos.alpha.copy_(z["alpha"])
    assert close(pos(pre(z["x"])), z["out"], 1e-5)


def test_postnet_and_heads_match_speecht5():
    z = load("postnet")
    c = OracleConfig(d_model=64, postnet_channels=48)
    post = Postnet(c).eval()
    with torch.no_grad():
        for i, cb in enumerate(post.convs):
            cb.conv.weight.copy_(z[f"conv{i}_w"])
            cb.conv.bias.zero_()              # SpeechT5 convs have no bias
            cb.bn.weight.copy_(z[f"bn{i}_g"])
            cb.bn.bias.copy_(z[f"bn{i}_b"])
            cb.bn.running_mean.copy_(z[f"bn{i}_rm"])
            cb.bn.running_var.copy_(z[f"bn{i}_rv"])
        before = torch.nn.functional.linear(z["h"], z["feat_w"], z["feat_b"])
        logits = torch.nn.functional.linear(z["h"], z["prob_w"], z["prob_b"]).squeeze(-1)
        after = post(before)
    assert close(before, z["before"], 1e-6)
    assert close(logits, z["logits"], 1e-6)
    assert close(after, z["after"], 1e-5)


def test_stop_bce_matches_speecht5():
    z = load("stop_bce")
    B, T = z["logits"].shape
    mel = torch.zeros(B, T, 80)
    _, parts = tts_loss(torch.zeros(B, T, 80), torch.zeros(B, T, 80), z["logits"], mel, z["mel_len"], 5.0)
    assert abs(parts["stop"].item() - z["bce"].item()) < 1e-6 * max(1.0, abs(z["bce"].item()))


def test_mha_matches_torch():
    z = load("mha")
    m = MHA(64, 4)
    with torch.no_grad():
        m.in_proj_weight.copy_(z["in_w"])
        m.in_proj_bias.copy_(z["in_b"])
        m.out_proj.weight.copy_(z["out_w"])
        m.out_proj.bias.copy_(z["out_b"])
        out, _ = m(z["q"], z["kv"], key_len=z["key_len"])
    assert close(out, z["out"], 1e-5)


def test_dropout_hash_known_answers():
    z = load("dropout_hash")
    assert np.array_equal(dropout_keep(1234, 77, 4096, 0.3), z["keep_a"].numpy())
    assert np.array_equal(dropout_keep(0xFFFFFFFF, 129, 4096, 0.5, offset=1 << 20), z["keep_b"].numpy())
    k = dropout_keep(7, 3, 200000, 0.25)
    assert abs(k.mean() - 0.75) < 0.005


def test_fully_masked_row_is_zero():
    m = MHA(64, 4)
    q = torch.randn(2, 5, 64)
    out, p = m(q, q, key_len=torch.tensor([5, 0]))
    assert torch.isfinite(out).all()
    assert p[1].abs().sum() == 0


def test_e2e_oracle_drift_guard():
    z = load("e2e_oracle")
    model = init_deterministic(TransformerTTSOracle(OracleConfig()), 0)
    model.train()
    model.set_seed(1234)
    b, a, s, _ = model(z["text"], z["text_len"], z["mel"], z["mel_len"])
    assert close(b, z["before"], 1e-5)
    assert close(a, z["after"], 1e-5)
    assert close(s, z["stop"], 1e-5)


@pytest.mark.parametrize("causal", [False, True])
def test_mha_causal_mask(causal):
    torch.manual_seed(0)
    m = MHA(64, 4)
    x = torch.randn(1, 6, 64)
    out1, _ = m(x, x, causal=causal)
    x2 = x.clone()
    x2[:, -1] += 1.0
    out2, _ = m(x2, x2, causal=causal)
    same = torch.allclose(out1[:, :-1], out2[:, :-1], atol=1e-6)
    assert same == causal
