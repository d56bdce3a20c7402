"""TTSConfig -- model hyper-parameters (SURVEY 8 defaults: d=512, 8 heads,
FFN 2048, 6+6 post-LN layers, 80 mels, 256-wide decoder pre-net, 5-layer
512-channel post-net, k=5 convs; 52.99M parameters)."""
from __future__ import annotations

from dataclasses import asdict, dataclass


@dataclass
class TTSConfig:
    vocab: int = 80
    d_model: int = 512
    n_heads: int = 8
    d_ffn: int = 2048
    n_enc: int = 6
    n_dec: int = 6
    n_mels: int = 80
    enc_conv_layers: int = 3
    enc_conv_kernel: int = 5
    dec_prenet: int = 256
    postnet_channels: int = 512
    postnet_layers: int = 5
    postnet_kernel: int = 5
    dropout: float = 0.1
    prenet_dropout: float = 0.5
    postnet_dropout: float = 0.5
    stop_pos_weight: float = 5.0
    max_len: int = 4096
    bn_momentum: float = 0.1
    bn_eps: float = 1e-5
    ln_eps: float = 1e-5

    def to_dict(self):
        return asdict(self)

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_heads


# dropout site ids (shared spec with oracle/tt2_oracle.py and DESIGN.md)
SITE_ENC_CONV = 1
SITE_ENC_PE = 4
SITE_ENC_LAYER = 16
SITE_DEC_FC1 = 64
SITE_DEC_FC2 = 65
SITE_DEC_PE = 66
SITE_DEC_LAYER = 80
SITE_POSTNET = 112
SITE_INFER_FC1 = 128
SITE_INFER_FC2 = 129
