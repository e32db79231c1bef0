"""torch.nn layer classes whose forward runs on libldm_amd.

Each subclasses the torch layer it stands in for, so parameter names, shapes, default init (and the
RNG draws it makes), state_dict keys and repr are exactly the reference's; only forward differs.
Fused multi-layer paths (conv+BN+ReLU, the whole UNet) live in models/model.py and ldm_amd.engine.
"""
import torch
import torch.nn as tnn

from . import functional as F
from . import ops


class Conv2d(tnn.Conv2d):
    def _check(self):
        if self.groups != 1 or tuple(self.dilation) != (1, 1) or self.padding_mode != "zeros" or \
                isinstance(self.padding, str) or self.padding[0] != self.padding[1] or self.stride[0] != self.stride[1]:
            raise NotImplementedError("ldm_amd.Conv2d: only groups=1, dilation=1, symmetric zero padding/stride")

    def forward(self, x, act="none", bcast=None, skip=None):
        self._check()
        return F.conv(x, self.weight, self.bias, stride=self.stride[0], padding=self.padding[0], act=act,
                      bcast=bcast, skip=skip)


class ConvTranspose2d(tnn.ConvTranspose2d):
    def forward(self, x, output_size=None, act="none", skip=None):
        if output_size is not None or self.groups != 1 or tuple(self.dilation) != (1, 1):
            raise NotImplementedError("ldm_amd.ConvTranspose2d: output_size/groups/dilation unsupported")
        return F.conv(x, self.weight, self.bias, stride=self.stride[0], padding=self.padding[0], transposed=True,
                      output_padding=self.output_padding[0], act=act, skip=skip)


class BatchNorm2d(tnn.BatchNorm2d):
    def forward(self, x, act="none"):
        return F.batchnorm(x, self, act)


class ReLU(tnn.ReLU):
    def forward(self, x):
        return F.activation(x, "relu")


class Tanh(tnn.Tanh):
    def forward(self, x):
        return F.activation(x, "tanh")


class GELU(tnn.GELU):
    def forward(self, x):
        if self.approximate != "none":
            raise NotImplementedError("ldm_amd.GELU: only the exact (erf) form")
        return F.activation(x, "gelu")


class Linear(tnn.Linear):
    def forward(self, x):
        return F.linear(x, self.weight, self.bias)


class MultiheadAttention(tnn.MultiheadAttention):
    """Sequence-first nn.MultiheadAttention (query [L,B,E], key/value [S,B,E]); no masks, no dropout.

    Returns (attn_output, None): the reference discards the averaged weights (model.py:153)."""

    def forward(self, query, key, value, key_padding_mask=None, need_weights=True, attn_mask=None,
                average_attn_weights=True, is_causal=False):
        if key_padding_mask is not None or attn_mask is not None or self.batch_first or \
                not self._qkv_same_embed_dim or self.bias_k is not None or (self.training and self.dropout > 0):
            raise NotImplementedError("ldm_amd.MultiheadAttention: masks / batch_first / kdim / dropout unsupported")
        if key is not value:
            raise NotImplementedError("ldm_amd.MultiheadAttention: key and value must be the same tensor "
                                      "(cross-attention on one style map, model.py:153)")
        # [L,B,E] -> channel-major [B,E,L] (layout copy), then the NCHW path of the UNet
        qc = query.permute(1, 2, 0).contiguous()
        kc = key.permute(1, 2, 0).contiguous()
        out = attention_nchw(self, qc.unsqueeze(2), kc.unsqueeze(2))
        return out.squeeze(2).permute(2, 0, 1), None


def attention_nchw(mha, q_nchw, kv_nchw):
    """CrossAttention on NCHW maps without the reference's permutes (model.py:140-160):
    Q = 1x1conv(q; W_q), KV = 1x1conv(kv; W_kv), per-head softmax attention, out = 1x1conv(.; W_o)."""
    B, E, h, w = q_nchw.shape
    ipw, ipb = mha.in_proj_weight, mha.in_proj_bias
    q, kv = F.in_proj(q_nchw, kv_nchw, ipw, ipb)
    a = F.attention_core(q.view(B, E, h * w), kv.view(B, 2 * E, -1), mha.num_heads)
    ow = mha.out_proj.weight
    out = F.conv(a.view(B, E, h, w), ow.view(E, E, 1, 1), mha.out_proj.bias, stride=1, padding=0, wkey=(ow, "o"))
    return out


__all__ = ["Conv2d", "ConvTranspose2d", "BatchNorm2d", "ReLU", "Tanh", "GELU", "Linear", "MultiheadAttention",
           "attention_nchw", "ops"]
