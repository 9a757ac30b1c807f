"""Crossmodal transformer encoder (MulT-style) — MI355X build of modules/crossmodal_transformer.py.

Same classes, signatures and parameter names.  Each layer's attention core is the fused HIP
flash kernel (see multihead_attention.py); the causal mask is passed as a diagonal, never
materialised on the device (buffered_future_mask returns a tiny host tensor tagged with it).
"""
import math

import torch
from torch import nn
import torch.nn.functional as F

from .position_embedding import SinusoidalPositionalEmbedding
from .multihead_attention import MultiheadAttention
from ..functional import (SplitKLinear, cast_params_bf16, dropout_seed, encoder_layer_rows, layer_norm,
                          splitk_linear)


class TransformerEncoder(nn.Module):
    """sqrt(E)-scaled input + sinusoidal positions + N pre-norm layers + final LN
    (crossmodal_transformer.py:9-96)."""

    def __init__(self, embed_dim, num_heads_mult, layers, attn_dropout=0.0, relu_dropout=0.0, res_dropout=0.0,
                 embed_dropout=0.0, attn_mask=False):
        super().__init__()
        self.dropout = embed_dropout
        self.attn_dropout = attn_dropout
        self.embed_dim = embed_dim
        self.embed_scale = math.sqrt(embed_dim)
        self.embed_positions = SinusoidalPositionalEmbedding(embed_dim)
        self.attn_mask = attn_mask
        self.layers = nn.ModuleList([
            TransformerEncoderLayer(embed_dim, num_heads_mult=num_heads_mult, attn_dropout=attn_dropout,
                                    relu_dropout=relu_dropout, res_dropout=res_dropout, attn_mask=attn_mask)
            for _ in range(layers)])
        self.register_buffer('version', torch.Tensor([2]))
        self.normalize = True
        if self.normalize:
            self.layer_norm = LayerNorm(embed_dim)

    def _embed(self, x_in):
        x = self.embed_scale * x_in
        if self.embed_positions is not None:
            x = x + self.embed_positions(x_in.transpose(0, 1)[:, :, 0]).transpose(0, 1)
        return F.dropout(x, p=self.dropout, training=self.training)

    def _gemm_params(self):
        for layer in self.layers:
            a = layer.self_attn
            yield from (a.in_proj_weight, a.in_proj_bias, a.out_proj.weight, a.out_proj.bias, layer.fc1.weight,
                        layer.fc1.bias, layer.fc2.weight, layer.fc2.bias)

    def forward(self, x_in, x_in_k=None, x_in_v=None):
        """x_in (T, B, E) [, x_in_k, x_in_v (Tk, B, E)] -> (T, B, E)."""
        if x_in.is_cuda and torch.is_autocast_enabled() and torch.get_autocast_dtype("cuda") == torch.bfloat16:
            # this step's bf16 copies of every layer's GEMM weights and biases in a few launches
            cast_params_bf16(list(self._gemm_params()))
        x = self._embed(x_in)
        cross = x_in_k is not None and x_in_v is not None
        if cross:
            x_k = self._embed(x_in_k)
            # the callers pass one tensor as key and value input (model.py:489-490); its two
            # embeddings are then equal unless dropout draws two masks, so compute it once and
            # let the layers project key and value from one LayerNorm (identical values)
            same = x_in_v is x_in_k and (self.dropout == 0.0 or not self.training)
            x_v = x_k if same else self._embed(x_in_v)
        for layer in self.layers:
            x = layer(x, x_k, x_v) if cross else layer(x)
        if self.normalize:
            x = layer_norm(x, self.layer_norm) if x.is_cuda else self.layer_norm(x)
        return x

    def max_positions(self):
        return self.embed_positions.max_positions()


class TransformerEncoderLayer(nn.Module):
    """Pre-norm layer: LN -> (cross) MHA -> residual; LN -> fc1/ReLU/fc2 -> residual
    (crossmodal_transformer.py:99-172).  The same layer_norms[0] normalises query, key and value
    (quirk kept: crossmodal_transformer.py:145,150-151)."""

    def __init__(self, embed_dim, num_heads_mult=4, attn_dropout=0.1, relu_dropout=0.1, res_dropout=0.1,
                 attn_mask=False):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads_mult = num_heads_mult
        self.self_attn = MultiheadAttention(embed_dim=self.embed_dim, num_heads_mult=self.num_heads_mult,
                                            attn_dropout=attn_dropout)
        self.attn_mask = attn_mask
        self.relu_dropout = relu_dropout
        self.res_dropout = res_dropout
        self.normalize_before = True
        self.fc1 = Linear(self.embed_dim, 4 * self.embed_dim)
        self.fc2 = Linear(4 * self.embed_dim, self.embed_dim)
        self.layer_norms = nn.ModuleList([LayerNorm(self.embed_dim) for _ in range(2)])

    def _fused_ok(self, x, x_k, x_v):
        inactive = lambda p: p == 0.0 or not self.training  # noqa: E731
        return (x.is_cuda and x.dtype == torch.float32 and not torch.is_autocast_enabled()
                and self.normalize_before and inactive(self.relu_dropout) and inactive(self.res_dropout)
                and (x_k is None and x_v is None or x_k is x_v) and self.embed_dim <= 256
                and self.embed_dim % self.num_heads_mult == 0 and self.embed_dim // self.num_heads_mult <= 16
                and self.self_attn.in_proj_bias is not None and self.self_attn.bias_k is None
                and not self.self_attn.add_zero_attn)

    def forward(self, x, x_k=None, x_v=None):
        if self._fused_ok(x, x_k, x_v):
            # HIP row-GEMM path (functional.encoder_layer_rows): LN0 + in_proj, attention core,
            # out_proj + residual, LN1 + fc1 + ReLU, fc2 + residual in 6 launches
            diag = (buffered_future_mask(x, x_k)._mmni_causal_diag if self.attn_mask else 0)
            p = float(self.self_attn.attn_dropout) if self.training else 0.0
            return encoder_layer_rows(x, x_k, self, diag, p, dropout_seed() if p > 0 else 0)
        residual = x
        x = self.maybe_layer_norm(0, x, before=True)
        mask = buffered_future_mask(x, x_k) if self.attn_mask else None
        if x_k is None and x_v is None:
            x, _ = self.self_attn(query=x, key=x, value=x, attn_mask=mask, need_weights=False)
        else:
            # one LayerNorm when key and value are one tensor (the encoder's shared embedding): the
            # two normalised copies are equal, and one tensor lets the attention project k and v in
            # one GEMM and keep them packed
            same = x_k is x_v
            x_k = self.maybe_layer_norm(0, x_k, before=True)
            x_v = x_k if same else self.maybe_layer_norm(0, x_v, before=True)
            x, _ = self.self_attn(query=x, key=x_k, value=x_v, attn_mask=mask, need_weights=False)
        x = F.dropout(x, p=self.res_dropout, training=self.training)
        x = residual + x
        x = self.maybe_layer_norm(0, x, after=True)
        residual = x
        x = self.maybe_layer_norm(1, x, before=True)
        if x.is_cuda:   # ReLU in the fc1 GEMM's epilogue
            x = splitk_linear(x, self.fc1.weight, self.fc1.bias, relu=True)
        else:
            x = F.relu(self.fc1(x))
        x = F.dropout(x, p=self.relu_dropout, training=self.training)
        x = self.fc2(x)
        x = F.dropout(x, p=self.res_dropout, training=self.training)
        x = residual + x
        return self.maybe_layer_norm(1, x, after=True)

    def maybe_layer_norm(self, i, x, before=False, after=False):
        assert before ^ after
        if not (after ^ self.normalize_before):
            return x
        if not x.is_cuda:
            return self.layer_norms[i](x)
        # a pre-norm feeds only the layer's Linears: under autocast its output is stored in the
        # GEMMs' dtype (no separate cast pass; same rounding as the autocast Linear's)
        out = torch.get_autocast_dtype("cuda") if (before and torch.is_autocast_enabled()) else None
        return layer_norm(x, self.layer_norms[i], out)


def fill_with_neg_inf(t):
    """FP16-compatible function that fills a tensor with -inf."""
    return t.float().fill_(float('-inf')).type_as(t)


def buffered_future_mask(tensor, tensor2=None):
    """Causal mask -inf where j - i >= 1 + |Tk - Tq| (crossmodal_transformer.py:179-186).

    Returns a small host tensor (the reference's value, for callers that inspect it) tagged with
    `_mmni_causal_diag`; the fused attention kernel applies the mask analytically from that
    diagonal, so nothing of size T x T is copied to or built on the device."""
    dim1 = dim2 = tensor.size(0)
    if tensor2 is not None:
        dim2 = tensor2.size(0)
    diag = 1 + abs(dim2 - dim1)
    mask = _CausalMask.get(dim1, dim2, diag)
    return mask


class _CausalMask:
    _cache = {}

    @classmethod
    def get(cls, dim1, dim2, diag):
        key = (dim1, dim2)
        m = cls._cache.get(key)
        if m is None:
            m = torch.triu(fill_with_neg_inf(torch.ones(dim1, dim2)), diag)[:dim1, :dim2]
            m._mmni_causal_diag = diag
            cls._cache[key] = m
        return m


def Linear(in_features, out_features, bias=True):
    """nn.Linear (crossmodal_transformer.py:189-194) whose weight gradient is split over the token
    rows (functional.SplitKLinear; same parameters and state_dict keys)."""
    m = SplitKLinear(in_features, out_features, bias)
    nn.init.xavier_uniform_(m.weight)
    if bias:
        nn.init.constant_(m.bias, 0.)
    return m


def LayerNorm(embedding_dim):
    return nn.LayerNorm(embedding_dim)
