"""fairseq-style multi-head attention — MI355X build.

Drop-in for the reference's modules/multihead_attention.py (same constructor, forward
signature, return tuple and parameter names).  The in/out projections stay GEMMs; the
bmm -> mask -> fp32 softmax -> bmm core (multihead_attention.py:109-130) is one flash-style
HIP kernel (libmmni.so mmni_mha_fwd/bwd) reading the time-major (T, B, E) projections in place.
The head-averaged weights (second return value) are produced by a separate kernel only when
asked for (need_weights=True, the reference's behaviour); TransformerEncoderLayer discards
them, so the encoder never materialises a T x T tensor.  Attention dropout (the reference's
F.dropout of the probabilities, multihead_attention.py:123; default --attn_dropout 0.1,
main.py:176) runs inside the kernels from a counter-based mask: one seed per call, drawn from
torch's default generator, regenerated in the backward.  The weights are differentiable with
respect to q and k (their backward rebuilds the per-head probabilities on the device; no caller of
the reference back-propagates through them, so that path is not optimised).
"""
import torch
from torch import nn
from torch.nn import Parameter
import torch.nn.functional as F

from ..functional import (SplitKLinear, dropout_seed, in_proj_q_kv, mha_core, mha_mean_probs, mha_packed,
                          splitk_linear)


def causal_diag_of(attn_mask, Tq, Tk):
    """Translate an attn_mask into the kernel's causal diagonal.  Masks produced by
    crossmodal_transformer.buffered_future_mask carry their diagonal; any other mask is not
    representable by the fused kernel."""
    if attn_mask is None:
        return 0
    diag = getattr(attn_mask, "_mmni_causal_diag", None)
    if diag is None:
        raise NotImplementedError("MultiheadAttention: only the causal mask of buffered_future_mask is supported "
                                  "by the fused kernel")
    if tuple(attn_mask.shape) != (Tq, Tk):
        raise ValueError(f"attn_mask shape {tuple(attn_mask.shape)} != ({Tq}, {Tk})")
    return diag


class MultiheadAttention(nn.Module):
    """Multi-headed attention (multihead_attention.py:9-157)."""

    def __init__(self, embed_dim, num_heads_mult, attn_dropout=0., bias=True, add_bias_kv=False,
                 add_zero_attn=False):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads_mult = num_heads_mult
        self.attn_dropout = attn_dropout
        self.head_dim = embed_dim // num_heads_mult
        assert self.head_dim * num_heads_mult == self.embed_dim, "embed_dim must be divisible by num_heads_mult"
        self.scaling = self.head_dim ** -0.5
        self.in_proj_weight = Parameter(torch.Tensor(3 * embed_dim, embed_dim))
        self.register_parameter('in_proj_bias', None)
        if bias:
            self.in_proj_bias = Parameter(torch.Tensor(3 * embed_dim))
        self.out_proj = SplitKLinear(embed_dim, embed_dim, bias=bias)
        if add_bias_kv:
            self.bias_k = Parameter(torch.Tensor(1, 1, embed_dim))
            self.bias_v = Parameter(torch.Tensor(1, 1, embed_dim))
        else:
            self.bias_k = self.bias_v = None
        self.add_zero_attn = add_zero_attn
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.xavier_uniform_(self.out_proj.weight)
        if self.in_proj_bias is not None:
            nn.init.constant_(self.in_proj_bias, 0.)
            nn.init.constant_(self.out_proj.bias, 0.)
        if self.bias_k is not None:
            nn.init.xavier_normal_(self.bias_k)
        if self.bias_v is not None:
            nn.init.xavier_normal_(self.bias_v)

    def forward(self, query, key, value, attn_mask=None, need_weights=True):
        """query (Tq, B, E), key/value (Tk, B, E) -> (attn (Tq, B, E), head-mean weights (B, Tq, Tk) or None)."""
        if self.bias_k is not None or self.add_zero_attn:
            raise NotImplementedError("add_bias_kv / add_zero_attn are not used by the reference callers and are "
                                      "not implemented by the fused kernel")
        tgt_len, bsz, embed_dim = query.size()
        assert embed_dim == self.embed_dim
        assert key.size() == value.size()
        src_len = key.size(0)
        diag = causal_diag_of(attn_mask, tgt_len, src_len)
        p = float(self.attn_dropout) if self.training else 0.0
        if not need_weights and query.is_cuda and key.data_ptr() == value.data_ptr():
            # packed projections straight into the attention core: self attention on one qkv GEMM,
            # cross attention on q + one kv GEMM of the packed weight (one autograd node, row-block
            # weight gradients); k / v stay column slices and their gradients arrive packed
            seed = dropout_seed() if p > 0 else 0
            if query.data_ptr() == key.data_ptr():
                attn = mha_packed(self._in_proj(query), None, self.num_heads_mult, diag, self.scaling, p, seed)
            else:
                q, kv = in_proj_q_kv(query, key, self.in_proj_weight, self.in_proj_bias)
                attn = mha_packed(q, kv, self.num_heads_mult, diag, self.scaling, p, seed)
            return self.out_proj(attn), None
        if query.data_ptr() == key.data_ptr() == value.data_ptr():
            q, k, v = self._in_proj(query).chunk(3, dim=-1)
        elif key.data_ptr() == value.data_ptr():
            q = self._in_proj(query, end=self.embed_dim)
            k, v = self._in_proj(key, start=self.embed_dim).chunk(2, dim=-1)
        else:
            q = self._in_proj(query, end=self.embed_dim)
            k = self._in_proj(key, start=self.embed_dim, end=2 * self.embed_dim)
            v = self._in_proj(value, start=2 * self.embed_dim)
        seed = dropout_seed() if p > 0 else 0
        attn, lse = mha_core(q, k, v, self.num_heads_mult, diag, self.scaling, dropout=p, seed=seed)
        attn = self.out_proj(attn)
        weights = None
        if need_weights:
            weights = mha_mean_probs(q, k, lse, self.num_heads_mult, diag, self.scaling, dropout=p, seed=seed)
        return attn, weights

    def in_proj_qkv(self, query):
        return self._in_proj(query).chunk(3, dim=-1)

    def in_proj_kv(self, key):
        return self._in_proj(key, start=self.embed_dim).chunk(2, dim=-1)

    def in_proj_q(self, query, **kwargs):
        return self._in_proj(query, end=self.embed_dim, **kwargs)

    def in_proj_k(self, key):
        return self._in_proj(key, start=self.embed_dim, end=2 * self.embed_dim)

    def in_proj_v(self, value):
        return self._in_proj(value, start=2 * self.embed_dim)

    def _in_proj(self, input, start=0, end=None, **kwargs):
        weight = kwargs.get('weight', self.in_proj_weight)
        bias = kwargs.get('bias', self.in_proj_bias)
        if start != 0 or end is not None:   # whole-weight projections stay unsliced (no slice gradient)
            weight = weight[start:end, :]
            if bias is not None:
                bias = bias[start:end]
        return splitk_linear(input, weight, bias)
