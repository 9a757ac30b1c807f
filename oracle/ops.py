"""torch-CPU restatement of the float ops on the hot path (oracle, tests only).

Every function works on un-partitioned channels-last token rows so it is directly comparable
with the fused HIP kernels, but internally it follows the reference's explicit data movement
(roll -> partition -> attention -> reverse -> roll back), dimension-generically.
Run it in float64 when checking kernels.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from .index_maps import shifted_window_rows, shift_labels, relative_position_index

LN100 = math.log(1.0 / 0.01)


def window_attention(q, k, v, table, batch, spatial, window, shift, heads, kind=0, scale=None, tau=None,
                     chunk=None):
    """Shifted-window attention on token rows.

    q, k, v: (batch*prod(spatial), C) token rows.  table: (Tsz, heads) additive bias table
    (kind 0: relative_position_bias_table, swinfusion_module.py:89-90,127-130; kind 1: the
    already-activated 16*sigmoid(cpb_mlp(coords)), swin_v2_module.py:158-162).  tau: (heads,)
    logit scale multiplier for kind 1 (swin_v2_module.py:153-156).
    Restates WindowAttention_fusion.forward (swinfusion_module.py:114-145),
    Cross_WindowAttention.forward (:213-246) and WindowAttention.forward (swin_v2_module.py:138-178)
    between their projections, plus the roll/partition/reverse of the blocks.

    Runs on whatever device q lives on.  chunk (windows per chunk, optional): the attention is
    evaluated chunk by chunk under activation checkpointing, so autograd keeps only the inputs and
    recomputes one chunk's N x N logits at a time in backward; windows are independent, so the
    result and every gradient are those of the unchunked computation.  This is what lets the
    float64 oracle run at the full 4 x 96^3 bench geometry (16,384 windows) on the GPU.
    """
    spatial, window, shift = tuple(spatial), tuple(window), tuple(shift)
    dev = q.device
    C = q.shape[1]
    hd = C // heads
    N = int(np.prod(window))
    rows = torch.from_numpy(shifted_window_rows(batch, spatial, window, shift)).to(dev)
    nwin = rows.shape[0]
    if kind == 0 and scale is None:
        scale = hd ** -0.5
    ridx = torch.from_numpy(relative_position_index(window)).reshape(-1).to(dev)
    labels = None
    if any(s > 0 for s in shift):
        labels = torch.from_numpy(shift_labels(spatial, window, shift)).to(dev)
    nW = nwin // batch

    def gather(t):
        return t[rows.reshape(-1)].reshape(nwin, N, heads, hd).permute(0, 2, 1, 3)

    def core(qw, kw, vw, table, tau, w0):
        if kind == 0:
            logits = (qw * scale) @ kw.transpose(-2, -1)
        else:
            logits = F.normalize(qw, dim=-1) @ F.normalize(kw, dim=-1).transpose(-2, -1)
            logits = logits * tau.reshape(1, heads, 1, 1)
        bias = table[ridx].reshape(N, N, heads).permute(2, 0, 1)
        logits = logits + bias.unsqueeze(0)
        if labels is not None:
            lab = labels[torch.arange(w0, w0 + qw.shape[0], device=dev) % nW]      # mask by w mod nW
            mask = (lab[:, None, :] != lab[:, :, None]).to(logits.dtype) * -100.0
            logits = logits + mask.unsqueeze(1)
        p = torch.softmax(logits, dim=-1)
        return (p @ vw).transpose(1, 2).reshape(qw.shape[0] * N, C)

    qw, kw, vw = gather(q), gather(k), gather(v)
    if chunk is None or chunk >= nwin:
        ow = core(qw, kw, vw, table, tau, 0)
    else:
        from torch.utils.checkpoint import checkpoint
        parts = []
        for w0 in range(0, nwin, chunk):
            sl = slice(w0, min(w0 + chunk, nwin))
            parts.append(checkpoint(core, qw[sl], kw[sl], vw[sl], table, tau, w0, use_reentrant=False))
        ow = torch.cat(parts, 0)
    out = torch.zeros_like(q)
    return out.index_copy(0, rows.reshape(-1), ow)


def swin_v2_tau(logit_scale):
    """exp(clamp(logit_scale, max=ln 100)) (swin_v2_module.py:154-155), flattened to (heads,)."""
    return torch.clamp(logit_scale, max=LN100).exp().reshape(-1)


def swin_v2_bias_table(cpb_mlp_params, coords_table, heads):
    """16*sigmoid(cpb_mlp(relative_coords_table)).view(-1, heads) (swin_v2_module.py:158-162).
    cpb_mlp_params = (w0, b0, w2): Linear(k,512) -> ReLU -> Linear(512, heads, no bias)."""
    w0, b0, w2 = cpb_mlp_params
    hdn = F.relu(F.linear(coords_table, w0, b0))
    return 16.0 * torch.sigmoid(F.linear(hdn, w2).reshape(-1, heads))


def causal_diag(Tq, Tk):
    """buffered_future_mask (crossmodal_transformer.py:179-186): -inf where j - i >= 1 + |Tk - Tq|."""
    return 1 + abs(Tk - Tq)


def mha_core(q, k, v, heads, diag=0, scale=None, drop_mask=None):
    """bmm / fp32 softmax / dropout / bmm core of MultiheadAttention.forward
    (multihead_attention.py:92-133) on time-major (T, B, E) tensors.  drop_mask (B, heads, Tq, Tk):
    the multipliers F.dropout applied to the probabilities (:123), None for no dropout.
    Returns (out (Tq,B,E), head-mean (dropped) weights (B,Tq,Tk))."""
    Tq, B, E = q.shape
    Tk = k.shape[0]
    hd = E // heads
    if scale is None:
        scale = hd ** -0.5
    qh = (q * scale).reshape(Tq, B * heads, hd).transpose(0, 1)
    kh = k.reshape(Tk, B * heads, hd).transpose(0, 1)
    vh = v.reshape(Tk, B * heads, hd).transpose(0, 1)
    w = torch.bmm(qh, kh.transpose(1, 2))
    if diag > 0:
        mask = torch.triu(torch.full((Tq, Tk), float("-inf"), dtype=w.dtype, device=w.device), diag)
        w = w + mask.unsqueeze(0)
    w = torch.softmax(w, dim=-1)
    if drop_mask is not None:
        w = w * drop_mask.reshape(B * heads, Tq, Tk).to(w.dtype)
    out = torch.bmm(w, vh).transpose(0, 1).reshape(Tq, B, E)
    mean_w = w.view(B, heads, Tq, Tk).sum(dim=1) / heads
    return out, mean_w


def sinusoidal_table(num, dim, padding_idx=0):
    """SinusoidalPositionalEmbedding.get_embedding (position_embedding.py:44-59)."""
    half = dim // 2
    freq = torch.exp(torch.arange(half, dtype=torch.float32) * -(math.log(10000) / (half - 1)))
    ang = torch.arange(num, dtype=torch.float32).unsqueeze(1) * freq.unsqueeze(0)
    emb = torch.cat([torch.sin(ang), torch.cos(ang)], dim=1).view(num, -1)
    if dim % 2 == 1:
        emb = torch.cat([emb, torch.zeros(num, 1)], dim=1)
    emb[padding_idx, :] = 0
    return emb


def sinusoidal_positions(tokens):
    """Positions for a (B, T) tensor: 1..T where tokens != 0, else 0 (make_positions,
    position_embedding.py:8-27, left_pad=0)."""
    B, T = tokens.shape
    pos = torch.arange(1, T + 1, device=tokens.device).unsqueeze(0).expand(B, T)
    return torch.where(tokens != 0, pos, torch.zeros_like(pos))


# Slope-pattern matching (tests only).  A LeakyReLU pre-activation within rounding of zero takes
# one slope in an fp32 forward and possibly the other in the float64 oracle; its gradient then
# differs by (1 - slope) over the receptive field of everything after it.  A test that wants to
# compare gradients pointwise records which slope the fp32 kernel took at every LeakyReLU (the
# sign of its output) and queues the masks here, in call order: each conv3d_cl with slope != 1
# pops one and applies exactly that slope pattern instead of re-deciding from its own sign.
SLOPE_PATTERNS = None


def conv3d_cl(x, weight, bias=None, stride=1, pad=0, slope=1.0):
    """Channels-last Conv3d + LeakyReLU(slope): the 3D semantics of nn.Conv3d
    (nvidia_blocks.py:43) / the k=s patch-embed conv (swin_v2_module.py:483)."""
    y = F.conv3d(x.permute(0, 4, 1, 2, 3), weight, bias, stride=stride, padding=pad)
    y = y.permute(0, 2, 3, 4, 1)
    if slope != 1.0:
        if SLOPE_PATTERNS:
            pos = SLOPE_PATTERNS.pop(0).to(y.device)
            assert pos.shape == y.shape, (pos.shape, y.shape)
            y = torch.where(pos, y, y * slope)
        else:
            y = F.leaky_relu(y, negative_slope=slope)
    return y.contiguous()
