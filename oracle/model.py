"""Functional torch-CPU restatement of the models on the path (oracle, tests + cpu_baseline only).

Every function takes a flat parameter dict `p` keyed exactly like the reference's state_dict
(and the build's), so the same recipe-filled weights drive the reference, the oracle and the
HIP product.  Dimension-generic: token grids are 2D (H, W) or 3D (D, H, W).

  swin_v2_logits      SwinTransformerV2.forward  (model.py:1100-1120)
  swinfusion_logits   SwinFusion.forward         (model.py:1396-1538)
  crossmodal_head     Transformer_Net_Cross_Attention.forward (model.py:489-537), feature_map_size 'same'
  swin_crossmodal_logits  the build-defined C4 composite from the pieces above
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import ops as O
from .index_maps import relative_coords_table


def _ln(p, pre, x):
    return F.layer_norm(x, (x.shape[-1],), p[pre + ".weight"], p[pre + ".bias"], 1e-5)


def _lin(p, pre, x):
    return F.linear(x, p[pre + ".weight"], p.get(pre + ".bias"))


def _mlp(p, pre, x):
    return _lin(p, pre + ".fc2", F.gelu(_lin(p, pre + ".fc1", x)))


def _window_for(res, ws, block_idx):
    """Per-block (window, shift) with the reference's clamp (swin_v2_module.py:226-229)."""
    shift = 0 if block_idx % 2 == 0 else ws // 2
    if min(res) <= ws:
        return min(res), 0
    return ws, shift


def _grid(res, ws, shift):
    nd = len(res)
    return tuple(res), (ws,) * nd, (shift,) * nd


# ------------------------------------------------------------------------------------------
# SwinFusion blocks (pre-norm, table bias)
# ------------------------------------------------------------------------------------------
def fusion_block(p, pre, x, x_size, heads, ws, shift):
    B, L, C = x.shape
    sp, win, sh = _grid(x_size, ws, shift)
    h = _ln(p, pre + ".norm1", x).reshape(-1, C)
    q, k, v = _lin(p, pre + ".attn.qkv", h).split(C, dim=-1)
    o = O.window_attention(q, k, v, p[pre + ".attn.relative_position_bias_table"], B, sp, win, sh, heads, 0,
                           chunk=ATTN_CHUNK)
    x = x + _lin(p, pre + ".attn.proj", o).view(B, L, C)
    return x + _mlp(p, pre + ".mlp", _ln(p, pre + ".norm2", x))


def cross_block(p, pre, x, y, x_size, heads, ws, shift):
    B, L, C = x.shape
    sp, win, sh = _grid(x_size, ws, shift)
    xn = _ln(p, pre + ".norm1_A", x).reshape(-1, C)
    yn = _ln(p, pre + ".norm1_B", y).reshape(-1, C)

    def attend(att, a, b):
        q = _lin(p, att + ".q", a)
        k, v = _lin(p, att + ".kv", b).split(C, dim=-1)
        o = O.window_attention(q, k, v, p[att + ".relative_position_bias_table"], B, sp, win, sh, heads, 0,
                               chunk=ATTN_CHUNK)
        return _lin(p, att + ".proj", o).view(B, L, C)

    xa = attend(pre + ".attn_A", xn, yn)
    yb = attend(pre + ".attn_B", yn, xn)
    x = x + xa
    x = x + _mlp(p, pre + ".mlp_A", _ln(p, pre + ".norm2_A", x))
    y = y + yb
    y = y + _mlp(p, pre + ".mlp_B", _ln(p, pre + ".norm2_B", y))
    return x, y


def fusion_layer(p, pre, x, x_size, depth, heads, ws, res):
    for i in range(depth):
        w, s = _window_for(res, ws, i)
        x = fusion_block(p, f"{pre}.blocks.{i}", x, x_size, heads, w, s)
    return x


def cross_layer(p, pre, x, y, x_size, depth, heads, ws, res):
    for i in range(depth):
        w, s = _window_for(res, ws, i)
        x, y = cross_block(p, f"{pre}.blocks.{i}", x, y, x_size, heads, w, s)
    return x, y


# ------------------------------------------------------------------------------------------
# Swin-V2 (res-post-norm, cosine attention)
# ------------------------------------------------------------------------------------------
def v2_block(p, pre, x, res, heads, ws, shift):
    B, L, C = x.shape
    sp, win, sh = _grid(res, ws, shift)
    a = pre + ".attn"
    bias = torch.cat((p[a + ".q_bias"], torch.zeros_like(p[a + ".v_bias"]), p[a + ".v_bias"]))
    q, k, v = F.linear(x.reshape(-1, C), p[a + ".qkv.weight"], bias).split(C, dim=-1)
    coords = torch.from_numpy(relative_coords_table(win)).to(x.device, x.dtype)
    table = O.swin_v2_bias_table((p[a + ".cpb_mlp.0.weight"], p[a + ".cpb_mlp.0.bias"], p[a + ".cpb_mlp.2.weight"]),
                                 coords, heads)
    o = O.window_attention(q, k, v, table, B, sp, win, sh, heads, 1, tau=O.swin_v2_tau(p[a + ".logit_scale"]),
                           chunk=ATTN_CHUNK)
    o = _lin(p, a + ".proj", o).view(B, L, C)
    x = x + _ln(p, pre + ".norm1", o)
    return x + _ln(p, pre + ".norm2", _mlp(p, pre + ".mlp", x))


def patch_merge(x, res):
    """2^k neighbour concat in the build's order (2D: the reference's (0,0),(1,0),(0,1),(1,1))."""
    B, L, C = x.shape
    g = x.view(B, *res, C)
    parts = []
    if len(res) == 2:
        for dx in (0, 1):
            for dy in (0, 1):
                parts.append(g[:, dy::2, dx::2])
    else:
        for dx in (0, 1):
            for dy in (0, 1):
                for dz in (0, 1):
                    parts.append(g[:, dz::2, dy::2, dx::2])
    return torch.cat(parts, -1).view(B, -1, len(parts) * C)


def swin_v2_logits(p, pre, img, patch, ws, depths=(2, 2, 6), heads=(3, 6, 12)):
    """img (B, *spatial) -> logits (B, 1)."""
    nd = img.dim() - 1
    B = img.shape[0]
    x_cl = img.unsqueeze(-1)
    w = p[pre + "patch_embed.proj.weight"]
    if nd == 2:
        x_cl = x_cl.unsqueeze(1)
        w = w.unsqueeze(2)
        st = (1, patch, patch)
    else:
        st = (patch,) * 3
    t = O.conv3d_cl(x_cl, w, p[pre + "patch_embed.proj.bias"], st, 0)
    res = tuple(t.shape[1:-1]) if nd == 3 else tuple(t.shape[2:-1])
    x = _ln(p, pre + "patch_embed.norm", t.reshape(B, -1, t.shape[-1]))
    for li, (d, h) in enumerate(zip(depths, heads)):
        for i in range(d):
            wsz, s = _window_for(res, ws, i)
            x = v2_block(p, f"{pre}layers.{li}.blocks.{i}", x, res, h, wsz, s)
        if li < len(depths) - 1:
            x = patch_merge(x, res)
            dpre = f"{pre}layers.{li}.downsample"
            x = _ln(p, dpre + ".norm", F.linear(x, p[dpre + ".reduction.weight"]))
            res = tuple(r // 2 for r in res)
    x = _ln(p, pre + "norm", x).mean(dim=1)
    return _lin(p, pre + "head", x)


# ------------------------------------------------------------------------------------------
# SwinFusion
# ------------------------------------------------------------------------------------------
def _conv(p, name, x_cl, slope):
    w = p[name + ".weight"]
    if w.dim() == 4:
        return O.conv3d_cl(x_cl.unsqueeze(1), w.unsqueeze(2), p[name + ".bias"], 1, (0, 1, 1), slope).squeeze(1)
    return O.conv3d_cl(x_cl, w, p[name + ".bias"], 1, 1, slope)


def swinfusion_logits(p, A, Bv, cfg):
    """cfg: dict(window_size, patch_size, Ex_depths, Fusion_depths, Re_depths, heads (int),
    resolution (patches resolution tuple), head_patch)."""
    return swin_v2_logits(p, "swin.", swinfusion_trunk(p, A, Bv, cfg), cfg["head_patch"], cfg["window_size"])


def swinfusion_trunk(p, A, Bv, cfg):
    """Ex / Fusion / Re trunk of SwinFusion (model.py:1396-1482): pair -> fused map (B, *spatial)."""
    ws = cfg["window_size"]
    res = tuple(cfg["resolution"])
    heads = cfg.get("heads", 6)

    def embed(x_cl):
        B, C = x_cl.shape[0], x_cl.shape[-1]
        return _ln(p, "patch_embed.norm", x_cl.reshape(B, -1, C))

    def unembed(t, x_size):
        return t.reshape(t.shape[0], *x_size, t.shape[-1])

    def extract(x_cl, tag):
        x = _conv(p, "conv_first1_A", x_cl, 0.2)
        x = _conv(p, "conv_first2_A", x, 0.2)
        x_size = tuple(x.shape[1:-1])
        t = embed(x)
        for li, d in enumerate(cfg["Ex_depths"]):
            t = fusion_layer(p, f"layers_Ex_{tag}.{li}.residual_group", t, x_size, d, heads, ws, res) + t
        return unembed(_ln(p, f"norm_Ex_{tag}", t), x_size)

    x = extract(A.unsqueeze(-1), "A")
    y = extract(Bv.unsqueeze(-1), "B")
    x_size = tuple(x.shape[1:-1])
    tx, ty = embed(x), embed(y)
    for li, d in enumerate(cfg["Fusion_depths"]):
        pre = f"layers_Fusion.{li}"
        tx = fusion_layer(p, pre + ".residual_group_A", tx, x_size, d, heads, ws, res) + tx
        ty = fusion_layer(p, pre + ".residual_group_B", ty, x_size, d, heads, ws, res) + ty
        cx, cy = cross_layer(p, pre + ".residual_group", tx, ty, x_size, d, heads, ws, res)
        tx, ty = cx + tx, cy + ty
    xf = unembed(_ln(p, "norm_Fusion_A", tx), x_size)
    yf = unembed(_ln(p, "norm_Fusion_B", ty), x_size)
    z = _conv(p, "conv_after_body_Fusion", torch.cat([xf, yf], -1), 0.2)
    t = embed(z)
    for li, d in enumerate(cfg["Re_depths"]):
        t = fusion_layer(p, f"layers_Re.{li}.residual_group", t, x_size, d, heads, ws, res) + t
    z = unembed(_ln(p, "norm_Re", t), x_size)
    z = _conv(p, "conv_last1", z, 0.2)
    z = _conv(p, "conv_last2", z, 0.2)
    return _conv(p, "conv_last3", z, 1.0)[..., 0]


# ------------------------------------------------------------------------------------------
# crossmodal transformer (crossmodal_transformer.py, multihead_attention.py) and the C4 composite
# ------------------------------------------------------------------------------------------
def mha(p, pre, q_in, k_in, v_in, heads, diag):
    """MultiheadAttention.forward without weights (multihead_attention.py:51-134): in_proj rows
    [0,E) / [E,2E) / [2E,3E) for q / k / v, scaled-dot core, out_proj."""
    E = q_in.shape[-1]
    W, b = p[pre + "in_proj_weight"], p[pre + "in_proj_bias"]
    q = F.linear(q_in, W[:E], b[:E])
    k = F.linear(k_in, W[E:2 * E], b[E:2 * E])
    v = F.linear(v_in, W[2 * E:], b[2 * E:])
    out, _ = O.mha_core(q, k, v, heads, diag)
    return F.linear(out, p[pre + "out_proj.weight"], p[pre + "out_proj.bias"])


def _embed_tokens(x_in):
    """sqrt(E) x + sinusoidal positions of x_in[..., 0] != 0 (crossmodal_transformer.py:72-77,
    position_embedding.py:30-79); x_in (T, B, E)."""
    T, B, E = x_in.shape
    pos = O.sinusoidal_positions(x_in.transpose(0, 1)[:, :, 0])          # (B, T)
    table = O.sinusoidal_table(T + 1, E).to(x_in.device, x_in.dtype)
    return math.sqrt(E) * x_in + table[pos].transpose(0, 1)


def encoder(p, pre, x_in, xk_in=None, xv_in=None, layers=12, heads=12, attn_mask=True):
    """TransformerEncoder.forward (crossmodal_transformer.py:49-90, 133-165): pre-norm layers,
    the same layer_norms.0 on query / key / value, causal mask diag 1 + |Tk - Tq|, final LN."""
    x = _embed_tokens(x_in)
    cross = xk_in is not None
    if cross:
        xk, xv = _embed_tokens(xk_in), _embed_tokens(xv_in)
    for i in range(layers):
        lp = f"{pre}layers.{i}."
        ln0 = lambda t: _ln(p, lp + "layer_norms.0", t)  # noqa: E731
        Tq = x.shape[0]
        Tk = xk.shape[0] if cross else Tq
        diag = O.causal_diag(Tq, Tk) if attn_mask else 0
        xn = ln0(x)
        a = mha(p, lp + "self_attn.", xn, ln0(xk) if cross else xn, ln0(xv) if cross else xn, heads, diag)
        x = x + a
        h = F.relu(_lin(p, lp + "fc1", _ln(p, lp + "layer_norms.1", x)))
        x = x + _lin(p, lp + "fc2", h)
    return _ln(p, pre + "layer_norm", x)


def crossmodal_head(p, pre, x_l, x_u, layers, heads, feature_map_gen="no", attn_mask=True):
    """Transformer_Net_Cross_Attention.forward (model.py:489-537), feature_map_size 'same',
    mixing 'U2L_and_L2U', concat: x_l, x_u (B, T, F) -> (out_cls (B, F), logits (B, 1))."""
    if feature_map_gen == "convolution_ul+l":
        w = p[pre + "proj_l.weight"][:, :, 0]                           # Conv1d(T, T, 1) over the time axis
        pl = torch.einsum("st,btf->bsf", w, x_l)
        pu = torch.einsum("st,btf->bsf", w, x_u)
    else:
        pl, pu = x_l, x_u
    pl, pu = pl.permute(1, 0, 2), pu.permute(1, 0, 2)                   # (T, B, F)
    h_l = encoder(p, pre + "trans_l_with_u.", pl, pu, pu, layers, heads, attn_mask)
    h_u = encoder(p, pre + "trans_u_with_l.", pu, pl, pl, layers, heads, attn_mask)
    # trans_mem is built with layers=3 -> max(nlevels, 3) (model.py:446-470)
    h = encoder(p, pre + "trans_mem.", torch.cat([h_l, h_u], dim=2), None, None, max(layers, 3), heads, attn_mask)
    out_cls = _lin(p, pre + "out_layer1", h[-1])
    return out_cls, _lin(p, pre + "out_layer2", out_cls)


def swin_crossmodal_logits(p, A, Bv, cfg, return_embedding=False):
    """SwinCrossmodal3D (SURVEY §8d C4 composite): per modality Conv3d(k=s=patch) + LN + Swin-V2
    stage 1, Cross_BasicLayer, Linear to d, crossmodal head.  cfg: patch, window_size, swin_heads,
    cross_heads, depth, layers, heads [, patch_B: modality B's patch (C5), default patch].
    return_embedding: also return the head's out_cls ('embedding_per_ROIs', model.py:512-537)."""
    ws = cfg["window_size"]
    patches = {"A": cfg["patch"], "B": cfg.get("patch_B", cfg["patch"])}

    def stage(img, tag):
        B = img.shape[0]
        P = patches[tag]
        t = O.conv3d_cl(img.unsqueeze(-1), p[f"patch_embed_{tag}.proj.weight"], p[f"patch_embed_{tag}.proj.bias"],
                        (P,) * 3, 0)
        res = tuple(t.shape[1:-1])
        x = _ln(p, f"patch_embed_{tag}.norm", t.reshape(B, -1, t.shape[-1]))
        for i in range(cfg["depth"]):
            wsz, s = _window_for(res, ws, i)
            x = v2_block(p, f"swin_{tag}.blocks.{i}", x, res, cfg["swin_heads"], wsz, s)
        return x, res

    x, res = stage(A, "A")
    y, _ = stage(Bv, "B")
    x, y = cross_layer(p, "cross", x, y, res, cfg["depth"], cfg["cross_heads"], ws, res)
    out_cls, logits = crossmodal_head(p, "crossmodal.", _lin(p, "to_seq_A", x), _lin(p, "to_seq_B", y),
                                      cfg["layers"], cfg["heads"])
    return (logits, out_cls) if return_embedding else logits


def params_of(module, dtype=torch.float64, device=None):
    """Detached parameter dict (leaf tensors, requires_grad) keyed like the state_dict."""
    return {k: v.detach().to(device=device, dtype=dtype).clone().requires_grad_(True)
            for k, v in module.named_parameters()}


# windows per checkpointed chunk of every window-attention call in the functions above (None:
# unchunked).  Tests that run the float64 oracle at full volume sizes on the GPU set it.
ATTN_CHUNK = None
