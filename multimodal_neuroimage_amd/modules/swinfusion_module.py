"""SwinFusion (SwinIR-derived) window / cross-window attention stack — MI355X build.

Drop-in for the reference's modules/swinfusion_module.py: same class names, constructor and
forward signatures and state_dict keys.  Inside, the shifted-window attention of
every block is ONE HIP launch (libmmni.so: mmni_wattn_fwd/bwd) that reads the qkv projection
straight from the un-partitioned channels-last token tensor: the roll, window_partition, mask
rebuild + H2D copy, bias gather, softmax, AV, window_reverse and reverse roll of the reference
(swinfusion_module.py:350-373, 114-145) collapse into it.  At C = 12 norm1 is fused into the
qkv / q / kv projections (blockops.hip) and norm2 + fc1 + GELU + fc2 + residual is one kernel
per direction (mlp.hip).  Every block also accepts 3D token grids (x_size = (D, H, W)), the
build's 3D lift; 2D inputs are the D = 1 special case.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.utils.checkpoint as checkpoint

from ..functional import (window_attention_self, window_attention_cross, conv3d_cl, layer_norm, linear, mlp, ln_linear,
                          ln_linear_ok, ln_mlp)
from ._common import (DropPath, inactive, to_2tuple, to_ntuple, trunc_normal_, relative_index_buffer, shift_mask_buffer,
                      attend_masked_windows, clamp_window, geometry, patch_merge_gather)


class Mlp_fusion(nn.Module):
    """fc1 -> act -> drop -> fc2 -> drop (swinfusion_module.py:14-30)."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.):
        super().__init__()
        hidden_features = hidden_features or in_features
        out_features = out_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)

    def forward(self, x, residual=None):
        return mlp(x, self.fc1, self.fc2, self.act, self.drop, residual)


def window_partition_fusion(x, window_size):
    """(B, *spatial, C) -> (num_windows*B, *window, C) (swinfusion_module.py:33-45; any rank)."""
    B, *spatial, C = x.shape
    win = to_ntuple(window_size, len(spatial))
    split = [B]
    for L, w in zip(spatial, win):
        split += [L // w, w]
    nd = len(spatial)
    perm = [0] + [1 + 2 * a for a in range(nd)] + [2 + 2 * a for a in range(nd)] + [1 + 2 * nd]
    return x.reshape(*split, C).permute(perm).reshape(-1, *win, C)


def window_reverse_fusion(windows, window_size, *spatial):
    """Inverse of window_partition_fusion (swinfusion_module.py:48-62); spatial = (H, W) or (D, H, W)."""
    nd = len(spatial)
    win = to_ntuple(window_size, nd)
    C = windows.shape[-1]
    nW = math.prod(L // w for L, w in zip(spatial, win))
    B = windows.shape[0] // nW
    split = [B] + [L // w for L, w in zip(spatial, win)] + list(win) + [C]
    perm = [0]
    for a in range(nd):
        perm += [1 + a, 1 + nd + a]
    perm += [1 + 2 * nd]
    return windows.reshape(split).permute(perm).reshape(B, *spatial, C)


def _no_attn_dropout(mod):
    if mod.training and mod.attn_drop.p > 0:
        raise NotImplementedError("mmni window attention: attention-probability dropout > 0 in training is not "
                                  "implemented by the fused kernel (reference default is 0)")


class WindowAttention_fusion(nn.Module):
    """Windowed multi-head self attention with a learned relative-position bias table
    (swinfusion_module.py:65-161).  window_size: 2- or 3-tuple."""

    def __init__(self, dim, window_size, num_heads, qkv_bias=True, qk_scale=None, attn_drop=0., proj_drop=0.):
        super().__init__()
        self.dim = dim
        self.window_size = tuple(window_size)
        self.num_heads = num_heads
        self.scale = qk_scale or (dim // num_heads) ** -0.5
        rows = math.prod(2 * w - 1 for w in self.window_size)
        self.relative_position_bias_table = nn.Parameter(torch.zeros(rows, num_heads))
        self.register_buffer("relative_position_index", relative_index_buffer(self.window_size))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        trunc_normal_(self.relative_position_bias_table, std=.02)
        self.softmax = nn.Softmax(dim=-1)

    def forward_tokens(self, x, geom, residual=None):
        """Fused path: x (rows, C) un-partitioned token rows of geometry `geom` -> (rows, C)."""
        return self.attend(linear(x, self.qkv), geom, residual)

    def attend(self, qkv, geom, residual=None):
        """Attention + proj (+ residual) from the projected (rows, 3C) qkv."""
        _no_attn_dropout(self)
        o = window_attention_self(qkv, self.relative_position_bias_table, geom, self.num_heads, kind=0,
                                  scale=self.scale)
        if residual is not None and inactive(self.proj_drop):
            return linear(o, self.proj, residual=residual)
        out = self.proj_drop(linear(o, self.proj))
        return out if residual is None else residual + out

    def forward(self, x, mask=None):
        """Reference signature: x (num_windows*B, N, C) already partitioned.  Without a mask each
        window is attended as its own unshifted volume; a shift mask (calculate_mask of the block,
        (nW, N, N)) is validated once and mapped back to the geometry the kernel derives it from."""
        if mask is not None:
            return attend_masked_windows(self.forward_tokens, [x], mask, self.window_size)
        B_, N, C = x.shape
        geom = geometry(B_, self.window_size, self.window_size, 0)
        return self.forward_tokens(x.reshape(B_ * N, C), geom).view(B_, N, C)

    def extra_repr(self):
        return f'dim={self.dim}, window_size={self.window_size}, num_heads={self.num_heads}'

    def flops(self, N):
        # multiply-accumulates per window, as the reference counts them (swinfusion_module.py:150-161)
        hd = self.dim // self.num_heads
        return N * self.dim * 3 * self.dim + 2 * self.num_heads * N * N * hd + N * self.dim * self.dim


class Cross_WindowAttention(nn.Module):
    """Window attention with queries from x and keys/values from y (swinfusion_module.py:163-262)."""

    def __init__(self, dim, window_size, num_heads, qkv_bias=True, qk_scale=None, attn_drop=0., proj_drop=0.):
        super().__init__()
        self.dim = dim
        self.window_size = tuple(window_size)
        self.num_heads = num_heads
        self.scale = qk_scale or (dim // num_heads) ** -0.5
        rows = math.prod(2 * w - 1 for w in self.window_size)
        self.relative_position_bias_table = nn.Parameter(torch.zeros(rows, num_heads))
        self.register_buffer("relative_position_index", relative_index_buffer(self.window_size))
        self.q = nn.Linear(dim, dim, bias=qkv_bias)
        self.kv = nn.Linear(dim, dim * 2, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        trunc_normal_(self.relative_position_bias_table, std=.02)
        self.softmax = nn.Softmax(dim=-1)

    def forward_tokens(self, x, y, geom, residual=None):
        return self.attend(linear(x, self.q), linear(y, self.kv), geom, residual)

    def attend(self, q, kv, geom, residual=None):
        """Cross attention + proj (+ residual) from the projected q (rows, C) and kv (rows, 2C)."""
        _no_attn_dropout(self)
        o = window_attention_cross(q, kv, self.relative_position_bias_table, geom, self.num_heads, kind=0,
                                   scale=self.scale)
        if residual is not None and inactive(self.proj_drop):
            return linear(o, self.proj, residual=residual)
        out = self.proj_drop(linear(o, self.proj))
        return out if residual is None else residual + out

    def forward(self, x, y, mask=None):
        if mask is not None:
            return attend_masked_windows(self.forward_tokens, [x, y], mask, self.window_size)
        B_, N, C = x.shape
        geom = geometry(B_, self.window_size, self.window_size, 0)
        return self.forward_tokens(x.reshape(B_ * N, C), y.reshape(B_ * N, C), geom).view(B_, N, C)

    def extra_repr(self):
        return f'dim={self.dim}, window_size={self.window_size}, num_heads={self.num_heads}'


class SwinTransformerBlock_fusion(nn.Module):
    """Pre-norm shifted-window block (swinfusion_module.py:265-398)."""

    def __init__(self, dim, input_resolution, num_heads, window_size=7, shift_size=0,
                 mlp_ratio=4., qkv_bias=True, qk_scale=None, drop=0., attn_drop=0., drop_path=0.,
                 act_layer=nn.GELU, norm_layer=nn.LayerNorm):
        super().__init__()
        self.dim = dim
        self.input_resolution = tuple(input_resolution)
        self.num_heads = num_heads
        self.mlp_ratio = mlp_ratio
        self.window_size, self.shift_size = clamp_window(self.input_resolution, window_size, shift_size)
        assert 0 <= self.shift_size < self.window_size, "shift_size must in 0-window_size"
        nd = len(self.input_resolution)
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention_fusion(dim, window_size=to_ntuple(self.window_size, nd), num_heads=num_heads,
                                           qkv_bias=qkv_bias, qk_scale=qk_scale, attn_drop=attn_drop,
                                           proj_drop=drop)
        self.drop_path = DropPath(drop_path) if drop_path > 0. else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp_fusion(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop)
        attn_mask = self.calculate_mask(self.input_resolution) if self.shift_size > 0 else None
        self.register_buffer("attn_mask", attn_mask)

    def calculate_mask(self, x_size):
        nd = len(x_size)
        return shift_mask_buffer(tuple(x_size), to_ntuple(self.window_size, nd), to_ntuple(self.shift_size, nd))

    def forward(self, x, x_size, skip=None, emit_skip=0):
        """skip: the identity skip of the residual group this block ends (RSTB / CRSTB), added in
        the MLP epilogue when the fused path runs (one full-size add less per group).
        emit_skip (the group's first block): 1 also returns the group input as a second view out
        of norm1 + qkv, to be the last block's skip, so that the skip's gradient joins this block's
        input gradient inside the LN + Linear backward (no autograd add); 2 does the same for a
        one-block group and uses the view as this block's own skip."""
        B, L, C = x.shape
        geom = geometry(B, x_size, self.window_size, self.shift_size)
        xs = x
        if inactive(self.drop_path) and ln_linear_ok(x, self.norm1, self.attn.qkv):
            # norm1 + qkv in one kernel; the residual's gradient joins inside its backward
            if emit_skip:
                qkv, xr, xs = ln_linear(x, self.norm1, self.attn.qkv, passthrough=2)
            else:
                qkv, xr = ln_linear(x, self.norm1, self.attn.qkv, passthrough=True)
            if emit_skip == 2:
                skip = xs
            x = self.attn.attend(qkv.reshape(B * L, 3 * C), geom, residual=xr.reshape(B * L, C)).view(B, L, C)
            out = ln_mlp(x, self.norm2, self.mlp, skip=skip)   # x + mlp(norm2(x)) [+ skip], one kernel
            return (out, xs) if emit_skip == 1 else out
        if emit_skip == 2:
            skip = x
        xn = layer_norm(x, self.norm1).reshape(B * L, C)
        if inactive(self.drop_path):   # residual adds fused into the proj / fc2 epilogues
            x = self.attn.forward_tokens(xn, geom, residual=x.reshape(B * L, C)).view(B, L, C)
            x = self.mlp(layer_norm(x, self.norm2), residual=x)
        else:
            x = x + self.drop_path(self.attn.forward_tokens(xn, geom).view(B, L, C))
            x = x + self.drop_path(self.mlp(layer_norm(x, self.norm2)))
        out = x if skip is None else x + skip
        return (out, xs) if emit_skip == 1 else out

    def extra_repr(self):
        return (f"dim={self.dim}, input_resolution={self.input_resolution}, num_heads={self.num_heads}, "
                f"window_size={self.window_size}, shift_size={self.shift_size}, mlp_ratio={self.mlp_ratio}")


class Cross_SwinTransformerBlock(nn.Module):
    """Two cross window attentions A<-B and B<-A sharing one geometry (swinfusion_module.py:400-558)."""

    def __init__(self, dim, input_resolution, num_heads, window_size=7, shift_size=0,
                 mlp_ratio=4., qkv_bias=True, qk_scale=None, drop=0., attn_drop=0., drop_path=0.,
                 act_layer=nn.GELU, norm_layer=nn.LayerNorm):
        super().__init__()
        self.dim = dim
        self.input_resolution = tuple(input_resolution)
        self.num_heads = num_heads
        self.mlp_ratio = mlp_ratio
        self.window_size, self.shift_size = clamp_window(self.input_resolution, window_size, shift_size)
        assert 0 <= self.shift_size < self.window_size, "shift_size must in 0-window_size"
        nd = len(self.input_resolution)
        win = to_ntuple(self.window_size, nd)
        self.norm1_A = norm_layer(dim)
        self.norm1_B = norm_layer(dim)
        self.attn_A = Cross_WindowAttention(dim, window_size=win, num_heads=num_heads, qkv_bias=qkv_bias,
                                            qk_scale=qk_scale, attn_drop=attn_drop, proj_drop=drop)
        self.attn_B = Cross_WindowAttention(dim, window_size=win, num_heads=num_heads, qkv_bias=qkv_bias,
                                            qk_scale=qk_scale, attn_drop=attn_drop, proj_drop=drop)
        self.drop_path_A = DropPath(drop_path) if drop_path > 0. else nn.Identity()
        self.drop_path_B = DropPath(drop_path) if drop_path > 0. else nn.Identity()
        self.norm2_A = norm_layer(dim)
        self.norm2_B = norm_layer(dim)
        hidden = int(dim * mlp_ratio)
        self.mlp_A = Mlp_fusion(in_features=dim, hidden_features=hidden, act_layer=act_layer, drop=drop)
        self.mlp_B = Mlp_fusion(in_features=dim, hidden_features=hidden, act_layer=act_layer, drop=drop)
        attn_mask = self.calculate_mask(self.input_resolution) if self.shift_size > 0 else None
        self.register_buffer("attn_mask", attn_mask)

    def calculate_mask(self, x_size):
        nd = len(x_size)
        return shift_mask_buffer(tuple(x_size), to_ntuple(self.window_size, nd), to_ntuple(self.shift_size, nd))

    def forward(self, x, y, x_size, skip=None, emit_skip=0):
        """skip: (skip_x, skip_y), the identity skips of the CRSTB inter-modal group this block
        ends, added in the MLP epilogues on the fused path.  emit_skip as in
        SwinTransformerBlock_fusion, for the pair (x, y)."""
        sx, sy = skip if skip is not None else (None, None)
        xs, ys = x, y
        B, L, C = x.shape
        geom = geometry(B, x_size, self.window_size, self.shift_size)
        if (inactive(self.drop_path_A) and inactive(self.drop_path_B)
                and ln_linear_ok(x, self.norm1_A, self.attn_A.q) and ln_linear_ok(x, self.norm1_A, self.attn_B.kv)):
            # norm1 fused into each projection that reads it (x -> q_A, kv_B; y -> q_B, kv_A)
            if emit_skip:
                qa, xr, xs = ln_linear(x, self.norm1_A, self.attn_A.q, passthrough=2)
                qb, yr, ys = ln_linear(y, self.norm1_B, self.attn_B.q, passthrough=2)
            else:
                qa, xr = ln_linear(x, self.norm1_A, self.attn_A.q, passthrough=True)
                qb, yr = ln_linear(y, self.norm1_B, self.attn_B.q, passthrough=True)
            if emit_skip == 2:
                sx, sy = xs, ys
            kvb = ln_linear(x, self.norm1_A, self.attn_B.kv)
            kva = ln_linear(y, self.norm1_B, self.attn_A.kv)
            xa = self.attn_A.attend(qa.reshape(B * L, C), kva.reshape(B * L, 2 * C), geom,
                                    residual=xr.reshape(B * L, C)).view(B, L, C)
            yb = self.attn_B.attend(qb.reshape(B * L, C), kvb.reshape(B * L, 2 * C), geom,
                                    residual=yr.reshape(B * L, C)).view(B, L, C)
            out = ln_mlp(xa, self.norm2_A, self.mlp_A, skip=sx), ln_mlp(yb, self.norm2_B, self.mlp_B, skip=sy)
            return (out, (xs, ys)) if emit_skip == 1 else out
        if emit_skip == 2:
            sx, sy = x, y
        xn = layer_norm(x, self.norm1_A).reshape(B * L, C)
        yn = layer_norm(y, self.norm1_B).reshape(B * L, C)
        if inactive(self.drop_path_A) and inactive(self.drop_path_B):   # fused residual adds
            xa = self.attn_A.forward_tokens(xn, yn, geom, residual=x.reshape(B * L, C)).view(B, L, C)
            yb = self.attn_B.forward_tokens(yn, xn, geom, residual=y.reshape(B * L, C)).view(B, L, C)
            x = self.mlp_A(layer_norm(xa, self.norm2_A), residual=xa)
            y = self.mlp_B(layer_norm(yb, self.norm2_B), residual=yb)
        else:
            a = self.attn_A.forward_tokens(xn, yn, geom).view(B, L, C)
            b = self.attn_B.forward_tokens(yn, xn, geom).view(B, L, C)
            x = x + self.drop_path_A(a)
            x = x + self.drop_path_A(self.mlp_A(layer_norm(x, self.norm2_A)))
            y = y + self.drop_path_B(b)
            y = y + self.drop_path_B(self.mlp_B(layer_norm(y, self.norm2_B)))
        out = (x if sx is None else x + sx), (y if sy is None else y + sy)
        return (out, (xs, ys)) if emit_skip == 1 else out

    def extra_repr(self):
        return (f"dim={self.dim}, input_resolution={self.input_resolution}, num_heads={self.num_heads}, "
                f"window_size={self.window_size}, shift_size={self.shift_size}, mlp_ratio={self.mlp_ratio}")


class PatchMerging_fusion(nn.Module):
    """Norm over the 2^k neighbour concat, then Linear(2^k C -> 2C) (swinfusion_module.py:560-606)."""

    def __init__(self, input_resolution, dim, norm_layer=nn.LayerNorm):
        super().__init__()
        self.input_resolution = tuple(input_resolution)
        self.dim = dim
        k = 2 ** len(self.input_resolution)
        self.reduction = nn.Linear(k * dim, 2 * dim, bias=False)
        self.norm = norm_layer(k * dim)

    def forward(self, x):
        assert x.shape[1] == math.prod(self.input_resolution), "input feature has wrong size"
        assert all(r % 2 == 0 for r in self.input_resolution), f"x size {self.input_resolution} are not even."
        return linear(layer_norm(patch_merge_gather(x, self.input_resolution), self.norm), self.reduction)

    def extra_repr(self):
        return f"input_resolution={self.input_resolution}, dim={self.dim}"


class BasicLayer_fusion(nn.Module):
    """depth x SwinTransformerBlock_fusion, shift on odd blocks (swinfusion_module.py:609-676)."""

    def __init__(self, dim, input_resolution, depth, num_heads, window_size,
                 mlp_ratio=4., qkv_bias=True, qk_scale=None, drop=0., attn_drop=0.,
                 drop_path=0., norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=False):
        super().__init__()
        self.dim = dim
        self.input_resolution = input_resolution
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            SwinTransformerBlock_fusion(dim=dim, input_resolution=input_resolution, num_heads=num_heads,
                                        window_size=window_size, shift_size=0 if i % 2 == 0 else window_size // 2,
                                        mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop,
                                        attn_drop=attn_drop,
                                        drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path,
                                        norm_layer=norm_layer)
            for i in range(depth)])
        self.downsample = downsample(input_resolution, dim=dim, norm_layer=norm_layer) if downsample else None

    def forward(self, x, x_size, skip=None):
        """skip: the enclosing residual group's identity skip (RSTB / CRSTB), handed to the last
        block so it joins that block's MLP epilogue; added after the downsample when there is one.
        When the skip is the group's own input, the first block re-emits it as a view of its
        norm1 + qkv (emit_skip) so the skip's gradient joins inside that block's backward."""
        last = len(self.blocks) - 1
        fold = skip is not None and skip is x and self.downsample is None and last >= 0

        def run(blk, *args):
            return checkpoint.checkpoint(blk, *args, use_reentrant=False) if self.use_checkpoint else blk(*args)
        for i, blk in enumerate(self.blocks):
            if fold and i == 0:
                if last == 0:
                    x = run(blk, x, x_size, None, 2)
                else:
                    x, skip = run(blk, x, x_size, None, 1)
                continue
            s = skip if (i == last and self.downsample is None) else None
            x = run(blk, x, x_size, s)
        if self.downsample is not None:
            x = self.downsample(x)
            return x if skip is None else x + skip
        return x if self.blocks or skip is None else x + skip

    def extra_repr(self):
        return f"dim={self.dim}, input_resolution={self.input_resolution}, depth={self.depth}"


class Cross_BasicLayer(nn.Module):
    """depth x Cross_SwinTransformerBlock (swinfusion_module.py:678-747)."""

    def __init__(self, dim, input_resolution, depth, num_heads, window_size,
                 mlp_ratio=4., qkv_bias=True, qk_scale=None, drop=0., attn_drop=0.,
                 drop_path=0., norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=False):
        super().__init__()
        self.dim = dim
        self.input_resolution = input_resolution
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            Cross_SwinTransformerBlock(dim=dim, input_resolution=input_resolution, num_heads=num_heads,
                                       window_size=window_size, shift_size=0 if i % 2 == 0 else window_size // 2,
                                       mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop,
                                       attn_drop=attn_drop,
                                       drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path,
                                       norm_layer=norm_layer)
            for i in range(depth)])
        self.downsample = downsample(input_resolution, dim=dim, norm_layer=norm_layer) if downsample else None

    def forward(self, x, y, x_size, skip=None):
        """skip: (skip_x, skip_y) of the enclosing CRSTB, joined in the last block's MLP epilogues
        (re-emitted by the first block when it is the group's input, as in BasicLayer_fusion)."""
        last = len(self.blocks) - 1
        fold = (skip is not None and skip[0] is x and skip[1] is y and self.downsample is None and last >= 0)

        def run(blk, *args):
            return checkpoint.checkpoint(blk, *args, use_reentrant=False) if self.use_checkpoint else blk(*args)
        for i, blk in enumerate(self.blocks):
            if fold and i == 0:
                if last == 0:
                    x, y = run(blk, x, y, x_size, None, 2)
                else:
                    (x, y), skip = run(blk, x, y, x_size, None, 1)
                continue
            s = skip if (i == last and self.downsample is None) else None
            x, y = run(blk, x, y, x_size, s)
        if self.downsample is not None:
            x, y = self.downsample(x), self.downsample(y)
            if skip is not None:
                x, y = x + skip[0], y + skip[1]
        elif skip is not None and not self.blocks:
            x, y = x + skip[0], y + skip[1]
        return x, y

    def extra_repr(self):
        return f"dim={self.dim}, input_resolution={self.input_resolution}, depth={self.depth}"


def _conv_like(nd, cin, cout):
    """nn.Conv2d / nn.Conv3d k3 s1 p1 matching the layer's rank (state_dict compatible in 2D)."""
    return (nn.Conv2d if nd == 2 else nn.Conv3d)(cin, cout, 3, 1, 1)


class RSTB(nn.Module):
    """Residual group: BasicLayer_fusion + identity skip (swinfusion_module.py:750-824).  The 1conv
    residual conv and patch (un)embed are constructed for state_dict parity but, as in the
    reference forward (:812-814), never applied."""

    def __init__(self, dim, input_resolution, depth, num_heads, window_size,
                 mlp_ratio=4., qkv_bias=True, qk_scale=None, drop=0., attn_drop=0.,
                 drop_path=0., norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=False,
                 img_size=224, patch_size=4, resi_connection='1conv'):
        super().__init__()
        self.dim = dim
        self.input_resolution = input_resolution
        nd = len(input_resolution)
        self.residual_group = BasicLayer_fusion(dim=dim, input_resolution=input_resolution, depth=depth,
                                                num_heads=num_heads, window_size=window_size, mlp_ratio=mlp_ratio,
                                                qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop,
                                                attn_drop=attn_drop, drop_path=drop_path, norm_layer=norm_layer,
                                                downsample=downsample, use_checkpoint=use_checkpoint)
        if resi_connection == '1conv':
            self.conv = _conv_like(nd, dim, dim)
        elif resi_connection == '3conv':
            C = nn.Conv2d if nd == 2 else nn.Conv3d
            self.conv = nn.Sequential(C(dim, dim // 4, 3, 1, 1), nn.LeakyReLU(0.2, inplace=True),
                                      C(dim // 4, dim // 4, 1, 1, 0), nn.LeakyReLU(0.2, inplace=True),
                                      C(dim // 4, dim, 3, 1, 1))
        self.patch_embed = PatchEmbed_fusion(img_size=img_size, patch_size=patch_size, in_chans=0, embed_dim=dim,
                                             norm_layer=None)
        self.patch_unembed = PatchUnEmbed(img_size=img_size, patch_size=patch_size, in_chans=0, embed_dim=dim,
                                          norm_layer=None)

    def forward(self, x, x_size):
        # residual_group(x) + x (:814), the "+ x" joined inside the group's last MLP epilogue
        return self.residual_group(x, x_size, skip=x)


class CRSTB(nn.Module):
    """Intra-modal groups A and B then the inter-modal Cross_BasicLayer, each with an identity
    skip (swinfusion_module.py:826-939)."""

    def __init__(self, dim, input_resolution, depth, num_heads, window_size,
                 mlp_ratio=4., qkv_bias=True, qk_scale=None, drop=0., attn_drop=0.,
                 drop_path=0., norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=False,
                 img_size=224, patch_size=4, resi_connection='1conv'):
        super().__init__()
        self.dim = dim
        self.input_resolution = input_resolution
        nd = len(input_resolution)
        kw = dict(dim=dim, input_resolution=input_resolution, depth=depth, num_heads=num_heads,
                  window_size=window_size, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop,
                  attn_drop=attn_drop, drop_path=drop_path, norm_layer=norm_layer, downsample=downsample,
                  use_checkpoint=use_checkpoint)
        self.residual_group = Cross_BasicLayer(**kw)
        self.residual_group_A = BasicLayer_fusion(**kw)
        self.residual_group_B = BasicLayer_fusion(**kw)
        if resi_connection == '1conv':
            self.conv_A = _conv_like(nd, dim, dim)
            self.conv_B = _conv_like(nd, dim, dim)
        elif resi_connection == '3conv':
            C = nn.Conv2d if nd == 2 else nn.Conv3d

            def three():
                return nn.Sequential(C(dim, dim // 4, 3, 1, 1), nn.LeakyReLU(0.2, inplace=True),
                                     C(dim // 4, dim // 4, 1, 1, 0), nn.LeakyReLU(0.2, inplace=True),
                                     C(dim // 4, dim, 3, 1, 1))
            self.conv_A, self.conv_B = three(), three()
        self.patch_embed = PatchEmbed_fusion(img_size=img_size, patch_size=patch_size, in_chans=0, embed_dim=dim,
                                             norm_layer=None)
        self.patch_unembed = PatchUnEmbed(img_size=img_size, patch_size=patch_size, in_chans=0, embed_dim=dim,
                                          norm_layer=None)

    def forward(self, x, y, x_size):
        # the three identity skips (:918-927) joined inside each group's last MLP epilogue
        x = self.residual_group_A(x, x_size, skip=x)
        y = self.residual_group_B(y, x_size, skip=y)
        return self.residual_group(x, y, x_size, skip=(x, y))


class PatchEmbed_fusion(nn.Module):
    """Flatten a (B, C, *spatial) map into tokens (+ optional LN) (swinfusion_module.py:941-981).
    Channels-last callers skip the transpose entirely (see model.SwinFusion)."""

    def __init__(self, img_size=224, patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        img_size = to_2tuple(img_size)
        patch_size = to_2tuple(patch_size)
        self.img_size = img_size
        self.patch_size = patch_size
        self.patches_resolution = [i // p for i, p in zip(img_size, patch_size)]
        self.num_patches = math.prod(self.patches_resolution)
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None

    def forward(self, x):
        x = x.flatten(2).transpose(1, 2)
        return layer_norm(x, self.norm) if self.norm is not None else x


class PatchUnEmbed(nn.Module):
    """Tokens (B, L, C) -> (B, C, *x_size) (swinfusion_module.py:984-1015)."""

    def __init__(self, img_size=224, patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        img_size = to_2tuple(img_size)
        patch_size = to_2tuple(patch_size)
        self.img_size = img_size
        self.patch_size = patch_size
        self.patches_resolution = [i // p for i, p in zip(img_size, patch_size)]
        self.num_patches = math.prod(self.patches_resolution)
        self.in_chans = in_chans
        self.embed_dim = embed_dim

    def forward(self, x, x_size):
        B = x.shape[0]
        return x.transpose(1, 2).reshape(B, self.embed_dim, *x_size)


class Upsample(nn.Sequential):
    """conv + PixelShuffle upsampler (swinfusion_module.py:1018-1037; unused by SwinFusion's forward)."""

    def __init__(self, scale, num_feat):
        m = []
        if (scale & (scale - 1)) == 0:
            for _ in range(int(math.log(scale, 2))):
                m += [nn.Conv2d(num_feat, 4 * num_feat, 3, 1, 1), nn.PixelShuffle(2)]
        elif scale == 3:
            m += [nn.Conv2d(num_feat, 9 * num_feat, 3, 1, 1), nn.PixelShuffle(3)]
        else:
            raise ValueError(f'scale {scale} is not supported. Supported scales: 2^n and 3.')
        super().__init__(*m)


class UpsampleOneStep(nn.Sequential):
    """Single conv + PixelShuffle (swinfusion_module.py:1040-1061)."""

    def __init__(self, scale, num_feat, num_out_ch, input_resolution=None):
        self.num_feat = num_feat
        self.input_resolution = input_resolution
        super().__init__(nn.Conv2d(num_feat, (scale ** 2) * num_out_ch, 3, 1, 1), nn.PixelShuffle(scale))


def conv_tokens(conv, x, slope=1.0):
    """Apply an nn.Conv2d/nn.Conv3d module to channels-last tokens (B, *spatial, Cin) through the
    HIP conv kernel (2D convs as kd = 1 on D = 1 volumes)."""
    w = conv.weight
    if w.dim() == 4:
        w = w.unsqueeze(2)
        x = x.unsqueeze(1)
        st = (1,) + tuple(conv.stride)
        pd = (0,) + tuple(conv.padding)
        return conv3d_cl(x, w, conv.bias, st, pd, slope).squeeze(1)
    return conv3d_cl(x, w, conv.bias, tuple(conv.stride), tuple(conv.padding), slope)
