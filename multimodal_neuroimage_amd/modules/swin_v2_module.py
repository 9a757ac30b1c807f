"""Swin Transformer V2 window-attention stack — MI355X build.

Drop-in for the reference's modules/swin_v2_module.py (same names, signatures, state_dict keys).
The cosine window attention (normalize, clamped logit scale, 16*sigmoid(cpb_mlp) bias, shift
mask, softmax, AV) plus the roll/partition/reverse runs as one HIP launch per block
(libmmni.so mmni_wattn_fwd/bwd, kind 1); the tiny cpb MLP (batch independent) stays in torch so
autograd carries its gradient.  PatchEmbed's strided conv runs on the channels-last HIP conv
kernel.  Blocks accept 2D (H, W) or 3D (D, H, W) resolutions (the build's 3D lift).
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.utils.checkpoint as checkpoint

from ..functional import window_attention_self, conv3d_cl, LN100, layer_norm, linear, mlp, cpb_table
from ._common import (DropPath, to_2tuple, to_ntuple, trunc_normal_, relative_index_buffer, shift_mask_buffer,
                      attend_masked_windows, clamp_window, geometry, patch_merge_gather)


class Mlp(nn.Module):
    """fc1 -> act -> drop -> fc2 -> drop (swin_v2_module.py:16-32)."""

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


def window_partition(x, window_size):
    """(B, *spatial, C) -> (num_windows*B, *window, C) (swin_v2_module.py:35-46; any rank)."""
    from .swinfusion_module import window_partition_fusion
    return window_partition_fusion(x, window_size)


def window_reverse(windows, window_size, *spatial):
    """Inverse of window_partition (swin_v2_module.py:49-62)."""
    from .swinfusion_module import window_reverse_fusion
    return window_reverse_fusion(windows, window_size, *spatial)


def _coords_table(window, pretrained):
    """Log-spaced relative coordinate table (swin_v2_module.py:96-111), any number of axes."""
    nd = len(window)
    axes = [torch.arange(-(w - 1), w, dtype=torch.float32) for w in window]
    tab = torch.stack(torch.meshgrid(*axes, indexing="ij"), dim=-1).unsqueeze(0)
    norm = pretrained if pretrained[0] > 0 else window
    for a in range(nd):
        tab[..., a] /= (norm[a] - 1)
    tab *= 8
    return torch.sign(tab) * torch.log2(torch.abs(tab) + 1.0) / np.log2(8)


class WindowAttention(nn.Module):
    """Cosine window attention with continuous position bias (swin_v2_module.py:65-195)."""

    def __init__(self, dim, window_size, num_heads_swin, qkv_bias=True, attn_drop=0., proj_drop=0.,
                 pretrained_window_size=[0, 0]):
        super().__init__()
        self.dim = dim
        self.window_size = tuple(window_size)
        nd = len(self.window_size)
        pw = pretrained_window_size
        pw = tuple(pw) if isinstance(pw, (list, tuple)) else (pw,) * nd
        self.pretrained_window_size = (pw + (0,) * nd)[:nd]
        self.num_heads_swin = num_heads_swin
        self.logit_scale = nn.Parameter(torch.log(10 * torch.ones((num_heads_swin, 1, 1))), requires_grad=True)
        self.cpb_mlp = nn.Sequential(nn.Linear(nd, 512, bias=True), nn.ReLU(inplace=True),
                                     nn.Linear(512, num_heads_swin, bias=False))
        self.register_buffer("relative_coords_table", _coords_table(self.window_size, self.pretrained_window_size))
        self.register_buffer("relative_position_index", relative_index_buffer(self.window_size))
        self.qkv = nn.Linear(dim, dim * 3, bias=False)
        if qkv_bias:
            self.q_bias = nn.Parameter(torch.zeros(dim))
            self.v_bias = nn.Parameter(torch.zeros(dim))
        else:
            self.q_bias = None
            self.v_bias = None
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        self.softmax = nn.Softmax(dim=-1)

    def bias_table(self):
        """16*sigmoid(cpb_mlp(relative_coords_table)) as a (Tsz, heads) table (swin_v2_module.py:158-162),
        one HIP launch per direction (functional.cpb_table)."""
        l1, l2 = self.cpb_mlp[0], self.cpb_mlp[2]
        return cpb_table(self.relative_coords_table, l1.weight, l1.bias, l2.weight)

    def tau(self):
        """exp(min(logit_scale, ln 100)) per head (swin_v2_module.py:154-155)."""
        return torch.clamp(self.logit_scale, max=LN100).exp().reshape(-1)

    def forward_tokens(self, x, geom):
        if self.training and self.attn_drop.p > 0:
            raise NotImplementedError("mmni window attention: attention dropout > 0 in training is not implemented")
        bias = None
        if self.q_bias is not None:
            bias = torch.cat((self.q_bias, torch.zeros_like(self.v_bias, requires_grad=False), self.v_bias))
        qkv = linear(x, self.qkv.weight, bias)
        o = window_attention_self(qkv, self.bias_table(), geom, self.num_heads_swin, kind=1, tau=self.tau())
        return self.proj_drop(linear(o, self.proj))

    def forward(self, x, mask=None):
        """Reference signature on pre-partitioned windows (num_windows*B, N, C); a shift mask
        (calculate_mask, (nW, N, N)) is validated once and mapped back to its geometry."""
        if mask is not None:
            return attend_masked_windows(self.forward_tokens, [x], mask, self.window_size)
        B_, N, C = x.shape
        geom = geometry(B_, self.window_size, self.window_size, 0)
        return self.forward_tokens(x.reshape(B_ * N, C), geom).view(B_, N, C)

    def extra_repr(self):
        return (f'dim={self.dim}, window_size={self.window_size}, '
                f'pretrained_window_size={self.pretrained_window_size}, num_heads_swin={self.num_heads_swin}')

    def flops(self, N):
        hd = self.dim // self.num_heads_swin
        return N * self.dim * 3 * self.dim + 2 * self.num_heads_swin * N * N * hd + N * self.dim * self.dim


class SwinTransformerBlock(nn.Module):
    """Res-post-norm shifted-window block (swin_v2_module.py:198-322)."""

    def __init__(self, dim, input_resolution, num_heads_swin, window_size=4, shift_size=0,
                 mlp_ratio=4., qkv_bias=True, drop=0., attn_drop=0., drop_path=0.,
                 act_layer=nn.GELU, norm_layer=nn.LayerNorm, pretrained_window_size=0):
        super().__init__()
        self.dim = dim
        self.input_resolution = tuple(input_resolution)
        self.num_heads_swin = num_heads_swin
        self.mlp_ratio = mlp_ratio
        self.window_size, self.shift_size = clamp_window(self.input_resolution, window_size, shift_size)
        assert 0 <= self.shift_size < self.window_size, "shift_size must in 0-window_size"
        nd = len(self.input_resolution)
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention(dim, window_size=to_ntuple(self.window_size, nd), num_heads_swin=num_heads_swin,
                                    qkv_bias=qkv_bias, attn_drop=attn_drop, proj_drop=drop,
                                    pretrained_window_size=to_ntuple(pretrained_window_size, nd))
        self.drop_path = DropPath(drop_path) if drop_path > 0. else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop)
        attn_mask = None
        if self.shift_size > 0:
            attn_mask = shift_mask_buffer(self.input_resolution, to_ntuple(self.window_size, nd),
                                          to_ntuple(self.shift_size, nd))
        self.register_buffer("attn_mask", attn_mask)

    def forward(self, x):
        B, L, C = x.shape
        assert L == math.prod(self.input_resolution), "input feature has wrong size"
        geom = geometry(B, self.input_resolution, self.window_size, self.shift_size)
        a = self.attn.forward_tokens(x.reshape(B * L, C), geom).view(B, L, C)
        x = x + self.drop_path(layer_norm(a, self.norm1))
        return x + self.drop_path(layer_norm(self.mlp(x), self.norm2))

    def extra_repr(self):
        return (f"dim={self.dim}, input_resolution={self.input_resolution}, num_heads_swin={self.num_heads_swin}, "
                f"window_size={self.window_size}, shift_size={self.shift_size}, mlp_ratio={self.mlp_ratio}")


class PatchMerging(nn.Module):
    """2^k neighbour concat -> Linear(2^k C -> 2C, no bias) -> LN(2C) (swin_v2_module.py:325-373)."""

    def __init__(self, input_resolution, dim, norm_layer=nn.LayerNorm):
        super().__init__()
        self.input_resolution = tuple(input_resolution)
        self.dim = dim
        k = 2 ** len(self.input_resolution)
        self.reduction = nn.Linear(k * dim, 2 * dim, bias=False)
        self.norm = norm_layer(2 * dim)

    def forward(self, x):
        assert x.shape[1] == math.prod(self.input_resolution), "input feature has wrong size"
        assert all(r % 2 == 0 for r in self.input_resolution), f"x size {self.input_resolution} are not even."
        return layer_norm(linear(patch_merge_gather(x, self.input_resolution), self.reduction), self.norm)

    def extra_repr(self):
        return f"input_resolution={self.input_resolution}, dim={self.dim}"


class BasicLayer(nn.Module):
    """depth x SwinTransformerBlock (+ PatchMerging) (swin_v2_module.py:376-451)."""

    def __init__(self, dim, input_resolution, depth, num_heads_swin, window_size,
                 mlp_ratio=4., qkv_bias=True, drop=0., attn_drop=0.,
                 drop_path=0., norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=False,
                 pretrained_window_size=0):
        super().__init__()
        self.dim = dim
        self.input_resolution = input_resolution
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(dim=dim, input_resolution=input_resolution, num_heads_swin=num_heads_swin,
                                 window_size=window_size, shift_size=0 if i % 2 == 0 else window_size // 2,
                                 mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, drop=drop, attn_drop=attn_drop,
                                 drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path,
                                 norm_layer=norm_layer, pretrained_window_size=pretrained_window_size)
            for i in range(depth)])
        self.downsample = downsample(input_resolution, dim=dim, norm_layer=norm_layer) if downsample else None

    def forward(self, x):
        for blk in self.blocks:
            x = checkpoint.checkpoint(blk, x, use_reentrant=False) if self.use_checkpoint else blk(x)
        return self.downsample(x) if self.downsample is not None else x

    def extra_repr(self):
        return f"dim={self.dim}, input_resolution={self.input_resolution}, depth={self.depth}"

    def _init_respostnorm(self):
        """Zero the post-norms (swin_v2_module.py:446-451)."""
        for blk in self.blocks:
            for n in (blk.norm1, blk.norm2):
                nn.init.constant_(n.bias, 0)
                nn.init.constant_(n.weight, 0)


class PatchEmbed(nn.Module):
    """Strided patch conv (+ LN) (swin_v2_module.py:454-499).  2D: Conv2d(k=s=patch) on (B,C,H,W);
    the 3D lift (img_size_d given) uses Conv3d(k=s=patch) on (B,C,D,H,W).  Either runs on the
    channels-last HIP conv kernel and lands directly in token order (B, L, embed)."""

    def __init__(self, img_size_w=1, img_size_h=84, patch_size=4, in_chans=1, embed_dim=96, norm_layer=None,
                 img_size_d=None):
        super().__init__()
        self.volumetric = img_size_d is not None
        if self.volumetric:
            patch_size = to_ntuple(patch_size, 3)
            patches_resolution = [img_size_d // patch_size[0], img_size_h // patch_size[1],
                                  img_size_w // patch_size[2]]
        else:
            patch_size = to_2tuple(patch_size)
            if img_size_w // patch_size[1] == 0:
                patches_resolution = [img_size_h // patch_size[0], img_size_w]
            else:
                patches_resolution = [img_size_h // patch_size[0], img_size_w // patch_size[1]]
        self.img_size_d = img_size_d
        self.img_size_h = img_size_h
        self.img_size_w = img_size_w
        self.patch_size = patch_size
        self.patches_resolution = patches_resolution
        self.num_patches = math.prod(patches_resolution)
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        conv = nn.Conv3d if self.volumetric else nn.Conv2d
        self.proj = conv(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None

    def forward(self, x):
        B, C = x.shape[:2]
        spatial = tuple(x.shape[2:])
        if self.volumetric:
            assert spatial == (self.img_size_d, self.img_size_h, self.img_size_w), \
                f"Input volume size {spatial} doesn't match model"
            x_cl = x.permute(0, 2, 3, 4, 1) if C > 1 else x.reshape(B, *spatial, 1)
            w, st = self.proj.weight, tuple(self.proj.stride)
        else:
            assert spatial == (self.img_size_h, self.img_size_w), \
                f"Input image size ({spatial[0]}*{spatial[1]}) doesn't match model ({self.img_size_h}*{self.img_size_w})."
            x_cl = (x.permute(0, 2, 3, 1) if C > 1 else x.reshape(B, *spatial, 1)).unsqueeze(1)
            w, st = self.proj.weight.unsqueeze(2), (1,) + tuple(self.proj.stride)
        y = conv3d_cl(x_cl, w, self.proj.bias, st, 0)
        y = y.reshape(B, -1, self.embed_dim)
        return layer_norm(y, self.norm) if self.norm is not None else y

    def flops(self):
        f = self.num_patches * self.embed_dim * self.in_chans * math.prod(self.patch_size)
        return f + (self.num_patches * self.embed_dim if self.norm is not None else 0)
