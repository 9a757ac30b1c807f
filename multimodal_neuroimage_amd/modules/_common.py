"""Helpers shared by the window-attention modules (host side, torch).

The buffers built here (relative_position_index, attn_mask, relative_coords_table) exist only so
state_dicts keep the reference's keys and shapes; the HIP kernels compute the
index and the mask analytically and never read them.
"""
import collections
import math
import weakref

import torch
import torch.nn as nn

from ..functional import WindowGeometry


def to_ntuple(x, n):
    if isinstance(x, (list, tuple)):
        return tuple(x)
    return (x,) * n


def to_2tuple(x):
    return to_ntuple(x, 2)


def trunc_normal_(t, std=1.0, mean=0.0, a=-2.0, b=2.0):
    return nn.init.trunc_normal_(t, mean=mean, std=std, a=a, b=b)


class DropPath(nn.Module):
    """Per-sample stochastic depth (timm.models.layers.DropPath semantics)."""

    def __init__(self, drop_prob=0.0):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        if self.drop_prob == 0.0 or not self.training:
            return x
        keep = 1.0 - self.drop_prob
        mask = x.new_empty((x.shape[0],) + (1,) * (x.ndim - 1)).bernoulli_(keep)
        return x * mask / keep


def inactive(m):
    """True when module m (DropPath / Dropout / Identity / None) is the identity right now, so a
    residual add can be fused into the producing kernel's epilogue."""
    if m is None or isinstance(m, nn.Identity):
        return True
    if isinstance(m, DropPath):
        return m.drop_prob == 0.0 or not m.training
    if isinstance(m, nn.Dropout):
        return m.p == 0.0 or not m.training
    return False


def relative_index_buffer(window):
    """relative_position_index of a window (any number of axes), int64 (N, N)."""
    axes = [torch.arange(w) for w in window]
    coords = torch.stack(torch.meshgrid(*axes, indexing="ij")).flatten(1)
    rel = coords[:, :, None] - coords[:, None, :]
    idx = torch.zeros(rel.shape[1:], dtype=torch.long)
    for a, w in enumerate(window):
        idx = idx * (2 * w - 1) + rel[a] + (w - 1)
    return idx


def shift_label_windows(resolution, window, shift, device=None):
    """(nW, N) region label of every window token of one sample: the labelled image of
    calculate_mask (swinfusion_module.py:317-329) partitioned into windows; axes with shift 0
    carry a single region (3D lift rule)."""
    nd = len(resolution)
    label = torch.zeros(resolution, dtype=torch.long, device=device)
    for a, (L, w, s) in enumerate(zip(resolution, window, shift)):
        lab = torch.zeros(L, dtype=torch.long, device=device)
        if s > 0:
            lab[L - w:L - s] = 1
            lab[L - s:] = 2
        view = [1] * nd
        view[a] = L
        label = label * 3 + lab.view(view)
    split = []
    for L, w in zip(resolution, window):
        split += [L // w, w]
    perm = [2 * a for a in range(nd)] + [2 * a + 1 for a in range(nd)]
    return label.view(split).permute(perm).reshape(-1, math.prod(window))


def shift_mask_buffer(resolution, window, shift):
    """(nW, N, N) {0, -100} mask of one sample for a shifted-window layer of `resolution`."""
    win = shift_label_windows(resolution, window, shift)
    diff = win.unsqueeze(1) - win.unsqueeze(2)
    return torch.zeros(diff.shape).masked_fill(diff != 0, -100.0)


def _factorizations(n, k):
    if k == 1:
        yield (n,)
        return
    for a in range(1, n + 1):
        if n % a == 0:
            for rest in _factorizations(n // a, k - 1):
                yield (a,) + rest


_MASK_GEOMETRY = collections.OrderedDict()   # (id, version, shape, window, device) -> (weakref, result)
_MASK_GEOMETRY_MAX = 64


def _mask_geometry_search(m, window):
    nW, N, _ = m.shape
    if N != math.prod(window):
        return None
    if not bool(m.any()):
        # an all-zero mask is an unshifted layer (no pair masked): nW windows along the first
        # non-trivial axis, shift 0
        a = next((i for i, w in enumerate(window) if w > 1), 0)
        return tuple(w * (nW if i == a else 1) for i, w in enumerate(window)), tuple(0 for _ in window)
    for counts in _factorizations(nW, len(window)):
        if any(c > 1 and w == 1 for c, w in zip(counts, window)):
            continue
        res = tuple(c * w for c, w in zip(counts, window))
        for s in range(1, max(window)):
            shift = tuple(s if w > s else 0 for w in window)
            lab = shift_label_windows(res, window, shift, device=m.device)
            ok = True
            for w0 in range(0, nW, 256):
                lb = lab[w0:w0 + 256]
                cand = (lb.unsqueeze(1) != lb.unsqueeze(2)).to(m.dtype) * -100.0
                if not torch.equal(cand, m[w0:w0 + 256]):
                    ok = False
                    break
            if ok:
                return res, shift
    return None


def geometry_for_mask(mask, window):
    """(resolution, shift) of a shifted-window layer whose calculate_mask equals `mask` (nW, N, N),
    or None.  An all-zero mask is shift 0.  The attention of a window depends only on its own tokens
    and mask[w mod nW], so any geometry reproducing the mask gives the reference's result.

    Cached per live mask tensor: the key holds the tensor's identity and in-place version, and the
    entry a weak reference to it, so a freed mask whose address (or id) a new tensor reuses is never
    taken for it; the cache keeps at most _MASK_GEOMETRY_MAX entries (least recently used out)."""
    window = tuple(int(w) for w in window)
    key = (id(mask), mask._version, tuple(mask.shape), window, str(mask.device))
    hit = _MASK_GEOMETRY.get(key)
    if hit is not None and hit[0]() is mask:
        _MASK_GEOMETRY.move_to_end(key)
        return hit[1]
    found = _mask_geometry_search(mask.detach(), window)
    _MASK_GEOMETRY[key] = (weakref.ref(mask), found)
    while len(_MASK_GEOMETRY) > _MASK_GEOMETRY_MAX:
        _MASK_GEOMETRY.popitem(last=False)
    return found


def attend_masked_windows(fn, windows, mask, window):
    """Run a fused window-attention `fn(rows..., geom) -> rows` on PRE-PARTITIONED shifted windows
    (num_windows*B, N, C) with the reference's explicit shift mask (WindowAttention*.forward(x, mask),
    swinfusion_module.py:114,213; swin_v2_module.py:138).  The windows are put back into their
    shifted frame, rolled back by the shift the mask encodes, attended by the kernel (which
    re-applies the roll and derives the same mask analytically) and re-partitioned."""
    from .swinfusion_module import window_partition_fusion, window_reverse_fusion
    geo = geometry_for_mask(mask, window)
    if geo is None:
        raise NotImplementedError("window attention: the mask is not a shifted-window calculate_mask of any "
                                  "geometry; the fused kernel derives masks analytically and takes no arbitrary ones")
    res, shift = geo
    nd = len(res)
    B_, N, C = windows[0].shape
    B = B_ // mask.shape[0]
    dims = tuple(range(1, nd + 1))
    rows = []
    for t in windows:
        xs = window_reverse_fusion(t.reshape(B_, *window, t.shape[-1]), window, *res)
        rows.append(torch.roll(xs, shifts=shift, dims=dims).reshape(-1, t.shape[-1]))
    out = fn(*rows, geometry(B, res, window, shift)).view(B, *res, C)
    out = torch.roll(out, shifts=tuple(-s for s in shift), dims=dims)
    return window_partition_fusion(out, window).reshape(B_, N, C)


def clamp_window(input_resolution, window_size, shift_size):
    """Window/shift clamp of the Swin blocks (swin_v2_module.py:226-231,
    swinfusion_module.py:294-298): a layer no larger than its window attends globally."""
    if min(input_resolution) <= window_size:
        return min(input_resolution), 0
    return window_size, shift_size


def geometry(batch, x_size, window_size, shift_size):
    """WindowGeometry of a block applied at spatial size x_size (2D or 3D)."""
    x_size = tuple(int(s) for s in x_size)
    nd = len(x_size)
    win = to_ntuple(window_size, nd)
    sh = to_ntuple(shift_size, nd)
    return WindowGeometry.make(batch, x_size, win if nd == 3 else (1,) + tuple(win),
                               sh if nd == 3 else (0,) + tuple(sh))


def patch_merge_gather(x, resolution):
    """Concatenate the 2^k neighbours of a token grid (B, prod(res), C) -> (B, prod(res/2), 2^k C).

    2D order is the reference's (h fastest): (0,0),(1,0),(0,1),(1,1) (swin_v2_module.py:354-358).
    The 3D lift extends it with the first axis fastest: offsets (dz,dy,dx) enumerated with dz
    varying fastest, then dy, then dx (so D = 1 reduces to the 2D order).
    """
    B, L, C = x.shape
    nd = len(resolution)
    x = x.view(B, *resolution, C)
    parts = []
    if nd == 2:
        for dx in (0, 1):
            for dy in (0, 1):
                parts.append(x[:, dy::2, dx::2, :])
    else:
        for dx in (0, 1):
            for dy in (0, 1):
                for dz in (0, 1):
                    parts.append(x[:, dz::2, dy::2, dx::2, :])
    y = torch.cat(parts, -1)
    return y.view(B, -1, (2 ** nd) * C)
