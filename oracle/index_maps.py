"""numpy restatement of the integer maps on the window-attention path (oracle, tests only).

All maps are dimension-generic over spatial axes (2D reference shapes, 3D lift).
"""
import numpy as np


def shifted_window_rows(batch, spatial, window, shift):
    """Gather map of roll(-shift) followed by window partition.

    Restates torch.roll(x, -s, dims) + window_partition (modules/swin_v2_module.py:35-46,278;
    modules/swinfusion_module.py:33-45,351): returns rows[w, t] = flat token row
    ((b*D + z)*H + y)*W + x read by window-local token t of window w, windows in row-major
    order of (b, window coords), tokens row-major inside a window.
    """
    spatial = tuple(spatial)
    window = tuple(window)
    shift = tuple(shift)
    nd = len(spatial)
    grid = np.arange(batch * int(np.prod(spatial)), dtype=np.int64).reshape((batch,) + spatial)
    # roll by -shift on every spatial axis: element at new position p came from p + shift
    rolled = np.roll(grid, tuple(-s for s in shift), axis=tuple(range(1, nd + 1)))
    # (b, n0, w0, n1, w1, ...) -> (b, n0, n1, ..., w0, w1, ...)
    split = [batch]
    for L, ws in zip(spatial, window):
        split += [L // ws, ws]
    blocks = rolled.reshape(split)
    order = [0] + [1 + 2 * a for a in range(nd)] + [2 + 2 * a for a in range(nd)]
    win = blocks.transpose(order).reshape(-1, int(np.prod(window)))
    return win.astype(np.int64)


def shift_labels(spatial, window, shift):
    """Per-window region labels of one sample, (nW, N) int64: the labelled image of
    calculate_mask (modules/swinfusion_module.py:317-338; modules/swin_v2_module.py:244-262)
    partitioned into windows.  Regions of the shifted frame are the slices (0,-ws), (-ws,-s),
    (-s,None) per axis (the cartesian product of per-axis labels); axes with shift 0 contribute
    a single region (the 3D lift rule of SURVEY Q19)."""
    spatial = tuple(spatial)
    nd = len(spatial)
    labels = np.zeros(spatial, dtype=np.int64)
    for a, (L, ws, s) in enumerate(zip(spatial, window, shift)):
        lab = np.zeros(L, dtype=np.int64)
        if s > 0:
            lab[L - ws:L - s] = 1
            lab[L - s:] = 2
        shape = [1] * nd
        shape[a] = L
        labels = labels * 3 + lab.reshape(shape)
    split = []
    for L, ws in zip(spatial, window):
        split += [L // ws, ws]
    order = [2 * a for a in range(nd)] + [2 * a + 1 for a in range(nd)]
    return labels.reshape(split).transpose(order).reshape(-1, int(np.prod(window)))


def shift_mask(spatial, window, shift):
    """Shifted-window attention mask of one sample, values {0, -100}: token pairs of a window
    with different region labels (shift_labels) get -100 (calculate_mask,
    modules/swinfusion_module.py:330-338)."""
    win = shift_labels(spatial, window, shift)
    diff = win[:, None, :] - win[:, :, None]
    return np.where(diff != 0, -100.0, 0.0).astype(np.float32)


def relative_position_index(window):
    """relative_position_index (modules/swinfusion_module.py:93-103, swin_v2_module.py:114-124),
    generalised to any number of axes: idx[i, j] = sum_a (c_a(i) - c_a(j) + ws_a - 1) * prod_{a'>a}(2 ws_a' - 1)."""
    window = tuple(window)
    coords = np.stack(np.meshgrid(*[np.arange(w) for w in window], indexing="ij")).reshape(len(window), -1)
    rel = coords[:, :, None] - coords[:, None, :]
    idx = np.zeros(rel.shape[1:], dtype=np.int64)
    for a, ws in enumerate(window):
        idx = idx * (2 * ws - 1) + (rel[a] + ws - 1)
    return idx


def relative_coords_table(window, pretrained_window=None):
    """Swin-V2 log-spaced relative coordinate table (modules/swin_v2_module.py:96-111):
    r = 8 * d / (ws - 1) per axis, then sign(r) * log2(|r| + 1) / log2(8); shape
    (1, 2ws_0-1, ..., len(window)) float32."""
    window = tuple(window)
    norm = tuple(pretrained_window) if pretrained_window and pretrained_window[0] > 0 else window
    axes = [np.arange(-(w - 1), w, dtype=np.float32) for w in window]
    grid = np.stack(np.meshgrid(*axes, indexing="ij"), axis=-1)
    for a, w in enumerate(norm):
        grid[..., a] = grid[..., a] / np.float32(w - 1)
    grid = grid * np.float32(8)
    tab = np.sign(grid) * np.log2(np.abs(grid) + np.float32(1.0)) / np.float32(np.log2(8))
    return tab[None].astype(np.float32)
