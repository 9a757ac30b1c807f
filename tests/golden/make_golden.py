"""Generate the golden fixtures in tests/golden/*.npz by running the REFERENCE's own Python.

Run in the build container only (the reference never travels to the GPU box):
    python tests/golden/make_golden.py
Every fixture holds inputs (or their seeds), outputs and gradients of one reference call at
the reference's own 2D shapes; parameters come from tests/golden/recipe.py.  The reference
code itself is imported, never copied (tests/golden/refload.py).
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import recipe  # noqa: E402
import refload  # noqa: E402

torch.set_num_threads(8)
torch.manual_seed(0)
R = refload.load()
SF, V2, MH, CM, PE, M = R["swinfusion"], R["swin_v2"], R["mha"], R["crossmodal"], R["pe"], R["model"]


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def npf(x):
    return x.detach().cpu().numpy().astype(np.float32)


def save(name, d):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **d)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB, {len(d)} arrays)")


def grads_of(module, prefix, out):
    for k, p in sorted(module.named_parameters()):
        if p.grad is not None:
            out[prefix + "d." + k] = npf(p.grad)


def grad_stats(module, prefix, out, full_below=4096):
    """Per-parameter gradient sum / sum of squares (+ full grad for small tensors)."""
    names, sums, sqs = [], [], []
    for k, p in sorted(module.named_parameters()):
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        names.append(k)
        sums.append(float(g.double().sum()))
        sqs.append(float((g.double() ** 2).sum()))
        if p.numel() <= full_below:
            out[prefix + "d." + k] = npf(g)
    out[prefix + "gnames"] = np.array(names)
    out[prefix + "gsum"] = np.array(sums)
    out[prefix + "gsq"] = np.array(sqs)


# ------------------------------------------------------------------------------------------
# 1. integer maps (rows of roll+partition, masks, relative index) + Swin-V2 coords table
# ------------------------------------------------------------------------------------------
def make_maps():
    d = {}
    for (H, W) in [(12, 12), (12, 18), (84, 84), (6, 6)]:
        ws = 3 if (H, W) == (6, 6) else 6
        shifts = (0, ws // 2)
        for s in shifts:
            grid = torch.arange(2 * H * W, dtype=torch.float64).reshape(2, H, W, 1)
            xs = torch.roll(grid, shifts=(-s, -s), dims=(1, 2)) if s else grid
            win = SF.window_partition_fusion(xs, ws).reshape(-1, ws * ws)
            d[f"rows_{H}x{W}_ws{ws}_s{s}"] = win.numpy().astype(np.int64)
        blk = SF.SwinTransformerBlock_fusion(dim=12, input_resolution=(H, W), num_heads=6, window_size=ws,
                                             shift_size=ws // 2)
        d[f"mask_{H}x{W}_ws{ws}_s{ws // 2}"] = blk.attn_mask.numpy()
    blk = V2.SwinTransformerBlock(dim=12, input_resolution=(12, 12), num_heads_swin=3, window_size=6, shift_size=3)
    d["v2mask_12x12_ws6_s3"] = blk.attn_mask.numpy()
    for ws in (6, 3, 4):
        wa = SF.WindowAttention_fusion(12, (ws, ws), 6)
        d[f"relidx_ws{ws}"] = wa.relative_position_index.numpy().astype(np.int64)
        wv = V2.WindowAttention(12, (ws, ws), 3)
        d[f"coords_ws{ws}"] = wv.relative_coords_table.numpy()
    save("maps.npz", d)


# ------------------------------------------------------------------------------------------
# 2. window attention (fusion, cross, Swin-V2) in the token formulation: roll + partition +
#    attention + reverse, exactly as the blocks use them
# ------------------------------------------------------------------------------------------
def shifted_call(attn, x, y, ws, s, mask, partition, reverse):
    B, H, W, C = x.shape
    xs = torch.roll(x, shifts=(-s, -s), dims=(1, 2)) if s else x
    xw = partition(xs, ws).view(-1, ws * ws, C)
    if y is not None:
        ys = torch.roll(y, shifts=(-s, -s), dims=(1, 2)) if s else y
        yw = partition(ys, ws).view(-1, ws * ws, C)
        ow = attn(xw, yw, mask=mask)
    else:
        ow = attn(xw, mask=mask)
    o = reverse(ow.view(-1, ws, ws, C), ws, H, W)
    return torch.roll(o, shifts=(s, s), dims=(1, 2)) if s else o


def make_wattn():
    d = {}
    cases = [
        # name, kind, B, H, W, C, heads, ws, shift, store_inputs
        ("f12s0", "fusion", 2, 12, 12, 12, 6, 6, 0, True),
        ("f12s3", "fusion", 2, 12, 12, 12, 6, 6, 3, True),
        ("f84s3", "fusion", 1, 84, 84, 12, 6, 6, 3, False),
        ("c12s3", "cross", 2, 12, 12, 12, 6, 6, 3, True),
        ("c84s3", "cross", 1, 84, 84, 12, 6, 6, 3, False),
        ("v12s0", "v2", 2, 12, 12, 12, 3, 6, 0, True),
        ("v12s3", "v2", 2, 12, 12, 12, 3, 6, 3, True),
        ("v6s0", "v2", 2, 6, 6, 24, 6, 6, 0, True),
        ("v3s0", "v2", 2, 3, 3, 48, 12, 3, 0, True),
    ]
    meta = {}
    for name, kind, B, H, W, C, heads, ws, s, store in cases:
        seed = 1000 + len(meta)
        if kind == "fusion":
            attn = SF.WindowAttention_fusion(C, (ws, ws), heads)
            part, rev = SF.window_partition_fusion, SF.window_reverse_fusion
        elif kind == "cross":
            attn = SF.Cross_WindowAttention(C, (ws, ws), heads)
            part, rev = SF.window_partition_fusion, SF.window_reverse_fusion
        else:
            attn = V2.WindowAttention(C, (ws, ws), heads)
            part, rev = V2.window_partition, V2.window_reverse
        recipe.fill_params(attn)
        x = t(recipe.randn(seed, (B, H, W, C))).requires_grad_(True)
        y = t(recipe.randn(seed + 1, (B, H, W, C))).requires_grad_(True) if kind == "cross" else None
        g = t(recipe.randn(seed + 2, (B, H, W, C)))
        mask = None
        if s:
            blk = SF.SwinTransformerBlock_fusion(dim=C, input_resolution=(H, W), num_heads=heads,
                                                 window_size=ws, shift_size=s)
            mask = blk.calculate_mask((H, W))
        out = shifted_call(attn, x, y, ws, s, mask, part, rev)
        (out * g).sum().backward()
        p = name + "."
        if store:
            d[p + "x"] = npf(x)
            if y is not None:
                d[p + "y"] = npf(y)
            d[p + "g"] = npf(g)
        d[p + "out"] = npf(out)
        d[p + "dx"] = npf(x.grad)
        if y is not None:
            d[p + "dy"] = npf(y.grad)
        grads_of(attn, p, d)
        meta[name] = dict(kind=kind, B=B, H=H, W=W, C=C, heads=heads, ws=ws, shift=s, seed=seed,
                          params=recipe.param_signature(attn))
    d["meta"] = np.array(json.dumps(meta))
    save("wattn.npz", d)


# ------------------------------------------------------------------------------------------
# 3. blocks / merging / patch-embed
# ------------------------------------------------------------------------------------------
def make_blocks():
    d, meta = {}, {}

    def run(name, mod, inputs, call, seed):
        recipe.fill_params(mod)
        xs = [t(recipe.randn(seed + i, shp)).requires_grad_(True) for i, shp in enumerate(inputs)]
        outs = call(mod, *xs)
        outs = outs if isinstance(outs, tuple) else (outs,)
        loss = 0
        for j, o in enumerate(outs):
            g = t(recipe.randn(seed + 100 + j, tuple(o.shape)))
            loss = loss + (o * g).sum()
            d[f"{name}.out{j}"] = npf(o)
        loss.backward()
        for i, x in enumerate(xs):
            d[f"{name}.dx{i}"] = npf(x.grad)
        grads_of(mod, name + ".", d)
        meta[name] = dict(inputs=[list(s) for s in inputs], seed=seed, params=recipe.param_signature(mod))

    blk = SF.SwinTransformerBlock_fusion(dim=12, input_resolution=(12, 12), num_heads=6, window_size=6, shift_size=3)
    run("bf12", blk, [(2, 144, 12)], lambda m, x: m(x, (12, 12)), 2000)
    blk = SF.SwinTransformerBlock_fusion(dim=12, input_resolution=(12, 12), num_heads=6, window_size=6, shift_size=3)
    run("bf84", blk, [(1, 84 * 84, 12)], lambda m, x: m(x, (84, 84)), 2100)
    blk = SF.SwinTransformerBlock_fusion(dim=12, input_resolution=(12, 12), num_heads=6, window_size=6, shift_size=0)
    run("bf12s0", blk, [(2, 144, 12)], lambda m, x: m(x, (12, 12)), 2150)
    blk = SF.Cross_SwinTransformerBlock(dim=12, input_resolution=(12, 12), num_heads=6, window_size=6, shift_size=3)
    run("bc12", blk, [(2, 144, 12), (2, 144, 12)], lambda m, x, y: m(x, y, (12, 12)), 2200)
    blk = V2.SwinTransformerBlock(dim=12, input_resolution=(12, 12), num_heads_swin=3, window_size=6, shift_size=3)
    run("bv12", blk, [(2, 144, 12)], lambda m, x: m(x), 2300)
    blk = V2.SwinTransformerBlock(dim=48, input_resolution=(3, 3), num_heads_swin=12, window_size=6, shift_size=3)
    run("bv3", blk, [(2, 9, 48)], lambda m, x: m(x), 2350)
    pm = V2.PatchMerging((12, 12), 12)
    run("pmv2", pm, [(2, 144, 12)], lambda m, x: m(x), 2400)
    pm = SF.PatchMerging_fusion((12, 12), 12)
    run("pmf", pm, [(2, 144, 12)], lambda m, x: m(x), 2500)
    pe = V2.PatchEmbed(img_size_w=84, img_size_h=84, patch_size=7, in_chans=1, embed_dim=12,
                       norm_layer=torch.nn.LayerNorm)
    run("pe", pe, [(2, 1, 84, 84)], lambda m, x: m(x), 2600)
    bl = SF.BasicLayer_fusion(dim=12, input_resolution=(12, 12), depth=2, num_heads=6, window_size=6)
    run("blf", bl, [(2, 144, 12)], lambda m, x: m(x, (12, 12)), 2700)
    crstb = SF.CRSTB(dim=12, input_resolution=(12, 12), depth=2, num_heads=6, window_size=6, img_size=12,
                     patch_size=1)
    run("crstb", crstb, [(2, 144, 12), (2, 144, 12)], lambda m, x, y: m(x, y, (12, 12)), 2800)
    d["meta"] = np.array(json.dumps(meta))
    save("blocks.npz", d)


# ------------------------------------------------------------------------------------------
# 4. crossmodal transformer
# ------------------------------------------------------------------------------------------
def make_mha():
    d, meta = {}, {}
    for T, store in ((16, True), (368, False)):
        name = f"mha{T}"
        seed = 3000 + T
        mha = MH.MultiheadAttention(84, 12)
        recipe.fill_params(mha)
        q = t(recipe.randn(seed, (T, 2, 84))).requires_grad_(True)
        k = t(recipe.randn(seed + 1, (T, 2, 84))).requires_grad_(True)
        v = t(recipe.randn(seed + 2, (T, 2, 84))).requires_grad_(True)
        mask = CM.buffered_future_mask(q, k)
        out, w = mha(q, k, v, attn_mask=mask)
        g = t(recipe.randn(seed + 3, tuple(out.shape)))
        gw = t(recipe.randn(seed + 4, tuple(w.shape)))
        ((out * g).sum() + (w * gw).sum()).backward()
        d[name + ".out"] = npf(out)
        d[name + ".w"] = npf(w) if store else npf(w[:, :32, :32])
        for nm, x in (("dq", q), ("dk", k), ("dv", v)):
            d[f"{name}.{nm}"] = npf(x.grad)
        grads_of(mha, name + ".", d)
        meta[name] = dict(T=T, seed=seed, params=recipe.param_signature(mha))
    # self attention path (qkv_same) without mask, E=168 (trans_mem shape)
    mha = MH.MultiheadAttention(168, 12)
    recipe.fill_params(mha)
    x = t(recipe.randn(3500, (24, 2, 168))).requires_grad_(True)
    out, w = mha(x, x, x)
    g = t(recipe.randn(3501, tuple(out.shape)))
    (out * g).sum().backward()
    d["mhaself.out"] = npf(out)
    d["mhaself.w"] = npf(w)
    d["mhaself.dx"] = npf(x.grad)
    grads_of(mha, "mhaself.", d)
    meta["mhaself"] = dict(T=24, seed=3500, params=recipe.param_signature(mha))
    # encoder: cross with causal mask and padding rows (zero feature 0 -> position 0)
    enc = CM.TransformerEncoder(84, 12, 2, attn_dropout=0.0, relu_dropout=0.0, res_dropout=0.0,
                                embed_dropout=0.0, attn_mask=True)
    recipe.fill_params(enc)
    xa = recipe.randn(3600, (20, 2, 84))
    xb = recipe.randn(3601, (20, 2, 84))
    xa[17:, 1, 0] = 0.0      # padding rows (position 0) in sample 1
    xb[0, 0, 0] = 0.0
    xa_t, xb_t = t(xa).requires_grad_(True), t(xb).requires_grad_(True)
    out = enc(xa_t, xb_t, xb_t)
    g = t(recipe.randn(3602, tuple(out.shape)))
    (out * g).sum().backward()
    d["enc.xa"], d["enc.xb"], d["enc.out"] = xa, xb, npf(out)
    d["enc.dxa"], d["enc.dxb"] = npf(xa_t.grad), npf(xb_t.grad)
    grads_of(enc, "enc.", d)
    meta["enc"] = dict(params=recipe.param_signature(enc))
    # positional embedding
    pe = PE.SinusoidalPositionalEmbedding(84)
    tok = recipe.randn(3700, (2, 30))
    tok[0, 5:9] = 0.0
    d["pe.tok"] = tok
    d["pe.out"] = npf(pe(t(tok)))
    d["meta"] = np.array(json.dumps(meta))
    save("mha.npz", d)


# ------------------------------------------------------------------------------------------
# 5. whole models at reference defaults (eval mode, dropout 0)
# ------------------------------------------------------------------------------------------
def make_models():
    d, meta = {}, {}
    bce = torch.nn.BCEWithLogitsLoss()
    # SwinFusion (step 6, dataset struct)
    kw = refload.default_kwargs("6", ["--dataset_name", "struct"])
    m = M.SwinFusion(**kw).eval()
    recipe.fill_params(m)
    A = t(recipe.randn(4000, (2, 84, 84))).requires_grad_(True)
    Bv = t(recipe.randn(4001, (2, 84, 84))).requires_grad_(True)
    out = m(A, Bv)["binary_classification"]
    lab = torch.tensor([[1.0], [0.0]])
    bce(out, lab).backward()
    d["swinfusion.logits"] = npf(out)
    d["swinfusion.dA"], d["swinfusion.dB"] = npf(A.grad), npf(Bv.grad)
    grad_stats(m, "swinfusion.", d)
    meta["swinfusion"] = dict(kwargs={k: v for k, v in kw.items() if isinstance(v, (int, float, str, bool))},
                              params=recipe.param_signature(m))
    # SwinTransformerV2 (step 3, sMRI)
    kw = refload.default_kwargs("3", ["--dataset_name", "sMRI"])
    m = M.SwinTransformerV2(**kw).eval()
    recipe.fill_params(m)
    X = t(recipe.randn(4100, (4, 84, 84))).requires_grad_(True)
    out = m(X)[kw["fine_tune_task"]]
    bce(out, torch.tensor([[1.0], [0.0], [1.0], [0.0]])).backward()
    d["swinv2.logits"] = npf(out)
    d["swinv2.dX"] = npf(X.grad)
    grad_stats(m, "swinv2.", d)
    meta["swinv2"] = dict(kwargs={k: v for k, v in kw.items() if isinstance(v, (int, float, str, bool))},
                          params=recipe.param_signature(m))
    # crossmodal trunk (step 2, lowfreqBERT cross attention), dropouts 0
    kw = refload.default_kwargs("2", ["--attn_dropout", "0", "--relu_dropout", "0", "--embed_dropout", "0",
                                      "--res_dropout", "0", "--attn_dropout_u", "0"])
    m = M.Transformer_Net_Cross_Attention(**kw).eval()
    recipe.fill_params(m)
    xl = t(recipe.randn(4200, (2, 368, 84))).requires_grad_(True)
    xu = t(recipe.randn(4201, (2, 368, 84))).requires_grad_(True)
    res = m(xl, xu)
    out = res[kw["fine_tune_task"]]
    bce(out, torch.tensor([[1.0], [0.0]])).backward()
    d["crossmodal.logits"] = npf(out)
    d["crossmodal.emb"] = npf(res["embedding_per_ROIs"])
    d["crossmodal.dxl"], d["crossmodal.dxu"] = npf(xl.grad), npf(xu.grad)
    grad_stats(m, "crossmodal.", d, full_below=512)
    meta["crossmodal"] = dict(kwargs={k: v for k, v in kw.items() if isinstance(v, (int, float, str, bool))},
                              params=recipe.param_signature(m))
    d["meta"] = np.array(json.dumps(meta))
    save("models.npz", d)


if __name__ == "__main__":
    which = sys.argv[1:] or ["maps", "wattn", "blocks", "mha", "models"]
    for w in which:
        globals()["make_" + w]()
