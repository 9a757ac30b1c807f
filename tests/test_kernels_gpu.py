"""HIP kernels (through the C ABI) vs the oracle, on seeded random inputs, 2D and 3D.

Integer maps: bit-exact.  Float kernels (fp32) vs the float64 oracle: max error relative to the
reference's max magnitude <= 1e-4 (the north-star bar is 1e-3 rel in fp32)."""
import numpy as np
import pytest
import torch

from oracle import ops as O
from oracle.index_maps import shifted_window_rows, shift_mask, relative_position_index
from multimodal_neuroimage_amd import functional as MF

pytestmark = pytest.mark.gpu
TOL = 1e-4


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-6))


GEOMS = [
    (2, (1, 12, 18), (1, 6, 6), (0, 3, 3)),
    (2, (1, 84, 84), (1, 6, 6), (0, 3, 3)),
    (2, (1, 6, 6), (1, 3, 3), (0, 1, 1)),
    (1, (12, 12, 12), (6, 6, 6), (3, 3, 3)),
    (2, (6, 12, 18), (3, 6, 6), (1, 3, 3)),
    (1, (12, 12, 12), (6, 6, 6), (0, 0, 0)),
]


@pytest.mark.parametrize("B,spatial,window,shift", GEOMS)
def test_window_maps_bit_exact(device, B, spatial, window, shift):
    g = MF.WindowGeometry(B, spatial, window, shift)
    rows = MF.window_rows(g, device).cpu().numpy().reshape(-1, g.N)
    np.testing.assert_array_equal(rows, shifted_window_rows(B, spatial, window, shift))
    mask = MF.window_mask(g, device).cpu().numpy()
    if any(shift):
        np.testing.assert_array_equal(mask, shift_mask(spatial, window, shift))
    else:
        assert (mask == 0).all()
    idx = MF.relative_index(g, device).cpu().numpy()
    np.testing.assert_array_equal(idx, relative_position_index(window))


def test_window_maps_full_volume_96(device):
    g = MF.WindowGeometry(1, (96, 96, 96), (6, 6, 6), (3, 3, 3))
    rows = MF.window_rows(g, device).cpu().numpy().reshape(-1, g.N)
    np.testing.assert_array_equal(rows, shifted_window_rows(1, (96, 96, 96), (6, 6, 6), (3, 3, 3)))


WATTN = [
    # kind, C, heads, B, spatial, window, shift, cross
    (0, 12, 6, 2, (1, 12, 12), (1, 6, 6), (0, 3, 3), False),
    (0, 12, 6, 2, (1, 12, 12), (1, 6, 6), (0, 0, 0), True),
    (0, 12, 6, 2, (1, 12, 18), (1, 6, 6), (0, 3, 3), True),
    (0, 12, 6, 1, (12, 12, 12), (6, 6, 6), (3, 3, 3), False),
    (0, 12, 6, 1, (12, 12, 12), (6, 6, 6), (3, 3, 3), True),
    (0, 12, 6, 2, (1, 6, 6), (1, 3, 3), (0, 1, 1), False),
    (0, 24, 12, 1, (1, 12, 12), (1, 6, 6), (0, 3, 3), False),
    (0, 6, 3, 2, (1, 12, 12), (1, 6, 6), (0, 3, 3), False),
    (1, 12, 3, 2, (1, 12, 12), (1, 6, 6), (0, 3, 3), False),
    (1, 12, 3, 1, (12, 12, 12), (6, 6, 6), (3, 3, 3), False),
    (1, 24, 6, 2, (1, 6, 6), (1, 6, 6), (0, 0, 0), False),
    (1, 24, 6, 1, (6, 6, 6), (6, 6, 6), (0, 0, 0), False),
    (1, 48, 12, 2, (1, 3, 3), (1, 3, 3), (0, 0, 0), False),
    (1, 48, 12, 2, (3, 3, 3), (3, 3, 3), (0, 0, 0), False),
    (0, 12, 6, 1, (12, 24, 6), (6, 6, 6), (3, 3, 3), False),
    (0, 12, 6, 1, (18, 18, 18), (6, 6, 6), (3, 3, 3), False),   # interior (mask-free) windows
    (0, 12, 6, 2, (18, 12, 6), (6, 6, 6), (3, 3, 3), True),
    # 6^3 kind-0 head pairs (merged quad backward) at 1, 2 and 4 head pairs per window
    (0, 4, 2, 1, (12, 12, 12), (6, 6, 6), (3, 3, 3), False),
    (0, 8, 4, 2, (6, 12, 6), (6, 6, 6), (3, 3, 3), True),
    (0, 16, 8, 1, (12, 6, 12), (6, 6, 6), (0, 0, 0), False),
]


@pytest.mark.parametrize("kind,C,heads,B,spatial,window,shift,cross", WATTN)
def test_window_attention_fwd_bwd_vs_oracle(device, kind, C, heads, B, spatial, window, shift, cross):
    gen = torch.Generator().manual_seed(hash((kind, C, B, spatial, window, shift, cross)) % (2 ** 31))
    geom = MF.WindowGeometry(B, spatial, window, shift)
    rows = geom.tokens
    Tsz = geom.table_rows
    q = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    k = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    v = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    table = torch.randn(Tsz, heads, generator=gen, dtype=torch.float64) * (0.5 if kind == 0 else 4.0)
    tau = (torch.rand(heads, generator=gen, dtype=torch.float64) * 15 + 5) if kind == 1 else None
    gout = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    scale = (C // heads) ** -0.5
    # oracle (float64, CPU, autograd)
    leaves = [t.clone().requires_grad_(True) for t in (q, k, v, table)]
    tau_l = tau.clone().requires_grad_(True) if tau is not None else None
    ref = O.window_attention(*leaves, B, spatial, window, shift, heads, kind, scale=scale, tau=tau_l)
    (ref * gout).sum().backward()
    # HIP kernel (fp32)
    f = lambda t: t.float().to(device).requires_grad_(True)  # noqa: E731
    tab_d = f(table)
    tau_d = f(tau) if tau is not None else None
    if cross:
        qd = f(q)
        kvd = f(torch.cat([k, v], dim=1))
        out = MF.window_attention_cross(qd, kvd, tab_d, geom, heads, kind=kind, scale=scale, tau=tau_d)
    else:
        qkvd = f(torch.cat([q, k, v], dim=1))
        out = MF.window_attention_self(qkvd, tab_d, geom, heads, kind=kind, scale=scale, tau=tau_d)
    (out * gout.float().to(device)).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(out, ref) < TOL
    if cross:
        dq, dk, dv = qd.grad, kvd.grad[:, :C], kvd.grad[:, C:]
    else:
        dq, dk, dv = qkvd.grad[:, :C], qkvd.grad[:, C:2 * C], qkvd.grad[:, 2 * C:]
    assert rel_err(dq, leaves[0].grad) < TOL
    assert rel_err(dk, leaves[1].grad) < TOL
    assert rel_err(dv, leaves[2].grad) < TOL
    assert rel_err(tab_d.grad, leaves[3].grad) < TOL
    if tau is not None:
        assert rel_err(tau_d.grad, tau_l.grad) < TOL


def test_window_attention_large_logits_and_masking(device):
    """Saturated logits (large tau and bias) stay finite and match the oracle: exercises the
    online-max rescale and the -100 mask interplay."""
    B, spatial, window, shift, C, heads = 1, (1, 12, 12), (1, 6, 6), (0, 3, 3), 12, 3
    geom = MF.WindowGeometry(B, spatial, window, shift)
    gen = torch.Generator().manual_seed(7)
    q = torch.randn(geom.tokens, C, generator=gen, dtype=torch.float64)
    k = q + 0.01 * torch.randn(geom.tokens, C, generator=gen, dtype=torch.float64)
    v = torch.randn(geom.tokens, C, generator=gen, dtype=torch.float64)
    table = torch.randn(geom.table_rows, heads, generator=gen, dtype=torch.float64) * 16
    tau = torch.full((heads,), 100.0, dtype=torch.float64)
    ref = O.window_attention(q, k, v, table, B, spatial, window, shift, heads, 1, tau=tau)
    qkv = torch.cat([q, k, v], 1).float().to(device)
    out = MF.window_attention_self(qkv, table.float().to(device), geom, heads, kind=1, tau=tau.float().to(device))
    assert torch.isfinite(out).all()
    assert rel_err(out, ref) < TOL


@pytest.mark.parametrize("cross", [False, True])
def test_window_attention_backward_large_lse_windows(device, cross):
    """6^3 kind-0 windows (the row-broadcast kernels) where some rows have |lse| far above the
    backward's fold bound (kFoldMax = 30 in log2 units) and others below it: both the folded and
    the subtracting loops run in one call, per wave (pass A) and per window (pass B)."""
    B, spatial, window, shift, C, heads = 1, (12, 12, 12), (6, 6, 6), (3, 3, 3), 12, 6
    geom = MF.WindowGeometry(B, spatial, window, shift)
    gen = torch.Generator().manual_seed(11)
    rows = geom.tokens
    q = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    k = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    v = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    q[: rows // 3] *= 40.0          # scores up to ~100 (natural log) in the first third of the volume
    table = torch.randn(geom.table_rows, heads, generator=gen, dtype=torch.float64) * 0.5
    table[:, 0] -= 60.0             # head 0: every score shifted down, lse ~ -60
    gout = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    scale = (C // heads) ** -0.5
    leaves = [t.clone().requires_grad_(True) for t in (q, k, v, table)]
    ref = O.window_attention(*leaves, B, spatial, window, shift, heads, 0, scale=scale)
    (ref * gout).sum().backward()
    f = lambda t: t.float().to(device).requires_grad_(True)  # noqa: E731
    tab_d = f(table)
    if cross:
        qd, kvd = f(q), f(torch.cat([k, v], dim=1))
        out = MF.window_attention_cross(qd, kvd, tab_d, geom, heads, kind=0, scale=scale)
    else:
        qkvd = f(torch.cat([q, k, v], dim=1))
        out = MF.window_attention_self(qkvd, tab_d, geom, heads, kind=0, scale=scale)
    (out * gout.float().to(device)).sum().backward()
    torch.cuda.synchronize()
    if cross:
        dq, dk, dv = qd.grad, kvd.grad[:, :C], kvd.grad[:, C:]
    else:
        dq, dk, dv = qkvd.grad[:, :C], qkvd.grad[:, C:2 * C], qkvd.grad[:, 2 * C:]
    assert rel_err(out, ref) < TOL
    # per head: the scaled third dominates the global maximum, so compare each head's columns
    # and the unscaled rows on their own scale as well
    for h in range(heads):
        cols = slice(2 * h, 2 * h + 2)
        for got, want in ((dq, leaves[0].grad), (dk, leaves[1].grad), (dv, leaves[2].grad)):
            assert rel_err(got[:, cols], want[:, cols]) < TOL
            assert rel_err(got[rows // 3:, cols], want[rows // 3:, cols]) < TOL
        assert rel_err(tab_d.grad[:, h], leaves[3].grad[:, h]) < TOL


MHA = [
    # Tq, Tk, B, heads, hd, causal
    (16, 16, 2, 12, 7, True),
    (368, 368, 2, 12, 7, True),
    (50, 70, 2, 12, 14, True),
    (70, 50, 2, 12, 14, True),
    (64, 64, 3, 4, 16, False),
    (33, 47, 1, 2, 8, False),
    (200, 200, 2, 12, 14, True),
    (130, 130, 1, 6, 4, True),
]


@pytest.mark.parametrize("Tq,Tk,B,heads,hd,causal", MHA)
def test_mha_fwd_bwd_vs_oracle(device, Tq, Tk, B, heads, hd, causal):
    gen = torch.Generator().manual_seed(Tq * 1000 + Tk + hd)
    E = heads * hd
    q, k, v = [torch.randn(T, B, E, generator=gen, dtype=torch.float64) for T in (Tq, Tk, Tk)]
    gout = torch.randn(Tq, B, E, generator=gen, dtype=torch.float64)
    diag = O.causal_diag(Tq, Tk) if causal else 0
    leaves = [t.clone().requires_grad_(True) for t in (q, k, v)]
    ref, ref_w = O.mha_core(*leaves, heads, diag)
    (ref * gout).sum().backward()
    dev = [t.float().to(device).requires_grad_(True) for t in (q, k, v)]
    out, lse = MF.mha_core(*dev, heads, diag)
    (out * gout.float().to(device)).sum().backward()
    w = MF.mha_mean_probs(dev[0], dev[1], lse, heads, diag)
    torch.cuda.synchronize()
    assert rel_err(out, ref) < TOL
    assert rel_err(w, ref_w) < TOL
    for a, b in zip(dev, leaves):
        assert rel_err(a.grad, b.grad) < TOL


@pytest.mark.parametrize("Tq,Tk,causal,p", [(64, 64, True, 0.0), (50, 70, True, 0.0), (64, 64, True, 0.2)])
def test_mha_mean_weights_gradient_vs_oracle(device, Tq, Tk, causal, p):
    """The second return value of MultiheadAttention (head-averaged, dropped weights) back-propagates
    into q and k as the reference's autograd would (multihead_attention.py:123,131-133)."""
    B, heads, hd = 2, 4, 7
    E = heads * hd
    gen = torch.Generator().manual_seed(Tq + Tk)
    q, k, v = [torch.randn(T, B, E, generator=gen, dtype=torch.float64) for T in (Tq, Tk, Tk)]
    gw = torch.randn(B, Tq, Tk, generator=gen, dtype=torch.float64)
    diag = O.causal_diag(Tq, Tk) if causal else 0
    seed = 1234
    dm = MF.mha_dropout_mask(Tq, Tk, B, heads, p, seed, device, diag).double().cpu() if p > 0 else None
    leaves = [t.clone().requires_grad_(True) for t in (q, k, v)]
    _, ref_w = O.mha_core(*leaves, heads, diag, drop_mask=dm)
    (ref_w * gw).sum().backward()
    dev = [t.float().to(device).requires_grad_(True) for t in (q, k, v)]
    _, lse = MF.mha_core(*dev, heads, diag, dropout=p, seed=seed)
    w = MF.mha_mean_probs(dev[0], dev[1], lse, heads, diag, dropout=p, seed=seed)
    (w * gw.float().to(device)).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(w, ref_w) < TOL
    assert rel_err(dev[0].grad, leaves[0].grad) < TOL
    assert rel_err(dev[1].grad, leaves[1].grad) < TOL


MHA_BF16 = [
    # Tq, Tk, B, heads, hd, causal  (C5: bf16 storage, one bf16 product, fp32 accumulation)
    (368, 368, 2, 12, 7, True),
    (200, 200, 2, 12, 14, True),
    (50, 70, 2, 12, 14, True),
    (64, 96, 1, 4, 8, False),
    (130, 130, 1, 6, 4, True),
    (1024, 1024, 1, 12, 7, True),
    (96, 80, 1, 3, 16, True),     # compact images at d = 16 (no padding dims)
    (77, 77, 2, 5, 11, True),     # d = 11: padded to 16, partial last tile
]
TOL_BF16 = 2e-2   # bf16 runs are held to 2e-2 rel against the fp32/fp64 golden


@pytest.mark.parametrize("Tq,Tk,B,heads,hd,causal", MHA_BF16)
def test_mha_bf16_vs_oracle(device, Tq, Tk, B, heads, hd, causal):
    """bf16 q/k/v/dout in, bf16 out/dq/dk/dv: against the fp64 oracle on the same bf16-rounded
    inputs, 2e-2 max-rel; the head-averaged weights (fp32) too."""
    gen = torch.Generator().manual_seed(Tq * 1000 + Tk + hd + 7)
    E = heads * hd
    q, k, v = [torch.randn(T, B, E, generator=gen, dtype=torch.float64).bfloat16().double() for T in (Tq, Tk, Tk)]
    gout = torch.randn(Tq, B, E, generator=gen, dtype=torch.float64).bfloat16().double()
    diag = O.causal_diag(Tq, Tk) if causal else 0
    leaves = [t.clone().requires_grad_(True) for t in (q, k, v)]
    ref, ref_w = O.mha_core(*leaves, heads, diag)
    (ref * gout).sum().backward()
    dev = [t.bfloat16().to(device).requires_grad_(True) for t in (q, k, v)]
    out, lse = MF.mha_core(*dev, heads, diag)
    assert out.dtype == torch.bfloat16
    out.backward(gout.bfloat16().to(device))
    w = MF.mha_mean_probs(dev[0], dev[1], lse, heads, diag)
    torch.cuda.synchronize()
    assert rel_err(out, ref) < TOL_BF16
    assert rel_err(w, ref_w) < TOL_BF16
    for a, b in zip(dev, leaves):
        assert a.grad.dtype == torch.bfloat16
        assert rel_err(a.grad, b.grad) < TOL_BF16


CONV = [
    # B, (D,H,W), Cin, Cout, k, stride, pad, slope
    (2, (16, 16, 16), 1, 12, (8, 8, 8), (8, 8, 8), (0, 0, 0), 1.0),
    (2, (10, 12, 14), 6, 12, (3, 3, 3), (1, 1, 1), (1, 1, 1), 0.2),
    (1, (8, 8, 8), 24, 12, (3, 3, 3), (1, 1, 1), (1, 1, 1), 0.2),
    (2, (9, 9, 9), 3, 1, (3, 3, 3), (1, 1, 1), (1, 1, 1), 1.0),
    (1, (9, 9, 9), 1, 6, (3, 3, 3), (1, 1, 1), (1, 1, 1), 0.2),
    (1, (9, 9, 9), 12, 6, (3, 3, 3), (1, 1, 1), (1, 1, 1), 0.2),
    (1, (9, 9, 9), 6, 3, (3, 3, 3), (1, 1, 1), (1, 1, 1), 0.2),
    (2, (1, 20, 24), 6, 12, (1, 3, 3), (1, 1, 1), (0, 1, 1), 0.2),
    (2, (1, 84, 84), 1, 12, (1, 7, 7), (1, 7, 7), (0, 0, 0), 1.0),
    # fewer (tap, Cin) pairs than output channels: db has columns no dW lane owns
    (1, (12, 12, 12), 1, 12, (2, 2, 2), (2, 2, 2), (0, 0, 0), 1.0),
    (2, (5, 6, 7), 1, 6, (1, 1, 1), (1, 1, 1), (0, 0, 0), 0.2),
]


@pytest.mark.parametrize("B,sp,Cin,Cout,k,stride,pad,slope", CONV)
def test_conv3d_fwd_bwd_vs_oracle(device, B, sp, Cin, Cout, k, stride, pad, slope):
    gen = torch.Generator().manual_seed(Cin * 100 + Cout + sum(sp))
    x = torch.randn(B, *sp, Cin, generator=gen, dtype=torch.float64)
    w = torch.randn(Cout, Cin, *k, generator=gen, dtype=torch.float64) * 0.2
    b = torch.randn(Cout, generator=gen, dtype=torch.float64)
    leaves = [t.clone().requires_grad_(True) for t in (x, w, b)]
    ref = O.conv3d_cl(*leaves, stride, pad, slope)
    gout = torch.randn(ref.shape, generator=gen, dtype=torch.float64)
    (ref * gout).sum().backward()
    dev = [t.float().to(device).requires_grad_(True) for t in (x, w, b)]
    out = MF.conv3d_cl(*dev, stride, pad, slope)
    (out * gout.float().to(device)).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(out, ref) < TOL
    for a, r in zip(dev, leaves):
        assert rel_err(a.grad, r.grad) < TOL


@pytest.mark.parametrize("Cin,Cout,sp,k,pad", [(24, 12, (40, 40, 40), 3, 1), (1, 6, (33, 34, 35), 3, 1),
                                               (12, 6, (24, 24, 24), 3, 1), (1, 12, (96, 96, 96), 8, 0)])
def test_conv3d_weight_grad_is_deterministic(device, Cin, Cout, sp, k, pad):
    """conv dW/db: per-workgroup partial rows reduced in a fixed order (no float atomics), so two
    identical backward passes agree bitwise (the DDP test's per-tensor 1e-4 bar depends on it)."""
    torch.manual_seed(Cin * 31 + Cout)
    x = torch.randn(2, *sp, Cin, device=device)
    w = (torch.randn(Cout, Cin, k, k, k, device=device) * 0.1).requires_grad_(True)
    b = torch.randn(Cout, device=device).requires_grad_(True)
    stride = 1 if k == 3 else k
    g = None
    grads = []
    for _ in range(3):
        w.grad = b.grad = None
        out = MF.conv3d_cl(x, w, b, stride, pad, 0.2 if k == 3 else 1.0)
        if g is None:
            g = torch.randn_like(out)
        (out * g).sum().backward()
        grads.append((w.grad.clone(), b.grad.clone()))
    for gw, gb in grads[1:]:
        assert torch.equal(gw, grads[0][0]) and torch.equal(gb, grads[0][1])


LN = [(1000, 12), (70001, 12), (513, 24), (4099, 48), (300, 96), (108, 48), (7, 24)]


@pytest.mark.parametrize("rows,C", LN)
def test_layernorm_fwd_bwd_vs_torch_fp64(device, rows, C):
    gen = torch.Generator().manual_seed(rows + C)
    x = torch.randn(rows, C, generator=gen, dtype=torch.float64) * 3 + 1
    w = torch.randn(C, generator=gen, dtype=torch.float64)
    b = torch.randn(C, generator=gen, dtype=torch.float64)
    g = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    leaves = [t.clone().requires_grad_(True) for t in (x, w, b)]
    ref = torch.nn.functional.layer_norm(leaves[0], (C,), leaves[1], leaves[2], 1e-5)
    (ref * g).sum().backward()
    ln = torch.nn.LayerNorm(C).to(device)
    with torch.no_grad():
        ln.weight.copy_(w.float())
        ln.bias.copy_(b.float())
    xd = x.float().to(device).requires_grad_(True)
    out = MF.layer_norm(xd, ln)
    (out * g.float().to(device)).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(out, ref) < TOL
    assert rel_err(xd.grad, leaves[0].grad) < TOL
    assert rel_err(ln.weight.grad, leaves[1].grad) < TOL
    assert rel_err(ln.bias.grad, leaves[2].grad) < TOL


LIN = [(5000, 12, 36), (4097, 12, 12), (3001, 12, 48), (3001, 48, 12), (2000, 48, 144), (1000, 24, 72), (777, 96, 48),
       (108, 48, 192), (13, 12, 12), (65, 24, 96), (70001, 12, 36)]


@pytest.mark.parametrize("rows,K,N", LIN)
def test_token_linear_weight_grad_vs_torch_fp64(device, rows, K, N):
    gen = torch.Generator().manual_seed(rows + K * 7 + N)
    x = torch.randn(rows, K, generator=gen, dtype=torch.float64)
    w = torch.randn(N, K, generator=gen, dtype=torch.float64) * 0.3
    b = torch.randn(N, generator=gen, dtype=torch.float64)
    g = torch.randn(rows, N, generator=gen, dtype=torch.float64)
    leaves = [t.clone().requires_grad_(True) for t in (x, w, b)]
    ref = torch.nn.functional.linear(*leaves)
    (ref * g).sum().backward()
    dev = [t.float().to(device).requires_grad_(True) for t in (x, w, b)]
    out = MF.linear(dev[0], dev[1], dev[2])
    (out * g.float().to(device)).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(out, ref) < TOL
    for a, r in zip(dev, leaves):
        assert rel_err(a.grad, r.grad) < TOL


def test_token_linear_weight_grad_is_deterministic(device):
    x = torch.randn(100003, 12, device=device)
    g = torch.randn(100003, 36, device=device)
    w = torch.randn(36, 12, device=device, requires_grad=True)
    grads = []
    for _ in range(3):
        w.grad = None
        (MF.linear(x, w) * g).sum().backward()
        grads.append(w.grad.clone())
    assert all(torch.equal(grads[0], gg) for gg in grads[1:])


TLIN = [(12, 36), (12, 12), (12, 24), (12, 48), (48, 12), (36, 12), (24, 12)]


@pytest.mark.parametrize("K,N", TLIN)
@pytest.mark.parametrize("with_res", [False, True])
def test_token_linear_fwd_dx_vs_torch_fp64(device, K, N, with_res):
    """HIP forward (epi 0, optional fused residual) and input gradient (transposed weight) of a
    token Linear."""
    rows = 70001
    gen = torch.Generator().manual_seed(K * 100 + N)
    x = torch.randn(rows, K, generator=gen, dtype=torch.float64)
    w = torch.randn(N, K, generator=gen, dtype=torch.float64) * 0.3
    b = torch.randn(N, generator=gen, dtype=torch.float64)
    g = torch.randn(rows, N, generator=gen, dtype=torch.float64)
    res = torch.randn(rows, N, generator=gen, dtype=torch.float64)
    leaves = [t.clone().requires_grad_(True) for t in (x, w, b, res)]
    ref = torch.nn.functional.linear(*leaves[:3]) + (leaves[3] if with_res else 0)
    (ref * g).sum().backward()
    dev = [t.float().to(device).requires_grad_(True) for t in (x, w, b, res)]
    out = MF.linear(dev[0], dev[1], dev[2], residual=dev[3] if with_res else None)
    (out * g.float().to(device)).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(out, ref) < TOL
    for a, r in zip(dev[:3], leaves[:3]):
        assert rel_err(a.grad, r.grad) < TOL
    if with_res:
        assert rel_err(dev[3].grad, leaves[3].grad) < TOL


@pytest.mark.parametrize("path", ["mfma", "tokenlinear"])
@pytest.mark.parametrize("rows,with_res", [(50003, True), (16, False), (33, True)])
def test_fused_mlp_gelu_vs_torch_fp64(device, path, rows, with_res):
    """fc1 + exact GELU + fc2 vs the float64 torch MLP, through both HIP paths: the one-kernel MFMA
    MLP (mlp.hip, hidden activation in registers, recomputed in backward) and the token-linear
    path with the GELU fused into the fc1 / fc2-input-gradient epilogues."""
    C, H = 12, 48
    gen = torch.Generator().manual_seed(C + H)
    x = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    w1 = torch.randn(H, C, generator=gen, dtype=torch.float64) * 0.4
    b1 = torch.randn(H, generator=gen, dtype=torch.float64) * 0.5
    w2 = torch.randn(C, H, generator=gen, dtype=torch.float64) * 0.2
    b2 = torch.randn(C, generator=gen, dtype=torch.float64)
    g = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    leaves = [t.clone().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    ref = torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(*leaves[:3])), *leaves[3:])
    (ref * g).sum().backward()
    fc1, fc2 = torch.nn.Linear(C, H).to(device), torch.nn.Linear(H, C).to(device)
    with torch.no_grad():
        fc1.weight.copy_(w1.float()); fc1.bias.copy_(b1.float())
        fc2.weight.copy_(w2.float()); fc2.bias.copy_(b2.float())
    xd = x.float().to(device).requires_grad_(True)
    rd = torch.randn(rows, C, device=device, requires_grad=True) if with_res else None
    if path == "mfma":
        out = MF.mlp(xd, fc1, fc2, torch.nn.GELU(), torch.nn.Dropout(0.0), residual=rd)
    else:
        out = MF._Mlp.apply(xd, fc1.weight, fc1.bias, fc2.weight, fc2.bias, rd)
    (out * g.float().to(device)).sum().backward()
    torch.cuda.synchronize()
    if with_res:
        ref = ref + rd.detach().double().cpu()
        assert rel_err(rd.grad, g) < TOL
    assert rel_err(out, ref) < TOL
    got = [xd.grad, fc1.weight.grad, fc1.bias.grad, fc2.weight.grad, fc2.bias.grad]
    for a, r in zip(got, leaves):
        assert rel_err(a, r.grad) < TOL


def test_fused_mlp_weight_grad_is_deterministic(device):
    """The MFMA MLP's weight gradients reduce per-wave partials in a fixed order: bitwise equal
    across runs."""
    C, H, rows = 12, 48, 200000
    torch.manual_seed(3)
    fc1, fc2 = torch.nn.Linear(C, H).to(device), torch.nn.Linear(H, C).to(device)
    x = torch.randn(rows, C, device=device, requires_grad=True)
    g = torch.randn(rows, C, device=device)
    grads = []
    for _ in range(2):
        for p in (fc1.weight, fc1.bias, fc2.weight, fc2.bias):
            p.grad = None
        MF.mlp(x, fc1, fc2, torch.nn.GELU(), torch.nn.Dropout(0.0)).backward(g)
        grads.append([p.grad.clone() for p in (fc1.weight, fc1.bias, fc2.weight, fc2.bias)])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


@pytest.mark.parametrize("N", [12, 24, 36])
@pytest.mark.parametrize("rows,passthrough", [(50003, True), (16, False), (33, True), (7, False), (50003, 2),
                                              (17, 2)])
def test_ln_linear_vs_torch_fp64(device, N, rows, passthrough):
    """norm1 + qkv/q/kv fused (blockops.hip): LN output never stored, backward recomputes it and
    adds the residual gradient (passthrough) in the same pass; passthrough=2 adds a second one (the
    residual group's skip, mmni_ln_linear_bwd2)."""
    C = 12
    gen = torch.Generator().manual_seed(rows * 3 + N)
    x = torch.randn(rows, C, generator=gen, dtype=torch.float64) * 2 + 0.5
    gm = torch.randn(C, generator=gen, dtype=torch.float64)
    bt = torch.randn(C, generator=gen, dtype=torch.float64)
    w = torch.randn(N, C, generator=gen, dtype=torch.float64) * 0.3
    b = torch.randn(N, generator=gen, dtype=torch.float64)
    g = torch.randn(rows, N, generator=gen, dtype=torch.float64)
    gr = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    gs = torch.randn(rows, C, generator=gen, dtype=torch.float64) * 3.0
    leaves = [t.clone().requires_grad_(True) for t in (x, gm, bt, w, b)]
    F_ = torch.nn.functional
    ref = F_.linear(F_.layer_norm(leaves[0], (C,), leaves[1], leaves[2], 1e-5), leaves[3], leaves[4])
    ((ref * g).sum() + ((leaves[0] * gr).sum() if passthrough else 0)
     + ((leaves[0] * gs).sum() if passthrough == 2 else 0)).backward()
    norm, lin = torch.nn.LayerNorm(C).to(device), torch.nn.Linear(C, N).to(device)
    with torch.no_grad():
        norm.weight.copy_(gm.float()); norm.bias.copy_(bt.float())
        lin.weight.copy_(w.float()); lin.bias.copy_(b.float())
    xd = x.float().to(device).requires_grad_(True)
    assert MF.ln_linear_ok(xd, norm, lin)
    out = MF.ln_linear(xd, norm, lin, passthrough=passthrough)
    if passthrough == 2:
        out, xr, xs = out
        assert xr.data_ptr() == xd.data_ptr() and xs.data_ptr() == xd.data_ptr()
        loss = ((out * g.float().to(device)).sum() + (xr * gr.float().to(device)).sum()
                + (xs * gs.float().to(device)).sum())
    elif passthrough:
        out, xr = out
        assert xr.data_ptr() == xd.data_ptr()
        loss = (out * g.float().to(device)).sum() + (xr * gr.float().to(device)).sum()
    else:
        loss = (out * g.float().to(device)).sum()
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(out, ref) < TOL
    got = [xd.grad, norm.weight.grad, norm.bias.grad, lin.weight.grad, lin.bias.grad]
    for a, r in zip(got, leaves):
        assert rel_err(a, r.grad) < TOL


def test_ln_linear_grads_are_deterministic(device):
    C, N, rows = 12, 36, 200003
    torch.manual_seed(5)
    norm, lin = torch.nn.LayerNorm(C).to(device), torch.nn.Linear(C, N).to(device)
    x = torch.randn(rows, C, device=device, requires_grad=True)
    g = torch.randn(rows, N, device=device)
    grads = []
    for _ in range(2):
        for p in (x, norm.weight, norm.bias, lin.weight, lin.bias):
            p.grad = None
        MF.ln_linear(x, norm, lin).backward(g)
        grads.append([p.grad.clone() for p in (x, norm.weight, norm.bias, lin.weight, lin.bias)])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


@pytest.mark.parametrize("rows", [33, 100003])
@pytest.mark.parametrize("bias", [True, False])
def test_linear_bwd_12x12_fused_vs_torch_fp64(device, rows, bias):
    """attn.proj backward (dx, dW, db in one pass, blockops.hip) through the token Linear."""
    C = 12
    gen = torch.Generator().manual_seed(rows + int(bias))
    x = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    w = torch.randn(C, C, generator=gen, dtype=torch.float64) * 0.3
    b = torch.randn(C, generator=gen, dtype=torch.float64)
    g = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    leaves = [t.clone().requires_grad_(True) for t in (x, w, b)]
    ref = torch.nn.functional.linear(leaves[0], leaves[1], leaves[2] if bias else None)
    (ref * g).sum().backward()
    dev = [t.float().to(device).requires_grad_(True) for t in (x, w, b)]
    out = MF.linear(dev[0], dev[1], dev[2] if bias else None)
    (out * g.float().to(device)).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(out, ref) < TOL
    for a, r in zip(dev[:2], leaves[:2]):
        assert rel_err(a.grad, r.grad) < TOL
    if bias:
        assert rel_err(dev[2].grad, leaves[2].grad) < TOL


@pytest.mark.parametrize("rows,residual_x,skip", [(50003, True, False), (16, False, False), (33, True, False),
                                                   (5, True, False), (50003, True, True), (17, False, True)])
def test_ln_mlp_vs_torch_fp64(device, rows, residual_x, skip):
    """norm2 + fc1 + GELU + fc2 (+ x) (+ the residual group's skip) in one kernel per direction
    (mlp.hip LN prologue; skip = mmni_ln_mlp_skip_fwd, its gradient dy)."""
    C, H = 12, 48
    gen = torch.Generator().manual_seed(rows + 17)
    x = torch.randn(rows, C, generator=gen, dtype=torch.float64) * 1.5 - 0.3
    gm = torch.randn(C, generator=gen, dtype=torch.float64)
    bt = torch.randn(C, generator=gen, dtype=torch.float64)
    w1 = torch.randn(H, C, generator=gen, dtype=torch.float64) * 0.4
    b1 = torch.randn(H, generator=gen, dtype=torch.float64) * 0.5
    w2 = torch.randn(C, H, generator=gen, dtype=torch.float64) * 0.2
    b2 = torch.randn(C, generator=gen, dtype=torch.float64)
    g = torch.randn(rows, C, generator=gen, dtype=torch.float64)
    sk = torch.randn(rows, C, generator=gen, dtype=torch.float64) * 2.0
    leaves = [t.clone().requires_grad_(True) for t in (x, gm, bt, w1, b1, w2, b2, sk)]
    F_ = torch.nn.functional
    xn = F_.layer_norm(leaves[0], (C,), leaves[1], leaves[2], 1e-5)
    ref = F_.linear(F_.gelu(F_.linear(xn, leaves[3], leaves[4])), leaves[5], leaves[6])
    if residual_x:
        ref = ref + leaves[0]
    if skip:
        ref = ref + leaves[7]
    (ref * g).sum().backward()

    class _M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.fc1, self.fc2 = torch.nn.Linear(C, H), torch.nn.Linear(H, C)
            self.act, self.drop = torch.nn.GELU(), torch.nn.Dropout(0.0)

    m, norm = _M().to(device), torch.nn.LayerNorm(C).to(device)
    with torch.no_grad():
        norm.weight.copy_(gm.float()); norm.bias.copy_(bt.float())
        m.fc1.weight.copy_(w1.float()); m.fc1.bias.copy_(b1.float())
        m.fc2.weight.copy_(w2.float()); m.fc2.bias.copy_(b2.float())
    xd = x.float().to(device).requires_grad_(True)
    sd = sk.float().to(device).requires_grad_(True) if skip else None
    assert MF.ln_mlp_ok(xd, norm, m)
    out = MF.ln_mlp(xd, norm, m, residual_x=residual_x, skip=sd)
    (out * g.float().to(device)).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(out, ref) < TOL
    got = [xd.grad, norm.weight.grad, norm.bias.grad, m.fc1.weight.grad, m.fc1.bias.grad, m.fc2.weight.grad,
           m.fc2.bias.grad] + ([sd.grad] if skip else [])
    for a, r in zip(got, leaves):
        assert rel_err(a, r.grad) < TOL


@pytest.mark.parametrize("cross", [False, True])
def test_window_attention_grads_are_deterministic(device, cross):
    """dq/dk/dv and the bias-table gradient (per-wave fp32 tables summed in a fixed order) are
    bitwise identical across runs at a 3D shifted geometry with masked and unmasked windows."""
    geom = MF.WindowGeometry(2, (24, 24, 18), (6, 6, 6), (3, 3, 3))
    torch.manual_seed(11)
    C, heads = 12, 6
    q = torch.randn(geom.tokens, C, device=device)
    kv = torch.randn(geom.tokens, 2 * C, device=device)
    table = (torch.randn(geom.table_rows, heads, device=device) * 0.3).requires_grad_(True)
    g = torch.randn(geom.tokens, C, device=device)
    res = []
    for _ in range(3):
        table.grad = None
        if cross:
            qd, kvd = q.clone().requires_grad_(True), kv.clone().requires_grad_(True)
            out = MF.window_attention_cross(qd, kvd, table, geom, heads)
            (out * g).sum().backward()
            res.append((qd.grad, kvd.grad, table.grad.clone()))
        else:
            qkv = torch.cat([q, kv], 1).requires_grad_(True)
            out = MF.window_attention_self(qkv, table, geom, heads)
            (out * g).sum().backward()
            res.append((qkv.grad, table.grad.clone()))
    for r in res[1:]:
        for a, b in zip(r, res[0]):
            assert torch.equal(a, b)


@pytest.mark.parametrize("C,heads,spatial,window", [(12, 3, (24, 24, 18), (6, 6, 6)), (12, 6, (16, 16, 16), (4, 4, 4)),
                                                    (48, 12, (3, 3, 3), (3, 3, 3)), (24, 6, (12, 12, 12), (6, 6, 6))])
def test_swin_v2_attention_grads_are_deterministic(device, C, heads, spatial, window):
    """Kind 1 (Swin-V2 cosine attention): dq/dk/dv, the bias-table gradient (64-bit fixed point) and
    dtau (logit_scale: per-block partial rows + a fixed-order column sum, no float atomics) are
    bitwise identical across runs, on the packed (head_dim 2) and generic (head_dim 4) kernels."""
    shift = tuple(w // 2 if s > w else 0 for s, w in zip(spatial, window))
    geom = MF.WindowGeometry(2, spatial, window, shift)
    torch.manual_seed(13 + C)
    qkv0 = torch.randn(geom.tokens, 3 * C, device=device)
    table = (torch.randn(geom.table_rows, heads, device=device) * 4).requires_grad_(True)
    tau = (torch.rand(heads, device=device) * 15 + 5).requires_grad_(True)
    g = torch.randn(geom.tokens, C, device=device)
    res = []
    for _ in range(3):
        table.grad = tau.grad = None
        qkv = qkv0.clone().requires_grad_(True)
        out = MF.window_attention_self(qkv, table, geom, heads, kind=1, tau=tau)
        (out * g).sum().backward()
        res.append((qkv.grad, table.grad.clone(), tau.grad.clone()))
    for r in res[1:]:
        for a, b in zip(r, res[0]):
            assert torch.equal(a, b)


MHA_DROP = [
    # Tq, Tk, B, heads, hd, causal, p
    (64, 64, 2, 4, 7, True, 0.1),
    (130, 100, 1, 3, 14, True, 0.3),
    (50, 70, 2, 12, 8, False, 0.5),
    (368, 368, 2, 12, 7, True, 0.1),
]


@pytest.mark.parametrize("Tq,Tk,B,heads,hd,causal,p", MHA_DROP)
def test_mha_dropout_vs_oracle_with_the_kernel_mask(device, Tq, Tk, B, heads, hd, causal, p):
    """Attention dropout (multihead_attention.py:123): the forward, the head-mean weights and all
    three gradients equal the fp64 oracle run with the very mask the kernels regenerate from the
    seed (exported by mmni_mha_dropout_mask), so forward and backward apply one mask."""
    gen = torch.Generator().manual_seed(Tq + 7 * Tk + hd)
    E = heads * hd
    q, k, v = [torch.randn(T, B, E, generator=gen, dtype=torch.float64) for T in (Tq, Tk, Tk)]
    gout = torch.randn(Tq, B, E, generator=gen, dtype=torch.float64)
    diag = O.causal_diag(Tq, Tk) if causal else 0
    seed = 1234 + Tq
    mask = MF.mha_dropout_mask(Tq, Tk, B, heads, p, seed, device)
    leaves = [t.clone().requires_grad_(True) for t in (q, k, v)]
    ref, ref_w = O.mha_core(*leaves, heads, diag, drop_mask=mask.double().cpu())
    (ref * gout).sum().backward()
    dev = [t.float().to(device).requires_grad_(True) for t in (q, k, v)]
    out, lse = MF.mha_core(*dev, heads, diag, dropout=p, seed=seed)
    (out * gout.float().to(device)).sum().backward()
    w = MF.mha_mean_probs(dev[0], dev[1], lse, heads, diag, dropout=p, seed=seed)
    torch.cuda.synchronize()
    assert rel_err(out, ref) < TOL
    assert rel_err(w, ref_w) < TOL
    for a, b in zip(dev, leaves):
        assert rel_err(a.grad, b.grad) < TOL


def test_mha_dropout_mask_statistics(device):
    """Keep rate 1 - p and unbiased multipliers (E[mask] = 1) within 5 sigma; masks differ across
    seeds, heads and rows; p = 0 is the no-dropout path bit for bit."""
    B, H, T, p = 2, 12, 368, 0.1
    m = MF.mha_dropout_mask(T, T, B, H, p, 99, device)
    n = m.numel()
    keep = float((m > 0).float().mean())
    sigma = (p * (1 - p) / n) ** 0.5
    assert abs(keep - (1 - p)) < 5 * sigma
    assert abs(float(m.double().mean()) - 1.0) < 5 * sigma / (1 - p)
    vals = torch.unique(m).tolist()
    assert len(vals) == 2 and vals[0] == 0.0 and abs(vals[1] - 1 / (1 - p)) < 1e-6
    m2 = MF.mha_dropout_mask(T, T, B, H, p, 100, device)
    assert not torch.equal(m, m2)
    assert not torch.equal(m[0, 0], m[0, 1]) and not torch.equal(m[0, 0, 0], m[0, 0, 1])
    # per-column keep rates stay near 1 - p (no column bias from the per-row hash)
    col = (m > 0).float().mean(dim=(0, 1, 2))
    assert float((col - (1 - p)).abs().max()) < 6 * (p * (1 - p) / (B * H * T)) ** 0.5
    torch.manual_seed(0)
    q, k, v = (torch.randn(T, B, H * 7, device=device) for _ in range(3))
    o0, _ = MF.mha_core(q, k, v, H, 1)
    o1, _ = MF.mha_core(q, k, v, H, 1, dropout=0.0, seed=5)
    assert torch.equal(o0, o1)


def test_crossmodal_model_trains_with_reference_dropout_defaults(device):
    """Transformer_Net_Cross_Attention with the reference's default dropouts (--attn_dropout 0.1
    etc., main.py:176-195) runs a training step (train mode, dropout in the kernels) and its eval
    forward equals the dropout-free path."""
    from multimodal_neuroimage_amd import model as M
    kw = dict(fine_tune_task="binary_classification", intermediate_vec=84, num_heads_mult=12, nlevels=2,
              attn_dropout=0.1, attn_dropout_u=0.1, relu_dropout=0.1, res_dropout=0.1, embed_dropout=0.1,
              out_dropout=0.0, attn_mask=True, sequence_length=368, feature_map_gen="convolution_ul+l",
              feature_map_size="same", mixing="U2L_and_L2U", concat_method="concat", fmri_type="divided_frequency")
    torch.manual_seed(0)
    m = M.Transformer_Net_Cross_Attention(**kw).to(device)
    xl, xu = torch.randn(2, 368, 84, device=device), torch.randn(2, 368, 84, device=device)
    m.train()
    out = m(xl, xu)["binary_classification"]
    loss = torch.nn.functional.binary_cross_entropy_with_logits(out, torch.ones_like(out))
    loss.backward()
    assert torch.isfinite(loss)
    assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)
    m.eval()
    with torch.no_grad():
        a = m(xl, xu)["binary_classification"]
        for mod in m.modules():
            if hasattr(mod, "attn_dropout"):
                mod.attn_dropout = 0.0
        b = m(xl, xu)["binary_classification"]
    assert torch.equal(a, b)


@pytest.mark.parametrize("window,heads", [((6, 6, 6), 3), ((6, 6, 6), 24), ((3, 3, 3), 12), ((7, 7), 6), ((2, 2, 2), 32)])
def test_cpb_table_vs_torch_fp64_and_deterministic(device, window, heads):
    """16 * sigmoid(cpb_mlp(relative_coords_table)) (swin_v2_module.py:158-162) on mmni_cpb_fwd /
    _bwd against the same MLP in torch float64: table 1e-5, dW1 / db1 / dW2 1e-5 max-rel, and bitwise
    repeatable gradients."""
    from multimodal_neuroimage_amd.modules.swin_v2_module import _coords_table
    nd = len(window)
    coords = _coords_table(window, (0,) * nd).to(device)
    g = torch.Generator().manual_seed(heads + nd)
    w1 = (torch.randn(512, nd, generator=g) * 0.5).to(device)
    b1 = (torch.randn(512, generator=g) * 0.5).to(device)
    w2 = (torch.randn(heads, 512, generator=g) * 0.05).to(device)
    dout = torch.randn(coords.reshape(-1, nd).shape[0], heads, generator=g).to(device)
    leaves = [t.double().clone().requires_grad_(True) for t in (w1, b1, w2)]
    c64 = coords.reshape(-1, nd).double()
    ref = 16 * torch.sigmoid(torch.relu(c64 @ leaves[0].t() + leaves[1]) @ leaves[2].t())
    ref.backward(dout.double())
    runs = []
    for _ in range(2):
        ps = [t.clone().requires_grad_(True) for t in (w1, b1, w2)]
        out = MF.cpb_table(coords, *ps)
        out.backward(dout)
        torch.cuda.synchronize()
        runs.append((out.detach(), [p.grad for p in ps]))
    out, grads = runs[0]
    assert rel_err(out, ref) < 1e-5
    for got, leaf in zip(grads, leaves):
        assert rel_err(got, leaf.grad) < 1e-5
    assert all(torch.equal(a, b) for a, b in zip(runs[0][1], runs[1][1]))
