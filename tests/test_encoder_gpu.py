"""The crossmodal encoder's HIP row-GEMM kernels (encoder.hip, ABI v6) against torch float64, and
the fused encoder layer against the module's per-op path (crossmodal_transformer.py:133-165).

Tolerances: 1e-5 max-rel for the fp32 kernels (exact-fp32 MFMA products, fp32 accumulation over
K <= 672 or over the token rows), bitwise repeatability for every weight / LayerNorm gradient
(fixed-order reductions), 1e-4 for a whole layer against the per-op path."""
import pytest
import torch

from multimodal_neuroimage_amd import functional as MF
from multimodal_neuroimage_amd.modules import crossmodal_transformer as CT

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.detach().double(), b.detach().double().to(a.device)
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


SHAPES = [  # rows, K, N
    (6912, 84, 84), (6912, 84, 168), (6912, 84, 336), (6912, 336, 84), (4096, 168, 504), (4096, 672, 168),
    (1000, 84, 252), (37, 84, 84), (130, 20, 13), (257, 83, 37), (64, 3, 130)]


@pytest.mark.parametrize("rows,K,N", SHAPES)
@pytest.mark.parametrize("ln,relu,res", [(False, False, False), (True, False, False), (True, True, False),
                                         (False, False, True)])
def test_rowgemm_vs_fp64(device, rows, K, N, ln, relu, res):
    if ln and K > 176:
        # the LayerNorm prologue holds a row in registers: K <= 176, else a loud refusal
        with pytest.raises(RuntimeError, match="LayerNorm prologue"):
            MF.rowgemm(torch.zeros(rows, K, device=device), torch.zeros(N, K, device=device),
                       ln=(torch.ones(K, device=device), torch.zeros(K, device=device), 1e-5), stats=True)
        return
    g = torch.Generator(device=device).manual_seed(rows + 7 * K + N)
    x = torch.randn(rows, K, device=device, generator=g) * 2 + 0.5
    w = torch.randn(N, K, device=device, generator=g) / K ** 0.5
    b = torch.randn(N, device=device, generator=g)
    gamma = torch.rand(K, device=device, generator=g) + 0.5
    beta = torch.randn(K, device=device, generator=g)
    r = torch.randn(rows, N, device=device, generator=g)
    xd = x.double()
    if ln:
        xd = torch.nn.functional.layer_norm(xd, (K,), gamma.double(), beta.double(), 1e-5)
    ref = xd @ w.double().t() + b.double()
    if relu:
        ref = ref.clamp_min(0)
    if res:
        ref = ref + r.double()
    out = MF.rowgemm(x, w, b, ln=(gamma, beta, 1e-5) if ln else None, relu=relu, res=r if res else None,
                     stats=ln)
    y = out[0] if ln else out
    torch.cuda.synchronize()
    assert rel_err(y, ref) < 1e-5
    if ln:
        mean = x.double().mean(-1)
        rstd = 1.0 / (x.double().var(-1, unbiased=False) + 1e-5).sqrt()
        assert rel_err(out[1], mean) < 1e-5 and rel_err(out[2], rstd) < 1e-5


@pytest.mark.parametrize("rows,K,N", [(6912, 84, 336), (4096, 168, 672), (333, 84, 84)])
def test_rowgemm_transposed_weight_and_relu_mask(device, rows, K, N):
    """dX = (dY W) * (a > 0): the input-gradient use (weight (N, K) read as its transpose)."""
    g = torch.Generator(device=device).manual_seed(rows + N)
    dy = torch.randn(rows, N, device=device, generator=g)
    w = torch.randn(N, K, device=device, generator=g) / N ** 0.5
    a = torch.randn(rows, K, device=device, generator=g).clamp_min(0)
    ref = (dy.double() @ w.double()) * (a > 0).double()
    y = MF.rowgemm(dy, w, transpose_w=True, aux=a)
    torch.cuda.synchronize()
    assert rel_err(y, ref) < 1e-5


@pytest.mark.parametrize("rows,K,N,ln", [(6912, 84, 84, True), (6912, 336, 84, False), (4096, 168, 504, True),
                                         (4096, 672, 168, False), (77, 84, 252, True)])
def test_rowgemm_dw_vs_fp64_and_deterministic(device, rows, K, N, ln):
    g = torch.Generator(device=device).manual_seed(rows * 3 + K + N)
    x = torch.randn(rows, K, device=device, generator=g)
    dy = torch.randn(rows, N, device=device, generator=g)
    gamma = torch.rand(K, device=device, generator=g) + 0.5
    beta = torch.randn(K, device=device, generator=g)
    mean = x.mean(-1)
    rstd = 1.0 / (x.var(-1, unbiased=False) + 1e-5).sqrt()
    xd = x.double()
    if ln:
        xd = (xd - mean.double()[:, None]) * rstd.double()[:, None] * gamma.double() + beta.double()
    ref_w = dy.double().t() @ xd
    ref_b = dy.double().sum(0)
    outs = [MF.rowgemm_dw(x, dy, N, K, True, ln=(gamma, beta, 1e-5) if ln else None, mean=mean, rstd=rstd)
            for _ in range(3)]
    torch.cuda.synchronize()
    assert rel_err(outs[0][0], ref_w) < 1e-5 and rel_err(outs[0][1], ref_b) < 1e-5
    for dw, db in outs[1:]:
        assert torch.equal(dw, outs[0][0]) and torch.equal(db, outs[0][1])


@pytest.mark.parametrize("rows,C,res", [(6912, 84, False), (4096, 168, True), (50, 84, True)])
def test_row_layernorm_bwd_vs_fp64(device, rows, C, res):
    g = torch.Generator(device=device).manual_seed(rows + C)
    x = (torch.randn(rows, C, device=device, generator=g) * 3 + 1).double()
    gamma = (torch.rand(C, device=device, generator=g) + 0.5).double()
    beta = torch.randn(C, device=device, generator=g).double()
    gy = torch.randn(rows, C, device=device, generator=g).double()
    dres = torch.randn(rows, C, device=device, generator=g).double()
    leaves = [t.clone().requires_grad_(True) for t in (x, gamma, beta)]
    y = torch.nn.functional.layer_norm(leaves[0], (C,), leaves[1], leaves[2], 1e-5)
    (y * gy).sum().backward()
    xf = x.float()
    mean = xf.mean(-1)
    rstd = 1.0 / (xf.var(-1, unbiased=False) + 1e-5).sqrt()
    outs = [MF.row_layernorm_bwd(gy.float(), xf, gamma.float(), mean, rstd, dres.float() if res else None)
            for _ in range(2)]
    torch.cuda.synchronize()
    dx, dg, db = outs[0]
    want = leaves[0].grad + (dres if res else 0)
    assert rel_err(dx, want) < 1e-5
    assert rel_err(dg, leaves[1].grad) < 1e-5 and rel_err(db, leaves[2].grad) < 1e-5
    assert all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))


@pytest.mark.parametrize("E,T,B,cross", [(84, 1728, 4, True), (168, 1728, 4, False), (84, 368, 2, True),
                                         (84, 100, 3, False)])
def test_fused_encoder_layer_matches_per_op_path(device, E, T, B, cross):
    """TransformerEncoderLayer on the HIP row-GEMM path (encoder_layer_rows) against the same layer
    on the per-op path (torch LayerNorm / GEMMs + the fused attention core), forward and every
    gradient, causal mask, fp32."""
    torch.manual_seed(E + T + B)
    layer = CT.TransformerEncoderLayer(E, num_heads_mult=12, attn_dropout=0.0, relu_dropout=0.0, res_dropout=0.0,
                                       attn_mask=True).to(device)
    with torch.no_grad():
        for m in layer.layer_norms:
            m.weight.uniform_(0.5, 1.5)
            m.bias.normal_()
        layer.self_attn.in_proj_bias.normal_(0, 0.1)
        layer.fc1.bias.normal_(0, 0.1)
    x = torch.randn(T, B, E, device=device)
    xk = torch.randn(T + 3, B, E, device=device) if cross else None
    gy = torch.randn(T, B, E, device=device)
    res = []
    for fused in (True, False):
        layer.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        ki = xk.clone().requires_grad_(True) if cross else None
        if fused:
            assert layer._fused_ok(xi, ki, ki)
            out = layer(xi, ki, ki)
        else:
            orig = CT.TransformerEncoderLayer._fused_ok
            CT.TransformerEncoderLayer._fused_ok = lambda self, *a: False
            try:
                out = layer(xi, ki, ki)
            finally:
                CT.TransformerEncoderLayer._fused_ok = orig
        (out * gy).sum().backward()
        torch.cuda.synchronize()
        res.append((out.detach(), xi.grad, ki.grad if cross else None,
                    {k: p.grad.clone() for k, p in layer.named_parameters()}))
    (o1, dx1, dk1, p1), (o2, dx2, dk2, p2) = res
    errs = dict(out=rel_err(o1, o2), dx=rel_err(dx1, dx2))
    if cross:
        errs["dxk"] = rel_err(dk1, dk2)
    for k in p1:
        errs[k] = rel_err(p1[k], p2[k])
    worst = max(errs.items(), key=lambda kv: kv[1])
    print(f"fused encoder layer E={E} T={T} B={B} cross={cross}: worst {worst[0]} {worst[1]:.2e}")
    assert worst[1] < 1e-4, errs


@pytest.mark.parametrize("rows,C,dtype", [(6912, 84, torch.float32), (32768, 168, torch.float32), (333, 84, torch.bfloat16),
                                          (50, 200, torch.float32)])
def test_row_layernorm_module_vs_fp64(device, rows, C, dtype):
    """functional.layer_norm at the crossmodal widths (mmni_row_layernorm_fwd / _bwd): output and
    every gradient against torch float64; fp32 output from bf16 input, as torch's autocast does."""
    ln = torch.nn.LayerNorm(C).to(device)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.normal_()
    g = torch.Generator(device=device).manual_seed(rows + C)
    x = (torch.randn(rows, C, device=device, generator=g) * 2 + 1).to(dtype).requires_grad_(True)
    gy = torch.randn(rows, C, device=device, generator=g)
    y = MF.layer_norm(x, ln)
    assert y.dtype == torch.float32
    y.backward(gy)
    xd = x.detach().double().requires_grad_(True)
    wd, bd = ln.weight.detach().double().requires_grad_(True), ln.bias.detach().double().requires_grad_(True)
    yd = torch.nn.functional.layer_norm(xd, (C,), wd, bd, ln.eps)
    yd.backward(gy.double())
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_err(y, yd) < 1e-5
    assert rel_err(x.grad.float(), xd.grad) < tol
    assert rel_err(ln.weight.grad, wd.grad) < 1e-5 and rel_err(ln.bias.grad, bd.grad) < 1e-5


@pytest.mark.parametrize("rows,C", [(4096 * 8, 84), (777, 168), (50, 200)])
def test_row_layernorm_bf16_output_vs_fp64(device, rows, C):
    """out_dtype=bf16 (the bf16 head's pre-norms, mmni_row_layernorm_fwd_t / _bwd_t): the output is the
    fp32 LayerNorm rounded once to bf16 (bit-equal to rounding the fp32 kernel's output), and a bf16
    output gradient gives the input / affine gradients of float64 autograd fed the same bf16 values."""
    ln = torch.nn.LayerNorm(C).to(device)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.normal_()
    g = torch.Generator(device=device).manual_seed(rows * 3 + C)
    x = (torch.randn(rows, C, device=device, generator=g) * 2 + 1).requires_grad_(True)
    gy = torch.randn(rows, C, device=device, generator=g).to(torch.bfloat16)
    y = MF.layer_norm(x, ln, torch.bfloat16)
    assert y.dtype == torch.bfloat16
    with torch.no_grad():
        y32 = MF.layer_norm(x, ln)
    assert torch.equal(y, y32.to(torch.bfloat16))
    y.backward(gy)
    xd = x.detach().double().requires_grad_(True)
    wd, bd = ln.weight.detach().double().requires_grad_(True), ln.bias.detach().double().requires_grad_(True)
    torch.nn.functional.layer_norm(xd, (C,), wd, bd, ln.eps).backward(gy.double())
    assert x.grad.dtype == torch.float32
    assert rel_err(x.grad, xd.grad) < 1e-5
    assert rel_err(ln.weight.grad, wd.grad) < 1e-5 and rel_err(ln.bias.grad, bd.grad) < 1e-5
