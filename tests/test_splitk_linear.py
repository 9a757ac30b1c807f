"""The crossmodal encoder's Linear with a split-K weight gradient (functional.SplitKLinear): the
row-chunk rule and the gradients against plain autograd on the CPU (float64), and its bf16
autocast path against F.linear's on the GPU."""
import pytest
import torch

from multimodal_neuroimage_amd.functional import SplitKLinear, _splitk_chunks, splitk_linear


def test_chunk_rule():
    assert _splitk_chunks(6912) == 27     # C4: 1,728 tokens x 4
    assert _splitk_chunks(32768) == 64    # C5: 4,096 tokens x 8
    assert _splitk_chunks(100) == 1       # fewer than 512 rows: no split
    for rows in (6912, 32768, 1000, 777):
        S = _splitk_chunks(rows)
        assert rows % S == 0 and (S == 1 or rows // S >= 256)


def test_gradients_match_autograd():
    g = torch.Generator().manual_seed(0)
    for rows_shape, N, K, bias in (((8, 864), 252, 84, True), ((4, 100), 84, 84, False)):
        x = torch.randn(*rows_shape, K, generator=g, dtype=torch.float64, requires_grad=True)
        w = torch.randn(N, K, generator=g, dtype=torch.float64, requires_grad=True)
        b = torch.randn(N, generator=g, dtype=torch.float64, requires_grad=True) if bias else None
        gy = torch.randn(*rows_shape, N, generator=g, dtype=torch.float64)
        (splitk_linear(x, w, b) * gy).sum().backward()
        got = [t.grad.clone() for t in (x, w, b) if t is not None]
        for t in (x, w, b):
            if t is not None:
                t.grad = None
        (torch.nn.functional.linear(x, w, b) * gy).sum().backward()
        ref = [t.grad for t in (x, w, b) if t is not None]
        for a, r in zip(got, ref):
            assert torch.allclose(a, r, rtol=1e-12, atol=1e-10)


def test_module_keeps_linear_state_dict():
    m = SplitKLinear(12, 84)
    assert isinstance(m, torch.nn.Linear)
    assert set(m.state_dict()) == {"weight", "bias"}


@pytest.mark.gpu
def test_bf16_autocast_matches_f_linear():
    """Under bf16 autocast (C5's head) the split-K Linear casts x and W once in its forward and keeps
    the bf16 copies: output and gradients match F.linear's autocast path (bf16 products, fp32
    parameter gradients), and the gradient dtypes follow the inputs'."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for x_dtype in (torch.float32, torch.bfloat16):
        x = torch.randn(4096, 2, 84, device=dev, generator=g).to(x_dtype).requires_grad_(True)
        w = torch.randn(336, 84, device=dev, generator=g).mul_(0.1).requires_grad_(True)
        b = torch.randn(336, device=dev, generator=g).requires_grad_(True)
        gy = torch.randn(4096, 2, 336, device=dev, generator=g).to(torch.bfloat16)
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
            y = splitk_linear(x, w, b)
        y.backward(gy)
        got = (y.detach().float(), x.grad.float(), w.grad, b.grad)
        assert y.dtype == torch.bfloat16 and x.grad.dtype == x_dtype
        assert w.grad.dtype == torch.float32 and b.grad.dtype == torch.float32
        x.grad = w.grad = b.grad = None
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
            yr = torch.nn.functional.linear(x, w, b)
        yr.backward(gy)
        ref = (yr.detach().float(), x.grad.float(), w.grad, b.grad)
        for a, r in zip(got, ref):
            err = float((a - r).abs().max() / r.abs().max())
            assert err < 2e-2, err


@pytest.mark.gpu
def test_device_reduction_fp32_matches_float64():
    """fp32 on the device (mmni_splitk_reduce for the chunk sum and db): gradients against float64
    autograd, for a split (6,912 rows: S = 27), an unsplit odd-width case and no bias; two runs are
    bitwise equal (fixed-order sums)."""
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(1)
    for rows_shape, N, K, bias in (((1728, 4), 84, 252, True), ((77, 3), 13, 84, True), ((512, 8), 168, 84, False)):
        x = torch.randn(*rows_shape, K, generator=g, dtype=torch.float64)
        w = torch.randn(N, K, generator=g, dtype=torch.float64) * 0.1
        b = torch.randn(N, generator=g, dtype=torch.float64) if bias else None
        gy = torch.randn(*rows_shape, N, generator=g, dtype=torch.float64)
        ref = []
        leaves = [t.clone().requires_grad_(True) if t is not None else None for t in (x, w, b)]
        (torch.nn.functional.linear(*leaves) * gy).sum().backward()
        ref = [t.grad for t in leaves if t is not None]
        runs = []
        for _ in range(2):
            lv = [t.float().to(dev).requires_grad_(True) if t is not None else None for t in (x, w, b)]
            splitk_linear(*lv).backward(gy.float().to(dev))
            runs.append([t.grad.clone() for t in lv if t is not None])
        for a, a2, r in zip(runs[0], runs[1], ref):
            assert torch.equal(a, a2)
            err = float((a.double().cpu() - r).abs().max() / r.abs().max())
            assert err < 1e-5, err


@pytest.mark.gpu
def test_cast_params_bf16_matches_torch_and_tracks_versions():
    """mmni_cast_bf16_multi (70 tensors: two launches) is bit-equal to torch's .to(bfloat16); the
    autocast Linears use a copy only while its parameter's version is unchanged."""
    from multimodal_neuroimage_amd import functional as MF
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    sizes = ([84 * 84, 84, 1, 336 * 84, 13, 672 * 168] * 12)[:70]
    ps = [torch.randn(n, device=dev, generator=g) * 10 for n in sizes]
    MF.cast_params_bf16(ps)
    for p in ps:
        c = MF._autocast_copy(p, torch.bfloat16)
        assert c.shape == p.shape and torch.equal(c, p.to(torch.bfloat16))
        assert c.data_ptr() % 128 == 0
    p = ps[0]
    p.add_(1.0)   # an optimizer step: version bump -> fresh cast
    assert torch.equal(MF._autocast_copy(p, torch.bfloat16), p.to(torch.bfloat16))


@pytest.mark.gpu
def test_relu_epilogue_matches_f_relu():
    """relu=True (the fc1 of the crossmodal layer: ReLU in the GEMM epilogue, mask from the saved
    output in the backward) against F.relu(F.linear(...)): fp32 to 1e-5, bf16 autocast to 2e-2."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    for auto, tol in ((False, 1e-5), (True, 2e-2)):
        x = torch.randn(4096, 2, 84, device=dev, generator=g).requires_grad_(True)
        w = (torch.randn(336, 84, device=dev, generator=g) * 0.1).requires_grad_(True)
        b = torch.randn(336, device=dev, generator=g).requires_grad_(True)
        gy = torch.randn(4096, 2, 336, device=dev, generator=g)
        outs = []
        for fused in (True, False):
            with torch.autocast(device_type="cuda", dtype=torch.bfloat16, enabled=auto):
                y = splitk_linear(x, w, b, relu=True) if fused else torch.relu(torch.nn.functional.linear(x, w, b))
            y.backward(gy.to(y.dtype))
            outs.append((y.detach().float(), x.grad.float(), w.grad.clone(), b.grad.clone()))
            x.grad = w.grad = b.grad = None
        for a, r in zip(*outs):
            err = float((a - r).abs().max() / r.abs().max())
            assert err < tol, (auto, err)
