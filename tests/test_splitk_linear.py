"""The crossmodal encoder's Linear with a split-K weight gradient (functional.SplitKLinear): the
row-chunk rule and the gradients against plain autograd, on the CPU (float64)."""
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
