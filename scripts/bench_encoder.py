"""Micro-benchmark of the crossmodal encoder's row-GEMM kernels (encoder.hip) and of one fused
encoder layer at the C4 / C5 shapes (rows = T * B).  Prints one JSON line per case:
{"case", "us"} (HIP events, median of reps).  Usage: python scripts/bench_encoder.py [reps]"""
import json
import sys

import torch

sys.path.insert(0, ".")
from multimodal_neuroimage_amd import functional as MF  # noqa: E402
from multimodal_neuroimage_amd.modules import crossmodal_transformer as CT  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda")
    torch.manual_seed(0)
    out = []
    for rows, E in ((6912, 84), (6912, 168), (16384, 84)):
        x = torch.randn(rows, E, device=dev)
        g, b = torch.rand(E, device=dev) + 0.5, torch.randn(E, device=dev)
        for K, N, ln, relu in ((E, 3 * E, True, False), (E, E, True, False), (E, 2 * E, True, False),
                               (E, 4 * E, True, True), (E, E, False, False), (4 * E, E, False, False)):
            xi = torch.randn(rows, K, device=dev)
            w = torch.randn(N, K, device=dev) / K ** 0.5
            bias = torch.randn(N, device=dev)
            lnp = (g, b, 1e-5) if ln else None
            us = timeit(lambda: MF.rowgemm(xi, w, bias, ln=lnp, relu=relu, stats=ln), reps)
            flop = 2.0 * rows * K * N
            out.append(dict(case=f"rowgemm rows={rows} K={K} N={N} ln={int(ln)}", us=us, tflops=flop / us / 1e6))
            dy = torch.randn(rows, N, device=dev)
            us = timeit(lambda: MF.rowgemm(dy, w, transpose_w=True), reps)
            out.append(dict(case=f"rowgemm_dx rows={rows} K={N} N={K}", us=us, tflops=flop / us / 1e6))
            mean = xi.mean(-1) if ln else None
            rstd = (1.0 / (xi.var(-1, unbiased=False) + 1e-5).sqrt()) if ln else None
            us = timeit(lambda: MF.rowgemm_dw(xi, dy, N, K, True, ln=lnp, mean=mean, rstd=rstd), reps)
            out.append(dict(case=f"rowgemm_dw rows={rows} K={K} N={N} ln={int(ln)}", us=us, tflops=flop / us / 1e6))
        mean = x.mean(-1)
        rstd = 1.0 / (x.var(-1, unbiased=False) + 1e-5).sqrt()
        dxn = torch.randn(rows, E, device=dev)
        us = timeit(lambda: MF.row_layernorm_bwd(dxn, x, g, mean, rstd, dxn), reps)
        out.append(dict(case=f"row_ln_bwd rows={rows} C={E}", us=us, gbps=4.0 * rows * E * 4 / us / 1e3))
    for E, T, B, cross in ((84, 1728, 4, True), (84, 1728, 4, False), (168, 1728, 4, False)):
        layer = CT.TransformerEncoderLayer(E, num_heads_mult=12, attn_dropout=0.0, relu_dropout=0.0,
                                           res_dropout=0.0, attn_mask=True).to(dev)
        x = torch.randn(T, B, E, device=dev, requires_grad=True)
        xk = torch.randn(T, B, E, device=dev, requires_grad=True) if cross else None
        gy = torch.randn(T, B, E, device=dev)

        def fwd_bwd():
            y = layer(x, xk, xk)
            y.backward(gy)

        us = timeit(fwd_bwd, reps)
        out.append(dict(case=f"encoder_layer fwd+bwd E={E} T={T} B={B} cross={int(cross)}", us=us))
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
