"""Input-pipeline micro-benchmark (GPU box): z-score HBM rate, band-split time per batch, and
the PairLoader's delivery rate from .npy files with and without a concurrent compute load."""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_neuroimage_amd import data as MD  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    dev = torch.device("cuda", 0)
    out = {}
    x = torch.randn(8, 96, 96, 96, device=dev)
    t = timed(lambda: MD.zscore(x))
    out["zscore_8x96^3_ms"] = round(t * 1e3, 4)
    out["zscore_GBps_algorithmic"] = round(x.numel() * 4 * 4 / t / 1e9, 1)   # 3 reads + 1 write
    y = torch.randn(32, 84, 361, device=dev).cumsum(-1)
    t = timed(lambda: MD.fmri_band_split(y, [353] * 32))
    out["band_split_32x84x353_ms"] = round(t * 1e3, 4)
    with tempfile.TemporaryDirectory() as d:
        paths_a, paths_b = [], []
        rng = np.random.default_rng(0)
        for i in range(16):
            for lst, tag in ((paths_a, "a"), (paths_b, "b")):
                p = os.path.join(d, f"{tag}{i}.npy")
                np.save(p, rng.standard_normal((96, 96, 96), dtype=np.float32))
                lst.append(p)
        ld = MD.PairLoader((MD.NpyVolumes(paths_a), MD.NpyVolumes(paths_b)), [0.0] * 16, 4, dev, prefetch=2)
        list(ld)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        for za, zb, lab in ld:
            n += za.shape[0]
        torch.cuda.synchronize()
        out["loader_npy_pairs_per_s"] = round(n / (time.perf_counter() - t0), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
