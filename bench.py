"""Throughput benchmark of the MI355X hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c4] [--batch B] [--size S]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Workload (default): two-modality SwinFusion in the build's 3D lift on synthetic
z-scored 96^3 sMRI+fMRI volume pairs, 4 pairs per GPU (weak scaling), fp32.  One step =
forward + backward + (RCCL gradient all-reduce, overlapped by DDP for N > 1) + AdamW, with the
inputs already resident in HBM.  Rank 0 prints ONE JSON line.

Extra fields:
  roofline      dominant HIP kernel over the timed region (HIP events on its launch stream);
                algorithmic FLOPs/bytes per launch as SURVEY §8d counts them; traffic from the
                committed rocprofv3 PMC summary when present (profiles/*pmc*.json), else null.
  cpu_baseline  the oracle's functional torch-CPU restatement of the same model, timed on this
                box's host cores on a bounded sample (trunk on one 36^3 pair fwd+bwd, scaled by the
                voxel ratio to 96^3 pairs/s); rank 0 at N = 1 only.
"""
import argparse
import glob
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "volume-pairs/sec fwd+bwd, 96³ 2-modality batch, 1/2/4/8 MI355X"
FP32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 vector = FP32 matrix dense peak
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=["c3", "c4"],
                    help="c3: SwinFusion 3D (default, the BASELINE metric's config); c4: SwinCrossmodal3D composite")
    ap.add_argument("--batch", type=int, default=4, help="volume pairs per GPU")
    ap.add_argument("--size", type=int, default=96, help="volume side (voxels)")
    ap.add_argument("--checkpoint", action="store_true", help="recompute blocks in backward (memory)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole step (fwd + bwd + AdamW) in one hipGraph and replay it (N = 1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-size", type=int, default=36)
    return ap.parse_args()


def model_kwargs(size):
    return dict(fine_tune_task="binary_classification", size_of_model="large", swin_embed_dim=12, drop_rate=0.0,
                attn_drop_rate=0.0, mlp_ratio=4.0, drop_path_rate=0.0, intermediate_vec=size, patch_size=8,
                window_size=6, no_init_weights=True, volume_size=size)


def c4_kwargs(size):
    """SURVEY §8d C4 composite: Swin-V2 stage 1 per modality (12^3 tokens at 96^3 / patch 8), 2 cross
    blocks, Linear(12 -> 84), the crossmodal head with 12 layers / 12 heads / causal mask on
    1,728-token sequences; dropouts 0 (the reference's default attention dropout 0.1 is RNG-only)."""
    return dict(fine_tune_task="binary_classification", volume_size=size, patch_size=8, swin_embed_dim=12,
                window_size=6, swin_heads=3, cross_heads=6, swin_depth=2, mlp_ratio=4.0, intermediate_vec=84,
                num_heads_mult=12, nlevels=12, attn_dropout=0.0, attn_dropout_u=0.0, relu_dropout=0.0,
                res_dropout=0.0, embed_dropout=0.0, out_dropout=0.0, attn_mask=True, mixing="U2L_and_L2U",
                concat_method="concat", fmri_type="divided_frequency")


def synthetic_pairs(n, size, device, seed):
    """z-scored N(0,1) volumes (datasets.py:416 zscore over the whole volume) + Bernoulli labels."""
    g = torch.Generator(device=device).manual_seed(seed)
    A = torch.randn(n, size, size, size, device=device, generator=g)
    B = torch.randn(n, size, size, size, device=device, generator=g)
    A = (A - A.mean(dim=(1, 2, 3), keepdim=True)) / A.std(dim=(1, 2, 3), keepdim=True)
    B = (B - B.mean(dim=(1, 2, 3), keepdim=True)) / B.std(dim=(1, 2, 3), keepdim=True)
    y = torch.bernoulli(torch.full((n, 1), 0.5, device=device), generator=g)
    return A, B, y


def latest_pmc(kernel_name):
    """HBM bytes per launch of `kernel_name` (bench naming, e.g. wattn_bwd_k0_C12_N216) from the
    newest committed PMC summary (scripts/summarize_profile.py), or (None, None)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        for k, v in d.get("kernels", {}).items():
            if kernel_name.startswith(k + "_") and v.get("hbm_bytes_per_launch") is not None:
                return v["hbm_bytes_per_launch"], os.path.basename(f)
    return None, None


def cpu_baseline_c4(size):
    """Oracle composite (fp32 CPU) fwd+bwd on one pair at the full size: the crossmodal head's cost
    does not scale with a smaller volume in a simple way, so no sampling."""
    from multimodal_neuroimage_amd import model as M
    from oracle import model as OM   # cpu_baseline leg: the oracle is the timed CPU port
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    m = M.SwinCrossmodal3D(**c4_kwargs(size))
    p = OM.params_of(m, torch.float32)
    g = torch.Generator().manual_seed(0)
    A = torch.randn(1, size, size, size, generator=g)
    B = torch.randn(1, size, size, size, generator=g)
    cfg = dict(patch=8, window_size=6, swin_heads=3, cross_heads=6, depth=2, layers=12, heads=12)
    t0 = time.perf_counter()
    out = OM.swin_crossmodal_logits(p, A, B, cfg)
    torch.nn.functional.binary_cross_entropy_with_logits(out, torch.ones_like(out)).backward()
    t = time.perf_counter() - t0
    return dict(value=round(1.0 / t, 6), unit="volume-pairs/s", cores=threads, kind="port",
                sample=f"oracle SwinCrossmodal3D fwd+bwd, 1 pair at {size}^3 ({t:.1f} s); fp32")


def cpu_baseline(size, sample):
    """Oracle (functional torch-CPU restatement) SwinFusion-3D fwd+bwd, bounded sample: the trunk
    (conv + 60 window-attention blocks, cost linear in voxels) on one sample^3 pair scaled by the
    voxel ratio, plus the Swin-V2 head at the full size^3 input (its cost does not scale)."""
    from multimodal_neuroimage_amd import model as M
    from oracle import model as OM   # cpu_baseline leg: the oracle is the timed CPU port
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    m = M.SwinFusion(**model_kwargs(size))
    p = OM.params_of(m, torch.float32)
    cfg = dict(window_size=6, Ex_depths=[6, 6], Fusion_depths=[2, 2, 2], Re_depths=[6, 6], heads=6,
               resolution=(size // 8,) * 3, head_patch=8)
    g = torch.Generator().manual_seed(0)
    A = torch.randn(1, sample, sample, sample, generator=g)
    B = torch.randn(1, sample, sample, sample, generator=g)
    t0 = time.perf_counter()
    OM.swinfusion_trunk(p, A, B, cfg).sum().backward()
    t_trunk = time.perf_counter() - t0
    z = torch.randn(1, size, size, size, generator=g)
    t0 = time.perf_counter()
    out = OM.swin_v2_logits(p, "swin.", z, 8, 6)
    torch.nn.functional.binary_cross_entropy_with_logits(out, torch.ones_like(out)).backward()
    t_head = time.perf_counter() - t0
    scale = (size / sample) ** 3
    t_pair = t_trunk * scale + t_head
    return dict(value=round(1.0 / t_pair, 6), unit="volume-pairs/s", cores=threads, kind="port",
                sample=f"oracle SwinFusion-3D fwd+bwd: trunk on 1 pair at {sample}^3 ({t_trunk:.1f} s, scaled "
                       f"x{scale:.0f} by voxel count) + Swin-V2 head at {size}^3 ({t_head:.1f} s); fp32")


def main():
    args = parse()
    from multimodal_neuroimage_amd import distributed as D
    env = D.init_from_env()            # one process per GPU, RCCL ("nccl") when WORLD_SIZE > 1
    world, rank, device = env.world, env.rank, env.device
    torch.manual_seed(55555555)

    from multimodal_neuroimage_amd import model as M
    from multimodal_neuroimage_amd.functional import KernelTimer

    if args.config == "c4":
        model = D.wrap_ddp(M.SwinCrossmodal3D(use_checkpoint=args.checkpoint, **c4_kwargs(args.size)).to(device), env)
    else:
        kw = model_kwargs(args.size)
        model = D.wrap_ddp(M.SwinFusion(use_checkpoint=args.checkpoint, **kw).to(device), env)
    graph = args.graph and world == 1
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=1e-5, capturable=graph)
    A, B, y = synthetic_pairs(args.batch, args.size, device, seed=1234 + rank)
    lossf = torch.nn.BCEWithLogitsLoss()

    def eager_step():
        opt.zero_grad(set_to_none=True)
        out = model(A, B)["binary_classification"]
        loss = lossf(out, y)
        loss.backward()
        opt.step()
        return loss

    step = eager_step
    if graph:
        # whole-step capture (torch.cuda.graphs whole-network recipe): warm up on a side stream,
        # capture fwd + bwd + AdamW once, then each step is one hipGraphLaunch.  The HIP kernels
        # launch on torch's current stream, so they are captured like torch's own.
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(args.warmup, 2)):
                eager_step()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(g):
            static_loss = lossf(model(A, B)["binary_classification"], y)
            static_loss.backward()
            opt.step()

        def step():
            g.replay()
            return static_loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    D.barrier(env)
    torch.cuda.synchronize()
    KernelTimer.reset()
    KernelTimer.enabled = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    D.barrier(env)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    KernelTimer.enabled = False
    elapsed = D.max_over_ranks(elapsed, env)
    if graph:
        # per-kernel HIP-event timings cannot be taken inside a graph replay: one eager step
        # after the timed region supplies them (same kernels, same shapes)
        torch.cuda.synchronize()
        KernelTimer.reset()
        KernelTimer.enabled = True
        eager_step()
        torch.cuda.synchronize()
        KernelTimer.enabled = False
    kern = KernelTimer.summary()
    loss_v = float(loss.item())

    if rank == 0:
        pairs = args.batch * world * args.steps
        value = pairs / elapsed
        ms = elapsed / args.steps * 1000.0
        steps_timed = 1 if graph else args.steps   # KernelTimer covers one eager step in graph mode
        dom_name, dom = max(kern.items(), key=lambda kv: kv[1]["total_ms"]) if kern else (None, None)
        roofline = None
        if dom is not None:
            tflops = dom["flops_per_launch"] / (dom["avg_ms"] * 1e-3) / 1e12
            traffic, pmc_file = latest_pmc(dom_name)
            roofline = dict(kernel=dom_name, bound="mfma", achieved=round(tflops, 3), peak=FP32_PEAK_TFLOPS,
                            unit="TFLOP/s", frac=round(tflops / FP32_PEAK_TFLOPS, 4), traffic=traffic,
                            avg_ms=round(dom["avg_ms"], 4), launches_per_step=dom["launches"] / steps_timed,
                            share_of_step=round(dom["total_ms"] / steps_timed / ms, 3),
                            algorithmic_bytes=dom["bytes_per_launch"],
                            algorithmic_gbs=round(dom["bytes_per_launch"] / (dom["avg_ms"] * 1e-3) / 1e9, 1),
                            note="fp32 compute roof (VALU = f32 MFMA rate); head_dim 2 leaves no MFMA-shaped "
                                 "contraction; traffic from " + (pmc_file or "no PMC summary yet"))
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline_c4(args.size) if args.config == "c4" else cpu_baseline(args.size,
                                                                                          args.cpu_sample_size)
            except Exception as e:  # the baseline is reported, never required
                cpu = dict(error=str(e))
        line = dict(metric=METRIC, value=round(value, 4), unit="volume-pairs/s", n_gpus=world, steps=args.steps,
                    warmup=args.warmup, ms_per_step=round(ms, 2), higher_is_better=True, scaling="weak",
                    vs_baseline=None, dtype="f32", data="synthetic (z-scored N(0,1) volumes, Bernoulli labels)",
                    config=(dict(workload=f"C3: SwinFusion 3D lift, {args.size}^3 sMRI+fMRI pairs",
                                 global_batch=args.batch * world, per_gpu_batch=args.batch, volume=args.size,
                                 patch=8, window=6, tokens_per_volume=args.size ** 3,
                                 parallelism=f"dp{world}", checkpoint=args.checkpoint, graph=graph)
                            if args.config == "c3" else
                            dict(workload=f"C4: SwinCrossmodal3D composite, {args.size}^3 pairs, crossmodal head "
                                          f"12 layers x 12 heads on {(args.size // 8) ** 3}-token sequences",
                                 global_batch=args.batch * world, per_gpu_batch=args.batch, volume=args.size,
                                 patch=8, window=6, sequence=(args.size // 8) ** 3, parallelism=f"dp{world}",
                                 checkpoint=args.checkpoint, graph=graph)),
                    roofline=roofline, cpu_baseline=cpu, loss=round(loss_v, 5),
                    kernels={k: dict(launches=v["launches"], avg_ms=round(v["avg_ms"], 4),
                                     total_ms=round(v["total_ms"], 2)) for k, v in kern.items()},
                    peak_mem_gb=round(torch.cuda.max_memory_allocated(device) / 1e9, 1))
        print(json.dumps(line), flush=True)
    D.shutdown(env)


if __name__ == "__main__":
    main()
