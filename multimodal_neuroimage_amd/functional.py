"""torch.autograd wrappers over the libmmni.so C ABI (include/mmni.h).

Every op here runs the hand-written HIP kernels; there is no eager/CPU fallback: inputs that
are not float32 ROCm-device tensors raise.  Outputs and saved tensors are allocated by torch
(caching allocator), the library only launches on torch's current stream.
"""
import ctypes
import math
import weakref
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import check, ptr, require_device, stream_handle

LN100 = math.log(1.0 / 0.01)


class KernelTimer:
    """Optional per-launch timing of the hot kernels with HIP events recorded on the stream the
    kernel is launched on (torch's current stream).  Off by default; bench.py enables it over its
    timed region.  records[name] = list of (start_event, end_event, algorithmic_flops, bytes)."""
    enabled = False
    records = {}

    @classmethod
    def start(cls):
        if not cls.enabled:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    @classmethod
    def stop(cls, name, ev, flops, nbytes):
        if ev is None:
            return
        end = torch.cuda.Event(enable_timing=True)
        end.record()
        cls.records.setdefault(name, []).append((ev, end, flops, nbytes))

    @classmethod
    def summary(cls):
        """{name: dict(launches, total_ms, avg_ms, flops_per_launch, bytes_per_launch)} (syncs)."""
        torch.cuda.synchronize()
        out = {}
        for name, recs in cls.records.items():
            ms = [a.elapsed_time(b) for a, b, _, _ in recs]
            out[name] = dict(launches=len(recs), total_ms=sum(ms), avg_ms=sum(ms) / len(ms),
                             flops_per_launch=sum(r[2] for r in recs) / len(recs),
                             bytes_per_launch=sum(r[3] for r in recs) / len(recs))
        return out

    @classmethod
    def reset(cls):
        cls.records = {}


@dataclass(frozen=True)
class WindowGeometry:
    """Volume grid + window + cyclic shift of one shifted-window attention call.

    2D reference shapes use D = 1, window (1, wh, ww), shift (0, sh, sw).
    """
    B: int
    spatial: tuple       # (D, H, W)
    window: tuple        # (wd, wh, ww)
    shift: tuple         # (sd, sh, sw)

    @property
    def tokens(self):
        D, H, W = self.spatial
        return self.B * D * H * W

    @property
    def N(self):
        wd, wh, ww = self.window
        return wd * wh * ww

    @property
    def table_rows(self):
        wd, wh, ww = self.window
        return (2 * wd - 1) * (2 * wh - 1) * (2 * ww - 1)

    @staticmethod
    def make(B, spatial, window, shift):
        spatial = tuple(int(s) for s in spatial)
        if len(spatial) == 2:
            spatial = (1,) + spatial
        if isinstance(window, int):
            window = (window,) * 3 if len(spatial) == 3 and spatial[0] > 1 else (1, window, window)
        window = tuple(int(w) for w in window)
        if len(window) == 2:
            window = (1,) + window
        if isinstance(shift, int):
            shift = tuple(shift if w > 1 else 0 for w in window)
        shift = tuple(int(s) for s in shift)
        if len(shift) == 2:
            shift = (0,) + shift
        return WindowGeometry(int(B), spatial, window, shift)


def _wattn_desc(g, C, heads, kind, scale, qs, ks, vs, os_):
    d = _lib.WAttnDesc()
    d.B = g.B
    d.D, d.H, d.W = g.spatial
    d.C = C
    d.heads = heads
    d.wd, d.wh, d.ww = g.window
    d.sd, d.sh, d.sw = g.shift
    d.kind = kind
    d.scale = float(scale)
    d.q_stride, d.k_stride, d.v_stride, d.o_stride = int(qs), int(ks), int(vs), int(os_)
    return d


def _row_view(t, C, offset):
    """(rows, stride) view of channels [offset, offset+C) of a (rows, stride) tensor."""
    return t[:, offset:offset + C]


class _WindowAttention(torch.autograd.Function):
    """Fused shift + partition + window attention + reverse, on token rows.

    q_src: (rows, Cq_total) with q in columns [0, C); kv_src: (rows, Ckv_total) with k in
    [k_off, k_off+C) and v in [v_off, v_off+C).  For self attention q_src is kv_src (packed
    qkv, offsets 0/C/2C).  Returns (rows, C).
    """

    @staticmethod
    def forward(ctx, q_src, kv_src, table, tau, geom, heads, kind, scale, k_off, v_off, packed):
        C = q_src.shape[1] // 3 if packed else q_src.shape[1]
        require_device(q_src, kv_src, table, tau, what="window_attention")
        rows = q_src.shape[0]
        assert rows == geom.tokens, f"window_attention: {rows} rows != geometry tokens {geom.tokens}"
        assert q_src.stride(1) == 1 and kv_src.stride(1) == 1
        table = table.contiguous()
        tau_c = tau.contiguous() if tau is not None else None
        out = torch.empty((rows, C), device=q_src.device, dtype=torch.float32)
        lse = torch.empty((rows, heads), device=q_src.device, dtype=torch.float32)
        q = q_src
        k = kv_src[:, k_off:]
        v = kv_src[:, v_off:]
        d = _wattn_desc(geom, C, heads, kind, scale, q.stride(0), k.stride(0), v.stride(0), C)
        L = _lib.load()
        vmax = torch.zeros(1, device=q_src.device, dtype=torch.int32)   # max|v| bits for the bwd bound
        ev = KernelTimer.start()
        check(L.mmni_wattn_fwd(d, ptr(q), ptr(k), ptr(v), ptr(table), ptr(tau_c), ptr(out), ptr(lse), ptr(vmax),
                               stream_handle(q_src.device)), "mmni_wattn_fwd")
        # SURVEY §8d counting: fwd 4*T*N*C FLOPs, 4*T*C*4 bytes (q, k, v read, o written)
        KernelTimer.stop(f"wattn_fwd_k{kind}_C{C}_N{geom.N}", ev, 4.0 * rows * geom.N * C, 16.0 * rows * C)
        ctx.save_for_backward(q_src, kv_src, table, tau_c, out, lse, vmax)
        ctx.cfg = (geom, heads, kind, scale, k_off, v_off, packed, C)
        return out

    @staticmethod
    def backward(ctx, dout):
        q_src, kv_src, table, tau, out, lse, vmax = ctx.saved_tensors
        geom, heads, kind, scale, k_off, v_off, packed, C = ctx.cfg
        dout = dout.contiguous()
        if packed:
            dq_src = torch.empty_like(q_src)
            dkv_src = dq_src
        else:
            dq_src = torch.empty_like(q_src)
            dkv_src = torch.empty_like(kv_src)
            if kv_src.shape[1] > 2 * C or (k_off, v_off) != (0, C):
                dkv_src.zero_()
        dtable = torch.zeros_like(table)
        dtau = torch.zeros_like(tau) if tau is not None else None
        q, k, v = q_src, kv_src[:, k_off:], kv_src[:, v_off:]
        dq, dk, dv = dq_src, dkv_src[:, k_off:], dkv_src[:, v_off:]
        d = _wattn_desc(geom, C, heads, kind, scale, q.stride(0), k.stride(0), v.stride(0), C)
        L = _lib.load()
        ws = torch.empty(L.mmni_wattn_bwd_workspace_bytes(d) // 8, device=q_src.device, dtype=torch.int64)
        ev = KernelTimer.start()
        check(L.mmni_wattn_bwd(d, ptr(q), ptr(k), ptr(v), ptr(table), ptr(tau), ptr(out), ptr(dout), ptr(lse),
                               ptr(dq), ptr(dk), ptr(dv), ptr(dtable), ptr(dtau), ptr(ws), ptr(vmax),
                               stream_handle(q_src.device)), "mmni_wattn_bwd")
        # SURVEY §8d counting: bwd 10*T*N*C FLOPs; bytes 8*T*C*4 + 4*T*heads (lse)
        rows = q_src.shape[0]
        KernelTimer.stop(f"wattn_bwd_k{kind}_C{C}_N{geom.N}", ev, 10.0 * rows * geom.N * C,
                         32.0 * rows * C + 4.0 * rows * heads)
        if packed:
            return dq_src, None, dtable, dtau, None, None, None, None, None, None, None
        return dq_src, dkv_src, dtable, dtau, None, None, None, None, None, None, None


def window_attention_self(qkv, table, geom, heads, *, kind=0, scale=None, tau=None):
    """Self window attention on packed qkv token rows (rows, 3C) -> (rows, C)."""
    C = qkv.shape[-1] // 3
    qkv2 = qkv.reshape(-1, 3 * C)
    if not qkv2.is_contiguous():
        qkv2 = qkv2.contiguous()
    if scale is None:
        scale = (C // heads) ** -0.5
    return _WindowAttention.apply(qkv2, qkv2, table, tau, geom, heads, kind, scale, C, 2 * C, True)


def window_attention_cross(q, kv, table, geom, heads, *, kind=0, scale=None, tau=None):
    """Cross window attention: q rows (rows, C) from x, kv rows (rows, 2C) from y."""
    C = q.shape[-1]
    q2 = q.reshape(-1, C).contiguous()
    kv2 = kv.reshape(-1, 2 * C).contiguous()
    if scale is None:
        scale = (C // heads) ** -0.5
    return _WindowAttention.apply(q2, kv2, table, tau, geom, heads, kind, scale, 0, C, False)


def window_rows(geom, device):
    """Integer gather map rows[w*N + t] used by the kernels (row a0)."""
    n = geom.B * (geom.spatial[0] // geom.window[0]) * (geom.spatial[1] // geom.window[1]) * \
        (geom.spatial[2] // geom.window[2]) * geom.N
    out = torch.empty(n, dtype=torch.int32, device=device)
    d = _wattn_desc(geom, 12, 6, 0, 1.0, 12, 12, 12, 12)
    check(_lib.load().mmni_window_rows(d, ptr(out), stream_handle(device)), "mmni_window_rows")
    return out


def window_mask(geom, device):
    """(nW, N, N) shift mask of one sample, {0, -100} (calculate_mask equivalent)."""
    nW = (geom.spatial[0] // geom.window[0]) * (geom.spatial[1] // geom.window[1]) * \
        (geom.spatial[2] // geom.window[2])
    out = torch.empty((nW, geom.N, geom.N), dtype=torch.float32, device=device)
    d = _wattn_desc(geom, 12, 6, 0, 1.0, 12, 12, 12, 12)
    check(_lib.load().mmni_window_mask(d, ptr(out), stream_handle(device)), "mmni_window_mask")
    return out


def relative_index(geom, device):
    out = torch.empty((geom.N, geom.N), dtype=torch.int32, device=device)
    d = _wattn_desc(geom, 12, 6, 0, 1.0, 12, 12, 12, 12)
    check(_lib.load().mmni_relative_index(d, ptr(out), stream_handle(device)), "mmni_relative_index")
    return out


# ----------------------------------------------------------------------------------------
# crossmodal multi-head attention core
# ----------------------------------------------------------------------------------------
def _workspace(nbytes, device):
    """Scratch for a kernel call (the caching allocator's blocks are >= 512-byte aligned)."""
    return torch.empty(max(int(nbytes), 256), device=device, dtype=torch.uint8)


def _mha_desc(Tq, Tk, B, heads, hd, causal_diag, scale, qs, ks, vs, os_, dropout=0.0, seed=0,
              dtype=torch.float32):
    d = _lib.MhaDesc()
    d.dtype = 1 if dtype == torch.bfloat16 else 0
    d.Tq, d.Tk, d.B, d.heads, d.head_dim = Tq, Tk, B, heads, hd
    d.causal_diag = int(causal_diag)
    d.scale = float(scale)
    d.q_stride, d.k_stride, d.v_stride, d.o_stride = int(qs), int(ks), int(vs), int(os_)
    d.dropout = float(dropout)
    d.seed = int(seed) & 0xffffffff
    return d


def dropout_seed():
    """A 32-bit seed for one attention-dropout mask, drawn from torch's default CPU generator (so
    torch.manual_seed makes runs reproducible, as the reference's F.dropout is)."""
    return int(torch.randint(0, 2 ** 31 - 1, (1,)).item())


class _MHA(torch.autograd.Function):
    """q (Tq, B, E), k/v (Tk, B, E) dense time-major tensors -> out (Tq, B, E), lse (B, h, Tq).
    dropout p > 0 applies the counter-based mask of `seed` to the probabilities (the backward
    regenerates it).  fp32 or bf16 storage (all three alike; out and the gradients follow it)."""

    @staticmethod
    def forward(ctx, q, k, v, heads, causal_diag, scale, dropout, seed):
        require_device(q, k, v, what="mha", dtypes=(torch.float32, torch.bfloat16))
        if not (q.dtype == k.dtype == v.dtype):
            raise RuntimeError(f"mha: q/k/v dtypes differ ({q.dtype}, {k.dtype}, {v.dtype})")
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        Tq, B, E = q.shape
        Tk = k.shape[0]
        out = torch.empty((Tq, B, E), device=q.device, dtype=q.dtype)
        lse = torch.empty((B, heads, Tq), device=q.device, dtype=torch.float32)
        d = _mha_desc(Tq, Tk, B, heads, E // heads, causal_diag, scale, E, E, E, E, dropout, seed, q.dtype)
        lib = _lib.load()
        ws = _workspace(lib.mmni_mha_fwd_workspace_bytes(d), q.device)
        ev = KernelTimer.start()
        check(lib.mmni_mha_fwd(d, ptr(q), ptr(k), ptr(v), ptr(out), ptr(lse), ptr(ws),
                               stream_handle(q.device)), "mmni_mha_fwd")
        sfx = "_bf16" if q.dtype == torch.bfloat16 else ""
        KernelTimer.stop(f"mha_fwd_E{E}{sfx}", ev, 4.0 * Tq * Tk * B * E, q.element_size() * B * E * (2 * Tq + 2 * Tk))
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.cfg = (heads, causal_diag, scale, dropout, seed)
        ctx.mark_non_differentiable(lse)
        return out, lse

    @staticmethod
    def backward(ctx, dout, _dlse):
        q, k, v, out, lse = ctx.saved_tensors
        heads, causal_diag, scale, dropout, seed = ctx.cfg
        Tq, B, E = q.shape
        Tk = k.shape[0]
        dout = dout.contiguous().to(q.dtype)
        dq = torch.empty_like(q)
        dk = torch.empty_like(k)
        dv = torch.empty_like(v)
        d = _mha_desc(Tq, Tk, B, heads, E // heads, causal_diag, scale, E, E, E, E, dropout, seed, q.dtype)
        lib = _lib.load()
        ws = _workspace(lib.mmni_mha_bwd_workspace_bytes(d), q.device)
        ev = KernelTimer.start()
        check(lib.mmni_mha_bwd(d, ptr(q), ptr(k), ptr(v), ptr(out), ptr(dout), ptr(lse),
                               ptr(dq), ptr(dk), ptr(dv), ptr(ws), stream_handle(q.device)),
              "mmni_mha_bwd")
        sfx = "_bf16" if q.dtype == torch.bfloat16 else ""
        KernelTimer.stop(f"mha_bwd_E{E}{sfx}", ev, 10.0 * Tq * Tk * B * E, q.element_size() * B * E * (4 * Tq + 4 * Tk))
        return dq, dk, dv, None, None, None, None, None


def mha_core(q, k, v, heads, causal_diag=0, scale=None, dropout=0.0, seed=None):
    """dropout(softmax(q*scale @ k^T + causal)) @ v over (T, B, E) time-major tensors.

    Returns (out, lse); lse (B, heads, Tq) feeds mha_mean_probs.  With dropout > 0 the mask comes
    from `seed` (drawn with dropout_seed() when None); pass the same seed to mha_mean_probs."""
    E = q.shape[-1]
    if scale is None:
        scale = (E // heads) ** -0.5
    if dropout > 0 and seed is None:
        seed = dropout_seed()
    return _MHA.apply(q, k, v, heads, causal_diag, scale, float(dropout), int(seed or 0))


class _MhaMeanProbs(torch.autograd.Function):
    """Head-averaged (dropped) probabilities from the kernel's lse.  Forward: the HIP kernel.
    Backward (rarely needed: no reference caller back-propagates through the weights, but the
    reference's autograd would): the per-head probabilities are rebuilt on the device in fp32 from
    q, k and lse, then dS = P (dP - rowsum(dP P)) and dq = scale dS k, dk = scale dS^T q."""

    @staticmethod
    def forward(ctx, q, k, lse, heads, causal_diag, scale, dropout, seed):
        Tq, B, E = q.shape
        Tk = k.shape[0]
        qc = q if (q.stride(1) == E and q.stride(0) == B * E) else q.contiguous()
        kc = k if (k.stride(1) == E and k.stride(0) == B * E) else k.contiguous()
        probs = torch.empty((B, Tq, Tk), device=q.device, dtype=torch.float32)
        d = _mha_desc(Tq, Tk, B, heads, E // heads, causal_diag, scale, E, E, E, E, dropout, seed, q.dtype)
        check(_lib.load().mmni_mha_mean_probs(d, ptr(qc), ptr(kc), ptr(lse), ptr(probs), stream_handle(q.device)),
              "mmni_mha_mean_probs")
        ctx.save_for_backward(q, k, lse)
        ctx.cfg = (heads, causal_diag, scale, dropout, seed)
        return probs

    @staticmethod
    def backward(ctx, dw):
        q, k, lse = ctx.saved_tensors
        heads, diag, scale, dropout, seed = ctx.cfg
        Tq, B, E = q.shape
        Tk = k.shape[0]
        hd = E // heads
        qh = q.float().reshape(Tq, B, heads, hd).permute(1, 2, 0, 3)     # (B, h, Tq, d)
        kh = k.float().reshape(Tk, B, heads, hd).permute(1, 2, 0, 3)     # (B, h, Tk, d)
        dq = torch.empty((B, heads, Tq, hd), device=q.device, dtype=torch.float32)
        dk = torch.empty((B, heads, Tk, hd), device=q.device, dtype=torch.float32)
        causal = (torch.triu(torch.full((Tq, Tk), float("-inf"), device=q.device), diag) if diag > 0 else None)
        # the dense (Tq, Tk) rebuild runs over (batch, head-chunk) slices sized to ~256 MB per
        # tensor, so C5-sized calls (8 x 12 x 4096^2) do not materialise 6.4 GB tensors
        hc = max(1, min(heads, (64 << 20) // max(1, Tq * Tk)))
        # (dropout: the kernels' mask is generated once for the whole call; only this rarely used
        # path, back-propagation through the returned weights with dropout on, holds it whole)
        dmask = mha_dropout_mask(Tq, Tk, B, heads, dropout, seed, q.device, diag) if dropout > 0 else None
        for b in range(B):
            dwb = dw[b].float() / heads                                   # (Tq, Tk), shared by the heads
            for h0 in range(0, heads, hc):
                h1 = min(heads, h0 + hc)
                s = torch.matmul(qh[b, h0:h1], kh[b, h0:h1].transpose(-1, -2)) * scale
                if causal is not None:
                    s = s + causal
                p = torch.exp(s - lse[b, h0:h1].unsqueeze(-1))           # the forward's softmax
                del s
                dp = dwb.expand(h1 - h0, Tq, Tk)
                if dropout > 0:
                    dp = dp * dmask[b, h0:h1]
                ds = p * (dp - (dp * p).sum(-1, keepdim=True))
                del p, dp
                dq[b, h0:h1] = torch.matmul(ds, kh[b, h0:h1]) * scale
                dk[b, h0:h1] = torch.matmul(ds.transpose(-1, -2), qh[b, h0:h1]) * scale
        dq = dq.permute(2, 0, 1, 3).reshape(Tq, B, E)
        dk = dk.permute(2, 0, 1, 3).reshape(Tk, B, E)
        return dq.to(q.dtype), dk.to(k.dtype), None, None, None, None, None, None


def mha_mean_probs(q, k, lse, heads, causal_diag=0, scale=None, dropout=0.0, seed=0):
    """Head-averaged (dropped) attention weights (B, Tq, Tk) (multihead_attention.py:123,131-133),
    differentiable with respect to q and k."""
    E = q.shape[-1]
    if scale is None:
        scale = (E // heads) ** -0.5
    return _MhaMeanProbs.apply(q, k, lse, heads, causal_diag, scale, float(dropout), int(seed or 0))


def mha_dropout_mask(Tq, Tk, B, heads, dropout, seed, device, causal_diag=0):
    """(B, heads, Tq, Tk) multipliers (0 or 1/(1-p)) of the kernels' dropout mask for `seed`."""
    mask = torch.empty((B, heads, Tq, Tk), device=device, dtype=torch.float32)
    d = _mha_desc(Tq, Tk, B, heads, 1, causal_diag, 1.0, heads, heads, heads, heads, dropout, seed)
    check(_lib.load().mmni_mha_dropout_mask(d, ptr(mask), stream_handle(device)), "mmni_mha_dropout_mask")
    return mask


# ----------------------------------------------------------------------------------------
# channels-last 3D convolution
# ----------------------------------------------------------------------------------------
def _triple(v):
    return tuple(int(a) for a in v) if isinstance(v, (tuple, list)) else (int(v),) * 3


def _conv_desc(x_shape, w_shape, stride, pad, slope):
    B, D, H, W, Cin = x_shape
    Cout, _, kd, kh, kw = w_shape
    sd, sh, sw = stride
    pd, ph, pw = pad
    d = _lib.Conv3dDesc()
    d.B, d.D, d.H, d.W, d.Cin, d.Cout = B, D, H, W, Cin, Cout
    d.kd, d.kh, d.kw, d.sd, d.sh, d.sw, d.pd, d.ph, d.pw = kd, kh, kw, sd, sh, sw, pd, ph, pw
    d.Do = (D + 2 * pd - kd) // sd + 1
    d.Ho = (H + 2 * ph - kh) // sh + 1
    d.Wo = (W + 2 * pw - kw) // sw + 1
    d.slope = float(slope)
    return d


class _Conv3d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad, slope):
        require_device(x, weight, bias, what="conv3d")
        x = x.contiguous()
        weight = weight.contiguous()
        if weight.data_ptr() % 8:
            weight = weight.clone()   # the k3 kernel reads 8-B aligned weight pairs (mmni.h)
        assert weight.dim() == 5 and x.dim() == 5 and x.shape[-1] == weight.shape[1]
        d = _conv_desc(tuple(x.shape), tuple(weight.shape), stride, pad, slope)
        y = torch.empty((d.B, d.Do, d.Ho, d.Wo, d.Cout), device=x.device, dtype=torch.float32)
        ev = KernelTimer.start()
        check(_lib.load().mmni_conv3d_fwd(d, ptr(x), ptr(weight), ptr(bias), ptr(y), stream_handle(x.device)),
              "mmni_conv3d_fwd")
        nout = y.numel() // d.Cout
        KernelTimer.stop(f"conv3d_fwd_{d.Cin}x{d.Cout}_k{d.kd}{d.kh}{d.kw}", ev,
                         2.0 * nout * d.Cout * d.Cin * d.kd * d.kh * d.kw, 4.0 * (x.numel() + y.numel()))
        ctx.save_for_backward(x, weight, y if slope != 1.0 else None)
        ctx.cfg = (stride, pad, slope, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        stride, pad, slope, has_bias = ctx.cfg
        dy = dy.contiguous()
        d = _conv_desc(tuple(x.shape), tuple(weight.shape), stride, pad, slope)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(weight)
        db = torch.empty(d.Cout, device=x.device, dtype=torch.float32) if has_bias else None
        L = _lib.load()
        ws = torch.empty(L.mmni_conv3d_bwd_workspace_bytes(d) // 4, device=x.device, dtype=torch.float32)
        ev = KernelTimer.start()
        check(L.mmni_conv3d_bwd(d, ptr(x), ptr(weight), ptr(y), ptr(dy), ptr(dx), ptr(dw), ptr(db), ptr(ws),
                                stream_handle(x.device)), "mmni_conv3d_bwd")
        nout = dy.numel() // d.Cout
        KernelTimer.stop(f"conv3d_bwd_{d.Cin}x{d.Cout}_k{d.kd}{d.kh}{d.kw}", ev,
                         4.0 * nout * d.Cout * d.Cin * d.kd * d.kh * d.kw,
                         4.0 * (2 * x.numel() + 2 * dy.numel()))
        return dx, dw, db, None, None, None


def conv3d_cl(x, weight, bias=None, stride=1, pad=0, slope=1.0):
    """Channels-last conv: x (B, D, H, W, Cin), weight (Cout, Cin, kd, kh, kw) ->
    (B, Do, Ho, Wo, Cout) with a fused LeakyReLU(slope) (slope 1 = identity)."""
    return _Conv3d.apply(x, weight, bias, _triple(stride), _triple(pad), slope)


# ----------------------------------------------------------------------------------------
# token-wise LayerNorm and Linear (weight gradient on the f32 MFMA)
# ----------------------------------------------------------------------------------------
LN_CHANNELS = (12, 24, 48, 96)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        require_device(x, weight, bias, what="layer_norm")
        C = x.shape[-1]
        x2 = x.reshape(-1, C).contiguous()
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        ev = KernelTimer.start()
        check(_lib.load().mmni_layernorm_fwd(rows, C, ptr(x2), ptr(weight), ptr(bias), float(eps), ptr(y),
                                              ptr(mean), ptr(rstd), stream_handle(x.device)), "mmni_layernorm_fwd")
        KernelTimer.stop(f"layernorm_fwd_C{C}", ev, 8.0 * rows * C, 8.0 * rows * C + 8.0 * rows)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, mean, rstd = ctx.saved_tensors
        C = x2.shape[1]
        rows = x2.shape[0]
        dy2 = dy.reshape(-1, C).contiguous()
        dx = torch.empty_like(x2)
        dgamma = torch.empty(C, device=x2.device, dtype=torch.float32)
        dbeta = torch.empty(C, device=x2.device, dtype=torch.float32)
        L = _lib.load()
        ws = torch.empty(L.mmni_layernorm_bwd_workspace_bytes(rows, C) // 4, device=x2.device, dtype=torch.float32)
        ev = KernelTimer.start()
        check(L.mmni_layernorm_bwd(rows, C, ptr(dy2), ptr(x2), ptr(weight), ptr(mean), ptr(rstd), ptr(dx),
                                   ptr(dgamma), ptr(dbeta), ptr(ws), stream_handle(x2.device)), "mmni_layernorm_bwd")
        KernelTimer.stop(f"layernorm_bwd_C{C}", ev, 12.0 * rows * C, 12.0 * rows * C + 8.0 * rows)
        return dx.view(ctx.shape), dgamma, dbeta, None


class _RowLayerNorm(torch.autograd.Function):
    """nn.LayerNorm over rows of C <= 256 (the crossmodal encoder's 84 / 168) on the wave-per-row
    kernels (mmni_row_layernorm_fwd_t / _bwd_t).  Computes in fp32 and returns fp32 — what torch's
    autocast does with layer_norm — from fp32 or bf16 input; out_dtype=bf16 stores the output
    rounded to bf16 for a consumer that is a bf16 GEMM (the autocast Linear would round the fp32
    output the same way), and then takes its gradient in bf16.  The input gradient comes back in the
    input's dtype."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, out_dtype):
        C = x.shape[-1]
        x2 = x.reshape(-1, C).float().contiguous()
        w, b = weight.float().contiguous(), bias.float().contiguous()
        rows = x2.shape[0]
        y = torch.empty(x2.shape, device=x.device, dtype=out_dtype)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        check(_lib.load().mmni_row_layernorm_fwd_t(rows, C, ptr(x2), C, ptr(w), ptr(b), float(eps), ptr(y),
                                                   1 if out_dtype == torch.bfloat16 else 0, C, ptr(mean), ptr(rstd),
                                                   stream_handle(x.device)), "mmni_row_layernorm_fwd")
        ctx.save_for_backward(x2, w, mean, rstd)
        ctx.shape, ctx.dtype, ctx.wdtype = x.shape, x.dtype, weight.dtype
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        dy2 = dy.reshape(x2.shape)
        if dy2.dtype not in (torch.float32, torch.bfloat16):
            dy2 = dy2.float()
        dx, dg, db = row_layernorm_bwd(dy2.contiguous(), x2, w, mean, rstd)
        return dx.view(ctx.shape).to(ctx.dtype), dg.to(ctx.wdtype), db.to(ctx.wdtype), None, None


def layer_norm(x, ln, out_dtype=None):
    """nn.LayerNorm `ln` applied to x (..., C) with the HIP kernels: the token kernels at C in
    12/24/48/96, the wave-per-row kernels up to C = 256 (the crossmodal stack's 84/168), torch's
    ROCm LayerNorm beyond.  out_dtype=torch.bfloat16 (row kernels only) stores the output in bf16 for
    a bf16 GEMM consumer.  No CPU path."""
    require_device(x, what="layer_norm", dtypes=(torch.float32, torch.bfloat16))
    C = x.shape[-1]
    if C in LN_CHANNELS and x.dtype == torch.float32 and out_dtype is None:
        return _LayerNorm.apply(x, ln.weight, ln.bias, ln.eps)
    if C <= 256 and ln.elementwise_affine and ln.bias is not None:
        return _RowLayerNorm.apply(x, ln.weight, ln.bias, ln.eps, out_dtype or torch.float32)
    y = ln(x)
    return y.to(out_dtype) if out_dtype is not None else y


_DW_TILES = {(1, 1), (1, 2), (1, 3), (2, 1), (3, 1), (2, 2), (3, 3), (1, 4), (4, 1), (2, 3), (3, 2), (9, 3), (3, 9),
             (6, 2), (2, 6), (4, 2), (2, 4), (5, 3), (3, 5), (6, 3), (3, 6), (8, 2), (2, 8), (12, 3), (3, 12),
             (4, 4), (6, 6), (4, 12), (12, 4)}


def _tlin_ok(K, N, epi=0, K2=0):
    return bool(_lib.load().mmni_token_linear_supported(K, N, epi, K2))


def _tlin(x2, w, bias, K, N, epi=0, transposed=False, aux=None, w2=None, b2=None, K2=0, residual=None):
    """HIP token Linear on (rows, K) rows -> (rows, N).  w is an nn.Linear weight (N, K), or
    with transposed=True the weight (K, N) of the Linear whose input gradient this is.
    residual (rows, N), contiguous, is added in the epilogue."""
    rows = x2.shape[0]
    y = torch.empty(rows, N, device=x2.device, dtype=torch.float32)
    d = _lib.TLinDesc()
    d.rows, d.K, d.N, d.epi, d.K2 = rows, K, N, epi, K2
    d.ldx, d.ldy, d.ldaux = x2.stride(0), N, (aux.stride(0) if aux is not None else 0)
    d.w_sn, d.w_sk = (1, N) if transposed else (K, 1)
    L = _lib.load()
    ev = KernelTimer.start()
    check(L.mmni_token_linear(ctypes.byref(d), ptr(x2), ptr(w), ptr(bias), ptr(aux), ptr(w2), ptr(b2),
                              ptr(residual), ptr(y), stream_handle(x2.device)), "mmni_token_linear")
    extra = 2.0 * rows * K2 * N if epi == 2 else 0.0
    KernelTimer.stop(f"token_linear_e{epi}_{K}x{N}", ev, 2.0 * rows * K * N + extra,
                     4.0 * rows * (K + N + (K2 if epi == 2 else 0)))
    return y


def _rows2d(t, C):
    t2 = t.reshape(-1, C)
    return t2 if (t2.stride(1) == 1 and t2.stride(0) % 4 == 0 and t2.data_ptr() % 16 == 0) else t2.contiguous()


def _linear_dw(x2, dy2, N, K, with_bias):
    rows = x2.shape[0]
    dw = torch.empty(N, K, device=x2.device, dtype=torch.float32)
    db = torch.empty(N, device=x2.device, dtype=torch.float32) if with_bias else None
    L = _lib.load()
    ws = torch.empty(L.mmni_linear_dw_workspace_bytes(N, K) // 4, device=x2.device, dtype=torch.float32)
    ev = KernelTimer.start()
    check(L.mmni_linear_dw(rows, N, K, ptr(x2), x2.stride(0), ptr(dy2), dy2.stride(0), ptr(dw), ptr(db), ptr(ws),
                           stream_handle(x2.device)), "mmni_linear_dw")
    KernelTimer.stop(f"linear_dw_{N}x{K}", ev, 2.0 * rows * N * K, 4.0 * rows * (N + K))
    return dw, db


class _TokenLinear(torch.autograd.Function):
    """y = x W^T + b on token rows.  Forward and dX on the HIP token-linear kernel when the shape
    is compiled (else hipBLASLt via torch), dW/db on the HIP MFMA reduction (the K = rows
    weight-gradient GEMM is where the library kernels stall)."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual):
        N, K = weight.shape
        x2 = _rows2d(x, K)
        ctx.save_for_backward(x2, weight)
        ctx.has_bias = bias is not None
        ctx.xshape = x.shape
        r2 = residual.reshape(-1, N).contiguous() if residual is not None else None
        if _tlin_ok(K, N):
            y = _tlin(x2, weight, bias, K, N, residual=r2)
        else:
            y = rowgemm(x2.contiguous(), weight.contiguous(), bias, res=r2)
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        N, K = weight.shape
        dy2 = _rows2d(dy, N)
        dx = None
        if (N == K == TOK_C and ctx.needs_input_grad[0] and x2.is_contiguous() and dy2.is_contiguous()
                and x2.data_ptr() % 16 == 0):
            dx, dw, db = _linear_bwd_fused(x2, dy2, weight, ctx.has_bias)
            return dx.view(ctx.xshape), dw, db, (dy if ctx.needs_input_grad[3] else None)
        if ctx.needs_input_grad[0]:
            dx = (_tlin(dy2, weight, None, N, K, transposed=True) if _tlin_ok(N, K)
                  else rowgemm(dy2.contiguous(), weight.contiguous(), transpose_w=True))
            dx = dx.view(ctx.xshape)
        dw, db = _linear_dw(x2, dy2, N, K, ctx.has_bias)
        return dx, dw, db, (dy if ctx.needs_input_grad[3] else None)


class _Mlp(torch.autograd.Function):
    """fc2(GELU(fc1(x))) on token rows (Mlp / Mlp_fusion, swin_v2_module.py:16-32,
    swinfusion_module.py:14-30) with the GELU fused into the fc1 kernel and, in backward, into
    the fc2 input-gradient kernel (the fc1 pre-activation is recomputed there, never stored)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, residual):
        H, C = w1.shape
        O = w2.shape[0]
        x2 = _rows2d(x, C)
        h = _tlin(x2, w1, b1, C, H, epi=1)
        r2 = residual.reshape(-1, O).contiguous() if residual is not None else None
        y = _tlin(h, w2, b2, H, O, residual=r2)
        ctx.save_for_backward(x2, h, w1, b1, w2)
        ctx.xshape = x.shape
        ctx.has_b = (b1 is not None, b2 is not None)
        return y.view(*x.shape[:-1], O)

    @staticmethod
    def backward(ctx, dy):
        x2, h, w1, b1, w2 = ctx.saved_tensors
        H, C = w1.shape
        O = w2.shape[0]
        dy2 = _rows2d(dy, O)
        dw2, db2 = _linear_dw(h, dy2, O, H, ctx.has_b[1])
        dpre = _tlin(dy2, w2, None, O, H, epi=2, transposed=True, aux=x2, w2=w1, b2=b1, K2=C)
        dw1, db1 = _linear_dw(x2, dpre, H, C, ctx.has_b[0])
        dx = _tlin(dpre, w1, None, H, C, transposed=True).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        return dx, dw1, db1, dw2, db2, (dy if ctx.needs_input_grad[5] else None)


def _mlp_desc(rows, C, H, ldx, ldy):
    d = _lib.MlpDesc()
    d.rows, d.C, d.H, d.ldx, d.ldy = rows, C, H, ldx, ldy
    return d


class _FusedMlp(torch.autograd.Function):
    """fc2(GELU(fc1(x))) (+ residual) in one HIP kernel per direction (mlp.hip, f32 MFMA): the
    hidden activation never reaches HBM; backward recomputes it from x."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, residual):
        H, C = w1.shape
        x2 = x.reshape(-1, C).contiguous()
        rows = x2.shape[0]
        y = torch.empty(rows, C, device=x2.device, dtype=torch.float32)
        r2 = residual.reshape(-1, C).contiguous() if residual is not None else None
        d = _mlp_desc(rows, C, H, C, C)
        ev = KernelTimer.start()
        check(_lib.load().mmni_mlp_fwd(ctypes.byref(d), ptr(x2), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(r2), ptr(y),
                                       stream_handle(x2.device)), "mmni_mlp_fwd")
        # algorithmic: 4*rows*C*H FLOPs (two GEMMs); bytes: x, y (+ residual) rows
        KernelTimer.stop(f"mlp_fwd_{C}x{H}", ev, 4.0 * rows * C * H, 4.0 * rows * C * (3 if r2 is not None else 2))
        ctx.save_for_backward(x2, w1, b1, w2)
        ctx.has_b = (b1 is not None, b2 is not None)
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], C)

    @staticmethod
    def backward(ctx, dy):
        x2, w1, b1, w2 = ctx.saved_tensors
        H, C = w1.shape
        dy2 = dy.reshape(-1, C).contiguous()
        rows = x2.shape[0]
        dx = torch.empty(rows, C, device=x2.device, dtype=torch.float32)
        dw1 = torch.empty_like(w1)
        dw2 = torch.empty_like(w2)
        db1 = torch.empty(H, device=x2.device, dtype=torch.float32)
        db2 = torch.empty(C, device=x2.device, dtype=torch.float32)
        L = _lib.load()
        d = _mlp_desc(rows, C, H, C, C)
        ws = torch.empty(L.mmni_mlp_bwd_workspace_bytes(ctypes.byref(d)) // 4, device=x2.device, dtype=torch.float32)
        ev = KernelTimer.start()
        check(L.mmni_mlp_bwd(ctypes.byref(d), ptr(x2), ptr(w1), ptr(b1), ptr(w2), ptr(dy2), ptr(dx), ptr(dw1), ptr(db1),
                             ptr(dw2), ptr(db2), ptr(ws), stream_handle(x2.device)), "mmni_mlp_bwd")
        # algorithmic: recompute (2*rows*C*H) + dgrad (2 GEMMs) + wgrad (2 GEMMs) = 10*rows*C*H
        KernelTimer.stop(f"mlp_bwd_{C}x{H}", ev, 10.0 * rows * C * H, 4.0 * rows * C * 3)
        return (dx.view(ctx.xshape), dw1, db1 if ctx.has_b[0] else None, dw2, db2 if ctx.has_b[1] else None,
                dy if ctx.needs_input_grad[5] else None)


class _LnMlp(torch.autograd.Function):
    """x + fc2(GELU(fc1(LN(x)))) (residual_x) or fc2(GELU(fc1(LN(x)))) in one HIP kernel per
    direction (mlp.hip, LN prologue): the norm2 output, the hidden activation and the LN
    statistics never reach HBM; the backward adds the LN backward and the residual gradient."""

    @staticmethod
    def forward(ctx, x, gamma, beta, w1, b1, w2, b2, eps, residual_x, skip):
        H, C = w1.shape
        x2 = x.reshape(-1, C).contiguous()
        rows = x2.shape[0]
        y = torch.empty(rows, C, device=x2.device, dtype=torch.float32)
        d = _mlp_desc(rows, C, H, C, C)
        L = _lib.load()
        ev = KernelTimer.start()
        if skip is None:
            check(L.mmni_ln_mlp_fwd(ctypes.byref(d), float(eps), ptr(x2), ptr(gamma), ptr(beta), ptr(w1), ptr(b1),
                                    ptr(w2), ptr(b2), int(residual_x), ptr(y), stream_handle(x2.device)),
                  "mmni_ln_mlp_fwd")
        else:
            s2 = skip.reshape(-1, C).contiguous()
            check(L.mmni_ln_mlp_skip_fwd(ctypes.byref(d), float(eps), ptr(x2), ptr(gamma), ptr(beta), ptr(w1),
                                         ptr(b1), ptr(w2), ptr(b2), int(residual_x), ptr(s2), ptr(y),
                                         stream_handle(x2.device)), "mmni_ln_mlp_skip_fwd")
        KernelTimer.stop(f"ln_mlp_fwd_{C}x{H}", ev, 4.0 * rows * C * H, 4.0 * rows * C * (2 if skip is None else 3))
        ctx.save_for_backward(x2, gamma, beta, w1, b1, w2)
        ctx.has_b = (b1 is not None, b2 is not None)
        ctx.eps, ctx.residual_x, ctx.xshape = float(eps), bool(residual_x), x.shape
        return y.view(*x.shape[:-1], C)

    @staticmethod
    def backward(ctx, dy):
        x2, gamma, beta, w1, b1, w2 = ctx.saved_tensors
        H, C = w1.shape
        dy2 = dy.reshape(-1, C).contiguous()
        rows = x2.shape[0]
        dev = x2.device
        dx = torch.empty(rows, C, device=dev, dtype=torch.float32)
        dgamma = torch.empty(C, device=dev, dtype=torch.float32)
        dbeta = torch.empty(C, device=dev, dtype=torch.float32)
        dw1, dw2 = torch.empty_like(w1), torch.empty_like(w2)
        db1 = torch.empty(H, device=dev, dtype=torch.float32)
        db2 = torch.empty(C, device=dev, dtype=torch.float32)
        L = _lib.load()
        d = _mlp_desc(rows, C, H, C, C)
        ws = torch.empty(L.mmni_mlp_bwd_workspace_bytes(ctypes.byref(d)) // 4, device=dev, dtype=torch.float32)
        ev = KernelTimer.start()
        check(L.mmni_ln_mlp_bwd(ctypes.byref(d), ctx.eps, ptr(x2), ptr(gamma), ptr(beta), ptr(w1), ptr(b1), ptr(w2),
                                ptr(dy2), int(ctx.residual_x), ptr(dx), ptr(dgamma), ptr(dbeta), ptr(dw1), ptr(db1),
                                ptr(dw2), ptr(db2), ptr(ws), stream_handle(dev)), "mmni_ln_mlp_bwd")
        KernelTimer.stop(f"ln_mlp_bwd_{C}x{H}", ev, 10.0 * rows * C * H, 4.0 * rows * C * 3)
        return (dx.view(ctx.xshape), dgamma, dbeta, dw1, db1 if ctx.has_b[0] else None, dw2,
                db2 if ctx.has_b[1] else None, None, None, dy if ctx.needs_input_grad[9] else None)


def ln_mlp_ok(x, norm, mlp_mod):
    fc1, fc2 = mlp_mod.fc1, mlp_mod.fc2
    H, C = fc1.weight.shape
    return (x.shape[-1] == C and isinstance(norm, torch.nn.LayerNorm) and norm.elementwise_affine
            and norm.bias is not None and isinstance(mlp_mod.act, torch.nn.GELU) and mlp_mod.act.approximate == "none"
            and (mlp_mod.drop.p == 0.0 or not mlp_mod.drop.training) and fc2.weight.shape[0] == C
            and bool(_lib.load().mmni_mlp_supported(C, H)))


def ln_mlp(x, norm, mlp_mod, residual_x=True, skip=None):
    """[x +] mlp_mod(norm(x)) [+ skip] for an Mlp / Mlp_fusion module (fc1, act, fc2, drop), fused
    into one kernel per direction when ln_mlp_ok; else LayerNorm + the MLP path.  skip is the
    identity skip of a residual group ending with this block (swinfusion_module.py:814,918-927),
    added in the same epilogue instead of by a separate full-size add."""
    require_device(x, what="ln_mlp")
    if skip is not None and (skip.shape != x.shape or skip.dtype != torch.float32):
        raise ValueError(f"ln_mlp: skip {tuple(skip.shape)} {skip.dtype} must match x {tuple(x.shape)} float32")
    if ln_mlp_ok(x, norm, mlp_mod):
        return _LnMlp.apply(x, norm.weight, norm.bias, mlp_mod.fc1.weight, mlp_mod.fc1.bias, mlp_mod.fc2.weight,
                            mlp_mod.fc2.bias, float(norm.eps), residual_x, skip)
    y = mlp(layer_norm(x, norm), mlp_mod.fc1, mlp_mod.fc2, mlp_mod.act, mlp_mod.drop,
            residual=x if residual_x else None)
    return y if skip is None else y + skip


def mlp(x, fc1, fc2, act, drop, residual=None):
    """The reference Mlp forward `drop(fc2(drop(act(fc1(x)))))` (+ residual) with the fused HIP
    path when act is exact nn.GELU, the dropouts are inactive and the shapes are compiled; else
    per-layer."""
    require_device(x, what="mlp")
    H, C = fc1.weight.shape
    O = fc2.weight.shape[0]
    if (isinstance(act, torch.nn.GELU) and act.approximate == "none" and (drop.p == 0.0 or not drop.training)
            and O == C and _lib.load().mmni_mlp_supported(C, H) and x.shape[-1] == C):
        return _FusedMlp.apply(x, fc1.weight, fc1.bias, fc2.weight, fc2.bias, residual)
    fused = (isinstance(act, torch.nn.GELU) and act.approximate == "none"
             and (drop.p == 0.0 or not drop.training)
             and _tlin_ok(C, H, 1) and _tlin_ok(O, H, 2, C) and _tlin_ok(H, C) and _tlin_ok(H, O)
             and ((H + 15) // 16, (C + 15) // 16) in _DW_TILES and ((O + 15) // 16, (H + 15) // 16) in _DW_TILES)
    if not fused:
        y = drop(linear(drop(act(linear(x, fc1))), fc2))
        return y if residual is None else residual + y
    return _Mlp.apply(x, fc1.weight, fc1.bias, fc2.weight, fc2.bias, residual)


# ----------------------------------------------------------------------------------------
# fused LayerNorm -> Linear (norm1 + attn.qkv / q / kv of a SwinFusion block, blockops.hip)
# ----------------------------------------------------------------------------------------
TOK_C = 12
TOK_LN_N = (12, 24, 36)


def _tok_desc(rows, C, N, eps=0.0):
    d = _lib.TokDesc()
    d.rows, d.C, d.N, d.eps = rows, C, N, eps
    return d


class _LnLinear(torch.autograd.Function):
    """y = LN(x) W^T + b in one pass; the LayerNorm output never reaches HBM (the backward
    recomputes it from x and the saved row statistics).  With passthrough=1 the Function also
    returns x itself (a view) to be used as the block's residual: its gradient arrives here and is
    added inside the fused backward instead of by a separate autograd add.  passthrough=2 returns
    a second view for the identity skip of the residual group this block opens (RSTB / CRSTB),
    whose gradient joins in the same kernel (mmni_ln_linear_bwd2)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, w, b, eps, passthrough):
        N, C = w.shape
        x2 = x.reshape(-1, C).contiguous()
        rows = x2.shape[0]
        y = torch.empty(rows, N, device=x2.device, dtype=torch.float32)
        mean = torch.empty(rows, device=x2.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x2.device, dtype=torch.float32)
        d = _tok_desc(rows, C, N, eps)
        ev = KernelTimer.start()
        check(_lib.load().mmni_ln_linear_fwd(ctypes.byref(d), ptr(x2), ptr(gamma), ptr(beta), ptr(w), ptr(b), ptr(y),
                                             ptr(mean), ptr(rstd), stream_handle(x2.device)), "mmni_ln_linear_fwd")
        # algorithmic: LN (~8 flops/elt) + 2*rows*C*N; bytes: x in, y + mean/rstd out
        KernelTimer.stop(f"ln_linear_fwd_{C}x{N}", ev, 2.0 * rows * C * N + 8.0 * rows * C,
                         4.0 * rows * (C + N + 2))
        ctx.save_for_backward(x2, gamma, beta, w, mean, rstd)
        ctx.has_b = b is not None
        ctx.xshape = x.shape
        y = y.view(*x.shape[:-1], N)
        if passthrough == 2:
            return y, x.view(x.shape), x.view(x.shape)
        return (y, x.view(x.shape)) if passthrough else y

    @staticmethod
    def backward(ctx, dy, dres=None, dres2=None):
        x2, gamma, beta, w, mean, rstd = ctx.saved_tensors
        N, C = w.shape
        rows = x2.shape[0]
        dy2 = dy.reshape(-1, N).contiguous()
        dr2 = dres.reshape(-1, C).contiguous() if dres is not None else None
        ds2 = dres2.reshape(-1, C).contiguous() if dres2 is not None else None
        dx = torch.empty(rows, C, device=x2.device, dtype=torch.float32)
        dw = torch.empty_like(w)
        db = torch.empty(N, device=x2.device, dtype=torch.float32) if ctx.has_b else None
        dgamma = torch.empty(C, device=x2.device, dtype=torch.float32)
        dbeta = torch.empty(C, device=x2.device, dtype=torch.float32)
        L = _lib.load()
        d = _tok_desc(rows, C, N)
        ws = torch.empty(L.mmni_tok_bwd_workspace_bytes(ctypes.byref(d)) // 4, device=x2.device, dtype=torch.float32)
        ev = KernelTimer.start()
        if ds2 is None:
            check(L.mmni_ln_linear_bwd(ctypes.byref(d), ptr(dy2), ptr(x2), ptr(mean), ptr(rstd), ptr(gamma),
                                       ptr(beta), ptr(w), ptr(dr2), ptr(dx), ptr(dw), ptr(db), ptr(dgamma), ptr(dbeta),
                                       ptr(ws), stream_handle(x2.device)), "mmni_ln_linear_bwd")
        else:
            check(L.mmni_ln_linear_bwd2(ctypes.byref(d), ptr(dy2), ptr(x2), ptr(mean), ptr(rstd), ptr(gamma),
                                        ptr(beta), ptr(w), ptr(dr2), ptr(ds2), ptr(dx), ptr(dw), ptr(db), ptr(dgamma),
                                        ptr(dbeta), ptr(ws), stream_handle(x2.device)), "mmni_ln_linear_bwd2")
        nres = (dr2 is not None) + (ds2 is not None)
        KernelTimer.stop(f"ln_linear_bwd_{C}x{N}", ev, 4.0 * rows * C * N + 16.0 * rows * C,
                         4.0 * rows * (N + 2 * C + 2 + C * nres))
        return dx.view(ctx.xshape), dgamma, dbeta, dw, db, None, None


def ln_linear_ok(x, norm, lin):
    return (x.shape[-1] == TOK_C and isinstance(norm, torch.nn.LayerNorm) and norm.elementwise_affine
            and norm.bias is not None and lin.weight.shape[1] == TOK_C and lin.weight.shape[0] in TOK_LN_N)


def ln_linear(x, norm, lin, passthrough=False):
    """lin(norm(x)) fused (x (..., 12), lin 12 -> 12/24/36); other shapes run LayerNorm and Linear
    as separate HIP kernels.  passthrough=True (1) also returns x for use as the residual, 2 returns
    it twice (residual, residual-group skip) (see _LnLinear)."""
    require_device(x, what="ln_linear")
    if ln_linear_ok(x, norm, lin):
        return _LnLinear.apply(x, norm.weight, norm.bias, lin.weight, lin.bias, float(norm.eps), int(passthrough))
    y = linear(layer_norm(x, norm), lin)
    if passthrough == 2:
        return y, x, x
    return (y, x) if passthrough else y


def _linear_bwd_fused(x2, dy2, weight, with_bias):
    """dx, dW, db of a 12 -> 12 token Linear in one pass over (dy, x) (blockops.hip)."""
    rows = x2.shape[0]
    C = TOK_C
    dx = torch.empty(rows, C, device=x2.device, dtype=torch.float32)
    dw = torch.empty_like(weight)
    db = torch.empty(C, device=x2.device, dtype=torch.float32) if with_bias else None
    L = _lib.load()
    d = _tok_desc(rows, C, C)
    ws = torch.empty(L.mmni_tok_bwd_workspace_bytes(ctypes.byref(d)) // 4, device=x2.device, dtype=torch.float32)
    ev = KernelTimer.start()
    check(L.mmni_linear_bwd(ctypes.byref(d), ptr(dy2), ptr(x2), ptr(weight), ptr(dx), ptr(dw), ptr(db), ptr(ws),
                            stream_handle(x2.device)), "mmni_linear_bwd")
    KernelTimer.stop(f"linear_bwd_{C}x{C}", ev, 4.0 * rows * C * C, 4.0 * rows * C * 3)
    return dx, dw, db


def linear(x, lin_or_weight, bias=None, residual=None):
    """Token Linear (+ residual) with the HIP kernels when the shape is compiled."""
    if isinstance(lin_or_weight, torch.nn.Linear):
        weight, bias = lin_or_weight.weight, lin_or_weight.bias
    else:
        weight = lin_or_weight
    require_device(x, what="linear")
    N, K = weight.shape
    if ((N + 15) // 16, (K + 15) // 16) not in _DW_TILES or K % 4:
        return _RowLinear.apply(x, weight, bias, residual)   # any shape, fp32, on the row-GEMM kernels
    return _TokenLinear.apply(x, weight, bias, residual)


class _RowLinear(torch.autograd.Function):
    """y = x W^T + b (+ residual) for the token-Linear shapes the tiled token kernels do not
    compile (the Swin-V2 deep stages' widths, PatchMerging reductions, heads): forward and dX on
    mmni_rowgemm, dW / db on mmni_rowgemm_dw (deterministic).  These ran as one-workgroup library
    GEMMs of ~11-13 us each at the deep stages' few hundred rows."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual):
        N, K = weight.shape
        x2 = _rows2d(x, K).contiguous()
        r2 = residual.reshape(-1, N).contiguous() if residual is not None else None
        y = rowgemm(x2, weight.contiguous(), bias, res=r2)
        ctx.save_for_backward(x2, weight)
        ctx.has_bias, ctx.xshape, ctx.has_res = bias is not None, x.shape, residual is not None
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        N, K = weight.shape
        dy2 = _rows2d(dy, N).contiguous()
        dx = rowgemm(dy2, weight.contiguous(), transpose_w=True).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        dw, db = rowgemm_dw(x2, dy2, N, K, ctx.has_bias)
        return dx, dw, db, (dy if ctx.has_res and ctx.needs_input_grad[3] else None)


# ------------------------------------------------------------------------------------------
# split-K weight gradient for the crossmodal encoder's Linears
# ------------------------------------------------------------------------------------------
def _splitk_chunks(rows):
    """Row chunks of a split-K weight gradient: the largest S <= 64 dividing `rows` with >= 256 rows
    per chunk (1: no split)."""
    best = 1
    for S in range(2, 65):
        if rows % S == 0 and rows // S >= 256:
            best = S
    return best


class _SplitKLinear(torch.autograd.Function):
    """y = x W^T + b whose weight gradient contracts over the token rows in S chunks (one batched
    GEMM of S small products, then a fixed-order fp32 sum over S; deterministic).  dW = dY^T X has a
    tiny N x K output and K = T*B = 6,912 (C4) to 32,768 (C5) rows, where the library's single
    GEMM tiles only the output and runs a few dozen workgroups (57-114 us a call, profiles/).
    Under bf16 autocast the products run in bf16 like F.linear's; the gradients come back in the
    parameters' own dtype.  The autocast casts of x and W are made once, in the forward, and the bf16
    copies are what the backward keeps (no re-cast per backward).  On the device the chunk-order
    sum of dW's partials and the column sums of db run in one HIP launch pair reading the bf16
    values directly (mmni_splitk_reduce; torch's two reductions took 24 us per Linear at C5)."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu=False):
        ctx.x_dtype = x.dtype
        if torch.is_autocast_enabled() and x.is_cuda:
            cdt = torch.get_autocast_dtype("cuda")
            xc, wc = x.to(cdt), _autocast_copy(weight, cdt)
            bc = _autocast_copy(bias, cdt)
        else:
            xc, wc, bc = x, weight, bias
        with torch.autocast(device_type="cuda", enabled=False):
            if relu and bc is not None and xc.is_cuda:
                # ReLU in the GEMM's epilogue (crossmodal_transformer.py:160 F.relu(self.fc1(x)))
                K = xc.shape[-1]
                y = torch._addmm_activation(bc, xc.reshape(-1, K), wc.t()).view(*xc.shape[:-1], wc.shape[0])
            else:
                y = F.linear(xc, wc, bc)
                if relu:
                    y = F.relu(y)
        if relu:
            ctx.save_for_backward(xc, wc, y)
        else:
            ctx.save_for_backward(xc, wc)
        ctx.relu = relu
        ctx.w_dtype = weight.dtype
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        if ctx.relu:
            x, w, y = ctx.saved_tensors
            dy = torch.ops.aten.threshold_backward(dy, y, 0)
        else:
            x, w = ctx.saved_tensors
        cdt = dy.dtype
        N, K = w.shape
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (dy @ w.to(cdt)).to(ctx.x_dtype)
        dy2 = dy.reshape(-1, N)
        x2 = x.reshape(-1, K).to(cdt)
        rows = dy2.shape[0]
        S = _splitk_chunks(rows)
        if dy.is_cuda and cdt in (torch.float32, torch.bfloat16):
            dw = torch.empty(N, K, device=dy.device, dtype=torch.float32)
            db = torch.empty(N, device=dy.device, dtype=torch.float32) if ctx.has_bias else None
            _splitk_wgrad(dy2, x2, dw, db)
            return dx, dw.to(ctx.w_dtype), (db.to(ctx.w_dtype) if db is not None else None), None
        # CPU tensors (the float64 gradient tests): the same chunking in torch
        acc = torch.promote_types(cdt, torch.float32)   # fp32 sums (fp64 stays fp64)
        if S > 1:
            r = rows // S
            dw = torch.bmm(dy2.view(S, r, N).transpose(1, 2), x2.view(S, r, K)).sum(0, dtype=acc)
        else:
            dw = (dy2.t() @ x2).to(acc)
        db = dy2.sum(0, dtype=acc).to(ctx.w_dtype) if ctx.has_bias else None
        return dx, dw.to(ctx.w_dtype), db, None


# bf16 copies of fp32 parameters made for the current step (cast_params_bf16), looked up by the
# autocast Linears instead of casting each weight and bias in its own launch
_BF16_CACHE = {}


def cast_params_bf16(params):
    """bf16 copies of fp32 device parameters, up to 64 per HIP launch (mmni_cast_bf16_multi), kept
    for this step's autocast Linears (_autocast_copy hands them out while the parameter's version
    is unchanged; an optimizer step bumps it, so a stale copy is never used)."""
    params = [p for p in params if p is not None and p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()]
    for k in [k for k, e in _BF16_CACHE.items() if e[0]() is None]:   # parameters that no longer exist
        del _BF16_CACHE[k]
    L = _lib.load()
    for i in range(0, len(params), 64):
        chunk = params[i:i + 64]
        offs, total = [], 0
        for p in chunk:   # 128-byte aligned pieces (the GEMMs' operand pointers)
            offs.append(total)
            total += (p.numel() + 63) // 64 * 64
        flat = torch.empty(total, device=chunk[0].device, dtype=torch.bfloat16)
        dsts = [flat[o:o + p.numel()].view(p.shape) for o, p in zip(offs, chunk)]
        n = len(chunk)
        src = (ctypes.c_void_p * n)(*[p.data_ptr() for p in chunk])
        dst = (ctypes.c_void_p * n)(*[d.data_ptr() for d in dsts])
        cnt = (ctypes.c_int64 * n)(*[p.numel() for p in chunk])
        check(L.mmni_cast_bf16_multi(n, src, dst, cnt, stream_handle(chunk[0].device)), "mmni_cast_bf16_multi")
        for p, d in zip(chunk, dsts):
            _BF16_CACHE[(p.data_ptr(), tuple(p.shape))] = (weakref.ref(p), p._version, d)


def _autocast_copy(t, cdt):
    """t.to(cdt), or this step's bf16 copy from cast_params_bf16 when it is current."""
    if t is None:
        return None
    if cdt == torch.bfloat16 and t.dtype == torch.float32:
        e = _BF16_CACHE.get((t.data_ptr(), tuple(t.shape)))
        if e is not None and e[0]() is t and e[1] == t._version:   # the same live tensor, unmodified
            return e[2]
    return t.to(cdt)


def _splitk_wgrad(dy2, x2, dw, db):
    """dw (N, K) = dy2^T x2 and db (N) = colsum dy2 (nullable) into fp32 destinations (contiguous
    row blocks of a larger gradient are fine): the S chunk products on the library GEMM, their
    chunk-order sum and db in one HIP launch pair (mmni_splitk_reduce, splitk.hip)."""
    rows, N = dy2.shape
    K = x2.shape[1]
    S = _splitk_chunks(rows)
    if S > 1:
        r = rows // S
        part = torch.bmm(dy2.view(S, r, N).transpose(1, 2), x2.view(S, r, K))
    else:
        part = dy2.t() @ x2
    dy2 = dy2.contiguous()
    L = _lib.load()
    ws = _workspace(L.mmni_splitk_reduce_workspace_bytes(rows, N), dy2.device) if db is not None else None
    ev = KernelTimer.start()
    check(L.mmni_splitk_reduce(S, N * K, ptr(part.contiguous()), rows, N, ptr(dy2), N,
                               1 if dy2.dtype == torch.bfloat16 else 0, ptr(dw), ptr(db), ptr(ws),
                               stream_handle(dy2.device)), "mmni_splitk_reduce")
    KernelTimer.stop(f"splitk_reduce_{N}x{K}", ev, float(S * N * K + rows * N),
                     float(part.element_size() * (S * N * K + rows * N) + 4 * (N * K + N)))


class _InProjQKV(torch.autograd.Function):
    """The cross-attention in_proj of MultiheadAttention (multihead_attention.py:71-84 in_proj_q /
    in_proj_kv on one packed (3E, E) weight): q = x_q W[:E]^T + b[:E], kv = x_kv W[E:]^T + b[E:]
    in one autograd node, so the weight and bias gradients are written as row blocks of one
    (3E, E) / (3E) gradient (no zero-filled slice gradients and accumulation adds) and the autocast
    casts of W and b happen once.  Weight gradients as _SplitKLinear (split-K, deterministic)."""

    @staticmethod
    def forward(ctx, xq, xkv, weight, bias):
        E = weight.shape[1]
        ctx.dtypes = (xq.dtype, xkv.dtype, weight.dtype)
        if torch.is_autocast_enabled() and xq.is_cuda:
            cdt = torch.get_autocast_dtype("cuda")
            xq, xkv, wc = xq.to(cdt), xkv.to(cdt), _autocast_copy(weight, cdt)
            bc = _autocast_copy(bias, cdt)
        else:
            wc, bc = weight, bias
        with torch.autocast(device_type="cuda", enabled=False):
            q = F.linear(xq, wc[:E], bc[:E] if bc is not None else None)
            kv = F.linear(xkv, wc[E:], bc[E:] if bc is not None else None)
        ctx.save_for_backward(xq, xkv, wc)
        ctx.has_bias = bias is not None
        return q, kv

    @staticmethod
    def backward(ctx, dq, dkv):
        xq, xkv, wc = ctx.saved_tensors
        xq_dtype, xkv_dtype, w_dtype = ctx.dtypes
        E = wc.shape[1]
        cdt = wc.dtype
        dq = dq.to(cdt)
        dkv = dkv.to(cdt)
        dxq = (dq @ wc[:E]).to(xq_dtype) if ctx.needs_input_grad[0] else None
        dxkv = (dkv @ wc[E:]).to(xkv_dtype) if ctx.needs_input_grad[1] else None
        dw = torch.empty(3 * E, E, device=wc.device, dtype=torch.float32)
        db = torch.empty(3 * E, device=wc.device, dtype=torch.float32) if ctx.has_bias else None
        _splitk_wgrad(dq.reshape(-1, E), xq.reshape(-1, E), dw[:E], db[:E] if db is not None else None)
        _splitk_wgrad(dkv.reshape(-1, 2 * E), xkv.reshape(-1, E), dw[E:], db[E:] if db is not None else None)
        return dxq, dxkv, dw.to(w_dtype), (db.to(w_dtype) if db is not None else None)


def in_proj_q_kv(xq, xkv, weight, bias=None):
    """(q, kv) = the cross-attention in_proj of one packed weight (see _InProjQKV); device only."""
    require_device(xq, xkv, weight, bias, what="in_proj_q_kv", dtypes=(torch.float32, torch.bfloat16))
    return _InProjQKV.apply(xq, xkv, weight, bias)


def mha_packed(q_src, kv_src, heads, causal_diag=0, scale=None, dropout=0.0, seed=None):
    """The attention core on packed projections (T, B, 3E) qkv (kv_src None: self attention) or
    (Tq, B, E) q + (Tk, B, 2E) kv: no slice copies forward, packed gradients backward (_MHARows).
    Returns the (Tq, B, E) output in the projections' dtype."""
    Tq, B = q_src.shape[0], q_src.shape[1]
    E = q_src.shape[-1] // 3 if kv_src is None else q_src.shape[-1]
    if scale is None:
        scale = (E // heads) ** -0.5
    if dropout > 0 and seed is None:
        seed = dropout_seed()
    q2 = _rows_view(q_src, q_src.shape[-1])
    kv2 = q2 if kv_src is None else _rows_view(kv_src, kv_src.shape[-1])
    Tk = Tq if kv_src is None else kv_src.shape[0]
    return _MHARows.apply(q2, kv2, Tq, Tk, B, heads, causal_diag, scale, float(dropout), int(seed or 0))


def splitk_linear(x, weight, bias=None, relu=False):
    """F.linear (F.relu of it with relu=True) with the split-K weight gradient (see _SplitKLinear)."""
    return _SplitKLinear.apply(x, weight, bias, relu)


class SplitKLinear(torch.nn.Linear):
    """nn.Linear (same parameters and state_dict keys) with the split-K weight gradient."""

    def forward(self, x):
        return _SplitKLinear.apply(x, self.weight, self.bias)


# ------------------------------------------------------------------------------------------
# crossmodal encoder layer on the HIP row-GEMM kernels (encoder.hip, ABI v6)
# ------------------------------------------------------------------------------------------
def _rg_desc(rows, K, N, ldx, ldy, w_sn, w_sk, ln=False, eps=0.0, relu=False, ldres=0, ldaux=0):
    d = _lib.RowGemmDesc()
    d.rows, d.K, d.N = int(rows), int(K), int(N)
    d.ldx, d.ldy, d.ldres, d.ldaux = int(ldx), int(ldy), int(ldres), int(ldaux)
    d.w_sn, d.w_sk = int(w_sn), int(w_sk)
    d.ln, d.eps, d.relu = int(bool(ln)), float(eps), int(bool(relu))
    return d


def _rows_view(t, C):
    """(rows, C) view of a tensor whose last dim is C with unit column stride and a uniform row
    stride (contiguous time-major (T, B, C) tensors and column slices of packed rows)."""
    if t.dim() == 2:
        assert t.stride(1) == 1
        return t
    t2 = t.reshape(-1, C)
    assert t2.stride(1) == 1
    return t2


class _CpbTable(torch.autograd.Function):
    """16 * sigmoid(cpb_mlp(relative_coords_table)) for a Swin-V2 WindowAttention
    (swin_v2_module.py:88-91,158-162) in one HIP launch per direction (mmni_cpb_fwd / _bwd, cpb.hip):
    Linear(nd, hidden) -> ReLU -> Linear(hidden, heads, no bias) -> 16 * sigmoid.  The coordinate
    table is a constant buffer (no gradient); dW1 / db1 / dW2 are fixed-order sums (deterministic)."""

    @staticmethod
    def forward(ctx, coords, w1, b1, w2):
        require_device(coords, w1, b1, w2)
        coords = coords.reshape(-1, coords.shape[-1]).contiguous()
        w1, b1, w2 = w1.contiguous(), b1.contiguous(), w2.contiguous()
        tsz, nd = coords.shape
        hidden, heads = w1.shape[0], w2.shape[0]
        out = torch.empty(tsz, heads, device=coords.device, dtype=torch.float32)
        check(_lib.load().mmni_cpb_fwd(tsz, nd, hidden, heads, ptr(coords), ptr(w1), ptr(b1), ptr(w2), ptr(out),
                                       stream_handle(coords.device)), "mmni_cpb_fwd")
        ctx.save_for_backward(coords, w1, b1, w2, out)
        return out

    @staticmethod
    def backward(ctx, dout):
        coords, w1, b1, w2, out = ctx.saved_tensors
        tsz, nd = coords.shape
        hidden, heads = w1.shape[0], w2.shape[0]
        dout = dout.contiguous()
        dw1, db1, dw2 = torch.empty_like(w1), torch.empty_like(b1), torch.empty_like(w2)
        L = _lib.load()
        ws = _workspace(L.mmni_cpb_bwd_workspace_bytes(tsz, nd, hidden, heads), coords.device)
        check(L.mmni_cpb_bwd(tsz, nd, hidden, heads, ptr(coords), ptr(w1), ptr(b1), ptr(w2), ptr(out), ptr(dout),
                             ptr(dw1), ptr(db1), ptr(dw2), ptr(ws), stream_handle(coords.device)), "mmni_cpb_bwd")
        return None, dw1, db1, dw2


def cpb_table(coords, w1, b1, w2):
    """(tsz, heads) = 16 * sigmoid(W2 relu(W1 coords + b1)) on the HIP kernels (fp32)."""
    return _CpbTable.apply(coords, w1, b1, w2)


def rowgemm(x2, w, bias=None, *, ln=None, relu=False, aux=None, res=None, transpose_w=False, stats=False):
    """y = epi(x' W^T) on token rows with the HIP row-GEMM (mmni_rowgemm).

    x2 (rows, K) with unit column stride; w an nn.Linear weight (N, K), or with transpose_w a weight
    (K_lin = N_out, N_lin = K) whose input gradient dY W this is.  ln = (gamma, beta, eps): LayerNorm
    prologue over the K columns; stats=True also returns the row (mean, rstd).  Epilogue: + bias,
    ReLU, * (aux > 0), + res (rows, N)."""
    require_device(x2, w, what="rowgemm")
    rows, K = x2.shape
    if transpose_w:
        Kw, N = w.shape
        w_sn, w_sk = 1, w.stride(0)
        assert w.stride(1) == 1 and Kw == K
    else:
        N, Kw = w.shape
        w_sn, w_sk = w.stride(0), 1
        assert w.stride(1) == 1 and Kw == K
    y = torch.empty(rows, N, device=x2.device, dtype=torch.float32)
    mean = rstd = None
    gamma = beta = None
    eps = 0.0
    if ln is not None:
        gamma, beta, eps = ln
        if stats:
            mean = torch.empty(rows, device=x2.device, dtype=torch.float32)
            rstd = torch.empty(rows, device=x2.device, dtype=torch.float32)
    d = _rg_desc(rows, K, N, x2.stride(0), N, w_sn, w_sk, ln is not None, eps, relu,
                 res.stride(0) if res is not None else 0, aux.stride(0) if aux is not None else 0)
    ev = KernelTimer.start()
    check(_lib.load().mmni_rowgemm(ctypes.byref(d), ptr(x2), ptr(gamma), ptr(beta), ptr(w), ptr(bias), ptr(aux),
                                   ptr(res), ptr(y), ptr(mean), ptr(rstd), stream_handle(x2.device)), "mmni_rowgemm")
    KernelTimer.stop(f"rowgemm_{K}x{N}{'_ln' if ln is not None else ''}", ev, 2.0 * rows * K * N,
                     4.0 * rows * (K + N + (N if res is not None else 0) + (N if aux is not None else 0)))
    return (y, mean, rstd) if stats else y


def rowgemm_dw(x2, dy2, N, K, with_bias, ln=None, mean=None, rstd=None, out=None):
    """dW (N, K) = dY^T X' and db (N) = colsum dY over token rows (fixed-order, deterministic);
    X' = LayerNorm(X) recomputed from the forward's row statistics when ln = (gamma, beta, eps).
    out = (dw, db): contiguous destinations (e.g. row blocks of a larger weight's gradient)."""
    rows = x2.shape[0]
    if out is not None:
        dw, db = out
    else:
        dw = torch.empty(N, K, device=x2.device, dtype=torch.float32)
        db = torch.empty(N, device=x2.device, dtype=torch.float32) if with_bias else None
    gamma = beta = None
    if ln is not None:
        gamma, beta, _ = ln
    d = _rg_desc(rows, K, N, x2.stride(0), dy2.stride(0), K, 1, ln is not None)
    L = _lib.load()
    ws = _workspace(L.mmni_rowgemm_dw_workspace_bytes(ctypes.byref(d)), x2.device)
    ev = KernelTimer.start()
    check(L.mmni_rowgemm_dw(ctypes.byref(d), ptr(x2), ptr(gamma), ptr(beta), ptr(mean), ptr(rstd), ptr(dy2), ptr(dw),
                            ptr(db), ptr(ws), stream_handle(x2.device)), "mmni_rowgemm_dw")
    KernelTimer.stop(f"rowgemm_dw_{N}x{K}", ev, 2.0 * rows * K * N, 4.0 * rows * (K + N))
    return dw, db


def row_layernorm_bwd(dxn2, x2, gamma, mean, rstd, dres2=None):
    """dX of a LayerNorm over the C columns of token rows from dL/d(LN output) (+ dres), and
    dgamma / dbeta (fixed-order sums)."""
    rows, C = x2.shape
    dx = torch.empty(rows, C, device=x2.device, dtype=torch.float32)
    dgamma = torch.empty(C, device=x2.device, dtype=torch.float32)
    dbeta = torch.empty(C, device=x2.device, dtype=torch.float32)
    L = _lib.load()
    ws = _workspace(L.mmni_row_layernorm_bwd_workspace_bytes(rows, C), x2.device)
    ev = KernelTimer.start()
    check(L.mmni_row_layernorm_bwd_t(rows, C, ptr(dxn2), 1 if dxn2.dtype == torch.bfloat16 else 0, dxn2.stride(0),
                                     ptr(x2), x2.stride(0), ptr(gamma), ptr(mean), ptr(rstd), ptr(dres2),
                                     dres2.stride(0) if dres2 is not None else 0, ptr(dx), C, ptr(dgamma), ptr(dbeta),
                                     ptr(ws), stream_handle(x2.device)), "mmni_row_layernorm_bwd")
    KernelTimer.stop(f"row_ln_bwd_C{C}", ev, 10.0 * rows * C, 4.0 * rows * C * (4 if dres2 is not None else 3))
    return dx, dgamma, dbeta


class _RowLnQKV(torch.autograd.Function):
    """LayerNorm0 + in_proj of one encoder layer (crossmodal_transformer.py:145,150-151 +
    multihead_attention.py:71-84) on token rows, LN fused into the projection (one launch per
    input; the LN output is recomputed in the backward from the saved row statistics).
      self attention (x_kv None): qkv = LN(x) W^T + b (N = 3E); returns (qkv, None, x)
      cross attention:            q = LN(x) W[:E]^T + b[:E], kv = LN(x_kv) W[E:]^T + b[E:];
                                  returns (q, kv, x)
    The third output is x itself (a view) for the layer's residual: its gradient arrives here and
    joins the LayerNorm backward in one kernel instead of an autograd add.  The weight gradient is
    written per row block of the whole in_proj_weight (no slice scatter)."""

    @staticmethod
    def forward(ctx, x, x_kv, gamma, beta, w, b, eps):
        E = x.shape[-1]
        x2 = _rows_view(x, E).contiguous()
        ln = (gamma, beta, eps)
        if x_kv is None:
            qkv, mean, rstd = rowgemm(x2, w, b, ln=ln, stats=True)
            ctx.save_for_backward(x2, gamma, beta, w, mean, rstd)
            q_out, kv_out = qkv, None
        else:
            k2 = _rows_view(x_kv, E).contiguous()
            q_out, mean, rstd = rowgemm(x2, w[:E], b[:E] if b is not None else None, ln=ln, stats=True)
            kv_out, mean_k, rstd_k = rowgemm(k2, w[E:], b[E:] if b is not None else None, ln=ln, stats=True)
            ctx.save_for_backward(x2, gamma, beta, w, mean, rstd, k2, mean_k, rstd_k)
        ctx.eps, ctx.has_b, ctx.xshape, ctx.kvshape = eps, b is not None, x.shape, (x_kv.shape if x_kv is not None
                                                                                    else None)
        return q_out, kv_out, x.view(x.shape)

    @staticmethod
    def backward(ctx, dq, dkv, dres):
        E = ctx.xshape[-1]
        ln_of = lambda g, b: (g, b, ctx.eps)  # noqa: E731
        dres2 = _rows_view(dres, E).contiguous() if dres is not None else None
        if ctx.kvshape is None:
            x2, gamma, beta, w, mean, rstd = ctx.saved_tensors
            dq2 = dq.contiguous()
            dw, db = rowgemm_dw(x2, dq2, 3 * E, E, ctx.has_b, ln=ln_of(gamma, beta), mean=mean, rstd=rstd)
            dxn = rowgemm(dq2, w, transpose_w=True)
            dx, dgamma, dbeta = row_layernorm_bwd(dxn, x2, gamma, mean, rstd, dres2)
            return dx.view(ctx.xshape), None, dgamma, dbeta, dw, db, None
        x2, gamma, beta, w, mean, rstd, k2, mean_k, rstd_k = ctx.saved_tensors
        dw = torch.empty_like(w)
        db = torch.empty(3 * E, device=w.device, dtype=torch.float32) if ctx.has_b else None
        ln = ln_of(gamma, beta)
        dq2 = dq.contiguous()
        rowgemm_dw(x2, dq2, E, E, ctx.has_b, ln=ln, mean=mean, rstd=rstd,
                   out=(dw[:E], db[:E] if db is not None else None))
        dxn = rowgemm(dq2, w[:E], transpose_w=True)
        dx, dgamma, dbeta = row_layernorm_bwd(dxn, x2, gamma, mean, rstd, dres2)
        dx_kv = None
        if dkv is not None:
            dkv2 = dkv.contiguous()
            rowgemm_dw(k2, dkv2, 2 * E, E, ctx.has_b, ln=ln, mean=mean_k, rstd=rstd_k,
                       out=(dw[E:], db[E:] if db is not None else None))
            dxn_k = rowgemm(dkv2, w[E:], transpose_w=True)
            dx_kv, dgk, dbk = row_layernorm_bwd(dxn_k, k2, gamma, mean_k, rstd_k)
            dgamma, dbeta = dgamma + dgk, dbeta + dbk
            dx_kv = dx_kv.view(ctx.kvshape)
        else:
            dw[E:].zero_()
            if db is not None:
                db[E:].zero_()
        return dx.view(ctx.xshape), dx_kv, dgamma, dbeta, dw, db, None


class _RowLinearResidual(torch.autograd.Function):
    """y = res + x W^T + b on token rows (out_proj + the residual add,
    multihead_attention.py:129, crossmodal_transformer.py:153-154)."""

    @staticmethod
    def forward(ctx, x, w, b, res):
        K = x.shape[-1]
        N = w.shape[0]
        x2 = _rows_view(x, K).contiguous()
        r2 = _rows_view(res, N).contiguous()
        y = rowgemm(x2, w, b, res=r2)
        ctx.save_for_backward(x2, w)
        ctx.has_b, ctx.xshape = b is not None, x.shape
        return y.view(*res.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        N, K = w.shape
        dy2 = _rows_view(dy, N).contiguous()
        dw, db = rowgemm_dw(x2, dy2, N, K, ctx.has_b)
        dx = rowgemm(dy2, w, transpose_w=True)
        return dx.view(ctx.xshape), dw, db, dy


class _RowLnFfn(torch.autograd.Function):
    """y = x + fc2(ReLU(fc1(LayerNorm(x)))) on token rows (crossmodal_transformer.py:155-165) in two
    launches (LN + fc1 + bias + ReLU; fc2 + bias + residual); the ReLU output (rows, 4E) is kept for
    the backward, whose ReLU mask is its sign."""

    @staticmethod
    def forward(ctx, x, gamma, beta, w1, b1, w2, b2, eps):
        E = x.shape[-1]
        x2 = _rows_view(x, E).contiguous()
        a, mean, rstd = rowgemm(x2, w1, b1, ln=(gamma, beta, eps), relu=True, stats=True)
        y = rowgemm(a, w2, b2, res=x2)
        ctx.save_for_backward(x2, gamma, beta, w1, w2, a, mean, rstd)
        ctx.eps, ctx.has_b, ctx.xshape = eps, (b1 is not None, b2 is not None), x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, gamma, beta, w1, w2, a, mean, rstd = ctx.saved_tensors
        H, E = w1.shape
        dy2 = _rows_view(dy, E).contiguous()
        dw2, db2 = rowgemm_dw(a, dy2, E, H, ctx.has_b[1])
        dh = rowgemm(dy2, w2, transpose_w=True, aux=a)          # (dY W2) * (a > 0)
        ln = (gamma, beta, ctx.eps)
        dw1, db1 = rowgemm_dw(x2, dh, H, E, ctx.has_b[0], ln=ln, mean=mean, rstd=rstd)
        dxn = rowgemm(dh, w1, transpose_w=True)
        dx, dgamma, dbeta = row_layernorm_bwd(dxn, x2, gamma, mean, rstd, dres2=dy2)
        return dx.view(ctx.xshape), dgamma, dbeta, dw1, db1, dw2, db2, None


class _MHARows(torch.autograd.Function):
    """The fused attention core on projections that stay packed: self attention reads q / k / v as
    column slices of one (T*B, 3E) qkv tensor, cross attention q (T*B, E) and k / v as slices of a
    (Tk*B, 2E) kv tensor; the backward writes dq / dk / dv straight into the packed gradients
    (the kernels take row strides), so no slice copies or gradient scatter run in between.  fp32 or
    bf16 storage (the output and gradients follow it)."""

    @staticmethod
    def forward(ctx, q_src, kv_src, Tq, Tk, B, heads, diag, scale, dropout, seed):
        require_device(q_src, kv_src, what="mha", dtypes=(torch.float32, torch.bfloat16))
        if q_src.dtype != kv_src.dtype:
            raise RuntimeError(f"mha: q / kv dtypes differ ({q_src.dtype}, {kv_src.dtype})")
        packed = q_src is kv_src
        E = q_src.shape[-1] // 3 if packed else q_src.shape[-1]
        qs = q_src.stride(0)
        if packed:
            q, k, v = q_src, q_src[:, E:], q_src[:, 2 * E:]
            ks = vs = qs
        else:
            q, k, v = q_src, kv_src, kv_src[:, E:]
            ks = vs = kv_src.stride(0)
        dt = q_src.dtype
        out = torch.empty((Tq, B, E), device=q_src.device, dtype=dt)
        lse = torch.empty((B, heads, Tq), device=q_src.device, dtype=torch.float32)
        d = _mha_desc(Tq, Tk, B, heads, E // heads, diag, scale, qs, ks, vs, E, dropout, seed, dt)
        lib = _lib.load()
        ws = _workspace(lib.mmni_mha_fwd_workspace_bytes(d), q_src.device)
        ev = KernelTimer.start()
        check(lib.mmni_mha_fwd(d, ptr(q), ptr(k), ptr(v), ptr(out), ptr(lse), ptr(ws), stream_handle(q_src.device)),
              "mmni_mha_fwd")
        sfx = "_bf16" if dt == torch.bfloat16 else ""
        KernelTimer.stop(f"mha_fwd_E{E}{sfx}", ev, 4.0 * Tq * Tk * B * E,
                         q_src.element_size() * B * E * (2 * Tq + 2 * Tk))
        ctx.save_for_backward(q_src, kv_src, out, lse)
        ctx.cfg = (Tq, Tk, B, heads, diag, scale, dropout, seed, packed, E, qs, ks, vs)
        return out

    @staticmethod
    def backward(ctx, dout):
        q_src, kv_src, out, lse = ctx.saved_tensors
        Tq, Tk, B, heads, diag, scale, dropout, seed, packed, E, qs, ks, vs = ctx.cfg
        dout = dout.contiguous().to(q_src.dtype)
        dq_src = torch.empty_like(q_src)
        if packed:
            q, k, v = q_src, q_src[:, E:], q_src[:, 2 * E:]
            dq, dk, dv = dq_src, dq_src[:, E:], dq_src[:, 2 * E:]
            dkv_src = None
        else:
            dkv_src = torch.empty_like(kv_src)
            q, k, v = q_src, kv_src, kv_src[:, E:]
            dq, dk, dv = dq_src, dkv_src, dkv_src[:, E:]
        dt = q_src.dtype
        d = _mha_desc(Tq, Tk, B, heads, E // heads, diag, scale, qs, ks, vs, E, dropout, seed, dt)
        lib = _lib.load()
        ws = _workspace(lib.mmni_mha_bwd_workspace_bytes(d), q_src.device)
        ev = KernelTimer.start()
        check(lib.mmni_mha_bwd(d, ptr(q), ptr(k), ptr(v), ptr(out), ptr(dout), ptr(lse), ptr(dq), ptr(dk), ptr(dv),
                               ptr(ws), stream_handle(q_src.device)), "mmni_mha_bwd")
        sfx = "_bf16" if dt == torch.bfloat16 else ""
        KernelTimer.stop(f"mha_bwd_E{E}{sfx}", ev, 10.0 * Tq * Tk * B * E,
                         q_src.element_size() * B * E * (4 * Tq + 4 * Tk))
        return dq_src, dkv_src, None, None, None, None, None, None, None, None


def encoder_layer_rows(x, x_kv, layer, diag, dropout_p, seed):
    """One pre-norm TransformerEncoderLayer (crossmodal_transformer.py:133-165) on the HIP kernels:
    LN0 + in_proj (q | kv, or qkv for self attention) -> fused attention core -> out_proj +
    residual -> LN1 + fc1 + ReLU -> fc2 + residual.  x (T, B, E); x_kv (Tk, B, E) shared by key and
    value (the encoder passes the same embedded tensor for both), or None for self attention.
    Residual / ReLU dropouts must be inactive (the caller checks)."""
    attn = layer.self_attn
    Tq, B = x.shape[0], x.shape[1]
    ln0, ln1 = layer.layer_norms[0], layer.layer_norms[1]
    q_src, kv_src, x_res = _RowLnQKV.apply(x, x_kv, ln0.weight, ln0.bias, attn.in_proj_weight, attn.in_proj_bias,
                                           float(ln0.eps))
    Tk = Tq if x_kv is None else x_kv.shape[0]
    a = _MHARows.apply(q_src, kv_src if x_kv is not None else q_src, Tq, Tk, B, attn.num_heads_mult, diag,
                       attn.scaling, dropout_p, seed)
    x = _RowLinearResidual.apply(a, attn.out_proj.weight, attn.out_proj.bias, x_res)
    return _RowLnFfn.apply(x, ln1.weight, ln1.bias, layer.fc1.weight, layer.fc1.bias, layer.fc2.weight,
                           layer.fc2.bias, float(ln1.eps))
