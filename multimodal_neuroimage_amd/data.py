"""Input pipeline of the data-parallel hot path.

Replaces what the reference does per subject inside DataLoader workers
(data_preprocess_and_load/datasets.py, dataloaders.py:55-99) with a GPU-side pipeline:

  * `PairLoader`: rank-sharded (ShardSampler = DistributedSampler semantics), drop-last batching
    of volume pairs; a host thread reads each batch from its source (memory-mapped .npy files or a
    seeded synthetic generator) into pinned buffers, a dedicated HIP stream copies them to HBM
    and z-scores them there (`zscore`), and the compute stream waits on an event only when it takes
    the batch: reading, H2D and normalisation of batch i+1 overlap the step on batch i.  No
    per-step host sync (the reference's trainer syncs on .item() every step).
  * `zscore`: scipy.stats.zscore(axis=None) per volume (datasets.py:416, 664), optionally through
    float16 like the reference's `.half()`.
  * `fmri_band_split`: the 'divided_frequency' fMRI preprocessing (datasets.py:665-698): nitime
    FIR high-pass band split into raw / low / ultralow, z-scored, padded to 368, time-major.

All GPU work runs in libmmni.so (preprocess.hip); there is no CPU fallback.
"""
import ctypes
import queue
import threading

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_handle
from .distributed import ShardSampler

FMRI_TR = 0.8
FMRI_LB = 0.0035
FMRI_SEQ = 368
FIR_ORDER = 64


def _require_cuda(t, what):
    if not t.is_cuda or t.dtype != torch.float32:
        raise RuntimeError(f"{what}: expected a float32 ROCm-device tensor (no CPU fallback), got {t.device} "
                           f"{t.dtype}")


def zscore(x, half_round=False, out=None):
    """(n, ...) -> per-leading-index whole-array z-score (ddof 0), on x's device and current stream."""
    _require_cuda(x, "zscore")
    x = x.contiguous()
    n = x.shape[0]
    count = x.numel() // max(n, 1)
    y = torch.empty_like(x) if out is None else out
    L = _lib.load()
    ws = torch.empty(L.mmni_zscore_workspace_bytes(n) // 8, device=x.device, dtype=torch.float64)
    check(L.mmni_zscore(n, count, ptr(x), ptr(y), int(bool(half_round)), ptr(ws), stream_handle(x.device)),
          "mmni_zscore")
    return y


_TAPS = {}


def fir_taps(device, tr=FMRI_TR, lb=FMRI_LB, order=FIR_ORDER):
    """nitime FilterAnalyzer.fir high-pass taps (float64) on `device` (cached)."""
    key = (str(device), tr, lb, order)
    if key not in _TAPS:
        n = order + 1
        buf = (ctypes.c_double * n)()
        check(_lib.load().mmni_fir_highpass_taps(n, lb / ((1.0 / tr) / 2.0), buf), "mmni_fir_highpass_taps")
        _TAPS[key] = torch.tensor(list(buf), dtype=torch.float64).to(device)
    return _TAPS[key]


def fmri_band_split(y, lens=None, seq=FMRI_SEQ, tr=FMRI_TR, lb=FMRI_LB, order=FIR_ORDER):
    """y (B, ROIs, Lmax) fMRI series (cropped [20:] and transposed as datasets.py:665 does), with
    lens (list of B ints, default Lmax) valid samples per subject -> (raw, low, ultralow), each
    (B, seq, ROIs) float32: the reference's fmri_raw / lowfreq / ultralowfreq sequences."""
    _require_cuda(y, "fmri_band_split")
    y = y.contiguous()
    B, R, Lmax = y.shape
    lens = [Lmax] * B if lens is None else [int(v) for v in lens]
    ntaps = order + 1
    if len(lens) != B or any(not (3 * ntaps < v <= Lmax) for v in lens) or Lmax > seq:
        raise ValueError(f"fmri_band_split: need 3*ntaps ({3 * ntaps}) < len <= Lmax ({Lmax}) <= seq ({seq}); "
                         f"got lens {lens}")
    d = _lib.BandSplitDesc()
    d.B, d.R, d.Lmax, d.seq, d.ntaps = B, R, Lmax, seq, ntaps
    lens_d = torch.tensor(lens, dtype=torch.int32).to(y.device, non_blocking=True)
    taps = fir_taps(y.device, tr, lb, order)
    outs = [torch.empty(B, seq, R, device=y.device, dtype=torch.float32) for _ in range(3)]
    check(_lib.load().mmni_fmri_band_split(ctypes.byref(d), ptr(y), ptr(lens_d), ptr(taps), *[ptr(o) for o in outs],
                                           stream_handle(y.device)), "mmni_fmri_band_split")
    return tuple(outs)


# ----------------------------------------------------------------------------------------
# sources
# ----------------------------------------------------------------------------------------
class NpyVolumes:
    """Volumes stored one per .npy file (the reference's per-subject files); read memory-mapped."""

    def __init__(self, paths):
        self.paths = list(paths)
        first = np.load(self.paths[0], mmap_mode="r")
        self.shape = tuple(first.shape)

    def __len__(self):
        return len(self.paths)

    def read_into(self, i, dst):
        a = np.load(self.paths[i], mmap_mode="r")
        if tuple(a.shape) != self.shape:
            raise ValueError(f"{self.paths[i]}: shape {a.shape} != {self.shape}")
        dst.numpy()[...] = a          # one copy, page cache -> pinned staging


class SyntheticVolumes:
    """Seeded N(0,1) volumes, one generator stream per index (reproducible under any sharding)."""

    def __init__(self, n, shape, seed=55555555):
        self.n, self.shape, self.seed = n, tuple(shape), seed

    def __len__(self):
        return self.n

    def read_into(self, i, dst):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        dst.copy_(torch.randn(self.shape, generator=g))


# ----------------------------------------------------------------------------------------
# loader
# ----------------------------------------------------------------------------------------
class PairLoader:
    """Batches of (A, B, labels) on `device`, rank-sharded, prefetched and z-scored on the GPU.

    sources: two volume sources of equal length (e.g. sMRI and fMRI-derived volumes); labels:
    sequence of per-subject targets.  Each rank sees len // world subjects per epoch (drop_last,
    like the reference's DistributedSampler + drop_last loaders); batches of `batch`, a short
    last batch dropped when drop_last.  `half_round` reproduces the reference's fp16 inputs."""

    def __init__(self, sources, labels, batch, device, rank=0, world=1, shuffle=True, seed=0, drop_last=True,
                 prefetch=2, half_round=False):
        a, b = sources
        if len(a) != len(b) or len(a) != len(labels) or a.shape != b.shape:
            raise ValueError("PairLoader: sources / labels disagree in length or shape")
        self.a, self.b = a, b
        self.labels = torch.as_tensor(labels, dtype=torch.float32).reshape(len(labels), -1)
        self.batch, self.device = batch, torch.device(device)
        self.sampler = ShardSampler(len(a), rank, world, shuffle=shuffle, seed=seed, drop_last=True)
        self.drop_last, self.prefetch, self.half_round = drop_last, max(1, prefetch), half_round
        self.copy_stream = torch.cuda.Stream(self.device)
        shape = (batch,) + tuple(a.shape)
        # pinned staging + device slots, one per in-flight batch (+1 for the one being consumed)
        nslots = self.prefetch + 1
        self._host = [(torch.empty(shape).pin_memory(), torch.empty(shape).pin_memory()) for _ in range(nslots)]
        self._dev = [(torch.empty(shape, device=self.device), torch.empty(shape, device=self.device))
                     for _ in range(nslots)]
        self._lab_host = [torch.empty((batch, self.labels.shape[1])).pin_memory() for _ in range(nslots)]

    def set_epoch(self, epoch):
        self.sampler.set_epoch(epoch)

    def _batches(self):
        idx = list(iter(self.sampler))
        nb = len(idx) // self.batch if self.drop_last else -(-len(idx) // self.batch)
        for k in range(nb):
            yield idx[k * self.batch:(k + 1) * self.batch]

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch if self.drop_last else -(-n // self.batch)

    def __iter__(self):
        batches = list(self._batches())
        nslots = len(self._host)
        q = queue.Queue(maxsize=self.prefetch)
        # per pinned slot: the event of the last H2D copy out of it (the host may refill the slot
        # only once that copy has completed); None = never used
        free = [queue.Queue() for _ in range(nslots)]
        for f in free:
            f.put(None)
        stop = threading.Event()

        def reader():
            try:
                for k, ids in enumerate(batches):
                    s = k % nslots
                    ev = free[s].get()
                    if stop.is_set():
                        return
                    if ev is not None:
                        ev.synchronize()      # host thread waits for the DMA out of this slot
                    ha, hb = self._host[s]
                    for j, i in enumerate(ids):
                        self.a.read_into(i, ha[j])
                        self.b.read_into(i, hb[j])
                    self._lab_host[s][:len(ids)].copy_(self.labels[ids])
                    q.put((s, len(ids)))
                q.put(None)
            except BaseException as e:  # surface reader errors in the consumer
                q.put(e)

        th = threading.Thread(target=reader, daemon=True)
        th.start()
        compute = torch.cuda.current_stream(self.device)
        try:
            while True:
                item = q.get()
                if item is None:
                    break
                if isinstance(item, BaseException):
                    raise item
                s, n = item
                ha, hb = self._host[s]
                da, db = self._dev[s]
                with torch.cuda.stream(self.copy_stream):
                    # da / db are read only by the z-score on this stream: in-order reuse is safe
                    da[:n].copy_(ha[:n], non_blocking=True)
                    db[:n].copy_(hb[:n], non_blocking=True)
                    lab = self._lab_host[s][:n].to(self.device, non_blocking=True)
                    copied = torch.cuda.Event()
                    copied.record(self.copy_stream)
                    za = zscore(da[:n], self.half_round)
                    zb = zscore(db[:n], self.half_round)
                    ready = torch.cuda.Event()
                    ready.record(self.copy_stream)
                free[s].put(copied)
                compute.wait_event(ready)
                for t in (za, zb, lab):
                    t.record_stream(compute)
                yield za, zb, lab
        finally:
            stop.set()
            for f in free:
                f.put(None)
            while th.is_alive():          # unblock a reader waiting on a full queue
                try:
                    q.get(timeout=0.05)
                except queue.Empty:
                    pass
