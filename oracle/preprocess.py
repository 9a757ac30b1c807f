"""numpy (float64) restatement of the reference's per-subject input preprocessing — oracle, test
infrastructure only (tests/, bench.py cpu_baseline).  Nothing in the product path imports it.

Covers SURVEY §8f rows 2-3, the steps between the .npy files and the model:
  * zscore(y, axis=None)                  whole-array z-score, then .half() for the struct / DTI
                                          inputs (datasets.py:414-416, 663-664); scipy.stats.zscore
                                          semantics (mean, population std, ddof = 0).
  * fMRI band split (datasets.py:665-698, the 'divided_frequency' / ABCD_multimodal path, FIR
    filtering, the default --filtering_type, main.py:166):
        func = np.load(...)[20:].T                (ROIs, L), L = 350..361
        FA = nitime FilterAnalyzer(TimeSeries(func, sampling_interval=0.8), lb=0.0035)
        raw = zscore(FA.data, axis=1); low = zscore(FA.fir.data, axis=1)
        ultralow = zscore(FA.data - FA.fir.data, axis=1)
        each zero-padded on time to 368 (pad//2 left), transposed to (368, ROIs), float32.
    nitime is not installed here (third-party, version unpinned by the reference: no requirements
    file).  FilterAnalyzer.fir is restated from nitime's published algorithm (nitime/analysis/
    spectral.py, FilterAnalyzer.fir + FilterAnalyzer.filtfilt, defaults filt_order = 64,
    fir_win = 'hamming', ub = None):
        n_taps = 65; lb_frac = lb / (fs / 2); no low-pass stage (ub = None);
        high-pass taps b = -firwin(n_taps, lb_frac, window='hamming'); b[n_taps // 2] += 1;
        per channel: out = scipy.signal.filtfilt(b, [1], x); out += mean(x) - mean(out)  (DC kept).
    scipy.signal.firwin / filtfilt (what nitime calls) are restated below in numpy and checked
    against scipy in tests/test_oracle_preprocess.py; the nitime wrapper itself (DC restore,
    spectral inversion) has no reference fixture: parity of that step is unpinned beyond the
    published algorithm.
"""
import numpy as np

FMRI_TR = 0.8          # sampling interval (s), datasets.py:669
FMRI_LB = 0.0035       # high-pass edge (Hz), datasets.py:670
FMRI_SEQ = 368         # padded sequence length, datasets.py:667
FIR_ORDER = 64         # nitime FilterAnalyzer default filt_order
FMRI_CROP = 20         # leading volumes dropped, datasets.py:665


def zscore(x, axis=None):
    """scipy.stats.zscore (ddof = 0) in float64."""
    x = np.asarray(x, dtype=np.float64)
    m = x.mean(axis=axis, keepdims=True)
    s = x.std(axis=axis, keepdims=True)
    return (x - m) / s


def zscore_half(y):
    """torch.Tensor(zscore(y, axis=None)).half() as float32 values (datasets.py:416, 664): the
    float64 z-score rounded to float32, then to float16."""
    return zscore(y).astype(np.float32).astype(np.float16).astype(np.float32)


def hamming(n):
    """scipy.signal.get_window('hamming', n) (symmetric: firwin asks for fftbins=False)."""
    k = np.arange(n, dtype=np.float64)
    return 0.54 - 0.46 * np.cos(2.0 * np.pi * k / (n - 1))


def firwin_lowpass(n_taps, cutoff):
    """scipy.signal.firwin(n_taps, cutoff, window='hamming') for a single cutoff given as a
    fraction of Nyquist (pass_zero=True, scale=True: unit gain at DC)."""
    alpha = 0.5 * (n_taps - 1)
    m = np.arange(n_taps, dtype=np.float64) - alpha
    h = cutoff * np.sinc(cutoff * m)
    h *= hamming(n_taps)
    return h / h.sum()


def fir_highpass_taps(tr=FMRI_TR, lb=FMRI_LB, order=FIR_ORDER):
    """nitime FilterAnalyzer.fir high-pass stage taps: spectral inversion of the low-pass."""
    n_taps = order + 1
    lb_frac = lb / ((1.0 / tr) / 2.0)
    b = -firwin_lowpass(n_taps, lb_frac)
    b[n_taps // 2] += 1.0
    return b


def _fir_steady(b, x):
    """lfilter(b, [1], x, zi=lfilter_zi(b, [1]) * x[0]): the FIR run as if x[0] had been held
    forever before the start (the steady state lfilter_zi encodes)."""
    n = len(b)
    xp = np.concatenate([np.full(n - 1, x[0]), x])
    return np.convolve(xp, b, mode="valid")


def filtfilt(b, x):
    """scipy.signal.filtfilt(b, [1], x) with its defaults (padtype 'odd', padlen 3 * len(b))."""
    x = np.asarray(x, dtype=np.float64)
    edge = 3 * len(b)
    if x.shape[-1] <= edge:
        raise ValueError("filtfilt: series shorter than the padding (3 * n_taps)")
    left = 2.0 * x[0] - x[edge:0:-1]
    right = 2.0 * x[-1] - x[-2:-(edge + 2):-1]
    ext = np.concatenate([left, x, right])
    y = _fir_steady(b, ext)
    y = _fir_steady(b, y[::-1])[::-1]
    return y[edge:-edge]


def fir_filter(data, tr=FMRI_TR, lb=FMRI_LB):
    """FilterAnalyzer(TimeSeries(data, sampling_interval=tr), lb=lb).fir.data for (channels, L)."""
    b = fir_highpass_taps(tr, lb)
    data = np.asarray(data, dtype=np.float64)
    out = np.empty_like(data)
    for i in range(data.shape[0]):
        o = filtfilt(b, data[i])
        out[i] = o - o.mean() + data[i].mean()
    return out


def _pad_t(a, seq):
    pad = seq - a.shape[1]
    return np.pad(a, ((0, 0), (pad // 2, pad - pad // 2))).T.astype(np.float32)


def fmri_band_split(func, seq=FMRI_SEQ):
    """(ROIs, L) fMRI series (already cropped and transposed, datasets.py:665) ->
    (raw, low, ultralow), each (seq, ROIs) float32 (datasets.py:669-698, FIR, no resample)."""
    func = np.asarray(func, dtype=np.float64)
    fir = fir_filter(func)
    raw = zscore(func, axis=1)
    low = zscore(fir, axis=1)
    ultralow = zscore(func - fir, axis=1)
    return _pad_t(raw, seq), _pad_t(low, seq), _pad_t(ultralow, seq)
