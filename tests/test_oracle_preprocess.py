"""The preprocessing oracle (oracle/preprocess.py) against scipy, which implements the published
routines nitime's FilterAnalyzer calls (firwin, filtfilt) and scipy.stats.zscore itself."""
import numpy as np
import pytest
import scipy.signal
import scipy.stats

from oracle import preprocess as P


def test_zscore_matches_scipy():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((84, 84)) * 3 + 2
    np.testing.assert_allclose(P.zscore(x), scipy.stats.zscore(x, axis=None), rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(P.zscore(x, axis=1), scipy.stats.zscore(x, axis=1), rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("cut", [0.0056, 0.1, 0.45])
def test_firwin_matches_scipy(cut):
    np.testing.assert_allclose(P.firwin_lowpass(65, cut), scipy.signal.firwin(65, cut, window="hamming"),
                               rtol=0, atol=1e-15)


def test_highpass_taps():
    b = P.fir_highpass_taps()
    ref = -scipy.signal.firwin(65, 0.0035 / 0.625, window="hamming")
    ref[32] += 1
    np.testing.assert_allclose(b, ref, rtol=0, atol=1e-15)
    assert abs(b.sum()) < 1e-12           # high-pass: no DC gain


@pytest.mark.parametrize("L", [196, 350, 361])
def test_filtfilt_matches_scipy(L):
    rng = np.random.default_rng(L)
    x = np.cumsum(rng.standard_normal(L)) + 5.0
    b = P.fir_highpass_taps()
    np.testing.assert_allclose(P.filtfilt(b, x), scipy.signal.filtfilt(b, [1.0], x), rtol=0, atol=1e-11)


def test_filtfilt_short_series_raises():
    with pytest.raises(ValueError):
        P.filtfilt(P.fir_highpass_taps(), np.zeros(195))


def test_band_split_shapes_and_identities():
    rng = np.random.default_rng(7)
    L = 353
    func = np.cumsum(rng.standard_normal((84, L)), axis=1)
    raw, low, ultra = P.fmri_band_split(func)
    assert raw.shape == low.shape == ultra.shape == (368, 84) and raw.dtype == np.float32
    pad = 368 - L
    for a in (raw, low, ultra):
        assert not a[:pad // 2].any() and not a[pad // 2 + L:].any()
        body = a[pad // 2:pad // 2 + L].astype(np.float64)
        np.testing.assert_allclose(body.mean(0), 0, atol=1e-5)
        np.testing.assert_allclose(body.std(0), 1, atol=1e-5)
    # the FIR output keeps the channel mean (nitime restores the DC)
    fir = P.fir_filter(func)
    np.testing.assert_allclose(fir.mean(1), func.mean(1), atol=1e-9)
