// Input preprocessing on the GPU: what the reference's Dataset.__getitem__
// does per subject on the host, batched into two kernels.
//
//   zscore       y = (x - mean) / std over each whole array (scipy.stats.zscore(axis=None),
//                ddof 0), optionally rounded through float16 (the reference's .half(),
//                datasets.py:416, 664).  Statistics in double, reduced in a fixed order
//                (deterministic): partial sums per block, then every normalising block re-adds the
//                same partials in the same order.  HBM-bound: 3 reads + 1 write of the array.
//   band split   datasets.py:665-698 (FIR path): per (subject, ROI) series, nitime
//                FilterAnalyzer(lb=0.0035, TR 0.8).fir = zero-phase FIR high-pass
//                (scipy.signal.filtfilt: odd extension by 3 * ntaps, steady-state initial
//                conditions, forward then backward pass) with the channel mean restored; then
//                raw / low (= fir) / ultralow (= raw - fir) z-scored over time, zero-padded to
//                `seq` (pad // 2 in front) and written time-major (seq, ROIs).  One workgroup per
//                series, everything in LDS, double arithmetic (the reference runs numpy float64).
// Oracle: oracle/preprocess.py.
#include "mmni_common.h"

#include <math.h>

namespace mmni {
namespace prep {

constexpr int kThreads = 256;
constexpr int kMaxTaps = 129;
constexpr int kMaxSeq = 1024;
constexpr int kMaxExt = kMaxSeq + 6 * kMaxTaps;

// Fixed-order block sum of one double per thread (tree over the 256 lanes of the block).
__device__ double block_sum(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < kThreads / 64; ++i) s += red[i];
    return s;
}

// ------------------------------------------------------------------------------------
// whole-array z-score
// ------------------------------------------------------------------------------------
constexpr int kZBlocks = 128;   // partial-sum blocks per array

// pass 0: partial sums of x; pass 1: partial sums of (x - mean)^2
template <int PASS>
__global__ __launch_bounds__(kThreads) void zscore_partial_kernel(const float* x, int64_t count, double* part) {
    __shared__ double red[kThreads / 64];
    const int64_t arr = blockIdx.y;
    const float* xa = x + arr * count;
    double mean = 0.0;
    if (PASS == 1) {
        const double* p = part + arr * kZBlocks * 2;
        double s = 0.0;
        for (int i = 0; i < kZBlocks; ++i) s += p[2 * i];
        mean = s / (double)count;
    }
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < count; i += (int64_t)kZBlocks * kThreads) {
        const double v = (double)xa[i];
        acc += PASS == 0 ? v : (v - mean) * (v - mean);
    }
    const double s = block_sum(acc, red);
    if (threadIdx.x == 0) part[(arr * kZBlocks + blockIdx.x) * 2 + PASS] = s;
}

__global__ __launch_bounds__(kThreads) void zscore_apply_kernel(const float* x, int64_t count, const double* part,
                                                               float* y, int half_round) {
    const int64_t arr = blockIdx.y;
    const double* p = part + arr * kZBlocks * 2;
    double s = 0.0, q = 0.0;
    for (int i = 0; i < kZBlocks; ++i) { s += p[2 * i]; q += p[2 * i + 1]; }
    const double mean = s / (double)count;
    const double inv = 1.0 / sqrt(q / (double)count);
    const float* xa = x + arr * count;
    float* ya = y + arr * count;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < count; i += (int64_t)gridDim.x * kThreads) {
        float v = (float)(((double)xa[i] - mean) * inv);
        if (half_round) v = (float)(_Float16)v;
        ya[i] = v;
    }
}

// ------------------------------------------------------------------------------------
// fMRI band split
// ------------------------------------------------------------------------------------
struct BandArgs {
    int R, Lmax, seq, ntaps;
    const float* y;        // (B, R, Lmax)
    const int32_t* lens;   // (B)
    const double* taps;    // (ntaps) high-pass FIR
    float* raw;            // (B, seq, R)
    float* low;
    float* ultralow;
};

__global__ __launch_bounds__(kThreads) void band_split_kernel(BandArgs a) {
    __shared__ double ext[kMaxExt];     // odd extension, later the FIR output
    __shared__ double y1[kMaxExt];      // forward pass
    __shared__ double xs[kMaxSeq];      // the series
    __shared__ double tp[kMaxTaps];
    __shared__ double red[kThreads / 64];
    const int r = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const int L = a.lens[b], nt = a.ntaps, edge = 3 * nt, E = L + 2 * edge;
    const float* x = a.y + ((int64_t)b * a.R + r) * a.Lmax;
    if (L <= edge || L > a.Lmax) {   // invalid length (the host wrapper validates): NaN rows, no OOB
        const int64_t base = (int64_t)b * a.seq * a.R + r;
        for (int t = tid; t < a.seq; t += kThreads) {
            const int64_t o = base + (int64_t)t * a.R;
            a.raw[o] = a.low[o] = a.ultralow[o] = __builtin_nanf("");
        }
        return;
    }
    for (int k = tid; k < nt; k += kThreads) tp[k] = a.taps[k];
    for (int t = tid; t < L; t += kThreads) xs[t] = (double)x[t];
    __syncthreads();
    for (int n = tid; n < E; n += kThreads) {
        const int m = n - edge;
        ext[n] = m < 0 ? 2.0 * xs[0] - xs[-m] : (m >= L ? 2.0 * xs[L - 1] - xs[2 * (L - 1) - m] : xs[m]);
    }
    __syncthreads();
    // forward pass; samples before the start hold ext[0] (lfilter_zi steady state)
    for (int n = tid; n < E; n += kThreads) {
        double s = 0.0;
        for (int k = 0; k < nt; ++k) s = fma(tp[k], ext[n - k < 0 ? 0 : n - k], s);
        y1[n] = s;
    }
    __syncthreads();
    // backward pass (only the kept window); samples past the end hold y1[E - 1]
    for (int t = tid; t < L; t += kThreads) {
        const int n = t + edge;
        double s = 0.0;
        for (int k = 0; k < nt; ++k) s = fma(tp[k], y1[n + k > E - 1 ? E - 1 : n + k], s);
        ext[t] = s;   // ext no longer needed: reuse for the FIR output
    }
    __syncthreads();
    double sx = 0.0, sf = 0.0;
    for (int t = tid; t < L; t += kThreads) { sx += xs[t]; sf += ext[t]; }
    const double mx = block_sum(sx, red) / L;
    const double mf = block_sum(sf, red) / L;
    // DC restore (nitime filtfilt), the three signals' means
    double s1 = 0.0, s2 = 0.0;
    for (int t = tid; t < L; t += kThreads) {
        const double f = ext[t] - mf + mx;
        ext[t] = f;
        s1 += f;
        s2 += xs[t] - f;
    }
    const double m1 = block_sum(s1, red) / L;
    const double m2 = block_sum(s2, red) / L;
    double q0 = 0.0, q1 = 0.0, q2 = 0.0;
    for (int t = tid; t < L; t += kThreads) {
        const double f = ext[t], u = xs[t] - f;
        q0 += (xs[t] - mx) * (xs[t] - mx);
        q1 += (f - m1) * (f - m1);
        q2 += (u - m2) * (u - m2);
    }
    const double i0 = 1.0 / sqrt(block_sum(q0, red) / L);
    const double i1 = 1.0 / sqrt(block_sum(q1, red) / L);
    const double i2 = 1.0 / sqrt(block_sum(q2, red) / L);
    const int front = (a.seq - L) / 2;
    const int64_t base = (int64_t)b * a.seq * a.R + r;
    for (int t = tid; t < a.seq; t += kThreads) {
        const int s = t - front;
        float v0 = 0.f, v1 = 0.f, v2 = 0.f;
        if (s >= 0 && s < L) {
            const double f = ext[s], u = xs[s] - f;
            v0 = (float)((xs[s] - mx) * i0);
            v1 = (float)((f - m1) * i1);
            v2 = (float)((u - m2) * i2);
        }
        const int64_t o = base + (int64_t)t * a.R;
        a.raw[o] = v0;
        a.low[o] = v1;
        a.ultralow[o] = v2;
    }
}

}  // namespace prep
}  // namespace mmni

using namespace mmni;

extern "C" size_t mmni_zscore_workspace_bytes(int64_t n_arrays) {
    return (size_t)(n_arrays > 0 ? n_arrays : 0) * prep::kZBlocks * 2 * sizeof(double);
}

extern "C" int mmni_zscore(int64_t n_arrays, int64_t count, const float* x, float* y, int half_round, void* workspace,
                           void* stream) {
    MMNI_ARG_CHECK(n_arrays > 0 && n_arrays <= 65535 && count > 0, "zscore: bad sizes (%lld arrays of %lld)",
                   (long long)n_arrays, (long long)count);
    MMNI_ARG_CHECK(x && y && workspace, "zscore: null pointer");
    hipStream_t s = (hipStream_t)stream;
    double* part = reinterpret_cast<double*>(workspace);
    const dim3 grid(prep::kZBlocks, (unsigned)n_arrays);
    prep::zscore_partial_kernel<0><<<grid, prep::kThreads, 0, s>>>(x, count, part);
    prep::zscore_partial_kernel<1><<<grid, prep::kThreads, 0, s>>>(x, count, part);
    int64_t blocks = (count + prep::kThreads * 4 - 1) / (prep::kThreads * 4);
    if (blocks > 1024) blocks = 1024;
    prep::zscore_apply_kernel<<<dim3((unsigned)blocks, (unsigned)n_arrays), prep::kThreads, 0, s>>>(x, count, part, y,
                                                                                                  half_round);
    return launch_status("zscore");
}

// scipy.signal.firwin(ntaps, cutoff, window='hamming') spectrally inverted (nitime
// FilterAnalyzer.fir high-pass taps); host-side, double.
extern "C" int mmni_fir_highpass_taps(int ntaps, double cutoff_frac, double* taps) {
    MMNI_ARG_CHECK(ntaps >= 3 && ntaps <= prep::kMaxTaps && ntaps % 2 == 1, "fir: ntaps must be odd, 3..%d",
                   prep::kMaxTaps);
    MMNI_ARG_CHECK(cutoff_frac > 0.0 && cutoff_frac < 1.0, "fir: cutoff must be in (0, 1) of Nyquist");
    MMNI_ARG_CHECK(taps != nullptr, "fir: null pointer");
    const double alpha = 0.5 * (ntaps - 1);
    double sum = 0.0;
    for (int k = 0; k < ntaps; ++k) {
        const double m = k - alpha, xm = M_PI * cutoff_frac * m;
        const double sinc = m == 0.0 ? 1.0 : sin(xm) / xm;
        const double win = 0.54 - 0.46 * cos(2.0 * M_PI * k / (ntaps - 1));
        taps[k] = cutoff_frac * sinc * win;
        sum += taps[k];
    }
    for (int k = 0; k < ntaps; ++k) taps[k] = -taps[k] / sum;
    taps[ntaps / 2] += 1.0;
    return 0;
}

extern "C" int mmni_fmri_band_split(const mmni_bandsplit_desc* d, const float* y, const int32_t* lens,
                                    const double* taps, float* raw, float* low, float* ultralow, void* stream) {
    MMNI_ARG_CHECK(d != nullptr && d->B > 0 && d->R > 0 && d->B <= 65535, "band_split: bad descriptor");
    MMNI_ARG_CHECK(d->ntaps >= 3 && d->ntaps <= prep::kMaxTaps && d->ntaps % 2 == 1, "band_split: ntaps");
    MMNI_ARG_CHECK(d->seq <= prep::kMaxSeq && d->Lmax <= d->seq, "band_split: seq %d > %d or Lmax %d > seq",
                   d->seq, prep::kMaxSeq, d->Lmax);
    MMNI_ARG_CHECK(d->Lmax > 3 * d->ntaps, "band_split: series must be longer than 3 * ntaps (%d)", 3 * d->ntaps);
    MMNI_ARG_CHECK(y && lens && taps && raw && low && ultralow, "band_split: null pointer");
    prep::BandArgs a{d->R, d->Lmax, d->seq, d->ntaps, y, lens, taps, raw, low, ultralow};
    prep::band_split_kernel<<<dim3((unsigned)d->R, (unsigned)d->B), prep::kThreads, 0, (hipStream_t)stream>>>(a);
    return launch_status("band_split");
}
