"""CPU restatement of the reference's ``pitch_shifting`` augmentation — TEST INFRASTRUCTURE ONLY.

``Dataset.pitch_shifting`` (dataset.py:225-235) draws a level from [-2, -1, 1, 2, None] and returns
``np.int16(librosa.effects.pitch_shift(sample.astype(float), SEQ_LENGTH, n_steps=level))`` — note
sr = SEQ_LENGTH = 16000 (dataset.py:235).  It is the checker of the K12 device kernel
(``srk_pitch_shift``); only ``tests/`` may import it.

**Parity unpinned.**  librosa and resampy are absent from this image and the reference pins no
version; the era evidence is librosa 0.6.x (positional ``sr``) with resampy 0.2.x.
This module restates their published algorithms with the dtypes those versions use:

``pitch_shift(y, sr, n_steps)`` (librosa.effects, bins_per_octave 12, res_type 'kaiser_best'):
    rate = 2 ** (-n_steps / 12)
    y_shift = resample(time_stretch(y, rate), sr / rate, sr); fix_length(y_shift, len(y))
``time_stretch(y, rate)``: stft (n_fft 2048, hop 512, periodic Hann, centred with reflect padding,
    complex64 result of a float64 FFT) -> phase_vocoder(rate) -> istft(dtype=y.dtype = float64)
    -> fix_length(round(len(y) / rate)).
``phase_vocoder`` (hop = n_fft // 4): time steps arange(0, n_frames, rate); per step the float32
    magnitude interpolation (1 - alpha) |D[:, s]| + alpha |D[:, s + 1]| (NumPy 1.x value-based
    casting: the float64 scalars are cast to float32), phase accumulator float32 (angle of the first
    column), dphase = float32(angle(D[:, s+1]) - angle(D[:, s])) - phi_advance in float64, wrapped by
    2 pi round-half-even, accumulated as float32(phase + (phi_advance + dphase)); output column
    mag * exp(1j * phase) in complex64.
``istft``: per column the Hermitian spectrum, float64 inverse FFT, real part times the periodic
    Hann window, overlap-added in column order; divided by the window sum-square envelope where it
    exceeds tiny(float64); centre trim n_fft // 2 each side.
``resample`` (librosa 0.6 -> resampy 0.2 ``resample(x, sr_orig, sr_new, filter='kaiser_best')``,
    then fix_length(ceil(len * ratio))): the kaiser_best filter is sinc_window(num_zeros=64,
    precision=9, window=kaiser(beta=14.769656459379492), rolloff=0.9475937167399596) — resampy ships
    it precomputed; here it is recomputed from those parameters — scaled by the ratio when
    downsampling; resampy's ``resample_f`` interpolation loop (time register accumulated by repeated
    addition, left wing then right wing, interpolated filter taps) in float64.
The int16 cast truncates toward zero (values outside int16 wrap as the device's int cast does).

Transcendentals: numpy evaluates ``np.angle`` / ``np.abs`` / ``np.exp`` of complex64 with the
platform's float32 libm (atan2f, hypotf, cosf / sinf); here, as on the device, they are evaluated in
float64 and rounded to float32 — the correctly rounded value, which libm's float32 functions return
in all but rare cases.
"""
import numpy as np
import scipy.signal

N_FFT = 2048
HOP = 512
SR = 16000
LEVELS = (-2, -1, 1, 2)
KAISER_BEST = dict(num_zeros=64, precision=9, beta=14.769656459379492, rolloff=0.9475937167399596)


def hann_periodic(n=N_FFT):
    """scipy.signal.get_window('hann', n, fftbins=True)."""
    return scipy.signal.get_window("hann", n, fftbins=True).astype(np.float64)


def _stft(y):
    """librosa 0.6 stft(y) with defaults: complex64 [1 + n_fft / 2, n_frames]."""
    w = hann_periodic()
    yp = np.pad(y, N_FFT // 2, mode="reflect")
    n_frames = 1 + (len(yp) - N_FFT) // HOP
    frames = np.stack([yp[HOP * t:HOP * t + N_FFT] for t in range(n_frames)], axis=1)
    return np.fft.fft(w[:, None] * frames, axis=0)[:N_FFT // 2 + 1].astype(np.complex64)


def _angle32(z):
    return np.arctan2(z.imag.astype(np.float64), z.real.astype(np.float64)).astype(np.float32)


def _abs32(z):
    return np.hypot(z.real.astype(np.float64), z.imag.astype(np.float64)).astype(np.float32)


def phase_vocoder(D, rate):
    n_bins, n_cols = D.shape
    time_steps = np.arange(0, n_cols, rate, dtype=np.float64)
    out = np.zeros((n_bins, len(time_steps)), np.complex64)
    phi_advance = np.linspace(0, np.pi * HOP, n_bins)
    phase_acc = _angle32(D[:, 0])
    D = np.pad(D, [(0, 0), (0, 2)], mode="constant")
    mags, angs = _abs32(D), _angle32(D)
    for t, step in enumerate(time_steps):
        s = int(step)
        alpha = np.mod(step, 1.0)
        mag = np.float32(1.0 - alpha) * mags[:, s] + np.float32(alpha) * mags[:, s + 1]
        ph = phase_acc.astype(np.float64)
        out[:, t] = (mag * np.cos(ph).astype(np.float32)) + 1j * (mag * np.sin(ph).astype(np.float32))
        dphase = (angs[:, s + 1] - angs[:, s]).astype(np.float64) - phi_advance
        dphase = dphase - 2.0 * np.pi * np.round(dphase / (2.0 * np.pi))
        phase_acc = (phase_acc.astype(np.float64) + (phi_advance + dphase)).astype(np.float32)
    return out


def window_sumsquare(n_frames):
    n = N_FFT + HOP * (n_frames - 1)
    x = np.zeros(n, np.float64)
    win_sq = hann_periodic() ** 2
    for i in range(n_frames):
        s = i * HOP
        x[s:min(n, s + N_FFT)] += win_sq[:max(0, min(N_FFT, n - s))]
    return x


def _istft(S):
    w = hann_periodic()
    n_frames = S.shape[1]
    y = np.zeros(N_FFT + HOP * (n_frames - 1), np.float64)
    for i in range(n_frames):
        spec = S[:, i]
        spec = np.concatenate((spec, spec[-2:0:-1].conj()), 0)
        y[i * HOP:i * HOP + N_FFT] += w * np.fft.ifft(spec).real
    wss = window_sumsquare(n_frames)
    nz = wss > np.finfo(np.float64).tiny
    y[nz] /= wss[nz]
    return y[N_FFT // 2:-(N_FFT // 2)]


def fix_length(y, n):
    return np.pad(y, (0, n - len(y)), mode="constant") if len(y) < n else y[:n]


def time_stretch(y, rate):
    y_stretch = _istft(phase_vocoder(_stft(y), rate))
    return fix_length(y_stretch, int(round(len(y) / rate)))


def sinc_window(num_zeros=64, precision=9, beta=14.769656459379492, rolloff=0.9475937167399596):
    """resampy.filters.sinc_window with window = kaiser(beta): the right wing, 2**precision taps per
    zero crossing."""
    num_bits = 2 ** precision
    n = num_bits * num_zeros
    sinc_win = rolloff * np.sinc(rolloff * np.linspace(0, num_zeros, num=n + 1, endpoint=True))
    taper = scipy.signal.windows.kaiser(2 * n + 1, beta)[n:]
    return taper * sinc_win, num_bits


def resample(x, sr_orig, sr_new):
    """librosa 0.6 core.resample(x, sr_orig, sr_new, res_type='kaiser_best', fix=True)."""
    ratio = float(sr_new) / sr_orig
    n_samples = int(np.ceil(x.shape[-1] * ratio))
    sample_ratio = float(sr_new) / sr_orig
    n_out = int(x.shape[-1] * sample_ratio)
    interp_win, num_table = sinc_window(**KAISER_BEST)
    if sample_ratio < 1:
        interp_win = interp_win * sample_ratio
    interp_delta = np.zeros_like(interp_win)
    interp_delta[:-1] = np.diff(interp_win)
    y = _resample_f(np.asarray(x, np.float64), n_out, sample_ratio, interp_win, interp_delta, num_table)
    return fix_length(y, n_samples)


def _resample_f(x, n_out, sample_ratio, interp_win, interp_delta, num_table):
    """resampy.interpn.resample_f, one channel, vectorised over the output samples (each output's
    taps are still summed in the loop's order: left wing i = 0.., then right wing k = 0..)."""
    scale = min(1.0, sample_ratio)
    time_increment = 1.0 / sample_ratio
    index_step = int(scale * num_table)
    nwin = interp_win.shape[0]
    n_orig = x.shape[0]
    tr = np.empty(n_out, np.float64)
    acc = 0.0
    for t in range(n_out):                   # the time register, accumulated as the loop does
        tr[t] = acc
        acc += time_increment
    n = tr.astype(np.int64)
    y = np.zeros(n_out, np.float64)
    frac = scale * (tr - n)
    index_frac = frac * num_table
    offset = index_frac.astype(np.int64)
    eta = index_frac - offset
    i_max = np.minimum(n + 1, (nwin - offset) // index_step)
    for i in range(int(i_max.max(initial=0))):
        m = i < i_max
        j = offset[m] + i * index_step
        weight = interp_win[j] + eta[m] * interp_delta[j]
        y[m] = y[m] + weight * x[n[m] - i]
    frac = scale - frac
    index_frac = frac * num_table
    offset = index_frac.astype(np.int64)
    eta = index_frac - offset
    k_max = np.minimum(n_orig - n - 1, (nwin - offset) // index_step)
    for k in range(int(k_max.max(initial=0))):
        m = k < k_max
        j = offset[m] + k * index_step
        weight = interp_win[j] + eta[m] * interp_delta[j]
        y[m] = y[m] + weight * x[n[m] + k + 1]
    return y


def pitch_shift(y, sr, n_steps):
    """librosa.effects.pitch_shift(y, sr, n_steps) (0.6.x), float64 in and out."""
    rate = 2.0 ** (-float(n_steps) / 12)
    y_shift = resample(time_stretch(y, rate), float(sr) / rate, sr)
    return fix_length(y_shift, len(y))


def int16_trunc(v):
    """np.int16(float64 array): truncation toward zero; out-of-range values wrap through int32 as
    the x86 conversion (and the device's (int16_t)(int) cast) does."""
    return np.trunc(v).astype(np.int64).astype(np.int32).astype(np.int16)


def pitch_shifting(sample, level):
    """dataset.py:225-235 with the level draw made explicit (None returns the sample)."""
    if level is None:
        return sample
    return int16_trunc(pitch_shift(np.asarray(sample).astype(float), SR, n_steps=level))
