"""CPU restatement of the reference's feature front-ends — TEST INFRASTRUCTURE ONLY.

This module is the parity *oracle*: a numpy (float64) restatement of the arithmetic the
reference performs on the CPU for each clip.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker / the timed
CPU baseline.  The product path (``speechrecognitionproject_amd``) never imports it.

Pinning status
--------------
* ``filter_banks``   — pinned: ``tests/golden/fbank_golden.npz`` was produced by importing
  the reference's own ``models/model_fbanks_cnn.py:filter_banks`` (see
  ``tests/golden/make_golden.py``).
* ``compute_spec``   — pinned: ``tests/golden/spec_golden.npz`` from the reference's
  ``models/model_spec_bgru.py:compute_spec`` (scipy.signal.spectrogram, scipy 1.15.3 here).
* ``compute_mfcc``   — **parity unpinned**: librosa (the reference's MFCC dependency,
  ``models/model_mfcc_bgru.py:5,13``) is not installed and has no pinned version (the repo has no
  requirements file; era evidence in SURVEY.md §8c points to librosa 0.6.x).  This restates the
  published librosa-0.6 algorithm and is pinned only by known-answer
  tests (silence → c0 = -100*sqrt(128); DCT orthonormality; tone band placement).
* ``add_noise_uniform`` — pinned: ``tests/golden/noise_mix_golden.npz`` from the reference's
  ``dataset.py:183-193`` with seeded draws.
* ``mfcc40x98``      — NOT a reference function: the perf-only "MFCC (40x98)" variant BASELINE.json
  names = scipy's orthonormal DCT-II of the pinned ``filter_banks``, first 40.
"""
import numpy as np

SR = 16000
SEQ_LENGTH = 16000  # dataset.py:13

# ----------------------------------------------------------------------------------------
# log-mel filter bank  (models/model_fbanks_cnn.py:15-66)
# ----------------------------------------------------------------------------------------
FB_NFFT = 512          # model_fbanks_cnn.py:42
FB_NFILT = 120         # model_fbanks_cnn.py:46
FB_FRAME_LEN = 400     # round(0.025*16000), model_fbanks_cnn.py:23-29
FB_FRAME_STEP = 160    # round(0.01*16000)
FB_NUM_FRAMES = 98     # ceil(|16000-400|/160), model_fbanks_cnn.py:30
FB_PRE_EMPHASIS = 0.97  # model_fbanks_cnn.py:20


def fbank_matrix():
    """The constant 120x257 triangular mel matrix of model_fbanks_cnn.py:46-59 (float64).

    The reference rebuilds it on every call (SURVEY.md §3.4 hot loop 1); the values depend only
    on constants, so it is built once here.
    """
    nfilt, nfft, sr = FB_NFILT, FB_NFFT, SR
    high_freq_mel = 2595 * np.log10(1 + (sr / 2) / 700)            # :48
    mel_points = np.linspace(0, high_freq_mel, nfilt + 2)           # :49
    hz_points = 700 * (10 ** (mel_points / 2595) - 1)               # :50
    bins = np.floor((nfft + 1) * hz_points / sr)                    # :51
    fbank = np.zeros((nfilt, int(np.floor(nfft / 2 + 1))))          # :52
    for m in range(1, nfilt + 1):                                   # :53-59
        f_m_minus, f_m, f_m_plus = int(bins[m - 1]), int(bins[m]), int(bins[m + 1])
        for k in range(f_m_minus, f_m):
            fbank[m - 1, k] = (k - bins[m - 1]) / (bins[m] - bins[m - 1])
        for k in range(f_m, f_m_plus):
            fbank[m - 1, k] = (bins[m + 1] - k) / (bins[m + 1] - bins[m])
    return fbank


_FBANK = None


def fbank_frame_index():
    """int64[98, 400] sample index read by (frame f, tap n): ``160 f + n`` into the pre-emphasised,
    zero-appended signal (model_fbanks_cnn.py:32-40; max 15919, so the 80 appended zeros are never
    read)."""
    return FB_FRAME_STEP * np.arange(FB_NUM_FRAMES)[:, None] + np.arange(FB_FRAME_LEN)[None, :]


def filter_banks(sample, index=None):
    """float32[16000] PCM (int16-valued) -> float32[98, 120] log-mel (dB), time x mel.

    Restates models/model_fbanks_cnn.py:15-66.  Precision follows numpy exactly: the
    pre-emphasis is float32 (:21), everything after the float64 zero-pad append (:33) is float64,
    the final cast is float32 (:65).
    """
    global _FBANK
    if _FBANK is None:
        _FBANK = fbank_matrix()
    signal = np.asarray(sample, dtype=np.float32)
    emph = np.append(signal[0], signal[1:] - np.float32(FB_PRE_EMPHASIS) * signal[:-1])   # :21
    pad_len = FB_NUM_FRAMES * FB_FRAME_STEP + FB_FRAME_LEN                              # :32
    pad = np.append(emph, np.zeros(pad_len - len(emph)))                                 # :33-34 -> f64
    idx = fbank_frame_index() if index is None else index
    frames = pad[idx] * np.hamming(FB_FRAME_LEN)                                         # :36-41
    mag = np.abs(np.fft.rfft(frames, FB_NFFT))                                           # :43
    pow_frames = (1.0 / FB_NFFT) * mag ** 2                                              # :44
    fb = pow_frames @ _FBANK.T                                                           # :60
    fb = np.where(fb == 0, np.finfo(float).eps, fb)                                      # :61
    return (20 * np.log10(fb)).astype(np.float32)                                        # :62-65


# ----------------------------------------------------------------------------------------
# log spectrogram  (models/model_spec_bgru.py:11-17, scipy.signal.spectrogram)
# ----------------------------------------------------------------------------------------
SPEC_NPERSEG = 640
SPEC_NOVERLAP = 320
SPEC_NUM_FRAMES = 49   # (16000 - 640)//320 + 1
SPEC_NBINS = 321


def tukey_window(n=SPEC_NPERSEG, alpha=0.25):
    """scipy.signal.get_window(('tukey', 0.25), 640) — periodic (fftbins=True): a symmetric
    Tukey window of length n+1 with the last sample dropped."""
    m = n + 1
    w = np.ones(m)
    width = int(np.floor(alpha * (m - 1) / 2.0))
    k1 = np.arange(0, width + 1)
    k3 = np.arange(m - width - 1, m)
    w[: width + 1] = 0.5 * (1 + np.cos(np.pi * (-1 + 2.0 * k1 / alpha / (m - 1))))
    w[m - width - 1:] = 0.5 * (1 + np.cos(np.pi * (-2.0 / alpha + 1 + 2.0 * k3 / alpha / (m - 1))))
    return w[:n]


def spec_frame_index():
    """int64[49, 640] sample index of (frame f, tap n): ``320 f + n`` (scipy.signal.spectrogram with
    nperseg=640, noverlap=320: no padding, the last 320 samples' second half never starts a frame)."""
    return (SPEC_NPERSEG - SPEC_NOVERLAP) * np.arange(SPEC_NUM_FRAMES)[:, None] + np.arange(SPEC_NPERSEG)[None, :]


def compute_spec(sample, transposed=False, index=None):
    """float32[16000] -> float32[321, 49] (freq x time); [49, 321] if ``transposed``
    (models/model_spec_cnn.py:14 applies ``.T``).

    scipy.signal.spectrogram(fs=16000, nperseg=640, noverlap=320, detrend=False): periodic
    Tukey(0.25) window, PSD density scaling 1/(fs*sum(w^2)), one-sided doubling of bins
    1..319 (DC and Nyquist not doubled), then ``np.log(S.astype(float32) + 1e-10)`` (:14).
    scipy itself computes in complex64 for float32 input; this restatement is float64.
    """
    x = np.asarray(sample, dtype=np.float64)
    w = tukey_window()
    idx = spec_frame_index() if index is None else index
    spec = np.abs(np.fft.rfft(x[idx] * w, SPEC_NPERSEG)) ** 2
    spec *= 1.0 / (SR * np.sum(w * w))
    spec[:, 1:-1] *= 2.0
    out = np.log(spec.astype(np.float32) + np.float32(1e-10)).astype(np.float32)   # (49, 321)
    return out if transposed else np.ascontiguousarray(out.T)


# ----------------------------------------------------------------------------------------
# MFCC (+ delta, delta-delta)  (models/model_mfcc_bgru.py:11-19; librosa 0.6 semantics)
# ----------------------------------------------------------------------------------------
MFCC_NFFT = 640
MFCC_HOP = 320
MFCC_NUM_FRAMES = 51   # 1 + 16000 // 320 (centred)
MFCC_NMELS = 128
MFCC_NCOEF = 13
MFCC_TOP_DB = 80.0
MFCC_AMIN = 1e-10


def hann_periodic(n=MFCC_NFFT):
    """scipy.signal.get_window('hann', n, fftbins=True)."""
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(n) / n)


def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep, mels)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_matrix(sr=SR, n_fft=MFCC_NFFT, n_mels=MFCC_NMELS):
    """librosa.filters.mel(sr, n_fft, n_mels=128, fmin=0, fmax=sr/2, htk=False, norm=1):
    Slaney-scale triangles with area normalisation, float64 [128, 321]."""
    fftfreqs = np.linspace(0, sr / 2.0, 1 + n_fft // 2)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(0.0), _hz_to_mel(sr / 2.0), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    w = np.zeros((n_mels, 1 + n_fft // 2))
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w


def dct_matrix(n_filters=MFCC_NCOEF, n_input=MFCC_NMELS):
    """librosa 0.6 ``filters.dct`` == scipy.fftpack.dct(type=2, norm='ortho') rows [:n_filters]."""
    basis = np.empty((n_filters, n_input))
    basis[0, :] = 1.0 / np.sqrt(n_input)
    samples = np.arange(1, 2 * n_input, 2) * np.pi / (2.0 * n_input)
    for i in range(1, n_filters):
        basis[i, :] = np.cos(i * samples) * np.sqrt(2.0 / n_input)
    return basis


_MEL = None
_DCT = None


def mfcc_frame_index():
    """int64[51, 640] ORIGINAL-clip sample index of (frame f, tap n) under librosa's
    ``stft(center=True, pad_mode='reflect')``: ``src = 320 f + n - 320`` into
    ``np.pad(x, 320, 'reflect')``, i.e. src < 0 -> -src and src > 15999 -> 31998 - src
    (p[:3] = x[320, 319, 318], p[-3:] = x[15681, 15680, 15679])."""
    src = MFCC_HOP * np.arange(MFCC_NUM_FRAMES)[:, None] + np.arange(MFCC_NFFT)[None, :] - MFCC_NFFT // 2
    src = np.where(src < 0, -src, src)
    return np.where(src > SEQ_LENGTH - 1, 2 * (SEQ_LENGTH - 1) - src, src)


def mfcc13(sample, index=None):
    """librosa.feature.mfcc(audio, 16000, n_mfcc=13, n_fft=640, hop_length=320) -> f64[13, 51].

    ``index`` (test hook): an alternative [51, 640] table of original-clip sample indices in place
    of :func:`mfcc_frame_index` (used to show that the parity tests reject a wrong index table)."""
    global _MEL, _DCT
    if _MEL is None:
        _MEL, _DCT = mel_matrix(), dct_matrix()
    y = np.asarray(sample, dtype=np.float32)
    if index is None:
        p = np.pad(y, MFCC_NFFT // 2, mode="reflect")                   # stft(center=True, 'reflect')
        idx = np.arange(MFCC_NFFT)[None, :] + MFCC_HOP * np.arange(MFCC_NUM_FRAMES)[:, None]
        fr = p[idx]
    else:
        fr = y[index]
    frames = fr.astype(np.float64) * hann_periodic()                     # f64 window * f32 frames
    stft = np.fft.rfft(frames, axis=1).astype(np.complex64)              # stored complex64 (0.6)
    S = (np.abs(stft) ** 2).T                                            # f32 [321, 51]
    mel = _MEL @ S                                                       # f64 [128, 51]
    db = 10.0 * np.log10(np.maximum(MFCC_AMIN, mel))                     # power_to_db(ref=1.0)
    db = np.maximum(db, db.max() - MFCC_TOP_DB)                          # top_db=80, per clip
    return _DCT @ db                                                     # [13, 51] f64


def compute_mfcc(sample, index=None):
    """float32[16000] -> float32[39, 51] = [mfcc; d mfcc; dd mfcc] (model_mfcc_bgru.py:11-19)."""
    m = mfcc13(sample, index)
    d = np.gradient(m, axis=1)                                           # :14
    dd = np.gradient(d, axis=1)                                          # :16
    return np.concatenate((m, d, dd)).astype(np.float32)                # :15-18


def mfcc40x98(sample, index=None):
    """float32[16000] -> float32[98, 40]: the perf-only variant (features.mfcc40x98) — scipy.fft.dct type 2,
    norm 'ortho', over the 120 mel bands of filter_banks (dB), coefficients 0..39, in float64."""
    import scipy.fft
    fb = filter_banks(sample, index).astype(np.float64)
    return scipy.fft.dct(fb, type=2, norm="ortho", axis=1)[:, :40].astype(np.float32)


# ----------------------------------------------------------------------------------------
# uniform noise mix  (dataset.py:183-193)
# ----------------------------------------------------------------------------------------
def add_noise_uniform(sample, noise, start, gain):
    """``np.int16(sample + gain * noise[start:start+16000])`` with the draws made explicit:
    ``start`` = randint(0, len(noise)-16000) (:191), ``gain`` = U(0, upper_bound) (:193).
    float64 arithmetic, truncation toward zero on the int16 cast."""
    seg = np.asarray(noise)[start:start + SEQ_LENGTH]
    return np.int16(np.asarray(sample) + gain * seg)
