"""K12 pitch_shifting oracle (oracle/pitch.py, dataset.py:225-235) on the CPU: known answers.

librosa / resampy are absent and the reference pins no version, so the restatement is
**parity-unpinned**; what pins it is first principles: a tone at f comes out at f * 2^(n/12), the
length is kept, silence stays silence, the level None returns the clip, the STFT -> inverse STFT
round trip (rate 1) reproduces the clip, the kaiser_best filter has unit DC gain."""
import numpy as np
import pytest

from oracle import pitch as P

SR = 16000


def _tone(f, amp=8000.0, n=SR):
    t = np.arange(n) / SR
    return np.int16(amp * np.sin(2 * np.pi * f * t))


def _peak_hz(y):
    seg = y[2000:14000].astype(np.float64) * np.hanning(12000)
    spec = np.abs(np.fft.rfft(seg, 4 * 12000))
    return np.argmax(spec) * SR / (4 * 12000)


@pytest.mark.parametrize("f", [440.0, 1000.0, 2500.0])
@pytest.mark.parametrize("n_steps", [-2, -1, 1, 2])
def test_tone_moves_by_the_semitone_ratio(f, n_steps):
    y = P.pitch_shifting(_tone(f), n_steps)
    assert y.dtype == np.int16 and y.shape == (SR,)
    want = f * 2.0 ** (n_steps / 12.0)
    assert abs(_peak_hz(y) - want) <= max(1.0, 1e-3 * want), (_peak_hz(y), want)


def test_level_none_and_silence():
    x = _tone(700.0)
    assert P.pitch_shifting(x, None) is x
    for n in (-2, -1, 1, 2):
        assert not P.pitch_shifting(np.zeros(SR, np.int16), n).any()


def test_stft_istft_round_trip_at_rate_one():
    """time_stretch(y, 1) = istft(phase_vocoder(stft(y), 1)) reproduces y up to the vocoder's float32
    phase accumulator (phases reach ~5e4 rad, a float32 ulp there is ~4e-3 rad), over the 512 * 31
    samples the inverse covers (librosa 0.6 drops the last 128: 16000 is not a multiple of the hop)."""
    rng = np.random.default_rng(3)
    x = np.clip(rng.normal(0, 3000, SR), -32768, 32767).astype(np.float64)
    y = P.time_stretch(x, 1.0)
    assert y.shape == x.shape
    body = 512 * 31     # the inverse STFT of 32 columns spans 512 * 31 samples; fix_length zero-pads
    assert np.linalg.norm(y[:body] - x[:body]) / np.linalg.norm(x[:body]) < 1e-2
    assert not y[body:].any()


def test_kaiser_best_filter():
    win, num_table = P.sinc_window(**P.KAISER_BEST)
    assert num_table == 512 and win.shape == (64 * 512 + 1,)
    assert win[0] == pytest.approx(P.KAISER_BEST["rolloff"], rel=1e-15)
    # DC gain of the interpolator: the taps at every fractional phase sum to ~1 per input sample
    for off in (0, 100, 300):
        assert abs(win[off::512].sum() + win[512 - off::512].sum() - 1.0) < 2e-3
    # resampling a constant keeps it (away from the edges)
    r = P.resample(np.ones(14254), SR / 2 ** (1 / 6), SR)
    assert r.shape == (SR,) and np.abs(r[2000:14000] - 1.0).max() < 1e-4


def test_lengths_follow_librosa():
    for n in (-2, -1, 1, 2):
        rate = 2.0 ** (-n / 12)
        ys = P.time_stretch(np.zeros(SR), rate)
        assert len(ys) == int(round(SR / rate))
