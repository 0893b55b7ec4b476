"""Deterministic synthetic 1-s 16 kHz clips (SURVEY.md §8d "Synthetic inputs").

There is no network and no Kaggle data on the GPU box, so every benchmark and parity test
runs on these.  The mix follows SURVEY.md §8d:

* 40 % N(0, 3000) clipped to int16,   * 20 % N(0, 30000) clipped,
* 20 % 440 Hz + 1 kHz tones at amplitude 8000,
* 10 % all-zero (silence, cf. dataset.py:152-154),   * 10 % half-zero.

Clips are int16-valued float32, NOT scaled to +-1 — exactly what ``Dataset.__getitem__``
returns (dataset.py:117).
"""
import numpy as np

SEQ_LENGTH = 16000
NUM_CLASSES = 12


def _kind(i):
    r = i % 10
    if r < 4:
        return "gauss3k"
    if r < 6:
        return "gauss30k"
    if r < 8:
        return "tones"
    if r == 8:
        return "zeros"
    return "halfzero"


def synthetic_clips(n, seed=0, clip=32767):
    """Return (pcm float32[n,16000], labels int64[n]).

    ``clip`` bounds |x| (the noise-mix config uses 30000 so int16(x + g*noise) cannot overflow,
    SURVEY.md §8d)."""
    rng = np.random.default_rng(seed)
    pcm = np.empty((n, SEQ_LENGTH), dtype=np.float32)
    t = np.arange(SEQ_LENGTH) / 16000.0
    for i in range(n):
        k = _kind(i)
        if k == "gauss3k":
            x = rng.normal(0, 3000, SEQ_LENGTH)
        elif k == "gauss30k":
            x = rng.normal(0, 30000, SEQ_LENGTH)
        elif k == "tones":
            ph = rng.uniform(0, 2 * np.pi, 2)
            x = 8000 * (0.5 * np.sin(2 * np.pi * 440 * t + ph[0]) + 0.5 * np.sin(2 * np.pi * 1000 * t + ph[1]))
        elif k == "zeros":
            x = np.zeros(SEQ_LENGTH)
        else:
            x = rng.normal(0, 3000, SEQ_LENGTH)
            x[SEQ_LENGTH // 2:] = 0
        pcm[i] = np.clip(np.rint(x), -min(clip, 32768), min(clip, 32767))
    labels = rng.integers(0, NUM_CLASSES, n).astype(np.int64)
    return pcm, labels


def synthetic_noise_bank(n_files=6, length=960000, seed=1):
    """Background-noise bank: 6 x 960,000-sample int16 N(0,2000) clipped to +-6000 (§8d)."""
    rng = np.random.default_rng(seed)
    return np.clip(np.rint(rng.normal(0, 2000, (n_files, length))), -6000, 6000).astype(np.int16)


def synthetic_noise_draws(n, bank_len=960000, n_files=6, upper_bound=0.1, seed=2):
    """Per-clip (file index, start offset, gain) draws, the explicit form of dataset.py:190-193."""
    rng = np.random.default_rng(seed)
    files = rng.integers(0, n_files, n).astype(np.int64)
    offs = rng.integers(0, bank_len - SEQ_LENGTH + 1, n).astype(np.int64)
    gains = rng.uniform(0, upper_bound, n).astype(np.float64)
    return files, offs, gains
