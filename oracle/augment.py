"""CPU restatement of the reference's training-mode augmentations — TEST INFRASTRUCTURE ONLY.

numpy restatement of ``dataset.py``'s per-item augmentations with every random draw made an
explicit argument, so that one call is a pure function of (sample, draws).  It is the checker of
the K10 device kernel (``srk_augment``); only ``tests/`` may import it.

Pinning status
--------------
* ``time_stretching``, ``add_noise_snr``, ``generate_silence_sample``, ``add_noise_uniform`` —
  pinned: ``tests/golden/augment_golden.npz`` was produced by calling the reference's own
  ``Dataset`` methods (dataset.py:148-204) under seeded ``random`` / ``np.random`` and recording
  the draws (``tests/golden/make_golden.py``).
* ``speed_tuning`` — **parity unpinned**: it calls ``cv2.resize(..., INTER_LINEAR)``
  (dataset.py:212) and OpenCV is not installed here (no version pinned by the reference either).
  ``resize_linear_cv2`` restates OpenCV's generic INTER_LINEAR path for a float64 column
  vector (resize.cpp ``resizeGeneric_`` with ``HResizeLinear`` / ``VResizeLinear<double, double,
  float>``): ``scale = 1 / (dst / src)``; per output row ``fy = float((dy + 0.5) * scale - 0.5)``,
  ``sy = floor(fy)``, ``fy -= sy`` (fp32), coefficients ``(1.f - fy, fy)`` in fp32, the two
  source rows ``sy`` and ``sy + 1`` clamped to ``[0, src - 1]`` (the weight is NOT clamped),
  value ``S0 * b0 + S1 * b1`` in float64 without fused multiply-add.
* ``pitch_shifting`` — needs librosa / resampy (absent): restated separately in ``oracle/pitch.py``
  (parity unpinned, known-answer tests), the checker of K12 ``srk_pitch_shift``.

Fill samples: the reference pads shifted / resampled clips with ``np.random.randint(-32, 32, k)``
(dataset.py:201,203,216,218).  The device draws them from a counter hash instead
(``aug_fill``); the functions below take the fill values as an array so both conventions can
be checked.
"""
import numpy as np

SEQ_LENGTH = 16000

OP_NONE, OP_SPEED, OP_SHIFT, OP_NOISE, OP_NOISE_SNR, OP_SILENCE, OP_PITCH = 0, 1, 2, 3, 4, 5, 6

_M64 = (1 << 64) - 1


def aug_fill(seed, clip, n=SEQ_LENGTH):
    """Device fill convention: int in [-32, 32) for output position i of clip ``clip``:
    splitmix64(seed + clip * 0x9E3779B97F4A7C15 + (i + 1) * 0xD1B54A32D192ED03) >> 58, minus 32."""
    i = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = (np.uint64(seed & _M64) + np.uint64(clip) * np.uint64(0x9E3779B97F4A7C15)
             + (i + np.uint64(1)) * np.uint64(0xD1B54A32D192ED03))
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return (x >> np.uint64(58)).astype(np.int64) - 32


def time_stretching(sample, shift, fill):
    """dataset.py:195-204 with ``shift`` = randint(-range, range) and ``fill`` the |shift| pad
    values: shift >= 0 drops the first ``shift`` samples and pads at the end, shift < 0 pads at
    the start."""
    sample = np.asarray(sample)
    fill = np.asarray(fill)[:abs(shift)]
    if shift >= 0:
        return np.int16(np.concatenate((sample[shift:], fill)))
    return np.int16(np.concatenate((fill, sample[:shift])))


def resize_linear_cv2(x, n_out):
    """cv2.resize(x, (1, n_out), interpolation=cv2.INTER_LINEAR) of a float64 column vector
    (see the module docstring; parity unpinned)."""
    x = np.asarray(x, dtype=np.float64)
    n_in = len(x)
    scale = 1.0 / (float(n_out) / float(n_in))
    dy = np.arange(n_out, dtype=np.float64)
    fy = ((dy + 0.5) * scale - 0.5).astype(np.float32)
    sy = np.floor(fy).astype(np.int64)
    fy = (fy - sy.astype(np.float32)).astype(np.float32)
    b0 = (np.float32(1.0) - fy).astype(np.float32).astype(np.float64)
    b1 = fy.astype(np.float64)
    r0 = np.clip(sy, 0, n_in - 1)
    r1 = np.clip(sy + 1, 0, n_in - 1)
    return x[r0] * b0 + x[r1] * b1


def speed_tuning(sample, n_out, fill):
    """dataset.py:206-223 with ``n_out`` = int(len(sample) * U(0.7, 1.3)); ``fill`` = the pad values
    (left part first, then right) when the resampled clip is shorter than 16000."""
    f = resize_linear_cv2(np.asarray(sample).astype(float), n_out)
    if n_out < SEQ_LENGTH:
        pad = SEQ_LENGTH - n_out
        left, right = int(pad / 2), int(np.ceil(pad / 2))
        fill = np.asarray(fill)
        return np.int16(np.r_[fill[:left], f, fill[left:left + right]])
    cut = n_out - SEQ_LENGTH
    return np.int16(f[int(cut / 2):int(cut / 2) + SEQ_LENGTH])


def add_noise_snr(sample, noise_seg, snr_db):
    """dataset.py:163-181 with the draws explicit: ``noise_seg`` = the 16000-sample noise window,
    ``snr_db`` in {-5, 0, 5, 10} (None returns the sample unchanged)."""
    sample = np.asarray(sample)
    if snr_db is None:
        return sample
    sp = np.sum((sample / 2 ** 15) ** 2) / len(sample)
    npow = np.sum((noise_seg / 2 ** 15) ** 2) / len(noise_seg)
    factor = np.sqrt((sp / npow) / (10 ** (snr_db / 10.0)))
    return np.int16(sample + factor * noise_seg)


def generate_silence_sample(noise_seg, gain):
    """dataset.py:148-161 after the first 185 all-zero samples: ``noise_seg * U(0, 1)`` cast to
    float32 (no int16 cast); ``noise_seg`` None -> the all-zero sample."""
    if noise_seg is None:
        return np.zeros(SEQ_LENGTH, dtype=np.float32)
    return (np.asarray(noise_seg) * gain).astype(np.float32)


def augment_batch(pcm, bank, op, iparam, noise_pos, dparam, seed):
    """The K10 contract (include/srk.h ``srk_augment``) restated per clip: float32 [n, 16000].
    ``bank`` is the flat int16 noise bank, ``noise_pos[b]`` an absolute start in it, ``dparam``
    the gain (noise / silence) or the linear SNR ratio 10 ** (snr / 10) (snr op)."""
    pcm = np.asarray(pcm)
    out = np.empty((len(pcm), SEQ_LENGTH), dtype=np.float32)
    for b in range(len(pcm)):
        x = pcm[b].astype(np.int64)
        o = int(op[b])
        seg = None if noise_pos[b] < 0 else bank[int(noise_pos[b]):int(noise_pos[b]) + SEQ_LENGTH]
        fill = aug_fill(seed, b)
        if o == OP_NONE:
            y = x
        elif o == OP_SPEED:
            n_out = int(iparam[b])
            if n_out < SEQ_LENGTH:
                pad = SEQ_LENGTH - n_out
                left = pad // 2
                # device convention: a fill value belongs to its OUTPUT position
                fill = np.concatenate((fill[:left], fill[left + n_out:]))
            y = speed_tuning(x, n_out, fill)
        elif o == OP_SHIFT:
            s = int(iparam[b])
            y = time_stretching(x, s, fill[SEQ_LENGTH - s:] if s >= 0 else fill[:-s])
        elif o == OP_NOISE:
            y = np.int16(x + float(dparam[b]) * seg)
        elif o == OP_NOISE_SNR:
            # snr given as the linear ratio r = 10 ** (snr / 10)
            sp = np.sum((x / 2 ** 15) ** 2) / len(x)
            npow = np.sum((seg / 2 ** 15) ** 2) / len(seg)
            y = np.int16(x + np.sqrt((sp / npow) / float(dparam[b])) * seg)
        elif o == OP_SILENCE:
            y = generate_silence_sample(seg, float(dparam[b]))
        elif o == OP_PITCH:   # iparam = n_steps (oracle/pitch.py, parity unpinned)
            from oracle import pitch
            y = pitch.pitch_shifting(x, int(iparam[b]))
        else:
            raise ValueError("bad op %d" % o)
        out[b] = np.asarray(y).astype(np.float32)
    return out
