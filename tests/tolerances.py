"""Parity tolerances, stated once (SURVEY.md Appendix A 'Tolerances').

* fbank (K2): per clip ||d||_inf / ||ref||_inf <= 1e-4, and
  elementwise <= 0.01 dB for every mel band within 80 dB of its frame's loudest band.  Bands
  deeper than that sit at the fp32-FFT noise floor (error ~ 1e-7 of the frame energy; measured
  <= 0.018 dB at >100 dB below the frame peak): they are held to <= 0.05 dB.  The DC bin, which
  pre-emphasis makes a catastrophic cancellation, is summed in fp64 on the GPU
  (csrc/features.hip), without which column 1 errs by up to 0.05-0.17 dB.
* MFCC (K1): ||d||_inf / ||ref||_inf <= 1e-4 per clip.
* spectrogram (K3): the reference itself (scipy) computes in complex64, so bins far below the
  clip's peak are float32 noise in BOTH implementations.  Bins within e^18 (~78 dB) of the clip's
  peak power: <= 2e-3 absolute in natural-log units; every bin: |e^a - e^b| <= 1e-7 * e^peak.
* noise-mix (K4), frame/window indexing, dataset PCM: bit-exact.
* logits: ||d||_inf / ||ref||_inf <= 1e-4 in fp32 mode; <= 2e-2 with bf16 / fp16 matrix-core
  operands (matmul_precision "bf16" / "fp16", SURVEY.md Appendix A, stated separately).
  Spectrogram-fed models on tonal clips: the reference's own arithmetic (scipy's complex64
  spectrogram) and the float64 restatement already differ by up to 2.5e-3 in logits (bins deep
  under a tone's peak are float32 noise, and the GRU reads them as features; measured at B=512,
  tests/test_lowprec_gpu.py).  There each clip is held to 1e-4 + 4 x that clip's own
  reference-vs-restatement spread (logits_ok) — the HIP spectrogram is a third float32 rounding of
  the same float64 quantity, so its distance to the restatement is of the reference's order, not
  bounded by it — and the model half alone (the oracle model fed the HIP features) to 1e-4.
* 16-bit train steps at the config shapes (tests/test_trainstep_lowprec_gpu.py): every gradient
  tensor ||g - g_oracle||_2 / ||g_oracle||_2 <= 2e-2 (LP_GRAD_REL, after unscaling the fp16 loss
  scale); the fused Adam update vs torch's Adam formula on the same gradient <= 2e-7 absolute
  (LP_ADAM_ABS; lr = 1e-4); the update's disagreement with the fp32 oracle's own Adam step, weighted
  by |g_oracle|, <= 2e-2 (LP_UPDATE_WEIGHTED).
* pitch_shifting (K12, parity unpinned): device vs oracle/pitch.py int16 outputs per clip, RMS
  difference <= 1e-3 of the clip's RMS and every sample within 64 int16 steps, modulo the int16 wrap
  (PITCH_REL_RMS, PITCH_MAX_LSB, pitch_close).  Not bitwise, measured (tools/pitch_diag.py): the STFT's
  first column is the reflect-padded frame centred on sample 0, an even signal, so its spectrum is real
  and the imaginary parts are FFT roundoff whose SIGN decides each phase between 0 and +-pi — any two
  FFT implementations (numpy's pocketfft and the device's radix-2) disagree on ~2 % of them; the phase
  vocoder starts its float32 phase accumulator there, so a 2 pi offset changes the float32 rounding of
  phases that reach ~5e4 rad (ulp 0.004 rad).  Measured: 1.6-2.8e-4 RMS, <= 20 steps on loud clips.
  Degenerate inputs are excluded: a tone with a whole number of periods per frame (1000 Hz at 16 kHz)
  leaves most bins exactly zero, so their phases — accumulated over the clip and loud again in the last,
  reflect-padded frame — are FFT roundoff in ANY implementation (measured: 8 % RMS device vs oracle).
* bf16 / fp16 GRU forward vs a float64 emulation of the same operand rounding: <= 2e-3 absolute on
  y (h in [-1, 1]; a rounding flip of one operand moves a gate pre-activation by ~1e-4).
"""
import numpy as np

FBANK_ABS_DB = 0.01
FBANK_DEPTH_DB = 80.0
FBANK_DEEP_ABS_DB = 0.05
FBANK_REL = 1e-4
MFCC_REL = 1e-4
SPEC_LOG_ABS = 2e-3
SPEC_LOG_WINDOW = 18.0
SPEC_LIN_REL = 1e-7
LOGITS_REL = 1e-4
LOGITS_REL_LOWPREC = 2e-2
GRU_LOWPREC_EMU_ABS = 2e-3
LP_GRAD_REL = 2e-2
LP_ADAM_ABS = 2e-7
LP_UPDATE_WEIGHTED = 2e-2
PITCH_REL_RMS = 1e-3
PITCH_MAX_LSB = 64


def pitch_close(out, ref):
    """K12 output vs oracle/pitch.py for one clip (int16-valued float arrays): (ok, (rel_rms, max_lsb)),
    differences taken modulo the int16 wrap (a value at the +-32768 edge wraps on one side only)."""
    d = np.abs(np.asarray(out, np.float64) - np.asarray(ref, np.float64))
    d = np.minimum(d, 65536.0 - d)
    rms = np.sqrt(np.mean(d ** 2)) / max(np.sqrt(np.mean(np.asarray(ref, np.float64) ** 2)), 1.0)
    return (rms <= PITCH_REL_RMS and d.max() <= PITCH_MAX_LSB), (rms, d.max())


def fbank_ok(out, ref):
    """out/ref: [98, 120] dB of ONE clip -> (ok, (norm_rel, shallow_abs, deep_abs))."""
    out = np.asarray(out, np.float64)
    ref = np.asarray(ref, np.float64)
    err = np.abs(out - ref)
    shallow = ref >= ref.max(axis=1, keepdims=True) - FBANK_DEPTH_DB
    rel = err.max() / max(np.abs(ref).max(), 1e-30)
    sh = err[shallow].max()
    dp = err[~shallow].max() if (~shallow).any() else 0.0
    return (rel <= FBANK_REL and sh <= FBANK_ABS_DB and dp <= FBANK_DEEP_ABS_DB), (rel, sh, dp)


def mfcc_err(out, ref):
    return float(np.abs(out - ref).max() / max(np.abs(ref).max(), 1e-30))


def spec_ok(out, ref):
    """out/ref: [321, 49] or [49, 321] log-power of ONE clip."""
    out = np.asarray(out, np.float64)
    ref = np.asarray(ref, np.float64)
    peak = ref.max()
    m = ref >= peak - SPEC_LOG_WINDOW
    log_err = np.abs(out - ref)[m].max()
    lin_err = np.abs(np.exp(out - peak) - np.exp(ref - peak))[~m].max() if (~m).any() else 0.0
    return log_err <= SPEC_LOG_ABS and lin_err <= SPEC_LIN_REL, (log_err, lin_err)


def rel_err(out, ref):
    return float(np.abs(np.asarray(out) - np.asarray(ref)).max() / max(np.abs(np.asarray(ref)).max(), 1e-30))


def spec_reference_spread(oracle_net, pcm, oracle_logits):
    """Per-clip |logits(scipy complex64 features) - logits(float64 restatement)|_inf / ||ref||_inf:
    the float32 spread of the reference's OWN spectrogram (models/model_spec_bgru.py:11-17 calls
    scipy.signal.spectrogram, which is importable here and on the GPU box) fed to the same oracle
    model.  oracle_net: an oracle.models spec model (features in [B, 321, 49] via .features)."""
    import scipy.signal as ss
    import torch

    def scipy_spec(c):
        _, _, S = ss.spectrogram(c, fs=16000, nperseg=640, noverlap=320, detrend=False)
        return np.log(S.astype(np.float32) + np.float32(1e-10))

    feats = torch.from_numpy(np.stack([scipy_spec(c) for c in pcm]))
    with torch.no_grad():
        out, _ = oracle_net.gru(feats.transpose(1, 2))
        alt = oracle_net.fc(out[:, -1, :]).numpy()
    scale = max(np.abs(oracle_logits).max(), 1e-30)
    return np.abs(alt - oracle_logits).max(axis=1) / scale


def logits_ok(out, ref, spread=None):
    """fp32-mode logits, per clip: ||d||_inf / ||ref||_inf <= LOGITS_REL (+ 4 x the reference's own
    float32 spread of that clip when given) -> (ok, worst (clip, err, bound))."""
    out = np.asarray(out, np.float64)
    ref = np.asarray(ref, np.float64)
    err = np.abs(out - ref).max(axis=1) / max(np.abs(ref).max(), 1e-30)
    bound = LOGITS_REL + (4.0 * np.asarray(spread) if spread is not None else 0.0)
    bound = np.broadcast_to(bound, err.shape)
    i = int(np.argmax(err - bound))
    return bool((err <= bound).all()), (i, float(err[i]), float(bound[i]))
