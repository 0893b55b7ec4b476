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
