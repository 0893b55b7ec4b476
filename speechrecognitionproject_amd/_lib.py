"""ctypes binding of libsrk.so (include/srk.h).  The product path has NO fallback: if the library
or a GPU is missing, every op raises.

torch is imported first on purpose: its bundled libamdhip64.so.7 is then the HIP runtime that
libsrk.so binds to (same SONAME), so torch tensors, streams and our kernels share one runtime.
"""
import ctypes
import os
import re

import torch  # noqa: F401  (load torch's HIP runtime before libsrk.so)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SRK_LIB") or os.path.join(_HERE, "libsrk.so")   # SRK_LIB: experiment builds
HEADER = os.path.join(os.path.dirname(_HERE), "include", "srk.h")
ABI_VERSION = 2

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_F = ctypes.c_float
_D = ctypes.c_double

# name -> argtypes (restype is int unless listed in _RESTYPE)
_SIGS = {
    "srk_version": [],
    "srk_last_error": [],
    "srk_init": [_I],
    "srk_prof_enable": [_I],
    "srk_prof_read": [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double),
                      ctypes.POINTER(ctypes.c_double)],
    "srk_prof_kernels": [ctypes.c_char_p, _I64, ctypes.POINTER(ctypes.c_int64)],
    "srk_source_stamp": [],
    "srk_diag_acc_store": [_P, _I64, _I, _P],
    "srk_diag_tr16_read": [_P, _I64, _P, _P],
    "srk_set_option": [ctypes.c_char_p, _I64],
    "srk_spin_timeouts": [],
    "srk_scratch_generation": [],
    "srk_gru_audit_words": [_I64, _I, _I, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                            ctypes.POINTER(ctypes.c_int64)],
    "srk_health_check": [_I],
    "srk_health_reset": [],
    "srk_fbank_fwd": [_P, _I64, _P, _P],
    "srk_mfcc_fwd": [_P, _I64, _P, _I, _P],
    "srk_spec_fwd": [_P, _I64, _P, _I, _P],
    "srk_fbank_fwd_i16": [_P, _I64, _P, _P],
    "srk_mfcc_fwd_i16": [_P, _I64, _P, _I, _P],
    "srk_spec_fwd_i16": [_P, _I64, _P, _I, _P],
    "srk_noise_mix": [_P, _P, _I64, _I64, _P, _P, _P, _I64, _P, _P],
    "srk_spec_noise_fwd": [_P, _P, _I64, _I64, _P, _P, _P, _I64, _P, _I, _P],
    "srk_augment": [_P, _I64, _P, _I64, _P, _P, _P, _P, ctypes.c_uint64, _P, _P],
    "srk_pitch_workspace_bytes": [_I64],
    "srk_pitch_shift": [_P, _I64, _P, _P, _I64, _P, _P, _I64, _P],
    "srk_wav_read_batch": [ctypes.POINTER(ctypes.c_char_p), _I64, _P, _P, _I],
    "srk_softmax_ensemble": [_P, _I64, _I64, _I64, _P, _P, _P, _P],
    "srk_gemm_f32": [_I, _I, _I64, _I64, _I64, _F, _P, _I64, _P, _I64, _F, _P, _I64, _P, _I, _P],
    "srk_gemm_rowsum_f32": [_I, _I, _I64, _I64, _I64, _F, _P, _I64, _P, _I64, _F, _P, _I64, _P, _P],
    "srk_gemm_16": [_I, _I, _I64, _I64, _I64, _F, _P, _I64, _P, _I64, _F, _P, _I64, _P, _I, _P],
    "srk_gemm_16_batched": [_I, _I, _I64, _I64, _I64, _F, _P, _I64, _I64, _P, _I64, _I64, _F, _P, _I64, _I64, _I, _P],
    "srk_colsum_f32": [_P, _I64, _I64, _I64, _P, _F, _P],
    "srk_gru_workspace_floats": [_I64, _I64, _I64, _I64, _I],
    "srk_gru_layer_fwd": [_P, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P],
    "srk_gru_layer_bwd": [_P, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P],
    "srk_gru_y16_offset": [_I64, _I64, _I64, _I64],
    "srk_gru_layer_fwd_x16": [_P, _P, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P],
    "srk_gru_layer_bwd_x16": [_P, _P, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P],
    "srk_conv2d_workspace_floats": [_I64, _I64, _I64, _I64],
    "srk_conv2d_nhwc_fwd": [_P, _I64, _I64, _I64, _I64, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P,
                            _P],
    "srk_conv2d_nhwc_bwd": [_P, _I64, _I64, _I64, _I64, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P, _P,
                            _P, _P, _P],
    "srk_conv2d_nhwc_fwd16": [_P, _I64, _I64, _I64, _I64, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P,
                              _P, ctypes.POINTER(_I), _P],
    "srk_conv2d_nhwc_bwd16": [_P, _I64, _I64, _I64, _I64, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P, _P,
                              _P, _P, _P, _P],
    "srk_conv2d_nhwc_bwd16_dy16": [_P, _I64, _I64, _I64, _I64, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P,
                                   _P, _P, _P, _P, _P, _P],
    "srk_conv2d_nhwc_bwd16_acc": [_P, _I64, _I64, _I64, _I64, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P,
                                  _P, _P, _P, _P, _P, _I, _P],
    "srk_conv2d_nhwc_fwd_pool": [_P, _I64, _I64, _I64, _I64, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P, _P,
                                 _P, ctypes.POINTER(_I), _P],
    "srk_conv2d_nhwc_bwd_pool": [_P, _I64, _I64, _I64, _I64, _P, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P, _P, _P,
                                 _P, _P, _P, _P],
    "srk_conv1_pool_workspace_floats": [_I64, _I64, _I64],
    "srk_conv1_pool_fwd": [_P, _I64, _I64, _I64, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P, _P],
    "srk_conv1_pool_fwd16": [_P, _I64, _I64, _I64, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P],
    "srk_conv1_pool_wgrad": [_P, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P],
    "srk_maxpool_nhwc_fwd": [_P, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P],
    "srk_maxpool_nhwc_bwd": [_P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P],
    "srk_batchnorm_fwd": [_P, _I64, _I64, _P, _P, _F, _F, _I, _P, _P, _P, _I, _P, _P, _P, _P],
    "srk_batchnorm_bwd": [_P, _P, _P, _I64, _I64, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P],
    "srk_batchnorm_fwd16": [_P, _I64, _I64, _P, _P, _F, _F, _I, _P, _P, _P, _I, _P, _P, ctypes.POINTER(_I), _P, _P,
                            _P],
    "srk_batchnorm_bwd16": [_P, _P, _P, _I64, _I64, _P, _P, _P, _I, _I, _P, _P, ctypes.POINTER(_I), _P, _P, _P, _P],
    "srk_batchnorm_bwd16_acc": [_P, _P, _P, _I64, _I64, _P, _P, _P, _I, _I, _P, _P, ctypes.POINTER(_I), _P, _P, _P,
                                _P, _P, _P],
    "srk_batchnorm_fwd16_mask": [_P, _I64, _I64, _P, _P, _F, _F, _I, _P, _P, _P, _I, _P, _P, ctypes.POINTER(_I), _P,
                                 _P, _P, _P],
    "srk_batchnorm_bwd16_mask": [_P, _P, _P, _P, _I64, _I64, _P, _P, _P, _I, _I, _P, _P, ctypes.POINTER(_I), _P, _P,
                                 _P, _P, _P, _P],
    "srk_batchnorm_stats": [_P, _I64, _I64, _P, _P],
    "srk_batchnorm_combine": [_P, _I, _I64, _F, _F, _P, _P, _P, _P, _P, _P],
    "srk_batchnorm_apply": [_P, _I64, _I64, _P, _P, _P, _P, _P, _I, _P, _P],
    "srk_batchnorm_bwd_reduce": [_P, _P, _P, _I64, _I64, _P, _P, _I, _P, _P],
    "srk_batchnorm_bwd_dx": [_P, _P, _P, _I64, _I64, _P, _P, _P, _P, _P, _I, _P, _P, _P],
    "srk_cross_entropy": [_P, _P, _I64, _I64, _P, _P, _P, _P],
    "srk_adam_step": [_P, _P, _P, _P, _I64, _F, _F, _F, _F, _I64, _F, _P],
    "srk_dropout_fwd": [_P, _I64, _F, ctypes.c_uint64, _P, _P, _P],
    "srk_dropout_fwd_state": [_P, _I64, _F, _P, _P, _P, _P],
    "srk_adam_step_state": [_P, _P, _P, _P, _I64, _F, _F, _F, _P, _F, _P],
    "srk_grad_scaler_init": [_P, _F, _F, _F, _I, _P],
    "srk_adam_step_scaled": [_P, _P, _P, _P, _I64, _F, _F, _F, _P, _F, _P, _P],
    "srk_dropout_apply": [_P, _P, _I64, _F, _P, _P],
}
_RESTYPE = {"srk_last_error": ctypes.c_char_p, "srk_spin_timeouts": ctypes.c_int64, "srk_scratch_generation": ctypes.c_int64, "srk_gru_workspace_floats": ctypes.c_int64, "srk_gru_y16_offset": ctypes.c_int64,
            "srk_conv2d_workspace_floats": ctypes.c_int64, "srk_conv1_pool_workspace_floats": ctypes.c_int64,
            "srk_pitch_workspace_bytes": ctypes.c_int64, "srk_source_stamp": ctypes.c_char_p}


class SrkError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libsrk.so once and declare every signature; raises if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SrkError("libsrk.so is not built (%s); run `python -m speechrecognitionproject_amd.build`" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, ctypes.c_int)
        v = L.srk_version()
        if v != ABI_VERSION:
            raise SrkError("libsrk.so ABI version %d != expected %d (rebuild)" % (v, ABI_VERSION))
        _lib = L
        # A/B measurements: SRK_OPTIONS="conv_tile=256,gru_lp2=0" applies srk_set_option at load
        for item in filter(None, os.environ.get("SRK_OPTIONS", "").split(",")):
            name, _, val = item.partition("=")
            call("srk_set_option", name.strip().encode(), int(val))
            _options[name.strip()] = int(val)
    return _lib


def source_stamp():
    """srk_source_stamp(): the source hash the loaded libsrk.so was built from (build.py)."""
    return lib().srk_source_stamp().decode()


def call(name, *args):
    """Invoke an srk_* entry point and raise SrkError with srk_last_error() on failure."""
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().srk_last_error().decode(errors="replace")
        raise SrkError("%s failed (status %d): %s" % (name, rc, msg))
    return rc


def prof_enable(on):
    call("srk_prof_enable", 1 if on else 0)


def prof_read(name):
    """(launch count, total ms, total algorithmic work) of the recorded launches of `name`."""
    n = ctypes.c_int64(0)
    ms = ctypes.c_double(0.0)
    w = ctypes.c_double(0.0)
    call("srk_prof_read", name.encode(), ctypes.byref(n), ctypes.byref(ms), ctypes.byref(w))
    return int(n.value), float(ms.value), float(w.value)


def prof_kernels():
    """Every recorded launch grouped by (category name, kernel template + shape):
    [{"name", "kernel", "launches", "ms_total", "work", "bytes"}] (bytes: algorithmic HBM bytes, 0 where
    the launch site does not state them)."""
    need = ctypes.c_int64(0)
    call("srk_prof_kernels", None, 0, ctypes.byref(need))
    buf = ctypes.create_string_buffer(int(need.value) + 256)
    call("srk_prof_kernels", buf, len(buf), ctypes.byref(need))
    out = []
    for line in buf.value.decode().splitlines():
        name, detail, n, ms, work, nbytes = line.split("\t")
        out.append({"name": name, "kernel": detail or name, "launches": int(n), "ms_total": float(ms),
                    "work": float(work), "bytes": float(nbytes)})
    return out


def scratch_generation():
    """srk_scratch_generation(): changes whenever a library scratch buffer is reallocated."""
    return int(lib().srk_scratch_generation())


_options = {}


def set_option(name, value):
    """srk_set_option (include/srk.h): e.g. set_option("gru_persistent", 0)."""
    call("srk_set_option", name.encode(), int(value))
    _options[name] = int(value)


def option(name, default=0):
    """The last value this process gave option `name` (set_option / SRK_OPTIONS), else `default`."""
    lib()
    return _options.get(name, default)


PRECISIONS = {"fp32": 0, "bf16": 1, "fp16": 2}
_precision = "fp32"


def set_matmul_precision(name):
    """Operand precision of the matrix-core kernels (GEMMs, GRU recurrence): "fp32" (default,
    exact fp32 MFMA = the reference's arithmetic), "bf16" or "fp16" (operands rounded on chip,
    fp32 accumulation, fp32 tensors in and out).  Process-wide, like torch's matmul precision
    switch; the models' constructors and state_dicts are unchanged."""
    global _precision
    if name not in PRECISIONS:
        raise ValueError("matmul precision must be one of %s, got %r" % (sorted(PRECISIONS), name))
    set_option("matmul_precision", PRECISIONS[name])
    _precision = name


def matmul_precision():
    return _precision


class precision_scope:
    """Run a block at a given matmul precision (restored after): autograd backward passes use the
    precision their forward ran at (the 16-bit GRU backward reads 16-bit operands its forward
    wrote)."""

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.prev = _precision
        if self.name != self.prev:
            set_matmul_precision(self.name)
        return self

    def __exit__(self, *exc):
        if _precision != self.prev:
            set_matmul_precision(self.prev)
        return False


_fused_conv_pool = [True]


def set_fused_conv_pool(on):
    """conv + (1, 4) max-pool in one launch (nn.conv_pool) or the separate kernels (A/B, tests)."""
    _fused_conv_pool[0] = bool(on)


def fused_conv_pool():
    return _fused_conv_pool[0]


def spin_timeouts():
    """Persistent-kernel spin waits that gave up since load (synchronizes; must stay 0)."""
    return int(lib().srk_spin_timeouts())


def check_health(sync=False):
    """Raise SrkError if a persistent kernel's spin-wait has ever timed out (its results are
    invalid).  sync=False reads a host-pinned word without synchronizing the device."""
    call("srk_health_check", 1 if sync else 0)


def header_symbols():
    """Every srk_* function declared in include/srk.h."""
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(srk_[a-z0-9_]+)\s*\(", text)))
