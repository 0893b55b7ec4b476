"""The C-ABI library loads and exports every symbol include/srk.h declares (no GPU needed)."""
import ctypes

from speechrecognitionproject_amd import _lib


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    syms = _lib.header_symbols()
    assert "srk_fbank_fwd" in syms and "srk_last_error" in syms
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    # every header symbol has a declared ctypes signature in the binding
    assert not [s for s in syms if s not in _lib._SIGS]


def test_version_and_error_channel():
    L = _lib.lib()
    assert L.srk_version() == _lib.ABI_VERSION
    assert isinstance(L.srk_last_error(), bytes)
    # argument validation happens before any device work
    rc = L.srk_mfcc_fwd(None, 4, None, 7, None)
    assert rc == -1 and b"layout" in L.srk_last_error()
    rc = L.srk_fbank_fwd(None, -1, None, None)
    assert rc == -1


def test_source_stamp_matches_tree():
    """The shipped libsrk.so was built from these sources: its srk_source_stamp() (build.py's sha256 over
    csrc/* and include/*.h) equals the stamp of the tree.  PMC records carry the same stamp, and bench.py
    attaches their counters only to a library with it (profiles/pmc_*.json)."""
    from speechrecognitionproject_amd import build
    assert _lib.source_stamp() == build.source_stamp()


def test_training_cli_flags():
    """training.py's reference CLI (-key / -lr, training.py:29-32) plus the 16-bit / checkpoint flags
    (SURVEY.md §5 "Config / flags": --precision {fp32,bf16,fp16}); parsed on the CPU."""
    import pytest
    from speechrecognitionproject_amd.training import parse
    a = parse(["-key", "k", "-lr", "0.001"])
    assert a.filekey == "k" and a.learning_rate == 0.001 and a.precision == "fp32" and a.loss_scale == "dynamic"
    assert not a.save_model
    a = parse(["--precision", "fp16", "--loss-scale", "512", "--save-model"])
    assert a.precision == "fp16" and float(a.loss_scale) == 512.0 and a.save_model
    with pytest.raises(SystemExit):
        parse(["--precision", "fp8"])


def test_new_entry_points_reject_bad_arguments():
    """The round-4 entry points validate on the host before touching the device (no GPU needed)."""
    import ctypes
    from speechrecognitionproject_amd import _lib
    L = _lib.lib()
    # null / misaligned scaler state, bad scale
    assert L.srk_grad_scaler_init(None, 1024.0, 2.0, 0.5, 2000, None) != 0
    assert L.srk_grad_scaler_init(ctypes.c_void_p(64), -1.0, 2.0, 0.5, 2000, None) != 0
    assert L.srk_adam_step_scaled(None, None, None, None, 10, 0.9, 0.999, 1e-8, None, 1.0, None, None) != 0
    # the pooled conv needs a (1, 4) window dividing the output width
    i64 = ctypes.c_int64
    rc = L.srk_conv2d_nhwc_fwd_pool(ctypes.c_void_p(256), 2, 98, 40, 64, ctypes.c_void_p(256), None, 128, 1, 7, 0, 3,
                                    3, ctypes.c_void_p(256), ctypes.c_void_p(256), ctypes.c_void_p(256), None, None, None)
    assert rc != 0 and b"window" in L.srk_last_error()
