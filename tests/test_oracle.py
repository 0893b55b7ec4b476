"""The CPU oracle (oracle/) against the golden vectors generated from the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import features as OF
from oracle import models as OM
from tolerances import spec_ok, rel_err


def test_fbank_oracle_bit_exact_vs_reference():
    g = golden("fbank_golden.npz")
    for c, ref in zip(g["pcm"], g["out"]):
        assert np.array_equal(OF.filter_banks(c), ref)


def test_fbank_matrix_properties():
    fb = OF.fbank_matrix()
    assert fb.shape == (120, 257)
    zero = [i for i in range(120) if not fb[i].any()]
    assert zero == [0, 2, 4, 7, 9, 11, 14, 17, 21, 25]
    assert (np.count_nonzero(fb, axis=0) <= 2).all()
    assert max(np.nonzero(fb)[1]) == 255


def test_spec_oracle_vs_reference():
    g = golden("spec_golden.npz")
    for c, ref in zip(g["pcm"], g["out"]):
        ok, errs = spec_ok(OF.compute_spec(c), ref)
        assert ok, errs
    assert np.array_equal(OF.compute_spec(g["pcm"][2], transposed=True), OF.compute_spec(g["pcm"][2]).T)


def test_windows_match_scipy():
    import scipy.signal as ss
    assert np.abs(OF.tukey_window() - ss.get_window(("tukey", 0.25), 640)).max() < 1e-15
    assert np.abs(OF.hann_periodic() - ss.get_window("hann", 640)).max() < 1e-15


def test_mfcc_glue_vs_reference():
    # the reference's compute_mfcc glue (np.gradient x2, concat, cast) around the librosa restatement
    g = golden("mfcc_glue_golden.npz")
    for c, ref in zip(g["pcm"], g["out"]):
        assert np.array_equal(OF.compute_mfcc(c), ref)


def test_mfcc_known_answers():
    # parity unpinned (no librosa): first-principles checks of the librosa-0.6 restatement
    z = OF.compute_mfcc(np.zeros(16000, np.float32))
    assert np.allclose(z[0], -100 * np.sqrt(128), rtol=1e-6)
    assert np.abs(z[1:]).max() < 1e-3
    d = OF.dct_matrix(128, 128)
    assert np.abs(d @ d.T - np.eye(128)).max() < 1e-12
    import scipy.fftpack
    v = np.random.default_rng(0).normal(size=128)
    assert np.allclose(OF.dct_matrix() @ v, scipy.fftpack.dct(v, type=2, norm="ortho")[:13])
    mel = OF.mel_matrix()
    assert mel.shape == (128, 321) and (mel >= 0).all()
    # a 1 kHz tone peaks in the mel band whose centre is nearest 1 kHz
    t = np.arange(16000) / 16000
    S = OF.mfcc13(np.float32(8000) * np.sin(2 * np.pi * 1000 * t).astype(np.float32))
    assert S.shape == (13, 51)
    centres = OF._mel_to_hz(np.linspace(OF._hz_to_mel(0), OF._hz_to_mel(8000), 130))[1:-1]
    x = np.float32(8000) * np.sin(2 * np.pi * 1000 * t).astype(np.float32)
    p = np.pad(x, 320, mode="reflect")
    fr = p[np.arange(640)[None] + 320 * np.arange(51)[:, None]] * OF.hann_periodic()
    m = OF.mel_matrix() @ (np.abs(np.fft.rfft(fr, axis=1)) ** 2).T
    assert abs(centres[m[:, 25].argmax()] - 1000) < 60


def test_noise_mix_oracle_vs_reference():
    g = golden("noise_mix_golden.npz")
    for i in range(len(g["out"])):
        out = OF.add_noise_uniform(g["pcm"][i], g["bank"][g["file_idx"][i]], int(g["start"][i]), float(g["gain"][i]))
        assert out.dtype == np.int16 and np.array_equal(out, g["out"][i])


@pytest.mark.parametrize("name,cls", [("fbanks_cnn", OM.FbanksCNN), ("mfcc_bgru", OM.MfccBGRU),
                                      ("spec_bgru", OM.SpecBGRU), ("resnet_bgru", OM.ResnetBGRU),
                                      ("mfrn_bgru", OM.MfrnBGRU), ("cnn_bgru", OM.CnnBGRU),
                                      ("spec_cnn", OM.SpecCNN), ("analyst", OM.Analyst),
                                      ("fbanks_cnn_train", OM.FbanksCNN),
                                      ("resnet_bgru_mode1", lambda: OM.ResnetBGRU(mode=1))])
def test_model_oracle_vs_reference(name, cls):
    g = golden(name + "_golden.npz")
    net = cls()
    net.load_state_dict(OM.seeded_state_dict(net, 0))
    net.train(bool(g["train_mode"]))
    if "dropout_keep" in g:
        net.dropout = OM.MaskDropout(g["dropout_keep"])
    params = dict(net.named_parameters())
    before = {k: v.detach().clone() for k, v in params.items()}
    out, loss, _ = OM.train_step(net, torch.from_numpy(g["pcm"]), torch.from_numpy(g["labels"]))
    assert rel_err(out.numpy(), g["logits"]) <= 1e-5
    assert abs(loss.item() - float(g["loss"])) <= 1e-5 * max(1.0, abs(float(g["loss"])))
    for k in g["names"]:
        gv = params[k].grad.reshape(-1).numpy()[g["gidx__" + k]]
        assert rel_err(gv, g["gval__" + k]) <= 1e-4, k
        dv = (params[k].detach() - before[k]).reshape(-1).numpy()[g["gidx__" + k]]
        assert np.abs(dv - g["dval__" + k]).max() <= 2e-6, k


def test_frame_index_tables():
    # SURVEY.md Appendix A "Frame/window index tables", stated as integer arithmetic and checked
    # against the padding / framing numpy itself performs in the reference's code paths
    T = OF.mfcc_frame_index()
    assert T.shape == (51, 640) and T.min() == 0 and T.max() == 15999
    y = np.random.default_rng(4).normal(size=16000).astype(np.float32)
    p = np.pad(y, 320, mode="reflect")                                   # librosa stft(center=True)
    assert np.array_equal(y[T], p[np.arange(640)[None] + 320 * np.arange(51)[:, None]])
    assert list(p[:3]) == list(y[[320, 319, 318]]) and list(p[-3:]) == list(y[[15681, 15680, 15679]])
    assert np.array_equal(OF.compute_mfcc(y), OF.compute_mfcc(y, T))
    F = OF.fbank_frame_index()
    assert F.shape == (98, 400) and F.max() == 15919 and np.array_equal(F[:, 0], 160 * np.arange(98))
    assert np.array_equal(OF.filter_banks(y), OF.filter_banks(y, F))
    S = OF.spec_frame_index()
    assert S.shape == (49, 640) and S.max() == 15999 and np.array_equal(S[:, 0], 320 * np.arange(49))
    assert np.array_equal(OF.compute_spec(y), OF.compute_spec(y, index=S))
    # the golden fbank / spec vectors (reference outputs) are reproduced through the explicit tables
    g = golden("fbank_golden.npz")
    for c, ref in zip(g["pcm"], g["out"]):
        assert np.array_equal(OF.filter_banks(c, F), ref)
