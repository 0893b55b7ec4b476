"""The training.py entry point end to end on the device path (synthetic clips), per plugin."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model", ["mfcc_bgru", "fbanks_cnn", "spec_bgru", "resnet_bgru"])
def test_training_entry_point(gpu, tmp_path, model):
    from speechrecognitionproject_amd.training import main
    main(["-key", "t", "-lr", "0.0001", "--model", model, "--synthetic", "48", "--batch-size", "16",
          "--output-path", str(tmp_path), "--log-every", "2"])
    losses = [float(l) for l in open(tmp_path / "loss_t.txt")]
    assert len(losses) == 3 and all(np.isfinite(losses))
    assert len(open(tmp_path / "val_t.txt").readlines()) == 1
    assert len(open(tmp_path / "train_t.txt").readlines()) == 1


def test_training_resnet_bgru_backend_head(gpu, tmp_path):
    """--mode 1: the staged training's auxiliary head (model_resnet_bgru.py:113-118) end to end."""
    from speechrecognitionproject_amd.training import main
    main(["-key", "m", "-lr", "0.0001", "--model", "resnet_bgru", "--mode", "1", "--synthetic", "48",
          "--batch-size", "16", "--output-path", str(tmp_path), "--log-every", "2"])
    losses = [float(l) for l in open(tmp_path / "loss_m.txt")]
    assert len(losses) == 3 and all(np.isfinite(losses))


def test_device_noise_mix_matches_numpy(gpu):
    from oracle import features as OF
    from speechrecognitionproject_amd.dataset import DeviceNoiseMix
    from speechrecognitionproject_amd.synthetic import synthetic_clips, synthetic_noise_bank
    x, _ = synthetic_clips(64, seed=4, clip=30000)
    bank = synthetic_noise_bank()
    mixer = DeviceNoiseMix(bank, seed=5)
    out = mixer(x.astype(np.int16)).cpu().numpy()
    rng = np.random.default_rng(5)
    files = rng.integers(0, bank.shape[0], 64)
    offs = rng.integers(0, bank.shape[1] - 16000 + 1, 64)
    gains = rng.uniform(0, 0.1, 64)
    ref = np.stack([OF.add_noise_uniform(x[i].astype(np.int16), bank[files[i]], int(offs[i]), float(gains[i]))
                    for i in range(64)])
    assert np.array_equal(out, ref.astype(np.float32))


@pytest.mark.parametrize("loader", ["device", "torch"])
def test_training_on_wav_tree(gpu, tmp_path, loader):
    """training.py on a Kaggle-layout WAV tree: the device input pipeline (native decode + K10
    augmentation) and the per-item DataLoader path both train; silence quota persists across epochs."""
    import random
    from scipy.io import wavfile
    from speechrecognitionproject_amd.training import main
    rng = np.random.default_rng(0)
    audio = tmp_path / "data" / "audio"
    os.makedirs(audio / "_background_noise_")
    open(audio / "_background_noise_" / "README.md", "w").close()
    wavfile.write(str(audio / "_background_noise_" / "n.wav"), 16000,
                  np.clip(np.rint(rng.normal(0, 2000, 48000)), -6000, 6000).astype(np.int16))
    names = []
    for d in ("yes", "no", "up", "bed"):
        os.makedirs(audio / d)
        for j in range(6):
            wavfile.write(str(audio / d / ("%d.wav" % j)), 16000,
                          np.clip(np.rint(rng.normal(0, 3000, 16000 - 1000 * j)), -32768, 32767).astype(np.int16))
            names.append("%s/%d.wav" % (d, j))
    (tmp_path / "data" / "training_list.txt").write_text("\n".join(names) + "\n")
    (tmp_path / "data" / "validation_list.txt").write_text("\n".join(names[::3]) + "\n")
    random.seed(0)
    np.random.seed(0)
    out = tmp_path / "out"
    main(["-key", "w", "--model", "mfcc_bgru", "--data-path", str(tmp_path / "data"), "--output-path", str(out),
          "--epochs", "2", "--batch-size", "16", "--reduce", "12", "--log-every", "4", "--loader", loader])
    losses = [float(l) for l in open(out / "loss_w.txt")]
    assert len(losses) == 2 * 3 and all(np.isfinite(losses))      # 18 commands + 12 unknown + 12 silence = 42
    assert len(open(out / "val_w.txt").readlines()) == 2


def test_spin_timeout_is_fatal(gpu, tmp_path):
    """A persistent-kernel spin-wait that gives up must stop training (its results are invalid),
    not continue silently.  The test hook "gru_spin_limit" = 1 makes every wait that is not
    satisfied on its first poll give up; training.py must exit non-zero with the SrkError."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from speechrecognitionproject_amd import _lib\n"
            "from speechrecognitionproject_amd.training import main\n"
            "_lib.set_option('gru_spin_limit', 1)\n"
            "main(['-key', 'x', '--model', 'mfcc_bgru', '--synthetic', '64', '--batch-size', '64', '--no-eval', "
            "'--output-path', %r])\n") % (repo, str(tmp_path))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode != 0, r.stdout + r.stderr
    assert "SrkError" in r.stderr and "timed out" in r.stderr, r.stderr[-2000:]
    # and in this (healthy) process the check passes
    from speechrecognitionproject_amd import _lib
    _lib.check_health(sync=True)


def test_training_graph_equals_eager(gpu, tmp_path):
    """training.py's graph path (two eager warm-up batches on a side stream, then a
    capture and replays) against --no-graph on a dropout-free model, 4 full batches x 2 epochs: the
    loss files and the final parameters must be identical."""
    import torch
    from speechrecognitionproject_amd.training import main
    res = {}
    for tag, extra in (("g", []), ("e", ["--no-graph"])):
        out = tmp_path / tag
        main(["-key", tag, "-lr", "0.0001", "--model", "mfcc_bgru", "--synthetic", "64", "--batch-size", "16",
              "--epochs", "2", "--output-path", str(out), "--log-every", "4", "--no-eval", "--save-model"] + extra)
        res[tag] = (open(out / ("loss_%s.txt" % tag)).read(),
                    torch.load(out / "models" / ("model_%s.ckpt" % tag), weights_only=True))
    assert len(res["g"][0].splitlines()) == 8
    assert res["g"][0] == res["e"][0]
    for k, v in res["g"][1].items():
        assert torch.equal(v, res["e"][1][k]), k


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_training_precision_flag(gpu, tmp_path, precision):
    """--precision (SURVEY.md §5 "Config / flags"): the 16-bit modes through the reference CLI; fp16
    trains with the dynamic loss scale and reports skipped steps."""
    from speechrecognitionproject_amd import _lib
    from speechrecognitionproject_amd.training import main
    main(["-key", "p", "-lr", "0.0001", "--model", "spec_bgru", "--synthetic", "48", "--batch-size", "16",
          "--output-path", str(tmp_path), "--log-every", "3", "--precision", precision])
    losses = [float(l) for l in open(tmp_path / "loss_p.txt")]
    assert len(losses) == 3 and all(np.isfinite(losses))
    assert _lib.matmul_precision() == "fp32"          # restored after the run
