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
