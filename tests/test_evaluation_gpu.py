"""Evaluation callers on the device: K11 softmax ensemble vs torch, the
predictions.py submission CSV vs the CPU oracle run clip by clip as the reference does, the
analyst stacking accuracy helper and analyst_training.py end to end."""
import csv
import os
import random

import numpy as np
import pytest
import torch

from oracle import models as OM
from speechrecognitionproject_amd.evaluation import softmax_ensemble

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,B", [(1, 1), (2, 7), (4, 1000), (8, 33)])
def test_softmax_ensemble_vs_torch(gpu, K, B):
    g = torch.Generator().manual_seed(K * 100 + B)
    logits = torch.randn(K, B, 12, generator=g) * 4
    logits[0, 0, :3] = 50.0                                       # large logits: max subtraction
    cat, mean, pred = softmax_ensemble(logits.cuda(), want_cat=True)
    p = torch.softmax(logits, dim=2)                              # [K, B, C]
    ref_cat = p.permute(1, 0, 2).reshape(B, K * 12)
    ref_mean = p[0].clone()
    for k in range(1, K):
        ref_mean = ref_mean + p[k]
    ref_mean = ref_mean / K
    assert torch.allclose(cat.cpu(), ref_cat, rtol=0, atol=2e-7)
    assert torch.allclose(mean.cpu(), ref_mean, rtol=0, atol=2e-7)
    top2 = ref_mean.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-5
    assert torch.equal(pred.cpu()[clear], ref_mean.argmax(1)[clear])


def _submission_tree(root, n, rng):
    from scipy.io import wavfile
    os.makedirs(root + "/test/audio")
    names = []
    for i in range(n):
        ln = 16000 if i % 4 else 11000
        x = np.clip(np.rint(rng.normal(0, [300, 3000, 12000][i % 3], ln)), -32768, 32767).astype(np.int16)
        wavfile.write(root + "/test/audio/clip_%03d.wav" % i, 16000, x)
        names.append("clip_%03d.wav" % i)
    with open(root + "/submission_list.txt", "w") as f:
        f.write("\n".join(names) + "\n")
    return names


def test_predictions_csv_vs_oracle(gpu, tmp_path):
    from speechrecognitionproject_amd.predictions import LABELS, main
    root = str(tmp_path)
    names = _submission_tree(root, 24, np.random.default_rng(0))
    refs = [OM.ResnetBGRU(), OM.SpecBGRU()]
    paths = []
    for i, r in enumerate(refs):
        sd = OM.seeded_state_dict(r, seed=i + 1)
        r.load_state_dict(sd)
        r.eval()
        paths.append(str(tmp_path / ("m%d.ckpt" % i)))
        torch.save(sd, paths[-1])
    out = main(["-k", "T", "--data-path", root, "--output-path", root, "--models", "resnet_bgru,spec_bgru",
                "--ckpt", ",".join(paths), "--batch-size", "10"])
    rows = list(csv.reader(open(out)))
    assert rows[0] == ["fname", "label"] and [r[0] for r in rows[1:]] == names
    from scipy.io import wavfile
    agree = 0
    with torch.no_grad():
        for (fname, label) in rows[1:]:
            x = wavfile.read(root + "/test/audio/" + fname)[1]
            x = torch.from_numpy(np.concatenate((x, np.zeros(16000 - len(x), dtype=int))).astype(np.float32))[None]
            res = (torch.softmax(refs[0](x).squeeze(0), 0) + torch.softmax(refs[1](x).squeeze(0), 0)) / 2
            top2 = res.topk(2).values
            if (top2[0] - top2[1]).item() > 1e-4:
                assert label == LABELS[int(res.argmax())], fname
                agree += 1
    assert agree >= 20


def test_analyst_accuracy_and_training(gpu, tmp_path):
    from scipy.io import wavfile
    from speechrecognitionproject_amd.analyst_training import main
    rng = np.random.default_rng(1)
    audio = tmp_path / "data" / "audio"
    os.makedirs(audio / "_background_noise_")
    open(audio / "_background_noise_" / "README.md", "w").close()
    wavfile.write(str(audio / "_background_noise_" / "n.wav"), 16000,
                  np.clip(np.rint(rng.normal(0, 2000, 40000)), -6000, 6000).astype(np.int16))
    names = []
    for d in ("yes", "no", "left", "dog"):
        os.makedirs(audio / d)
        for j in range(3):
            wavfile.write(str(audio / d / ("%d.wav" % j)), 16000,
                          np.clip(np.rint(rng.normal(0, 3000, 16000)), -32768, 32767).astype(np.int16))
            names.append("%s/%d.wav" % (d, j))
    (tmp_path / "data" / "training_list.txt").write_text("\n".join(names) + "\n")
    (tmp_path / "data" / "validation_list.txt").write_text("\n".join(names[1::2]) + "\n")
    random.seed(0)
    np.random.seed(0)
    out = tmp_path / "out"
    maxval, epochs = main(["-k", "a", "--data-path", str(tmp_path / "data"), "--output-path", str(out),
                           "--epochs", "3", "--batch-size", "4", "--reduce", "2"])
    assert 1 <= epochs <= 3
    losses = [float(l) for l in open(out / "loss_a.txt")]
    assert losses and all(np.isfinite(losses))
    assert len(open(out / "val_a.txt").readlines()) == epochs
    if maxval > 0:
        sd = torch.load(out / "models" / "model_a.ckpt", weights_only=True)
        OM.Analyst().load_state_dict(sd)


@pytest.mark.parametrize("name", ["fbanks_cnn", "mfcc_bgru"])
def test_plugin_eval_helpers_vs_reference_golden(gpu, tmp_path, name):
    """``accuracy`` / ``class_accuracy`` of the GPU plugin write byte-identical files to the
    reference's own run (tests/golden/make_golden.py: eval_helpers_golden; model_mfcc_bgru.py:39-82):
    accuracy appends one line and over-counts the short last batch (3 clips at batchsize 2 -> 50.0),
    class_accuracy overwrites a 12-line file; both leave the model in training mode."""
    import importlib
    from conftest import golden
    mod = importlib.import_module("speechrecognitionproject_amd.models.model_" + name)
    ocls = {"fbanks_cnn": OM.FbanksCNN, "mfcc_bgru": OM.MfccBGRU}[name]
    g = golden("eval_helpers_%s_golden.npz" % name)
    net = mod.Network().cuda()
    sd = OM.seeded_state_dict(ocls(), 0)
    sd[str(g["bias_key"])] = torch.from_numpy(g["bias"])     # the fixture's centred output bias
    net.load_state_dict(sd)
    net.train()
    ds_a = [{"audio": a, "label": int(l)} for a, l in zip(g["acc_pcm"], g["acc_labels"])]
    ds_c = [{"audio": a, "label": int(l)} for a, l in zip(g["cls_pcm"], g["cls_labels"])]
    fa, fc = tmp_path / "val.txt", tmp_path / "class.txt"
    fa.write_text(str(g["acc_prior"]))
    fc.write_text("stale\n")
    ret = mod.accuracy(net, ds_a, str(fa), int(g["acc_batch"]))
    assert net.training
    assert ret == float(g["acc_return"])
    assert fa.read_text() == str(g["acc_file"])
    mod.class_accuracy(net, ds_c, str(fc), int(g["cls_batch"]))
    assert net.training
    assert fc.read_text() == str(g["cls_file"])
    # the reference's own quirk: a batch size that does not divide the dataset walks past the
    # short last batch (model_mfcc_bgru.py:74-77) and raises
    with pytest.raises(IndexError):
        mod.class_accuracy(net, ds_c[:6], str(tmp_path / "c2.txt"), 4)
