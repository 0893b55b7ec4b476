"""Generate the golden parity fixtures in tests/golden/ FROM THE REFERENCE ITSELF.

Run in the build container only (``/root/reference`` does not exist on the GPU box):

    python tests/golden/make_golden.py

The reference is imported read-only from /root/reference.  Three third-party modules it imports
are absent from this image: ``librosa`` (model_mfcc_bgru.py:5, dataset.py:9) and
``cv2`` (dataset.py:8).  They are replaced by stubs that raise if called — except
``librosa.feature.mfcc``, which is bound to the oracle's librosa-0.6 restatement so that the
reference's MFCC *glue* (np.gradient x2, concat, cast; model_mfcc_bgru.py:12-18) and its
GRU/FC run unmodified.  The librosa arithmetic itself stays "parity unpinned".

Outputs are data only (inputs + expected outputs), no reference source.
"""
import os
import random
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.path.insert(0, REPO)
# the reference tree is read-only: importing it must not leave __pycache__/*.pyc behind
sys.dont_write_bytecode = True

from oracle import features as OF            # noqa: E402
from oracle import models as OM              # noqa: E402
from speechrecognitionproject_amd.synthetic import synthetic_clips   # noqa: E402


def _install_stubs():
    def _absent(*a, **k):
        raise RuntimeError("stubbed third-party call (absent in this image)")

    librosa = types.ModuleType("librosa")
    feat = types.ModuleType("librosa.feature")
    eff = types.ModuleType("librosa.effects")

    def mfcc(y, sr=22050, n_mfcc=20, n_fft=2048, hop_length=512):
        assert (sr, n_mfcc, n_fft, hop_length) == (16000, 13, 640, 320)
        return OF.mfcc13(y)

    feat.mfcc = mfcc
    eff.pitch_shift = _absent
    librosa.feature, librosa.effects = feat, eff
    cv2 = types.ModuleType("cv2")
    cv2.resize = _absent
    sys.modules.update({"librosa": librosa, "librosa.feature": feat, "librosa.effects": eff, "cv2": cv2})


def golden_clips():
    """8 clips covering the amplitude range named in SURVEY.md §8c."""
    rng = np.random.default_rng(123)
    t = np.arange(16000) / 16000.0
    clips = [
        rng.normal(0, 1, 16000),
        rng.normal(0, 30, 16000),
        rng.normal(0, 3000, 16000),
        rng.normal(0, 30000, 16000),
        np.zeros(16000),
        np.concatenate([rng.normal(0, 3000, 8000), np.zeros(8000)]),
        8000 * np.sin(2 * np.pi * 440 * t) + 4000 * np.sin(2 * np.pi * 1000 * t + 0.3),
        1000 + rng.normal(0, 200, 16000),   # strong DC: stresses the pre-emphasis/DC bin
    ]
    return np.stack([np.clip(np.rint(c), -32768, 32767) for c in clips]).astype(np.float32)


def sample_entries(t, n=256, seed=99):
    flat = t.detach().reshape(-1).numpy()
    if flat.size <= 4096:
        return np.arange(flat.size), flat.copy()
    idx = np.sort(np.random.default_rng(seed).choice(flat.size, n, replace=False))
    return idx, flat[idx].copy()


ONLY = set(sys.argv[1:])   # optional subset of fixture file names to (re)write
if ONLY:
    _savez = np.savez_compressed

    def _savez_only(path, **kw):
        if os.path.basename(path) in ONLY:
            _savez(path, **kw)

    np.savez_compressed = _savez_only


class _MaskDropout(torch.nn.Module):
    """Stands in for the reference's ``nn.Dropout`` (model_fbanks_cnn.py:79,98) with an exported
    Bernoulli(1 - p) keep mask: y = x * keep / (1 - p), what nn.Dropout computes for that draw."""

    def __init__(self, keep, p=0.5):
        super().__init__()
        self.keep, self.p = keep, p

    def forward(self, x):
        return x * self.keep / (1.0 - self.p) if self.training else x


def model_golden(name, net, x, labels, train_mode=False, dropout_keep=None):
    if ONLY and name not in ONLY:
        return
    sd = OM.seeded_state_dict(net, seed=0)
    net.load_state_dict(sd)
    net.train(train_mode)
    if dropout_keep is not None:
        net.dropout = _MaskDropout(torch.from_numpy(dropout_keep.astype(np.float32)))
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    before = {k: v.detach().clone() for k, v in net.named_parameters()}
    opt.zero_grad()
    out = net(torch.from_numpy(x))
    loss = torch.nn.CrossEntropyLoss()(out, torch.from_numpy(labels))
    loss.backward()
    grads = {k: v.grad.detach().clone() for k, v in net.named_parameters() if v.grad is not None}
    opt.step()
    rec = {"pcm": x, "labels": labels, "logits": out.detach().numpy(), "loss": np.float32(loss.item()),
           "train_mode": np.int64(train_mode), "names": np.array(list(grads.keys()))}
    if dropout_keep is not None:
        rec["dropout_keep"] = dropout_keep.astype(np.uint8)
    for k in grads:
        gi, gv = sample_entries(grads[k])
        di, dv = sample_entries(dict(net.named_parameters())[k].detach() - before[k])
        rec["gidx__" + k], rec["gval__" + k] = gi, gv
        rec["dval__" + k] = dv
        rec["gsum__" + k] = np.float64(grads[k].double().sum())
        rec["gabs__" + k] = np.float64(grads[k].double().abs().sum())
    np.savez_compressed(os.path.join(HERE, name), **rec)
    print("wrote", name, "logits", out.shape)


def eval_helpers_golden(name, R_mod, ocls, seed):
    """The plugin eval helpers ``accuracy`` / ``class_accuracy`` (model_mfcc_bgru.py:39-82; the same
    text in every model_*.py) run by the reference on a seeded model in eval mode, recording the
    files they write.  Clips are kept only where the reference's top-2 logit gap is wide (> 1e-2 of
    the largest logit), so a 1e-4 logit difference cannot change a prediction.
    * ``accuracy`` on 3 clips at batchsize 2 (labels: right, wrong, right): the last batch is short
      and ``total += batchsize`` counts it as 2 -> 2 / 4 = 50.0, appended after an existing line.
    * ``class_accuracy`` on 36 clips at batchsize 4: clips 0..23 carry labels i % 12 (every class
      present; the reference divides by each class count) and clips 24..35 carry the reference's
      own prediction; the file is overwritten."""
    if ONLY and name not in ONLY:
        return
    net = R_mod.Network()
    sd = OM.seeded_state_dict(ocls(), 0)
    net.load_state_dict(sd)
    net.eval()
    x, _ = synthetic_clips(160, seed=seed)
    with torch.no_grad():
        lg = net(torch.from_numpy(x)).numpy()
    # a random-init model predicts one class for every clip: centre the output bias on these
    # clips' mean logits so the predictions spread over the classes (stored in the fixture)
    bias_key = [k for k in sd if k.endswith("bias")][-1]
    sd[bias_key] = (sd[bias_key].double() - torch.from_numpy(lg.mean(0))).float()
    net.load_state_dict(sd)
    with torch.no_grad():
        lg = net(torch.from_numpy(x)).numpy()
    top2 = np.sort(lg, axis=1)[:, -2:]
    wide = np.nonzero(top2[:, 1] - top2[:, 0] > 1e-2 * np.abs(lg).max())[0]
    assert len(wide) >= 39, len(wide)
    pred = lg.argmax(1)
    a_idx = wide[:3]
    a_lab = np.array([pred[a_idx[0]], (pred[a_idx[1]] + 5) % 12, pred[a_idx[2]]])
    c_idx = wide[3:39]
    c_lab = np.concatenate([np.arange(24) % 12, pred[c_idx[24:]]])
    ds_a = [{"audio": x[i], "label": int(l)} for i, l in zip(a_idx, a_lab)]
    ds_c = [{"audio": x[i], "label": int(l)} for i, l in zip(c_idx, c_lab)]
    with tempfile.TemporaryDirectory() as d:
        fa, fc = d + "/val.txt", d + "/class.txt"
        with open(fa, "w") as f:
            f.write("12.5\n")
        with open(fc, "w") as f:
            f.write("stale\n")
        net.train()
        ret = R_mod.accuracy(net, ds_a, fa, 2)
        assert net.training
        R_mod.class_accuracy(net, ds_c, fc, 4)
        ta, tc = open(fa).read(), open(fc).read()
    np.savez_compressed(os.path.join(HERE, name), acc_pcm=x[a_idx], acc_labels=a_lab, acc_batch=np.int64(2),
                        acc_return=np.float64(ret), acc_file=np.array(ta), acc_prior=np.array("12.5\n"),
                        cls_pcm=x[c_idx], cls_labels=c_lab, cls_batch=np.int64(4), cls_file=np.array(tc),
                        acc_pred=pred[a_idx], cls_pred=pred[c_idx], bias_key=np.array(bias_key),
                        bias=sd[bias_key].numpy())
    print("wrote", name, repr(ta), tc.count("\n"), "lines")


def main():
    _install_stubs()
    sys.path.insert(0, REF)
    sys.path.insert(0, REF + "/models")
    import model_fbanks_cnn as R_fb
    import model_spec_bgru as R_sb
    import model_spec_cnn as R_sc
    import model_mfcc_bgru as R_mb
    import model_mfrn_bgru as R_mr
    import model_cnn_bgru as R_cb
    import model_analyst as R_an
    import model_resnet_bgru as R_rb
    import dataset as R_ds
    torch.set_default_dtype(torch.float32)

    pcm = golden_clips()
    # ---- K2 fbank (model_fbanks_cnn.py:15-66)
    fb = np.stack([R_fb.filter_banks(torch.from_numpy(c)).numpy() for c in pcm])
    np.savez_compressed(os.path.join(HERE, "fbank_golden.npz"), pcm=pcm, out=fb)
    # ---- K3 spectrogram (model_spec_bgru.py:11-17; model_spec_cnn.py:12-18 is its transpose)
    sp = np.stack([R_sb.compute_spec(torch.from_numpy(c)).numpy() for c in pcm])
    spt = np.stack([R_sc.compute_spec(torch.from_numpy(c)).numpy() for c in pcm])
    assert np.array_equal(sp.transpose(0, 2, 1), spt)
    np.savez_compressed(os.path.join(HERE, "spec_golden.npz"), pcm=pcm, out=sp)
    # ---- K1 MFCC glue with the oracle's librosa restatement (arithmetic unpinned, glue pinned)
    mf = np.stack([R_mb.compute_mfcc(torch.from_numpy(c)).numpy() for c in pcm])
    np.savez_compressed(os.path.join(HERE, "mfcc_glue_golden.npz"), pcm=pcm, out=mf)

    # ---- K4 noise-mix + Dataset PCM path on a synthetic Kaggle-layout tree (dataset.py)
    from scipy.io import wavfile
    with tempfile.TemporaryDirectory() as root:
        rng = np.random.default_rng(7)
        os.makedirs(root + "/_background_noise_")
        open(root + "/_background_noise_/README.md", "w").close()
        bank = np.clip(np.rint(rng.normal(0, 2000, (2, 60000))), -6000, 6000).astype(np.int16)
        for i in range(2):
            wavfile.write(root + "/_background_noise_/noise%d.wav" % i, 16000, bank[i])
        for d in ("yes", "go", "bed"):
            os.makedirs(root + "/" + d)
        lens = {"yes/a.wav": 12000, "go/b.wav": 16000, "bed/c.wav": 9000}
        wavs = {}
        for f, n in lens.items():
            w = np.clip(np.rint(rng.normal(0, 3000, n)), -32768, 32767).astype(np.int16)
            wavfile.write(root + "/" + f, 16000, w)
            wavs[f] = w
        with open(root + "/validation_list.txt", "w") as fh:
            fh.write("\n".join(lens) + "\n")
        ds = R_ds.Dataset(root + "/validation_list.txt", root)
        items = [ds[i] for i in range(len(ds))]
        np.savez_compressed(os.path.join(HERE, "dataset_golden.npz"),
                            names=np.array(list(lens)), audio=np.stack([it["audio"] for it in items]),
                            labels=np.array([it["label"] for it in items]),
                            wav_a=wavs["yes/a.wav"], wav_b=wavs["go/b.wav"], wav_c=wavs["bed/c.wav"])
        # add_noise_uniform with seeded draws; the draws are re-derived in the same order
        names = sorted(ds.noise_list)
        samples, outs, files, starts, gains = [], [], [], [], []
        for i in range(6):
            s = np.concatenate((wavs["yes/a.wav"], np.zeros(4000, dtype=int))) if i % 2 == 0 else wavs["go/b.wav"]
            random.seed(i)
            np.random.seed(i)
            out = ds.add_noise_uniform(s, 0.1)
            random.seed(i)
            np.random.seed(i)
            fname = ds.noise_list[random.randint(0, len(ds.noise_list) - 1)]
            start = random.randint(0, 60000 - 16000)
            gain = np.random.uniform(0, 0.1)
            assert np.array_equal(out, OF.add_noise_uniform(s, bank[names.index(fname)], start, gain))
            samples.append(s.astype(np.int64))
            outs.append(out)
            files.append(names.index(fname))
            starts.append(start)
            gains.append(gain)
        np.savez_compressed(os.path.join(HERE, "noise_mix_golden.npz"), bank=bank, pcm=np.stack(samples),
                            file_idx=np.array(files), start=np.array(starts), gain=np.array(gains), out=np.stack(outs))

        # time_stretching / add_noise_snr / generate_silence_sample (dataset.py:148-204): call the
        # reference under a seed, then replay the same draws to record them explicitly
        from oracle import augment as OA
        base = np.concatenate((wavs["yes/a.wav"], np.zeros(4000, dtype=int)))
        shifts, shift_fill, shift_out = [], np.zeros((8, 4800), dtype=np.int64), []
        for i in range(8):
            random.seed(100 + i)
            np.random.seed(100 + i)
            out = ds.time_stretching(base, 4800)
            random.seed(100 + i)
            np.random.seed(100 + i)
            sh = random.randint(-4800, 4800)
            fill = np.random.randint(-32, 32, abs(sh))
            assert np.array_equal(out, OA.time_stretching(base, sh, fill))
            shifts.append(sh)
            shift_fill[i, :abs(sh)] = fill
            shift_out.append(out)
        snr_pcm, snr_files, snr_starts, snr_db, snr_out = [], [], [], [], []
        for i in range(10):
            s = wavs["go/b.wav"].astype(np.int64) // (1 + 7 * (i % 2))
            random.seed(200 + i)
            np.random.seed(200 + i)
            out = ds.add_noise_snr(s)
            random.seed(200 + i)
            np.random.seed(200 + i)
            fname = ds.noise_list[random.randint(0, len(ds.noise_list) - 1)]
            start = random.randint(0, 60000 - 16000)
            snr = [-5, 0, 5, 10, None][random.randint(0, 4)]
            seg = bank[names.index(fname)][start:start + 16000]
            assert np.array_equal(out, OA.add_noise_snr(s, seg, snr))
            snr_pcm.append(s)
            snr_files.append(names.index(fname))
            snr_starts.append(start)
            snr_db.append(np.nan if snr is None else snr)
            snr_out.append(np.asarray(out).astype(np.int64))
        sil_files, sil_starts, sil_gains, sil_out = [], [], [], []
        ds.silence_class_zeros_count = 185
        for i in range(4):
            random.seed(300 + i)
            np.random.seed(300 + i)
            out = ds.generate_silence_sample()
            random.seed(300 + i)
            np.random.seed(300 + i)
            fname = ds.noise_list[random.randint(0, len(ds.noise_list) - 1)]
            start = random.randint(0, 60000 - 16000)
            gain = np.random.uniform(0, 1)
            assert np.array_equal(out, OA.generate_silence_sample(bank[names.index(fname)][start:start + 16000], gain))
            sil_files.append(names.index(fname))
            sil_starts.append(start)
            sil_gains.append(gain)
            sil_out.append(out)
        np.savez_compressed(os.path.join(HERE, "augment_golden.npz"), bank=bank, shift_pcm=base.astype(np.int64),
                            shift=np.array(shifts), shift_fill=shift_fill, shift_out=np.stack(shift_out),
                            snr_pcm=np.stack(snr_pcm), snr_file=np.array(snr_files), snr_start=np.array(snr_starts),
                            snr_db=np.array(snr_db, dtype=np.float64), snr_out=np.stack(snr_out),
                            sil_file=np.array(sil_files), sil_start=np.array(sil_starts),
                            sil_gain=np.array(sil_gains), sil_out=np.stack(sil_out))

    # ---- module-level goldens (logits, CE loss, sampled grads, 1-step Adam delta)
    x, y = synthetic_clips(4, seed=5)
    torch.manual_seed(0)
    model_golden("fbanks_cnn_golden.npz", R_fb.Network(), x, y, train_mode=False)
    # train mode: dropout on [B, 512] after maxpool3 with an exported keep mask
    keep = (np.random.default_rng(55).random((4, 512)) >= 0.5).astype(np.uint8)
    model_golden("fbanks_cnn_train_golden.npz", R_fb.Network(), x, y, train_mode=True, dropout_keep=keep)
    model_golden("mfcc_bgru_golden.npz", R_mb.Network(), x, y)
    model_golden("spec_bgru_golden.npz", R_sb.Network(), x, y)
    x2, y2 = synthetic_clips(2, seed=6)
    model_golden("resnet_bgru_golden.npz", R_rb.Network(), x2, y2, train_mode=True)
    torch.manual_seed(0)
    model_golden("resnet_bgru_mode1_golden.npz", R_rb.Network(mode=1), x2, y2, train_mode=True)
    x3, y3 = synthetic_clips(2, seed=7)
    torch.manual_seed(0)
    model_golden("mfrn_bgru_golden.npz", R_mr.Network(), x3, y3, train_mode=True)
    x4, y4 = synthetic_clips(2, seed=8)
    torch.manual_seed(0)
    model_golden("cnn_bgru_golden.npz", R_cb.Network(), x4, y4, train_mode=True)
    x5, y5 = synthetic_clips(4, seed=9)
    torch.manual_seed(0)
    model_golden("spec_cnn_golden.npz", R_sc.Network(), x5, y5, train_mode=False)
    # the analyst's input: 4 concatenated 12-way softmax vectors per clip (analyst_training.py:94-99)
    lg = np.random.default_rng(10).normal(0, 3, (6, 4, 12))
    probs = (np.exp(lg) / np.exp(lg).sum(-1, keepdims=True)).reshape(6, 48).astype(np.float32)
    torch.manual_seed(0)
    model_golden("analyst_golden.npz", R_an.Network(), probs, np.array([0, 3, 11, 5, 5, 10]), train_mode=True)
    # ---- plugin eval helpers (SURVEY.md §8c "Python-harness rows" item 3)
    torch.manual_seed(0)
    eval_helpers_golden("eval_helpers_fbanks_cnn_golden.npz", R_fb, OM.FbanksCNN, seed=61)
    eval_helpers_golden("eval_helpers_mfcc_bgru_golden.npz", R_mb, OM.MfccBGRU, seed=62)


if __name__ == "__main__":
    main()
