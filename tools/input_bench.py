"""Input-pipeline throughput: the reference's per-item path vs the device
pipeline, on a synthetic Kaggle-layout WAV tree written to a temporary directory.

    python tools/input_bench.py [--files 4096] [--batch 512] [--threads 16]

Prints one JSON line: clips/s of
  scipy_read        scipy.io.wavfile.read per file (the reference's decoder, dataset.py:98)
  native_read       srk_wav_read_batch (host threads) per batch
  dataset_loader    DataLoader(Dataset, batch) in training mode: per-item decode + numpy augmentation
  device_loader     DeviceBatchLoader: native decode -> pinned -> H2D -> K10 augmentation (one launch)
and the K10 kernel alone on 65,536 resident clips (algorithmic bytes / time vs 8 TB/s).
"""
import argparse
import json
import os
import random
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from speechrecognitionproject_amd import _lib, features as K              # noqa: E402
from speechrecognitionproject_amd.dataset import Dataset, DeviceBatchLoader, read_wav_batch   # noqa: E402


def make_tree(root, n_files, rng):
    from scipy.io import wavfile
    os.makedirs(root + "/_background_noise_")
    open(root + "/_background_noise_/README.md", "w").close()
    for i in range(6):
        wavfile.write(root + "/_background_noise_/n%d.wav" % i, 16000,
                      np.clip(np.rint(rng.normal(0, 2000, 960000)), -6000, 6000).astype(np.int16))
    words = ["yes", "no", "up", "down", "left", "right", "on", "off", "stop", "go", "bed", "cat"]
    names = []
    for w in words:
        os.makedirs(root + "/" + w)
    for i in range(n_files):
        w = words[i % len(words)]
        n = 16000 if i % 5 else int(rng.integers(8000, 16000))
        x = np.clip(np.rint(rng.normal(0, 3000, n)), -32768, 32767).astype(np.int16)
        wavfile.write(root + "/%s/%05d.wav" % (w, i), 16000, x)
        names.append("%s/%05d.wav" % (w, i))
    with open(root + "/training_list.txt", "w") as f:
        f.write("\n".join(names) + "\n")
    return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    from scipy.io import wavfile
    res = {}
    with tempfile.TemporaryDirectory() as root:
        rng = np.random.default_rng(0)
        names = make_tree(root, args.files, rng)
        paths = [root + "/" + n for n in names]
        t0 = time.perf_counter()
        for p in paths:
            wavfile.read(p)
        res["scipy_read"] = len(paths) / (time.perf_counter() - t0)
        read_wav_batch(paths[:args.batch], threads=args.threads)
        t0 = time.perf_counter()
        for s in range(0, len(paths), args.batch):
            read_wav_batch(paths[s:s + args.batch], threads=args.threads)
        res["native_read"] = len(paths) / (time.perf_counter() - t0)
        random.seed(0)
        np.random.seed(0)
        ds = Dataset(root + "/training_list.txt", root)
        n_items = len(ds)
        loader = torch.utils.data.DataLoader(ds, batch_size=args.batch, shuffle=True)
        t0 = time.perf_counter()
        seen = 0
        for b in loader:
            b["audio"].cuda()
            seen += len(b["label"])
            if seen >= 2048:
                break
        torch.cuda.synchronize()
        res["dataset_loader"] = seen / (time.perf_counter() - t0)
        dl = DeviceBatchLoader(ds, batch_size=args.batch, shuffle=True, threads=args.threads)
        it = iter(dl)
        next(it)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        seen = 0
        for b in it:
            seen += b["audio"].shape[0]
        torch.cuda.synchronize()
        res["device_loader"] = seen / (time.perf_counter() - t0)
        res["items"] = n_items
    # K10 alone: 65,536 resident clips, a mix of ops
    n = 65536
    rng = np.random.default_rng(1)
    pcm = torch.from_numpy(np.clip(np.rint(rng.normal(0, 3000, (4096, 16000))), -32768, 32767).astype(np.int16))
    pcm = pcm.cuda().repeat(n // 4096, 1)
    bank = torch.from_numpy(np.clip(np.rint(rng.normal(0, 2000, 6 * 960000)), -6000, 6000).astype(np.int16)).cuda()
    op = rng.integers(0, 6, n)
    ip = np.where(op == 1, (16000 * rng.uniform(0.7, 1.3, n)).astype(np.int64), rng.integers(-4800, 4801, n))
    pos = rng.integers(0, bank.numel() - 16000 + 1, n)
    dp = np.where(op == 4, 10 ** (rng.choice([-5, 0, 5, 10], n) / 10.0), rng.uniform(0, 0.1, n))
    out = torch.empty((n, 16000), device="cuda")
    for _ in range(2):
        K.augment(pcm, bank, op, ip, pos, dp, 1, out=out)
    torch.cuda.synchronize()
    _lib.prof_enable(True)
    for _ in range(5):
        K.augment(pcm, bank, op, ip, pos, dp, 1, out=out)
    cnt, ms, work = _lib.prof_read("augment")
    _lib.prof_enable(False)
    gbs = work / (ms * 1e-3) / 1e9
    res["augment_kernel"] = {"clips_per_launch": n, "ms_per_launch": round(ms / cnt, 4), "GB_s": round(gbs, 1),
                             "frac_of_8TBs": round(gbs / 8000.0, 4), "bytes_per_clip": 96000}
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
