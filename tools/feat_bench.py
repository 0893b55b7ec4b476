"""Time the feature kernels on a large batch (HBM roofline check)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from speechrecognitionproject_amd import _lib, features as K
from speechrecognitionproject_amd.synthetic import synthetic_clips
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
x, _ = synthetic_clips(1024, seed=123)
xd = torch.from_numpy(x).cuda().repeat(n // 1024, 1)
res = {}
for name, fn in [("mfcc", lambda: K.mfcc(xd, time_major=True)), ("mfcc_coef_major", lambda: K.mfcc(xd)), ("fbank", lambda: K.fbank(xd)), ("spec", lambda: K.spec(xd, transposed=True)), ("spec_freq_major", lambda: K.spec(xd))]:
    if os.environ.get("FEAT_ONLY") and name not in os.environ["FEAT_ONLY"].split(","):
        continue
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    _lib.prof_enable(True)
    for _ in range(5):
        fn()
    c, ms, w = _lib.prof_read(name.split("_")[0])
    _lib.prof_enable(False)
    res[name] = {"ms": round(ms / c, 3), "GB/s": round(w / (ms * 1e-3) / 1e9, 1), "frac_8TBs": round(w / (ms * 1e-3) / 8e12, 4)}
print(json.dumps(res))
