import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from speechrecognitionproject_amd import features as K
from speechrecognitionproject_amd.synthetic import synthetic_clips
which = sys.argv[1] if len(sys.argv) > 1 else "mfcc"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
x, _ = synthetic_clips(1024, seed=123)
xd = torch.from_numpy(x).cuda().repeat(n // 1024, 1)
# the models' layouts (bench.py feature_roofline): MFCC time-major, spectrogram transposed
fn = {"mfcc": lambda x: K.mfcc(x, time_major=True), "spec": lambda x: K.spec(x, transposed=True),
      "fbank": K.fbank}[which]
for _ in range(3):
    fn(xd)
torch.cuda.synchronize()
