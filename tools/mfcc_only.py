import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from speechrecognitionproject_amd import features as K
from speechrecognitionproject_amd.synthetic import synthetic_clips
which = sys.argv[1] if len(sys.argv) > 1 else "mfcc"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
x, _ = synthetic_clips(1024, seed=123)
xd = torch.from_numpy(x).cuda().repeat(n // 1024, 1)
for _ in range(3):
    getattr(K, which)(xd)
torch.cuda.synchronize()
