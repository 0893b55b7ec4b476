"""Debug helper: run the feature kernels on the golden + synthetic clips, save raw outputs."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from speechrecognitionproject_amd import features as K
from speechrecognitionproject_amd.synthetic import synthetic_clips
g = np.load("tests/golden/fbank_golden.npz")
x = np.concatenate([g["pcm"], synthetic_clips(16, seed=11)[0]])
xt = torch.from_numpy(x)
np.savez("gpurun_out/feat_dump.npz", pcm=x, fbank=K.fbank(xt).cpu().numpy(), spec=K.spec(xt).cpu().numpy(),
         mfcc=K.mfcc(xt).cpu().numpy())
print("ok")
