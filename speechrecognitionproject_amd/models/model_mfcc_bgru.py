"""Drop-in for the reference plugin ``models/model_mfcc_bgru.py``: MFCC(+deltas) -> 2-layer
BiGRU(39 -> 512) -> Linear(1024 -> 12) on the last time step.

Same constructor signature, ``state_dict`` keys/shapes and helpers as the reference
(model_mfcc_bgru.py:11-82).  The difference is where the arithmetic runs: the per-clip CPU
librosa loop (:29-32) becomes ONE batched HIP kernel launch (K1, srk_mfcc_fwd) on the device,
and the GRU / Linear run on the hand-written kernels of libsrk.so.
"""
import torch
import torch.nn as nn

from .. import features
from ..nn import BiGRU, Linear, last_step
from ._common import DEVICE, accuracy, class_accuracy   # noqa: F401  (plugin API)


def compute_mfcc(sample):
    """FloatTensor[16000] (int16-valued) -> FloatTensor[39, 51] on the CPU, like the reference
    (model_mfcc_bgru.py:11-19); computed by the K1 kernel."""
    return features.mfcc(sample.reshape(1, -1))[0].cpu()


class Network(nn.Module):
    """features="mfcc39x51" is the reference model.  features="mfcc40x98" is a PERF-ONLY, NON-REFERENCE
    variant for BASELINE.json configs[1]'s literal "MFCC (40x98)" (features.mfcc40x98: 40 MFCCs over 98
    frames, GRU input 40, 98 steps) — its state_dict differs in the first GRU layer."""

    def __init__(self, num_features=512, num_layers=2, features="mfcc39x51"):
        super().__init__()
        if features not in ("mfcc39x51", "mfcc40x98"):
            raise ValueError("features must be 'mfcc39x51' (the reference) or 'mfcc40x98' (perf-only)")
        self.features = features
        n_in = 39 if features == "mfcc39x51" else 40
        self.gru = BiGRU(n_in, num_features, num_layers=num_layers, bidirectional=True, batch_first=True)
        self.fc = Linear(num_features * 2, 12)

    def forward(self, x):
        with torch.no_grad():
            if self.features == "mfcc39x51":
                inx = features.mfcc(x, time_major=True)     # [B, 51, 39] = transpose(mfcc, 1, 2)
            else:
                inx = features.mfcc40x98(x)                 # [B, 98, 40] (perf-only variant)
        inx, _ = self.gru(inx)
        return self.fc(last_step(inx))
