"""Drop-in for the reference plugin ``models/model_spec_bgru.py``: log spectrogram (321 x 49)
-> 2-layer BiGRU(321 -> 512) -> Linear(1024 -> 12) on the last time step
(model_spec_bgru.py:11-79).  Spectrogram = K3 (srk_spec_fwd), GRU/Linear = libsrk kernels."""
import torch
import torch.nn as nn

from .. import features
from ..nn import BiGRU, Linear, last_step
from ._common import DEVICE, accuracy, class_accuracy   # noqa: F401


def compute_spec(sample):
    """FloatTensor[16000] -> FloatTensor[321, 49] (freq x time) on the CPU (model_spec_bgru.py:11-17)."""
    return features.spec(sample.reshape(1, -1))[0].cpu()


class Network(nn.Module):
    def __init__(self, num_features=512, num_layers=2):
        super().__init__()
        self.gru = BiGRU(321, num_features, num_layers=num_layers, bidirectional=True, batch_first=True)
        self.fc = Linear(num_features * 2, 12)

    def forward(self, x):
        with torch.no_grad():
            inx = features.spec(x, transposed=True)     # [B, 49, 321] = transpose(spec, 1, 2)
        inx, _ = self.gru(inx)
        return self.fc(last_step(inx))
