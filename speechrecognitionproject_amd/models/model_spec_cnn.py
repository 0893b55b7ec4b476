"""Drop-in for the reference plugin ``models/model_spec_cnn.py``: log spectrogram (49 x 321,
time x frequency) -> conv1 (3x7) -> maxpool (1,5) -> conv2 (1x7) -> maxpool (1,5) -> conv3 (1x12)
-> conv4 (5x1) -> max over time -> dropout -> fc1 -> fc2, no nonlinearities
(model_spec_cnn.py:12-57).

Same constructor, ``state_dict`` keys/shapes and helpers.  ``bn1`` (BatchNorm2d(1), :23) is
constructed but never called by the reference's forward; it is kept (a plain torch module, so
reference checkpoints load) and likewise unused.  The per-clip CPU ``compute_spec`` loop (:39-41)
becomes one batched HIP launch (K3, transposed output), conv1 + maxpool1 run as one fused
one-channel kernel (srk_conv1_pool_*), conv2-4 as channels-last implicit GEMMs (K6).
"""
import torch
import torch.nn as nn

from .. import features
from ..nn import Conv2d, Dropout, Linear, MaxPool1d, MaxPool2d, conv1_pool
from ._common import DEVICE, accuracy, class_accuracy   # noqa: F401


def compute_spec(sample):
    """FloatTensor[16000] -> FloatTensor[49, 321] (time x freq) on the CPU (model_spec_cnn.py:12-18)."""
    return features.spec(sample.reshape(1, -1), transposed=True)[0].cpu()


class Network(nn.Module):
    def __init__(self):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(1)
        self.conv1 = Conv2d(1, 64, (3, 7), padding=(1, 3))
        self.maxpool1 = MaxPool2d((1, 5))
        self.conv2 = Conv2d(64, 128, (1, 7), padding=(0, 3))
        self.maxpool2 = MaxPool2d((1, 5))
        self.conv3 = Conv2d(128, 256, (1, 12))
        self.conv4 = Conv2d(256, 512, (5, 1), padding=(2, 0))
        self.maxpool3 = MaxPool1d(49)
        self.dropout = Dropout(0.5)
        self.fc1 = Linear(512, 256)
        self.fc2 = Linear(256, 12)

    def forward(self, x):
        with torch.no_grad():
            inx = features.spec(x, transposed=True)        # [B, 49, 321]
        h = conv1_pool(inx, self.conv1, self.maxpool1)   # fused conv1 + maxpool1: NHWC [B, 49, 64, 64]
        h = self.maxpool2(self.conv2(h))                  # [B, 49, 12, 128]
        h = self.conv4(self.conv3(h))                     # [B, 49, 1, 512]
        h = self.maxpool3(h.squeeze(2)).squeeze(1)        # [B, 512]
        h = self.dropout(h)
        return self.fc2(self.fc1(h))
