"""Drop-in for the reference plugin ``models/model_cnn_bgru.py``: raw-waveform 1-D CNN
(Conv1d(1, 64, k80, s4, p38) -> 3 x Conv1d(k4, s2), each + BatchNorm + ReLU, no biases)
-> Linear(512, 512) per step -> 2-layer BiGRU(512) over T = 498 steps -> Linear(1024, 12) on the
last step (model_cnn_bgru.py:11-56).

Same constructor ``Network()``, ``state_dict`` keys/shapes (``cnn.*``, ``gru.gru.*``, ``gru.fc2.*``)
and helpers.  Activations stay channels-last [B, L, C], so the reference's transpose before ``fc``
(:29) is free.  Convolutions = K6 implicit GEMMs, BatchNorm + ReLU = K9 (one fused kernel per
layer), GRU = K5 (the persistent recurrence; T = 498 is ten times the MFCC model's 51 steps).
BatchNorm under data parallelism uses per-rank batch statistics.
"""
import torch
import torch.nn as nn

from ..nn import BatchNorm1d, BiGRU, Conv1d, Linear, last_step
from ._common import DEVICE, accuracy, class_accuracy   # noqa: F401


class CNN(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = Conv1d(1, 64, kernel_size=80, stride=4, padding=38, bias=False)
        self.bn1 = BatchNorm1d(64)
        self.conv2 = Conv1d(64, 128, kernel_size=4, stride=2, padding=0, bias=False)
        self.bn2 = BatchNorm1d(128)
        self.conv3 = Conv1d(128, 256, kernel_size=4, stride=2, padding=0, bias=False)
        self.bn3 = BatchNorm1d(256)
        self.conv4 = Conv1d(256, 512, kernel_size=4, stride=2, padding=0, bias=False)
        self.bn4 = BatchNorm1d(512)
        self.fc = Linear(512, 512)

    def forward(self, x):
        # x: [B, 16000, 1] channels-last waveform
        x = self.bn1(self.conv1(x), relu=True)   # [B, 4000, 64]
        x = self.bn2(self.conv2(x), relu=True)   # [B, 1999, 128]
        x = self.bn3(self.conv3(x), relu=True)   # [B, 998, 256]
        x = self.bn4(self.conv4(x), relu=True)   # [B, 498, 512]
        bs, sl, _ = x.shape
        return self.fc(x.reshape(bs * sl, -1)).view(bs, sl, 512)


class GRU(nn.Module):
    def __init__(self):
        super().__init__()
        self.gru = BiGRU(512, 512, num_layers=2, bidirectional=True, batch_first=True)
        self.fc2 = Linear(512 * 2, 12)

    def forward(self, x):
        x, _ = self.gru(x)
        return self.fc2(last_step(x))


class Network(nn.Module):
    def __init__(self):
        super().__init__()
        self.cnn = CNN()
        self.gru = GRU()

    def forward(self, x):
        if not torch.is_tensor(x):
            x = torch.as_tensor(x)
        x = x.to(DEVICE, torch.float32).reshape(x.shape[0], -1, 1)   # [B, 16000, 1] (:52)
        return self.gru(self.cnn(x))
