"""Drop-in for the reference plugin ``models/model_mfrn_bgru.py`` (the literal
"MFCC + CNN-BiGRU"): MFCC(+deltas) [51 x 39] concatenated with a raw-waveform ResNet-1D branch
(Conv1d(1, 64, 640, stride 40, padding 320) stem -> 401 steps, 4 stages x 2 BasicBlocks with k=15
convs, BatchNorm, ReLU -> 51 steps, Linear(512, 512) per step) -> 2-layer BiGRU(551 -> 512) ->
Linear(1024, 12) on the last step (model_mfrn_bgru.py:11-140).

Same constructor ``Network(num_features=512, num_layers=2)``, ``state_dict`` keys/shapes and
helpers.  MFCC = K1 (one batched launch instead of the per-clip librosa loop, :128-131), convs =
K6 (channels-last implicit GEMM), BatchNorm(+residual+ReLU) = K9, GRU = K5, Linear = GEMM.  The
branch concatenation (:135) is the only torch op on the path (a [B, 51, 551] copy).
"""
import torch
import torch.nn as nn

from .. import features
from ..nn import BatchNorm1d, BiGRU, Conv1d, Linear, last_step
from ._common import DEVICE, accuracy, class_accuracy   # noqa: F401  (plugin API)
from .model_mfcc_bgru import compute_mfcc               # noqa: F401  (same function, :11-19)
from .model_resnet_bgru import BasicBlock, _kaiming


class ResNet(nn.Module):
    """model_mfrn_bgru.py:49-106 (no auxiliary backend head, unlike model_resnet_bgru)."""

    def __init__(self, block):
        super().__init__()
        self.inplanes = 64
        self.conv1 = Conv1d(1, 64, kernel_size=640, stride=40, padding=320, bias=False)
        self.bn1 = BatchNorm1d(64)
        self.relu = nn.ReLU(inplace=True)
        self.layer1 = self._make_layer(block, 64, 2)
        self.layer2 = self._make_layer(block, 128, 2, stride=2)
        self.layer3 = self._make_layer(block, 256, 2, stride=2)
        self.layer4 = self._make_layer(block, 512, 2, stride=2)
        self.fc1 = Linear(512, 512)
        for m in self.modules():
            if isinstance(m, Conv1d):
                _kaiming(m)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes:
            downsample = nn.Sequential(Conv1d(self.inplanes, planes, kernel_size=1, stride=stride, bias=False),
                                       BatchNorm1d(planes))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        # x: [B, 16000, 1] channels-last waveform
        x = self.bn1(self.conv1(x), relu=True)                        # [B, 401, 64]
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))     # [B, 51, 512]
        bs, sl, _ = x.shape
        return self.fc1(x.reshape(bs * sl, -1)).view(bs, sl, 512)


class GRU(nn.Module):
    def __init__(self, num_features=512, num_layers=2):
        super().__init__()
        self.gru = BiGRU(551, num_features, num_layers=num_layers, bidirectional=True, batch_first=True)
        self.fc2 = Linear(num_features * 2, 12)

    def forward(self, x):
        x, _ = self.gru(x)
        return self.fc2(last_step(x))


class Network(nn.Module):
    def __init__(self, num_features=512, num_layers=2):
        super().__init__()
        self.resnet = ResNet(BasicBlock)
        self.gru = GRU(num_features=num_features, num_layers=num_layers)

    def forward(self, x):
        with torch.no_grad():
            mfcc = features.mfcc(x, time_major=True)                 # [B, 51, 39] (:128-131)
        if not torch.is_tensor(x):
            x = torch.as_tensor(x)
        x = x.to(mfcc.device, torch.float32).reshape(x.shape[0], -1, 1)
        r = self.resnet(x)                                            # [B, 51, 512]
        return self.gru(torch.cat((r, mfcc), 2))                      # (:135-136)
