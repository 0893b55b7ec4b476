"""Drop-in for the reference plugin ``models/model_resnet_bgru.py``: raw-waveform ResNet-18-style
1-D front end (Conv1d k=80/s=16 stem, 4 stages x 2 BasicBlocks with k=15 convs, BatchNorm, ReLU)
-> Linear(512, 512) per step -> 2-layer BiGRU(512) -> Linear(1024, 12) on the last step
(model_resnet_bgru.py:14-150).

Same constructor ``Network(num_features=512, num_layers=2, mode=0)``, ``state_dict`` keys/shapes
(including the ``mode == 1`` backend head, :57-71, so reference checkpoints load) and helpers.
Activations stay channels-last [B, L, C] through the ResNet, so the reference's transpose before
``fc1`` (:107-111) is free.  Convolutions = K6, BatchNorm(+residual+ReLU) = K9, GRU = K5.
``mode == 1`` (the auxiliary backend of the staged training, :57-71, :113-118) runs on the same
kernels: the fc1 output's 125 time steps are the backend's channels, so the [B, 125, 512] view is
transposed to channels-last [B, 512, 125] once, then K6 1-D convs, K9 BatchNorm (+ReLU; 250 / 125
channels on zero-padded float4 groups), the channels-last max-pool, the length mean and two Linear
layers give [B, 12] logits; the GRU is skipped (:147-149).

BatchNorm under data parallelism uses per-rank batch statistics.
"""
import torch
import torch.nn as nn

from ..nn import BatchNorm1d, BiGRU, Conv1d, Linear, MaxPool1d, conv1d_nlc, last_step
from ._common import DEVICE, accuracy, class_accuracy   # noqa: F401


def _kaiming(conv):
    nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")


class BasicBlock(nn.Module):
    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.kernel_size, self.padding = 15, 7
        self.conv1 = Conv1d(inplanes, planes, 15, stride=stride, padding=7, bias=False)
        self.bn1 = BatchNorm1d(planes)
        self.conv2 = Conv1d(planes, planes, 15, stride=1, padding=7, bias=False)
        self.bn2 = BatchNorm1d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        residual = x
        if self.downsample is not None:
            residual = self.downsample[1](self.downsample[0](x))
        out = self.bn1(self.conv1(x), relu=True)
        return self.bn2(self.conv2(out), residual=residual, relu=True)


class ResNet(nn.Module):
    def __init__(self, block, mode):
        super().__init__()
        self.mode = mode
        self.inplanes = 64
        self.dim = 125
        self.conv1 = Conv1d(1, 64, kernel_size=80, stride=16, padding=38, bias=False)
        self.bn1 = BatchNorm1d(64)
        self.relu = nn.ReLU(inplace=True)
        self.layer1 = self._make_layer(block, 64, 2)
        self.layer2 = self._make_layer(block, 128, 2, stride=2)
        self.layer3 = self._make_layer(block, 256, 2, stride=2)
        self.layer4 = self._make_layer(block, 512, 2, stride=2)
        self.fc1 = Linear(512, 512)
        # mode == 1 auxiliary head (model_resnet_bgru.py:57-71): same module indices / state_dict keys;
        # the ReLUs are fused into the BatchNorm kernels in forward
        self.backend_conv1 = nn.Sequential(
            Conv1d(self.dim, 2 * self.dim, 5, stride=2, padding=0, bias=False), BatchNorm1d(2 * self.dim), nn.ReLU(True),
            MaxPool1d(2),
            Conv1d(2 * self.dim, 4 * self.dim, 5, stride=2, padding=0, bias=False), BatchNorm1d(4 * self.dim),
            nn.ReLU(True))
        self.backend_conv2 = nn.Sequential(
            Linear(4 * self.dim, self.dim), BatchNorm1d(self.dim), nn.ReLU(True), Linear(self.dim, 12))
        for m in self.modules():
            if isinstance(m, (Conv1d, nn.Conv1d)):
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
        # x: [B, L, 1] channels-last waveform
        x = self.bn1(self.conv1(x), relu=True)            # [B, 1000, 64]
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))   # [B, 125, 512]
        bs, sl, _ = x.shape
        x = self.fc1(x.reshape(bs * sl, -1))
        if self.mode == 1:   # :113-117, channels = the sl time steps, length = the 512 features
            x = x.view(bs, sl, 512).transpose(1, 2).contiguous()     # [B, 512, sl] channels-last
            conv_a, bn_a, _, pool, conv_b, bn_b, _ = self.backend_conv1
            # 250 channels run as 252 (float4 groups for K9 and the pool): conv_a gets 2 zero output
            # filters, BatchNorm keeps them 0, conv_b gets 2 zero input channels
            pa = (-conv_a.out_channels) % 4
            wa = torch.cat([conv_a.weight, conv_a.weight.new_zeros((pa,) + tuple(conv_a.weight.shape[1:]))])
            wb = torch.cat([conv_b.weight, conv_b.weight.new_zeros((conv_b.out_channels, pa, conv_b.kernel_size[0]))], 1)
            x = bn_a.forward_padded(conv1d_nlc(x, wa, None, conv_a.stride[0]), relu=True)   # [B, 254, 252]
            x = bn_b(conv1d_nlc(pool(x), wb, None, conv_b.stride[0]), relu=True)           # [B, 62, 500]
            fc_a, bn_h, _, fc_b = self.backend_conv2
            return fc_b(bn_h(fc_a(x.mean(1)), relu=True))            # torch.mean(x, 2) of the NCL layout
        return x.view(bs, sl, 512)


class GRU(nn.Module):
    def __init__(self, num_features=512, num_layers=2):
        super().__init__()
        self.gru = BiGRU(512, num_features, num_layers=num_layers, bidirectional=True, batch_first=True)
        self.fc2 = Linear(num_features * 2, 12)

    def forward(self, x):
        x, _ = self.gru(x)
        return self.fc2(last_step(x))


class Network(nn.Module):
    def __init__(self, num_features=512, num_layers=2, mode=0):
        super().__init__()
        self.mode = mode
        self.resnet = ResNet(BasicBlock, mode=mode)
        self.gru = GRU(num_features=num_features, num_layers=num_layers)

    def forward(self, x):
        if not torch.is_tensor(x):
            x = torch.as_tensor(x)
        x = x.to(DEVICE, torch.float32).reshape(x.shape[0], -1, 1)   # [B, 16000, 1]
        x = self.resnet(x)
        if self.mode != 1:
            x = self.gru(x)
        return x
