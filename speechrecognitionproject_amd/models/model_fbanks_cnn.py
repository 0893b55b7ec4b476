"""Drop-in for the reference plugin ``models/model_fbanks_cnn.py``: log-mel filter banks (98 x 120)
-> conv1 (7x3) -> maxpool (1,3) -> conv2 (1x7) -> maxpool (1,4) -> conv3 (1x10) -> conv4 (7x1)
-> max over time -> dropout -> fc1 -> fc2, no nonlinearities (model_fbanks_cnn.py:68-147).

Same constructor, ``state_dict`` keys/shapes and helpers.  The per-clip CPU ``filter_banks`` loop
(:84-87) becomes one batched HIP launch (K2); conv1 + maxpool1 run as one fused one-channel kernel
(srk_conv1_pool_*: the pre-pool activation is never written), conv2-4 as channels-last implicit GEMMs
on the matrix cores (K6), conv2's maxpool in its GEMM epilogue (srk_conv2d_nhwc_fwd_pool).
"""
import torch
import torch.nn as nn

from .. import features
from ..nn import Conv2d, Dropout, Linear, MaxPool1d, MaxPool2d, conv1_pool, conv_pool
from ._common import DEVICE, accuracy, class_accuracy   # noqa: F401


def filter_banks(sample):
    """FloatTensor[16000] -> FloatTensor[98, 120] (time x mel) on the CPU (model_fbanks_cnn.py:15-66)."""
    return features.fbank(sample.reshape(1, -1))[0].cpu()


class Network(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = Conv2d(1, 64, kernel_size=(7, 3), padding=(3, 1))
        self.maxpool1 = MaxPool2d((1, 3))
        self.conv2 = Conv2d(64, 128, (1, 7), padding=(0, 3))
        self.maxpool2 = MaxPool2d((1, 4))
        self.conv3 = Conv2d(128, 256, (1, 10))
        self.conv4 = Conv2d(256, 512, (7, 1), padding=(3, 0))
        self.maxpool3 = MaxPool1d(98)
        self.dropout = Dropout()
        self.fc1 = Linear(512, 256)
        self.fc2 = Linear(256, 12)

    def forward(self, x):
        with torch.no_grad():
            inx = features.fbank(x)                       # [B, 98, 120]
        # fused conv1 + maxpool1: NHWC [B, 98, 40, 64] (its fp32 copy skipped when conv2 reads the 16-bit one)
        h = conv1_pool(inx, self.conv1, self.maxpool1, next_conv_pool16=True)
        h = conv_pool(h, self.conv2, self.maxpool2)      # fused conv2 + maxpool2: [B, 98, 10, 128]
        h = self.conv4(self.conv3(h))                     # [B, 98, 1, 512]
        h = self.maxpool3(h.squeeze(2)).squeeze(1)        # [B, 512]
        h = self.dropout(h)
        return self.fc2(self.fc1(h))
