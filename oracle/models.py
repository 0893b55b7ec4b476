"""CPU restatement of the reference acoustic models — TEST INFRASTRUCTURE ONLY.

PyTorch-CPU modules with the reference's arithmetic (fp32, torch.nn.GRU / Conv / Linear on the
CPU), fed by the numpy feature oracle of ``oracle/features.py`` in a per-clip Python loop exactly
as the reference's ``forward`` does.  Used by the parity tests as the checker and by
``bench.py``'s ``cpu_baseline`` leg ("kind": "port").  Never imported by the product package.

Pinned by ``tests/golden/*_golden.npz`` (generated from the reference modules themselves by
``tests/golden/make_golden.py``): logits, loss, sampled gradients and the 1-step Adam update.
"""
import numpy as np
import torch
import torch.nn as nn

from . import features as F

NUM_CLASSES = 12


def seeded_state_dict(module, seed=0):
    """Deterministic weights shared by the reference, the oracle and the HIP path:
    every tensor ~ U(-a, a), a = 1/sqrt(fan_in) of its owning weight (BN weight=1, bias=0,
    running stats default).  Keys iterate in ``state_dict`` order."""
    rng = np.random.default_rng(seed)
    sd = module.state_dict()
    out = {k: v.clone() for k, v in sd.items()}
    for mname, m in module.named_modules():
        pre = mname + "." if mname else ""
        if isinstance(m, nn.GRU):
            a = 1.0 / np.sqrt(m.hidden_size)
            names = [n for n, _ in m.named_parameters(recurse=False)]
        elif isinstance(m, (nn.Conv1d, nn.Conv2d, nn.Linear)):
            a = 1.0 / np.sqrt(int(np.prod(m.weight.shape[1:])))
            names = [n for n, _ in m.named_parameters(recurse=False)]
        else:
            continue   # BatchNorm keeps weight=1, bias=0, running stats (0, 1)
        for n in names:
            k = pre + n
            out[k] = torch.from_numpy(rng.uniform(-a, a, tuple(sd[k].shape)).astype(np.float32))
    return out


# ---------------------------------------------------------------- model_mfcc_bgru.py:21-37
class MfccBGRU(nn.Module):
    def __init__(self, num_features=512, num_layers=2):
        super().__init__()
        self.gru = nn.GRU(39, hidden_size=num_features, num_layers=num_layers, bidirectional=True, batch_first=True)
        self.fc = nn.Linear(num_features * 2, NUM_CLASSES)

    @staticmethod
    def features(x):
        return torch.from_numpy(np.stack([F.compute_mfcc(c) for c in x.numpy()]))   # per clip, :31-32

    def forward(self, x):
        with torch.no_grad():
            inx = self.features(x)
        out, _ = self.gru(inx.transpose(1, 2))
        return self.fc(out[:, -1, :])


# ---------------------------------------------------------------- model_spec_bgru.py:19-35
class SpecBGRU(nn.Module):
    def __init__(self, num_features=512, num_layers=2):
        super().__init__()
        self.gru = nn.GRU(321, hidden_size=num_features, num_layers=num_layers, bidirectional=True, batch_first=True)
        self.fc = nn.Linear(num_features * 2, NUM_CLASSES)

    @staticmethod
    def features(x):
        return torch.from_numpy(np.stack([F.compute_spec(c) for c in x.numpy()]))

    def forward(self, x):
        with torch.no_grad():
            inx = self.features(x)
        out, _ = self.gru(inx.transpose(1, 2))
        return self.fc(out[:, -1, :])


class MaskDropout(nn.Module):
    """``nn.Dropout(p)`` with the Bernoulli(1 - p) keep mask supplied instead of drawn:
    y = x * keep / (1 - p) in training mode, identity in eval (the draw the reference's
    model_fbanks_cnn.py:79,98 would make is exported into the golden fixture instead)."""

    def __init__(self, keep, p=0.5):
        super().__init__()
        self.keep, self.p = torch.as_tensor(keep, dtype=torch.float32), p

    def forward(self, x):
        return x * self.keep / (1.0 - self.p) if self.training else x


# ---------------------------------------------------------------- model_fbanks_cnn.py:68-102
class FbanksCNN(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 64, kernel_size=(7, 3), padding=(3, 1))
        self.maxpool1 = nn.MaxPool2d((1, 3))
        self.conv2 = nn.Conv2d(64, 128, (1, 7), padding=(0, 3))
        self.maxpool2 = nn.MaxPool2d((1, 4))
        self.conv3 = nn.Conv2d(128, 256, (1, 10))
        self.conv4 = nn.Conv2d(256, 512, (7, 1), padding=(3, 0))
        self.maxpool3 = nn.MaxPool1d(98)
        self.dropout = nn.Dropout()
        self.fc1 = nn.Linear(512, 256)
        self.fc2 = nn.Linear(256, NUM_CLASSES)

    @staticmethod
    def features(x):
        return torch.from_numpy(np.stack([F.filter_banks(c) for c in x.numpy()]))

    def forward_features(self, inx):
        h = self.maxpool1(self.conv1(inx.unsqueeze(1)))
        h = self.maxpool2(self.conv2(h))
        h = self.conv4(self.conv3(h)).squeeze(3)
        h = self.maxpool3(h).squeeze(2)
        return self.fc2(self.fc1(self.dropout(h)))

    def forward(self, x):
        with torch.no_grad():
            inx = self.features(x)
        return self.forward_features(inx)


# ---------------------------------------------------------------- model_resnet_bgru.py:14-150
class _Block(nn.Module):
    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv1d(inplanes, planes, 15, stride=stride, padding=7, bias=False)
        self.bn1 = nn.BatchNorm1d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv1d(planes, planes, 15, stride=1, padding=7, bias=False)
        self.bn2 = nn.BatchNorm1d(planes)
        self.downsample = downsample

    def forward(self, x):
        res = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + res)


class _ResNet1d(nn.Module):
    def __init__(self, stem=(80, 16, 38), backend=True, mode=0):
        super().__init__()
        self.mode = mode
        self.inplanes = 64
        k, st, pd = stem
        self.conv1 = nn.Conv1d(1, 64, kernel_size=k, stride=st, padding=pd, bias=False)
        self.bn1 = nn.BatchNorm1d(64)
        self.relu = nn.ReLU(inplace=True)
        self.layer1 = self._layer(64, 2)
        self.layer2 = self._layer(128, 2, 2)
        self.layer3 = self._layer(256, 2, 2)
        self.layer4 = self._layer(512, 2, 2)
        self.fc1 = nn.Linear(512, 512)
        if not backend:   # model_mfrn_bgru.py:49-66 has no auxiliary head
            return
        dim = 125   # the mode==1 backend exists in the state_dict (model_resnet_bgru.py:57-71)
        self.backend_conv1 = nn.Sequential(
            nn.Conv1d(dim, 2 * dim, 5, 2, 0, bias=False), nn.BatchNorm1d(2 * dim), nn.ReLU(True),
            nn.MaxPool1d(2, 2),
            nn.Conv1d(2 * dim, 4 * dim, 5, 2, 0, bias=False), nn.BatchNorm1d(4 * dim), nn.ReLU(True))
        self.backend_conv2 = nn.Sequential(
            nn.Linear(4 * dim, dim), nn.BatchNorm1d(dim), nn.ReLU(True), nn.Linear(dim, NUM_CLASSES))

    def _layer(self, planes, blocks, stride=1):
        ds = None
        if stride != 1 or self.inplanes != planes:
            ds = nn.Sequential(nn.Conv1d(self.inplanes, planes, 1, stride=stride, bias=False), nn.BatchNorm1d(planes))
        layers = [_Block(self.inplanes, planes, stride, ds)]
        self.inplanes = planes
        layers += [_Block(planes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.relu(self.bn1(self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        b, _, t = x.shape
        x = self.fc1(x.transpose(1, 2).reshape(b * t, -1))
        if self.mode == 1:   # model_resnet_bgru.py:113-117: the time steps are the backend's channels
            x = self.backend_conv1(x.view(b, t, 512))
            return self.backend_conv2(torch.mean(x, 2))
        return x.view(b, t, 512)


class _GRUHead(nn.Module):
    def __init__(self, num_features=512, num_layers=2, input_size=512):
        super().__init__()
        self.gru = nn.GRU(input_size, hidden_size=num_features, num_layers=num_layers, bidirectional=True,
                          batch_first=True)
        self.fc2 = nn.Linear(num_features * 2, NUM_CLASSES)

    def forward(self, x):
        out, _ = self.gru(x)
        return self.fc2(out[:, -1, :])


class ResnetBGRU(nn.Module):
    def __init__(self, num_features=512, num_layers=2, mode=0):
        super().__init__()
        self.mode = mode
        self.resnet = _ResNet1d(mode=mode)
        self.gru = _GRUHead(num_features, num_layers)

    def forward(self, x):   # model_resnet_bgru.py:145-150: mode 1 returns the backend head's logits
        x = self.resnet(x.float().unsqueeze(1))
        return x if self.mode == 1 else self.gru(x)


# ---------------------------------------------------------------- model_mfrn_bgru.py:11-140
class MfrnBGRU(nn.Module):
    """MFCC [51, 39] (per clip, as compute_mfcc) concatenated with a raw-wave ResNet-1D (stem
    Conv1d(1, 64, 640, stride 40, padding 320) -> 401 -> 51 steps) + fc1, then BiGRU(551) + fc2."""

    def __init__(self, num_features=512, num_layers=2):
        super().__init__()
        self.resnet = _ResNet1d(stem=(640, 40, 320), backend=False)
        self.gru = _GRUHead(num_features, num_layers, input_size=551)

    @staticmethod
    def features(x):
        return torch.from_numpy(np.stack([F.compute_mfcc(c) for c in x.numpy()]))

    def forward(self, x):
        with torch.no_grad():
            mf = self.features(x).transpose(1, 2)               # [B, 51, 39] (:128-131)
        r = self.resnet(x.float().unsqueeze(1))                 # [B, 51, 512] (:133)
        return self.gru(torch.cat((r, mf), 2))                  # (:135-136)


# ---------------------------------------------------------------- model_cnn_bgru.py:11-56
class _CNN1d(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv1d(1, 64, kernel_size=80, stride=4, padding=38, bias=False)
        self.bn1 = nn.BatchNorm1d(64)
        self.conv2 = nn.Conv1d(64, 128, kernel_size=4, stride=2, padding=0, bias=False)
        self.bn2 = nn.BatchNorm1d(128)
        self.conv3 = nn.Conv1d(128, 256, kernel_size=4, stride=2, padding=0, bias=False)
        self.bn3 = nn.BatchNorm1d(256)
        self.conv4 = nn.Conv1d(256, 512, kernel_size=4, stride=2, padding=0, bias=False)
        self.bn4 = nn.BatchNorm1d(512)
        self.fc = nn.Linear(512, 512)

    def forward(self, x):
        for i in range(1, 5):
            x = torch.relu(getattr(self, "bn%d" % i)(getattr(self, "conv%d" % i)(x)))
        return self.fc(x.transpose(1, 2))


class CnnBGRU(nn.Module):
    """Raw wave [B, 16000] -> 4 strided Conv1d + BN + ReLU (T = 498) -> fc -> BiGRU(512) -> fc2."""

    def __init__(self):
        super().__init__()
        self.cnn = _CNN1d()
        self.gru = _GRUHead(512, 2)

    def forward(self, x):
        return self.gru(self.cnn(x.float().unsqueeze(1)))


# ---------------------------------------------------------------- model_spec_cnn.py:20-57
class SpecCNN(nn.Module):
    def __init__(self):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(1)   # constructed, never called (:23)
        self.conv1 = nn.Conv2d(1, 64, (3, 7), padding=(1, 3))
        self.maxpool1 = nn.MaxPool2d((1, 5))
        self.conv2 = nn.Conv2d(64, 128, (1, 7), padding=(0, 3))
        self.maxpool2 = nn.MaxPool2d((1, 5))
        self.conv3 = nn.Conv2d(128, 256, (1, 12))
        self.conv4 = nn.Conv2d(256, 512, (5, 1), padding=(2, 0))
        self.maxpool3 = nn.MaxPool1d(49)
        self.dropout = nn.Dropout(0.5)
        self.fc1 = nn.Linear(512, 256)
        self.fc2 = nn.Linear(256, NUM_CLASSES)

    @staticmethod
    def features(x):
        return torch.from_numpy(np.stack([F.compute_spec(c).T for c in x.numpy()]))   # [B, 49, 321]

    def forward(self, x):
        with torch.no_grad():
            inx = self.features(x)
        h = self.maxpool1(self.conv1(inx.unsqueeze(1)))
        h = self.maxpool2(self.conv2(h))
        h = self.conv4(self.conv3(h)).squeeze(3)
        h = self.maxpool3(h).squeeze(2)
        return self.fc2(self.fc1(self.dropout(h)))


# ---------------------------------------------------------------- models/model_analyst.py:10-20
class Analyst(nn.Module):
    """Stacking head over 4 x 12 softmax outputs: fc1 (48 -> 96) -> fc2 (96 -> 12), no activation."""

    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(48, 96)
        self.fc2 = nn.Linear(96, NUM_CLASSES)

    def forward(self, x):
        return self.fc2(self.fc1(x.float()))


def train_step(model, x, labels, lr=1e-4, optimizer=None):
    """One training.py:85-91 step on the CPU: zero_grad, forward, CE(mean), backward, Adam."""
    crit = nn.CrossEntropyLoss()
    opt = optimizer or torch.optim.Adam(model.parameters(), lr=lr)
    opt.zero_grad()
    out = model(x)
    loss = crit(out, labels)
    loss.backward()
    opt.step()
    return out.detach(), loss.detach(), opt
