"""Drop-in for the reference plugin ``models/model_analyst.py``: the stacking head of the
ensemble — Linear(48, 96) -> Linear(96, 12) (no nonlinearity) over the concatenated softmax
outputs of four frozen base models (model_analyst.py:10-20), and its ``accuracy(models, dataset,
filename, batchsize=1)`` with ``models = [analyst, m1, m2, m3, m4]`` (:22-53).

The softmax/concat of the base models' outputs is K11 (evaluation.stacked_inputs), one launch
per batch instead of four host-side softmaxes per clip.
"""
import torch
import torch.nn as nn
from torch.utils.data import DataLoader

from ..evaluation import stacked_inputs
from ..nn import Linear
from ._common import DEVICE


class Network(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = Linear(48, 96)
        self.fc2 = Linear(96, 12)

    def forward(self, x):
        x = torch.as_tensor(x).to(DEVICE, torch.float32)
        return self.fc2(self.fc1(x))


def accuracy(models, dataset, filename, batchsize=1):
    """Accuracy (%) of the stacked ensemble; appends one line to ``filename``.  Every clip counts
    once (the reference's loop is batch_size=1 with ``total += 1``, :38-49), for any ``batchsize``."""
    analyst, bases = models[0], models[1:5]
    analyst.eval()
    total, correct = 0, 0
    data = DataLoader(dataset, batch_size=batchsize, drop_last=False)
    with torch.no_grad():
        for batch in data:
            outputs = analyst(stacked_inputs(bases, batch['audio']))
            _, predicted = torch.max(outputs.data, 1)
            total += predicted.shape[0]
            correct += (predicted == batch['label'].to(outputs.device)).sum().item()
    with open(filename, 'a') as f:
        f.write(str(100 * correct / float(total)) + '\n')
    analyst.train()
    return 100 * correct / float(total)
