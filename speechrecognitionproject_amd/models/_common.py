"""Evaluation helpers shared by every model plugin — same behaviour as the reference's
per-module copies (e.g. models/model_mfcc_bgru.py:39-82), including its quirks:
``total += batchsize`` over-counts a short last batch (:51), and ``class_accuracy`` iterates
``range(batchsize)`` (:67), so it needs a dataset length divisible by ``batchsize``."""
import torch
from torch.utils.data import DataLoader

LABELS = ['yes', 'no', 'up', 'down', 'left', 'right', 'on', 'off', 'stop', 'go', 'unknown', 'silence']
DEVICE = torch.device('cuda' if torch.cuda.is_available() else 'cpu')


def accuracy(model, dataset, filename, batchsize=2):
    """Overall accuracy (%) on ``dataset``; appends it as one line to ``filename``."""
    total, correct = 0, 0
    model.eval()
    dataloader = DataLoader(dataset, batch_size=batchsize, drop_last=False)
    with torch.no_grad():
        for batch in dataloader:
            outputs = model(batch['audio'])
            _, predicted = torch.max(outputs.data, 1)
            total += batchsize
            correct += (predicted == batch['label'].to(outputs.device)).sum().item()
    with open(filename, 'a') as f:
        f.write(str(100 * correct / float(total)) + '\n')
    model.train()
    return 100 * correct / float(total)


def class_accuracy(model, dataset, filename, batchsize=2):
    """Per-class accuracy; overwrites ``filename`` with 12 lines."""
    class_correct = [0.0] * 12
    class_total = [0.0] * 12
    model.eval()
    dataloader = DataLoader(dataset, batch_size=batchsize, drop_last=False)
    with torch.no_grad():
        for batch in dataloader:
            outputs = model(batch['audio'])
            _, predicted = torch.max(outputs.data, 1)
            c = (predicted == batch['label'].to(outputs.device)).squeeze()
            for i in range(batchsize):
                label = batch['label'][i]
                class_correct[label] += c[i].item()
                class_total[label] += 1
    with open(filename, 'w') as f:
        for i in range(12):
            f.write('Accuracy of %5s : %2d %%' % (LABELS[i], 100 * class_correct[i] / class_total[i]) + '\n')
    model.train()
