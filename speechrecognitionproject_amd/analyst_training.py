"""The reference's ``analyst_training.py`` (analyst_training.py:1-122) on the MI355X path: train
the stacking analyst (models/model_analyst.py) on the concatenated softmax outputs of four frozen
base plugins, with per-epoch validation, best-checkpoint saving and early stopping.

    python -m speechrecognitionproject_amd.analyst_training -k KEY -lr LR --data-path DATA \
        --output-path OUT [--base-models fbanks_cnn,resnet_bgru,spec_bgru,spec_cnn] [--ckpt ...]

Same loop: Adam(lr, default 1e-4) over the analyst only, CrossEntropyLoss, NUM_EPOCHS = 10, the
reference's ExponentialLR(0.87) scheduler is created but never stepped (:81-82, kept as is), one
``str(loss)`` line per step to ``loss_<KEY>.txt``, ``accuracy`` line per epoch to
``val_<KEY>.txt``, the best analyst ``state_dict`` to ``models/model_<KEY>.ckpt``, stop once an
epoch brings no improvement (:114-118), ``resample_unknown_class`` after each epoch.  The
reference reduces both datasets to one clip per class (:47-48, ``--reduce 1``, the default here
too; ``--reduce 0`` keeps everything).  Batches default to the reference's batch_size = 1; the
base models and K11 run a whole batch per step either way.
"""
import argparse
import os

import torch
from torch.utils.data import DataLoader

from .dataset import Dataset, DeviceBatchLoader
from .evaluation import stacked_inputs
from .models import model_analyst
from .nn import CrossEntropyLoss
from .optim import Adam
from .predictions import load_models


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('-k', '--key', type=str, help='key')
    p.add_argument('-lr', '--learning_rate', type=float, help='LEARNING_RATE')
    p.add_argument('--data-path', required=True, help="parent of 'audio' and the *_list.txt files")
    p.add_argument('--output-path', default='.')
    p.add_argument('--base-models', default='fbanks_cnn,resnet_bgru,spec_bgru,spec_cnn')
    p.add_argument('--ckpt', default='', help='comma-separated base-model state_dict files (:65-68)')
    p.add_argument('--epochs', type=int, default=10)
    p.add_argument('--batch-size', type=int, default=1)
    p.add_argument('--reduce', type=int, default=1)
    p.add_argument('--loader', choices=('device', 'torch'), default='device')
    return p.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    key = args.key or ''
    lr = args.learning_rate if args.learning_rate is not None else 0.0001
    device = torch.device('cuda')
    data = Dataset(args.data_path + '/training_list.txt', args.data_path + '/audio')
    valset = Dataset(args.data_path + '/validation_list.txt', args.data_path + '/audio')
    if args.reduce:
        data.reduce_dataset(args.reduce)
        valset.reduce_dataset(args.reduce)
    bases = load_models(args.base_models.split(','), args.ckpt.split(',') if args.ckpt else [], device)
    for m in bases:
        for q in m.parameters():
            q.requires_grad = False
    analyzer = model_analyst.Network().to(device)
    criterion = CrossEntropyLoss()
    optimizer = Adam([q for q in analyzer.parameters() if q.requires_grad], lr=lr)
    torch.optim.lr_scheduler.ExponentialLR(optimizer, 0.87)   # created, never stepped (:81)
    os.makedirs(os.path.join(args.output_path, 'models'), exist_ok=True)
    models = [analyzer] + bases
    epoch, estop, maxval, maxind = 0, False, 0, 0
    while epoch < args.epochs and not estop:
        if args.loader == 'device':
            loader = DeviceBatchLoader(data, batch_size=args.batch_size, shuffle=True, seed=epoch)
        else:
            loader = DataLoader(data, batch_size=args.batch_size, shuffle=True, drop_last=False)
        losses = []
        for batch in loader:
            inp = stacked_inputs(bases, batch['audio'])
            optimizer.zero_grad()
            outputs = analyzer(inp)
            loss = criterion(outputs, batch['label'].to(device))
            loss.backward()
            optimizer.step()
            losses.append(loss.detach())
        if losses:
            with open(os.path.join(args.output_path, 'loss_' + key + '.txt'), 'a') as f:
                for v in torch.stack(losses).tolist():
                    f.write(str(v) + '\n')
        newval = model_analyst.accuracy(models, valset, os.path.join(args.output_path, 'val_' + key + '.txt'),
                                        batchsize=max(1, args.batch_size))
        if newval > maxval:
            maxval, maxind = newval, epoch
            torch.save(analyzer.state_dict(), os.path.join(args.output_path, 'models', 'model_' + key + '.ckpt'))
        if epoch > maxind:
            estop = True
        epoch += 1
        data.resample_unknown_class()
    return maxval, epoch


if __name__ == '__main__':
    main()
