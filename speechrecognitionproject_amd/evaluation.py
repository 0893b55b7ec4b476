"""Evaluation callers of the path: the softmax ensemble of
``predictions.py`` and the stacked "analyst" inputs of ``models/model_analyst.py`` /
``analyst_training.py``, batched on the device (K11 ``srk_softmax_ensemble``).

The reference evaluates one clip at a time (DataLoader batch_size=1) and combines
``softmax(model_k(x).squeeze(0), dim=0)`` on the host side of the model outputs
(predictions.py:59-64, analyst_training.py:94-99); here a batch of clips goes through every
model and ONE kernel launch produces the per-clip probabilities, their concatenation, their
mean and its arg-max.
"""
import torch

from ._lib import SrkError, call
from .features import ptr, require_gpu, stream_ptr


def softmax_ensemble(logits, want_cat=False, want_mean=True, want_pred=True):
    """logits: list of K float32 device tensors [B, C] (or one [K, B, C] tensor).
    Returns (cat [B, K*C] | None, mean [B, C] | None, pred int64 [B] | None)."""
    require_gpu()
    x = torch.stack(list(logits)) if isinstance(logits, (list, tuple)) else logits
    x = x.detach().to(torch.float32).contiguous()
    if x.dim() != 3 or x.device.type != "cuda":
        raise SrkError("softmax_ensemble: expected K device tensors [B, C]")
    K, B, C = x.shape
    cat = torch.empty((B, K * C), device=x.device) if want_cat else None
    mean = torch.empty((B, C), device=x.device) if want_mean else None
    pred = torch.empty((B,), device=x.device, dtype=torch.int64) if want_pred else None
    nul = None
    call("srk_softmax_ensemble", ptr(x), K, B, C, ptr(cat) if want_cat else nul, ptr(mean) if want_mean else nul,
         ptr(pred) if want_pred else nul, stream_ptr())
    return cat, mean, pred


@torch.no_grad()
def stacked_inputs(models, audio):
    """The analyst input of analyst_training.py:94-99 for a batch: [B, 12 * len(models)] =
    concat_k softmax(model_k(audio)) (models in eval mode, no gradient)."""
    cat, _, _ = softmax_ensemble([m(audio) for m in models], want_cat=True, want_mean=False, want_pred=False)
    return cat
