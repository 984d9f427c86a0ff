"""Which native path a model's ``forward`` takes: the fused inference kernels or the training
composition (native operators under ``torch.autograd``).

The reference trains with ``model.train(); pred = model(graph); loss.backward()``
(trainer.py:233-358) and validates under ``torch.no_grad()`` in eval mode (trainer.py:417).
The fused inference kernels never keep the activations a backward needs, so a forward whose
output must carry gradients has to run the training composition (slower: one launch per
operator instead of a few fused kernels per layer).

Rule, per module attribute ``native_train`` (default ``"auto"``):

* ``"auto"``: the training composition when autograd is recording (``torch.is_grad_enabled()``)
  and at least one parameter requires grad; otherwise the fused kernels.  A model in ``eval()``
  that takes the training composition this way warns once (``NativePathWarning``): that is
  usually a validation / inference loop that forgot ``torch.no_grad()``.
* ``True``: the training composition whenever autograd is recording (no warning).
* ``False``: always the fused kernels; the output carries no autograd graph.
"""
import warnings

import torch

MODES = ("auto", True, False)


class NativePathWarning(UserWarning):
    pass


def use_training_path(module) -> bool:
    mode = getattr(module, "native_train", "auto")
    # by identity: 1 / 0 compare equal to True / False but are not accepted (they would fall through
    # the `is` tests below to "auto")
    if not any(mode is m for m in (True, False)) and not (isinstance(mode, str) and mode == "auto"):
        raise ValueError(f"native_train must be one of {MODES}, got {mode!r}")
    if mode is False or not torch.is_grad_enabled():
        return False
    if mode is True:
        return True
    if not any(p.requires_grad for p in module.parameters()):
        return False
    if not module.training and not getattr(module, "_warned_eval_grad", False):
        warnings.warn(
            f"{type(module).__name__}: a grad-mode forward in eval() runs the native training composition "
            "(autograd through per-operator kernels), not the fused inference kernels; wrap inference in "
            "torch.no_grad() or set model.native_train = False for the fused path, or set "
            "model.native_train = True to silence this warning", NativePathWarning, stacklevel=3)
        module._warned_eval_grad = True
    return True
