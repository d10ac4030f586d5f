"""Drop-in for the reference's lipreading/huggingface_vivit_model.py on libvdiff.

Same names: `ViViT(vivit_model, num_classes, num_frames)` (:18-33) and
`train_huggingface_model` (:35-95).  `VivitModel` / `VivitConfig` stand in for the
transformers classes the reference imports (:1); transformers-format state dicts load
unchanged.  The reference's loop reads module-level X_train / X_test / Y_train_p /
Y_test_p globals (set by main.py, :38-41); the one-argument call
`train_huggingface_model(VIVIT)` does the same here, and the data may also be passed as
arguments, with the same shapes (N x 5 x 1 x 32 x 32 clips, integer labels).  Differences: data are moved to the GPU
once per epoch-batch as in the reference, `best_model_wts` uses copy.deepcopy (the
reference imports `deepcopy` but calls `copy.deepcopy`, :90, a NameError), and the
validation loss is computed rather than reusing the last training loss (:80-84).  Training
accuracy counts the train-mode predictions of each step's own forward, as the reference
does (:52-64).
"""
from __future__ import annotations

import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vdiff.vivit import (ViViT, VivitConfig, VivitModel, VivitTrainer,  # noqa: E402,F401
                         lipreading_config)


# module-level data the reference's one-argument call reads (:38-41); main.py sets them
X_train = X_test = Y_train_p = Y_test_p = None


def train_huggingface_model(VIVIT, X_train=None, Y_train=None, X_test=None, Y_test=None,
                            num_epochs=10, batch_size=16, device="cuda", log=print):
    """huggingface_vivit_model.py:35-95: CE + AdamW(1e-4), StepLR(2, 0.2) per epoch; keeps
    the weights of the best validation-accuracy epoch.  Data arguments left as None are
    read from this module's globals X_train / Y_train_p / X_test / Y_test_p, as the
    reference does."""
    g = globals()
    X_train = g["X_train"] if X_train is None else X_train
    Y_train = g["Y_train_p"] if Y_train is None else Y_train
    X_test = g["X_test"] if X_test is None else X_test
    Y_test = g["Y_test_p"] if Y_test is None else Y_test
    if any(v is None for v in (X_train, Y_train, X_test, Y_test)):
        raise NameError("train_huggingface_model: set X_train / Y_train_p / X_test / Y_test_p "
                        "on this module (as main.py does for the reference) or pass them")
    VIVIT = VIVIT.to(device)
    X_train = torch.as_tensor(X_train).reshape(len(X_train), 5, 1, 32, 32).float()
    X_test = torch.as_tensor(X_test).reshape(len(X_test), 5, 1, 32, 32).float()
    Y_train = torch.as_tensor(Y_train).reshape(len(Y_train)).long()
    Y_test = torch.as_tensor(Y_test).reshape(len(Y_test)).long()
    tr = VivitTrainer(VIVIT, lr=1e-4)
    best_acc, best = -1.0, copy.deepcopy(VIVIT.state_dict())
    for epoch in range(num_epochs):
        run_loss, run_ok = 0.0, 0
        for i in range(0, len(X_train), batch_size):
            data = X_train[i:i + batch_size].to(device)
            labels = Y_train[i:i + batch_size].to(device)
            loss = tr.step(data, labels)
            run_loss += float(loss) * len(labels)
            # training accuracy from the step's own train-mode predictions (:52-64)
            run_ok += int((tr.logits.argmax(1) == labels).sum())
        VIVIT.eval()
        log(f"train loss is {run_loss / len(X_train)}, epoch_acc is {run_ok / len(X_train)}")
        val_loss, val_ok = 0.0, 0
        with torch.no_grad():
            for i in range(0, len(X_test), batch_size):
                labels = Y_test[i:i + batch_size]
                out = VIVIT(X_test[i:i + batch_size].to(device))
                val_loss += float(F.cross_entropy(out, labels.to(device))) * len(labels)
                val_ok += int((out.argmax(1).cpu() == labels).sum())
        acc = val_ok / max(1, len(X_test))
        log(f"val loss is {val_loss / max(1, len(X_test))}, epoch_acc is {acc}")
        if acc > best_acc:
            best_acc, best = acc, copy.deepcopy(VIVIT.state_dict())
        tr.epoch_end()
    VIVIT.load_state_dict(best)
    return VIVIT
