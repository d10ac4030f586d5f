"""Generate tests/golden/vivit.npz from transformers' own VivitModel (CPU, fp32).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_vivit_golden.py

The reference's lipreading/huggingface_vivit_model.py imports tensorflow / cv2 at module
level (absent here), so its 8-line ViViT wrapper (:18-33: last_hidden_state -> mean over
tokens -> Linear(256, num_classes)) is restated around transformers.VivitModel, which is
the installed library the reference builds on (main.py:57-58).  Config: the reference's
(image 32, 1 channel, hidden 256, 8 heads; 5-frame clips as main.py:32 feeds them) with
2 layers, batch 3, 7 classes, seeded non-trivial weights (oracle.vivit.seeded_state)."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from transformers import VivitConfig, VivitModel  # noqa: E402

from oracle.vivit import seeded_state  # noqa: E402

LAYERS, HEADS, CLASSES, B = 2, 8, 7, 3


def main():
    cfg = VivitConfig(image_size=32, num_frames=5, num_channels=1, hidden_size=256,
                      num_attention_heads=HEADS, num_hidden_layers=LAYERS, intermediate_size=512,
                      attn_implementation="eager")
    vit = VivitModel(cfg).eval()
    shapes = {"vit." + k: tuple(v.shape) for k, v in vit.state_dict().items()}
    shapes["fc.weight"], shapes["fc.bias"] = (CLASSES, 256), (CLASSES,)
    P = seeded_state(shapes, 11)
    vit.load_state_dict({k[4:]: v for k, v in P.items() if k.startswith("vit.")})
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, 5, 1, 32, 32, generator=g)
    labels = torch.tensor([1, 6, 3])
    for p in vit.parameters():
        p.requires_grad_(True)
    fcw = P["fc.weight"].clone().requires_grad_(True)
    fcb = P["fc.bias"].clone().requires_grad_(True)
    hs = vit(pixel_values=x).last_hidden_state
    logits = F.linear(hs.mean(dim=1), fcw, fcb)
    loss = F.cross_entropy(logits, labels)
    loss.backward()
    grads = {"vit." + n: p.grad for n, p in vit.named_parameters() if p.grad is not None}
    pick = ["vit.embeddings.patch_embeddings.projection.weight", "vit.layers.0.attention.q_proj.weight",
            "vit.layers.1.mlp.fc1.weight", "vit.layers.1.layernorm_after.weight", "vit.layernorm.bias"]
    out = {"x": x.numpy(), "labels": labels.numpy(), "last_hidden": hs.detach().numpy(),
           "logits": logits.detach().numpy(), "loss": np.float32(loss.item()),
           "grad_fc.weight": fcw.grad.numpy()}
    for k in pick:  # large gradients: the first 8 rows (the fixture stays small)
        out["grad_" + k] = grads[k].numpy()[:8]
    # the weights are not stored: oracle.vivit.seeded_state(shapes, 11) regenerates them
    np.savez_compressed(os.path.join(HERE, "vivit.npz"), **out)
    print("wrote vivit.npz", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
