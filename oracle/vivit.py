"""Oracle restatement of the ViViT lipreading classifier (CPU, fp32) -- TEST
INFRASTRUCTURE ONLY: imported by tests/ (and bench's cpu leg) as the checker, never by
the product path.

Functional forward over a state dict with transformers' VivitModel key names (5.15):
  * lipreading/huggingface_vivit_model.py:25-33  ViViT.forward: vit(x).last_hidden_state,
    mean over tokens, Linear(256, num_classes);
  * transformers VivitTubeletEmbeddings / VivitEmbeddings: Conv3d(kernel = stride =
    tubelet) over [B, C, T, H, W], flatten, CLS prepended, + position table;
  * VivitLayer: x + o_proj(MHA(LN_before(x))), then x + fc2(gelu_fast(fc1(LN_after(x))));
    MHA = softmax(q k^T * head_dim^-1/2) v per head (eager_attention_forward);
  * final VivitModel.layernorm.
Pinned against transformers' VivitModel itself by tests/golden/gen_vivit_golden.py
(tests/golden/vivit.npz)."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def gelu_fast(x):
    """transformers.activations.FastGELUActivation."""
    return 0.5 * x * (1.0 + torch.tanh(x * 0.7978845608 * (1.0 + 0.044715 * x * x)))


def vivit_forward(P: dict, x: torch.Tensor, heads: int, layers: int, tubelet=(2, 16, 16),
                  eps: float = 1e-6) -> torch.Tensor:
    """VivitModel.forward(...).last_hidden_state for pixel_values x [B, T, C, H, W]."""
    e = "embeddings."
    h = F.conv3d(x.transpose(1, 2).float(), P[e + "patch_embeddings.projection.weight"],
                 P[e + "patch_embeddings.projection.bias"], stride=tubelet)
    h = h.flatten(2).transpose(1, 2)
    B = h.shape[0]
    h = torch.cat((P[e + "cls_token"].expand(B, -1, -1), h), dim=1) + P[e + "position_embeddings"]
    C = h.shape[-1]
    D = C // heads
    for i in range(layers):
        p = f"layers.{i}."
        y = F.layer_norm(h, (C,), P[p + "layernorm_before.weight"], P[p + "layernorm_before.bias"], eps)
        q, k, v = (F.linear(y, P[p + f"attention.{n}_proj.weight"], P[p + f"attention.{n}_proj.bias"])
                   .reshape(B, -1, heads, D).transpose(1, 2) for n in "qkv")
        a = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(D), dim=-1) @ v
        a = a.transpose(1, 2).reshape(B, -1, C)
        h = h + F.linear(a, P[p + "attention.o_proj.weight"], P[p + "attention.o_proj.bias"])
        y = F.layer_norm(h, (C,), P[p + "layernorm_after.weight"], P[p + "layernorm_after.bias"], eps)
        y = F.linear(gelu_fast(F.linear(y, P[p + "mlp.fc1.weight"], P[p + "mlp.fc1.bias"])),
                     P[p + "mlp.fc2.weight"], P[p + "mlp.fc2.bias"])
        h = h + y
    return F.layer_norm(h, (C,), P["layernorm.weight"], P["layernorm.bias"], eps)


def vivit_classifier(P: dict, x: torch.Tensor, heads: int, layers: int, **kw) -> torch.Tensor:
    """huggingface_vivit_model.py:25-33: keys of the wrapper are vit.* and fc.*."""
    V = {k[4:]: v for k, v in P.items() if k.startswith("vit.")}
    h = vivit_forward(V, x, heads, layers, **kw)
    return F.linear(h.mean(dim=1), P["fc.weight"], P["fc.bias"])


def seeded_state(shapes: dict, seed: int, scale: float = 1.0) -> dict:
    """Deterministic non-trivial weights: randn / sqrt(fan_in) for >= 2-D tensors,
    1 + 0.1 randn for LayerNorm weights, 0.1 randn for biases and the token tables."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k in sorted(shapes):
        s = shapes[k]
        r = torch.randn(s, generator=g)
        if "layernorm" in k and k.endswith("weight"):
            out[k] = 1 + 0.1 * r
        elif len(s) >= 2 and not k.endswith(("cls_token", "position_embeddings")):
            out[k] = scale * r / math.sqrt(math.prod(s[1:]))
        else:
            out[k] = 0.1 * r
    return out
