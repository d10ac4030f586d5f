"""ViViT lipreading classifier on libvdiff (BASELINE config 5).

Reference: lipreading/huggingface_vivit_model.py:18-33 (`ViViT`: VivitModel ->
last_hidden_state -> mean over tokens -> Linear(256, num_classes)) and :35-95 (the
fine-tune loop: CrossEntropy, AdamW lr 1e-4, StepLR(step_size=2, gamma=0.2) per epoch,
batch 16); lipreading/main.py:57-58 builds `VivitConfig(image_size=32, num_frames=15,
num_channels=1, hidden_size=256, num_attention_heads=8, ...)`.

`VivitModel` here mirrors transformers' VivitModel (the version installed in this image,
5.15: module names `layers.N.attention.q_proj` ..., `mlp.fc1/fc2`), so its state_dict
loads and saves checkpoints of that class unchanged.  The compute is MI355X-native:
  * tubelet embedding (Conv3d, kernel = stride = tubelet) = patch gather + one GEMM;
  * q/k/v/o, fc1, fc2 on the implicit-GEMM kernel (1x1 conv), residual adds fused into
    the o_proj / fc2 epilogues;
  * multi-head attention on the flash kernel (q|k|v channel chunks, heads as pointer
    arithmetic: QKVAttention order, scale head_dim^-1/2 as transformers' sdpa/eager);
  * LayerNorm and the tanh GELU ("gelu_fast") on layernorm.hip.
The reference config as written cannot run: num_frames=15 sizes the position table for
7 tubelets in time while main.py feeds 5-frame clips (2 tubelets).  `lipreading_config`
takes the frame count the data has (5), which is what the reference must have meant.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import hipgraph, ops


@dataclass
class VivitConfig:
    """The fields of transformers.VivitConfig the model reads (same names and defaults)."""
    image_size: int = 224
    num_frames: int = 32
    tubelet_size: tuple = (2, 16, 16)
    num_channels: int = 3
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    hidden_act: str = "gelu_fast"
    hidden_dropout_prob: float = 0.0
    attention_probs_dropout_prob: float = 0.0
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-6
    qkv_bias: bool = True

    @classmethod
    def from_hf(cls, hf_config) -> "VivitConfig":
        names = cls.__dataclass_fields__
        return cls(**{k: getattr(hf_config, k) for k in names if hasattr(hf_config, k)})


def lipreading_config(num_frames: int = 5, **kw) -> VivitConfig:
    """main.py:57 with the clip length the data has (MAX_SEQ_LENGTH = 5, main.py:32)."""
    base = dict(image_size=32, num_frames=num_frames, num_channels=1, hidden_size=256,
                num_attention_heads=8)
    base.update(kw)
    return VivitConfig(**base)


def tubelets(pixel_values: torch.Tensor, tubelet) -> torch.Tensor:
    """[B, T, C, H, W] -> [B, nt*nh*nw, C*t*h*w]: the non-overlapping tubelets (trailing
    frames / pixels that do not fill one are dropped, as Conv3d with kernel = stride does),
    each flattened in the (C, kt, kh, kw) order of the Conv3d weight, tokens in (t, h, w)
    order as Conv3d(...).flatten(2)."""
    B, T, C, H, W = pixel_values.shape
    t, h, w = tubelet
    nt, nh, nw = T // t, H // h, W // w
    x = pixel_values[:, :nt * t, :, :nh * h, :nw * w]
    x = x.reshape(B, nt, t, C, nh, h, nw, w).permute(0, 1, 4, 6, 3, 2, 5, 7)
    return x.reshape(B, nt * nh * nw, C * t * h * w)


class VivitTubeletEmbeddings(nn.Module):
    def __init__(self, config: VivitConfig):
        super().__init__()
        t, h, w = config.tubelet_size
        self.tubelet = (t, h, w)
        self.num_patches = ((config.num_frames // t) * (config.image_size // h)
                            * (config.image_size // w))
        self.projection = nn.Conv3d(config.num_channels, config.hidden_size,
                                    kernel_size=self.tubelet, stride=self.tubelet)

    def forward(self, pixel_values: torch.Tensor) -> torch.Tensor:
        """[B, T, C, H, W] -> [B, patches, hidden]: the tubelet gather, then one GEMM."""
        x = tubelets(pixel_values, self.tubelet)
        wgt = self.projection.weight.reshape(self.projection.weight.shape[0], -1)
        return ops.linear(x, wgt, self.projection.bias)


class VivitEmbeddings(nn.Module):
    def __init__(self, config: VivitConfig):
        super().__init__()
        self.cls_token = nn.Parameter(torch.zeros(1, 1, config.hidden_size))
        self.patch_embeddings = VivitTubeletEmbeddings(config)
        self.position_embeddings = nn.Parameter(
            torch.zeros(1, self.patch_embeddings.num_patches + 1, config.hidden_size))

    def forward(self, pixel_values: torch.Tensor) -> torch.Tensor:
        emb = self.patch_embeddings(pixel_values)
        if emb.shape[1] + 1 != self.position_embeddings.shape[1]:
            raise ValueError(f"{emb.shape[1]} tubelets but a position table for "
                             f"{self.position_embeddings.shape[1] - 1} (num_frames / image_size "
                             "of the config must match the clips)")
        cls = self.cls_token.to(emb.dtype).expand(emb.shape[0], -1, -1)
        return torch.cat((cls, emb), dim=1) + self.position_embeddings.to(emb.dtype)


class VivitAttention(nn.Module):
    def __init__(self, config: VivitConfig):
        super().__init__()
        C = config.hidden_size
        self.heads = config.num_attention_heads
        self.q_proj = nn.Linear(C, C, bias=config.qkv_bias)
        self.k_proj = nn.Linear(C, C, bias=config.qkv_bias)
        self.v_proj = nn.Linear(C, C, bias=config.qkv_bias)
        self.o_proj = nn.Linear(C, C, bias=True)

    def forward(self, h: torch.Tensor, residual: torch.Tensor) -> torch.Tensor:
        """h [B, N, C] (normalised) -> residual + o_proj(MHA(h))."""
        B, N, C = h.shape
        w = torch.cat((self.q_proj.weight, self.k_proj.weight, self.v_proj.weight))
        b = (torch.cat((self.q_proj.bias, self.k_proj.bias, self.v_proj.bias))
             if self.q_proj.bias is not None else None)
        qkv = ops.linear(h, w, b)                          # [B, N, 3C]: tokens are rows
        a = ops.attention(qkv.transpose(1, 2), self.heads, legacy=False)  # [B, C, N] (cl)
        return ops.linear(a.transpose(1, 2), self.o_proj.weight, self.o_proj.bias,
                          residual=residual)


class VivitMLP(nn.Module):
    def __init__(self, config: VivitConfig):
        super().__init__()
        if config.hidden_act not in ("gelu_fast", "gelu_pytorch_tanh", "gelu_new"):
            raise NotImplementedError(f"hidden_act {config.hidden_act!r}: the tanh GELU only")
        self.fc1 = nn.Linear(config.hidden_size, config.intermediate_size)
        self.fc2 = nn.Linear(config.intermediate_size, config.hidden_size)

    def forward(self, h: torch.Tensor, residual: torch.Tensor) -> torch.Tensor:
        h = ops.gelu_tanh(ops.linear(h, self.fc1.weight, self.fc1.bias))
        return ops.linear(h, self.fc2.weight, self.fc2.bias, residual=residual)


class VivitLayer(nn.Module):
    """Pre-norm block: x + attn(LN(x)), then x + mlp(LN(x)) (dropout 0 in the config)."""

    def __init__(self, config: VivitConfig):
        super().__init__()
        self.attention = VivitAttention(config)
        self.layernorm_before = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.layernorm_after = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.mlp = VivitMLP(config)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        ln = self.layernorm_before
        x = self.attention(ops.layer_norm(x, ln.weight, ln.bias, ln.eps), x)
        ln = self.layernorm_after
        return self.mlp(ops.layer_norm(x, ln.weight, ln.bias, ln.eps), x)


class VivitPooler(nn.Module):
    def __init__(self, config: VivitConfig):
        super().__init__()
        self.dense = nn.Linear(config.hidden_size, config.hidden_size)


@dataclass
class VivitOutput:
    last_hidden_state: torch.Tensor
    pooler: Optional[VivitPooler] = None

    @property
    def pooler_output(self):
        """tanh(dense(CLS)) as transformers' VivitPooler; computed on request (the
        reference classifier never reads it)."""
        if self.pooler is None:
            return None
        cls = self.last_hidden_state[:, 0]
        return torch.tanh(ops.linear(cls, self.pooler.dense.weight, self.pooler.dense.bias))


class VivitModel(nn.Module):
    def __init__(self, config: VivitConfig, add_pooling_layer: bool = True, use_bf16=False):
        super().__init__()
        self.config = config
        self.dtype_ = torch.bfloat16 if use_bf16 else torch.float32
        self.embeddings = VivitEmbeddings(config)
        self.layers = nn.ModuleList(VivitLayer(config) for _ in range(config.num_hidden_layers))
        self.layernorm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.pooler = VivitPooler(config) if add_pooling_layer else None
        self.init_weights()

    def init_weights(self, seed: Optional[int] = None):
        """transformers' _init_weights: N(0, initializer_range) for Linear / Conv3d weights
        and the CLS / position tables, zero biases, LayerNorm (1, 0)."""
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        std = self.config.initializer_range
        with torch.no_grad():
            for m in self.modules():
                if isinstance(m, (nn.Linear, nn.Conv3d)):
                    m.weight.copy_(torch.randn(m.weight.shape, generator=g) * std)
                    if m.bias is not None:
                        m.bias.zero_()
                elif isinstance(m, nn.LayerNorm):
                    m.weight.fill_(1.0)
                    m.bias.zero_()
            for p in (self.embeddings.cls_token, self.embeddings.position_embeddings):
                p.copy_(torch.randn(p.shape, generator=g) * std)

    def forward(self, pixel_values: torch.Tensor) -> VivitOutput:
        x = self.embeddings(pixel_values.to(self.dtype_))
        for layer in self.layers:
            x = layer(x)
        ln = self.layernorm
        return VivitOutput(ops.layer_norm(x, ln.weight, ln.bias, ln.eps), self.pooler)


class ViViT(nn.Module):
    """huggingface_vivit_model.py:18-33: vit(x).last_hidden_state -> mean over tokens ->
    Linear(256, num_classes) (the reference hard-codes 256 = its hidden size)."""

    def __init__(self, vivit_model: VivitModel, num_classes: int, num_frames: int):
        super().__init__()
        self.num_frames = num_frames
        self.vit = vivit_model
        self.fc = nn.Linear(256, num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = self.vit(x).last_hidden_state
        return ops.linear(h.mean(dim=1), self.fc.weight, self.fc.bias).float()


class VivitTrainer:
    """One fine-tune step of train_huggingface_model (huggingface_vivit_model.py:35-60):
    CrossEntropy -> backward -> (all-reduce) -> AdamW(lr 1e-4); `epoch_end()` steps the
    StepLR(step_size=2, gamma=0.2) as the reference does once per epoch."""

    def __init__(self, model: ViViT, lr=1e-4, bucket_mb=25.0, graph=False):
        """graph=True: the step runs as captured HIP graphs.  At 9 tokens x 256 hidden every
        kernel runs for microseconds, so an eager step is bound by host-side launch
        overhead.  One process: forward, backward and AdamW in one graph.  Under DDP: graph
        1 = forward + backward + gradient flatten into one fp32 buffer, then ONE eager
        all-reduce of that buffer (the collective stays outside the capture), then graph 2 =
        unflatten / average + AdamW."""
        from .ddp import GradBucketer
        self.model = model
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.distributed = (torch.distributed.is_initialized()
                            and torch.distributed.get_world_size() > 1)
        self.world = torch.distributed.get_world_size() if self.distributed else 1
        self.bucketer = (GradBucketer(self.params, bucket_mb)
                         if self.distributed and not graph else None)
        kw = {"fused": True} if self.params and self.params[0].is_cuda else {}
        if graph:
            kw["capturable"] = True
            lr = torch.tensor(lr, device=self.params[0].device)
        self.opt = torch.optim.AdamW(self.params, lr=lr, **kw)
        self.sched = torch.optim.lr_scheduler.StepLR(self.opt, step_size=2, gamma=0.2)
        self.use_graph = graph
        self.graph = None

    def step(self, data: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        if not self.use_graph:
            return self._step(data, labels)
        if self.graph is None:
            self._capture(data, labels)
        self.static_x.copy_(data)
        self.static_y.copy_(labels)
        self.graph.replay()
        if self.distributed:
            torch.distributed.all_reduce(self.flat)
            self.graph_opt.replay()
        return self.static_loss

    def node_types(self):
        """{node type: count} of the captured step graph (vdiff.hipgraph): the graph must hold
        no memset node -- torch's reductions that reset a semaphore by a captured memset went
        stale under HIP's graph packet capture."""
        from .hipgraph import graph_nodes
        nodes = graph_nodes(self.graph.raw_cuda_graph())
        return {t: sum(1 for n in nodes if n["type"] == t) for t in {n["type"] for n in nodes}}

    def _fwd_bwd(self, x, y):
        self.model.train()
        out = self.model(x)
        self.logits = out.detach()  # the step's train-mode predictions (graph: static buffer)
        loss = F.cross_entropy(out, y)
        loss.backward()
        return loss.detach()

    def _capture(self, data, labels):
        self.static_x = data.clone()
        self.static_y = labels.clone()
        dev = data.device
        # the warm-up steps below are real updates: snapshot the weights so that the first
        # replay is the first update the caller sees (optimizer state is reset below)
        snapshot = [p.detach().clone() for p in self.params]
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(3):  # warm the allocator and autograd outside the capture
                if self.distributed:  # identical updates on every rank: average first
                    self._fwd_bwd(self.static_x, self.static_y)
                    for p in self.params:
                        if p.grad is not None:
                            torch.distributed.all_reduce(p.grad)
                            p.grad.div_(self.world)
                    self.opt.step()
                    self.opt.zero_grad(set_to_none=True)
                else:
                    self._step(self.static_x, self.static_y)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.opt.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph(keep_graph=True)  # node list kept (node_types)
        if not self.distributed:
            with hipgraph.capture(self.graph):
                self.static_loss = self._step(self.static_x, self.static_y, zero=False)
            self.graph.instantiate()
            self._restore(snapshot)
            return
        # parameters with a gradient (the pooler has none: the classifier never reads it).
        # thread_local: the process group's watchdog thread may query events meanwhile.
        torch.cuda.synchronize(dev)
        torch.distributed.barrier()
        with hipgraph.capture(self.graph, capture_error_mode="thread_local"):
            self.static_loss = self._fwd_bwd(self.static_x, self.static_y)
            grads = [p.grad for p in self.params if p.grad is not None]
            self.flat = torch.cat([g.reshape(-1).float() for g in grads])
        self.graph_opt = torch.cuda.CUDAGraph()
        with hipgraph.capture(self.graph_opt, capture_error_mode="thread_local"):
            views = self.flat.split([g.numel() for g in grads])
            torch._foreach_mul_(list(views), 1.0 / self.world)
            torch._foreach_copy_(grads, [v.view_as(g) for v, g in zip(views, grads)])
            self.opt.step()
        self._restore(snapshot)

    @torch.no_grad()
    def _restore(self, snapshot):
        """Undo the capture warm-up in place (the graphs hold these addresses): weights back
        to the snapshot, AdamW moments and step counts to zero -- the state of a fresh
        optimizer, so the first replay applies bias-corrected step 1."""
        for p, v in zip(self.params, snapshot):
            p.copy_(v)
        for st in self.opt.state.values():
            for v in st.values():
                if torch.is_tensor(v):
                    v.zero_()

    def _step(self, data, labels, zero=True):
        self.model.train()
        out = self.model(data)
        self.logits = out.detach()  # the step's train-mode predictions (graph: static buffer)
        loss = F.cross_entropy(out, labels)
        loss.backward()
        if self.bucketer is not None:
            self.bucketer.finish()
            self.bucketer.step(self.opt)
            self.bucketer.zero_grad()
            return loss.detach()
        self.opt.step()
        if zero:
            self.opt.zero_grad(set_to_none=True)
        return loss.detach()

    def epoch_end(self):
        self.sched.step()


def vivit_flops(config: VivitConfig, batch: int) -> float:
    """Forward FLOP (2 per MAC) of VivitModel + ViViT head for one batch."""
    C, I, L = config.hidden_size, config.intermediate_size, config.num_hidden_layers
    t, h, w = config.tubelet_size
    P = (config.num_frames // t) * (config.image_size // h) * (config.image_size // w)
    N = P + 1
    patch = 2 * P * C * config.num_channels * t * h * w
    per_layer = 2 * N * (4 * C * C + 2 * C * I) + 4 * N * N * C
    return float(batch * (patch + L * per_layer))
