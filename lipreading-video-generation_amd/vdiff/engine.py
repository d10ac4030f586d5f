"""Training step and samplers around the drop-in model (the loops of the reference
train.py:107-134 and test.py:51-83), plus synthetic clip generation.

Differences from the reference loops (all deliberate):
  * t ~ U{0, ..., num_timesteps-1}: the reference draws randint(0, 500) against a
    100-step schedule (train.py:125) and crashes;
  * no per-step torch.cuda.empty_cache() in sampling (test.py:58), and the audio
    encoder runs once per clip instead of at every denoising step;
  * gradients are averaged across ranks by vdiff.ddp.GradBucketer (world > 1).
"""
from __future__ import annotations

import contextlib
import math
import os
import warnings
import weakref
from dataclasses import dataclass

import torch

from . import hipgraph, ops
from .ddp import GradBucketer


@dataclass
class Clip:
    """One synthetic minibatch: target frames, reference image, audio windows, noise, t."""
    x0: torch.Tensor      # [B, 3, T, H, W] (or [B, 3, H, W])
    cond: torch.Tensor    # [B, 3, H, W]
    audio: dict           # {'input_values': [B*T, samples]}
    eps: torch.Tensor     # like x0
    t: torch.Tensor       # [B] int64


def synthetic_clip(batch, frames, size, num_timesteps, device, seed=0, samples=4000,
                   dims=3) -> Clip:
    """Seeded synthetic inputs: x0, cond ~ U[-1, 1]; eps ~ N(0, 1);
    audio ~ N(0, 1) [B*T, 4000]; t ~ U{0..N-1}.  Generated on the device."""
    g = torch.Generator(device=device).manual_seed(seed)
    shape = (batch, 3, frames, size, size) if dims == 3 else (batch, 3, size, size)
    x0 = torch.rand(shape, generator=g, device=device) * 2 - 1
    cond = torch.rand((batch, 3, size, size), generator=g, device=device) * 2 - 1
    eps = torch.randn(shape, generator=g, device=device)
    nwin = batch * (frames if dims == 3 else 1)
    audio = {"input_values": torch.randn((nwin, samples), generator=g, device=device)}
    t = torch.randint(0, num_timesteps, (batch,), generator=g, device=device)
    return Clip(x0, cond, audio, eps, t)


def reinit_nonzero(model, seed=1234, std=0.02):
    """Product-side deterministic init for benchmarks / smoke runs: the reference's
    zero_module layers (unet.py:222-224, 306, 627) would make the denoiser output 0."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in model.named_parameters():
            if name.startswith("audio_encoder."):
                continue
            if p.dim() >= 2 and float(p.detach().abs().max()) == 0.0:
                fan_in = math.prod(p.shape[1:])
                p.copy_(torch.randn(p.shape, generator=g) / math.sqrt(fan_in))
            elif p.dim() == 1 and float(p.detach().abs().max()) == 0.0 and name.endswith("bias"):
                p.copy_(std * torch.randn(p.shape, generator=g))
    return model


class Trainer:
    """q_sample -> denoiser -> MSE(eps_pred, eps) -> backward -> all-reduce -> Adam.

    train.py:102-103: Adam(model.parameters(), lr=1e-2), MSELoss."""

    def __init__(self, model, scheduler, lr=1e-2, bucket_mb=25.0, fused_adam=True,
                 check_every=50, batch_pack=True, graph=False, loss_fn=None):
        """check_every: the loss finiteness flag (kept on the device, updated every step) is
        read on the host every `check_every` steps and by check_finite(); a non-finite
        loss raises FloatingPointError naming the first bad step.  0 disables it.
        batch_pack: re-pack the conv operands once per step in one launch
        (ops.step_packed_weights) instead of per conv call.
        graph: replay the denoiser's forward + backward as one HIP graph (TrainStepGraph);
        one process only.
        loss_fn: (pred, eps) -> scalar loss; default ops.mse_loss (vd_mse_loss, fixed-order).
        Host-logic tests on CPU pass torch's F.mse_loss (the product ops refuse CPU tensors)."""
        self.model = model
        self.loss_fn = loss_fn or ops.mse_loss
        self.scheduler = scheduler
        self.check_every = int(check_every)
        self.steps_done = 0
        self._first_bad = None  # device int64: first step with a non-finite loss, or -1
        params = [p for p in model.parameters() if p.requires_grad]
        # one process: no all-reduce, so no bucket views -- autograd hands each gradient over
        # without the accumulate-into-view add, and zero_grad drops them (no fills)
        distributed = torch.distributed.is_initialized() and torch.distributed.get_world_size() > 1
        self.bucketer = GradBucketer(params, bucket_mb) if distributed else None
        kw = {"fused": True} if fused_adam and params and params[0].is_cuda else {}
        self.opt = torch.optim.Adam(params, lr=lr, **kw)
        # conv operands re-packed once per step in one launch (ops.step_packed_weights)
        self.packs = ops.step_packed_weights() if batch_pack else contextlib.nullcontext()
        if graph and self.bucketer is not None:
            raise ValueError("Trainer(graph=True) is single-process (the gradient buckets are "
                             "launched from autograd hooks)")
        if graph and not batch_pack:
            raise ValueError("Trainer(graph=True) needs batch_pack (per-call packs would be "
                             "frozen into the graph)")
        if graph and os.environ.get("VDIFF_TRAIN_GRAPH_EXPERIMENTAL") != "1":
            # advisor r03: a known defect must not be one keyword away from a user
            raise RuntimeError("Trainer(graph=True) is opt-in: it measured no gain over the eager "
                               "step (kernel-bound; DESIGN section 9 item 3); set "
                               "VDIFF_TRAIN_GRAPH_EXPERIMENTAL=1 to run it")
        self.graph = TrainStepGraph(self) if graph else None

    def step(self, clip: Clip) -> torch.Tensor:
        if self.graph is not None:
            return self.graph.step(clip)
        return self._eager_step(clip)

    def _eager_step(self, clip: Clip) -> torch.Tensor:
        self.model.train()
        with self.packs:
            xt = self.scheduler.add_noise(clip.x0, clip.eps, clip.t)
            pred = self.model(xt, clip.cond, clip.audio, clip.t)
            loss = self.loss_fn(pred, clip.eps)
            loss.backward()
        if self.bucketer is not None:
            self.bucketer.finish()
            self.bucketer.step(self.opt)
            self.bucketer.zero_grad()
        else:
            self.opt.step()
            self.opt.zero_grad(set_to_none=True)
        loss = loss.detach()
        self._track_finite(loss)
        return loss

    def _track_finite(self, loss):
        """SURVEY 5 failure detection without a per-step host sync: a device-side record of
        the first step whose loss is NaN/Inf (the reference skips nothing and checks
        nothing, train.py:111-112), read every check_every steps."""
        if self.check_every <= 0:
            return
        if self._first_bad is None:
            self._first_bad = torch.full((), -1, dtype=torch.int64, device=loss.device)
        bad = ~torch.isfinite(loss) & (self._first_bad < 0)
        self._first_bad.copy_(torch.where(bad, self.steps_done, self._first_bad))
        self.steps_done += 1
        if self.steps_done % self.check_every == 0:
            self.check_finite()

    def check_finite(self):
        """Raise FloatingPointError if any step so far had a non-finite loss (host sync).

        Under DDP (the gradient bucketer active) the first bad step is MIN-all-reduced over
        the ranks first, so a loss that went non-finite on one rank makes EVERY rank raise
        here together instead of leaving the others blocked in the next gradient
        all-reduce (advisor r03).  Every rank reaches this call at the same step count."""
        if self._first_bad is None and self.bucketer is None:
            return
        if self._first_bad is None:
            dev = next(self.model.parameters()).device
            self._first_bad = torch.full((), -1, dtype=torch.int64, device=dev)
        fb = self._first_bad
        if self.bucketer is not None:
            big = torch.iinfo(torch.int64).max
            v = torch.where(fb >= 0, fb, torch.full_like(fb, big)).reshape(1)
            if v.is_cuda and torch.distributed.get_backend() == "gloo":
                v = v.cpu()
            torch.distributed.all_reduce(v, op=torch.distributed.ReduceOp.MIN)
            first = int(v[0])
            first = -1 if first == big else first
        else:
            first = int(fb)
        if first >= 0:
            raise FloatingPointError(f"non-finite training loss at step {first} "
                                     f"(of {self.steps_done})")


class TrainStepGraph:
    """Trainer.step with the denoiser replayed as one HIP graph (the
    ~600 launch gaps of an eager step).

    Captured: the batched weight pack, q_sample, the conditioning concat and the UNet forward,
    the MSE (vd_mse_loss, whose value step() returns) and the whole backward down to the UNet
    parameters' gradients and the gradient of the pooled audio features.  Eager around it: the wav2vec2 encoder (transformers draws its
    LayerDrop and SpecAugment decisions on the host every step, which changes the launch
    sequence, so it cannot be frozen), its backward (fed the replayed feature gradient) and
    the fused Adam step over all parameters.  Same math as the eager step: the first `warmup`
    steps run eagerly (lazy initialisation, the packed-weight plan), the capture itself does not
    update anything, and the ResBlock dropout draws a new mask per replay through the device
    counter the GroupNorm kernels read (vd_set_dropout_counter).  The UNet parameters' .grad
    tensors live in the graph's memory pool and are overwritten by each replay; they are never
    reset to None."""

    def __init__(self, trainer, warmup=2):
        # a weak reference: Trainer -> TrainStepGraph -> Trainer would be a reference cycle,
        # so a dropped trainer's CUDAGraph would be destroyed by the cyclic collector -- which
        # may run inside a later capture, where ~CUDAGraph's device synchronisation is refused
        # and the process aborts (round 5; DESIGN section 9.3, hipgraph.capture)
        self._tr = weakref.ref(trainer)
        self.warmup = int(warmup)
        self.g = None
        self.steps = 0

    @property
    def tr(self):
        return self._tr()

    def step(self, clip: Clip) -> torch.Tensor:
        tr = self.tr
        if self.steps < self.warmup:
            self.steps += 1
            return tr._eager_step(clip)
        model = tr.model
        model.train()
        enc = model.encode_audio(clip.audio).float()
        if self.g is None:
            self._capture(clip, enc)
        elif self._shapes(clip, enc) != self.shapes:
            # a batch of another shape (a short last batch): eager, with every gradient
            # released first so that the eager backward does not accumulate into the graph's
            tr.opt.zero_grad(set_to_none=True)
            self.steps += 1
            return tr._eager_step(clip)
        for p, g in self.grads:  # (an eager step in between may have released them)
            p.grad = g
        with torch.no_grad():
            for dst, src in ((self.x0, clip.x0), (self.eps, clip.eps), (self.t, clip.t),
                             (self.cond, clip.cond), (self.feats, enc)):
                dst.copy_(src)
        self.g.replay()
        if enc.requires_grad:
            enc.backward(self.feats.grad)
        tr.opt.step()
        for p in self.eager_params:
            p.grad = None
        self.steps += 1
        loss = self.loss.clone()  # the replay's own MSE (vd_mse_loss, captured)
        tr._track_finite(loss)
        return loss

    def node_types(self):
        """{node type: count} of the captured graph (vdiff.hipgraph; memset nodes must be 0)."""
        from .hipgraph import graph_nodes
        nodes = graph_nodes(self.g.raw_cuda_graph())
        return {t: sum(1 for n in nodes if n["type"] == t) for t in {n["type"] for n in nodes}}

    @staticmethod
    def _shapes(clip, enc):
        return tuple((tuple(x.shape), x.dtype) for x in (clip.x0, clip.eps, clip.t, clip.cond, enc))

    def _body(self):
        """The captured region.  The loss is vd_mse_loss (ops.mse_loss), a fixed-order
        two-launch reduction: round 4 found torch's one-launch multi-block mean (per-block
        partials, a semaphore reset by a captured hipMemsetAsync, a last-block combine)
        returning a stale value from some replay on -- the replay's output kept an earlier
        value while every gradient stayed exact -- and round 5 reproduced that with torch alone
        (tools/graph_reduce_repro.py) and saw it vanish under DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
        (DESIGN section 9.3).  The captured step holds no memset node
        (tests/test_gpu_train_graph.py), and step() returns this in-graph value."""
        tr = self.tr
        with tr.packs:
            xt = tr.scheduler.add_noise(self.x0, self.eps, self.t)
            pred = tr.model(xt, self.cond, self.feats, self.t)
            loss = tr.loss_fn(pred, self.eps)
            self.loss = loss.detach()  # lives in the graph's pool, rewritten by each replay
            loss.backward()

    def _capture(self, clip, enc):
        from . import _lib
        tr, model = self.tr, self.tr.model
        self.x0, self.eps = clip.x0.clone(), clip.eps.clone()
        self.t, self.cond = clip.t.clone(), clip.cond.clone()
        self.feats = enc.detach().clone().requires_grad_(enc.requires_grad)
        enc_ids = {id(p) for p in model.audio_encoder.parameters()} \
            if getattr(model, "audio_encoder", None) is not None else set()
        self.eager_params = [p for p in model.parameters() if p.requires_grad and id(p) in enc_ids]
        self.ctr = torch.zeros((), dtype=torch.int64, device=enc.device)
        tr.opt.zero_grad(set_to_none=True)
        # one run of the region on a side stream before capture (torch's graph recipe: lazy
        # allocator / autograd state), its gradients discarded
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self._body()
        torch.cuda.current_stream().wait_stream(side)
        tr.opt.zero_grad(set_to_none=True)
        self.feats.grad = None
        self.g = torch.cuda.CUDAGraph(keep_graph=True)  # node list kept (graph_nodes)
        lib = _lib.lib()
        lib.vd_set_dropout_counter(self.ctr.data_ptr())
        try:
            with hipgraph.capture(self.g, capture_error_mode="thread_local"):
                self.ctr.add_(1)
                self._body()
        finally:
            lib.vd_set_dropout_counter(None)
        self.g.instantiate()
        self.shapes = self._shapes(clip, enc)
        tr.packs.frozen = True  # the graph replays the pack launch into these buffers
        self.grads = [(p, p.grad) for p in model.parameters() if p.grad is not None]
        missing = [n for n, p in model.named_parameters()
                   if p.requires_grad and id(p) not in enc_ids and p.grad is None]
        if missing:  # a parameter off the captured path would silently never train
            raise RuntimeError(f"TrainStepGraph: no captured gradient for {missing[:4]}")


@torch.no_grad()
def sample_ddim(model, sampler, cond, audio, shape, generator=None, callback=None):
    """DDIM sampling (build extension of test.py:51-83): audio encoded once, packed conv
    weights reused across steps (ops.frozen_weights)."""
    with ops.frozen_weights():
        return _sample_ddim(model, sampler, cond, audio, shape, generator, callback)


class GraphUnsafe(RuntimeError):
    """A captured graph holds a node type that is not safe to replay (a memset node)."""


class DDIMGraph:
    """One deterministic DDIM denoising step -- UNet forward + vd_ddim_step -- captured once
    as a HIP graph and replayed per step (no per-kernel launch gaps, no host work per
    step).  The sample lives in a static buffer updated in place; the step's timesteps are
    copied device-to-device from the sampler's table before each replay.  Use inside
    ops.frozen_weights() (the graph reads the cached packed conv weights); eta must be 0."""

    def __init__(self, model, sampler, cond, feats, xt):
        if sampler.eta != 0:
            raise ValueError("DDIMGraph: eta = 0 (deterministic DDIM) only")
        dev = xt.device
        B = xt.shape[0]
        self.model, self.sampler = model, sampler
        self.cond, self.feats = cond, feats
        self.xt = xt.clone()
        self.t_all = sampler.timesteps.to(dev).view(-1, 1).expand(-1, B).contiguous()
        self.tp_all = sampler.prev_timesteps.to(dev).view(-1, 1).expand(-1, B).contiguous()
        self.t = self.t_all[0].clone()
        self.tp = self.tp_all[0].clone()
        self.acp = sampler._acp(dev)
        self.graph = None
        self.x0 = None

    def _body(self):
        eps = self.model(self.xt, self.cond, self.feats, self.t)
        xp, x0 = ops.ddim_step(self.xt, eps.to(self.xt.dtype), self.t, self.tp, self.acp,
                               eta=0.0, clip=self.sampler.clip_x0)
        self.xt.copy_(xp.view_as(self.xt))
        return x0

    def capture(self):
        """Warm up eagerly and capture one step (step() does this on first use).  Raises
        GraphUnsafe if the captured step holds a memset node."""
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream(device=self.xt.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):  # eager warm-up: packed weights, tables, workspaces
            keep = self.xt.clone()
            self._body()
            self.xt.copy_(keep)
        cur.wait_stream(side)
        self.graph = torch.cuda.CUDAGraph(keep_graph=True)  # node list kept (node_types)
        with hipgraph.capture(self.graph):
            self.x0 = self._body()
        self.graph.instantiate()
        types = self.node_types()
        if types.get("memset", 0):
            # a memset node replayed with eager work between replays is
            # where a captured reduction went stale on this HIP runtime; sample() steps
            # eagerly instead of trusting such a graph
            raise GraphUnsafe(f"DDIMGraph: captured step holds memset nodes {types}")

    def node_types(self):
        """{node type: count} of the captured step (vdiff.hipgraph; memset nodes must be 0)."""
        return hipgraph.node_counts(self.graph)

    def step(self, i):
        """Denoise from sampler.timesteps[i]; returns (x_prev, x0) (static buffers)."""
        self.t.copy_(self.t_all[i])
        self.tp.copy_(self.tp_all[i])
        if self.graph is None:
            self.capture()
        self.graph.replay()
        return self.xt, self.x0.view_as(self.xt)


def _use_graph(device, sampler):
    return (device.type == "cuda" and sampler.eta == 0
            and os.environ.get("VDIFF_DDIM_GRAPH", "1") != "0")


def _sample_ddim(model, sampler, cond, audio, shape, generator, callback):
    model.eval()
    device = cond.device
    feats = model.encode_audio(audio) if hasattr(model, "encode_audio") else audio
    xt = torch.randn(shape, generator=generator, device=device)
    x0 = None
    if _use_graph(device, sampler):
        g = DDIMGraph(model, sampler, cond, feats, xt)
        try:
            g.capture()
        except GraphUnsafe as e:
            warnings.warn(f"{e}; sampling eagerly")
            g = None
        if g is not None:
            for i in range(sampler.steps):
                xt, x0 = g.step(i)
                if callback is not None:  # the graph's static buffers: the next replay rewrites them
                    callback(i, xt.clone(), x0.clone())
            return xt.clone(), x0.clone()
    for i in range(sampler.steps):
        t = torch.full((shape[0],), int(sampler.timesteps[i]), dtype=torch.int64, device=device)
        eps = model(xt, cond, feats, t)
        xt, x0 = sampler.step(xt, eps, i)
        if callback is not None:
            callback(i, xt, x0)
    return xt, x0


@torch.no_grad()
def sample_ddpm(model, scheduler, cond, audio, shape, n_timesteps=None, generator=None,
                callback=None):
    """Ancestral sampling as test.py:51-83 (V2 scheduler by default there)."""
    with ops.frozen_weights():
        return _sample_ddpm(model, scheduler, cond, audio, shape, n_timesteps, generator,
                            callback)


def _sample_ddpm(model, scheduler, cond, audio, shape, n_timesteps, generator, callback):
    model.eval()
    device = cond.device
    feats = model.encode_audio(audio) if hasattr(model, "encode_audio") else audio
    n = n_timesteps or scheduler.num_timesteps
    xt = torch.randn(shape, generator=generator, device=device)
    x0 = None
    for i in reversed(range(n)):
        t = torch.full((shape[0],), i, dtype=torch.int64, device=device)
        eps = model(xt, cond, feats, t)
        z = torch.randn(xt.shape, generator=generator, device=device)
        xt, x0 = scheduler.sample_prev_timestep(xt, eps, t, z=z)
        if callback is not None:
            callback(i, xt, x0)
    return xt, x0
