"""Data-parallel training over torch.distributed (backend "nccl" = RCCL on ROCm).

One process per GPU; each rank holds a full replica and a disjoint minibatch of
clips.  GroupNorm is per-sample, so no activation exchange exists: the only
collective is the gradient all-reduce.  Gradients live in flat fp32
bucket buffers (p.grad is a view into them), and a bucket's all-reduce is launched
asynchronously from the post-accumulate-grad hook of the last parameter that
fills it, so RCCL traffic over xGMI overlaps the rest of the backward pass.
Buckets are filled in reverse registration order (the order backward produces
gradients), ~25 MB each: large enough to run the 7 xGMI links near their per-link
rate, small enough that the first bucket launches early in the backward.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def local_device_index(local: int) -> int:
    """GPU of a local rank: one per GPU.  More local ranks than GPUs (a multi-rank rehearsal
    on a one-GPU box, VDIFF_DIST_BACKEND=gloo) share the GPUs round-robin."""
    count = torch.cuda.device_count()  # does not initialise the GPU
    return local % count if count > 0 else local


def init_from_env(backend: str | None = None):
    """Initialise the default process group from torchrun's env; returns (rank, world, local).

    backend: None = VDIFF_DIST_BACKEND if set, else "nccl" (RCCL) with a GPU, else "gloo".
    `local` is the GPU index (local_device_index), not necessarily LOCAL_RANK."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = local_device_index(int(os.environ.get("LOCAL_RANK", "0")))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("VDIFF_DIST_BACKEND") or (
                "nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


class _Bucket:
    __slots__ = ("params", "flat", "pending", "work", "launched")

    def __init__(self, params, flat):
        self.params = params
        self.flat = flat
        self.pending = len(params)  # parameters still without this step's gradient
        self.work = None
        self.launched = False


class GradBucketer:
    """Bucketed, backward-overlapped gradient averaging.

    Usage per step:  loss.backward(); bucketer.finish(); optimizer.step();
    bucketer.zero_grad()  (never optimizer.zero_grad(set_to_none=True): p.grad must
    stay a view of the bucket buffer).

    Buckets are launched strictly in bucket order on every rank: a ready bucket waits for
    its predecessors.  Which parameters receive a gradient can differ between ranks
    (wav2vec2's LayerDrop and SpecAugment in train mode skip layers / the mask embedding at
    random), so launching in hook-completion order would pair different buckets in one
    collective.  A bucket with a parameter that got no gradient launches from finish(),
    carrying zeros for it -- what DDP's find_unused_parameters does.  A parameter that got
    no gradient on ANY rank (e.g. the ViViT pooler) has its .grad set to None for the
    optimizer step, as in a single process, so weight decay does not touch it.
    """

    def __init__(self, params, bucket_mb: float = 25.0, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        params = [p for p in params if p.requires_grad]
        cap = int(bucket_mb * 2 ** 20)
        self.buckets: list[_Bucket] = []
        cur, size = [], 0
        for p in reversed(params):
            nbytes = p.numel() * 4
            if cur and size + nbytes > cap:
                self.buckets.append(self._make(cur))
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            self.buckets.append(self._make(cur))
        self.next = 0  # first bucket not yet launched
        self.bucket_of = {}
        self.index = {}  # param -> position in self.used
        self.views = []  # (param, its gradient view into the bucket buffer)
        for b in self.buckets:
            for p in b.params:
                self.bucket_of[p] = b
                self.index[p] = len(self.views)
                self.views.append((p, p.grad))
                if self.world > 1:
                    p.register_post_accumulate_grad_hook(self._hook)
        self.used = [0] * len(self.views)  # this rank: did the parameter get a gradient

    def _make(self, params):
        dev = params[0].device
        flat = torch.zeros(sum(p.numel() for p in params), dtype=torch.float32, device=dev)
        off = 0
        for p in params:
            if p.dtype != torch.float32:
                raise TypeError("GradBucketer expects fp32 master parameters")
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        return _Bucket(params, flat)

    def _launch(self, b: _Bucket):
        b.launched = True
        b.work = dist.all_reduce(b.flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def _hook(self, p):
        self.used[self.index[p]] = 1
        self.bucket_of[p].pending -= 1
        while self.next < len(self.buckets) and self.buckets[self.next].pending == 0:
            self._launch(self.buckets[self.next])
            self.next += 1

    def finish(self):
        """Launch the remaining buckets in order (those with parameters that got no
        gradient, and their successors), wait for all, and average."""
        if self.world == 1:
            return
        for b in self.buckets[self.next:]:
            self._launch(b)
        self.next = len(self.buckets)
        used = None
        if not all(self.used):  # some parameter got no gradient here: is it unused anywhere?
            used = torch.tensor(self.used, dtype=torch.int32, device=self.buckets[0].flat.device)
        flag = torch.tensor([0 if used is None else 1], dtype=torch.int32,
                            device=self.buckets[0].flat.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        if int(flag.item()):
            if used is None:
                used = torch.ones(len(self.used), dtype=torch.int32,
                                  device=self.buckets[0].flat.device)
            dist.all_reduce(used, op=dist.ReduceOp.MAX, group=self.group)
            for (p, _), u in zip(self.views, used.tolist()):
                if not u:
                    p.grad = None  # restored by zero_grad()
        for b in self.buckets:
            b.work.wait()
            b.flat.mul_(1.0 / self.world)
            b.work = None

    def zero_grad(self):
        for b in self.buckets:
            b.flat.zero_()
            b.pending = len(b.params)
            b.launched = False
        for p, v in self.views:
            if p.grad is None:
                p.grad = v
        self.used = [0] * len(self.views)
        self.next = 0

    @property
    def nbytes(self):
        return sum(b.flat.numel() * 4 for b in self.buckets)


def broadcast_parameters(module, src=0, group=None):
    """Make every rank start from rank `src`'s weights."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src, group=group)
