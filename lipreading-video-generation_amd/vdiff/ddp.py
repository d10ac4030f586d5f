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

The reference has no multi-GPU training at all (test.py:101 wraps sampling in
nn.DataParallel); this replaces that with one process per GPU.
"""
from __future__ import annotations

import os

import weakref

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
    """Bucketed, backward-overlapped gradient averaging with no host synchronisation.

    Usage per step:  loss.backward(); bucketer.finish(); bucketer.step(optimizer);
    bucketer.zero_grad()  (never optimizer.zero_grad(set_to_none=True): p.grad must
    stay a view of the bucket buffer).

    Buckets are launched strictly in bucket order on every rank: a ready bucket waits for
    its predecessors.  Which parameters receive a gradient can differ between ranks
    (wav2vec2's LayerDrop and SpecAugment in train mode skip layers / the mask embedding at
    random), so launching in hook-completion order would pair different buckets in one
    collective.  A bucket with a parameter that got no gradient launches from finish(),
    carrying zeros for it -- what DDP's find_unused_parameters does.

    Unused-everywhere parameters.  In one process a parameter that got no gradient keeps
    .grad = None and the optimizer leaves it (and its moments) alone.  Here every rank
    must agree on which parameters that applies to, without the host waiting for the GPU.
    The LAST bucket (launched last on every rank, and only once every hook of the step
    has run or finish() has been called) carries one fp32 "used" flag per parameter
    after its gradients, uploaded from pinned host memory right before its all-reduce;
    after the sum, flag > 0 means "used on some rank".  step(optimizer) snapshots only
    the parameters this rank did not use (the host knows them from its hooks), runs the
    optimizer, and restores parameter and optimizer state on the device where the summed
    flag is 0 -- all stream-ordered, so the host queues the next step at once.  With
    every parameter used on this rank, step() is plain optimizer.step().
    """

    def __init__(self, params, bucket_mb: float = 25.0, group=None, timing: bool = False):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        params = [p for p in params if p.requires_grad]
        for p in params:
            if p.dtype != torch.float32:
                raise TypeError("GradBucketer expects fp32 master parameters")
        cap = int(bucket_mb * 2 ** 20)
        groups, cur, size = [], [], 0
        for p in reversed(params):
            nbytes = p.numel() * 4
            if cur and size + nbytes > cap:
                groups.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            groups.append(cur)
        nparams = len(params)
        self.buckets: list[_Bucket] = [
            self._make(g, extra=nparams if i == len(groups) - 1 else 0)
            for i, g in enumerate(groups)]
        self.next = 0  # first bucket not yet launched
        self.bucket_of = {}
        self.index = {}  # param -> position in self.used
        self.views = []  # (param, its gradient view into the bucket buffer)
        # the hooks hold the bucketer weakly: a bound method would make a parameter -> hook ->
        # bucketer -> parameter cycle, so a dropped bucketer (its gradient buffers and pinned
        # flags) would wait for the cyclic collector instead of being released at once
        ref = weakref.ref(self)

        def hook(p):
            me = ref()
            if me is not None:
                me._hook(p)
        for b in self.buckets:
            for p in b.params:
                self.bucket_of[p] = b
                self.index[p] = len(self.views)
                self.views.append((p, p.grad))
                if self.world > 1:
                    p.register_post_accumulate_grad_hook(hook)
        self.used = [0] * len(self.views)  # this rank: did the parameter get a gradient
        self.unused_local: list[int] = []
        if self.buckets:
            last = self.buckets[-1].flat
            self.flags = last[last.numel() - nparams:]  # summed "used" flags after finish()
            pin = last.is_cuda
            self._flags_host = torch.zeros(nparams, dtype=torch.float32, pin_memory=pin)
            self._flags_evt = torch.cuda.Event() if pin else None
        self.timing = timing and bool(self.buckets) and self.buckets[0].flat.is_cuda
        self._times = []  # (event after backward, event after the averaged buckets)

    def _make(self, params, extra=0):
        dev = params[0].device
        flat = torch.zeros(sum(p.numel() for p in params) + extra, dtype=torch.float32,
                           device=dev)
        off = 0
        for p in params:
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        return _Bucket(params, flat)

    def _launch(self, b: _Bucket):
        if b is self.buckets[-1]:
            # every hook of this step has run (or finish() was called): the flags are final
            if self._flags_evt is not None:
                self._flags_evt.synchronize()  # the previous step's upload has left the buffer
            self._flags_host.numpy()[:] = self.used
            self.flags.copy_(self._flags_host, non_blocking=True)
            if self._flags_evt is not None:
                self._flags_evt.record()
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
        gradient, and their successors), make the current stream wait for all of them, and
        average.  No host synchronisation with RCCL (work.wait() is a stream wait)."""
        if self.world == 1:
            return
        if self.timing:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        for b in self.buckets[self.next:]:
            self._launch(b)
        self.next = len(self.buckets)
        self.unused_local = [i for i, u in enumerate(self.used) if not u]
        for b in self.buckets:
            b.work.wait()
            b.flat.mul_(1.0 / self.world)
            b.work = None
        if self.timing:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self._times.append((e0, e1))

    @torch.no_grad()
    def step(self, optimizer):
        """optimizer.step(), except that parameters no rank produced a gradient for keep
        their values and optimizer state (as with .grad = None in one process).  Call after
        finish()."""
        if self.world == 1 or not self.unused_local:
            optimizer.step()
            return
        snaps = []
        for i in self.unused_local:
            p = self.views[i][0]
            st = optimizer.state.get(p, {})
            snaps.append((i, p, p.detach().clone(),
                          {k: v.clone() for k, v in st.items() if torch.is_tensor(v)}))
        optimizer.step()
        for i, p, p0, s0 in snaps:
            keep = self.flags[i] > 0  # summed over ranks: used somewhere
            p.copy_(torch.where(keep, p, p0))
            for k, v in optimizer.state.get(p, {}).items():
                if torch.is_tensor(v):
                    old = s0.get(k)
                    v.copy_(torch.where(keep, v, old if old is not None else torch.zeros_like(v)))

    def globally_unused(self) -> list[int]:
        """Indices (into self.views) of the parameters no rank used in the last step.
        Reads the summed flags: a host synchronisation, for tests and diagnostics only."""
        return [i for i, f in enumerate(self.flags.tolist()) if f == 0]

    def zero_grad(self):
        for b in self.buckets:
            b.flat.zero_()
            b.pending = len(b.params)
            b.launched = False
        self.used = [0] * len(self.views)
        self.next = 0

    def comm_times_ms(self) -> list[float]:
        """Per-step exposed gradient-exchange time (timing=True): from the end of the
        backward on the compute stream to the averaged buckets, i.e. the all-reduce time
        NOT hidden under the backward.  Synchronises; call after the timed region."""
        torch.cuda.synchronize()
        out = [a.elapsed_time(b) for a, b in self._times]
        self._times = []
        return out

    @torch.no_grad()
    def standalone_allreduce_ms(self, iters: int = 3) -> float:
        """Time of the step's whole gradient exchange issued alone (every bucket back to
        back, no backward to hide under), averaged over `iters`; synchronises."""
        if self.world == 1 or not self.buckets:
            return 0.0
        keep = [b.flat.clone() for b in self.buckets]
        dist.barrier(group=self.group)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            works = [dist.all_reduce(b.flat, group=self.group, async_op=True)
                     for b in self.buckets]
            for w in works:
                w.wait()
        e1.record()
        torch.cuda.synchronize()
        for b, k in zip(self.buckets, keep):
            b.flat.copy_(k)
        return e0.elapsed_time(e1) / iters

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
