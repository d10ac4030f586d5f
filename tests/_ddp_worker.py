"""One rank of tests/test_gpu_ddp.py (not collected by pytest): the tiny audio-conditioned
UNet3D in fp32 on the one GPU, its half of a 2-clip batch, gradients averaged by
vdiff.ddp.GradBucketer over gloo (VDIFF_DIST_BACKEND=gloo, set before any GPU call).

    RANK=r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tests/_ddp_worker.py OUT
Writes OUT.rank<r>.pt: {"grads": {name: grad}, "launched_in_backward": k, "buckets": n}.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("VDIFF_DIST_BACKEND", "gloo")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from vdiff.ddp import GradBucketer, broadcast_parameters, init_from_env  # noqa: E402

TINY = dict(image_size=16, in_channels=3, model_channels=32, out_channels=3, num_res_blocks=1,
            attention_resolutions=(2,), channel_mult=(1, 2), dims=3, audio_feature_dim=64,
            projected_audio_dim=16, im_cond_output_ch=16, dropout=0.0)


def build(dev):
    from oracle.unet import init_params
    from vdiff.unet_audio import UNetAudio
    m = UNetAudio(**TINY, audio_encoder=False)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    m.load_state_dict(init_params(shapes, 21))
    return m.to(dev)


def batch(dev):
    """Two clips [2, 3, 4, 16, 16] + cond images, pooled audio [2*4, 64], eps, t."""
    from oracle.fixtures import seeded
    x0 = seeded((2, 3, 4, 16, 16), 31, "uniform")
    cond = seeded((2, 3, 16, 16), 32, "uniform")
    feat = seeded((8, 64), 33)
    eps = seeded((2, 3, 4, 16, 16), 34)
    t = torch.tensor([12, 81])
    return [u.to(dev) for u in (x0, cond, feat, eps, t)]


def loss_of(m, sched, x0, cond, feat, eps, t):
    xt = sched.add_noise(x0, eps, t)
    return F.mse_loss(m(xt, cond, feat, t), eps)


def main(out):
    rank, world, local = init_from_env()          # gloo: no GPU call before this point
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    from vdiff.schedulers import LinearNoiseScheduler
    m = build(dev)
    broadcast_parameters(m)
    bk = GradBucketer([p for p in m.parameters()], bucket_mb=0.25)
    sched = LinearNoiseScheduler(100, 0.00085, 0.012)
    x0, cond, feat, eps, t = batch(dev)
    T = x0.shape[2]
    sl = slice(rank, rank + 1)
    loss = loss_of(m, sched, x0[sl], cond[sl], feat[rank * T:(rank + 1) * T], eps[sl], t[sl])
    loss.backward()
    launched = bk.next                            # buckets whose all-reduce began in backward
    bk.finish()
    torch.save({"grads": {n: p.grad.detach().cpu() for n, p in m.named_parameters()},
                "launched_in_backward": launched, "buckets": len(bk.buckets)},
               f"{out}.rank{rank}.pt")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
