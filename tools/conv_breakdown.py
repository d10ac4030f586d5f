"""Per-shape conv kernel time of the config-2 train step (HIP events per launch over 3 timed
steps): which convolutions the 20 ms of conv per step go to.   python tools/conv_breakdown.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    import bench
    from vdiff import ops
    from vdiff.engine import Trainer, synthetic_clip
    from vdiff.schedulers import LinearNoiseScheduler
    dev = torch.device("cuda", 0)
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    torch.manual_seed(0)
    model = bench.build_model(args, dev)
    tr = Trainer(model, LinearNoiseScheduler(100, 0.00085, 0.012), lr=1e-2)
    clip = synthetic_clip(1, 16, 128, 100, dev, seed=0)
    for _ in range(2):
        tr.step(clip)
    timer = ops.KernelTimer()
    ops.set_timer(timer)
    steps = 3
    for _ in range(steps):
        tr.step(clip)
    ops.set_timer(None)
    rows = sorted(timer.conv_summary().items(), key=lambda kv: -kv[1][1])
    tot = sum(v[1] for v in timer.conv_summary().values()) / steps
    print(f"conv total {tot:.2f} ms/step")
    for (kind, key), (cnt, ms, flop) in rows:
        per = ms / cnt
        print(f"{kind:16s} {key:45s} x{cnt // steps:3d}  {ms / steps:7.3f} ms/step  "
              f"{per * 1e3:8.1f} us  {flop / per / 1e9:7.1f} TF/s")


if __name__ == "__main__":
    main()
