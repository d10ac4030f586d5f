"""Config-2 train step (vdiff.engine.Trainer, bench model): per step, HIP events at its
start and end on the current stream give the GPU period (start -> next start) and the
boundary gap (end -> next start: the time the GPU waits for the host to issue the next
step's first kernel).  Blocks of steps are repeated to show the period's drift (GPU box).
    python tools/step_gap.py [--steps 4] [--rounds 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from vdiff import ops  # noqa: E402
from vdiff.engine import Trainer, synthetic_clip  # noqa: E402
from vdiff.schedulers import LinearNoiseScheduler  # noqa: E402


def run(trainer, clip, steps):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps + 1)]
    for i in range(steps + 1):
        ev[i][0].record()
        if i < steps:
            trainer.step(clip)
        ev[i][1].record()
    torch.cuda.synchronize()
    period = [ev[i][0].elapsed_time(ev[i + 1][0]) for i in range(steps)]
    gap = [ev[i][1].elapsed_time(ev[i + 1][0]) for i in range(steps)]
    return period, gap


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lr", type=float, default=1e-2, help="0 keeps the weights fixed")
    ap.add_argument("--no-timer", action="store_true",
                    help="no per-launch attention events (for a kernel trace: tools/idle_gaps.py)")
    a = ap.parse_args()
    args = argparse.Namespace(size=128, frames=16, dtype="bf16", mode="joint")
    dev = torch.device("cuda", 0)
    model = bench.build_model(args, dev)
    sched = LinearNoiseScheduler(100, 0.00085, 0.012)
    tr = Trainer(model, sched, lr=a.lr)
    clip = synthetic_clip(1, 16, 128, 100, dev, seed=0)
    tr.step(clip)  # warm-up: state, tables, packed weights
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)  # trace marker (spin kernel): the timed rounds start after it
    ps, gs = [], []
    for r in range(a.rounds):
        timer = ops.KernelTimer() if not a.no_timer else None
        ops.set_timer(timer)
        p, g = run(tr, clip, a.steps)
        ops.set_timer(None)
        ps.extend(p)
        gs.extend(g)
        per = {}
        for (kind, hd, n, nseq), (cnt, ms) in (timer.summary().items() if timer else ()):
            per[(kind, hd)] = per.get((kind, hd), 0.0) + ms / a.steps
        print(f"round {r} period " + " ".join(f"{x:.2f}" for x in p)
              + " | boundary gap " + " ".join(f"{x:.3f}" for x in g), flush=True)
        print("   attention ms/step: " + ", ".join(
            f"{k} d{hd} {v:.1f}" for (k, hd), v in sorted(per.items(), key=lambda kv: -kv[1])
            if v > 1.0), flush=True)
    print(f"mean period {sum(ps) / len(ps):.2f} ms, mean boundary gap "
          f"{sum(gs) / len(gs):.3f} ms ({len(ps)} steps)")


if __name__ == "__main__":
    main()
