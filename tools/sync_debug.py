"""Find host<->GPU synchronisations inside the bench train step (GPU box).

torch's sync debug mode warns at every synchronising call (item(), nonzero, pageable
copies, ...); each warning is printed once with the Python stack that issued it.
    python tools/sync_debug.py [--steps 2]
"""
import argparse
import os
import sys
import traceback
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from vdiff.engine import Trainer, synthetic_clip  # noqa: E402
from vdiff.schedulers import LinearNoiseScheduler  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--frames", type=int, default=16)
    a = ap.parse_args()
    args = argparse.Namespace(size=a.size, frames=a.frames, dtype="bf16", mode="joint")
    dev = torch.device("cuda", 0)
    model = bench.build_model(args, dev)
    tr = Trainer(model, LinearNoiseScheduler(100, 0.00085, 0.012), lr=1e-2)
    clip = synthetic_clip(1, a.frames, a.size, 100, dev, seed=0)
    tr.step(clip)  # warm-up: first-call allocations and tables
    torch.cuda.synchronize()

    seen = {}

    def show(message, category, filename, lineno, file=None, line=None):
        stack = "".join(traceback.format_stack()[:-1][-8:])
        key = (str(message), stack)
        seen[key] = seen.get(key, 0) + 1

    warnings.showwarning = show
    warnings.simplefilter("always")
    torch.cuda.set_sync_debug_mode("warn")
    for _ in range(a.steps):
        tr.step(clip)
    torch.cuda.set_sync_debug_mode("default")
    torch.cuda.synchronize()
    print(f"{len(seen)} distinct synchronising call sites in {a.steps} steps")
    for (msg, stack), n in seen.items():
        print(f"--- x{n}: {msg}\n{stack}")


if __name__ == "__main__":
    main()
