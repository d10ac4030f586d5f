"""Which Python lines launch the torch (non-libvdiff) kernels of a config-2 train step: one
profiled step under torch.profiler with stacks, grouped by the aten op and the innermost
frames inside this repository (vdiff / bench), sorted by device time.

    python tools/op_census.py [--mode spatial_temporal|joint] [--top 40]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="spatial_temporal")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    from vdiff.engine import Trainer
    from vdiff.schedulers import LinearNoiseScheduler
    argv, sys.argv = sys.argv, ["bench.py", "--mode", a.mode]
    args = bench.parse()  # the bench's defaults (lr, dropout, sizes)
    sys.argv = argv
    dev = torch.device("cuda:0")
    bench.seed_host(1234)
    model = bench.build_model(args, dev)
    tr = Trainer(model, LinearNoiseScheduler(100, 0.00085, 0.012), lr=args.lr)
    bank = bench.clip_bank(args, 4, dev, 0)
    for i in range(3):
        tr.step(bank[i])
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    cfg = torch._C._profiler._ExperimentalConfig(verbose=True)  # Python stacks on this torch
    with torch.profiler.profile(activities=acts, with_stack=True, experimental_config=cfg) as prof:
        tr.step(bank[3])
        torch.cuda.synchronize()
    rows = {}
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CPU or not ev.name.startswith("aten::"):
            continue
        dev_us = sum(k.duration for k in ev.kernels) if ev.kernels else 0.0
        if not dev_us:
            continue
        while ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
            ev = ev.cpu_parent  # attribute the kernel to its outermost aten op
        frames = [f for f in (ev.stack or []) if "op_census" not in f and "site-packages" not in
                  f and "dist-packages" not in f and "torch/" not in f]
        where = " < ".join(f.split("/")[-1] for f in frames[:3])
        if not where:  # backward: the autograd node that ran it
            par = ev.cpu_parent
            while par is not None and not par.name.startswith("autograd::engine"):
                par = par.cpu_parent
            where = par.name.replace("autograd::engine::evaluate_function: ", "bwd ") if par \
                else "(no Python frame)"
        if any("transformers" in f for f in (ev.stack or [])):
            where += " [transformers]"
        key = (ev.name, where)
        n, t = rows.get(key, (0, 0.0))
        rows[key] = (n + 1, t + dev_us)
    tot = sum(t for _, t in rows.values())
    print(f"torch-launched kernels in one {a.mode} train step: {tot / 1e3:.2f} ms "
          f"(device time of the outermost aten ops with kernels)")
    for (name, where), (n, t) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / 1e3:8.3f} ms  x{n:<4d} {name:28s} {where}")


if __name__ == "__main__":
    main()
