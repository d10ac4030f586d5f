"""DDIM sampling as a replayed HIP graph against the eager loop at the BASELINE config-2 shape
(128x128x16, joint attention, bf16; the bench's model): max |diff| and rel-L2 of the samples
after --steps DDIM steps.  The tests (tests/test_gpu_ddim_graph.py) pin this at 32x32;
this tool checks the full-size graph, whose train-step counterpart returned impossible
losses.   python tools/ddim_graph_check.py [--steps 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lipreading-video-generation_amd"), ROOT]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--frames", type=int, default=16)
    a = ap.parse_args()
    import bench
    from vdiff import ops
    from vdiff.engine import sample_ddim, synthetic_clip
    from vdiff.schedulers import DDIMSampler, LinearNoiseSchedulerV2
    dev = torch.device("cuda", 0)
    ns = argparse.Namespace(size=a.size, frames=a.frames, dtype="bf16", mode="joint")
    model = bench.build_model(ns, dev).eval()
    clip = synthetic_clip(1, a.frames, a.size, 500, dev, seed=5)
    sampler = DDIMSampler(LinearNoiseSchedulerV2(500, 0.00005, 0.015), steps=a.steps)
    out = {}
    with torch.no_grad(), ops.frozen_weights():
        feats = model.encode_audio(clip.audio)
        for mode in ("0", "1"):
            os.environ["VDIFF_DDIM_GRAPH"] = mode
            g = torch.Generator(device=dev).manual_seed(9)
            seen = []
            sample_ddim(model, sampler, clip.cond, feats, tuple(clip.x0.shape), generator=g,
                        callback=lambda i, xt, x0: seen.append(xt.float()))
            out[mode] = seen
    res = []
    for i, (e, gr) in enumerate(zip(out["0"], out["1"])):
        d = (gr - e)
        res.append({"step": i, "max_abs": float(d.abs().max()),
                    "rel_l2": float(d.norm() / e.norm().clamp_min(1e-30)),
                    "finite": bool(torch.isfinite(gr).all())})
    print(json.dumps({"shape": list(clip.x0.shape), "steps": res}))


if __name__ == "__main__":
    main()
