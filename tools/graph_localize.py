"""Localise the graph-replayed train-step defect: two copies of the
bench UNet3D from one init (no audio encoder: pooled features in, so no host-side random
masks; ResBlock dropout 0), one Trainer eager and one Trainer(graph=True), both at lr 0 so the
weights never move and every step sees the same operands.  With every reduction fixed-order
(round 4), each replay must equal the eager step BIT FOR BIT: loss and every parameter
gradient.  Prints, per step, the loss pair and the parameters whose gradients differ
(backward order: the first listed is the earliest-computed difference).
With --lr > 0 the weights move (Adam, eager after each replay) and the parameters after each
step are compared as well; --audio runs the wav2vec2 encoder (random init) with the host RNGs
(torch, numpy, random) re-seeded identically before each trainer's step, so both trainers draw
the same SpecAugment / LayerDrop decisions; --dropout sets the ResBlock dropout (the graph's
masks come from the device counter, so with dropout the two runs differ by design).
    python tools/graph_localize.py [--size 64] [--steps 4] [--lr 0] [--audio] [--dropout 0]"""
import argparse
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lipreading-video-generation_amd"), ROOT]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--mult", default="1,2,4")
    ap.add_argument("--lr", type=float, default=0.0)
    ap.add_argument("--audio", action="store_true")
    ap.add_argument("--dropout", type=float, default=0.0)
    ap.add_argument("--no-grads", action="store_true",
                    help="compare losses and weights only (no gradient copies)")
    ap.add_argument("--loss-first", action="store_true",
                    help="read the returned loss right after the step, before the copies")
    a = ap.parse_args()
    import random
    import numpy as np
    os.environ["VDIFF_TRAIN_GRAPH_EXPERIMENTAL"] = "1"
    from vdiff.engine import Clip, Trainer, reinit_nonzero
    from vdiff.schedulers import LinearNoiseScheduler
    from vdiff.unet_audio import UNetAudio
    dev = torch.device("cuda", 0)
    mult = tuple(int(x) for x in a.mult.split(","))
    torch.manual_seed(1234)
    m = UNetAudio(image_size=a.size, in_channels=3, model_channels=64, out_channels=3,
                  num_res_blocks=2, attention_resolutions=(1, 2, 4)[:len(mult)],
                  channel_mult=mult, audio_feature_dim=768, projected_audio_dim=128, dims=3,
                  use_bf16=True, audio_encoder=a.audio, audio_encoder_pretrained=False,
                  dropout=a.dropout)
    reinit_nonzero(m, seed=1234)
    m = m.to(dev)
    models = {"eager": m, "graph": copy.deepcopy(m)}
    sched = LinearNoiseScheduler(100, 0.00085, 0.012)
    trs = {k: Trainer(v, sched, lr=a.lr, graph=(k == "graph")) for k, v in models.items()}
    g = torch.Generator(device=dev).manual_seed(0)
    T, S = a.frames, a.size
    clip = Clip(torch.rand((1, 3, T, S, S), generator=g, device=dev) * 2 - 1,
                torch.rand((1, 3, S, S), generator=g, device=dev) * 2 - 1,
                ({"input_values": torch.randn((T, 4000), generator=g, device=dev)} if a.audio
                 else torch.randn((T, 768), generator=g, device=dev)),
                torch.randn((1, 3, T, S, S), generator=g, device=dev),
                torch.tensor([37], device=dev))
    names = [n for n, _ in m.named_parameters()]
    report = []
    for step in range(a.steps):
        rec = {}
        for k, tr in trs.items():
            grads = {}
            hooks = []
            if k == "eager" and not a.no_grads:  # graph grads: p.grad after the replay
                hooks = [p.register_post_accumulate_grad_hook(
                    lambda p, n=n: grads.__setitem__(n, p.grad.detach().clone()))
                    for n, p in models[k].named_parameters()]
            torch.manual_seed(1000 + step)
            np.random.seed(1000 + step)
            random.seed(1000 + step)
            loss = tr.step(clip)
            lval = float(loss) if a.loss_first else None
            for h in hooks:
                h.remove()
            if k == "graph" and tr.graph.g is not None and not a.no_grads:
                grads = {n: p.grad.detach().clone() for n, p in models[k].named_parameters()
                         if p.grad is not None}
            torch.cuda.synchronize()
            rec[k] = (float(loss) if lval is None else lval, grads)
            if lval is not None and lval != float(loss):
                print(json.dumps({"step": step, "trainer": k, "loss_changed_after_copies":
                                  [lval, float(loss)]}), flush=True)
        le, ge = rec["eager"]
        lg, gg = rec["graph"]
        diff = []
        for n in reversed(names):  # backward order
            if n in ge and n in gg and not torch.equal(ge[n], gg[n]):
                d = (gg[n].float() - ge[n].float())
                diff.append((n, float(d.abs().max()),
                             float(d.norm() / ge[n].float().norm().clamp_min(1e-30))))
        wdiff = [n for (n, pe), (_, pg) in zip(models["eager"].named_parameters(),
                                                 models["graph"].named_parameters())
                 if not torch.equal(pe, pg)]
        line = {"step": step, "loss_eager": le, "loss_graph": lg,
                "n_weights_differ": len(wdiff), "weights_differ": wdiff[:8],
                "graph_active": trs["graph"].graph.g is not None,
                "n_grads_compared": len(set(ge) & set(gg)), "n_differ": len(diff),
                "first_differing": diff[:12]}
        print(json.dumps(line), flush=True)
        report.append(line)
    bad = [r for r in report if r["n_differ"] or r["n_weights_differ"]
           or r["loss_eager"] != r["loss_graph"] or not r["loss_graph"] >= 0]
    print(json.dumps({"size": a.size, "frames": a.frames, "mult": mult, "lr": a.lr,
                      "audio": a.audio, "dropout": a.dropout, "steps_bad": len(bad)}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
