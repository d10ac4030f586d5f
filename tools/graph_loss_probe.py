"""Where does the graph-replayed train step's wrong LOSS come from?  (tools/graph_localize.py,
batch r04d: with the weights moving, every replayed gradient and every weight after Adam is
bit-identical to the eager step's, but from the third replay on the returned loss is a
bf16-exact garbage value, e.g. -0.85546875.)  One graph Trainer (64x64x16, no audio encoder,
dropout 0, lr 1e-2); per step after the replay this reads, with a sync between each:
  loss_out   the graph's captured loss output (TrainStepGraph.loss) right after the replay
  mse_pred   F.mse_loss recomputed eagerly from the graph's own prediction buffer
  loss_after the same output after the eager Adam step
  returned   the value Trainer.step returned
and checks the packed-operand plan: every descriptor's source and destination pointer must be
a live parameter / plan buffer, and the loss buffer must lie outside every plan buffer.
--sync 0 drops the synchronised reads; --keep-pred 0 --sync 0 runs the product's own
TrainStepGraph.step (since round 4 it reports the eager MSE of the kept prediction).
    python tools/graph_loss_probe.py [--steps 7] [--twin] [--keep-pred 0|1] [--sync 0|1]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lipreading-video-generation_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--steps", type=int, default=7)
    ap.add_argument("--twin", action="store_true", help="an eager twin trainer alternates")
    ap.add_argument("--keep-pred", type=int, default=1,
                    help="1: report the old in-graph loss output from the probe's own step; "
                         "0 (with --sync 0 and no --snap): the product's step, which reports the "
                         "eager MSE of the replayed prediction (round-4 fix)")
    ap.add_argument("--sync", type=int, default=1, help="synchronise and read after the replay")
    ap.add_argument("--seed-each-step", action="store_true",
                    help="torch / numpy / random re-seeded before every step (graph_localize)")
    ap.add_argument("--snap", action="store_true",
                    help="inside the graph: copy the MSE to a second buffer before the "
                         "backward; after the replay: clone the loss output before Adam")
    ap.add_argument("--compare-weights", action="store_true",
                    help="torch.equal of every parameter pair after each step (needs --twin)")
    a = ap.parse_args()
    os.environ["VDIFF_TRAIN_GRAPH_EXPERIMENTAL"] = "1"
    import copy
    from vdiff import engine
    from vdiff.engine import Clip, Trainer, reinit_nonzero
    from vdiff.schedulers import LinearNoiseScheduler
    from vdiff.unet_audio import UNetAudio
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    m = UNetAudio(image_size=a.size, in_channels=3, model_channels=64, out_channels=3,
                  num_res_blocks=2, attention_resolutions=(1, 2, 4), channel_mult=(1, 2, 4),
                  audio_feature_dim=768, projected_audio_dim=128, dims=3, use_bf16=True,
                  audio_encoder=False, dropout=0.0)
    reinit_nonzero(m, seed=1234)
    m = m.to(dev)
    twin = copy.deepcopy(m) if a.twin else None
    sched = LinearNoiseScheduler(100, 0.00085, 0.012)
    tr = Trainer(m, sched, lr=1e-2, graph=True)
    tw = Trainer(twin, sched, lr=1e-2) if twin is not None else None
    g = torch.Generator(device=dev).manual_seed(0)
    T, S = 16, a.size
    clip = Clip(torch.rand((1, 3, T, S, S), generator=g, device=dev) * 2 - 1,
                torch.rand((1, 3, S, S), generator=g, device=dev) * 2 - 1,
                torch.randn((T, 768), generator=g, device=dev),
                torch.randn((1, 3, T, S, S), generator=g, device=dev),
                torch.tensor([37], device=dev))
    probe = {}
    G = engine.TrainStepGraph
    orig_body, orig_step = G._body, G.step

    def body(self):
        # the round-4 product body plus the old design's in-graph loss output (self.loss, a
        # buffer outside the graph pool, written by a copy after the backward)
        tr_ = self.tr
        with tr_.packs:
            xt = tr_.scheduler.add_noise(self.x0, self.eps, self.t)
            pred = tr_.model(xt, self.cond, self.feats, self.t)
            self.pred = pred.detach()
            loss = F.mse_loss(pred, self.eps)
            if a.snap:
                self.loss_pre.copy_(loss.detach())
            loss.backward()
        self.loss.copy_(loss.detach())

    def probe_step(self, clip_):
        if self.g is None or self.steps < self.warmup:
            return orig_step(self, clip_)
        enc = self.tr.model.encode_audio(clip_.audio).float()
        for p, gr in self.grads:
            p.grad = gr
        with torch.no_grad():
            for dst, src in ((self.x0, clip_.x0), (self.eps, clip_.eps), (self.t, clip_.t),
                             (self.cond, clip_.cond), (self.feats, enc)):
                dst.copy_(src)
        self.g.replay()
        if a.snap:
            probe["_snap_t"] = self.loss.clone()
            probe["_pre_t"] = self.loss_pre.clone()
        if a.sync:
            torch.cuda.synchronize()
            probe["loss_out"] = float(self.loss)
            probe["mse_pred"] = float(F.mse_loss(self.pred, self.eps))
        self.tr.opt.step()
        if a.sync:
            torch.cuda.synchronize()
            probe["loss_after"] = float(self.loss)
        self.steps += 1
        loss = self.loss.clone()
        self.tr._track_finite(loss)
        return loss

    G._body = body
    G.loss = torch.zeros((), dtype=torch.float32, device=dev)
    if a.snap:
        G.loss_pre = torch.zeros((), dtype=torch.float32, device=dev)
    report = []
    import random
    for step in range(a.steps):
        probe.clear()
        if tw is not None:
            if a.seed_each_step:
                torch.manual_seed(1000 + step)
                np.random.seed(1000 + step)
                random.seed(1000 + step)
            le = float(tw.step(clip))
        else:
            le = None
        if tr.graph.g is not None and (a.sync or a.keep_pred or a.snap):
            G.step = probe_step
        if a.seed_each_step:
            torch.manual_seed(1000 + step)
            np.random.seed(1000 + step)
            random.seed(1000 + step)
        lr_ = tr.step(clip)
        G.step = orig_step
        if a.compare_weights and twin is not None:
            probe["n_weights_differ"] = sum(1 for pe, pg in zip(twin.parameters(), m.parameters())
                                            if not torch.equal(pe, pg))
        for key in ("_snap_t", "_pre_t"):
            if key in probe:
                probe[key[1:-2]] = float(probe.pop(key))
        rec = {"step": step, "graph": tr.graph.g is not None, "returned": float(lr_),
               "eager_twin": le, **probe}
        if tr.graph.g is not None:
            pk = tr.packs
            live_out = {b.data_ptr(): b.numel() * b.element_size() for b in pk.bufs.values()}
            live_w = {p.data_ptr() for p in m.parameters()}
            bad = 0
            for dt, table, n, total in pk.plans:
                desc = np.dtype([("w", "<u8"), ("out", "<u8"), ("Co", "<i4"), ("Ci", "<i4"),
                                 ("taps", "<i4"), ("Cip", "<i4"), ("Cop", "<i4"),
                                 ("tr", "<i4"), ("start", "<i8")])
                rows = table.cpu().numpy().view(desc)
                bad += sum(1 for r in rows if int(r["w"]) not in live_w
                           or int(r["out"]) not in live_out)
            lp = tr.graph.loss.data_ptr()
            inside = [hex(o) for o, nb in live_out.items() if o <= lp < o + nb]
            rec.update({"plan_rows_bad": bad, "loss_ptr": hex(lp), "loss_inside_plan_buf": inside,
                        "n_plan_bufs": len(live_out)})
        print(json.dumps(rec), flush=True)
        report.append(rec)
    return 0


if __name__ == "__main__":
    sys.exit(main())
