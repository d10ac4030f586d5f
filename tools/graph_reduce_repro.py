"""Torch-only reproducer for the wrong in-graph MSE value of the graph-replayed train step
(DESIGN section 9 item 3): no libvdiff call anywhere.

A small bf16 "denoiser" (two GEMMs + SiLU on a 1x3x16x64x64 clip) -> F.mse_loss(pred, eps)
(fp32; torch's multi-block mean: per-block partials in a staging buffer, the last block found
through an atomic semaphore) -> a copy of the loss to a buffer outside the graph pool ->
backward, captured as one HIP graph and replayed with new inputs every step.  After each
replay the in-graph loss is compared with F.mse_loss recomputed eagerly from the graph's own
prediction buffer; between replays the host does what the round-4 probe did (an SGD update,
torch.equal over the parameters and clones of every gradient) unless --quiet-host.

    python tools/graph_reduce_repro.py [--replays 300] [--quiet-host] [--impl torch|twostage]
Prints one JSON line: replays, mismatches, the first few (replay, in-graph, eager) triples."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replays", type=int, default=300)
    ap.add_argument("--quiet-host", action="store_true", help="no host work between replays")
    ap.add_argument("--impl", default="torch", choices=["torch", "twostage"])
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--check-grads", action="store_true",
                    help="also recompute the step eagerly and compare the graph's gradients")
    ap.add_argument("--probe-sem", action="store_true",
                    help="read every memset node's destination (the reduction's semaphore) "
                         "after each replay through the HIP runtime (tools/hipgraph.py)")
    ap.add_argument("--host-ops", type=int, default=1,
                    help="repetitions of the host work between replays (launch count scale)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    T, S = 16, a.size
    shape = (1, 3, T, S, S)
    n = 3 * T * S * S
    W1 = torch.nn.Parameter(torch.randn(3, 256, device=dev) * 0.5)
    W2 = torch.nn.Parameter(torch.randn(256, 3, device=dev) * 0.05)
    params = [W1, W2]
    x = torch.randn(shape, device=dev)
    eps = torch.randn(shape, device=dev)
    snap = torch.zeros((), device=dev)
    state = {}

    def fwd(W1, W2):
        h = x.permute(0, 2, 3, 4, 1).reshape(-1, 3).bfloat16() @ W1.bfloat16()
        h = F.silu(h)
        return (h @ W2.bfloat16()).reshape(1, T, S, S, 3).permute(0, 4, 1, 2, 3).float()

    def body():
        h = x.permute(0, 2, 3, 4, 1).reshape(-1, 3).bfloat16() @ W1.bfloat16()
        h = F.silu(h)
        pred = (h @ W2.bfloat16()).reshape(1, T, S, S, 3).permute(0, 4, 1, 2, 3).float()
        state["pred"] = pred.detach()
        if a.impl == "torch":
            loss = F.mse_loss(pred, eps)
        else:  # per-row sums (no cross-block staging) then one small sum
            d = (pred.float() - eps).reshape(256, -1)
            loss = (d * d).sum(1).sum() * (1.0 / n)
        snap.copy_(loss.detach())
        loss.backward()

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        body()
    torch.cuda.current_stream().wait_stream(side)
    for p in params:
        p.grad = None
    g = torch.cuda.CUDAGraph(keep_graph=a.probe_sem)
    with torch.cuda.graph(g):
        body()
    grads = [p.grad for p in params]
    sems, sem_log = [], []
    if a.probe_sem:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(
            __file__))), "lipreading-video-generation_amd"))
        from vdiff.hipgraph import graph_nodes, read_i32
        nodes = graph_nodes(g.raw_cuda_graph())
        sems = [nd for nd in nodes if nd["type"] == "memset"]
        print(json.dumps({"node_types": {t: sum(1 for nd in nodes if nd["type"] == t)
                                          for t in {nd["type"] for nd in nodes}},
                          "memset_nodes": sems}), flush=True)
        g.instantiate()
    bad, bad_grads = [], []
    gen = torch.Generator(device=dev).manual_seed(1)
    for r in range(a.replays):
        with torch.no_grad():
            x.copy_(torch.randn(shape, generator=gen, device=dev) * (1 + r % 7))
            eps.copy_(torch.randn(shape, generator=gen, device=dev))
        g.replay()
        with torch.no_grad():
            ref = F.mse_loss(state["pred"], eps)
        got, want = float(snap), float(ref)
        if sems:
            torch.cuda.synchronize()
            sem_log.append((r, [read_i32(nd["dst"], max(1, nd["bytes"] // 4)) for nd in sems]))
        if got != want:
            bad.append((r, got, want))
        if a.check_grads:
            w = [p.detach().clone().requires_grad_(True) for p in params]
            ge = torch.autograd.grad(F.mse_loss(fwd(*w), eps), w)
            if not all(torch.equal(u, v) for u, v in zip(ge, grads)):
                bad_grads.append(r)
        for _ in range(0 if a.quiet_host else a.host_ops):
            with torch.no_grad():
                kept = [gr.clone() for gr in grads]
                for p, gr in zip(params, grads):
                    p.sub_(1e-3 * gr / a.host_ops)
                _ = [torch.equal(p, k) for p, k in zip(params, kept)]
                _ = [float(k.abs().sum()) for k in kept]
    print(json.dumps({"impl": a.impl, "quiet_host": a.quiet_host, "replays": a.replays,
                      "host_ops": a.host_ops, "mismatches": len(bad), "first": bad[:5],
                      "grad_mismatches": len(bad_grads) if a.check_grads else None,
                      "first_grad_mismatch": bad_grads[:3],
                      "semaphores_around_first_mismatch":
                          [x for x in sem_log if bad and bad[0][0] - 3 <= x[0] <= bad[0][0] + 3]
                          or sem_log[:3],
                      "DEBUG_CLR_GRAPH_PACKET_CAPTURE":
                          os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE")}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
