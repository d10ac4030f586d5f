"""Which finalizer aborts a HIP graph capture?

Round 5 saw one `-m gpu` run die with "Fatal Python error: Aborted" while the interpreter was
"Garbage-collecting" inside TrainStepGraph._capture.  torch.cuda.graph does NOT collect before
capture_begin (torch.compiler.config.force_cudagraph_gc is False), so reference cycles left by
earlier tests are collected by whatever allocation crosses the collector's threshold -- inside
the capture, on the capturing thread.  Each case below builds one candidate object that owns a
HIP resource, strands it in an unreachable reference cycle, starts a capture in torch's
thread_local mode (TrainStepGraph's) and runs gc.collect() inside it, in its own child process.

Round 6 result (profiles/r06_capture_probe.jsonl): every case completes except a dead
CUDAGraph in a cycle ("gc_graph"), which aborts: "terminate called after throwing an instance of
'c10::AcceleratorError' what(): HIP error: operation not permitted when stream is capturing ...
Exception raised from ~CUDAGraph at HIPGraph.cpp:324".  The same graph collected by
vdiff.hipgraph.capture before capture_begin ("fixed_graph") completes, and a graph Trainer is
now freed by reference counting ("gc_trainer_graph": TrainStepGraph holds it weakly).

Cases run in order; the probe stops at the first child killed by a signal (nothing more is
started on the GPU after an abort).  The case expected to abort runs last.
    python tools/capture_finalizer_probe.py [--out gpurun_out/capture_probe.jsonl]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = ["record_null_stream", "record_pool_stream", "gc_pinned_unused", "gc_pinned_recorded",
         "gc_event", "gc_thread_pool", "gc_trainer_graph", "fixed_graph", "gc_graph"]


def _cycle(obj):
    box = {"obj": obj}
    box["self"] = box
    return box


def child(case):
    import gc
    import torch
    sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
    sys.path.insert(0, ROOT)
    dev = "cuda"
    x = torch.zeros(1 << 16, device=dev)
    torch.cuda.synchronize()
    res = {"case": case}
    gc.disable()  # the candidate must survive until the collection inside the capture
    if case == "gc_pinned_unused":
        p = torch.empty(1 << 16, pin_memory=True)
        _cycle(p)
        del p
    elif case == "gc_pinned_recorded":
        # what ClipBatcher.next, the SpecAugment mask upload and GradBucketer's flag upload do:
        # a non_blocking copy from pinned host memory records the stream on the host block
        p = torch.ones(1 << 16, pin_memory=True)
        d = p.to(dev, non_blocking=True)
        torch.cuda.synchronize()
        _cycle(p)
        del p, d
    elif case == "gc_event":
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        torch.cuda.synchronize()
        _cycle(e)
        del e
    elif case in ("gc_graph", "fixed_graph"):
        g0 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g0):
            x.add_(1.0)
        g0.replay()
        torch.cuda.synchronize()
        _cycle(g0)
        del g0
    elif case == "gc_thread_pool":
        from concurrent.futures import ThreadPoolExecutor

        class Owner:  # ClipBatcher's shape: a pool, pending pinned batches, a __del__
            def __init__(self):
                self.pool = ThreadPoolExecutor(max_workers=1)
                self.pending = [self.pool.submit(lambda: torch.ones(4096).pin_memory())
                                for _ in range(3)]

            def __del__(self):
                self.pool.shutdown(wait=True)
        o = Owner()
        [f.result() for f in o.pending]
        o.me = o
        del o
    elif case == "gc_trainer_graph":
        os.environ["VDIFF_TRAIN_GRAPH_EXPERIMENTAL"] = "1"
        from oracle.unet import init_params
        from vdiff.engine import Clip, Trainer
        from vdiff.schedulers import LinearNoiseScheduler
        from vdiff.unet_audio import UNetAudio
        m = UNetAudio(image_size=32, in_channels=3, model_channels=32, out_channels=3,
                      num_res_blocks=1, attention_resolutions=(2,), channel_mult=(1, 2), dims=3,
                      audio_feature_dim=64, projected_audio_dim=16, im_cond_output_ch=16,
                      audio_encoder=False)
        m.load_state_dict(init_params({k: tuple(v.shape) for k, v in m.state_dict().items()}, 5))
        m = m.to(dev)
        gen = torch.Generator(device=dev).manual_seed(1)
        x0 = torch.rand((1, 3, 4, 32, 32), generator=gen, device=dev)
        c = Clip(x0, x0[:, :, 0].clone(), torch.randn((4, 64), device=dev), torch.randn_like(x0),
                 torch.tensor([3], device=dev))
        tr = Trainer(m, LinearNoiseScheduler(100, 0.00085, 0.012), lr=1e-3, graph=True)
        for _ in range(4):
            tr.step(c)
        torch.cuda.synchronize()
        import weakref
        ref = weakref.ref(tr)
        del tr, m, c, x0
        res["trainer_freed_by_refcount"] = ref() is None
    g = torch.cuda.CUDAGraph()
    try:
        if case == "fixed_graph":
            from vdiff import hipgraph
            gc.enable()
            with hipgraph.capture(g, capture_error_mode="thread_local"):
                x.add_(1.0)
                res["gc_enabled_inside"] = gc.isenabled()
                res["collected"] = gc.collect()
        else:
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                x.add_(1.0)
                if case == "record_null_stream":
                    try:
                        torch.cuda.Event().record(torch.cuda.default_stream())
                        res["record"] = "ok"
                    except RuntimeError as e:
                        res["record"] = str(e).splitlines()[0]
                elif case == "record_pool_stream":
                    s = torch.cuda.Stream()
                    try:
                        torch.cuda.Event().record(s)
                        res["record"] = "ok"
                    except RuntimeError as e:
                        res["record"] = str(e).splitlines()[0]
                else:
                    res["collected"] = gc.collect()
        res["capture"] = "ok"
        g.replay()
        torch.cuda.synchronize()
        res["replay"] = float(x[0])
    except RuntimeError as e:
        res["capture"] = str(e).splitlines()[0]
    print("RESULT " + json.dumps(res), flush=True)


def main():
    out = None
    if "--out" in sys.argv:
        out = sys.argv[sys.argv.index("--out") + 1]
    rows = []
    for case in CASES:
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", case],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
        row = {"case": case, "returncode": p.returncode}
        for line in p.stdout.splitlines():
            if line.startswith("RESULT "):
                row.update(json.loads(line[7:]))
        err = [s for s in p.stderr.splitlines() if s.strip() and "amdgpu.ids" not in s]
        row["stderr_key"] = [s for s in err if any(k in s for k in (
            "terminate", "what()", "Error", "error", "Exception", "Fatal", "hip", "CUDA"))][:12]
        row["stderr_head"] = err[:8]
        rows.append(row)
        print(json.dumps(row), flush=True)
        if out:
            with open(out, "a") as f:
                f.write(json.dumps(row) + "\n")
        if p.returncode < 0 or p.returncode == 134:
            print(f"case {case} died by signal {-p.returncode}: stopping", flush=True)
            break
    return 0


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        sys.exit(main())
