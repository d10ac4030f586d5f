"""Trainer(graph=True): the denoiser's forward + backward replayed as one HIP graph
(vdiff.engine.TrainStepGraph) against the eager step, and the
GroupNorm dropout step counter the replays advance (vd_set_dropout_counter)."""
import copy

import pytest
import torch

from oracle.fixtures import rel_l2

pytestmark = pytest.mark.gpu
dev = "cuda"

GOLDEN = 0x9E3779B97F4A7C15


@pytest.fixture(autouse=True)
def _experimental(monkeypatch):
    """Trainer(graph=True) is gated behind VDIFF_TRAIN_GRAPH_EXPERIMENTAL (advisor r03)."""
    monkeypatch.setenv("VDIFF_TRAIN_GRAPH_EXPERIMENTAL", "1")


def _tiny_w2v(hidden=64):
    """A one-layer wav2vec2 with every stochastic part off (dropouts, LayerDrop, SpecAugment),
    so the eager and the graph runs see the same encoder computation."""
    from transformers import Wav2Vec2Config, Wav2Vec2Model
    from vdiff.unet_audio import Wav2Vec2Encoder, _patch_wav2vec2
    cfg = Wav2Vec2Config(num_hidden_layers=1, hidden_size=hidden, intermediate_size=128,
                         num_attention_heads=4, conv_dim=(64,) * 7, hidden_dropout=0.0,
                         attention_dropout=0.0, activation_dropout=0.0, feat_proj_dropout=0.0,
                         final_dropout=0.0, layerdrop=0.0, mask_time_prob=0.0,
                         mask_feature_prob=0.0)
    torch.manual_seed(11)
    w = Wav2Vec2Model(cfg)
    _patch_wav2vec2(w)
    enc = Wav2Vec2Encoder.__new__(Wav2Vec2Encoder)
    torch.nn.Module.__init__(enc)
    enc.wav2vec2 = w
    return enc


def _model(dropout=0.0, audio=False, bf16=False):
    from oracle.unet import init_params
    from vdiff.unet_audio import UNetAudio
    m = UNetAudio(image_size=32, in_channels=3, model_channels=32, out_channels=3,
                  num_res_blocks=1, attention_resolutions=(2,), channel_mult=(1, 2), dims=3,
                  audio_feature_dim=64, projected_audio_dim=16, im_cond_output_ch=16,
                  dropout=dropout, audio_encoder=False)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    m.load_state_dict(init_params(shapes, 5))
    if audio:
        m.audio_encoder = _tiny_w2v()
    if bf16:
        m.convert_to_fp16()
    return m.to(dev)


def _clip(s, audio, frames=4):
    from vdiff.engine import Clip
    gen = torch.Generator(device=dev).manual_seed(100 + s)
    x0 = torch.rand((1, 3, frames, 32, 32), generator=gen, device=dev) * 2 - 1
    cond = torch.rand((1, 3, 32, 32), generator=gen, device=dev) * 2 - 1
    a = ({"input_values": torch.randn((frames, 4000), generator=gen, device=dev)} if audio
         else torch.randn((frames, 64), generator=gen, device=dev))
    eps = torch.randn(x0.shape, generator=gen, device=dev)
    return Clip(x0, cond, a, eps, torch.tensor([3 + 7 * s], device=dev))


def _run(m, graph, steps, audio, lr=1e-3):
    from vdiff.engine import Trainer
    from vdiff.schedulers import LinearNoiseScheduler
    tr = Trainer(m, LinearNoiseScheduler(100, 0.00085, 0.012), lr=lr, graph=graph)
    losses = torch.stack([tr.step(_clip(s, audio)) for s in range(steps)])
    return tr, losses


def _close_to_eager(ref, again, got, tol):
    """got (graph run) vs ref (eager run) per tensor, with the eager run's own repeat `again`
    as the noise floor: the split-K weight-gradient atomics reorder fp32 sums, and Adam's
    g / (|g| + eps) turns rounding noise into full +-lr steps where a gradient is zero in exact
    arithmetic (e.g. the bias of a conv whose output is GroupNorm-ed with one channel per
    group), so such tensors drift apart between any two runs."""
    bad = []
    for n, a, a2, b in zip(ref[0], ref[1], again[1], got[1]):
        d, floor = rel_l2(b, a), rel_l2(a2, a)
        if d > tol and d > 4 * floor + tol:
            bad.append((n, d, floor))
    return bad


def _params(m):
    return ([n for n, _ in m.named_parameters()], [p.detach().clone() for p in m.parameters()])


@pytest.mark.parametrize("audio,bf16", [(False, False), (True, False), (False, True)])
def test_graph_step_equals_eager(audio, bf16):
    """Six steps (two eager warm-up steps, the capture, four replays) track the eager
    Trainer: the losses (fp32 1e-5 / bf16 1e-4) and every parameter after the last Adam step,
    against the eager run's own run-to-run spread (_close_to_eager).  With a trainable (tiny,
    deterministic) wav2vec2 the encoder's backward is fed the replayed feature gradient."""
    m = _model(audio=audio, bf16=bf16)
    runs = []
    for graph in (False, False, True):
        mm = copy.deepcopy(m)
        tr, losses = _run(mm, graph, 6, audio)
        runs.append((losses, _params(mm)))
    assert tr.graph.g is not None and tr.graph.steps == 6
    tol = 1e-4 if bf16 else 1e-5
    assert rel_l2(runs[2][0], runs[0][0]) < tol, (runs[2][0], runs[0][0])
    bad = _close_to_eager(runs[0][1], runs[1][1], runs[2][1], tol)
    assert not bad, bad
    if audio:  # the encoder trained in both runs
        w0 = dict(m.named_parameters())
        moved = [n for n, p in zip(*runs[2][1])
                 if n.startswith("audio_encoder.") and not torch.equal(p, w0[n])]
        assert len(moved) > 5


def test_graph_gradients_equal_eager():
    """At lr 0 (the weights never move) the gradients a replay leaves in .grad equal the
    eager step's on the same clip, every parameter with a gradient above the rounding level
    (fp32, 1e-4 relative)."""
    from vdiff.engine import Trainer
    from vdiff.schedulers import LinearNoiseScheduler
    m = _model(audio=True)
    c = _clip(0, True)
    me, mg = copy.deepcopy(m), copy.deepcopy(m)
    eager = {}
    hooks = [p.register_post_accumulate_grad_hook(
        lambda p, n=n: eager.__setitem__(n, p.grad.detach().clone()))
        for n, p in me.named_parameters()]
    Trainer(me, LinearNoiseScheduler(100, 0.00085, 0.012), lr=0.0).step(c)
    for h in hooks:
        h.remove()
    tr = Trainer(mg, LinearNoiseScheduler(100, 0.00085, 0.012), lr=0.0, graph=True)
    for _ in range(4):
        tr.step(c)
    assert tr.graph.g is not None
    # the encoder's gradients are released after Adam; the denoiser's stay in the graph pool
    got = {n: p.grad for n, p in mg.named_parameters() if p.grad is not None}
    assert len(got) >= len(eager) - sum(n.startswith("audio_encoder.") for n in eager)
    top = max(float(g.norm()) for g in eager.values())
    for n, g in got.items():
        if float(eager[n].norm()) > 1e-5 * top:
            assert rel_l2(g, eager[n]) < 1e-4, n


def test_graph_step_other_shape_runs_eager():
    """A batch of another shape after the capture (a short last batch) runs eagerly and the
    replays after it still train every parameter: the sequence 4-frame x4, 2-frame, 4-frame x2
    tracks the eager Trainer (fp32, 1e-5 against the eager run-to-run spread)."""
    from vdiff.engine import Trainer
    from vdiff.schedulers import LinearNoiseScheduler
    m = _model()
    seq = [(0, 4), (1, 4), (2, 4), (3, 4), (4, 2), (5, 4), (6, 4)]
    out = []
    for graph in (False, False, True):
        mm = copy.deepcopy(m)
        tr = Trainer(mm, LinearNoiseScheduler(100, 0.00085, 0.012), lr=1e-3, graph=graph)
        losses = torch.stack([tr.step(_clip(s, False, f)) for s, f in seq])
        out.append((losses, _params(mm)))
    assert rel_l2(out[2][0], out[0][0]) < 1e-5
    bad = _close_to_eager(out[0][1], out[1][1], out[2][1], 1e-5)
    assert not bad, bad


def test_graph_replays_draw_new_dropout_masks():
    """ResBlock dropout (0.1) in the graph: at lr 0 the same clip replayed twice gives two
    different losses (a frozen seed would repeat the mask), while without dropout the two
    replays agree."""
    for dropout, differ in ((0.1, True), (0.0, False)):
        from vdiff.engine import Trainer
        from vdiff.schedulers import LinearNoiseScheduler
        tr = Trainer(_model(dropout=dropout), LinearNoiseScheduler(100, 0.00085, 0.012), lr=0.0,
                     graph=True)
        c = _clip(0, False)
        losses = [float(tr.step(c)) for _ in range(5)]
        d = abs(losses[4] - losses[3])
        if differ:
            assert d > 1e-6 * abs(losses[3]), losses
        else:
            assert d < 1e-5 * abs(losses[3]), losses


def test_dropout_counter_mixes_into_seed():
    """vd_set_dropout_counter: a GroupNorm+SiLU+dropout launch that reads counter value k
    equals the launch with seed ^ ((k + 1) * 0x9E3779B97F4A7C15) and no counter, forward and
    backward."""
    from vdiff import _lib, ops
    lib = _lib.lib()
    torch.manual_seed(3)
    x = ops.to_cl(torch.randn(1, 64, 4, 8, 8, device=dev).bfloat16())
    g = torch.randn(64, device=dev, requires_grad=True)
    b = torch.randn(64, device=dev, requires_grad=True)
    dy = torch.randn(x.shape, device=dev).bfloat16()

    def run(seed, ctr=None):
        xx = x.detach().clone().requires_grad_(True)
        lib.vd_set_dropout_counter(ctr.data_ptr() if ctr is not None else None)
        try:
            y = ops.group_norm_silu(xx, g, b, 32, 1e-5, True, dropout=0.1, seed=seed)
            dx, = torch.autograd.grad(y, xx, ops.to_cl(dy))
        finally:
            lib.vd_set_dropout_counter(None)
        return y.detach(), dx

    ctr = torch.full((), 5, dtype=torch.int64, device=dev)
    y1, d1 = run(123, ctr)
    y2, d2 = run(123 ^ ((6 * GOLDEN) % 2 ** 64))
    y0, _ = run(123)
    assert torch.equal(y1, y2) and torch.equal(d1, d2)
    assert not torch.equal(y1, y0)


# ------------------------------------------------------------------ config-2 scale (round 4)
def _bench_unet(size, dropout):
    """The bench model (config 2 topology, bf16, joint attention) without the wav2vec2
    encoder: pooled audio features in, so both trainers see identical inputs."""
    from vdiff.engine import reinit_nonzero
    from vdiff.unet_audio import UNetAudio
    torch.manual_seed(1234)
    m = UNetAudio(image_size=size, in_channels=3, model_channels=64, out_channels=3,
                  num_res_blocks=2, attention_resolutions=(1, 2, 4), channel_mult=(1, 2, 4),
                  audio_feature_dim=768, projected_audio_dim=128, dims=3, use_bf16=True,
                  audio_encoder=False, dropout=dropout)
    reinit_nonzero(m, seed=1234)
    return m.to(dev)


def _bench_clip(size, frames=16):
    from vdiff.engine import Clip
    g = torch.Generator(device=dev).manual_seed(0)
    return Clip(torch.rand((1, 3, frames, size, size), generator=g, device=dev) * 2 - 1,
                torch.rand((1, 3, size, size), generator=g, device=dev) * 2 - 1,
                torch.randn((frames, 768), generator=g, device=dev),
                torch.randn((1, 3, frames, size, size), generator=g, device=dev),
                torch.tensor([37], device=dev))


def test_graph_config2_lr0_replays_equal_eager():
    """VERDICT r03 item 3 at the config-2 shape (128x128x16, bf16, joint attention): two
    eager warm-up steps, the capture, three replays.  With every reduction fixed-order the
    replayed step equals the eager step bit for bit -- the loss and every gradient -- and the
    loss is a finite, non-negative mean of squares."""
    from vdiff.engine import Trainer
    from vdiff.schedulers import LinearNoiseScheduler
    m = _bench_unet(128, 0.0)
    models = {"eager": m, "graph": copy.deepcopy(m)}
    sched = LinearNoiseScheduler(100, 0.00085, 0.012)
    trs = {k: Trainer(v, sched, lr=0.0, graph=(k == "graph")) for k, v in models.items()}
    clip = _bench_clip(128)
    for step in range(5):
        ge = {}
        hooks = [p.register_post_accumulate_grad_hook(
            lambda p, n=n: ge.__setitem__(n, p.grad.detach().clone()))
            for n, p in models["eager"].named_parameters()]
        le = trs["eager"].step(clip)
        for h in hooks:
            h.remove()
        lg = trs["graph"].step(clip)
        torch.cuda.synchronize()
        assert torch.isfinite(lg) and float(lg) >= 0.0, (step, float(lg))
        assert torch.equal(le, lg), (step, float(le), float(lg))
        if trs["graph"].graph.g is not None:
            for n, p in models["graph"].named_parameters():
                assert torch.equal(p.grad, ge[n]), (step, n)
    assert trs["graph"].graph.steps == 5 and trs["graph"].graph.g is not None


def test_graph_loss_with_moving_weights_and_host_reductions():
    """The round-4 reproducer of the wrong replay losses: 64x64x16, lr 1e-2 (the weights
    move), an eager twin stepped alternately, and torch.equal over every parameter pair plus
    clones and sums of every gradient after each step (host-side GPU work between the
    replays).  Round 4 saw -0.855 and -0.707 (bf16-exact garbage) at steps 4-5 from torch's
    in-graph mean while every weight and gradient stayed bit-identical; round 5 traced it to
    that reduction under HIP's graph packet capture and replaced it with
    vd_mse_loss.  The value returned is the graph's OWN captured loss, and it must equal the
    eager twin's bit for bit at every one of 12 steps; the captured graph holds no memset
    node."""
    from vdiff.engine import Trainer
    from vdiff.schedulers import LinearNoiseScheduler
    m = _bench_unet(64, 0.0)
    twin = copy.deepcopy(m)
    sched = LinearNoiseScheduler(100, 0.00085, 0.012)
    tg = Trainer(m, sched, lr=1e-2, graph=True)
    te = Trainer(twin, sched, lr=1e-2)
    clip = _bench_clip(64)
    for step in range(12):
        le = float(te.step(clip))
        lg = float(tg.step(clip))
        assert lg >= 0.0 and lg == le, (step, le, lg)
        assert all(torch.equal(a, b) for a, b in zip(twin.parameters(), m.parameters())), step
        kept = [p.grad.clone() for p in m.parameters() if p.grad is not None]
        assert all(torch.isfinite(k.abs().sum()) for k in kept)
    types = tg.graph.node_types()
    assert types.get("memset", 0) == 0 and types.get("kernel", 0) > 100, types


def test_graph_step_holds_no_memset_nodes():
    """The captured train step (tiny model, trainable wav2vec2 fed by the replayed feature
    gradient) contains no memset node, whose replay under HIP's graph
    packet capture is where torch's in-graph reduction went stale -- and
    its in-graph loss equals the eager step's over five replays at lr 0."""
    from vdiff.engine import Trainer
    from vdiff.schedulers import LinearNoiseScheduler
    m = _model(audio=True)
    me = copy.deepcopy(m)
    sched = LinearNoiseScheduler(100, 0.00085, 0.012)
    tg = Trainer(m, sched, lr=0.0, graph=True)
    te = Trainer(me, sched, lr=0.0)
    c = _clip(0, True)
    for _ in range(7):
        assert torch.equal(tg.step(c), te.step(c))
    types = tg.graph.node_types()
    assert types.get("memset", 0) == 0 and types["kernel"] > 20, types


def test_graph_config2_dropout_replays():
    """Config-2 shape with the ResBlock dropout at 0.1 and lr 0: three replays draw fresh
    masks through the device step counter (so they are not comparable to the eager steps,
    whose masks come from host seeds); each replayed loss is finite, non-negative, differs
    from the previous replay's, and stays within the spread of eager dropout steps."""
    from vdiff.engine import Trainer
    from vdiff.schedulers import LinearNoiseScheduler
    m = _bench_unet(128, 0.1)
    twin = copy.deepcopy(m)
    sched = LinearNoiseScheduler(100, 0.00085, 0.012)
    tg = Trainer(m, sched, lr=0.0, graph=True)
    te = Trainer(twin, sched, lr=0.0)
    clip = _bench_clip(128)
    eager = [float(te.step(clip)) for _ in range(5)]
    graph = [float(tg.step(clip)) for _ in range(5)]
    assert tg.graph.g is not None
    lo, hi = min(eager), max(eager)
    for i, v in enumerate(graph):
        assert v == v and v >= 0.0, (i, v)
        assert 0.5 * lo <= v <= 2.0 * hi, (i, v, eager)
    assert len(set(graph[2:])) == 3, graph


def test_capture_runs_without_garbage_collection():
    """vdiff.hipgraph.capture keeps Python's collector off while the capture runs (a
    collection inside a capture runs finalizers on the capturing thread) and restores it."""
    import gc
    from vdiff import hipgraph
    x = torch.zeros(1024, device="cuda")
    seen = []
    g = torch.cuda.CUDAGraph()
    assert gc.isenabled()
    with hipgraph.capture(g):
        seen.append(gc.isenabled())
        x.add_(1.0)
    assert seen == [False] and gc.isenabled()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == 2.0


def test_capture_completes_with_a_dead_graph_in_a_cycle():
    """the object behind the round-5 abort -- a captured, replayed
    torch.cuda.CUDAGraph stranded in an unreachable reference cycle (as the Trainer <->
    TrainStepGraph cycle of an earlier test held one).  Destroyed by the cyclic collector inside
    a capture, ~CUDAGraph's device synchronisation (HIPGraph.cpp:324, ROCm builds) returns
    hipErrorStreamCaptureUnsupported, AT_CUDA_CHECK throws in a destructor and std::terminate
    aborts (tools/capture_finalizer_probe.py, profiles/r06_capture_probe.jsonl).
    hipgraph.capture collects it before capture_begin and keeps the collector off while
    allocation-heavy host code runs inside."""
    import gc
    import weakref
    from vdiff import hipgraph

    class Holder:
        pass
    x = torch.zeros(1024, device=dev)
    h = Holder()
    h.me = h
    h.graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(h.graph):
        x.add_(1.0)
    h.graph.replay()
    torch.cuda.synchronize()
    ref = weakref.ref(h)
    del h
    assert ref() is not None and gc.isenabled()
    g = torch.cuda.CUDAGraph()
    seen = []
    with hipgraph.capture(g, capture_error_mode="thread_local"):
        seen.append(ref() is None)
        junk = [[i] for i in range(100000)]  # container allocations past gc thresholds
        x.add_(1.0)
    del junk
    g.replay()
    torch.cuda.synchronize()
    assert seen == [True] and float(x[0]) == 2.0


def test_dropped_graph_trainer_is_freed_without_the_collector():
    """Trainer <-> TrainStepGraph hold each other weakly in one direction, so a dropped
    graph trainer (its captured graph, memory pool and static buffers) is released at once by
    reference counting, never by a collection that could fall inside a later capture."""
    import gc
    import weakref
    from vdiff.engine import Trainer
    from vdiff.schedulers import LinearNoiseScheduler
    m = _model()
    tr = Trainer(m, LinearNoiseScheduler(100, 0.00085, 0.012), lr=1e-3, graph=True)
    c = _clip(0, False)
    for _ in range(3):
        tr.step(c)
    assert tr.graph.g is not None
    refs = [weakref.ref(tr), weakref.ref(tr.graph), weakref.ref(tr.graph.g)]
    gc.disable()
    try:
        del tr
        assert all(r() is None for r in refs)
    finally:
        gc.enable()
