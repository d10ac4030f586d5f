"""The drop-in flat modules (video-generation/diffusion/{unet,unet_audio,utils,
linear_noise_scheduler,noise_scheduler}.py) expose the reference names, constructor
signatures and state-dict keys; the product path refuses CPU tensors.  CPU only: each
check runs in a subprocess because the flat names (utils, unet) are generic."""
import json
import subprocess
import sys
import textwrap

from conftest import DROPIN, ROOT


def run(code):
    src = textwrap.dedent(code)
    env_code = f"import sys; sys.path.insert(0, {DROPIN!r}); sys.path.insert(1, {ROOT!r})\n" + src
    out = subprocess.run([sys.executable, "-c", env_code], capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    return out.stdout


def test_reference_names_exist():
    out = run("""
        import json, inspect
        import unet, unet_audio, utils, linear_noise_scheduler as lns, noise_scheduler as ns
        names = {
          "unet": [n for n in ("UNetModel", "ResBlock", "AttentionBlock", "QKVAttention",
                   "QKVAttentionLegacy", "Upsample", "Downsample", "TimestepBlock",
                   "TimestepEmbedSequential", "SuperResModel", "Wav2Vec2Encoder") if hasattr(unet, n)],
          "unet_audio": [n for n in ("UNetAudio", "Wav2Vec2Encoder", "AudioFeatureTransformer")
                         if hasattr(unet_audio, n)],
          "utils": [n for n in ("conv_nd", "linear", "avg_pool_nd", "zero_module", "normalization",
                    "timestep_embedding", "checkpoint", "CheckpointFunction", "GroupNorm32",
                    "set_visible_devices", "update_ema", "mean_flat") if hasattr(utils, n)],
          "sched": [n for n in ("LinearNoiseScheduler", "LinearNoiseSchedulerV2") if hasattr(lns, n)]
                   + [n for n in ("CosineNoiseScheduler", "DDIMSampler") if hasattr(ns, n)],
        }
        sig = list(inspect.signature(unet.UNetModel.__init__).parameters)[1:19]
        asig = list(inspect.signature(unet_audio.UNetAudio.__init__).parameters)[1:25]
        print(json.dumps({"names": names, "sig": sig, "asig": asig}))
    """)
    d = json.loads(out.strip().splitlines()[-1])
    assert len(d["names"]["unet"]) == 11
    assert len(d["names"]["unet_audio"]) == 3
    assert len(d["names"]["utils"]) == 12
    assert len(d["names"]["sched"]) == 4
    assert d["sig"] == ["image_size", "in_channels", "model_channels", "out_channels",
                        "num_res_blocks", "attention_resolutions", "dropout", "channel_mult",
                        "conv_resample", "dims", "num_classes", "use_checkpoint", "use_fp16",
                        "num_heads", "num_head_channels", "num_heads_upsample",
                        "use_scale_shift_norm", "resblock_updown"]
    assert d["asig"][:9] == ["image_size", "in_channels", "model_channels", "out_channels",
                             "num_res_blocks", "attention_resolutions", "image_cond",
                             "im_cond_input_ch", "im_cond_output_ch"]
    assert d["asig"][-2:] == ["audio_feature_dim", "projected_audio_dim"]


def test_state_dict_keys_and_schedules_match_oracle():
    out = run("""
        import json, torch
        import unet, linear_noise_scheduler as lns, noise_scheduler as ns
        from oracle.unet import build_plan, param_shapes
        from oracle.fixtures import FULL2D, FULL3D
        from oracle import schedulers as osch
        ok = []
        for cfg in (FULL2D, FULL3D):
            with torch.device("meta"):
                m = unet.UNetModel(image_size=32, **cfg)
            sd = {k: tuple(v.shape) for k, v in m.state_dict().items()}
            ok.append(sd == dict(param_shapes(build_plan(**cfg))))
        s = lns.LinearNoiseScheduler(100, 0.00085, 0.012)
        ok.append(torch.equal(s.alpha_cum_prod, osch.linear_tables(100, 0.00085, 0.012)["acp"]))
        s2 = lns.LinearNoiseSchedulerV2(500, 0.00005, 0.015)
        ok.append(torch.equal(s2.betas, osch.linear_tables(500, 0.00005, 0.015)["betas"]))
        c = ns.CosineNoiseScheduler(2000)
        ok.append(torch.equal(c.alphas_cumprod, osch.cosine_tables(2000)["acp"]))
        d = ns.DDIMSampler(s2, steps=50)
        ok.append(int(d.timesteps[0]) == 499 and int(d.prev_timesteps[-1]) == -1)
        print(json.dumps(ok))
    """)
    assert json.loads(out.strip().splitlines()[-1]) == [True] * 6


def test_product_path_refuses_cpu():
    out = run("""
        import torch, unet
        m = unet.UNetModel(image_size=8, in_channels=3, model_channels=32, out_channels=3,
                           num_res_blocks=1, attention_resolutions=(), channel_mult=(1,))
        try:
            m(torch.zeros(1, 3, 8, 8), torch.tensor([1]))
            print("NO-ERROR")
        except RuntimeError as e:
            print("RAISED", "no CPU fallback" in str(e) or "GPU only" in str(e))
    """)
    assert "RAISED True" in out


def test_train_entry_parses_reference_defaults():
    out = run("""
        import json, train
        a = train.parse([])
        print(json.dumps([a.lr, a.num_timesteps, a.batch_size, a.epochs, a.model_channels,
                          a.channel_mult, a.attention_resolutions, a.dropout]))
    """)
    assert json.loads(out.strip().splitlines()[-1]) == [0.01, 100, 8, 10, 64, [1, 2, 4],
                                                        [1, 2, 4], 0.1]


def test_sampling_entry_reference_signatures():
    """test.py keeps the reference's API: config, load_model_and_scheduler(config) and
    sample_images(model, scheduler, img_cond, audio_cond, n_timesteps=500) (test.py:33-113),
    importable without running the script."""
    out = run("""
        import json, inspect, test
        print(json.dumps({
          "sample": list(inspect.signature(test.sample_images).parameters)[:5],
          "n_default": inspect.signature(test.sample_images).parameters["n_timesteps"].default,
          "load": [p for p, v in inspect.signature(test.load_model_and_scheduler).parameters.items()
                   if v.kind == v.POSITIONAL_OR_KEYWORD],
          "cfg": sorted(test.config), "ldm": test.config["ldm_params"]["model_channels"]}))
    """)
    d = json.loads(out.strip().splitlines()[-1])
    assert d["sample"] == ["model", "scheduler", "img_cond", "audio_cond", "n_timesteps"]
    assert d["n_default"] == 500 and d["load"] == ["config"]
    assert d["cfg"] == ["dataset_params", "ldm_params", "train_params"] and d["ldm"] == 64


def test_vivit_train_entry_one_argument_call():
    """train_huggingface_model(VIVIT) reads the module-level X_train / Y_train_p / X_test /
    Y_test_p as the reference does (huggingface_vivit_model.py:35-41)."""
    import os
    from conftest import PKG
    out = run(f"""
        import inspect, sys
        sys.path.insert(0, {os.path.join(PKG, "lipreading")!r})
        import huggingface_vivit_model as h
        ps = inspect.signature(h.train_huggingface_model).parameters
        print(list(ps)[0], all(ps[n].default is None for n in ("X_train", "Y_train", "X_test", "Y_test")))
        try:
            h.train_huggingface_model(object())
        except NameError as e:
            print("NameError", "X_train" in str(e))
    """)
    assert "VIVIT True" in out and "NameError True" in out
