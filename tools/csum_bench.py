"""Per-(sample, channel) sums of the conv bias / emb-add gradients (vd_channel_sums) at the
config-2 train step's dY shapes, bf16, GPU time of back-to-back C-ABI calls (HIP events);
checked against torch's fp32 sum.   [VDIFF_CSUM_BLOCKS=n VDIFF_CSUM_UNROLL=u] python tools/csum_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))

import torch  # noqa: E402

from vdiff import _lib, ops  # noqa: E402

# (channels, pixels, calls per train step)
SHAPES = ((64, 262144, 14), (128, 262144, 6), (192, 262144, 5), (128, 65536, 12),
          (256, 65536, 12), (384, 65536, 5), (256, 16384, 14), (512, 16384, 4),
          (768, 16384, 6), (8, 262144, 1))


def main():
    tot = 0.0
    for C, S, per in SHAPES:
        x = torch.randn(1, S, C, device="cuda").bfloat16()
        out = torch.empty(1, C, device="cuda")
        ws = torch.empty(_lib.lib().vd_channel_sums_workspace_size(1, C), dtype=torch.uint8,
                         device="cuda")
        st = torch.cuda.current_stream().cuda_stream

        def run():
            _lib.call("vd_channel_sums", x.data_ptr(), 1, S, C, 0, ops._DT[torch.bfloat16],
                      out.data_ptr(), ws.data_ptr(), st)
        run()
        torch.cuda.synchronize()
        ref = x.float().sum(1)
        err = float((out - ref).norm() / ref.norm())
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1e3
        tot += us * per
        print(f"channel_sums C={C:4d} S={S:7d}: {us:6.1f} us ({S * C * 2 / us / 1e3:6.0f} GB/s)  "
              f"rel-L2 {err:.1e}", flush=True)
        assert err < 1e-5
    print(f"per train step (shape counts estimated): {tot / 1e3:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
