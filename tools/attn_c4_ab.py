"""Forward attention at the BASELINE config-4 shapes (256x256x25, joint): D=64 N=1638400,
D=128 N=409600, D=256 N=102400; per kernel shape (ops.attention_config), HIP-event timed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
import torch  # noqa: E402

from vdiff import ops  # noqa: E402

shapes = [(128, 409600, ("nb2", "d8n")), (64, 1638400, ("w8", "d8n"))]
for C, N, cfgs in shapes:
    qkv = ops.to_cl(torch.randn(1, 3 * C, N, device="cuda", dtype=torch.bfloat16))
    for rep in range(2):
        for cfg in cfgs:
            with ops.attention_config(cfg), torch.no_grad():
                ops.attention(qkv, 1)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(2):
                    ops.attention(qkv, 1)
                e1.record()
                torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 2
            tf = 4 * N * N * C / (ms / 1e3) / 1e12
            print(f"D={C} N={N} cfg={cfg}: {ms:.2f} ms {tf:.0f} TF/s", flush=True)
