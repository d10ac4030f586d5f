"""The batched weight pack of the bench's train step: the plan's jobs (count, elements, LDS
tiles by layout and tap count) and the launch's time alone (HIP events, 20 launches)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lipreading-video-generation_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import bench
    from vdiff import _lib
    from vdiff.engine import Trainer, synthetic_clip
    from vdiff.schedulers import LinearNoiseScheduler
    args = bench.parse()
    dev = torch.device("cuda", 0)
    m = bench.build_model(args, dev)
    tr = Trainer(m, LinearNoiseScheduler(100, 0.00085, 0.012), lr=1e-3)
    clip = synthetic_clip(1, 16, 128, 100, dev)
    tr.step(clip)
    tr.step(clip)
    desc = np.dtype([("w", "<u8"), ("out", "<u8"), ("Co", "<i4"), ("Ci", "<i4"), ("taps", "<i4"),
                     ("Cip", "<i4"), ("Cop", "<i4"), ("tr", "<i4"), ("start", "<i8")])
    for dt, table, n, total in tr.packs.plans:
        rows = table.cpu().numpy().view(desc)
        tiles = {}
        for r in rows:
            key = ("tr" if r["tr"] else "fwd", int(r["taps"]))
            t = ((r["Cip"] + 7) // 8) * ((r["Cop"] + 63) // 64) if r["tr"] else \
                ((r["Co"] + 3) // 4) * ((r["Cip"] + 63) // 64)
            tiles[key] = tiles.get(key, 0) + int(t)
        print(f"dtype {dt}: {n} jobs, {total / 1e6:.2f} M elements, tiles {tiles}", flush=True)
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(3):
            _lib.call("vd_conv_pack_weights", table.data_ptr(), n, total, _lib.VD_BF16, st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            _lib.call("vd_conv_pack_weights", table.data_ptr(), n, total, _lib.VD_BF16, st)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        w_bytes = sum(int(r["Co"]) * int(r["Ci"]) * int(r["taps"]) * 4 for r in rows)
        print(f"  {us:.1f} us per launch; fp32 reads {w_bytes / 1e6:.1f} MB, bf16 writes "
              f"{total * 2 / 1e6:.1f} MB: {(w_bytes + 2 * total) / us / 1e6:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
