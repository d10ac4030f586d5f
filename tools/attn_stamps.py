"""Per-tile cycle breakdown of the forward attention loop from s_memtime stamps.

  tools/build_variant.sh stamps -DVD_ATTN_STAMPS
  VDIFF_LIB=lipreading-video-generation_amd/vdiff/libvdiff_stamps.so VDIFF_ATTN_CFG=w8 \\
      python tools/attn_stamps.py [head_dim] [seq_len]

Stamps (lane 0 of each wave, workgroups 0..63, tiles 0..63): 0 = before the ring's
vmcnt + barrier, 1 = after it, 2 = after S' MFMA + softmax VALU (before the rare-path
branch), 3 = after the PV products are issued.  Prints medians over workgroups / tiles
8..63 per wave: barrier wait (1-0), S+softmax (2-1), PV issue (3-2), tile period."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
import torch  # noqa: E402

from vdiff import _lib, ops  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 64
N = int(sys.argv[2]) if len(sys.argv) > 2 else 262144
qkv = ops.to_cl(torch.randn(1, 3 * D, N, device="cuda", dtype=torch.bfloat16))
for _ in range(3):
    ops.attention(qkv, 1)
torch.cuda.synchronize()
buf = np.zeros((64, 8, 4, 64), dtype=np.uint64)
lib = _lib.lib()
lib.vd_debug_attn_stamps.argtypes = [C.c_void_p, C.c_size_t]
assert lib.vd_debug_attn_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.astype(np.int64)
for w in range(8):
    s = st[:, w, :, 8:64]
    if not s.any():
        continue
    wait = np.median(s[:, 1] - s[:, 0])
    sv = np.median(s[:, 2] - s[:, 1])
    pv = np.median(s[:, 3] - s[:, 2])
    per = np.median(np.diff(s[:, 0], axis=1))
    print(f"wave {w}: barrier wait {wait:7.0f}  S+softmax {sv:7.0f}  PV issue {pv:7.0f}  "
          f"tile period {per:7.0f} cycles")
