"""Per-step kernel time by category from a rocprofv3 --kernel-trace database of a bench run:
steps are cut at each q_sample launch (one per train step); prints the categories of the
last steps (the timed ones) in ms per step.   python tools/prof_steps.py run_results.db [cut]
cut: a kernel-name substring that starts each step (default QSample; ddim_kernel for DDIM).
Also prints the per-kernel table (name, launches, ms) of the last step."""
import sqlite3
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def cat(n):
    if n.startswith(("attn_", "vd_attn_")):
        return "attention (vdiff)"
    if n.startswith(("wgrad_dma", "wgrad_strip", "wgrad_finish", "conv_wgrad")):
        return "conv weight gradient (vdiff)"
    if n.startswith("channel_sums"):
        return "conv bias / emb-add gradient (vdiff)"
    if n.startswith(("igemm_dma", "pw_gemm", "igemm_bf16", "conv_gemm", "pack_weight",
                     "halo_conv")):
        return "conv (vdiff)"
    if n.startswith("gn_"):
        return "groupnorm (vdiff)"
    if n.startswith("Cijk"):
        return "rocBLAS / hipBLASLt GEMM"
    if n.startswith("naive_conv"):
        return "MIOpen naive conv"
    low = n.lower()
    if ("miopen" in low or "gtcx" in n or "im2d" in low or "col2im" in low or n.startswith("_ZN2ck")
            or n.startswith("ck::") or "batched_transpose" in n or "subtensor" in low):
        return "MIOpen / CK (wav2vec2 convs)"
    if n.startswith("at::native") or n.startswith("__amd"):
        return "torch elementwise / copies / fills"
    return "other vdiff"


c = sqlite3.connect(sys.argv[1])
ks = [(short(n), s, e) for n, s, e in
      c.execute("select name, start, end from kernels order by start")]
CUT = sys.argv[2] if len(sys.argv) > 2 else "QSample"
cuts = [s for n, s, e in ks if CUT in n]
print(f"{len(cuts)} steps ({CUT} launches)")
for i in range(max(0, len(cuts) - 4), len(cuts)):
    lo, hi = cuts[i], cuts[i + 1] if i + 1 < len(cuts) else float("inf")
    agg, wall0, wall1 = {}, None, None
    for n, s, e in ks:
        if lo <= s < hi:
            agg[cat(n)] = agg.get(cat(n), 0) + (e - s) / 1e6
            wall0 = s if wall0 is None else wall0
            wall1 = e
    tot = sum(agg.values())
    print(f"step {i}: kernels {tot:.1f} ms, first->last {(wall1 - wall0) / 1e6:.1f} ms")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(f"   {k:38s} {v:8.2f}")

# the last complete step's kernels by name
lo, hi = cuts[-2], cuts[-1]
per = {}
for n, s, e in ks:
    if lo <= s < hi:
        r = per.setdefault(n[:90], [0, 0.0])
        r[0] += 1
        r[1] += (e - s) / 1e6
print("last complete step, per kernel (launches, ms):")
for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"   {t:8.3f} ms  x{c:<4d} {n}")

# idle gaps of the last step: the 12 largest, with the kernels on either side
lo = cuts[-1]
last = [(n, s, e) for n, s, e in ks if s >= lo]
gaps = []
end = None
for i, (n, s, e) in enumerate(last):
    if end is not None and s > end:
        gaps.append(((s - end) / 1e3, last[i - 1][0][:50], n[:50], i))
    end = e if end is None else max(end, e)
tot = sum(g[0] for g in gaps)
print(f"last step: {len(gaps)} gaps, {tot / 1e3:.2f} ms idle in all; largest:")
for g in sorted(gaps, reverse=True)[:12]:
    print(f"   {g[0]:8.1f} us  after {g[1]:50s} before {g[2]:50s} (#{g[3]})")
# where the idle time sits: per 100-kernel window of the last step, idle ms and the most
# frequent kernel name in the window
print("idle by position (kernel index window, idle ms, busy ms, typical kernel):")
for w0 in range(0, len(last), 100):
    idle = sum(g[0] for g in gaps if w0 <= g[3] < w0 + 100) / 1e3
    busy = sum((e - s) for n, s, e in last[w0:w0 + 100]) / 1e6
    names = {}
    for n, s, e in last[w0:w0 + 100]:
        names[n[:40]] = names.get(n[:40], 0) + 1
    top = max(names.items(), key=lambda kv: kv[1])[0]
    print(f"   {w0:5d}  idle {idle:6.2f}  busy {busy:7.2f}  {top}")
