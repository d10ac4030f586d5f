"""Reduce the rocprofv3 PMC passes of tools/pmc_attn.sh to per-kernel averages.

  python tools/pmc_traffic.py gpurun_out/pmc profiles/pmc_traffic.json profiles/r01_pmc_attn.md

HBM bytes follow MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE / WRITE_SIZE are the L2
memory-side request counters, reported in KiB; on gfx950 FETCH_SIZE tallies half the bytes
of 16-B-per-lane streaming reads, WRITE_SIZE is exact for 16-B stores.  Rather than trust
the factor blindly, the run includes a calibration launch (tools/attn_bench.py --calib:
q_sample over 2 x 256 MiB bf16 reads + 256 MiB write) and the read / write scale factors are
taken from it; both are written next to the per-kernel numbers.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

CALIB_ELEMS = 1 << 27
CALIB_READ = 2 * CALIB_ELEMS * 2
CALIB_WRITE = CALIB_ELEMS * 2

_ATTN = re.compile(r"(attn_\w+?)_kernel<(?:[^,<>]+,\s*)?(\d+)")
_VARIANT = re.compile(r"_(pipe|defer|pair)$")  # kernel variants share the launch's key
_ASM = re.compile(r"^vd_(attn_\w+)_d(\d+)$")   # hand-scheduled kernels (asm/gen_attn_asm.py)


_SHORT = re.compile(r"short_attn_(fwd|bwd)_kernel<(\d+)")  # attn_short.hip (temporal mode)


def kernel_key(name: str) -> str:
    m = _SHORT.search(name)
    if m:
        return f"short_attn_{m.group(1)}_d{m.group(2)}"
    m = _ASM.match(name)
    if m:
        return f"{m.group(1)}_d{m.group(2)}"
    m = _ATTN.search(name)
    if m:
        return f"{_VARIANT.sub('', m.group(1))}_d{m.group(2)}"
    if "QSample" in name:
        return "calib_q_sample"
    base = re.sub(r"^void\s+", "", name).split("(")[0]
    return base.split("<")[0][:60]


def load(d: str):
    """-> {kernel_key: {counter: [per-dispatch values]}}"""
    per = defaultdict(lambda: defaultdict(float))  # (key, dispatch) -> counter -> value
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = (kernel_key(row["Kernel_Name"]), row["Dispatch_Id"])
                per[k][row["Counter_Name"]] += float(row["Counter_Value"])
    out = defaultdict(lambda: defaultdict(list))
    for (key, _), ctrs in per.items():
        for c, v in ctrs.items():
            out[key][c].append(v)
    return out


def main(src, js, md):
    tab = defaultdict(dict)
    for d in sorted(glob.glob(os.path.join(src, "p*"))):
        if not os.path.isdir(d):
            continue
        for key, ctrs in load(d).items():
            for c, vals in ctrs.items():
                tab[key][c] = sum(vals) / len(vals)
    cal = tab.get("calib_q_sample", {})
    rf = CALIB_READ / (cal["FETCH_SIZE"] * 1024) if cal.get("FETCH_SIZE") else 2.0
    wf = CALIB_WRITE / (cal["WRITE_SIZE"] * 1024) if cal.get("WRITE_SIZE") else 1.0
    res = {"_calibration": {"read_factor": round(rf, 4), "write_factor": round(wf, 4),
                            "source": "q_sample, 2x256 MiB bf16 read + 256 MiB write"}}
    for key, c in sorted(tab.items()):
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rd = c["FETCH_SIZE"] * 1024 * rf
            wr = c["WRITE_SIZE"] * 1024 * wf
            res[key] = {"hbm_read_bytes": int(rd), "hbm_write_bytes": int(wr),
                        "hbm_bytes_per_launch": int(rd + wr)}
    with open(js, "w") as f:
        json.dump(res, f, indent=1)
    cols = sorted({c for v in tab.values() for c in v})
    lines = ["# PMC counters per launch (rocprofv3 --pmc, one group per pass)", "",
             f"read factor {rf:.3f}, write factor {wf:.3f} (calibration launch)", "",
             "| kernel | " + " | ".join(cols) + " |", "|---" * (len(cols) + 1) + "|"]
    for key, c in sorted(tab.items()):
        lines.append(f"| {key} | " + " | ".join(f"{c[x]:.4g}" if x in c else "" for x in cols)
                     + " |")
    with open(md, "w") as f:
        f.write("\n".join(lines) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
