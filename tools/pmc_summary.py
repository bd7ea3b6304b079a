"""Summarise rocprofv3 --pmc CSVs: per-counter mean per dispatch for the kernels matching a regex,
optionally per kernel, with derived ratios (MFMA busy share, clock).

  python tools/pmc_summary.py [--by-kernel] <regex> <root> [--json out.json]

Units (MI355X_MICROARCH.md 'Per-instruction cycle constants'): SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* / SQ_BUSY_CYCLES count quad-cycles summed over waves / SEs;
SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs; GRBM_GUI_ACTIVE sums the 8 XCDs."""
import argparse
import csv
import glob
import json
import re
from collections import defaultdict

SIMDS = 256 * 4


def collect(root, regex, by_kernel):
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if not regex.search(name):
                    continue
                short = name.replace("(anonymous namespace)::", "").replace("void ", "")
                key = re.sub(r"\(.*", "", short) if by_kernel else "all"
                vals[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def derive(c):
    d = {}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c and c["GRBM_GUI_ACTIVE"] > 0:
        # per-XCD active cycles = GRBM_GUI_ACTIVE / 8; MFMA-busy share of SIMD cycles over the kernel
        d["mfma_busy_frac_of_simd_cycles"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * c["GRBM_GUI_ACTIVE"] / 8)
    if "SQ_WAVE_CYCLES" in c:
        w = c["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in c and w:
                d[k.lower() + "_frac_of_wave_cycles"] = c[k] / w
    if "SQ_INSTS_MFMA" in c and c["SQ_INSTS_MFMA"]:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            if k in c:
                d[k.lower() + "_per_mfma"] = c[k] / c["SQ_INSTS_MFMA"]
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--by-kernel", action="store_true")
    ap.add_argument("regex", nargs="?", default="fwd_f16")
    ap.add_argument("root", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--json")
    a = ap.parse_args()
    vals = collect(a.root, re.compile(a.regex), a.by_kernel)
    out = {}
    for key, cs in vals.items():
        means = {k: sum(v) / len(v) for k, v in cs.items()}
        out[key] = {"mean_per_dispatch": means, "dispatches": {k: len(v) for k, v in cs.items()},
                    "derived": derive(means)}
        print(key)
        for k in sorted(means):
            print(f"  {k:32s} n={len(cs[k]):3d} mean={means[k]:.6g}")
        for k, v in out[key]["derived"].items():
            print(f"  {k:40s} {v:.4f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
