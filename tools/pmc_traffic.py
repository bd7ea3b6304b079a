"""HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes -> profiles/traffic_<cfg>.json.

Usage: python tools/pmc_traffic.py <cfg> <kernel-regex> <pmc-root> [--out profiles/traffic_<cfg>.json]

Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): both counters are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of 16-B/lane coalesced streaming
reads (all of this repo's global loads on the hot kernels are 16 B/lane), so it
is doubled; WRITE_SIZE is exact for 16-B stores and for float atomics.  The
kernels' 2/4-B epilogue stores are uncalibrated: compare `write_bytes` with the
algorithmic write bytes printed alongside."""
import argparse
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def counter_values(root, regex):
    vals = {}
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if regex.search(name):
                    vals.setdefault(row["Counter_Name"], {}).setdefault(name, []).append(float(row["Counter_Value"]))
    return vals


def counter_means(root, regex):
    """Per counter: the sum over matching kernels of each kernel's mean per dispatch (a step that
    launches several kernels, e.g. forward + backward, is priced as one step), and the dispatches."""
    return {c: (sum(sum(v) / len(v) for v in per.values()), sum(len(v) for v in per.values()))
            for c, per in counter_values(root, regex).items()}


def per_kernel(root, regex):
    """Corrected read / write bytes per launch of each matching kernel (where a step's traffic goes)."""
    vals = counter_values(root, regex)
    out = {}
    for c, scale, key in (("FETCH_SIZE", 2048, "read_bytes"), ("WRITE_SIZE", 1024, "write_bytes")):
        for name, v in vals.get(c, {}).items():
            out.setdefault(name, {})[key] = sum(v) / len(v) * scale
    return out


def algorithmic_bytes(cfg_key):
    import numpy as np
    import bench
    cfg = bench.CONFIGS[cfg_key]
    return bench.algorithmic_bytes(cfg, int(np.prod(cfg[3])))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg")
    ap.add_argument("regex")
    ap.add_argument("root")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    m = counter_means(a.root, re.compile(a.regex))
    if "FETCH_SIZE" not in m or "WRITE_SIZE" not in m:
        sys.exit(f"missing counters under {a.root}: {sorted(m)}")
    fetch_kib, n_f = m["FETCH_SIZE"]
    write_kib, n_w = m["WRITE_SIZE"]
    read_b = fetch_kib * 1024 * 2
    write_b = write_kib * 1024
    alg_r, alg_w = algorithmic_bytes(a.cfg)
    out = {
        "config": a.cfg, "kernel_regex": a.regex, "dispatches": [n_f, n_w],
        "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib,
        "read_bytes": read_b, "write_bytes": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "algorithmic_read_bytes": alg_r, "algorithmic_write_bytes": alg_w,
        "traffic_over_algorithmic": (read_b + write_b) / (alg_r + alg_w),
        "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 16-B/lane read half-count); WRITE_SIZE KiB x1024",
        "per_kernel": per_kernel(a.root, re.compile(a.regex)),
    }
    path = a.out or os.path.join(ROOT, "profiles", f"traffic_{a.cfg}.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
