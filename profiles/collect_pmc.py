"""Collect rocprofv3 PMC counters for the shuffle kernels, one pass per counter group.

Run ON THE GPU BOX (it spawns `rocprofv3 --pmc ... -- python3 bench.py ...`, one pass each):

    python3 profiles/collect_pmc.py --out gpurun_out/pmc [--tag r01] [bench args...]

Summary: profiles/pmc_<tag>.json with, per kernel, the mean of every counter per dispatch and
the HBM bytes per launch computed as the MI355X guide prescribes (MI355X_MICROARCH.md §HBM):
FETCH_SIZE (KiB) is doubled — on gfx950 it reports half the bytes of a wide streaming read —
and WRITE_SIZE (KiB) is taken as is; FETCH_SIZE and WRITE_SIZE need separate passes (TCC slots).
This script never imports torch and never touches the GPU itself.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [
    ["FETCH_SIZE"],
    ["WRITE_SIZE"],
    ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
     "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD"],
    ["SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_SALU",
     "SQ_LDS_IDX_ACTIVE", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS", "SQ_INST_LEVEL_VMEM"],
    ["TA_TA_BUSY", "TA_ADDR_STALLED_BY_TC_CYCLES", "GRBM_GUI_ACTIVE", "GRBM_COUNT"],
    ["TCC_HIT_sum", "TCC_MISS_sum"],
]
KERNELS = {"k_hist": "hist", "k_scatter": "scatter", "k_tile_scan": "tile_scan",
           "k_group_scan": "group_scan", "k_gather_copy": "copy"}


def short(name: str) -> str | None:
    for k in KERNELS:
        if k in name:
            # keep the template signature (v1/v2 variants) in the key
            base = name.split("(")[0].replace("void ", "").replace("sux::", "")
            return base
    return None


def run_pass(counters, outdir, bench_args, i):
    d = os.path.join(outdir, f"pass{i}")
    cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", *counters, "-d", d, "-o", "run",
           "--output-format", "csv", "--", sys.executable, os.path.join(ROOT, "bench.py"),
           *bench_args]
    print("+", " ".join(cmd), flush=True)
    with open(os.path.join(outdir, f"pass{i}.log"), "w") as log:
        rc = subprocess.call(cmd, stdout=log, stderr=subprocess.STDOUT, cwd=ROOT)
    if rc != 0:
        raise SystemExit(f"pass {i} ({counters}) failed with rc={rc}")
    return d


def parse(d):
    """{kernel: {counter: [values per dispatch]}}"""
    out = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if not k:
                    continue
                out[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return out


def summarize(dirs):
    acc = defaultdict(dict)
    for d in dirs:
        for k, cs in parse(d).items():
            for c, vals in cs.items():
                acc[k][c] = sum(vals) / len(vals)
                acc[k][c + "_dispatches"] = len(vals)
    res = {}
    for k, cs in acc.items():
        e = dict(cs)
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            e["hbm_read_bytes_per_launch"] = cs["FETCH_SIZE"] * 1024 * 2  # gfx950: x2
            e["hbm_write_bytes_per_launch"] = cs["WRITE_SIZE"] * 1024
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes_per_launch"] + e["hbm_write_bytes_per_launch"]
        res[k] = e
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/pmc")
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--summarize-only", action="store_true")
    a, bench_args = ap.parse_known_args()
    if not bench_args:
        bench_args = ["--steps", "1", "--warmup", "1", "--records", "268435456",
                      "--no-cpu-baseline", "--varlen-rows", "0", "--compress-maps", "0",
                      "--file-maps", "0", "--reduce-sort-records", "0"]
    os.makedirs(a.out, exist_ok=True)
    dirs = []
    for i, cs in enumerate(PASSES):
        d = os.path.join(a.out, f"pass{i}")
        if not a.summarize_only:
            run_pass(cs, a.out, bench_args, i)
        dirs.append(d)
    res = summarize(dirs)
    summary = {"bench_args": bench_args, "note": "per-dispatch means; hbm bytes = 2*FETCH_SIZE + "
               "WRITE_SIZE (KiB->B), MI355X_MICROARCH.md §HBM", "kernels": res}
    # bench.py reads the map-side scatter entry under the plain name (the default k_scatter7,
    # never the reduce-sort's k_scatter16 if that leg ran)
    for pref in ("k_scatter7", "k_scatter6", "k_scatter"):
        hit = [k for k in res if k.startswith(pref) and not k.startswith("k_scatter16")]
        if hit:
            summary["kernels"]["k_scatter"] = res[hit[0]]
            summary["k_scatter_is"] = hit[0]
            break
    path = os.path.join(ROOT, "profiles", f"pmc_{a.tag}.json")
    with open(os.path.join(a.out, f"pmc_{a.tag}.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1, sort_keys=True))
    print("wrote", os.path.join(a.out, f"pmc_{a.tag}.json"), "(copy to", path, "to commit)")


if __name__ == "__main__":
    main()
