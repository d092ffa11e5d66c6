"""Collect rocprofv3 PMC counters for the shuffle kernels, one pass per counter group.

Run ON THE GPU BOX (it spawns `rocprofv3 --pmc ... -- python3 bench.py ...`, one pass each):

    python3 profiles/collect_pmc.py --out gpurun_out/pmc --workload terasort [bench args...]
    python3 profiles/collect_pmc.py --merge gpurun_out/pmc --tag r02      (on the CPU side)

The first form writes <out>/<workload>/summary.json; --merge folds every workload's summary into
profiles/pmc_<tag>.json = {"workloads": {workload: {"bench_args", "records_per_launch",
"kernels": {kernel: {...}}}}}, the file bench.py reads its `traffic` from (keyed by workload and
by the kernel the library reports it launched).  Per kernel: the mean of every counter per
dispatch and the HBM bytes per launch computed as the MI355X guide prescribes (MI355X_MICROARCH.md §HBM):
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
           "k_map_scan": "map_scan", "k_onepass": "onepass", "k_sweep": "sweep",
           "k_gather_copy": "copy", "k_msd16": "msd"}
WORKLOAD_ARGS = {  # one PMC run: 8 launch groups of 32 maps x 2^20 records per workload (the
    # traffic per record is what bench.py reads; it does not depend on the group size)
    "terasort": ["--workload", "terasort", "--records", str(8 * 32 * (1 << 20)), "--group-maps", "32"],
    "zipf": ["--workload", "zipf", "--records", str(8 * 32 * (1 << 20)), "--group-maps", "32"],
    "small": ["--workload", "small", "--records", str(8 * 32 * (1 << 20)), "--group-maps", "32"],
}
COMMON = ["--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--varlen-rows", "0",
          "--compress-maps", "0", "--file-maps", "0", "--reduce-sort-records", "0",
          "--plugin-groups", "0", "--self-check", "0", "--maps-2e27", "0", "--resolve", "0",
          "--plugin-host-maps", "0"]


def short(name: str) -> str | None:
    """Kernel base name ('k_scatter7'), the name sux_kernel_variant reports."""
    for k in KERNELS:
        if k in name:
            return name.split("(")[0].replace("void ", "").replace("sux::", "").split("<")[0]
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
    ap.add_argument("--workload", default="terasort", choices=sorted(WORKLOAD_ARGS))
    ap.add_argument("--tag", default="r02")
    ap.add_argument("--merge", default=None, help="fold <dir>/*/summary.json into profiles/pmc_<tag>.json")
    a, extra = ap.parse_known_args()
    if a.merge:
        path = os.path.join(ROOT, "profiles", f"pmc_{a.tag}.json")
        merged = {"note": "per-dispatch means; hbm bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB->B), "
                          "MI355X_MICROARCH.md §HBM; written by profiles/collect_pmc.py",
                  "workloads": {}}
        if os.path.exists(path):
            with open(path) as f:
                merged["workloads"].update(json.load(f).get("workloads", {}))
        for f in sorted(glob.glob(os.path.join(a.merge, "*", "summary.json"))):
            with open(f) as fh:
                sm = json.load(fh)
            # kernels profiled earlier under the same workload (other tuning shapes) are kept
            old = merged["workloads"].get(sm["workload"], {}).get("kernels", {})
            merged["workloads"][sm["workload"]] = dict(sm, kernels={**old, **sm["kernels"]})
        with open(path, "w") as f:
            json.dump(merged, f, indent=1, sort_keys=True)
        print("wrote", path, sorted(merged["workloads"]))
        return
    bench_args = WORKLOAD_ARGS[a.workload] + COMMON + extra
    out = os.path.join(a.out, a.workload)
    os.makedirs(out, exist_ok=True)
    dirs = [run_pass(cs, out, bench_args, i) for i, cs in enumerate(PASSES)]
    res = summarize(dirs)
    gm = int(bench_args[bench_args.index("--group-maps") + 1]) if "--group-maps" in bench_args else 32
    rpm = int(bench_args[bench_args.index("--map-records") + 1]) if "--map-records" in bench_args else 1 << 20
    for e in res.values():
        e["records_per_launch"] = gm * rpm
    summary = {"workload": a.workload, "bench_args": bench_args, "records_per_launch": gm * rpm,
               "kernels": res}
    with open(os.path.join(out, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
