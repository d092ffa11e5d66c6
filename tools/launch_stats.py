"""Per-kernel launch statistics of a rocprofv3 kernel trace, restricted to the timed steps.

rocprofv3 --stats averages every launch of a kernel name, warm-up launches included; bench.py's
roofline `avg_launch_ms` covers the timed steps only.  This reads run_kernel_trace.csv, drops the
first `skip` launches of each kernel (the warm-up: --warmup x launch groups per step) and writes
count / mean / median / min / max per kernel, so a line's `frac` recomputes from a tracked file:
frac = alg_bytes_per_launch / mean_ns / 8000 GB/s.
usage: python tools/launch_stats.py run_kernel_trace.csv SKIP OUT.csv
"""
import csv
import statistics
import sys
from collections import defaultdict


def main(trace: str, skip: int, out: str) -> None:
    per = defaultdict(list)
    with open(trace) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            per[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "LaunchesKept", "LaunchesSkipped", "MeanNs", "MedianNs", "MinNs", "MaxNs"])
        for name, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            kept = d[skip:] if len(d) > skip else d
            w.writerow([name, len(kept), len(d) - len(kept), f"{statistics.mean(kept):.1f}",
                        f"{statistics.median(kept):.1f}", min(kept), max(kept)])


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
