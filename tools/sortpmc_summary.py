"""Summarise tools/r04_sortpmc.sh: per sort kernel, the mean of each counter over the timed calls
(the last 5 dispatches of each kernel name), HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B,
MI355X_MICROARCH.md HBM rules), and the TA stall share.
usage: python tools/sortpmc_summary.py gpurun_out/r04_sortpmc OUT.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d, out):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values by dispatch]
    for f in sorted(glob.glob(os.path.join(d, "pass*", "**", "*counter_collection.csv"), recursive=True)):
        rows = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            rows[(k, int(r["Dispatch_Id"]))][r["Counter_Name"]] = float(r["Counter_Value"])
        for (k, _), cs in sorted(rows.items(), key=lambda x: x[0][1]):
            for c, v in cs.items():
                per[k][c].append(v)
    res = {}
    for k, cs in per.items():
        if "sort" not in k and "top_" not in k and "span" not in k and "gather" not in k:
            continue
        m = {c: sum(v[-5:]) / len(v[-5:]) for c, v in cs.items()}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_read_bytes"] = 2 * m["FETCH_SIZE"] * 1024
            m["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        if m.get("TA_TA_BUSY"):
            m["ta_stalled_by_tc_share"] = m.get("TA_ADDR_STALLED_BY_TC_CYCLES", 0) / m["TA_TA_BUSY"]
        if m.get("SQ_LDS_IDX_ACTIVE"):
            m["lds_conflict_share"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"]
        res[k] = m
    json.dump({"note": "tools/r04_sortpmc.sh: 5 M random TeraSort records (tools/sort_prof.py 5); "
               "means of the last 5 dispatches; hbm_read_bytes = 2 x FETCH_SIZE (gfx950), "
               "hbm_write_bytes = WRITE_SIZE", "kernels": res}, open(out, "w"), indent=1, sort_keys=True)
    for k, m in sorted(res.items(), key=lambda x: -x[1].get("hbm_read_bytes", 0)):
        print(f"{k[:50]:50s} read {m.get('hbm_read_bytes', 0) / 1e6:8.1f} MB  write "
              f"{m.get('hbm_write_bytes', 0) / 1e6:8.1f} MB  TA stall {m.get('ta_stalled_by_tc_share', 0):.2f}"
              f"  LDS conflicts {m.get('lds_conflict_share', 0):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
