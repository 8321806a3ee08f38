"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel, the counters of its LARGEST
dispatch (by grid size; the bench's timed launch, not the small latency probes), averaged over
the dispatches of that size.  Usage: python3 tools/pmc_parse.py <pmc dir> <out.json>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(root, out):
    rows = defaultdict(list)  # kernel -> [(grid, counter, value)]
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                short = row.get("Kernel_Name", "").split("(")[0].replace("gbv::", "")
                if short.startswith("void "):  # template instances: "void gbv::k_sm_prepare<false>"
                    short = short[5:]
                rows[short].append((float(row["Grid_Size"]), row["Counter_Name"], float(row["Counter_Value"])))
                dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
                rows[short].append((float(row["Grid_Size"]), "duration_ms", dur))
    res = {}
    for k, rs in rows.items():
        gmax = max(g for g, _, _ in rs)
        acc = defaultdict(list)
        for g, c, v in rs:
            if g == gmax:
                acc[c].append(v)
        d = {c: sum(v) / len(v) for c, v in acc.items()}
        d["grid_size"] = gmax
        d["dispatches_at_grid"] = max(len(v) for v in acc.values())
        res[k] = d
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
