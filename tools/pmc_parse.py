"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel and per grid size (work-items), the
counters averaged over the dispatches of that size.  bench.py attaches a kernel's counters to a
roofline only at the grid its own launch had (bench.pmc_at).
Usage: python3 tools/pmc_parse.py <pmc dir> <out.json> [tag]"""
import csv
import glob
import json
import os
import subprocess
import sys
import time
from collections import defaultdict


def short_name(k):
    k = k.split("(")[0]
    if k.startswith("void "):  # template instances: "void gbv::k_sm_prepare<false>"
        k = k[5:]
    return k.replace("gbv::", "")


def main(root, out, tag=""):
    acc = defaultdict(lambda: defaultdict(list))  # (kernel, grid) -> counter -> [values]
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                key = (short_name(row.get("Kernel_Name", "")), int(float(row["Grid_Size"])))
                acc[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
                dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
                acc[key]["duration_ms"].append(dur)
    kernels = defaultdict(dict)
    for (k, g), cs in acc.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["dispatches"] = max(len(v) for c, v in cs.items() if c != "duration_ms")
        kernels[k][str(g)] = d
    try:
        head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True).stdout.strip()
    except OSError:
        head = ""
    res = {"collected": {"tag": tag, "date_utc": time.strftime("%Y-%m-%d %H:%M", time.gmtime()), "tree": head or None,
                         "passes": "FETCH_SIZE | WRITE_SIZE | SQ (separate rocprofv3 --pmc runs, tools/pmc.sh)"},
           "kernels": {k: kernels[k] for k in sorted(kernels)}}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
