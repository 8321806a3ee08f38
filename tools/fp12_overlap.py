"""For every k_fp12_check dispatch of a kernel trace: the kernels of other queues that ran during it
(what ran beside the multi-GPU exchange's final check).  Usage: python3 tools/fp12_overlap.py trace.csv"""
import csv
import sys
from collections import Counter

rows = list(csv.DictReader(open(sys.argv[1])))
k = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?")) for r in rows]
k.sort(key=lambda x: x[1])
checks = [x for x in k if "k_fp12_check" in x[0]]
print("k_fp12_check dispatches: %d" % len(checks))
beside = Counter()
n_overlap = 0
for name, s, e, q in checks:
    others = [x for x in k if x[3] != q and x[1] < e and x[2] > s]
    if others:
        n_overlap += 1
    for o in others:
        beside[o[0].split("(")[0].replace("gbv::", "")] += 1
    print("%8.3f ms  queue %s  beside: %s" % ((e - s) / 1e6, q, ", ".join(sorted({o[0].split("(")[0].replace("gbv::", "") for o in others})) or "-"))
print("checks with another queue's kernel running beside them: %d of %d" % (n_overlap, len(checks)))
print("kernels beside the checks:", dict(beside.most_common()))
