"""Medians of tools/latency_probe.py output: per call kind, wall time and per-stage kernel times.
    python tools/lat_summary.py gpurun_out/<tag>/lat_*.txt"""
import collections
import re
import statistics as st
import sys

for fn in sys.argv[1:]:
    wall = collections.defaultdict(list)
    kern = collections.defaultdict(lambda: collections.defaultdict(list))
    for line in open(fn):
        m = re.match(r"(call|bad call|c1 call|c4 block|c4e block) ([\d.]+) ms\s+kernels \{(.*)\}", line)
        if not m:
            continue
        wall[m.group(1)].append(float(m.group(2)))
        for k, v in re.findall(r"'(\w+)': ([\d.]+)", m.group(3)):
            kern[m.group(1)][k].append(float(v))
    print(fn)
    for kind, w in wall.items():
        ks = {k: round(st.median(v), 2) for k, v in kern[kind].items() if st.median(v) > 0.05}
        print(f"  {kind:10s} {st.median(w):6.2f} ms  {ks}")
