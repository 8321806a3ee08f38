#!/bin/bash
# Thread-form Miller doubling step without products for the halvings and 3 b' C: full GPU parity,
# then the C1 / C3 / C5 probes against r05p's base lines (same tree otherwise).
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 240 python -u tools/vs_probe.py --steps 9 > $O/vs.txt 2>&1 || { echo "vs probe failed"; tail -5 $O/vs.txt; exit 1; }
grep "^C" $O/vs.txt; grep "k_vs_miller\b" $O/vs.txt
timeout -k 10 300 python -u tools/c5_probe.py > $O/c5.txt 2>&1 || { echo "c5 probe failed"; tail -5 $O/c5.txt; exit 1; }
grep "^C5" $O/c5.txt
