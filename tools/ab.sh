#!/bin/bash
# A/B bench of library variants: bash tools/ab.sh name1 name2 ...  ("base" = lodestar_amd/libgbv.so)
mkdir -p gpurun_out/ab
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=lodestar_amd/variants/libgbv_$v.so; fi
  LODESTAR_AMD_LIB=$lib timeout -k 10 240 python3 -u bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-signing-roots > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
done
