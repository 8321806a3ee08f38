set -o pipefail
OUT=gpurun_out/r04o; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_c5.py tests/test_gpu_scale.py tests/test_gpu_stream.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then lib=""; else lib=lodestar_amd/variants/libgbv_$v.so; fi
  LODESTAR_AMD_LIB=$lib GBV_DL_DEBUG=1 timeout -k 10 300 python3 -u tools/c5_probe.py --steps 9 --depth ${DEPTH:-3} > $OUT/c5_$v.txt 2>$OUT/c5_$v.err || { tail -5 $OUT/c5_$v.err; exit 1; }
  echo "$v $(cut -c1-250 $OUT/c5_$v.txt) | $(grep '\[gbv\]' $OUT/c5_$v.err | tail -1)"
done
