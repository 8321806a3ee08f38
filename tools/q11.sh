# Timing runs of bench.py with per-step completion times; usage: bash tools/q11.sh
mkdir -p gpurun_out/q11
run() { # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 8 --warmup 1 --inflight 3 --no-cpu-baseline --no-signing-roots > gpurun_out/q11/$tag.json 2> gpurun_out/q11/$tag.err || exit 1
  echo "$tag $(grep 'step done' gpurun_out/q11/$tag.err | sed 's/.bench.   step done at//' | tr '\n' ' ') $(python3 -c "import json;d=json.load(open('gpurun_out/q11/$tag.json'));print(d['value'], d['p50_batch_latency_ms'], d['roofline']['kernel_ms_per_step'])")"
}
GBV_MSM_STREAM=h timeout -k 10 300 python3 -u -m pytest tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q11/scale.log 2>&1 || { tail -30 gpurun_out/q11/scale.log; exit 1; }
tail -1 gpurun_out/q11/scale.log
for r in 1 2 3; do
  run H$r GBV_MSM_STREAM=h
done
run A1
