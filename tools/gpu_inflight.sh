set -o pipefail
mkdir -p gpurun_out/r06o; export TMPDIR=/tmp
for k in 3 4 5 3 4 5; do
  timeout -k 10 200 python3 -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-signing-roots --no-extras --no-api --no-vs-shard --inflight $k > gpurun_out/r06o/inf$k.json 2> gpurun_out/r06o/inf$k.err || { tail -20 gpurun_out/r06o/inf$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r06o/inf$k.json')); k=d['roofline']['kernel_ms_per_step']; print('inflight $k: %.3f M ms/step %.2f prep %.2f msm %.2f' % (d['value']/1e6, d['ms_per_step'], k['prepare'], k['msm']))"
done
