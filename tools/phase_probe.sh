set -u
mkdir -p gpurun_out/ph
for e in "MIVS_PF_FLAGS=32" "MIVS_PF_FLAGS=32 MIVS_PF_CHUNK_ROWS=8192" "MIVS_PF_FLAGS=0"; do
  env $e timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --gt-queries 200 --json-out gpurun_out/ph/b.json > gpurun_out/ph/b.log 2>&1 || exit 1
  echo "== $e"; grep "k10 phases" gpurun_out/ph/b.log | tail -2
  python3 -c "import json;j=json.load(open('gpurun_out/ph/b.json'));print(round(j['value']), j['roofline']['launch_ms'], j['ms_per_step'])"
done
