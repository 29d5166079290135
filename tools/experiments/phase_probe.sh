set -u
# in-kernel phase clocks of the pre-filter scans (MIVS_PF_FLAGS=32), K12 and K10
mkdir -p gpurun_out/ph
for e in "MIVS_PF_FLAGS=32" "MIVS_PF_FLAGS=32 MIVS_PF_REG=0" "$@"; do
  env $e timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --gt-queries 100 --json-out gpurun_out/ph/b.json > gpurun_out/ph/b.log 2>&1 || exit 1
  echo "== $e"; grep "phases" gpurun_out/ph/b.log | tail -1
  python3 -c "import json;j=json.load(open('gpurun_out/ph/b.json'));print(round(j['value']), j['roofline']['launch_ms'], j['ms_per_step'])"
done
