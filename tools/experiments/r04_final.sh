#!/bin/bash
# Round-end evidence: every -m gpu test, the default bench, and the same under rocprofv3 --kernel-trace --stats
set -u
O=gpurun_out/r04final4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 11; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python3 -u bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 12; }
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['value'], b['ms_per_step'], b['roofline']['frac'], b['ivf_pq_12m5']['qps_pq_refined'], b['ivf_pq_12m5']['recall_at_10_pq_refined'])"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o prof -- python3 -u bench.py --json-out $O/bench_prof.json > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 13; }
rm -f $O/prof/prof_kernel_trace.csv
bash tools/step_prof.sh r04final4/step > /dev/null && head -1 $O/step/breakdown.txt
echo done
