#!/bin/bash
# A/B of K13 build variants (variants/libmivs_*.so via MIVS_LIB), alternating with the default build
set -u
O=gpurun_out/r04var
mkdir -p $O
run() {  # name lib
  local nm=$1 lib=$2
  MIVS_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --json-out $O/$nm.json > $O/$nm.log 2>&1 || return 1
  python3 -c "import json;b=json.load(open('$O/$nm.json'));print('$nm', b['ms_per_step'], b['roofline']['launch_ms'])"
}
B=cuvs-rag_amd/mivs/libmivs.so
run base1 $B && run pd2 variants/libmivs_pd2.so && run pd4 variants/libmivs_pd4.so && run spin0 variants/libmivs_spin0.so && run base2 $B && run pd2b variants/libmivs_pd2.so && run pd4b variants/libmivs_pd4.so && run spin0b variants/libmivs_spin0.so
