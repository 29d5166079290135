#!/bin/bash
# K13a epilogue with v_med3: the build parity tests, then the build A/B (variants via MIVS_LIB)
set -u
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_engine_switches.py tests/test_gpu_baseline_configs.py > gpurun_out/r05med3_tests.log 2>&1 || { tail -30 gpurun_out/r05med3_tests.log; exit 11; }
tail -2 gpurun_out/r05med3_tests.log
bash tools/experiments/r05_varb.sh r05med3 base med3
