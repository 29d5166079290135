#!/bin/bash
# the -m gpu suite, then the step breakdown (rocprofv3 kernel trace of the default bench's timed steps)
set -u
export TMPDIR=/tmp
bash tools/gpu_tests.sh ${1:-r05k11} || exit 11
bash tools/step_prof.sh ${1:-r05k11}_step || exit 12
