#!/bin/bash
# K13 probe: tile pieces gathered from the query array vs copied from tile images
set -u
O=gpurun_out/${1:-r05g}
mkdir -p $O
timeout -k 10 120 ./tools/k13_probe 3000 > $O/probe.log 2>&1; rc=$?
cat $O/probe.log
exit $rc
