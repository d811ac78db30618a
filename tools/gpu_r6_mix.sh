#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 python -u tools/fetch_probe.py mix > gpurun_out/r6_mix_probe.txt 2>&1; rc=$?; cat gpurun_out/r6_mix_probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u tools/fetch_probe.py > gpurun_out/r6_fetch_probe2.txt 2>&1; rc=$?; cat gpurun_out/r6_fetch_probe2.txt; exit $rc
