#!/bin/bash
# vst_gemm_tn in the training backward: the training tests (gradient gates vs the fp32 oracle / the CPU-autocast
# yardstick), the weight-gradient shape bench, then the configs[4] train bench with and without it (same box)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() { local lim=$1 log=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "[step] $log rc=$rc";
        if [ $rc -ne 0 ]; then tail -30 gpurun_out/$log; exit $rc; fi; }
run 600 r6_tn_tests.txt python -u -m pytest tests/test_training_gpu.py tests/test_train_step_gpu.py tests/test_kernels_gpu.py -m gpu -x -v -s -k "train or grad or gemm_tn or lora or geglu" --timeout 500 --timeout-method thread
grep -E "passed|failed" gpurun_out/r6_tn_tests.txt | tail -2
run 200 r6_tn_bench.txt python -u tools/tn_bench.py
run 400 r6_tn_train_on.json python -u bench.py --train --no-cpu-baseline --no-roofline
VST_GEMM_TN=0 run 400 r6_tn_train_off.json python -u bench.py --train --no-cpu-baseline --no-roofline
run 400 r6_tn_train_on2.json python -u bench.py --train --no-cpu-baseline --no-roofline
for f in on off on2; do python -c "import json;d=json.loads([l for l in open('gpurun_out/r6_tn_train_$f.json') if l.startswith('{')][-1]);print('$f', d['ms_per_step'], d['value'], d.get('loss'))"; done
