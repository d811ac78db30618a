#!/bin/bash
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_training_gpu.py -m gpu -x -q -k "layer_norm or unet_training" --timeout 250 --timeout-method thread > gpurun_out/r6_lnb_tests.txt 2>&1 || { tail -20 gpurun_out/r6_lnb_tests.txt; exit 1; }
tail -1 gpurun_out/r6_lnb_tests.txt
for v in new old new; do
  if [ $v = old ]; then export VST_LIB_AB=ablib/libvst_old.so; else unset VST_LIB_AB; fi
  timeout -k 10 400 python -u bench.py --train --no-cpu-baseline --no-roofline > gpurun_out/r6_lnb_$v.json 2>&1 || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/r6_lnb_$v.json') if l.startswith('{')][-1]);print('$v', d['ms_per_step'], d['value'], d.get('loss'))"
done
