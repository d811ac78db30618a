#!/bin/bash
# round-6 measurement session: PMC HBM traffic of the shipped library (2 passes) -> profiles/pmc_traffic_r6.json (read by
# bench.py), the headline bench, the rocprof kernel stats of the same command, the training bench
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ]; then echo "[step] stopping after rc=$rc"; tail -20 gpurun_out/$log; exit $rc; fi
  return 0
}
md5sum video_style_transfer_amd/libvst_hip.so > gpurun_out/pmc_so.md5
run 300 r6f_pmc_fetch.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o pmc -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-vae --no-peaks --no-roofline
run 300 r6f_pmc_write.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o pmc -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-vae --no-peaks --no-roofline
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_so.md5 > gpurun_out/pmc_traffic_r6.json && cp gpurun_out/pmc_traffic_r6.json profiles/ && echo "[step] pmc json ok"
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
run 420 r6f_bench.json python -u bench.py
tail -c 400 gpurun_out/r6f_bench.json
run 400 r6f_rocprof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6f_prof -o r6f -- python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vae --no-peaks
mkdir -p gpurun_out/r6f_keep
for f in $(find gpurun_out/r6f_prof -name "*kernel_stats.csv"); do cp $f gpurun_out/r6f_keep/; done
rm -rf gpurun_out/r6f_prof
run 400 r6f_bench_train.json python -u bench.py --train --no-cpu-baseline
tail -c 300 gpurun_out/r6f_bench_train.json
