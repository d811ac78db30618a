# round-4 GPU session h: headline bench, rocprof kernel stats of the same command, PMC HBM traffic (2 passes)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ]; then echo "[step] stopping after rc=$rc"; tail -5 gpurun_out/$log; exit $rc; fi
  return 0
}
md5sum video_style_transfer_amd/libvst_hip.so > gpurun_out/pmc_so.md5
run 400 r4h_bench.json python -u bench.py
run 400 r4h_rocprof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4h_prof -o r4h -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-vae --no-peaks
run 300 r4h_pmc_fetch.log rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o pmc -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-vae --no-peaks --no-roofline
run 300 r4h_pmc_write.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o pmc -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-vae --no-peaks --no-roofline
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_so.md5 > gpurun_out/pmc_traffic_r4h.json && echo "[step] pmc json ok"
# keep the summaries only (the raw traces exceed gpurun's 64 MiB copy-back)
mkdir -p gpurun_out/r4h_keep
for f in $(find gpurun_out/r4h_prof -name "*kernel_stats.csv"); do cp $f gpurun_out/r4h_keep/; done
rm -rf gpurun_out/r4h_prof gpurun_out/pmc_fetch gpurun_out/pmc_write
ls -la gpurun_out/r4h_keep; du -sh gpurun_out
