# round-4 GPU session l: LayerNorm row stream — bitwise tests, in-step A/B (VST_LN_STREAM 0/1, VST_LN_WPC 4/8/16)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ]; then echo "[step] stopping after rc=$rc"; tail -30 gpurun_out/$log; exit $rc; fi
  return 0
}
run 300 r4l_tests.log python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "layer_norm or persistent"
run 600 r4l_shard.log python -u -m pytest -v -x --timeout 300 --timeout-method thread tests/test_frame_shard.py -k "sdxl_768_32_frames_two"
grep -E "FAILED|passed|failed|\[shard\]" gpurun_out/r4l_shard.log | tail -6
grep -E "FAILED|passed|failed" gpurun_out/r4l_tests.log | tail -3
for v in "0 8" "1 8" "1 4" "1 16" "0 8" "1 8" "1 4" "1 16"; do
  set -- $v
  VST_LN_STREAM=$1 VST_LN_WPC=$2 run 300 r4l_bench_ln$1_wpc$2_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
for f in gpurun_out/r4l_bench_*.json; do python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); k=d['kernels']; print('$f', d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'layernorm' in n})"; done
