# temporal attention: kernel tests, then the build in abx/libvst_old.so vs the in-tree build, two alternating passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k "temporal" > gpurun_out/tcheck_pytest.log 2>&1 || { tail -30 gpurun_out/tcheck_pytest.log; exit 1; }
grep passed gpurun_out/tcheck_pytest.log
for r in 1 2; do
  VST_LIB_AB=abx/libvst_old.so timeout -k 10 120 python -u tools/attn_bench.py temp64 temp32 temp16 > gpurun_out/tcheck_old$r.txt 2>&1 || exit 1
  timeout -k 10 120 python -u tools/attn_bench.py temp64 temp32 temp16 > gpurun_out/tcheck_new$r.txt 2>&1 || exit 1
  for t in old new; do echo "$t $r: $(grep '^{' gpurun_out/tcheck_$t$r.txt | grep -v bwd | tr -d '\n')"; done
done
