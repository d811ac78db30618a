set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_lora_gpu.py tests/test_host.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_lora.log 2>&1 || { echo "lora tests failed"; tail -40 gpurun_out/pytest_lora.log; exit 1; }
tail -3 gpurun_out/pytest_lora.log
timeout -k 10 800 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_bf16_gpu.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/pytest_parity_lora.log 2>&1 || { echo "parity failed"; grep -E "parity|PASS|FAIL|Error" gpurun_out/pytest_parity_lora.log | tail -40; exit 1; }
grep -E "\[parity\]|\[bf16-parity\]|passed|failed" gpurun_out/pytest_parity_lora.log | tail -30
bash tools/ab_bench.sh new nolora new2 nolora2
