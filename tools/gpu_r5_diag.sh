#!/bin/bash
# round 5: the captured all_to_all_single with the graph destroyed before destroy_process_group (RCCL's persistent
# plan lives as long as the graph), then the same without (the round-4 hang) to confirm the cause
set -o pipefail
mkdir -p gpurun_out
export NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,COLL,P2P
timeout -k 10 100 python -u tools/rccl_diag.py a2a+del > gpurun_out/r5_rccl_diag_del.log 2>&1 || { echo "a2a+del failed rc=$?"; exit 1; }
echo "a2a+del ok"
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vae > gpurun_out/r5_bench_base.json 2> gpurun_out/r5_bench_base.err
echo "bench rc=$?"
