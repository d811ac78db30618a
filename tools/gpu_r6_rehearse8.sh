#!/bin/bash
# bench.py's 8-rank path at the driver's full sizes (16 x 512^2, 8 clips, frame-sharded x8), all ranks on the one
# GPU over gloo (VST_BENCH_REHEARSAL=gloo): the shard preflight (rank 0's unsharded forward of all 8 clips x CFG pair),
# piecewise capture and one eager step.  A correctness drill, never a scaling number.
mkdir -p gpurun_out
export VST_BENCH_REHEARSAL=gloo OMP_NUM_THREADS=2 PYTHONUNBUFFERED=1
EXTRA=${1:---strong-record off --gather-record off --configs3 off}
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 8 --steps 1 --warmup 0 --no-cpu-baseline --no-vae --no-roofline $EXTRA \
  > gpurun_out/r6_rehearse8.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do
  sleep 30
  echo "[hb] $(date +%T) $(nvidia-smi >/dev/null 2>&1; rocm-smi --showmemuse 2>/dev/null | grep -m1 'GPU\[0\]' | tr -s ' ' | cut -c1-80)"
done
wait $pid
rc=$?
tail -c 3000 gpurun_out/r6_rehearse8.log
exit $rc
