set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --train --steps 5 --warmup 2 > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err || { tail -30 gpurun_out/bench_train.err; exit 1; }
cat gpurun_out/bench_train.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.pop('kernels'); print(json.dumps(d, indent=1)); print(list(k.items())[:12])"
