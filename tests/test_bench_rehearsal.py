"""bench.py's N-GPU path rehearsed on one GPU (VERDICT r2 "RCCL readiness"): `torch.distributed.run` with two ranks,
both on cuda:0 over gloo (VST_BENCH_REHEARSAL=gloo; RCCL cannot put two ranks on one device), frame sharding of every
clip over the ranks.  Before anything is timed, bench.py runs its shard preflight -- one eager frame-sharded UNet
forward, gathered to rank 0 and compared with rank 0's unsharded forward of the same clips -- and exits non-zero
unless the two are bit-identical (weak scaling, clips == ranks; and the strong-scaling sub-records: one clip split over the
ranks, configs[3]'s shape class); the JSON line carries the results.  The driver's 8-GPU run goes through the same code with
the nccl backend (and the step captured in a HIP graph)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_bench_two_rank_frame_shard_rehearsal():
    if torch.cuda.device_count() == 0:
        pytest.skip("no HIP device")
    env = dict(os.environ, VST_BENCH_REHEARSAL="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "1", "--warmup", "0", "--frames", "16", "--size", "256", "--no-cpu-baseline", "--no-vae", "--no-roofline",
           "--configs3", "on", "--configs3-frames", "8", "--configs3-size", "256"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    pf = d["shard_preflight"]
    print(f"[rehearsal] {d['config']['parallelism']}: {d['ms_per_step']} ms/step, preflight {pf}")
    assert d["n_gpus"] == 2 and d["finite"]
    assert pf is not None and pf["bitwise_equal"] and pf["rel_l2"] == 0.0
    # the sub-records the driver's N-GPU run adds: one clip split over the ranks (strong scaling) and configs[3]'s
    # shape class (here 8 frames at 256^2 so the rehearsal stays short), each with its own bitwise preflight
    subs = d["sub_records"]
    assert d["config"]["exchange_overlap"] is True  # the headline runs the overlapped all-to-all (CFG pair halves)
    for name in ("strong_1clip", "configs3", "all_gather"):
        r = subs[name]
        print(f"[rehearsal] {name}: {r['ms_per_step']} ms/step, {r['frames_per_gpu']} frames/GPU, "
              f"exchange {r['exchange']} (overlap {r['overlap']}), preflight {r['shard_preflight']}")
        assert r["scaling"] == ("weak" if name == "all_gather" else "strong") and r["finite"] and r["value"] > 0
        assert r["shard_preflight"]["bitwise_equal"], r["shard_preflight"]
    # the north star's exchange on the headline workload (sub_records.all_gather): same clips, same bits
    assert subs["all_gather"]["exchange"] == "all_gather" and subs["all_gather"]["clips"] == 2
