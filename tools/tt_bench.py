"""TemporalTransformer (animatediff/temporal_transformer.py) on the HIP path vs the fp32 CPU oracle restatement,
at the shape SURVEY.md §6 timed the reference on: TemporalTransformer(320, 2 layers, 8 heads), (1, 320, 16, 64, 64).
Prints one JSON line (GPU ms, CPU ms, threads, rel-L2 vs the oracle)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.ref_ops import temporal_transformer  # noqa: E402  (checker / CPU baseline only)
from video_style_transfer_amd.temporal_transformer import TemporalTransformer  # noqa: E402


def main():
    torch.manual_seed(0)
    C, shape = 320, (1, 320, 16, 64, 64)
    tt = TemporalTransformer(C, 2, 8)
    with torch.no_grad():
        for p in tt.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    x = torch.randn(shape).to(torch.bfloat16).float()
    dev = torch.device("cuda")
    ttd = tt.to(dev)
    xd = x.to(dev)
    for _ in range(3):
        out = ttd(xd, num_frames=16)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        out = ttd(xd, num_frames=16)
    e.record()
    torch.cuda.synchronize()
    gpu_ms = s.elapsed_time(e) / 20
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    P = {k: v.float().cpu() for k, v in tt.state_dict().items()}
    with torch.no_grad():
        t0 = time.perf_counter()
        ref = temporal_transformer(x, P, 2, 8)
        cpu_ms = (time.perf_counter() - t0) * 1e3
    o = out.float().cpu()
    print(json.dumps({"module": "TemporalTransformer(320, 2, 8)", "input": list(shape), "gpu_ms": round(gpu_ms, 3),
                      "cpu_oracle_ms": round(cpu_ms, 1), "cpu_threads": threads,
                      "speedup": round(cpu_ms / gpu_ms, 1),
                      "rel_l2_vs_oracle": float((o - ref).norm() / ref.norm())}))


if __name__ == "__main__":
    main()
