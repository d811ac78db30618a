"""Per-shape timing of the HBM-bound normalisation kernels at the 16x512^2 CFG-pair step shapes
(GroupNorm: 2 reads + 1 write; LayerNorm: read + write; LayerNorm+LoRA-down: read + write + u).
Prints one JSON line per shape with us and GB/s of algorithmic traffic."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

BF16 = torch.bfloat16


def timeit(fn, reps=20):
    """Device time per call: `reps` calls captured in one HIP graph (eager launches of these 10-50 us
    kernels are bounded by the Python launch path, not the GPU)."""
    fn()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        fn()  # warm the caching allocator on the capture stream
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(reps):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    graph.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    gn = [("res64", 32, 4096, 320, 0, True), ("res64_cat", 32, 4096, 320, 320, True), ("res64_cat960", 32, 4096, 640, 320, True),
          ("res32", 32, 1024, 640, 0, True), ("res32_cat", 32, 1024, 640, 640, True), ("res16", 32, 256, 1280, 0, True),
          ("res16_cat", 32, 256, 1280, 1280, True), ("t2d32", 32, 1024, 640, 0, False), ("t2d16", 32, 256, 1280, 0, False),
          ("motion64", 2, 65536, 320, 0, False), ("motion32", 2, 16384, 640, 0, False), ("motion16", 2, 4096, 1280, 0, False)]
    for name, ns, rps, C1, C2, act in gn:
        x1 = torch.randn(ns * rps, C1, device=dev, generator=g).to(BF16)
        x2 = torch.randn(ns * rps, C2, device=dev, generator=g).to(BF16) if C2 else None
        C = C1 + C2
        gam, bet = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        out = torch.empty(ns * rps, C, dtype=BF16, device=dev)
        us = timeit(lambda: K.group_norm(x1, ns, rps, 32, 1e-5, gam, bet, silu=act, x2=x2, out=out))
        sums = torch.empty(ns * 64, dtype=torch.float64, device=dev)
        us_s = timeit(lambda: K.group_norm_sums(x1, ns, rps, 32, x2=x2, out=sums))
        nb = 2.0 * ns * rps * C
        print(json.dumps({"kind": "groupnorm", "shape": name, "rows": ns * rps, "C": C, "us": round(us, 1),
                          "gbs": round(3 * nb / us / 1e3, 1), "stats_us": round(us_s, 1),
                          "stats_gbs": round(nb / us_s / 1e3, 1)}), flush=True)
    for rows, C in [(131072, 320), (32768, 640), (8192, 1280)]:
        x = torch.randn(rows, C, device=dev, generator=g).to(BF16)
        gam, bet = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        out = torch.empty_like(x)
        us = timeit(lambda: K.layer_norm(x, gam, bet, 1e-5, out=out))
        print(json.dumps({"kind": "layernorm", "rows": rows, "C": C, "us": round(us, 1),
                          "gbs": round(2 * 2.0 * rows * C / us / 1e3, 1)}), flush=True)
        for R in (16, 64):
            A = (torch.randn(R, C, device=dev, generator=g) * C ** -0.5).to(BF16)
            us = timeit(lambda: K.layer_norm_lora(x, gam, bet, 1e-5, A, out=out))
            print(json.dumps({"kind": "layernorm_lora", "rows": rows, "C": C, "R": R, "us": round(us, 1),
                              "gbs": round((2 * 2.0 * rows * C + 2.0 * rows * R) / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
