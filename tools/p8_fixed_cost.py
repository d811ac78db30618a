"""Fixed per-tile cost of the 8-phase GEMM: time one launch shape at several K (same M, N, so the same tile count and
rounds) and fit t = rounds * (fixed + nk * per_ktile); `fixed` is what a tile pays outside its k-loop (fill + epilogue
+ launch ramp), `per_ktile` the steady-state cost of one 64-deep k-tile.  One JSON line per (kind, M, N).
python tools/p8_fixed_cost.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from video_style_transfer_amd import kernels as K  # noqa: E402

CASES = [("geglu", 8192, 10240), ("plain", 8192, 1280), ("plain", 131072, 320), ("geglu", 131072, 2560),
         ("plain", 32768, 640)]
KS = [320, 640, 1280, 2560, 5120]


def time_us(fn, reps=20):
    for _ in range(3):
        fn()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / reps)
    return best


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for kind, M, N in CASES:
        geglu = kind == "geglu"
        pts = []
        for Kd in KS:
            x = torch.randn(M, Kd, device=dev, generator=g).to(torch.bfloat16)
            w = (torch.randn(N, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
            b = torch.randn(N, device=dev, generator=g) * 0.1
            r = None if geglu else torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
            us = time_us(lambda: K.linear(x, w, b, geglu=geglu, residual=r))
            pts.append((Kd // 64, us, K.gemm_kernel_name(M, N, Kd, 1 if geglu else 0)))
            del x, w, r
            print(f"[fc] {kind} {M}x{N}x{Kd}: {us:.1f} us  {2.0 * M * N * Kd / us / 1e6:.0f} TF/s  {pts[-1][2]}",
                  flush=True)
        nk = torch.tensor([p[0] for p in pts], dtype=torch.float64)
        t = torch.tensor([p[1] for p in pts], dtype=torch.float64)
        A = torch.stack([torch.ones_like(nk), nk], 1)
        coef = torch.linalg.lstsq(A, t[:, None]).solution[:, 0]
        print(json.dumps({"kind": kind, "M": M, "N": N, "points_us": {int(p[0] * 64): round(p[1], 1) for p in pts},
                          "kernels": sorted({p[2] for p in pts}), "fixed_us_per_launch": round(coef[0].item(), 2),
                          "us_per_ktile_per_launch": round(coef[1].item(), 3)}), flush=True)


if __name__ == "__main__":
    main()
