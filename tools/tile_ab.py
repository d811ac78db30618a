"""Per-shape A/B of the GEMM tile configurations (ring 256x256 = 3, 256x128 = 4, 256x160 = 6, 192x256 = 7, 8-phase
256x256 = 8) on the under-filled and odd-N shapes of the denoise step, interleaved in one process.
python tools/tile_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

BF = torch.bfloat16
SHAPES = [  # name, M, N, K1, K2, geglu, residual, bias
    ("sp1280_qkv_lora", 8192, 3840, 1280, 64, False, False, True),
    ("sp640_qkv_lora", 32768, 1920, 640, 64, False, False, True),
    ("tr1280_out_lora", 4096, 1280, 1280, 32, False, True, True),
    ("tr1280_ff2", 4096, 1280, 5120, 0, False, True, True),
    ("tr1280_dx", 4096, 1280, 1280, 0, False, False, False),
    ("tr1280_dw", 1280, 1280, 4096, 0, False, False, False),
    ("tr1280_dx_ff", 4096, 5120, 1280, 0, False, False, False),
    ("sp1280_out_lora", 8192, 1280, 1280, 32, False, True, True),
    ("sp1280_ff2", 8192, 1280, 5120, 0, False, True, True),
    ("sp1280_proj", 8192, 1280, 1280, 0, False, False, True),
    ("mm320_proj", 131072, 320, 320, 0, False, True, True),
    ("sp640_out_lora", 32768, 640, 640, 32, False, True, True),
    ("sp640_proj", 32768, 640, 640, 0, False, False, True),
    ("sp640_ff2", 32768, 640, 2560, 0, False, True, True),
    ("mm320_ff2", 131072, 320, 1280, 0, False, True, True),
]
TILES = [(0, 0), (8, 1), (3, 1), (6, 1), (7, 1)]  # (tile, splits), 0 = auto
# VST_TILE_AB_TILES="0:0,1:1,9:1" / VST_TILE_AB_SHAPES="sp1280_out_lora,sp1280_ff2": another tile set / shape subset
if os.environ.get("VST_TILE_AB_TILES"):
    TILES = [tuple(int(v) for v in t.split(":")) for t in os.environ["VST_TILE_AB_TILES"].split(",")]
if os.environ.get("VST_TILE_AB_SHAPES"):
    SHAPES = [s for s in SHAPES if s[0] in os.environ["VST_TILE_AB_SHAPES"].split(",")]


def run(x, x2, w, b, r, geglu, tile):
    K.GEMM_POLICY["tile"], K.GEMM_POLICY["splits"] = tile
    try:
        return K.linear(x, w, b, x2=x2, residual=r, geglu=geglu)
    finally:
        K.GEMM_POLICY["tile"], K.GEMM_POLICY["splits"] = 0, 0


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for name, M, N, K1, K2, geglu, res, bias in SHAPES:
        Kt = K1 + K2
        x = torch.randn(M, K1, device=dev, generator=g).to(BF)
        x2 = torch.randn(M, K2, device=dev, generator=g).to(BF) if K2 else None
        w = (torch.randn(N, Kt, device=dev, generator=g) * Kt ** -0.5).to(BF)
        b = torch.randn(N, device=dev, generator=g) * 0.1 if bias else None
        r = torch.randn(M, N, device=dev, generator=g).to(BF) if res else None
        ref = run(x, x2, w, b, r, geglu, (3, 1)).float()
        fl = 2.0 * M * N * Kt
        best = {}
        for rnd in range(3):
            for t in TILES:
                if t[0] == 8 and K2 and (K1 % 64):
                    continue
                us = timeit(lambda: run(x, x2, w, b, r, geglu, t)) * 1e3
                best[t] = min(best.get(t, 1e9), us)
        errs = {t: ((run(x, x2, w, b, r, geglu, t).float() - ref).norm() / ref.norm()).item() for t in best}
        line = "  ".join(f"t{t[0]}s{t[1]}:{us:6.1f}us {fl / us / 1e6:6.1f}TF" + ("" if errs[t] < 1e-2 else f"(ERR {errs[t]:.1e})")
                         for t, us in best.items())
        print(f"{name:16s} {M}x{N}x{Kt} auto={K.gemm_kernel_name(M, N, Kt, 1 if geglu else 0)}\n   {line}", flush=True)


if __name__ == "__main__":
    main()
