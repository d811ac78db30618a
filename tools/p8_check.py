"""A/B of the 8-phase GEMM (gemm_p8.hip, tile code 8) against the ring kernel (tile 3) on the denoise path's
projection / GEGLU shapes: bitwise equality of the outputs (same MFMA accumulation order over k) and TF/s,
interleaved in one process.  python tools/p8_check.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

BF = torch.bfloat16
SHAPES = [  # name, M, N, K1, K2 (LoRA cols), geglu, residual, bias
    ("tail_test", 1000, 640, 320, 32, False, True, True),
    ("mm320_qkv", 131072, 960, 320, 0, False, False, False),
    ("mm320_ff1", 131072, 2560, 320, 0, True, False, True),
    ("mm320_ff2", 131072, 320, 1280, 0, False, True, True),
    ("sp640_qkv_lora", 32768, 1920, 640, 64, False, False, False),
    ("sp640_out_lora", 32768, 640, 640, 32, False, True, True),
    ("sp640_ff1", 32768, 5120, 640, 0, True, False, True),
    ("sp640_ff2", 32768, 640, 2560, 0, False, True, True),
    ("sp1280_qkv_lora", 8192, 3840, 1280, 64, False, False, False),
    ("sp1280_out_lora", 8192, 1280, 1280, 32, False, True, True),
    ("sp1280_ff1", 8192, 10240, 1280, 0, True, False, True),
    ("sp1280_ff2", 8192, 1280, 5120, 0, False, True, True),
    ("mm1280_qkv", 8192, 3840, 1280, 0, False, False, False),
]


def run(x, x2, w, b, r, geglu, tile):
    K.GEMM_POLICY["tile"] = tile
    try:
        return K.linear(x, w, b, x2=x2, residual=r, geglu=geglu)
    finally:
        K.GEMM_POLICY["tile"] = 0


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
    ok = True
    for name, M, N, K1, K2, geglu, res, bias in SHAPES:
        Kt = K1 + K2
        x = torch.randn(M, K1, device=dev, generator=g).to(BF)
        x2 = torch.randn(M, K2, device=dev, generator=g).to(BF) if K2 else None
        w = (torch.randn(N, Kt, device=dev, generator=g) * Kt ** -0.5).to(BF)
        b = torch.randn(N, device=dev, generator=g) * 0.1 if bias else None
        r = torch.randn(M, N // 2 if geglu else N, device=dev, generator=g).to(BF) if res else None
        a = run(x, x2, w, b, r, geglu, 3)
        c = run(x, x2, w, b, r, geglu, 8)
        same = torch.equal(a, c)
        ok &= same
        fl = 2.0 * M * N * Kt
        t3 = [timeit(lambda: run(x, x2, w, b, r, geglu, 3)) for _ in range(2)]
        t8 = [timeit(lambda: run(x, x2, w, b, r, geglu, 8)) for _ in range(2)]
        t3, t8 = min(t3), min(t8)
        print(f"{name:16s} M={M:6d} N={N:5d} K={Kt:5d} bitwise={same} "
              f"ring {t3 * 1e3:8.1f} us {fl / t3 / 1e9:7.1f} TF   p8 {t8 * 1e3:8.1f} us {fl / t8 / 1e9:7.1f} TF  "
              f"x{t3 / t8:.3f}" + ("" if same else f"  maxdiff {(a.float() - c.float()).abs().max().item():.3e}"),
              flush=True)
    print("ALL BITWISE EQUAL" if ok else "MISMATCH")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
