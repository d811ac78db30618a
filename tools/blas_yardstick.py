"""The step's plain GEMM shapes through vst_gemm (the 8-phase / ring kernels, default policy) against torch's
hipBLASLt (F.linear, no bias) on the same operands: a library yardstick, not part of the product path.
python tools/blas_yardstick.py [passes]  -> one line per shape: us per launch and TF/s of each, alternated."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

SHAPES = [  # name, M, N, K (16x512^2 CFG pair: 16^2 level M = 8192, 32^2 32768, 64^2 131072)
    ("out1280", 8192, 1280, 1280), ("ff2_1280", 8192, 1280, 5120), ("qkv1280", 8192, 3840, 1280),
    ("ff1_1280", 8192, 10240, 1280), ("out640", 32768, 640, 640), ("ff2_640", 32768, 640, 2560),
    ("qkv640", 32768, 1920, 640), ("ff1_640", 32768, 5120, 640), ("mproj320", 131072, 320, 320),
    ("mqkv320", 131072, 960, 320), ("mff2_320", 131072, 320, 1280),
]


def timed(fn, iters=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for name, M, N, Kd in SHAPES:
        x = torch.randn(M, Kd, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * Kd
        vs, bl = [], []
        for _ in range(passes):
            vs.append(timed(lambda: K.linear(x, w, None, out=out)))
            bl.append(timed(lambda: torch.nn.functional.linear(x, w)))
        v, b = min(vs), min(bl)
        err = (K.linear(x, w).float() - torch.nn.functional.linear(x, w).float()).abs().max().item()
        print(json.dumps({"shape": name, "M": M, "N": N, "K": Kd, "vst_us": round(v, 1), "blas_us": round(b, 1),
                          "vst_tf": round(fl / v / 1e6, 1), "blas_tf": round(fl / b / 1e6, 1),
                          "kernel": K.gemm_kernel_name(M, N, Kd, 0),
                          "max_abs_diff": err}), flush=True)


if __name__ == "__main__":
    main()
