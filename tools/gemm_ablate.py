"""Ablation of the ring GEMM main loop (run once per VST_GEMM_ABLATE value: 0 full,
1 no loop DMA, 2 no MFMA, 3 neither).  Prints TF/s-equivalent per (shape, tile)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

BF = torch.bfloat16
SHAPES = [("qkv1280", 8192, 3840, 1344), ("ff2_1280", 8192, 1280, 5120), ("ff2_640", 32768, 640, 2560),
          ("big4k", 4096, 4096, 4096), ("ff1_1280", 8192, 10240, 1280), ("out_lora1280", 8192, 1280, 1312),
          ("proj320", 131072, 320, 320), ("qkv320", 131072, 960, 320), ("ff1_320", 131072, 2560, 320),
          ("ff1_1280_geglu", 8192, 10240, 1280), ("ff1_320_geglu", 131072, 2560, 320),
          ("down1280x32_skinny", 8192, 32, 1280), ("down1280x64_skinny", 8192, 64, 1280),
          ("down640x32_skinny", 32768, 32, 640), ("down640x64_skinny", 32768, 64, 640),
          ("proj1280", 8192, 1280, 1280)]
if os.environ.get("SHAPES"):
    SHAPES = [sh for sh in SHAPES if sh[0] in os.environ["SHAPES"].split()]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda")
    ab = os.environ.get("VST_GEMM_ABLATE", "0")
    for name, M, N, Kd in SHAPES:
        x = torch.randn(M, Kd, device=dev).to(BF)
        w = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).to(BF)
        geglu = name.endswith("_geglu")
        out = torch.empty(M, N // 2 if geglu else N, device=dev, dtype=BF)
        fl = 2.0 * M * N * Kd
        row = {"ablate": ab, "shape": name}
        for t in [int(v) for v in os.environ.get("TILES", "3").split()]:
            K.GEMM_POLICY.update(tile=5 if name.endswith("_skinny") else t, splits=1)
            ms = timeit(lambda: K.linear(x, w, None, out=out, geglu=geglu))
            row[f"t{t}_tf"] = round(fl / ms / 1e9, 1)
            row[f"t{t}_us"] = round(ms * 1e3, 1)
        if ab == "0" and not geglu and not name.endswith("_skinny"):
            ms = timeit(lambda: torch.nn.functional.linear(x, w))
            row["hipblaslt_tf"] = round(fl / ms / 1e9, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
