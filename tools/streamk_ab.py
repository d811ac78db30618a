"""A/B timing of ring GEMM tile choices on the UNet's under-filled shapes: 256x256 vs 192x256
(and stream-K when run with VST_STREAMK=1)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

SHAPES = [("ff2_1280", 8192, 1280, 5120), ("out_lora_1280", 8192, 1280, 1312), ("proj_640", 32768, 640, 640),
          ("ff2_640", 32768, 640, 2560)]


def main():
    dev = torch.device("cuda")
    for name, M, N, Kd in SHAPES:
        x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fn = lambda: K.linear(x, w, b, residual=r, out=out)  # noqa: E731
        for tile in (0, 3, 7):
            K.GEMM_POLICY.update(tile=tile, splits=0)
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                fn()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 20
            print(json.dumps({"streamk_env": os.environ.get("VST_STREAMK", "0"), "shape": name, "tile": tile,
                              "kernel": K.gemm_kernel_name(M, N, Kd, 0), "us": round(ms * 1e3, 1),
                              "tf": round(2 * M * N * Kd / ms / 1e9, 1)}), flush=True)
        K.GEMM_POLICY.update(tile=0, splits=0)


if __name__ == "__main__":
    main()
