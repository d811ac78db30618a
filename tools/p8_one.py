"""Isolated 8-phase GEMM launches for counter passes (tools/p8_pmc.sh): each named shape on its production tile
(tile 9 = 256x192 for N = 1280 / 640 / 320 grids, tile 8 = 256x256 otherwise), 20 timed launches, TF/s printed.
python tools/p8_one.py [name ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

BF = torch.bfloat16
SHAPES = {  # name: M, N, K, geglu, tile
    "proj1280": (8192, 1280, 1280, False, 9),
    "ff2_1280": (8192, 1280, 5120, False, 9),
    "geglu1280": (8192, 10240, 1280, True, 8),
    "qkv1280": (8192, 3840, 1280, False, 8),
    "proj320": (131072, 320, 320, False, 9),
    "qkv320_256": (131072, 960, 320, False, 8),
    "qkv320_192": (131072, 960, 320, False, 9),
    "qkv640_256": (32768, 1920, 640, False, 8),
    "qkv640_192": (32768, 1920, 640, False, 9),
    "mqkv1280_256": (8192, 3840, 1280, False, 8),
    "mqkv1280_192": (8192, 3840, 1280, False, 9),
}


def main():
    dev = torch.device("cuda")
    names = sys.argv[1:] or list(SHAPES)
    for name in names:
        M, N, Kd, geglu, tile = SHAPES[name]
        g = torch.Generator(device="cpu").manual_seed(1)
        x = (torch.randn(M, Kd, generator=g) * 0.5).to(BF).to(dev)
        w = (torch.randn(N, Kd, generator=g) * Kd ** -0.5).to(BF).to(dev)
        K.GEMM_POLICY.update(tile=tile, splits=1)
        try:
            for _ in range(3):
                K.linear(x, w, geglu=geglu)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                K.linear(x, w, geglu=geglu)
            e.record()
            torch.cuda.synchronize()
        finally:
            K.GEMM_POLICY.update(tile=0, splits=0)
        us = s.elapsed_time(e) / 20 * 1e3
        print(f"{name} {M}x{N}x{Kd} tile {tile}: {us:.1f} us {2.0 * M * N * Kd / us / 1e6:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
