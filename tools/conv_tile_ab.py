"""Per-shape A/B of the conv tile configurations (ring 256x256 = 3, 256x160 = 6, auto = 0) on the denoise step's
3x3 conv shapes (16 frames x CFG pair = 32 images), interleaved in one process.  python tools/conv_tile_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

BF = torch.bfloat16
SHAPES = [  # name, nimg, H, W, C1, C2, Cout
    ("c320", 32, 64, 64, 320, 0, 320),
    ("c640", 32, 32, 32, 640, 0, 640),
    ("c1280", 32, 16, 16, 1280, 0, 1280),
    ("cat640_320", 32, 64, 64, 320, 320, 320),
    ("cat1280_640", 32, 32, 32, 640, 640, 640),
]
TILES = [(0, 0), (3, 1), (6, 1)]


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for name, n, H, W, C1, C2, Co in SHAPES:
        x1 = torch.randn(n * H * W, C1, device=dev, generator=g).to(BF)
        x2 = torch.randn(n * H * W, C2, device=dev, generator=g).to(BF) if C2 else None
        Kr = 9 * (C1 + C2)
        w = (torch.randn(Co, Kr, device=dev, generator=g) * Kr ** -0.5).to(BF)
        b = torch.randn(Co, device=dev, generator=g) * 0.1

        def run(t):
            K.GEMM_POLICY["tile"], K.GEMM_POLICY["splits"] = t
            try:
                return K.conv3x3(x1, n, H, W, w, b, x2=x2)
            finally:
                K.GEMM_POLICY["tile"], K.GEMM_POLICY["splits"] = 0, 0
        ref = run((3, 1)).float()
        fl = 2.0 * n * H * W * Co * Kr
        best = {}
        for _ in range(3):
            for t in TILES:
                for _ in range(2):
                    run(t)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    run(t)
                e.record()
                e.synchronize()
                best[t] = min(best.get(t, 1e9), s.elapsed_time(e) / 10 * 1e3)
        errs = {t: ((run(t).float() - ref).norm() / ref.norm()).item() for t in best}
        print(f"{name:12s} M={n * H * W} N={Co} K={Kr}  " + "  ".join(
            f"t{t[0]}:{us:7.1f}us {fl / us / 1e6:6.1f}TF" + ("" if errs[t] < 1e-2 else f"(ERR {errs[t]:.1e})")
            for t, us in best.items()), flush=True)


if __name__ == "__main__":
    main()
