"""The VAE's Cout = 128 / 256 / 512 3x3 convs on the tile the library picks vs forced ring tiles (256x128 = tile 4,
256x256 = tile 3): us per launch and whether the outputs are bit-identical.  python tools/vae_conv_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

SHAPES = [  # nimg, H, W, Cin, Cout (the SDXL VAE encoder at 512^2, 4-frame chunks; the decoder's 512^2 up block)
    (4, 512, 512, 128, 128), (4, 256, 256, 256, 256), (4, 128, 128, 256, 256), (4, 64, 64, 512, 512),
    (4, 512, 512, 256, 128),
]
if os.environ.get("VST_CONV_AB") == "unet":  # the denoise step's UNet convs (CFG pair x 16 frames = 32 images)
    SHAPES = [(32, 64, 64, 320, 320), (32, 32, 32, 640, 640), (32, 16, 16, 1280, 1280), (32, 32, 32, 320, 640)]
TILES = (("auto", 0), ("ring256x128", 4), ("ring256x256", 3), ("auto", 0))
if os.environ.get("VST_CONV_AB") == "unet":
    TILES = (("auto", 0), ("ring256x160", 6), ("ring256x256", 3), ("ring256x128", 4), ("auto", 0))


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for n, H, W, ci, co in SHAPES:
        x = torch.randn(n * H * W, ci, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(co, 9 * ci, device=dev, generator=g) * (9 * ci) ** -0.5).to(torch.bfloat16)
        b = torch.randn(co, device=dev, generator=g) * 0.1
        res = {}
        outs = {}
        for name, tile in TILES:
            K.GEMM_POLICY.update(tile=tile, splits=1 if tile else 0)
            try:
                for _ in range(2):
                    y = K.conv3x3(x, n, H, W, w, b)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    y = K.conv3x3(x, n, H, W, w, b)
                e.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(e) / 10 * 1e3
                sym = K.gemm_kernel_name(n * H * W, co, w.shape[1], 2)
            finally:
                K.GEMM_POLICY.update(tile=0, splits=0)
            res[name] = min(res.get(name, 1e12), us)
            outs[name] = y.clone()
            print(f"  {name:12s} {sym}: {us:.1f} us", flush=True)
        fl = 2.0 * n * H * W * co * 9 * ci
        same = all(torch.equal(outs["auto"], o) for o in outs.values())
        print(f"conv {n}x{H}x{W} {ci}->{co}: " + ", ".join(f"{k} {v:.1f} us ({fl / v / 1e6:.0f} TF/s)"
                                                          for k, v in res.items()) + f"; bit-identical {same}",
              flush=True)


if __name__ == "__main__":
    main()
