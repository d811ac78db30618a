"""How chaotic is a synthetic-init family?  (weights.INIT_SCALES)

For the SDXL UNet (UnZipLoRA r=8, F=2) on the fp32 oracle, at a small latent so it runs on the CPU:
  gain      = rel change of the output / rel change of the input, for a 1e-3 relative input perturbation;
  autocast  = rel-L2 of the oracle under torch.autocast(cpu, bf16) from its fp32 run.
A gain >> 1 means single bf16 rounding flips are amplified through the depth of the network, so end-to-end parity
gates on that init measure the init, not the kernels.

  python tools/init_conditioning.py [latent] [legacy|conditioned ...]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.unet import unet_forward  # noqa: E402
from video_style_transfer_amd.config import UNetMotionConfig  # noqa: E402
from video_style_transfer_amd.weights import synthetic_state_dict  # noqa: E402


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def main():
    h = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    inits = sys.argv[2:] or ["legacy", "conditioned"]
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = UNetMotionConfig.sdxl()
    g = torch.Generator().manual_seed(1)
    lat = torch.randn(1, 4, 2, h, h, generator=g)
    enc = torch.randn(1, 77, 2048, generator=g)
    pooled = torch.randn(1, 1280, generator=g)
    tids = torch.tensor([[8. * h, 8 * h, 0, 0, 8 * h, 8 * h]])
    t = torch.tensor([501.0])
    lat2 = lat * (1 + 1e-3 * torch.randn(lat.shape, generator=torch.Generator().manual_seed(9)))
    for init in inits:
        sd = {k: v.float() for k, v in synthetic_state_dict(cfg, 0, 8, dtype=torch.bfloat16, init=init).items()}
        t0 = time.time()
        with torch.no_grad():
            y = unet_forward(sd, cfg.to_dict(), lat, t, enc, pooled, tids)
            y2 = unet_forward(sd, cfg.to_dict(), lat2, t, enc, pooled, tids)
            with torch.autocast("cpu", torch.bfloat16):
                yb = unet_forward(sd, cfg.to_dict(), lat, t, enc, pooled, tids).float()
        print(f"{init:12s} latent {h}x{h}: output std {y.std():.3f}  gain {rel(y2, y) / rel(lat2, lat):6.2f}  "
              f"autocast-vs-fp32 {rel(yb, y):.3e}  ({time.time() - t0:.0f}s)", flush=True)


if __name__ == "__main__":
    main()
