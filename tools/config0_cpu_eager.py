"""BASELINE configs[0] ("Single 256x256 latent, 1 SDXL UNet forward (no motion module, no LoRA), PyTorch CPU eager")
read literally: the fp32 oracle UNet2DConditionModel forward on ONE 256x256 latent (2048^2 px, 35.9 TF), CPU eager,
timed on this host's cores (thread count and CPU model printed).  Synthetic weights (conditioned init), as every
config here.  The HIP-vs-emulation parity of the same forward is tests/test_parity_bf16_gpu.py::
test_configs0_sdxl_image_unet_256_latent.

  python tools/config0_cpu_eager.py [latent=256] [threads=min(16, cpus)]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.unet import unet_forward  # noqa: E402
from video_style_transfer_amd.config import UNetMotionConfig  # noqa: E402
from video_style_transfer_amd.weights import synthetic_state_dict  # noqa: E402


def main():
    hw = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    cfg = UNetMotionConfig.sdxl_image()
    sd = synthetic_state_dict(cfg, 24, None)
    g = torch.Generator().manual_seed(36)
    lat = torch.randn(1, 4, 1, hw, hw, generator=g)
    enc = torch.randn(1, 77, cfg.cross_attention_dim, generator=g)
    pooled = torch.randn(1, cfg.text_embed_dim, generator=g)
    tids = torch.tensor([[8.0 * hw, 8.0 * hw, 0, 0, 8.0 * hw, 8.0 * hw]])
    cpu = next((ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")), "?")
    with torch.no_grad():
        t0 = time.perf_counter()
        y = unet_forward(sd, cfg.to_dict(), lat, torch.tensor([901.0]), enc, pooled, tids)
        dt = time.perf_counter() - t0
    print(f"configs[0] CPU eager fp32 SDXL UNet forward, 1 x {hw}x{hw} latent ({8 * hw}^2 px): {dt:.2f} s on "
          f"{threads} threads of {cpu}; output std {y.std():.4f}", flush=True)


if __name__ == "__main__":
    main()
