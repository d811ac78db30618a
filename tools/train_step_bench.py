"""One train_animatediff.py step on one MI355X with the HIP training path (BASELINE configs[4]
on one GPU, no DDP): SDXL UNet + AnimateDiff-SDXL motion modules (synthetic weights), UnZipLoRA r=8 frozen,
temporal LoRA r=32 injected, freeze_spatial_layers; 16x512x512 clip (1 x 16 frames, 64x64 latent); Euler add_noise
x_t = x_0 + sigma * eps (train_animatediff.py:234-236); MSE on eps; backward through unet_train_tokens (every
gradient on HIP kernels); torch AdamW.  Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402
from video_style_transfer_amd.autograd import unet_train_tokens  # noqa: E402
from video_style_transfer_amd.config import UNetMotionConfig  # noqa: E402
from video_style_transfer_amd.temporal_lora import inject_temporal_lora  # noqa: E402
from video_style_transfer_amd.utils import build_unet, freeze_spatial_layers  # noqa: E402

BF = torch.bfloat16


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dev = torch.device("cuda")
    cfg = UNetMotionConfig.sdxl()
    unet = build_unet(cfg, seed=0, lora_rank=8, device=dev)
    n_wrapped = inject_temporal_lora(unet, rank=32, alpha=1.0)
    freeze_spatial_layers(unet)
    params = [p for p in unet.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=1e-5)
    B, F, h = 1, 16, 64
    g = torch.Generator(device="cpu").manual_seed(0)
    x0 = torch.randn(B, 4, F, h, h, generator=g).to(dev)
    enc = torch.randn(B, 77, cfg.cross_attention_dim, generator=g).to(dev, BF)
    pooled = torch.randn(B, cfg.text_embed_dim, generator=g).to(dev, BF)
    tids = torch.tensor([[512, 512, 0, 0, 512, 512]], dtype=torch.float32, device=dev)
    sigma = 5.0

    def step():
        eps = torch.randn_like(x0)
        xt = x0 + sigma * eps
        x = torch.empty(B * F * h * h, 4, dtype=BF, device=dev)
        K.pack_latents(xt.contiguous(), x)
        with torch.no_grad():
            emb = unet.embed(torch.tensor([500.0], device=dev), pooled, tids, B)
        y = unet_train_tokens(unet, x, B, F, h, h, emb, enc.reshape(-1, cfg.cross_attention_dim))
        tgt = eps.permute(0, 2, 3, 4, 1).reshape(-1, 4)
        loss = ((y.float() - tgt) ** 2).mean()
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    loss = step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(json.dumps({"metric": "train step (fwd+bwd+AdamW), 16x512x512 clip, 1 GPU, no DDP", "ms_per_step":
                      round(dt * 1e3, 1), "frames_per_s": round(F / dt, 2), "loss": round(float(loss), 4),
                      "finite": bool(torch.isfinite(loss).item()), "trainable_params": sum(p.numel() for p in params),
                      "temporal_lora_layers": n_wrapped, "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
