"""Forward+backward time of one motion module (temporal LoRA r=32 on its attention projections, FF / proj / norms
trainable) on the HIP autograd path at the 16x512^2 CFG-free training shapes (train_animatediff.py: B=1 clip,
16 frames; latent 64^2 / 32^2 / 16^2 -> C = 320 / 640 / 1280).  Prints one JSON line per level."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd.autograd import motion_module_train  # noqa: E402
from video_style_transfer_amd.temporal_lora import TemporalLoRALinear  # noqa: E402
from video_style_transfer_amd.unet_motion import MotionModule  # noqa: E402


def build(C, dev):
    mm = MotionModule(C, heads=8)
    blk = mm.transformer_blocks[0]
    for attn in (blk.attn1, blk.attn2):
        attn.to_q, attn.to_k, attn.to_v = (TemporalLoRALinear(l, 32, 1.0) for l in (attn.to_q, attn.to_k, attn.to_v))
        attn.to_out[0] = TemporalLoRALinear(attn.to_out[0], 32, 1.0)
    mm = mm.to(dev)
    for n, p in mm.named_parameters():
        if p.dim() == 2 and "lora_" not in n:
            p.data = p.data.to(torch.bfloat16)
    return mm


def main():
    dev = torch.device("cuda")
    for C, hw in ((320, 64), (640, 32), (1280, 16)):
        mm = build(C, dev)
        nclip, F, HW = 1, 16, hw * hw
        x = torch.randn(nclip * F * HW, C, device=dev).to(torch.bfloat16).requires_grad_(True)
        gy = torch.randn(nclip * F * HW, C, device=dev).to(torch.bfloat16)
        for _ in range(2):
            motion_module_train(mm, x, nclip, F, HW).backward(gy)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 5
        for _ in range(n):
            y = motion_module_train(mm, x, nclip, F, HW)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(n):
            motion_module_train(mm, x, nclip, F, HW).backward(gy)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        fwd = (t1 - t0) / n * 1e3
        tot = (t2 - t1) / n * 1e3
        T = nclip * F * HW
        flops_fwd = 2 * T * C * C * (1 + 1 + 2 * 4) + 2 * T * C * 8 * C + 2 * T * 4 * C * C  # proj, attn qkvo x2, FF
        print(json.dumps({"C": C, "tokens": T, "fwd_ms": round(fwd, 3), "fwd_bwd_ms": round(tot, 3),
                          "bwd_ms": round(tot - fwd, 3), "fwd_tflops": round(flops_fwd / fwd / 1e9, 1)}), flush=True)
        del mm, x, y


if __name__ == "__main__":
    main()
