"""Isolated launches of two 8-phase GEMMs for SQ counter passes: the 16^2 out-projection + UnZipLoRA
(8192x1280x1312, residual; one round of 224 256x192 tiles) and the 16^2 GEGLU (8192x10240x1280, persistent 256x256).
python tools/sq_gemm.py  (under rocprofv3 --pmc ...)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    M, N, Kd = 8192, 1280, 1280
    x = torch.randn(M, Kd, device=dev, generator=g).to(torch.bfloat16)
    r = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    b = torch.randn(N, device=dev, generator=g) * 0.1
    w = (torch.randn(N, Kd + 32, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
    a = torch.zeros(32, Kd, device=dev)
    a[:16] = torch.randn(16, Kd, device=dev, generator=g) * Kd ** -0.5
    a = a.to(torch.bfloat16)
    wg = (torch.randn(10240, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
    bg = torch.randn(10240, device=dev, generator=g) * 0.1
    for _ in range(10):
        K.linear_lora(x, w, a, N, 16, b, residual=r)
        K.linear(x, wg, bg, geglu=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
