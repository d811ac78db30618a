"""Spatial attention vs fp32 torch at the UNet's shapes, with score scales from flat to peaky (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

BF = torch.bfloat16


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for name, nb, heads, Nq, Nk, kv_div in [("self32", 4, 10, 1024, 1024, 1), ("self16", 4, 20, 256, 256, 1),
                                            ("cross32", 4, 10, 1024, 77, 2), ("cross16", 4, 20, 256, 77, 4)]:
        for amp in (1.0, 3.0, 8.0):
            C = heads * 64
            q = (torch.randn(nb * Nq, C, device=dev, generator=g) * amp).to(BF)
            k = (torch.randn(nb // kv_div * Nk, C, device=dev, generator=g) * amp).to(BF)
            v = torch.randn(nb // kv_div * Nk, C, device=dev, generator=g).to(BF)
            out = K.spatial_attention(q, k, v, nb, heads, Nq, Nk, kv_div)
            qf = q.float().view(nb, Nq, heads, 64).transpose(1, 2)
            kf = k.float().view(nb // kv_div, Nk, heads, 64).transpose(1, 2).repeat_interleave(kv_div, 0)
            vf = v.float().view(nb // kv_div, Nk, heads, 64).transpose(1, 2).repeat_interleave(kv_div, 0)
            ref = torch.nn.functional.scaled_dot_product_attention(qf, kf, vf).transpose(1, 2).reshape(nb * Nq, C)
            e = ((out.float() - ref).norm() / ref.norm()).item()
            mx = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            print(f"{name} amp={amp}: rel_l2={e:.2e} rel_max={mx:.2e}", flush=True)


if __name__ == "__main__":
    main()
