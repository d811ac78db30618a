"""Run a fixed set of kernels on seeded inputs and save the outputs (diagnostic: compare two library builds
bitwise, each in its own process via VST_LIB_AB).  python tools/ab_bitwise.py out.pt | compare a.pt b.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BF = torch.bfloat16


def run(path):
    from video_style_transfer_amd import kernels as K
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s, a=1.0: (torch.randn(*s, device=dev, generator=g) * a).to(BF)  # noqa: E731
    out = {}
    x, w, b = r(8192, 1280), r(3840, 1280, a=0.03), torch.randn(3840, device=dev, generator=g)
    out["gemm_qkv"] = K.linear(x, w, b)
    out["gemm_256"] = K.linear(r(8192, 1312), r(1280, 1312, a=0.03), None, residual=r(8192, 1280))
    q = r(32 * 256, 3 * 1280)
    out["attn_self16"] = K.spatial_attention(q[:, :1280], q[:, 1280:2560], q[:, 2560:], 32, 20, 256, 256, 1)
    kv = r(2 * 77, 2 * 640)
    out["attn_cross32"] = K.spatial_attention(r(32 * 1024, 640), kv[:, :640], kv[:, 640:], 32, 10, 1024, 77, 16)
    out["ln"] = K.layer_norm(r(4096, 640), torch.ones(640, device=dev), torch.zeros(640, device=dev))
    out["ln_lora"] = K.layer_norm_lora(r(4096, 640), torch.ones(640, device=dev), torch.zeros(640, device=dev), 1e-5,
                                       r(48, 640, a=0.05))
    out["silu"] = K.silu(r(1 << 20))
    out["add"] = K.add(r(1 << 20), r(1 << 20, a=1e-3))
    xt = r(2 * 16 * 1024, 3 * 640)
    out["temporal"] = K.temporal_attention(xt[:, :640], xt[:, 640:1280], xt[:, 1280:], 2, 16, 1024, 8, 80)
    out["geglu_p8"] = K.linear(r(8192, 1280), r(10240, 1280, a=0.03), torch.randn(10240, device=dev, generator=g),
                               geglu=True)
    out["geglu_ring"] = K.linear(r(1024, 640), r(2560, 640, a=0.04), torch.randn(2560, device=dev, generator=g),
                                 geglu=True)
    out["conv"] = K.conv3x3(r(8 * 32 * 32, 320), 8, 32, 32, r(640, 9 * 320, a=0.02), None)
    torch.cuda.synchronize()
    torch.save({k: (v[0] if isinstance(v, tuple) else v).cpu() for k, v in out.items()}, path)


def compare(a, b):
    A, B = torch.load(a), torch.load(b)
    for k in A:
        x, y = A[k].float(), B[k].float()
        nd = (A[k].view(torch.int16) != B[k].view(torch.int16)).sum().item() if A[k].dtype == BF else -1
        e = ((x - y).norm() / max(y.norm().item(), 1e-30)).item()
        print(f"{k:14s} differing={nd} of {A[k].numel()} rel_l2={e:.2e}")


if __name__ == "__main__":
    if sys.argv[1] == "compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
