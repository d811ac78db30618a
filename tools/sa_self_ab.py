"""Spatial self-attention kernel variants (VST_SA_SELF, read once per process): time at the 32x32 / 16x16 levels
(CFG batch 2 x 16 frames) and the rel-L2 error against a torch fp32 reference on the same inputs.
Usage (one variant per process): VST_SA_SELF=41 python tools/sa_self_ab.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

BF = torch.bfloat16
SHAPES = [("self32", 32, 10, 1024), ("self16", 32, 20, 256), ("self64_2", 2, 5, 4096)]


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    var = os.environ.get("SA_LABEL", os.environ.get("VST_SA_SELF", "0"))  # SA_LABEL: a build's name (VST_LIB_AB A/B)
    only = sys.argv[1:]
    for name, nb, heads, N in SHAPES:
        if only and name not in only:
            continue
        C = heads * 64
        qkv = (torch.randn(nb * N, 3 * C, generator=g) * float(os.environ.get("SA_GAIN", "1"))).to(dev).to(BF)
        q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
        out = torch.empty(nb * N, C, device=dev, dtype=BF)
        lse = torch.empty(nb * heads * N, device=dev, dtype=torch.float32)
        ms = timeit(lambda: K.spatial_attention(q, k, v, nb, heads, N, N, out=out))
        K.spatial_attention(q, k, v, nb, heads, N, N, out=out, lse=lse)
        torch.cuda.synchronize()
        # fp32 reference on a few batches
        bs = [0, nb - 1]
        err, lerr = 0.0, 0.0
        for b in bs:
            qq = q[b * N:(b + 1) * N].float().view(N, heads, 64).transpose(0, 1)
            kk = k[b * N:(b + 1) * N].float().view(N, heads, 64).transpose(0, 1)
            vv = v[b * N:(b + 1) * N].float().view(N, heads, 64).transpose(0, 1)
            s = qq @ kk.transpose(1, 2) / 8.0
            ref = (torch.softmax(s, -1) @ vv).transpose(0, 1).reshape(N, C)
            o = out[b * N:(b + 1) * N].float()
            err = max(err, ((o - ref).norm() / ref.norm()).item())
            ref_lse = torch.logsumexp(s, -1) * 1.4426950408889634  # [heads, N], log2 domain
            got = lse[b * heads * N:(b + 1) * heads * N].view(heads, N)
            lerr = max(lerr, (got - ref_lse).abs().max().item())
        fl = 4.0 * nb * heads * N * N * 64
        print(json.dumps({"variant": var, "shape": name, "us": round(ms * 1e3, 2), "tflops": round(fl / ms / 1e9, 1),
                          "rel_l2": float("%.3e" % err), "lse_maxabs": float("%.3e" % lerr),
                          "out_hash": int((out.view(torch.int16).long() * torch.arange(1, out.numel() + 1, device=dev)
                                           .view_as(out)).sum().item()),
                          "lse_hash": float(lse.double().sum().item())}), flush=True)


if __name__ == "__main__":
    main()
