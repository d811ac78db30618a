"""Spatial / temporal attention kernel timings at the UNet's shapes (16x512^2, CFG batch 2)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

BF = torch.bfloat16
SPATIAL = [("self32", 32, 10, 1024, 1024, 1), ("self16", 32, 20, 256, 256, 1), ("cross32", 32, 10, 1024, 77, 16),
           ("cross16", 32, 20, 256, 77, 16)]
TEMPORAL = [("temp64", 2, 16, 4096, 320), ("temp32", 2, 16, 1024, 640), ("temp16", 2, 16, 256, 1280)]


def timeit(fn, iters=20):
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
    only = sys.argv[1:]  # optional shape names (profiling passes)
    for name, nb, heads, Nq, Nk, kv_div in SPATIAL:
        if only and name not in only:
            continue
        C = heads * 64
        q = torch.randn(nb * Nq, 3 * C, device=dev).to(BF)
        kv = torch.randn(nb // kv_div * Nk, 2 * C, device=dev).to(BF)
        if kv_div == 1:
            qq, kk, vv = q[:, :C], q[:, C:2 * C], q[:, 2 * C:]
        else:
            qq, kk, vv = q[:, :C], kv[:, :C], kv[:, C:]
        out = torch.empty(nb * Nq, C, device=dev, dtype=BF)
        ms = timeit(lambda: K.spatial_attention(qq, kk, vv, nb, heads, Nq, Nk, kv_div, out=out))
        fl = 4.0 * nb * heads * Nq * Nk * 64
        print(json.dumps({"shape": name, "us": round(ms * 1e3, 1), "tflops": round(fl / ms / 1e9, 1)}), flush=True)
    for name, nclip, Fr, HW, C in TEMPORAL:
        if only and name not in only:
            continue
        qkv = torch.randn(nclip * Fr * HW, 3 * C, device=dev).to(BF)
        out = torch.empty(nclip * Fr * HW, C, device=dev, dtype=BF)
        ms = timeit(lambda: K.temporal_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], nclip, Fr, HW, 8, C // 8,
                                                 out=out))
        by = 2.0 * 4 * nclip * Fr * HW * C
        print(json.dumps({"shape": name, "us": round(ms * 1e3, 1), "gbs": round(by / ms / 1e6, 1)}), flush=True)
        dout = torch.randn(nclip * Fr * HW, C, device=dev).to(BF)
        grad = torch.empty(nclip * Fr * HW, 3 * C, device=dev, dtype=BF)
        ms = timeit(lambda: K.temporal_attention_bwd(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], dout, nclip, Fr, HW,
                                                     8, C // 8, out=grad))
        by = 2.0 * 7 * nclip * Fr * HW * C
        print(json.dumps({"shape": name + "_bwd", "us": round(ms * 1e3, 1), "gbs": round(by / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
