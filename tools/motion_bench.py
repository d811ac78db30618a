"""Graph-timed fused motion-module attention block vs its four launches at the 64x64-level step shape (CFG pair of
16 frames, C = 320, HW = 4096).  python tools/motion_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

C, HEADS, F, HW, NCLIP = 320, 8, 16, 4096, 2


def graph_us(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    dev = torch.device("cuda")
    T = NCLIP * F * HW
    x = (torch.randn(T, C, device=dev) * 0.7).to(torch.bfloat16)
    gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    pe = torch.randn(32, C, device=dev) * 0.5
    wqkv = (torch.randn(3 * C, C, device=dev) * C ** -0.5).to(torch.bfloat16)
    wo = (torch.randn(C, C, device=dev) * C ** -0.5).to(torch.bfloat16)
    bo = torch.zeros(C, device=dev)
    y = torch.empty_like(x)

    def fused():
        K.motion_attention_block(x, NCLIP, F, HW, HEADS, gamma, beta, 1e-5, pe, wqkv, None, wo, bo, out=y)

    def four():
        n = K.layer_norm(x, gamma, beta, 1e-5, pe=pe, pe_div=HW, pe_mod=F)
        qkv = K.linear(n, wqkv)
        o = K.temporal_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], NCLIP, F, HW, HEADS, C // HEADS)
        K.linear(o, wo, bo, residual=x)

    for _ in range(2):
        print(f"fused {graph_us(fused):.1f} us   four-launch {graph_us(four):.1f} us", flush=True)


if __name__ == "__main__":
    main()
