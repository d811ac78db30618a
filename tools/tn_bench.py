"""The training step's weight-gradient shapes: vst_gemm_tn (a^T b over the tokens, no transposes) against the path it
replaces (two vst_transpose launches + the split-K ring GEMM on the transposed operands).  python tools/tn_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

SHAPES = [  # tokens M, N (gradient rows), K (gradient columns): the 4-clip window at 64^2 / 32^2 / 16^2
    (262144, 320, 320), (262144, 2560, 320), (262144, 320, 1280), (65536, 640, 640), (65536, 5120, 640),
    (16384, 1280, 1280), (16384, 10240, 1280), (16384, 1280, 5120), (262144, 32, 320), (262144, 320, 32),
]


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for M, N, Kc in SHAPES:
        a = torch.randn(M, N, generator=g, device=dev).to(torch.bfloat16)
        b = (torch.randn(M, Kc, generator=g, device=dev) * M ** -0.5).to(torch.bfloat16)
        old = lambda: K.linear(K.transpose(a), K.transpose(b))  # noqa: E731
        new = lambda: K.linear_tn(a, b)  # noqa: E731
        t_old, t_new = timeit(old), timeit(new)
        fl = 2.0 * M * N * Kc
        err = ((new().float() - old().float()).norm() / old().float().norm()).item()
        print(f"{M}x{N}x{Kc}: transpose+GEMM {t_old:8.1f} us ({fl / t_old / 1e6:6.0f} TF/s)  gemm_tn {t_new:8.1f} us "
              f"({fl / t_new / 1e6:6.0f} TF/s)  rel_l2 {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
