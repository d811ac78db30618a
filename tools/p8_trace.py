"""Per-workgroup phase timeline of the 8-phase GEMM (diagnostics build): entry -> first operands landed (fill),
-> k-loop done (main loop), -> epilogue stores drained.  Build: bash tools/p8_trace.sh (abx/libvst_trace.so with
-DVST_P8_TRACE); run: VST_LIB_AB=abx/libvst_trace.so python tools/p8_trace.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import _lib, kernels as K  # noqa: E402

BF = torch.bfloat16
SHAPES = [  # name, M, N, K1, K2, geglu, residual
    ("out_lora1280", 8192, 1280, 1280, 32, False, True),
    ("qkv_lora1280", 8192, 3840, 1280, 64, False, False),
    ("geglu1280", 8192, 10240, 1280, 0, True, False),
    ("out_lora640", 32768, 640, 640, 32, False, True),
    ("qkv_lora640", 32768, 1920, 640, 64, False, False),
]


def main():
    lib = _lib.load()
    fn = lib.vst_p8_trace_read
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    want = sys.argv[1:]
    abl = int(os.environ.get("VST_GEMM_ABLATE", "0"))
    for name, M, N, K1, K2, geglu, res in SHAPES:
        if want and name not in want:
            continue
        Kt = K1 + K2
        x = torch.randn(M, K1, device=dev, generator=g).to(BF)
        x2 = torch.randn(M, K2, device=dev, generator=g).to(BF) if K2 else None
        w = (torch.randn(N, Kt, device=dev, generator=g) * Kt ** -0.5).to(BF)
        b = torch.randn(N, device=dev, generator=g) * 0.1
        r = torch.randn(M, N // 2 if geglu else N, device=dev, generator=g).to(BF) if res else None
        fl = 2.0 * M * N * Kt
        if not geglu and not abl:  # correctness of this build against fp32 torch on the same bf16 operands
            xc = torch.cat([x, x2], 1) if K2 else x
            ref = xc.float() @ w.float().t() + b
            if res:
                ref = ref.to(BF).float() + r.float()
            out = K.linear(x, w, b, x2=x2, residual=r).float()
            print(f"{name} rel-L2 vs fp32 torch {((out - ref).norm() / ref.norm()).item():.2e}", flush=True)
            del xc, ref, out
        for _ in range(5):
            K.linear(x, w, b, x2=x2, residual=r, geglu=geglu)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            K.linear(x, w, b, x2=x2, residual=r, geglu=geglu)
        e.record()
        e.synchronize()
        us = s.elapsed_time(e) / 20 * 1e3
        # one more launch with a cold-ish L2: flush by writing a 512 MiB buffer first
        junk = torch.empty(256 << 20, dtype=BF, device=dev)
        for cold in ((False,) if abl else (False, True)):
            if cold:
                junk.fill_(1.0)
            torch.cuda.synchronize()
            K.linear(x, w, b, x2=x2, residual=r, geglu=geglu)
            torch.cuda.synchronize()
            nwg = ((M + 255) // 256) * ((N + 255) // 256)
            buf = np.zeros((min(nwg, 8192), 8), dtype=np.uint64)
            assert fn(buf.ctypes.data, buf.shape[0]) == 0
            wall = buf[:, 0::2].astype(np.float64) * 0.01  # 100 MHz -> us
            clk = buf[:, 1::2].astype(np.float64)
            t0 = wall[:, 0].min()
            fill, loop, epi = wall[:, 1] - wall[:, 0], wall[:, 2] - wall[:, 1], wall[:, 3] - wall[:, 2]
            ghz = np.median((clk[:, 3] - clk[:, 0]) / np.maximum(wall[:, 3] - wall[:, 0], 1e-3) / 1e3)
            start = wall[:, 0] - t0
            end = wall[:, 3] - t0
            nk = (Kt + 63) // 64
            ideal_loop = 2 * 256 * 256 * 64 * nk / (2.5e15 / 256) * 1e6
            print(f"abl={abl} {name:14s} {M}x{N}x{Kt} {'cold' if cold else 'warm'} event {us:6.1f}us = {fl / us / 1e6:6.1f}TF  "
                  f"wg={nwg} span {end.max():6.1f}us  start p50/max {np.median(start):5.1f}/{start.max():5.1f}  "
                  f"fill p50/max {np.median(fill):5.2f}/{fill.max():5.2f}  loop p50/max {np.median(loop):5.1f}/{loop.max():5.1f}"
                  f" (ideal {ideal_loop:4.1f})  epi p50/max {np.median(epi):5.2f}/{epi.max():5.2f}  clk {ghz:4.2f}GHz",
                  flush=True)
            if nwg > 256:  # second-round workgroups: when did they start relative to the first round's ends
                order = np.argsort(start)
                late = start[order[256:]]
                print(f"   round-2 start p50 {np.median(late):5.1f}us, first-round end p50 {np.median(end[order[:256]]):5.1f}us",
                      flush=True)
        del junk


if __name__ == "__main__":
    main()
