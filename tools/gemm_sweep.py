"""GEMM variant sweep over the UNet's projection/conv shapes (16x512^2, CFG B=2).

python tools/gemm_sweep.py  -> one line per (shape, variant): TF/s, plus torch.matmul (hipBLASLt)
as a library yardstick for the plain GEMMs.  Used to tune the tile/split heuristic in gemm.hip.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

BF = torch.bfloat16
SHAPES = [
    # (name, M, N, K, K2(lora cols) , geglu)
    ("mm320_proj", 131072, 320, 320, 0, False),
    ("mm320_qkv", 131072, 960, 320, 0, False),
    ("mm320_ff1", 131072, 2560, 320, 0, True),
    ("mm320_ff2", 131072, 320, 1280, 0, False),
    ("sp640_qkv_lora", 32768, 1920, 640, 64, False),
    ("sp640_lora_down", 32768, 64, 640, 0, False),
    ("sp640_out_lora", 32768, 640, 640, 32, False),
    ("sp640_proj", 32768, 640, 640, 0, False),
    ("sp640_ff1", 32768, 5120, 640, 0, True),
    ("sp640_ff2", 32768, 640, 2560, 0, False),
    ("sp1280_qkv_lora", 8192, 3840, 1280, 64, False),
    ("sp1280_lora_down", 8192, 64, 1280, 0, False),
    ("sp1280_out_lora", 8192, 1280, 1280, 32, False),
    ("sp1280_proj", 8192, 1280, 1280, 0, False),
    ("sp1280_ff1", 8192, 10240, 1280, 0, True),
    ("sp1280_ff2", 8192, 1280, 5120, 0, False),
    ("text_kv_lora", 154, 2560, 2048, 64, False),
    ("text_lora_down", 154, 64, 2048, 0, False),
    ("temb", 2, 13760, 1280, 0, False),
    ("mm640_qkv", 32768, 1920, 640, 0, False),
    ("mm1280_qkv", 8192, 3840, 1280, 0, False),
]
CONVS = [
    # (name, nimg, H, W, Cin, Cout, stride, up, C2)
    ("conv320", 32, 64, 64, 320, 320, 1, False, 0),
    ("conv640", 32, 32, 32, 640, 640, 1, False, 0),
    ("conv1280", 32, 16, 16, 1280, 1280, 1, False, 0),
    ("conv_up2560", 32, 16, 16, 1280, 1280, 1, False, 1280),
    ("conv_up960", 32, 64, 64, 640, 320, 1, False, 320),
    ("down320", 32, 64, 64, 320, 320, 2, False, 0),
    ("up1280", 32, 16, 16, 1280, 1280, 1, True, 0),
]


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
    variants = [(0, 0), (1, 1), (2, 1), (3, 1), (4, 1), (6, 1), (7, 1), (3, 2)]
    res = []
    for name, M, N, Kd, K2, geglu in SHAPES:
        x = torch.randn(M, Kd, device=dev).to(BF)
        x2 = torch.randn(M, K2, device=dev).to(BF) if K2 else None
        w = (torch.randn(N, Kd + K2, device=dev) / (Kd ** 0.5)).to(BF)
        b = torch.randn(N, device=dev)
        fl = 2.0 * M * N * (Kd + K2)
        row = {"shape": name, "M": M, "N": N, "K": Kd + K2}
        for t, s in variants:
            if geglu and t in (2, 6):
                continue
            K.GEMM_POLICY.update(tile=t, splits=s)
            try:
                ms = timeit(lambda: K.linear(x, w, b, x2=x2, geglu=geglu))
                row[f"t{t}s{s}"] = round(fl / ms / 1e9, 1)
            except Exception as ex:  # noqa
                row[f"t{t}s{s}"] = str(ex)[:40]
        K.GEMM_POLICY.update(tile=0, splits=0)
        if not geglu and not os.environ.get("NO_BLAS"):
            xx = torch.cat([x, x2], 1) if x2 is not None else x
            ms = timeit(lambda: torch.nn.functional.linear(xx, w, None))
            row["hipblaslt"] = round(fl / ms / 1e9, 1)
        print(json.dumps(row), flush=True)
        res.append(row)
    for name, n, H, W, Ci, Co, st, up, C2 in CONVS:
        x = torch.randn(n * H * W, Ci, device=dev).to(BF)
        x2 = torch.randn(n * H * W, C2, device=dev).to(BF) if C2 else None
        w = (torch.randn(Co, 9 * (Ci + C2), device=dev) / 50).to(BF)
        b = torch.randn(Co, device=dev)
        OH = 2 * H if up else (H // st)
        fl = 2.0 * n * OH * OH * Co * 9 * (Ci + C2)
        row = {"shape": name}
        for t, s in variants:
            K.GEMM_POLICY.update(tile=t, splits=s)
            ms = timeit(lambda: K.conv3x3(x, n, H, W, w, b, x2=x2, stride=st, upsample=up))
            row[f"t{t}s{s}"] = round(fl / ms / 1e9, 1)
        K.GEMM_POLICY.update(tile=0, splits=0)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
