"""Per-CU operand fetch rate (vst_probe_fetch): LDS-DMA vs buffer loads into VGPRs vs buffer loads + ds_write_b128,
from an L2-resident region, one 512-thread workgroup per CU.  python tools/fetch_probe.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import _lib  # noqa: E402


def main():
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.zeros(4096, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    for mb in (1, 2, 64):
        src = torch.randint(0, 1 << 30, (mb << 18,), dtype=torch.int32, device=dev)
        for mode, name in ((1, "LDS-DMA"), (0, "buffer_load -> VGPR"), (2, "buffer_load + ds_write_b128")):
            for grid in (cus, 2 * cus):
                iters = 4096
                for _ in range(2):
                    assert lib.vst_probe_fetch(mode, ctypes.c_void_p(src.data_ptr()), src.numel() * 4, grid, iters,
                                               ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(st)) == 0
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(5):
                    lib.vst_probe_fetch(mode, ctypes.c_void_p(src.data_ptr()), src.numel() * 4, grid, iters,
                                        ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(st))
                b.record()
                torch.cuda.synchronize()
                ms = a.elapsed_time(b) / 5
                byts = grid * 8 * iters * 1024
                print(f"region {mb:3d} MB  {name:28s} grid {grid:4d}: {ms:8.3f} ms  {byts / ms / 1e6:8.1f} GB/s chip  "
                      f"{byts / ms / 1e6 / cus:6.1f} GB/s per CU", flush=True)


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def mix():
    """vst_probe_mix: per iteration and wave 32 register-operand MFMAs + P one-KiB pieces (LDS-DMA vs buffer_load +
    ds_write_b128); the P = 0 run fixes the clock (2 waves x 32 MFMAs x 16 cycles per SIMD and iteration)."""
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.zeros(4096, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    src = torch.randint(0, 1 << 30, (2 << 18,), dtype=torch.int32, device=dev)  # 2 MB: L2-resident
    iters = 4000

    def run(mode, pc):
        args = (mode, pc, ctypes.c_void_p(src.data_ptr()), src.numel() * 4, cus, iters, ctypes.c_void_p(out.data_ptr()),
                ctypes.c_void_p(st))
        for _ in range(2):
            assert lib.vst_probe_mix(*args) == 0
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            lib.vst_probe_mix(*args)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / 5 * 1e3 / iters  # us per iteration
    base = run(0, 0)
    clk = 1024 / (base * 1e-6) / 1e9  # GHz if the MFMAs alone set the pace
    print(f"mix: MFMA only {base * 1e3:.1f} ns per iteration (=> {clk:.2f} GHz at 1024 SIMD cycles)", flush=True)
    for mode, name in ((1, "LDS-DMA"), (2, "buffer_load + ds_write_b128")):
        for pc in (2, 4, 8):
            t = run(mode, pc)
            extra = (t - base) * 1e-6 * clk * 1e9
            print(f"mix: {name:28s} {pc} pieces/wave/iter: {t * 1e3:.1f} ns per iteration, +{extra:.0f} cycles "
                  f"(+{extra / pc:.0f} per piece per wave; 2 waves per SIMD), "
                  f"{8 * pc * 1024 / (t * 1e-6) / 1e9:.1f} GB/s per CU", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "mix":
    mix()
