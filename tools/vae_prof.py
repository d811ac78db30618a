"""Per-kernel time of the VAE encode inside the configs[4] training step (4 clips x 16 frames at 512^2) and of the
clip decode, from the launch profiler (HIP events around every instrumented launch).  python tools/vae_prof.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import _roofline_from  # noqa: E402
from video_style_transfer_amd import kernels as K  # noqa: E402
from video_style_transfer_amd.config import VAEConfig  # noqa: E402
from video_style_transfer_amd.train import encode_frames  # noqa: E402
from video_style_transfer_amd.vae import build_vae  # noqa: E402


def main():
    dev = torch.device("cuda")
    vae = build_vae(VAEConfig.sdxl(), seed=1, device=dev)
    g = torch.Generator().manual_seed(0)
    frames = (torch.rand(4, 16, 3, 512, 512, generator=g) * 2 - 1).to(dev)
    gen = torch.Generator(device=dev).manual_seed(3)
    encode_frames(vae, frames, gen)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        lat = encode_frames(vae, frames, gen)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 3 * 1e3
    K.profile_launches(True)
    encode_frames(vae, frames, gen)
    rec = K.collect_launches()
    K.profile_launches(False)
    rl, table = _roofline_from(rec, ms)
    print(f"encode 64 frames 512^2: {ms:.1f} ms, {rl['step_flops'] / 1e12:.1f} TF alg -> "
          f"{rl['step_flops'] / (ms * 1e-3) / 1e12:.0f} TF/s; instrumented kernel time "
          f"{rl['event_kernel_time_ms_per_step']:.1f} ms")
    for k, v in list(table.items())[:14]:
        print(f"  {v['event_ms_per_step']:8.2f} ms {v['launches']:4d}x {v['tflops']} TF/s  {k}")
    shapes = {}
    for kind, sym, fl, nb, t, shape in rec:
        key = f"{kind} {shape} {sym}"
        d = shapes.setdefault(key, [0, 0.0, 0.0])
        d[0] += 1
        d[1] += t
        d[2] += fl
    for key, (n, t, fl) in sorted(shapes.items(), key=lambda kv: -kv[1][1])[:14]:
        print(f"  shape {t:8.2f} ms {n:3d}x {fl / (t * 1e-3) / 1e12 if t else 0:7.1f} TF/s  {key}")
    print(tuple(lat.shape))


if __name__ == "__main__":
    main()
