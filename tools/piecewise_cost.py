"""What piecewise capture (frame_shard.PiecewiseGraph) costs a denoise step, measured on one GPU: the configs[2] step
captured as ONE HIP graph vs the same step split where a frame-sharded step splits -- three splits per motion module
(the GroupNorm partials all-gather, the to-pixels and the to-frames all-to-all), 46 graphs and 45 no-op host calls --
replayed alternately.  The difference is the graph-boundary cost a sharded step pays on top of its collectives.
python tools/piecewise_cost.py [--steps 20] [--rounds 3]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    from video_style_transfer_amd import unet_motion as UM
    from video_style_transfer_amd.config import UNetMotionConfig
    from video_style_transfer_amd.frame_shard import PiecewiseGraph
    from video_style_transfer_amd.pipeline import AnimateDiffDenoiser
    from video_style_transfer_amd.utils import build_unet
    dev = torch.device("cuda", 0)
    cfg = UNetMotionConfig.sdxl()
    unet = build_unet(cfg, seed=0, lora_rank=8, device=dev)
    den = AnimateDiffDenoiser(unet, 16, 512, 512, device=dev)
    g = torch.Generator().manual_seed(7)
    enc = torch.randn(2, 77, cfg.cross_attention_dim, generator=g)
    pooled = torch.randn(2, cfg.text_embed_dim, generator=g)
    den.set_prompt_embeds(enc[1:], pooled[1:], enc[:1], pooled[:1])
    den.init_latents(seed=42)
    den.capture()
    whole = den.graph

    class Splitter:
        _pw = None
    sp = Splitter()
    orig = UM.MotionModule.run

    def run(self, x, nimg, H, W, ctx):
        if sp._pw is not None:
            sp._pw.collective(lambda: None)  # (GroupNorm partials all-gather)
        y = orig(self, x, nimg, H, W, ctx)
        if sp._pw is not None:
            sp._pw.collective(lambda: None)  # (to-pixels all-to-all)
            sp._pw.collective(lambda: None)  # (to-frames all-to-all)
        return y
    UM.MotionModule.run = run
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    pw = PiecewiseGraph().capture(den._step, [sp], s)
    UM.MotionModule.run = orig

    def timed(g):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps * 1e3
    res = {"one_graph_ms": [], "piecewise_ms": []}
    for g in (whole, pw):
        for _ in range(3):
            g.replay()
    for _ in range(args.rounds):
        res["one_graph_ms"].append(round(timed(whole), 3))
        res["piecewise_ms"].append(round(timed(pw), 3))
    a, b = min(res["one_graph_ms"]), min(res["piecewise_ms"])
    res.update(pieces=pw.num_graphs, host_calls=len(pw.items) - pw.num_graphs, best_one_graph_ms=a,
               best_piecewise_ms=b, overhead_ms=round(b - a, 3), overhead_frac=round((b - a) / a, 4))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
