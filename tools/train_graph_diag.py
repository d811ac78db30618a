"""Where does a captured TrainStep differ from the eager one?  (diagnostic, GPU)

Runs, from the same starting weights and the same draws: eager step A, eager step B (fresh optimizer), captured step
G; prints for each pair how many trainable elements differ and by how many bf16 ulps, and whether the gradients of
A and B are equal.

  python tools/train_graph_diag.py [tiny|sdxl]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd.config import UNetMotionConfig  # noqa: E402
from video_style_transfer_amd.scheduler import EulerDiscreteScheduler  # noqa: E402
from video_style_transfer_amd.temporal_lora import TemporalLoRALinear, build_spatial_lora_index, \
    inject_temporal_lora  # noqa: E402
from video_style_transfer_amd.train import TrainStep, make_adamw  # noqa: E402
from video_style_transfer_amd.utils import build_unet, freeze_spatial_layers  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "sdxl"
    dev = torch.device("cuda")
    cfg = UNetMotionConfig.sdxl() if which == "sdxl" else UNetMotionConfig.tiny()
    F, h, tr = (16, 64, 32) if which == "sdxl" else (4, 8, 4)
    unet = build_unet(cfg, seed=21, lora_rank=8, device=dev)
    torch.manual_seed(22)
    inject_temporal_lora(unet, rank=tr, alpha=1.0)
    with torch.no_grad():
        for m in unet.modules():
            if isinstance(m, TemporalLoRALinear):
                m.lora_B.normal_(0, 0.02)
    freeze_spatial_layers(unet)
    index = build_spatial_lora_index(unet)
    params = [p for p in unet.parameters() if p.requires_grad]
    g = torch.Generator().manual_seed(6)
    enc = torch.randn(1, 77, cfg.cross_attention_dim, generator=g)
    pooled = torch.randn(1, cfg.text_embed_dim, generator=g)
    lat = torch.randn(1, 4, F, h, h, generator=g).to(dev)
    kw = dict(lambda_orth=1e-4, spatial_index=index, max_grad_norm=0.5, resolution=8 * h, seed=11)
    snap = [p.detach().clone() for p in params]

    def restore():
        with torch.no_grad():
            for p, q in zip(params, snap):
                p.copy_(q)
                p.grad = None

    def eager():
        opt = make_adamw(params, lr=2e-5, capturable=True)
        out = TrainStep(unet, opt, EulerDiscreteScheduler(), **kw)(lat, enc, pooled)
        torch.cuda.synchronize()
        grads = [p.grad.detach().clone() for p in params]
        res = [p.detach().clone() for p in params]
        restore()
        return out, grads, res

    oa, ga, ra = eager()
    ob, gb, rb = eager()
    opt = make_adamw(params, lr=2e-5, capturable=True)
    step = TrainStep(unet, opt, EulerDiscreteScheduler(), **kw)
    step.capture(lat, enc, pooled)
    og = step.replay()
    torch.cuda.synchronize()
    rg = [p.detach().clone() for p in params]

    def cmp(name, x, y):
        n = sum(int((a != b).sum()) for a, b in zip(x, y))
        tot = sum(a.numel() for a in x)
        worst = None
        for (pn, _), a, b in zip([(n_, p) for n_, p in unet.named_parameters() if p.requires_grad], x, y):
            if not torch.equal(a, b):
                worst = pn if worst is None else worst
        print(f"{name}: {n} of {tot} elements differ; first differing tensor {worst}", flush=True)

    print(f"loss A {float(oa['loss'])!r} B {float(ob['loss'])!r} G {float(og['loss'])!r}")
    print(f"gnorm A {float(oa['grad_norm'])!r} B {float(ob['grad_norm'])!r} G {float(og['grad_norm'])!r}")
    cmp("grads A vs B", ga, gb)
    cmp("weights A vs B", ra, rb)
    cmp("weights A vs G", ra, rg)
    cmp("weights B vs G", rb, rg)


if __name__ == "__main__":
    main()
