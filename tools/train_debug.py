"""Bisect the training-path UNet forward against the inference path, block by block (tiny config)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402
from video_style_transfer_amd import autograd as AG  # noqa: E402
from video_style_transfer_amd.config import UNetMotionConfig  # noqa: E402
from video_style_transfer_amd.temporal_lora import TemporalLoRALinear, inject_temporal_lora  # noqa: E402
from video_style_transfer_amd.unet_motion import FwdCtx  # noqa: E402
from video_style_transfer_amd.utils import build_unet  # noqa: E402
from video_style_transfer_amd.weights import synthetic_state_dict  # noqa: E402

BF = torch.bfloat16
dev = torch.device("cuda")
cfg = UNetMotionConfig.tiny()
sd = synthetic_state_dict(cfg, 0, 4)
unet = build_unet(cfg, state_dict=sd, lora_rank=4, device=dev)
inject_temporal_lora(unet, rank=4, alpha=1.0)
with torch.no_grad():
    for m in unet.modules():
        if isinstance(m, TemporalLoRALinear):
            m.lora_B.normal_(0, 0.05)
B, F, h = 1, 2, 16
g = torch.Generator().manual_seed(2)
enc = torch.randn(B, 77, cfg.cross_attention_dim, generator=g).to(dev, BF)
pooled = torch.randn(B, cfg.text_embed_dim, generator=g).to(dev, BF)
tids = torch.tensor([[128, 128, 0, 0, 128, 128]], dtype=torch.float32, device=dev)
emb = unet.embed(torch.tensor([500.0], device=dev), pooled, tids, B)
ctx = FwdCtx(B, F, emb, enc, {}, None, unet.batched_temb(emb))
temb = ctx.temb
nimg = B * F


def cmp(name, a, b):
    e = ((a.float() - b.float()).norm() / b.float().norm()).item()
    print(f"{name}: rel={e:.3e}", flush=True)


with torch.no_grad():
    H = W = h
    x = torch.randn(nimg * H * W, 64, generator=g).to(dev, BF)
    blk = unet.down_blocks[0]
    res = blk.resnets[0]
    cmp("resnet d0", AG.resnet_train(res, x, nimg, H, W, temb[res], F * H * W), res.run(x, nimg, H, W, ctx))
    mm = blk.motion_modules[0]
    cmp("motion d0", AG.motion_module_train(mm, x, B, F, H * W), mm.run(x, nimg, H, W, ctx))
    cmp("down conv", AG.Conv3x3Fn.apply(x, blk.downsamplers[0].conv, nimg, H, W),
        blk.downsamplers[0].run(x, nimg, H, W)[0])
    blk1 = unet.down_blocks[1]
    H = W = h // 2
    x1 = torch.randn(nimg * H * W, 128, generator=g).to(dev, BF)
    t2 = blk1.attentions[0]
    cmp("t2d d1", AG.transformer2d_train(t2, x1, nimg, H, W, enc.reshape(-1, cfg.cross_attention_dim), F),
        t2.run(x1, nimg, H, W, ctx))
    ub = unet.up_blocks[0]
    H = W = h // 4
    xa = torch.randn(nimg * H * W, 256, generator=g).to(dev, BF)
    sk = torch.randn(nimg * H * W, 256, generator=g).to(dev, BF)
    r0 = ub.resnets[0]
    cmp("resnet u0 cat", AG.resnet_train(r0, AG.CatFn.apply(xa, sk), nimg, H, W, temb[r0], F * H * W),
        r0.run(xa, nimg, H, W, ctx, x2=sk))
    cmp("up conv", AG.Conv3x3Fn.apply(xa, ub.upsamplers[0].conv, nimg, H, W, None, 1, True),
        ub.upsamplers[0].run(xa, nimg, H, W)[0])
    # walk both paths side by side
    xs0 = torch.empty(B * F * h * h, 4, dtype=BF, device=dev)
    K.pack_latents(torch.randn(B, 4, F, h, h, generator=g).to(dev), xs0)
    H = W = h
    e2 = enc.reshape(-1, cfg.cross_attention_dim)
    a = unet.conv_in.run(xs0, nimg, H, W)
    b = AG.Conv3x3Fn.apply(xs0, unet.conv_in, nimg, H, W)
    cmp("conv_in", b, a)
    sa, sb = [(a, H, W)], [(b, H, W)]
    for i, blk in enumerate(unet.down_blocks):
        for j, res in enumerate(blk.resnets):
            a = res.run(a, nimg, H, W, ctx)
            b = AG.resnet_train(res, b, nimg, H, W, temb[res], F * H * W)
            cmp(f"down{i}.res{j}", b, a)
            if blk.attentions is not None:
                a = blk.attentions[j].run(a, nimg, H, W, ctx)
                b = AG.transformer2d_train(blk.attentions[j], b, nimg, H, W, e2, F)
                cmp(f"down{i}.attn{j}", b, a)
            a = blk.motion_modules[j].run(a, nimg, H, W, ctx)
            b = AG.motion_module_train(blk.motion_modules[j], b, B, F, H * W)
            cmp(f"down{i}.motion{j}", b, a)
            sa.append((a, H, W)); sb.append((b, H, W))
        if blk.downsamplers is not None:
            a = blk.downsamplers[0].run(a, nimg, H, W)[0]
            b = AG.Conv3x3Fn.apply(b, blk.downsamplers[0].conv, nimg, H, W)
            H, W = H // 2, W // 2
            cmp(f"down{i}.ds", b, a)
            sa.append((a, H, W)); sb.append((b, H, W))
    mid = unet.mid_block
    a = mid.run(a, nimg, H, W, ctx)
    b = AG.resnet_train(mid.resnets[0], b, nimg, H, W, temb[mid.resnets[0]], F * H * W)
    b = AG.transformer2d_train(mid.attentions[0], b, nimg, H, W, e2, F)
    b = AG.resnet_train(mid.resnets[1], b, nimg, H, W, temb[mid.resnets[1]], F * H * W)
    cmp("mid", b, a)
    for i, blk in enumerate(unet.up_blocks):
        for j, res in enumerate(blk.resnets):
            ska = sa.pop()[0]
            skb = sb.pop()[0]
            a = res.run(a, nimg, H, W, ctx, x2=ska)
            b = AG.resnet_train(res, AG.CatFn.apply(b, skb), nimg, H, W, temb[res], F * H * W)
            cmp(f"up{i}.res{j}", b, a)
            if blk.attentions is not None:
                a = blk.attentions[j].run(a, nimg, H, W, ctx)
                b = AG.transformer2d_train(blk.attentions[j], b, nimg, H, W, e2, F)
                cmp(f"up{i}.attn{j}", b, a)
            a = blk.motion_modules[j].run(a, nimg, H, W, ctx)
            b = AG.motion_module_train(blk.motion_modules[j], b, B, F, H * W)
            cmp(f"up{i}.motion{j}", b, a)
        if blk.upsamplers is not None:
            a = blk.upsamplers[0].run(a, nimg, H, W)[0]
            b = AG.Conv3x3Fn.apply(b, blk.upsamplers[0].conv, nimg, H, W, None, 1, True)
            H, W = 2 * H, 2 * W
            cmp(f"up{i}.us", b, a)
    xs = torch.empty(B * F * h * h, 4, dtype=BF, device=dev)
    K.pack_latents(torch.randn(B, 4, F, h, h, generator=g).to(dev), xs)
    y_tr = AG.unet_train_tokens(unet, xs, B, F, h, h, emb, enc.reshape(-1, cfg.cross_attention_dim))
    y_inf = unet.forward_tokens(xs, B, F, h, h, emb, enc)
    cmp("unet", y_tr, y_inf)
