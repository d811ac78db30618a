"""Isolate the C=256 transformer mismatch (tiny config down_blocks[2].attentions[0])."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402
from video_style_transfer_amd import autograd as AG  # noqa: E402
from video_style_transfer_amd.config import UNetMotionConfig  # noqa: E402
from video_style_transfer_amd.lora_linear import build_ops, run_ops  # noqa: E402
from video_style_transfer_amd.unet_motion import FwdCtx  # noqa: E402
from video_style_transfer_amd.utils import build_unet  # noqa: E402
from video_style_transfer_amd.weights import synthetic_state_dict  # noqa: E402

BF = torch.bfloat16
dev = torch.device("cuda")
cfg = UNetMotionConfig.tiny()
unet = build_unet(cfg, state_dict=synthetic_state_dict(cfg, 0, 4), lora_rank=4, device=dev)
g = torch.Generator().manual_seed(2)
B, F = 1, 2
nimg, H = 2, 4
HW = H * H
enc = torch.randn(B, 77, cfg.cross_attention_dim, generator=g).to(dev, BF)
e2 = enc.reshape(-1, cfg.cross_attention_dim)
pooled = torch.randn(B, cfg.text_embed_dim, generator=g).to(dev, BF)
tids = torch.tensor([[128, 128, 0, 0, 128, 128]], dtype=torch.float32, device=dev)
emb = unet.embed(torch.tensor([500.0], device=dev), pooled, tids, B)
ctx = FwdCtx(B, F, emb, enc, {}, None, unet.batched_temb(emb))


def cmp(name, a, b):
    print(f"{name}: rel={((a.float() - b.float()).norm() / b.float().norm()).item():.3e}", flush=True)


with torch.no_grad():
    for bi, C in ((1, 128), (2, 256)):
        t2 = unet.down_blocks[bi].attentions[0]
        blk = t2.transformer_blocks[0]
        x = torch.randn(nimg * HW, C, generator=g).to(dev, BF)
        cmp(f"C={C} t2d", AG.transformer2d_train(t2, x, nimg, H, H, e2, F), t2.run(x, nimg, H, H, ctx))
        a1, a2 = blk.attn1, blk.attn2
        cmp(f"C={C} qkv", AG.proj_train([a1.to_q, a1.to_k, a1.to_v], x),
            run_ops(x, build_ops([a1.to_q, a1.to_k, a1.to_v], 1.0)))
        cmp(f"C={C} to_out", AG.proj_train([a1.to_out[0]], x), run_ops(x, build_ops([a1.to_out[0]], 1.0)))
        cmp(f"C={C} q2", AG.proj_train([a2.to_q], x), run_ops(x, build_ops([a2.to_q], 1.0)))
        cmp(f"C={C} kv", AG.proj_train([a2.to_k, a2.to_v], e2), run_ops(e2, build_ops([a2.to_k, a2.to_v], 1.0)))
        w, b = blk.ff.net[0].geglu_ops()
        cmp(f"C={C} geglu", AG.GEGLUFn.apply(x, blk.ff.net[0].proj.weight, blk.ff.net[0].proj.bias),
            K.linear(x, w, b, geglu=True))
        n = AG.LayerNormFn.apply(x, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps)
        cmp(f"C={C} ln", n, blk.norm1.run(x))
        heads = a1.heads
        qkv = run_ops(x, build_ops([a1.to_q, a1.to_k, a1.to_v], 1.0))
        inner = qkv.shape[1] // 3
        cmp(f"C={C} sattn", AG.SpatialAttentionFn.apply(qkv[:, :inner], qkv[:, inner:2 * inner], qkv[:, 2 * inner:],
                                                        nimg, heads, HW, HW, 1),
            K.spatial_attention(qkv[:, :inner], qkv[:, inner:2 * inner], qkv[:, 2 * inner:], nimg, heads, HW, HW, 1,
                                scale=0.125))
        print(C, "heads", heads, "inner", inner, "attn2 heads", a2.heads, flush=True)

    # block-level: inference BasicTransformerBlock.run vs the training composition of one block
    t2 = unet.down_blocks[2].attentions[0]
    C = 256
    for bi, blk in enumerate(t2.transformer_blocks):
        x = torch.randn(nimg * HW, C, generator=g).to(dev, BF)
        a1, a2 = blk.attn1, blk.attn2
        ref = blk.run(x, nimg, HW, ctx)
        h = x
        n = AG.LayerNormFn.apply(h, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps)
        qkv = AG.proj_train([a1.to_q, a1.to_k, a1.to_v], n)
        inner = qkv.shape[1] // 3
        o = AG.SpatialAttentionFn.apply(qkv[:, :inner], qkv[:, inner:2 * inner], qkv[:, 2 * inner:], nimg, a1.heads,
                                        HW, HW, 1)
        h1 = AG.AddFn.apply(h, AG.proj_train([a1.to_out[0]], o))
        ref1 = a1(blk.norm1.run(x).view(nimg, HW, C), _vst_residual=x).view(-1, C)
        cmp(f"blk{bi} after attn1 (plain LN path)", h1, ref1)
        nl, u = blk.norm1.run_lora(x, __import__("video_style_transfer_amd.attention_processor", fromlist=["x"]).input_lora_ops(a1, True, 1.0))
        cmp(f"blk{bi} LN vs LN-LoRA y", n, nl)
        u2 = K.linear(n, build_ops([a1.to_q, a1.to_k, a1.to_v], 1.0).a)
        cmp(f"blk{bi} u fused vs skinny", u, u2)
        ref_l = a1(nl.view(nimg, HW, C), _vst_residual=x, _vst_lora_u=u).view(-1, C)
        cmp(f"blk{bi} after attn1 (LN-LoRA path)", h1, ref_l)
