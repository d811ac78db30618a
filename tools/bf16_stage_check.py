"""Stage-by-stage bf16 parity of one ResnetBlock2D / Transformer2D block (HIP kernel output vs oracle/unet_bf16.py
on the identical bf16 input of that stage): locates where the HIP path departs from bf16-emulated reference math."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import unet_bf16 as E  # noqa: E402
from oracle import unet as O  # noqa: E402
from video_style_transfer_amd import kernels as K  # noqa: E402
from video_style_transfer_amd.config import UNetMotionConfig  # noqa: E402
from video_style_transfer_amd.utils import build_unet  # noqa: E402

dev = torch.device("cuda")
BF = torch.bfloat16


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return f"rel_l2={((a - b).norm() / b.norm()).item():.2e} rel_max={((a - b).abs().max() / b.abs().max()).item():.2e}"


unet = build_unet(UNetMotionConfig.sdxl(), seed=21, lora_rank=8, device=dev)
P = {k: v.detach().float().cpu() for k, v in unet.state_dict().items()}
rb = unet.down_blocks[1].resnets[0]
name = "down_blocks.1.resnets.0"
g = torch.Generator().manual_seed(0)
nimg, H = 4, 32
x = torch.randn(nimg * H * H, 320, generator=g).to(BF)
xd = x.to(dev)
f32 = lambda t: t.detach().float().contiguous()  # noqa: E731
h1 = K.group_norm(xd, nimg, H * H, 32, 1e-5, f32(rb.norm1.weight), f32(rb.norm1.bias), silu=True)
e1 = E.group_norm(x.float(), nimg, 32, P[name + ".norm1.weight"], P[name + ".norm1.bias"], 1e-5, silu=True)
print("GN1+SiLU", rel(h1, e1))
temb = torch.randn(1, 640, generator=g).to(BF).float()
c1 = rb.conv1.run(h1, nimg, H, H, row_bias=temb.to(dev), row_bias_div=nimg * H * H)
ec1, _, _ = E.conv3x3(P, name + ".conv1", h1.float().cpu(), nimg, H, H, row_bias=temb, rows_per_bias=nimg * H * H)
print("conv1+temb", rel(c1, ec1))
c1n = rb.conv1.run(h1, nimg, H, H)
ec1n, _, _ = E.conv3x3(P, name + ".conv1", h1.float().cpu(), nimg, H, H)
print("conv1 (no temb)", rel(c1n, ec1n))
h2 = K.group_norm(c1, nimg, H * H, 32, 1e-5, f32(rb.norm2.weight), f32(rb.norm2.bias), silu=True)
e2 = E.group_norm(c1.float().cpu(), nimg, 32, P[name + ".norm2.weight"], P[name + ".norm2.bias"], 1e-5, silu=True)
print("GN2+SiLU", rel(h2, e2))
sc = rb.conv_shortcut.run(xd)
Wsc = P[name + ".conv_shortcut.weight"].reshape(640, 320)
esc = E.q(x.float() @ Wsc.t() + P[name + ".conv_shortcut.bias"])
print("shortcut", rel(sc, esc))
y = rb.conv2.run(h2, nimg, H, H, residual=sc)
ey, _, _ = E.conv3x3(P, name + ".conv2", h2.float().cpu(), nimg, H, H, residual=sc.float().cpu())
print("conv2+res", rel(y, ey))
# plain GEMM: proj_in of a transformer
t2d = unet.down_blocks[1].attentions[0]
xin = torch.randn(nimg * H * H, 640, generator=g).to(BF)
yp = t2d.proj_in.run(xin.to(dev))
ep = E.proj(P, ["down_blocks.1.attentions.0.proj_in"], xin.float())
print("proj_in GEMM", rel(yp, ep))
# LN
blk = t2d.transformer_blocks[0]
ln = blk.norm3.run(xin.to(dev))
el = E.layer_norm(xin.float(), P["down_blocks.1.attentions.0.transformer_blocks.0.norm3.weight"],
                  P["down_blocks.1.attentions.0.transformer_blocks.0.norm3.bias"])
print("LayerNorm", rel(ln, el))
# attention core
qkv = torch.randn(nimg * H * H, 3 * 640, generator=g).to(BF)
qd = qkv.to(dev)
o = K.spatial_attention(qd[:, :640], qd[:, 640:1280], qd[:, 1280:], nimg, 10, H * H, H * H, 1)
eo = E.attention_core(qkv[:, :640].float(), qkv[:, 640:1280].float(), qkv[:, 1280:].float(), 10, nimg, H * H, H * H,
                      tile=64)
print("spatial attention", rel(o, eo))
# GEGLU
w, b = blk.ff.net[0].geglu_ops()
hg = K.linear(ln, w, b, geglu=True)
eg = E.proj(P, ["down_blocks.1.attentions.0.transformer_blocks.0.ff.net.0.proj"], ln.float().cpu(), geglu=True)
print("GEGLU", rel(hg, eg))
# attn1 full
n, u = blk.norm1.run_lora(xin.to(dev), __import__("video_style_transfer_amd.attention_processor", fromlist=["x"]).input_lora_ops(blk.attn1, True, 1.0))
A = E.lowrank_A(P, [f"down_blocks.1.attentions.0.transformer_blocks.0.attn1.{p}" for p in ("to_q", "to_k", "to_v")], O.LoRAState())
en = E.layer_norm(xin.float(), P["down_blocks.1.attentions.0.transformer_blocks.0.norm1.weight"], P["down_blocks.1.attentions.0.transformer_blocks.0.norm1.bias"])
print("LN(+lora) n", rel(n, en), "u", rel(u[:, :A.shape[0]], E.q(n.float().cpu() @ A.t())))
# ---- motion module pieces: clip-wide GroupNorm, LayerNorm + PE, frame-axis attention, whole module
from video_style_transfer_amd.unet_motion import FwdCtx  # noqa: E402


def motion_stages(mm, mname, C, HW, Fr=16, nclip=1):
    heads = 8
    xm = torch.randn(nclip * Fr * HW, C, generator=g).to(BF)
    gm = K.group_norm(xm.to(dev), nclip, Fr * HW, 32, 1e-6, f32(mm.norm.weight), f32(mm.norm.bias))
    egm = E.group_norm(xm.float(), nclip, 32, P[mname + ".norm.weight"], P[mname + ".norm.bias"], 1e-6)
    print(f"[C={C}] motion GN (clip-wide)", rel(gm, egm))
    tb = mm.transformer_blocks[0]
    pe = f32(tb.pos_embed.pe).view(-1, C)
    lnp = tb.norm1.run(xm.to(dev), pe=pe, pe_div=HW, pe_mod=Fr)
    pe_rows = P[mname + ".transformer_blocks.0.pos_embed.pe"].reshape(-1, C)[:Fr].repeat_interleave(HW, 0).repeat(nclip, 1)
    elnp = E.layer_norm(xm.float(), P[mname + ".transformer_blocks.0.norm1.weight"],
                        P[mname + ".transformer_blocks.0.norm1.bias"], pe=pe_rows)
    print(f"[C={C}] LayerNorm + PE", rel(lnp, elnp))
    qkv = torch.randn(nclip * Fr * HW, 3 * C, generator=g).to(BF)
    qd = qkv.to(dev)
    to = K.temporal_attention(qd[:, :C], qd[:, C:2 * C], qd[:, 2 * C:], nclip, Fr, HW, heads, C // heads)
    eto = E.temporal_core(qkv[:, :C].float(), qkv[:, C:2 * C].float(), qkv[:, 2 * C:].float(), heads, nclip, Fr, HW)
    print(f"[C={C}] temporal attention", rel(to, eto))
    # the block's stages chained on the HIP outputs
    h = tb.norm1.run(gm, pe=pe, pe_div=HW, pe_mod=Fr)
    eh = E.layer_norm(gm.float().cpu(), P[mname + ".transformer_blocks.0.norm1.weight"],
                      P[mname + ".transformer_blocks.0.norm1.bias"], pe=pe_rows)
    print(f"[C={C}] LN+PE on GN output", rel(h, eh))
    from video_style_transfer_amd.lora_linear import build_ops, run_ops
    a1 = tb.attn1
    qkv2 = run_ops(h, build_ops([a1.to_q, a1.to_k, a1.to_v], 1.0))
    eqkv2 = E.proj(P, [f"{mname}.transformer_blocks.0.attn1.{p}" for p in ("to_q", "to_k", "to_v")], h.float().cpu())
    print(f"[C={C}] motion qkv GEMM", rel(qkv2, eqkv2))
    o2 = K.temporal_attention(qkv2[:, :C], qkv2[:, C:2 * C], qkv2[:, 2 * C:], nclip, Fr, HW, heads, C // heads)
    eo2 = E.temporal_core(qkv2[:, :C].float().cpu(), qkv2[:, C:2 * C].float().cpu(), qkv2[:, 2 * C:].float().cpu(),
                          heads, nclip, Fr, HW)
    print(f"[C={C}] temporal attention on real q/k/v", rel(o2, eo2))
    bn = f"{mname}.transformer_blocks.0"
    res = torch.randn(nclip * Fr * HW, C, generator=g).to(BF).to(dev)
    y1 = run_ops(o2, build_ops([a1.to_out[0]], 1.0), residual=res)
    ey1 = E.proj(P, [bn + ".attn1.to_out.0"], o2.float().cpu(), residual=res.float().cpu())
    print(f"[C={C}] to_out + residual", rel(y1, ey1), K.gemm_kernel_name(y1.shape[0], C, C, 0))
    w, b = tb.ff.net[0].geglu_ops()
    ff1 = K.linear(h, w, b, geglu=True)
    eff1 = E.proj(P, [bn + ".ff.net.0.proj"], h.float().cpu(), geglu=True)
    print(f"[C={C}] GEGLU", rel(ff1, eff1), K.gemm_kernel_name(h.shape[0], 8 * C, C, 1))
    ff2 = tb.ff.net[2].run(ff1, residual=res)
    eff2 = E.proj(P, [bn + ".ff.net.2"], ff1.float().cpu(), residual=res.float().cpu())
    print(f"[C={C}] ff.net.2 + residual", rel(ff2, eff2), K.gemm_kernel_name(h.shape[0], C, 4 * C, 0))
    po = mm.proj_out.run(ff2, residual=xm.to(dev))
    epo = E.proj(P, [mname + ".proj_out"], ff2.float().cpu(), residual=xm.float())
    print(f"[C={C}] proj_out + residual", rel(po, epo))
    ctx = FwdCtx(nclip, Fr, None, None, {}, None, None)
    ym = mm.run(xm.to(dev), nclip * Fr, 1, HW, ctx)
    eym = E.motion_module(P, mname, xm.float(), nclip, Fr, HW)
    with E.split_k_reassociation():
        fym = E.motion_module(P, mname, xm.float(), nclip, Fr, HW)
    print(f"[C={C}] motion module (whole)", rel(ym, eym), "floor", rel(fym, eym))


motion_stages(unet.down_blocks[0].motion_modules[0], "down_blocks.0.motion_modules.0", 320, 1024)
