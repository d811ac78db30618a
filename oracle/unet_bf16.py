"""ORACLE (test infrastructure only): the UNetMotionModel forward of oracle/unet.py -- the same reference semantics,
restated op for op -- in "bf16 emulation": every tensor the MI355X path stores in bf16 is rounded to bf16 at exactly
that boundary, everything between two stores is fp32 (as the kernels' fp32 accumulators and fp32 epilogues are).

Purpose ("Parity ... next best thing"): an fp32 oracle cannot separate "different arithmetic" from
"same arithmetic in bf16", so the HIP path is also gated against this restatement.  What remains between the two is
fp32 reassociation (MFMA accumulation order, online-softmax tiling, fused epilogues), which flips an occasional
bf16 rounding by one ulp.

Boundaries (what the HIP path stores in bf16; kernel names in video_style_transfer_amd/):
  * every GEMM / conv output after its fp32 bias; a fused residual / per-frame temb add is applied to that bf16
    value and rounded again (the reference's separate add), the fused GEGLU multiplies the bf16 h and gate;
  * GroupNorm(+SiLU) and LayerNorm(+sinusoidal PE) outputs;
  * the UnZipLoRA down-projection u = x . Acat^T (vst_layernorm_lora / gemm_skinny), which enters the projection
    GEMM as extra K columns against V = scale * [B_c * m_c | B_s * m_s] rounded to bf16 (lora_linear.build_ops);
  * attention: P = exp(S - max) rounded to bf16 before the P.V product, normalised by the fp32 row sum l; O stored
    bf16; the spatial kernel's online softmax over 64-key tiles is followed step by step (running max, rescale);
  * timestep embeddings, SiLU, the latent pack (scale_model_input) -- all bf16 outputs.
Weights are the bf16 device values (LoRA factors fp32, as the reference keeps them).  Layout: token-major
[(b*F + f)*H*W + p, C], like the device path.

Reference citations: the math of every block is oracle/unet.py's (diffusers ~0.30 semantics for the glue; the
processor animatediff/attention_processor.py:18-96 and UnZipLoRA unziplora_unet/unziplora_linear_layer.py:298-346,
both golden-pinned); this file only adds the rounding points.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from .unet import LoRAState, euler_schedule, timestep_embedding


def q(t: torch.Tensor) -> torch.Tensor:
    """Round to bf16 (round-to-nearest-even) and return fp32."""
    return t.to(torch.bfloat16).float()


# Reassociation probe: with _SPLIT_K on, every contraction (GEMM, conv, attention products) sums its K axis as two
# separately accumulated halves -- the same math with a different fp32 summation order.  The distance between the
# probed and the plain emulation is the bf16-rounding noise floor that fp32 reassociation alone produces on a given
# layer: the yardstick for "the HIP path equals bf16 reference arithmetic up to reassociation".
# The second probe, fp64_accumulation, accumulates every contraction exactly (fp64) before the same bf16 roundings.
_SPLIT_K = False
_FP64 = False


class split_k_reassociation:
    def __enter__(self):
        global _SPLIT_K
        _SPLIT_K = True

    def __exit__(self, *a):
        global _SPLIT_K
        _SPLIT_K = False


class fp64_accumulation:
    def __enter__(self):
        global _FP64
        _FP64 = True

    def __exit__(self, *a):
        global _FP64
        _FP64 = False


def mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b in fp32 (two K halves under split_k_reassociation, fp64 under fp64_accumulation)."""
    k = a.shape[-1]
    if _FP64:
        return (a.double() @ b.double()).float()
    if not _SPLIT_K or k < 2:
        return a @ b
    h = k // 2
    return a[..., :h] @ b[..., :h, :] + a[..., h:] @ b[..., h:, :]


def conv2d(img, w, b, stride):
    """3x3 conv (pad 1) in fp32 as an explicit im2col GEMM: the (channel, ky, kx) patch matrix of F.unfold times the
    flattened weights through mm(), so the split_k_reassociation / fp64_accumulation probes apply to it like to every
    other contraction (the split falls between the two channel halves).  Not F.conv2d: on the GPU that dispatches to
    MIOpen, whose algorithm choice (and so the fp32 summation order) may differ from box to box (VERDICT r5 weak #1,
    lead 2), and the emulation is the yardstick the HIP path is gated against."""
    n, c, H, W = img.shape
    co = w.shape[0]
    OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
    cols = F.unfold(img, 3, padding=1, stride=stride)            # [n, c*9, OH*OW], rows ordered (c, ky, kx)
    y = mm(cols.transpose(1, 2), w.reshape(co, c * 9).t())       # [n, OH*OW, co]
    if b is not None:
        y = y + b
    return y.transpose(1, 2).reshape(n, co, OH, OW)


def _w(P, k):
    return P[k].float()


# ------------------------------------------------------------------------------------ projections
def _lowrank(P, name, lora: LoRAState):
    """(A [R, in], V [out, R]) fp32 of an UnZipLoRA layer under the forward type (unziplora_linear_layer.py:298-346,
    low-rank form of lowrank_factors()), scale folded into V, or None."""
    pre = name + ".lora_layer."
    if lora is None or pre + "lora_matrix_dic.content_down.weight" not in P:
        return None
    ft = lora.forward_type
    As, Vs = [], []
    for key in ("content", "style"):
        if ft not in ("both", key) or lora.masked.get((name, key), False):
            continue
        A = P[pre + f"lora_matrix_dic.{key}_down.weight"].float()
        B = P[pre + f"lora_matrix_dic.{key}_up.weight"].float()
        if ft == "both":
            B = B * P[pre + f"merge_{key}"].float()[:, None]
        As.append(A)
        Vs.append(B * lora.scale)
    if not As:
        return None
    return torch.cat(As, 0), torch.cat(Vs, 1)


def proj(P, names, x, lora: Optional[LoRAState] = None, residual=None, u=None, geglu=False):
    """lora_linear.run_ops(build_ops(names)) in fused mode: [x | u] . [W | V]^T + b (+ residual) with the GEMM
    epilogue's rounding points.
    names share the input x (q/k/v concatenated); u = q(x . Acat^T) unless given (LayerNorm-fused)."""
    Ws, bs, As, Vs = [], [], [], []
    for n in names:
        W = _w(P, n + ".weight")
        Ws.append(W)
        bs.append(P[n + ".bias"].float() if n + ".bias" in P else torch.zeros(W.shape[0], device=W.device))
        lr = _lowrank(P, n, lora)
        As.append(None if lr is None else lr[0])
        Vs.append(None if lr is None else lr[1])
    y = mm(x, torch.cat(Ws, 0).t())
    if any(a is not None for a in As):
        A = q(torch.cat([a for a in As if a is not None], 0))
        if u is None:
            u = q(mm(x, A.t()))
        R = A.shape[0]
        V = torch.zeros(y.shape[1], R, device=y.device)
        o_n = o_r = 0
        for W, v in zip(Ws, Vs):
            if v is not None:
                V[o_n:o_n + W.shape[0], o_r:o_r + v.shape[1]] = v
                o_r += v.shape[1]
            o_n += W.shape[0]
        y = y + mm(u[:, :R], q(V).t())
    y = y + torch.cat(bs)
    if geglu:  # the projection output is staged in bf16, then h * gelu(gate) is rounded again
        h, g = q(y).chunk(2, dim=-1)
        return q(h * F.gelu(g))
    if residual is not None:  # bf16 linear output, then the residual add (the reference's separate add)
        return q(q(y) + residual)
    return q(y)


def lowrank_A(P, names, lora):
    """q(Acat) of the projections sharing an input (the LayerNorm-fused down-projection operand), or None."""
    As = [lr[0] for lr in (_lowrank(P, n, lora) for n in names) if lr is not None]
    return None if not As else q(torch.cat(As, 0))


# ------------------------------------------------------------------------------------ norms
def group_norm(x, nsamples, groups, gamma, beta, eps, silu=False):
    """x [nsamples * rows, C]: statistics per (sample, group) over the sample's rows (vst_groupnorm)."""
    R, C = x.shape
    xs = x.double().view(nsamples, R // nsamples, groups, C // groups)
    mean = xs.mean((1, 3), keepdim=True)
    var = ((xs - mean) ** 2).mean((1, 3), keepdim=True)
    y = ((xs - mean) / torch.sqrt(var + eps)).float().reshape(R, C) * gamma.float() + beta.float()
    return q(F.silu(y) if silu else y)


def layer_norm(x, gamma, beta, eps=1e-5, pe=None):
    y = F.layer_norm(x, (x.shape[-1],), gamma.float(), beta.float(), eps)
    return q(y if pe is None else y + pe)


# ------------------------------------------------------------------------------------ attention
def attention_core(qm, km, vm, heads, nbatch, Nq, Nk, kv_div=1, scale=None, tile=None):
    """softmax(q k^T * scale) v per (batch, head) with bf16 P.  tile=None: one pass with the row max (the temporal
    kernel, F <= 32 frames at once); tile=64: the spatial kernel's online softmax over 64-key tiles -- running max
    m, P = exp(scale (s - m)) rounded to bf16 per tile, o and l rescaled by exp(scale (m_old - m_new))."""
    C = qm.shape[1]
    hd = C // heads
    scale = hd ** -0.5 if scale is None else scale
    qh = qm.view(nbatch, Nq, heads, hd).transpose(1, 2)
    kh = km.view(nbatch // kv_div, Nk, heads, hd).transpose(1, 2).repeat_interleave(kv_div, 0)
    vh = vm.view(nbatch // kv_div, Nk, heads, hd).transpose(1, 2).repeat_interleave(kv_div, 0)
    s = mm(qh, kh.transpose(-1, -2))
    if tile is None:
        p = torch.exp((s - s.amax(-1, keepdim=True)) * scale)
        o = mm(q(p), vh) / p.sum(-1, keepdim=True)
    else:
        m = torch.full(s.shape[:-1] + (1,), -float("inf"), device=s.device)
        l = torch.zeros_like(m)
        o = torch.zeros(s.shape[:-1] + (hd,), device=s.device)
        for k0 in range(0, Nk, tile):
            st = s[..., k0:k0 + tile]
            m_new = torch.maximum(m, st.amax(-1, keepdim=True))
            alpha = torch.exp((m - m_new) * scale)
            p = torch.exp((st - m_new) * scale)
            l = l * alpha + p.sum(-1, keepdim=True)
            o = o * alpha + mm(q(p), vh[..., k0:k0 + tile, :])
            m = m_new
        o = o / l
    return q(o.transpose(1, 2).reshape(nbatch * Nq, C))


def temporal_core(qm, km, vm, heads, nclip, Fr, HW):
    """Frame-axis attention on token rows (b*F + f)*HW + p."""
    C = qm.shape[1]

    def to_seq(t):
        return t.view(nclip, Fr, HW, C).transpose(1, 2).reshape(nclip * HW * Fr, C)
    o = attention_core(to_seq(qm), to_seq(km), to_seq(vm), heads, nclip * HW, Fr, Fr)
    return o.view(nclip, HW, Fr, C).transpose(1, 2).reshape(-1, C)


# ------------------------------------------------------------------------------------ blocks
def basic_block_spatial(P, name, x, nimg, N, enc, frames_per_text, heads, lora):
    """BasicTransformerBlock (unzip_attention.py:113-239) with AnimateDiffAttnProcessor2_0 on both attentions."""
    C = x.shape[1]
    qkv_names = [f"{name}.attn1.{p}" for p in ("to_q", "to_k", "to_v")]
    A = lowrank_A(P, qkv_names, lora)
    n = layer_norm(x, P[name + ".norm1.weight"], P[name + ".norm1.bias"])
    u = None if A is None else q(mm(n, A.t()))
    qkv = proj(P, qkv_names, n, lora, u=u)
    o = attention_core(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], heads, nimg, N, N, tile=64)
    x = proj(P, [name + ".attn1.to_out.0"], o, lora, residual=x)
    qn = [name + ".attn2.to_q"]
    A = lowrank_A(P, qn, lora)
    n = layer_norm(x, P[name + ".norm2.weight"], P[name + ".norm2.bias"])
    u = None if A is None else q(mm(n, A.t()))
    qq = proj(P, qn, n, lora, u=u)
    kv = proj(P, [name + ".attn2.to_k", name + ".attn2.to_v"], enc, lora)   # text K/V once per clip
    L = enc.shape[0] // (nimg // frames_per_text)
    o = attention_core(qq, kv[:, :C], kv[:, C:], heads, nimg, N, L, frames_per_text, tile=64)
    x = proj(P, [name + ".attn2.to_out.0"], o, lora, residual=x)
    n = layer_norm(x, P[name + ".norm3.weight"], P[name + ".norm3.bias"])
    h = proj(P, [name + ".ff.net.0.proj"], n, None, geglu=True)
    return proj(P, [name + ".ff.net.2"], h, None, residual=x)


def transformer2d(P, name, x, nimg, HW, enc, frames_per_text, heads, layers, lora):
    h = group_norm(x, nimg, 32, P[name + ".norm.weight"], P[name + ".norm.bias"], 1e-6)
    h = proj(P, [name + ".proj_in"], h)
    for i in range(layers):
        h = basic_block_spatial(P, f"{name}.transformer_blocks.{i}", h, nimg, HW, enc, frames_per_text, heads, lora)
    return proj(P, [name + ".proj_out"], h, residual=x)


def motion_module(P, name, x, nclip, Fr, HW, heads=8):
    """diffusers AnimateDiffTransformer3D: clip-wide GroupNorm, proj_in, one block (two frame-axis self-attentions
    with the sinusoidal PE added after norm1/norm2), GEGLU FF, proj_out + residual."""
    C = x.shape[1]
    h = group_norm(x, nclip, 32, P[name + ".norm.weight"], P[name + ".norm.bias"], 1e-6)
    h = proj(P, [name + ".proj_in"], h)
    blk = name + ".transformer_blocks.0"
    pe_tab = P[blk + ".pos_embed.pe"].float().reshape(-1, C)[:Fr]
    pe = pe_tab.repeat_interleave(HW, 0).repeat(nclip, 1)        # row (b*F + f)*HW + p -> pe[f]
    for a, nn_ in (("attn1", "norm1"), ("attn2", "norm2")):
        n = layer_norm(h, P[f"{blk}.{nn_}.weight"], P[f"{blk}.{nn_}.bias"], pe=pe)
        qkv = proj(P, [f"{blk}.{a}.{p}" for p in ("to_q", "to_k", "to_v")], n)
        o = temporal_core(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], heads, nclip, Fr, HW)
        h = proj(P, [f"{blk}.{a}.to_out.0"], o, residual=h)
    n = layer_norm(h, P[blk + ".norm3.weight"], P[blk + ".norm3.bias"])
    f = proj(P, [blk + ".ff.net.0.proj"], n, geglu=True)
    h = proj(P, [blk + ".ff.net.2"], f, residual=h)
    return proj(P, [name + ".proj_out"], h, residual=x)


def conv3x3(P, name, x, nimg, H, W, stride=1, upsample=False, row_bias=None, rows_per_bias=1, residual=None):
    """Implicit-GEMM conv on token rows: bf16 weights, fp32 bias / temb row bias / residual epilogue, one rounding."""
    C = x.shape[1]
    img = x.view(nimg, H, W, C).permute(0, 3, 1, 2)
    if upsample:
        img = F.interpolate(img, scale_factor=2.0, mode="nearest")
    y = conv2d(img, _w(P, name + ".weight"), P[name + ".bias"].float(), stride)
    OH, OW = y.shape[-2:]
    y = y.permute(0, 2, 3, 1).reshape(nimg * OH * OW, -1)
    if row_bias is None and residual is None:
        return q(y), OH, OW
    y = q(y)  # bf16 conv output, then the temb / residual adds (one more rounding)
    if row_bias is not None:
        y = y + row_bias.repeat_interleave(rows_per_bias, 0)
    if residual is not None:
        y = y + residual
    return q(y), OH, OW


def resnet(P, name, x, nimg, H, W, temb_row, rows_per_bias, skip=None):
    """ResnetBlock2D: GN+SiLU (over [x | skip]) -> conv1 (+temb) -> GN+SiLU -> conv2 + shortcut."""
    xc = x if skip is None else torch.cat([x, skip], 1)
    h = group_norm(xc, nimg, 32, P[name + ".norm1.weight"], P[name + ".norm1.bias"], 1e-5, silu=True)
    h, _, _ = conv3x3(P, name + ".conv1", h, nimg, H, W, row_bias=temb_row, rows_per_bias=rows_per_bias)
    h = group_norm(h, nimg, 32, P[name + ".norm2.weight"], P[name + ".norm2.bias"], 1e-5, silu=True)
    if name + ".conv_shortcut.weight" in P:
        Wsc = _w(P, name + ".conv_shortcut.weight").reshape(-1, xc.shape[1])
        sc = q(mm(xc, Wsc.t()) + P[name + ".conv_shortcut.bias"].float())
    else:
        sc = xc
    y, _, _ = conv3x3(P, name + ".conv2", h, nimg, H, W, residual=sc)
    return y


def embed(P, cfg, t, text_embeds, time_ids):
    """UNetMotionModel.embed: SiLU(time_embedding(Timesteps(t)) + add_embedding([text_embeds, Timesteps(ids)]))."""
    ch0 = cfg["block_out_channels"][0]
    B = t.shape[0]
    t_in = q(timestep_embedding(t.float(), ch0))
    h = q(F.silu(proj(P, ["time_embedding.linear_1"], t_in)))
    temb = proj(P, ["time_embedding.linear_2"], h)
    tid = q(timestep_embedding(time_ids.float().reshape(-1), cfg["addition_time_embed_dim"]).reshape(B, -1))
    add_in = torch.cat([q(text_embeds.float()), tid], 1)
    h = q(F.silu(proj(P, ["add_embedding.linear_1"], add_in)))
    emb = proj(P, ["add_embedding.linear_2"], h, residual=temb)
    return q(F.silu(emb))


def unet_forward_tokens(P, cfg, x, B, Fr, h, w, emb_silu, enc, lora: LoRAState = None):
    """UNetMotionModel.forward_tokens: x [B*F*h*w, Cin] (bf16 values) -> noise [B*F*h*w, Cout] (bf16 values).
    enc: [B*L, D] text states (bf16 values), shared by the F frames of a clip."""
    lora = lora if lora is not None else LoRAState()
    ch = list(cfg["block_out_channels"])
    nimg = B * Fr
    H, W = h, w
    motion = cfg.get("motion_modules", True)
    mh = cfg.get("motion_num_attention_heads", 8)
    Lb = cfg["layers_per_block"]

    def temb(name):
        return q(mm(emb_silu, _w(P, name + ".time_emb_proj.weight").t()) + P[name + ".time_emb_proj.bias"].float())

    x, _, _ = conv3x3(P, "conv_in", x, nimg, H, W)
    skips = [(x, H, W)]
    for i, bt in enumerate(cfg["down_block_types"]):
        for j in range(Lb):
            nm = f"down_blocks.{i}"
            x = resnet(P, f"{nm}.resnets.{j}", x, nimg, H, W, temb(f"{nm}.resnets.{j}"), Fr * H * W)
            if bt.startswith("CrossAttn"):
                x = transformer2d(P, f"{nm}.attentions.{j}", x, nimg, H * W, enc, Fr, cfg["num_attention_heads"][i],
                                  cfg["transformer_layers_per_block"][i], lora)
            if motion:
                x = motion_module(P, f"{nm}.motion_modules.{j}", x, B, Fr, H * W, mh)
            skips.append((x, H, W))
        if i < len(ch) - 1:
            x, H, W = conv3x3(P, f"down_blocks.{i}.downsamplers.0.conv", x, nimg, H, W, stride=2)
            skips.append((x, H, W))
    x = resnet(P, "mid_block.resnets.0", x, nimg, H, W, temb("mid_block.resnets.0"), Fr * H * W)
    x = transformer2d(P, "mid_block.attentions.0", x, nimg, H * W, enc, Fr, cfg["num_attention_heads"][-1],
                      cfg["transformer_layers_per_block"][-1], lora)
    if cfg.get("use_motion_mid_block", False) and motion:
        x = motion_module(P, "mid_block.motion_modules.0", x, B, Fr, H * W, mh)
    x = resnet(P, "mid_block.resnets.1", x, nimg, H, W, temb("mid_block.resnets.1"), Fr * H * W)
    rtl = list(reversed(cfg["transformer_layers_per_block"]))
    rheads = list(reversed(cfg["num_attention_heads"]))
    for i, bt in enumerate(cfg["up_block_types"]):
        for j in range(Lb + 1):
            s, sh, sw = skips.pop()
            assert (sh, sw) == (H, W)
            nm = f"up_blocks.{i}"
            x = resnet(P, f"{nm}.resnets.{j}", x, nimg, H, W, temb(f"{nm}.resnets.{j}"), Fr * H * W, skip=s)
            if bt.startswith("CrossAttn"):
                x = transformer2d(P, f"{nm}.attentions.{j}", x, nimg, H * W, enc, Fr, rheads[i], rtl[i], lora)
            if motion:
                x = motion_module(P, f"{nm}.motion_modules.{j}", x, B, Fr, H * W, mh)
        if i < len(ch) - 1:
            x, H, W = conv3x3(P, f"up_blocks.{i}.upsamplers.0.conv", x, nimg, H, W, upsample=True)
    x = group_norm(x, nimg, 32, P["conv_norm_out.weight"], P["conv_norm_out.bias"], 1e-5, silu=True)
    x, _, _ = conv3x3(P, "conv_out", x, nimg, H, W)
    return x


def pack(sample, scale=1.0):
    """(B, C, F, h, w) fp32 -> token rows [(b*F + f)*h*w + p, C] rounded to bf16 (vst_pack_latents)."""
    B, C, Fr, h, w = sample.shape
    return q(sample.float().permute(0, 2, 3, 4, 1).reshape(-1, C) * scale)


def unet_forward(P, cfg, sample, timestep, encoder_hidden_states, text_embeds, time_ids, lora: LoRAState = None):
    """UNetMotionModel.forward (inference_animatediff.py:110-121) in bf16 emulation; 5-D in, 5-D fp32 out."""
    B, Cin, Fr, h, w = sample.shape
    dev = sample.device
    t = timestep.float().reshape(-1).to(dev)
    if t.numel() == 1:
        t = t.expand(B)
    emb = embed(P, cfg, t, text_embeds.to(dev), time_ids.to(dev))
    encoder_hidden_states = encoder_hidden_states.to(dev)
    enc = q(encoder_hidden_states.float()).reshape(-1, encoder_hidden_states.shape[-1])
    y = unet_forward_tokens(P, cfg, pack(sample), B, Fr, h, w, emb, enc, lora)
    return y.view(B, Fr, h, w, -1).permute(0, 4, 1, 2, 3)


def denoise(P, cfg, latents, cond, uncond, time_ids, num_steps, guidance, lora=None, steps=None):
    """pipeline.AnimateDiffDenoiser's step (= generate_video's loop, inference_animatediff.py:104-131) in bf16
    emulation: CFG batched as [uncond, cond], fp32 latents, Euler update from the bf16 noise."""
    ts, sigmas, _ = euler_schedule(num_steps)
    lat = latents.float().clone()
    dev = lat.device
    B, Cl, Fr, h, w = lat.shape
    enc = q(torch.cat([uncond[0], cond[0]], 0).float().to(dev))
    pooled = torch.cat([uncond[1], cond[1]], 0).to(dev)
    tids = time_ids.float().reshape(1, -1).repeat(2 * B, 1).to(dev)
    n = num_steps if steps is None else steps
    for i in range(n):
        x = pack(lat, 1.0 / math.sqrt(float(sigmas[i]) ** 2 + 1.0))
        x = torch.cat([x, x], 0)
        emb = embed(P, cfg, ts[i:i + 1].float().to(dev).expand(2 * B), pooled, tids)
        noise = unet_forward_tokens(P, cfg, x, 2 * B, Fr, h, w, emb, enc.reshape(-1, enc.shape[-1]), lora)
        rows = B * Fr * h * w
        u, c = noise[:rows], noise[rows:]
        eps = (u + guidance * (c - u)).view(B, Fr, h, w, Cl).permute(0, 4, 1, 2, 3)
        lat = lat + (sigmas[i + 1] - sigmas[i]) * eps
    return lat
