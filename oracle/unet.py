"""ORACLE (test infrastructure only): UNetMotionModel forward in fp32 NCHW, reference semantics.

Restates, from diffusers ~0.30 public semantics (the library the reference builds its UNet with,
animatediff/utils.py:13-45; not vendored, so PARITY UNPINNED for the glue itself):
  UNetMotionModel.forward, Timesteps/TimestepEmbedding, SDXL text_time add-embedding,
  ResnetBlock2D, Downsample2D, Upsample2D, Transformer2DModel (linear projection),
  BasicTransformerBlock, GEGLU FeedForward, AnimateDiffTransformer3D motion module.
The attention inside runs the reference processor semantics (ref_ops.attn_processor,
animatediff/attention_processor.py:18-96) with the UnZipLoRA delta (ref_ops.unziplora_delta,
unziplora_unet/unziplora_linear_layer.py:298-346) — both pinned by tests/golden fixtures.

Parameters: a flat dict with the diffusers/reference state-dict key names (any dtype; used in fp32).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .ref_ops import attn_processor, lora_compatible_linear, unziplora_delta


def _p(P, k):
    return P[k].float()


def timestep_embedding(t, dim, flip_sin_to_cos=True, shift=0.0):
    """diffusers get_timestep_embedding (max_period 10000, scale 1)."""
    half = dim // 2
    exponent = -math.log(10000) * torch.arange(half, dtype=torch.float32, device=t.device) / (half - shift)
    emb = t.float()[:, None] * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


def linear(P, name, x):
    return F.linear(x, _p(P, name + ".weight"), _p(P, name + ".bias") if name + ".bias" in P else None)


class LoRAState:
    def __init__(self, forward_type="both", scale=1.0, masked=None):
        self.forward_type = forward_type
        self.scale = scale
        self.masked = masked or {}


def proj(P, name, x, lora: LoRAState):
    """LoRACompatibleLinear.forward with an optional UnZipLoRA layer (lora_linear.py:74-81)."""
    W = _p(P, name + ".weight")
    b = _p(P, name + ".bias") if name + ".bias" in P else None
    delta = None
    lk = name + ".lora_layer.lora_matrix_dic.content_down.weight"
    if lora is not None and lk in P:
        pre = name + ".lora_layer."
        delta = unziplora_delta(x, P[pre + "lora_matrix_dic.content_down.weight"],
                                P[pre + "lora_matrix_dic.content_up.weight"], P[pre + "merge_content"],
                                P[pre + "lora_matrix_dic.style_down.weight"], P[pre + "lora_matrix_dic.style_up.weight"],
                                P[pre + "merge_style"], lora.forward_type, lora.masked.get((name, "content"), False),
                                lora.masked.get((name, "style"), False))
    return lora_compatible_linear(x, W, b, delta, lora.scale if lora is not None else 1.0)


def attention(P, name, x, enc, heads, lora):
    def pr(n, t):
        return proj(P, f"{name}.{'to_out.0' if n == 'to_out' else n}", t, lora)

    return attn_processor(x, enc, heads, pr)


def layer_norm(P, name, x, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), _p(P, name + ".weight"), _p(P, name + ".bias"), eps)


def geglu_ff(P, name, x):
    h = linear(P, name + ".net.0.proj", x)
    hidden, gate = h.chunk(2, dim=-1)
    return linear(P, name + ".net.2", hidden * F.gelu(gate))


def basic_block(P, name, x, enc, heads, lora, pe=None):
    """diffusers BasicTransformerBlock (layer_norm); PE added after norm1/norm2 when present."""
    n = layer_norm(P, name + ".norm1", x)
    if pe is not None:
        n = n + pe[:, : n.shape[1]]
    x = attention(P, name + ".attn1", n, None, heads, lora) + x
    n = layer_norm(P, name + ".norm2", x)
    if pe is not None:
        n = n + pe[:, : n.shape[1]]
    x = attention(P, name + ".attn2", n, enc, heads, lora) + x
    n = layer_norm(P, name + ".norm3", x)
    return geglu_ff(P, name + ".ff", n) + x


def transformer2d(P, name, x, enc, heads, layers, lora):
    BF, C, H, W = x.shape
    res = x
    h = F.group_norm(x, 32, _p(P, name + ".norm.weight"), _p(P, name + ".norm.bias"), 1e-6)
    h = h.permute(0, 2, 3, 1).reshape(BF, H * W, C)
    h = linear(P, name + ".proj_in", h)
    for i in range(layers):
        h = basic_block(P, f"{name}.transformer_blocks.{i}", h, enc, heads, lora)
    h = linear(P, name + ".proj_out", h)
    return h.reshape(BF, H, W, C).permute(0, 3, 1, 2) + res


def motion_module(P, name, x, num_frames, heads=8, lora=None):
    """diffusers AnimateDiffTransformer3D: GroupNorm over the 5-D (B,C,F,H,W) tensor."""
    BF, C, H, W = x.shape
    B = BF // num_frames
    res = x
    h = x.reshape(B, num_frames, C, H, W).permute(0, 2, 1, 3, 4)
    h = F.group_norm(h, 32, _p(P, name + ".norm.weight"), _p(P, name + ".norm.bias"), 1e-6)
    h = h.permute(0, 3, 4, 2, 1).reshape(B * H * W, num_frames, C)
    h = linear(P, name + ".proj_in", h)
    blk = name + ".transformer_blocks.0"
    pe = _p(P, blk + ".pos_embed.pe")
    h = basic_block(P, blk, h, None, heads, lora, pe=pe)
    h = linear(P, name + ".proj_out", h)
    h = h.reshape(B, H, W, num_frames, C).permute(0, 3, 4, 1, 2).reshape(BF, C, H, W)
    return h + res


def conv(P, name, x, stride=1):
    return F.conv2d(x, _p(P, name + ".weight"), _p(P, name + ".bias"), stride=stride,
                    padding=P[name + ".weight"].shape[-1] // 2)


def resnet(P, name, x, temb, eps=1e-5):
    """diffusers ResnetBlock2D (default time-embedding norm, output_scale_factor 1)."""
    h = F.silu(F.group_norm(x, 32, _p(P, name + ".norm1.weight"), _p(P, name + ".norm1.bias"), eps))
    h = conv(P, name + ".conv1", h)
    h = h + linear(P, name + ".time_emb_proj", F.silu(temb))[:, :, None, None]
    h = F.silu(F.group_norm(h, 32, _p(P, name + ".norm2.weight"), _p(P, name + ".norm2.bias"), eps))
    h = conv(P, name + ".conv2", h)
    if name + ".conv_shortcut.weight" in P:
        x = conv(P, name + ".conv_shortcut", x)
    return x + h


def unet_forward(P, cfg, sample, timestep, encoder_hidden_states, text_embeds, time_ids, lora: LoRAState = None):
    """UNetMotionModel.forward (called at inference_animatediff.py:110-121), fp32.

    cfg: dict with block_out_channels, down_block_types, up_block_types, layers_per_block,
    transformer_layers_per_block, num_attention_heads, addition_time_embed_dim,
    use_motion_mid_block, motion_num_attention_heads, motion_modules (default True; False = the SDXL
    UNet2DConditionModel forward, sample (B, C, 1, h, w)).
    """
    lora = lora if lora is not None else LoRAState()
    sample = sample.float()
    dev = sample.device  # the restatement runs wherever its inputs live (CPU; torch fp32 on a GPU for big loops)
    encoder_hidden_states, text_embeds, time_ids = (encoder_hidden_states.to(dev), text_embeds.to(dev),
                                                    time_ids.to(dev))
    B, Cin, Fr, h, w = sample.shape
    ch = list(cfg["block_out_channels"])
    t = timestep.float().reshape(-1).to(dev)
    if t.numel() == 1:
        t = t.expand(B)
    t_emb = timestep_embedding(t, ch[0])
    emb = linear(P, "time_embedding.linear_2", F.silu(linear(P, "time_embedding.linear_1", t_emb)))
    tid = timestep_embedding(time_ids.float().reshape(-1), cfg["addition_time_embed_dim"]).reshape(B, -1)
    add = torch.cat([text_embeds.float(), tid], dim=-1)
    aug = linear(P, "add_embedding.linear_2", F.silu(linear(P, "add_embedding.linear_1", add)))
    emb = (emb + aug).repeat_interleave(Fr, dim=0)
    enc = encoder_hidden_states.float().repeat_interleave(Fr, dim=0)
    x = sample.permute(0, 2, 1, 3, 4).reshape(B * Fr, Cin, h, w)
    x = conv(P, "conv_in", x)
    skips = [x]
    L = cfg["layers_per_block"]
    mh = cfg.get("motion_num_attention_heads", 8)
    motion = cfg.get("motion_modules", True)  # False: plain SDXL UNet2DConditionModel (animatediff/utils.py:20)
    for i, bt in enumerate(cfg["down_block_types"]):
        for j in range(L):
            x = resnet(P, f"down_blocks.{i}.resnets.{j}", x, emb)
            if bt.startswith("CrossAttn"):
                x = transformer2d(P, f"down_blocks.{i}.attentions.{j}", x, enc, cfg["num_attention_heads"][i],
                                  cfg["transformer_layers_per_block"][i], lora)
            if motion:
                x = motion_module(P, f"down_blocks.{i}.motion_modules.{j}", x, Fr, mh)
            skips.append(x)
        if i < len(ch) - 1:
            x = conv(P, f"down_blocks.{i}.downsamplers.0.conv", x, stride=2)
            skips.append(x)
    x = resnet(P, "mid_block.resnets.0", x, emb)
    x = transformer2d(P, "mid_block.attentions.0", x, enc, cfg["num_attention_heads"][-1],
                      cfg["transformer_layers_per_block"][-1], lora)
    if cfg.get("use_motion_mid_block", False) and motion:
        x = motion_module(P, "mid_block.motion_modules.0", x, Fr, mh)
    x = resnet(P, "mid_block.resnets.1", x, emb)
    rtl = list(reversed(cfg["transformer_layers_per_block"]))
    rheads = list(reversed(cfg["num_attention_heads"]))
    for i, bt in enumerate(cfg["up_block_types"]):
        for j in range(L + 1):
            x = torch.cat([x, skips.pop()], dim=1)
            x = resnet(P, f"up_blocks.{i}.resnets.{j}", x, emb)
            if bt.startswith("CrossAttn"):
                x = transformer2d(P, f"up_blocks.{i}.attentions.{j}", x, enc, rheads[i], rtl[i], lora)
            if motion:
                x = motion_module(P, f"up_blocks.{i}.motion_modules.{j}", x, Fr, mh)
        if i < len(ch) - 1:
            x = F.interpolate(x, scale_factor=2.0, mode="nearest")
            x = conv(P, f"up_blocks.{i}.upsamplers.0.conv", x)
    x = F.silu(F.group_norm(x, 32, _p(P, "conv_norm_out.weight"), _p(P, "conv_norm_out.bias"), 1e-5))
    x = conv(P, "conv_out", x)
    return x.reshape(B, Fr, -1, h, w).permute(0, 2, 1, 3, 4)


# ------------------------------------------------------------------------------- scheduler
def euler_schedule(num_inference_steps, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012,
                   steps_offset=1):
    """EulerDiscreteScheduler (SDXL scheduler config: scaled_linear betas, 'leading' spacing,
    steps_offset 1, epsilon prediction) — set_timesteps + sigmas; init_noise_sigma = sqrt(max^2+1)."""
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float32) ** 2
    alphas_cumprod = torch.cumprod(1.0 - betas, dim=0)
    step_ratio = num_train_timesteps // num_inference_steps
    timesteps = (torch.arange(0, num_inference_steps) * step_ratio).round().flip(0).double() + steps_offset
    sig_all = ((1 - alphas_cumprod) / alphas_cumprod) ** 0.5
    sig = torch.from_numpy(__import__("numpy").interp(timesteps.numpy(), torch.arange(num_train_timesteps).numpy(),
                                                      sig_all.numpy()))
    sigmas = torch.cat([sig, torch.zeros(1, dtype=sig.dtype)]).float()
    init_noise_sigma = float((sigmas.max() ** 2 + 1) ** 0.5)
    return timesteps.float(), sigmas, init_noise_sigma


def denoise(P, cfg, latents, cond, uncond, time_ids, num_steps, guidance, lora=None, steps=None):
    """generate_video's loop (inference_animatediff.py:104-131) in fp32: CFG as two UNet calls,
    Euler step.  `steps` limits the number of iterations run (for bounded tests)."""
    ts, sigmas, _ = euler_schedule(num_steps)
    lat = latents.float().clone()
    n = num_steps if steps is None else steps
    for i in range(n):
        scaled = lat / ((sigmas[i] ** 2 + 1) ** 0.5)
        t = ts[i:i + 1]
        nu = unet_forward(P, cfg, scaled, t, uncond[0], uncond[1], time_ids, lora)
        nc = unet_forward(P, cfg, scaled, t, cond[0], cond[1], time_ids, lora)
        eps = nu + guidance * (nc - nu)
        lat = lat + (sigmas[i + 1] - sigmas[i]) * eps
    return lat
