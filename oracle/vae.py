"""ORACLE (test infrastructure only): SDXL VAE (diffusers AutoencoderKL) encode / decode in fp32 NCHW.

The reference loads the VAE with diffusers (fp32: inference_animatediff.py:164-169, train_animatediff.py:67-72) and
calls `vae.decode(latents / scaling_factor).sample` per frame (inference_animatediff.py:137-144) and
`vae.encode(frames).latent_dist.sample() * scaling_factor` (train_animatediff.py:219-224).  Diffusers is not vendored
and not installed, so this is a restatement of its public semantics (~0.30) -- PARITY UNPINNED for the VAE:
  Encoder: conv_in -> DownEncoderBlock2D* (ResnetBlock2D x layers, Downsample2D(padding=0) = F.pad (0,1,0,1) +
           conv k3 s2 p0) -> UNetMidBlock2D -> GroupNorm -> SiLU -> conv_out (2 x latent)
  Decoder: conv_in -> UNetMidBlock2D -> UpDecoderBlock2D* (ResnetBlock2D x (layers + 1), Upsample2D = nearest 2x +
           conv k3 p1) -> GroupNorm -> SiLU -> conv_out
  UNetMidBlock2D: resnet -> Attention(heads 1, dim_head C, GroupNorm(32, eps 1e-6) on the input, q/k/v/out with
           bias, softmax(q k^T / sqrt(C)) v, residual) -> resnet
  ResnetBlock2D (temb None): GN+SiLU -> conv3x3 -> GN+SiLU -> conv3x3, + (1x1 conv_shortcut if cin != cout)
  AutoencoderKL: encode = quant_conv(encoder(x)) -> DiagonalGaussianDistribution (mean, logvar clamp [-30, 20]);
                 decode = decoder(post_quant_conv(z))
Parameters: a flat dict with the diffusers AutoencoderKL state-dict key names (any dtype; used in fp32).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _p(P, k):
    return P[k].float()


def conv(P, name, x, stride=1, padding=1):
    return F.conv2d(x, _p(P, name + ".weight"), _p(P, name + ".bias"), stride=stride, padding=padding)


def gn(P, name, x, eps=1e-6, groups=32, silu=False):
    y = F.group_norm(x, groups, _p(P, name + ".weight"), _p(P, name + ".bias"), eps)
    return F.silu(y) if silu else y


def resnet(P, name, x):
    h = gn(P, name + ".norm1", x, silu=True)
    h = conv(P, name + ".conv1", h)
    h = gn(P, name + ".norm2", h, silu=True)
    h = conv(P, name + ".conv2", h)
    if name + ".conv_shortcut.weight" in P:
        x = conv(P, name + ".conv_shortcut", x, padding=0)
    return x + h


def attention(P, name, x):
    B, C, H, W = x.shape
    h = gn(P, name + ".group_norm", x).view(B, C, H * W).transpose(1, 2)
    q = F.linear(h, _p(P, name + ".to_q.weight"), _p(P, name + ".to_q.bias"))
    k = F.linear(h, _p(P, name + ".to_k.weight"), _p(P, name + ".to_k.bias"))
    v = F.linear(h, _p(P, name + ".to_v.weight"), _p(P, name + ".to_v.bias"))
    a = torch.softmax(q @ k.transpose(1, 2) / (C ** 0.5), dim=-1) @ v
    o = F.linear(a, _p(P, name + ".to_out.0.weight"), _p(P, name + ".to_out.0.bias"))
    return o.transpose(1, 2).reshape(B, C, H, W) + x


def mid_block(P, name, x):
    x = resnet(P, name + ".resnets.0", x)
    x = attention(P, name + ".attentions.0", x)
    return resnet(P, name + ".resnets.1", x)


def encoder(P, cfg, x):
    ch, n = cfg["block_out_channels"], cfg["layers_per_block"]
    x = conv(P, "encoder.conv_in", x)
    for i in range(len(ch)):
        for j in range(n):
            x = resnet(P, f"encoder.down_blocks.{i}.resnets.{j}", x)
        if i < len(ch) - 1:
            x = conv(P, f"encoder.down_blocks.{i}.downsamplers.0.conv", F.pad(x, (0, 1, 0, 1)), stride=2, padding=0)
    x = mid_block(P, "encoder.mid_block", x)
    x = gn(P, "encoder.conv_norm_out", x, silu=True)
    return conv(P, "encoder.conv_out", x)


def decoder(P, cfg, z):
    ch, n = cfg["block_out_channels"], cfg["layers_per_block"]
    x = conv(P, "decoder.conv_in", z)
    x = mid_block(P, "decoder.mid_block", x)
    for i in range(len(ch)):
        for j in range(n + 1):
            x = resnet(P, f"decoder.up_blocks.{i}.resnets.{j}", x)
        if i < len(ch) - 1:
            x = conv(P, f"decoder.up_blocks.{i}.upsamplers.0.conv", F.interpolate(x, scale_factor=2.0, mode="nearest"))
    x = gn(P, "decoder.conv_norm_out", x, silu=True)
    return conv(P, "decoder.conv_out", x)


def encode_moments(P, cfg, x):
    """quant_conv(encoder(x)): (n, 2*latent, H/2^k, W/2^k)."""
    return conv(P, "quant_conv", encoder(P, cfg, x.float()), padding=0)


def latent_sample(moments, eps=None):
    """DiagonalGaussianDistribution(moments).sample() with the given standard-normal eps (None: the mode)."""
    mean, logvar = moments.chunk(2, dim=1)
    if eps is None:
        return mean
    return mean + torch.exp(0.5 * logvar.clamp(-30.0, 20.0)) * eps


def decode(P, cfg, z):
    """decoder(post_quant_conv(z)) -> (n, 3, 8h, 8w) for z already divided by scaling_factor."""
    return decoder(P, cfg, conv(P, "post_quant_conv", z.float(), padding=0))


def frames_u8(img):
    """inference_animatediff.py:141-143: (x / 2 + 0.5).clamp(0, 1) * 255 -> uint8 (truncation), (n, H, W, 3)."""
    return ((img.float() / 2 + 0.5).clamp(0, 1).permute(0, 2, 3, 1) * 255).to(torch.uint8)
