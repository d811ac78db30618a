"""Parameter inventory (diffusers key names) and seeded synthetic weights.

The state-dict layout is exactly what the reference's UNet carries after
`load_unet_with_motion` (animatediff/utils.py:13-45) + `insert_unziplora_to_unet`
(unziplora_unet/utils.py:388-484): diffusers UNetMotionModel names, plus for every spatial
attention projection `...{to_q,to_k,to_v,to_out.0}.lora_layer.lora_matrix_dic.{content,style}_{down,up}.weight`
and `...lora_layer.merge_{content,style}`.  No real checkpoints exist offline, so benchmarks and
parity tests use seeded synthetic weights of this exact architecture.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch

from .config import UNetMotionConfig


def sinusoid_table(dim: int, max_len: int = 32) -> torch.Tensor:
    """diffusers SinusoidalPositionalEmbedding table == reference PositionalEncoding
    (animatediff/temporal_transformer.py:11-21).  Shape (1, max_len, dim)."""
    position = torch.arange(max_len).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, dim, 2) * (-math.log(10000.0) / dim))
    pe = torch.zeros(1, max_len, dim)
    pe[0, :, 0::2] = torch.sin(position * div_term)
    pe[0, :, 1::2] = torch.cos(position * div_term)
    return pe


def _linear(S, name, out_f, in_f, bias=True, kind="w"):
    S[name + ".weight"] = ((out_f, in_f), kind)
    if bias:
        S[name + ".bias"] = ((out_f,), "b")


def _norm(S, name, C):
    S[name + ".weight"] = ((C,), "g")
    S[name + ".bias"] = ((C,), "b")


def _conv(S, name, cout, cin, k=3, kind="w"):
    S[name + ".weight"] = ((cout, cin, k, k), kind)
    S[name + ".bias"] = ((cout,), "b")


def _lora(S, name, in_f, out_f, rank):
    for key in ("content", "style"):
        S[f"{name}.lora_layer.lora_matrix_dic.{key}_down.weight"] = ((rank, in_f), "lora")
        S[f"{name}.lora_layer.lora_matrix_dic.{key}_up.weight"] = ((out_f, rank), "lora")
        S[f"{name}.lora_layer.merge_{key}"] = ((out_f,), "merger")


def _attention(S, name, q_dim, kv_dim, lora_rank=None):
    _linear(S, name + ".to_q", q_dim, q_dim, bias=False)
    _linear(S, name + ".to_k", q_dim, kv_dim, bias=False)
    _linear(S, name + ".to_v", q_dim, kv_dim, bias=False)
    _linear(S, name + ".to_out.0", q_dim, q_dim, bias=True, kind="wo")
    if lora_rank:
        _lora(S, name + ".to_q", q_dim, q_dim, lora_rank)
        _lora(S, name + ".to_k", kv_dim, q_dim, lora_rank)
        _lora(S, name + ".to_v", kv_dim, q_dim, lora_rank)
        _lora(S, name + ".to_out.0", q_dim, q_dim, lora_rank)


def _basic_block(S, name, C, cross_dim, lora_rank=None, temporal=False):
    _norm(S, name + ".norm1", C)
    _attention(S, name + ".attn1", C, C, lora_rank)
    _norm(S, name + ".norm2", C)
    _attention(S, name + ".attn2", C, C if temporal else cross_dim, lora_rank)
    _norm(S, name + ".norm3", C)
    _linear(S, name + ".ff.net.0.proj", 8 * C, C)
    _linear(S, name + ".ff.net.2", C, 4 * C, kind="wo")
    if temporal:
        S[name + ".pos_embed.pe"] = ((1, 32, C), "pe")


def _transformer2d(S, name, C, layers, cross_dim, lora_rank):
    _norm(S, name + ".norm", C)
    _linear(S, name + ".proj_in", C, C)
    for i in range(layers):
        _basic_block(S, f"{name}.transformer_blocks.{i}", C, cross_dim, lora_rank)
    _linear(S, name + ".proj_out", C, C, kind="wo")


def _motion(S, name, C):
    _norm(S, name + ".norm", C)
    _linear(S, name + ".proj_in", C, C)
    _basic_block(S, name + ".transformer_blocks.0", C, None, None, temporal=True)
    _linear(S, name + ".proj_out", C, C, kind="wo")


def _resnet(S, name, cin, cout, temb):
    _norm(S, name + ".norm1", cin)
    _conv(S, name + ".conv1", cout, cin)
    _linear(S, name + ".time_emb_proj", cout, temb)
    _norm(S, name + ".norm2", cout)
    _conv(S, name + ".conv2", cout, cout, kind="wo")
    if cin != cout:
        _conv(S, name + ".conv_shortcut", cout, cin, k=1)


def param_shapes(cfg: UNetMotionConfig, lora_rank: int | None = 8) -> "OrderedDict[str, tuple]":
    """name -> (shape, init kind) for every parameter/buffer of the LoRA-injected UNetMotionModel."""
    S: "OrderedDict[str, tuple]" = OrderedDict()
    ch = cfg.block_out_channels
    T = cfg.time_embed_dim
    _conv(S, "conv_in", ch[0], cfg.in_channels)
    _linear(S, "time_embedding.linear_1", T, ch[0])
    _linear(S, "time_embedding.linear_2", T, T)
    _linear(S, "add_embedding.linear_1", T, cfg.projection_class_embeddings_input_dim)
    _linear(S, "add_embedding.linear_2", T, T)
    out_c = ch[0]
    for i, bt in enumerate(cfg.down_block_types):
        in_c, out_c = out_c, ch[i]
        for j in range(cfg.layers_per_block):
            _resnet(S, f"down_blocks.{i}.resnets.{j}", in_c if j == 0 else out_c, out_c, T)
            if bt.startswith("CrossAttn"):
                _transformer2d(S, f"down_blocks.{i}.attentions.{j}", out_c, cfg.transformer_layers_per_block[i],
                               cfg.cross_attention_dim, lora_rank)
            if cfg.motion_modules:
                _motion(S, f"down_blocks.{i}.motion_modules.{j}", out_c)
        if i < len(ch) - 1:
            _conv(S, f"down_blocks.{i}.downsamplers.0.conv", out_c, out_c)
    C = ch[-1]
    _resnet(S, "mid_block.resnets.0", C, C, T)
    _transformer2d(S, "mid_block.attentions.0", C, cfg.transformer_layers_per_block[-1], cfg.cross_attention_dim,
                   lora_rank)
    if cfg.use_motion_mid_block and cfg.motion_modules:
        _motion(S, "mid_block.motion_modules.0", C)
    _resnet(S, "mid_block.resnets.1", C, C, T)
    rch = list(reversed(ch))
    rtl = list(reversed(cfg.transformer_layers_per_block))
    out_c = rch[0]
    for i, bt in enumerate(cfg.up_block_types):
        prev_c, out_c = out_c, rch[i]
        in_c = rch[min(i + 1, len(ch) - 1)]
        n = cfg.layers_per_block + 1
        for j in range(n):
            skip = in_c if j == n - 1 else out_c
            rin = prev_c if j == 0 else out_c
            _resnet(S, f"up_blocks.{i}.resnets.{j}", rin + skip, out_c, T)
            if bt.startswith("CrossAttn"):
                _transformer2d(S, f"up_blocks.{i}.attentions.{j}", out_c, rtl[i], cfg.cross_attention_dim, lora_rank)
            if cfg.motion_modules:
                _motion(S, f"up_blocks.{i}.motion_modules.{j}", out_c)
        if i < len(ch) - 1:
            _conv(S, f"up_blocks.{i}.upsamplers.0.conv", out_c, out_c)
    _norm(S, "conv_norm_out", ch[0])
    _conv(S, "conv_out", cfg.out_channels, ch[0], kind="wo")
    return S


# Synthetic-init families.  "legacy" (rounds 1-2): unit-gain projections, residual-branch outputs at 0.5/sqrt(fan_in).
# With q and k at unit gain the attention logits have std ~1 before any LoRA delta, and the 70 spatial blocks of the
# SDXL UNet amplify a 1e-3 input perturbation ~47x (F=2, 16x16 latent, fp32 oracle): every end-to-end parity gate
# then measures that chaos instead of the kernels.  "conditioned" (default) keeps the same random streams but sets
# q/k at 0.4/sqrt(fan_in) (softer attention, as trained SDXL heads mostly are) and residual-branch outputs at
# 0.25/sqrt(fan_in): the same perturbation then grows 1.3-1.4x at 16x16 and 32x32 latents, and bf16 autocast lands
# 1.8e-2 / 2.3e-2 from fp32 instead of 4.8e-1 (tools/init_conditioning.py).
INIT_SCALES = {"legacy": {"wo": 0.5, "qk": 1.0}, "conditioned": {"wo": 0.25, "qk": 0.4}}
DEFAULT_INIT = "conditioned"


def _init_value(name, shape, kind, g, device, init=DEFAULT_INIT):
    if kind in ("w", "wo"):
        sc = INIT_SCALES[init]
        fan_in = int(math.prod(shape[1:]))
        gain = sc["wo"] if kind == "wo" else 1.0
        if name.endswith((".to_q.weight", ".to_k.weight")):
            gain *= sc["qk"]
        return torch.randn(shape, generator=g, device=device) * (gain / math.sqrt(fan_in))
    if kind == "b":
        return torch.randn(shape, generator=g, device=device) * 0.02
    if kind == "g":
        return 1.0 + torch.randn(shape, generator=g, device=device) * 0.05
    if kind == "lora":
        r = shape[0] if "_down" in name else shape[1]
        return torch.randn(shape, generator=g, device=device) / r
    if kind == "merger":
        return torch.rand(shape, generator=g, device=device)
    if kind == "pe":
        return sinusoid_table(shape[-1], shape[1]).to(device)
    raise ValueError(kind)


@torch.no_grad()
def init_synthetic_(module, cfg: UNetMotionConfig, seed: int = 0, lora_rank: int | None = 8, init: str = DEFAULT_INIT):
    """Fill an existing (e.g. to_empty'd) module in place, on its own device, with the same
    distributions as synthetic_state_dict (device RNG: values differ from the CPU stream)."""
    sd = module.state_dict()
    dev = next(iter(sd.values())).device
    g = torch.Generator(device=dev).manual_seed(seed)
    for name, (shape, kind) in param_shapes(cfg, lora_rank).items():
        t = sd[name]
        t.copy_(_init_value(name, shape, kind, g, dev, init).to(t.dtype))
    return module


def synthetic_state_dict(cfg: UNetMotionConfig, seed: int = 0, lora_rank: int | None = 8,
                         dtype: torch.dtype = torch.float32, init: str = DEFAULT_INIT) -> "OrderedDict[str, torch.Tensor]":
    """Seeded synthetic weights: linear/conv ~ N(0,1)/sqrt(fan_in) (q/k and the
    residual-branch outputs scaled per INIT_SCALES[init]), biases N(0, 0.02), norm gamma 1+N(0,0.05) / beta N(0,0.02),
    UnZipLoRA A,B ~ N(0, 1/r) (unziplora_linear_layer.py:281-282), mergers ~ U(0,1).
    Values are generated in fp32 on CPU, then rounded to `dtype` (bf16 for the device path; the
    oracle consumes the same bf16-rounded values in fp32)."""
    g = torch.Generator().manual_seed(seed)
    out = OrderedDict()
    for name, (shape, kind) in param_shapes(cfg, lora_rank).items():
        out[name] = _init_value(name, shape, kind, g, "cpu", init).to(dtype)
    return out


def _vae_resnet(S, name, cin, cout):
    _norm(S, name + ".norm1", cin)
    _conv(S, name + ".conv1", cout, cin)
    _norm(S, name + ".norm2", cout)
    _conv(S, name + ".conv2", cout, cout, kind="wo")
    if cin != cout:
        _conv(S, name + ".conv_shortcut", cout, cin, k=1)


def _vae_mid(S, name, C):
    _vae_resnet(S, name + ".resnets.0", C, C)
    a = name + ".attentions.0"
    _norm(S, a + ".group_norm", C)
    for p in ("to_q", "to_k", "to_v"):
        _linear(S, f"{a}.{p}", C, C)
    _linear(S, a + ".to_out.0", C, C, kind="wo")
    _vae_resnet(S, name + ".resnets.1", C, C)


def vae_param_shapes(cfg) -> "OrderedDict[str, tuple]":
    """name -> (shape, init kind) of diffusers AutoencoderKL (encoder / decoder / quant_conv / post_quant_conv)."""
    S: "OrderedDict[str, tuple]" = OrderedDict()
    ch, L, n = cfg.block_out_channels, cfg.latent_channels, cfg.layers_per_block
    _conv(S, "encoder.conv_in", ch[0], cfg.in_channels)
    out_c = ch[0]
    for i in range(len(ch)):
        in_c, out_c = out_c, ch[i]
        for j in range(n):
            _vae_resnet(S, f"encoder.down_blocks.{i}.resnets.{j}", in_c if j == 0 else out_c, out_c)
        if i < len(ch) - 1:
            _conv(S, f"encoder.down_blocks.{i}.downsamplers.0.conv", out_c, out_c)
    _vae_mid(S, "encoder.mid_block", ch[-1])
    _norm(S, "encoder.conv_norm_out", ch[-1])
    _conv(S, "encoder.conv_out", 2 * L, ch[-1])
    _conv(S, "quant_conv", 2 * L, 2 * L, k=1)
    _conv(S, "post_quant_conv", L, L, k=1)
    _conv(S, "decoder.conv_in", ch[-1], L)
    _vae_mid(S, "decoder.mid_block", ch[-1])
    rch = list(reversed(ch))
    out_c = rch[0]
    for i in range(len(ch)):
        prev_c, out_c = out_c, rch[i]
        for j in range(n + 1):
            _vae_resnet(S, f"decoder.up_blocks.{i}.resnets.{j}", prev_c if j == 0 else out_c, out_c)
        if i < len(ch) - 1:
            _conv(S, f"decoder.up_blocks.{i}.upsamplers.0.conv", out_c, out_c)
    _norm(S, "decoder.conv_norm_out", ch[0])
    _conv(S, "decoder.conv_out", cfg.out_channels, ch[0], kind="wo")
    return S


def vae_synthetic_state_dict(cfg, seed: int = 0, dtype: torch.dtype = torch.float32) -> "OrderedDict[str, torch.Tensor]":
    """Seeded synthetic AutoencoderKL weights (same distributions as synthetic_state_dict; no checkpoint offline)."""
    g = torch.Generator().manual_seed(seed)
    return OrderedDict((name, _init_value(name, shape, kind, g, "cpu", "legacy").to(dtype))
                       for name, (shape, kind) in vae_param_shapes(cfg).items())
