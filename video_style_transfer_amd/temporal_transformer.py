"""TemporalTransformer — MI355X-native mirror of animatediff/temporal_transformer.py.

The reference module (PositionalEncoding :6-27, TemporalTransformerBlock :30-76, TemporalTransformer
:79-146) is the repo's own frame-axis transformer: (B, C, F, H, W) -> (B*H*W, F, C) sequences,
+ sinusoidal PE once, N x [LN -> nn.MultiheadAttention -> +res ; LN -> Linear(C,4C) -> GELU ->
Linear(4C,C) -> +res], final LN, back to (B, C, F, H, W).  This mirror keeps the reference's module
tree and parameter names (`pos_encoding.pe`, `blocks.{i}.norm1`, `blocks.{i}.attn.in_proj_weight`,
`blocks.{i}.attn.out_proj`, `blocks.{i}.ffn.{0,3}`, `norm`), so a reference state_dict loads as is.

Execution never leaves the token-major layout [(b*F + f)*H*W + p, C] (bf16) and never permutes:
  vst_pack_latents (5-D -> tokens) ; vst_add_row_table (+ PE[f], PositionalEncoding.forward) ;
  per block: vst_layernorm -> ONE in_proj GEMM (+bias) -> vst_temporal_attention (frame axis read
  with stride H*W, q/k/v read in place from the fused output) -> out_proj GEMM (+bias, residual
  fused) ; vst_layernorm -> ffn.0 GEMM (+bias, GELU epilogue) -> ffn.3 GEMM (+bias, residual fused) ;
  final vst_layernorm -> vst_unpack_tokens (tokens -> 5-D).
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import kernels as K

BF16 = torch.bfloat16


def _cached(p: torch.Tensor, tag: str, fn):
    key = (p.data_ptr(), p._version)
    c = p.__dict__.get(tag)
    if c is None or c[0] != key:
        c = (key, fn(p.detach()))
        p.__dict__[tag] = c
    return c[1]


def _f32(p):
    return _cached(p, "_vst_f32", lambda t: t.float().contiguous())


def _bf16(p):
    return _cached(p, "_vst_bf16", lambda t: t.to(BF16).contiguous())


class PositionalEncoding(nn.Module):
    """temporal_transformer.py:6-27: pe (1, max_len, d), sin on even and cos on odd channels."""

    def __init__(self, d_model: int, max_len: int = 32):
        super().__init__()
        position = torch.arange(max_len).unsqueeze(1)
        div_term = torch.exp(torch.arange(0, d_model, 2) * (-math.log(10000.0) / d_model))
        pe = torch.zeros(1, max_len, d_model)
        pe[0, :, 0::2] = torch.sin(position * div_term)
        pe[0, :, 1::2] = torch.cos(position * div_term)
        self.register_buffer("pe", pe)


class TemporalTransformerBlock(nn.Module):
    """temporal_transformer.py:30-76 (parameter containers; run() is the HIP path)."""

    def __init__(self, channels: int, num_heads: int = 8, dropout: float = 0.0):
        super().__init__()
        self.num_heads = num_heads
        self.norm1 = nn.LayerNorm(channels)
        self.attn = nn.MultiheadAttention(embed_dim=channels, num_heads=num_heads, dropout=dropout, batch_first=True)
        self.norm2 = nn.LayerNorm(channels)
        self.ffn = nn.Sequential(nn.Linear(channels, channels * 4), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(channels * 4, channels), nn.Dropout(dropout))

    def run(self, h, nclip, F, HW):
        """h: [nclip*F*HW, C] tokens -> new [nclip*F*HW, C] tokens."""
        C = h.shape[1]
        n1 = K.layer_norm(h, _f32(self.norm1.weight), _f32(self.norm1.bias), self.norm1.eps)
        qkv = K.linear(n1, _bf16(self.attn.in_proj_weight), _f32(self.attn.in_proj_bias))
        o = K.temporal_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], nclip, F, HW, self.num_heads,
                                 C // self.num_heads)
        h = K.linear(o, _bf16(self.attn.out_proj.weight), _f32(self.attn.out_proj.bias), residual=h)
        n2 = K.layer_norm(h, _f32(self.norm2.weight), _f32(self.norm2.bias), self.norm2.eps)
        f = K.linear(n2, _bf16(self.ffn[0].weight), _f32(self.ffn[0].bias), act="gelu")
        return K.linear(f, _bf16(self.ffn[3].weight), _f32(self.ffn[3].bias), residual=h)


class TemporalTransformer(nn.Module):
    """temporal_transformer.py:79-146.  forward((B, C, F, H, W), num_frames) -> (B, C, F, H, W)."""

    def __init__(self, in_channels: int, num_layers: int = 2, num_heads: int = 8, dropout: float = 0.0):
        super().__init__()
        self.in_channels = in_channels
        self.num_layers = num_layers
        self.pos_encoding = PositionalEncoding(in_channels, max_len=32)
        self.blocks = nn.ModuleList([TemporalTransformerBlock(in_channels, num_heads, dropout)
                                     for _ in range(num_layers)])
        self.norm = nn.LayerNorm(in_channels)

    def run_tokens(self, x, nclip, F, HW):
        """x: [nclip*F*HW, C] bf16 tokens (row (b*F + f)*HW + p) -> output tokens, same layout."""
        max_len = self.pos_encoding.pe.shape[1]
        if F > max_len:
            raise ValueError(f"{F} frames exceed the positional table length {max_len}")
        pe = _f32(self.pos_encoding.pe).view(-1, self.in_channels)
        h = K.add_row_table(x, pe, div=HW, mod=F)
        for blk in self.blocks:
            h = blk.run(h, nclip, F, HW)
        return K.layer_norm(h, _f32(self.norm.weight), _f32(self.norm.bias), self.norm.eps)

    def forward(self, hidden_states: torch.Tensor, num_frames: int = 1) -> torch.Tensor:
        if not hidden_states.is_cuda:
            raise K._lib.VstError("TemporalTransformer: input is on CPU; the HIP path has no CPU fallback")
        B, C, F, H, W = hidden_states.shape
        if C != self.in_channels:
            raise ValueError(f"expected {self.in_channels} channels, got {C}")
        x = torch.empty(B * F * H * W, C, dtype=BF16, device=hidden_states.device)
        K.pack_latents(hidden_states.float().contiguous(), x)
        y = self.run_tokens(x, B, F, H * W)
        out = torch.empty(B, C, F, H, W, dtype=torch.float32, device=hidden_states.device)
        K.unpack_tokens(y, out)
        return out.to(hidden_states.dtype)
