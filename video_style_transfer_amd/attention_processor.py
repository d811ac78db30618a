"""Attention module + processors — the plug-in surface the reference swaps.

* `Attention`: the attributes/methods diffusers' Attention exposes to processors
  (heads, to_q/to_k/to_v/to_out, norm_cross, spatial_norm, group_norm, residual_connection,
  rescale_output_factor, prepare_attention_mask, set_processor/processor).
* `AnimateDiffAttnProcessor2_0`: same call signature and semantics as
  animatediff/attention_processor.py:18-96 (spatial self/cross attention of UNetMotionModel,
  text states repeat_interleave'd to B*F, LoRA `scale` forwarded to the projections only when
  to_q has a lora_layer).  Kernel mapping: self-attn q/k/v -> ONE fused GEMM (UnZipLoRA delta
  as augmented K), SDPA -> vst_spatial_attention, to_out -> GEMM with the block residual fused
  in the epilogue.  Cross-attn K/V are projected once per clip (not per frame) and indexed by
  frame // F inside the attention kernel.
* `AttnProcessor2_0`: the default processor the reference leaves on motion modules
  (inference_animatediff.py:211-215): frame-axis self-attention -> vst_temporal_attention.

Hidden-state layout.  Spatial: (B*F, H*W, C).  Motion: the reference/diffusers permute to
(B*H*W, F, C); our blocks keep (B*F, H*W, C) and pass `num_frames=F`, the kernel reads the frame
axis with stride H*W.  Both layouts are accepted by AttnProcessor2_0 (without `num_frames` the
input is taken as (batch, seq=F, C), the diffusers layout).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn

from . import kernels as K
from .lora_linear import LoRACompatibleLinear, build_ops, run_ops


class Attention(nn.Module):
    def __init__(self, query_dim: int, cross_attention_dim: Optional[int] = None, heads: int = 8,
                 dim_head: int = 64, bias: bool = False, out_bias: bool = True, processor=None,
                 temporal: bool = False):
        super().__init__()
        inner = heads * dim_head
        kv_dim = cross_attention_dim if cross_attention_dim is not None else query_dim
        self.heads = heads
        self.dim_head = dim_head
        self.inner_dim = inner
        self.is_cross_attention = cross_attention_dim is not None
        self.scale = dim_head ** -0.5
        self.to_q = LoRACompatibleLinear(query_dim, inner, bias=bias)
        self.to_k = LoRACompatibleLinear(kv_dim, inner, bias=bias)
        self.to_v = LoRACompatibleLinear(kv_dim, inner, bias=bias)
        self.to_out = nn.ModuleList([LoRACompatibleLinear(inner, query_dim, bias=out_bias), nn.Dropout(0.0)])
        self.norm_cross = None
        self.spatial_norm = None
        self.group_norm = None
        self.residual_connection = False
        self.rescale_output_factor = 1.0
        self.temporal = temporal
        self.processor = processor if processor is not None else (
            AttnProcessor2_0() if temporal else AnimateDiffAttnProcessor2_0())

    def set_processor(self, processor):
        self.processor = processor

    def get_processor(self):
        return self.processor

    def prepare_attention_mask(self, attention_mask, target_length, batch_size, out_dim=3):
        raise NotImplementedError("attention masks are not used on the AnimateDiff-XL denoise path")

    def norm_encoder_hidden_states(self, encoder_hidden_states):
        raise NotImplementedError("norm_cross is None for SDXL attention")

    def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None, **cross_attention_kwargs):
        return self.processor(self, hidden_states, encoder_hidden_states=encoder_hidden_states,
                              attention_mask=attention_mask, **cross_attention_kwargs)


def _proj_scale(attn, scale):
    # attention_processor.py:54 — LoRA scale only reaches layers that have a lora_layer
    return scale if hasattr(attn.to_q, "lora_layer") else 1.0


def _finish(attn, out, residual_for_flag):
    if attn.residual_connection:
        out = out + residual_for_flag
    if attn.rescale_output_factor != 1.0:
        out = out / attn.rescale_output_factor
    return out


class AnimateDiffAttnProcessor2_0:
    """animatediff/attention_processor.py:6-96, kernel-backed."""

    def __init__(self):
        if not hasattr(F, "scaled_dot_product_attention"):
            raise ImportError("AnimateDiffAttnProcessor2_0 requires PyTorch 2.0+.")

    def __call__(self, attn, hidden_states, encoder_hidden_states=None, attention_mask=None, temb=None, scale=1.0,
                 **kwargs):
        fused_residual = kwargs.pop("_vst_residual", None)
        lora_u = kwargs.pop("_vst_lora_u", None)  # x @ Acat^T of the q(/k/v) ops, from K.layer_norm_lora
        if attn.spatial_norm is not None or attn.group_norm is not None or attn.norm_cross:
            raise NotImplementedError("spatial_norm/group_norm/norm_cross are inert for SDXL (attention_processor.py:30-60)")
        if attention_mask is not None:
            raise NotImplementedError("attention_mask is None on the reference path (attention_processor.py:46-48)")
        input_ndim = hidden_states.ndim
        if input_ndim == 4:  # (B, C, H, W) -> tokens (attention_processor.py:34-36)
            b4, c4, h4, w4 = hidden_states.shape
            hidden_states = hidden_states.reshape(b4, c4, h4 * w4).transpose(1, 2).contiguous()
        batch, N, C = hidden_states.shape
        s = _proj_scale(attn, scale)
        heads, inner = attn.heads, attn.to_q.out_features
        hd = inner // heads
        x = hidden_states.reshape(batch * N, C)
        if encoder_hidden_states is None:
            qkv = run_ops(x, build_ops([attn.to_q, attn.to_k, attn.to_v], s), u=lora_u)
            o = K.spatial_attention(qkv[:, :inner], qkv[:, inner:2 * inner], qkv[:, 2 * inner:], batch, heads, N, N,
                                    1, scale=hd ** -0.5) if hd == 64 else _generic_attention(qkv, batch, heads, N)
        else:
            enc = encoder_hidden_states
            be, L, D = enc.shape
            if batch % be:
                raise ValueError(f"encoder batch {be} does not divide hidden batch {batch}")
            q_ops = build_ops([attn.to_q], s)
            kv = _text_kv(attn, enc, s)
            if hd != 64:
                raise NotImplementedError("spatial cross-attention kernel is specialised for head_dim 64 (SDXL)")
            if lora_u is None and _cross_fusable(q_ops, batch * N, N, L):
                # q projection (+ in-GEMM UnZipLoRA) and the text cross-attention as one launch: q stays on chip
                o = K.linear_cross_attention(x, q_ops.w, q_ops.a, q_ops.gn, q_ops.gr, q_ops.bias, kv[:, :inner],
                                             kv[:, inner:], Nq=N, Nk=L, kv_div=batch // be, scale=hd ** -0.5,
                                             r_alg=q_ops.r)
            else:
                q = run_ops(x, q_ops, u=lora_u)
                o = K.spatial_attention(q, kv[:, :inner], kv[:, inner:], batch, heads, N, L, batch // be,
                                        scale=hd ** -0.5)
        res2d = None if fused_residual is None else fused_residual.reshape(batch * N, -1)
        out = run_ops(o, build_ops([attn.to_out[0]], s), residual=res2d)
        out = out.view(batch, N, -1)
        if input_ndim == 4:
            out = out.transpose(-1, -2).reshape(b4, c4, h4, w4)
        return _finish(attn, out, hidden_states)


def _cross_fusable(ops, M: int, Nq: int, Nk: int) -> bool:
    """attn2's q projection ops (as build_ops made them) and the cross-attention fit vst_gemm_cross_attention."""
    lora = ops.a is not None
    if lora and ops.gn <= 0:
        return False
    return K.cross_attention_fusable(M, ops.n, ops.k1, lora, 0 if not lora else ops.a.shape[0], ops.gn, ops.gr, Nq, Nk)


def input_lora_ops(attn, self_attention: bool, scale: float = 1.0):
    """The projection operands AnimateDiffAttnProcessor2_0 will apply to this attention's hidden states
    (q/k/v for self-attention, q for cross-attention), or None when another processor is installed.
    Lets the producer of the hidden states (the block's LayerNorm) emit the LoRA down-projection."""
    if not isinstance(attn.processor, AnimateDiffAttnProcessor2_0):
        return None
    s = _proj_scale(attn, scale)
    return build_ops([attn.to_q, attn.to_k, attn.to_v] if self_attention else [attn.to_q], s)


def _text_kv(attn, enc, s):
    """Cross-attention K/V of the text states (to_k/to_v + LoRA on encoder_hidden_states).

    They depend only on the prompt and the weights, not on the latents, so across the 50 denoise
    steps of a clip they are projected once: cached on the module and keyed on the text tensor
    object (weakref + in-place version) and on the projection operands (build_ops is itself keyed
    on the parameter versions, LoRA scale and mode).  Inside a captured step graph the cached
    buffer is simply read.  A few texts are kept (the two CFG branches run as separate calls on two streams,
    pipeline.py), oldest dropped first."""
    import weakref
    ops = build_ops([attn.to_k, attn.to_v], s)
    cache = attn.__dict__.setdefault("_vst_text_kv", [])
    for ref, ver, ops_c, kv in cache:
        if ref() is enc and ver == enc._version and ops_c is ops:
            return kv
    be, L, D = enc.shape
    kv = run_ops(enc.reshape(be * L, D), ops)
    cache[:] = [c for c in cache if c[0]() is not None][-3:] + [(weakref.ref(enc), enc._version, ops, kv)]
    return kv


def _generic_attention(qkv, batch, heads, N):
    raise NotImplementedError("spatial self-attention kernel is specialised for head_dim 64 (SDXL)")


def _tattn_enabled() -> bool:
    """VST_TATTN=0 keeps the motion attention as q/k/v GEMM + vst_temporal_attention (A/B)."""
    return os.environ.get("VST_TATTN", "1") != "0"


def _tattn_operands(attn, ops, heads, head_dim):
    """The fused q/k/v weight re-laid out per pair of heads for vst_gemm_temporal_attention, cached on the module
    against the fused operand it was made from (build_ops caches that one per parameter version; trained weights get
    a fresh operand, hence a fresh layout, every call)."""
    c = attn.__dict__.get("_vst_tattn")
    if c is None or c[0] is not ops:
        c = (ops,) + K.temporal_qkv_layout(ops.w, ops.bias, heads, head_dim)
        attn.__dict__["_vst_tattn"] = c
    return c[1], c[2]


class AttnProcessor2_0:
    """Default (motion-module) processor: self-attention along the frame axis."""

    def __call__(self, attn, hidden_states, encoder_hidden_states=None, attention_mask=None, temb=None,
                 num_frames: Optional[int] = None, **kwargs):
        fused_residual = kwargs.pop("_vst_residual", None)
        if encoder_hidden_states is not None or attention_mask is not None:
            raise NotImplementedError("motion-module attention is self-attention without mask")
        batch, N, C = hidden_states.shape
        if num_frames is not None:  # our layout: (B*F, HW, C)
            nclip, Fr, HW = batch // num_frames, num_frames, N
        else:  # diffusers layout: (B*HW, F, C)
            nclip, Fr, HW = batch, N, 1
        heads = attn.heads
        inner = attn.to_q.out_features
        D = inner // heads
        x = hidden_states.reshape(batch * N, C)
        ops = build_ops([attn.to_q, attn.to_k, attn.to_v], 1.0)
        # (HW % (16 P) under K.fusion_world(P): a P-way all-to-all rank holds HW / P pixels and fuses only when that
        # is a multiple of 16, so the unsharded forward it is compared with decides the same way)
        if num_frames is not None and _tattn_enabled() and ops.a is None and ops.w.shape[1] == C and \
                HW % (16 * K.fusion_pixel_div()) == 0 and \
                K.temporal_attention_fusable(batch * N, C, nclip, Fr, HW, heads, D):
            # q/k/v projection + frame attention in one launch (vst_gemm_temporal_attention; 16 frames, heads of 40)
            w_t, b_t = _tattn_operands(attn, ops, heads, D)
            o = K.linear_temporal_attention(x, w_t, b_t, nclip=nclip, F=Fr, HW=HW, heads=heads, head_dim=D,
                                            scale=D ** -0.5)
        else:
            qkv = run_ops(x, ops)
            o = K.temporal_attention(qkv[:, :inner], qkv[:, inner:2 * inner], qkv[:, 2 * inner:], nclip, Fr, HW,
                                     heads, D)
        res2d = None if fused_residual is None else fused_residual.reshape(batch * N, -1)
        out = run_ops(o, build_ops([attn.to_out[0]], 1.0), residual=res2d).view(batch, N, -1)
        return _finish(attn, out, hidden_states)
