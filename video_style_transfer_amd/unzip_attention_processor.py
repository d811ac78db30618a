"""Image-path attention of Stage 1 (unziplora_unet/unzip_attention_processor.py), kernel-backed — SURVEY §8 a4.

* `Attention`: the reference's Attention subclass (:25-181) whose forward carries
  `encoder_hidden_states_content` / `encoder_hidden_states_style` to the processor; its projections are the
  dual-prompt `lora_unzip.LoRACompatibleLinear`.
* `AttnProcessor2_0.__call__(attn, hidden_states, encoder_hidden_states, encoder_hidden_states_content,
  encoder_hidden_states_style, attention_mask, temb, scale)` (:662-759): q = to_q(x | x, x); k/v =
  to_{k,v}(joint text | content text, style text); SDPA -> vst_spatial_attention; to_out(o | o, o).  Each projection
  is one fused GEMM (lora_unzip.py); self-attention q/k/v share their input and run as one GEMM.

The 4-D input, spatial_norm, group_norm and norm_cross branches follow the reference's code; attention masks are
not supported (the Stage-1 image path passes none).
"""
from __future__ import annotations

import torch

from . import kernels as K
from .attention_processor import Attention as _TextAttention
from .attention_processor import _finish
from .lora_linear import build_ops, run_ops
from .lora_unzip import LoRACompatibleLinear


def _project(lin, x, x1, x2, scale):
    if isinstance(lin, LoRACompatibleLinear):
        return lin(x, scale, x1, x2)
    if hasattr(lin, "lora_layer"):
        return lin(x, scale)
    return lin(x)


class AttnProcessor2_0:
    """unzip_attention_processor.py:662-759."""

    def __init__(self):
        import torch.nn.functional as F
        if not hasattr(F, "scaled_dot_product_attention"):
            raise ImportError("AttnProcessor2_0 requires PyTorch 2.0, to use it, please upgrade PyTorch to 2.0.")

    def __call__(self, attn, hidden_states, encoder_hidden_states=None, encoder_hidden_states_content=None,
                 encoder_hidden_states_style=None, attention_mask=None, temb=None, scale: float = 1.0):
        if attention_mask is not None:
            raise NotImplementedError("attention masks are not used on the Stage-1 image path")
        residual = hidden_states
        if attn.spatial_norm is not None:
            hidden_states = attn.spatial_norm(hidden_states, temb)
        input_ndim = hidden_states.ndim
        if input_ndim == 4:
            b4, c4, h4, w4 = hidden_states.shape
            hidden_states = hidden_states.view(b4, c4, h4 * w4).transpose(1, 2).contiguous()
        if attn.group_norm is not None:
            hidden_states = attn.group_norm(hidden_states.transpose(1, 2)).transpose(1, 2).contiguous()
        batch, N, C = hidden_states.shape
        heads, inner = attn.heads, attn.to_q.out_features
        hd = inner // heads
        x = hidden_states
        if encoder_hidden_states is None:
            enc = enc_c = enc_s = x
        else:
            enc = encoder_hidden_states
            enc_c = enc if encoder_hidden_states_content is None else encoder_hidden_states_content
            enc_s = enc if encoder_hidden_states_style is None else encoder_hidden_states_style
            if attn.norm_cross:
                enc = attn.norm_encoder_hidden_states(enc)
                enc_c = attn.norm_encoder_hidden_states(enc_c)
                enc_s = attn.norm_encoder_hidden_states(enc_s)
        if enc is x and enc_c is x and enc_s is x:
            # self-attention: every branch reads x -> one fused q/k/v GEMM
            qkv = run_ops(x.reshape(batch * N, C), build_ops([attn.to_q, attn.to_k, attn.to_v], scale, mode="fused"))
            q, k, v = qkv[:, :inner], qkv[:, inner:2 * inner], qkv[:, 2 * inner:]
            Nk = N
        else:
            q = _project(attn.to_q, x, x, x, scale).reshape(batch * N, inner)
            k = _project(attn.to_k, enc, enc_c, enc_s, scale)
            v = _project(attn.to_v, enc, enc_c, enc_s, scale)
            if k.shape[0] != batch:
                raise ValueError(f"encoder batch {k.shape[0]} != hidden batch {batch} (the image path does not "
                                 "repeat text states)")
            Nk = k.shape[1]
            k, v = k.reshape(batch * Nk, inner), v.reshape(batch * Nk, inner)
        if hd == 64:  # k and v may be separate buffers: the kernel only needs one row stride for both
            o = K.spatial_attention(q, k, v, batch, heads, N, Nk, 1, scale=hd ** -0.5)
        else:
            raise NotImplementedError("the spatial attention kernel is specialised for head_dim 64 (SDXL)")
        out = _project(attn.to_out[0], o, o, o, scale).view(batch, N, -1)
        out = attn.to_out[1](out)
        if input_ndim == 4:
            out = out.transpose(-1, -2).reshape(b4, c4, h4, w4)
        return _finish(attn, out, residual)


class Attention(_TextAttention):
    """unzip_attention_processor.py:25-181: projections are dual-prompt LoRACompatibleLinear, forward carries the
    content/style encoder states to the processor."""

    def __init__(self, query_dim: int, cross_attention_dim=None, heads: int = 8, dim_head: int = 64,
                 bias: bool = False, out_bias: bool = True, processor=None):
        super().__init__(query_dim, cross_attention_dim, heads, dim_head, bias, out_bias,
                         processor=processor or AttnProcessor2_0())
        inner = heads * dim_head
        kv_dim = cross_attention_dim if cross_attention_dim is not None else query_dim
        self.to_q = LoRACompatibleLinear(query_dim, inner, bias=bias)
        self.to_k = LoRACompatibleLinear(kv_dim, inner, bias=bias)
        self.to_v = LoRACompatibleLinear(kv_dim, inner, bias=bias)
        self.to_out = torch.nn.ModuleList([LoRACompatibleLinear(inner, query_dim, bias=out_bias),
                                           torch.nn.Dropout(0.0)])

    def forward(self, hidden_states, encoder_hidden_states=None, encoder_hidden_states_content=None,
                encoder_hidden_states_style=None, attention_mask=None, **cross_attention_kwargs):
        return self.processor(self, hidden_states, encoder_hidden_states=encoder_hidden_states,
                              encoder_hidden_states_content=encoder_hidden_states_content,
                              encoder_hidden_states_style=encoder_hidden_states_style,
                              attention_mask=attention_mask, **cross_attention_kwargs)
