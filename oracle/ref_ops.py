"""ORACLE (test infrastructure only): reference-semantics building blocks, fp32 CPU.

Each function restates one reference call site; the citation is in its docstring.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------- UnZipLoRA
def unziplora_delta(x, A_c, B_c, m_c, A_s, B_s, m_s, forward_type="both", masked_c=False, masked_s=False,
                    x_style=None):
    """UnZipLoRALinearLayerInfer.forward (unziplora_unet/unziplora_linear_layer.py:298-346).

    A: (r, in) = lora_matrix_dic.{key}_down.weight, B: (out, r) = {key}_up.weight,
    m: (out,) merger.  "both": x @ (A_c^T B_c^T * m_c) + x_s @ (A_s^T B_s^T * m_s);
    "content"/"style" use the single branch WITHOUT the merger (:331, :343).  A masked key
    contributes zeros (:308-317).  x_style defaults to x (:306-307).
    """
    x = x.float()
    xs = x if x_style is None else x_style.float()
    out_f = B_c.shape[0]
    zeros = x.new_zeros(x.shape[:-1] + (out_f,))

    def merged(A, B):
        return A.float().t() @ B.float().t()  # (in, out)

    if forward_type == "both":
        dc = zeros if masked_c else x @ (merged(A_c, B_c) * m_c.float())
        ds = zeros if masked_s else xs @ (merged(A_s, B_s) * m_s.float())
        return ds + dc
    if forward_type == "content":
        return zeros if masked_c else x @ merged(A_c, B_c)
    if forward_type == "style":
        return zeros if masked_s else xs @ merged(A_s, B_s)
    raise AssertionError(forward_type)


def lora_compatible_linear(x, W, b=None, delta=None, scale=1.0):
    """LoRACompatibleLinear.forward (unziplora_unet/lora_linear.py:74-81): out + scale * lora(x)."""
    out = F.linear(x.float(), W.float(), None if b is None else b.float())
    if delta is not None:
        out = out + scale * delta
    return out


def lora_unzip_linear(x, W, b=None, x1=None, x2=None, lora=None, forward_type="both", scale=1.0):
    """lora_unzip.LoRACompatibleLinear.forward (unziplora_unet/lora_unzip.py:66-75): F.linear(x) + scale *
    lora_layer(x1, x2) — base on the joint-prompt states x, the content LoRA on x1, the style LoRA on x2 (the
    UnZipLoRALinearLayerInfer two-input forward, unziplora_linear_layer.py:298-346).  lora = (A_c, B_c, m_c,
    A_s, B_s, m_s) or None."""
    d = None if lora is None else unziplora_delta(x1, *lora, forward_type=forward_type, x_style=x2)
    return lora_compatible_linear(x, W, b, d, scale)


def unzip_attn_processor(hidden_states, encoder_hidden_states, enc_content, enc_style, heads, proj):
    """AttnProcessor2_0.__call__ of the image path (unziplora_unet/unzip_attention_processor.py:671-759), 3-D
    input, no mask: q = to_q(x | x, x); k, v = to_{k,v}(enc | enc_content, enc_style); SDPA; to_out(o | o, o).
    proj(name, x, x1, x2) applies the projection.  Missing content/style states fall back to the joint ones
    (the reference passes None through, which its LoRA layer cannot take)."""
    enc = hidden_states if encoder_hidden_states is None else encoder_hidden_states
    enc_c = enc if enc_content is None else enc_content
    enc_s = enc if enc_style is None else enc_style
    batch = hidden_states.shape[0]
    q = proj("to_q", hidden_states, hidden_states, hidden_states)
    k = proj("to_k", enc, enc_c, enc_s)
    v = proj("to_v", enc, enc_c, enc_s)
    hd = k.shape[-1] // heads
    q = q.view(batch, -1, heads, hd).transpose(1, 2)
    k = k.view(batch, -1, heads, hd).transpose(1, 2)
    v = v.view(batch, -1, heads, hd).transpose(1, 2)
    o = sdpa(q, k, v).transpose(1, 2).reshape(batch, -1, heads * hd)
    return proj("to_out", o, o, o)


# ----------------------------------------------------------------------------- attention
def sdpa(q, k, v, scale=None):
    """F.scaled_dot_product_attention without mask/dropout (attention_processor.py:78-80), fp32."""
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else scale
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    return torch.softmax(s, dim=-1) @ v.float()


def attn_processor(hidden_states, encoder_hidden_states, heads, proj, scale=1.0):
    """AnimateDiffAttnProcessor2_0.__call__, 3-D input path (animatediff/attention_processor.py:28-96).

    proj: callable(name, x) -> projected x for name in {to_q,to_k,to_v,to_out}; it applies the
    base linear plus `scale` * LoRA delta when the layer has one (:54).  Text states with batch
    smaller than hidden_states' are repeat_interleave'd to it (:63-66).
    """
    batch = hidden_states.shape[0]
    q = proj("to_q", hidden_states)
    enc = hidden_states if encoder_hidden_states is None else encoder_hidden_states
    if enc.shape[0] != batch:
        enc = enc.repeat_interleave(batch // enc.shape[0], dim=0)
    k = proj("to_k", enc)
    v = proj("to_v", enc)
    inner = k.shape[-1]
    hd = inner // heads
    q = q.view(batch, -1, heads, hd).transpose(1, 2)
    k = k.view(batch, -1, heads, hd).transpose(1, 2)
    v = v.view(batch, -1, heads, hd).transpose(1, 2)
    o = sdpa(q, k, v)
    o = o.transpose(1, 2).reshape(batch, -1, heads * hd)
    return proj("to_out", o)


# ----------------------------------------------------------------------------- temporal
def positional_encoding(d_model, max_len=32):
    """PositionalEncoding.__init__ (animatediff/temporal_transformer.py:11-21) -> (max_len, d)."""
    position = torch.arange(max_len).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d_model, 2) * (-math.log(10000.0) / d_model))
    pe = torch.zeros(max_len, d_model)
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    return pe


def mha(x, in_w, in_b, out_w, out_b, heads):
    """nn.MultiheadAttention(batch_first) self-attention as used at temporal_transformer.py:67-68."""
    C = x.shape[-1]
    qkv = F.linear(x, in_w, in_b)
    q, k, v = qkv.split(C, dim=-1)
    B, S, _ = x.shape
    hd = C // heads
    q = q.view(B, S, heads, hd).transpose(1, 2)
    k = k.view(B, S, heads, hd).transpose(1, 2)
    v = v.view(B, S, heads, hd).transpose(1, 2)
    o = sdpa(q, k, v).transpose(1, 2).reshape(B, S, C)
    return F.linear(o, out_w, out_b)


def temporal_transformer(x, P, num_layers, heads, prefix=""):
    """TemporalTransformer.forward (animatediff/temporal_transformer.py:110-146) on (B,C,F,H,W).

    P holds the module's state_dict (keys as in the reference module).
    """
    x = x.float()
    B, C, Fr, H, W = x.shape
    h = x.permute(0, 3, 4, 2, 1).reshape(-1, Fr, C)
    h = h + P[prefix + "pos_encoding.pe"][:, :Fr, :].float()
    for i in range(num_layers):
        p = f"{prefix}blocks.{i}."
        n = F.layer_norm(h, (C,), P[p + "norm1.weight"].float(), P[p + "norm1.bias"].float())
        h = h + mha(n, P[p + "attn.in_proj_weight"].float(), P[p + "attn.in_proj_bias"].float(),
                    P[p + "attn.out_proj.weight"].float(), P[p + "attn.out_proj.bias"].float(), heads)
        n = F.layer_norm(h, (C,), P[p + "norm2.weight"].float(), P[p + "norm2.bias"].float())
        f = F.linear(n, P[p + "ffn.0.weight"].float(), P[p + "ffn.0.bias"].float())
        f = F.gelu(f)
        f = F.linear(f, P[p + "ffn.3.weight"].float(), P[p + "ffn.3.bias"].float())
        h = h + f
    h = F.layer_norm(h, (C,), P[prefix + "norm.weight"].float(), P[prefix + "norm.bias"].float())
    return h.view(B, H, W, Fr, C).permute(0, 4, 3, 1, 2).contiguous()


def temporal_lora_forward(x, W, b, A, Bm, alpha, rank):
    """TemporalLoRALinear.forward (animatediff/temporal_lora.py:29-32)."""
    scale = alpha / rank
    return F.linear(x.float(), W.float(), None if b is None else b.float()) + F.linear(
        F.linear(x.float(), A.float()), Bm.float()) * scale


def temporal_lora_delta(A, Bm, alpha, rank):
    """TemporalLoRALinear.get_delta (animatediff/temporal_lora.py:34-36)."""
    return (Bm.float() @ A.float()) * (alpha / rank)


def orth_loss(pairs, lambda_orth):
    """compute_orth_loss (animatediff/temporal_lora.py:126-166).

    pairs: list of (delta_temporal (out,in), A_c, B_c, A_s, B_s).
    """
    if lambda_orth == 0.0 or not pairs:
        return torch.tensor(0.0)
    total = None
    for dt, A_c, B_c, A_s, B_s in pairs:
        dc = B_c.float() @ A_c.float()
        ds = B_s.float() @ A_s.float()
        W = dt.float()
        c = torch.sum((W.t() @ dc) ** 2) + torch.sum((W.t() @ ds) ** 2)
        total = c if total is None else total + c
    return lambda_orth * total / len(pairs)
