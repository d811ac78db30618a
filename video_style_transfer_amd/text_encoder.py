"""The SDXL text encoders on the HIP path: encode_prompt of inference_animatediff.py:16-35 /
train_animatediff.py:29-50, i.e. transformers' CLIPTextModel (openai CLIP ViT-L/14 text tower, `text_encoder`) and
CLIPTextModelWithProjection (OpenCLIP ViT-bigG/14 text tower, `text_encoder_2`), loaded by the reference from the
SDXL checkpoint (train_animatediff.py:74-80).

Same module tree and state-dict keys as transformers (`text_model.embeddings.token_embedding.weight`,
`text_model.encoder.layers.{i}.self_attn.{q,k,v,out}_proj`, `layer_norm1/2`, `mlp.fc1/fc2`,
`text_model.final_layer_norm`, `text_projection`), so a checkpoint's text encoders load unchanged.  The forward is
the transformers CLIPTextTransformer:
  h = token_embedding[ids] + position_embedding[pos]                         (vst_embed_tokens)
  per layer: h += out_proj(causal_attention(q, k, v of LN1(h)));  h += fc2(act(fc1(LN2(h))))
                                      (vst_gemm_ex, vst_causal_attention, GELU(erf) in the GEMM epilogue /
                                       vst_quick_gelu; each residual add fused with the next LayerNorm:
                                       vst_residual_layernorm)
  last_hidden_state = final_layer_norm(h); pooled = last_hidden_state at the EOS token; text_embeds = pooled @ P^T.
Weights bf16, GEMM accumulation fp32, GEMM outputs bf16 and the residual stream h fp32 -- the precision of the
reference's fp32 towers under bf16 autocast (a bf16 residual stream measured 2.3x that run's distance from fp32 over
the 32 bigG layers).  No tokenizer vocabulary ships offline: the boundary is the token ids (a tokenizer callable may
be passed to encode_prompt).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch
from torch import nn

from . import _lib
from . import kernels as K

BF16 = torch.bfloat16


@dataclass
class CLIPTextConfig:
    """transformers.CLIPTextConfig fields the SDXL text towers use (the two `config.json`s of
    stabilityai/stable-diffusion-xl-base-1.0 text_encoder / text_encoder_2)."""
    vocab_size: int = 49408
    hidden_size: int = 768
    intermediate_size: int = 3072
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    max_position_embeddings: int = 77
    hidden_act: str = "quick_gelu"
    layer_norm_eps: float = 1e-5
    projection_dim: int = 768
    eos_token_id: int = 2  # 2: the legacy pooling, the EOS token is the largest id (transformers CLIPTextTransformer)

    @classmethod
    def sdxl_text_encoder(cls) -> "CLIPTextConfig":
        return cls()

    @classmethod
    def sdxl_text_encoder_2(cls) -> "CLIPTextConfig":
        return cls(hidden_size=1280, intermediate_size=5120, num_hidden_layers=32, num_attention_heads=20,
                   hidden_act="gelu", projection_dim=1280)

    @classmethod
    def tiny(cls, act: str = "quick_gelu") -> "CLIPTextConfig":
        return cls(vocab_size=1000, hidden_size=128, intermediate_size=512, num_hidden_layers=3,
                   num_attention_heads=2, hidden_act=act, projection_dim=128)


class _Linear(nn.Linear):
    def f32_bias(self):
        c = self.__dict__.get("_vst_b")
        if c is None or c[0] != self.bias._version:
            c = (self.bias._version, self.bias.detach().float().contiguous())
            self.__dict__["_vst_b"] = c
        return c[1]


class CLIPAttention(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        C = cfg.hidden_size
        self.heads = cfg.num_attention_heads
        self.head_dim = C // self.heads
        self.k_proj, self.v_proj, self.q_proj, self.out_proj = (_Linear(C, C) for _ in range(4))

    def qkv_operands(self):
        """[Wq; Wk; Wv] bf16 and the fp32 bias, built once per parameter version."""
        ver = tuple(p._version for p in self.parameters())
        c = self.__dict__.get("_vst_qkv")
        if c is None or c[0] != ver:
            W = torch.cat([self.q_proj.weight, self.k_proj.weight, self.v_proj.weight], 0).to(BF16).contiguous()
            b = torch.cat([self.q_proj.bias, self.k_proj.bias, self.v_proj.bias], 0).float().contiguous()
            c = (ver, W, b)
            self.__dict__["_vst_qkv"] = c
        return c[1], c[2]

    def run(self, n, B, L):
        C = n.shape[1]
        W, b = self.qkv_operands()
        qkv = K.linear(n, W, b)
        o = torch.empty((B * L, C), dtype=BF16, device=n.device)
        _lib.call("vst_causal_attention", qkv.data_ptr(), qkv.stride(0), qkv[:, C:].data_ptr(),
                  qkv[:, 2 * C:].data_ptr(), qkv.stride(0), o.data_ptr(), o.stride(0), B, self.heads, L,
                  self.head_dim, float(self.head_dim ** -0.5), K._stream())
        return K.linear(o, self.out_proj.weight, self.out_proj.f32_bias())


class CLIPMLP(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.act = cfg.hidden_act
        if self.act not in ("quick_gelu", "gelu"):
            raise ValueError(f"CLIPMLP: hidden_act {self.act!r} (SDXL uses quick_gelu / gelu)")
        self.fc1 = _Linear(cfg.hidden_size, cfg.intermediate_size)
        self.fc2 = _Linear(cfg.intermediate_size, cfg.hidden_size)

    def run(self, n):
        if self.act == "gelu":  # exact GELU in the GEMM epilogue (transformers ACT2FN["gelu"])
            h = K.linear(n, self.fc1.weight, self.fc1.f32_bias(), act="gelu")
        else:
            h = K.linear(n, self.fc1.weight, self.fc1.f32_bias())
            _lib.call("vst_quick_gelu", h.data_ptr(), h.data_ptr(), h.numel(), K._stream())
        return K.linear(h, self.fc2.weight, self.fc2.f32_bias())


class _LayerNorm(nn.LayerNorm):
    def f32(self):
        c = self.__dict__.get("_vst_f32")
        ver = (self.weight._version, self.bias._version)
        if c is None or c[0] != ver:
            c = (ver, self.weight.detach().float().contiguous(), self.bias.detach().float().contiguous())
            self.__dict__["_vst_f32"] = c
        return c[1], c[2]

    def add_run(self, h, y=None):
        """(h + y fp32, LayerNorm of it bf16): vst_residual_layernorm."""
        g, b = self.f32()
        rows, C = h.shape
        ho = torch.empty_like(h)
        n = torch.empty((rows, C), dtype=BF16, device=h.device)
        _lib.call("vst_residual_layernorm", h.data_ptr(), h.stride(0), None if y is None else y.data_ptr(),
                  0 if y is None else y.stride(0), rows, C, g.data_ptr(), b.data_ptr(), float(self.eps),
                  ho.data_ptr(), ho.stride(0), n.data_ptr(), n.stride(0), K._stream())
        return ho, n


class CLIPEncoderLayer(nn.Module):
    """transformers CLIPEncoderLayer: h += self_attn(layer_norm1(h)); h += mlp(layer_norm2(h)).  The residual adds
    run fused with the following LayerNorm on the fp32 residual stream (CLIPTextTransformer.run)."""

    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.self_attn = CLIPAttention(cfg)
        self.layer_norm1 = _LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)
        self.mlp = CLIPMLP(cfg)
        self.layer_norm2 = _LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)


class _Encoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.layers = nn.ModuleList([CLIPEncoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])


class _Embeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.token_embedding = nn.Embedding(cfg.vocab_size, cfg.hidden_size)
        self.position_embedding = nn.Embedding(cfg.max_position_embeddings, cfg.hidden_size)
        self.register_buffer("position_ids", torch.arange(cfg.max_position_embeddings).unsqueeze(0), persistent=False)


class CLIPTextTransformer(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.config = cfg
        self.embeddings = _Embeddings(cfg)
        self.encoder = _Encoder(cfg)
        self.final_layer_norm = _LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)

    def run(self, input_ids: torch.Tensor, n_layers: Optional[int] = None):
        """(hidden_states tuple [embeddings, layer 1 .. layer n] as (B, L, C) fp32 -- the residual stream, fp32 as in
        the reference's fp32 towers under autocast -- , last_hidden_state (final LayerNorm, bf16), pooled (bf16))."""
        cfg = self.config
        if input_ids.dim() != 2:
            raise ValueError("input_ids must be (batch, sequence)")
        B, L = input_ids.shape
        if L > cfg.max_position_embeddings:
            raise ValueError(f"sequence of {L} tokens > max_position_embeddings {cfg.max_position_embeddings}")
        dev = self.embeddings.token_embedding.weight.device
        if dev.type != "cuda":
            raise _lib.VstError("CLIP text encoder: weights are on CPU; the HIP path has no CPU fallback")
        ids_cpu = input_ids.detach().to("cpu", torch.int64)
        if int(ids_cpu.min()) < 0 or int(ids_cpu.max()) >= cfg.vocab_size:
            raise IndexError("input_ids out of the vocabulary range")  # nn.Embedding's error, checked on the host
        ids = ids_cpu.to(torch.int32).to(dev)
        C = cfg.hidden_size
        tok, pos = self.embeddings.token_embedding.weight, self.embeddings.position_embedding.weight
        h = torch.empty((B * L, C), dtype=torch.float32, device=dev)
        _lib.call("vst_embed_tokens", ids.data_ptr(), B * L, L, tok.data_ptr(), pos.data_ptr(), C, h.data_ptr(), C,
                  K._stream())
        states = [h]
        n = cfg.num_hidden_layers if n_layers is None else n_layers
        layers = list(self.encoder.layers[:n])
        lns = [ly.layer_norm1 for ly in layers[1:]] + [self.final_layer_norm]
        _, x = layers[0].layer_norm1.add_run(h) if layers else (h, None)
        for ly, ln_next in zip(layers, lns):
            h, x = ly.layer_norm2.add_run(h, ly.self_attn.run(x, B, L))    # h += attn; x = LN2(h)
            h, x = ln_next.add_run(h, ly.mlp.run(x))                     # h += mlp;  x = next LN1 / final LN
            states.append(h)
        if not layers:
            _, x = self.final_layer_norm.add_run(h)
        last = x
        if cfg.eos_token_id == 2:
            eos = ids_cpu.argmax(-1)
        else:
            eos = (ids_cpu == cfg.eos_token_id).int().argmax(-1)
        rows = (torch.arange(B) * L + eos).to(dev)
        pooled = last.index_select(0, rows)
        return tuple(s.view(B, L, C) for s in states), last.view(B, L, C), pooled


@dataclass
class CLIPTextOutput:
    """transformers BaseModelOutputWithPooling / CLIPTextModelOutput: [0] is last_hidden_state (CLIPTextModel) or
    text_embeds (CLIPTextModelWithProjection), as the reference indexes it (inference_animatediff.py:29-31)."""
    last_hidden_state: torch.Tensor
    pooler_output: Optional[torch.Tensor] = None
    text_embeds: Optional[torch.Tensor] = None
    hidden_states: Optional[Tuple[torch.Tensor, ...]] = None

    def __getitem__(self, i):
        first = self.text_embeds if self.text_embeds is not None else self.last_hidden_state
        return (first, self.last_hidden_state, self.hidden_states)[i]


class CLIPTextModel(nn.Module):
    """transformers.CLIPTextModel surface: model(input_ids, output_hidden_states=True).hidden_states[-2]."""

    def __init__(self, cfg: Optional[CLIPTextConfig] = None):
        super().__init__()
        self.config = cfg or CLIPTextConfig.sdxl_text_encoder()
        self.text_model = CLIPTextTransformer(self.config)

    def forward(self, input_ids, attention_mask=None, output_hidden_states: bool = False, **kw):
        if attention_mask is not None:
            raise NotImplementedError("encode_prompt passes no attention mask (inference_animatediff.py:25-33)")
        states, last, pooled = self.text_model.run(input_ids)
        return CLIPTextOutput(last, pooled, None, states if output_hidden_states else None)


class CLIPTextModelWithProjection(nn.Module):
    """transformers.CLIPTextModelWithProjection surface: model(input_ids, output_hidden_states=True)[0] is the
    projected pooled embedding (text_embeds), .hidden_states[-2] the penultimate layer."""

    def __init__(self, cfg: Optional[CLIPTextConfig] = None):
        super().__init__()
        self.config = cfg or CLIPTextConfig.sdxl_text_encoder_2()
        self.text_model = CLIPTextTransformer(self.config)
        self.text_projection = nn.Linear(self.config.hidden_size, self.config.projection_dim, bias=False)

    def forward(self, input_ids, attention_mask=None, output_hidden_states: bool = False, **kw):
        if attention_mask is not None:
            raise NotImplementedError("encode_prompt passes no attention mask (inference_animatediff.py:25-33)")
        states, last, pooled = self.text_model.run(input_ids)
        emb = K.linear(pooled.contiguous(), self.text_projection.weight)
        return CLIPTextOutput(last, pooled, emb, states if output_hidden_states else None)


def build_text_encoder(cls, cfg: Optional[CLIPTextConfig] = None, *, state_dict=None, seed: int = 0,
                       device="cuda"):
    """A text encoder with bf16 weights on the device: from a transformers-format state dict, or seeded synthetic
    (N(0, 0.02) projections / embeddings, LayerNorm gamma 1 beta 0: transformers' CLIP init)."""
    model = cls(cfg)
    if state_dict is not None:
        # checkpoints name the tower "text_model.*" (SDXL text_encoder / text_encoder_2); recent transformers drop
        # the prefix from CLIPTextModel's own state_dict: accept both
        state_dict = {(k if k.startswith("text_model.") or k.startswith("text_projection") else "text_model." + k): v
                      for k, v in state_dict.items()}
        missing, unexpected = model.load_state_dict(state_dict, strict=False)
        missing = [k for k in missing if not k.endswith("position_ids")]
        unexpected = [k for k in unexpected if not k.endswith("position_ids")]
        if missing or unexpected:
            raise KeyError(f"text encoder checkpoint mismatch: missing {missing[:4]}, unexpected {unexpected[:4]}")
        return model.to(device=device, dtype=BF16).requires_grad_(False)
    model = model.to(device=device, dtype=BF16).requires_grad_(False)
    g = torch.Generator(device=device).manual_seed(seed)
    with torch.no_grad():
        for name, p in model.named_parameters():
            if "layer_norm" in name:
                p.fill_(1.0 if name.endswith("weight") else 0.0)
            elif name.endswith("bias"):
                p.zero_()
            else:
                p.copy_(torch.randn(p.shape, generator=g, device=p.device) * 0.02)
    return model


def encode_prompt(text_encoder, text_encoder_2, tokenizer, tokenizer_2, prompt, device=None):
    """inference_animatediff.py:16-35: (prompt_embeds (B, 77, 768 + 1280), pooled (B, 1280)).  `tokenizer*` are
    callables returning an object with .input_ids (B, 77), as transformers' CLIPTokenizer(prompt, padding=
    "max_length", max_length=77, truncation=True, return_tensors="pt") does; `prompt` may also be given directly as
    token ids (B, 77) when no tokenizer vocabulary is available (tokenizer = None)."""
    def ids(tok, p):
        if tok is None:
            return p if torch.is_tensor(p) else torch.as_tensor(p)
        t = tok(p, padding="max_length", max_length=getattr(tok, "model_max_length", 77), truncation=True,
                return_tensors="pt")
        return t.input_ids
    prompt_embeds = text_encoder(ids(tokenizer, prompt), output_hidden_states=True).hidden_states[-2]
    out2 = text_encoder_2(ids(tokenizer_2, prompt), output_hidden_states=True)
    pooled = out2[0]
    prompt_embeds_2 = out2.hidden_states[-2]
    return torch.cat([prompt_embeds, prompt_embeds_2], dim=-1), pooled
