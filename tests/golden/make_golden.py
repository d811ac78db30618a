"""Generate golden input/output vectors by running the REFERENCE's own torch-only modules.

Run in the build container only (it reads /root/reference, which never travels to the GPU
box):   python tests/golden/make_golden.py
Outputs tests/golden/*.safetensors (data only: seeded inputs, parameters and the reference's
outputs).  Modules exercised:
  animatediff/attention_processor.py   AnimateDiffAttnProcessor2_0 (spatial self/cross, temporal core)
  animatediff/temporal_transformer.py  PositionalEncoding, TemporalTransformer
  animatediff/temporal_lora.py         TemporalLoRALinear, compute_orth_loss, build_spatial_lora_index,
                                       get_merged_motion_state_dict
  unziplora_unet/unziplora_linear_layer.py  UnZipLoRALinearLayerInfer (both/content/style, masked)
  unziplora_unet/lora_linear.py        LoRACompatibleLinear (+ UnZipLoRA layer)
  unziplora_unet/lora_unzip.py         LoRACompatibleLinear, image-path dual-prompt variant (x, x_content, x_style)
"""
import json
import os
import sys

import torch
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import structured as S  # noqa: E402

REF = "/root/reference"
sys.path.insert(0, REF)

from animatediff.attention_processor import AnimateDiffAttnProcessor2_0  # noqa: E402
from animatediff.temporal_lora import (TemporalLoRALinear, build_spatial_lora_index,  # noqa: E402
                                       compute_orth_loss, get_merged_motion_state_dict, inject_temporal_lora)
from animatediff.temporal_transformer import PositionalEncoding, TemporalTransformer  # noqa: E402
from unziplora_unet.lora_linear import LoRACompatibleLinear  # noqa: E402
from unziplora_unet.lora_unzip import LoRACompatibleLinear as UnzipLoRACompatibleLinear  # noqa: E402
from unziplora_unet.unziplora_linear_layer import UnZipLoRALinearLayerInfer  # noqa: E402

torch.set_grad_enabled(False)


def bf(t):
    """round to bf16-representable fp32 (inputs are bf16-exact so the GPU path sees them exactly)"""
    return t.to(torch.bfloat16).float()


def save(name, tensors, meta):
    out = {}
    for k, v in tensors.items():
        v = v.detach().contiguous()
        # bf16-exact fp32 data is stored as bf16 (exact); consumers call .float()
        if v.dtype == torch.float32 and v.numel() > 64 and torch.equal(v, v.to(torch.bfloat16).float()):
            v = v.to(torch.bfloat16)
        out[k] = v
    tensors = out
    save_file(tensors, os.path.join(HERE, name + ".safetensors"), metadata={"meta": json.dumps(meta)})
    n = sum(v.numel() * v.element_size() for v in tensors.values())
    print(f"{name}: {len(tensors)} tensors, {n / 1e6:.2f} MB")


def make_unziplora(gen, in_f, out_f, r, merger=True):
    layer = UnZipLoRALinearLayerInfer(in_f, out_f, rank=r, lora_matrix_key=["content", "style"])
    for k in ("content_down", "content_up", "style_down", "style_up"):
        w = layer.lora_matrix_dic[k].weight
        w.copy_(bf(torch.randn(w.shape, generator=gen) / r))
    if merger:
        layer.merge_content.copy_(bf(torch.rand(out_f, generator=gen)))
        layer.merge_style.copy_(bf(torch.rand(out_f, generator=gen)))
    return layer


def dump_unziplora(layer, prefix, dst):
    d = layer.lora_matrix_dic
    dst[prefix + "A_c"] = d["content_down"].weight.detach().clone()
    dst[prefix + "B_c"] = d["content_up"].weight.detach().clone()
    dst[prefix + "A_s"] = d["style_down"].weight.detach().clone()
    dst[prefix + "B_s"] = d["style_up"].weight.detach().clone()
    dst[prefix + "m_c"] = layer.merge_content.detach().clone()
    dst[prefix + "m_s"] = layer.merge_style.detach().clone()


# --------------------------------------------------------------------------- 1. UnZipLoRA
def gen_unziplora():
    gen = torch.Generator().manual_seed(1)
    T, meta = {}, {"cases": []}
    for (in_f, out_f, r) in [(640, 640, 8), (2048, 1280, 8), (1280, 1280, 64)]:
        tag = f"i{in_f}_o{out_f}_r{r}"
        layer = make_unziplora(gen, in_f, out_f, r)
        x = bf(torch.randn(2, 8, in_f, generator=gen))
        xs = bf(torch.randn(2, 8, in_f, generator=gen))
        T[tag + ".x"] = x
        T[tag + ".xs"] = xs
        dump_unziplora(layer, tag + ".", T)
        for mode in ("both", "content", "style"):
            layer.set_forward(mode)
            T[f"{tag}.out_{mode}"] = layer(x)
            if mode == "both":
                T[f"{tag}.out_both_xs"] = layer(x, xs)  # image-path 2-input variant (lora_unzip.py:66)
        layer.set_forward("both")
        layer.set_layer_mask("style", True)
        T[f"{tag}.out_both_masked_style"] = layer(x)
        layer.set_layer_mask("style", False)
        meta["cases"].append([in_f, out_f, r])
    save("unziplora", T, meta)


# --------------------------------------------------------------------------- 2. LoRACompatibleLinear
def gen_lora_linear():
    gen = torch.Generator().manual_seed(2)
    T = {}
    in_f = out_f = 640
    lin = LoRACompatibleLinear(in_f, out_f, bias=True)
    wf = S.make(out_f, in_f, 8, gen)
    lin.weight.copy_(S.rebuild(wf, out_f, in_f))
    lin.bias.copy_(bf(torch.randn(out_f, generator=gen) * 0.1))
    layer = make_unziplora(gen, in_f, out_f, 8)
    lin.set_lora_layer(layer)
    x = bf(torch.randn(2, 16, in_f, generator=gen))
    S.store("W", wf, T)
    T["b"] = lin.bias.detach().clone()
    T["x"] = x
    dump_unziplora(layer, "lora.", T)
    for mode in ("both", "content", "style"):
        layer.set_forward(mode)
        T[f"out_{mode}_s1"] = lin(x)
        T[f"out_{mode}_s07"] = lin(x, 0.7)
    lin.set_lora_layer(None)
    T["out_nolora"] = lin(x)
    save("lora_linear", T, {"in": in_f, "out": out_f, "rank": 8})


# --------------------------------------------------------------------------- 2b. lora_unzip dual-prompt linear
def gen_lora_unzip():
    """lora_unzip.py:66-75: base on x (joint prompt), content LoRA on x_1, style LoRA on x_2.
    Text-token-shaped inputs (77 tokens, 2048 -> 640), as the K/V projections of cross-attention see them."""
    gen = torch.Generator().manual_seed(9)
    T = {}
    in_f, out_f, r = 2048, 640, 8
    lin = UnzipLoRACompatibleLinear(in_f, out_f, bias=False)
    wf = S.make(out_f, in_f, 8, gen)
    lin.weight.copy_(S.rebuild(wf, out_f, in_f))
    layer = make_unziplora(gen, in_f, out_f, r)
    lin.set_lora_layer(layer)
    x, x1, x2 = (bf(torch.randn(1, 77, in_f, generator=gen)) for _ in range(3))
    S.store("W", wf, T)
    T["x"], T["x1"], T["x2"] = x, x1, x2
    dump_unziplora(layer, "lora.", T)
    for mode in ("both", "content", "style"):
        layer.set_forward(mode)
        T[f"out_{mode}_s1"] = lin(x, 1.0, x1, x2)
        T[f"out_{mode}_s07"] = lin(x, 0.7, x1, x2)
    lin.set_lora_layer(None)
    T["out_nolora"] = lin(x)
    save("lora_unzip", T, {"in": in_f, "out": out_f, "rank": r})


# --------------------------------------------------------------------------- 3/4. attention processor
class DuckAttention(torch.nn.Module):
    """The attributes AnimateDiffAttnProcessor2_0 reads (attention_processor.py:28-96)."""

    def __init__(self, q_dim, kv_dim, heads, out_bias=True, lora=False):
        super().__init__()
        self.heads = heads
        L = LoRACompatibleLinear if lora else torch.nn.Linear
        self.to_q = L(q_dim, q_dim, bias=False)
        self.to_k = L(kv_dim, q_dim, bias=False)
        self.to_v = L(kv_dim, q_dim, bias=False)
        self.to_out = torch.nn.ModuleList([L(q_dim, q_dim, bias=out_bias), torch.nn.Dropout(0.0)])
        self.spatial_norm = None
        self.group_norm = None
        self.norm_cross = None
        self.residual_connection = False
        self.rescale_output_factor = 1.0


def fill_attention(attn, gen, T, prefix, lora_rank=None, lowrank=8):
    for name in ("to_q", "to_k", "to_v", "to_out.0"):
        lin = attn.to_out[0] if name == "to_out.0" else getattr(attn, name)
        of, inf = lin.weight.shape
        wf = S.make(of, inf, lowrank, gen)
        lin.weight.copy_(S.rebuild(wf, of, inf))
        S.store(f"{prefix}{name}.W", wf, T)
        if lin.bias is not None:
            lin.bias.copy_(bf(torch.randn(of, generator=gen) * 0.1))
            T[f"{prefix}{name}.b"] = lin.bias.detach().clone()
        if lora_rank:
            layer = make_unziplora(gen, inf, of, lora_rank)
            lin.set_lora_layer(layer)
            dump_unziplora(layer, f"{prefix}{name}.lora.", T)


def gen_processor():
    gen = torch.Generator().manual_seed(3)
    proc = AnimateDiffAttnProcessor2_0()
    T, meta = {}, {}
    # spatial self-attention with UnZipLoRA on q/k/v/out (C=320, 5 heads of 64, N=64 tokens)
    a = DuckAttention(320, 320, 5, lora=True)
    fill_attention(a, gen, T, "self.", lora_rank=8)
    x = bf(torch.randn(2, 64, 320, generator=gen))
    T["self.x"] = x
    for mode in ("both", "content", "style"):
        for m in (a.to_q, a.to_k, a.to_v, a.to_out[0]):
            m.lora_layer.set_forward(mode)
        T[f"self.out_{mode}"] = proc(a, x)
        T[f"self.out_{mode}_s05"] = proc(a, x, scale=0.5)
    for m in (a.to_q, a.to_k, a.to_v, a.to_out[0]):
        m.lora_layer.set_forward("both")
    with torch.autocast("cpu", dtype=torch.bfloat16):
        T["self.out_both_autocast_bf16"] = proc(a, x).float()
    meta["self"] = {"C": 320, "heads": 5, "N": 64, "batch": 2, "rank": 8}
    # cross-attention: hidden (B*F=4, 16, 128), text (B=1... repeat to 4) 77 x 2048, 2 heads of 64
    c = DuckAttention(128, 2048, 2, lora=True)
    fill_attention(c, gen, T, "cross.", lora_rank=8)
    xh = bf(torch.randn(4, 16, 128, generator=gen))
    enc = bf(torch.randn(2, 77, 2048, generator=gen))
    T["cross.x"] = xh
    T["cross.enc"] = enc
    T["cross.out_both"] = proc(c, xh, encoder_hidden_states=enc)
    meta["cross"] = {"C": 128, "heads": 2, "Nq": 16, "Nk": 77, "batch": 4, "kv_batch": 2, "rank": 8}
    save("processor", T, meta)


def gen_temporal_core():
    """motion-module attention core: processor with heads=8, d=C/8, over (B*HW, F, C)."""
    gen = torch.Generator().manual_seed(4)
    proc = AnimateDiffAttnProcessor2_0()
    T, meta = {}, {"cases": []}
    for (C, Fr, nseq) in [(320, 16, 8), (640, 32, 4), (1280, 16, 2), (64, 5, 6)]:
        tag = f"C{C}_F{Fr}"
        a = DuckAttention(C, C, 8, lora=False)
        fill_attention(a, gen, T, tag + ".")
        x = bf(torch.randn(nseq, Fr, C, generator=gen))
        T[tag + ".x"] = x
        T[tag + ".out"] = proc(a, x)
        meta["cases"].append([C, Fr, nseq])
    save("temporal_core", T, meta)


# --------------------------------------------------------------------------- 5. TemporalTransformer
def gen_temporal_transformer():
    gen = torch.Generator().manual_seed(5)
    T = {}
    C = 320
    tt = TemporalTransformer(C, num_layers=2, num_heads=8)
    tt.eval()
    for name, p in tt.named_parameters():
        if p.dim() == 2:
            wf = S.make(p.shape[0], p.shape[1], 8, gen, diag_scale=0.5)
            p.copy_(S.rebuild(wf, p.shape[0], p.shape[1]))
            S.store(name, wf, T)
        else:
            if name.endswith("weight"):
                p.copy_(bf(1.0 + 0.1 * torch.randn(p.shape, generator=gen)))
            else:
                p.copy_(bf(0.1 * torch.randn(p.shape, generator=gen)))
            T[name] = p.detach().clone()
    x = bf(torch.randn(1, C, 16, 8, 8, generator=gen))
    T["x"] = x
    T["out"] = tt(x, num_frames=16)
    T["pe"] = PositionalEncoding(C, 32).pe.clone()
    T["pe_d80"] = PositionalEncoding(80, 32).pe.clone()
    save("temporal_transformer", T, {"C": C, "layers": 2, "heads": 8, "shape": [1, C, 16, 8, 8]})


# --------------------------------------------------------------------------- 6-8. temporal LoRA
class _Attn(torch.nn.Module):
    def __init__(self, C, with_lora):
        super().__init__()
        L = LoRACompatibleLinear if with_lora else torch.nn.Linear
        self.to_q = L(C, C, bias=False)
        self.to_k = L(C, C, bias=False)
        self.to_v = L(C, C, bias=False)
        self.to_out = torch.nn.ModuleList([L(C, C, bias=True), torch.nn.Dropout(0.0)])


class _Block(torch.nn.Module):
    def __init__(self, C, with_lora):
        super().__init__()
        self.attn1 = _Attn(C, with_lora)
        self.attn2 = _Attn(C, with_lora)


class _Tr(torch.nn.Module):
    def __init__(self, C, with_lora):
        super().__init__()
        self.transformer_blocks = torch.nn.ModuleList([_Block(C, with_lora)])


class _Down(torch.nn.Module):
    def __init__(self, C):
        super().__init__()
        self.attentions = torch.nn.ModuleList([_Tr(C, True), _Tr(C, True)])
        self.motion_modules = torch.nn.ModuleList([_Tr(C, False), _Tr(C, False)])


class _Unet(torch.nn.Module):
    def __init__(self, C):
        super().__init__()
        self.down_blocks = torch.nn.ModuleList([_Down(C)])


def gen_temporal_lora():
    gen = torch.Generator().manual_seed(6)
    T = {}
    C = 64
    u = _Unet(C)
    for n, p in u.named_parameters():
        p.copy_(bf(torch.randn(p.shape, generator=gen) * 0.1))
    for n, m in u.named_modules():
        if isinstance(m, LoRACompatibleLinear):
            m.set_lora_layer(make_unziplora(gen, m.in_features, m.out_features, 8))
    n_wrapped = inject_temporal_lora(u, rank=32, alpha=1.0)
    for n, m in u.named_modules():
        if isinstance(m, TemporalLoRALinear):
            m.lora_A.copy_(bf(torch.randn(m.lora_A.shape, generator=gen) * 0.01))
            m.lora_B.copy_(bf(torch.randn(m.lora_B.shape, generator=gen) * 0.01))
    sd = {k: v.detach().clone() for k, v in u.state_dict().items()}
    for k, v in sd.items():
        T["sd." + k] = v
    # one TemporalLoRALinear forward / get_delta / merged_weight
    mod = u.down_blocks[0].motion_modules[0].transformer_blocks[0].attn1.to_out[0]
    x = bf(torch.randn(3, 16, C, generator=gen))
    T["x"] = x
    T["fwd"] = mod(x)
    T["delta"] = mod.get_delta()
    T["merged"] = mod.merged_weight()
    idx = build_spatial_lora_index(u)
    T["orth_loss"] = compute_orth_loss(u, idx, 0.1).reshape(1)
    merged = get_merged_motion_state_dict(u)
    for k, v in merged.items():
        T["merged_sd." + k] = v
    meta = {"C": C, "rank": 32, "alpha": 1.0, "lambda": 0.1, "n_wrapped": n_wrapped, "index": sorted(idx.keys()),
            "merged_keys": sorted(merged.keys()),
            "fwd_module": "down_blocks.0.motion_modules.0.transformer_blocks.0.attn1.to_out.0"}
    save("temporal_lora", T, meta)


if __name__ == "__main__":
    gen_unziplora()
    gen_lora_linear()
    gen_lora_unzip()
    gen_processor()
    gen_temporal_core()
    gen_temporal_transformer()
    gen_temporal_lora()
