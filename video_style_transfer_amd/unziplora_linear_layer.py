"""UnZipLoRA inference layer — kernel-backed mirror of
unziplora_unet/unziplora_linear_layer.py:265-346 (UnZipLoRALinearLayerInfer).

Same constructor, parameters (`lora_matrix_dic.{content,style}_{down,up}`, `merge_content`,
`merge_style`), state-dict keys, `set_forward` / `set_layer_mask` API and forward semantics:
  "both":    x_c @ ((A_c^T B_c^T) * m_c) + x_s @ ((A_s^T B_s^T) * m_s)
  "content": x_c @ (A_c^T B_c^T)            (no merger — reference :331)
  "style":   x_s @ (A_s^T B_s^T)            (no merger — reference :343)
  a masked key contributes zeros (:308-317).
The reference materialises two dense in x out matrices and runs two full-rank GEMMs per call.
Here the delta stays low-rank: `fused_operands()` returns (Acat, V) with
Acat = [A_c; A_s] (zero-padded to a multiple of 32 rows) and V = [B_c * m_c | B_s * m_s], so the
delta is (x Acat^T) V^T; LoRACompatibleLinear folds V into extra K columns of its base GEMM.
"""
from __future__ import annotations

from typing import List, Optional, Union

import torch
from torch import nn

from . import kernels as K

KEYS = ("content", "style")


def pad32(n: int) -> int:
    return (n + 31) // 32 * 32


class UnZipLoRALinearLayerInfer(nn.Module):
    def __init__(self, in_features: int, out_features: int, rank: int = 64, lora_matrix_key: List[str] = None,
                 device: Optional[Union[torch.device, str]] = None, dtype: Optional[torch.dtype] = None):
        super().__init__()
        lora_matrix_key = list(lora_matrix_key or KEYS)
        self.lora_matrix_dic = nn.ModuleDict()
        self.masked_matrix = {}
        for key in lora_matrix_key:
            self.lora_matrix_dic[f"{key}_down"] = nn.Linear(in_features, rank, bias=False, device=device, dtype=dtype)
            self.lora_matrix_dic[f"{key}_up"] = nn.Linear(rank, out_features, bias=False, device=device, dtype=dtype)
            nn.init.normal_(self.lora_matrix_dic[f"{key}_down"].weight, std=1 / rank)
            nn.init.normal_(self.lora_matrix_dic[f"{key}_up"].weight, std=1 / rank)
            self.masked_matrix[key] = False
        self.lora_matrix_key = lora_matrix_key
        self.in_features = in_features
        self.out_features = out_features
        self.rank = rank
        self.forward_type = "both"
        self.dtype = dtype
        self.merge_content = nn.Parameter(torch.ones(out_features, device=device, dtype=dtype))
        self.merge_style = nn.Parameter(torch.ones(out_features, device=device, dtype=dtype))

    # ---- reference API -----------------------------------------------------------------
    def set_layer_mask(self, key, value=True):
        self.masked_matrix[key] = value

    def set_forward(self, type: str = "both"):
        assert type in ["both", "content", "style"]
        self.forward_type = type

    # ---- low-rank operands -------------------------------------------------------------
    def active_terms(self):
        """[(key, use_merger)] that contribute under the current forward type / masks."""
        ft = self.forward_type
        terms = []
        if ft in ("both", "content") and not self.masked_matrix.get("content", False):
            terms.append(("content", ft == "both"))
        if ft in ("both", "style") and not self.masked_matrix.get("style", False):
            terms.append(("style", ft == "both"))
        return terms

    def state_key(self):
        ps = [self.merge_content, self.merge_style] + [m.weight for m in self.lora_matrix_dic.values()]
        return (self.forward_type, tuple(sorted(self.masked_matrix.items())),
                tuple((p.data_ptr(), p._version) for p in ps))

    def lowrank_factors(self, scale: float = 1.0, split: bool = False):
        """fp32 (A [R, in], V [out, R]) with delta(x) = (x A^T) V^T, R = #active terms * rank
        (unpadded; V carries `scale` and the mergers).  split=True -> {key: (A_key, V_key)}."""
        parts = {}
        for key, use_m in self.active_terms():
            A = self.lora_matrix_dic[f"{key}_down"].weight.float()
            B = self.lora_matrix_dic[f"{key}_up"].weight.float()
            if use_m:
                B = B * getattr(self, f"merge_{key}").float()[:, None]
            parts[key] = (A, B * scale)
        if split:
            return parts
        dev = self.merge_content.device
        if not parts:
            return torch.zeros(0, self.in_features, device=dev), torch.zeros(self.out_features, 0, device=dev)
        return torch.cat([a for a, _ in parts.values()], 0), torch.cat([v for _, v in parts.values()], 1)

    # ---- forward (standalone use; the projection path fuses instead) --------------------
    def forward(self, hidden_states_content: torch.Tensor, hidden_states_style: torch.Tensor = None) -> torch.Tensor:
        xc = hidden_states_content
        xs = xc if hidden_states_style is None else hidden_states_style
        if self.forward_type == "style" and hidden_states_style is None:
            xs = xc
        shape = xc.shape[:-1] + (self.out_features,)
        xc2 = xc.reshape(-1, self.in_features)
        xs2 = xs.reshape(-1, self.in_features)
        parts = self.lowrank_factors(1.0, split=True)
        out = None
        for key, (A, V) in parts.items():
            x = xc2 if key == "content" else xs2
            Ap = torch.zeros(pad32(A.shape[0]), A.shape[1], device=A.device)
            Vp = torch.zeros(V.shape[0], pad32(A.shape[0]), device=A.device)
            Ap[: A.shape[0]] = A
            Vp[:, : A.shape[0]] = V
            U = K.linear(x, Ap.to(torch.bfloat16))
            out = K.linear(U, Vp.to(torch.bfloat16), residual=out)
        if out is None:
            out = torch.zeros(xc2.shape[0], self.out_features, dtype=xc.dtype, device=xc.device)
        return out.view(shape)
