"""Image-path dual-prompt LoRA linear — kernel-backed mirror of unziplora_unet/lora_unzip.py.

`LoRACompatibleLinear.forward(hidden_states, scale, hidden_states_1, hidden_states_2)` (lora_unzip.py:66-75)
= hidden_states W^T + b + scale * lora_layer(hidden_states_1, hidden_states_2): the base weight sees the joint
prompt, the UnZipLoRA content branch the content prompt and the style branch the style prompt
(unzip_attention_processor.py:707-725).  On the device it is the same single fused GEMM as the text-path
projection, with the low-rank activations taken from different inputs:
    u = [x_1 A_c^T | x_2 A_s^T]            (skinny GEMMs; the style columns of the second are copied in)
    y = [x | u] . [W | scale * (B_c*m_c | B_s*m_s)]^T + b
so x_1 != x_2 != x costs two skinny GEMMs and one column copy more than the text path, nothing dense.

Reference defect handled: its AttnProcessor2_0 passes `hidden_states_content=` /
`hidden_states_style=` while this forward names them `hidden_states_1` / `_2` (a TypeError in the reference);
both spellings are accepted here.  A missing branch input falls back to `hidden_states` (the reference would hand
None to its LoRA layer and fail).
"""
from __future__ import annotations

import torch

from . import kernels as K
from .lora_linear import LoRACompatibleLinear as _TextPathLinear
from .lora_linear import build_ops, run_ops


def _pick(*cands):
    for c in cands:
        if c is not None:
            return c
    return None


def dual_prompt_lora_down(lin, ops, x1: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """u = [x1 A_c^T | x2 A_s^T | 0-pad] in the column order build_ops stacked the active branches."""
    u = K.linear(x1, ops.a, kind="gemm_lora_down", alg_n=ops.r)
    if x2 is x1:
        return u
    parts = lin.lora_layer.lowrank_factors(1.0, split=True)
    col = 0
    for key, (A, _) in parts.items():
        r = A.shape[0]
        if key == "style" and r:
            u2 = K.linear(x2, ops.a, kind="gemm_lora_down", alg_n=ops.r)
            K.copy2d(u2[:, col:col + r], u[:, col:col + r])
        col += r
    return u


class LoRACompatibleLinear(_TextPathLinear):
    """lora_unzip.py:6-75 (set_lora_layer / _fuse_lora / _unfuse_lora as the text-path class)."""

    def forward(self, hidden_states: torch.Tensor, scale: float = 1.0, hidden_states_1: torch.Tensor = None,
                hidden_states_2: torch.Tensor = None, *, hidden_states_content: torch.Tensor = None,
                hidden_states_style: torch.Tensor = None) -> torch.Tensor:
        if not hidden_states.is_cuda:
            raise K._lib.VstError("lora_unzip.LoRACompatibleLinear: input is on CPU; the HIP path has no CPU fallback")
        shape = hidden_states.shape[:-1] + (self.out_features,)
        x = hidden_states.reshape(-1, self.in_features)
        if self.lora_layer is None:
            return run_ops(x, build_ops([self], scale)).view(shape)
        x1 = _pick(hidden_states_1, hidden_states_content, hidden_states).reshape(-1, self.in_features)
        x2 = _pick(hidden_states_2, hidden_states_style, hidden_states).reshape(-1, self.in_features)
        if x1.shape != x.shape or x2.shape != x.shape:
            raise ValueError(f"lora_unzip: branch inputs {tuple(x1.shape)}/{tuple(x2.shape)} vs {tuple(x.shape)}")
        # the low-rank terms read other inputs than the base: never pre-fold them into W
        ops = build_ops([self], scale, mode="fused")
        if ops.a is None:
            return run_ops(x, ops).view(shape)
        same = (x1.data_ptr() == x.data_ptr() and x2.data_ptr() == x.data_ptr())
        if same:
            return run_ops(x, ops).view(shape)
        if x2.data_ptr() == x1.data_ptr():
            x2 = x1
        u = dual_prompt_lora_down(self, ops, x1.contiguous(), x2 if x2 is x1 else x2.contiguous())
        return run_ops(x, ops, u=u).view(shape)
