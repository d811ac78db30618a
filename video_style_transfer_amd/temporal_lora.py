"""Temporal LoRA for the motion modules — mirror of animatediff/temporal_lora.py.

TemporalLoRALinear keeps the reference's attribute names (`base`, `lora_A`, `lora_B`, `scale`,
`rank`) because `freeze_spatial_layers` string-matches them (animatediff/utils.py:79-85).
Its forward is the same augmented-K GEMM as every other projection (lora_linear.build_ops):
[x | x A^T] . [W | scale * B]^T + b.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn

from .lora_linear import build_ops, run_ops


class TemporalLoRALinear(nn.Module):
    """temporal_lora.py:10-41.  W_base + (alpha/rank) * lora_B @ lora_A; A ~ N(0, 0.01), B = 0."""
    is_temporal_lora = True

    def __init__(self, base: nn.Linear, rank: int = 32, alpha: float = 1.0):
        super().__init__()
        self.base = base
        self.base.weight.requires_grad_(False)
        if self.base.bias is not None:
            self.base.bias.requires_grad_(False)
        self.in_features = base.in_features
        self.out_features = base.out_features
        self.rank = rank
        self.scale = alpha / rank
        dev = base.weight.device
        self.lora_A = nn.Parameter(torch.randn(rank, base.in_features, device=dev) * 0.01)
        self.lora_B = nn.Parameter(torch.zeros(base.out_features, rank, device=dev))

    # operand-builder protocol
    def state_key(self):
        return ("tlora", self.scale, tuple((p.data_ptr(), p._version) for p in (self.lora_A, self.lora_B)))

    def lowrank_factors(self, scale: float = 1.0):
        return self.lora_A.float(), self.lora_B.float() * self.scale

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if torch.is_grad_enabled() and (self.lora_A.requires_grad or self.lora_B.requires_grad
                                        or self.base.weight.requires_grad):
            # training (train_animatediff.py:265-319): HIP forward + backward through autograd.LoRALinearFn
            from .autograd import lora_linear
            return lora_linear(x, self.base.weight, self.base.bias, self.lora_A, self.lora_B, self.scale, self)
        x2 = x.reshape(-1, self.in_features)
        out = run_ops(x2, build_ops([self], 1.0))
        return out.view(x.shape[:-1] + (self.out_features,))

    def get_delta(self) -> torch.Tensor:
        """(out, in) low-rank delta (temporal_lora.py:34-36)."""
        return (self.lora_B @ self.lora_A) * self.scale

    def merged_weight(self) -> torch.Tensor:
        with torch.no_grad():
            return (self.base.weight.float() + self.get_delta().float()).to(self.base.weight.dtype).detach()


def inject_temporal_lora(unet, rank: int = 32, alpha: float = 1.0) -> int:
    """temporal_lora.py:44-69: wrap motion-module to_q/k/v/to_out[0] (idempotent)."""
    count = 0
    for name, module in list(unet.named_modules()):
        if "motion_modules" not in name:
            continue
        if not all(hasattr(module, a) for a in ("to_q", "to_k", "to_v", "to_out")):
            continue
        if isinstance(getattr(module, "to_q", None), TemporalLoRALinear):
            continue
        for proj in ("to_q", "to_k", "to_v"):
            lin = getattr(module, proj, None)
            if isinstance(lin, nn.Linear):
                setattr(module, proj, TemporalLoRALinear(lin, rank, alpha))
                count += 1
        if len(module.to_out) > 0 and isinstance(module.to_out[0], nn.Linear):
            module.to_out[0] = TemporalLoRALinear(module.to_out[0], rank, alpha)
            count += 1
    return count


def build_spatial_lora_index(unet) -> Dict[str, object]:
    """temporal_lora.py:72-123: temporal wrapped linear name -> paired spatial UnZipLoRA layer."""
    spatial = {}
    for name, module in unet.named_modules():
        if "motion_modules" in name:
            continue
        lora = getattr(module, "lora_layer", None)
        if lora is not None:
            spatial[name] = lora
    index = {}
    for name, module in unet.named_modules():
        if "motion_modules" not in name or not isinstance(module, TemporalLoRALinear):
            continue
        parts = name.split(".")
        mm = parts.index("motion_modules")
        prefix = ".".join(parts[:mm])
        mm_index = parts[mm + 1]
        after = parts[mm + 2:]
        if "temporal_transformer" in after:
            after = after[after.index("temporal_transformer") + 1:]
        path = prefix + ".attentions." + mm_index + "." + ".".join(after)
        lora = spatial.get(path)
        if lora is None:
            continue
        try:
            B_c = lora.lora_matrix_dic.content_up.weight
            A_c = lora.lora_matrix_dic.content_down.weight
        except AttributeError:
            continue
        if B_c.shape[0] == module.out_features and A_c.shape[1] == module.in_features:
            index[name] = lora
    return index


def compute_orth_loss(unet, spatial_index: Dict, lambda_orth: float) -> torch.Tensor:
    """temporal_lora.py:126-166: lambda/N * sum ||dT^T dC||_F^2 + ||dT^T dS||_F^2.

    Evaluated low-rank: dT^T dC = A_t^T (B_t^T B_c)(A_c) scaled, so ||.||_F^2 =
    trace(G_t (B_t^T B_c) G_c (B_t^T B_c)^T) with G = A A^T (r x r) — O(r^2 * C) instead of the
    reference's two dense C x C x C products per pair.  Same value, same gradient."""
    if lambda_orth == 0.0 or not spatial_index:
        return torch.tensor(0.0)
    total: Optional[torch.Tensor] = None
    count = 0
    for name, module in unet.named_modules():
        if name not in spatial_index or not isinstance(module, TemporalLoRALinear):
            continue
        lora = spatial_index[name]
        At = module.lora_A.float()
        Bt = module.lora_B.float() * module.scale
        Gt = At @ At.t()
        contrib = None
        for key in ("content", "style"):
            with torch.no_grad():
                Bs = lora.lora_matrix_dic[f"{key}_up"].weight.float()
                As = lora.lora_matrix_dic[f"{key}_down"].weight.float()
                Gs = As @ As.t()
            M = Bt.t() @ Bs  # (r_t, r_s)
            val = torch.sum((Gt @ M) * (M @ Gs))  # trace(Gt M Gs M^T)
            contrib = val if contrib is None else contrib + val
        total = contrib if total is None else total + contrib
        count += 1
    if total is None:
        return torch.tensor(0.0)
    return lambda_orth * total / count


def get_merged_motion_state_dict(unet) -> Dict[str, torch.Tensor]:
    """temporal_lora.py:169-192: motion_modules state dict with deltas folded, original key names."""
    merged, wrapped = {}, set()
    for name, module in unet.named_modules():
        if not isinstance(module, TemporalLoRALinear) or "motion_modules" not in name:
            continue
        merged[name + ".weight"] = module.merged_weight().cpu()
        if module.base.bias is not None:
            merged[name + ".bias"] = module.base.bias.detach().cpu()
        wrapped.add(name)
    for k, v in unet.state_dict().items():
        if "motion_modules" not in k or any(k.startswith(w + ".") for w in wrapped):
            continue
        merged[k] = v.detach().cpu()
    return merged
