"""LoRA-capable linear layers — kernel-backed mirror of unziplora_unet/lora_linear.py
(itself diffusers 0.27 `lora.py`), plus the projection-operand builder every attention
processor uses.

`LoRACompatibleLinear.forward(x, scale)` = x W^T + b + scale * lora_layer(x)  (lora_linear.py:74-81).
On the device this is ONE bf16 MFMA GEMM over an augmented K dimension:
    [x | x A^T] . [W | scale * V]^T + b
where (A, V) are the layer's low-rank factors (UnZipLoRA: A = [A_c; A_s], V = [B_c*m_c | B_s*m_s];
plain LoRA: A = down, V = up * alpha/rank; TemporalLoRALinear: A = lora_A, V = lora_B * alpha/rank),
and x A^T is one skinny GEMM.  Projections that share an input (q/k/v, or k/v of cross-attention)
are concatenated into one GEMM with their factors stacked.

LoRA mode (set_lora_mode): "fused" (default) keeps the delta low-rank inside the GEMM every call;
"folded" pre-merges W + scale * V A once per weight/forward-type change (exactly the
reference's `_fuse_lora` arithmetic, lora_linear.py:49-62) — zero per-call overhead for frozen
inference weights.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

import torch
from torch import nn

from . import kernels as K

_LORA_MODE = "fused"


def set_lora_mode(mode: str):
    global _LORA_MODE
    assert mode in ("fused", "folded")
    _LORA_MODE = mode


def get_lora_mode() -> str:
    return _LORA_MODE


def pad32(n: int) -> int:
    return (n + 31) // 32 * 32


class LoRALinearLayer(nn.Module):
    """lora_linear.py:10-38 (diffusers LoRALinearLayer): up(down(x)) * alpha/rank."""

    def __init__(self, in_features, out_features, rank=4, network_alpha=None, device=None, dtype=None):
        super().__init__()
        self.down = nn.Linear(in_features, rank, bias=False, device=device, dtype=dtype)
        self.up = nn.Linear(rank, out_features, bias=False, device=device, dtype=dtype)
        self.network_alpha = network_alpha
        self.rank = rank
        self.out_features = out_features
        self.in_features = in_features
        nn.init.normal_(self.down.weight, std=1 / rank)
        nn.init.zeros_(self.up.weight)

    def state_key(self):
        return ("lora", self.network_alpha, tuple((p.data_ptr(), p._version) for p in (self.down.weight, self.up.weight)))

    def lowrank_factors(self, scale=1.0):
        s = scale * (self.network_alpha / self.rank if self.network_alpha is not None else 1.0)
        return self.down.weight.float(), self.up.weight.float() * s

    def forward(self, hidden_states):
        A, V = self.lowrank_factors(1.0)
        x = hidden_states.reshape(-1, self.in_features)
        Ap = _pad_rows(A).to(torch.bfloat16)
        Vp = _pad_cols(V).to(torch.bfloat16)
        out = K.linear(K.linear(x, Ap), Vp)
        return out.view(hidden_states.shape[:-1] + (self.out_features,))


def _pad_rows(A):
    P = pad32(max(A.shape[0], 1))
    if P == A.shape[0]:
        return A.contiguous()
    out = A.new_zeros(P, A.shape[1])
    out[: A.shape[0]] = A
    return out


def _pad_cols(V):
    P = pad32(max(V.shape[1], 1))
    if P == V.shape[1]:
        return V.contiguous()
    out = V.new_zeros(V.shape[0], P)
    out[:, : V.shape[1]] = V
    return out


@dataclass
class ProjOps:
    w: torch.Tensor                  # bf16 [N, K1 (+P)]
    a: Optional[torch.Tensor]        # bf16 [P, K1] or None
    bias: Optional[torch.Tensor]     # fp32 [N] or None
    k1: int
    n: int
    r: int = 0                       # real (unpadded) low-rank width
    gn: int = 0                      # output columns per projection when every projection has the same width and
    gr: int = 0                      # rank (u columns [g gr, (g+1) gr) feed rows [g gn, (g+1) gn)); 0 = irregular


def _linear_parts(lin):
    """(W, b, lowrank_source or None) for any projection module on the path."""
    from .temporal_lora import TemporalLoRALinear  # local import: temporal_lora imports this module
    if isinstance(lin, TemporalLoRALinear):
        return lin.base.weight, lin.base.bias, lin
    lora = getattr(lin, "lora_layer", None)
    return lin.weight, lin.bias, lora


def _state_key(lin, scale, mode):
    W, b, lora = _linear_parts(lin)
    k = (W.data_ptr(), W._version, None if b is None else (b.data_ptr(), b._version))
    if lora is not None:
        k = k + (lora.state_key(), scale)
    return k + (mode,)


def build_ops(lins: Sequence[nn.Module], scale: float = 1.0, mode: Optional[str] = None) -> ProjOps:
    """Concatenated operands for projections sharing one input (cached on lins[0])."""
    mode = mode or _LORA_MODE
    key = (tuple(id(l) for l in lins), float(scale), mode)
    skey = tuple(_state_key(l, scale, mode) for l in lins)
    # operands of parameters that train are rebuilt per call: HIP-graph replay of a training step updates them
    # without a version bump, so a version-keyed cache would go stale
    cacheable = not any(p.requires_grad for l in lins for p in l.parameters())
    cache = lins[0].__dict__.setdefault("_vst_ops_cache", {})
    hit = cache.get(key) if cacheable else None
    if hit is not None and hit[0] == skey:
        return hit[1]
    with torch.no_grad():
        Ws, bs, As, Vs = [], [], [], []
        for l in lins:
            W, b, lora = _linear_parts(l)
            Wf = W.float()
            A = V = None
            if lora is not None:
                s = scale if not hasattr(lora, "is_temporal_lora") else 1.0
                A, V = lora.lowrank_factors(s)
                if A.shape[0] == 0:
                    A = V = None
            if mode == "folded" and A is not None:
                Wf = Wf + V @ A
                A = V = None
            Ws.append(Wf)
            bs.append(None if b is None else b.float())
            As.append(A)
            Vs.append(V)
        dev = Ws[0].device
        N = sum(w.shape[0] for w in Ws)
        K1 = Ws[0].shape[1]
        R = sum(0 if a is None else a.shape[0] for a in As)
        if R > 0:
            P = pad32(R)
            A_all = torch.zeros(P, K1, device=dev)
            W_all = torch.zeros(N, K1 + P, device=dev)
            o_r = o_n = 0
            for w, a, v in zip(Ws, As, Vs):
                W_all[o_n:o_n + w.shape[0], :K1] = w
                if a is not None:
                    A_all[o_r:o_r + a.shape[0]] = a
                    W_all[o_n:o_n + w.shape[0], K1 + o_r:K1 + o_r + a.shape[0]] = v
                    o_r += a.shape[0]
                o_n += w.shape[0]
            a_bf = A_all.to(torch.bfloat16).contiguous()
        else:
            W_all = torch.cat(Ws, 0)
            a_bf = None
        bias = None
        if any(b is not None for b in bs):
            bias = torch.cat([b if b is not None else torch.zeros(w.shape[0], device=dev) for w, b in zip(Ws, bs)])
            bias = bias.contiguous()
        gn = gr = 0
        if a_bf is not None and len({w.shape[0] for w in Ws}) == 1 and \
                len({0 if a is None else a.shape[0] for a in As}) == 1:
            gn, gr = Ws[0].shape[0], As[0].shape[0]
        ops = ProjOps(W_all.to(torch.bfloat16).contiguous(), a_bf, bias, K1, N, R if a_bf is not None else 0, gn, gr)
    if cacheable:
        cache[key] = (skey, ops)
    return ops


def lora_in_gemm(ops: ProjOps, rows: int) -> bool:
    """True when run_ops(x, ops) over `rows` rows computes the LoRA down-projection inside the projection GEMM
    (K.linear_lora), so a producer need not emit u = x @ ops.a^T (LayerNorm.run_lora checks this first)."""
    return ops.a is not None and ops.gn > 0 and \
        K.gemm_lora_tile(rows, ops.n, ops.k1, ops.a.shape[0], ops.gn, ops.gr) > 0


def run_ops(x2d: torch.Tensor, ops: ProjOps, residual=None, out=None, geglu=False, u=None) -> torch.Tensor:
    """`u` = x2d @ ops.a^T when the producer already computed it (K.layer_norm_lora); otherwise the down-projection
    runs inside the projection GEMM where the shape allows (K.linear_lora), else as its own skinny GEMM."""
    if ops.a is None:
        return K.linear(x2d, ops.w, ops.bias, residual=residual, out=out, geglu=geglu)
    if u is None and not geglu and lora_in_gemm(ops, x2d.shape[0]):
        return K.linear_lora(x2d, ops.w, ops.a, ops.gn, ops.gr, ops.bias, residual=residual, out=out, r_alg=ops.r)
    if u is None:
        u = K.linear(x2d, ops.a, kind="gemm_lora_down", alg_n=ops.r)
    return K.linear(x2d, ops.w, ops.bias, x2=u, residual=residual, out=out, geglu=geglu, alg_k2=ops.r)


class LoRACompatibleLinear(nn.Linear):
    """lora_linear.py:41-81.  forward(hidden_states, scale) -> base + scale * lora_layer(hidden_states)."""

    def __init__(self, *args, lora_layer: Optional[nn.Module] = None, **kwargs):
        super().__init__(*args, **kwargs)
        self.lora_layer = lora_layer

    def set_lora_layer(self, lora_layer: Optional[nn.Module]):
        self.lora_layer = lora_layer

    def _fuse_lora(self, lora_scale: float = 1.0, safe_fusing: bool = False):
        """lora_linear.py:49-62: W <- W + scale * (up @ down), drop the layer."""
        if self.lora_layer is None:
            return
        A, V = self.lora_layer.lowrank_factors(lora_scale)
        fused = self.weight.data.float() + V @ A
        if safe_fusing and torch.isnan(fused).any().item():
            raise ValueError("NaN detected in fused LoRA weight.")
        self.w_up, self.w_down, self.lora_scale = V.detach().clone(), A.detach().clone(), 1.0
        self.weight.data = fused.to(self.weight.dtype)
        self.lora_layer = None

    def _unfuse_lora(self):
        if getattr(self, "w_up", None) is None or getattr(self, "w_down", None) is None:
            return
        self.weight.data = (self.weight.data.float() - self.lora_scale * (self.w_up @ self.w_down)).to(self.weight.dtype)
        self.w_up = self.w_down = None

    def forward(self, hidden_states: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
        if not hidden_states.is_cuda:
            # CPU tensors: plain eager semantics are NOT provided — the product path is the HIP kernel.
            raise K._lib.VstError("LoRACompatibleLinear: input is on CPU; the HIP path has no CPU fallback")
        x = hidden_states.reshape(-1, self.in_features)
        ops = build_ops([self], scale)
        out = run_ops(x, ops)
        return out.view(hidden_states.shape[:-1] + (self.out_features,))


def plain_linear_ops(lin: nn.Linear) -> ProjOps:
    return build_ops([lin], 1.0)

