"""Compact, exactly reconstructible weights for golden fixtures.

Large matrices in the fixtures are stored as W = diag-like(d) + U @ V^T (rank k) so the
committed files stay small; tests rebuild W with `rebuild`.  Used by make_golden.py and by
the tests that consume its fixtures.
"""
import torch


def make(out_f, in_f, rank, gen, diag_scale=1.0, lr_scale=None):
    n = min(out_f, in_f)
    d = (torch.rand(n, generator=gen) * 0.5 + 0.75) * diag_scale
    lr_scale = lr_scale if lr_scale is not None else 1.0 / (in_f ** 0.5)
    U = torch.randn(out_f, rank, generator=gen) * lr_scale
    V = torch.randn(in_f, rank, generator=gen)
    return {"d": d, "U": U, "V": V}


def rebuild(f, out_f, in_f):
    W = f["U"].float() @ f["V"].float().t()
    n = f["d"].numel()
    W[torch.arange(n), torch.arange(n)] += f["d"].float()
    return W


def store(prefix, factors, dst):
    for k, v in factors.items():
        dst[f"{prefix}.{k}"] = v.contiguous()


def load(prefix, src):
    return {k: src[f"{prefix}.{k}"] for k in ("d", "U", "V")}
