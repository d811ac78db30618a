"""Locate GroupNorm mismatches: per (sample, group) and per-row error of K.group_norm vs torch."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from video_style_transfer_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
for ns, rps, C in [(1, 4096, 1280), (1, 4096, 320), (2, 1000, 640)]:
    g = torch.Generator().manual_seed(ns * rps + C)
    x = (torch.randn(ns * rps, C, generator=g)).to(torch.bfloat16) + 0.5
    gam, bet = torch.ones(C), torch.zeros(C)
    out = K.group_norm(x.to(dev), ns, rps, 32, 1e-5, gam.to(dev), bet.to(dev)).float().cpu()
    ref = F.group_norm(x.float().view(ns, rps, C).permute(0, 2, 1), 32, gam, bet, 1e-5).permute(0, 2, 1).reshape(-1, C)
    err = (out - ref).abs()
    eg = err.view(ns, rps, 32, C // 32).amax((1, 3))
    er = err.view(ns, rps, C).amax(2)
    print(ns, rps, C, "max", err.max().item(), "groups>0.02:", (eg > 0.02).nonzero().tolist()[:10],
          "rows>0.02:", (er > 0.02).nonzero()[:, 1].tolist()[:20], flush=True)
    og = out.view(ns, rps, 32, C // 32)
    print("  out |mean| max", og.mean((1, 3)).abs().max().item(), "|std-1| max",
          (og.std((1, 3)) - 1).abs().max().item(), flush=True)
