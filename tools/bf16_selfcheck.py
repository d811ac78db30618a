"""Precision yardstick for the SDXL-architecture parity gate: the fp32 oracle UNet forward (F=2, 64x64 latent, seed 11)
vs the SAME oracle under torch.autocast(cpu, bf16) -- what a plain bf16 implementation of the reference math (the
reference runs under autocast bf16, inference_animatediff.py:98-101) deviates by.  Measured: rel-L2 1.53e-1, rel-max 2.1e-1."""
import sys, time, torch
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from oracle.unet import unet_forward
from video_style_transfer_amd.config import UNetMotionConfig
from video_style_transfer_amd.weights import synthetic_state_dict
torch.set_num_threads(8)
cfg = UNetMotionConfig.sdxl()
sd = synthetic_state_dict(cfg, 11, 8)
sd = {k: (v if "lora_layer" in k else v.to(torch.bfloat16).float()) for k, v in sd.items()}
g = torch.Generator().manual_seed(12)
B, Fr, hw = 2, 2, 64
BF = torch.bfloat16
lat = torch.randn(B, 4, Fr, hw, hw, generator=g).to(BF).float()
enc = torch.randn(B, 77, cfg.cross_attention_dim, generator=g).to(BF).float()
pooled = torch.randn(B, cfg.text_embed_dim, generator=g).to(BF).float()
tids = torch.tensor([[512, 512, 0, 0, 512, 512]] * B, dtype=torch.float32)
t = torch.tensor([601.0, 601.0])
with torch.no_grad():
    t0 = time.time(); ref = unet_forward(sd, cfg.to_dict(), lat, t, enc, pooled, tids); print('fp32', time.time() - t0, flush=True)
    t0 = time.time()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        rb = unet_forward(sd, cfg.to_dict(), lat, t, enc, pooled, tids).float()
    print('bf16 autocast', time.time() - t0)
print('oracle bf16-autocast vs fp32: rel_l2 %.3e rel_max %.3e' % (((rb - ref).norm() / ref.norm()).item(), ((rb - ref).abs().max() / ref.abs().max()).item()))
