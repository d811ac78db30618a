"""CPU checks of the VAE host side: diffusers AutoencoderKL parameter names / shapes, oracle shapes, and that the HIP
module refuses CPU tensors (no CPU fallback)."""
import pytest
import torch

from oracle import vae as OV
from video_style_transfer_amd.config import VAEConfig
from video_style_transfer_amd.vae import AutoencoderKL
from video_style_transfer_amd.weights import vae_param_shapes, vae_synthetic_state_dict


def test_sdxl_vae_inventory():
    cfg = VAEConfig.sdxl()
    S = vae_param_shapes(cfg)
    assert sum(torch.Size(s).numel() for s, _ in S.values()) == 83653863  # SDXL VAE parameter count
    for k in ("decoder.mid_block.attentions.0.to_out.0.weight", "encoder.down_blocks.0.downsamplers.0.conv.weight",
              "decoder.up_blocks.2.resnets.0.conv_shortcut.weight", "post_quant_conv.weight", "quant_conv.bias"):
        assert k in S
    m = AutoencoderKL(cfg)
    assert {k: tuple(v.shape) for k, v in m.state_dict().items()} == {k: tuple(s) for k, (s, _) in S.items()}


def test_oracle_shapes_tiny():
    cfg = VAEConfig.tiny()
    P = vae_synthetic_state_dict(cfg, 0)
    x = torch.rand(2, 3, 32, 32) * 2 - 1
    mom = OV.encode_moments(P, cfg.to_dict(), x)
    assert mom.shape == (2, 8, 8, 8)
    z = OV.latent_sample(mom, torch.randn(2, 4, 8, 8))
    y = OV.decode(P, cfg.to_dict(), z)
    assert y.shape == (2, 3, 32, 32) and torch.isfinite(y).all()
    assert OV.frames_u8(y).dtype == torch.uint8


def test_vae_refuses_cpu_tensors():
    pytest.importorskip("ctypes")
    vae = AutoencoderKL(VAEConfig.tiny())
    with pytest.raises(RuntimeError):
        vae.decode(torch.zeros(1, 4, 8, 8))
    with pytest.raises(RuntimeError):
        vae.encode(torch.zeros(1, 3, 32, 32))
