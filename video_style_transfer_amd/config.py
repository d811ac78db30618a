"""Architecture config of the UNetMotionModel the reference builds.

The reference loads SDXL base + the AnimateDiff SDXL motion adapter through diffusers
(`animatediff/utils.py:13-45`: UNet2DConditionModel.from_pretrained + UNetMotionModel.from_unet2d).
The values in `sdxl()` are the stabilityai/stable-diffusion-xl-base-1.0 unet config and the
guoyww/animatediff-motion-adapter-sdxl-beta adapter config (motion_layers_per_block=2, 8 motion
heads, motion_max_seq_length=32, no mid-block motion module).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field
from typing import Tuple


@dataclass
class UNetMotionConfig:
    in_channels: int = 4
    out_channels: int = 4
    block_out_channels: Tuple[int, ...] = (320, 640, 1280)
    down_block_types: Tuple[str, ...] = ("DownBlockMotion", "CrossAttnDownBlockMotion", "CrossAttnDownBlockMotion")
    up_block_types: Tuple[str, ...] = ("CrossAttnUpBlockMotion", "CrossAttnUpBlockMotion", "UpBlockMotion")
    layers_per_block: int = 2
    transformer_layers_per_block: Tuple[int, ...] = (1, 2, 10)
    num_attention_heads: Tuple[int, ...] = (5, 10, 20)  # head_dim 64 everywhere (SDXL)
    cross_attention_dim: int = 2048
    norm_num_groups: int = 32
    norm_eps: float = 1e-5
    addition_time_embed_dim: int = 256
    text_embed_dim: int = 1280  # pooled text embedding width
    num_time_ids: int = 6
    motion_num_attention_heads: int = 8
    motion_max_seq_length: int = 32
    motion_norm_num_groups: int = 32
    use_motion_mid_block: bool = False
    motion_modules: bool = True  # False: the plain SDXL UNet2DConditionModel (animatediff/utils.py:20), F = 1
    extra: dict = field(default_factory=dict)

    @property
    def time_embed_dim(self) -> int:
        return 4 * self.block_out_channels[0]

    @property
    def projection_class_embeddings_input_dim(self) -> int:
        return self.text_embed_dim + self.num_time_ids * self.addition_time_embed_dim

    def to_dict(self):
        return asdict(self)

    @classmethod
    def sdxl(cls) -> "UNetMotionConfig":
        return cls()

    @classmethod
    def sdxl_image(cls) -> "UNetMotionConfig":
        """The SDXL UNet2DConditionModel before the motion adapter (BASELINE configs[0];
        `UNet2DConditionModel.from_pretrained(subfolder="unet")`, animatediff/utils.py:20): same blocks, no motion
        modules; used with one frame per sample."""
        return cls(motion_modules=False)

    @classmethod
    def tiny(cls) -> "UNetMotionConfig":
        """Same topology as SDXL at test scale (head_dim 64 spatial, motion head_dim 8/16/32)."""
        return cls(block_out_channels=(64, 128, 256), transformer_layers_per_block=(1, 1, 2),
                   num_attention_heads=(1, 2, 4), cross_attention_dim=256, addition_time_embed_dim=32,
                   text_embed_dim=64)

    @classmethod
    def from_dict(cls, d):
        d = dict(d)
        for k in ("block_out_channels", "down_block_types", "up_block_types", "transformer_layers_per_block",
                  "num_attention_heads"):
            if k in d:
                d[k] = tuple(d[k])
        return cls(**d)


@dataclass
class VAEConfig:
    """diffusers AutoencoderKL config of stabilityai/stable-diffusion-xl-base-1.0/vae (loaded fp32 by the reference:
    inference_animatediff.py:164-169, train_animatediff.py:67-72): 4 DownEncoderBlock2D / UpDecoderBlock2D levels,
    2 resnets per down level (3 per up level), GroupNorm(32, eps 1e-6), one single-head attention in each mid block,
    latent 4 channels, scaling_factor 0.13025."""
    in_channels: int = 3
    out_channels: int = 3
    latent_channels: int = 4
    block_out_channels: Tuple[int, ...] = (128, 256, 512, 512)
    layers_per_block: int = 2
    norm_num_groups: int = 32
    scaling_factor: float = 0.13025

    def to_dict(self):
        return asdict(self)

    @classmethod
    def sdxl(cls) -> "VAEConfig":
        return cls()

    @classmethod
    def tiny(cls) -> "VAEConfig":
        """Same topology at test scale (channels multiples of 64 for the implicit-GEMM convs)."""
        return cls(block_out_channels=(64, 128, 128))
