"""SDXL VAE (diffusers AutoencoderKL) on the HIP path: the decode of the denoised clip and the encode of training
frames.

Reference calls (diffusers AutoencoderKL, loaded fp32):
  decode: inference_animatediff.py:137-144 -- latents / scaling_factor, one `vae.decode(frame).sample` per frame,
          then (x / 2 + 0.5).clamp(0, 1) * 255 -> uint8;
  encode: train_animatediff.py:219-224 -- `vae.encode(frames).latent_dist.sample() * scaling_factor`.
Module tree and parameter names follow diffusers AutoencoderKL (encoder / decoder / quant_conv / post_quant_conv), so
a real `vae/diffusion_pytorch_model.safetensors` loads with `load_state_dict`.

MI355X-first execution: the frames of a clip are decoded TOGETHER (chunks of several frames, not one frame per call),
NHWC bf16 activations with fp32 accumulation, every 3x3 conv an implicit GEMM (nearest-2x upsample fused into the
next conv, the encoder's asymmetric-pad stride-2 conv a kernel mode), GroupNorm+SiLU one pass, 1x1 shortcuts as GEMMs
with the residual add fused into conv2's epilogue.  The mid-block attention (one head of dim 512 over the latent's
h*w tokens) runs as fused q/k/v GEMM -> fp32 scores (vst_gemm_f32out) -> row softmax -> P.V GEMM -> out-projection
with the residual fused.  Precision: bf16 storage / fp32 accumulate, where the reference runs fp32 (its comment: "SDXL
VAE is numerically unstable at lower precision" -- fp16 overflow; bf16 keeps fp32's exponent range).  The deviation
from the fp32 oracle is measured and gated in tests/test_vae_gpu.py.
Frame sharding (bench --gpus N, frame_shard.py): every rank decodes the frames it holds; no exchange.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import nn

from . import kernels as K
from .config import VAEConfig
from .unet_motion import Conv1x1, Conv3x3, GroupNorm, f32

BF16 = torch.bfloat16
_CHUNK_BYTES = 1 << 30  # largest activation of one frame chunk (keeps every buffer offset in 31 bits)


def _padded_kernel_weight(conv: nn.Conv2d, cin_pad: int, cout_pad: int | None = None) -> torch.Tensor:
    """[Cout(_pad), k*k*cin_pad] bf16 (ky, kx, ci) with zero columns for channels cin..cin_pad-1 (and zero rows past
    Cout): the 4-channel latent enters the 1x1 / 3x3 convs as an 8-channel (16-B) NHWC row."""
    key = (conv.weight.data_ptr(), conv.weight._version, cin_pad, cout_pad)
    c = conv.__dict__.get("_vst_wpad")
    if c is None or c[0] != key:
        co, ci, kh, kw = conv.weight.shape
        w = conv.weight.detach().float().permute(0, 2, 3, 1)
        wp = w.new_zeros(cout_pad or co, kh, kw, cin_pad)
        wp[:co, :, :, :ci] = w
        b = conv.bias.detach().float()
        bp = b.new_zeros(cout_pad or co)
        bp[:co] = b
        c = (key, (wp.reshape(wp.shape[0], -1).to(BF16).contiguous(), bp.contiguous()))
        conv.__dict__["_vst_wpad"] = c
    return c[1]


class ResnetBlock2D(nn.Module):
    """diffusers ResnetBlock2D with temb_channels=None, eps 1e-6, output_scale_factor 1."""

    def __init__(self, cin, cout, groups=32, eps=1e-6):
        super().__init__()
        self.norm1 = GroupNorm(groups, cin, eps=eps)
        self.conv1 = Conv3x3(cin, cout)
        self.norm2 = GroupNorm(groups, cout, eps=eps)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = Conv3x3(cout, cout)
        self.conv_shortcut = Conv1x1(cin, cout) if cin != cout else None

    def run(self, x, n, H, W):
        h = self.norm1.run(x, n, H * W, silu=True)
        h = self.conv1.run(h, n, H, W)
        h = self.norm2.run(h, n, H * W, silu=True)
        sc = self.conv_shortcut.run(x) if self.conv_shortcut is not None else x
        return self.conv2.run(h, n, H, W, residual=sc)


class _Linear(nn.Linear):
    pass


class Attention(nn.Module):
    """diffusers Attention of the VAE mid block (heads 1, dim_head C, group_norm, residual_connection, bias)."""

    def __init__(self, C, groups=32, eps=1e-6):
        super().__init__()
        self.group_norm = GroupNorm(groups, C, eps=eps)
        self.to_q, self.to_k, self.to_v = _Linear(C, C), _Linear(C, C), _Linear(C, C)
        self.to_out = nn.ModuleList([_Linear(C, C), nn.Dropout(0.0)])

    def _qkv(self):
        ps = (self.to_q.weight, self.to_k.weight, self.to_v.weight, self.to_q.bias, self.to_k.bias, self.to_v.bias,
              self.to_out[0].weight, self.to_out[0].bias)
        key = tuple((p.data_ptr(), p._version) for p in ps)
        c = self.__dict__.get("_vst_qkv")
        if c is None or c[0] != key:
            w = torch.cat([p.detach() for p in ps[:3]]).to(BF16).contiguous()
            b = torch.cat([p.detach() for p in ps[3:6]]).float().contiguous()
            c = (key, (w, b, ps[6].detach().to(BF16).contiguous(), ps[7].detach().float().contiguous()))
            self.__dict__["_vst_qkv"] = c
        return c[1]

    def run(self, x, n, H, W):
        C, HW = x.shape[1], H * W
        wqkv, bqkv, wo, bo = self._qkv()
        h = self.group_norm.run(x, n, HW)
        qkv = K.linear(h, wqkv, bqkv)  # [n*HW, 3C]
        o = torch.empty((n * HW, C), dtype=BF16, device=x.device)
        s = torch.empty((HW, HW), dtype=torch.float32, device=x.device)
        p = torch.empty((HW, HW), dtype=BF16, device=x.device)
        vt = torch.empty((C, HW), dtype=BF16, device=x.device)
        for i in range(n):
            rows = slice(i * HW, (i + 1) * HW)
            K.gemm_f32out(qkv[rows, :C], qkv[rows, C:2 * C], out=s)
            K.softmax_rows(s, C ** -0.5, out=p)
            K.transpose(qkv[rows, 2 * C:], out=vt)
            K.linear(p, vt, out=o[rows])
        return K.linear(o, wo, bo, residual=x)


class UNetMidBlock2D(nn.Module):
    def __init__(self, C, groups=32):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(C, C, groups), ResnetBlock2D(C, C, groups)])
        self.attentions = nn.ModuleList([Attention(C, groups)])

    def run(self, x, n, H, W):
        x = self.resnets[0].run(x, n, H, W)
        x = self.attentions[0].run(x, n, H, W)
        return self.resnets[1].run(x, n, H, W)


class _Sampler(nn.Module):
    def __init__(self, C, stride):
        super().__init__()
        self.conv = Conv3x3(C, C, stride=stride)


class DownEncoderBlock2D(nn.Module):
    def __init__(self, cin, cout, layers, add_down, groups=32):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if j == 0 else cout, cout, groups) for j in range(layers)])
        self.downsamplers = nn.ModuleList([_Sampler(cout, 2)]) if add_down else None

    def run(self, x, n, H, W):
        for r in self.resnets:
            x = r.run(x, n, H, W)
        if self.downsamplers is not None:
            conv = self.downsamplers[0].conv
            x = K.conv3x3_down_pad0(x, n, H, W, conv.kernel_weight(), f32(conv.bias))
            H, W = (H - 2) // 2 + 1, (W - 2) // 2 + 1
        return x, H, W


class UpDecoderBlock2D(nn.Module):
    def __init__(self, cin, cout, layers, add_up, groups=32):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if j == 0 else cout, cout, groups) for j in range(layers)])
        self.upsamplers = nn.ModuleList([_Sampler(cout, 1)]) if add_up else None

    def run(self, x, n, H, W):
        for r in self.resnets:
            x = r.run(x, n, H, W)
        if self.upsamplers is not None:
            x = self.upsamplers[0].conv.run(x, n, H, W, upsample=True)
            H, W = 2 * H, 2 * W
        return x, H, W


class Encoder(nn.Module):
    def __init__(self, cfg: VAEConfig):
        super().__init__()
        ch, g = cfg.block_out_channels, cfg.norm_num_groups
        self.conv_in = Conv3x3(cfg.in_channels, ch[0])
        self.down_blocks = nn.ModuleList(
            [DownEncoderBlock2D(ch[max(i - 1, 0)], ch[i], cfg.layers_per_block, i < len(ch) - 1, g)
             for i in range(len(ch))])
        self.mid_block = UNetMidBlock2D(ch[-1], g)
        self.conv_norm_out = GroupNorm(g, ch[-1], eps=1e-6)
        self.conv_act = nn.SiLU()
        self.conv_out = Conv3x3(ch[-1], 2 * cfg.latent_channels)

    def run(self, x, n, H, W):
        x = self.conv_in.run(x, n, H, W)
        for blk in self.down_blocks:
            x, H, W = blk.run(x, n, H, W)
        x = self.mid_block.run(x, n, H, W)
        x = self.conv_norm_out.run(x, n, H * W, silu=True)
        return self.conv_out.run(x, n, H, W), H, W


class Decoder(nn.Module):
    def __init__(self, cfg: VAEConfig):
        super().__init__()
        ch, g = cfg.block_out_channels, cfg.norm_num_groups
        rch = list(reversed(ch))
        self.conv_in = Conv3x3(cfg.latent_channels, ch[-1])
        self.mid_block = UNetMidBlock2D(ch[-1], g)
        self.up_blocks = nn.ModuleList(
            [UpDecoderBlock2D(rch[max(i - 1, 0)], rch[i], cfg.layers_per_block + 1, i < len(ch) - 1, g)
             for i in range(len(ch))])
        self.conv_norm_out = GroupNorm(g, ch[0], eps=1e-6)
        self.conv_act = nn.SiLU()
        self.conv_out = Conv3x3(ch[0], cfg.out_channels)

    def run(self, z8, n, H, W):
        """z8: [n*H*W, 8] bf16 (post_quant_conv output, channels 4..7 zero)."""
        w, b = _padded_kernel_weight(self.conv_in, z8.shape[1])
        x = K.conv3x3(z8, n, H, W, w, b)
        x = self.mid_block.run(x, n, H, W)
        for blk in self.up_blocks:
            x, H, W = blk.run(x, n, H, W)
        x = self.conv_norm_out.run(x, n, H * W, silu=True)
        return self.conv_out.run(x, n, H, W), H, W


@dataclass
class DecoderOutput:
    sample: torch.Tensor


class DiagonalGaussianDistribution:
    """diffusers DiagonalGaussianDistribution over NHWC bf16 moments (mean = ch 0-3, logvar = ch 4-7)."""

    def __init__(self, moments, n, H, W):
        self.moments, self.n, self.H, self.W = moments, n, H, W

    def sample(self, generator: torch.Generator | None = None, scale: float = 1.0) -> torch.Tensor:
        """mean + exp(logvar / 2) * eps (eps ~ N(0, 1) from `generator`), times `scale`: fp32 (n, 4, H, W)."""
        eps = torch.randn((self.n, 4, self.H, self.W), generator=generator, device=self.moments.device,
                          dtype=torch.float32)
        return K.vae_sample(self.moments, self.n, self.H, self.W, eps, scale)

    def mode(self, scale: float = 1.0) -> torch.Tensor:
        return K.vae_sample(self.moments, self.n, self.H, self.W, None, scale)

    @property
    def mean(self):
        return self.mode()


@dataclass
class AutoencoderKLOutput:
    latent_dist: DiagonalGaussianDistribution


class AutoencoderKL(nn.Module):
    """diffusers AutoencoderKL surface the reference uses: `decode(z).sample`, `encode(x).latent_dist.sample()`,
    `config.scaling_factor`.  Inputs / outputs are fp32 NCHW device tensors like the reference's fp32 VAE."""

    def __init__(self, cfg: VAEConfig | None = None):
        super().__init__()
        self.cfg = cfg = cfg or VAEConfig.sdxl()
        self.config = cfg
        self.encoder = Encoder(cfg)
        self.decoder = Decoder(cfg)
        self.quant_conv = nn.Conv2d(2 * cfg.latent_channels, 2 * cfg.latent_channels, 1)
        self.post_quant_conv = nn.Conv2d(cfg.latent_channels, cfg.latent_channels, 1)

    def _chunk(self, n, H, W, pixel_scale):
        per = H * pixel_scale * W * pixel_scale * max(self.cfg.block_out_channels) * 2
        return max(1, min(n, _CHUNK_BYTES // per))

    def _decode_nhwc(self, z: torch.Tensor):
        """z (n, 4, h, w) fp32 device -> list of (bf16 [c*8h*8w, 3] NHWC, c) per frame chunk."""
        if not z.is_cuda:
            raise K._lib.VstError("AutoencoderKL.decode: the HIP path has no CPU fallback")
        n, L, h, w = z.shape
        wq, bq = _padded_kernel_weight(self.post_quant_conv, 8, 8)
        outs = []
        f = 2 ** (len(self.cfg.block_out_channels) - 1)
        step = self._chunk(n, h, w, f)
        for i in range(0, n, step):
            c = min(step, n - i)
            z8 = K.nchw_to_nhwc(z[i:i + c].float().contiguous(), 1.0, ldd=8)
            z8 = K.linear(z8, wq, bq)
            y, H, W = self.decoder.run(z8, c, h, w)
            outs.append((y, c))
        return outs, f * h, f * w

    def decode(self, z: torch.Tensor, return_dict: bool = True):
        """z: (n, latent, h, w) (already divided by scaling_factor) -> DecoderOutput(sample (n, 3, 8h, 8w) fp32)."""
        outs, H, W = self._decode_nhwc(z)
        C = self.cfg.out_channels
        sample = torch.cat([K.nhwc_to_nchw(y, c, C, H, W) for y, c in outs])
        return DecoderOutput(sample) if return_dict else (sample,)

    def decode_to_frames(self, latents: torch.Tensor) -> torch.Tensor:
        """inference_animatediff.py:137-144 on the device: latents (1, 4, F, h, w) from the denoise loop ->
        uint8 frames (F, 8h, 8w, 3): / scaling_factor, decode, (x / 2 + 0.5).clamp(0, 1) * 255."""
        z = (latents.float() / self.cfg.scaling_factor).squeeze(0).permute(1, 0, 2, 3).contiguous()
        outs, H, W = self._decode_nhwc(z)
        C = self.cfg.out_channels
        return torch.cat([K.frames_to_u8(y, c, C, H, W) for y, c in outs])

    def encode(self, x: torch.Tensor, return_dict: bool = True):
        """x: (n, 3, H, W) fp32 in [-1, 1] -> AutoencoderKLOutput(latent_dist)."""
        if not x.is_cuda:
            raise K._lib.VstError("AutoencoderKL.encode: the HIP path has no CPU fallback")
        n, _, H, W = x.shape
        wq, bq = _padded_kernel_weight(self.quant_conv, 8)
        moms = []
        step = self._chunk(n, H, W, 1)
        h = w = None
        for i in range(0, n, step):
            c = min(step, n - i)
            xi = K.nchw_to_nhwc(x[i:i + c].float().contiguous(), 1.0)
            m, h, w = self.encoder.run(xi, c, H, W)
            moms.append(K.linear(m, wq, bq))
        dist = DiagonalGaussianDistribution(torch.cat(moms), n, h, w)
        return AutoencoderKLOutput(dist) if return_dict else (dist,)


def build_vae(cfg: VAEConfig | None = None, state_dict=None, seed: int = 0, device="cuda") -> AutoencoderKL:
    """AutoencoderKL on `device` with a given (diffusers-named) state dict or seeded synthetic weights."""
    from .weights import vae_synthetic_state_dict
    cfg = cfg or VAEConfig.sdxl()
    vae = AutoencoderKL(cfg)
    sd = state_dict if state_dict is not None else vae_synthetic_state_dict(cfg, seed)
    vae.load_state_dict(sd, strict=True)
    return vae.to(device).requires_grad_(False)
