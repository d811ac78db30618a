"""The denoise loop of `generate_video` (inference_animatediff.py:53-151), MI355X-native.

Per step the reference does: scale_model_input -> unet(uncond) -> unet(cond) -> CFG combine ->
Euler step (two B=1 UNet calls, :109-121).  Here one step is:
  vst_pack_latents (scale_model_input, both CFG branches, NHWC bf16)
  -> embed (timestep read from the device schedule table)
  -> ONE UNet forward over the CFG-batched B=2 clip (results identical to two B=1 calls: no op mixes
     batch elements)
  -> vst_euler_cfg_step (CFG combine + Euler update of the fp32 latents)
  -> vst_step_advance (device step counter).
Because every per-step scalar lives in device tables indexed by the device counter, the whole step
is captured once into a HIP graph and replayed for all 50 steps (no per-launch host overhead).
Latents stay fp32 on the device (the reference keeps them in the UNet dtype between steps).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import kernels as K
from .scheduler import EulerDiscreteScheduler
from .unet_motion import UNetMotionModel

BF16 = torch.bfloat16


class AnimateDiffDenoiser:
    def __init__(self, unet: UNetMotionModel, num_frames: int, height: int, width: int, *,
                 num_inference_steps: int = 50, guidance_scale: float = 7.5, device=None,
                 scheduler: Optional[EulerDiscreteScheduler] = None, use_graph: bool = True, shard=None,
                 num_clips: int = 1):
        """`num_clips` clips are denoised together (the reference loop is one clip, B=1).
        `shard` (frame_shard.FrameShard): this process denoises frames [f0, f0 + F/P) of every clip and
        exchanges with the other ranks inside every motion module.
        The CFG branches always run as ONE batched B=2 forward on one stream (running them as two B=1 chains on two
        forked streams measured slower, 76.6 vs 72.8 ms per step, profiles/r3_ab_cfg_streams.txt; removed)."""
        self.unet = unet
        self.nclips = num_clips
        self.shard = shard
        self.F_total = num_frames
        self.F, self.f0 = shard.local_frames(num_frames) if shard is not None else (num_frames, 0)
        self.h, self.w = height // 8, width // 8
        self.height, self.width = height, width
        self.guidance = guidance_scale
        self.cfg = guidance_scale > 1.0
        self.ncopy = 2 if self.cfg else 1
        self.device = torch.device(device or "cuda")
        self.scheduler = scheduler or EulerDiscreteScheduler()
        self.scheduler.set_timesteps(num_inference_steps, device=self.device)
        self.num_steps = num_inference_steps
        self.use_graph = use_graph
        cfg = unet.config
        dev = self.device
        self.lat = torch.zeros(num_clips, cfg.in_channels, self.F, self.h, self.w, dtype=torch.float32, device=dev)
        self.x = torch.empty(self.ncopy * num_clips * self.F * self.h * self.w, cfg.in_channels, dtype=BF16,
                             device=dev)
        self.step_idx = torch.zeros(1, dtype=torch.int32, device=dev)
        self.timesteps = self.scheduler.timesteps.to(dev, torch.float32).contiguous()
        self.sigmas = self.scheduler.sigmas.to(dev, torch.float32).contiguous()
        self.enc = None
        self.graph = None

    def set_prompt_embeds(self, cond_embeds, cond_pooled, uncond_embeds=None, uncond_pooled=None):
        """(1 or num_clips, L, D) text states and (1 or num_clips, P) pooled embeds per branch
        (encode_prompt output).  UNet batch order: [uncond clips..., cond clips...]."""
        dev = self.device
        n = self.nclips

        def per_clip(t):
            return t if t is None or t.shape[0] == n else t.expand(n, *t.shape[1:])
        cond_embeds, cond_pooled = per_clip(cond_embeds), per_clip(cond_pooled)
        uncond_embeds, uncond_pooled = per_clip(uncond_embeds), per_clip(uncond_pooled)
        if self.cfg:
            enc = torch.cat([uncond_embeds, cond_embeds], 0)
            pooled = torch.cat([uncond_pooled, cond_pooled], 0)
        else:
            enc, pooled = cond_embeds, cond_pooled
        self.enc = enc.to(dev, BF16).contiguous()
        self.pooled = pooled.to(dev, BF16).contiguous()
        # SDXL time ids (inference_animatediff.py:81-85)
        tid = torch.tensor([self.height, self.width, 0, 0, self.height, self.width], dtype=torch.float32)
        self.time_ids = tid.unsqueeze(0).repeat(self.ncopy * n, 1).to(dev).contiguous()
        self.graph = None

    def _step(self):
        B = self.ncopy * self.nclips
        K.pack_latents(self.lat, self.x, sigmas=self.sigmas, step_idx=self.step_idx, ncopy=self.ncopy)
        emb = self.unet.embed(self.timesteps, self.pooled, self.time_ids, B, step_idx=self.step_idx)
        noise = self.unet.forward_tokens(self.x, B, self.F, self.h, self.w, emb, self.enc, shard=self.shard)
        K.euler_cfg_step(noise, self.lat, self.sigmas, self.step_idx, guidance=self.guidance, ncopy=self.ncopy)
        K.step_advance(self.step_idx, self.num_steps)

    def capture(self):
        """Warm up (fills every derived-weight cache), then capture one step into a HIP graph.  Frame-sharded over
        several ranks: piecewise (frame_shard.PiecewiseGraph), the graphs split at the collectives, which run between
        them."""
        saved = self.lat.clone()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self.step_idx.zero_()
            self._step()
        torch.cuda.current_stream(self.device).wait_stream(s)
        if self.shard is not None and self.shard.world > 1:
            from .frame_shard import PiecewiseGraph
            self.graph = PiecewiseGraph().capture(self._step, [self.shard], s)
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._step()
            self.graph = g
        self.lat.copy_(saved)
        self.step_idx.zero_()

    def set_latents(self, latents):
        """latents: (num_clips, C, F_total, h, w) for whole clips (this rank keeps its frames) or
        (num_clips, C, F_local, h, w)."""
        lat = latents.to(self.device, torch.float32)
        if lat.dim() == 5 and lat.shape[2] == self.F_total and self.F != self.F_total:
            lat = lat[:, :, self.f0:self.f0 + self.F]
        self.lat.copy_(lat.reshape(self.lat.shape))
        self.step_idx.zero_()

    def init_latents(self, seed: int = 42):
        """randn((1,4,F,h,w), generator=seed) * init_noise_sigma (inference_animatediff.py:88-95); with
        frame sharding every rank draws the whole clip and keeps its frames."""
        g = torch.Generator(device="cpu").manual_seed(seed)
        shape = (self.nclips, self.lat.shape[1], self.F_total, self.h, self.w)
        lat = torch.randn(shape, generator=g) * self.scheduler.init_noise_sigma
        self.set_latents(lat)
        return lat

    def run_steps(self, n: Optional[int] = None):
        n = self.num_steps if n is None else n
        if self.use_graph and self.graph is None:
            self.capture()
        for _ in range(n):
            if self.graph is not None:
                self.graph.replay()
            else:
                self._step()
        return self.lat

    def __call__(self, latents=None, seed: int = 42):
        if latents is None:
            self.init_latents(seed)
        else:
            self.set_latents(latents)
        return self.run_steps()

    def decode(self, vae) -> torch.Tensor:
        """inference_animatediff.py:137-144 for the frames this rank holds: latents / scaling_factor -> VAE decode ->
        uint8 (clips * F_local, 8h, 8w, 3) on the device.  Frame-sharded runs decode their own frames (no exchange);
        the frames of a clip are decoded together instead of one vae.decode call per frame."""
        return torch.cat([vae.decode_to_frames(self.lat[c:c + 1]) for c in range(self.lat.shape[0])])
