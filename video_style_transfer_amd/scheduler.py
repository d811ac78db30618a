"""EulerDiscreteScheduler tables for the denoise loop (inference_animatediff.py:217-219, :104-131).

SDXL scheduler config: scaled_linear betas (0.00085 -> 0.012, 1000 train steps), 'leading'
timestep spacing, steps_offset 1, epsilon prediction, linear sigma interpolation, no Karras.
Host-side math only (once per schedule); the per-step arithmetic (scale_model_input, CFG
combine, Euler update) runs in vst_pack_latents / vst_euler_cfg_step on the device, reading
these tables through a device step counter so a captured HIP graph replays every step.
"""
from __future__ import annotations

import numpy as np
import torch


class EulerDiscreteScheduler:
    def __init__(self, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012, steps_offset=1,
                 timestep_spacing="leading"):
        self.num_train_timesteps = num_train_timesteps
        betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float32) ** 2
        self.alphas_cumprod = torch.cumprod(1.0 - betas, dim=0)
        self.steps_offset = steps_offset
        self.timestep_spacing = timestep_spacing
        self.timesteps = None
        self.sigmas = None

    def set_timesteps(self, num_inference_steps: int, device=None):
        n = num_inference_steps
        if self.timestep_spacing == "leading":
            ratio = self.num_train_timesteps // n
            ts = (np.arange(0, n) * ratio).round()[::-1].copy().astype(np.float32) + self.steps_offset
        elif self.timestep_spacing == "trailing":
            ratio = self.num_train_timesteps / n
            ts = (np.arange(self.num_train_timesteps, 0, -ratio)).round().copy().astype(np.float32) - 1
        else:  # linspace
            ts = np.linspace(0, self.num_train_timesteps - 1, n, dtype=np.float32)[::-1].copy()
        sig = (((1 - self.alphas_cumprod) / self.alphas_cumprod) ** 0.5).numpy()
        sig = np.interp(ts, np.arange(0, len(sig)), sig)
        sig = np.concatenate([sig, [0.0]]).astype(np.float32)
        self.timesteps = torch.from_numpy(ts).to(device)
        self.sigmas = torch.from_numpy(sig).to(device)
        self.num_inference_steps = n

    @property
    def init_noise_sigma(self) -> float:
        m = float(self.sigmas.max())
        return m if self.timestep_spacing in ("linspace", "trailing") else (m ** 2 + 1) ** 0.5

    def scale_model_input(self, sample, step_index):
        return sample / ((self.sigmas[step_index] ** 2 + 1) ** 0.5)

    def add_noise(self, original_samples, noise, timesteps):
        """Training noising (train_animatediff.py:234-236): x + sigma(t) * eps (no input scaling).  The sigma table
        is kept on the samples' device, so the call issues no host copy (graph-capturable)."""
        dev = original_samples.device
        cache = self.__dict__.setdefault("_sig_dev", {})
        if dev not in cache:
            cache[dev] = (((1 - self.alphas_cumprod) / self.alphas_cumprod) ** 0.5).to(dev)
        s = cache[dev][timesteps.long()].to(original_samples.dtype)
        while s.dim() < original_samples.dim():
            s = s.unsqueeze(-1)
        return original_samples + s * noise
