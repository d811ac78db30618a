"""The optimisation step of train_animatediff.py (BASELINE configs[4]) on the HIP training path,
with data-parallel gradient averaging over RCCL.

- `GradBucketAllReducer` replaces accelerate's DDP wrapper (train_animatediff.py:314-319 `accelerator.backward`,
  `clip_grad_norm_`): gradients of the trainable set are copied into fp32 buckets by post-accumulate hooks as the
  backward produces them, and each full bucket's all-reduce is launched asynchronously at once, so the exchange of
  the up-block gradients overlaps the backward through the down blocks. Buckets are large (64 MB by default): xGMI
  is point-to-point, a ring all-reduce is per-link bound, and fewer, larger messages amortise the per-call latency.
  fp32 reduction keeps the 1/N averaging exact for the bf16 motion weights (the trainable set is ~156 M params,
  626 MB of fp32 buckets, ~7 ms of ring time per step next to a ~1.2 s step).
- `TrainStep` is one iteration of the loop body train_animatediff.py:214-319: Euler `add_noise` x + sigma(t)*eps
  (:228-236, no input scaling), optional unconditional prompt with p = 0.1 (:248-254), the UNet forward through
  `autograd.unet_train_tokens` (every forward and backward kernel on HIP), epsilon-prediction MSE in fp32
  (:294-300), the orthogonality loss (:307-312, evaluated low-rank by `temporal_lora.compute_orth_loss`),
  backward, gradient averaging, clip_grad_norm_ (:316), optimizer step (:317).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional

import torch
import torch.distributed as dist

BF16 = torch.bfloat16


class GradBucketAllReducer:
    """Bucketed, backward-overlapped gradient averaging over a torch.distributed group (RCCL on ROCm, gloo on CPU).

    Usage per step: loss.backward(); reducer.finish(); optimizer.step().  Parameters that received no gradient in a
    step contribute zeros (as DDP with find_unused_parameters would) and get an averaged gradient back, so every rank
    takes the same optimizer step."""

    def __init__(self, params: Iterable[torch.nn.Parameter], group=None, bucket_mb: float = 64.0,
                 reduce_dtype: torch.dtype = torch.float32):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.reduce_dtype = reduce_dtype
        cap = max(1, int(bucket_mb * 2 ** 20) // torch.tensor([], dtype=reduce_dtype).element_size())
        # autograd produces gradients roughly in reverse registration order: fill buckets in that order so the
        # first bucket completes early in the backward.
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, n = [], 0
        for p in reversed(self.params):
            if cur and n + p.numel() > cap:
                self.buckets.append(cur)
                cur, n = [], 0
            cur.append(p)
            n += p.numel()
        if cur:
            self.buckets.append(cur)
        self.flat: List[torch.Tensor] = []
        self.where: Dict[int, tuple] = {}
        for b, plist in enumerate(self.buckets):
            off = 0
            for p in plist:
                self.where[id(p)] = (b, off)
                off += p.numel()
            self.flat.append(torch.zeros(off, dtype=reduce_dtype, device=plist[0].device))
        self._ready = [set() for _ in self.buckets]
        self._works: List[Optional[object]] = [None] * len(self.buckets)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    def bucket_sizes_mb(self) -> List[float]:
        return [t.numel() * t.element_size() / 2 ** 20 for t in self.flat]

    def _on_grad(self, p: torch.nn.Parameter) -> None:
        b, off = self.where[id(p)]
        self.flat[b][off:off + p.numel()].copy_(p.grad.reshape(-1))
        self._ready[b].add(id(p))
        if len(self._ready[b]) == len(self.buckets[b]):
            self._launch(b)

    def _launch(self, b: int) -> None:
        if self._works[b] is not None:
            raise RuntimeError(f"GradBucketAllReducer: bucket {b} launched twice in one step "
                               "(a parameter received two gradients; call finish() after every backward)")
        if self.world == 1:
            self._works[b] = True
            return
        self._works[b] = dist.all_reduce(self.flat[b], group=self.group, async_op=True)

    def finish(self) -> None:
        """Launch the buckets that still wait for unused parameters (their segments are zero-filled), wait for every
        all-reduce, divide by the world size and write the averages back into p.grad."""
        for b, plist in enumerate(self.buckets):
            if self._works[b] is None:
                for p in plist:
                    if id(p) not in self._ready[b]:
                        _, off = self.where[id(p)]
                        self.flat[b][off:off + p.numel()].zero_()
                self._launch(b)
        for b, plist in enumerate(self.buckets):
            w = self._works[b]
            if w is not True:
                w.wait()
            flat = self.flat[b]
            if self.world > 1:
                flat.div_(self.world)
            for p in plist:
                _, off = self.where[id(p)]
                seg = flat[off:off + p.numel()].view(p.shape)
                if p.grad is None:
                    p.grad = seg.to(p.dtype).clone()
                else:
                    p.grad.copy_(seg)
            self._ready[b].clear()
            self._works[b] = None

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []


def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Same initial weights on every rank (accelerate.prepare broadcasts rank 0's module state)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src, group=group)


class TrainStep:
    """One train_animatediff.py iteration (:214-319) for a UNetMotionModel with temporal LoRA injected and the spatial
    path frozen (`utils.freeze_spatial_layers`).  Inputs are VAE latents already scaled by vae.scaling_factor
    (B, 4, F, h, w) fp32 on the device; prompt embeddings are (1, 77, D) / (1, Dp) as encode_prompt returns them."""

    def __init__(self, unet, optimizer, scheduler, *, reducer: Optional[GradBucketAllReducer] = None,
                 lambda_orth: float = 0.0, spatial_index: Optional[Dict] = None, max_grad_norm: float = 1.0,
                 p_uncond: float = 0.1, resolution: int = 512, seed: int = 0, lr_scheduler=None):
        """`seed` is offset by the process rank: every data-parallel rank draws its own noise, timesteps and
        unconditional-prompt coin (the reference's per-process RNG streams).  `lr_scheduler` (optional) steps after
        the optimizer (train_animatediff.py:318)."""
        self.unet = unet
        self.opt = optimizer
        self.sched = scheduler
        self.lr_scheduler = lr_scheduler
        self.reducer = reducer
        self.lambda_orth = lambda_orth
        self.spatial_index = spatial_index or {}
        self.max_grad_norm = max_grad_norm
        self.p_uncond = p_uncond
        self.resolution = resolution
        self.params = [p for p in unet.parameters() if p.requires_grad]
        rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.gen = torch.Generator(device="cpu").manual_seed(seed + 1000003 * rank)

    def _draw(self, latents, noise=None, timesteps=None, use_uncond=None, has_uncond=False):
        """The step's random draws (train_animatediff.py:228-254) from this rank's generator; overrides win."""
        B = latents.shape[0]
        draw_noise = torch.randn(latents.shape, generator=self.gen)                         # :228
        draw_t = torch.randint(0, self.sched.num_train_timesteps, (B,), generator=self.gen)  # :229-232
        draw_u = float(torch.rand(1, generator=self.gen)) < self.p_uncond                  # :248-254
        noise = draw_noise if noise is None else noise
        t = draw_t if timesteps is None else timesteps
        return noise, t.cpu(), has_uncond and (draw_u if use_uncond is None else use_uncond)

    def _text(self, prompt, pooled, B, dev):
        enc = prompt.to(dev, BF16)
        pool = pooled.to(dev, BF16)
        enc = enc.expand(B, -1, -1).reshape(-1, enc.shape[-1]).contiguous()               # .repeat(B, 1, 1)
        pool = pool.expand(B, -1).contiguous()
        return enc, pool

    def _body(self, latents, noise, t, enc, pool) -> Dict:
        """Forward, losses, backward, gradient averaging, clipping and the optimizer step on device tensors only (no
        host synchronisation: the body is what TrainStep.capture records into a HIP graph).  Gradients must be
        None or zero on entry."""
        from . import kernels as K
        from .autograd import unet_train_tokens
        from .temporal_lora import compute_orth_loss

        unet = self.unet
        B, Cl, F, h, w = latents.shape
        dev = latents.device
        # add_noise with the clip's timestep on every frame (:233-236); sigma broadcasts over (C, F, h, w)
        noisy = self.sched.add_noise(latents, noise, t).contiguous()
        tids = self._tids(B, dev)                                                          # :256-262
        x = torch.empty(B * F * h * w, Cl, dtype=BF16, device=dev)
        K.pack_latents(noisy, x)
        with torch.no_grad():
            emb = unet.embed(t.to(torch.float32), pool, tids, B)
        pred = unet_train_tokens(unet, x, B, F, h, w, emb, enc)                            # :265-273
        target = noise.permute(0, 2, 3, 4, 1).reshape(-1, Cl)                              # epsilon, :276-277
        loss_mse = torch.mean((pred.float() - target) ** 2)                                # :298-300
        if self.lambda_orth > 0 and self.spatial_index:
            loss_orth = compute_orth_loss(unet, self.spatial_index, self.lambda_orth).to(dev)
        else:
            loss_orth = torch.zeros((), device=dev)
        loss = loss_mse + loss_orth
        loss.backward()                                                                    # :314
        if self.reducer is not None:
            self.reducer.finish()
        gnorm = torch.nn.utils.clip_grad_norm_(self.params, self.max_grad_norm)           # :316
        self.opt.step()                                                                    # :317
        return {"loss": loss.detach(), "loss_mse": loss_mse.detach(), "loss_orth": loss_orth.detach(),
                "grad_norm": gnorm.detach()}

    def _tids(self, B, dev):
        key = (B, dev)
        c = self.__dict__.setdefault("_tids_cache", {})
        if key not in c:
            r = float(self.resolution)
            c[key] = torch.tensor([[r, r, 0.0, 0.0, r, r]], device=dev).expand(B, -1).contiguous()
        return c[key]

    def __call__(self, latents: torch.Tensor, prompt, pooled, uncond_prompt=None, uncond_pooled=None, *,
                 noise: Optional[torch.Tensor] = None, timesteps: Optional[torch.Tensor] = None,
                 use_uncond: Optional[bool] = None) -> Dict:
        """noise / timesteps / use_uncond override the step's random draws (tests compare a data-parallel step
        with a single-process step on the concatenated batch)."""
        dev = latents.device
        B = latents.shape[0]
        noise, t, use_uncond = self._draw(latents, noise, timesteps, use_uncond, uncond_prompt is not None)
        enc, pool = self._text(uncond_prompt if use_uncond else prompt, uncond_pooled if use_uncond else pooled, B,
                               dev)
        self.opt.zero_grad(set_to_none=True)
        out = self._body(latents, noise.to(dev, torch.float32), t.to(dev), enc, pool)
        if self.lr_scheduler is not None:
            self.lr_scheduler.step()                                                       # :318
        out.update(uncond=use_uncond, timesteps=t)
        return out

    # ---- HIP-graph capture of the whole step (single process) ------------------------------------------------
    def capture(self, latents: torch.Tensor, prompt, pooled, warmup: int = 2, uncond_prompt=None, uncond_pooled=None):
        """Record one whole training step (forward, backward, clipping, AdamW) into a HIP graph on static buffers,
        after `warmup` eager steps on a side stream (they fill every frozen-operand cache).  The optimizer must be
        built with capturable=True; per-step host work left outside the graph: the random draws (copied into the
        static noise / timestep buffers) and the lr schedule.  Single-process only (the reducer's collectives stay
        eager)."""
        if self.reducer is not None and self.reducer.world > 1:
            raise NotImplementedError("TrainStep.capture: data-parallel steps run eagerly")
        dev = latents.device
        B = latents.shape[0]
        self.s_lat = latents.detach().clone()
        self.s_noise = torch.zeros_like(self.s_lat)
        self.s_t = torch.zeros(B, dtype=torch.long, device=dev)
        self.s_enc, self.s_pool = self._text(prompt, pooled, B, dev)
        # the two text conditions a step can draw (:248-254), copied into the static buffers before each replay
        self.text_cond = (self.s_enc.clone(), self.s_pool.clone())
        self.text_uncond = None if uncond_prompt is None else self._text(uncond_prompt, uncond_pooled, B, dev)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                noise, t, _ = self._draw(self.s_lat)
                self.s_noise.copy_(noise)
                self.s_t.copy_(t)
                self.opt.zero_grad(set_to_none=True)
                self._body(self.s_lat, self.s_noise, self.s_t, self.s_enc, self.s_pool)
        torch.cuda.current_stream(dev).wait_stream(s)
        self.opt.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.s_out = self._body(self.s_lat, self.s_noise, self.s_t, self.s_enc, self.s_pool)
        return self.graph

    def replay(self, latents: Optional[torch.Tensor] = None) -> Dict:
        """One captured step on new latents (or the static ones) with fresh noise / timestep draws."""
        if latents is not None:
            self.s_lat.copy_(latents)
        noise, t, use_uncond = self._draw(self.s_lat, has_uncond=self.text_uncond is not None)
        self.s_noise.copy_(noise)
        self.s_t.copy_(t)
        enc, pool = self.text_uncond if use_uncond else self.text_cond
        self.s_enc.copy_(enc)
        self.s_pool.copy_(pool)
        self.graph.replay()
        if self.lr_scheduler is not None:
            self.lr_scheduler.step()
        return self.s_out


def encode_frames(vae, frames: torch.Tensor, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """train_animatediff.py:219-224 + :238-246: frames (B, F, 3, H, W) in [-1, 1] -> VAE encode (no grad) ->
    latent_dist.sample() * scaling_factor -> (B, 4, F, h, w) fp32, the layout TrainStep takes."""
    B, F = frames.shape[:2]
    with torch.no_grad():
        flat = frames.reshape(B * F, *frames.shape[2:]).float()
        lat = vae.encode(flat).latent_dist.sample(generator, scale=vae.config.scaling_factor)
    return lat.view(B, F, *lat.shape[1:]).permute(0, 2, 1, 3, 4).contiguous()

