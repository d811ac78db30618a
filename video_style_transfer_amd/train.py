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

import functools
import math
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
        # False inside an accumulation window (DDP's no_sync): gradients only accumulate locally; the sync call's
        # hooks then see the accumulated p.grad and reduce it
        self.sync = True

    def bucket_sizes_mb(self) -> List[float]:
        return [t.numel() * t.element_size() / 2 ** 20 for t in self.flat]

    def _on_grad(self, p: torch.nn.Parameter) -> None:
        if not self.sync:
            return
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
        if not self.sync:
            raise RuntimeError("GradBucketAllReducer.finish() inside an accumulation window (sync=False)")
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


def _cosine_with_warmup(step: int, warmup: int, total: int, num_cycles: float = 0.5) -> float:
    if step < warmup:
        return float(step) / float(max(1, warmup))
    progress = float(step - warmup) / float(max(1, total - warmup))
    return max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress)))


def _linear_with_warmup(step: int, warmup: int, total: int) -> float:
    if step < warmup:
        return float(step) / float(max(1, warmup))
    return max(0.0, float(total - step) / float(max(1, total - warmup)))


def get_scheduler(name: str, optimizer, num_warmup_steps: int = 0, num_training_steps: int = 0):
    """diffusers.optimization.get_scheduler (train_animatediff.py:180-184; `--lr_scheduler` default "cosine", 100
    warmup steps, :403-404): a LambdaLR over the optimizer's lr.  "cosine" is half a cosine cycle after a linear
    warmup, "linear" a linear decay after it, "constant_with_warmup" / "constant" what they say.  With a device-tensor
    lr (make_adamw(..., capturable=True)) every step() writes the new value into that tensor in place, so a captured
    AdamW reads it on the next replay."""
    w, n = num_warmup_steps, num_training_steps
    if name == "cosine":
        fn = functools.partial(_cosine_with_warmup, warmup=w, total=n)
    elif name == "linear":
        fn = functools.partial(_linear_with_warmup, warmup=w, total=n)
    elif name == "constant_with_warmup":
        def fn(step):
            return float(step) / float(max(1, w)) if step < w else 1.0
    elif name == "constant":
        def fn(step):
            return 1.0
    else:
        raise ValueError(f"get_scheduler: unsupported schedule {name!r} (cosine, linear, constant_with_warmup, "
                         "constant)")
    return torch.optim.lr_scheduler.LambdaLR(optimizer, fn)


def make_adamw(params, lr: float = 2e-5, betas=(0.9, 0.999), weight_decay: float = 1e-2, eps: float = 1e-8, *,
               capturable: bool = False, device=None):
    """The reference's optimizer (train_animatediff.py:163-169: AdamW, --learning_rate 2e-5, betas 0.9/0.999, weight
    decay 1e-2, eps 1e-8).  capturable=True (for TrainStep.capture) keeps lr as a one-element fp32 tensor on the
    parameters' device: a Python-float lr would be baked into the captured update kernels (both the step size and the
    decoupled decay 1 - lr*wd), and the lr schedule would never reach the replayed graph."""
    params = list(params)
    if capturable:
        dev = device if device is not None else params[0].device
        lr = torch.tensor(float(lr), dtype=torch.float32, device=dev)
    return torch.optim.AdamW(params, lr=lr, betas=betas, weight_decay=weight_decay, eps=eps, capturable=capturable)


class TrainStep:
    """One train_animatediff.py iteration (:214-319) for a UNetMotionModel with temporal LoRA injected and the spatial
    path frozen (`utils.freeze_spatial_layers`).  Inputs are VAE latents already scaled by vae.scaling_factor
    (B, 4, F, h, w) fp32 on the device; prompt embeddings are (1, 77, D) / (1, Dp) as encode_prompt returns them.

    Gradient accumulation follows `accelerator.accumulate(unet)` with `Accelerator(gradient_accumulation_steps=N)`
    (:51-54, :214; accelerate 1.x semantics, pinned against accelerate itself by tests/test_train_host.py): every call
    is one micro-batch; the loss is divided by N before the backward (`accelerator.backward`); the gradients of N
    consecutive calls accumulate; only the N-th call (`sync_gradients`) all-reduces them over the data-parallel ranks
    (DDP's no_sync on the others), clips (:315-316), steps the optimizer and zeroes the gradients (:317-319).  The lr
    scheduler, wrapped by accelerate, advances only on sync calls and then once per process
    (AcceleratedScheduler.step with split_batches=False), so on P ranks the schedule runs P times as fast per
    optimizer step, as in the reference."""

    def __init__(self, unet, optimizer, scheduler, *, reducer: Optional[GradBucketAllReducer] = None,
                 lambda_orth: float = 0.0, spatial_index: Optional[Dict] = None, max_grad_norm: float = 1.0,
                 p_uncond: float = 0.1, resolution: int = 512, seed: int = 0, lr_scheduler=None,
                 gradient_accumulation_steps: int = 1, num_processes: Optional[int] = None):
        """`seed` is offset by the process rank: every data-parallel rank draws its own noise, timesteps and
        unconditional-prompt coin (the reference's per-process RNG streams).  `lr_scheduler` (optional) steps after
        the optimizer (train_animatediff.py:318), `num_processes` times per optimizer step (default: the world
        size)."""
        if gradient_accumulation_steps < 1:
            raise ValueError("gradient_accumulation_steps must be >= 1")
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
        self.accum = int(gradient_accumulation_steps)
        self.micro = 0  # calls since the last sync (accelerator.step)
        self.graph = self.graph_micro = None
        self.params = [p for p in unet.parameters() if p.requires_grad]
        dist_on = dist.is_available() and dist.is_initialized()
        rank = dist.get_rank() if dist_on else 0
        self.num_processes = num_processes or (dist.get_world_size() if dist_on else 1)
        self.gen = torch.Generator(device="cpu").manual_seed(seed + 1000003 * rank)

    @property
    def sync_gradients(self) -> bool:
        """Whether the next call ends an accumulation window (accelerate's GradientState.sync_gradients)."""
        return (self.micro + 1) % self.accum == 0

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

    def _body(self, latents, noise, t, enc, pool, sync: bool = True, zero_in_place: bool = False,
              div: Optional[int] = None) -> Dict:
        """Forward, losses, backward (gradients accumulate into p.grad); on a sync call also gradient averaging,
        clipping and the optimizer step.  Device tensors only (no host synchronisation: the body is what
        TrainStep.capture records into a HIP graph).  zero_in_place: the sync body ends by zeroing the gradient
        tensors in place (the captured graphs keep static .grad tensors), instead of the eager zero_grad(None)."""
        dev = latents.device
        loss, loss_mse, loss_orth = self._loss(latents, noise, t, enc, pool)
        if self.reducer is not None:
            self.reducer.sync = sync                                                       # DDP no_sync otherwise
        div = self.accum if div is None else div
        (loss / div if div > 1 else loss).backward()                                       # :314 accelerator.backward
        if sync:
            if self.reducer is not None:
                self.reducer.finish()
            gnorm = torch.nn.utils.clip_grad_norm_(self.params, self.max_grad_norm)       # :315-316
            self.opt.step()                                                                # :317
            if zero_in_place:
                torch._foreach_zero_([p.grad for p in self.params])                        # :319
        else:
            gnorm = torch.full((), float("nan"), device=dev)                               # no clip on this call
        return {"loss": loss.detach(), "loss_mse": loss_mse.detach(), "loss_orth": loss_orth.detach(),
                "grad_norm": gnorm.detach()}

    def _loss(self, latents, noise, t, enc, pool):
        """The micro-batch loss (train_animatediff.py:228-312): Euler add_noise, the HIP UNet forward, epsilon MSE in
        fp32 and the orthogonality loss."""
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
        return loss_mse + loss_orth, loss_mse, loss_orth

    def _tids(self, B, dev):
        key = (B, dev)
        c = self.__dict__.setdefault("_tids_cache", {})
        if key not in c:
            r = float(self.resolution)
            c[key] = torch.tensor([[r, r, 0.0, 0.0, r, r]], device=dev).expand(B, -1).contiguous()
        return c[key]

    def _advance(self, sync: bool) -> None:
        """accelerate's bookkeeping after a call: the step counter, and AcceleratedScheduler.step (:318)."""
        self.micro = 0 if sync else self.micro + 1
        if self.lr_scheduler is None:
            return
        if not sync:
            self.lr_scheduler._step_count += 1  # GradientAccumulationPlugin.adjust_scheduler: counted, lr unchanged
            return
        for _ in range(self.num_processes):
            self.lr_scheduler.step()

    def __call__(self, latents: torch.Tensor, prompt, pooled, uncond_prompt=None, uncond_pooled=None, *,
                 noise: Optional[torch.Tensor] = None, timesteps: Optional[torch.Tensor] = None,
                 use_uncond: Optional[bool] = None) -> Dict:
        """One eager micro-batch.  noise / timesteps / use_uncond override the step's random draws (tests compare a
        data-parallel step with a single-process step on the concatenated batch).  The returned "loss" is the
        undivided micro-batch loss (what the reference logs); "grad_norm" is NaN on calls that do not sync."""
        dev = latents.device
        B = latents.shape[0]
        noise, t, use_uncond = self._draw(latents, noise, timesteps, use_uncond, uncond_prompt is not None)
        enc, pool = self._text(uncond_prompt if use_uncond else prompt, uncond_pooled if use_uncond else pooled, B,
                               dev)
        sync = self.sync_gradients
        if self.micro == 0:  # the previous window's :319 (accelerate zeroes only on sync calls)
            if self.graph is not None:
                torch._foreach_zero_([p.grad for p in self.params if p.grad is not None])  # keep the static grads
            else:
                self.opt.zero_grad(set_to_none=True)
        out = self._body(latents, noise.to(dev, torch.float32), t.to(dev), enc, pool, sync=sync)
        self._advance(sync)
        out.update(uncond=use_uncond, timesteps=t, sync=sync)
        return out

    # ---- a whole accumulation window as one batched forward + backward -----------------------------------------
    def _window_draws(self, latents, has_uncond, noise=None, timesteps=None, use_uncond=None):
        """The draws of the window's N sequential calls, in their order (so the RNG stream is the per-call one)."""
        N = self.accum
        B = latents.shape[0]
        if B % N:
            raise ValueError(f"TrainStep.window: {B} clips do not split into {N} micro-batches")
        mb = B // N
        ns, ts, us = [], [], []
        for i in range(N):
            sl = slice(i * mb, (i + 1) * mb)
            n_i, t_i, u_i = self._draw(latents[sl], None if noise is None else noise[sl],
                                       None if timesteps is None else timesteps[sl],
                                       None if use_uncond is None else use_uncond[i], has_uncond)
            ns.append(n_i)
            ts.append(t_i)
            us.append(bool(u_i))
        return torch.cat(ns), torch.cat(ts), us

    def window(self, latents: torch.Tensor, prompt, pooled, uncond_prompt=None, uncond_pooled=None, *,
               noise: Optional[torch.Tensor] = None, timesteps: Optional[torch.Tensor] = None,
               use_uncond: Optional[List[bool]] = None) -> Dict:
        """A whole accumulation window -- the gradient_accumulation_steps calls of one optimizer step -- as ONE
        forward + backward over the window's clips stacked on the batch axis (latents: (N * micro_batch, C, F, h,
        w)), then the sync call's all-reduce / clip / AdamW / zero and the scheduler bookkeeping of N calls.

        Same gradient as the N sequential calls: every op of the UNet is per clip (no batch mixing), the mean MSE
        over the N equal-sized micro-batches is the mean of their means, and the orth loss, identical in every call
        of a window (the weights only change at its end), enters once instead of N times 1/N.  Each clip keeps its
        own noise, timestep and unconditional-prompt coin, drawn in the sequential calls' order.  What changes is
        only the shape of every GEMM (M x N clips), i.e. fp32 summation orders."""
        if self.micro != 0:
            raise RuntimeError("TrainStep.window: call at the start of an accumulation window")
        dev = latents.device
        has_u = uncond_prompt is not None
        noise, t, us = self._window_draws(latents, has_u, noise, timesteps, use_uncond)
        mb = latents.shape[0] // self.accum
        encs, pools = [], []
        for u in us:
            e, p_ = self._text(uncond_prompt if u else prompt, uncond_pooled if u else pooled, mb, dev)
            encs.append(e)
            pools.append(p_)
        if self.graph is not None:
            torch._foreach_zero_([p.grad for p in self.params if p.grad is not None])
        else:
            self.opt.zero_grad(set_to_none=True)
        out = self._body(latents, noise.to(dev, torch.float32), t.to(dev), torch.cat(encs), torch.cat(pools),
                         sync=True, div=1)
        for _ in range(self.accum - 1):
            self._advance(False)
        self._advance(True)
        out.update(uncond=us, timesteps=t, sync=True)
        return out

    # ---- HIP-graph capture of the whole step (single process) ------------------------------------------------
    def capture(self, latents: torch.Tensor, prompt, pooled, warmup: int = 2, uncond_prompt=None, uncond_pooled=None,
                window: bool = False):
        """Record the step into HIP graphs on static buffers: one graph for the sync call (forward, backward,
        clipping, AdamW, zeroing) and, with gradient accumulation, one for the other calls (forward + backward
        accumulating into the static .grad tensors).  `warmup` eager windows run first on a side stream (they fill
        every frozen-operand cache and create the optimizer state); the trainable parameters, the optimizer state,
        the gradients and this rank's random generator are then restored, so capturing changes no training state.
        The optimizer must be capturable; with an lr scheduler its lr must be a device tensor (make_adamw) so the
        schedule reaches the replays.  Per-call host work left outside the graphs: the random draws (copied into
        the static noise / timestep / text buffers) and the scheduler step.  Single process only (the reducer's
        collectives stay eager).  window=True: one graph of the whole accumulation window as TrainStep.window runs
        it (latents then hold the window's N micro-batches); replay() then runs a whole optimizer step."""
        if self.reducer is not None and self.reducer.world > 1:
            raise NotImplementedError("TrainStep.capture: data-parallel steps run eagerly")
        dev = latents.device
        for g in self.opt.param_groups:
            if not g.get("capturable", False):
                raise ValueError("TrainStep.capture: the optimizer must be built with capturable=True")
            if self.lr_scheduler is not None and not (isinstance(g["lr"], torch.Tensor) and g["lr"].device == dev):
                raise ValueError("TrainStep.capture: with an lr scheduler the optimizer's lr must be a device tensor "
                                 "(train.make_adamw(..., capturable=True)); a float lr is baked into the graph")
        if self.micro != 0:
            raise RuntimeError("TrainStep.capture: call at the start of an accumulation window")
        B = latents.shape[0]
        if window and B % self.accum:
            raise ValueError(f"TrainStep.capture(window=True): {B} clips do not split into {self.accum} micro-batches")
        self.window_mode = window
        mb = B // self.accum if window else B
        self.s_lat = latents.detach().clone()
        self.s_noise = torch.zeros_like(self.s_lat)
        self.s_t = torch.zeros(B, dtype=torch.long, device=dev)
        self.s_enc, self.s_pool = self._text(prompt, pooled, B, dev)
        # the two text conditions a call can draw (:248-254), per micro-batch, copied into the static buffers
        self.text_cond = self._text(prompt, pooled, mb, dev)
        self.text_uncond = None if uncond_prompt is None else self._text(uncond_prompt, uncond_pooled, mb, dev)

        # training state the warm-up must not change
        gen_state = self.gen.get_state()
        with torch.no_grad():
            p_snap = [p.detach().clone() for p in self.params]
        st_snap = {id(p): {k: (v.detach().clone() if isinstance(v, torch.Tensor) else v)
                           for k, v in self.opt.state[p].items()} for p in self.params if p in self.opt.state}
        for p in self.params:  # static gradient tensors, shared by both graphs (accumulation across replays)
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            else:
                p.grad.zero_()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                if window:
                    noise, t, _ = self._window_draws(self.s_lat, False)
                    self.s_noise.copy_(noise)
                    self.s_t.copy_(t)
                    self._body(self.s_lat, self.s_noise, self.s_t, self.s_enc, self.s_pool, sync=True,
                               zero_in_place=True, div=1)
                    continue
                for k in range(self.accum):
                    noise, t, _ = self._draw(self.s_lat)
                    self.s_noise.copy_(noise)
                    self.s_t.copy_(t)
                    self._body(self.s_lat, self.s_noise, self.s_t, self.s_enc, self.s_pool,
                               sync=k == self.accum - 1, zero_in_place=True)
            with torch.no_grad():
                for p, v in zip(self.params, p_snap):
                    p.copy_(v)
                for p in self.params:
                    st = self.opt.state.get(p)
                    if not st:
                        continue
                    old = st_snap.get(id(p))
                    for k, v in st.items():
                        if isinstance(v, torch.Tensor):
                            if old is not None and isinstance(old.get(k), torch.Tensor):
                                v.copy_(old[k])
                            else:
                                v.zero_()           # state created by the warm-up: back to its initial zeros
                torch._foreach_zero_([p.grad for p in self.params])
        torch.cuda.current_stream(dev).wait_stream(s)
        self.gen.set_state(gen_state)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.s_out = self._body(self.s_lat, self.s_noise, self.s_t, self.s_enc, self.s_pool, sync=True,
                                    zero_in_place=True, div=1 if window else None)
        if self.accum > 1 and not window:
            self.graph_micro = torch.cuda.CUDAGraph()  # own memory pool: its temporaries never alias s_out
            with torch.cuda.graph(self.graph_micro):
                self.s_out_micro = self._body(self.s_lat, self.s_noise, self.s_t, self.s_enc, self.s_pool,
                                              sync=False)
        return self.graph

    def replay(self, latents: Optional[torch.Tensor] = None) -> Dict:
        """One captured micro-batch on new latents (or the static ones) with fresh noise / timestep draws.  The
        returned tensors are the graph's static outputs: read them before the next replay of the same graph."""
        if latents is not None:
            self.s_lat.copy_(latents)
        if getattr(self, "window_mode", False):
            noise, t, us = self._window_draws(self.s_lat, self.text_uncond is not None)
            self.s_noise.copy_(noise)
            self.s_t.copy_(t)
            L, mb = self.text_cond[0].shape[0], self.text_cond[1].shape[0]
            for i, u in enumerate(us):
                enc, pool = self.text_uncond if u else self.text_cond
                self.s_enc[i * L:(i + 1) * L].copy_(enc)
                self.s_pool[i * mb:(i + 1) * mb].copy_(pool)
            self.graph.replay()
            for _ in range(self.accum - 1):
                self._advance(False)
            self._advance(True)
            return dict(self.s_out, uncond=us, timesteps=t, sync=True)
        noise, t, use_uncond = self._draw(self.s_lat, has_uncond=self.text_uncond is not None)
        self.s_noise.copy_(noise)
        self.s_t.copy_(t)
        enc, pool = self.text_uncond if use_uncond else self.text_cond
        self.s_enc.copy_(enc)
        self.s_pool.copy_(pool)
        sync = self.sync_gradients
        (self.graph if sync else self.graph_micro).replay()
        self._advance(sync)
        return dict(self.s_out if sync else self.s_out_micro, uncond=use_uncond, timesteps=t, sync=sync)


def encode_frames(vae, frames: torch.Tensor, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """train_animatediff.py:219-224 + :238-246: frames (B, F, 3, H, W) in [-1, 1] -> VAE encode (no grad) ->
    latent_dist.sample() * scaling_factor -> (B, 4, F, h, w) fp32, the layout TrainStep takes."""
    B, F = frames.shape[:2]
    with torch.no_grad():
        flat = frames.reshape(B * F, *frames.shape[2:]).float()
        lat = vae.encode(flat).latent_dist.sample(generator, scale=vae.config.scaling_factor)
    return lat.view(B, F, *lat.shape[1:]).permute(0, 2, 1, 3, 4).contiguous()

