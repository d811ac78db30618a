"""Frame sharding of a clip across the GPUs of a node (one process per GPU, torch.distributed / RCCL).

SURVEY.md §8(e): everything in the UNet is frame-local except the 15 motion modules, whose frame-axis
attention needs every frame of a clip at each pixel, and whose GroupNorm takes its statistics over the
whole clip (diffusers AnimateDiffTransformer3D, built at animatediff/utils.py:31).

With P ranks each holding F/P contiguous frames of every clip, a motion module runs as:
  1. GroupNorm statistics: fp32 (sum, sumsq) chunk partials of each of this rank's frames
     -> all-gather (B*F/P frames x 8 chunks x 32 groups x 2 floats per rank) -> every rank merges the
     clip's partials in one fixed frame order (fp64) and normalises its own frames, then applies proj_in
     (per token, frame-local).  The unsharded forward merges the same per-frame partials in the same
     order, so the statistics -- and with them the whole sharded forward -- are bit-identical to the
     unsharded one;
  2. frame shard -> pixel shard: one all-to-all hands rank q the pixel slab q (H*W/P pixels) of every
     frame. Each rank now holds all F frames for H*W/P pixels. That is exactly the data the
     frame-axis attention needs. The whole transformer block runs unchanged on it (LN, q/k/v, temporal
     attention, out, GEGLU FF are all per token or per pixel);
  3. pixel shard -> frame shard: the inverse all-to-all, then proj_out + residual frame-local.
Per module and rank this moves 2 x (P-1)/P of the rank's activation over xGMI. That is P x less than
an all-gather of the clip before the attention (the north-star formulation), and no motion-module
work is duplicated across ranks.

exchange="all_gather" (opt-in; bench.py --exchange all_gather) is the north-star formulation itself: one all-gather
of the module's input hands every rank the whole clip, every rank runs the motion module over all frames (GroupNorm,
proj_in, both frame-attention blocks: frame 0's attn2 K/V depend on every frame's attn1 output, so nothing short of
the whole module is needed), and keeps its own frames' rows for proj_out + residual.  (P-1)/P of the clip's
activation per rank and module, and P x the motion-module work; bit-identical to the unsharded forward as well.

The layout permutations around the all-to-all are one HIP kernel each (vst_permute_rows).  A step is captured
PIECEWISE (PiecewiseGraph): the kernels between two collectives form one HIP graph, and the collectives run between
the graph replays on the same stream.  So no collective is ever inside a captured graph (RCCL's own graph capture is
not relied on), and the gloo backend (CPU transport, host staging; used by tests to run several ranks on one GPU or on
CPU) gets the same captured step as nccl (= RCCL).
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Sequence

import torch
import torch.distributed as dist

from . import kernels as K

Permute = Callable[[torch.Tensor, Sequence[int], Sequence[int]], torch.Tensor]


class PiecewiseGraph:
    """A HIP-graph capture split at the collectives: capture() runs `fn` once under capture; every collective that
    FrameShard issues meanwhile closes the current graph, is recorded as a host call, and a new graph opens after it.
    replay() replays graph, collective, graph, ... in capture order on the current stream.  All pieces share one
    memory pool (replayed in capture order, as torch requires for pool sharing).

    Why the collectives stay outside the graphs: a collective captured INTO a graph makes RCCL keep a persistent plan
    that references the communicator for as long as the graph lives; destroy_process_group with such a graph still
    alive waits for it forever (round 4's hang, profiles/r4_rccl_diag.log: a captured all_to_all_single -- RCCL
    send/recv -- at world 1).  Destroying the graph first exits cleanly (profiles/r5_rccl_diag_del.log), so whole-step
    capture is possible with that teardown order; the piecewise form is kept because it is the one the 1-GPU box can
    exercise with real collectives (gloo, 2-8 ranks) and it costs ~1 % of a step."""

    def __init__(self):
        self.items = []
        self.pool = None
        self._g = None

    def _begin(self):
        self._g = torch.cuda.CUDAGraph()
        # thread-local: the process group's watchdog thread may query events of earlier (eager) collectives
        self._g.capture_begin(pool=self.pool, capture_error_mode="thread_local")

    def _end(self):
        self._g.capture_end()
        if self.pool is None:
            self.pool = self._g.pool()
        self.items.append(self._g)
        self._g = None

    def collective(self, fn):
        """Called by FrameShard in place of issuing a collective while capturing."""
        self._end()
        self.items.append(fn)
        self._begin()

    def capture(self, fn, shards, stream):
        """Capture fn() on `stream` (a side stream, as torch capture requires) with `shards` in piecewise mode."""
        for sh in shards:
            sh._pw = self
        try:
            torch.cuda.synchronize()
            with torch.cuda.stream(stream):
                self._begin()
                fn()
                self._end()
            torch.cuda.current_stream().wait_stream(stream)
        except BaseException:
            # end the open capture (else the side stream stays in capture mode and every later HIP call fails
            # confusingly) and drop every piece: a half-captured step is never replayed
            if self._g is not None:
                try:
                    with torch.cuda.stream(stream):
                        self._g.capture_end()
                except Exception:  # noqa: BLE001 -- the original error is the one to report
                    pass
                self._g = None
            self.items.clear()
            raise
        finally:
            for sh in shards:
                sh._pw = None
        return self

    @property
    def num_graphs(self):
        return sum(1 for it in self.items if isinstance(it, torch.cuda.CUDAGraph))

    def replay(self):
        for it in self.items:
            if isinstance(it, torch.cuda.CUDAGraph):
                it.replay()
            else:
                it()


class FrameShard:
    EXCHANGES = ("all_to_all", "all_gather")

    def __init__(self, group=None, permute: Optional[Permute] = None, exchange: str = "all_to_all",
                 overlap: Optional[bool] = None):
        """overlap: run each motion module's batch as two halves whose exchanges overlap the other half's compute
        (all_to_all: pipelined; all_gather: half 1's gather under half 0's module; same bits either way).  Default:
        VST_SHARD_OVERLAP, else on."""
        if not dist.is_initialized():
            raise RuntimeError("FrameShard needs an initialised torch.distributed process group")
        if exchange not in self.EXCHANGES:
            raise ValueError(f"exchange {exchange!r}: one of {self.EXCHANGES}")
        self.exchange = exchange
        if overlap is None:
            overlap = os.environ.get("VST_SHARD_OVERLAP", "1") != "0"
        self.overlap = bool(overlap)
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = str(dist.get_backend(group)).lower()
        self._permute = permute or K.permute_rows
        self._pw = None  # PiecewiseGraph while a step is being captured

    @property
    def graph_capturable(self) -> bool:
        """Piecewise capture works on every backend (the collectives stay outside the graphs)."""
        return True

    def _issue(self, fn):
        if self._pw is not None:
            self._pw.collective(fn)
        else:
            fn()

    def local_frames(self, F: int):
        """(frames per rank, first global frame of this rank)."""
        if F % self.world:
            raise ValueError(f"{F} frames do not split over {self.world} ranks")
        fl = F // self.world
        return fl, self.rank * fl

    # ---- collectives ----------------------------------------------------------------------
    def _staged(self, t: torch.Tensor) -> bool:
        return t.is_cuda and self.backend != "nccl"

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return t

        def op():
            if self._staged(t):
                h = t.cpu()
                dist.all_reduce(h, group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, group=self.group)
        self._issue(op)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """Every rank's equal-shaped `t` stacked rank-major: [world, *t.shape]."""
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        if self.world == 1:
            out[0].copy_(t)
            return out
        src = t.contiguous()

        def op():
            if self.backend != "nccl":  # gloo: list all-gather through host memory
                parts = [torch.empty(src.shape, dtype=src.dtype) for _ in range(self.world)]
                dist.all_gather(parts, src.cpu(), group=self.group)
                out.copy_(torch.stack(parts))
            else:
                dist.all_gather_into_tensor(out, src, group=self.group)
        self._issue(op)
        return out

    def _all_to_all(self, out: torch.Tensor, inp: torch.Tensor):
        def op():
            if self._staged(inp):
                ho = torch.empty(out.shape, dtype=out.dtype)
                dist.all_to_all_single(ho, inp.cpu(), group=self.group)
                out.copy_(ho)
            else:
                dist.all_to_all_single(out, inp, group=self.group)
        self._issue(op)

    def _all_gather_begin(self, out: torch.Tensor, src: torch.Tensor):
        """all_gather_into_tensor(out [world * rows, C], src [rows, C]) issued like _all_to_all_begin; returns its wait."""
        slot = {}

        def issue():
            if self.backend != "nccl":  # gloo: list all-gather through host memory (done at issue)
                parts = [torch.empty(src.shape, dtype=src.dtype) for _ in range(self.world)]
                dist.all_gather(parts, src.cpu(), group=self.group)
                out.copy_(torch.cat(parts))
            else:
                slot["work"] = dist.all_gather_into_tensor(out, src, group=self.group, async_op=True)

        def wait():
            w = slot.pop("work", None)
            if w is not None:
                w.wait()
        self._issue(issue)
        return lambda: self._issue(wait)

    def gather_frames_begin(self, h: torch.Tensor, B: int, Fl: int, HW: int):
        """gather_frames issued without waiting: returns end() -> rows (b, f_global, p) of the whole clip (the all-gather
        runs on RCCL's stream until end() makes the compute stream wait for it)."""
        src = h.contiguous()
        g = torch.empty((self.world * src.shape[0], src.shape[1]), dtype=src.dtype, device=src.device)
        wait = self._all_gather_begin(g, src)

        def end():
            wait()
            return self._permute(g, (self.world, B, Fl, HW), (1, 0, 2, 3))
        return end, src

    def _all_to_all_begin(self, out: torch.Tensor, inp: torch.Tensor):
        """Issue the all-to-all without making the compute stream wait for it; returns the `wait` to call before `out`
        is read.  nccl (RCCL): async_op=True -- the collective runs on RCCL's stream after the work already queued on
        the current stream, so the kernels queued between begin and wait overlap it.  gloo (host-staged): done at
        begin (no overlap; same result).  Under piecewise capture both halves are host items between graph pieces."""
        slot = {}

        def issue():
            if self._staged(inp):
                ho = torch.empty(out.shape, dtype=out.dtype)
                dist.all_to_all_single(ho, inp.cpu(), group=self.group)
                out.copy_(ho)
            else:
                slot["work"] = dist.all_to_all_single(out, inp, group=self.group, async_op=True)

        def wait():
            w = slot.pop("work", None)
            if w is not None:
                w.wait()  # the current stream waits for RCCL's (no host block)
        self._issue(issue)
        return lambda: self._issue(wait)

    # ---- layout exchange ------------------------------------------------------------------
    def to_pixels(self, h: torch.Tensor, B: int, Fl: int, HW: int) -> torch.Tensor:
        """rows (b, f_local, p) over this rank's frames -> rows (b, f_global, p') over pixel slab `rank`
        (p' < HW/P), every frame of every clip."""
        P = self.world
        if P == 1:
            return h
        if HW % P:
            raise ValueError(f"{HW} pixels do not split over {P} ranks")
        hp = HW // P
        send = self._permute(h, (B, Fl, P, hp), (2, 0, 1, 3))   # (dest rank q, b, f_local, p')
        recv = torch.empty_like(send)
        self._all_to_all(recv, send)                             # (source rank r, b, f_local, p')
        return self._permute(recv, (P, B, Fl, hp), (1, 0, 2, 3))  # (b, r*Fl + f_local, p')

    def gather_frames(self, h: torch.Tensor, B: int, Fl: int, HW: int) -> torch.Tensor:
        """rows (b, f_local, p) of this rank's frames -> rows (b, f_global, p) of the whole clip on every rank."""
        P = self.world
        if P == 1:
            return h
        g = self.all_gather(h)                                          # (rank r, b, f_local, p)
        return self._permute(g.view(-1, h.shape[1]), (P, B, Fl, HW), (1, 0, 2, 3))  # (b, r*Fl + f_local, p)

    def local_frames_of(self, h: torch.Tensor, B: int, Fl: int, HW: int) -> torch.Tensor:
        """rows (b, f_global, p) of the whole clip -> rows (b, f_local, p) of this rank's frames."""
        P = self.world
        if P == 1:
            return h
        return h.view(B, P, Fl * HW, h.shape[1])[:, self.rank].reshape(B * Fl * HW, h.shape[1])

    def to_frames(self, h: torch.Tensor, B: int, Fl: int, HW: int) -> torch.Tensor:
        """Inverse of to_pixels."""
        P = self.world
        if P == 1:
            return h
        hp = HW // P
        send = self._permute(h, (B, P, Fl, hp), (1, 0, 2, 3))   # (dest rank r, b, f_local, p')
        recv = torch.empty_like(send)
        self._all_to_all(recv, send)                             # (source slab q, b, f_local, p')
        return self._permute(recv, (P, B, Fl, hp), (1, 2, 0, 3))  # (b, f_local, q*hp + p')

    # ---- the exchange overlapped with compute -------------------------------------------------
    def _to_pixels_begin(self, h, B, Fl, HW):
        P, hp = self.world, HW // self.world
        send = self._permute(h, (B, Fl, P, hp), (2, 0, 1, 3))
        recv = torch.empty_like(send)
        wait = self._all_to_all_begin(recv, send)

        def end():
            wait()
            return self._permute(recv, (P, B, Fl, hp), (1, 0, 2, 3))
        return end, send  # (send is held until end: the collective reads it)

    def _to_frames_begin(self, h, B, Fl, HW):
        P, hp = self.world, HW // self.world
        send = self._permute(h, (B, P, Fl, hp), (1, 0, 2, 3))
        recv = torch.empty_like(send)
        wait = self._all_to_all_begin(recv, send)

        def end():
            wait()
            return self._permute(recv, (P, B, Fl, hp), (1, 2, 0, 3))
        return end, send

    def pipelined(self, nparts: int, pre, mid, post, B: int, Fl: int, HW: int) -> None:
        """The all-to-all motion-module schedule over `nparts` equal slices of the batch (B = clips per slice), so
        that each slice's exchange runs while the previous slice computes (the exchange overlapped with
        compute):
            pre(0) x0  pre(1) x1  w0 mid(0) x0'  w1 mid(1) x1'  w0' post(0)  w1' post(1)
        pre(i) -> rows (b, f_local, p) of slice i (GroupNorm + proj_in); mid(i, h) on rows (b, f_global, p') of
        pixel slab `rank` (the transformer block); post(i, h) consumes rows (b, f_local, p) (proj_out + residual).
        x = an all-to-all issued (to_pixels / to_frames), w = its wait.  Every slice runs the same row-wise ops on
        its own rows as the one-slice schedule, so the result is the same bits (test_frame_shard.py)."""
        if self.world == 1 or HW % self.world:
            raise ValueError(f"pipelined exchange: {HW} pixels over {self.world} ranks")
        ends = []
        for i in range(nparts):
            ends.append(self._to_pixels_begin(pre(i), B, Fl, HW))
        for i in range(nparts):
            end, _send = ends[i]
            ends[i] = self._to_frames_begin(mid(i, end()), B, Fl, HW)
        for i in range(nparts):
            end, _send = ends[i]
            post(i, end())
            ends[i] = None

