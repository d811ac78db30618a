"""UNetMotionModel (SDXL + AnimateDiff motion modules), MI355X-native.

Module tree and parameter names follow diffusers' UNetMotionModel, which the reference builds with
`UNetMotionModel.from_unet2d` (animatediff/utils.py:13-45) and then patches with UnZipLoRA
(unziplora_unet/utils.py:388-484) and AnimateDiffAttnProcessor2_0 (inference_animatediff.py:209-215).
So `load_state_dict` of a reference/diffusers checkpoint (plus Stage-1 LoRA keys) drops in.

Execution is MI355X-first: activations never leave the token-major NHWC layout
[(b*F + f)*H*W + p, C] (bf16); every conv is an implicit GEMM, every projection a fused MFMA
GEMM with bias / residual / GEGLU / temb epilogues, GroupNorm+SiLU and LayerNorm(+PE) are single
passes, the skip concatenation of the up path is read from two sources instead of copied, and the
motion modules read the frame axis in place (no permutes).  The public forward keeps the
reference signature and 5-D (B, C, F, h, w) in/out.

Block semantics (diffusers ~0.30, restated in oracle/unet.py with citations):
  ResnetBlock2D:        GN+SiLU -> conv3x3 (+ time_emb_proj(SiLU(emb))) -> GN+SiLU -> conv3x3 (+ shortcut)
  Transformer2DModel:   GN(eps 1e-6) -> proj_in -> BasicTransformerBlock* -> proj_out -> + residual
  BasicTransformerBlock: LN -> attn1 -> +res ; LN -> attn2(text) -> +res ; LN -> GEGLU FF -> +res
  motion module:        GN over (C-group, F, H, W) -> proj_in -> block(self, self, PE before each attn)
                        -> proj_out -> + residual
"""
from __future__ import annotations

import os

import dataclasses
from dataclasses import dataclass
from typing import Optional

import torch
from torch import nn

from . import kernels as K
from .attention_processor import Attention, input_lora_ops
from .config import UNetMotionConfig
from .lora_linear import LoRACompatibleLinear, build_ops, lora_in_gemm, run_ops
from .weights import sinusoid_table

BF16 = torch.bfloat16


class _F32Cache:
    """fp32 device copies of bf16 params (norm affine, conv/linear bias) keyed by tensor version."""

    @staticmethod
    def get(p: torch.Tensor) -> torch.Tensor:
        if p.requires_grad:  # trained parameters change under graph replay without a version bump: no cache
            return p.detach().float().contiguous()
        key = (p.data_ptr(), p._version)
        c = p.__dict__.get("_vst_f32")
        if c is None or c[0] != key:
            c = (key, p.detach().float().contiguous())
            p.__dict__["_vst_f32"] = c
        return c[1]


f32 = _F32Cache.get


class GroupNorm(nn.GroupNorm):
    def run(self, x1, nsamples, rows_per_sample, *, silu=False, x2=None, out=None):
        # statistics from column statistics (128-row chunks): the producing conv's epilogue wrote them
        # (K.conv3x3(colstat=True)) or vst_colstat makes them, the same bits either way, so a frame shard (whose convs
        # may run on other tiles) normalises exactly as the whole clip does
        cs = K.group_norm_stats(x1, x2) if rows_per_sample % 128 == 0 and K.colstat_enabled() else None
        return K.group_norm(x1, nsamples, rows_per_sample, self.num_groups, self.eps, f32(self.weight), f32(self.bias),
                            silu=silu, x2=x2, out=out, colstat=cs)


class LayerNorm(nn.LayerNorm):
    def run(self, x, *, pe=None, pe_div=1, pe_mod=1, out=None):
        return K.layer_norm(x, f32(self.weight), f32(self.bias), self.eps, pe=pe, pe_div=pe_div, pe_mod=pe_mod,
                            out=out)

    def run_lora(self, x, ops):
        """(LN(x), LN(x) @ ops.a^T or None): the LoRA down-projection fused into the normalisation pass when
        the consuming projections carry one and the shapes suit the fused kernel."""
        C = x.shape[1]
        if ops is None or ops.a is None or ops.a.shape[0] > 64 or C % 32 or C > 1280 or lora_in_gemm(ops, x.shape[0]):
            return self.run(x), None
        return K.layer_norm_lora(x, f32(self.weight), f32(self.bias), self.eps, ops.a, r_alg=ops.r)


class Conv3x3(nn.Conv2d):
    """nn.Conv2d(k=3, pad=1) whose device weight is re-laid out once to [Cout, (ky,kx,ci)]."""

    def __init__(self, cin, cout, stride=1):
        super().__init__(cin, cout, 3, stride=stride, padding=1)

    def kernel_weight(self):
        key = (self.weight.data_ptr(), self.weight._version)
        c = self.__dict__.get("_vst_w")
        if c is None or c[0] != key:
            co, ci = self.weight.shape[:2]
            w = self.weight.detach().permute(0, 2, 3, 1).reshape(co, 9 * ci)
            kp = (9 * ci + 7) & ~7
            if kp != 9 * ci:
                w = torch.cat([w, w.new_zeros(co, kp - 9 * ci)], 1)
            c = (key, w.to(BF16).contiguous())
            self.__dict__["_vst_w"] = c
        return c[1]

    def run(self, x1, nimg, H, W, *, x2=None, upsample=False, row_bias=None, row_bias_div=1, residual=None,
            colstat=False):
        return K.conv3x3(x1, nimg, H, W, self.kernel_weight(), f32(self.bias), x2=x2, stride=self.stride[0],
                         upsample=upsample, row_bias=row_bias, row_bias_div=row_bias_div, residual=residual,
                         colstat=colstat)


class Conv1x1(nn.Conv2d):
    def __init__(self, cin, cout):
        super().__init__(cin, cout, 1)

    def kernel_weight(self):
        key = (self.weight.data_ptr(), self.weight._version)
        c = self.__dict__.get("_vst_w")
        if c is None or c[0] != key:
            c = (key, self.weight.detach().reshape(self.weight.shape[0], -1).to(BF16).contiguous())
            self.__dict__["_vst_w"] = c
        return c[1]

    def run(self, x1, x2=None):
        return K.linear(x1, self.kernel_weight(), f32(self.bias), x2=x2)


class Linear(LoRACompatibleLinear):
    """Plain projection (proj_in/out, FF, embeddings) — LoRACompatibleLinear without a lora layer."""

    def run(self, x, *, residual=None, out=None):
        return run_ops(x, build_ops([self], 1.0), residual=residual, out=out)


@dataclass
class FwdCtx:
    B: int                 # clips in the batch (CFG-batched: 2x)
    F: int                 # frames per clip
    emb_silu: torch.Tensor  # [B, T] bf16, SiLU(time + add embedding)
    enc: Optional[torch.Tensor]  # [B, L, D] bf16 text states
    cross_kwargs: dict
    shard: Optional[object] = None  # frame_shard.FrameShard when the clip's frames span ranks (F is per rank)
    temb: Optional[dict] = None     # ResnetBlock2D -> fp32 [B, Cout] view of the batched time_emb_proj output


# --------------------------------------------------------------------------------------- blocks
class GEGLU(nn.Module):
    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.proj = Linear(dim_in, dim_out * 2)

    def geglu_ops(self):
        """proj weight with hidden/gate rows interleaved per 32-output block (GEMM GEGLU epilogue).  Cached per
        parameter version while the weights are frozen; trained weights are re-interleaved on every call (a cache
        keyed on the version would go stale under HIP-graph replay, which updates parameters without Python)."""
        w, b = self.proj.weight, self.proj.bias
        if w.requires_grad or b.requires_grad:
            return self._interleaved(w, b)
        key = (w.data_ptr(), w._version, b.data_ptr(), b._version)
        c = self.__dict__.get("_vst_geglu")
        if c is None or c[0] != key:
            c = (key, self._interleaved(w, b))
            self.__dict__["_vst_geglu"] = c
        return c[1]

    @staticmethod
    def _interleaved(w, b):
        inner = w.shape[0] // 2
        idx = torch.arange(inner, device=w.device).view(-1, 32)
        idx = torch.cat([idx, idx + inner], 1).reshape(-1)
        return w.detach()[idx].to(BF16).contiguous(), b.detach()[idx].float().contiguous()


class FeedForward(nn.Module):
    """diffusers FeedForward(activation_fn="geglu"): net = [GEGLU, Dropout, Linear]."""

    def __init__(self, dim, mult=4):
        super().__init__()
        inner = dim * mult
        self.net = nn.ModuleList([GEGLU(dim, inner), nn.Dropout(0.0), Linear(inner, dim)])

    def run(self, x, residual):
        w, b = self.net[0].geglu_ops()
        h = K.linear(x, w, b, geglu=True)
        return self.net[2].run(h, residual=residual)


class BasicTransformerBlock(nn.Module):
    """unziplora_unet/unzip_attention.py:13-239 / diffusers BasicTransformerBlock (norm_type layer_norm)."""

    def __init__(self, dim, heads, head_dim, cross_attention_dim=None, temporal=False, max_seq_length=32):
        super().__init__()
        self.temporal = temporal
        self.norm1 = LayerNorm(dim)
        self.attn1 = Attention(dim, None, heads, head_dim, temporal=temporal)
        self.norm2 = LayerNorm(dim)
        self.attn2 = Attention(dim, None if temporal else cross_attention_dim, heads, head_dim, temporal=temporal)
        self.norm3 = LayerNorm(dim)
        self.ff = FeedForward(dim)
        if temporal:
            self.pos_embed = _SinusoidalPE(dim, max_seq_length)

    def _fused_motion_ops(self, C, F, HW):
        return _fused_motion_ops_impl(self, C, F, HW)

    def run(self, x, nimg, N, ctx: FwdCtx):
        """x: [nimg*N, C] -> same."""
        C = x.shape[1]
        if self.temporal:
            pe = f32(self.pos_embed.pe).view(-1, C)
            fused = self._fused_motion_ops(C, ctx.F, N)
            if fused is not None:
                # each attention half (norm + PE, q/k/v, frame attention, to_out, residual) as one launch
                for norm, (qkv, o) in zip((self.norm1, self.norm2), fused):
                    x = K.motion_attention_block(x, nimg // ctx.F, ctx.F, N, self.attn1.heads, f32(norm.weight),
                                                 f32(norm.bias), norm.eps, pe, qkv.w, qkv.bias, o.w, o.bias)
                n = self.norm3.run(x)
                return self.ff.run(n, residual=x)
            kw = dict(pe=pe, pe_div=N, pe_mod=ctx.F)
            n = self.norm1.run(x, **kw)
            x = self.attn1(n.view(nimg, N, C), num_frames=ctx.F, _vst_residual=x).view(-1, C)
            n = self.norm2.run(x, **kw)
            x = self.attn2(n.view(nimg, N, C), num_frames=ctx.F, _vst_residual=x).view(-1, C)
        else:
            scale = ctx.cross_kwargs.get("scale", 1.0)
            n, u = self.norm1.run_lora(x, input_lora_ops(self.attn1, True, scale))
            x = self.attn1(n.view(nimg, N, C), _vst_residual=x, _vst_lora_u=u, **ctx.cross_kwargs).view(-1, C)
            n, u = self.norm2.run_lora(x, input_lora_ops(self.attn2, False, scale))
            x = self.attn2(n.view(nimg, N, C), encoder_hidden_states=ctx.enc, _vst_residual=x, _vst_lora_u=u,
                           **ctx.cross_kwargs).view(-1, C)
        n = self.norm3.run(x)
        return self.ff.run(n, residual=x)


def _fused_motion_ops_impl(block, C, F, HW):
    """[(qkv ops, out ops)] for attn1 / attn2 when vst_motion_attention_block can run them: the default processor,
    no LoRA on any projection (temporal LoRA trains through the autograd path), the kernel's shape."""
    from .attention_processor import AttnProcessor2_0
    # opt-in (VST_MOTION_FUSE=1): the fused block is correct but measured slower than the four launches
    if os.environ.get("VST_MOTION_FUSE") != "1" or not K.motion_block_fusable(C, F, HW, block.attn1.heads):
        return None
    # shape-dependent like the fused frame attention (kernels.fusion_world): decide as a P-way all-to-all rank, which
    # holds HW / P pixels, decides, so an unsharded forward under fusion_world(P) equals the shards bit for bit
    P = K.fusion_pixel_div()
    if P > 1 and (HW % P or not K.motion_block_fusable(C, F, HW // P, block.attn1.heads)):
        return None
    out = []
    for attn in (block.attn1, block.attn2):
        if type(attn.processor) is not AttnProcessor2_0 or attn.heads != block.attn1.heads:
            return None
        qkv = build_ops([attn.to_q, attn.to_k, attn.to_v], 1.0)
        o = build_ops([attn.to_out[0]], 1.0)
        if qkv.a is not None or o.a is not None or qkv.w.shape != (3 * C, C) or o.w.shape != (C, C):
            return None
        out.append((qkv, o))
    return out


class _SinusoidalPE(nn.Module):
    def __init__(self, dim, max_len=32):
        super().__init__()
        self.register_buffer("pe", sinusoid_table(dim, max_len))


class Transformer2DModel(nn.Module):
    """unziplora_unet/transformer_2d.py:137-352 (continuous input, use_linear_projection=True)."""

    def __init__(self, heads, head_dim, C, layers, cross_attention_dim, groups=32):
        super().__init__()
        self.norm = GroupNorm(groups, C, eps=1e-6)
        self.proj_in = Linear(C, C)
        self.transformer_blocks = nn.ModuleList(
            [BasicTransformerBlock(C, heads, head_dim, cross_attention_dim) for _ in range(layers)])
        self.proj_out = Linear(C, C)

    def run(self, x, nimg, H, W, ctx):
        h = self.norm.run(x, nimg, H * W)
        h = self.proj_in.run(h)
        for blk in self.transformer_blocks:
            h = blk.run(h, nimg, H * W, ctx)
        return self.proj_out.run(h, residual=x)


class MotionModule(nn.Module):
    """diffusers AnimateDiffTransformer3D (motion module built by UNetMotionModel.from_unet2d)."""

    def __init__(self, C, heads=8, groups=32, max_seq_length=32):
        super().__init__()
        self.norm = GroupNorm(groups, C, eps=1e-6)
        self.proj_in = Linear(C, C)
        self.transformer_blocks = nn.ModuleList(
            [BasicTransformerBlock(C, heads, C // heads, None, temporal=True, max_seq_length=max_seq_length)])
        self.proj_out = Linear(C, C)

    def run(self, x, nimg, H, W, ctx):
        HW = H * W
        shard = ctx.shard
        B, G = nimg // ctx.F, self.norm.num_groups
        if shard is not None and shard.world > 1 and shard.exchange == "all_gather":
            # north-star exchange (frame_shard.py): the whole clip on every rank, this rank's frames kept at the end.
            # With overlap, the batch's two halves (the CFG pair) are gathered by two async all-gathers issued up front,
            # so half 1's gather runs under half 0's module (the gather overlapped with compute)
            Fl, P = ctx.F, shard.world
            F = Fl * P
            tctx = dataclasses.replace(ctx, F=F)
            halves = 2 if shard.overlap and B % 2 == 0 else 1
            nb, rows = B // halves, (B // halves) * Fl * HW
            ends = [shard.gather_frames_begin(x[i * rows:(i + 1) * rows], nb, Fl, HW) for i in range(halves)]
            out = torch.empty_like(x) if halves > 1 else None
            for i in range(halves):
                end, _src = ends[i]
                xf = end()
                part = K.group_norm_frame_partials(xf, nb * F, HW, G)
                h = K.group_norm_apply_partials(xf, nb, F, HW, G, self.norm.eps, f32(self.norm.weight),
                                                f32(self.norm.bias), part, 1)
                h = self.proj_in.run(h)
                for blk in self.transformer_blocks:
                    h = blk.run(h, nb * F, HW, tctx)
                ends[i] = None
                if halves == 1:
                    return self.proj_out.run(shard.local_frames_of(h, nb, Fl, HW), residual=x)
                self.proj_out.run(shard.local_frames_of(h, nb, Fl, HW), residual=x[i * rows:(i + 1) * rows],
                                  out=out[i * rows:(i + 1) * rows])
            return out
        # GroupNorm statistics over every frame of a clip, from per-frame partials merged in one fixed frame order:
        # the same bits whether this process holds the whole clip or a frame shard of it
        part = K.group_norm_frame_partials(x, nimg, HW, G)
        P = 1 if shard is None else shard.world
        if P > 1:
            part = shard.all_gather(part)
            if shard.overlap and B % 2 == 0 and HW % P == 0:
                return self._run_overlapped(x, B, ctx.F, HW, P, ctx, part)
        h = K.group_norm_apply_partials(x, B, ctx.F, HW, G, self.norm.eps, f32(self.norm.weight), f32(self.norm.bias),
                                        part, P)
        h = self.proj_in.run(h)
        if P == 1:
            for blk in self.transformer_blocks:
                h = blk.run(h, nimg, HW, ctx)
            return self.proj_out.run(h, residual=x)
        # frames of each clip spread over ranks (frame_shard.py): frame-axis work on a pixel shard holding every frame
        Fl = ctx.F
        h = shard.to_pixels(h, B, Fl, HW)
        tctx = dataclasses.replace(ctx, F=Fl * P)
        with K.fusion_world(1):  # (these HW // P pixels are this rank's share already)
            for blk in self.transformer_blocks:
                h = blk.run(h, B * Fl * P, HW // P, tctx)
        h = shard.to_frames(h, B, Fl, HW)
        return self.proj_out.run(h, residual=x)

    def _run_overlapped(self, x, B, Fl, HW, P, ctx, part):
        """The all-to-all branch with the batch in two halves (the CFG pair's uncond / cond clips), so each half's
        exchange runs while the other half computes (FrameShard.pipelined): GroupNorm + proj_in of half 1 under half
        0's frame -> pixel exchange, half 0's transformer block under half 1's, and so on.  Every op is row-wise on
        its half's rows (the GroupNorm statistics are per clip, from the all-gathered partials), so the output is the
        one-half schedule's bits (tests/test_frame_shard.py)."""
        G, nb = self.norm.num_groups, B // 2
        rows = nb * Fl * HW
        out = torch.empty_like(x)
        tctx = dataclasses.replace(ctx, F=Fl * P)
        w, bias = f32(self.norm.weight), f32(self.norm.bias)

        def pre(i):
            xs = x[i * rows:(i + 1) * rows]
            ps = part[:, i * nb * Fl:(i + 1) * nb * Fl].contiguous()  # [P, nb*Fl, chunks, G, 2]: this half's clips
            h = K.group_norm_apply_partials(xs, nb, Fl, HW, G, self.norm.eps, w, bias, ps, P)
            return self.proj_in.run(h)

        def mid(i, h):
            with K.fusion_world(1):  # (these HW // P pixels are this rank's share already)
                for blk in self.transformer_blocks:
                    h = blk.run(h, nb * Fl * P, HW // P, tctx)
            return h

        def post(i, h):
            self.proj_out.run(h, residual=x[i * rows:(i + 1) * rows], out=out[i * rows:(i + 1) * rows])

        ctx.shard.pipelined(2, pre, mid, post, nb, Fl, HW)
        return out


class ResnetBlock2D(nn.Module):
    def __init__(self, cin, cout, temb, groups=32, eps=1e-5):
        super().__init__()
        self.in_channels, self.out_channels = cin, cout
        self.norm1 = GroupNorm(groups, cin, eps=eps)
        self.conv1 = Conv3x3(cin, cout)
        self.time_emb_proj = Linear(temb, cout)
        self.norm2 = GroupNorm(groups, cout, eps=eps)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = Conv3x3(cout, cout)
        self.conv_shortcut = Conv1x1(cin, cout) if cin != cout else None

    def run(self, x1, nimg, H, W, ctx, x2=None):
        HW = H * W
        h = self.norm1.run(x1, nimg, HW, silu=True, x2=x2)
        if ctx.temb is not None and self in ctx.temb:
            temb = ctx.temb[self]  # view of the one batched projection (UNetMotionModel.batched_temb)
        else:
            temb = self.time_emb_proj.run(ctx.emb_silu).float()  # [B, cout]; bf16-rounded like the reference
        h = self.conv1.run(h, nimg, H, W, row_bias=temb, row_bias_div=ctx.F * HW, colstat=True)
        h = self.norm2.run(h, nimg, HW, silu=True)
        sc = self.conv_shortcut.run(x1, x2) if self.conv_shortcut is not None else x1
        return self.conv2.run(h, nimg, H, W, residual=sc, colstat=True)


class Downsample2D(nn.Module):
    def __init__(self, C):
        super().__init__()
        self.conv = Conv3x3(C, C, stride=2)

    def run(self, x, nimg, H, W):
        return self.conv.run(x, nimg, H, W, colstat=True), (H + 1) // 2, (W + 1) // 2


class Upsample2D(nn.Module):
    def __init__(self, C):
        super().__init__()
        self.conv = Conv3x3(C, C)

    def run(self, x, nimg, H, W):
        return self.conv.run(x, nimg, H, W, upsample=True, colstat=True), 2 * H, 2 * W


class DownBlock(nn.Module):
    """DownBlockMotion / CrossAttnDownBlockMotion."""

    def __init__(self, cin, cout, temb, layers, cross, t_layers, heads, cross_dim, add_down, motion_heads, motion=True):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if j == 0 else cout, cout, temb) for j in range(layers)])
        self.attentions = nn.ModuleList(
            [Transformer2DModel(heads, cout // heads, cout, t_layers, cross_dim) for _ in range(layers)]) if cross else None
        self.motion_modules = nn.ModuleList([MotionModule(cout, motion_heads) for _ in range(layers)]) if motion else None
        self.downsamplers = nn.ModuleList([Downsample2D(cout)]) if add_down else None

    def run(self, x, nimg, H, W, ctx):
        outs = []
        for j, res in enumerate(self.resnets):
            x = res.run(x, nimg, H, W, ctx)
            if self.attentions is not None:
                x = self.attentions[j].run(x, nimg, H, W, ctx)
            if self.motion_modules is not None:
                x = self.motion_modules[j].run(x, nimg, H, W, ctx)
            outs.append((x, H, W))
        if self.downsamplers is not None:
            x, H, W = self.downsamplers[0].run(x, nimg, H, W)
            outs.append((x, H, W))
        return x, H, W, outs


class UpBlock(nn.Module):
    """UpBlockMotion / CrossAttnUpBlockMotion."""

    def __init__(self, prev_c, cout, skip_in, temb, layers, cross, t_layers, heads, cross_dim, add_up, motion_heads,
                 motion=True):
        super().__init__()
        n = layers + 1
        self.resnets = nn.ModuleList([
            ResnetBlock2D((prev_c if j == 0 else cout) + (skip_in if j == n - 1 else cout), cout, temb)
            for j in range(n)])
        self.attentions = nn.ModuleList(
            [Transformer2DModel(heads, cout // heads, cout, t_layers, cross_dim) for _ in range(n)]) if cross else None
        self.motion_modules = nn.ModuleList([MotionModule(cout, motion_heads) for _ in range(n)]) if motion else None
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if add_up else None

    def run(self, x, nimg, H, W, ctx, skips):
        for j, res in enumerate(self.resnets):
            s, sh, sw = skips.pop()
            assert (sh, sw) == (H, W)
            x = res.run(x, nimg, H, W, ctx, x2=s)  # channel concat [x, skip] read from two sources
            if self.attentions is not None:
                x = self.attentions[j].run(x, nimg, H, W, ctx)
            if self.motion_modules is not None:
                x = self.motion_modules[j].run(x, nimg, H, W, ctx)
        if self.upsamplers is not None:
            x, H, W = self.upsamplers[0].run(x, nimg, H, W)
        return x, H, W


class MidBlock(nn.Module):
    """UNetMidBlockCrossAttnMotion (no motion module for the SDXL-beta adapter)."""

    def __init__(self, C, temb, t_layers, heads, cross_dim, motion, motion_heads):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(C, C, temb), ResnetBlock2D(C, C, temb)])
        self.attentions = nn.ModuleList([Transformer2DModel(heads, C // heads, C, t_layers, cross_dim)])
        self.motion_modules = nn.ModuleList([MotionModule(C, motion_heads)]) if motion else None

    def run(self, x, nimg, H, W, ctx):
        x = self.resnets[0].run(x, nimg, H, W, ctx)
        x = self.attentions[0].run(x, nimg, H, W, ctx)
        if self.motion_modules is not None:
            x = self.motion_modules[0].run(x, nimg, H, W, ctx)
        return self.resnets[1].run(x, nimg, H, W, ctx)


class TimestepEmbedding(nn.Module):
    def __init__(self, cin, T):
        super().__init__()
        self.linear_1 = Linear(cin, T)
        self.linear_2 = Linear(T, T)

    def run(self, x, residual=None):
        h = self.linear_1.run(x)
        h = K.silu(h)
        return self.linear_2.run(h, residual=residual)


@dataclass
class UNetMotionOutput:
    sample: torch.Tensor


class UNetMotionModel(nn.Module):
    def __init__(self, config: Optional[UNetMotionConfig] = None):
        super().__init__()
        cfg = config or UNetMotionConfig.sdxl()
        self.config = cfg
        ch = cfg.block_out_channels
        T = cfg.time_embed_dim
        self.conv_in = Conv3x3(cfg.in_channels, ch[0])
        self.time_embedding = TimestepEmbedding(ch[0], T)
        self.add_embedding = TimestepEmbedding(cfg.projection_class_embeddings_input_dim, T)
        self.down_blocks = nn.ModuleList()
        out_c = ch[0]
        for i, bt in enumerate(cfg.down_block_types):
            in_c, out_c = out_c, ch[i]
            self.down_blocks.append(DownBlock(in_c, out_c, T, cfg.layers_per_block, bt.startswith("CrossAttn"),
                                              cfg.transformer_layers_per_block[i], cfg.num_attention_heads[i],
                                              cfg.cross_attention_dim, i < len(ch) - 1, cfg.motion_num_attention_heads,
                                              cfg.motion_modules))
        self.mid_block = MidBlock(ch[-1], T, cfg.transformer_layers_per_block[-1], cfg.num_attention_heads[-1],
                                  cfg.cross_attention_dim, cfg.use_motion_mid_block and cfg.motion_modules,
                                  cfg.motion_num_attention_heads)
        rch = list(reversed(ch))
        rtl = list(reversed(cfg.transformer_layers_per_block))
        rheads = list(reversed(cfg.num_attention_heads))
        self.up_blocks = nn.ModuleList()
        out_c = rch[0]
        for i, bt in enumerate(cfg.up_block_types):
            prev_c, out_c = out_c, rch[i]
            skip_in = rch[min(i + 1, len(ch) - 1)]
            self.up_blocks.append(UpBlock(prev_c, out_c, skip_in, T, cfg.layers_per_block, bt.startswith("CrossAttn"),
                                          rtl[i], rheads[i], cfg.cross_attention_dim, i < len(ch) - 1,
                                          cfg.motion_num_attention_heads, cfg.motion_modules))
        self.conv_norm_out = GroupNorm(cfg.norm_num_groups, ch[0], eps=cfg.norm_eps)
        self.conv_out = Conv3x3(ch[0], cfg.out_channels)

    # ---- diffusers surface ----------------------------------------------------------------
    @property
    def dtype(self):
        return self.conv_in.weight.dtype

    @property
    def attn_processors(self):
        return {f"{n}.processor": m.processor for n, m in self.named_modules() if isinstance(m, Attention)}

    def set_attn_processor(self, processor):
        mods = {f"{n}.processor": m for n, m in self.named_modules() if isinstance(m, Attention)}
        if isinstance(processor, dict):
            if set(processor) != set(mods):
                raise ValueError("processor dict keys must match attn_processors")
            for k, p in processor.items():
                mods[k].set_processor(p)
        else:
            for m in mods.values():
                m.set_processor(processor)

    # ---- embeddings -----------------------------------------------------------------------
    def embed(self, timestep, text_embeds, time_ids, B, step_idx=None, out=None):
        """SiLU(time_embedding(Timesteps(t)) + add_embedding([text_embeds, Timesteps(time_ids)])) -> [B, T].
        `timestep`: fp32 device tensor [B] (or a schedule table with step_idx)."""
        cfg = self.config
        ch0 = cfg.block_out_channels[0]
        dev = text_embeds.device
        t_in = torch.empty(B, ch0, dtype=BF16, device=dev)
        K.timestep_embedding(timestep, B, ch0, t_in, step_idx=step_idx)
        add_in = torch.empty(B, cfg.projection_class_embeddings_input_dim, dtype=BF16, device=dev)
        K.copy2d(text_embeds, add_in[:, : cfg.text_embed_dim])
        tid = time_ids.float().reshape(-1).contiguous()
        K.timestep_embedding(tid, B * cfg.num_time_ids, cfg.addition_time_embed_dim, add_in,
                             col0=cfg.text_embed_dim, per_row=cfg.num_time_ids)
        temb = self.time_embedding.run(t_in)
        emb = self.add_embedding.run(add_in, residual=temb)  # emb = temb + aug_emb
        return K.silu(emb, out=out)

    def batched_temb(self, emb_silu):
        """time_emb_proj(SiLU(emb)) of EVERY ResnetBlock2D as one GEMM over the concatenated weights
        ([B, sum Cout], bf16-rounded like the reference's per-block Linear, then fp32 once): 17 M=2
        projections become one launch.  Returns {resnet: fp32 [B, Cout] view}."""
        res = [m for m in self.modules() if isinstance(m, ResnetBlock2D)]
        ops = build_ops([m.time_emb_proj for m in res], 1.0)
        allt = run_ops(emb_silu, ops).float()
        out, o = {}, 0
        for m in res:
            c = m.out_channels
            out[m] = allt[:, o:o + c]
            o += c
        return out

    # ---- core (NHWC tokens) -----------------------------------------------------------------
    def forward_tokens(self, x, B, F, h, w, emb_silu, enc, cross_kwargs=None, shard=None, fusion_world=None):
        """x: [B*F*h*w, in_channels] bf16 -> noise prediction [B*F*h*w, out_channels] bf16.
        With `shard` (frame_shard.FrameShard), F is this rank's frames of each clip.  `fusion_world` P (default: the
        shard's world size, else 1): take the shape-dependent fusion decisions a P-way frame-sharded rank takes
        (kernels.fusion_world), so an unsharded forward equals a P-way sharded one bit for bit."""
        if fusion_world is None:
            fusion_world = shard.world if shard is not None else 1
        # no split-K: a row's bits do not depend on the launch's row count (frame shards)
        K.colstat_reset()
        with K.row_invariant(), K.fusion_world(fusion_world):
            ctx = FwdCtx(B, F, emb_silu, enc, cross_kwargs or {}, shard, self.batched_temb(emb_silu))
            nimg = B * F
            H, W = h, w
            x = self.conv_in.run(x, nimg, H, W)
            skips = [(x, H, W)]
            for blk in self.down_blocks:
                x, H, W, outs = blk.run(x, nimg, H, W, ctx)
                skips.extend(outs)
            x = self.mid_block.run(x, nimg, H, W, ctx)
            for blk in self.up_blocks:
                x, H, W = blk.run(x, nimg, H, W, ctx, skips)
            x = self.conv_norm_out.run(x, nimg, H * W, silu=True)
            return self.conv_out.run(x, nimg, H, W)

    def forward(self, sample, timestep, encoder_hidden_states, timestep_cond=None, attention_mask=None,
                cross_attention_kwargs=None, added_cond_kwargs=None, return_dict=True, frame_shard=None,
                fusion_world=None, **kwargs):
        """diffusers UNetMotionModel.forward signature (inference_animatediff.py:110-121).  With
        `frame_shard` (frame_shard.FrameShard) `sample` holds this rank's frames of each clip; `fusion_world`: see
        forward_tokens."""
        if not sample.is_cuda:
            raise K._lib.VstError("UNetMotionModel: sample is on CPU; the HIP path has no CPU fallback")
        B, Cin, F, h, w = sample.shape
        dev = sample.device
        t = timestep if torch.is_tensor(timestep) else torch.tensor([timestep])
        t = t.to(device=dev, dtype=torch.float32).reshape(-1)
        if t.numel() == 1:
            t = t.expand(B)
        t = t.contiguous()
        text_embeds = added_cond_kwargs["text_embeds"].to(dev, BF16).reshape(B, -1).contiguous()
        time_ids = added_cond_kwargs["time_ids"].to(dev).reshape(B, -1)
        emb_silu = self.embed(t, text_embeds, time_ids, B)
        enc = encoder_hidden_states.to(dev, BF16).contiguous()
        x = torch.empty(B * F * h * w, Cin, dtype=BF16, device=dev)
        K.pack_latents(sample.float().contiguous(), x)
        y = self.forward_tokens(x, B, F, h, w, emb_silu, enc, cross_attention_kwargs, shard=frame_shard,
                                fusion_world=fusion_world)
        out = y.view(B, F, h, w, -1).permute(0, 4, 1, 2, 3).contiguous().to(sample.dtype)
        return UNetMotionOutput(out) if return_dict else (out,)
