"""Training path, first piece: autograd Functions whose forward AND backward run on the HIP
kernels, for the projections `train_animatediff.py` trains (train_animatediff.py:212-319).

`LoRALinearFn`: y = x W^T + b + s (x A^T) B^T — `TemporalLoRALinear` (animatediff/temporal_lora.py:10-41, W frozen,
A/B trainable) and the motion-module linears whose W/b are trainable (animatediff/utils.py:79-85 leaves FF and
proj_in/out unfrozen).  With g = dL/dy (bf16, tokens x out):
    forward   u = x A^T (skinny GEMM)            y = [x | u] . [W | s B]^T + b      (one fused GEMM)
    backward  v = g B                            dX = [g | v] . [W^T | s A^T]^T     (one fused GEMM)
              dA = s v^T x,  dB = s g^T u,  db = g^T 1 (a ones row appended to u^T),  dW = g^T x
The weight-side products contract over the token axis: vst_gemm_tn reads g, x, u, v as they lie ([tokens,
features]) and reads both MFMA operands transposed from the LDS (`_tdot`); only the largest gradient outputs keep the
older form (both operands transposed by vst_transpose into [features, tokens], then the split-K ring GEMM), which is
faster there (tools/tn_bench.py).  W^T is cached per weight version when W is frozen.
Gradients come out of bf16 MFMA GEMMs with fp32 accumulation (as under the reference's bf16 autocast) and are
cast to the parameters' dtypes.
"""
from __future__ import annotations

import contextlib

import torch

from . import kernels as K
from .lora_linear import pad32

BF16 = torch.bfloat16


def _wt(W: torch.Tensor) -> torch.Tensor:
    """W^T (bf16, [in, out]), cached on the parameter per version while it is frozen; a trained weight is transposed
    on every call (HIP-graph replay updates it without a version bump, so a cache would go stale)."""
    if W.requires_grad:
        return K.transpose(W.detach().to(BF16).contiguous())
    key = (W.data_ptr(), W._version)
    c = W.__dict__.get("_vst_wt")
    if c is None or c[0] != key:
        c = (key, K.transpose(W.detach().to(BF16).contiguous()))
        W.__dict__["_vst_wt"] = c
    return c[1]


# a^T b over the token axis (weight gradients): vst_gemm_tn up to this many output elements; past it the transposed
# operands' split-K GEMM measured faster (16384 x 10240 x 1280: 509 vs 671 us; every smaller training shape 1.2-3.4x
# slower than vst_gemm_tn, profiles/r6_gemm_tn.txt).  VST_GEMM_TN=0: always the transposed form (A/B).
_TN_MAX_OUT = 8 << 20
_TN_ON = None


def _tdot(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 [a.shape[1], b.shape[1]] = a^T b for token-major a [M, N], b [M, K]."""
    global _TN_ON
    if _TN_ON is None:
        import os
        _TN_ON = os.environ.get("VST_GEMM_TN", "1") != "0"
    if _TN_ON and a.shape[1] * b.shape[1] <= _TN_MAX_OUT:
        return K.linear_tn(a, b)
    Mp = (a.shape[0] + 7) // 8 * 8  # the ring GEMM's K granule: zero-padded token columns
    return K.linear(_transpose_padded(a, Mp), _transpose_padded(b, Mp))


def _transpose_padded(t: torch.Tensor, Mp: int) -> torch.Tensor:
    """[M, C] -> [C, Mp] bf16 with zero columns M..Mp (Mp = M: a plain vst_transpose)."""
    M = t.shape[0]
    if Mp == M:
        return K.transpose(t)
    out = torch.zeros(t.shape[1], Mp, device=t.device, dtype=BF16)
    K.transpose(t, out=out[:, :M])
    return out


class _AugOperands:
    """Persistent augmented operands of a LoRA projection whose base W is frozen: W_aug = [W | s B] ([N, K + P]) and
    WT_aug = [W^T | s A^T] ([K, N + P]) hold W / W^T from construction; each call rewrites only the r LoRA columns
    (A and B train), instead of rebuilding the whole augmented matrices."""

    def __init__(self, W: torch.Tensor, P: int):
        N, K1 = W.shape
        dev = W.device
        self.P = P
        self.W_aug = torch.zeros(N, K1 + P, device=dev, dtype=BF16)
        self.W_aug[:, :K1] = W.detach().to(BF16)
        self.WT_aug = torch.zeros(K1, N + P, device=dev, dtype=BF16)
        K.transpose(self.W_aug[:, :K1], out=self.WT_aug[:, :N])
        self.A_pad = torch.zeros(P, K1, device=dev, dtype=BF16)
        self.BT = torch.zeros(P, N, device=dev, dtype=BF16)


def _aug_operands(owner, W: torch.Tensor, P: int) -> _AugOperands:
    key = (W.data_ptr(), W._version, tuple(W.shape), P)
    c = owner.__dict__.get("_vst_aug")
    if c is None or c[0] != key:
        c = (key, _AugOperands(W, P))
        owner.__dict__["_vst_aug"] = c
    return c[1]


class LoRALinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2d, W, b, A, B, s: float, owner=None):
        """owner: a module to hold the persistent augmented operands of a frozen W (None: rebuilt per call)."""
        if x2d.shape[1] % 64 or W.shape[0] % 64:
            raise ValueError("LoRALinearFn: in/out features must be multiples of 64 (two-source GEMM K split)")
        r = A.shape[0]
        P = pad32(max(r, 1))
        x2d = x2d.to(BF16).contiguous()
        N, K1 = W.shape
        if owner is not None and not W.requires_grad:
            aug = _aug_operands(owner, W, P)
        else:
            aug = _AugOperands(W, P)
        aug.A_pad[:r] = A.detach().to(BF16)
        aug.W_aug[:, K1:K1 + r] = (B.detach().float() * s).to(BF16)
        aug.WT_aug[:, N:N + r] = (A.detach().float().t() * s).to(BF16)
        aug.BT[:r] = B.detach().t().to(BF16)
        bias = None if b is None else b.detach().float().contiguous()
        u = K.linear(x2d, aug.A_pad, kind="gemm_lora_down", alg_n=r)
        y = K.linear(x2d, aug.W_aug, bias, x2=u, alg_k2=r)
        ctx.save_for_backward(x2d, W, A, B, u)
        ctx.aug = aug
        ctx.s = s
        ctx.b_dtype = None if b is None else b.dtype
        return y

    @staticmethod
    def backward(ctx, g):
        x2d, W, A, B, u = ctx.saved_tensors
        aug = ctx.aug
        s = ctx.s
        g = g.to(BF16).contiguous()
        r = A.shape[0]
        v = K.linear(g, aug.BT, kind="gemm_lora_down", alg_n=r)                # [M, P] = g B
        need_x, need_w, need_b, need_a, need_bb = ctx.needs_input_grad[:5]
        dX = dW = db = dA = dB = None
        if need_x:
            dX = K.linear(g, aug.WT_aug, x2=v, alg_k2=r)                         # [M, in]
        if need_w:
            dW = _tdot(g, x2d).to(W.dtype)                                       # [N, in] = g^T x
        if need_a:
            dA = (_tdot(v, x2d)[:r].float() * s).to(A.dtype)                    # [r, in] = s v^T x
        if need_bb:
            dB = (_tdot(g, u)[:, :r].float() * s).to(B.dtype)                   # [N, r] = s g^T u
        if need_b:
            db = K.colsum(g).to(ctx.b_dtype)                                     # [N] = g^T 1
        return dX, dW, db, dA, dB, None, None


class PlainLinearFn(torch.autograd.Function):
    """A trainable linear without LoRA (motion-module proj_in / proj_out / ff.net.2, animatediff/utils.py:79-85):
    y = x W^T + b; dX = g W (W^T cached per optimizer step), dW = g^T x, db = g^T 1."""

    @staticmethod
    def forward(ctx, x2d, W, b):
        from .unet_motion import f32
        x2d = x2d.to(BF16).contiguous()
        y = K.linear(x2d, W.detach().to(BF16).contiguous(), None if b is None else f32(b))
        ctx.save_for_backward(x2d, W)
        ctx.b_dtype = None if b is None else b.dtype
        return y

    @staticmethod
    def backward(ctx, g):
        x2d, W = ctx.saved_tensors
        g = g.to(BF16).contiguous()
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        dX = dW = db = None
        if need_x:
            dX = K.linear(g, _wt(W))
        if need_w:
            dW = _tdot(g, x2d).to(W.dtype)
        if need_b:
            db = K.colsum(g).to(ctx.b_dtype)
        return dX, dW, db


def _frozen_bwd_operands(ops):
    """(W_aug^T = [W^T | A^T] [K1, N + P] or W^T, V^T [P, N] or None) of a frozen projection's inference operands
    (lora_linear.ProjOps), cached on the ops object (which is itself rebuilt when a parameter version changes)."""
    c = ops.__dict__.get("_vst_bwd")
    if c is None:
        K1, N = ops.k1, ops.n
        W = ops.w[:, :K1]
        if ops.a is None:
            c = (K.transpose(W), None)
        else:
            P = ops.a.shape[0]
            wt = torch.empty(K1, N + P, device=W.device, dtype=BF16)
            K.transpose(W, out=wt[:, :N])
            K.transpose(ops.a, out=wt[:, N:])
            c = (wt, K.transpose(ops.w[:, K1:K1 + P]))
        ops.__dict__["_vst_bwd"] = c
    return c


class FrozenProjFn(torch.autograd.Function):
    """Projections whose parameters are all frozen (the Stage-2 spatial path with its UnZipLoRA layers, frozen conv
    shortcuts): forward = the inference operands ([x | x A^T] . [W | V]^T + b, lora_linear.build_ops, cached per
    parameter version), backward = dX = [g | g V] . [W^T | A^T]^T only, on cached transposed operands."""

    @staticmethod
    def forward(ctx, x2d, ops):
        from .lora_linear import run_ops
        x2d = x2d.to(BF16).contiguous()
        ctx.ops = ops
        return run_ops(x2d, ops)

    @staticmethod
    def backward(ctx, g):
        ops = ctx.ops
        g = g.to(BF16).contiguous()
        wt, vt = _frozen_bwd_operands(ops)
        if vt is None:
            return K.linear(g, wt), None
        v = K.linear(g, vt, kind="gemm_lora_down", alg_n=ops.r)
        return K.linear(g, wt, x2=v, alg_k2=ops.r), None


def lora_linear(x, W, b, A, B, s: float, owner=None):
    """y[..., out] = x W^T + b + s (x A^T) B^T with the HIP forward/backward (any leading shape); `owner` keeps the
    augmented operands of a frozen W across calls."""
    x2 = x.reshape(-1, x.shape[-1])
    y = LoRALinearFn.apply(x2, W, b, A, B, s, owner)
    return y.view(x.shape[:-1] + (W.shape[0],))


class LayerNormFn(torch.autograd.Function):
    """BasicTransformerBlock LayerNorm (unziplora_unet/unzip_attention.py:113-239; diffusers nn.LayerNorm) with the
    HIP forward (vst_layernorm) and backward (vst_layernorm_bwd: dx, dgamma, dbeta; statistics recomputed)."""

    @staticmethod
    def forward(ctx, x2d, gamma, beta, eps: float, pe=None, pe_div: int = 1, pe_mod: int = 1):
        """pe: optional [max_len, C] fp32 table added after the affine, row r gets pe[(r // pe_div) % pe_mod]
        (motion-module norm1/norm2 + sinusoidal PE); a constant, so the backward is unchanged."""
        x2d = x2d.to(BF16).contiguous()
        g32 = gamma.detach().float().contiguous()
        y = K.layer_norm(x2d, g32, beta.detach().float().contiguous(), eps, pe=pe, pe_div=pe_div, pe_mod=pe_mod)
        ctx.save_for_backward(x2d, gamma)
        ctx.eps = eps
        ctx.beta_dtype = beta.dtype
        return y

    @staticmethod
    def backward(ctx, g):
        x2d, gamma = ctx.saved_tensors
        affine = bool(ctx.needs_input_grad[1] or ctx.needs_input_grad[2])  # frozen spatial norms: dx only
        dx, dgam, dbet = K.layer_norm_bwd(x2d, g.to(BF16).contiguous(), gamma.detach().float().contiguous(), ctx.eps,
                                          need_affine=affine)
        if not affine:
            return dx, None, None, None, None, None, None
        return dx, dgam.to(gamma.dtype), dbet.to(ctx.beta_dtype), None, None, None, None


def _interleave32(t: torch.Tensor) -> torch.Tensor:
    """diffusers GEGLU proj rows [h; gate] -> the fused epilogue's [h_b (32) | gate_b (32)] blocks."""
    two_nh = t.shape[0]
    return t.reshape(2, two_nh // 64, 32, *t.shape[1:]).transpose(0, 1).reshape(t.shape)


def _deinterleave32(t: torch.Tensor) -> torch.Tensor:
    two_nh = t.shape[0]
    return t.reshape(two_nh // 64, 2, 32, *t.shape[1:]).transpose(0, 1).reshape(t.shape)


def _geglu_wt(geglu):
    """(interleaved GEGLU weight)^T, cached on the module per weight version while frozen."""
    w = geglu.proj.weight
    if w.requires_grad:
        return K.transpose(geglu.geglu_ops()[0])
    key = (w.data_ptr(), w._version)
    c = geglu.__dict__.get("_vst_geglu_wt")
    if c is None or c[0] != key:
        c = (key, K.transpose(geglu.geglu_ops()[0]))
        geglu.__dict__["_vst_geglu_wt"] = c
    return c[1]


class GEGLUFn(torch.autograd.Function):
    """diffusers GEGLU (proj = Linear(C, 2 Nh); out = h * gelu(gate)) of the motion / spatial FF: forward is the
    fused GEGLU GEMM on the module's interleaved operands (unet_motion.GEGLU.geglu_ops, cached per weight version);
    backward recomputes p = x W^T + b, then vst_geglu_bwd -> dp, dX = dp W (cached W^T), dW = dp^T x, db = dp^T 1,
    in the 32-interleaved column order (de-interleaved for the parameters)."""

    @staticmethod
    def forward(ctx, x2d, W, b, geglu):
        if W.shape[0] % 64 or x2d.shape[1] % 8:
            raise ValueError("GEGLUFn: 2*Nh must be a multiple of 64")
        x2d = x2d.to(BF16).contiguous()
        Wi, bi = geglu.geglu_ops()
        y = K.linear(x2d, Wi, bi, geglu=True)
        ctx.save_for_backward(x2d)
        ctx.geglu = geglu
        ctx.w_dtype, ctx.b_dtype = W.dtype, b.dtype
        return y

    @staticmethod
    def backward(ctx, g):
        (x2d,) = ctx.saved_tensors
        Wi, bi = ctx.geglu.geglu_ops()
        p = K.linear(x2d, Wi, bi)                                              # [M, 2Nh] pre-activation
        dp = K.geglu_bwd(p, g.to(BF16).contiguous())
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        dX = dW = db = None
        if need_x:
            dX = K.linear(dp, _geglu_wt(ctx.geglu))                            # [M, C] = dp W
        if need_w:
            dW = _deinterleave32(_tdot(dp, x2d)).to(ctx.w_dtype)
        if need_b:
            db = _deinterleave32(K.colsum(dp)).to(ctx.b_dtype)
        return dX, dW, db, None


class TemporalAttentionFn(torch.autograd.Function):
    """Motion-module attention core over the frame axis (the diffusers AnimateDiffTransformer3D attention as
    restated in animatediff/attention_processor.py; tokens [(b*F + f)*HW + p, C]).  Input: the fused q/k/v
    projection output [tokens, 3C]; its gradient comes back as one [tokens, 3C] buffer (vst_temporal_attention_bwd),
    which is what the fused projection's backward consumes."""

    @staticmethod
    def forward(ctx, qkv, nclip: int, F: int, HW: int, heads: int):
        qkv = qkv.to(BF16).contiguous()
        C = qkv.shape[1] // 3
        o = K.temporal_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], nclip, F, HW, heads, C // heads)
        ctx.save_for_backward(qkv)
        ctx.dims = (nclip, F, HW, heads)
        return o

    @staticmethod
    def backward(ctx, g):
        (qkv,) = ctx.saved_tensors
        nclip, F, HW, heads = ctx.dims
        C = qkv.shape[1] // 3
        dqkv = torch.empty_like(qkv)
        K.temporal_attention_bwd(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], g.to(BF16).contiguous(), nclip, F, HW,
                                 heads, C // heads, out=dqkv)
        return dqkv, None, None, None, None


class GroupNormFn(torch.autograd.Function):
    """GroupNorm (+SiLU) over `nsamples` groups of `rows_per_sample` token rows (the motion module's clip-wide GN:
    rows_per_sample = F*H*W, frames = F; per-frame GN: H*W) with the HIP forward (vst_groupnorm, or for a clip-wide
    GN the inference path's per-frame partials, vst_groupnorm_frame_partials / _apply_partials) and backward
    (vst_groupnorm_bwd)."""

    @staticmethod
    def forward(ctx, x2d, gamma, beta, nsamples: int, rows_per_sample: int, groups: int, eps: float, silu: bool,
                frames: int = 1):
        x2d = x2d.to(BF16).contiguous()
        g32, b32 = gamma.detach().float().contiguous(), beta.detach().float().contiguous()
        # (not taken: vst_groupnorm_bwd recomputes mean / rstd in its own chunking, so for the clip-wide
        # motion GroupNorm the backward's statistics can differ from these fp64-merged ones by fp32 ulps.  Moving the
        # forward to vst_groupnorm with the backward's statistics in its chunking was built and measured in round 5:
        # it moves single tiny-UNet gradients (tensors of a few hundred elements) by up to 2.5x their CPU bf16-autocast
        # yardstick error -- the gradients of this test are that sensitive to ulp-level changes -- while the
        # production-size gradients are unaffected; the inference path's bits are kept, profiles/r5_gn_bwd_stats.log.)
        if frames > 1 and not silu:
            hw = rows_per_sample // frames
            part = K.group_norm_frame_partials(x2d, nsamples * frames, hw, groups)
            y = K.group_norm_apply_partials(x2d, nsamples, frames, hw, groups, eps, g32, b32, part, 1)
        else:
            y = K.group_norm(x2d, nsamples, rows_per_sample, groups, eps, g32, b32, silu=silu)
        ctx.save_for_backward(x2d, gamma, beta)
        ctx.cfg = (nsamples, rows_per_sample, groups, eps, silu)
        return y

    @staticmethod
    def backward(ctx, g):
        x2d, gamma, beta = ctx.saved_tensors
        ns, rps, groups, eps, silu = ctx.cfg
        dx, dg, db = K.group_norm_bwd(x2d, g.to(BF16).contiguous(), ns, rps, groups, eps,
                                      gamma.detach().float().contiguous(), beta.detach().float().contiguous(), silu=silu)
        return dx, dg.to(gamma.dtype), db.to(beta.dtype), None, None, None, None, None, None



class AddFn(torch.autograd.Function):
    """Residual add on the HIP path (vst_add); the gradient passes to both operands."""

    @staticmethod
    def forward(ctx, a, b):
        return K.add(a.contiguous(), b.contiguous())

    @staticmethod
    def backward(ctx, g):
        return g, g


def _mergers_trainable(lora) -> bool:
    return any(getattr(lora, n, None) is not None and getattr(lora, n).requires_grad
               for n in ("merge_content", "merge_style"))


def _any_merger_trainable(lins) -> bool:
    return any(getattr(lin, "lora_layer", None) is not None and _mergers_trainable(lin.lora_layer) for lin in lins)


def _proj_parts(lins, scale: float = 1.0):
    """(W [sum out, in], b or None, A [sum r, in], B [sum out, sum r] with the LoRA scales folded in) of projections
    sharing one input, as autograd-tracked concatenations of the modules' own parameters.  Frozen UnZipLoRA layers
    (Stage 2 keeps the spatial LoRA frozen) contribute their low-rank factors (lowrank_factors(scale)) as constants."""
    from .temporal_lora import TemporalLoRALinear
    Ws, bs, As, Bs = [], [], [], []
    for lin in lins:
        base = lin.base if isinstance(lin, TemporalLoRALinear) else lin
        Ws.append(base.weight)
        bs.append(base.bias)
        lora = getattr(lin, "lora_layer", None)
        if isinstance(lin, TemporalLoRALinear):
            As.append(lin.lora_A)
            Bs.append(lin.lora_B * lin.scale)
        elif lora is not None:
            A, V = lora.lowrank_factors(scale)
            As.append(A.detach().float())
            # trainable mergers (--unfreeze_mergers, animatediff/utils.py:86-88): V = B * m stays on the autograd
            # graph, so LoRALinearFn's dB = s g^T u reaches merge_content / merge_style
            Bs.append(V.float() if _mergers_trainable(lora) else V.detach().float())
        else:
            As.append(base.weight.new_zeros(0, base.in_features, dtype=torch.float32))
            Bs.append(base.weight.new_zeros(base.out_features, 0, dtype=torch.float32))
    if len(Ws) == 1:
        W = Ws[0]
    elif any(w.requires_grad for w in Ws):
        W = torch.cat(Ws, 0)
    else:  # frozen bases (temporal LoRA q/k/v): concatenate once per weight version
        key = tuple((w.data_ptr(), w._version) for w in Ws)
        c = lins[0].__dict__.get("_vst_wcat")
        if c is None or c[0] != key:
            c = (key, torch.cat([w.detach() for w in Ws], 0))
            lins[0].__dict__["_vst_wcat"] = c
        W = c[1]
    b = None
    if any(x is not None for x in bs):
        b = torch.cat([x.float() if x is not None else torch.zeros(w.shape[0], device=w.device) for w, x in zip(Ws, bs)])
    A = torch.cat([a.float() for a in As], 0)
    B = torch.block_diag(*[bb.float() for bb in Bs])
    return W, b, A, B


def proj_train(lins, x2d, scale: float = 1.0):
    """Projections sharing the input x2d on the training path: all frozen -> FrozenProjFn (inference operands, dX
    only); one plain trainable linear -> PlainLinearFn; otherwise (temporal LoRA, trainable mergers) LoRALinearFn
    over the concatenated parameters, with the frozen base's augmented operands kept on lins[0]."""
    from .lora_linear import build_ops
    from .temporal_lora import TemporalLoRALinear
    if not any(p.requires_grad for lin in lins for p in lin.parameters()):
        return FrozenProjFn.apply(x2d, build_ops(lins, scale))
    if len(lins) == 1 and not isinstance(lins[0], TemporalLoRALinear) and getattr(lins[0], "lora_layer", None) is None:
        return PlainLinearFn.apply(x2d, lins[0].weight, lins[0].bias)
    W, b, A, B = _proj_parts(lins, scale)
    return LoRALinearFn.apply(x2d, W, b, A, B, 1.0, lins[0])


def transformer2d_train(t2d, x2d, nimg: int, H: int, W: int, enc=None, frames_per_text: int = 1, scale: float = 1.0):
    """Transformer2DModel of the frozen spatial path (unziplora_unet/transformer_2d.py:137-352; BasicTransformerBlock
    unzip_attention.py:113-239 with the UnZipLoRA delta on every q/k/v/out) on autograd Functions, so dL/dx flows
    back on HIP kernels: per-frame GroupNorm, proj_in, [LN -> fused q/k/v (+LoRA) -> self-attention -> to_out
    (+LoRA) + res; LN -> q (+LoRA) x text K/V -> cross-attention -> to_out + res; LN -> GEGLU -> ff.2 + res],
    proj_out + x.  enc: [nimg / frames_per_text * L, D] bf16 text states (constants: no gradient is taken)."""
    HW = H * W
    C = x2d.shape[1]
    h = GroupNormFn.apply(x2d, t2d.norm.weight, t2d.norm.bias, nimg, HW, t2d.norm.num_groups, t2d.norm.eps, False)
    h = proj_train([t2d.proj_in], h)
    for blk in t2d.transformer_blocks:
        a1, a2 = blk.attn1, blk.attn2
        n = LayerNormFn.apply(h, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps)
        qkv = proj_train([a1.to_q, a1.to_k, a1.to_v], n, scale)
        inner = qkv.shape[1] // 3
        o = SpatialAttentionFn.apply(qkv[:, :inner], qkv[:, inner:2 * inner], qkv[:, 2 * inner:], nimg, a1.heads, HW,
                                     HW, 1)
        h = AddFn.apply(h, proj_train([a1.to_out[0]], o, scale))
        n = LayerNormFn.apply(h, blk.norm2.weight, blk.norm2.bias, blk.norm2.eps)
        q = proj_train([a2.to_q], n, scale)
        L = enc.shape[0] // (nimg // frames_per_text)
        # text K/V are constants of the frozen path unless their UnZipLoRA mergers train
        with contextlib.nullcontext() if _any_merger_trainable([a2.to_k, a2.to_v]) else torch.no_grad():
            kv = proj_train([a2.to_k, a2.to_v], enc, scale)
        o = SpatialAttentionFn.apply(q, kv[:, :inner], kv[:, inner:], nimg, a2.heads, HW, L, frames_per_text)
        h = AddFn.apply(h, proj_train([a2.to_out[0]], o, scale))
        n = LayerNormFn.apply(h, blk.norm3.weight, blk.norm3.bias, blk.norm3.eps)
        f = GEGLUFn.apply(n, blk.ff.net[0].proj.weight, blk.ff.net[0].proj.bias, blk.ff.net[0])
        h = AddFn.apply(h, proj_train([blk.ff.net[2]], f))
    return AddFn.apply(x2d, proj_train([t2d.proj_out], h))


def motion_module_train(mm, x2d, nclip: int, F: int, HW: int):
    """Forward of a motion module (unet_motion.MotionModule = diffusers AnimateDiffTransformer3D) built from the
    autograd Functions above, so loss.backward() runs the whole module backward on HIP kernels: GroupNorm over the
    clip, proj_in, [LN+PE -> fused q/k/v (+temporal LoRA) -> frame-axis attention -> to_out (+LoRA) -> +res] x2,
    LN -> GEGLU -> ff.2 -> +res, proj_out -> +x.  Tokens [(b*F + f)*HW + p, C] bf16."""
    C = x2d.shape[1]
    h = GroupNormFn.apply(x2d, mm.norm.weight, mm.norm.bias, nclip, F * HW, mm.norm.num_groups, mm.norm.eps, False, F)
    h = proj_train([mm.proj_in], h)
    for blk in mm.transformer_blocks:
        pe = blk.pos_embed.pe.detach().float().reshape(-1, C).contiguous()
        for norm, attn in ((blk.norm1, blk.attn1), (blk.norm2, blk.attn2)):
            n = LayerNormFn.apply(h, norm.weight, norm.bias, norm.eps, pe, HW, F)
            qkv = proj_train([attn.to_q, attn.to_k, attn.to_v], n)
            o = TemporalAttentionFn.apply(qkv, nclip, F, HW, attn.heads)
            h = AddFn.apply(h, proj_train([attn.to_out[0]], o))
        n = LayerNormFn.apply(h, blk.norm3.weight, blk.norm3.bias, blk.norm3.eps)
        f = GEGLUFn.apply(n, blk.ff.net[0].proj.weight, blk.ff.net[0].proj.bias, blk.ff.net[0])
        h = AddFn.apply(h, proj_train([blk.ff.net[2]], f))
    return AddFn.apply(x2d, proj_train([mm.proj_out], h))


def _conv_dgrad_weight(conv):
    """Kernel-layout weight of the stride-1 3x3 conv's data gradient: W'[ci, co, ky, kx] = W[co, ci, 2-ky, 2-kx]
    (flipped taps, swapped channels), laid out [ci, (ky, kx, co)] like Conv3x3.kernel_weight; cached per version."""
    W = conv.weight
    key = (W.data_ptr(), W._version)
    c = conv.__dict__.get("_vst_wdgrad")
    if c is None or c[0] != key:
        wf = W.detach().flip(2, 3).transpose(0, 1)                      # [ci, co, 3, 3]
        ci, co = wf.shape[:2]
        w = wf.permute(0, 2, 3, 1).reshape(ci, 9 * co)
        kp = (9 * co + 7) & ~7
        if kp != 9 * co:
            w = torch.cat([w, w.new_zeros(ci, kp - 9 * co)], 1)
        c = (key, w.to(BF16).contiguous())
        conv.__dict__["_vst_wdgrad"] = c
    return c[1]


class Conv3x3Fn(torch.autograd.Function):
    """Frozen 3x3 conv of the spatial path (frozen in train_animatediff.py): forward = the implicit-GEMM conv
    (+ per-frame temb row bias, a constant here); backward dX = the same conv kernel on dY with flipped,
    channel-swapped weights — stride 1 directly; stride 2 (Downsample2D) on the zero-inserted dY; the
    nearest-2x-upsampled conv (Upsample2D) at the upsampled size followed by the 2x2 sum-pool adjoint."""

    @staticmethod
    def forward(ctx, x2d, conv, nimg: int, H: int, W: int, row_bias=None, row_bias_div: int = 1,
                upsample: bool = False):
        if conv.weight.requires_grad:
            raise NotImplementedError("Conv3x3Fn: frozen convs only (dgrad); dW is not on the training path")
        stride = conv.stride[0]
        if stride == 2 and (H % 2 or W % 2):
            raise NotImplementedError("Conv3x3Fn: stride-2 dgrad assumes even spatial sizes")
        x2d = x2d.to(BF16).contiguous()
        y = conv.run(x2d, nimg, H, W, upsample=upsample, row_bias=row_bias, row_bias_div=row_bias_div)
        ctx.conv, ctx.dims, ctx.mode = conv, (nimg, H, W), ("up" if upsample else stride)
        return y

    @staticmethod
    def backward(ctx, g):
        nimg, H, W = ctx.dims
        wd = _conv_dgrad_weight(ctx.conv)
        g = g.to(BF16).contiguous()
        if ctx.mode == 2:
            dx = K.conv3x3(K.zero_insert(g, nimg, H // 2, W // 2), nimg, H, W, wd, None)
        elif ctx.mode == "up":
            dx = K.sumpool2x2(K.conv3x3(g, nimg, 2 * H, 2 * W, wd, None), nimg, H, W)
        else:
            dx = K.conv3x3(g, nimg, H, W, wd, None)
        return dx, None, None, None, None, None, None, None


class CatFn(torch.autograd.Function):
    """Up-block skip concat [x | skip] on channels (the inference path reads the two sources in place; the training
    path materialises it once for the GroupNorm / conv / shortcut backward)."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.ca = a.shape[1]
        return torch.cat([a.to(BF16), b.to(BF16)], 1)

    @staticmethod
    def backward(ctx, g):
        return g[:, :ctx.ca].contiguous(), g[:, ctx.ca:].contiguous()


def _conv1x1_ops(sc):
    """ProjOps of a frozen 1x1 conv shortcut (kernel weight [Cout, Cin] bf16, fp32 bias), cached per version."""
    from .lora_linear import ProjOps
    from .unet_motion import f32
    if sc.weight.requires_grad:
        raise NotImplementedError("conv shortcut: frozen (spatial path) only")
    key = (sc.weight.data_ptr(), sc.weight._version, sc.bias.data_ptr(), sc.bias._version)
    c = sc.__dict__.get("_vst_train_ops")
    if c is None or c[0] != key:
        w = sc.kernel_weight()
        c = (key, ProjOps(w, None, f32(sc.bias), w.shape[1], w.shape[0], 0))
        sc.__dict__["_vst_train_ops"] = c
    return c[1]


def resnet_train(rb, x2d, nimg: int, H: int, W: int, temb_rows=None, rows_per_bias: int = 1):
    """ResnetBlock2D (frozen spatial path) forward on autograd Functions, so the gradient w.r.t. its input flows back
    on HIP kernels: GN+SiLU -> conv1 (+temb row bias) -> GN+SiLU -> conv2 -> + shortcut.
    temb_rows: fp32 [n, Cout] time-embedding projection rows (row r of the output adds temb_rows[r // rows_per_bias])."""
    HW = H * W
    h = GroupNormFn.apply(x2d, rb.norm1.weight, rb.norm1.bias, nimg, HW, rb.norm1.num_groups, rb.norm1.eps, True)
    h = Conv3x3Fn.apply(h, rb.conv1, nimg, H, W, temb_rows, rows_per_bias)
    h = GroupNormFn.apply(h, rb.norm2.weight, rb.norm2.bias, nimg, HW, rb.norm2.num_groups, rb.norm2.eps, True)
    h = Conv3x3Fn.apply(h, rb.conv2, nimg, H, W)
    if rb.conv_shortcut is not None:
        x2d = FrozenProjFn.apply(x2d, _conv1x1_ops(rb.conv_shortcut))
    return AddFn.apply(x2d, h)


class SpatialAttentionFn(torch.autograd.Function):
    """SDPA core of AnimateDiffAttnProcessor2_0 (animatediff/attention_processor.py:78-80), head_dim 64: forward =
    vst_spatial_attention (MFMA), backward = vst_spatial_attention_bwd.  q: [nbatch*Nq, C]; k, v: [nkv*Nk, C] with
    nkv = nbatch / kv_div (text K/V shared by the frames of a clip: their gradient sums over those frames)."""

    @staticmethod
    def forward(ctx, q, k, v, nbatch: int, heads: int, Nq: int, Nk: int, kv_div: int):
        q, k, v = (t.to(BF16).contiguous() for t in (q, k, v))
        lse = torch.empty(nbatch * heads * Nq, dtype=torch.float32, device=q.device)
        o = K.spatial_attention(q, k, v, nbatch, heads, Nq, Nk, kv_div, scale=0.125, lse=lse)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.dims = (nbatch, heads, Nq, Nk, kv_div)
        return o

    @staticmethod
    def backward(ctx, g):
        q, k, v, o, lse = ctx.saved_tensors
        nbatch, heads, Nq, Nk, kv_div = ctx.dims
        # frozen K/V (the cross-attention over text states of the frozen spatial path) skip the dK/dV pass
        need_dkv = bool(ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        dq, dk, dv = K.spatial_attention_bwd(q, k, v, o, g.to(BF16).contiguous(), lse, nbatch, heads, Nq, Nk, kv_div,
                                             scale=0.125, need_dkv=need_dkv)
        return dq, dk, dv, None, None, None, None, None


def unet_train_tokens(unet, x, B: int, F: int, h: int, w: int, emb_silu, enc2d, scale: float = 1.0):
    """UNetMotionModel.forward_tokens (unet_motion.py) on the autograd Functions: the training forward of
    train_animatediff.py:265-273 whose loss.backward() runs on HIP kernels end to end — frozen spatial path (convs,
    ResnetBlock2D, Transformer2DModel with UnZipLoRA) dX only, motion modules with their trainable parameters.
    x: [B*F*h*w, in] bf16 tokens of the noisy latents; emb_silu: SiLU(time + add embedding) [B, T] (constant);
    enc2d: [B*L, D] text states (constant)."""
    temb = unet.batched_temb(emb_silu)
    nimg = B * F
    H, W = h, w

    def res_block(res, t):
        return resnet_train(res, t, nimg, H, W, temb[res], F * H * W)

    x = Conv3x3Fn.apply(x, unet.conv_in, nimg, H, W)
    skips = [(x, H, W)]
    for blk in unet.down_blocks:
        for j, res in enumerate(blk.resnets):
            x = res_block(res, x)
            if blk.attentions is not None:
                x = transformer2d_train(blk.attentions[j], x, nimg, H, W, enc2d, F, scale)
            if blk.motion_modules is not None:
                x = motion_module_train(blk.motion_modules[j], x, B, F, H * W)
            skips.append((x, H, W))
        if blk.downsamplers is not None:
            x = Conv3x3Fn.apply(x, blk.downsamplers[0].conv, nimg, H, W)
            H, W = H // 2, W // 2
            skips.append((x, H, W))
    mid = unet.mid_block
    x = res_block(mid.resnets[0], x)
    x = transformer2d_train(mid.attentions[0], x, nimg, H, W, enc2d, F, scale)
    if mid.motion_modules is not None:
        x = motion_module_train(mid.motion_modules[0], x, B, F, H * W)
    x = res_block(mid.resnets[1], x)
    for blk in unet.up_blocks:
        for j, res in enumerate(blk.resnets):
            sk, sh, sw = skips.pop()
            assert (sh, sw) == (H, W)
            x = res_block(res, CatFn.apply(x, sk))
            if blk.attentions is not None:
                x = transformer2d_train(blk.attentions[j], x, nimg, H, W, enc2d, F, scale)
            if blk.motion_modules is not None:
                x = motion_module_train(blk.motion_modules[j], x, B, F, H * W)
        if blk.upsamplers is not None:
            x = Conv3x3Fn.apply(x, blk.upsamplers[0].conv, nimg, H, W, None, 1, True)
            H, W = 2 * H, 2 * W
    n = unet.conv_norm_out
    x = GroupNormFn.apply(x, n.weight, n.bias, nimg, H * W, n.num_groups, n.eps, True)
    return Conv3x3Fn.apply(x, unet.conv_out, nimg, H, W)
