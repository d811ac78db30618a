"""Tensor-level wrappers over the C ABI (libvst_hip.so).

Every function takes device tensors (bf16 activations/weights, fp32 bias/norm params), checks
shapes, and launches on torch's current HIP stream.  Activations are token-major 2-D views
[rows, C] (row stride may exceed C, e.g. a column slice of a fused QKV buffer).
No CPU fallback exists: a CPU tensor or a missing library raises.
"""
from __future__ import annotations

import os
import weakref

import torch

from . import _lib

BF16 = torch.bfloat16
F32 = torch.float32


def _stream():
    return torch.cuda.current_stream().cuda_stream


# ---- launch profiler (bench.py roofline): HIP events around every launch of an instrumented op
_PROF = None  # list of (kind, symbol, flops, bytes, ev_start, ev_end) while active


def profile_launches(active: bool):
    global _PROF
    _PROF = [] if active else None


def collect_launches():
    """[(kind, kernel symbol or None, flops, bytes, ms, shape)] for the launches recorded since
    profile_launches(True)."""
    torch.cuda.synchronize()
    out = [(k, y, f, b, s.elapsed_time(e), sh) for k, y, f, b, s, e, sh in (_PROF or [])]
    return out


class _Rec:
    __slots__ = ("kind", "flops", "nbytes", "s", "sym", "shape")

    def __init__(self, kind, flops, nbytes, sym=None, shape=None):
        self.kind, self.flops, self.nbytes = kind, flops, nbytes
        self.s = None
        self.sym = sym  # callable -> kernel symbol (evaluated only while profiling)
        self.shape = shape

    def __enter__(self):
        if _PROF is not None:
            self.s = torch.cuda.Event(enable_timing=True)
            self.s.record()
        return self

    def __exit__(self, *a):
        if _PROF is not None and self.s is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            _PROF.append((self.kind, self.sym() if self.sym else None, self.flops, self.nbytes, self.s, e,
                          self.shape))


GEMM_POLICY = {"tile": 0, "splits": 0}  # 0 = library heuristic (tuning / tests may force)
_ROW_INVARIANT = [0]


class row_invariant:
    """Inside: GEMMs and convs run without split-K (splits = 1 unless GEMM_POLICY forces a count), so every output
    row's bits depend on that row's inputs only, never on how many rows the launch has.  The denoise forward runs
    under it (UNetMotionModel.forward_tokens): a frame-sharded rank then computes exactly the unsharded forward's
    bits for its frames.  (Split-K only ever applied to grids under half a wave of tiles; the forward's token GEMMs
    at the step's shapes never split anyway.)"""

    def __enter__(self):
        _ROW_INVARIANT[0] += 1
        return self

    def __exit__(self, *a):
        _ROW_INVARIANT[0] -= 1


_FUSION_WORLD = [1]


class fusion_world:
    """Inside: shape-dependent fusion decisions are taken as a P-way frame-sharded rank takes them, so a forward here
    computes exactly the bits of a P-way sharded forward.  Two decisions depend on the pixels a rank holds (with the
    all-to-all exchange H*W/P of them): the motion attention fused into its q/k/v GEMM (vst_gemm_temporal_attention,
    default), which needs a multiple of 16 pixels, so an unsharded forward (or an all-gather rank, which holds all
    H*W) under fusion_world(P) fuses a layer only when (H*W) % (16 P) == 0; and the opt-in whole-block motion kernel
    (VST_MOTION_FUSE=1, unet_motion._fused_motion_ops_impl), which also asks vst_motion_attention_block_supported
    for H*W/P.  UNetMotionModel.forward_tokens enters it
    with the shard's world size (or its `fusion_world` argument); the all-to-all branch of MotionModule, whose
    pixels are already split, re-enters it with 1."""

    def __init__(self, world: int):
        if world < 1:
            raise ValueError(f"fusion_world({world})")
        self.world = int(world)

    def __enter__(self):
        self._prev = _FUSION_WORLD[0]
        _FUSION_WORLD[0] = self.world
        return self

    def __exit__(self, *a):
        _FUSION_WORLD[0] = self._prev


def fusion_pixel_div() -> int:
    """The P of the enclosing fusion_world (1 outside any)."""
    return _FUSION_WORLD[0]


def _splits():
    s = GEMM_POLICY["splits"]
    return s if s or not _ROW_INVARIANT[0] else 1


def gemm_kernel_name(M, N, K, kind):
    """Kernel the library launches for a GEMM / conv of this size (kind: 0 linear, 1 GEGLU, 2 conv,
    3 scalar-gather conv) under the current GEMM_POLICY."""
    name = _lib.load().vst_gemm_kernel_name(M, N, K, kind, GEMM_POLICY["tile"], _splits(), _WS_BYTES)
    return name.decode() if name else None
_WS = {}
_WS_BYTES = 80 << 20  # fp32 split-K slabs


def _workspace(device):
    """GEMM workspace per (device, stream) (allocated once, reused stream-ordered): the fp32 split-K slabs.  One per
    stream, so GEMMs queued on two streams never share slabs."""
    key = (device, _stream())
    ws = _WS.get(key)
    if ws is None:
        ws = torch.zeros(_WS_BYTES // 4, dtype=F32, device=device)
        _WS[key] = ws
    return ws


def _wrote(t):
    """A launch is about to write t through a raw pointer (which does not bump t._version): drop any GroupNorm column
    statistics registered for its storage (colstat_of), so they are never read for overwritten data."""
    if _COLSTAT and t is not None:
        _COLSTAT.pop(t.data_ptr(), None)


def _dev(t: torch.Tensor, dtype, name):
    if name == "out":
        _wrote(t)
    if not t.is_cuda:
        raise _lib.VstError(f"{name}: tensor is on {t.device}; the HIP path has no CPU fallback")
    if t.dtype != dtype:
        raise _lib.VstError(f"{name}: expected {dtype}, got {t.dtype}")
    if t.dim() != 2 or t.stride(1) != 1:
        raise _lib.VstError(f"{name}: expected a 2-D row-major view, got shape {tuple(t.shape)} stride {t.stride()}")
    return t


def _p(t):
    return None if t is None else t.data_ptr()


def _ld(t):
    return t.stride(0) if t.shape[0] > 1 else t.shape[1]


def linear(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, *, x2: torch.Tensor | None = None,
           residual: torch.Tensor | None = None, row_bias: torch.Tensor | None = None, row_bias_div: int = 1,
           out: torch.Tensor | None = None, geglu: bool = False, alg_k2: int | None = None,
           kind: str | None = None, alg_n: int | None = None, act: str | None = None) -> torch.Tensor:
    """out[M, N'] = epilogue([x | x2] @ w^T + bias + row_bias[m // div] + residual); N' = N or N/2 (GEGLU).
    act="gelu": GELU(erf) of (x @ w^T + bias) — no residual / row bias with it."""
    _dev(x, BF16, "x")
    _dev(w, BF16, "w")
    M, K1 = x.shape
    N, K = w.shape
    if x2 is not None:
        _dev(x2, BF16, "x2")
        if x2.shape[0] != M or K1 + x2.shape[1] != K:
            raise _lib.VstError(f"linear: x {tuple(x.shape)} + x2 {tuple(x2.shape)} vs w {tuple(w.shape)}")
    elif K1 != K:
        raise _lib.VstError(f"linear: x {tuple(x.shape)} vs w {tuple(w.shape)}")
    if act not in (None, "gelu") or (act and (geglu or residual is not None or row_bias is not None)):
        raise _lib.VstError(f"linear: act={act!r} supports only bias (no GEGLU / residual / row bias)")
    n_out = N // 2 if geglu else N
    if out is None:
        out = torch.empty((M, n_out), dtype=BF16, device=x.device)
    _dev(out, BF16, "out")
    if out.shape != (M, n_out):
        raise _lib.VstError(f"linear: out shape {tuple(out.shape)} != {(M, n_out)}")
    if bias is not None and (bias.dtype != F32 or bias.numel() != N or not bias.is_cuda):
        raise _lib.VstError("linear: bias must be fp32 [N] on device")
    if residual is not None:
        _dev(residual, BF16, "residual")
        if residual.shape != (M, n_out):
            raise _lib.VstError("linear: residual shape mismatch")
    if row_bias is not None:
        if row_bias.dtype != F32 or not row_bias.is_cuda or row_bias.shape[-1] != N:
            raise _lib.VstError("linear: row_bias must be fp32 [M/div, N]")
    # algorithmic work: the LoRA columns count only their real rank (alg_k2), not the zero padding
    k_alg = K1 + (0 if x2 is None else (x2.shape[1] if alg_k2 is None else alg_k2))
    kind = kind or ("gemm_geglu" if geglu else ("gemm_lora" if x2 is not None and alg_k2 is not None else "gemm"))
    n_alg = N if alg_n is None else alg_n
    with _Rec(kind, 2.0 * M * n_alg * k_alg, 2.0 * (M * k_alg + N * k_alg + M * n_out * (2 if residual is not None else 1)),
              lambda: gemm_kernel_name(M, N, K, 1 if geglu else 0), (M, N, K)):
        ws = _workspace(x.device)
        _lib.call("vst_gemm_ex", _p(x), _ld(x), _p(x2), 0 if x2 is None else _ld(x2), K1, _p(w), _ld(w), M, N, K,
                  _p(bias), _p(row_bias), row_bias_div, N if row_bias is not None else 0, _p(residual),
                  0 if residual is None else _ld(residual), _p(out), _ld(out), 1 if geglu else (2 if act else 0),
                  GEMM_POLICY["tile"], _splits(), _p(ws), _WS_BYTES, _stream())
    return out


def linear_tn(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """out[N, K] (bf16) = a^T b with a [M, N] and b [M, K] row-major over the M tokens (vst_gemm_tn): the weight
    gradients of the training backward (dW = g^T x, dA = s v^T x, dB = s g^T u) without transposed copies."""
    _dev(a, BF16, "a")
    _dev(b, BF16, "b")
    M, N = a.shape
    if b.shape[0] != M:
        raise _lib.VstError(f"linear_tn: a {tuple(a.shape)} and b {tuple(b.shape)} differ in tokens")
    K = b.shape[1]
    if out is None:
        out = torch.empty((N, K), dtype=BF16, device=a.device)
    _dev(out, BF16, "out")
    if out.shape != (N, K):
        raise _lib.VstError(f"linear_tn: out shape {tuple(out.shape)} != {(N, K)}")
    wsb = int(_lib.load().vst_gemm_tn_workspace_bytes(M, N, K))
    ws = torch.empty(max(wsb // 4, 1), dtype=F32, device=a.device) if wsb else None
    with _Rec("gemm_tn", 2.0 * M * N * K, 2.0 * (M * N + M * K + N * K), lambda: "gemm_tn", (N, K, M)):
        _lib.call("vst_gemm_tn", _p(a), _ld(a), _p(b), _ld(b), M, N, K, _p(out), _ld(out), _p(ws), wsb, _stream())
    return out


_LORA_BN = {}


class p8_conv:
    """Context manager routing 3x3 convs to the 8-phase kernel (on=True) or the ring kernel (vst_p8_conv); tests and
    A/B runs only."""

    def __init__(self, on=True):
        self.on = int(bool(on))

    def __enter__(self):
        self.prev = int(_lib.load().vst_p8_conv(self.on))
        return self

    def __exit__(self, *a):
        _lib.load().vst_p8_conv(self.prev)


class p8_persist:
    """Context manager switching the 8-phase GEMM's persistent grid on / off (vst_p8_persist) for the GEMMs launched
    inside it; tests and A/B runs only (the outputs are the same bits either way)."""

    def __init__(self, on=True):
        self.on = int(bool(on))

    def __enter__(self):
        self.prev = int(_lib.load().vst_p8_persist(self.on))
        return self

    def __exit__(self, *a):
        _lib.load().vst_p8_persist(self.prev)


class sa_self:
    """Context manager routing the long self-attention to sa_self_kernel (on=True, the default) or to the general
    spatial kernel (vst_sa_self); tests and A/B runs only (the outputs are the same bits either way)."""

    def __init__(self, on=True):
        self.on = int(bool(on))

    def __enter__(self):
        self.prev = int(_lib.load().vst_sa_self(self.on))
        return self

    def __exit__(self, *a):
        _lib.load().vst_sa_self(self.prev)


class p8_tile_width:
    """Context manager forcing the 8-phase GEMM's tile width (256 / 192 / 320 where legal; 0 = the library's
    policy) for the GEMMs launched inside it (vst_p8_force_bn); tests and A/B runs only."""

    def __init__(self, bn):
        self.bn = int(bn)

    def __enter__(self):
        self.prev = int(_lib.load().vst_p8_force_bn(self.bn))
        _LORA_BN.clear()
        _XATTN_OK.clear()
        return self

    def __exit__(self, *a):
        _lib.load().vst_p8_force_bn(self.prev)
        _LORA_BN.clear()
        _XATTN_OK.clear()


def gemm_lora_tile(M, N, K, P, group_n, group_r):
    """Tile width (256 / 192) of the in-GEMM LoRA projection (vst_gemm_lora) for this shape, 0 = not supported
    (the caller then runs the down-projection as its own pass).  Host-side policy only; no launch."""
    key = (M, N, K, P, group_n, group_r)
    bn = _LORA_BN.get(key)
    if bn is None:
        bn = _LORA_BN[key] = int(_lib.load().vst_gemm_lora_supported(M, N, K, P, group_n, group_r))
    return bn


def linear_lora(x: torch.Tensor, w: torch.Tensor, a: torch.Tensor, group_n: int, group_r: int,
                bias: torch.Tensor | None = None, *, residual: torch.Tensor | None = None,
                out: torch.Tensor | None = None, r_alg: int | None = None) -> torch.Tensor:
    """out = [x | bf16(x @ a^T)] @ w^T + bias (+ residual), the down-projection computed inside the GEMM
    (vst_gemm_lora).  w: [N, K + P] = [W | V], a: [P, K]; output columns n use u columns of group n // group_n."""
    _dev(x, BF16, "x")
    _dev(w, BF16, "w")
    _dev(a, BF16, "a")
    M, K = x.shape
    N = w.shape[0]
    P = a.shape[0]
    if a.shape[1] != K or w.shape[1] != K + P:
        raise _lib.VstError(f"linear_lora: x {tuple(x.shape)} a {tuple(a.shape)} w {tuple(w.shape)}")
    if out is None:
        out = torch.empty((M, N), dtype=BF16, device=x.device)
    _dev(out, BF16, "out")
    if out.shape != (M, N):
        raise _lib.VstError(f"linear_lora: out shape {tuple(out.shape)} != {(M, N)}")
    if bias is not None and (bias.dtype != F32 or bias.numel() != N or not bias.is_cuda):
        raise _lib.VstError("linear_lora: bias must be fp32 [N] on device")
    if residual is not None:
        _dev(residual, BF16, "residual")
        if residual.shape != (M, N):
            raise _lib.VstError("linear_lora: residual shape mismatch")
    bn = gemm_lora_tile(M, N, K, P, group_n, group_r)
    if not bn:
        raise _lib.VstError(f"linear_lora: shape M={M} N={N} K={K} P={P} groups ({group_n}, {group_r}) unsupported")
    r = P if r_alg is None else r_alg
    # algorithmic work: base + up-projection (as the unfused "gemm_lora" counts it) + the down-projection once
    flops = 2.0 * M * N * (K + r) + 2.0 * M * K * r
    nbytes = 2.0 * (M * K + N * (K + r) + r * K + M * N * (2 if residual is not None else 1))
    sym = f"gemm_p8<128x{bn},lora>" if bn == 320 else f"gemm_p8<256x{bn},lora>"
    with _Rec("gemm_lora", flops, nbytes, lambda: sym, (M, N, K + P)):
        _lib.call("vst_gemm_lora", _p(x), _ld(x), _p(a), _ld(a), P, group_n, group_r, _p(w), _ld(w), M, N, K,
                  _p(bias), _p(residual), 0 if residual is None else _ld(residual), _p(out), _ld(out), _stream())
    return out


_XATTN_OK = {}


def cross_attention_fusable(M, N, K, lora, P, group_n, group_r, Nq, Nk):
    """Whether vst_gemm_cross_attention runs attn2 (q projection + text cross-attention) as one launch for this shape
    (host policy only, no launch)."""
    key = (M, N, K, bool(lora), P, group_n, group_r, Nq, Nk)
    ok = _XATTN_OK.get(key)
    if ok is None:
        ok = _XATTN_OK[key] = bool(_lib.load().vst_gemm_cross_attention_supported(M, N, K, int(bool(lora)), P,
                                                                                   group_n, group_r, Nq, Nk))
    return ok


def linear_cross_attention(x: torch.Tensor, w: torch.Tensor, a: torch.Tensor | None, group_n: int, group_r: int,
                           bias: torch.Tensor | None, k: torch.Tensor, v: torch.Tensor, *, Nq: int, Nk: int,
                           kv_div: int, scale: float, out: torch.Tensor | None = None,
                           r_alg: int | None = None) -> torch.Tensor:
    """o = softmax(q_h k_h^T scale) v_h per head (head_dim 64) with q = [x | bf16(x a^T)] w^T + bias computed in the
    same launch (vst_gemm_cross_attention); k / v: [text_batches * Nk, N] views (row stride >= N), the text batch of
    frame f = (m // Nq) is f // kv_div."""
    _dev(x, BF16, "x")
    _dev(w, BF16, "w")
    _dev(k, BF16, "k")
    _dev(v, BF16, "v")
    M, K = x.shape
    N = w.shape[0]
    P = 0 if a is None else a.shape[0]
    if a is not None:
        _dev(a, BF16, "a")
        if a.shape[1] != K or w.shape[1] != K + P:
            raise _lib.VstError(f"linear_cross_attention: x {tuple(x.shape)} a {tuple(a.shape)} w {tuple(w.shape)}")
    elif w.shape[1] != K:
        raise _lib.VstError(f"linear_cross_attention: x {tuple(x.shape)} w {tuple(w.shape)}")
    if k.shape != v.shape or k.shape[1] != N or k.shape[0] % Nk or _ld(k) != _ld(v):
        raise _lib.VstError(f"linear_cross_attention: k {tuple(k.shape)} v {tuple(v.shape)} N={N} Nk={Nk}")
    if M % Nq or (M // Nq - 1) // kv_div >= k.shape[0] // Nk:
        raise _lib.VstError(f"linear_cross_attention: M={M} Nq={Nq} kv_div={kv_div} vs {k.shape[0] // Nk} text rows")
    if bias is not None and (bias.dtype != F32 or bias.numel() != N or not bias.is_cuda):
        raise _lib.VstError("linear_cross_attention: bias must be fp32 [N] on device")
    if not cross_attention_fusable(M, N, K, a is not None, P, group_n, group_r, Nq, Nk):
        raise _lib.VstError(f"linear_cross_attention: M={M} N={N} K={K} Nq={Nq} Nk={Nk} not fusable")
    if out is None:
        out = torch.empty((M, N), dtype=BF16, device=x.device)
    _dev(out, BF16, "out")
    if out.shape != (M, N):
        raise _lib.VstError(f"linear_cross_attention: out shape {tuple(out.shape)} != {(M, N)}")
    r = P if r_alg is None else r_alg
    flops = 2.0 * M * N * (K + r) + 2.0 * M * K * r + 4.0 * M * N * Nk
    nbytes = 2.0 * (M * K + N * (K + r) + r * K + 2 * (k.shape[0]) * N + M * N)
    sym = "gemm_p8<256x192,lora,xattn>" if a is not None else "gemm_p8<256x192,xattn>"
    with _Rec("gemm_xattn", flops, nbytes, lambda: sym, (M, N, K + P)):
        _lib.call("vst_gemm_cross_attention", _p(x), _ld(x), _p(a), 0 if a is None else _ld(a), P, group_n, group_r,
                  _p(w), _ld(w), _p(bias), M, N, K, _p(k), _p(v), _ld(k), k.shape[0], Nq, Nk, kv_div, float(scale),
                  _p(out), _ld(out), _stream())
    return out


_TATTN_OK = {}


def temporal_attention_fusable(M: int, K: int, nclip: int, F: int, HW: int, heads: int, head_dim: int) -> bool:
    """vst_gemm_temporal_attention_supported (host policy, cached): the motion modules' q/k/v + frame attention in one
    launch (16 frames, heads of 40)."""
    key = (M, K, nclip, F, HW, heads, head_dim)
    ok = _TATTN_OK.get(key)
    if ok is None:
        ok = _TATTN_OK[key] = bool(_lib.load().vst_gemm_temporal_attention_supported(*key))
    return ok


def temporal_qkv_layout(w: torch.Tensor, b: torch.Tensor | None, heads: int, head_dim: int):
    """The fused q/k/v weight [3C, K] (+ bias [3C]) re-laid out for vst_gemm_temporal_attention: per group of
    hpt = 256 // (3 head_dim) heads (2 of 40, 1 of 80) [q k v of each head] then zero rows up to 256.
    Returns (w_t bf16, b_t fp32)."""
    C = heads * head_dim
    hpt = 256 // (3 * head_dim)
    if w.shape[0] != 3 * C or hpt == 0 or heads % hpt:
        raise _lib.VstError(f"temporal_qkv_layout: w {tuple(w.shape)} heads={heads} head_dim={head_dim}")
    d = torch.arange(head_dim, device=w.device)
    rows, valid = [], []
    for t in range(heads // hpt):
        for h in range(hpt * t, hpt * t + hpt):
            for part in range(3):
                rows.append(part * C + h * head_dim + d)
        pad = 256 - 3 * hpt * head_dim
        rows.append(torch.zeros(pad, dtype=torch.long, device=w.device))
        valid.append(torch.cat([torch.ones(3 * hpt * head_dim, device=w.device), torch.zeros(pad, device=w.device)]))
    idx = torch.cat(rows)
    keep = torch.cat(valid)
    w_t = (w.detach().float()[idx] * keep[:, None]).to(BF16).contiguous()
    b_t = None if b is None else (b.detach().float()[idx] * keep).contiguous()
    return w_t, b_t


def linear_temporal_attention(x: torch.Tensor, w_t: torch.Tensor, b_t: torch.Tensor | None, *, nclip: int, F: int,
                              HW: int, heads: int, head_dim: int, scale: float,
                              out: torch.Tensor | None = None) -> torch.Tensor:
    """o = the motion modules' frame-axis attention of q/k/v = x w^T + b, in one launch (vst_gemm_temporal_attention);
    x: [nclip*F*HW, K] rows (clip, frame, pixel), w_t / b_t from temporal_qkv_layout.  Returns [M, heads*head_dim]."""
    _dev(x, BF16, "x")
    _dev(w_t, BF16, "w_t")
    M, K = x.shape
    N = heads // (256 // (3 * head_dim)) * 256
    if w_t.shape != (N, K):
        raise _lib.VstError(f"linear_temporal_attention: w_t {tuple(w_t.shape)} != {(N, K)}")
    if b_t is not None and (b_t.dtype != F32 or b_t.numel() != N or not b_t.is_cuda):
        raise _lib.VstError("linear_temporal_attention: b_t must be fp32 [N] on device")
    if not temporal_attention_fusable(M, K, nclip, F, HW, heads, head_dim):
        raise _lib.VstError(f"linear_temporal_attention: M={M} K={K} F={F} HW={HW} heads={heads} not fusable")
    C = heads * head_dim
    if out is None:
        out = torch.empty((M, C), dtype=BF16, device=x.device)
    _dev(out, BF16, "out")
    flops = 2.0 * M * 3 * C * K + 4.0 * M * F * C
    nbytes = 2.0 * (M * K + 3 * C * K + M * C)
    with _Rec("gemm_tattn", flops, nbytes, lambda: "gemm_p8<256x256,tattn>", (M, N, K)):
        _lib.call("vst_gemm_temporal_attention", _p(x), _ld(x), _p(w_t), _ld(w_t), _p(b_t), M, K, nclip, F, HW, heads,
                  head_dim, float(scale), _p(out), _ld(out), _stream())
    return out


# GroupNorm column statistics of conv outputs (vst_conv3x3_colstat -> vst_groupnorm_colstat): output data_ptr ->
# (weakref to the output, its version counter at the conv, colstat [ceil(M/128), Cout, 2] fp32).  Filled by
# conv3x3(colstat=True) and read by colstat_of(); an entry is valid only for the very tensor the conv wrote, not
# modified since (version), still alive (weakref).  colstat_reset() at the start of each UNet forward.
_COLSTAT: dict = {}


def colstat_enabled() -> bool:
    """VST_GN_COLSTAT=1: the UNet's GroupNorms take their statistics from column statistics (opt-in).  Measured in
    the denoise step (profiles/r5_ab_gn_colstat.txt): GroupNorm 2.22 -> 2.00 ms, the convs that write the statistics
    10.80 -> 10.92 ms (the epilogue's two extra barriers and row-group sums), net -0.08 ms per step, within the
    run-to-run spread; and every GroupNorm's statistics change bits (another summation order), which moved one
    configs[2] block's max-element error past its gate (1.76e-2 against 1.6e-2, rel_l2 unchanged)."""
    return os.environ.get("VST_GN_COLSTAT", "0") == "1"


def colstat_reset() -> None:
    _COLSTAT.clear()


def colstat_of(t: torch.Tensor | None):
    """The column statistics a conv3x3(colstat=True) registered for exactly this tensor, else None."""
    if t is None:
        return None
    e = _COLSTAT.get(t.data_ptr())
    if e is None:
        return None
    base = e[0]()
    if base is None or base.shape != t.shape or base.stride() != t.stride() or t._version != e[1]:
        return None
    return e[2]


def colstat(x: torch.Tensor) -> torch.Tensor:
    """Column statistics of x [M, C] in the conv epilogue's arithmetic (vst_colstat): [ceil(M/128), C, 2] fp32."""
    _dev(x, BF16, "x")
    M, C = x.shape
    cs = torch.empty(((M + 127) // 128, C, 2), dtype=F32, device=x.device)
    with _Rec("groupnorm", 0.0, 2.0 * M * C):
        _lib.call("vst_colstat", _p(x), _ld(x), M, C, _p(cs), _stream())
    return cs


def group_norm_stats(x1, x2=None):
    """(cs1, cs2) for group_norm(colstat=...): each source's column statistics from its producing conv when it wrote
    them (colstat_of), else from vst_colstat -- the same bits either way."""
    c1 = colstat_of(x1)
    c1 = colstat(x1) if c1 is None else c1
    if x2 is None:
        return c1, None
    c2 = colstat_of(x2)
    return c1, colstat(x2) if c2 is None else c2


def conv3x3(x1: torch.Tensor, nimg: int, H: int, W: int, w: torch.Tensor, bias: torch.Tensor | None, *,
            x2: torch.Tensor | None = None, stride: int = 1, upsample: bool = False,
            row_bias: torch.Tensor | None = None, row_bias_div: int = 1, residual: torch.Tensor | None = None,
            out: torch.Tensor | None = None, colstat: bool = False) -> torch.Tensor:
    """NHWC 3x3 conv (pad 1).  x1: [nimg*H*W, C1] (+ x2: [nimg*H*W, C2] concatenated on channels).
    w: [Cout, 9*(C1+C2)] laid out (ky, kx, ci).  Returns [nimg*OH*OW, Cout].
    colstat: also write the GroupNorm column statistics of the output where the 128x320 8-phase tiles run it
    (vst_conv3x3_colstat), registered for colstat_of(out)."""
    _dev(x1, BF16, "x1")
    C1 = x1.shape[1]
    C2 = 0
    if x2 is not None:
        _dev(x2, BF16, "x2")
        C2 = x2.shape[1]
    for t, c in ((x1, C1), (x2, C2)):
        if t is not None and (not t.is_contiguous() or t.shape[0] != nimg * H * W):
            raise _lib.VstError("conv3x3: inputs must be contiguous [nimg*H*W, C]")
    _dev(w, BF16, "w")
    Cout = w.shape[0]
    kreal = 9 * (C1 + C2)
    if w.shape[1] != ((kreal + 7) & ~7) and w.shape[1] != kreal:
        raise _lib.VstError(f"conv3x3: weight {tuple(w.shape)} vs K={kreal}")
    if upsample:
        OH, OW = 2 * H, 2 * W
    elif stride == 2:
        OH, OW = (H + 1) // 2, (W + 1) // 2
    else:
        OH, OW = H, W
    M = nimg * OH * OW
    if out is None:
        out = torch.empty((M, Cout), dtype=BF16, device=x1.device)
    _wrote(out)
    if bias is not None and (bias.dtype != F32 or bias.numel() != Cout):
        raise _lib.VstError("conv3x3: bias must be fp32 [Cout]")
    if residual is not None:
        _dev(residual, BF16, "residual")
    if row_bias is not None and (row_bias.dtype != F32 or not row_bias.is_cuda or row_bias.dim() != 2
                                 or row_bias.stride(1) != 1 or row_bias.shape[1] != Cout):
        raise _lib.VstError("conv3x3: row_bias must be an fp32 [nimg/div, Cout] device view with unit column stride")
    kind = "conv3x3" if (C1 + C2) % 64 == 0 else "conv3x3_small_cin"
    with _Rec(kind, 2.0 * M * Cout * kreal, 2.0 * (nimg * H * W * (C1 + C2) + Cout * kreal + M * Cout),
              lambda: gemm_kernel_name(M, Cout, w.shape[1], 2 if kind == "conv3x3" else 3), (M, Cout, w.shape[1])):
        if colstat and colstat_enabled() and Cout % 320 == 0 and out.is_contiguous() and GEMM_POLICY["tile"] == 0 \
                and _splits() <= 1:
            cs = torch.empty(((M + 127) // 128, Cout, 2), dtype=F32, device=x1.device)
            rc = _lib.load().vst_conv3x3_colstat(
                _p(x1), C1, _p(x2), C2, nimg, H, W, stride, 1 if upsample else 0, _p(w), Cout, _p(bias),
                _p(row_bias), row_bias_div, 0 if row_bias is None else _ld(row_bias), _p(residual),
                0 if residual is None else _ld(residual), _p(out), _ld(out), _p(cs), _stream())
            if rc == 0:
                _COLSTAT[out.data_ptr()] = (weakref.ref(out), out._version, cs)
                return out
            if rc != 3:
                raise _lib.VstError(f"vst_conv3x3_colstat failed with status {rc}")
        ws = _workspace(x1.device)
        _lib.call("vst_conv3x3_ex", _p(x1), C1, _p(x2), C2, nimg, H, W, stride, 1 if upsample else 0, _p(w), Cout,
                  _p(bias), _p(row_bias), row_bias_div, 0 if row_bias is None else _ld(row_bias), _p(residual), 0 if residual is None else _ld(residual),
                  _p(out), _ld(out) if Cout >= 8 else Cout, GEMM_POLICY["tile"], _splits(), _p(ws),
                  _WS_BYTES, _stream())
    return out


def spatial_attention(q, k, v, nbatch, heads, Nq, Nk, kv_div=1, out=None, scale=None, lse=None):
    """q: [nbatch*Nq, >=heads*64] view; k/v: [nbatch/kv_div*Nk, >=heads*64] views.  lse: optional fp32
    [nbatch*heads*Nq] output of the log2-domain logsumexp per query (the training backward recomputes P from it)."""
    for n, t in (("q", q), ("k", k), ("v", v)):
        _dev(t, BF16, n)
    if q.shape[0] != nbatch * Nq or k.shape[0] != (nbatch // kv_div) * Nk or v.shape[0] != k.shape[0]:
        raise _lib.VstError("spatial_attention: row counts do not match batch/Nq/Nk")
    if k.stride(0) != v.stride(0):
        raise _lib.VstError("spatial_attention: k and v must share a row stride")
    if out is None:
        out = torch.empty((nbatch * Nq, heads * 64), dtype=BF16, device=q.device)
    _dev(out, BF16, "out")
    if lse is not None and (lse.dtype != F32 or not lse.is_cuda or lse.numel() != nbatch * heads * Nq):
        raise _lib.VstError("spatial_attention: lse must be fp32 [nbatch*heads*Nq] on device")
    scale = 0.125 if scale is None else scale
    with _Rec("spatial_attention", 4.0 * nbatch * heads * Nq * Nk * 64,
              2.0 * 64 * heads * (2 * nbatch * Nq + 2 * (nbatch // kv_div) * Nk), None, (nbatch * heads, Nq, Nk)):
        _lib.call("vst_spatial_attention", _p(q), _ld(q), _p(k), _p(v), k.stride(0), _p(out), _ld(out), nbatch,
                  heads, Nq, Nk, kv_div, 64, float(scale), _p(lse), _stream())
    return out


def temporal_attention(q, k, v, nclip, F, HW, heads, head_dim, out=None, scale=None):
    """Frame-axis attention; rows (b*F + f)*HW + p.  q/k/v views share one row stride."""
    for n, t in (("q", q), ("k", k), ("v", v)):
        _dev(t, BF16, n)
    if not (q.stride(0) == k.stride(0) == v.stride(0)):
        raise _lib.VstError("temporal_attention: q/k/v must share a row stride")
    if q.shape[0] != nclip * F * HW:
        raise _lib.VstError("temporal_attention: rows != nclip*F*HW")
    if out is None:
        out = torch.empty((q.shape[0], heads * head_dim), dtype=BF16, device=q.device)
    _wrote(out)
    scale = head_dim ** -0.5 if scale is None else scale
    T = nclip * F * HW
    with _Rec("temporal_attention", 4.0 * T * F * heads * head_dim, 2.0 * 4 * T * heads * head_dim):
        _lib.call("vst_temporal_attention", _p(q), _p(k), _p(v), q.stride(0), _p(out), _ld(out), nclip, F, HW, heads,
                  head_dim, float(scale), _stream())
    return out


def motion_block_fusable(C, F, HW, heads):
    """vst_motion_attention_block takes this motion-module shape (host policy only)."""
    return bool(_lib.load().vst_motion_attention_block_supported(C, F, HW, heads))


def motion_attention_block(x, nclip, F, HW, heads, gamma, beta, eps, pe, wqkv, bqkv, wo, bo, *, scale=None, out=None):
    """y = x + (attention over the F frames of (LayerNorm(x) * gamma + beta + pe[frame]) . wqkv^T (+ bqkv)) . wo^T + bo
    in one launch; x: [nclip * F * HW, C] token rows (b * F + f) * HW + p."""
    _dev(x, BF16, "x")
    _dev(wqkv, BF16, "wqkv")
    _dev(wo, BF16, "wo")
    T, C = x.shape
    if T != nclip * F * HW or wqkv.shape != (3 * C, C) or wo.shape != (C, C):
        raise _lib.VstError(f"motion_attention_block: x {tuple(x.shape)} wqkv {tuple(wqkv.shape)} wo {tuple(wo.shape)}")
    for n, t, k in (("gamma", gamma, C), ("beta", beta, C), ("bqkv", bqkv, 3 * C), ("bo", bo, C)):
        if t is not None and (t.dtype != F32 or not t.is_cuda or t.numel() != k or not t.is_contiguous()):
            raise _lib.VstError(f"motion_attention_block: {n} must be fp32 [{k}] on device")
    if pe is not None and (pe.dtype != F32 or not pe.is_cuda or pe.shape[0] < F or pe.shape[-1] != C
                           or not pe.is_contiguous()):
        raise _lib.VstError("motion_attention_block: pe must be fp32 [>= F, C] on device")
    if any(t is not None and t.data_ptr() % 16 for t in (gamma, beta, pe)):
        raise _lib.VstError("motion_attention_block: gamma / beta / pe must be 16-byte aligned (vector loads)")
    if gamma is None or beta is None:
        raise _lib.VstError("motion_attention_block: gamma and beta are required")
    if out is None:
        out = torch.empty((T, C), dtype=BF16, device=x.device)
    _dev(out, BF16, "out")
    if out.shape != (T, C):
        raise _lib.VstError(f"motion_attention_block: out shape {tuple(out.shape)} != {(T, C)}")
    D = C // heads
    scale = D ** -0.5 if scale is None else scale
    flops = 2.0 * T * C * 4 * C + 4.0 * T * F * C
    with _Rec("motion_block", flops, 2.0 * (2 * T * C + 4 * C * C), lambda: "motion_attn_block_kernel", (T, 4 * C, C)):
        _lib.call("vst_motion_attention_block", _p(x), _ld(x), nclip, F, HW, C, heads, _p(gamma), _p(beta), float(eps),
                  _p(pe), _p(wqkv), _ld(wqkv), _p(bqkv), _p(wo), _ld(wo), _p(bo), float(scale), _p(out), _ld(out),
                  _stream())
    return out


def group_norm(x1, nsamples, rows_per_sample, groups, eps, gamma, beta, *, silu=False, x2=None, out=None,
               colstat=None):
    """colstat: (cs1, cs2 or None) column statistics of x1 / x2 from their producing convs (colstat_of):
    the statistics pass over x is skipped (vst_groupnorm_colstat)."""
    _dev(x1, BF16, "x1")
    C = x1.shape[1] + (0 if x2 is None else x2.shape[1])
    if x2 is not None:
        _dev(x2, BF16, "x2")
    if x1.shape[0] != nsamples * rows_per_sample:
        raise _lib.VstError("group_norm: rows != nsamples*rows_per_sample")
    if out is None:
        out = torch.empty((x1.shape[0], C), dtype=BF16, device=x1.device)
    _wrote(out)
    ws_bytes = _lib.load().vst_groupnorm_workspace_bytes(nsamples, rows_per_sample, groups, C)
    ws = torch.empty((ws_bytes + 3) // 4, dtype=F32, device=x1.device)
    if colstat is not None:
        cs1, cs2 = colstat
        for nm, cs, src in (("cs1", cs1, x1), ("cs2", cs2, x2)):
            if (cs is None) != (src is None):
                raise _lib.VstError(f"group_norm: {nm} must be given exactly when its source is")
            if cs is None:
                continue
            want = ((src.shape[0] + 127) // 128, src.shape[1], 2)
            if tuple(cs.shape) != want or cs.dtype != F32 or cs.device != src.device or not cs.is_contiguous():
                raise _lib.VstError(f"group_norm: {nm} must be contiguous fp32 {want} on {src.device}, got "
                                    f"{tuple(cs.shape)} {cs.dtype} on {cs.device}")
        with _Rec("groupnorm", 0.0, 2.0 * 2 * x1.shape[0] * C):  # one read + one write
            _lib.call("vst_groupnorm_colstat", _p(x1), _ld(x1), x1.shape[1], _p(cs1), _p(x2),
                      0 if x2 is None else _ld(x2), 0 if x2 is None else x2.shape[1], _p(cs2), nsamples,
                      rows_per_sample, groups, float(eps), _p(gamma), _p(beta), 1 if silu else 0, _p(out), _ld(out),
                      _p(ws), _stream())
        return out
    with _Rec("groupnorm", 0.0, 2.0 * 3 * x1.shape[0] * C):  # two reads + one write
        _lib.call("vst_groupnorm", _p(x1), _ld(x1), x1.shape[1], _p(x2), 0 if x2 is None else _ld(x2),
                  0 if x2 is None else x2.shape[1], nsamples, rows_per_sample, groups, float(eps), _p(gamma),
                  _p(beta), 1 if silu else 0, _p(out), _ld(out), _p(ws), _stream())
    return out


def group_norm_frame_partials(x, nframes, rows_per_frame, groups, *, out=None):
    """fp32 (sum, sumsq) chunk partials of every frame, [nframes, chunks, groups, 2] (vst_groupnorm_frame_partials):
    a frame's partials depend on that frame only, so the frame-sharded motion GroupNorm all-gathers them."""
    _dev(x, BF16, "x")
    C = x.shape[1]
    if x.shape[0] != nframes * rows_per_frame:
        raise _lib.VstError("group_norm_frame_partials: rows != nframes*rows_per_frame")
    nck = int(_lib.load().vst_groupnorm_frame_chunks(rows_per_frame))
    if out is None:
        out = torch.empty((nframes, nck, groups, 2), dtype=F32, device=x.device)
    if out.dtype != F32 or not out.is_cuda or not out.is_contiguous() or out.numel() != nframes * nck * groups * 2:
        raise _lib.VstError("group_norm_frame_partials: out must be contiguous fp32 [nframes, chunks, groups, 2]")
    with _Rec("groupnorm", 0.0, 2.0 * x.shape[0] * C):
        _lib.call("vst_groupnorm_frame_partials", _p(x), _ld(x), C, nframes, rows_per_frame, groups, _p(out),
                  _stream())
    return out


def group_norm_apply_partials(x, nclips, frames_local, rows_per_frame, groups, eps, gamma, beta, part, nranks, *,
                              silu=False, out=None):
    """GroupNorm of this rank's rows (clips x frames_local frames) with statistics over all nranks * frames_local
    frames of each clip, merged in one fixed order from `part` = [nranks, nclips, frames_local, chunks, groups, 2]
    (the all-gather of every rank's group_norm_frame_partials; nranks = 1: the whole clip is here)."""
    _dev(x, BF16, "x")
    C = x.shape[1]
    nck = int(_lib.load().vst_groupnorm_frame_chunks(rows_per_frame))
    if x.shape[0] != nclips * frames_local * rows_per_frame:
        raise _lib.VstError("group_norm_apply_partials: rows != nclips*frames_local*rows_per_frame")
    if part.dtype != F32 or not part.is_cuda or not part.is_contiguous() or \
            part.numel() != nranks * nclips * frames_local * nck * groups * 2:
        raise _lib.VstError("group_norm_apply_partials: part must be contiguous fp32 "
                            "[nranks, nclips, frames_local, chunks, groups, 2] on device")
    if out is None:
        out = torch.empty((x.shape[0], C), dtype=BF16, device=x.device)
    _dev(out, BF16, "out")
    ss = torch.empty(2 * nclips * C, dtype=F32, device=x.device)
    with _Rec("groupnorm", 0.0, 2.0 * 2 * x.shape[0] * C):
        _lib.call("vst_groupnorm_apply_partials", _p(x), _ld(x), C, nclips, frames_local, rows_per_frame, groups,
                  _p(part), nranks, float(eps), _p(gamma), _p(beta), 1 if silu else 0, _p(out), _ld(out), _p(ss),
                  _stream())
    return out


def permute_rows(src, dims, perm, out=None):
    """src rows indexed (i0,i1,i2,i3) over `dims`; returns rows in order (i_perm[0], .., i_perm[3])."""
    _dev(src, BF16, "src")
    if not src.is_contiguous() or src.shape[0] != dims[0] * dims[1] * dims[2] * dims[3]:
        raise _lib.VstError("permute_rows: src must be contiguous with prod(dims) rows")
    if out is None:
        out = torch.empty_like(src)
    _wrote(out)
    with _Rec("permute", 0.0, 2.0 * 2 * src.numel()):
        _lib.call("vst_permute_rows", _p(src), _p(out), src.shape[1], *dims, *perm, _stream())
    return out


def add_row_table(x, table, *, div=1, mod=1, out=None):
    """out[row] = x[row] + table[(row // div) % mod]; table fp32 [>= mod, C] on device."""
    _dev(x, BF16, "x")
    rows, C = x.shape
    if table.dtype != F32 or not table.is_cuda or table.dim() != 2 or table.shape[1] != C or table.shape[0] < mod:
        raise _lib.VstError("add_row_table: table must be fp32 [>= mod, C] on device")
    if out is None:
        out = torch.empty((rows, C), dtype=BF16, device=x.device)
    _wrote(out)
    with _Rec("add_row_table", 0.0, 2.0 * 2 * rows * C):
        _lib.call("vst_add_row_table", _p(x), _ld(x), C, rows, _p(table.contiguous()), div, mod, _p(out), _ld(out),
                  _stream())
    return out


def unpack_tokens(src, out):
    """bf16 token rows ((b*F + f)*HW + p, C) -> fp32 out (B, C, F, H, W) (contiguous)."""
    _dev(src, BF16, "src")
    if out.dtype != F32 or not out.is_cuda or not out.is_contiguous() or out.dim() != 5:
        raise _lib.VstError("unpack_tokens: out must be a contiguous fp32 (B, C, F, H, W) device tensor")
    B, C, F, H, W = out.shape
    if not src.is_contiguous() or src.shape != (B * F * H * W, C):
        raise _lib.VstError(f"unpack_tokens: src {tuple(src.shape)} vs out {tuple(out.shape)}")
    _lib.call("vst_unpack_tokens", _p(src), B, C, F, H * W, _p(out), _stream())
    return out


def layer_norm_lora(x, gamma, beta, eps, A, *, r_alg=None, out=None):
    """(LN(x), LN(x) @ A^T) in one pass; A: bf16 [R, C] (R % 16 == 0, <= 64) — LayerNorm + UnZipLoRA down."""
    _dev(x, BF16, "x")
    _dev(A, BF16, "A")
    rows, C = x.shape
    R = A.shape[0]
    if A.shape[1] != C or R % 16 or R > 64 or C % 32 or C > 1280 or not A.is_contiguous():
        raise _lib.VstError(f"layer_norm_lora: x {tuple(x.shape)} A {tuple(A.shape)}")
    if out is None:
        out = torch.empty((rows, C), dtype=BF16, device=x.device)
    _wrote(out)
    u = torch.empty((rows, R), dtype=BF16, device=x.device)
    with _Rec("layernorm_lora", 2.0 * rows * C * (r_alg or R), 2.0 * (2 * rows * C + rows * R)):
        _lib.call("vst_layernorm_lora", _p(x), _ld(x), C, rows, _p(gamma), _p(beta), float(eps), _p(A), R, _p(out),
                  _ld(out), _p(u), R, _stream())
    return out, u


def layer_norm(x, gamma, beta, eps=1e-5, *, pe=None, pe_div=1, pe_mod=1, out=None):
    _dev(x, BF16, "x")
    rows, C = x.shape
    if out is None:
        out = torch.empty((rows, C), dtype=BF16, device=x.device)
    _wrote(out)
    with _Rec("layernorm", 0.0, 2.0 * 2 * rows * C):
        _lib.call("vst_layernorm", _p(x), _ld(x), C, rows, _p(gamma), _p(beta), float(eps), _p(pe), pe_div, pe_mod,
                  _p(out), _ld(out), _stream())
    return out


def timestep_embedding(t, n, dim, out, *, col0=0, per_row=1, step_idx=None, flip=True, shift=0.0):
    """diffusers Timesteps(dim, flip_sin_to_cos, shift): value i -> out[i // per_row, col0 + (i % per_row)*dim]."""
    if t.dtype != F32 or not t.is_cuda:
        raise _lib.VstError("timestep_embedding: t must be fp32 on device")
    _lib.call("vst_timestep_embedding", _p(t), _p(step_idx), n, dim, 1 if flip else 0, float(shift), _p(out),
              _ld(out), col0, per_row, _stream())
    return out


def silu(x, out=None):
    out = torch.empty_like(x) if out is None else out
    _wrote(out)
    _lib.call("vst_silu", _p(x), _p(out), x.numel(), _stream())
    return out


def add(a, b, out=None):
    out = torch.empty_like(a) if out is None else out
    _wrote(out)
    _lib.call("vst_add", _p(a), _p(b), _p(out), a.numel(), _stream())
    return out


def transpose(x, out=None):
    """bf16 [rows, cols] (row-major view) -> [cols, rows]."""
    _dev(x, BF16, "x")
    rows, cols = x.shape
    if out is None:
        out = torch.empty((cols, rows), dtype=BF16, device=x.device)
    _wrote(out)
    with _Rec("transpose", 0.0, 2.0 * 2 * rows * cols):
        _lib.call("vst_transpose", _p(x), _ld(x), rows, cols, _p(out), _ld(out), _stream())
    return out


def layer_norm_bwd(x, g, gamma, eps=1e-5, need_affine=True):
    """LayerNorm backward: (dx bf16 [rows, C], dgamma fp32 [C], dbeta fp32 [C]); need_affine=False (frozen
    affine) computes dx only and returns (dx, None, None)."""
    _dev(x, BF16, "x")
    _dev(g, BF16, "g")
    rows, C = x.shape
    dx = torch.empty((rows, C), dtype=BF16, device=x.device)
    dgamma = dbeta = ws = None
    if need_affine:
        dgamma = torch.empty(C, dtype=F32, device=x.device)
        dbeta = torch.empty(C, dtype=F32, device=x.device)
        ws = torch.empty((_lib.load().vst_layernorm_bwd_workspace_bytes(C, rows) + 3) // 4, dtype=F32,
                         device=x.device)
    with _Rec("layernorm_bwd", 0.0, 2.0 * 3 * rows * C):
        _lib.call("vst_layernorm_bwd", _p(x), _ld(x), _p(g), _ld(g), C, rows, _p(gamma), float(eps), _p(dx), _ld(dx),
                  _p(dgamma), _p(dbeta), _p(ws), _stream())
    return dx, dgamma, dbeta


def group_norm_bwd(x, g, nsamples, rows_per_sample, groups, eps, gamma, beta, *, silu=False):
    """GroupNorm (+SiLU) backward: (dx bf16, dgamma fp32 [C], dbeta fp32 [C])."""
    _dev(x, BF16, "x")
    _dev(g, BF16, "g")
    rows, C = x.shape
    if rows != nsamples * rows_per_sample or g.shape != x.shape:
        raise _lib.VstError("group_norm_bwd: shapes")
    dx = torch.empty((rows, C), dtype=BF16, device=x.device)
    dgamma = torch.empty(C, dtype=F32, device=x.device)
    dbeta = torch.empty(C, dtype=F32, device=x.device)
    ws = torch.empty((_lib.load().vst_groupnorm_bwd_workspace_bytes(nsamples, rows_per_sample, groups, C) + 3) // 4,
                     dtype=F32, device=x.device)
    with _Rec("groupnorm_bwd", 0.0, 2.0 * 5 * rows * C):
        _lib.call("vst_groupnorm_bwd", _p(x), _ld(x), _p(g), _ld(g), C, nsamples, rows_per_sample, groups, float(eps),
                  _p(gamma), _p(beta), int(silu), _p(dx), _ld(dx), _p(dgamma), _p(dbeta), _p(ws), _stream())
    return dx, dgamma, dbeta


def colsum(x, out=None):
    """fp32 [N] column sums of a bf16 [M, N] row-major view (bias gradients), deterministic (vst_colsum).  The kernel
    reads 16-B chunks of 8 columns: a view whose width, row stride or base is not 8-column aligned is first copied
    into a zero-padded [M, ceil8(N)] buffer (the padding columns sum to zero and are dropped)."""
    _dev(x, BF16, "x")
    M, N = x.shape
    if out is None:
        out = torch.empty(N, dtype=F32, device=x.device)
    if N % 8 or _ld(x) % 8 or x.data_ptr() % 16:
        n8 = (N + 7) // 8 * 8
        xp = torch.zeros((M, n8), dtype=BF16, device=x.device)
        xp[:, :N].copy_(x)  # (stream-ordered scratch: no cached buffer, which a captured graph would alias)
        full = colsum(xp)
        out.copy_(full[:N])
        return out
    ws = torch.empty((_lib.load().vst_colsum_workspace_bytes(M, N) + 3) // 4, dtype=F32, device=x.device)
    with _Rec("colsum", 0.0, 2.0 * M * N):
        _lib.call("vst_colsum", _p(x), _ld(x), M, N, _p(out), _p(ws), _stream())
    return out


def geglu_bwd(p, g, out=None):
    """dp (32-interleaved like p) from p = the GEGLU projection output and g = dL/d(h * gelu(gate))."""
    _dev(p, BF16, "p")
    _dev(g, BF16, "g")
    M, Nh = g.shape
    if p.shape != (M, 2 * Nh):
        raise _lib.VstError(f"geglu_bwd: p {tuple(p.shape)} vs g {tuple(g.shape)}")
    if out is None:
        out = torch.empty((M, 2 * Nh), dtype=BF16, device=p.device)
    with _Rec("geglu_bwd", 0.0, 2.0 * 5 * M * Nh):
        _lib.call("vst_geglu_bwd", _p(p), _ld(p), _p(g), _ld(g), M, Nh, _p(out), _ld(out), _stream())
    return out


def spatial_attention_bwd(q, k, v, o, dout, lse, nbatch, heads, Nq, Nk, kv_div=1, scale=None, dq=None, dkv=None,
                          need_dkv=True):
    """(dq [nbatch*Nq, heads*64], dk, dv [nbatch/kv_div*Nk, heads*64] as column views of one [.., 2*heads*64], or
    None, None when need_dkv is False: frozen K/V skip the dK/dV kernel).  lse: the forward's logsumexp output."""
    for n, t in (("q", q), ("k", k), ("v", v), ("o", o), ("dout", dout)):
        _dev(t, BF16, n)
    if k.stride(0) != v.stride(0):
        raise _lib.VstError("spatial_attention_bwd: k and v must share a row stride")
    if lse.dtype != F32 or not lse.is_cuda or lse.numel() != nbatch * heads * Nq:
        raise _lib.VstError("spatial_attention_bwd: lse must be the forward's fp32 [nbatch*heads*Nq] logsumexp")
    C = heads * 64
    nkv = nbatch // kv_div
    if dq is None:
        dq = torch.empty((nbatch * Nq, C), dtype=BF16, device=q.device)
    if need_dkv and dkv is None:
        dkv = torch.empty((nkv * Nk, 2 * C), dtype=BF16, device=q.device)
    ws = torch.empty((_lib.load().vst_spatial_attention_bwd_workspace_bytes(nbatch, heads, Nq, Nk) + 3) // 4,
                     dtype=F32, device=q.device)
    scale = 0.125 if scale is None else scale
    # MFMA work: dQ pass 3 products (S, dP, dQ), dK/dV pass 4 (S, dP, dV, dK), 2*64 flop per (q, key) each
    with _Rec("spatial_attention_bwd", (6.0 + (8.0 if need_dkv else 0.0)) * nbatch * heads * Nq * Nk * 64, 0.0):
        _lib.call("vst_spatial_attention_bwd", _p(q), _ld(q), _p(k), _p(v), k.stride(0), _p(o), _ld(o), _p(dout),
                  _ld(dout), _p(lse), _p(dq), _ld(dq), _p(dkv[:, :C]) if need_dkv else None,
                  _p(dkv[:, C:]) if need_dkv else None, dkv.stride(0) if need_dkv else 0, nbatch, heads, Nq, Nk,
                  kv_div, 64, float(scale), _p(ws), _stream())
    if not need_dkv:
        return dq, None, None
    return dq, dkv[:, :C], dkv[:, C:]


def temporal_attention_bwd(q, k, v, dout, nclip, F, HW, heads, head_dim, scale=None, out=None):
    """(dq, dk, dv) of temporal_attention as column views of one [tokens, 3C] bf16 buffer."""
    for n, t in (("q", q), ("k", k), ("v", v), ("dout", dout)):
        _dev(t, BF16, n)
    if not (q.stride(0) == k.stride(0) == v.stride(0)):
        raise _lib.VstError("temporal_attention_bwd: q/k/v must share a row stride")
    C = heads * head_dim
    rows = nclip * F * HW
    if out is None:
        out = torch.empty((rows, 3 * C), dtype=BF16, device=q.device)
    scale = head_dim ** -0.5 if scale is None else scale
    with _Rec("temporal_attention_bwd", 0.0, 2.0 * 7 * rows * C):
        _lib.call("vst_temporal_attention_bwd", _p(q), _p(k), _p(v), q.stride(0), _p(dout), _ld(dout), _p(out[:, :C]),
                  _p(out[:, C:2 * C]), _p(out[:, 2 * C:]), out.stride(0), nclip, F, HW, heads, head_dim, float(scale),
                  _stream())
    return out[:, :C], out[:, C:2 * C], out[:, 2 * C:]


def zero_insert(x, nimg, h, w):
    """[nimg*h*w, C] -> [nimg*2h*2w, C] with x on the even (2i, 2j) pixels, zeros elsewhere."""
    _dev(x, BF16, "x")
    C = x.shape[1]
    out = torch.zeros((nimg * 4 * h * w, C), dtype=BF16, device=x.device)
    _lib.call("vst_zero_insert", _p(x), nimg, h, w, C, _p(out), _stream())
    return out


def sumpool2x2(x, nimg, h, w):
    """[nimg*2h*2w, C] -> [nimg*h*w, C], 2x2 block sums (h, w: output size)."""
    _dev(x, BF16, "x")
    C = x.shape[1]
    out = torch.empty((nimg * h * w, C), dtype=BF16, device=x.device)
    _lib.call("vst_sumpool2x2", _p(x), nimg, h, w, C, _p(out), _stream())
    return out


def copy2d(x, out):
    _lib.call("vst_copy2d", _p(x), _ld(x), _p(out), _ld(out), x.shape[0], x.shape[1], _stream())
    return out


def pack_latents(lat, out, *, sigmas=None, step_idx=None, fixed_scale=1.0, ncopy=1):
    B, Cl, F, H, W = lat.shape
    if lat.dtype != F32 or not lat.is_contiguous():
        raise _lib.VstError("pack_latents: latents must be contiguous fp32 (B,C,F,H,W)")
    _lib.call("vst_pack_latents", _p(lat), B, Cl, F, H * W, _p(sigmas), _p(step_idx), float(fixed_scale), ncopy,
              _p(out), _stream())
    return out


def euler_cfg_step(noise, lat, sigmas, step_idx, *, guidance=7.5, ncopy=2):
    B, Cl, F, H, W = lat.shape
    _lib.call("vst_euler_cfg_step", _p(noise), ncopy, float(guidance), _p(lat), B, Cl, F, H * W, _p(sigmas),
              _p(step_idx), _stream())


def step_advance(step_idx, num_steps):
    """step_idx <- (step_idx + 1) mod num_steps on the device (a schedule of num_steps steps)."""
    _lib.call("vst_step_advance", _p(step_idx), int(num_steps), _stream())


# ---- ceiling probes (bench.py: measured peaks next to the vendor figures) ----
def probe_mfma_tflops(device, grid=1024, iters=20000, reps=3):
    """Best-of-`reps` bf16 MFMA rate of vst_probe_mfma (16 independent 16x16x32 chains per wave)."""
    sink = torch.empty(grid, dtype=F32, device=device)
    flops = float(grid) * 8 * iters * 16 * 16384
    best = 0.0
    for _ in range(reps + 1):  # first launch warms the clocks
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        _lib.call("vst_probe_mfma", grid, iters, sink.data_ptr(), _stream())
        e.record()
        e.synchronize()
        best = max(best, flops / (s.elapsed_time(e) * 1e-3) / 1e12)
    return best


def probe_hbm_read_gbs(device, nbytes=4 << 30, grid=4096, reps=3):
    """Best-of-`reps` streaming read rate of vst_probe_hbm_read over an `nbytes` buffer (>> the 256 MB
    Infinity Cache, so it is HBM)."""
    buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
    sink = torch.empty(grid, dtype=torch.int32, device=device)
    best = 0.0
    for _ in range(reps + 1):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        _lib.call("vst_probe_hbm_read", buf.data_ptr(), nbytes, grid, sink.data_ptr(), _stream())
        e.record()
        e.synchronize()
        best = max(best, nbytes / (s.elapsed_time(e) * 1e-3) / 1e9)
    del buf
    return best


# ---- SDXL VAE (AutoencoderKL) pieces (vae.py) ----
def conv3x3_down_pad0(x: torch.Tensor, nimg: int, H: int, W: int, w: torch.Tensor, bias: torch.Tensor | None,
                      out: torch.Tensor | None = None) -> torch.Tensor:
    """diffusers Downsample2D(padding=0): F.pad(x, (0,1,0,1)) + 3x3 stride-2 conv, NHWC.  Returns
    [nimg*((H-2)//2+1)*((W-2)//2+1), Cout]."""
    _dev(x, BF16, "x")
    _dev(w, BF16, "w")
    C, Cout = x.shape[1], w.shape[0]
    if not x.is_contiguous() or x.shape[0] != nimg * H * W or w.shape[1] != 9 * C or C % 64:
        raise _lib.VstError("conv3x3_down_pad0: x [nimg*H*W, C] contiguous, C % 64 == 0, w [Cout, 9C]")
    OH, OW = (H - 2) // 2 + 1, (W - 2) // 2 + 1
    M = nimg * OH * OW
    if out is None:
        out = torch.empty((M, Cout), dtype=BF16, device=x.device)
    if bias is not None and (bias.dtype != F32 or bias.numel() != Cout):
        raise _lib.VstError("conv3x3_down_pad0: bias must be fp32 [Cout]")
    with _Rec("conv3x3", 2.0 * M * Cout * 9 * C, 2.0 * (nimg * H * W * C + Cout * 9 * C + M * Cout),
              lambda: gemm_kernel_name(M, Cout, 9 * C, 2), (M, Cout, 9 * C)):
        ws = _workspace(x.device)
        _lib.call("vst_conv3x3_down_pad0", _p(x), C, nimg, H, W, _p(w), Cout, _p(bias), _p(out), _ld(out), _p(ws),
                  _WS_BYTES, _stream())
    return out


def gemm_f32out(a: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """fp32 [M, N] = a[M, K] @ w[N, K]^T without rounding the accumulator."""
    _dev(a, BF16, "a")
    _dev(w, BF16, "w")
    M, K = a.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise _lib.VstError(f"gemm_f32out: a {tuple(a.shape)} vs w {tuple(w.shape)}")
    if out is None:
        out = torch.empty((M, N), dtype=F32, device=a.device)
    if out.dtype != F32 or not out.is_contiguous() or out.shape != (M, N):
        raise _lib.VstError("gemm_f32out: out must be contiguous fp32 [M, N]")
    with _Rec("gemm_f32out", 2.0 * M * N * K, 2.0 * (M * K + N * K) + 4.0 * M * N,
              lambda: gemm_kernel_name(M, N, K, 0), (M, N, K)):
        _lib.call("vst_gemm_f32out", _p(a), _ld(a), _p(w), _ld(w), M, N, K, _p(out), _stream())
    return out


def softmax_rows(s: torch.Tensor, scale: float, out: torch.Tensor | None = None) -> torch.Tensor:
    """bf16 softmax(scale * s) over the last dim of an fp32 [rows, n] matrix."""
    if not s.is_cuda or s.dtype != F32 or s.dim() != 2 or s.stride(1) != 1:
        raise _lib.VstError("softmax_rows: s must be an fp32 2-D row-major device view")
    rows, n = s.shape
    if out is None:
        out = torch.empty((rows, n), dtype=BF16, device=s.device)
    _dev(out, BF16, "out")
    with _Rec("softmax", 0.0, 4.0 * rows * n + 2.0 * rows * n):
        _lib.call("vst_softmax_rows", _p(s), _ld(s), rows, n, float(scale), _p(out), _ld(out), _stream())
    return out


def nchw_to_nhwc(x: torch.Tensor, mul: float = 1.0, ldd: int | None = None) -> torch.Tensor:
    """fp32 (n, C, H, W) -> bf16 [n*H*W, ldd] (channels >= C zero)."""
    if not x.is_cuda or x.dtype != F32 or x.dim() != 4 or not x.is_contiguous():
        raise _lib.VstError("nchw_to_nhwc: x must be a contiguous fp32 (n, C, H, W) device tensor")
    n, C, H, W = x.shape
    ldd = ldd or C
    if ldd < C:
        raise _lib.VstError(f"nchw_to_nhwc: ldd {ldd} < C {C}")
    out = torch.empty((n * H * W, ldd), dtype=BF16, device=x.device)
    _lib.call("vst_nchw_to_nhwc", _p(x), n, C, H * W, float(mul), _p(out), ldd, _stream())
    return out


def nhwc_to_nchw(x: torch.Tensor, n: int, C: int, H: int, W: int) -> torch.Tensor:
    """bf16 [n*H*W, >=C] -> fp32 (n, C, H, W)."""
    _dev(x, BF16, "x")
    if x.shape[0] != n * H * W or _ld(x) < C or x.shape[1] < C:
        raise _lib.VstError(f"nhwc_to_nchw: x {tuple(x.shape)} (ld {_ld(x)}) vs n*H*W = {n * H * W} rows of >= C channels")
    out = torch.empty((n, C, H, W), dtype=F32, device=x.device)
    _lib.call("vst_nhwc_to_nchw", _p(x), _ld(x), n, C, H * W, _p(out), _stream())
    return out


def frames_to_u8(x: torch.Tensor, n: int, C: int, H: int, W: int) -> torch.Tensor:
    """bf16 [n*H*W, >=C] decoder output -> uint8 (n, H, W, C) frames (inference_animatediff.py:141-143)."""
    _dev(x, BF16, "x")
    if x.shape[0] != n * H * W or _ld(x) < C or x.shape[1] < C:
        raise _lib.VstError(f"frames_to_u8: x {tuple(x.shape)} (ld {_ld(x)}) vs n*H*W = {n * H * W} rows of >= C channels")
    out = torch.empty((n, H, W, C), dtype=torch.uint8, device=x.device)
    _lib.call("vst_frames_to_u8", _p(x), _ld(x), n, C, H * W, _p(out), _stream())
    return out


def vae_sample(moments: torch.Tensor, n: int, H: int, W: int, eps: torch.Tensor | None, mul: float) -> torch.Tensor:
    """moments bf16 [n*H*W, >=8] -> fp32 (n, 4, H, W) = (mean + exp(logvar/2) * eps) * mul (eps None: mean * mul)."""
    _dev(moments, BF16, "moments")
    if moments.shape[0] != n * H * W or _ld(moments) < 8 or moments.shape[1] < 8:
        raise _lib.VstError(f"vae_sample: moments {tuple(moments.shape)} vs n*H*W = {n * H * W} rows of >= 8 "
                            "channels (mean | logvar)")
    if eps is not None and (eps.dtype != F32 or not eps.is_contiguous() or eps.shape != (n, 4, H, W)):
        raise _lib.VstError("vae_sample: eps must be contiguous fp32 (n, 4, H, W)")
    out = torch.empty((n, 4, H, W), dtype=F32, device=moments.device)
    _lib.call("vst_vae_sample", _p(moments), _ld(moments), n, H * W, _p(eps), float(mul), _p(out), _stream())
    return out
