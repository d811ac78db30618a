"""Kernel-level numerics: each HIP kernel vs a plain PyTorch fp32 reference of the same op.

Tolerance: bf16 inputs are exact on both sides; kernels accumulate in fp32 and round the
output once to bf16, so |err| <= ~1 bf16 ulp of the output (rel 2^-8) plus fp32 reassociation.
We assert max|err| / max|ref| <= 1e-2 and rel-L2 <= 5e-3 per op.
"""
import math

import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rnd(*shape, scale=1.0, gen=None):
    return (torch.randn(*shape, generator=gen) * scale).to(torch.bfloat16)


def check(out, ref, rel_l2=5e-3, rel_max=1e-2, name=""):
    out = out.float().cpu()
    ref = ref.float().cpu()
    assert out.shape == ref.shape, (name, out.shape, ref.shape)
    assert torch.isfinite(out).all(), name
    err = (out - ref)
    l2 = err.norm() / ref.norm().clamp_min(1e-12)
    mx = err.abs().max() / ref.abs().max().clamp_min(1e-12)
    assert l2 <= rel_l2 and mx <= rel_max, f"{name}: rel_l2={l2:.3e} rel_max={mx:.3e}"


@pytest.fixture(scope="module")
def K():
    from video_style_transfer_amd import kernels
    return kernels


@pytest.mark.parametrize("M,N,Kd", [(300, 200, 192), (1024, 640, 640), (4096, 1920, 640), (77, 1280, 2048), (2, 1280, 320)])
def test_gemm_bias_residual(cuda, K, M, N, Kd):
    g = torch.Generator().manual_seed(M + N + Kd)
    x, w = rnd(M, Kd, gen=g), rnd(N, Kd, scale=Kd ** -0.5, gen=g)
    b = torch.randn(N, generator=g)
    r = rnd(M, N, gen=g)
    out = K.linear(x.to(cuda), w.to(cuda), b.to(cuda), residual=r.to(cuda))
    ref = x.float() @ w.float().t() + b + r.float()
    check(out, ref, name="gemm")


@pytest.mark.parametrize("M,N,Kd,tile", [(8192, 32, 1280, 0), (32768, 64, 640, 0), (1030, 48, 640, 5),
                                         (2048, 16, 2048, 0), (100, 40, 96, 5), (4099, 64, 1344, 0)])
def test_gemm_skinny_lora_down(cuda, K, M, N, Kd, tile):
    g = torch.Generator().manual_seed(M + N)
    x, w = rnd(M, Kd, gen=g), rnd(N, Kd, scale=Kd ** -0.5, gen=g)
    K.GEMM_POLICY.update(tile=tile, splits=0)
    try:
        assert K.gemm_kernel_name(M, N, Kd, 0) == "gemm_skinny"
        out = K.linear(x.to(cuda), w.to(cuda), None, kind="gemm_lora_down")
    finally:
        K.GEMM_POLICY.update(tile=0, splits=0)
    check(out, x.float() @ w.float().t(), name="gemm_skinny")


@pytest.mark.parametrize("M,N,Kd,K2", [(4096, 1280, 1280, 32), (4000, 1200, 640, 0), (8192, 1280, 2048, 64)])
def test_gemm_underfilled_grids(cuda, K, M, N, Kd, K2):
    """Tile counts that leave CUs idle under 256x256 (160 tiles on 256 CUs: the policy takes the 8-phase kernel's
    256x192 tiles, 224 of them; 80 tiles: 128x128), and the same GEMMs forced onto the ring's 192x256 tile."""
    g = torch.Generator().manual_seed(M + N + Kd)
    x, x2 = rnd(M, Kd, gen=g), (rnd(M, K2, gen=g) if K2 else None)
    w = rnd(N, Kd + K2, scale=(Kd + K2) ** -0.5, gen=g)
    b = torch.randn(N, generator=g)
    rb = torch.randn(M // 1000 + 1, N, generator=g)
    r = rnd(M, N, gen=g)
    name = K.gemm_kernel_name(M, N, Kd + K2, 0)
    t256 = ((M + 255) // 256) * ((N + 255) // 256)
    assert ("256x192" if t256 >= 128 else "128x128") in name, name
    for tile in (0, 7, 0):  # policy tile, forced 192x256, policy again
        K.GEMM_POLICY.update(tile=tile, splits=0)
        try:
            out = K.linear(x.to(cuda), w.to(cuda), b.to(cuda), x2=None if x2 is None else x2.to(cuda),
                           row_bias=rb.to(cuda), row_bias_div=1000, residual=r.to(cuda))
        finally:
            K.GEMM_POLICY.update(tile=0, splits=0)
        xx = x if x2 is None else torch.cat([x, x2], 1)
        ref = xx.float() @ w.float().t() + b + rb.repeat_interleave(1000, 0)[:M] + r.float()
        check(out, ref, name=f"gemm {name} {M}x{N}x{Kd + K2}")


@pytest.mark.parametrize("M,N,K1,K2,geglu", [(8192, 1280, 1280, 32, False), (2000, 640, 320, 0, False),
                                             (4096, 2560, 640, 64, True), (1024, 320, 2048, 0, False),
                                             (8200, 1920, 1344, 0, False), (131072, 320, 320, 0, False)])
def test_gemm_8phase_bitwise_equals_ring(cuda, K, M, N, K1, K2, geglu):
    """The 8-phase kernel (gemm_p8.hip: 256x256 tile 8, 256x192 tile 9, 128x320 tile 10) accumulates every output
    over k in the same MFMA order as the ring kernel (tile 3, no split): identical bits, tails in M / N / K (LoRA
    columns) included."""
    g = torch.Generator().manual_seed(M + N + K1)
    x, x2 = rnd(M, K1, gen=g).to(cuda), (rnd(M, K2, gen=g).to(cuda) if K2 else None)
    w = rnd(N, K1 + K2, scale=(K1 + K2) ** -0.5, gen=g).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    r = None if geglu else rnd(M, N, gen=g).to(cuda)
    outs = []
    # tile 9: the 8-phase kernel at 256x192, tile 10 at 128x320 (no GEGLU; N a multiple of 320)
    for tile in ((3, 8) if geglu else (3, 8, 9) + ((10,) if N % 320 == 0 else ())):
        K.GEMM_POLICY.update(tile=tile, splits=1)
        try:
            outs.append(K.linear(x, w, b, x2=x2, residual=r, geglu=geglu))
        finally:
            K.GEMM_POLICY.update(tile=0, splits=0)
    for o in outs[1:]:
        assert torch.equal(outs[0], o)


@pytest.mark.parametrize("M,N,Kd,mode,bn", [
    (131072, 320, 320, "residual", 0), (131072, 320, 320, "residual", 320), (131072, 2560, 320, "geglu", 0),
    (8192, 10240, 1280, "geglu", 0), (32768, 640, 640, "rowbias", 0), (32868, 640, 640, "residual", 192),
    (32868, 1920, 640, "gelu", 0), (32768, 640, 2560, "residual", 320), (131072, 960, 320, "bias", 0),
    (65536, 1280, 128, "residual", 256)])
def test_gemm_8phase_persistent_bitwise(cuda, K, M, N, Kd, mode, bn):
    """The persistent grid of the 8-phase kernel (one workgroup per CU walking the tiles; each tile's last two
    k-tiles stream the next tile's first two, and the epilogue stages through the LDS past the ring) gives the same
    bits as one workgroup per tile: every epilogue (residual, row bias, GEGLU, GELU, bias only), every tile width,
    M tails (32868 = 128 x 256 + 100), K = 128 (the shortest stream)."""
    g = torch.Generator().manual_seed(M + N + Kd)
    x = rnd(M, Kd, gen=g).to(cuda)
    w = rnd(N, Kd, scale=Kd ** -0.5, gen=g).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    kw = {}
    if mode == "residual":
        kw["residual"] = rnd(M, N, gen=g).to(cuda)
    if mode == "rowbias":
        kw.update(row_bias=torch.randn(M // 4096, N, generator=g).to(cuda), row_bias_div=4096)
    if mode == "geglu":
        kw["geglu"] = True
    if mode == "gelu":
        kw["act"] = "gelu"
    outs = []
    with K.p8_tile_width(bn):
        for on in (False, True):
            with K.p8_persist(on):
                name = K.gemm_kernel_name(M, N, Kd, 1 if mode == "geglu" else 0)
                assert name.startswith("gemm_p8<") and name.endswith(",persist>") == on, name
                outs.append(K.linear(x, w, b, **kw))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]), f"{name}: {(outs[0].float() - outs[1].float()).abs().max().item()}"


@pytest.mark.parametrize("M,N,K1,K2,act", [(8192, 1280, 1280, 32, None), (32768, 640, 640, 32, None),
                                           (1000, 320, 192, 0, "gelu"), (8292, 3840, 1280, 64, None)])
def test_gemm_8phase_128x320_vs_torch(cuda, K, M, N, K1, K2, act):
    """The 128x320 tiles of the 8-phase kernel (tile 10: 4 x 2 waves of 64 x 80) against fp32 torch, with an M tail
    (8292 = 64 x 128 + 100), the two-source A (LoRA columns) and the GELU epilogue."""
    g = torch.Generator().manual_seed(M + N + 3)
    x, x2 = rnd(M, K1, gen=g).to(cuda), (rnd(M, K2, gen=g).to(cuda) if K2 else None)
    w = rnd(N, K1 + K2, scale=(K1 + K2) ** -0.5, gen=g).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    r = None if act else rnd(M, N, gen=g).to(cuda)
    K.GEMM_POLICY.update(tile=10, splits=1)
    try:
        assert K.gemm_kernel_name(M, N, K1 + K2, 0).startswith("gemm_p8<128x320")
        out = K.linear(x, w, b, x2=x2, residual=r, act=act)
    finally:
        K.GEMM_POLICY.update(tile=0, splits=0)
    xx = x.float() if x2 is None else torch.cat([x, x2], 1).float()
    ref = xx @ w.float().t() + b
    if act:
        ref = torch.nn.functional.gelu(ref)
    if r is not None:
        ref = ref.to(torch.bfloat16).float() + r.float()
    check(out, ref, name=f"gemm_p8<128x320> {M}x{N}x{K1 + K2}")


@pytest.mark.parametrize("M,N,K1,K2,act", [(8192, 1280, 1280, 32, None), (32768, 640, 640, 32, None),
                                           (131072, 320, 320, 0, None), (1000, 200, 192, 0, "gelu"),
                                           (4096, 576, 1344, 0, None)])
def test_gemm_8phase_256x192_vs_torch(cuda, K, M, N, K1, K2, act):
    """The 256x192 tiles of the 8-phase kernel, chosen automatically for N = 320 / 640 / 1280 on full grids
    (gemm.hip p8_bn192): against fp32 torch, with M / N tails (N = 200: a 192 + 8 split) and the GELU epilogue."""
    g = torch.Generator().manual_seed(M + N)
    x, x2 = rnd(M, K1, gen=g).to(cuda), (rnd(M, K2, gen=g).to(cuda) if K2 else None)
    w = rnd(N, K1 + K2, scale=(K1 + K2) ** -0.5, gen=g).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    r = None if act else rnd(M, N, gen=g).to(cuda)
    K.GEMM_POLICY.update(tile=9, splits=1)
    try:
        out = K.linear(x, w, b, x2=x2, residual=r, act=act)
    finally:
        K.GEMM_POLICY.update(tile=0, splits=0)
    xc = torch.cat([x, x2], 1) if K2 else x
    ref = xc.float() @ w.float().t() + b
    if act:
        ref = torch.nn.functional.gelu(ref)
    if r is not None:
        ref = ref.to(torch.bfloat16).float() + r.float()
    check(out, ref, name=f"gemm_p8<256x192> {M}x{N}x{K1 + K2}")
    if not act and M >= 8192:
        assert "256x192" in K.gemm_kernel_name(M, N, K1 + K2, 0), K.gemm_kernel_name(M, N, K1 + K2, 0)


def test_conv_underfilled_grid(cuda, K):
    g = torch.Generator().manual_seed(77)
    n, Ci, Co, H, W = 16, 320, 1280, 16, 16
    x = rnd(n, Ci, H, W, gen=g)
    w = rnd(Co, Ci, 3, 3, scale=(9 * Ci) ** -0.5, gen=g)
    b = torch.randn(Co, generator=g) * 0.1
    name = K.gemm_kernel_name(n * H * W, Co, 9 * Ci, 2)
    assert "128x128" in name, name  # 80 tiles of 256x256 -> 320 of 128x128
    out = K.conv3x3(to_nhwc(x).to(cuda), n, H, W, wflat(w).to(cuda), b.to(cuda))
    check(out, to_nhwc(conv_ref(x.float(), w.float(), b)), name=f"conv {name}")


@pytest.mark.parametrize("tile,splits", [(1, 1), (2, 1), (1, 3), (2, 5), (0, 0), (3, 1), (4, 1), (6, 1), (6, 3),
                                         (7, 1), (7, 2), (8, 1), (8, 0)])
@pytest.mark.parametrize("geglu", [False, True])
def test_gemm_tile_and_splitk_variants(cuda, K, tile, splits, geglu):
    g = torch.Generator().manual_seed(tile * 10 + splits)
    M, N, Kd, K2 = 300, 384, 640, 32
    x, x2 = rnd(M, Kd, gen=g), rnd(M, K2, gen=g)
    w = rnd(N, Kd + K2, scale=0.04, gen=g)
    b = torch.randn(N, generator=g)
    rb = torch.randn(M // 100, N, generator=g)
    r = rnd(M, N // 2 if geglu else N, gen=g)
    K.GEMM_POLICY.update(tile=tile, splits=splits)
    try:
        if geglu:
            out = K.linear(x.to(cuda), w.to(cuda), b.to(cuda), x2=x2.to(cuda), geglu=True)
        else:
            out = K.linear(x.to(cuda), w.to(cuda), b.to(cuda), x2=x2.to(cuda), row_bias=rb.to(cuda),
                           row_bias_div=100, residual=r.to(cuda))
    finally:
        K.GEMM_POLICY.update(tile=0, splits=0)
    y = torch.cat([x, x2], 1).float() @ w.float().t() + b
    if geglu:
        idx = torch.arange(N).view(-1, 64)
        h, gt = y[:, idx[:, :32].reshape(-1)], y[:, idx[:, 32:].reshape(-1)]
        ref = h * F.gelu(gt)
    else:
        ref = y + rb.repeat_interleave(100, 0) + r.float()
    check(out, ref, name=f"gemm t{tile} s{splits} geglu={geglu}")


@pytest.mark.parametrize("tile,splits", [(2, 1), (1, 4), (2, 3), (3, 1), (4, 1), (6, 1), (6, 2), (7, 1), (7, 3)])
def test_conv_tile_and_splitk_variants(cuda, K, tile, splits):
    g = torch.Generator().manual_seed(31 + splits)
    n, C1, C2, Co, H, W = 2, 128, 64, 192, 8, 8
    x1, x2 = rnd(n, C1, H, W, gen=g), rnd(n, C2, H, W, gen=g)
    w = rnd(Co, C1 + C2, 3, 3, scale=(9 * (C1 + C2)) ** -0.5, gen=g)
    b = torch.randn(Co, generator=g) * 0.1
    r = rnd(n, Co, H, W, gen=g)
    K.GEMM_POLICY.update(tile=tile, splits=splits)
    try:
        out = K.conv3x3(to_nhwc(x1).to(cuda), n, H, W, wflat(w).to(cuda), b.to(cuda), x2=to_nhwc(x2).to(cuda),
                        residual=to_nhwc(r).to(cuda))
    finally:
        K.GEMM_POLICY.update(tile=0, splits=0)
    ref = conv_ref(torch.cat([x1, x2], 1).float(), w.float(), b) + r.float()
    check(out, to_nhwc(ref), name=f"conv t{tile} s{splits}")


def test_gemm_two_source_and_rowbias(cuda, K):
    g = torch.Generator().manual_seed(7)
    M, K1, K2, N = 640, 640, 32, 384
    x, x2 = rnd(M, K1, gen=g), rnd(M, K2, gen=g)
    w = rnd(N, K1 + K2, scale=0.04, gen=g)
    rb = torch.randn(M // 64, N, generator=g)
    out = K.linear(x.to(cuda), w.to(cuda), None, x2=x2.to(cuda), row_bias=rb.to(cuda), row_bias_div=64)
    ref = torch.cat([x, x2], 1).float() @ w.float().t() + rb.repeat_interleave(64, 0)
    check(out, ref, name="gemm2src")


def test_gemm_strided_views(cuda, K):
    g = torch.Generator().manual_seed(8)
    big = rnd(512, 3 * 256, gen=g).to(cuda)
    x = big[:, 256:512]  # column view, ld = 768
    w = rnd(128, 256, scale=0.06, gen=g)
    out = torch.zeros(512, 3 * 128, dtype=torch.bfloat16, device=cuda)
    K.linear(x, w.to(cuda), None, out=out[:, 128:256])
    ref = x.float().cpu() @ w.float().t()
    check(out[:, 128:256], ref, name="gemm-views")
    assert out[:, :128].abs().max() == 0 and out[:, 256:].abs().max() == 0


def test_gemm_geglu(cuda, K):
    g = torch.Generator().manual_seed(9)
    M, C = 700, 128
    inner = 4 * C
    x = rnd(M, C, gen=g)
    w = rnd(2 * inner, C, scale=C ** -0.5, gen=g)
    b = torch.randn(2 * inner, generator=g) * 0.1
    # interleave rows: per 32-output block j: hidden rows [32j,32j+32) then gate rows [inner+32j, ...)
    idx = torch.cat([torch.cat([torch.arange(32 * j, 32 * j + 32), inner + torch.arange(32 * j, 32 * j + 32)])
                     for j in range(inner // 32)])
    out = K.linear(x.to(cuda), w[idx].contiguous().to(cuda), b[idx].contiguous().to(cuda), geglu=True)
    y = x.float() @ w.float().t() + b
    hdn, gate = y.chunk(2, dim=-1)
    ref = hdn * F.gelu(gate)
    check(out, ref, name="geglu")


def conv_ref(x_nchw, w, b, stride=1, up=False):
    if up:
        x_nchw = F.interpolate(x_nchw, scale_factor=2.0, mode="nearest")
    return F.conv2d(x_nchw, w, b, stride=stride, padding=1)


def to_nhwc(x):  # (N,C,H,W) -> [N*H*W, C]
    return x.permute(0, 2, 3, 1).reshape(-1, x.shape[1]).contiguous()


def wflat(w):  # (Cout,Cin,3,3) -> [Cout, 9*Cin] (ky,kx,ci), K padded to 8
    co, ci = w.shape[:2]
    f = w.permute(0, 2, 3, 1).reshape(co, 9 * ci)
    kp = (9 * ci + 7) & ~7
    if kp != 9 * ci:
        f = torch.cat([f, torch.zeros(co, kp - 9 * ci, dtype=f.dtype)], 1)
    return f.contiguous()


@pytest.mark.parametrize("n,Ci,Co,H,W,stride,up", [
    (2, 64, 128, 16, 16, 1, False), (3, 320, 320, 8, 8, 2, False), (2, 128, 64, 8, 8, 1, True),
    (2, 4, 320, 16, 16, 1, False), (2, 320, 4, 8, 8, 1, False), (1, 64, 64, 7, 5, 2, False)])
def test_conv3x3(cuda, K, n, Ci, Co, H, W, stride, up):
    g = torch.Generator().manual_seed(Ci * 7 + Co)
    x = rnd(n, Ci, H, W, gen=g)
    w = rnd(Co, Ci, 3, 3, scale=(9 * Ci) ** -0.5, gen=g)
    b = torch.randn(Co, generator=g) * 0.1
    out = K.conv3x3(to_nhwc(x).to(cuda), n, H, W, wflat(w).to(cuda), b.to(cuda), stride=stride, upsample=up)
    ref = conv_ref(x.float(), w.float(), b, stride, up)
    check(out, to_nhwc(ref), name="conv")


@pytest.mark.parametrize("n,C1,C2,Co,H,W,stride,up", [
    (8, 320, 0, 320, 64, 64, 1, False),     # 64x64 level, Cout 320: 128x320 tiles
    (16, 640, 320, 640, 32, 32, 1, False),  # up path: skip concat, Cout 640
    (16, 320, 0, 640, 64, 64, 2, False),    # downsample (stride 2)
    (16, 640, 0, 640, 16, 16, 1, True),     # upsample (nearest 2x)
    (32, 1280, 0, 1280, 16, 16, 1, False),  # 16x16 level, Cout 1280: 256-row tiles
])
def test_conv3x3_8phase_bitwise_equals_ring(cuda, K, n, C1, C2, Co, H, W, stride, up):
    """3x3 convs on the 8-phase kernel (vst_p8_conv: implicit im2col into its A slots, a (tap, channel) cursor per slot)
    against the ring kernel's conv bit for bit (same k order), and against fp32 torch; temb row bias and residual."""
    g = torch.Generator().manual_seed(n + C1 + Co + stride)
    x1 = rnd(n, C1, H, W, gen=g)
    x2 = rnd(n, C2, H, W, gen=g) if C2 else None
    Ci = C1 + C2
    w = rnd(Co, Ci, 3, 3, scale=(9 * Ci) ** -0.5, gen=g)
    b = torch.randn(Co, generator=g) * 0.1
    OH, OW = (2 * H, 2 * W) if up else ((H + 1) // 2, (W + 1) // 2) if stride == 2 else (H, W)
    temb = torch.randn(n, Co, generator=g)
    r = rnd(n, Co, OH, OW, gen=g)
    args = (to_nhwc(x1).to(cuda), n, H, W, wflat(w).to(cuda), b.to(cuda))
    kw = dict(x2=None if x2 is None else to_nhwc(x2).to(cuda), stride=stride, upsample=up, row_bias=temb.to(cuda),
              row_bias_div=OH * OW, residual=to_nhwc(r).to(cuda))
    ring = K.conv3x3(*args, **kw)
    with K.p8_conv(True):
        assert "gemm_p8" in K.gemm_kernel_name(n * OH * OW, Co, 9 * Ci, 2)
        p8 = K.conv3x3(*args, **kw)
    assert torch.equal(p8, ring)
    xx = x1.float() if x2 is None else torch.cat([x1, x2], 1).float()
    ref = conv_ref(xx, w.float(), b, stride, up).to(torch.bfloat16).float() + temb[:, :, None, None] + r.float()
    check(p8, to_nhwc(ref), name="conv p8")


@pytest.mark.parametrize("n,Ci,Co,H,W", [(2, 128, 128, 128, 128), (4, 512, 512, 64, 64), (2, 256, 128, 128, 128)])
def test_conv3x3_vae_ring128(cuda, K, n, Ci, Co, H, W):
    """The VAE's Cout = 128 / 512 convs that the 8-phase policy would put on 192-wide tiles run on the ring kernel's
    256x128 tiles (gemm.hip conv_ring128): the same bits as the 256x256 ring tiles, and fp32 torch's values."""
    g = torch.Generator().manual_seed(n + Ci + Co + H)
    x = rnd(n, Ci, H, W, gen=g)
    w = rnd(Co, Ci, 3, 3, scale=(9 * Ci) ** -0.5, gen=g)
    b = torch.randn(Co, generator=g) * 0.1
    args = (to_nhwc(x).to(cuda), n, H, W, wflat(w).to(cuda), b.to(cuda))
    assert K.gemm_kernel_name(n * H * W, Co, 9 * Ci, 2) == "gemm_ring<256x128,conv>"
    out = K.conv3x3(*args)
    K.GEMM_POLICY.update(tile=3, splits=1)
    try:
        ring256 = K.conv3x3(*args)
    finally:
        K.GEMM_POLICY.update(tile=0, splits=0)
    assert torch.equal(out, ring256)
    check(out, to_nhwc(conv_ref(x.float(), w.float(), b)), name="conv ring128")


@pytest.mark.parametrize("M,N,Kd", [(2, 1280, 320), (2, 1280, 2816), (2, 13760, 1280), (1, 8, 8), (3, 104, 40),
                                    (5, 640, 1288), (8, 336, 4096)])
@pytest.mark.parametrize("epi", ["bias", "residual", "gelu", "rowbias"])
def test_gemm_rows_small_m(cuda, K, M, N, Kd, epi):
    """gemm_rows_kernel (M <= 8: the time-embedding MLPs, the batched time_emb_proj) vs fp32, every epilogue."""
    g = torch.Generator().manual_seed(M * 1000 + N + Kd)
    x, w = rnd(M, Kd, gen=g), rnd(N, Kd, scale=Kd ** -0.5, gen=g)
    b = torch.randn(N, generator=g)
    y = x.float() @ w.float().t() + b
    assert K.gemm_kernel_name(M, N, Kd, 0) == "gemm_rows"
    if epi == "bias":
        out, ref = K.linear(x.to(cuda), w.to(cuda), b.to(cuda)), y
    elif epi == "gelu":
        out, ref = K.linear(x.to(cuda), w.to(cuda), b.to(cuda), act="gelu"), F.gelu(y)
    elif epi == "residual":
        r = rnd(M, N, gen=g)
        out = K.linear(x.to(cuda), w.to(cuda), b.to(cuda), residual=r.to(cuda))
        ref = y.to(torch.bfloat16).float() + r.float()
    else:
        rb = torch.randn(1, N, generator=g)
        out = K.linear(x.to(cuda), w.to(cuda), b.to(cuda), row_bias=rb.to(cuda), row_bias_div=8)
        ref = y.to(torch.bfloat16).float() + rb
    check(out, ref, name=f"gemm_rows {M}x{N}x{Kd} {epi}")


def test_gemm_rows_column_independent_of_n(cuda, K):
    """The batched time_emb_proj (one GEMM over every resnet's rows) equals each resnet's own Linear bit for bit."""
    g = torch.Generator().manual_seed(5)
    x = rnd(2, 1280, gen=g).to(cuda)
    w = rnd(13760, 1280, scale=1280 ** -0.5, gen=g).to(cuda)
    b = torch.randn(13760, generator=g).to(cuda)
    full = K.linear(x, w, b)
    o = 0
    for c in (320, 640, 1280, 960, 40):
        assert torch.equal(K.linear(x, w[o:o + c], b[o:o + c]), full[:, o:o + c]), (o, c)
        o += c


def test_conv3x3_concat_temb_residual(cuda, K):
    g = torch.Generator().manual_seed(11)
    n, C1, C2, Co, H, W = 4, 128, 64, 128, 8, 8
    x1, x2 = rnd(n, C1, H, W, gen=g), rnd(n, C2, H, W, gen=g)
    w = rnd(Co, C1 + C2, 3, 3, scale=(9 * (C1 + C2)) ** -0.5, gen=g)
    b = torch.randn(Co, generator=g) * 0.1
    temb = torch.randn(n, Co, generator=g)
    r = rnd(n, Co, H, W, gen=g)
    out = K.conv3x3(to_nhwc(x1).to(cuda), n, H, W, wflat(w).to(cuda), b.to(cuda), x2=to_nhwc(x2).to(cuda),
                    row_bias=temb.to(cuda), row_bias_div=H * W, residual=to_nhwc(r).to(cuda))
    ref = conv_ref(torch.cat([x1, x2], 1).float(), w.float(), b) + temb[:, :, None, None] + r.float()
    check(out, to_nhwc(ref), name="conv-cat")


@pytest.mark.parametrize("nb,heads,Nq,Nk,kv_div", [(4, 2, 256, 256, 1), (2, 3, 1024, 1024, 1), (8, 2, 100, 77, 4),
                                                   (2, 1, 64, 64, 1), (2, 2, 200, 300, 1), (4, 1, 50, 150, 2),
                                                   (1, 1, 130, 1, 1)])
@pytest.mark.parametrize("qs", [1.0, 3.0])
def test_spatial_attention(cuda, K, nb, heads, Nq, Nk, kv_div, qs):
    """qs scales q: logit std 1 (near-uniform softmax) and 3 (peaked: max tracking / tile rescale matter)."""
    g = torch.Generator().manual_seed(Nq + Nk + heads)
    C = heads * 64
    q = rnd(nb * Nq, C, scale=qs, gen=g)
    kv = rnd(nb // kv_div * Nk, 2 * C, gen=g)
    qd, kvd = q.to(cuda), kv.to(cuda)
    out = K.spatial_attention(qd, kvd[:, :C], kvd[:, C:], nb, heads, Nq, Nk, kv_div)
    qh = q.float().view(nb, Nq, heads, 64).transpose(1, 2)
    k = kv[:, :C].float().view(nb // kv_div, Nk, heads, 64).repeat_interleave(kv_div, 0).transpose(1, 2)
    v = kv[:, C:].float().view(nb // kv_div, Nk, heads, 64).repeat_interleave(kv_div, 0).transpose(1, 2)
    ref = torch.softmax(qh @ k.transpose(-1, -2) / 8.0, -1) @ v
    check(out, ref.transpose(1, 2).reshape(nb * Nq, C), name="sdpa")


@pytest.mark.parametrize("nb,heads,Nq,Nk", [(4, 2, 256, 256), (2, 3, 1024, 1024), (2, 2, 200, 300), (1, 1, 130, 130)])
@pytest.mark.parametrize("qs", [1.0, 3.0])
def test_sa_self_bitwise_equals_spatial_attn(cuda, K, nb, heads, Nq, Nk, qs):
    """The long self-attention kernel (sa_self_kernel, inference and the training forward) and the general spatial
    kernel compute the same bits -- output and logsumexp -- so inference and training run one forward arithmetic
    (VERDICT r5 weak #7)."""
    g = torch.Generator().manual_seed(Nq * 7 + Nk + heads)
    C = heads * 64
    q = rnd(nb * Nq, C, scale=qs, gen=g).to(cuda)
    kv = rnd(nb * Nk, 2 * C, gen=g).to(cuda)
    outs = {}
    for on in (1, 0):
        with K.sa_self(on):
            lse = torch.empty(nb * heads * Nq, dtype=torch.float32, device=cuda)
            o_inf = K.spatial_attention(q, kv[:, :C], kv[:, C:], nb, heads, Nq, Nk)
            o_tr = K.spatial_attention(q, kv[:, :C], kv[:, C:], nb, heads, Nq, Nk, lse=lse)
            outs[on] = (o_inf, o_tr, lse)
    assert torch.equal(outs[1][0], outs[0][0])
    assert torch.equal(outs[1][1], outs[0][1])
    assert torch.equal(outs[1][0], outs[1][1])
    assert torch.equal(outs[1][2], outs[0][2])


@pytest.mark.parametrize("nclip,Fr,HW,C", [(2, 16, 64, 320), (1, 32, 16, 640), (1, 16, 8, 1280), (1, 32, 4, 1280), (3, 5, 7, 64),
                                           (2, 16, 1, 128)])
@pytest.mark.parametrize("qs", [1.0, 3.0])
def test_temporal_attention(cuda, K, nclip, Fr, HW, C, qs):
    """qs scales q: logit std 1 and 3 (peaked softmax)."""
    g = torch.Generator().manual_seed(nclip * Fr + C)
    heads, d = 8, C // 8
    qkv = rnd(nclip * Fr * HW, 3 * C, gen=g)
    qkv[:, :C] = (qkv[:, :C].float() * qs).to(torch.bfloat16)
    qd = qkv.to(cuda)
    out = K.temporal_attention(qd[:, :C], qd[:, C:2 * C], qd[:, 2 * C:], nclip, Fr, HW, heads, d)

    def seq(t):  # rows (b*F+f)*HW+p -> (b*HW+p, heads, F, d)
        return t.float().view(nclip, Fr, HW, heads, d).permute(0, 2, 3, 1, 4).reshape(nclip * HW, heads, Fr, d)

    q, k, v = seq(qkv[:, :C]), seq(qkv[:, C:2 * C]), seq(qkv[:, 2 * C:])
    o = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(d), -1) @ v
    ref = o.view(nclip, HW, heads, Fr, d).permute(0, 3, 1, 2, 4).reshape(nclip * Fr * HW, C)
    check(out, ref, name="temporal")


@pytest.mark.parametrize("nclip,HW,d,bias,ws", [(2, 4096, 40, False, 1.0), (1, 256, 40, True, 1.0),
                                             (2, 512, 40, True, 3.0), (3, 1024, 40, False, 2.0),
                                             (2, 1024, 80, False, 1.0), (1, 512, 80, True, 3.0)])
def test_gemm_temporal_attention(cuda, K, nclip, HW, d, bias, ws):
    """The motion modules' q/k/v projection with the frame-axis attention as its epilogue (vst_gemm_temporal_attention,
    16 frames, 8 heads of 40 (K = 320, the 64^2 level) or 80 (K = 640, 32^2)) against the two-launch path (q/k/v GEMM
    + vst_temporal_attention) and against fp32 torch on the bf16-rounded q/k/v; ws scales the weights (ws = 3: logit
    std ~3, a peaked softmax)."""
    g = torch.Generator().manual_seed(nclip * HW + int(ws) + d)
    Fr, heads = 16, 8
    C = heads * d
    M = nclip * Fr * HW
    x = rnd(M, C, gen=g)
    w = rnd(3 * C, C, scale=ws * C ** -0.5, gen=g)
    b = (torch.randn(3 * C, generator=g) * 0.1) if bias else None
    xd, wd, bd = x.to(cuda), w.to(cuda), None if b is None else b.to(cuda)
    assert K.temporal_attention_fusable(M, C, nclip, Fr, HW, heads, d)
    w_t, b_t = K.temporal_qkv_layout(wd, None if bd is None else bd.float(), heads, d)
    fused = K.linear_temporal_attention(xd, w_t, b_t, nclip=nclip, F=Fr, HW=HW, heads=heads, head_dim=d,
                                        scale=d ** -0.5)
    qkv = K.linear(xd, wd, bd)
    two = K.temporal_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], nclip, Fr, HW, heads, d)
    check(fused, two.float(), rel_l2=2e-3, rel_max=1e-2, name="tattn fused vs two launches")
    qf = (x.float() @ w.float().t() + (0 if b is None else b)).to(torch.bfloat16).float()

    def seq(t):  # rows (b*F+f)*HW+p -> (b*HW+p, heads, F, d)
        return t.view(nclip, Fr, HW, heads, d).permute(0, 2, 3, 1, 4).reshape(nclip * HW, heads, Fr, d)

    q, k, v = seq(qf[:, :C]), seq(qf[:, C:2 * C]), seq(qf[:, 2 * C:])
    o = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(d), -1) @ v
    ref = o.view(nclip, HW, heads, Fr, d).permute(0, 3, 1, 2, 4).reshape(M, C)
    check(fused, ref, name="tattn fused vs fp32")


def test_gemm_temporal_attention_refuses(cuda, K):
    """Outside the fused kernel's contract the policy says no (the processor then takes the two launches)."""
    assert not K.temporal_attention_fusable(2 * 16 * 4096, 320, 2, 32, 4096, 8, 40)   # 32 frames
    assert not K.temporal_attention_fusable(2 * 16 * 256, 1280, 2, 16, 256, 8, 160)   # heads of 160 (16^2)
    assert not K.temporal_attention_fusable(2 * 16 * 100, 320, 2, 16, 100, 8, 40)     # HW % 16
    assert K.temporal_attention_fusable(2 * 16 * 4096, 320, 2, 16, 4096, 8, 40)       # the 64^2 level
    assert K.temporal_attention_fusable(2 * 16 * 1024, 640, 2, 16, 1024, 8, 80)       # the 32^2 level


@pytest.mark.parametrize("ns,rps,C1,C2,silu", [(4, 64, 320, 0, True), (2, 1000, 640, 0, False),
                                               (3, 64, 128, 64, True), (1, 16 * 256, 1280, 0, False),
                                               (32, 256, 1280, 1280, True), (5, 77, 640, 320, True),
                                               (2, 9, 64, 0, False), (3, 700, 4096, 0, False)])
def test_group_norm(cuda, K, ns, rps, C1, C2, silu):
    g = torch.Generator().manual_seed(ns * rps + C1)
    x1 = rnd(ns * rps, C1, gen=g) + 0.5
    x2 = rnd(ns * rps, C2, gen=g) if C2 else None
    C = C1 + C2
    gam, bet = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.1
    out = K.group_norm(x1.to(cuda), ns, rps, 32, 1e-5, gam.to(cuda), bet.to(cuda), silu=silu,
                       x2=None if x2 is None else x2.to(cuda))
    x = x1.float() if x2 is None else torch.cat([x1, x2], 1).float()
    xs = x.view(ns, rps, C).permute(0, 2, 1)  # (N, C, L)
    ref = F.group_norm(xs, 32, gam, bet, 1e-5).permute(0, 2, 1).reshape(ns * rps, C)
    if silu:
        ref = F.silu(ref)
    check(out, ref, name="groupnorm")


def test_conv_colstat_groupnorm(cuda, K, monkeypatch):
    """GroupNorm statistics from the producing convs' epilogues (vst_conv3x3_colstat -> vst_groupnorm_colstat):
    the conv output is the same bits with or without the statistics; the column statistics equal fp64 sums of the
    stored bf16 output per 128-row tile and vst_colstat's bit for bit; the GroupNorm over [x1 | x2] (an up block's
    concat, groups straddling the seam) matches the statistics-pass GroupNorm to within one bf16 rounding and torch
    fp32."""
    monkeypatch.setenv("VST_GN_COLSTAT", "1")  # (opt-in in the step)
    g = torch.Generator().manual_seed(5)
    n, H, W = 32, 32, 32  # 32768 rows: the 8-phase 128x320 conv path
    outs, stats = [], []
    xin = rnd(n * H * W, 320, gen=g).to(cuda)
    r = rnd(n * H * W, 640, gen=g).to(cuda)
    for Co, res in ((640, r), (320, None)):
        w = rnd(Co, 320, 3, 3, scale=(9 * 320) ** -0.5, gen=g)
        b = torch.randn(Co, generator=g) * 0.1
        wd, bd = wflat(w).to(cuda), b.to(cuda)
        plain = K.conv3x3(xin, n, H, W, wd, bd, residual=res)
        y = K.conv3x3(xin, n, H, W, wd, bd, residual=res, colstat=True)
        assert torch.equal(y, plain), Co
        cs = K.colstat_of(y)
        assert cs is not None and cs.shape == (n * H * W // 128, Co, 2)
        yt = y.double().view(-1, 128, Co)
        ref = torch.stack([yt.sum(1), (yt * yt).sum(1)], -1)
        torch.testing.assert_close(cs.double(), ref, rtol=1e-5, atol=1e-3)
        outs.append(y)
        stats.append(cs)
    x1, x2 = outs
    C = 960
    gam = (torch.rand(C, generator=g) + 0.5).to(cuda)
    bet = (torch.randn(C, generator=g) * 0.1).to(cuda)
    want = K.group_norm(x1, n, H * W, 32, 1e-5, gam, bet, silu=True, x2=x2)
    got = K.group_norm(x1, n, H * W, 32, 1e-5, gam, bet, silu=True, x2=x2, colstat=(stats[0], stats[1]))
    d = (got.float() - want.float()).abs()
    assert (d <= want.float().abs() * 2 ** -7 + 1e-6).all(), d.max()
    assert (got == want).float().mean() > 0.98
    xs = torch.cat([x1, x2], 1).float().cpu().view(n, H * W, C).permute(0, 2, 1)
    ref = F.silu(F.group_norm(xs, 32, gam.cpu(), bet.cpu(), 1e-5)).permute(0, 2, 1).reshape(-1, C)
    check(got.cpu(), ref, name="groupnorm_colstat")
    # vst_colstat restates the epilogue's arithmetic: the same bits as the conv wrote
    for y, c in zip(outs, stats):
        assert torch.equal(K.colstat(y), c)
    # a tensor modified after its conv loses its statistics
    x2.add_(0)
    assert K.colstat_of(x2) is None and K.colstat_of(x1) is not None
    # ... and so does one overwritten through a raw-pointer launch (out=), which does not bump its version
    K.conv3x3(xin, n, H, W, wflat(rnd(640, 320, 3, 3, scale=0.02, gen=g)).to(cuda), None, out=x1)
    assert K.colstat_of(x1) is None
    # statistics of the wrong shape are refused on the host (the kernel indexes them without bounds)
    with pytest.raises(K._lib.VstError):
        K.group_norm(x1, n, H * W, 32, 1e-5, gam, bet, silu=True, x2=x2, colstat=(stats[1], stats[0]))
    with pytest.raises(K._lib.VstError):
        K.group_norm(x1, n, H * W, 32, 1e-5, gam, bet, silu=True, x2=x2, colstat=(stats[0], None))
    K.colstat_reset()
    assert K.colstat_of(x1) is None


@pytest.mark.parametrize("P,nclip,Fr,HW,C", [(1, 2, 16, 256, 1280), (2, 2, 16, 256, 1280), (4, 2, 16, 64, 320),
                                              (8, 1, 32, 576, 640), (2, 3, 4, 100, 64)])
def test_group_norm_frame_partials_sharded(cuda, K, P, nclip, Fr, HW, C):
    """Motion GN: P 'ranks' holding F/P frames of every clip, partials all-gathered rank-major; every rank's rows
    == the same rows of the whole-clip GN bit for bit, and the whole-clip GN matches torch fp32."""
    g = torch.Generator().manual_seed(P * 100 + HW)
    x = (rnd(nclip * Fr * HW, C, gen=g) + 0.3).to(cuda)
    gam = (torch.rand(C, generator=g) + 0.5).to(cuda)
    bet = (torch.randn(C, generator=g) * 0.1).to(cuda)
    xv = x.view(nclip, Fr, HW, C)
    whole = K.group_norm_apply_partials(x, nclip, Fr, HW, 32, 1e-6, gam, bet,
                                        K.group_norm_frame_partials(x, nclip * Fr, HW, 32), 1)
    Fl = Fr // P
    shards = [xv[:, r * Fl:(r + 1) * Fl].reshape(-1, C).contiguous() for r in range(P)]
    part = torch.stack([K.group_norm_frame_partials(s, nclip * Fl, HW, 32) for s in shards]).contiguous()
    for r, s in enumerate(shards):
        y = K.group_norm_apply_partials(s, nclip, Fl, HW, 32, 1e-6, gam, bet, part, P)
        assert torch.equal(y.view(nclip, Fl, HW, C), whole.view(nclip, Fr, HW, C)[:, r * Fl:(r + 1) * Fl]), f"rank {r}"
    ref = F.group_norm(x.float().cpu().view(nclip, Fr * HW, C).permute(0, 2, 1), 32, gam.cpu(), bet.cpu(), 1e-6)
    check(whole.cpu(), ref.permute(0, 2, 1).reshape(-1, C), name="groupnorm_frames")


@pytest.mark.parametrize("nimg,HW,C", [(32, 256, 1280), (32, 1024, 640), (8, 4096, 320), (6, 576, 1280)])
def test_group_norm_frame_invariant(cuda, K, nimg, HW, C):
    """Per-frame GroupNorm: a frame's output does not depend on how many frames share the launch (the chunking is a
    function of the frame's row count only), so a frame-sharded rank gets the unsharded bits."""
    g = torch.Generator().manual_seed(nimg + HW)
    x = (rnd(nimg * HW, C, gen=g) + 0.2).to(cuda)
    gam = (torch.rand(C, generator=g) + 0.5).to(cuda)
    bet = (torch.randn(C, generator=g) * 0.1).to(cuda)
    full = K.group_norm(x, nimg, HW, 32, 1e-5, gam, bet, silu=True)
    for lo, hi in ((0, nimg // 2), (nimg // 2, nimg), (1, 2)):
        part = K.group_norm(x[lo * HW:hi * HW], hi - lo, HW, 32, 1e-5, gam, bet, silu=True)
        assert torch.equal(part, full[lo * HW:hi * HW]), (lo, hi)


@pytest.mark.parametrize("dims,perm", [((2, 3, 4, 5), (2, 0, 1, 3)), ((4, 2, 3, 8), (1, 0, 2, 3)),
                                       ((4, 2, 3, 8), (1, 2, 0, 3)), ((3, 1, 2, 2), (3, 2, 1, 0))])
def test_permute_rows(cuda, K, dims, perm):
    C = 40
    n = dims[0] * dims[1] * dims[2] * dims[3]
    x = torch.arange(n * C, dtype=torch.float32).remainder(251).view(n, C).to(torch.bfloat16)
    out = K.permute_rows(x.to(cuda), dims, perm).cpu()
    ref = x.view(*dims, C).permute(*perm, 4).reshape(n, C)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("rows,C,use_pe,offset", [(300, 320, False, 0.0), (64, 1280, True, 0.0), (513, 640, True, 0.0),
                                                 (10, 64, False, 0.0), (256, 1280, False, 40.0), (96, 320, False, -25.0)])
def test_layer_norm(cuda, K, rows, C, use_pe, offset):
    """offset: rows whose mean is far from 0 relative to their spread (the statistics' cancellation case)."""
    g = torch.Generator().manual_seed(rows + C)
    x = (rnd(rows, C, gen=g).float() + offset).to(torch.bfloat16)
    gam, bet = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.1
    pe = torch.randn(32, C, generator=g) if use_pe else None
    HW, Fr = 4, 8
    out = K.layer_norm(x.to(cuda), gam.to(cuda), bet.to(cuda), 1e-5, pe=None if pe is None else pe.to(cuda),
                       pe_div=HW, pe_mod=Fr)
    ref = F.layer_norm(x.float(), (C,), gam, bet, 1e-5)
    if use_pe:
        ref = ref + pe[(torch.arange(rows) // HW) % Fr]
    check(out, ref, name="layernorm")


def test_timestep_and_euler(cuda, K):
    t = torch.tensor([981.0, 1.0, 500.0], device=cuda)
    out = torch.zeros(3, 320, dtype=torch.bfloat16, device=cuda)
    K.timestep_embedding(t, 3, 320, out)
    half = 160
    ex = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32) / half)
    e = t.cpu()[:, None] * ex[None]
    ref = torch.cat([torch.cos(e), torch.sin(e)], -1)
    check(out, ref, rel_max=2e-2, name="temb")
    # Euler + CFG
    B, Cl, Fr, H, W = 1, 4, 3, 4, 4
    lat = torch.randn(B, Cl, Fr, H, W)
    sig = torch.tensor([14.6, 10.0, 0.0])
    step = torch.zeros(1, dtype=torch.int32, device=cuda)
    packed = torch.empty(2 * B * Fr * H * W, Cl, dtype=torch.bfloat16, device=cuda)
    K.pack_latents(lat.to(cuda), packed, sigmas=sig.to(cuda), step_idx=step, ncopy=2)
    ref_pack = (lat / math.sqrt(14.6 ** 2 + 1)).permute(0, 2, 3, 4, 1).reshape(-1, Cl)
    check(packed[: B * Fr * H * W], ref_pack, name="pack")
    check(packed[B * Fr * H * W:], ref_pack, name="pack2")
    noise = rnd(2 * B * Fr * H * W, Cl)
    latd = lat.to(cuda)
    K.euler_cfg_step(noise.to(cuda), latd, sig.to(cuda), step, guidance=7.5, ncopy=2)
    u = noise[: B * Fr * H * W].float().view(B, Fr, H, W, Cl).permute(0, 4, 1, 2, 3)
    c = noise[B * Fr * H * W:].float().view(B, Fr, H, W, Cl).permute(0, 4, 1, 2, 3)
    ref = lat + (0.0 - 0.0 + 10.0 - 14.6) * (u + 7.5 * (c - u))
    check(latd, ref, rel_l2=1e-5, rel_max=1e-5, name="euler")
    K.step_advance(step, 50)
    assert int(step.item()) == 1
    step.fill_(49)
    K.step_advance(step, 50)  # end of the schedule wraps instead of indexing sigmas[51]
    assert int(step.item()) == 0


@pytest.mark.parametrize("M,N,Kd,tile,splits", [(700, 1280, 320, 0, 0), (4096, 2560, 640, 0, 0), (300, 384, 640, 1, 3),
                                               (1024, 512, 256, 3, 1)])
def test_gemm_gelu(cuda, K, M, N, Kd, tile, splits):
    g = torch.Generator().manual_seed(M + N + 5)
    x, w = rnd(M, Kd, gen=g), rnd(N, Kd, scale=Kd ** -0.5, gen=g)
    b = torch.randn(N, generator=g) * 0.3
    K.GEMM_POLICY.update(tile=tile, splits=splits)
    try:
        out = K.linear(x.to(cuda), w.to(cuda), b.to(cuda), act="gelu")
    finally:
        K.GEMM_POLICY.update(tile=0, splits=0)
    check(out, F.gelu(x.float() @ w.float().t() + b), name="gemm+gelu")


def test_add_row_table_and_unpack(cuda, K):
    g = torch.Generator().manual_seed(3)
    B, C, Fr, H, W = 2, 96, 5, 9, 7
    x5 = torch.randn(B, C, Fr, H, W, generator=g)
    tok = torch.empty(B * Fr * H * W, C, dtype=torch.bfloat16, device=cuda)
    K.pack_latents(x5.to(cuda), tok)
    pe = torch.randn(32, C, generator=g)
    y = K.add_row_table(tok, pe.to(cuda), div=H * W, mod=Fr)
    ref = x5.to(torch.bfloat16).float().permute(0, 2, 3, 4, 1).reshape(-1, C) + pe[(torch.arange(y.shape[0]) // (H * W)) % Fr]
    check(y, ref, name="add_row_table")
    out = torch.empty(B, C, Fr, H, W, device=cuda)
    K.unpack_tokens(tok, out)
    assert torch.equal(out.cpu(), x5.to(torch.bfloat16).float())


@pytest.mark.parametrize("rows,C,R", [(300, 320, 64), (1000, 1280, 32), (77, 640, 48), (64, 64, 16), (33, 1280, 64),
                                      (8192, 1280, 48), (4100, 640, 16), (2049, 96, 32)])
def test_layer_norm_lora(cuda, K, rows, C, R):
    """LayerNorm + UnZipLoRA down-projection in one pass: y = LN(x) (bf16), u = y @ A^T."""
    g = torch.Generator().manual_seed(rows + C + R)
    x = rnd(rows, C, gen=g) + 0.3
    gam, bet = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.1
    A = rnd(R, C, scale=C ** -0.5, gen=g)
    y, u = K.layer_norm_lora(x.to(cuda), gam.to(cuda), bet.to(cuda), 1e-5, A.to(cuda))
    ref_y = F.layer_norm(x.float(), (C,), gam, bet, 1e-5)
    check(y, ref_y, name="ln_lora.y")
    check(u, ref_y.to(torch.bfloat16).float() @ A.float().t(), name="ln_lora.u")


def test_ceiling_probes(cuda, K):
    """The measured-peak probes bench.py reports: plausible MI355X magnitudes (well above any
    kernel of the path, at or below the vendor peaks with some slack for clocks)."""
    tf = K.probe_mfma_tflops(cuda, grid=512, iters=4000, reps=1)
    gbs = K.probe_hbm_read_gbs(cuda, nbytes=1 << 30, reps=1)
    assert 500.0 < tf < 3000.0, tf
    assert 1000.0 < gbs < 9000.0, gbs


@pytest.mark.parametrize("row_bias", [False, True])
def test_gemm_rows_past_2gb(cuda, K, row_bias):
    """An A operand of 2.3 GB (the 64^2 ff.net.2 of an 8-clip CFG batch reads 2.7 GB): the kernels' buffer descriptors
    take 32-bit byte offsets, so vst_gemm_ex runs such a call as row chunks (gemm.hip row_chunk; with a row bias the
    chunks start on its row groups, here 4096-row frames).  The rows past 2 GiB are checked against fp32 torch and
    bitwise against a launch over those rows alone."""
    div = 4096
    M, Kd, N = 220 * div, 1280, 320
    g = torch.Generator(device=cuda).manual_seed(5)
    x = torch.randn(M, Kd, generator=g, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, Kd, generator=g, device=cuda) * Kd ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g, device=cuda) * 0.1
    r = torch.randn(M, N, generator=g, device=cuda).to(torch.bfloat16)
    rb = torch.randn(M // div, N, generator=g, device=cuda) if row_bias else None
    kw = dict(row_bias=rb, row_bias_div=div) if row_bias else {}
    assert (M - 1) * Kd * 2 > 2 ** 31
    out = K.linear(x, w, b, residual=r, **kw)
    tail = slice(M - 16 * div, M)
    kt = dict(row_bias=rb[-16:].contiguous(), row_bias_div=div) if row_bias else {}
    alone = K.linear(x[tail].contiguous(), w, b, residual=r[tail].contiguous(), **kt)
    torch.cuda.synchronize()
    assert torch.equal(out[tail], alone)

    def ref(rows):
        y = x[rows].float() @ w.float().t() + b + r[rows].float()
        if row_bias:
            y = y + rb.repeat_interleave(div, 0)[rows]
        return y
    check(out[tail], ref(tail), name="gemm rows past 2 GiB")
    check(out[0:4096], ref(slice(0, 4096)), name="gemm first rows")


@pytest.mark.parametrize("row_bias", [False, True])
def test_conv3x3_images_past_2gb(cuda, K, row_bias):
    """A conv input of 2.2 GB: vst_conv3x3_ex runs it as chunks of whole images; the last images (past 2 GiB) equal a
    conv of those 8 images alone (both on the 8-phase kernel), and fp32 torch on the last one."""
    n, Ci, Co, H, W = 42, 1024, 64, 160, 160
    g = torch.Generator(device=cuda).manual_seed(6)
    x = torch.randn(n * H * W, Ci, generator=g, device=cuda).to(torch.bfloat16)
    w = (torch.randn(Co, Ci, 3, 3, generator=g, device=cuda) * (9 * Ci) ** -0.5).to(torch.bfloat16)
    b = torch.randn(Co, generator=g, device=cuda) * 0.1
    assert x.numel() * 2 > 2 ** 31
    wf = wflat(w.cpu()).to(cuda)
    rb = torch.randn(n, Co, generator=g, device=cuda) if row_bias else None  # per image (the resnets' temb)
    kw = dict(row_bias=rb, row_bias_div=H * W) if row_bias else {}
    out = K.conv3x3(x, n, H, W, wf, b, **kw)
    kt = dict(row_bias=rb[n - 8:].contiguous(), row_bias_div=H * W) if row_bias else {}
    alone = K.conv3x3(x[(n - 8) * H * W:].contiguous(), 8, H, W, wf, b, **kt)
    torch.cuda.synchronize()
    assert torch.equal(out[(n - 8) * H * W:], alone)
    xi = x[(n - 1) * H * W:].float().view(1, H, W, Ci).permute(0, 3, 1, 2)
    ref = to_nhwc(conv_ref(xi, w.float(), b)) + (rb[n - 1] if row_bias else 0)
    check(out[(n - 1) * H * W:], ref, name="conv image past 2 GiB")


def test_unchunked_entry_points_refuse_past_2gb(cuda, K):
    """Entry points that do not chunk (attention here) refuse operands past the kernels' 32-bit buffer offsets with
    VST_ERR_ARG instead of computing on the zeros those offsets would read (vst_common.h Fit31)."""
    from video_style_transfer_amd._lib import VstError
    heads, Nq, Nk = 10, 4096, 77
    nb = 420  # q: 1.72M rows x 640 bf16 = 2.2 GB
    q = torch.empty(nb * Nq, heads * 64, dtype=torch.bfloat16, device=cuda)
    kv = torch.zeros(nb * Nk, heads * 64, dtype=torch.bfloat16, device=cuda)
    o = torch.empty(1, heads * 64, dtype=torch.bfloat16, device=cuda).expand(nb * Nq, heads * 64)
    assert (nb * Nq - 1) * heads * 64 * 2 > 2 ** 31
    with pytest.raises(VstError, match="status 1"):
        K.spatial_attention(q, kv, kv, nb, heads, Nq, Nk, out=o)
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,N,Kc", [(262144, 320, 320), (65536, 640, 640), (20000, 1280, 1280), (4096, 2560, 320),
                                    (1000, 32, 640), (300, 1280, 32), (16384, 1280, 5120), (77, 64, 8)])
def test_gemm_tn_vs_torch(cuda, K, M, N, Kc):
    """vst_gemm_tn (the training step's weight gradients, C = a^T b over M tokens) against fp32 torch: token tails
    (M not a multiple of 64), N / K not multiples of 128, the split-token fp32 partials and the direct bf16 path."""
    g = torch.Generator(device=cuda).manual_seed(M + N)
    a = torch.randn(M, N, generator=g, device=cuda).to(torch.bfloat16)
    b = (torch.randn(M, Kc, generator=g, device=cuda) * M ** -0.5).to(torch.bfloat16)
    out = K.linear_tn(a, b)
    ref = a.float().t() @ b.float()
    check(out, ref, name=f"gemm_tn {M}x{N}x{Kc}")
    again = K.linear_tn(a, b)
    torch.cuda.synchronize()
    assert torch.equal(out, again)  # deterministic (fixed-order split sum)
