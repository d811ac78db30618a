"""The fused base + LoRA projection with the down-projection inside the 8-phase GEMM (vst_gemm_lora,
gemm_p8.hip LORA) against (a) fp32 torch of the reference's arithmetic — u = x.Acat^T rounded to bf16 (the
output of UnZipLoRALinearLayerInfer's down factors under autocast, unziplora_unet/unziplora_linear_layer.py:298-346),
then [x | u].[W | V]^T + b, rounded once, + residual — and (b) the two-pass path it replaces (u from its own pass,
then vst_gemm_ex over [x | u]): the same operands in the same k order, so the two agree to the rounding of u.

Tolerances: (a) the kernel tests' 5e-3 rel-L2 / 1e-2 rel-max (one bf16 rounding of the output + fp32
reassociation); (b) 1e-3 / 4e-3 (an occasional 1-ulp difference of a bf16 u element, whose fp32 sum runs in
another order in the two passes).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rnd(*shape, scale=1.0, gen=None):
    return (torch.randn(*shape, generator=gen) * scale).to(torch.bfloat16)


def check(out, ref, rel_l2, rel_max, name=""):
    out = out.float().cpu()
    ref = ref.float().cpu()
    assert out.shape == ref.shape, (name, out.shape, ref.shape)
    assert torch.isfinite(out).all(), name
    err = out - ref
    l2 = (err.norm() / ref.norm().clamp_min(1e-12)).item()
    mx = (err.abs().max() / ref.abs().max().clamp_min(1e-12)).item()
    assert l2 <= rel_l2 and mx <= rel_max, f"{name}: rel_l2={l2:.3e} rel_max={mx:.3e}"
    return l2, mx


@pytest.fixture(scope="module")
def K():
    from video_style_transfer_amd import kernels
    return kernels


def _operands(M, Kd, nproj, n_per, r_per, P, gen, dev):
    """x [M, Kd]; Acat [P, Kd] (rows past nproj*r_per zero); W_aug [nproj*n_per, Kd + P] with projection i's up
    factors in columns Kd + i*r_per (the build_ops layout)."""
    x = rnd(M, Kd, gen=gen)
    A = torch.zeros(P, Kd)
    A[: nproj * r_per] = torch.randn(nproj * r_per, Kd, generator=gen) * Kd ** -0.5
    A = A.to(torch.bfloat16)
    N = nproj * n_per
    W = torch.zeros(N, Kd + P)
    W[:, :Kd] = torch.randn(N, Kd, generator=gen) * Kd ** -0.5
    for i in range(nproj):
        W[i * n_per:(i + 1) * n_per, Kd + i * r_per:Kd + (i + 1) * r_per] = \
            torch.randn(n_per, r_per, generator=gen) * r_per ** -0.5
    W = W.to(torch.bfloat16)
    return x.to(dev), A.to(dev), W.to(dev)


CASES = [
    # M, Kd, nproj, n_per, r_per, P, bias, residual, expected tile
    (8192, 1280, 1, 1280, 16, 32, True, True, 192),    # to_out + UnZipLoRA r=8 at the 16x16 level (+ bias, residual)
    (8192, 1280, 3, 1280, 16, 64, False, False, 256),  # attn1 q/k/v stacked
    (8192, 1280, 1, 1280, 16, 32, False, False, 192),  # attn2 q
    (32768, 640, 1, 640, 16, 32, True, True, 320),     # to_out at the 32x32 level (the persistent LoRA grid)
    (32768, 640, 3, 640, 16, 64, False, False, 320),   # attn1 q/k/v at the 32x32 level (persistent, 6 rounds)
    (8192, 1280, 3, 1280, 8, 32, False, False, 256),   # content-only (r = 8 per projection: 8-column groups)
    (7000, 1000, 1, 1280, 16, 32, True, True, 192),    # M tail (7000 = 27 x 256 + 88), K tail (1000 = 15 x 64 + 40)
]


@pytest.mark.parametrize("M,Kd,nproj,n_per,r_per,P", [(32768, 640, 1, 640, 16, 32), (32768, 640, 3, 640, 16, 64)])
def test_gemm_lora_persistent_bitwise(cuda, K, M, Kd, nproj, n_per, r_per, P):
    """The persistent LoRA grid (128x320 tiles, each tile's fill under the previous tile's epilogue) gives the bits of
    the one-workgroup-per-tile launches (VST_P8_LORA_PERSIST=0 in a child process: the switch is read once)."""
    import os
    import subprocess
    import sys
    if os.environ.get("VST_P8_LORA_PERSIST", "1") != "1":
        pytest.skip("VST_P8_LORA_PERSIST is off in this process: both sides would run the one-tile-per-workgroup grid")
    g = torch.Generator().manual_seed(M + nproj)
    x, A, W = _operands(M, Kd, nproj, n_per, r_per, P, g, cuda)
    N = W.shape[0]
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    r = rnd(M, N, gen=g).to(cuda)
    assert K.gemm_lora_tile(M, N, Kd, P, n_per, r_per) == 320
    out = K.linear_lora(x, W, A, n_per, r_per, b, residual=r)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        torch.save({"x": x.cpu(), "A": A.cpu(), "W": W.cpu(), "b": b.cpu(), "r": r.cpu()}, os.path.join(d, "in.pt"))
        code = (
            "import sys, torch; sys.path.insert(0, %r)\n"
            "from video_style_transfer_amd import kernels as K\n"
            "t = torch.load(%r, weights_only=True)\n"
            "c = {k: v.cuda() for k, v in t.items()}\n"
            "y = K.linear_lora(c['x'], c['W'], c['A'], %d, %d, c['b'], residual=c['r'])\n"
            "torch.save(y.cpu(), %r)\n" % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                             os.path.join(d, "in.pt"), n_per, r_per, os.path.join(d, "out.pt")))
        env = dict(os.environ, VST_P8_LORA_PERSIST="0")
        subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=240)
        ref = torch.load(os.path.join(d, "out.pt"), weights_only=True)
    assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("M,Kd,nproj,n_per,r_per,P,use_bias,use_res,bn", CASES)
def test_gemm_lora_vs_torch_and_two_pass(cuda, K, M, Kd, nproj, n_per, r_per, P, use_bias, use_res, bn):
    g = torch.Generator().manual_seed(M + Kd + nproj * 7 + r_per)
    x, A, W = _operands(M, Kd, nproj, n_per, r_per, P, g, cuda)
    N = W.shape[0]
    b = (torch.randn(N, generator=g) * 0.1).to(cuda) if use_bias else None
    r = rnd(M, N, gen=g).to(cuda) if use_res else None
    assert K.gemm_lora_tile(M, N, Kd, P, n_per, r_per) == bn
    out = K.linear_lora(x, W, A, n_per, r_per, b, residual=r)
    # (a) fp32 torch of the reference arithmetic
    u = (x.float() @ A.float().t()).to(torch.bfloat16)
    ref = x.float() @ W[:, :Kd].float().t() + u.float() @ W[:, Kd:].float().t()
    if b is not None:
        ref = ref + b
    if r is not None:
        ref = ref.to(torch.bfloat16).float() + r.float()
    check(out, ref, 5e-3, 1e-2, f"gemm_lora {M}x{N}x{Kd}+{P} vs fp32")
    # (b) the two-pass path (u from torch, then the [x | u] GEMM) — the kernel's own u is the only difference
    if Kd % 64 == 0:
        two = K.linear(x, W, b, x2=u, residual=r)
        check(out, two, 1e-3, 4e-3, f"gemm_lora {M}x{N}x{Kd}+{P} vs two-pass")


def test_gemm_lora_u_only(cuda, K):
    """W_base = 0, no bias: the output is u.V^T alone, so a wrong u block (group / window / row mapping) shows
    as a large error instead of hiding under the base product."""
    g = torch.Generator().manual_seed(5)
    M, Kd = 8192, 1280
    x, A, W = _operands(M, Kd, 3, 1280, 16, 64, g, cuda)
    W[:, :Kd] = 0
    out = K.linear_lora(x, W, A, 1280, 16)
    u = (x.float() @ A.float().t()).to(torch.bfloat16).float()
    ref = u @ W[:, Kd:].float().t()
    check(out, ref, 5e-3, 1e-2, "gemm_lora u.V^T only")


def test_gemm_lora_unsupported_falls_back(cuda, K):
    """A shape where every tile width would put two u blocks in one tile (q/k/v of width 600: 192-, 256-wide tiles
    straddle a projection boundary, and 600 is not a multiple of 320) is refused (status 3) and run_ops takes the
    two-pass path with the same result as the explicit two-pass call.  The decision depends on the shape only, not on
    M (a frame-sharded rank must take the unsharded forward's path)."""
    from video_style_transfer_amd import _lib
    from video_style_transfer_amd.lora_linear import ProjOps, lora_in_gemm, run_ops
    g = torch.Generator().manual_seed(9)
    M, Kd = 32768, 640
    x, A, W = _operands(M, Kd, 3, 600, 16, 64, g, cuda)
    for m in (M, 4096, 300):
        assert K.gemm_lora_tile(m, 1800, Kd, 64, 600, 16) == 0
    assert K.gemm_lora_tile(32768, 1920, Kd, 64, 640, 16) == K.gemm_lora_tile(2048, 1920, Kd, 64, 640, 16) == 320
    with pytest.raises(_lib.VstError):
        K.linear_lora(x, W, A, 600, 16)
    ops = ProjOps(W, A, None, Kd, 1800, 48, 600, 16)
    assert not lora_in_gemm(ops, M)
    out = run_ops(x, ops)
    u = K.linear(x, A, kind="gemm_lora_down")
    two = K.linear(x, W, None, x2=u)
    assert torch.equal(out, two)


def test_run_ops_uses_in_gemm_lora(cuda, K):
    """run_ops on an UnZipLoRA to_out projection takes the in-GEMM path (one launch, no separate u pass) and
    matches the two-pass result."""
    from video_style_transfer_amd.lora_linear import ProjOps, lora_in_gemm, run_ops
    g = torch.Generator().manual_seed(11)
    M, Kd = 8192, 1280
    x, A, W = _operands(M, Kd, 1, 1280, 16, 32, g, cuda)
    b = torch.randn(1280, generator=g).to(cuda)
    ops = ProjOps(W, A, b, Kd, 1280, 16, 1280, 16)
    assert lora_in_gemm(ops, M)
    K.profile_launches(True)
    out = run_ops(x, ops)
    rec = K.collect_launches()
    K.profile_launches(False)
    assert [k for k, *_ in rec] == ["gemm_lora"], rec
    assert rec[0][1] == "gemm_p8<256x192,lora>"
    u = (x.float() @ A.float().t()).to(torch.bfloat16)
    check(out, K.linear(x, W, b, x2=u), 1e-3, 4e-3, "run_ops in-GEMM vs two-pass")


@pytest.mark.parametrize("M,Kd,nproj,n_per,r_per,P,use_bias,use_res", [
    (8192, 1280, 1, 1280, 16, 32, True, True),     # to_out at 16x16 on 128x320 tiles (one full round)
    (32768, 640, 3, 640, 16, 64, False, False),    # the 32x32 q/k/v: 256-wide tiles straddle q/k, 320-wide do not
    (8292, 1000, 1, 1280, 16, 32, True, True),     # M tail (8292 = 64 x 128 + 100), K tail
    (131072, 320, 1, 320, 16, 32, True, False),
])
def test_gemm_lora_128x320(cuda, K, M, Kd, nproj, n_per, r_per, P, use_bias, use_res):
    """vst_gemm_lora on the 128x320 tiles (forced with vst_p8_force_bn): against fp32 torch and the two-pass path,
    and bit for bit equal to the 256-row tiles where those support the shape (same k order for x.W^T and for u)."""
    g = torch.Generator().manual_seed(M + Kd + nproj)
    x, A, W = _operands(M, Kd, nproj, n_per, r_per, P, g, cuda)
    N = W.shape[0]
    b = (torch.randn(N, generator=g) * 0.1).to(cuda) if use_bias else None
    r = rnd(M, N, gen=g).to(cuda) if use_res else None
    with K.p8_tile_width(320):
        assert K.gemm_lora_tile(M, N, Kd, P, n_per, r_per) == 320
        out = K.linear_lora(x, W, A, n_per, r_per, b, residual=r)
    u = (x.float() @ A.float().t()).to(torch.bfloat16)
    ref = x.float() @ W[:, :Kd].float().t() + u.float() @ W[:, Kd:].float().t()
    if b is not None:
        ref = ref + b
    if r is not None:
        ref = ref.to(torch.bfloat16).float() + r.float()
    check(out, ref, 5e-3, 1e-2, f"gemm_lora 128x320 {M}x{N}x{Kd}+{P} vs fp32")
    if Kd % 64 == 0:
        two = K.linear(x, W, b, x2=u, residual=r)
        check(out, two, 1e-3, 4e-3, f"gemm_lora 128x320 {M}x{N}x{Kd}+{P} vs two-pass")
    for bn in (192, 256):
        with K.p8_tile_width(bn):
            if K.gemm_lora_tile(M, N, Kd, P, n_per, r_per) == bn:
                assert torch.equal(out, K.linear_lora(x, W, A, n_per, r_per, b, residual=r)), bn
