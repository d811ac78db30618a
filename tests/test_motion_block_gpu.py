"""The fused motion-module attention block (vst_motion_attention_block, csrc/motion.hip): LayerNorm + sinusoidal PE,
the q/k/v projection, attention over the 16 frames of every pixel, to_out and the residual add in one launch, against
(a) the four-launch path it replaces (vst_layernorm with the PE, the q/k/v GEMM, vst_temporal_attention, the
out-projection GEMM with the residual fused) and (b) fp32 torch of the same block (diffusers BasicTransformerBlock
norm1 -> +PE -> attn1 -> +residual inside AnimateDiff's motion module; reference copy of the block:
unziplora_unet/unzip_attention.py:150-151, 196-197; core: animatediff/temporal_transformer.py:66-68).

Tolerances on y: (a) 2e-3 rel-L2 / 1e-2 rel-max -- the same bf16 rounding points, the projections summed over k in
another order; (b) the kernel tests' 5e-3 / 1e-2 against fp32.  On the block's update y - x alone: rel-L2 2e-3 against
the four-launch path (rel-max not gated: one bf16 ulp of y is ~1e-2 of a typical |y - x|), and against fp32 no worse
than 1.1x the four-launch path's own distance (~1e-2, set by y's bf16 rounding)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

C, HEADS, F = 320, 8, 16


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


def _operands(nclip, HW, qkv_bias, seed, dev):
    g = torch.Generator().manual_seed(seed)
    T = nclip * F * HW
    x = (torch.randn(T, C, generator=g) * 0.7).to(torch.bfloat16).to(dev)
    gamma = (1.0 + 0.1 * torch.randn(C, generator=g)).to(dev)
    beta = (0.1 * torch.randn(C, generator=g)).to(dev)
    pe = (0.5 * torch.randn(32, C, generator=g)).to(dev)
    wqkv = (torch.randn(3 * C, C, generator=g) * C ** -0.5).to(torch.bfloat16).to(dev)
    bqkv = (0.1 * torch.randn(3 * C, generator=g)).to(dev) if qkv_bias else None
    wo = (torch.randn(C, C, generator=g) * 0.25 * C ** -0.5).to(torch.bfloat16).to(dev)
    bo = (0.05 * torch.randn(C, generator=g)).to(dev)
    return x, gamma, beta, pe, wqkv, bqkv, wo, bo


def _four_launch(K, x, nclip, HW, gamma, beta, pe, wqkv, bqkv, wo, bo):
    n = K.layer_norm(x, gamma, beta, 1e-5, pe=pe, pe_div=HW, pe_mod=F)
    qkv = K.linear(n, wqkv, bqkv)
    o = K.temporal_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], nclip, F, HW, HEADS, C // HEADS)
    return K.linear(o, wo, bo, residual=x)


def _fp32(x, nclip, HW, gamma, beta, pe, wqkv, bqkv, wo, bo):
    xf = x.float()
    n = torch.nn.functional.layer_norm(xf, (C,), gamma, beta, 1e-5)
    n = n + pe[:F].repeat_interleave(HW, 0).repeat(nclip, 1)
    qkv = n @ wqkv.float().t() + (0 if bqkv is None else bqkv)
    q, k, v = (t.view(nclip, F, HW, HEADS, C // HEADS).permute(0, 2, 3, 1, 4) for t in qkv.split(C, 1))
    o = torch.nn.functional.scaled_dot_product_attention(q, k, v)  # over the frame axis
    o = o.permute(0, 3, 1, 2, 4).reshape(nclip * F * HW, C)
    return xf + o @ wo.float().t() + bo


@pytest.mark.parametrize("nclip,HW,qkv_bias", [(2, 256, False), (2, 4096, False), (1, 64, True)])
def test_motion_block_vs_four_launch_and_fp32(cuda, K, nclip, HW, qkv_bias):
    ops = _operands(nclip, HW, qkv_bias, nclip * 7 + HW, cuda)
    x, gamma, beta, pe, wqkv, bqkv, wo, bo = ops
    assert K.motion_block_fusable(C, F, HW, HEADS)
    y = K.motion_attention_block(x, nclip, F, HW, HEADS, gamma, beta, 1e-5, pe, wqkv, bqkv, wo, bo)
    y4 = _four_launch(K, x, nclip, HW, gamma, beta, pe, wqkv, bqkv, wo, bo)
    check(y, y4, 2e-3, 1e-2, f"fused vs four-launch HW={HW}")
    # the block's update alone (y - x): rel-L2 only -- one bf16 ulp of y is ~1e-2 of a typical |y - x|
    check(y.float() - x.float(), y4.float() - x.float(), 2e-3, 1.0, f"fused vs four-launch update HW={HW}")
    ref = _fp32(x, nclip, HW, gamma, beta, pe, wqkv, bqkv, wo, bo)
    check(y, ref, 5e-3, 1e-2, f"fused vs fp32 HW={HW}")
    # the update against fp32 is dominated by y's own bf16 rounding: no worse than the four-launch path's
    e_fused = ((y.float() - ref).norm() / (ref - x.float()).norm()).item()
    e_four = ((y4.float() - ref).norm() / (ref - x.float()).norm()).item()
    assert e_fused <= 1.1 * e_four + 1e-4, (e_fused, e_four)


def test_motion_block_refuses_other_shapes(cuda, K):
    from video_style_transfer_amd import _lib
    assert not K.motion_block_fusable(640, F, 1024, HEADS)   # the 32x32 level keeps the four launches
    assert not K.motion_block_fusable(C, 32, 4096, HEADS)    # configs[3]: 32 frames
    assert not K.motion_block_fusable(C, F, 4092, HEADS)     # pixels not a multiple of 8
    x, gamma, beta, pe, wqkv, bqkv, wo, bo = _operands(1, 64, False, 1, cuda)
    with pytest.raises(_lib.VstError):
        K.motion_attention_block(x, 2, 8, 64, HEADS, gamma, beta, 1e-5, pe, wqkv, bqkv, wo, bo)


def test_motion_module_opt_in_matches_default(cuda, K, monkeypatch):
    """A whole MotionModule (GroupNorm, proj_in, the transformer block, proj_out) at the 64x64-level shape with the
    fused attention halves switched on (VST_MOTION_FUSE=1) against the default four-launch path: the opt-in is a
    drop-in for the same module tree and weights."""
    from video_style_transfer_amd.unet_motion import FwdCtx, MotionModule
    torch.manual_seed(5)
    mm = MotionModule(C).to(cuda)
    with torch.no_grad():
        for name, p in mm.named_parameters():
            if p.dim() == 2:
                p.normal_(0.0, 0.4 * p.shape[1] ** -0.5)
            elif "norm" in name and name.endswith("weight"):
                p.normal_(1.0, 0.1)
            else:
                p.normal_(0.0, 0.05)
    for p in mm.parameters():
        p.requires_grad_(False)
    nclip, H, W = 2, 16, 16
    x = (torch.randn(nclip * F * H * W, C, device=cuda) * 0.7).to(torch.bfloat16)
    ctx = FwdCtx(B=nclip, F=F, emb_silu=None, enc=None, cross_kwargs={})
    monkeypatch.delenv("VST_MOTION_FUSE", raising=False)
    K.profile_launches(True)
    y_def = mm.run(x, nclip * F, H, W, ctx)
    kinds_def = [r[0] for r in K.collect_launches()]
    K.profile_launches(False)
    monkeypatch.setenv("VST_MOTION_FUSE", "1")
    K.profile_launches(True)
    y_fused = mm.run(x, nclip * F, H, W, ctx)
    kinds_fused = [r[0] for r in K.collect_launches()]
    K.profile_launches(False)
    assert "motion_block" not in kinds_def and kinds_fused.count("motion_block") == 2, (kinds_def, kinds_fused)
    check(y_fused, y_def, 2e-3, 1e-2, "motion module fused vs default")
