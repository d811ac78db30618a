"""CPU tests of the host-side fusion policy (no launch, no GPU): which SDXL projections take the in-GEMM UnZipLoRA
down-projection (vst_gemm_lora), which attn2 calls run as one launch (vst_gemm_cross_attention), which motion-module
shapes the fused attention block accepts, and the operand grouping build_ops hands them."""
import pytest
import torch


def _attn(C, cross, r=8):
    from video_style_transfer_amd.attention_processor import Attention
    from video_style_transfer_amd.utils import attach_unziplora_layers
    holder = torch.nn.Module()
    holder.blk = torch.nn.Module()
    holder.blk.attn2 = Attention(C, 2048 if cross else None, C // 64, 64)
    attach_unziplora_layers(holder, r)
    for p in holder.parameters():
        p.requires_grad_(False)
    return holder.blk.attn2


@pytest.mark.parametrize("C", [640, 1280])
def test_build_ops_groups_unziplora_projections(C):
    """q/k/v stacked: every projection C output rows and 2r = 16 u columns (content + style), padded to 64."""
    from video_style_transfer_amd.lora_linear import build_ops
    attn = _attn(C, cross=False)
    qkv = build_ops([attn.to_q, attn.to_k, attn.to_v], 1.0)
    assert qkv.w.shape == (3 * C, C + 64) and qkv.a.shape == (64, C)
    assert (qkv.gn, qkv.gr, qkv.r) == (C, 16, 48)
    out = build_ops([attn.to_out[0]], 1.0)
    assert out.w.shape == (C, C + 32) and (out.gn, out.gr, out.r) == (C, 16, 16)
    # projection i's up factors sit in its own u columns only
    for i in range(3):
        rows = qkv.w[i * C:(i + 1) * C, C:].float()
        assert rows[:, :16 * i].abs().sum() == 0 and rows[:, 16 * (i + 1):].abs().sum() == 0


def test_lora_in_gemm_policy_at_sdxl_shapes():
    """Every SDXL projection absorbs the down-projection: 16x16 level (M = 8192 CFG-batched tokens) q/k/v, attn2 q and
    to_out; 32x32 (M = 32768) to_out and q/k/v (on 128x320 tiles: 256-wide ones straddle the q/k boundary at C = 640).
    The decision depends on the shape, not on M: a frame-sharded rank with 1/P of the rows takes the same path."""
    from video_style_transfer_amd import kernels as K
    from video_style_transfer_amd.lora_linear import build_ops, lora_in_gemm
    a16, a32 = _attn(1280, cross=False), _attn(640, cross=False)
    for m in (8192, 1024, 512):
        assert lora_in_gemm(build_ops([a16.to_q, a16.to_k, a16.to_v], 1.0), m)
        assert lora_in_gemm(build_ops([a16.to_q], 1.0), m)
        assert lora_in_gemm(build_ops([a16.to_out[0]], 1.0), m)
    for m in (32768, 4096):
        assert lora_in_gemm(build_ops([a32.to_out[0]], 1.0), m)
        qkv = build_ops([a32.to_q, a32.to_k, a32.to_v], 1.0)
        assert lora_in_gemm(qkv, m) and K.gemm_lora_tile(m, qkv.n, qkv.k1, qkv.a.shape[0], qkv.gn, qkv.gr) == 320


def test_cross_attention_fusion_policy():
    """attn2 (to_q + SDPA over 77 text keys) is one launch at both transformer levels of the step, with or without
    the UnZipLoRA layer, and not when a 256-row tile would straddle two frames."""
    from video_style_transfer_amd import attention_processor as AP
    from video_style_transfer_amd.lora_linear import build_ops
    for C, Nq in ((1280, 256), (640, 1024)):
        attn = _attn(C, cross=True)
        ops = build_ops([attn.to_q], 1.0)
        assert AP._cross_fusable(ops, 32 * Nq, Nq, 77)
        assert AP._cross_fusable(ops, 4 * Nq, Nq, 77)  # shape-only: a frame shard fuses where the whole clip does
        assert not AP._cross_fusable(ops, 32 * 320, 320, 77)
    plain = AP.Attention(1280, 2048, 20, 64)
    assert AP._cross_fusable(build_ops([plain.to_q], 1.0), 8192, 256, 77)


def test_motion_block_policy_is_opt_in(monkeypatch):
    """The fused motion attention block accepts the 64x64 level only and is used only with VST_MOTION_FUSE=1."""
    from video_style_transfer_amd import kernels as K
    from video_style_transfer_amd.unet_motion import BasicTransformerBlock, _fused_motion_ops_impl
    assert K.motion_block_fusable(320, 16, 4096, 8) and not K.motion_block_fusable(640, 16, 1024, 8)
    blk = BasicTransformerBlock(320, 8, 40, None, temporal=True)
    for p in blk.parameters():
        p.requires_grad_(False)
    monkeypatch.delenv("VST_MOTION_FUSE", raising=False)
    assert _fused_motion_ops_impl(blk, 320, 16, 4096) is None
    monkeypatch.setenv("VST_MOTION_FUSE", "1")
    ops = _fused_motion_ops_impl(blk, 320, 16, 4096)
    assert ops is not None and [o.w.shape for pair in ops for o in pair] == [(960, 320), (320, 320)] * 2
    assert _fused_motion_ops_impl(blk, 320, 32, 4096) is None  # 32 frames (configs[3])
