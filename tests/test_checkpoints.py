"""CPU tests of the offline checkpoint formats, so real weights drop in:
  * a diffusers SDXL `unet/` snapshot + a MotionAdapter snapshot (animatediff/utils.py:13-45),
  * a trained `checkpoint-{step}/motion_modules.pth` (animatediff/utils.py:102-144, _find_pth :56-63),
  * Stage-1 UnZipLoRA `pytorch_lora_weights.safetensors` + merger .pth files
    (unziplora_unet/utils.py:27,347-484).
The files are synthesised here in those layouts (no real checkpoint exists offline); loading goes through
safetensors / torch.load(weights_only=True) only."""
import json
import os

import pytest
import torch

from video_style_transfer_amd.config import UNetMotionConfig
from video_style_transfer_amd.utils import (PARTS, build_unet, insert_unziplora_to_unet, load_unet_with_motion,
                                            save_checkpoint, unet_config_from_diffusers)
from video_style_transfer_amd.weights import synthetic_state_dict

TINY_DIFFUSERS_UNET = {
    "_class_name": "UNet2DConditionModel", "in_channels": 4, "out_channels": 4,
    "block_out_channels": [64, 128, 256], "layers_per_block": 2,
    "down_block_types": ["DownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D"],
    "up_block_types": ["CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "UpBlock2D"],
    "attention_head_dim": [1, 2, 4], "transformer_layers_per_block": [1, 1, 2], "cross_attention_dim": 256,
    "addition_time_embed_dim": 32, "projection_class_embeddings_input_dim": 64 + 6 * 32, "norm_num_groups": 32,
    "norm_eps": 1e-5, "use_linear_projection": True, "addition_embed_type": "text_time",
}
ADAPTER = {"_class_name": "MotionAdapter", "motion_layers_per_block": 2, "motion_num_attention_heads": 8,
           "motion_max_seq_length": 32, "motion_norm_num_groups": 32, "use_motion_mid_block": False}


def _write_snapshot(root, sd):
    from safetensors.torch import save_file
    os.makedirs(os.path.join(root, "sdxl", "unet"))
    os.makedirs(os.path.join(root, "adapter"))
    with open(os.path.join(root, "sdxl", "unet", "config.json"), "w") as f:
        json.dump(TINY_DIFFUSERS_UNET, f)
    with open(os.path.join(root, "adapter", "config.json"), "w") as f:
        json.dump(ADAPTER, f)
    base = {k: v.contiguous() for k, v in sd.items() if "motion_modules" not in k}
    motion = {k: v.contiguous() for k, v in sd.items() if "motion_modules" in k and not k.endswith(".pe")}
    save_file(base, os.path.join(root, "sdxl", "unet", "diffusion_pytorch_model.safetensors"))
    save_file(motion, os.path.join(root, "adapter", "diffusion_pytorch_model.fp16.safetensors"))
    return os.path.join(root, "sdxl"), os.path.join(root, "adapter")


def test_sdxl_diffusers_config_maps_to_architecture():
    sdxl = {"block_out_channels": [320, 640, 1280], "attention_head_dim": [5, 10, 20],
            "transformer_layers_per_block": [1, 2, 10], "cross_attention_dim": 2048, "addition_time_embed_dim": 256,
            "projection_class_embeddings_input_dim": 2816, "layers_per_block": 2, "norm_num_groups": 32,
            "down_block_types": ["DownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D"],
            "up_block_types": ["CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "UpBlock2D"]}
    assert unet_config_from_diffusers(sdxl, ADAPTER).to_dict() == UNetMotionConfig.sdxl().to_dict()


def test_load_unet_with_motion_from_diffusers_snapshots(tmp_path):
    cfg = UNetMotionConfig.tiny()
    sd = synthetic_state_dict(cfg, seed=5, lora_rank=None)
    base, adapter = _write_snapshot(str(tmp_path), sd)
    unet, max_seq = load_unet_with_motion(base, adapter, torch_dtype=torch.float32, device="cpu")
    assert max_seq == 32
    got = unet.state_dict()
    assert set(got) == set(sd)
    for k, v in sd.items():
        assert torch.equal(got[k], v), k  # PE tables rebuilt equal to the synthetic ones


def test_motion_modules_pth_roundtrip(tmp_path):
    cfg = UNetMotionConfig.tiny()
    sd = synthetic_state_dict(cfg, seed=6, lora_rank=None)
    base, _ = _write_snapshot(str(tmp_path), sd)
    trained = build_unet(cfg, state_dict=sd, lora_rank=None, device="cpu", dtype=torch.float32)
    with torch.no_grad():
        for n, p in trained.named_parameters():
            if "motion_modules" in n:
                p.add_(0.25)  # "trained" motion weights
    save_checkpoint(trained, str(tmp_path / "out"), 100)
    ckpt = str(tmp_path / "out" / "checkpoint-100")
    unet, max_seq = load_unet_with_motion(base, ckpt, torch_dtype=torch.float32, device="cpu")
    assert max_seq is None
    ref = trained.state_dict()
    for k, v in unet.state_dict().items():
        assert torch.equal(v, ref[k]), k
    with pytest.raises(KeyError):  # a checkpoint that does not fit the architecture fails loudly
        bad = dict(sd)
        bad.pop("conv_in.weight")
        build_unet(cfg, state_dict=bad, lora_rank=None, device="cpu", dtype=torch.float32, strict=False)


def test_insert_unziplora_from_stage1_files(tmp_path):
    from safetensors.torch import save_file
    cfg = UNetMotionConfig.tiny()
    unet = build_unet(cfg, state_dict=synthetic_state_dict(cfg, seed=7, lora_rank=None), lora_rank=None,
                      device="cpu", dtype=torch.float32)
    g = torch.Generator().manual_seed(0)
    r = 4
    content, style, mc, ms = {}, {}, {}, {}
    names = [n[: -len(".processor")] for n in unet.attn_processors if "motion_modules" not in n]
    assert names
    for attn_name in names:
        attn = unet.get_submodule(attn_name)
        for part in PARTS:
            lin = attn.get_submodule(part)
            for tens, tag in ((content, "c"), (style, "s")):
                tens[f"unet.unet.{attn_name}.{part}.lora.down.weight"] = torch.randn(r, lin.in_features, generator=g)
                tens[f"unet.unet.{attn_name}.{part}.lora.up.weight"] = torch.randn(lin.out_features, r, generator=g)
            mc[f"unet.{attn_name}.{part}.lora.merge_content"] = torch.rand(lin.out_features, generator=g)
            ms[f"unet.{attn_name}.{part}.lora.merge_style"] = torch.rand(lin.out_features, generator=g)
    os.makedirs(tmp_path / "content")
    save_file(content, str(tmp_path / "content" / "pytorch_lora_weights.safetensors"))
    save_file(style, str(tmp_path / "style.safetensors"))
    torch.save(mc, str(tmp_path / "merger_content.pth"))
    torch.save(ms, str(tmp_path / "merger_style.pth"))
    insert_unziplora_to_unet(unet, str(tmp_path / "content"), str(tmp_path / "style.safetensors"),
                             str(tmp_path / "merger_content.pth"), str(tmp_path / "merger_style.pth"), rank=r,
                             device="cpu")
    for attn_name in names:
        for part in PARTS:
            layer = unet.get_submodule(f"{attn_name}.{part}").lora_layer
            d = layer.lora_matrix_dic
            assert torch.equal(d["content_down"].weight, content[f"unet.unet.{attn_name}.{part}.lora.down.weight"])
            assert torch.equal(d["style_up"].weight, style[f"unet.unet.{attn_name}.{part}.lora.up.weight"])
            assert torch.equal(layer.merge_content.detach(), mc[f"unet.{attn_name}.{part}.lora.merge_content"])
            assert torch.equal(layer.merge_style.detach(), ms[f"unet.{attn_name}.{part}.lora.merge_style"])


# ---------------------------------------------------------------------------- pinned to the reference's own output
class _GoldAttn(torch.nn.Module):
    """The module tree tests/golden/make_golden.py gave the reference's temporal_lora.py (duck-typed attention with
    to_q/to_k/to_v/to_out), rebuilt from this package's classes."""

    def __init__(self, C, with_lora):
        super().__init__()
        from video_style_transfer_amd.lora_linear import LoRACompatibleLinear
        L = LoRACompatibleLinear if with_lora else torch.nn.Linear
        self.to_q = L(C, C, bias=False)
        self.to_k = L(C, C, bias=False)
        self.to_v = L(C, C, bias=False)
        self.to_out = torch.nn.ModuleList([L(C, C, bias=True), torch.nn.Dropout(0.0)])


class _GoldTr(torch.nn.Module):
    def __init__(self, C, with_lora):
        super().__init__()
        blk = torch.nn.Module()
        blk.attn1, blk.attn2 = _GoldAttn(C, with_lora), _GoldAttn(C, with_lora)
        self.transformer_blocks = torch.nn.ModuleList([blk])


def test_temporal_lora_formats_match_reference_golden(tmp_path):
    """inject_temporal_lora / build_spatial_lora_index / compute_orth_loss / get_merged_motion_state_dict /
    save_checkpoint against the reference's own outputs on the same tree and weights (tests/golden/temporal_lora,
    produced by animatediff/temporal_lora.py:44-192): same wrapped-layer count, same orth-loss pairs and value, the
    merged motion_modules state dict with exactly the reference's key set and values (what the reference writes to
    checkpoint-{step}/motion_modules.pth, animatediff/utils.py:102-144)."""
    from safetensors import safe_open
    from safetensors.torch import load_file
    from video_style_transfer_amd.temporal_lora import (build_spatial_lora_index, compute_orth_loss,
                                                        get_merged_motion_state_dict, inject_temporal_lora)
    from video_style_transfer_amd.unziplora_linear_layer import UnZipLoRALinearLayerInfer
    path = os.path.join(os.path.dirname(__file__), "golden", "temporal_lora.safetensors")
    T = load_file(path)
    with safe_open(path, "pt") as f:
        meta = json.loads(f.metadata()["meta"])
    C = meta["C"]
    u = torch.nn.Module()
    down = torch.nn.Module()
    down.attentions = torch.nn.ModuleList([_GoldTr(C, True), _GoldTr(C, True)])
    down.motion_modules = torch.nn.ModuleList([_GoldTr(C, False), _GoldTr(C, False)])
    u.down_blocks = torch.nn.ModuleList([down])
    for n, m in u.named_modules():
        if hasattr(m, "set_lora_layer"):
            m.set_lora_layer(UnZipLoRALinearLayerInfer(m.in_features, m.out_features, 8, ["content", "style"]))
    assert inject_temporal_lora(u, rank=meta["rank"], alpha=meta["alpha"]) == meta["n_wrapped"]
    sd = {k[3:]: v for k, v in T.items() if k.startswith("sd.")}
    u.load_state_dict(sd, strict=True)  # the reference's parameter names load as they are
    idx = build_spatial_lora_index(u)
    assert sorted(idx) == sorted(meta["index"])
    orth = compute_orth_loss(u, idx, meta["lambda"])
    assert torch.allclose(orth.detach(), T["orth_loss"][0], rtol=1e-4), (orth, T["orth_loss"])
    merged = get_merged_motion_state_dict(u)
    gold_keys = meta["merged_keys"]
    assert sorted(merged) == sorted(gold_keys)
    for k in gold_keys:
        assert torch.allclose(merged[k].float(), T["merged_sd." + k].float(), rtol=1e-5, atol=1e-7), k
    save_checkpoint(u, str(tmp_path), 7)
    saved = torch.load(os.path.join(tmp_path, "checkpoint-7", "motion_modules.pth"), map_location="cpu",
                       weights_only=True)
    assert sorted(saved) == sorted(gold_keys)
