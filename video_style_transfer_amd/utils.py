"""Model-assembly helpers mirroring unziplora_unet/utils.py and animatediff/utils.py.

insert_unziplora_to_unet (unziplora_unet/utils.py:388-484), unziplora_set_forward_type (:162-174),
get_lora_weights (:131-160; safetensors only, local path — no hub download offline),
use_lora_weights_for_inference / use_lora_mergers_for_inference (:347-387),
_make_lora_compatible (:712-725), freeze_spatial_layers / save_checkpoint /
_extract_merger_state_dicts (animatediff/utils.py:66-163), load_unet_with_motion / _find_pth
(animatediff/utils.py:13-63: a diffusers SDXL `unet/` snapshot + a MotionAdapter snapshot or a trained
motion_modules.pth, read offline with loaders that execute nothing), synthetic UNet construction.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional, Tuple, Union

import torch

from .config import UNetMotionConfig
from .lora_linear import LoRACompatibleLinear
from .unet_motion import UNetMotionModel
from .unziplora_linear_layer import UnZipLoRALinearLayerInfer
from .weights import init_synthetic_, synthetic_state_dict  # noqa: F401

LORA_WEIGHT_NAME_SAFE = "pytorch_lora_weights.safetensors"
PARTS = ("to_q", "to_k", "to_v", "to_out.0")


def get_lora_weights(lora_name_or_path: Union[str, Dict[str, torch.Tensor]], subfolder: Optional[str] = None):
    if isinstance(lora_name_or_path, dict):
        return lora_name_or_path
    path = lora_name_or_path
    if subfolder is not None:
        path = os.path.join(path, subfolder)
    if os.path.isdir(path):
        path = os.path.join(path, LORA_WEIGHT_NAME_SAFE)
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} (hub download is unavailable offline)")
    assert path.endswith(".safetensors"), "Currently only safetensors is supported"
    from safetensors.torch import load_file
    return load_file(path, device="cpu")


def use_lora_weights_for_inference(tensors, key, prefix="unet.unet."):
    down, up = {}, {}
    for part in PARTS:
        down[part] = tensors[f"{prefix}{key}.{part}.lora.down.weight"]
        up[part] = tensors[f"{prefix}{key}.{part}.lora.up.weight"]
    return down, up


def use_lora_mergers_for_inference(tensors_content, tensors_style, key, prefix="unet.unet."):
    mc, ms = {}, {}
    for part in PARTS:
        mc[part] = tensors_content[f"{prefix}{key}.{part}.lora.merge_content"]
        ms[part] = tensors_style[f"{prefix}{key}.{part}.lora.merge_style"]
    return mc, ms


def _make_lora_compatible(module, attr):
    layer = getattr(module, attr)
    if not hasattr(layer, "set_lora_layer"):
        new = LoRACompatibleLinear(layer.in_features, layer.out_features, bias=layer.bias is not None,
                                   device=layer.weight.device, dtype=layer.weight.dtype)
        new.weight = layer.weight
        if layer.bias is not None:
            new.bias = layer.bias
        setattr(module, attr, new)


def _safe_load(path_or_dict):
    if path_or_dict is None or isinstance(path_or_dict, dict):
        return path_or_dict
    return torch.load(path_or_dict, map_location="cpu", weights_only=True)


def insert_unziplora_to_unet(unet, content_lora_path, style_lora_path, weight_content_path=None,
                             weight_style_path=None, rank: int = 64, device=None, **kwargs):
    """Inject UnZipLoRALinearLayerInfer into every non-motion attention projection.
    `rank` is a parameter here (the reference hard-wires 64 — SURVEY §9.4)."""
    tc = get_lora_weights(content_lora_path)
    ts = get_lora_weights(style_lora_path)
    wc = _safe_load(weight_content_path)
    ws = _safe_load(weight_style_path)
    for proc_name in unet.attn_processors:
        if "motion_modules" in proc_name:
            continue
        attn = unet
        for n in proc_name.split(".")[:-1]:
            attn = getattr(attn, n)
        attn_name = ".".join(proc_name.split(".")[:-1])
        cd, cu = use_lora_weights_for_inference(tc, attn_name)
        sd, su = use_lora_weights_for_inference(ts, attn_name)
        mc = ms = None
        if wc is not None and ws is not None:
            mc, ms = use_lora_mergers_for_inference(wc, ws, attn_name, prefix="unet.")
        _make_lora_compatible(attn, "to_q")
        _make_lora_compatible(attn, "to_k")
        _make_lora_compatible(attn, "to_v")
        _make_lora_compatible(attn.to_out, "0")
        for part, lin in (("to_q", attn.to_q), ("to_k", attn.to_k), ("to_v", attn.to_v), ("to_out.0", attn.to_out[0])):
            r = cd[part].shape[0] if rank is None else rank
            layer = UnZipLoRALinearLayerInfer(lin.in_features, lin.out_features, rank=r,
                                              lora_matrix_key=["content", "style"],
                                              device=device or lin.weight.device)
            sd_ = {"lora_matrix_dic.content_down.weight": cd[part], "lora_matrix_dic.content_up.weight": cu[part],
                   "lora_matrix_dic.style_down.weight": sd[part], "lora_matrix_dic.style_up.weight": su[part]}
            if mc is not None:
                sd_["merge_content"] = mc[part]
                sd_["merge_style"] = ms[part]
            layer.load_state_dict(sd_, strict=False)
            lin.set_lora_layer(layer)
    return unet


def unziplora_set_forward_type(unet, type: str = "both"):
    assert type in ["both", "content", "style"]
    for _, module in unet.named_modules():
        if hasattr(module, "set_lora_layer"):
            lora = getattr(module, "lora_layer")
            if lora is not None:
                assert hasattr(lora, "set_forward"), lora
                lora.set_forward(type)
    return unet


def attach_unziplora_layers(unet, rank: int):
    """Create (empty) UnZipLoRA layers on every spatial projection so a full state dict with
    `...lora_layer...` keys can be loaded directly."""
    for name, mod in unet.named_modules():
        if "motion_modules" in name or not isinstance(mod, LoRACompatibleLinear):
            continue
        if name.split(".")[-1] in ("to_q", "to_k", "to_v", "0") and (".attn1." in name + "." or ".attn2." in name + "."):
            mod.set_lora_layer(UnZipLoRALinearLayerInfer(mod.in_features, mod.out_features, rank=rank,
                                                         lora_matrix_key=["content", "style"],
                                                         device=mod.weight.device))
    return unet


def build_unet(cfg: Optional[UNetMotionConfig] = None, *, state_dict=None, seed: int = 0, lora_rank: Optional[int] = 8,
               device="cuda", dtype=torch.bfloat16, strict: bool = True, init: Optional[str] = None) -> UNetMotionModel:
    """UNetMotionModel with UnZipLoRA layers, weights from `state_dict` or seeded synthetic ones (`init`: the
    synthetic-init family, weights.INIT_SCALES; default weights.DEFAULT_INIT)."""
    cfg = cfg or UNetMotionConfig.sdxl()
    with torch.device("meta"):
        unet = UNetMotionModel(cfg)
    if state_dict is None:
        # seeded synthetic weights generated directly on the target device
        unet = unet.to_empty(device=device)
        if lora_rank:
            attach_unziplora_layers(unet, lora_rank)
        for name, p in unet.named_parameters():
            if "lora_layer" not in name:
                p.data = p.data.to(dtype)
        init_synthetic_(unet, cfg, seed, lora_rank, **({} if init is None else {"init": init}))
        return unet.requires_grad_(False)
    unet = unet.to_empty(device="cpu")
    if lora_rank:
        attach_unziplora_layers(unet, lora_rank)
    if not strict:
        # the only keys a checkpoint may omit are the sinusoidal PE tables (diffusers rebuilds them too);
        # UnZipLoRA factors come from insert_unziplora_to_unet (lora_rank=None here); anything else is an error
        from .weights import sinusoid_table
        for name, buf in unet.named_buffers():
            if name.endswith("pos_embed.pe") or name.endswith("pos_encoding.pe"):
                buf.copy_(sinusoid_table(buf.shape[-1], buf.shape[-2]).view_as(buf))
        missing, unexpected = unet.load_state_dict(state_dict, strict=False)
        missing = [k for k in missing if not k.endswith(".pe")]
        if missing or unexpected:
            raise KeyError(f"checkpoint does not match the architecture: missing {missing[:5]} "
                           f"({len(missing)}), unexpected {unexpected[:5]} ({len(unexpected)})")
    else:
        unet.load_state_dict(state_dict, strict=True)
    unet.requires_grad_(False)
    # UNet weights in the compute dtype; UnZipLoRA params stay fp32 like the reference (dtype=None)
    for name, p in unet.named_parameters():
        if "lora_layer" not in name:
            p.data = p.data.to(dtype)
    return unet.to(device)


def freeze_spatial_layers(unet, unfreeze_mergers: bool = False):
    """animatediff/utils.py:66-95."""
    for name, param in unet.named_parameters():
        if "motion_modules" in name:
            param.requires_grad_(not (".base.weight" in name or ".base.bias" in name))
        elif unfreeze_mergers and ("merge_content" in name or "merge_style" in name):
            param.requires_grad_(True)
        else:
            param.requires_grad_(False)


def _extract_merger_state_dicts(unet):
    mc, ms = {}, {}
    for name, module in unet.named_modules():
        if "motion_modules" in name:
            continue
        lora = getattr(module, "lora_layer", None)
        if lora is None or getattr(lora, "merge_content", None) is None:
            continue
        mc[f"unet.{name}.lora.merge_content"] = lora.merge_content.detach().cpu()
        ms[f"unet.{name}.lora.merge_style"] = lora.merge_style.detach().cpu()
    return mc, ms


def save_checkpoint(unet, output_dir: str, step, save_mergers: bool = False):
    """animatediff/utils.py:102-144: checkpoint-{step}/motion_modules.pth (temporal LoRA folded)."""
    from .temporal_lora import TemporalLoRALinear, get_merged_motion_state_dict
    path = os.path.join(output_dir, f"checkpoint-{step}")
    os.makedirs(path, exist_ok=True)
    if any(isinstance(m, TemporalLoRALinear) for m in unet.modules()):
        state = get_merged_motion_state_dict(unet)
    else:
        state = {k: v.cpu() for k, v in unet.state_dict().items() if "motion_modules" in k}
    torch.save(state, os.path.join(path, "motion_modules.pth"))
    if save_mergers:
        mc, ms = _extract_merger_state_dicts(unet)
        torch.save(mc, os.path.join(path, "merger_content_stage2.pth"))
        torch.save(ms, os.path.join(path, "merger_style_stage2.pth"))
    return path


# ---------------------------------------------------------------------------------------------------------
# Offline checkpoint formats: diffusers snapshots and the reference's motion_modules.pth
# ---------------------------------------------------------------------------------------------------------
def _load_tensor_file(path: str) -> Dict[str, torch.Tensor]:
    """safetensors, or a torch pickle read with weights_only=True (nothing in the file is executed)."""
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path, device="cpu")
    return torch.load(path, map_location="cpu", weights_only=True)


def load_diffusers_weights(path: str, stem: str = "diffusion_pytorch_model") -> Dict[str, torch.Tensor]:
    """State dict of a diffusers model folder (single file, fp16 variant, or a sharded index), or of a file."""
    if os.path.isfile(path):
        return _load_tensor_file(path)
    for name in (f"{stem}.safetensors", f"{stem}.fp16.safetensors", f"{stem}.bin", f"{stem}.fp16.bin"):
        p = os.path.join(path, name)
        if os.path.isfile(p):
            return _load_tensor_file(p)
    for name in (f"{stem}.safetensors.index.json", f"{stem}.safetensors.index.fp16.json", f"{stem}.bin.index.json"):
        p = os.path.join(path, name)
        if os.path.isfile(p):
            with open(p) as f:
                shards = sorted(set(json.load(f)["weight_map"].values()))
            sd = {}
            for sh in shards:
                sd.update(_load_tensor_file(os.path.join(path, sh)))
            return sd
    raise FileNotFoundError(f"no {stem} weights under {path}")


def unet_config_from_diffusers(unet_cfg: dict, adapter_cfg: Optional[dict] = None) -> UNetMotionConfig:
    """UNetMotionConfig from a diffusers UNet2DConditionModel config.json (+ MotionAdapter config.json).
    diffusers' SDXL config names the per-block head COUNT `attention_head_dim` ([5, 10, 20]); a
    `num_attention_heads` entry, when present, takes precedence (diffusers does the same)."""
    heads = unet_cfg.get("num_attention_heads") or unet_cfg.get("attention_head_dim")
    nb = len(unet_cfg["block_out_channels"])
    as_tuple = lambda v: tuple(v) if isinstance(v, (list, tuple)) else (v,) * nb  # noqa: E731
    motion = lambda t: t.replace("2D", "Motion")  # noqa: E731
    add_dim = unet_cfg.get("addition_time_embed_dim") or 256
    proj_in = unet_cfg.get("projection_class_embeddings_input_dim") or (1280 + 6 * add_dim)
    kw = dict(in_channels=unet_cfg.get("in_channels", 4), out_channels=unet_cfg.get("out_channels", 4),
              block_out_channels=tuple(unet_cfg["block_out_channels"]),
              down_block_types=tuple(motion(t) for t in unet_cfg["down_block_types"]),
              up_block_types=tuple(motion(t) for t in unet_cfg["up_block_types"]),
              layers_per_block=unet_cfg.get("layers_per_block", 2),
              transformer_layers_per_block=as_tuple(unet_cfg.get("transformer_layers_per_block", 1)),
              num_attention_heads=as_tuple(heads), cross_attention_dim=unet_cfg.get("cross_attention_dim", 2048),
              norm_num_groups=unet_cfg.get("norm_num_groups", 32), norm_eps=unet_cfg.get("norm_eps", 1e-5),
              addition_time_embed_dim=add_dim, num_time_ids=6, text_embed_dim=proj_in - 6 * add_dim)
    if adapter_cfg:
        kw.update(motion_num_attention_heads=adapter_cfg.get("motion_num_attention_heads", 8),
                  motion_max_seq_length=adapter_cfg.get("motion_max_seq_length", 32),
                  motion_norm_num_groups=adapter_cfg.get("motion_norm_num_groups", 32),
                  use_motion_mid_block=bool(adapter_cfg.get("use_motion_mid_block", False)))
    return UNetMotionConfig(**kw)


def _find_pth(path: str) -> Optional[str]:
    """animatediff/utils.py:56-63: a trained motion_modules.pth given directly or inside a directory."""
    if path.endswith(".pth") and os.path.isfile(path):
        return path
    if os.path.isdir(path):
        cand = os.path.join(path, "motion_modules.pth")
        if os.path.isfile(cand):
            return cand
    return None


def load_unet_with_motion(pretrained_model_name_or_path: str, motion_adapter_path: str,
                          torch_dtype: torch.dtype = torch.bfloat16, device: str = "cuda",
                          lora_rank: Optional[int] = None) -> Tuple[UNetMotionModel, Optional[int]]:
    """animatediff/utils.py:13-45 offline: SDXL `unet/` (config.json + weights) + the motion adapter folder,
    or a trained `motion_modules.pth` (then the architecture's default adapter config applies, as the reference's
    from_unet2d(base, None) does).  Returns (unet, motion_max_seq_length or None), like the reference."""
    base = os.path.join(pretrained_model_name_or_path, "unet")
    if not os.path.isdir(base):
        base = pretrained_model_name_or_path
    with open(os.path.join(base, "config.json")) as f:
        unet_cfg = json.load(f)
    pth = _find_pth(motion_adapter_path)
    adapter_cfg = None
    if pth is not None:
        motion_sd = _load_tensor_file(pth)
    else:
        with open(os.path.join(motion_adapter_path, "config.json")) as f:
            adapter_cfg = json.load(f)
        motion_sd = load_diffusers_weights(motion_adapter_path)
    cfg = unet_config_from_diffusers(unet_cfg, adapter_cfg)
    sd = load_diffusers_weights(base)
    sd.update({k: v for k, v in motion_sd.items() if "motion_modules" in k})
    unet = build_unet(cfg, state_dict=sd, lora_rank=lora_rank, device=device, dtype=torch_dtype, strict=False)
    return unet, (adapter_cfg.get("motion_max_seq_length") if adapter_cfg else None)
