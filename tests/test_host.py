"""CPU tests: C-ABI library loads and exports every declared symbol, architecture inventory,
scheduler tables vs the oracle, host-side LoRA/temporal-LoRA bookkeeping."""
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_header_symbols():
    from video_style_transfer_amd import _lib
    lib = _lib.load()
    hdr = open(os.path.join(ROOT, "include", "vst.h")).read()
    declared = set(re.findall(r"\b(vst_[a-z0-9_]+)\s*\(", hdr))
    assert declared, "no declarations parsed"
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.vst_version().startswith(b"vst-hip")


def test_calls_fail_loudly_on_cpu_tensors():
    from video_style_transfer_amd import _lib, kernels as K
    x = torch.zeros(4, 64, dtype=torch.bfloat16)
    with pytest.raises(_lib.VstError):
        K.linear(x, x)


def test_bad_arguments_rejected_without_gpu():
    from video_style_transfer_amd import _lib
    lib = _lib.load()
    # K not a multiple of 8 -> VST_ERR_ARG before any launch
    assert lib.vst_gemm(1, 8, None, 0, 0, 1, 8, 4, 4, 6, None, None, 1, 0, None, 0, 1, 8, 0, None) == 1
    assert lib.vst_temporal_attention(1, 1, 1, 8, 1, 8, 1, 64, 1, 8, 8, 1.0, None) == 1  # F > 32
    assert lib.vst_spatial_attention(1, 64, 1, 1, 64, 1, 64, 1, 1, 8, 8, 1, 40, 1.0, None, None) == 1  # head_dim != 64
    assert lib.vst_step_advance(1, 0, None) == 1  # empty schedule
    assert lib.vst_spatial_attention_bwd(1, 64, 1, 1, 64, 1, 64, 1, 64, None, 1, 64, None, None, 0, 1, 1, 8, 8, 1, 64,
                                         0.125, 1, None) == 1  # no lse


def test_gemm_lora_policy_without_gpu():
    """vst_gemm_lora_supported (host policy, no launch): the SDXL UnZipLoRA r=8 projections run the down-projection
    inside the 8-phase GEMM, whatever M is (whether the in-GEMM path is taken is shape-only, so a frame-sharded rank
    takes the unsharded forward's path; the tile width it returns may follow the grid's rounds); a shape where every
    tile width straddles two u blocks, or a rank wider than one block, is refused."""
    from video_style_transfer_amd import _lib
    lib = _lib.load()
    q = lib.vst_gemm_lora_supported
    assert q(8192, 1280, 1280, 32, 1280, 16) == 192   # to_out / attn2 q at 16x16
    assert q(8192, 3840, 1280, 64, 1280, 16) == 256   # attn1 q/k/v at 16x16
    assert q(32768, 640, 640, 32, 640, 16) == 320     # to_out at 32x32: two rounds -> the persistent 128x320 grid
    #   (the tile width may follow M; the k order, and so the bits, do not -- test_gemm_lora_persistent_bitwise)
    assert q(16384, 640, 640, 32, 640, 16) == 192     # ... one round at a 2-way frame shard: one workgroup per tile
    assert q(32768, 1920, 640, 64, 640, 16) == 320    # q/k boundary inside a 256-wide tile: 128x320 tiles
    assert q(32768, 1800, 640, 64, 600, 16) == 0      # every width straddles (600 wide, not a multiple of 320)
    assert q(8192, 1280, 1280, 32, 1280, 32) == 0     # r = 16 UnZipLoRA: 32 u columns per projection
    assert q(1024, 1280, 1280, 32, 1280, 16) == 192   # small grids too (shape-only decision)
    # attn2 as one launch (q projection + text cross-attention epilogue): 256-row tiles inside a frame, <= 80 keys
    xq = lib.vst_gemm_cross_attention_supported
    assert xq(8192, 1280, 1280, 1, 32, 1280, 16, 256, 77) == 1    # 16x16 level, UnZipLoRA r=8
    assert xq(8192, 1280, 1280, 0, 0, 0, 0, 256, 77) == 1         # no LoRA (configs[1])
    assert xq(32768, 640, 640, 1, 32, 640, 16, 1024, 77) == 1     # 32x32 level
    assert xq(8192, 1280, 1280, 1, 32, 1280, 16, 320, 77) == 0    # tiles would straddle frames
    assert xq(8192, 1280, 1280, 1, 32, 1280, 16, 256, 81) == 0    # more keys than the LDS holds
    # a refused shape returns status 3 from the launch entry as well, before touching the pointers
    assert lib.vst_gemm_lora(1, 1280, 1, 640, 64, 600, 16, 1, 704, 32768, 1800, 640, None, None, 0, 1, 1800,
                             None) == 3


@pytest.mark.parametrize("cfgname", ["tiny", "sdxl"])
def test_param_inventory_matches_module_tree(cfgname):
    from video_style_transfer_amd.config import UNetMotionConfig
    from video_style_transfer_amd.unet_motion import UNetMotionModel
    from video_style_transfer_amd.utils import attach_unziplora_layers
    from video_style_transfer_amd.weights import param_shapes
    cfg = getattr(UNetMotionConfig, cfgname)()
    with torch.device("meta"):
        unet = UNetMotionModel(cfg)
        attach_unziplora_layers(unet, 8)
    sd = unet.state_dict()
    inv = param_shapes(cfg, 8)
    assert set(sd) == set(inv), sorted(set(sd) ^ set(inv))[:10]
    for k, (shape, _) in inv.items():
        assert tuple(sd[k].shape) == tuple(shape), k
    # SDXL topology facts from SURVEY.md §3.A: 70 spatial transformer blocks (140 attention
    # modules, 560 LoRA-wrapped projections), 15 motion modules, 17 resnets
    blocks = {k.split(".attn1.")[0] for k in sd if ".attn1.to_q.weight" in k and "motion" not in k}
    motion = {k.split(".motion_modules.")[0] + k.split(".motion_modules.")[1][:2] for k in sd if ".motion_modules." in k}
    resnets = {k.rsplit(".conv1.", 1)[0] for k in sd if k.endswith("conv1.weight")}
    loras = [k for k in sd if k.endswith("lora_layer.merge_content")]
    if cfgname == "sdxl":
        assert len(blocks) == 70 and len(loras) == 560 and len(motion) == 15 and len(resnets) == 17


def test_attn_processor_surface():
    from video_style_transfer_amd.attention_processor import AnimateDiffAttnProcessor2_0, AttnProcessor2_0
    from video_style_transfer_amd.config import UNetMotionConfig
    from video_style_transfer_amd.unet_motion import UNetMotionModel
    with torch.device("meta"):
        unet = UNetMotionModel(UNetMotionConfig.tiny())
    procs = unet.attn_processors
    spatial = [k for k in procs if "motion_modules" not in k]
    motion = [k for k in procs if "motion_modules" in k]
    assert all(isinstance(procs[k], AnimateDiffAttnProcessor2_0) for k in spatial)
    assert all(isinstance(procs[k], AttnProcessor2_0) for k in motion)
    # the reference's processor swap (inference_animatediff.py:209-215) round-trips
    new = {n: (p if "motion_modules" in n else AnimateDiffAttnProcessor2_0()) for n, p in procs.items()}
    unet.set_attn_processor(new)
    assert unet.attn_processors.keys() == procs.keys()


def test_scheduler_matches_oracle():
    from oracle.unet import euler_schedule
    from video_style_transfer_amd.scheduler import EulerDiscreteScheduler
    s = EulerDiscreteScheduler()
    s.set_timesteps(50)
    ts, sig, init = euler_schedule(50)
    assert torch.equal(s.timesteps.float(), ts.float())
    assert torch.allclose(s.sigmas, sig, rtol=1e-6, atol=1e-7)
    assert abs(s.init_noise_sigma - init) < 1e-5
    assert s.timesteps[0] == 981 and s.timesteps[-1] == 1


def test_temporal_lora_bookkeeping_cpu():
    from video_style_transfer_amd.config import UNetMotionConfig
    from video_style_transfer_amd.temporal_lora import (TemporalLoRALinear, build_spatial_lora_index,
                                                        get_merged_motion_state_dict, inject_temporal_lora)
    from video_style_transfer_amd.unet_motion import UNetMotionModel
    from video_style_transfer_amd.utils import attach_unziplora_layers, freeze_spatial_layers
    unet = UNetMotionModel(UNetMotionConfig.tiny())
    attach_unziplora_layers(unet, 8)
    n = inject_temporal_lora(unet, rank=32, alpha=1.0)
    assert n == 15 * 2 * 4  # 15 motion modules x (attn1, attn2) x (q, k, v, out)
    assert inject_temporal_lora(unet) == 0  # idempotent
    idx = build_spatial_lora_index(unet)
    # motion module i of a cross-attn block pairs with attentions.i of the same block
    assert idx and all(".motion_modules." in k for k in idx)
    assert "down_blocks.1.motion_modules.0.transformer_blocks.0.attn1.to_q" in idx
    freeze_spatial_layers(unet)
    trainable = {n for n, p in unet.named_parameters() if p.requires_grad}
    assert all("motion_modules" in n for n in trainable)
    assert not any(".base." in n for n in trainable)
    merged = get_merged_motion_state_dict(unet)
    assert not any(".base." in k or "lora_A" in k for k in merged)
    assert "down_blocks.0.motion_modules.0.transformer_blocks.0.attn1.to_q.weight" in merged
    assert isinstance(unet.down_blocks[0].motion_modules[0].transformer_blocks[0].attn1.to_q, TemporalLoRALinear)


def test_orth_loss_lowrank_matches_dense():
    """compute_orth_loss evaluated low-rank equals the reference's dense formula."""
    from oracle.ref_ops import orth_loss
    from video_style_transfer_amd.config import UNetMotionConfig
    from video_style_transfer_amd.temporal_lora import build_spatial_lora_index, compute_orth_loss, inject_temporal_lora
    from video_style_transfer_amd.unet_motion import UNetMotionModel
    from video_style_transfer_amd.utils import attach_unziplora_layers
    torch.manual_seed(0)
    unet = UNetMotionModel(UNetMotionConfig.tiny())
    attach_unziplora_layers(unet, 8)
    inject_temporal_lora(unet, rank=32, alpha=1.0)
    for n, p in unet.named_parameters():
        if "lora_B" in n:
            p.data.normal_(0, 0.01)
    idx = build_spatial_lora_index(unet)
    got = compute_orth_loss(unet, idx, 0.1)
    pairs = []
    mods = dict(unet.named_modules())
    for name, lora in idx.items():
        m = mods[name]
        d = lora.lora_matrix_dic
        pairs.append((m.get_delta().detach(), d["content_down"].weight, d["content_up"].weight,
                      d["style_down"].weight, d["style_up"].weight))
    ref = orth_loss(pairs, 0.1)
    assert torch.allclose(got.detach(), ref, rtol=1e-4), (got, ref)


def test_gemm_kernel_policy_host_only():
    """vst_gemm_kernel_name is pure host logic: the tile / split-K / skinny choice for the UNet's shapes."""
    from video_style_transfer_amd import kernels as K
    name = K.gemm_kernel_name
    assert name(8192, 32, 1280, 0) == "gemm_skinny"            # UnZipLoRA down-projection
    assert name(131072, 320, 40, 3) == "gemm_kernel<conv_in>"  # Cin = 4 gather conv
    assert name(8192, 10240, 1280, 1) == "gemm_p8<256x256,geglu,persist>"  # GEGLU epilogue, persistent grid
    assert name(8192, 1280, 5120, 0) == "gemm_p8<256x192>"      # one round of tiles: one workgroup per tile
    assert name(2, 1280, 1280, 0) == "gemm_rows"                # temb projection: M = 2
    assert name(2, 13760, 1280, 0) == "gemm_rows"               # batched time_emb_proj of every resnet
    assert name(9, 1280, 1280, 0).endswith("splitk>")           # M > 8: split-K tiles
    assert name(131072, 320, 2880, 2).endswith("conv>")
    assert name(131072, 4, 2880, 2) == "gemm_ring<128x64,conv>"  # conv_out: Cout not a multiple of 64
    assert name(8192, 1280, 11520, 2) == "gemm_p8<128x320,conv>"  # 16^2 resnet conv: implicit im2col, 8-phase
    assert name(32768, 640, 5760, 2) == "gemm_p8<128x320,conv>"


def test_text_encoder_surface_cpu():
    """The SDXL text towers keep transformers' module tree / state-dict keys (a checkpoint's text_encoder and
    text_encoder_2 load unchanged, with or without the "text_model." prefix recent transformers drop), and refuse
    to run from CPU weights (no CPU fallback)."""
    import transformers
    from video_style_transfer_amd import _lib
    from video_style_transfer_amd import text_encoder as T
    for cfg, ours_cls, ref_cls in ((T.CLIPTextConfig.tiny(), T.CLIPTextModel, transformers.CLIPTextModel),
                                   (T.CLIPTextConfig.tiny("gelu"), T.CLIPTextModelWithProjection,
                                    transformers.CLIPTextModelWithProjection)):
        tc = transformers.CLIPTextConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                                         intermediate_size=cfg.intermediate_size,
                                         num_hidden_layers=cfg.num_hidden_layers,
                                         num_attention_heads=cfg.num_attention_heads, hidden_act=cfg.hidden_act,
                                         projection_dim=cfg.projection_dim, eos_token_id=2, bos_token_id=0)
        sd = ref_cls(tc).state_dict()
        model = T.build_text_encoder(ours_cls, cfg, state_dict=sd, device="cpu")
        ours = {k if k.startswith(("text_model.", "text_projection")) else "text_model." + k for k in sd}
        assert ours == set(model.state_dict())
        with pytest.raises(_lib.VstError):
            model(torch.zeros(1, 77, dtype=torch.long))


def test_colstat_registry_host_logic():
    """kernels.colstat_of (the GroupNorm column-statistics hand-off, opt-in VST_GN_COLSTAT): an entry is valid only
    for the very tensor its conv wrote -- same storage, shape and strides, not modified since, still alive -- and
    colstat_reset() drops every entry (each UNet forward starts with it)."""
    import weakref
    from video_style_transfer_amd import kernels as K
    K.colstat_reset()
    out = torch.zeros(256, 320, dtype=torch.bfloat16)
    cs = torch.zeros(2, 320, 2)
    K._COLSTAT[out.data_ptr()] = (weakref.ref(out), out._version, cs)
    assert K.colstat_of(out) is cs
    assert K.colstat_of(out.view(128, 640)) is None          # another shape over the same storage
    assert K.colstat_of(out[:, :160]) is None                # a column slice (other strides)
    assert K.colstat_of(None) is None
    out.add_(1)                                              # modified after the conv wrote it
    assert K.colstat_of(out) is None
    K._COLSTAT[out.data_ptr()] = (weakref.ref(out), out._version, cs)
    assert K.colstat_of(out) is cs
    K.colstat_reset()
    assert K.colstat_of(out) is None
    # a raw-pointer write into the tensor (a K.* wrapper given out=, which does not bump _version) drops the entry
    K._COLSTAT[out.data_ptr()] = (weakref.ref(out), out._version, cs)
    K._wrote(out)
    assert K.colstat_of(out) is None
    K._COLSTAT[out.data_ptr()] = (weakref.ref(out), out._version, cs)
    with pytest.raises(K._lib.VstError):                     # _dev(out, ...) drops it too (then refuses the CPU tensor)
        K._dev(out, torch.bfloat16, "out")
    assert K.colstat_of(out) is None
