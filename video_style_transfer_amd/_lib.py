"""ctypes binding of libvst_hip.so (the C ABI declared in include/vst.h).

This is the only place the shared library is touched.  There is deliberately no CPU or
PyTorch fallback: if the library is missing, or a tensor is not on a HIP device, the call
raises.  (The reference path is PyTorch eager; our kernels replace it, they do not wrap it.)
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libvst_hip.so")

# name -> (restype, argtypes)
_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_S = ctypes.c_size_t
SIGNATURES = {
    "vst_gemm": (_I, [_P, _I, _P, _I, _I, _P, _I, _I, _I, _I, _P, _P, _I, _I, _P, _I, _P, _I, _I, _P]),
    "vst_gemm_ex": (_I, [_P, _I, _P, _I, _I, _P, _I, _I, _I, _I, _P, _P, _I, _I, _P, _I, _P, _I, _I, _I, _I, _P, _S,
                         _P]),
    "vst_gemm_workspace_bytes": (_S, [_I, _I, _I]),
    "vst_gemm_lora": (_I, [_P, _I, _P, _I, _I, _I, _I, _P, _I, _I, _I, _I, _P, _P, _I, _P, _I, _P]),
    "vst_gemm_lora_supported": (_I, [_I, _I, _I, _I, _I, _I]),
    "vst_gemm_cross_attention": (_I, [_P, _I, _P, _I, _I, _I, _I, _P, _I, _P, _I, _I, _I, _P, _P, _I, _I, _I, _I, _I,
                                      _F, _P, _I, _P]),
    "vst_gemm_cross_attention_supported": (_I, [_I, _I, _I, _I, _I, _I, _I, _I, _I]),
    "vst_gemm_temporal_attention": (_I, [_P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _F, _P, _I, _P]),
    "vst_gemm_temporal_attention_supported": (_I, [_I, _I, _I, _I, _I, _I, _I]),
    "vst_gemm_kernel_name": (ctypes.c_char_p, [_I, _I, _I, _I, _I, _I, _S]),
    "vst_conv3x3": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _I, _P, _I, _P, _P, _I, _P, _I, _P, _I, _P]),
    "vst_conv3x3_ex": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _I, _P, _I, _P, _P, _I, _I, _P, _I, _P, _I, _I, _I, _P,
                            _S, _P]),
    "vst_spatial_attention": (_I, [_P, _I, _P, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _F, _P, _P]),
    "vst_temporal_attention": (_I, [_P, _P, _P, _I, _P, _I, _I, _I, _I, _I, _I, _F, _P]),
    "vst_motion_attention_block": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _F, _P, _P, _I, _P, _P, _I, _P, _F, _P, _I,
                                        _P]),
    "vst_motion_attention_block_supported": (_I, [_I, _I, _I, _I]),
    "vst_groupnorm_workspace_bytes": (_S, [_I, _I, _I, _I]),
    "vst_groupnorm_frame_chunks": (_I, [_I]),
    "vst_p8_force_bn": (_I, [_I]),
    "vst_p8_conv": (_I, [_I]),
    "vst_p8_persist": (_I, [_I]),
    "vst_sa_self": (_I, [_I]),
    "vst_groupnorm_frame_partials": (_I, [_P, _I, _I, _I, _I, _I, _P, _P]),
    "vst_groupnorm_apply_partials": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _I, _F, _P, _P, _I, _P, _I, _P, _P]),
    "vst_permute_rows": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "vst_groupnorm": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _F, _P, _P, _I, _P, _I, _P, _P]),
    "vst_colstat": (_I, [_P, _I, _I, _I, _P, _P]),
    "vst_groupnorm_colstat": (_I, [_P, _I, _I, _P, _P, _I, _I, _P, _I, _I, _I, _F, _P, _P, _I, _P, _I, _P, _P]),
    "vst_conv3x3_colstat": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _I, _P, _I, _P, _P, _I, _I, _P, _I, _P, _I, _P,
                                 _P]),
    "vst_layernorm_lora": (_I, [_P, _I, _I, _I, _P, _P, _F, _P, _I, _P, _I, _P, _I, _P]),
    "vst_layernorm": (_I, [_P, _I, _I, _I, _P, _P, _F, _P, _I, _I, _P, _I, _P]),
    "vst_add_row_table": (_I, [_P, _I, _I, _I, _P, _I, _I, _P, _I, _P]),
    "vst_unpack_tokens": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "vst_timestep_embedding": (_I, [_P, _P, _I, _I, _I, _F, _P, _I, _I, _I, _P]),
    "vst_pack_latents": (_I, [_P, _I, _I, _I, _I, _P, _P, _F, _I, _P, _P]),
    "vst_euler_cfg_step": (_I, [_P, _I, _F, _P, _I, _I, _I, _I, _P, _P, _P]),
    "vst_step_advance": (_I, [_P, _I, _P]),
    "vst_silu": (_I, [_P, _P, _S, _P]),
    "vst_add": (_I, [_P, _P, _P, _S, _P]),
    "vst_quick_gelu": (_I, [_P, _P, _S, _P]),
    "vst_embed_tokens": (_I, [_P, _I, _I, _P, _P, _I, _P, _I, _P]),
    "vst_causal_attention": (_I, [_P, _I, _P, _P, _I, _P, _I, _I, _I, _I, _I, _F, _P]),
    "vst_residual_layernorm": (_I, [_P, _I, _P, _I, _I, _I, _P, _P, _F, _P, _I, _P, _I, _P]),
    "vst_copy2d": (_I, [_P, _I, _P, _I, _I, _I, _P]),
    "vst_transpose": (_I, [_P, _I, _I, _I, _P, _I, _P]),
    "vst_layernorm_bwd_workspace_bytes": (_S, [_I, _I]),
    "vst_layernorm_bwd": (_I, [_P, _I, _P, _I, _I, _I, _P, _F, _P, _I, _P, _P, _P, _P]),
    "vst_geglu_bwd": (_I, [_P, _I, _P, _I, _I, _I, _P, _I, _P]),
    "vst_colsum_workspace_bytes": (_S, [_I, _I]),
    "vst_colsum": (_I, [_P, _I, _I, _I, _P, _P, _P]),
    "vst_groupnorm_bwd_workspace_bytes": (_S, [_I, _I, _I, _I]),
    "vst_groupnorm_bwd": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _F, _P, _P, _I, _P, _I, _P, _P, _P, _P]),
    "vst_spatial_attention_bwd_workspace_bytes": (_S, [_I, _I, _I, _I]),
    "vst_spatial_attention_bwd": (_I, [_P, _I, _P, _P, _I, _P, _I, _P, _I, _P, _P, _I, _P, _P, _I, _I, _I, _I, _I, _I,
                                       _I, _F, _P, _P]),
    "vst_zero_insert": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "vst_sumpool2x2": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "vst_temporal_attention_bwd": (_I, [_P, _P, _P, _I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _P]),
    "vst_conv3x3_down_pad0": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _P, _I, _P, _S, _P]),
    "vst_gemm_f32out": (_I, [_P, _I, _P, _I, _I, _I, _I, _P, _P]),
    "vst_gemm_tn": (_I, [_P, _I, _P, _I, _I, _I, _I, _P, _I, _P, _S, _P]),
    "vst_gemm_tn_workspace_bytes": (_S, [_I, _I, _I]),
    "vst_softmax_rows": (_I, [_P, _I, _I, _I, _F, _P, _I, _P]),
    "vst_nchw_to_nhwc": (_I, [_P, _I, _I, _I, _F, _P, _I, _P]),
    "vst_nhwc_to_nchw": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "vst_frames_to_u8": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "vst_vae_sample": (_I, [_P, _I, _I, _I, _P, _F, _P, _P]),
    "vst_probe_mfma": (_I, [_I, _I, _P, _P]),
    "vst_probe_hbm_read": (_I, [_P, _S, _I, _P, _P]),
    "vst_probe_fetch": (_I, [_I, _P, _I, _I, _I, _P, _P]),
    "vst_probe_mix": (_I, [_I, _I, _P, _I, _I, _I, _P, _P]),
    "vst_version": (ctypes.c_char_p, []),
}

_lib = None


class VstError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load the HIP library (idempotent).  Raises VstError when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    alt = os.environ.get("VST_LIB_AB")  # diagnostics only (tools/gemm_ablate.py A/B of two builds)
    path = path or alt or LIB_PATH
    if not os.path.exists(path):
        raise VstError(f"libvst_hip.so not found at {path}; build it with `make` (hipcc --offload-arch=gfx950)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if alt and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols() -> list[str]:
    return list(SIGNATURES)


def call(name: str, *args):
    rc = getattr(load(), name)(*args)
    if rc != 0:
        why = {1: "bad argument", 2: "launch failure", 3: "unsupported shape"}.get(rc, "error")
        raise VstError(f"{name} failed with status {rc} ({why})")
    return rc
