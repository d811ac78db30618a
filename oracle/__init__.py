"""ORACLE — TEST INFRASTRUCTURE ONLY.

A CPU, fp32, PyTorch-eager restatement of the reference algorithm for the AnimateDiff-XL +
UnZipLoRA denoising path (tanmud/video_style_transfer).  Every function cites the reference
file:line it follows.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg may import this package, and only as the checker / CPU baseline; the
product package (`video_style_transfer_amd`) never imports it and has no CPU fallback.

Pinning:
  * pinned against golden vectors produced by importing the reference's own torch-only
    modules in the build container (tests/golden/make_golden.py -> tests/golden/*.safetensors):
    UnZipLoRALinearLayerInfer, LoRACompatibleLinear, AnimateDiffAttnProcessor2_0 (spatial
    self/cross and the frame-axis core), TemporalTransformer / PositionalEncoding,
    TemporalLoRALinear, compute_orth_loss, get_merged_motion_state_dict;
  * the diffusers-owned pieces (UNetMotionModel glue, ResnetBlock2D, Transformer2DModel,
    motion module AnimateDiffTransformer3D, EulerDiscreteScheduler) are restated from the
    public diffusers ~0.30 semantics the reference depends on (diffusers is not vendored in
    the reference and not installed here): PARITY UNPINNED for those glue pieces beyond the
    attention core and the sinusoidal PE, which are pinned through the reference modules.
"""
