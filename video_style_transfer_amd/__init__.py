"""MI355X-native AnimateDiff-XL + UnZipLoRA denoising path (drop-in for tanmud/video_style_transfer).

Host side: PyTorch-ROCm modules mirroring the reference's plug-in surface.  Compute: the
hand-written gfx950 HIP kernels in libvst_hip.so (C ABI: include/vst.h), loaded via ctypes.
"""
__version__ = "0.1.0"
