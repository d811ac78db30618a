"""bench.py's roofline bookkeeping on synthetic launch records (CPU): the dominant kernel's rate, the per-shape view
of the fused base + UnZipLoRA GEMMs and attn2, and each shape's binding roof (MFMA floor vs HBM floor)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_roofline_bounds_per_shape():
    M, N, K, r = 32768, 640, 640, 16
    fl = 2.0 * M * N * (K + r) + 2.0 * M * K * r
    nb = 2.0 * (M * K + N * (K + r) + r * K + 2 * M * N)  # x, w, a, residual + output
    M2, N2, K2 = 8192, 3840, 1280
    fl2 = 2.0 * M2 * N2 * (K2 + r) + 2.0 * M2 * K2 * r * 3
    nb2 = 2.0 * (M2 * K2 + N2 * (K2 + r) + M2 * N2)
    rec = [("gemm_lora", "gemm_p8<256x192,lora>", fl, nb, 0.048, (M, N, K + 32)) for _ in range(2)]
    rec += [("gemm_lora", "gemm_p8<256x256,lora>", fl2, nb2, 0.080, (M2, N2, K2 + 64))]
    rec += [("gemm_xattn", "gemm_p8<256x192,lora,xattn>", fl2 / 3, nb2 / 3, 0.043, (8192, 1280, 1312))]
    rl, table = bench._roofline_from(rec, step_ms=None)
    assert rl["kernel"] == "gemm_p8<256x192,lora>"  # the largest summed time (2 x 48 us)
    v = rl["fused_lora_gemms"]
    out = v["32768x640x672"]
    assert out["launches"] == 2 and out["bound"] == "hbm"  # 126 MB against 28 GF: below the 312 flop/B ridge
    assert abs(out["floor_us"] - nb / 8e12 * 1e6) < 0.01
    assert abs(out["roof_frac"] - out["floor_us"] / 48.0) < 1e-3
    qkv = v["8192x3840x1344"]
    assert qkv["bound"] == "mfma" and abs(qkv["frac"] - fl2 / 80e-6 / 2.5e15) < 1e-3
    assert "8192x1280x1312 xattn" in v
    assert set(table) == {"gemm_p8<256x192,lora>", "gemm_p8<256x256,lora>", "gemm_p8<256x192,lora,xattn>"}
