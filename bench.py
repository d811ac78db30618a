#!/usr/bin/env python3
"""Denoised frames/s of the AnimateDiff-XL (+UnZipLoRA r=8) 50-step CFG denoise loop on MI355X.

Metric (BASELINE.json): denoised frames/sec, 16x512x512 clip, 50-step AnimateDiff-XL.
A "step" = one denoise step of the loop (inference_animatediff.py:105-131): scale_model_input ->
UNet forward of the CFG pair (batched, B=2) -> CFG combine -> Euler update; captured once as a HIP
graph and replayed.  value = frames / (50 steps x mean step time) — the rate at which whole clips
are produced; weights are seeded synthetic SDXL + AnimateDiff-SDXL motion + UnZipLoRA r=8 (no
checkpoints offline), text embeddings synthetic N(0,1).

  python bench.py [--gpus N --steps K --warmup W] [--frames 16 --size 512 --lora-rank 8 --lora-mode fused]
N>1 (torch.distributed.run, one rank per GPU): see --parallel.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table; no sparsity)
PEAK_HBM_GBS = 8000.0
HBM_MEASURED_GBS = 6300.0       # vst_probe_hbm_read / MI355X_MICROARCH.md ("6.29 TB/s measured")
MFMA_MEASURED_TFLOPS = 2440.0   # vst_probe_mfma

KERNEL_OF_KIND = {  # non-GEMM kinds; GEMM/conv launches carry the library's own kernel name
    "spatial_attention": "spatial_attn_kernel",
    "temporal_attention": "temporal_attn_kernel",
    "groupnorm": "gn_stats/gn_finalize/gn_apply",
    "layernorm": "layernorm_kernel",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--lora-rank", type=int, default=8)
    ap.add_argument("--lora-mode", default="fused", choices=["fused", "folded"])
    ap.add_argument("--num-inference-steps", type=int, default=50)
    ap.add_argument("--guidance", type=float, default=7.5)
    ap.add_argument("--parallel", default="frames", choices=["frames", "replicas"],
                    help="N>1: 'frames' shards the frames of every clip over the ranks (all-to-all around each "
                         "motion module, frame_shard.py); 'replicas' runs an independent clip per rank")
    ap.add_argument("--exchange", default="all_to_all", choices=["all_to_all", "all_gather"],
                    help="frames mode: the motion modules' exchange; all_to_all (default: frame shard <-> pixel shard, "
                         "no duplicated work) or all_gather (the north star's: every rank gathers the clip and runs the "
                         "module over all frames)")
    ap.add_argument("--clips", type=int, default=0,
                    help="frames mode: clips denoised together (default N: per-GPU work fixed at one clip's "
                         "frames = weak scaling; 1 = one clip split N ways = strong scaling); N=1 or replicas: "
                         "clips batched per GPU (throughput mode, not the headline)")
    ap.add_argument("--strong-record", default="auto", choices=["auto", "on", "off"],
                    help="frames mode, N>1: also time ONE --frames clip split over the N ranks (strong scaling) and "
                         "report it under sub_records.strong_1clip (auto: whenever the headline has more than 1 clip)")
    ap.add_argument("--configs3", default="auto", choices=["auto", "on", "off"],
                    help="frames mode, N>1: also time BASELINE configs[3] (one --configs3-frames x --configs3-size^2 "
                         "clip frame-sharded over the ranks) under sub_records.configs3 (auto: at N=8)")
    ap.add_argument("--gather-record", default="auto", choices=["auto", "on", "off"],
                    help="frames mode, N>1, --exchange all_to_all: also time the headline workload with the north "
                         "star's exchange (an all-gather of the clip before each motion module) under "
                         "sub_records.all_gather (auto: whenever N>1)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="frames mode, all_to_all: run each motion module's exchange as one blocking collective "
                         "(default: the CFG pair in two halves whose all-to-alls overlap the other half's compute)")
    ap.add_argument("--configs3-frames", type=int, default=32)
    ap.add_argument("--configs3-size", type=int, default=768)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-peaks", action="store_true", help="skip the MFMA / HBM ceiling probes")
    ap.add_argument("--cpu-sample-frames", type=int, default=2)
    ap.add_argument("--no-vae", action="store_true", help="skip the VAE decode record (denoise) / the per-step VAE "
                    "encode of the training frames (--train: the step then starts from synthetic latents)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--train", action="store_true",
                    help="BASELINE configs[4]: one train_animatediff.py optimizer step per rank (fwd+bwd on "
                         "--grad-accum 16-frame clips, orth loss, clip_grad_norm_, AdamW, cosine lr; RCCL gradient "
                         "all-reduce for N>1) instead of the denoise loop")
    ap.add_argument("--grad-accum", type=int, default=4,
                    help="--train: gradient_accumulation_steps (train_animatediff.py:395, default 4): clips per rank "
                         "per optimizer step")
    ap.add_argument("--sequential-accum", action="store_true",
                    help="--train: one forward / backward per clip (the reference's loop shape) instead of the whole "
                         "accumulation window batched (TrainStep.window; same gradient)")
    return ap.parse_args()


def _lib_md5():
    import hashlib
    from video_style_transfer_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.md5(f.read()).hexdigest()


def src_hash():
    """sha256 over the library's sources and build recipe (csrc/*.hip, *.h, include/vst.h, Makefile): the hipcc
    build is deterministic, so equal hashes mean the same libvst_hip.so even after a rebuild."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "video_style_transfer_amd", "csrc", "*")))
    files += [os.path.join(ROOT, "include", "vst.h"), os.path.join(ROOT, "Makefile")]
    for fn in files:
        with open(fn, "rb") as f:
            h.update(os.path.basename(fn).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def pmc_traffic(symbol):
    """HBM bytes per launch of `symbol` from the profiles/pmc_traffic_*.json (tools/pmc_traffic.py: rocprofv3
    FETCH_SIZE / WRITE_SIZE passes with the gfx950 corrections) that was measured on this exact libvst_hip.so
    (same md5, or same source hash); the newest such file wins.  (bytes, source) or (None, reason)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic_*.json")), key=os.path.getmtime)
    if not files:
        return None, "no PMC profile"
    md5, sh = _lib_md5(), src_hash()
    for fn in reversed(files):
        with open(fn) as f:
            d = json.load(f)
        if d.get("lib_md5") != md5 and d.get("src_hash") != sh:
            continue
        k = d.get("kernels", {}).get(symbol)
        if k is None:
            return None, f"{symbol} not in {os.path.basename(fn)}"
        return k["traffic_bytes"], os.path.basename(fn)
    return None, "no PMC profile of this build of libvst_hip.so"


def _gpu_busy(ms):
    """Keep the stream busy for ~`ms` (torch.cuda._sleep, calibrated once), so the host can enqueue a whole
    instrumented step behind it: the step's launches then run back to back as in the graph replay, and an event
    interval measures its kernel, not the host's enqueue gap before it (tiny kernels were inflated 2-3x by those)."""
    global _SLEEP_CYC_PER_MS
    if _SLEEP_CYC_PER_MS is None:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1000)  # warm-up
        a.record()
        torch.cuda._sleep(10_000_000)
        b.record()
        torch.cuda.synchronize()
        _SLEEP_CYC_PER_MS = 10_000_000 / max(a.elapsed_time(b), 1e-3)
    torch.cuda._sleep(int(ms * _SLEEP_CYC_PER_MS))


_SLEEP_CYC_PER_MS = None


def roofline(den, step_ms=None):
    """One instrumented eager step: HIP events around every launch on its stream, enqueued behind a ~0.4 s busy
    kernel so the launches execute back to back (their sum is then comparable with the replayed step)."""
    from video_style_transfer_amd import kernels as K
    den.step_idx.zero_()
    torch.cuda.synchronize()
    _gpu_busy(400.0)
    K.profile_launches(True)
    den._step()
    rec = K.collect_launches()
    K.profile_launches(False)
    den.step_idx.zero_()
    return _roofline_from(rec, step_ms)


def _roofline_from(rec, step_ms=None):
    """Group instrumented launches by kernel symbol; the dominant kernel's achieved rate against its roofline.
    The per-kernel event intervals of the eager step also hold each launch's dispatch gap, so they sum to more than the
    replayed step; the `kernels` table is scaled to the replayed step (`step_ms`) when it does (factor in
    `table_scale`), while the dominant kernel's rate uses its raw event time (the conservative side)."""
    by = {}
    shapes = {}
    for kind, sym, fl, nb, ms, shape in rec:
        sym = sym or KERNEL_OF_KIND.get(kind, kind)
        if shape is not None:
            d = shapes.setdefault(f"{kind} {shape[0]}x{shape[1]}x{shape[2]} {sym}", [0, 0.0, 0.0, 0.0])
            d[0] += 1
            d[1] += ms
            d[2] += fl
            d[3] += nb
        d = by.setdefault(sym, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
        d["launches"] += 1
        d["ms"] += ms
        d["flops"] += fl
        d["bytes"] += nb
    total_ms = sum(d["ms"] for d in by.values())
    scale = min(1.0, step_ms / total_ms) if step_ms else 1.0
    if os.environ.get("VST_BENCH_SHAPES"):
        for key, (n, ms, fl, nb) in sorted(shapes.items(), key=lambda kv: -kv[1][1]):
            # the shape's own roofline floor: MFMA (flops / 2.5 PF) or HBM (algorithmic bytes / 8 TB/s), whichever is
            # longer, and the fraction of it this launch reaches
            t_mfma, t_hbm = fl / (PEAK_BF16_TFLOPS * 1e12), nb / (PEAK_HBM_GBS * 1e9)
            print(f"[shape] {ms:8.3f} ms {n:4d}x {fl / (ms * 1e-3) / 1e12:7.1f} TF {nb / (ms * 1e-3) / 1e9:7.1f} GB/s "
                  f"{'mfma' if t_mfma >= t_hbm else 'hbm ':4s} roof {max(t_mfma, t_hbm) / (ms * 1e-3):.3f}  {key}",
                  file=sys.stderr)
    # north-star view: the fused base + UnZipLoRA projection GEMMs (q/k/v, out) and attn2 (to_q + UnZipLoRA + the
    # text attention) per shape.  frac is against the 2.5 PF MFMA peak (the north star's measure); each entry also
    # carries its roofline bound: the MFMA time floor (flops / 2.5 PF) against the HBM floor (algorithmic bytes /
    # 8 TB/s, and at the measured 6.3 TB/s) -- the 32^2 out-projection moves more bytes than its flops cover
    lora = {}
    for key, (n, ms, fl, nb) in shapes.items():
        kind = key.split()[0]
        if kind in ("gemm_lora", "gemm_xattn"):
            per = ms / n * 1e3  # us per launch
            t_mfma = fl / n / (PEAK_BF16_TFLOPS * 1e12) * 1e6
            t_hbm = nb / n / (PEAK_HBM_GBS * 1e9) * 1e6
            t_hbm_meas = nb / n / (HBM_MEASURED_GBS * 1e9) * 1e6
            name = key.split()[1] + (" xattn" if kind == "gemm_xattn" else "")
            lora[name] = {"launches": n, "ms_per_step": round(ms, 3), "us_per_launch": round(per, 2),
                          "tflops": round(fl / (ms * 1e-3) / 1e12, 1),
                          "frac": round(fl / (ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
                          "alg_mb_per_launch": round(nb / n / 1e6, 1),
                          "bound": "mfma" if t_mfma >= t_hbm else "hbm",
                          "floor_us": round(max(t_mfma, t_hbm), 2),
                          "roof_frac": round(max(t_mfma, t_hbm) / per, 4),
                          "roof_frac_measured_hbm": round(max(t_mfma * PEAK_BF16_TFLOPS / MFMA_MEASURED_TFLOPS,
                                                              t_hbm_meas) / per, 4)}
    dom_sym, dom = max(by.items(), key=lambda kv: kv[1]["ms"])
    mfma = dom["flops"] > 0
    if mfma:
        achieved = dom["flops"] / (dom["ms"] * 1e-3) / 1e12
        peak, unit = PEAK_BF16_TFLOPS, "TFLOP/s"
    else:
        achieved = dom["bytes"] / (dom["ms"] * 1e-3) / 1e9
        peak, unit = PEAK_HBM_GBS, "GB/s"
    table = {}
    for sym, d in sorted(by.items(), key=lambda kv: -kv[1]["ms"]):
        ms = d["ms"] * scale
        table[sym] = {"launches": d["launches"], "ms_per_step": round(ms, 3), "event_ms_per_step": round(d["ms"], 3),
                      "share": round(d["ms"] / total_ms, 4),
                      "tflops": round(d["flops"] / (ms * 1e-3) / 1e12, 1) if d["flops"] else None,
                      "gbs": round(d["bytes"] / (ms * 1e-3) / 1e9, 1)}
    traffic, tsrc = pmc_traffic(dom_sym)
    step_flops = sum(d["flops"] for d in by.values())
    return {
        "bound": "mfma" if mfma else "hbm", "kernel": dom_sym, "achieved": round(achieved, 1), "peak": peak,
        "unit": unit, "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_source": tsrc,
        "alg_bytes_per_launch": round(dom["bytes"] / dom["launches"]),
        "avg_launch_ms": round(dom["ms"] / dom["launches"], 4),
        "flops_per_launch": dom["flops"] / dom["launches"],
        "kernel_time_ms_per_step": round(total_ms * scale, 3),
        "event_kernel_time_ms_per_step": round(total_ms, 3), "table_scale": round(scale, 4),
        "fused_lora_gemms": lora,
        "step_flops": step_flops,
    }, table


def measured_peaks(dev, rl):
    """Measured ceilings (vst_probe_mfma / vst_probe_hbm_read) next to the vendor peaks, and the dominant
    kernel's fraction of the measured one (report both)."""
    from video_style_transfer_amd import kernels as K
    mf = K.probe_mfma_tflops(dev)
    hb = K.probe_hbm_read_gbs(dev)
    meas = mf if rl["bound"] == "mfma" else hb
    return {"mfma_bf16_tflops": round(mf, 1), "hbm_read_gbs": round(hb, 1),
            "frac_of_measured": round(rl["achieved"] / meas, 4),
            "probes": "vst_probe_mfma: 1024 WGs x 8 waves x 16 independent 16x16x32 bf16 chains; "
                      "vst_probe_hbm_read: 4 GiB streamed with 16-B non-temporal loads"}


def vae_decode_timing(args, den, dev, ms_step):
    """The clip's VAE decode after the loop (inference_animatediff.py:137-144; outside the metric):
    SDXL AutoencoderKL (synthetic weights) decoding this rank's frames to uint8, timed over 3 runs, with its
    algorithmic flops from the instrumented launches and the end-to-end rate (50 denoise steps + decode)."""
    from video_style_transfer_amd import kernels as K
    from video_style_transfer_amd.config import VAEConfig
    from video_style_transfer_amd.vae import build_vae
    vae = build_vae(VAEConfig.sdxl(), seed=args.seed, device=dev)
    frames = den.decode(vae)  # warm-up (weight layouts, workspaces)
    K.profile_launches(True)
    den.decode(vae)
    fl = sum(r[2] for r in K.collect_launches())
    K.profile_launches(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        frames = den.decode(vae)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 3 * 1e3
    n = frames.shape[0]
    del vae
    torch.cuda.empty_cache()
    return {"ms_per_clip": round(ms, 2), "frames": n, "frames_per_s": round(n / (ms * 1e-3), 2),
            "alg_tflop": round(fl / 1e12, 2), "tflops": round(fl / (ms * 1e-3) / 1e12, 1),
            "frac": round(fl / (ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4), "output": list(frames.shape[1:]),
            "end_to_end_frames_per_s": round(n / (args.num_inference_steps * ms_step * 1e-3 + ms * 1e-3), 4),
            "note": "SDXL VAE decode to uint8 frames (bf16, frames batched); not part of the denoise metric"}


def cpu_baseline(args, cfg):
    """Oracle (fp32 CPU restatement) timed on a bounded sample: one UNet forward (one CFG branch)
    of a `cpu_sample_frames`-frame clip at the bench resolution; extrapolated to frames/s of the
    50-step CFG loop = frames / (2 * steps * t_forward)."""
    from oracle.unet import unet_forward
    from video_style_transfer_amd.weights import synthetic_state_dict
    threads = _cpu_threads()
    torch.set_num_threads(threads)
    sd = synthetic_state_dict(cfg, args.seed, args.lora_rank or None)
    fr, h = args.cpu_sample_frames, args.size // 8
    g = torch.Generator().manual_seed(1)
    lat = torch.randn(1, 4, fr, h, h, generator=g)
    enc = torch.randn(1, 77, cfg.cross_attention_dim, generator=g)
    pooled = torch.randn(1, cfg.text_embed_dim, generator=g)
    tids = torch.tensor([[args.size, args.size, 0, 0, args.size, args.size]], dtype=torch.float32)
    with torch.no_grad():
        t0 = time.perf_counter()
        unet_forward(sd, cfg.to_dict(), lat, torch.tensor([981.0]), enc, pooled, tids)
        dt = time.perf_counter() - t0
    del sd
    fps = fr / (2 * args.num_inference_steps * dt)
    return {"value": fps, "unit": "frames/s", "cores": threads, "kind": "port", "cpu": _cpu_model(), **_cpu_share(),
            "sample": f"1 UNet forward (one CFG branch) of a {fr}-frame {args.size}x{args.size} clip, fp32, "
                      f"{dt:.2f}s, extrapolated x{2 * args.num_inference_steps} forwards"}


def train_cpu_baseline(args, cfg):
    """Oracle (fp32 CPU restatement) forward + backward of the trainable motion parameters on a bounded sample
    (`cpu_sample_frames` frames at the bench resolution), extrapolated to training frames/s."""
    from oracle.unet import unet_forward
    from video_style_transfer_amd.weights import synthetic_state_dict
    threads = _cpu_threads()
    torch.set_num_threads(threads)
    sd = synthetic_state_dict(cfg, args.seed, args.lora_rank or None)
    for k, v in sd.items():
        v.requires_grad_("motion_modules" in k and not k.endswith(".pe"))
    fr, h = args.cpu_sample_frames, args.size // 8
    g = torch.Generator().manual_seed(1)
    lat = torch.randn(1, 4, fr, h, h, generator=g)
    enc = torch.randn(1, 77, cfg.cross_attention_dim, generator=g)
    pooled = torch.randn(1, cfg.text_embed_dim, generator=g)
    tids = torch.tensor([[args.size, args.size, 0, 0, args.size, args.size]], dtype=torch.float32)
    t0 = time.perf_counter()
    pred = unet_forward(sd, cfg.to_dict(), lat, torch.tensor([501.0]), enc, pooled, tids)
    ((pred - torch.randn_like(pred)) ** 2).mean().backward()
    dt = time.perf_counter() - t0
    del sd
    return {"value": fr / dt, "unit": "frames/s", "cores": threads, "kind": "port", "cpu": _cpu_model(), **_cpu_share(),
            "sample": f"fp32 oracle forward + backward (motion-module parameters trainable) of a {fr}-frame "
                      f"{args.size}x{args.size} clip: {dt:.2f}s"}


def _cpu_threads():
    """Host threads for the CPU baseline: this GPU's share of the box's cores.  The GPU box gives each GPU a 16-core
    share and exports OMP_NUM_THREADS=16 for it (the machine's other cores belong to the other GPUs' jobs); elsewhere
    every core this process may run on."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0"))
    return env or len(os.sched_getaffinity(0))


def _cpu_share():
    return {"host_cpus": os.cpu_count(), "cpus_allowed": len(os.sched_getaffinity(0)),
            "threads_note": "OMP_NUM_THREADS (this GPU's host-core share on the box) threads"}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


# Frame-sharded N-GPU runs, weak (clips == ranks, the driver's default) and strong (fewer clips than ranks, the
# sub-records) alike: every rank runs the unsharded forward's GEMM / norm kernels with a k order that does not depend on
# the row count (kernels.row_invariant), takes every shape-dependent fusion decision as the unsharded forward does
# under kernels.fusion_world(P), merges the motion GroupNorm's per-frame partials in the same order, and the exchange
# only moves rows -- so the sharded forward must equal the unsharded one bit for bit in both modes
# (tests/test_frame_shard.py: 2, 4 and 8 ranks on one GPU, configs[3]'s 8 x 4 frames of 32 x 768^2 included).
def _gather0(t, world, rank):
    """All ranks' equal-shaped tensors -> list on rank 0 (None elsewhere); staged through host memory on gloo."""
    import torch.distributed as dist
    staged = str(dist.get_backend()).lower() != "nccl"
    src = t.cpu() if staged else t.contiguous()
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src)
    return [p.to(t.device) for p in parts] if rank == 0 else None


def shard_preflight(den, unet, world, rank):
    """Before any timing of a frame-sharded N-GPU run: one eager sharded UNet forward of the step's CFG-batched
    input (the collectives included); every rank's noise prediction is gathered to rank 0 and compared with rank 0's
    unsharded forward of the same clips (all frames, the same CFG batch, so every text / embedding GEMM has the same
    row count on both sides).  Weak scaling must be bit-exact; returns {"rel_l2", "rel_max", "bitwise_equal"} on
    rank 0 (None elsewhere); the run fails on a mismatch."""
    from video_style_transfer_amd import kernels as K
    n, F, h, w = den.nclips, den.F, den.h, den.w
    B = den.ncopy * n
    den.step_idx.zero_()
    K.pack_latents(den.lat, den.x, sigmas=den.sigmas, step_idx=den.step_idx, ncopy=den.ncopy)
    emb = unet.embed(den.timesteps, den.pooled, den.time_ids, B, step_idx=den.step_idx)
    with torch.no_grad():
        noise = unet.forward_tokens(den.x, B, F, h, w, emb, den.enc, shard=den.shard)  # rows (b, f_local, p)
    rows = F * h * w
    parts = _gather0(noise, world, rank)
    lat_parts = _gather0(den.lat.contiguous(), world, rank)                              # (n, C, F_local, h, w)
    out, ok = None, True
    if rank == 0:
        Cl = den.lat.shape[1]
        got = torch.stack([p.view(B, F, h * w, -1) for p in parts], 1)                  # (b, rank, f_local, p)
        got = got.reshape(B * world * rows, -1)
        lat_full = torch.cat(lat_parts, 2).contiguous()                                  # (n, C, F_total, h, w)
        x = torch.empty(B * world * rows, Cl, dtype=torch.bfloat16, device=den.x.device)
        K.pack_latents(lat_full, x, sigmas=den.sigmas, step_idx=den.step_idx, ncopy=den.ncopy)
        with torch.no_grad():
            ref = unet.forward_tokens(x, B, F * world, h, w, emb, den.enc, fusion_world=world)
        e2 = ((got.float() - ref.float()).norm() / ref.float().norm()).item()
        em = ((got.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        exact = bool(torch.equal(got, ref))
        out = {"rel_l2": round(e2, 9), "rel_max": round(em, 9), "bitwise_equal": exact,
               "gate": "bitwise equality (" + ("weak" if n == world else "strong") + " scaling)",
               "what": f"{n} clip(s) x CFG pair noise prediction at {8 * h}x{8 * w}, {world}-way frame-sharded eager "
                       f"forward ({F} frames per rank) vs rank 0's unsharded forward of all {F * world} frames"}
        ok = exact and bool(torch.isfinite(got.float()).all())
        if not ok:
            print(json.dumps({"preflight_failed": out}), file=sys.stderr)
        del ref, x, got
    import torch.distributed as dist
    bad = torch.tensor([0 if rank != 0 or ok else 1], dtype=torch.int32)
    bad = bad if str(dist.get_backend()).lower() != "nccl" else bad.to(den.x.device)
    dist.all_reduce(bad)
    if int(bad.item()):
        raise SystemExit(3)
    return out


def bench_train(args, world, rank, local, dev):
    """BASELINE configs[4] (train_animatediff.py:212-319): SDXL UNet + AnimateDiff-SDXL motion modules (synthetic
    weights), UnZipLoRA r=8 frozen on all spatial projections, temporal LoRA r=32 injected, freeze_spatial_layers,
    --grad-accum 16x512x512 clips (VAE-encoded synthetic frames) per rank per optimizer step (accelerator.accumulate,
    default 4): Euler add_noise, UNet fwd, MSE + orth loss (lambda 1e-4), backward; on the window's last clip gradient
    all-reduce (RCCL, N>1), clip_grad_norm_(0.5), AdamW(2e-5, cosine schedule with 100 warm-up steps).  N=1: every
    clip replays one of two captured HIP graphs (accumulate / sync); N>1: eager calls with the bucketed all-reduce
    overlapping the last clip's backward."""
    from video_style_transfer_amd import kernels as K
    from video_style_transfer_amd.config import UNetMotionConfig
    from video_style_transfer_amd.scheduler import EulerDiscreteScheduler
    from video_style_transfer_amd.temporal_lora import build_spatial_lora_index, inject_temporal_lora
    from video_style_transfer_amd.train import GradBucketAllReducer, TrainStep, broadcast_parameters, get_scheduler, \
        make_adamw
    from video_style_transfer_amd.utils import build_unet, freeze_spatial_layers
    cfg = UNetMotionConfig.sdxl()
    t_build = time.perf_counter()
    unet = build_unet(cfg, seed=args.seed, lora_rank=args.lora_rank or None, device=dev)
    torch.manual_seed(args.seed)
    inject_temporal_lora(unet, rank=32, alpha=1.0)
    freeze_spatial_layers(unet)
    if world > 1:
        broadcast_parameters(unet)
    params = [p for p in unet.parameters() if p.requires_grad]
    graph = world == 1 and not args.no_graph
    # train_animatediff.py:163-169, :180-184 defaults: AdamW(2e-5, wd 1e-2), cosine schedule, 100 warm-up steps of
    # --max_train_steps 1000; the lr lives in a device tensor so the schedule reaches the captured step
    opt = make_adamw(params, lr=2e-5, betas=(0.9, 0.999), weight_decay=1e-2, eps=1e-8, capturable=graph, device=dev)
    lr_sched = get_scheduler("cosine", opt, num_warmup_steps=100, num_training_steps=1000)
    reducer = GradBucketAllReducer(params) if world > 1 else None
    step = TrainStep(unet, opt, EulerDiscreteScheduler(), reducer=reducer, lambda_orth=1e-4,
                     spatial_index=build_spatial_lora_index(unet), max_grad_norm=0.5, resolution=args.size,
                     seed=args.seed, lr_scheduler=lr_sched, gradient_accumulation_steps=args.grad_accum)
    g = torch.Generator().manual_seed(100 + rank)
    h = args.size // 8
    window = not args.sequential_accum and args.grad_accum > 1
    nclip = args.grad_accum if window else 1   # clips per forward / backward
    lat = torch.randn(nclip, 4, args.frames, h, h, generator=g).to(dev)
    vae = frames = None
    if not args.no_vae:
        # train_animatediff.py:219-224 inside every step: the clip's frames (synthetic, in [-1, 1]) -> VAE encode ->
        # latent_dist.sample() * scaling_factor (fp32 VAE in the reference; the HIP VAE, bf16, frames batched)
        from video_style_transfer_amd.config import VAEConfig
        from video_style_transfer_amd.train import encode_frames
        from video_style_transfer_amd.vae import build_vae
        vae = build_vae(VAEConfig.sdxl(), seed=args.seed + 1, device=dev)
        frames = (torch.rand(nclip, args.frames, 3, args.size, args.size, generator=g) * 2 - 1).to(dev)
        vgen = torch.Generator(device=dev).manual_seed(200 + rank)
        lat = encode_frames(vae, frames, vgen)
    enc = torch.randn(1, 77, cfg.cross_attention_dim, generator=g)
    pooled = torch.randn(1, cfg.text_embed_dim, generator=g)
    unc, unp = torch.zeros_like(enc), torch.zeros_like(pooled)
    if graph:
        step.capture(lat, enc, pooled, uncond_prompt=unc, uncond_pooled=unp, window=window)

        def micro():
            return step.replay(None if vae is None else encode_frames(vae, frames, vgen))
    elif window:
        def micro():
            return step.window(lat if vae is None else encode_frames(vae, frames, vgen), enc, pooled, unc, unp)
    else:
        def micro():
            return step(lat if vae is None else encode_frames(vae, frames, vgen), enc, pooled, unc, unp)

    def run():  # one optimizer step = one accumulation window of --grad-accum clips per rank
        for _ in range(1 if window else args.grad_accum):
            out = micro()
        assert out["sync"]
        return out
    t_build = time.perf_counter() - t_build
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms_step = dt / args.steps * 1e3
    value = args.frames * args.grad_accum * world / (ms_step * 1e-3)
    ok = bool(torch.isfinite(out["loss"]).item())
    lr_now = float(opt.param_groups[0]["lr"])
    rl = table = step_rl = None
    if not args.no_roofline:
        # one instrumented eager step (HIP events around every launch on its stream), enqueued behind a busy kernel
        lat_e = lat if vae is None else encode_frames(vae, frames, vgen)
        torch.cuda.synchronize()
        _gpu_busy(1500.0)
        K.profile_launches(True)
        if window:  # one whole window, so the optimizer / clip launches are counted once
            step.window(lat_e, enc, pooled)
        else:
            for _ in range(args.grad_accum):
                step(lat_e, enc, pooled)
        rl, table = _roofline_from(K.collect_launches(), ms_step)
        K.profile_launches(False)
        fl = rl.pop("step_flops")
        step_rl = {"alg_tflop": round(fl / 1e12, 2), "achieved_tflops": round(fl / (ms_step * 1e-3) / 1e12, 1),
                   "frac": round(fl / (ms_step * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4)}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        del step, opt, unet
        torch.cuda.empty_cache()
        cpu = train_cpu_baseline(args, cfg)
    if rank == 0:
        print(json.dumps({
            "metric": f"train frames/sec (fwd+bwd, AdamW step per {args.grad_accum} clips), {args.frames}x{args.size}x"
                      f"{args.size} clips per GPU, AnimateDiff-XL temporal LoRA",
            "value": round(value, 3), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": f"BASELINE configs[4]: train_animatediff.py step, {args.frames}x{args.size}x"
                                   f"{args.size} clip/GPU, temporal LoRA r=32, UnZipLoRA r={args.lora_rank} frozen, "
                                   f"orth loss 1e-4, clip 0.5, AdamW, cosine lr (100 warm-up), gradient accumulation "
                                   f"{args.grad_accum} (one step = {args.grad_accum} clips per GPU"
                                   + (", the window batched in one fwd+bwd)" if window else ", one fwd+bwd per clip)")
                                   + (
                                       ", from synthetic latents (no VAE encode)" if vae is None else
                                       ", VAE encode of the synthetic frames in every step"),
                       "model": "SDXL UNet + AnimateDiff-SDXL motion modules (synthetic weights)",
                       "global_batch": world * args.grad_accum, "frames": args.frames, "resolution": args.size,
                       "gradient_accumulation_steps": args.grad_accum,
                       "parallelism": f"dp{world}" + (" (RCCL bucketed all-reduce)" if world > 1 else ""),
                       "graph": graph, "trainable_params": sum(p.numel() for p in params)},
            "loss": round(float(out["loss"]), 5), "finite": ok, "lr": lr_now,
            "ms_per_clip": round(ms_step / args.grad_accum, 3),
            "roofline": rl, "step_roofline": step_rl, "cpu_baseline": cpu, "kernels": table,
            "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1), "setup_s": round(t_build, 1)}))


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # VST_BENCH_REHEARSAL=gloo: rehearse the N-rank orchestration on a one-GPU box (every rank on cuda:0, gloo
    # transport, eager steps) -- a correctness drill for the launcher path, never a scaling number.
    rehearsal = os.environ.get("VST_BENCH_REHEARSAL") == "gloo"
    if rehearsal:
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if args.train:
        return bench_train(args, world, rank, local, dev)

    from video_style_transfer_amd.config import UNetMotionConfig
    from video_style_transfer_amd.lora_linear import set_lora_mode
    from video_style_transfer_amd.utils import build_unet

    cfg = UNetMotionConfig.sdxl()
    set_lora_mode(args.lora_mode)
    t_build = time.perf_counter()
    unet = build_unet(cfg, seed=args.seed, lora_rank=args.lora_rank or None, device=dev)
    t_build = time.perf_counter() - t_build
    sharded = world > 1 and args.parallel == "frames"
    nclips = (args.clips or world) if sharded else max(1, args.clips)
    head = timed_denoise(args, unet, cfg, world, rank, dev, rehearsal, frames=args.frames, size=args.size,
                         nclips=nclips, sharded=sharded)
    den, ms_step, value = head["den"], head["ms_per_step"], head["value"]
    ok = bool(torch.isfinite(den.lat).all().item())

    rl, table = (None, None) if args.no_roofline else roofline(den, ms_step)
    step = None
    if rl is not None:
        # whole denoise step against the chip: algorithmic flops of every launch (table in DESIGN.md 3) per
        # graph-replayed step time
        fl = rl.pop("step_flops")
        step = {"alg_tflop": round(fl / 1e12, 2), "achieved_tflops": round(fl / (ms_step * 1e-3) / 1e12, 1),
                "frac": round(fl / (ms_step * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4)}
        if rank == 0 and not rehearsal and not args.no_peaks:
            rl["peak_measured"] = measured_peaks(dev, rl)
            step["frac_of_measured"] = round(step["achieved_tflops"] / rl["peak_measured"]["mfma_bf16_tflops"], 4)
    graphed = den.graph is not None
    vae_rec = None if args.no_vae else vae_decode_timing(args, den, dev, ms_step)
    den.graph = None  # (piecewise graphs hold no collective; released before the next run's memory)
    del den, head["den"]
    torch.cuda.empty_cache()

    # N-GPU frame sharding: the north star's curve needs more than the weak-scaling headline -- one 16-frame clip split
    # N ways (strong scaling) and, on 8 GPUs, BASELINE configs[3] (one 32 x 768^2 clip, 4 frames per GPU); each runs
    # its own bitwise preflight, piecewise capture and timing with the same --steps / --warmup
    subs = {}
    if sharded and world > 1:
        want_strong = args.strong_record == "on" or (args.strong_record == "auto" and nclips != 1)
        want_c3 = args.configs3 == "on" or (args.configs3 == "auto" and world == 8)
        plans = []
        if want_strong:
            plans.append(("strong_1clip", args.frames, args.size))
        want_gather = args.exchange == "all_to_all" and (
            args.gather_record == "on" or args.gather_record == "auto")
        if want_gather:  # the north star's own exchange on the headline workload, next to the all-to-all headline
            plans.append(("all_gather", args.frames, args.size, nclips, "all_gather"))
        if want_c3:
            plans.append(("configs3", args.configs3_frames, args.configs3_size, 1, args.exchange))
        plans = [p if len(p) == 5 else p + (1, args.exchange) for p in plans]
        for name, fr, sz, ncl, exch in plans:
            if fr % world:
                subs[name] = {"skipped": f"{fr} frames do not split over {world} ranks"}
                continue
            r = timed_denoise(args, unet, cfg, world, rank, dev, rehearsal, frames=fr, size=sz, nclips=ncl,
                              sharded=True, exchange=exch)
            subs[name] = {
                "value": round(r["value"], 4), "unit": "frames/s", "ms_per_step": round(r["ms_per_step"], 3),
                "n_gpus": world, "scaling": "strong" if ncl < world else "weak", "frames": fr, "resolution": sz,
                "clips": ncl, "frames_per_gpu": fr // world, "graph": r["den"].graph is not None,
                "note": r["graph_note"], "exchange": exch, "overlap": r["overlap"],
                "shard_preflight": r["preflight"],
                "finite": bool(torch.isfinite(r["den"].lat).all().item()),
                "workload": ("BASELINE configs[3]: " if name == "configs3" else "") +
                            f"{ncl} {fr}x{sz}x{sz} clip(s) + UnZipLoRA rank-{args.lora_rank}, CFG pair, frame-sharded "
                            f"x{world} ({fr // world} frames/clip/GPU, "
                            + ("all-to-all" if exch == "all_to_all" else "all-gather of the clip before each motion "
                                                                         "module (the north star's exchange)") + ")"}
            r["den"].graph = None
            del r
            torch.cuda.empty_cache()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        del unet
        torch.cuda.empty_cache()
        cpu = cpu_baseline(args, cfg)
    if rank == 0:
        out = {
            "metric": f"denoised frames/sec, {args.frames}x{args.size}x{args.size} clip, "
                      f"{args.num_inference_steps}-step AnimateDiff-XL",
            "value": round(value, 4), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "strong" if (sharded and nclips < world) else "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": f"BASELINE configs[2]: {args.frames}x{args.size}x{args.size} clip + UnZipLoRA "
                                   f"rank-{args.lora_rank} ({args.lora_mode}) on all 560 spatial q/k/v/out, "
                                   f"{args.num_inference_steps}-step Euler, CFG {args.guidance} batched (B=2)",
                       "model": "SDXL UNet + AnimateDiff-SDXL motion modules (synthetic weights)",
                       "global_batch": nclips if sharded else nclips * world, "frames": args.frames,
                       "resolution": args.size,
                       "parallelism": (f"frame-shard x{world} ({nclips} clips, {args.frames // world} frames/clip/GPU, "
                                       + ("RCCL all-to-all around each motion module)" if args.exchange == "all_to_all"
                                          else "RCCL all-gather of the clip before each motion module)")
                                       if sharded else
                                       f"replicas x{world}" if world > 1 else "single") + (
                                       f", {nclips} clips batched per GPU" if not sharded and nclips > 1 else ""),
                       "graph": graphed, "exchange_overlap": head["overlap"],
                       "note": head["graph_note"]},
            "roofline": rl, "step_roofline": step, "vae_decode": vae_rec, "cpu_baseline": cpu, "kernels": table,
            "finite": ok, "shard_preflight": head["preflight"], "sub_records": subs or None,
            "setup_s": round(t_build, 1),
        }
        print(json.dumps(out))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()  # (every HIP graph released above: a graph must not outlive the communicator)


def timed_denoise(args, unet, cfg, world, rank, dev, rehearsal, *, frames, size, nclips, sharded, exchange=None):
    """One denoiser of `nclips` clips of `frames` x size^2 (frame-sharded over the ranks when `sharded`): preflight
    (sharded), capture (one HIP graph; piecewise at N > 1), --warmup untimed and --steps timed replays bracketed by
    barrier + synchronize, the max over ranks.  Returns the denoiser (for the roofline / VAE records) and the timing."""
    from video_style_transfer_amd.pipeline import AnimateDiffDenoiser
    shard = None
    if sharded:
        from video_style_transfer_amd.frame_shard import FrameShard
        shard = FrameShard(exchange=exchange or args.exchange, overlap=not args.no_overlap)
    den = AnimateDiffDenoiser(unet, frames, size, size, num_inference_steps=args.num_inference_steps,
                              guidance_scale=args.guidance, device=dev, shard=shard, num_clips=nclips)
    seed_rank = 0 if shard is not None else rank  # sharded ranks hold frames of the SAME clips
    g = torch.Generator().manual_seed(7 + seed_rank)
    enc = torch.randn(2, 77, cfg.cross_attention_dim, generator=g)
    pooled = torch.randn(2, cfg.text_embed_dim, generator=g)
    den.set_prompt_embeds(enc[1:], pooled[1:], enc[:1], pooled[:1])
    den.init_latents(seed=42 + seed_rank)
    graph_note = None
    preflight = shard_preflight(den, unet, world, rank) if shard is not None else None
    if not args.no_graph:
        # N = 1: one HIP graph per step; a step that cannot be captured fails the run.  Frame-sharded N > 1: the step
        # is captured piecewise (frame_shard.PiecewiseGraph: the graphs split at the collectives, which run between
        # the replays), so no collective is inside a graph.  If capture still fails on any rank, ALL ranks time eager
        # steps, reported loudly in the line ("graph": false, "note"), never silently
        err = None
        try:
            den.capture()
        except Exception as e:  # noqa: BLE001 -- re-raised at N = 1
            if world == 1:
                raise
            err = e
            den.graph = None
            torch.cuda.synchronize()
        if world > 1:
            import torch.distributed as dist
            flag = torch.tensor([0.0 if err is None else 1.0], device="cpu" if rehearsal else dev)
            dist.all_reduce(flag)
            if flag.item() > 0:
                den.graph = None
                graph_note = (f"HIP-graph capture of the frame-sharded step failed on {int(flag.item())} of {world} "
                              f"ranks{'' if err is None else ' (' + type(err).__name__ + ': ' + str(err)[:160] + ')'}; "
                              f"eager steps")
                print(f"[bench] rank {rank}: {graph_note}", file=sys.stderr, flush=True)
            elif shard is not None:
                graph_note = (f"piecewise capture: {den.graph.num_graphs} HIP graphs per step, the "
                              f"{len(den.graph.items) - den.graph.num_graphs} collectives ({shard.backend}) between them")

    def one_step():
        if den.graph is not None:
            den.graph.replay()
        else:
            den._step()
    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([dt], device="cpu" if rehearsal else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms_step = dt / args.steps * 1e3
    # frames mode: nclips whole clips spread over all ranks; replicas: every rank denoises its own clip
    frames_total = frames * nclips if shard is not None else frames * nclips * world
    value = frames_total / (args.num_inference_steps * ms_step * 1e-3)
    return {"den": den, "ms_per_step": ms_step, "value": value, "preflight": preflight, "graph_note": graph_note,
            "overlap": None if shard is None else shard.overlap}


if __name__ == "__main__":
    main()
