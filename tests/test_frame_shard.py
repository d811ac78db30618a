"""Frame sharding of a clip over ranks (video_style_transfer_amd/frame_shard.py).

CPU (gloo, world sizes 2, 4 and 8 -- the last is configs[3]'s 8 ranks x 4 frames): the layout algebra of the frame <-> pixel shard exchange, and that the
sharded motion module (all-reduced GroupNorm statistics + frame-axis work on pixel shards) equals the
oracle's unsharded motion module (oracle/unet.py motion_module) on each rank's frames.

GPU (gloo transport, 2-8 ranks on one GPU, HIP kernels): a frame-sharded tiny-UNet forward is as close
to the fp32 oracle's whole-clip forward as the unsharded HIP forward is (both bf16); at configs[3]'s SDXL 32 x 768^2
shape (B = 1 over 2 ranks, and the CFG pair over 4 and 8 ranks -- 8 x 4 frames is configs[3]'s own split), the
16 x 512^2 clip over 8 ranks (2 frames each) and 16 x 576^2 over 2 ranks (a motion level whose per-rank pixel count is
not a multiple of 16) the gathered shards ARE the unsharded HIP forward, bit for bit.
"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def torch_permute_rows(src, dims, perm):
    """Semantics of vst_permute_rows, restated in torch for CPU ranks."""
    C = src.shape[1]
    return src.view(*dims, C).permute(*perm, 4).reshape(-1, C).contiguous()


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)


# ------------------------------------------------------------------------------------- CPU
def _cpu_worker(rank, world, port, q, F=4):
    try:
        sys.path.insert(0, ROOT)
        _init(rank, world, port)
        from oracle import unet as OU
        from video_style_transfer_amd.frame_shard import FrameShard
        sh = FrameShard(permute=torch_permute_rows)
        torch.manual_seed(0)
        B, H, W, C = 2, 4, 6, 64
        HW = H * W
        X = torch.randn(B, F, HW, C)
        Fl, f0 = sh.local_frames(F)
        x_loc = X[:, f0:f0 + Fl].reshape(-1, C).contiguous()
        # (a) frame shard -> pixel shard: rank r holds pixel slab r of every frame
        hp = HW // world
        px = sh.to_pixels(x_loc, B, Fl, HW)
        ref = X[:, :, rank * hp:(rank + 1) * hp].reshape(-1, C)
        assert torch.equal(px, ref), "to_pixels layout"
        # (b) round trip
        assert torch.equal(sh.to_frames(px, B, Fl, HW), x_loc), "to_frames(to_pixels(x)) != x"
        # (b') the north-star exchange: the all-gather hands every rank the whole clip in (b, f, p) row order, and
        # local_frames_of takes this rank's frames back out of it
        gx = sh.gather_frames(x_loc, B, Fl, HW)
        assert torch.equal(gx, X.reshape(-1, C)), "gather_frames layout"
        assert torch.equal(sh.local_frames_of(gx, B, Fl, HW), x_loc), "local_frames_of(gather_frames(x)) != x"
        # the async form the overlapped all-gather exchange issues per CFG half: each half gathered on its own
        nbh, rws = B // 2, (B // 2) * Fl * HW
        halves = [sh.gather_frames_begin(x_loc[i * rws:(i + 1) * rws], nbh, Fl, HW) for i in range(2)]
        got_g = torch.cat([end() for end, _src in halves])
        assert torch.equal(got_g, X.reshape(-1, C)), "gather_frames_begin per half != gather_frames"
        # (b'') the overlapped schedule (FrameShard.pipelined: the batch in two halves, each half's exchange issued
        # before the other half computes) gives the one-slice schedule's bits; mid() is a frame-axis op (a running sum
        # over every frame of each pixel), so it only matches if each half really holds all frames of its pixels
        def mid_op(h, nb):
            return h.view(nb, F, hp, C).cumsum(1).reshape(-1, C) * 0.5

        ref_all = sh.to_frames(mid_op(sh.to_pixels(x_loc * 3.0, B, Fl, HW), B), B, Fl, HW) + x_loc
        nb, rows = B // 2, (B // 2) * Fl * HW
        got = torch.empty_like(x_loc)
        order = []

        def pre(i):
            order.append(("pre", i))
            return x_loc[i * rows:(i + 1) * rows] * 3.0

        def mid(i, h):
            order.append(("mid", i))
            return mid_op(h, nb)

        def post(i, h):
            order.append(("post", i))
            got[i * rows:(i + 1) * rows] = h + x_loc[i * rows:(i + 1) * rows]
        sh.pipelined(2, pre, mid, post, nb, Fl, HW)
        assert torch.equal(got, ref_all), "pipelined exchange != one-slice exchange"
        assert order == [("pre", 0), ("pre", 1), ("mid", 0), ("mid", 1), ("post", 0), ("post", 1)], order
        # (c) sharded motion module == oracle motion module
        P = {}
        g = torch.Generator().manual_seed(1)
        name = "mm"
        P[name + ".norm.weight"] = 1 + 0.1 * torch.randn(C, generator=g)
        P[name + ".norm.bias"] = 0.1 * torch.randn(C, generator=g)
        for lin in ("proj_in", "proj_out"):
            P[f"{name}.{lin}.weight"] = torch.randn(C, C, generator=g) / C ** 0.5
            P[f"{name}.{lin}.bias"] = 0.1 * torch.randn(C, generator=g)
        blk = name + ".transformer_blocks.0"
        for a in ("attn1", "attn2"):
            for pj in ("to_q", "to_k", "to_v"):
                P[f"{blk}.{a}.{pj}.weight"] = torch.randn(C, C, generator=g) / C ** 0.5
            P[f"{blk}.{a}.to_out.0.weight"] = torch.randn(C, C, generator=g) / C ** 0.5
            P[f"{blk}.{a}.to_out.0.bias"] = 0.1 * torch.randn(C, generator=g)
        for n in ("norm1", "norm2", "norm3"):
            P[f"{blk}.{n}.weight"] = 1 + 0.1 * torch.randn(C, generator=g)
            P[f"{blk}.{n}.bias"] = 0.1 * torch.randn(C, generator=g)
        P[f"{blk}.ff.net.0.proj.weight"] = torch.randn(8 * C, C, generator=g) / C ** 0.5
        P[f"{blk}.ff.net.0.proj.bias"] = 0.1 * torch.randn(8 * C, generator=g)
        P[f"{blk}.ff.net.2.weight"] = torch.randn(C, 4 * C, generator=g) / (4 * C) ** 0.5
        P[f"{blk}.ff.net.2.bias"] = 0.1 * torch.randn(C, generator=g)
        from video_style_transfer_amd.weights import sinusoid_table
        P[f"{blk}.pos_embed.pe"] = sinusoid_table(C, 32)
        x_nchw = X.reshape(B * F, H, W, C).permute(0, 3, 1, 2).contiguous()
        full = OU.motion_module(P, name, x_nchw, F)                       # (B*F, C, H, W)
        full_tok = full.permute(0, 2, 3, 1).reshape(B, F, HW, C)[:, f0:f0 + Fl].reshape(-1, C)
        # sharded: per-frame GN partials all-gathered rank-major ([P, B, Fl, G, 2]) and merged in global frame order
        # (the layout vst_groupnorm_apply_partials reads)
        G = 32
        xs = x_loc.double().view(B, Fl, HW, G, C // G)
        part = torch.stack([xs.sum((2, 4)), (xs * xs).sum((2, 4))], -1)        # [B, Fl, G, 2]
        allp = sh.all_gather(part)                                              # [P, B, Fl, G, 2]
        assert allp.shape == (world,) + tuple(part.shape) and torch.equal(allp[rank], part)
        sums = allp.permute(1, 0, 2, 3, 4).reshape(B, F, G, 2).sum(1)           # frames 0..F-1 of each clip
        cnt = F * HW * (C // G)
        mean = sums[..., 0] / cnt
        var = sums[..., 1] / cnt - mean * mean
        xs = xs.reshape(B, Fl * HW, G, C // G)
        h = (xs - mean[:, None, :, None]) / torch.sqrt(var[:, None, :, None] + 1e-6)
        h = h.float().reshape(B, Fl * HW, C) * P[name + ".norm.weight"] + P[name + ".norm.bias"]
        h = OU.linear(P, name + ".proj_in", h.reshape(-1, C))
        h = sh.to_pixels(h, B, Fl, HW)                                    # rows (b, f, p')
        h = h.view(B, F, hp, C).permute(0, 2, 1, 3).reshape(B * hp, F, C)  # oracle layout (B*HW', F, C)
        h = OU.basic_block(P, blk, h, None, 8, None, pe=P[f"{blk}.pos_embed.pe"])
        h = h.view(B, hp, F, C).permute(0, 2, 1, 3).reshape(-1, C)
        h = sh.to_frames(h, B, Fl, HW)
        out = OU.linear(P, name + ".proj_out", h) + x_loc
        err = ((out - full_tok).norm() / full_tok.norm()).item()
        assert err < 1e-5, f"sharded motion module rel err {err}"
        q.put((rank, "ok", err))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, "fail", repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _spawn(fn, world, *extra):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q) + extra) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("world,F", [(2, 4), (4, 8), (8, 32)])
def test_frame_shard_cpu(world, F):
    """(8, 32): BASELINE configs[3]'s split, 32 frames over 8 ranks (4 each), CFG pair (B = 2)."""
    res = _spawn(_cpu_worker, world, F)
    for rank, status, info in res:
        assert status == "ok", f"rank {rank}: {info}"


# ------------------------------------------------------------------------------------- GPU
def _gpu_worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        _init(rank, world, port)
        from oracle.unet import unet_forward
        from test_parity_gpu import _setup
        from video_style_transfer_amd.frame_shard import FrameShard
        from video_style_transfer_amd.utils import build_unet
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        F = 8
        cfg, sd, lat, enc, pooled, tids = _setup("tiny", F, 16)
        t = torch.tensor([761.0, 761.0])
        ref = unet_forward(sd, cfg.to_dict(), lat, t, enc, pooled, tids)        # fp32 oracle, whole clip
        unet = build_unet(cfg, state_dict=sd, device=dev)
        sh = FrameShard()
        Fl, f0 = sh.local_frames(F)
        kw = dict(added_cond_kwargs={"text_embeds": pooled.to(dev), "time_ids": tids.to(dev)})
        full = unet(lat.to(dev), t.to(dev), enc.to(dev), **kw).sample.float().cpu()
        part = unet(lat[:, :, f0:f0 + Fl].contiguous().to(dev), t.to(dev), enc.to(dev), frame_shard=sh,
                    **kw).sample.float().cpu()
        r = ref[:, :, f0:f0 + Fl]

        def rel(a, b):
            return ((a - b).norm() / b.norm()).item()
        e_full, e_shard = rel(full[:, :, f0:f0 + Fl], r), rel(part, r)
        ok = e_shard <= 3e-2 and e_shard <= 1.25 * e_full + 2e-3
        q.put((rank, "ok" if ok else "fail", f"vs fp32 oracle: sharded {e_shard:.3e}, unsharded {e_full:.3e}"))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, "fail", repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.gpu
def test_frame_shard_unet_two_ranks_one_gpu():
    if torch.cuda.device_count() == 0:
        pytest.skip("no HIP device")
    res = _spawn(_gpu_worker, 2)
    for rank, status, info in res:
        print(f"[shard] rank {rank}: {status} {info}")
        assert status == "ok", f"rank {rank}: {info}"


def _gpu_worker_sdxl768(rank, world, port, q, exchange="all_to_all"):
    """BASELINE configs[3] shapes: SDXL + motion modules + UnZipLoRA r=8, 32 frames at 768x768 (96x96 latent),
    frames split over 2 ranks (16 each) on one GPU, vs the unsharded HIP forward of the whole clip; both exchanges
    (all-to-all around the motion modules, and the north star's all-gather of the clip before them)."""
    try:
        sys.path.insert(0, ROOT)
        _init(rank, world, port)
        from video_style_transfer_amd.config import UNetMotionConfig
        from video_style_transfer_amd.frame_shard import FrameShard
        from video_style_transfer_amd.utils import build_unet
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        cfg = UNetMotionConfig.sdxl()
        unet = build_unet(cfg, seed=41, lora_rank=8, device=dev)
        F, hw = 32, 96
        g = torch.Generator().manual_seed(42)
        lat = torch.randn(1, 4, F, hw, hw, generator=g)
        enc = torch.randn(1, 77, cfg.cross_attention_dim, generator=g)
        pooled = torch.randn(1, cfg.text_embed_dim, generator=g)
        tids = torch.tensor([[768, 768, 0, 0, 768, 768]], dtype=torch.float32)
        t = torch.tensor([501.0])
        kw = dict(added_cond_kwargs={"text_embeds": pooled.to(dev), "time_ids": tids.to(dev)})
        sh = FrameShard(exchange=exchange)
        Fl, f0 = sh.local_frames(F)
        part = unet(lat[:, :, f0:f0 + Fl].contiguous().to(dev), t.to(dev), enc.to(dev), frame_shard=sh,
                    **kw).sample.cpu()
        full = unet(lat.to(dev), t.to(dev), enc.to(dev), fusion_world=world, **kw).sample.cpu()[:, :, f0:f0 + Fl]
        # every op outside the motion modules is frame-local with frame-invariant bits (GroupNorm chunking and GEMM
        # k order depend on the frame shape only); the motion GroupNorm merges the same per-frame partials in the
        # same order; the exchange only moves rows: the shards must be the unsharded bits exactly
        same = torch.equal(part, full)
        d = (part.float() - full.float()).abs().max().item()
        q.put((rank, "ok" if same else "fail", f"frames {f0}..{f0 + Fl - 1}: sharded == unsharded: {same} "
                                               f"(max |diff| {d:.3e})"))
    except BaseException:  # noqa: BLE001
        import traceback
        q.put((rank, "fail", traceback.format_exc()[-2000:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["all_to_all", "all_gather"])
def test_frame_shard_sdxl_768_32_frames_two_ranks_one_gpu(exchange):
    if torch.cuda.device_count() == 0:
        pytest.skip("no HIP device")
    res = _spawn(_gpu_worker_sdxl768, 2, exchange)
    for rank, status, info in res:
        print(f"[shard] configs[3] {exchange} rank {rank}: {status} {info}")
        assert status == "ok", f"rank {rank}: {info}"


def _gpu_worker_sdxl_cfg(rank, world, port, q, F=32, hw=96, exchange="all_to_all"):
    """The CFG pair (B = 2: uncond + cond text states, as the denoise loop batches them) of one SDXL clip of F frames
    at (8 hw)^2, split over `world` ranks (F / world frames each) on one GPU.  Rank 0 gathers the shards and compares
    them with its unsharded forward of the whole clip under kernels.fusion_world(world) (the other ranks run the sharded
    forward only): BASELINE configs[3] (32 x 768^2) over 4 and 8 ranks -- 8 x 4 frames is configs[3]'s own split --
    the 16 x 512^2 clip split 8 ways (bench.py's strong-scaling sub-record at N = 8), and 16 x 576^2 over 2 ranks, whose
    36 x 36 motion level gives each all-to-all rank 648 pixels (not a multiple of 16: that layer's motion attention
    is not fused into its q/k/v GEMM on the ranks, so the unsharded forward must not fuse it either)."""
    try:
        sys.path.insert(0, ROOT)
        _init(rank, world, port)
        from video_style_transfer_amd import kernels as K
        from video_style_transfer_amd.config import UNetMotionConfig
        from video_style_transfer_amd.frame_shard import FrameShard
        from video_style_transfer_amd.utils import build_unet
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        cfg = UNetMotionConfig.sdxl()
        unet = build_unet(cfg, seed=43, lora_rank=8, device=dev)
        print(f"[shard] rank {rank}/{world}: UNet built", flush=True)
        g = torch.Generator().manual_seed(44)
        lat1 = torch.randn(1, 4, F, hw, hw, generator=g)
        lat = torch.cat([lat1, lat1])  # the CFG pair shares the latents
        enc = torch.randn(2, 77, cfg.cross_attention_dim, generator=g)
        pooled = torch.randn(2, cfg.text_embed_dim, generator=g)
        tids = torch.tensor([[8 * hw, 8 * hw, 0, 0, 8 * hw, 8 * hw]] * 2, dtype=torch.float32)
        t = torch.tensor([501.0, 501.0])
        kw = dict(added_cond_kwargs={"text_embeds": pooled.to(dev), "time_ids": tids.to(dev)})
        sh = FrameShard(exchange=exchange)
        Fl, f0 = sh.local_frames(F)
        part = unet(lat[:, :, f0:f0 + Fl].contiguous().to(dev), t.to(dev), enc.to(dev), frame_shard=sh,
                    **kw).sample.float().cpu()
        print(f"[shard] rank {rank}/{world}: sharded forward done", flush=True)
        parts = [torch.empty_like(part) for _ in range(world)]
        dist.all_gather(parts, part)
        if rank != 0:
            q.put((rank, "ok", f"frames {f0}..{f0 + Fl - 1} sent to rank 0"))
            return
        whole = torch.cat(parts, 2)
        full = unet(lat.to(dev), t.to(dev), enc.to(dev), fusion_world=world, **kw).sample.float().cpu()
        print(f"[shard] rank 0: unsharded forward done", flush=True)
        same = torch.equal(whole, full)
        d = [(whole[b] - full[b]).abs().max().item() for b in range(2)]
        msg = (f"{F}x{8 * hw}^2, {world} shards x {Fl} frames, CFG pair: gathered shards == unsharded: {same} "
               f"(max |diff| uncond {d[0]:.3e}, cond {d[1]:.3e})")
        if same and any(s_ * s_ % (16 * world) for s_ in (hw, hw // 2)):
            # the case the policy exists for: without it the unsharded forward fuses a layer the ranks cannot
            fused = unet(lat.to(dev), t.to(dev), enc.to(dev), **kw).sample.float().cpu()
            msg += f"; unsharded without the policy differs: {not torch.equal(fused, full)}"
        q.put((rank, "ok" if same else "fail", msg))
    except BaseException:  # noqa: BLE001
        import traceback
        q.put((rank, "fail", traceback.format_exc()[-2000:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,F,hw", [(4, 32, 96), (8, 32, 96), (8, 16, 64), (2, 16, 72)],
                         ids=["configs3_4ranks", "configs3_8ranks_x4frames", "strong_16x512_8ranks",
                              "576_2ranks_fusion_policy"])
def test_frame_shard_sdxl_cfg_pair_one_gpu(world, F, hw):
    if torch.cuda.device_count() == 0:
        pytest.skip("no HIP device")
    res = _spawn(_gpu_worker_sdxl_cfg, world, F, hw)
    for rank, status, info in res:
        print(f"[shard] CFG pair rank {rank}: {status} {info}")
        assert status == "ok", f"rank {rank}: {info}"


def _gpu_worker_overlap(rank, world, port, q):
    """The overlapped exchanges (FrameShard(overlap=True): each motion module's CFG pair as two halves whose all-to-alls
    -- or, for the north star's all-gather, whose gathers -- run under the other half's compute) against the one-slice
    exchange and against the unsharded forward: the tiny UNet, CFG pair, 8 frames over `world` ranks; bit-identical."""
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        _init(rank, world, port)
        from test_parity_gpu import _setup
        from video_style_transfer_amd.frame_shard import FrameShard
        from video_style_transfer_amd.utils import build_unet
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        F = 8
        cfg, sd, lat, enc, pooled, tids = _setup("tiny", F, 16, seed=9, B=2)
        unet = build_unet(cfg, state_dict=sd, device=dev)
        kw = dict(added_cond_kwargs={"text_embeds": pooled.to(dev), "time_ids": tids.to(dev)})
        t = torch.tensor([421.0, 421.0])
        full = unet(lat.to(dev), t.to(dev), enc.to(dev), fusion_world=world, **kw).sample.float().cpu()
        msgs, ok = [], True
        for exchange in ("all_to_all", "all_gather"):
            outs = {}
            for ov in (True, False):
                sh = FrameShard(exchange=exchange, overlap=ov)
                Fl, f0 = sh.local_frames(F)
                outs[ov] = unet(lat[:, :, f0:f0 + Fl].contiguous().to(dev), t.to(dev), enc.to(dev), frame_shard=sh,
                                **kw).sample.float().cpu()
            same_ov = torch.equal(outs[True], outs[False])
            same_full = torch.equal(outs[True], full[:, :, f0:f0 + Fl])
            ok = ok and same_ov and same_full
            msgs.append(f"{exchange}: overlapped == one-slice: {same_ov}; == unsharded: {same_full}")
        q.put((rank, "ok" if ok else "fail", "; ".join(msgs)))
    except BaseException:  # noqa: BLE001
        import traceback
        q.put((rank, "fail", traceback.format_exc()[-2000:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.gpu
def test_frame_shard_overlapped_exchange_two_ranks_one_gpu():
    if torch.cuda.device_count() == 0:
        pytest.skip("no HIP device")
    res = _spawn(_gpu_worker_overlap, 2)
    for rank, status, info in res:
        print(f"[shard] overlap rank {rank}: {status} {info}")
        assert status == "ok", f"rank {rank}: {info}"


def _gpu_worker_piecewise(rank, world, port, q):
    """Piecewise capture of the frame-sharded denoise step (frame_shard.PiecewiseGraph: HIP graphs split at the
    collectives, which run between the replays): 3 replayed steps == 3 eager steps, bit for bit."""
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        _init(rank, world, port)
        from test_parity_gpu import _setup
        from video_style_transfer_amd.frame_shard import FrameShard, PiecewiseGraph
        from video_style_transfer_amd.pipeline import AnimateDiffDenoiser
        from video_style_transfer_amd.utils import build_unet
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        cfg, sd, lat, enc, pooled, tids = _setup("tiny", 8, 16, seed=6, B=2)
        unet = build_unet(cfg, state_dict=sd, device=dev)
        sh = FrameShard()
        den = AnimateDiffDenoiser(unet, 8, 128, 128, num_inference_steps=10, device=dev, shard=sh, num_clips=1,
                                  use_graph=False)
        den.set_prompt_embeds(enc[1:2], pooled[1:2], enc[0:1], pooled[0:1])
        lat0 = den.init_latents(seed=3)
        eager = den.run_steps(3).clone()
        den.set_latents(lat0)
        den.use_graph = True
        den.capture()
        assert isinstance(den.graph, PiecewiseGraph) and den.graph.num_graphs > 1
        den.set_latents(lat0)
        graph = den.run_steps(3).clone()
        same = torch.equal(eager, graph)
        q.put((rank, "ok" if same else "fail", f"piecewise graph ({den.graph.num_graphs} graphs, "
                                               f"{len(den.graph.items) - den.graph.num_graphs} collectives) == eager: "
                                               f"{same}, max |diff| {(eager - graph).abs().max().item():.3e}"))
    except BaseException:  # noqa: BLE001
        import traceback
        q.put((rank, "fail", traceback.format_exc()[-2000:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.gpu
def test_frame_shard_piecewise_graph_two_ranks_one_gpu():
    if torch.cuda.device_count() == 0:
        pytest.skip("no HIP device")
    res = _spawn(_gpu_worker_piecewise, 2)
    for rank, status, info in res:
        print(f"[shard] piecewise rank {rank}: {status} {info}")
        assert status == "ok", f"rank {rank}: {info}"
