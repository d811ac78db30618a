"""Where does a frame-sharded UNet forward first differ from the unsharded one?  Two gloo ranks on one GPU run the
sharded forward of the bench's input (`--clips` clips x CFG pair, `--frames` frames at `--size`), recording the output
of every ResnetBlock2D / Transformer2DModel / BasicTransformerBlock / MotionModule / Down- / Upsample2D; rank 0 also
runs the unsharded forward of the same clips and compares layer by layer (shards re-assembled on the frame axis).
Prints the first layers whose outputs are not bit-identical, with the max |diff| and whether their inputs matched.
python tools/shard_diag.py [--frames 16 --size 256 --clips 2 --world 2]"""
import argparse
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _recorder(U, unet, rec):
    names = {id(m): n for n, m in unet.named_modules()}
    saved = {}

    def wrap(cls, kind):
        orig = cls.run
        saved[cls] = orig

        def run(mod, x, nimg, *a, **kw):
            y = orig(mod, x, nimg, *a, **kw)
            out = y[0] if isinstance(y, tuple) else y
            rec.append((kind, names.get(id(mod), "?"), nimg, x.detach().cpu().clone(), out.detach().cpu().clone()))
            return y
        cls.run = run
    for cls, kind in ((U.ResnetBlock2D, "resnet"), (U.Transformer2DModel, "t2d"), (U.MotionModule, "motion"),
                      (U.Downsample2D, "down"), (U.Upsample2D, "up")):
        wrap(cls, kind)
    orig_blk = U.BasicTransformerBlock.run
    saved[U.BasicTransformerBlock] = orig_blk

    def blk_run(mod, x, nimg, N, ctx):
        y = orig_blk(mod, x, nimg, N, ctx)
        if not mod.temporal:
            rec.append(("block", names.get(id(mod), "?"), nimg, x.detach().cpu().clone(), y.detach().cpu().clone()))
        return y
    U.BasicTransformerBlock.run = blk_run
    return saved


def _worker(rank, world, port, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    from video_style_transfer_amd import kernels as K
    from video_style_transfer_amd import unet_motion as U
    from video_style_transfer_amd.config import UNetMotionConfig
    from video_style_transfer_amd.frame_shard import FrameShard
    from video_style_transfer_amd.pipeline import AnimateDiffDenoiser
    from video_style_transfer_amd.utils import build_unet
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = UNetMotionConfig.sdxl()
    unet = build_unet(cfg, seed=0, lora_rank=8, device=dev)
    sh = FrameShard()
    n = args.clips
    den = AnimateDiffDenoiser(unet, args.frames, args.size, args.size, device=dev, shard=sh, num_clips=n)
    g = torch.Generator().manual_seed(7)
    enc = torch.randn(2, 77, cfg.cross_attention_dim, generator=g)
    pooled = torch.randn(2, cfg.text_embed_dim, generator=g)
    den.set_prompt_embeds(enc[1:], pooled[1:], enc[:1], pooled[:1])
    den.init_latents(seed=42)
    B, F, h, w = den.ncopy * n, den.F, den.h, den.w
    den.step_idx.zero_()
    K.pack_latents(den.lat, den.x, sigmas=den.sigmas, step_idx=den.step_idx, ncopy=den.ncopy)
    emb = unet.embed(den.timesteps, den.pooled, den.time_ids, B, step_idx=den.step_idx)
    rec = []
    saved = _recorder(U, unet, rec)
    with torch.no_grad():
        unet.forward_tokens(den.x, B, F, h, w, emb, den.enc, shard=sh)
    torch.save(rec, f"/tmp/shard_diag_rank{rank}.pt")
    lat_parts = [torch.empty_like(den.lat.cpu()) for _ in range(world)]
    dist.all_gather(lat_parts, den.lat.cpu())
    dist.barrier()
    if rank == 0:
        lat_full = torch.cat(lat_parts, 2).contiguous().to(dev)
        x = torch.empty(B * world * F * h * w, den.x.shape[1], dtype=torch.bfloat16, device=dev)
        K.pack_latents(lat_full, x, sigmas=den.sigmas, step_idx=den.step_idx, ncopy=den.ncopy)
        ref = []
        for cls, fn in saved.items():
            cls.run = fn
        _recorder(U, unet, ref)
        with torch.no_grad():
            unet.forward_tokens(x, B, F * world, h, w, emb, den.enc)
        shards = [torch.load(f"/tmp/shard_diag_rank{r}.pt") for r in range(world)]
        assert all(len(s) == len(ref) for s in shards), (len(ref), [len(s) for s in shards])
        shown = 0
        for i, (kind, name, nimg_u, xin_u, y_u) in enumerate(ref):
            def assemble(idx):  # rows (b, f_local, p) per rank -> (b, f, p)
                parts = [s[i][idx] for s in shards]
                rows = parts[0].shape[0]
                per_b = rows // B
                return torch.cat([torch.stack([p[b * per_b:(b + 1) * per_b] for p in parts]) for b in range(B)]
                                 ).reshape(B * world * per_b, -1)
            y_s, x_s = assemble(4), assemble(3)
            if y_s.shape != y_u.shape:
                print(f"[{i}] {kind} {name}: shape {tuple(y_s.shape)} vs {tuple(y_u.shape)}")
                continue
            same_y, same_x = torch.equal(y_s, y_u), torch.equal(x_s, xin_u)
            if not same_y or not same_x:
                d = (y_s.float() - y_u.float()).abs().max().item()
                print(f"[{i}] {kind:7s} {name:50s} rows {y_u.shape[0]} C {y_u.shape[1]}: input equal {same_x}, "
                      f"output equal {same_y}, max|dy| {d:.3e}", flush=True)
                shown += 1
                if shown >= 12:
                    break
        if shown == 0:
            print(f"all {len(ref)} recorded layers bit-identical", flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--clips", type=int, default=2)
    ap.add_argument("--world", type=int, default=2)
    args = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_worker, args=(args.world, port, args), nprocs=args.world, join=True)


if __name__ == "__main__":
    main()
