"""Data-parallel training step (BASELINE configs[4], SURVEY 8(e) "Training (cfg 5)"): train.GradBucketAllReducer
replaces accelerate's DDP wrapper (train_animatediff.py:185-187 `accelerator.prepare`, :314 `accelerator.backward`),
train.TrainStep is the loop body (:214-319).

CPU (gloo, world size 2, spawned before anything touches a GPU):
  * the reducer's averaged gradients equal the mean of the per-rank gradients, over several buckets, with a parameter
    that one rank never uses (zero-filled, as DDP with find_unused_parameters) and one no rank uses, for two
    consecutive steps (bucket state resets);
  * full buckets launch during the backward (overlap), each bucket exactly once per step.
GPU (gloo transport, 2 ranks on one MI355X, HIP kernels): one TrainStep (orth loss, clip_grad_norm_, reducer) per
rank on its own clip equals one single-process TrainStep on the concatenated 2-clip batch with the same noise and
timesteps: same loss, same averaged + clipped gradients.
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


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _spawn(fn, world, *extra):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q) + extra) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=900) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    return res


# ------------------------------------------------------------------------------------- CPU
class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(32, 64)
        self.b = torch.nn.Linear(64, 64)
        self.c = torch.nn.Linear(64, 16)
        self.only_rank0 = torch.nn.Linear(16, 16)   # used by rank 0 only
        self.never = torch.nn.Linear(16, 16)        # used by no rank

    def forward(self, x, rank):
        h = self.c(torch.tanh(self.b(torch.tanh(self.a(x)))))
        if rank == 0:
            h = h + self.only_rank0(h)
        return h


def _data(rank, step):
    g = torch.Generator().manual_seed(100 * step + rank)
    return torch.randn(8, 32, generator=g), torch.randn(8, 16, generator=g)


def _reducer_worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        _init(rank, world, port)
        from video_style_transfer_amd.train import GradBucketAllReducer
        torch.manual_seed(0)
        net = _Net()
        # ~0.02 MB buckets: several buckets over the 5 layers
        red = GradBucketAllReducer(net.parameters(), bucket_mb=0.02)
        assert len(red.buckets) >= 3, red.bucket_sizes_mb()
        launched = []
        orig = red._launch

        def spy(b):
            launched.append((b, in_backward[0]))
            orig(b)
        red._launch = spy
        for step in range(2):
            launched.clear()
            net.zero_grad(set_to_none=True)
            x, y = _data(rank, step)
            in_backward = [True]
            ((net(x, rank) - y) ** 2).mean().backward()
            in_backward[0] = False
            red.finish()
            got = {n: p.grad.clone() for n, p in net.named_parameters()}
            # reference: the per-rank gradients, averaged (every rank recomputes all ranks' data locally)
            ref = {n: torch.zeros_like(p) for n, p in net.named_parameters()}
            for r in range(world):
                ref_net = _Net()
                ref_net.load_state_dict(net.state_dict())
                xr, yr = _data(r, step)
                ((ref_net(xr, r) - yr) ** 2).mean().backward()
                for n, p in ref_net.named_parameters():
                    if p.grad is not None:
                        ref[n] += p.grad / world
            for n in got:
                err = (got[n] - ref[n]).abs().max().item()
                assert err < 1e-6, f"step {step} {n}: max err {err}"
            assert torch.count_nonzero(got["never.weight"]) == 0
            ids = sorted(b for b, _ in launched)
            assert ids == list(range(len(red.buckets))), f"each bucket once per step: {launched}"
            assert any(during for _, during in launched), "no bucket launched during the backward"
            with torch.no_grad():  # a plain SGD step so step 2 runs on new weights
                for p in net.parameters():
                    p -= 0.1 * p.grad
        q.put((rank, "ok", f"{len(red.buckets)} buckets"))
    except BaseException as e:  # noqa: BLE001
        import traceback
        q.put((rank, "fail", traceback.format_exc()[-2000:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_grad_bucket_all_reducer_cpu_world2():
    res = _spawn(_reducer_worker, 2)
    for rank, status, info in res:
        assert status == "ok", f"rank {rank}: {info}"


# ------------------------------------------------------------------------------------- GPU
def _train_setup(dev, config="tiny"):
    from video_style_transfer_amd.config import UNetMotionConfig
    from video_style_transfer_amd.temporal_lora import TemporalLoRALinear, build_spatial_lora_index, \
        inject_temporal_lora
    from video_style_transfer_amd.utils import build_unet, freeze_spatial_layers
    cfg = UNetMotionConfig.tiny() if config == "tiny" else UNetMotionConfig.sdxl()
    unet = build_unet(cfg, seed=3, lora_rank=8, device=dev)
    torch.manual_seed(4)
    inject_temporal_lora(unet, rank=4 if config == "tiny" else 32, alpha=1.0)
    with torch.no_grad():
        for m in unet.modules():
            if isinstance(m, TemporalLoRALinear):
                m.lora_B.normal_(0, 0.02)  # B = 0 at init would make the orth loss and its gradient vanish
    freeze_spatial_layers(unet)
    return cfg, unet, build_spatial_lora_index(unet)


def _clip_inputs(cfg, nclip=2, F=4, h=8):
    if cfg.block_out_channels[0] == 320:  # SDXL: BASELINE configs[4]'s clip, 16 frames at 512^2
        F, h = 16, 64
    g = torch.Generator().manual_seed(5)
    lat = torch.randn(nclip, 4, F, h, h, generator=g)
    noise = torch.randn(nclip, 4, F, h, h, generator=g)
    t = torch.tensor([101, 777])[:nclip]
    enc = torch.randn(1, 77, cfg.cross_attention_dim, generator=g)
    pooled = torch.randn(1, cfg.text_embed_dim, generator=g)
    return lat, noise, t, enc, pooled


def _run_step(unet, index, lat, noise, t, enc, pooled, reducer=None, sdxl=False):
    from video_style_transfer_amd.scheduler import EulerDiscreteScheduler
    from video_style_transfer_amd.train import TrainStep
    params = [p for p in unet.parameters() if p.requires_grad]
    opt = torch.optim.SGD(params, lr=0.0)  # lr 0: the weights stay comparable; the gradients are the check
    # SDXL: the reference's orth weight and clip (train_animatediff.py:414, :394); tiny: large enough to matter
    step = TrainStep(unet, opt, EulerDiscreteScheduler(), reducer=reducer, lambda_orth=1e-4 if sdxl else 0.5,
                     spatial_index=index, max_grad_norm=0.5 if sdxl else 0.05, resolution=512 if sdxl else 64)
    dev = next(unet.parameters()).device
    out = step(lat.to(dev), enc, pooled, noise=noise, timesteps=t, use_uncond=False)
    grads = {n: p.grad.detach().float().cpu() for n, p in unet.named_parameters() if p.requires_grad}
    return out, grads


def _dp_gpu_worker(rank, world, port, q, config="tiny"):
    try:
        sys.path.insert(0, ROOT)
        _init(rank, world, port)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        from video_style_transfer_amd.train import GradBucketAllReducer
        sdxl = config == "sdxl"
        cfg, unet, index = _train_setup(dev, config)
        assert index, "orth-loss pairing found no spatial partner"
        lat, noise, t, enc, pooled = _clip_inputs(cfg)
        sl = slice(rank, rank + 1)
        red = GradBucketAllReducer([p for p in unet.parameters() if p.requires_grad],
                                   bucket_mb=64.0 if sdxl else 1.0)
        out, grads = _run_step(unet, index, lat[sl], noise[sl], t[sl], enc, pooled, red, sdxl)
        red.remove()
        del unet, red
        torch.cuda.empty_cache()
        loss = torch.tensor([float(out["loss_mse"])])
        dist.all_reduce(loss)
        if rank == 0:
            cfg, unet1, index1 = _train_setup(dev, config)
            out1, grads1 = _run_step(unet1, index1, lat, noise, t, enc, pooled, sdxl=sdxl)
            errs = {n: ((grads[n] - grads1[n]).norm() / grads1[n].norm().clamp_min(1e-20)).item() for n in grads1}
            worst = max(errs, key=errs.get)
            lm, l1 = float(loss) / world, float(out1["loss_mse"])
            info = (f"loss_mse dp {lm:.6f} single {l1:.6f}; orth {float(out['loss_orth']):.4e} vs "
                    f"{float(out1['loss_orth']):.4e}; grad_norm {float(out['grad_norm']):.4e} vs "
                    f"{float(out1['grad_norm']):.4e}; worst grad {worst} rel {errs[worst]:.2e} over {len(errs)}")
            # SDXL: the two ranks' B=1 backward and the B=2 backward round differently in bf16 through the 70-block
            # spatial stack (each is ~4e-2 from fp32, test_training_gpu.py), so 5e-2; tiny: 2e-2
            ok = (abs(lm - l1) <= 1e-3 * abs(l1) and errs[worst] < (5e-2 if sdxl else 2e-2)
                  and float(out1["loss_orth"]) > 0
                  and abs(float(out["loss_orth"]) - float(out1["loss_orth"])) <= 1e-5 * float(out1["loss_orth"]))
            q.put((rank, "ok" if ok else "fail", info))
        else:
            q.put((rank, "ok", ""))
        dist.barrier()
    except BaseException:  # noqa: BLE001
        import traceback
        q.put((rank, "fail", traceback.format_exc()[-2000:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["tiny", "sdxl"])
def test_train_step_data_parallel_two_ranks_one_gpu(config):
    """sdxl: BASELINE configs[4]'s workload (SDXL + motion modules, UnZipLoRA r=8 frozen, temporal LoRA r=32, one
    16x512^2 clip per rank, 64 MB buckets) -- the two ranks' bucketed average equals the 2-clip batch."""
    if torch.cuda.device_count() == 0:
        pytest.skip("no HIP device")
    res = _spawn(_dp_gpu_worker, 2, config)
    for rank, status, info in res:
        print(f"[dp] rank {rank}: {status} {info}")
        assert status == "ok", f"rank {rank}: {info}"
