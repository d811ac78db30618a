"""Host logic of the training step (BASELINE configs[4], train_animatediff.py:51-54, :180-184, :214-319), on the CPU.

The optimisation bookkeeping of train.TrainStep -- gradient accumulation, when the gradients are all-reduced, clipped,
stepped and zeroed, and how the lr scheduler advances -- is pinned against the reference's own dependencies, which
are importable here: accelerate (the `Accelerator(gradient_accumulation_steps=N)` / `accelerator.accumulate` loop
of the reference, run verbatim on a toy model) and transformers (whose get_*_schedule_with_warmup diffusers'
get_scheduler restates).  The UNet forward is replaced by a toy model through TrainStep._loss, so only the
bookkeeping is under test here; tests/test_training_gpu.py runs the same logic on the HIP UNet.
"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Sched:
    num_train_timesteps = 1000


class _Toy(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(16, 32)
        self.b = torch.nn.Linear(32, 16)
        self.frozen = torch.nn.Linear(16, 16).requires_grad_(False)

    def loss(self, latents, noise, t):
        x = (latents + noise * (t.float().view(-1, 1, 1, 1, 1) / 1000.0)).reshape(-1, 16)
        pred = self.b(torch.tanh(self.a(self.frozen(x))))
        return torch.mean((pred - noise.reshape(-1, 16)) ** 2)


def _toy_step_cls():
    from video_style_transfer_amd.train import TrainStep

    class ToyStep(TrainStep):
        def _loss(self, latents, noise, t, enc, pool):
            mse = self.unet.loss(latents, noise, t)
            return mse, mse, torch.zeros(())
    return ToyStep


def _batches(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(1, 4, 2, 2, 2, generator=g), torch.randn(1, 4, 2, 2, 2, generator=g),
             torch.randint(0, 1000, (1,), generator=g)) for _ in range(n)]


def test_get_scheduler_matches_transformers():
    """diffusers' get_scheduler restated (train.get_scheduler) == transformers' published schedules (diffusers copies
    them): the reference's default cosine with 100 warm-up steps over 1000, and the linear / constant variants."""
    import transformers
    from video_style_transfer_amd.train import get_scheduler

    def lrs(make, n):
        p = torch.nn.Parameter(torch.zeros(2))
        opt = torch.optim.SGD([p], lr=2e-5)
        s = make(opt)
        out = []
        for _ in range(n):
            out.append(opt.param_groups[0]["lr"])
            opt.step()
            s.step()
        return out

    cases = [("cosine", transformers.get_cosine_schedule_with_warmup, 100, 1000),
             ("linear", transformers.get_linear_schedule_with_warmup, 10, 50),
             ("constant_with_warmup", lambda o, w, n: transformers.get_constant_schedule_with_warmup(o, w), 7, 30)]
    for name, ref, w, n in cases:
        got = lrs(lambda o: get_scheduler(name, o, w, n), n + 5)
        want = lrs(lambda o: ref(o, w, n), n + 5)
        assert got == pytest.approx(want, rel=1e-12, abs=1e-18), name
    assert lrs(lambda o: get_scheduler("constant", o), 3) == [2e-5] * 3
    with pytest.raises(ValueError):
        get_scheduler("cosine_with_restarts", torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=1.0))


@pytest.mark.parametrize("accum", [1, 4])
def test_train_step_accumulation_matches_accelerate(accum):
    """train_animatediff.py's loop (:214-319) run verbatim through accelerate 1.x on a toy model vs TrainStep on the
    same model and micro-batches: the parameters after every call, the lr after every call, and which calls stepped
    the optimizer, for gradient_accumulation_steps 1 and 4 (the reference default), with the reference's cosine
    schedule (warm-up 3 of 20 here, so the lr moves every optimizer step), AdamW and clip_grad_norm_."""
    from accelerate import Accelerator
    from accelerate.state import AcceleratorState, GradientState
    from video_style_transfer_amd.train import get_scheduler
    AcceleratorState._reset_state(True)
    GradientState._reset_state()
    ToyStep = _toy_step_cls()
    n_calls = 4 * accum + 2
    batches = _batches(n_calls)
    torch.manual_seed(0)
    ref_model = _Toy()
    ours = _Toy()
    ours.load_state_dict(ref_model.state_dict())

    acc = Accelerator(gradient_accumulation_steps=accum, mixed_precision="no", cpu=True)
    r_params = [p for p in ref_model.parameters() if p.requires_grad]
    r_opt = torch.optim.AdamW(r_params, lr=1e-2, betas=(0.9, 0.999), weight_decay=1e-2, eps=1e-8)
    r_sched = get_scheduler("cosine", r_opt, 3, 20)
    ref_model, r_opt, r_sched = acc.prepare(ref_model, r_opt, r_sched)
    ref_traj = []
    for lat, noise, t in batches:
        with acc.accumulate(ref_model):
            loss = ref_model.loss(lat, noise, t)
            acc.backward(loss)
            if acc.sync_gradients:
                acc.clip_grad_norm_(r_params, 0.05)
            r_opt.step()
            r_sched.step()
            r_opt.zero_grad()
        ref_traj.append(([p.detach().clone() for p in r_params], r_opt.param_groups[0]["lr"], acc.sync_gradients))

    o_params = [p for p in ours.parameters() if p.requires_grad]
    o_opt = torch.optim.AdamW(o_params, lr=1e-2, betas=(0.9, 0.999), weight_decay=1e-2, eps=1e-8)
    step = ToyStep(ours, o_opt, _Sched(), max_grad_norm=0.05, lr_scheduler=get_scheduler("cosine", o_opt, 3, 20),
                   gradient_accumulation_steps=accum, num_processes=1)
    enc, pool = torch.zeros(1, 77, 8), torch.zeros(1, 8)
    moved = 0
    for i, (lat, noise, t) in enumerate(batches):
        before = [p.detach().clone() for p in o_params]
        out = step(lat, enc, pool, noise=noise, timesteps=t, use_uncond=False)
        want_p, want_lr, want_sync = ref_traj[i]
        assert out["sync"] == want_sync, i
        assert o_opt.param_groups[0]["lr"] == pytest.approx(want_lr, rel=1e-12, abs=0), i
        for p, w in zip(o_params, want_p):
            torch.testing.assert_close(p.detach(), w, rtol=1e-6, atol=1e-7, msg=f"call {i}")
        changed = any(not torch.equal(p, b) for p, b in zip(o_params, before))
        moved += changed
        # the first optimizer step runs at lr 0 (warm-up from 0), so it only shows up in the moments
        assert changed == (want_sync and i >= accum), i
        if not out["sync"]:
            assert torch.isnan(out["grad_norm"]), i
    assert moved == n_calls // accum - 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dp_accum_worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from video_style_transfer_amd.train import GradBucketAllReducer, get_scheduler
        ToyStep = _toy_step_cls()
        accum = 3
        batches = _batches(world * accum, seed=11)
        torch.manual_seed(0)
        model = _Toy()
        params = [p for p in model.parameters() if p.requires_grad]
        red = GradBucketAllReducer(params, bucket_mb=0.002)
        launched = []
        orig = red._launch

        def spy(b):
            launched.append(b)
            orig(b)
        red._launch = spy
        opt = torch.optim.SGD(params, lr=0.5)
        sched = get_scheduler("constant_with_warmup", opt, 8, 100)
        step = ToyStep(model, opt, _Sched(), reducer=red, max_grad_norm=1e9, lr_scheduler=sched,
                       gradient_accumulation_steps=accum)
        assert step.num_processes == world
        enc, pool = torch.zeros(1, 77, 8), torch.zeros(1, 8)
        mine = batches[rank * accum:(rank + 1) * accum]   # this rank's micro-batches of the window
        import copy
        ref = copy.deepcopy(model)
        for k, (lat, noise, t) in enumerate(mine):
            out = step(lat, enc, pool, noise=noise, timesteps=t, use_uncond=False)
            if k < accum - 1:
                assert not out["sync"] and not launched, f"collective on a no_sync call {k}: {launched}"
        assert out["sync"] and sorted(launched) == list(range(len(red.buckets))), launched
        # DDP + accumulation == the gradient of the mean loss over all world*accum micro-batches, one SGD step at the
        # lr of scheduler step 0, i.e. 0: the weights stay put and the reduced .grad is compared)
        rp = [p for p in ref.parameters() if p.requires_grad]
        for lat, noise, t in batches:
            (ref.loss(lat, noise, t) / len(batches)).backward()
        for p, r in zip(params, rp):
            torch.testing.assert_close(p.grad, r.grad, rtol=1e-5, atol=1e-7)
        # the scheduler advanced once per process on the sync call (AcceleratedScheduler, split_batches=False)
        assert sched.last_epoch == world and opt.param_groups[0]["lr"] == pytest.approx(0.5 * world / 8)
        q.put((rank, "ok", f"{len(red.buckets)} buckets"))
    except BaseException:  # noqa: BLE001
        import traceback
        q.put((rank, "fail", traceback.format_exc()[-2000:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_train_step_accumulation_data_parallel_cpu_world2():
    """gloo world 2, gradient_accumulation_steps 3: no collective on the two no_sync calls, every bucket reduced once
    on the sync call, the averaged gradient equals that of the mean loss over all 6 micro-batches, and the lr
    scheduler advanced world-size times."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_accum_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, status, info in res:
        assert status == "ok", f"rank {rank}: {info}"


def test_train_step_window_equals_sequential_calls():
    """TrainStep.window (the accumulation window as ONE batched forward / backward) == the N sequential calls it
    replaces: same random draws (in the calls' order), same accumulated gradient, weights and lr after the step."""
    from video_style_transfer_amd.train import get_scheduler
    ToyStep = _toy_step_cls()
    accum = 3
    lat = torch.cat([b[0] for b in _batches(2 * accum, seed=21)])
    enc, pool = torch.zeros(1, 77, 8), torch.zeros(1, 8)

    def make():
        torch.manual_seed(3)
        m = _Toy()
        ps = [p for p in m.parameters() if p.requires_grad]
        opt = torch.optim.AdamW(ps, lr=1e-2)
        return m, ps, opt, ToyStep(m, opt, _Sched(), max_grad_norm=0.05, seed=4,
                                   lr_scheduler=get_scheduler("cosine", opt, 2, 10), gradient_accumulation_steps=accum,
                                   num_processes=1)
    m1, p1, o1, s1 = make()
    m2, p2, o2, s2 = make()
    for w in range(2):  # two windows: the second one moves the weights (warm-up lr 0 on the first)
        chunk = lat[w * accum:(w + 1) * accum]
        outs = [s1(chunk[i:i + 1], enc, pool, enc, pool) for i in range(accum)]
        ow = s2.window(chunk, enc, pool, enc, pool)
        assert [o["uncond"] for o in outs] == ow["uncond"]
        assert torch.equal(torch.cat([o["timesteps"] for o in outs]), ow["timesteps"])
        assert float(ow["loss"]) == pytest.approx(sum(float(o["loss"]) for o in outs) / accum, rel=1e-5)
        assert float(ow["grad_norm"]) == pytest.approx(float(outs[-1]["grad_norm"]), rel=1e-5)
        for a, b in zip(p1, p2):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7)
        assert o1.param_groups[0]["lr"] == o2.param_groups[0]["lr"] and s1.micro == s2.micro == 0
        assert s1.lr_scheduler._step_count == s2.lr_scheduler._step_count
