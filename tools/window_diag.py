"""Where does a captured accumulation window differ from the eager one?  (diagnostic, GPU)

Tiny UNet, 2 micro-batches, the three models built first (as tests/test_train_step_gpu.py does): gradients of
TrainStep.window (eager), of the captured window (its final in-place zeroing disabled so they survive the replay)
and of the two sequential calls, per trainable tensor.

  python tools/window_diag.py [clip] [lr] [sched 0|1]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_train_step_gpu import _model, _text  # noqa: E402
from video_style_transfer_amd.config import UNetMotionConfig  # noqa: E402
from video_style_transfer_amd.scheduler import EulerDiscreteScheduler  # noqa: E402
from video_style_transfer_amd.train import TrainStep, get_scheduler, make_adamw  # noqa: E402


def main():
    clip = float(sys.argv[1]) if len(sys.argv) > 1 else 0.5
    lr = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-3
    sched = len(sys.argv) > 3 and sys.argv[3] == "1"
    print(f"clip {clip} lr {lr} sched {sched}")
    dev = torch.device("cuda")
    cfg = UNetMotionConfig.tiny()
    accum = 2
    enc, pooled, unc, unp = _text(cfg)
    lat = torch.randn(accum, 4, 4, 8, 8, generator=torch.Generator().manual_seed(31)).to(dev)
    kw = dict(lambda_orth=1e-2, max_grad_norm=clip, resolution=64, seed=13, gradient_accumulation_steps=accum)
    modes = ("window", "graph", "seq")
    steps = {}
    for mode in modes:
        u, idx = _model(cfg, dev, 8, 4)
        names = [n for n, p in u.named_parameters() if p.requires_grad]
        ps = [p for p in u.parameters() if p.requires_grad]
        opt = make_adamw(ps, lr=lr, capturable=True)
        steps[mode] = (TrainStep(u, opt, EulerDiscreteScheduler(), spatial_index=idx,
                                 lr_scheduler=get_scheduler("cosine", opt, 1, 6) if sched else None, **kw), ps)
    rec = []
    if os.environ.get("DIAG_REC"):
        from video_style_transfer_amd import autograd as A
        from video_style_transfer_amd import kernels as K
        variant = os.environ["DIAG_REC"]

        def bw(ctx, g):  # GEGLUFn.backward with the bias reduction recorded (and optionally changed)
            (x2d,) = ctx.saved_tensors
            Wi, bi = ctx.geglu.geglu_ops()
            M = x2d.shape[0]
            pp = K.linear(x2d, Wi, bi)
            dp = K.geglu_bwd(pp, g.to(torch.bfloat16).contiguous())
            need_x, need_w, need_b = ctx.needs_input_grad[:3]
            dX = dW = db = None
            if need_x:
                dX = K.linear(dp, A._geglu_wt(ctx.geglu))
            if need_w:
                Mp = (M + 7) // 8 * 8
                dW = A._deinterleave32(K.linear(A._transpose_padded(dp, Mp), A._transpose_padded(x2d, Mp))).to(
                    ctx.w_dtype)
            if need_b:
                t_early = None
                if variant == "dtype":
                    s_ = dp.sum(0, dtype=torch.float32)
                else:
                    t = dp.float()
                    if torch.cuda.is_current_stream_capturing():
                        t_early = t.clone()
                    s_ = t.sum(0)
                early = s_.clone() if torch.cuda.is_current_stream_capturing() else None
                db = A._deinterleave32(s_).to(ctx.b_dtype)
                if early is not None:
                    rec.append((ctx.geglu, db, early, s_, dp.clone(), t_early))
            return dX, dW, db, None
        A.GEGLUFn.backward = staticmethod(bw)
    real = torch._foreach_zero_
    torch._foreach_zero_ = lambda ts: None if torch.cuda.is_current_stream_capturing() else real(ts)
    try:
        steps["graph"][0].capture(lat, enc, pooled, uncond_prompt=unc, uncond_pooled=unp, window=True)
    finally:
        torch._foreach_zero_ = real
    res = {}
    for mode in modes:
        st, ps = steps[mode]
        if mode == "window":
            out = st.window(lat, enc, pooled, unc, unp)
        elif mode == "graph":
            out = st.replay(lat)
        else:
            for i in range(accum):
                out = st(lat[i:i + 1], enc, pooled, unc, unp)
        torch.cuda.synchronize()
        res[mode] = (float(out["loss"]), float(out["grad_norm"]), [p.grad.detach().float().clone() for p in ps])
        print(f"{mode}: loss {res[mode][0]:.7f} grad_norm {res[mode][1]:.6e} uncond {out['uncond']}", flush=True)
    if rec:
        u = steps["graph"][0].unet
        mod2name = {m: n for n, m in u.named_modules()}
        gmap = dict(u.named_parameters())
        for m, db, early, s_, dp, t_early in rec:
            n = mod2name.get(m, "?")
            ref = dp.float().sum(0)
            if t_early is not None:
                print(f"  t(early clone) vs dp.float(): rel {((t_early - dp.float()).norm() / dp.float().norm()):.3e};"
                      f" |t_early.sum(0)| {t_early.sum(0).norm():.4e}")
            print(f"  rec {n}: |dp| {dp.float().norm():.4e} |sum ref| {ref.norm():.4e} |sum early clone| "
                  f"{early.norm():.4e} |sum after| {s_.norm():.4e} |db| {db.float().norm():.4e}", flush=True)
    for a, b in (("window", "graph"), ("window", "seq")):
        bad = []
        for n, x, y in zip(names, res[a][2], res[b][2]):
            e = ((x - y).norm() / y.norm().clamp_min(1e-30)).item()
            if e > 1e-2:
                bad.append((n, e, x.norm().item(), y.norm().item()))
        print(f"{a} vs {b}: {len(bad)} of {len(names)} tensors differ > 1e-2")
        for row in bad[:12]:
            print("   ", row)


if __name__ == "__main__":
    main()
