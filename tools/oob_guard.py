"""Out-of-bounds write detector for the HIP launches (diagnostic, GPU; eager only).

Every device tensor made through torch.empty / zeros / empty_like / zeros_like / full is carved out of a larger
buffer with GUARD bytes of a sentinel pattern before and after it.  After every libvst_hip launch (_lib.call) the
stream is synchronised and the guards of every buffer that one of the launch's pointer arguments points into are
checked; the first launch that changed a guard is reported with its arguments, and the script stops.

  python tools/oob_guard.py [tiny|tiny-seq] [accum]
"""
import bisect
import os
import sys
import weakref

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

GUARD = 1 << 16
SENT = 0xA5
_bufs = {}      # start address of the whole buffer -> (weakref to the uint8 buffer, payload bytes)
_starts = []    # sorted start addresses
_real = {n: getattr(torch, n) for n in ("empty", "zeros", "empty_like", "zeros_like", "full")}
_checked = [0]


def _is_cuda(device):
    return device is not None and torch.device(device).type == "cuda"


def _carve(shape, dtype, device, fill=None):
    if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)):
        shape = tuple(shape[0])
    shape = tuple(int(s) for s in shape)
    dtype = dtype or torch.get_default_dtype()
    n = 1
    for s in shape:
        n *= s
    es = torch.empty((), dtype=dtype).element_size()
    nbytes = n * es
    buf = _real["empty"](GUARD * 2 + nbytes, dtype=torch.uint8, device=device)
    buf.fill_(SENT)
    t = buf[GUARD:GUARD + nbytes].view(dtype).view(shape)
    if fill is not None:
        t.fill_(fill)
    a = buf.data_ptr()
    _bufs[a] = (weakref.ref(buf), nbytes)
    bisect.insort(_starts, a)
    t._oob_buf = buf  # keep the guarded buffer alive with the view
    return t


def _mk(name, fill):
    def f(*shape, dtype=None, device=None, **kw):
        if not _is_cuda(device) or kw.get("out") is not None or kw.get("layout") not in (None, torch.strided):
            return _real[name](*shape, dtype=dtype, device=device, **kw)
        return _carve(shape, dtype, device, fill)
    return f


def _mk_like(name, fill):
    def f(x, dtype=None, device=None, **kw):
        dev = device if device is not None else x.device
        if not _is_cuda(dev) or kw.get("memory_format") not in (None, torch.preserve_format, torch.contiguous_format):
            return _real[name](x, dtype=dtype, device=device, **kw)
        return _carve(tuple(x.shape), dtype or x.dtype, dev, fill)
    return f


def _full(size, fill_value, dtype=None, device=None, **kw):
    if not _is_cuda(device) or kw:
        return _real["full"](size, fill_value, dtype=dtype, device=device, **kw)
    return _carve(tuple(size), dtype, device, fill_value)


def install():
    torch.empty = _mk("empty", None)
    torch.zeros = _mk("zeros", 0)
    torch.empty_like = _mk_like("empty_like", None)
    torch.zeros_like = _mk_like("zeros_like", 0)
    torch.full = _full
    from video_style_transfer_amd import _lib
    real_call = _lib.call

    def call(name, *args):
        rc = real_call(name, *args)
        torch.cuda.synchronize()
        _checked[0] += 1
        for a in args:
            if not isinstance(a, int) or a < 1 << 20:
                continue
            i = bisect.bisect_right(_starts, a) - 1
            if i < 0:
                continue
            start = _starts[i]
            ref, nbytes = _bufs[start]
            buf = ref()
            if buf is None or not (start <= a < start + 2 * GUARD + nbytes):
                continue
            lo = buf[:GUARD]
            hi = buf[GUARD + nbytes:]
            blo = int((lo != SENT).sum())
            bhi = int((hi != SENT).sum())
            if blo or bhi:
                first = int((hi != SENT).nonzero()[0]) if bhi else -int((lo != SENT).nonzero()[-1])
                print(f"OOB after launch #{_checked[0]} {name}: buffer of {nbytes} bytes (arg at offset "
                      f"{a - start - GUARD}); {blo} guard bytes changed before it, {bhi} after it (first at +{first})")
                print("   args:", args)
                import traceback
                traceback.print_stack(limit=12)
                sys.exit(3)
        return rc
    _lib.call = call


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "tiny"
    accum = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    from test_train_step_gpu import _model, _text
    from video_style_transfer_amd.config import UNetMotionConfig
    from video_style_transfer_amd.scheduler import EulerDiscreteScheduler
    from video_style_transfer_amd.train import TrainStep, make_adamw
    dev = torch.device("cuda")
    cfg = UNetMotionConfig.tiny()
    enc, pooled, unc, unp = _text(cfg)
    lat = torch.randn(accum, 4, 4, 8, 8, generator=torch.Generator().manual_seed(31)).to(dev)
    u, idx = _model(cfg, dev, 8, 4)
    install()  # after construction (meta-device init); every activation, gradient and workspace is guarded
    ps = [p for p in u.parameters() if p.requires_grad]
    opt = make_adamw(ps, lr=1e-3, capturable=True)
    st = TrainStep(u, opt, EulerDiscreteScheduler(), spatial_index=idx, lambda_orth=1e-2, max_grad_norm=0.5,
                   resolution=64, seed=13, gradient_accumulation_steps=accum)
    for w in range(2):
        if which == "tiny-seq":
            for i in range(accum):
                st(lat[i:i + 1], enc, pooled, unc, unp)
        else:
            st.window(lat, enc, pooled, unc, unp)
        torch.cuda.synchronize()
        print(f"window {w}: {_checked[0]} launches checked, no guard changed", flush=True)


if __name__ == "__main__":
    main()
