"""Do torch's own reductions give eager results inside a captured HIP graph?  (diagnostic, GPU)

Each case captures a graph of R repetitions of a reduction on fresh inputs, with scratch tensors filled with junk
and freed in between (so the graph pool hands recycled, dirty memory to the next allocation), replays it, and
compares every result with the same reduction run eagerly.  Column sums of [M, N] with large M reduce across
workgroups through a global staging buffer whose semaphores torch zeroes with a memset; if a captured memset does
not take effect the column sums come back wrong.

  python tools/graph_reduce_check.py
"""
import torch


def case(name, fn, shape, dtype, R=24):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(1)
    xs = [torch.randn(*shape, generator=g, device=dev).to(dtype) for _ in range(R)]
    want = [fn(x) for x in xs]
    torch.cuda.synchronize()
    outs = []
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up
        for x in xs[:2]:
            fn(x)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for i, x in enumerate(xs):
            junk = torch.empty(128 * (1 + i % 5), device=dev).fill_(12345.0)
            del junk  # freed before the reduction: its (small-pool) block is what the next small allocation gets
            outs.append(fn(x))
    graph.replay()
    torch.cuda.synchronize()
    bad = 0
    worst = 0.0
    for o, w in zip(outs, want):
        e = ((o.float() - w.float()).norm() / w.float().norm().clamp_min(1e-30)).item()
        worst = max(worst, e)
        bad += e > 1e-4
    print(f"{name:38s} {str(shape):16s} {str(dtype):15s}: {bad:2d} of {R} replayed results differ from eager "
          f"(worst rel {worst:.2e})", flush=True)
    return bad


def memset_case(nbytes, R=16):
    """hipMemsetAsync captured into the graph on a recycled, dirty block; the zeroed bytes are copied out."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    dev = torch.device("cuda")
    n = max(1, nbytes // 4)
    outs = []
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for i in range(R):
            junk = torch.empty(n, device=dev).fill_(777.0)
            del junk
            z = torch.empty(n, device=dev)
            rc = hip.hipMemsetAsync(z.data_ptr(), 0, n * 4, torch.cuda.current_stream().cuda_stream)
            assert rc == 0, rc
            outs.append(z.clone())
    graph.replay()
    torch.cuda.synchronize()
    bad = sum(int((o != 0).any()) for o in outs)
    print(f"captured hipMemsetAsync of {n * 4:8d} B on a dirty recycled block: {bad:2d} of {R} not zero", flush=True)
    return bad


def main():
    total = 0
    for nb in (16, 512, 4096, 65536, 1 << 20):
        total += memset_case(nb)
    for shape in ((512, 512), (2048, 64), (65536, 1280), (16384, 2560), (4096, 320)):
        total += case("x.float().sum(0)", lambda x: x.float().sum(0), shape, torch.bfloat16)
        total += case("x.sum(0, dtype=float32)", lambda x: x.sum(0, dtype=torch.float32), shape, torch.bfloat16)
        total += case("x.sum(0) fp32", lambda x: x.sum(0), shape, torch.float32)
    for n in (1 << 20, 1 << 22):
        total += case("mean((x - 0.5)**2)", lambda x: torch.mean((x.float() - 0.5) ** 2), (n,), torch.bfloat16)
    print(f"total mismatching results: {total}")


if __name__ == "__main__":
    main()
