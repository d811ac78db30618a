"""RCCL (torch.distributed "nccl" backend) on the GPU box, between HIP-graph replays.

The frame-sharded denoise step is captured piecewise (frame_shard.PiecewiseGraph): the kernels between two
collectives form one HIP graph and the collectives -- all_gather_into_tensor (motion-module GroupNorm partials),
all_to_all_single (frame shard <-> pixel shard), all_reduce -- run between the replays on the same stream.  (Capturing
the collectives themselves was measured on this box: all_reduce and all_gather_into_tensor replay, and a captured
all_to_all_single replays too but left the process hanging in destroy_process_group while the graph holding it was
still alive (profiles/r4_rccl_diag.log): RCCL keeps a persistent plan of a captured send/recv for as long as the graph
lives.  Destroying the graph first exits cleanly (profiles/r5_rccl_diag_del.log); the second test below pins that
teardown order.)
A one-GPU box can only run world size 1 (RCCL refuses two ranks on one device), so this test runs the piecewise
pattern with the nccl backend at world 1 in a child process -- eager step, piecewise capture, three replays checked,
process-group teardown -- so the driver's 8-GPU run is not the first execution of that pattern on RCCL."""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, time
t0 = time.time()
def log(m):
    print(f"[rccl child {time.time() - t0:6.1f}s] {m}", flush=True)
import torch, torch.distributed as dist
sys.path.insert(0, os.environ["VST_ROOT"])
from video_style_transfer_amd.frame_shard import PiecewiseGraph
log("torch imported")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
assert str(dist.get_backend()).lower() == "nccl"
log("nccl process group up")
n = 1 << 20
a = torch.zeros(n, device=dev); b = torch.zeros(n, device=dev); c = torch.zeros(3, 5, device=dev)
ga = torch.empty(1, 3, 5, device=dev); ta = torch.empty(n, device=dev)
def step(pw=None):
    issue = (lambda fn: pw.collective(fn)) if pw is not None else (lambda fn: fn())
    a.mul_(2.0); issue(lambda: dist.all_reduce(a)); a.add_(1.0)
    issue(lambda: dist.all_to_all_single(ta, b)); ta.mul_(3.0)
    issue(lambda: dist.all_gather_into_tensor(ga, c))
    ga.mul_(0.5)
step(); torch.cuda.synchronize()
log("eager step ok")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
pw = PiecewiseGraph()
pw.capture(lambda: step(pw), [], s)
assert pw.num_graphs == 4 and len(pw.items) == 7, (pw.num_graphs, len(pw.items))
log("captured piecewise: 4 graphs, 3 collectives")
for it in range(3):
    x = torch.randn(n, device=dev); y = torch.randn(n, device=dev); z = torch.randn(3, 5, device=dev)
    a.copy_(x); b.copy_(y); c.copy_(z)
    pw.replay()
    torch.cuda.synchronize()
    assert torch.equal(a, x * 2 + 1), "all_reduce between graphs"
    assert torch.equal(ta, y * 3), "all_to_all_single between graphs"
    assert torch.equal(ga[0], z * 0.5), "all_gather_into_tensor between graphs"
    log(f"replay {it} ok")
dist.destroy_process_group()
log("process group destroyed")
print("rccl piecewise ok: all_reduce, all_to_all_single, all_gather_into_tensor between HIP-graph replays, 3x")
"""


CHILD_WHOLE = r"""
import gc, os, sys, time
t0 = time.time()
def log(m):
    print(f"[rccl child {time.time() - t0:6.1f}s] {m}", flush=True)
import torch, torch.distributed as dist
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
n = 1 << 20
a = torch.zeros(n, device=dev); b = torch.zeros(n, device=dev); c = torch.zeros(3, 5, device=dev)
ga = torch.empty(1, 3, 5, device=dev); ta = torch.empty(n, device=dev)
def step():
    a.mul_(2.0); dist.all_reduce(a); a.add_(1.0)
    dist.all_to_all_single(ta, b); ta.mul_(3.0)
    dist.all_gather_into_tensor(ga, c); ga.mul_(0.5)
step(); torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    with torch.cuda.graph(g):
        step()
torch.cuda.current_stream().wait_stream(s)
log("captured: all_reduce, all_to_all_single, all_gather_into_tensor inside one graph")
for it in range(3):
    x = torch.randn(n, device=dev); y = torch.randn(n, device=dev); z = torch.randn(3, 5, device=dev)
    a.copy_(x); b.copy_(y); c.copy_(z)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(a, x * 2 + 1) and torch.equal(ta, y * 3) and torch.equal(ga[0], z * 0.5)
    log(f"replay {it} ok")
del g  # the graph (and RCCL's persistent plans of its collectives) before the communicator
gc.collect()
torch.cuda.synchronize()
dist.destroy_process_group()
log("graph released, then process group destroyed")
print("rccl whole-graph ok")
"""


CHILD_ASYNC = r"""
import os, sys, time
t0 = time.time()
def log(m):
    print(f"[rccl child {time.time() - t0:6.1f}s] {m}", flush=True)
import torch, torch.distributed as dist
sys.path.insert(0, os.environ["VST_ROOT"])
from video_style_transfer_amd.frame_shard import FrameShard, PiecewiseGraph
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
sh = FrameShard(exchange="all_to_all")
assert sh.backend == "nccl" and not sh._staged(torch.zeros(1, device=dev))
n = 1 << 22
a = torch.zeros(n, device=dev); b = torch.zeros(n, device=dev); c = torch.zeros(3, 5, device=dev)
ta = torch.empty(n, device=dev); g2 = torch.empty(3, 5, device=dev)
def step():
    # FrameShard's overlapped exchange primitives: the collective issued async on RCCL's stream, kernels queued
    # between the issue and the wait, then the compute stream waits for RCCL's
    b.mul_(2.0)
    w1 = sh._all_to_all_begin(ta, b)
    c.add_(1.0)
    for _ in range(4):
        a.mul_(1.0)
    w1()
    ta.mul_(3.0)
    w2 = sh._all_gather_begin(g2, c)
    a.mul_(2.0)
    w2()
    g2.mul_(0.5)
x = torch.randn(n, device=dev); y = torch.randn(n, device=dev); z = torch.randn(3, 5, device=dev)
a.copy_(x); b.copy_(y); c.copy_(z)
step(); torch.cuda.synchronize()
assert torch.equal(ta, y * 2 * 3) and torch.equal(g2, (z + 1) * 0.5) and torch.equal(a, x * 2)
log("eager async step ok")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
pw = PiecewiseGraph()
pw.capture(step, [sh], s)
assert pw.num_graphs == 5 and len(pw.items) == 9, (pw.num_graphs, len(pw.items))
log("captured piecewise: 5 graphs, 2 async issues + 2 waits")
for it in range(3):
    x = torch.randn(n, device=dev); y = torch.randn(n, device=dev); z = torch.randn(3, 5, device=dev)
    a.copy_(x); b.copy_(y); c.copy_(z)
    pw.replay()
    torch.cuda.synchronize()
    assert torch.equal(ta, y * 2 * 3), "async all_to_all_single between graphs"
    assert torch.equal(g2, (z + 1) * 0.5), "async all_gather_into_tensor between graphs"
    assert torch.equal(a, x * 2)
    log(f"replay {it} ok")
pw.items.clear()
dist.destroy_process_group()
log("process group destroyed")
print("rccl async piecewise ok")
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_world1_collectives_between_graph_replays():
    if torch.cuda.device_count() == 0:
        pytest.skip("no HIP device")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), VST_ROOT=ROOT,
               HSA_ENABLE_IPC_MODE_LEGACY="0", NCCL_DEBUG=os.environ.get("NCCL_DEBUG", "INFO"))
    # the child's output streams straight through (a first import on a fresh box can take a minute)
    out = os.path.join(ROOT, "gpurun_out", "rccl_child.log")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        r = subprocess.run([sys.executable, "-u", "-c", CHILD], env=env, stdout=f, stderr=subprocess.STDOUT, timeout=150)
    text = open(out).read()
    print(text[-4000:])
    assert r.returncode == 0 and "rccl piecewise ok" in text, text[-3000:]


@pytest.mark.gpu
def test_rccl_world1_collectives_captured_then_graph_released_first():
    """The round-4 hang's cause, pinned: collectives captured inside one HIP graph replay correctly, and with the graph
    released before destroy_process_group the process exits (the hang needed the graph to outlive the communicator)."""
    if torch.cuda.device_count() == 0:
        pytest.skip("no HIP device")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), VST_ROOT=ROOT,
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = os.path.join(ROOT, "gpurun_out", "rccl_child_whole.log")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        r = subprocess.run([sys.executable, "-u", "-c", CHILD_WHOLE], env=env, stdout=f, stderr=subprocess.STDOUT,
                           timeout=150)
    text = open(out).read()
    print(text[-3000:])
    assert r.returncode == 0 and "rccl whole-graph ok" in text, text[-3000:]


@pytest.mark.gpu
def test_rccl_world1_async_exchange_between_graph_replays():
    """FrameShard's overlapped-exchange primitives (_all_to_all_begin / _all_gather_begin: async_op=True on RCCL's
    stream, the wait as a later host item) under piecewise capture with the nccl backend at world 1: the exact code the
    N-GPU overlapped motion-module schedule runs between its graph pieces, on RCCL before any 8-GPU run."""
    if torch.cuda.device_count() == 0:
        pytest.skip("no HIP device")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), VST_ROOT=ROOT,
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = os.path.join(ROOT, "gpurun_out", "rccl_child_async.log")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        r = subprocess.run([sys.executable, "-u", "-c", CHILD_ASYNC], env=env, stdout=f, stderr=subprocess.STDOUT,
                           timeout=150)
    text = open(out).read()
    print(text[-3000:])
    assert r.returncode == 0 and "rccl async piecewise ok" in text, text[-3000:]
