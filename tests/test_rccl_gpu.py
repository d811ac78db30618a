"""RCCL (torch.distributed "nccl" backend) on the GPU box, captured in a HIP graph.

The frame-sharded denoise step (frame_shard.py) and the data-parallel training step put RCCL collectives inside
the step's captured HIP graph: all_gather_into_tensor (motion-module GroupNorm partials), all_to_all_single (frame
shard <-> pixel shard) and all_reduce (the DP gradient buckets, train.GradBucketAllReducer).  A one-GPU box can
only run world size 1 (RCCL refuses two ranks on one device), so this test initialises the nccl backend at world
1 in a child process, captures the three collectives in a torch.cuda.graph on a side stream, replays the graph
with new inputs and checks every output; then the same through FrameShard's own methods.  The driver's 8-GPU run
is then not the first time RCCL stream capture executes."""
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
log("torch imported")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
assert str(dist.get_backend()).lower() == "nccl"
log("nccl process group up")
n = 1 << 20
a = torch.zeros(n, device=dev); b = torch.zeros(n, device=dev); c = torch.zeros(3, 5, device=dev)
ga = torch.empty(1, 3, 5, device=dev); ta = torch.empty(n, device=dev)
for _ in range(2):  # warm-up on a side stream (communicator setup outside the capture)
    dist.all_reduce(a); dist.all_to_all_single(ta, b); dist.all_gather_into_tensor(ga, c)
torch.cuda.synchronize()
log("eager collectives done")
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    with torch.cuda.graph(g):
        a.mul_(2.0); dist.all_reduce(a); a.add_(1.0)
        dist.all_to_all_single(ta, b); ta.mul_(3.0)
        dist.all_gather_into_tensor(ga, c)
torch.cuda.current_stream().wait_stream(s)
log("captured")
for it in range(3):
    x = torch.randn(n, device=dev); y = torch.randn(n, device=dev); z = torch.randn(3, 5, device=dev)
    a.copy_(x); b.copy_(y); c.copy_(z)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(a, x * 2 + 1), "all_reduce in graph"
    assert torch.equal(ta, y * 3), "all_to_all_single in graph"
    assert torch.equal(ga[0], z), "all_gather_into_tensor in graph"
# FrameShard's own methods on the nccl backend (world 1: the collectives short-circuit only where P == 1 is exact)
from video_style_transfer_amd.frame_shard import FrameShard
sh = FrameShard()
assert sh.graph_capturable and sh.world == 1
p = torch.randn(4, 8, 32, 2, device=dev)
g2 = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    with torch.cuda.graph(g2):
        out = sh.all_gather(p)
torch.cuda.current_stream().wait_stream(s)
p.copy_(torch.randn_like(p)); g2.replay(); torch.cuda.synchronize()
assert out.shape == (1, 4, 8, 32, 2) and torch.equal(out[0], p), "FrameShard.all_gather in graph"
dist.destroy_process_group()
print("rccl capture ok: all_reduce, all_to_all_single, all_gather_into_tensor replayed 3x in a HIP graph")
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_world1_collectives_in_hip_graph():
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
    assert r.returncode == 0 and "rccl capture ok" in text, text[-3000:]
