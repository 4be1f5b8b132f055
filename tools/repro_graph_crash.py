"""Does multi-stream HIP graph capture / replay crash without this library?

Round 2's GPU suite died with host-side SIGSEGVs inside torch.cuda.graph's
capture_end (hipStreamEndCapture + instantiate) and CUDAGraph.replay
(hipGraphLaunch) of the 4-stream pipelined step graphs.  This probe builds
graphs of the same SHAPE from torch ops only -- no librvhip call anywhere:
per stage, a fork of three side streams from the capture stream
(wait_stream), a chain of small kernels on each, a device->pinned-host copy
on one of them (the result hand-back), and the join back -- 8 stages per
graph, several graphs, then replays them in a loop.  A crash here puts the
fault in the runtime's graph path, not in the library's kernels or host
code.  Prints progress every 50 replays.

usage: python tools/repro_graph_crash.py [graphs] [replays] [mode]
  mode "multi" (default): the 4-stream fork/join stages
  mode "single": the same kernels captured on one stream (control)
"""
import faulthandler
import sys
import time

import torch

faulthandler.enable()
G = int(sys.argv[1]) if len(sys.argv) > 1 else 4
R = int(sys.argv[2]) if len(sys.argv) > 2 else 400
MODE = sys.argv[3] if len(sys.argv) > 3 else "multi"
dev = torch.device("cuda:0")
n = 1 << 20
bufs = [torch.rand(n, device=dev) for _ in range(8)]
host = [torch.empty(4096, dtype=torch.float32, pin_memory=True) for _ in range(G * 8)]
side = [torch.cuda.Stream(dev) for _ in range(3)]


def stage(j, g):
    cur = torch.cuda.current_stream()
    if MODE == "multi":
        for s in side:
            s.wait_stream(cur)
        for i, s in enumerate(side):
            with torch.cuda.stream(s):
                a = bufs[2 * i]
                for _ in range(6):
                    a.mul_(0.999).add_(bufs[2 * i + 1], alpha=1e-3)
                if i == 2:
                    host[g * 8 + j].copy_(a[:4096], non_blocking=True)
        bufs[6].add_(bufs[7], alpha=1e-3)
        for s in side:
            cur.wait_stream(s)
    else:
        for i in range(3):
            a = bufs[2 * i]
            for _ in range(6):
                a.mul_(0.999).add_(bufs[2 * i + 1], alpha=1e-3)
            if i == 2:
                host[g * 8 + j].copy_(a[:4096], non_blocking=True)
        bufs[6].add_(bufs[7], alpha=1e-3)


graphs = []
for g in range(G):
    for j in range(8):  # warm the allocator and kernels outside capture
        stage(j, g)
torch.cuda.synchronize()
t0 = time.time()
for g in range(G):
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for j in range(8):
            stage(j, g)
    graphs.append(gr)
print(f"captured {G} graphs ({MODE}) in {time.time() - t0:.2f} s", flush=True)
for r in range(R):
    for gr in graphs:
        gr.replay()
    if r % 50 == 0:
        torch.cuda.synchronize()
        print(f"replay round {r}", flush=True)
torch.cuda.synchronize()
print(f"done: {R} rounds x {G} graphs ({MODE}), no crash", flush=True)
