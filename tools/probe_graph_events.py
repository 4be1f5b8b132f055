"""Probe: do HIP events recorded inside captured graphs time correctly on
this ROCm?  Captures S=4 OverlappedSteps with per-conv-launch events, replays,
reads the event timings, and compares with an eager profiled pass."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def read(lib, h, n):
    ms = np.zeros(n)
    fl = np.zeros(n)
    cv = np.zeros(n, np.int32)
    nf = lib.rv_yolo_profile_read(h, ms.ctypes.data, fl.ctypes.data, cv.ctypes.data, n)
    return nf, ms, cv


def main():
    import bench
    from rvs_amd import _lib
    from rvs_amd.engine import OverlappedSteps, RoadVisionEngine
    from rvs_amd.synth import road_frames
    dev = torch.device("cuda:0")
    S, K = 8, 4
    eng = RoadVisionEngine(bench.bench_config(), S, (1080, 1920), device=dev)
    fr = road_frames(S, K + 1, 1080, 1920, device=dev)
    ts = torch.tensor([[f / 30.0] * S for f in range(K + 1)], dtype=torch.float64, device=dev)
    eng.step(fr[0], ts[0])
    torch.cuda.synchronize()
    lib = _lib.load()
    h = eng.detector._h
    n = lib.rv_yolo_num_convs(0)
    lib.rv_yolo_profile(h, K)
    for k in range(K):
        eng.step(fr[k + 1], ts[k + 1])
    torch.cuda.synchronize()
    nf, ms, cv = read(lib, h, n)
    print("eager: forwards", nf, "conv ms/step", ms[cv >= 0].sum() / max(nf, 1), flush=True)
    lib.rv_yolo_profile(h, 0)
    lib.rv_yolo_profile(h, K)
    run = OverlappedSteps(eng, [fr[k + 1] for k in range(K)], [ts[k + 1] for k in range(K)],
                          depth=3, chunk=8)
    torch.cuda.synchronize()
    print("captured", flush=True)
    run.run()
    torch.cuda.synchronize()
    print("replayed", flush=True)
    nf, ms, cv = read(lib, h, n)
    print("graph: forwards", nf, "conv ms/step", ms[cv >= 0].sum() / max(nf, 1), flush=True)
    print("per-launch us (first 10):", np.round(ms[:10] / max(nf, 1) * 1e3, 1), flush=True)
    del run
    torch.cuda.synchronize()
    lib.rv_yolo_profile(h, 0)
    x = fr[0, 0].cpu()
    print("ok after teardown", int(x.sum()), flush=True)


if __name__ == "__main__":
    main()
