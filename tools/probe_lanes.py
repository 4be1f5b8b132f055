"""Probe the multi-lane OverlappedSteps schedule: eager (capture=0) or
captured (capture=1); compares every step's results with sequential steps.
usage: python tools/probe_lanes.py CAPTURE LANES CHUNK"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch  # noqa: E402


def main():
    import bench
    from rvs_amd.engine import OverlappedSteps, RoadVisionEngine
    from rvs_amd.synth import road_frames
    cap, L, chunk = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    dev = torch.device("cuda:0")
    S, F = 4, 6
    cfg = bench.bench_config()
    fr = road_frames(S, F, 1080, 1920, device=dev)
    ts = torch.tensor([[f / 30.0] * S for f in range(F)], dtype=torch.float64, device=dev)
    seq = RoadVisionEngine(cfg, S, (1080, 1920), device=dev)
    want = []
    for f in range(F):
        want.append(seq.results(seq.step(fr[f], ts[f])))
    eng = RoadVisionEngine(cfg, S, (1080, 1920), device=dev, lanes=L)
    eng.step(fr[0], ts[0])
    torch.cuda.synchronize()
    print("building", flush=True)
    run = OverlappedSteps(eng, [fr[f] for f in range(1, F)], [ts[f] for f in range(1, F)],
                          depth=3, chunk=chunk, capture=bool(cap))
    torch.cuda.synchronize()
    print("built", len(run.graphs), "graphs", flush=True)
    run.run()
    torch.cuda.synchronize()
    key = lambda r: [[(d.x1, d.y1, d.track_id) for d in s] for s in r]  # noqa
    ok = all(key(want[k + 1]) == key(eng.results(o)) for k, o in enumerate(run.outs))
    print("match", ok, flush=True)


if __name__ == "__main__":
    main()
