"""Isolated timing of rv_sort_update (no concurrent stages): S streams of
synthetic drifting detections (oracle/sort_ref.synthetic_detections) run
for W warm-up frames (the live track count grows to its steady state), then
K frames are timed with HIP events.  usage: python tools/time_sort.py [S] [NOBJ]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from oracle import sort_ref
    from rvs_amd.track.sort_hip import MultiStreamSort
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    nobj = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    dev = torch.device("cuda:0")
    W, K, dmax = 60, 30, 100
    cfg = {"max_staleness": 1.2, "min_hits": 3, "iou_threshold": 0.35, "speed_window": 0.8}
    st = [sort_ref.synthetic_detections(W + K, seed=s, n_obj=nobj, p_clutter=8.0) for s in range(S)]
    dets = np.zeros((W + K, S, dmax, 6), np.float32)
    cnt = np.zeros((W + K, S), np.int32)
    ts = np.zeros((W + K, S), np.float64)
    for s in range(S):
        for f in range(W + K):
            r = st[s][0][f][:dmax]
            dets[f, s, :len(r)] = r
            cnt[f, s] = len(r)
            ts[f, s] = st[s][1][f]
    dets, cnt, ts = (torch.from_numpy(x).to(dev) for x in (dets, cnt, ts))
    ms = MultiStreamSort(cfg, S, tmax=1024, dmax=dmax, device=dev)
    for f in range(W):
        ms.update(dets[f], cnt[f], ts[f])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for f in range(W, W + K):
        ms.update(dets[f], cnt[f], ts[f])
    e1.record()
    torch.cuda.synchronize()
    stt = ms.stats()
    print(f"S={S} dets/frame {float(cnt.float().mean()):.1f} tracks mean {stt['T'].mean():.1f} "
          f"max {stt['T'].max()}: rv_sort_update {e0.elapsed_time(e1) / K * 1e3:.1f} us/frame",
          flush=True)


if __name__ == "__main__":
    main()
