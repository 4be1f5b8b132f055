"""Phase split of the fused SORT kernel (a -DRV_SORT_PHASE build:
RV_LIB_VARIANT=sph, tools/build_defs_variant.sh): time_sort.py's synthetic
streams, then the summed per-phase wall-clock ticks of every block of the
timed frames.  usage: RV_LIB_VARIANT=sph python tools/sort_phase.py [S] [NOBJ] [CLUTTER]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

PHASES = ["predict+load", "iou pairs", "sort", "greedy", "bookkeeping", "kf update+metrics"]


def main():
    from oracle import sort_ref
    from rvs_amd import _lib
    from rvs_amd.track.sort_hip import MultiStreamSort
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    nobj = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    clutter = float(sys.argv[3]) if len(sys.argv) > 3 else 8.0
    dev = torch.device("cuda:0")
    W, K, dmax = 60, 30, 300
    cfg = {"max_staleness": 1.2, "min_hits": 3, "iou_threshold": 0.35, "speed_window": 0.8}
    st = [sort_ref.synthetic_detections(W + K, seed=s, n_obj=nobj, p_clutter=clutter) for s in range(S)]
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
    lib = _lib.load()
    rd = lib.rv_sort_phase_read
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 8)()
    for f in range(W):
        ms.update(dets[f], cnt[f], ts[f])
    torch.cuda.synchronize()
    rd(buf, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for f in range(W, W + K):
        ms.update(dets[f], cnt[f], ts[f])
    e1.record()
    torch.cuda.synchronize()
    rd(buf, 0)
    stt = ms.stats()
    per = [buf[i] / (K * S) / 100.0 for i in range(6)]  # us per block per frame (100 MHz ticks)
    print(f"S={S} dets/frame {float(cnt.float().mean()):.1f} tracks mean {stt['T'].mean():.1f} "
          f"max {stt['T'].max()}: {e0.elapsed_time(e1) / K * 1e3:.1f} us/frame; per block: " +
          ", ".join(f"{n} {v:.1f}" for n, v in zip(PHASES, per)) + f" (sum {sum(per):.1f} us)",
          flush=True)


if __name__ == "__main__":
    main()
