"""BASELINE config 2 (configs[1]): "YOLOv8n 640x640 batch=1 bf16 on one
MI355X (Conv/C2f/SPPF MFMA kernels, fused SiLU)" -- per-frame LATENCY.

The reference detects one frame per call (main_preview.py:99 ->
YOLOUltralytics.infer, src/detect/yolo_ultralytics.py:26-53), so batch 1 is
its native shape.  Measured here, all at 640x640 (the letterbox is a no-op
copy at that size) on u8 frames resident in HBM:

  forward_eager   letterbox + YOLOv8n forward + fused decode, launched from
                  the host each call (~40 launches)
  detect_eager    the same + NMS / scale_boxes / class filter
  detect_native   letterbox + forward + NMS recorded once as a native launch
                  list (rvs_amd.schedule.Schedule) and issued with one C call
                  per frame (the serving form; no HIP graph capture, which
                  crashed intermittently in r02: DESIGN.md §3)
  chain_native    the whole per-frame chain (CLAHE + median + letterbox +
                  forward + NMS + SORT + result hand-back to pinned host) as
                  one recorded step of RoadVisionEngine(S=1)
  infer_host      YOLOHip.infer(np.ndarray) exactly as the reference calls
                  it: H2D of the frame, the device path, D2H and Detection
                  construction

Each is timed per call (host clock, synchronised after every call: a
latency, not a throughput) over --iters calls after --warmup; the JSON line
reports median / p90 / p99 in ms.  `roofline` prices the launch-list
forward against the dense bf16 MFMA peak (8.742 GFLOP per 640^2 frame,
SURVEY 8(d)); at batch 1 the forward is ~40 dependent launches of a few
microseconds each, so the fraction is a latency statement.  cpu_baseline =
the torch-CPU fp32 restatement of the same forward + restated NMS, one frame
per call.  Synthetic weights (no checkpoint here)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

GFLOP = 8.742  # YOLOv8n at 640x640
PEAK_BF16 = 2500.0


def stats(ts):
    a = np.sort(np.asarray(ts) * 1e3)
    return {"median_ms": round(float(np.median(a)), 4), "p90_ms": round(float(np.percentile(a, 90)), 4),
            "p99_ms": round(float(np.percentile(a, 99)), 4), "min_ms": round(float(a[0]), 4),
            "calls": len(a)}


def timed(fn, iters, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append(time.perf_counter() - t0)
    return out


def device_ms(fn, n=50):
    """Back-to-back device time per call (events on the current stream)."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def cpu_baseline(frame, flat, frames, threads):
    from oracle import yolo_ref
    torch.set_num_threads(threads)
    model = yolo_ref.YoloRef(0, flat)
    x = yolo_ref.preprocess(frame[None])
    model.forward(x)
    ts = []
    for _ in range(frames):
        t0 = time.perf_counter()
        raw = model.forward(yolo_ref.preprocess(frame[None])).numpy()
        yolo_ref.postprocess(raw, (640, 640), (640, 640), classes_keep=[0, 2, 3, 5, 7])
        ts.append(time.perf_counter() - t0)
    return {"value": round(1e3 * float(np.median(ts)), 3), "unit": "ms/frame (median)",
            "cores": threads, "kind": "port", "host_cpus": os.cpu_count(),
            "sample": f"{frames} calls of torch-CPU fp32 YOLOv8n 640x640 b=1 + restated NMS "
                      f"({threads} threads)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--autotune", type=int, default=1)
    ap.add_argument("--cpu-frames", type=int, default=20, help="0 skips the CPU baseline")
    args = ap.parse_args()
    from conftest import road_frame
    from rvs_amd.config import load_config
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YOLOHip, YoloEngine
    from rvs_amd.engine import RoadVisionEngine

    dev = torch.device("cuda:0")
    H = W = 640
    host = road_frame(H, W, seed=0)
    frame = torch.from_numpy(host).to(dev)[None].contiguous()
    flat = weights.synthetic_weights(0, seed=0)
    keep = [0, 2, 3, 5, 7]
    eng = YoloEngine(0, flat, 1, (H, W), imgsz=640, device=dev, classes_keep=keep)
    lb = eng.letterbox(frame)
    if args.autotune:
        eng.autotune(lb, reps=10)
    tuned = eng.tuned_configs()
    res = {}
    res["forward_eager"] = stats(timed(lambda: eng.forward_raw(eng.letterbox(frame)), args.iters,
                                       args.warmup))
    res["detect_eager"] = stats(timed(lambda: eng.run(frame), args.iters, args.warmup))

    from rvs_amd.schedule import Schedule
    g = Schedule()
    with g.recording():
        eng.run(frame)
    res["detect_native"] = stats(timed(g.run, args.iters, args.warmup))
    gf = Schedule()
    with gf.recording():
        eng.forward_raw(eng.letterbox(frame))
    res["forward_native"] = stats(timed(gf.run, args.iters, args.warmup))
    fwd_dev_ms = device_ms(gf.run)
    det_dev_ms = device_ms(g.run)

    # the whole per-frame chain, one stream, one recorded step
    cfg = load_config()
    cfg["detect"]["weights"] = "synthetic"
    rve = RoadVisionEngine(cfg, 1, (H, W), device=dev, weights=flat)
    rve.detector.load_tuned(tuned)
    ts = torch.zeros(1, dtype=torch.float64, device=dev)
    for _ in range(3):
        rve.step(frame, ts)
    torch.cuda.synchronize()
    gc = Schedule()
    with gc.recording():
        out = rve.step(frame, ts)
    k = [0]

    def chain():
        ts.fill_(k[0] / 30.0)
        k[0] += 1
        gc.run()
    res["chain_native"] = stats(timed(chain, args.iters, args.warmup))
    torch.cuda.synchronize()
    out["seq"] = out["record"].seq
    n_chain = len(rve.results(out)[0])

    det = YOLOHip({"model": "yolov8n.pt", "weights": "synthetic", "classes_keep": keep})
    det.flat = flat
    e1 = det.engine(H, W, 1)
    e1.load_tuned(tuned)
    res["infer_host"] = stats(timed(lambda: det.infer(host), args.iters // 2, args.warmup))
    n_det = len(det.infer(host))

    lat = res["detect_native"]["median_ms"]
    tf = GFLOP / (fwd_dev_ms * 1e-3) / 1e3
    line = {
        "metric": "YOLOv8n 640x640 batch=1 detect latency (letterbox+forward+NMS, native launch list)",
        "value": lat, "unit": "ms", "n_gpus": 1, "steps": args.iters, "warmup": args.warmup,
        "higher_is_better": False, "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (one 640x640 road frame, synthetic YOLOv8n weights)",
        "config": {"workload": "configs[1]: YOLOv8n 640x640 batch=1 bf16", "batch": 1,
                   "imgsz": 640, "autotune": bool(args.autotune)},
        "latency": res,
        "device_ms_back_to_back": {"forward_native": round(fwd_dev_ms, 4),
                                   "detect_native": round(det_dev_ms, 4)},
        "roofline": {"kernel": "YOLOv8n forward, launch list back to back (one frame)",
                     "bound": "mfma", "achieved": round(tf, 2), "peak": PEAK_BF16,
                     "unit": "TFLOP/s", "frac": round(tf / PEAK_BF16, 5), "traffic": None},
        "detections": {"infer_host": n_det, "chain": n_chain},
    }
    if args.cpu_frames > 0:
        thr = int(os.environ.get("OMP_NUM_THREADS", 0)) or min(16, os.cpu_count())
        line["cpu_baseline"] = cpu_baseline(host, flat, args.cpu_frames, thr)
    print(json.dumps(line))
    rve.close()
    det.close()
    eng.close()


if __name__ == "__main__":
    main()
