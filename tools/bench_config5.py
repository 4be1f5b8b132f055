"""BASELINE config 5 (configs[4]): "YOLOv8m 1280x1280 fp8 MFMA conv path,
batch=16, fog/rain-augmented frames (tools/fog_batch)".

A step = fog/rain synthesis on the device (rv_fog_full_u8 with
tools/fog_batch.py's settings, or the one-pass core rv_fog_rain_u8 with
--fog core; from clean frames resident in HBM) -> letterbox -> YOLOv8m forward at imgsz 1280 -> NMS, for a
batch of 16.  --dtype fp8 (default) runs the conv stack on
v_mfma_f32_16x16x32_fp8_fp8 with e4m3 weights / activations (scales
calibrated once on the first batch), bf16 the bf16 plan.

Prints ONE JSON line with bench.py's fields: value = frames/s of the whole
step; roofline = the conv family (every conv launch of a forward, HIP events
on the launch stream, rv_yolo_profile) against the dense MFMA peak of its
dtype (fp8: 5000 TFLOP/s; the non-scaled fp8 instruction itself issues at
the bf16 rate, 2500, reported as instruction_peak); cpu_baseline = the CPU
restatement of the same step (oracle fog_frame + torch-CPU fp32 YOLOv8m +
restated NMS) on a bounded sample.  Synthetic weights (no checkpoint here).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK = {"fp8": 5000.0, "bf16": 2500.0}  # dense MFMA TFLOP/s, MI355X_MICROARCH.md
GFLOP_PER_FRAME = 315.7  # YOLOv8m at 1280x1280: 2*M*N*K over all convs


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--dtype", default="fp8", choices=["fp8", "bf16"])
    p.add_argument("--batch", type=int, default=16)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--autotune", type=int, default=1)
    p.add_argument("--cpu-frames", type=int, default=1,
                   help="CPU baseline frames (the full fog oracle takes ~1 min per 1280x1280 frame); "
                        "0 skips it")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--fog", default="full", choices=["full", "core"],
                   help="full: the reference's whole synthesize with tools/fog_batch.py's "
                        "settings (rv_fog_full_u8); core: the one-pass scattering core")
    return p.parse_args()


def conv_profile(eng, lb, n=3):
    """Per-launch HIP-event timing of n eager forwards: conv ms per forward,
    algorithmic FLOPs and bytes per forward."""
    from rvs_amd import _lib
    lib = _lib.load()
    h = eng._h
    _lib.check(lib.rv_yolo_profile(h, n), "rv_yolo_profile")
    for _ in range(n):
        eng.forward_raw(lb)
    torch.cuda.synchronize()
    k = lib.rv_yolo_num_convs(eng.variant)
    ms, fl, cv, by = (np.zeros(k), np.zeros(k), np.zeros(k, np.int32), np.zeros(k))
    nf = lib.rv_yolo_profile_read(h, ms.ctypes.data, fl.ctypes.data, cv.ctypes.data, k)
    lib.rv_yolo_profile_bytes(h, by.ctypes.data, k)
    lib.rv_yolo_profile(h, 0)
    v = cv >= 0
    return float(ms[v].sum()) / max(nf, 1), float(fl[v].sum()), float(by[v].sum()), int(v.sum())


def cpu_baseline(clean_host, flat, frames, threads, fog="full"):
    """The CPU restatement of the same step on a bounded sample: the fog
    oracle (fog="full": fog_frame_full, every stage of the reference's
    synthesize, src/augment/fog.py:227-299, with tools/fog_batch.py:20-28's
    settings -- the GPU leg's work; "core": the scattering core only),
    letterbox, torch-CPU fp32 YOLOv8m, restated NMS."""
    from oracle import cpu, fog_ref, yolo_ref
    torch.set_num_threads(threads)
    model = yolo_ref.YoloRef(2, flat)
    rng = np.random.RandomState(5)
    H, W = clean_host.shape[1:3]
    t = np.zeros(3)
    t0 = time.perf_counter()
    for i in range(frames):
        a = time.perf_counter()
        if fog == "full":
            prm = fog_ref.draw_full(rng, H, W, level="medium", rain=True)
            img = fog_ref.fog_frame_full(clean_host[i % len(clean_host)], prm, y_h_ratio=0.42,
                                         softness_ratio=0.07, global_veil=0.5,
                                         depth_blur_max=4.0, rain_p=0.002)
        else:
            prm = fog_ref.draw(rng, H, W, level="medium", rain=True)
            img = fog_ref.fog_frame(clean_host[i % len(clean_host)], prm, rain_p=0.002)
        lb = cpu.letterbox(img, cpu.letterbox_geometry(H, W, 1280))[None]
        b = time.perf_counter()
        raw = model.forward(yolo_ref.preprocess(lb)).numpy()
        c = time.perf_counter()
        yolo_ref.postprocess(raw, (1280, 1280), (H, W), classes_keep=[0, 2, 3, 5, 7])
        d = time.perf_counter()
        t += [b - a, c - b, d - c]
    dt = time.perf_counter() - t0
    return {"value": round(frames / dt, 4), "unit": "frames/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "stage_s_per_frame": {
                k: round(v / frames, 3) for k, v in zip(["fog+letterbox", "yolov8m_fp32", "nms"], t)},
            "sample": f"{frames} frame(s) of 1280x1280: oracle "
                      + ("fog_frame_full (numpy f32, every stage of the reference's synthesize "
                         "with tools/fog_batch.py's settings)" if fog == "full" else
                         "fog_frame (numpy f32, the scattering core)")
                      + f" + torch-CPU fp32 YOLOv8m ({threads} threads) + restated NMS; "
                      f"{dt:.1f} s"}


def main():
    args = parse()
    from conftest import road_frame
    from rvs_amd.augment import FogSynthesizer
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    B, H, W = args.batch, 1280, 1280
    dev = torch.device("cuda:0")
    clean_host = np.stack([road_frame(H, W, seed=70 + b) for b in range(4)])
    clean = torch.from_numpy(clean_host).to(dev).repeat((B + 3) // 4, 1, 1, 1)[:B].contiguous()
    if args.fog == "full":  # tools/fog_batch.py:20-28
        syn = FogSynthesizer(level="medium", seed=5, rain_p=0.002, device=dev, y_h_ratio=0.42,
                             perlin_scale_ratio=0.18, perlin_octaves=2, horizon_softness=0.07,
                             global_veil=0.5, depth_blur_max=4.0)
    else:
        syn = FogSynthesizer(level="medium", seed=5, rain_p=0.002, device=dev, filters=False)
    prep = syn.prepare([syn.draw(H, W) for _ in range(B)])
    fog = syn.synthesize_batch(clean, prepared=prep)
    flat = weights.synthetic_weights(2, seed=0)
    eng = YoloEngine(2, flat, B, (H, W), imgsz=1280, device=dev, dtype=args.dtype,
                     classes_keep=[0, 2, 3, 5, 7])
    lb = eng.letterbox(fog)
    if args.dtype == "fp8":
        eng.calibrate(lb)
    if args.autotune:
        eng.autotune(lb, reps=2)

    def step():
        syn.synthesize_batch(clean, out=fog, prepared=prep)
        eng.run(fog)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ms_step = (time.perf_counter() - t0) / args.steps * 1e3
    # stage split (events on the current stream)
    def t_of(fn, n=5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / n
    ms_fog = t_of(lambda: syn.synthesize_batch(clean, out=fog, prepared=prep))
    ms_fwd = t_of(lambda: eng.forward_raw(lb))
    ms_nms = t_of(lambda: eng.nms(B))
    conv_ms, flop, byts, nl = conv_profile(eng, lb)
    tf = flop / (conv_ms * 1e-3) / 1e12
    peak = PEAK[args.dtype]
    out = {
        "metric": "config 5 frames/s (fog/rain -> YOLOv8m 1280 -> NMS)", "value":
            round(B / ms_step * 1e3, 1), "unit": "frames/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
        "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (road frames + device fog/rain; "
        "synthetic YOLOv8m weights)",
        "config": {"workload": f"configs[4]: YOLOv8m 1280x1280 {args.dtype} conv path, batch {B}, "
                               "fog/rain frames", "batch": B, "imgsz": 1280, "fog": args.fog,
                   "autotune": bool(args.autotune)},
        "stage_ms": {"fog": round(ms_fog, 4), "forward": round(ms_fwd, 4), "nms": round(ms_nms, 4)},
        "roofline": {
            "kernel": "conv family (every conv launch of one YOLOv8m forward; HIP events on the "
                      "launch stream)", "bound": "mfma", "achieved": round(tf, 1), "peak": peak,
            "unit": "TFLOP/s", "frac": round(tf / peak, 4), "traffic": None,
            "instruction_peak": 2500.0 if args.dtype == "fp8" else peak,
            "instruction_frac": round(tf / 2500.0, 4),
            "conv_ms_per_forward": round(conv_ms, 4), "launches": nl,
            "algorithmic_gflop_per_forward": round(flop / 1e9, 1),
            "algorithmic_gb_per_forward": round(byts / 1e9, 3)},
        "forward_tflops": round(GFLOP_PER_FRAME * B / ms_fwd, 1),
        "dets_per_frame": round(eng.det_n[:B].float().mean().item(), 2),
    }
    if args.cpu_frames > 0:
        thr = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", 0)) or min(16, os.cpu_count())
        out["cpu_baseline"] = cpu_baseline(clean_host, flat, args.cpu_frames, thr, args.fog)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
