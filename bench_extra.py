"""Secondary legs of bench.py's line (rank 0, one GPU): the other BASELINE
configurations and the host-fed rate, each a few seconds of device work.

  config2_latency   configs[1]: YOLOv8n 640x640 batch 1 -- the reference's
                    per-call shape (main_preview.py:99 -> YOLOUltralytics.infer,
                    src/detect/yolo_ultralytics.py:26-53): letterbox + forward +
                    NMS recorded once as a native launch list, one C call per
                    frame, host clock around each call with a sync after it
  config5_fp8       configs[4]: fog/rain synthesis (tools/fog_batch.py:7-34's
                    settings, every stage of src/augment/fog.py:227-299) ->
                    letterbox -> YOLOv8m at imgsz 1280 on the fp8 MFMA -> NMS,
                    batch 16; conv-family roofline against the fp8 peaks
  hostfed_nv12      configs[2] fed from pinned host memory (BASELINE.md §4
                    item 5): NV12 frames (what a decoder hands over) copied
                    H2D and converted on the device on a copy stream, one
                    window of K steps ahead of the recorded K-step pipeline
                    that consumes the previous window

None of these is the headline `value`; synthetic frames and weights (no
checkpoint or dataset exists here)."""
from __future__ import annotations

import time

import numpy as np
import torch

PEAK_BF16 = 2500.0   # dense TFLOP/s (MI355X_MICROARCH.md)
PEAK_FP8 = 5000.0    # dense, block-scaled f8f6f4 MFMA
GFLOP_V8N_640 = 8.742      # YOLOv8n at 640x640
GFLOP_V8M_1280 = 315.7     # YOLOv8m at 1280x1280


def _stats_ms(ts):
    a = np.sort(np.asarray(ts) * 1e3)
    return {"median_ms": round(float(np.median(a)), 4), "p90_ms": round(float(np.percentile(a, 90)), 4),
            "p99_ms": round(float(np.percentile(a, 99)), 4), "calls": len(a)}


def _per_call(fn, iters, warmup):
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


def _device_ms(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def _conv_profile(eng, fwd, n=2):
    """Conv-family device time per forward (HIP events on the launch stream
    around every conv launch, rv_yolo_profile) and its algorithmic FLOPs."""
    from rvs_amd import _lib
    lib = _lib.load()
    h = eng._h
    _lib.check(lib.rv_yolo_profile(h, n), "rv_yolo_profile")
    for _ in range(n):
        fwd()
    torch.cuda.synchronize()
    k = lib.rv_yolo_num_convs(eng.variant)
    ms, fl, cv = np.zeros(k), np.zeros(k), np.zeros(k, np.int32)
    nf = lib.rv_yolo_profile_read(h, ms.ctypes.data, fl.ctypes.data, cv.ctypes.data, k)
    lib.rv_yolo_profile(h, 0)
    v = cv >= 0
    return float(ms[v].sum()) / max(nf, 1), float(fl[v].sum())


def config2_latency(dev, iters=200, warmup=20) -> dict:
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    from rvs_amd.schedule import Schedule
    from rvs_amd.synth import road_frames
    frame = road_frames(1, 1, 640, 640, device=dev)[0].contiguous()
    eng = YoloEngine(0, weights.synthetic_weights(0, seed=0), 1, (640, 640), imgsz=640, device=dev,
                     classes_keep=[0, 2, 3, 5, 7])
    eng.autotune(eng.letterbox(frame), reps=5)
    det = Schedule()
    with det.recording():
        eng.run(frame)
    fwd = Schedule()
    with fwd.recording():
        eng.forward_raw(eng.letterbox(frame))
    lat = _stats_ms(_per_call(det.run, iters, warmup))
    fwd_ms = _device_ms(fwd.run, 50)
    conv_ms, flop = _conv_profile(eng, lambda: eng.forward_raw(eng.letterbox(frame)))
    tf = GFLOP_V8N_640 / (fwd_ms * 1e-3) / 1e3
    n_det = int(eng.det_n[0].item())
    det.close()
    fwd.close()
    eng.close()
    return {"workload": "configs[1]: YOLOv8n 640x640 batch=1 bf16, letterbox + forward + NMS per "
                        "call (native launch list), host clock around each call with a sync",
            "value": lat["median_ms"], "unit": "ms (median per-frame latency)",
            "higher_is_better": False, **lat,
            "forward_device_ms_back_to_back": round(fwd_ms, 4),
            "roofline": {"kernel": "YOLOv8n forward at batch 1 (launch list back to back)",
                         "bound": "mfma", "achieved": round(tf, 2), "peak": PEAK_BF16,
                         "unit": "TFLOP/s", "frac": round(tf / PEAK_BF16, 5),
                         "conv_ms_per_forward": round(conv_ms, 4),
                         "algorithmic_gflop_per_forward": round(flop / 1e9, 3)},
            "detections": n_det}


def config5_fp8(dev, steps=5, warmup=2, B=16) -> dict:
    from rvs_amd.augment import FogSynthesizer
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    from rvs_amd.synth import road_frames
    H = W = 1280
    base = road_frames(4, 1, H, W, device=dev)[0]
    clean = base.repeat((B + 3) // 4, 1, 1, 1)[:B].contiguous()
    # tools/fog_batch.py:20-28's settings
    syn = FogSynthesizer(level="medium", seed=5, rain_p=0.002, device=dev, y_h_ratio=0.42,
                         perlin_scale_ratio=0.18, perlin_octaves=2, horizon_softness=0.07,
                         global_veil=0.5, depth_blur_max=4.0)
    prep = syn.prepare([syn.draw(H, W) for _ in range(B)])
    fog = syn.synthesize_batch(clean, prepared=prep)
    eng = YoloEngine(2, weights.synthetic_weights(2, seed=0), B, (H, W), imgsz=1280, device=dev,
                     dtype="fp8", classes_keep=[0, 2, 3, 5, 7])
    lb = eng.letterbox(fog)
    eng.calibrate(lb)
    eng.autotune(lb, reps=2)

    def step():
        syn.synthesize_batch(clean, out=fog, prepared=prep)
        eng.run(fog)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ms_step = (time.perf_counter() - t0) / steps * 1e3
    fwd_ms = _device_ms(lambda: eng.forward_raw(lb), 3)
    conv_ms, flop = _conv_profile(eng, lambda: eng.forward_raw(lb))
    tf = flop / (conv_ms * 1e-3) / 1e12
    dets = round(eng.det_n[:B].float().mean().item(), 2)
    eng.close()
    return {"workload": "configs[4]: fog/rain synthesis (every stage, tools/fog_batch.py settings) -> "
                        "letterbox -> YOLOv8m 1280x1280 fp8 (e4m3) MFMA conv path -> NMS, batch 16",
            "value": round(B / ms_step * 1e3, 1), "unit": "frames/s", "ms_per_step": round(ms_step, 3),
            "steps": steps, "dtype": "fp8",
            "forward_ms": round(fwd_ms, 3),
            "forward_tflops": round(GFLOP_V8M_1280 * B / fwd_ms, 1),
            "roofline": {"kernel": "conv family of one YOLOv8m forward (HIP events on the launch "
                                   "stream)", "bound": "mfma", "achieved": round(tf, 1),
                         "peak": PEAK_FP8, "unit": "TFLOP/s", "frac": round(tf / PEAK_FP8, 4),
                         "instruction_peak": PEAK_BF16,
                         "instruction_frac": round(tf / PEAK_BF16, 4),
                         "peak_note": "5 PF = the block-scaled f8f6f4 MFMA; the non-scaled "
                                      "16x16x32 fp8 instruction issues at the bf16 rate, 2.5 PF",
                         "conv_ms_per_forward": round(conv_ms, 4),
                         "algorithmic_gflop_per_forward": round(flop / 1e9, 1)},
            "dets_per_frame": dets}


def hostfed_nv12(job, windows=3) -> dict:
    """The bench's K-step pipeline fed from pinned host NV12 frames: window
    w's K x S frames are copied H2D and converted (rv_nv12_to_bgr_u8) on a
    copy stream while the recorded pipeline runs window w - 1; two device
    frame windows alternate.  A pinned ring of 2 steps of NV12 stands in
    for the decoder's output buffers."""
    from rvs_amd import kernels
    from rvs_amd.schedule import PipelinedRun
    eng, S, K, dev = job.eng, job.S, job.K, job.dev
    H, W = eng.H, eng.W
    ring = [torch.randint(0, 256, (S, H * 3 // 2, W), dtype=torch.uint8).pin_memory()
            for _ in range(2)]
    nv = [torch.empty((S, H * 3 // 2, W), dtype=torch.uint8, device=dev) for _ in range(2)]
    bgr = [[torch.empty((S, H, W, 3), dtype=torch.uint8, device=dev) for _ in range(K)]
           for _ in range(2)]
    ts = [job.ts[job.Wm + k] for k in range(K)]
    runs = [PipelinedRun(eng, bgr[b], ts, mode="native", sync=job.args.sync, units=job.unit_sizes)
            for b in range(2)]
    copy = torch.cuda.Stream(dev)
    main = torch.cuda.current_stream()
    saved = eng.tracker.state[0].clone()

    def upload(b, after=None):
        with torch.cuda.stream(copy):
            if after is not None:
                copy.wait_event(after)
            for k in range(K):
                nv[k % 2].copy_(ring[k % 2], non_blocking=True)
                kernels.nv12_to_bgr(nv[k % 2], out=bgr[b][k])
            ev = torch.cuda.Event()
            ev.record(copy)
        return ev

    # H2D alone (the PCIe ceiling of this leg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(copy):
        for k in range(K):
            nv[k % 2].copy_(ring[k % 2], non_blocking=True)
    torch.cuda.synchronize()
    h2d_s = (time.perf_counter() - t0) / K
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    up = upload(0)
    done = [None, None]
    for w in range(windows):
        b = w % 2
        nxt = None
        if w + 1 < windows:  # next window's frames, after the run that last read them
            nxt = upload(1 - b, done[1 - b])
        main.wait_event(up)
        runs[b].run()
        ev = torch.cuda.Event()
        ev.record(main)
        done[b] = ev
        up = nxt
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    eng.tracker.state[0].copy_(saved)
    for r in runs:
        r.close()
    torch.cuda.synchronize()
    frame_b = H * W * 3 // 2
    return {"workload": f"configs[2] fed from pinned host NV12: {windows} windows of {K} steps x {S} "
                        "streams, H2D + NV12->BGR on a copy stream one window ahead of the "
                        "recorded pipeline",
            "value": round(windows * K * S / el, 1), "unit": "frames/s",
            "h2d_only_frames_per_s": round(S / h2d_s, 1),
            "h2d_gbs": round(S * frame_b / h2d_s / 1e9, 1),
            "bytes_per_frame_h2d": frame_b}
