"""End-to-end benchmark of the MI355X road-vision hot path.

Metric (BASELINE.json): end-to-end frames/sec @1080p (preproc + YOLOv8n +
SORT).  Workload at N=1: configs[2] -- "Full chain 1920x1080 batch=32 on one
MI355X: CLAHE+Median+YOLOv8n+NMS+SORT IoU".  A step = one pass of the hot path
over one stream-major batch (32 camera streams x 1 frame): fused CLAHE+median
(proc frames written to HBM), letterbox, YOLOv8n forward (bf16 MFMA), NMS +
scale_boxes + class filter, SORT (KF + IoU + greedy association) with
ground-plane homography metrics.  Inputs are synthetic road frames generated
on the device before the timed region (resident in HBM).

Multi-GPU (torchrun, one process per GPU): camera streams are sharded
(stream s -> rank s // 32), no collective on the data path (weak scaling);
rank timings are reduced with a MAX for the reported time.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

H, W = 1080, 1920
FLOP_PER_FRAME = 2 * 2.623e9           # YOLOv8n @ 384x640
BYTES_PER_FRAME = 15.39e6              # SURVEY 8(d) algorithmic HBM bytes / 1080p frame
PEAK_BF16 = 2500.0                     # TFLOP/s dense (MI355X_MICROARCH.md)
PEAK_HBM = 8000.0                      # GB/s
IMAGE_POINTS = [[560, 1000], [1360, 1000], [1160, 620], [760, 620]]
WORLD_POINTS = [[-3.5, 5.0], [3.5, 5.0], [3.5, 30.0], [-3.5, 30.0]]


def bench_config():
    from rvs_amd.config import load_config
    cfg = load_config()
    cfg["geometry"]["enabled"] = True
    cfg["geometry"]["projector"]["image_points"] = IMAGE_POINTS
    cfg["geometry"]["projector"]["world_points"] = WORLD_POINTS
    return cfg


def cpu_baseline(frames_host: np.ndarray, ts: np.ndarray, cfg: dict, threads: int):
    """The CPU oracle port of the reference path timed on this host: C restatement
    of CLAHE/median/letterbox (1 thread), torch-CPU fp32 YOLOv8n (batch 1, `threads`
    intra-op threads), restated NMS, reference-semantics Python SORT + homography."""
    from oracle import cpu, sort_ref, yolo_ref
    from rvs_amd.detect.weights import synthetic_weights
    from rvs_amd.geometry import find_homography
    torch.set_num_threads(threads)
    model = yolo_ref.YoloRef(0, synthetic_weights(0, 0))
    proj = sort_ref.HomographyProjector(find_homography(np.array(IMAGE_POINTS, np.float32),
                                                        np.array(WORLD_POINTS, np.float32)),
                                        (0.0, 0.0), 1000.0)
    trk = sort_ref.SortTracker(cfg["tracking"])
    geo = cpu.letterbox_geometry(H, W)
    keep = cfg["detect"]["classes_keep"]
    t0 = time.perf_counter()
    n = 0
    for img, t in zip(frames_host, ts):
        proc = cpu.median(cpu.clahe_ycrcb(img, 8, 2.0), 3)
        lb = cpu.letterbox(proc, geo)[None]
        raw = model.forward(yolo_ref.preprocess(lb)).numpy()
        dets = yolo_ref.postprocess(raw, geo[:2], (H, W), classes_keep=keep)[0]
        trk.update([sort_ref.Det(*map(float, r[:5]), int(r[5])) for r in dets], float(t), proj)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} consecutive 1080p frames of one stream, full chain (C oracle "
                      f"CLAHE+median+letterbox 1 thread, torch-CPU fp32 YOLOv8n "
                      f"{threads} threads, restated NMS, Python SORT+homography); "
                      f"{dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)  # pipeline fill/drain < 1 %
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--streams", type=int, default=32, help="camera streams per GPU")
    ap.add_argument("--cpu-frames", type=int, default=int(os.environ.get("RV_CPU_FRAMES", 6)))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="launch kernels eagerly (no HIP graph)")
    ap.add_argument("--no-autotune", action="store_true",
                    help="skip the per-layer conv kernel autotuning before the timed region")
    ap.add_argument("--depth", type=int, default=int(os.environ.get("RV_PIPE_DEPTH", 3)),
                    help="pipelined steps: 3 = Y(k) || P(k+1) || T(k-1), 2 = [T(k-1) || P(k)] -> Y(k)")
    ap.add_argument("--graph-chunk", type=int, default=None,
                    help="pipeline steps per captured graph (default 8, RV_GRAPH_CHUNK; 0 = all)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one graph per step; no overlap of step k's NMS+SORT with step k+1")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from rvs_amd import _lib
    from rvs_amd.engine import OverlappedSteps, RoadVisionEngine
    from rvs_amd.shard import job_throughput, max_over_ranks, rank_streams
    from rvs_amd.synth import road_frames

    cfg = bench_config()
    S, K, Wm = args.streams, args.steps, args.warmup
    eng = RoadVisionEngine(cfg, S, (H, W), device=dev)
    frames = road_frames(S, Wm + K, H, W, device=dev,
                         stream_offset=rank_streams(S, rank).start)
    ts_all = torch.tensor([[f / 30.0] * S for f in range(Wm + K)], dtype=torch.float64,
                          device=dev)
    torch.cuda.synchronize()

    for f in range(Wm):
        eng.step(frames[f], ts_all[f])
    if not args.no_autotune:  # per-layer conv kernel choice, on real activations
        eng.autotune(frames[0], reps=int(os.environ.get("RV_AUTOTUNE_REPS", "10")))
    torch.cuda.synchronize()
    lib = _lib.load()
    graphs = runner = None
    if not args.eager and not args.no_pipeline:
        # the track stage of step k (NMS + SORT, latency-bound) overlaps the
        # preprocess of step k+1 inside one graph (engine.OverlappedSteps)
        runner = OverlappedSteps(eng, [frames[Wm + k] for k in range(K)],
                                 [ts_all[Wm + k] for k in range(K)], depth=args.depth,
                                 chunk=args.graph_chunk)
        torch.cuda.synchronize()
    elif not args.eager:
        # one HIP graph per timed step (its own frame batch); replayed in order
        graphs = [eng.capture(frames[Wm + k], ts_all[Wm + k])[0] for k in range(K)]
        torch.cuda.synchronize()
    else:
        _lib.check(lib.rv_yolo_profile(eng.detector._h, K), "rv_yolo_profile")
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if runner is not None:
        runner.run()
    else:
        for k in range(K):
            if graphs is not None:
                graphs[k].replay()
            else:
                eng.step(frames[Wm + k], ts_all[Wm + k])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        torch.distributed.barrier()
    elapsed = max_over_ranks(elapsed, dev)

    # live conv timing (HIP events on the launch stream): a separate eager
    # pass over the same K steps (event records cannot live inside graphs)
    if graphs is not None or runner is not None:
        _lib.check(lib.rv_yolo_profile(eng.detector._h, K), "rv_yolo_profile")
        for k in range(K):
            eng.step(frames[Wm + k], ts_all[Wm + k])
        torch.cuda.synchronize()
    n = lib.rv_yolo_num_convs(eng.variant)
    ms = np.zeros(n, np.float64)
    fl = np.zeros(n, np.float64)
    cv = np.zeros(n, np.int32)
    nf = lib.rv_yolo_profile_read(eng.detector._h, ms.ctypes.data, fl.ctypes.data, cv.ctypes.data, n)
    by = np.zeros(n, np.float64)
    lib.rv_yolo_profile_bytes(eng.detector._h, by.ctypes.data, n)
    lib.rv_yolo_profile(eng.detector._h, 0)
    valid = cv >= 0
    conv_ms_per_step = float(ms[valid].sum()) / max(nf, 1)
    conv_flop_per_step = float(fl[valid].sum())
    conv_bytes_per_step = float(by[valid].sum())
    n_launch = int(valid.sum())
    achieved = conv_flop_per_step / (conv_ms_per_step * 1e-3) / 1e12 if conv_ms_per_step else 0.0
    achieved_bw = conv_bytes_per_step / (conv_ms_per_step * 1e-3) / 1e9 if conv_ms_per_step else 0.0
    # which roofline binds the conv family: its algorithmic bytes at peak HBM
    # vs its FLOPs at peak bf16 MFMA (small channel counts: bytes win)
    t_hbm = conv_bytes_per_step / (PEAK_HBM * 1e9)
    t_mfma = conv_flop_per_step / (PEAK_BF16 * 1e12)

    # HBM bytes of the conv launches of one step, from the committed
    # PMC passes of this configuration (tools/gpu_pmc.sh -> pmc_traffic.json)
    traffic = None
    tp = os.path.join(REPO, "profiles", "r01", "pmc_traffic.json")
    if os.path.exists(tp):
        traffic = json.load(open(tp)).get("conv_bytes_per_step")
    value = job_throughput(S * K, world, elapsed)
    chunk_desc = (args.graph_chunk if args.graph_chunk is not None
                  else int(os.environ.get("RV_GRAPH_CHUNK", "8")))
    chunk_desc = "all" if chunk_desc <= 0 else str(chunk_desc)
    res = {
        "metric": "end-to-end frames/sec @1080p (preproc+YOLOv8n+SORT), 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": K,
        "warmup": Wm,
        "ms_per_step": round(elapsed / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic 1080p road frames generated on device (resident in HBM); "
                "synthetic LSUV-calibrated YOLOv8n weights (no checkpoint available)",
        "config": {"workload": "full chain 1920x1080, 32 camera streams x 1 frame per step per GPU: "
                               "CLAHE+Median (fused) -> letterbox -> YOLOv8n -> NMS -> SORT+homography",
                   "streams_per_gpu": S, "frame": [H, W], "detector_input": [eng.detector.in_h,
                                                                           eng.detector.in_w],
                   "parallelism": f"streams sharded {S}/GPU, no collective",
                   "conv_autotune": not args.no_autotune,
                   "execution": "eager" if args.eager else
                                ("graph per step" if args.no_pipeline else
                                 f"graphs, {args.depth}-stage software pipeline over steps "
                                 "(preprocess / YOLO / NMS+SORT of consecutive steps overlap), "
                                 f"{chunk_desc} steps per graph")},
        "roofline": {
            "kernel": "conv family: conv_patch_kernel + conv1x1_direct_kernel (all YOLOv8n conv "
                      "launches of a step, HIP events on the launch stream)",
            "bound": "hbm" if t_hbm >= t_mfma else "mfma",
            "achieved": round(achieved_bw if t_hbm >= t_mfma else achieved, 2),
            "peak": PEAK_HBM if t_hbm >= t_mfma else PEAK_BF16,
            "unit": "GB/s" if t_hbm >= t_mfma else "TFLOP/s",
            "frac": round(achieved_bw / PEAK_HBM if t_hbm >= t_mfma else achieved / PEAK_BF16, 5),
            "traffic": traffic,
            "traffic_unit": "bytes per step (all conv launches; rocprofv3 PMC FETCH_SIZE x2 "
                            "+ WRITE_SIZE, profiles/r01/pmc_traffic.json)",
            "algorithmic_bytes_per_step": round(conv_bytes_per_step),
            "algorithmic_gflop_per_step": round(conv_flop_per_step / 1e9, 2),
            "mfma_tflops": round(achieved, 2), "mfma_frac": round(achieved / PEAK_BF16, 5),
            "hbm_gbs": round(achieved_bw, 1), "hbm_frac": round(achieved_bw / PEAK_HBM, 5),
            "launches_per_step": n_launch,
            "conv_ms_per_step": round(conv_ms_per_step, 4),
        },
        "end_to_end_roofline_frac": round(value / world * (BYTES_PER_FRAME / (PEAK_HBM * 1e9) +
                                                           FLOP_PER_FRAME / (PEAK_BF16 * 1e12)), 5),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_frames > 0:
        nfr = args.cpu_frames
        host = frames[Wm:Wm + nfr, 0].cpu().numpy()
        threads = min(16, os.cpu_count() or 1)
        res["cpu_baseline"] = cpu_baseline(host, np.arange(nfr) / 30.0, cfg, threads)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
