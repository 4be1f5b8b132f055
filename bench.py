"""End-to-end benchmark of the MI355X road-vision hot path.

Metric (BASELINE.json): end-to-end frames/sec @1080p (preproc + YOLOv8n +
SORT).  Workload at N=1: configs[2] -- "Full chain 1920x1080 batch=32 on one
MI355X: CLAHE+Median+YOLOv8n+NMS+SORT IoU".  A step = one pass of the hot path
over one stream-major batch (32 camera streams x 1 frame): fused CLAHE+median
(proc frames written to HBM), letterbox, YOLOv8n forward (bf16 MFMA), NMS +
scale_boxes + class filter, SORT (KF + IoU + greedy association) with
ground-plane homography metrics, and the hand-back of the step's detections,
track ids and metrics to pinned host memory (the reference's .cpu().numpy(),
src/detect/yolo_ultralytics.py:44-52).  Inputs are synthetic road frames
generated on the device before the timed region (resident in HBM).

Multi-GPU (torchrun, one process per GPU): camera streams are sharded
(stream s -> rank s // 32), no collective on the data path (weak scaling);
rank timings are reduced with a MAX for the reported time (rvs_amd.shard:
init_from_env, timed_job -- the same code the gloo test drives on the CPU).

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "road-vision-system_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

H, W = 1080, 1920
FLOP_PER_FRAME = 2 * 2.623e9           # YOLOv8n @ 384x640
BYTES_PER_FRAME = 15.39e6              # SURVEY 8(d) algorithmic HBM bytes / 1080p frame
PEAK_BF16 = 2500.0                     # TFLOP/s dense (MI355X_MICROARCH.md)
PEAK_HBM = 8000.0                      # GB/s
IMAGE_POINTS = [[560, 1000], [1360, 1000], [1160, 620], [760, 620]]
WORLD_POINTS = [[-3.5, 5.0], [3.5, 5.0], [3.5, 30.0], [-3.5, 30.0]]
METRIC = "end-to-end frames/sec @1080p (preproc+YOLOv8n+SORT), 1/2/4/8 MI355X"
PMC_TRAFFIC = os.path.join(REPO, "profiles", "r02", "pmc_traffic.json")


def bench_config():
    from rvs_amd.config import load_config
    cfg = load_config()
    cfg["geometry"]["enabled"] = True
    cfg["geometry"]["projector"]["image_points"] = IMAGE_POINTS
    cfg["geometry"]["projector"]["world_points"] = WORLD_POINTS
    cfg["detect"]["weights"] = "synthetic"  # no checkpoint exists here (explicit opt-in)
    return cfg


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)  # pipeline fill/drain < 1 %
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--streams", type=int, default=32, help="camera streams per GPU")
    ap.add_argument("--tmax", type=int, default=int(os.environ.get("RV_TMAX", 1024)),
                    help="SORT track capacity per stream")
    ap.add_argument("--cpu-frames", type=int, default=int(os.environ.get("RV_CPU_FRAMES", 30)))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="launch kernels eagerly (no HIP graph)")
    ap.add_argument("--no-autotune", action="store_true",
                    help="skip the per-layer conv kernel autotuning before the timed region")
    ap.add_argument("--conv-grid", choices=["persistent", "tuned"],
                    default=os.environ.get("RV_CONV_GRID", "persistent"),
                    help="pipelined runs: keep the autotuned tile of every conv launch but run it "
                         "on a persistent grid (default), or keep the autotuner's grid choice")
    ap.add_argument("--tune-save", default=None, help="write the autotuned conv configs (JSON)")
    ap.add_argument("--tune-load", default=None,
                    help="load conv configs saved by --tune-save instead of autotuning")
    ap.add_argument("--conv-timing", choices=["both", "overlap", "eager", "none"], default="both",
                    help="per-launch conv timing after the timed region: HIP events around "
                         "every conv launch while the timed region's multi-stream schedule runs "
                         "eagerly (overlap: same concurrency as the graphs), a plain sequential "
                         "eager pass, or none")
    ap.add_argument("--depth", type=int, default=int(os.environ.get("RV_PIPE_DEPTH", 4)),
                    help="pipelined steps: 4 = Y2(k-1) || P(k+1) || Y1(k) || T(k-2) (the forward "
                         "split in two halves on two forward lanes), 3 = Y(k) || P(k+1) || T(k-1), "
                         "2 = [T(k-1) || P(k)] -> Y(k)")
    ap.add_argument("--graph-chunk", type=int, default=None,
                    help="pipeline steps per captured graph (default 8, RV_GRAPH_CHUNK; 0 = all)")
    ap.add_argument("--pair", type=int, default=int(os.environ.get("RV_PAIR", 4)),
                    help="depth 4: run the forwards of this many consecutive steps as one batch "
                         "(pair x streams frames; SORT still sees every stream in order); the "
                         "largest divisor of --steps not above it is used")
    ap.add_argument("--lanes", type=int, default=int(os.environ.get("RV_LANES", 1)),
                    help="forward lanes: the YOLO forwards of this many consecutive steps run "
                         "concurrently (engine.OverlappedSteps dependency-graph schedule)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one graph per step; no overlap of step k's NMS+SORT with step k+1")
    return ap.parse_args(argv)


def pick_pair(steps: int, pair: int) -> int:
    """Steps per pipeline unit: the largest p <= pair that divides `steps`
    (a driver may pass any --steps)."""
    return max(p for p in range(1, max(1, pair) + 1) if steps % p == 0)


class BenchJob:
    """What one rank runs: its 32 camera streams through the full chain."""

    def __init__(self, args, rank: int, dev):
        from rvs_amd.engine import RoadVisionEngine
        from rvs_amd.shard import rank_streams
        from rvs_amd.synth import road_frames
        self.args, self.dev = args, dev
        self.cfg = bench_config()
        self.S, self.K, self.Wm = args.streams, args.steps, args.warmup
        # depth 4 runs the two halves of consecutive forwards on two lanes
        lanes = 2 if args.depth == 4 and not args.no_pipeline and not args.eager else args.lanes
        pair = 1
        if args.depth == 4 and not args.no_pipeline and not args.eager:
            pair = pick_pair(args.steps, args.pair)
        self.eng = RoadVisionEngine(self.cfg, self.S, (H, W), device=dev, tmax=args.tmax,
                                    lanes=lanes, pair=pair)
        self.frames = road_frames(self.S, self.Wm + self.K, H, W, device=dev,
                                  stream_offset=rank_streams(self.S, rank).start)
        self.ts = torch.tensor([[f / 30.0] * self.S for f in range(self.Wm + self.K)],
                               dtype=torch.float64, device=dev)
        self.units = self.S * self.K
        self.runner = self.graphs = None
        torch.cuda.synchronize()

    def warmup(self):
        for f in range(self.Wm):
            self.eng.step(self.frames[f], self.ts[f])
        torch.cuda.synchronize()

    def prepare(self):
        a, eng = self.args, self.eng
        if a.tune_load:
            with open(a.tune_load) as f:
                eng.detector.load_tuned([tuple(c) for c in json.load(f)["configs"]])
        elif not a.no_autotune:  # per-layer conv kernel choice, on real activations
            eng.autotune(self.frames[0], reps=int(os.environ.get("RV_AUTOTUNE_REPS", "10")))
            if a.conv_grid == "persistent" and not a.eager and not a.no_pipeline:
                # every conv on a persistent grid: the autotuner times each
                # launch alone, but inside the pipelined graphs persistent
                # grids share the chip better (A/B: +0.6 %)
                eng.detector.load_tuned([tuple(c[:4]) + (1,) + tuple(c[5:])
                                         for c in eng.detector.tuned_configs()])
            if a.tune_save:
                with open(a.tune_save, "w") as f:
                    json.dump({"configs": eng.detector.tuned_configs()}, f)
        torch.cuda.synchronize()
        K, Wm = self.K, self.Wm
        if not a.eager and not a.no_pipeline:
            from rvs_amd.engine import OverlappedSteps
            # NMS + SORT + hand-back of step k overlap the preprocess of step k+1
            # and the forward of step k+1 runs beside both (engine.OverlappedSteps)
            self.runner = OverlappedSteps(eng, [self.frames[Wm + k] for k in range(K)],
                                          [self.ts[Wm + k] for k in range(K)], depth=a.depth,
                                          chunk=a.graph_chunk)
        elif not a.eager:
            self.graphs = [eng.capture(self.frames[Wm + k], self.ts[Wm + k])[0] for k in range(K)]
        torch.cuda.synchronize()

    def run(self):
        from rvs_amd import _lib
        st = _lib.stream_ptr()
        _lib.call("rv_trace_marker", 1, st)  # brackets the timed region in a kernel trace
        if self.runner is not None:
            self.runner.run()
        else:
            for k in range(self.K):
                if self.graphs is not None:
                    self.graphs[k].replay()
                else:
                    self.eng.step(self.frames[self.Wm + k], self.ts[self.Wm + k])
        _lib.call("rv_trace_marker", 2, st)

    @staticmethod
    def sync():
        torch.cuda.synchronize()

    def materialise(self) -> dict:
        """Detection-list construction from the handed-back host records of
        the timed steps (host work after the hand-back; reported separately)."""
        from rvs_amd.handback import to_detections
        if self.runner is None:
            return {"in_timed_region": True, "materialise_ms_per_step": None}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        nd = 0
        for rec in self.runner.records:
            n, rows = rec.arrays()
            nd += sum(len(x) for x in to_detections(n, rows, self.eng.names))
        dt = time.perf_counter() - t0
        return {"in_timed_region": True, "record_bytes_per_step": self.runner.records[0].nbytes,
                "detections_per_step": round(nd / self.K, 1),
                "materialise_ms_per_step": round(dt / self.K * 1e3, 3)}

    def track_report(self) -> dict:
        st = self.eng.track_stats()
        return {"tmax": self.args.tmax, "tracks_mean": round(float(st["T"].mean()), 1),
                "tracks_max": int(st["T"].max()), "overflow_streams": int(st["overflow"].sum())}


def rank_job(job, device) -> dict:
    """warm-up, preparation (autotune + capture), then the timed region
    (rvs_amd.shard.timed_job: barrier, sync, K steps, sync, max over ranks)."""
    from rvs_amd.shard import timed_job
    job.warmup()
    job.prepare()
    return timed_job(job.run, job.sync, job.units, device)


def _conv_pass(job, mode: str, tags):
    """One profiled pass over the K steps: HIP events around every conv
    launch of lane 0's forwards (rv_yolo_profile), bracketed by trace
    markers `tags` so tools/trace_window.py can cut the same window out of
    a rocprofv3 trace.  Returns (ms per forward, FLOPs, bytes, launches)."""
    from rvs_amd import _lib
    from rvs_amd.engine import OverlappedSteps
    eng, K, Wm = job.eng, job.K, job.Wm
    lib = _lib.load()
    h = eng.detector._h
    # eager: each conv launched 5x back to back between its events, so an
    # event pair times kernels, not the dispatch gap in front of one kernel
    _lib.check(lib.rv_yolo_profile_reps(h, K, 5 if mode == "eager" else 1), "rv_yolo_profile")
    st = _lib.stream_ptr()
    _lib.call("rv_trace_marker", tags[0], st)
    prof = None
    if mode == "overlap":
        prof = OverlappedSteps(eng, [job.frames[Wm + k] for k in range(K)],
                               [job.ts[Wm + k] for k in range(K)], depth=job.args.depth,
                               chunk=job.args.graph_chunk, capture=False)
    elif eng.pair > 1:  # each launch alone, on the timed region's forward batch
        from rvs_amd.handback import Record
        P = eng.pair
        recs = [Record(eng.S, eng.detector.max_det, eng.device) for _ in range(P)]
        for u in range(K // P):
            eng.step_unit([job.frames[Wm + u * P + h] for h in range(P)],
                          [job.ts[Wm + u * P + h] for h in range(P)], recs)
    else:
        for k in range(K):
            eng.step(job.frames[Wm + k], job.ts[Wm + k])
    _lib.call("rv_trace_marker", tags[1], st)
    torch.cuda.synchronize()
    n = lib.rv_yolo_num_convs(eng.variant)
    ms, fl, by = np.zeros(n), np.zeros(n), np.zeros(n)
    cv = np.zeros(n, np.int32)
    nf = lib.rv_yolo_profile_read(h, ms.ctypes.data, fl.ctypes.data, cv.ctypes.data, n)
    lib.rv_yolo_profile_bytes(h, by.ctypes.data, n)
    prof = None  # noqa: F841 -- eager schedule objects before the events
    torch.cuda.synchronize()
    lib.rv_yolo_profile(h, 0)
    valid = cv >= 0
    # pair mode: every profiled forward covers `pair` steps -> per step
    per = eng.pair
    return (float(ms[valid].sum()) / max(nf, 1) / per, float(fl[valid].sum()) / per,
            float(by[valid].sum()) / per, int(valid.sum()) / per)


def conv_roofline(job, mode: str) -> dict:
    """Roofline of the conv family (every conv launch of a step:
    conv_patch_kernel, conv1x1_direct_kernel, c2f_chain_kernel) from HIP
    events recorded on the launch stream around every conv launch
    (rv_yolo_profile; HIP events recorded inside captured graphs read zero
    elapsed time on ROCm 7.2, so the timed graphs themselves cannot be timed
    this way).  achieved = algorithmic bytes (or FLOPs) of the family per
    step / its measured time per step.
      "eager": one step at a time, each launch alone, five times back to
               back between its events -- the kernels' own speed (the
               headline `roofline`; rocprofv3 cross-check: the trace window
               between the 5th and 6th rv_trace_marker);
      "overlap": the timed region's multi-stream schedule run eagerly, so
               each launch sees the concurrency it sees inside the timed
               graphs (`in_pipeline`; window: markers 3 and 4).
    "both" measures both."""
    eng = job.eng
    job.runner = None  # release the timed graphs (and their memory pool) first
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    res = {}
    for m, tags in (("overlap", (3, 4)), ("eager", (5, 6))):
        if mode in (m, "both"):
            res[m] = _conv_pass(job, m, tags)
    traffic = None
    if os.path.exists(PMC_TRAFFIC):
        traffic = json.load(open(PMC_TRAFFIC)).get("conv_bytes_per_step")

    def view(conv_ms, flop, byts, nl):
        tflops = flop / (conv_ms * 1e-3) / 1e12
        gbs = byts / (conv_ms * 1e-3) / 1e9
        # which roofline binds the conv family: its algorithmic bytes at peak
        # HBM vs its FLOPs at peak bf16 MFMA (small channel counts: bytes win)
        hbm = byts / (PEAK_HBM * 1e9) >= flop / (PEAK_BF16 * 1e12)
        return {"bound": "hbm" if hbm else "mfma",
                "achieved": round(gbs if hbm else tflops, 2),
                "peak": PEAK_HBM if hbm else PEAK_BF16,
                "unit": "GB/s" if hbm else "TFLOP/s",
                "frac": round(gbs / PEAK_HBM if hbm else tflops / PEAK_BF16, 5),
                "mfma_tflops": round(tflops, 2), "mfma_frac": round(tflops / PEAK_BF16, 5),
                "hbm_gbs": round(gbs, 1), "hbm_frac": round(gbs / PEAK_HBM, 5),
                "launches_per_step": nl, "conv_ms_per_step": round(conv_ms, 4),
                "algorithmic_bytes_per_step": round(byts),
                "algorithmic_gflop_per_step": round(flop / 1e9, 2)}
    if not res or any(v[0] <= 0 for v in res.values()):
        return {"error": "no event timings"}
    main = "eager" if "eager" in res else "overlap"
    out = {"kernel": "conv family: conv_patch_kernel + conv1x1_direct_kernel + c2f_chain_kernel "
                     "(all YOLOv8n conv launches of a step; HIP events on the launch stream)",
           "timing": main + (" (one pipeline unit at a time: each launch alone, on the timed "
                             "region's forward batch)" if main == "eager" else
                             " (the timed region's schedule run eagerly)")}
    out.update(view(*res[main]))
    out["traffic"] = traffic
    out["traffic_unit"] = ("bytes per step (all conv launches; rocprofv3 PMC 2 x FETCH_SIZE + "
                           "WRITE_SIZE, separate passes over one eager step; "
                           "profiles/r02/pmc_traffic.json)")
    if main == "eager" and "overlap" in res:
        out["in_pipeline"] = dict(view(*res["overlap"]), timing=(
            "the timed region's schedule run eagerly: each conv launch timed under the "
            "concurrency it has inside the timed graphs"))
    return out


def host_cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(frames_host: np.ndarray, ts: np.ndarray, cfg: dict, threads: int) -> dict:
    """The CPU oracle port of the reference path timed on this host's cores:
    C restatement of CLAHE/median/letterbox (OpenMP over `threads`), torch-CPU
    fp32 YOLOv8n (batch 1, `threads` intra-op threads), restated NMS,
    reference-semantics Python SORT + homography -- frame by frame, as
    main_preview.py:94-109 runs it.  Plus the reference's SORT association
    alone (_iou_matrix Python double loop + greedy, sort_tracker.py:182-210)
    at T = D = 100."""
    from oracle import cpu, sort_ref, yolo_ref
    from rvs_amd.detect.weights import synthetic_weights
    from rvs_amd.geometry import find_homography
    torch.set_num_threads(threads)  # also the OpenMP team of the C oracle
    model = yolo_ref.YoloRef(0, synthetic_weights(0, 0))
    proj = sort_ref.HomographyProjector(find_homography(np.array(IMAGE_POINTS, np.float32),
                                                        np.array(WORLD_POINTS, np.float32)),
                                        (0.0, 0.0), 1000.0)
    trk = sort_ref.SortTracker(cfg["tracking"])
    geo = cpu.letterbox_geometry(H, W)
    keep = cfg["detect"]["classes_keep"]
    stage = np.zeros(4)
    t0 = time.perf_counter()
    n = 0
    for img, t in zip(frames_host, ts):
        a = time.perf_counter()
        proc = cpu.median(cpu.clahe_ycrcb(img, 8, 2.0), 3)
        lb = cpu.letterbox(proc, geo)[None]
        b = time.perf_counter()
        raw = model.forward(yolo_ref.preprocess(lb)).numpy()
        c = time.perf_counter()
        dets = yolo_ref.postprocess(raw, geo[:2], (H, W), classes_keep=keep)[0]
        d = time.perf_counter()
        trk.update([sort_ref.Det(*map(float, r[:5]), int(r[5])) for r in dets], float(t), proj)
        e = time.perf_counter()
        stage += [b - a, c - b, d - c, e - d]
        n += 1
    dt = time.perf_counter() - t0
    # the reference's association at T = D = 100 (72.9 ms on the container Xeon)
    rng = np.random.default_rng(0)
    xy = rng.uniform(0, 1800, (100, 2)).astype(np.float32)
    wh = rng.uniform(20, 200, (100, 2)).astype(np.float32)
    tb = np.concatenate([xy, xy + wh], 1)
    db = tb + rng.normal(0, 3, tb.shape).astype(np.float32)
    reps = 5
    a = time.perf_counter()
    for _ in range(reps):
        sort_ref.greedy(sort_ref.iou_matrix(tb, db), cfg["tracking"]["iou_threshold"])
    assoc_ms = (time.perf_counter() - a) / reps * 1e3
    return {"value": n / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "cpu_model": host_cpu_model(),
            "torch_threads": torch.get_num_threads(),
            "stage_ms_per_frame": {k: round(v / n * 1e3, 2) for k, v in
                                   zip(["preprocess+letterbox", "yolov8n_fp32", "nms",
                                        "sort+homography"], stage)},
            "sort_associate_ms_T100_D100": round(assoc_ms, 2),
            "sample": f"{n} consecutive 1080p frames of one stream, full chain (C oracle "
                      f"CLAHE+median+letterbox on {threads} OpenMP threads, torch-CPU fp32 "
                      f"YOLOv8n {threads} threads, restated NMS, Python SORT+homography); "
                      f"{dt:.1f} s"}


def main(argv=None):
    args = parse_args(argv)
    from rvs_amd.shard import init_from_env
    rank, world, local = init_from_env("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    job = BenchJob(args, rank, dev)
    t = rank_job(job, dev)
    elapsed, value = t["elapsed_s"], t["value"]
    K, S = job.K, job.S
    handback = job.materialise()
    sort_rep = job.track_report()
    roof = conv_roofline(job, args.conv_timing) if args.conv_timing != "none" else None

    P = job.eng.pair
    if args.graph_chunk is not None:
        chunk_desc = args.graph_chunk
    else:
        chunk_desc = int(os.environ.get("RV_GRAPH_CHUNK", "8"))
        chunk_desc = max(1, chunk_desc // P) if chunk_desc > 0 and P > 1 else chunk_desc
    chunk_desc = "all" if chunk_desc <= 0 else str(chunk_desc)
    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": K,
        "warmup": job.Wm,
        "ms_per_step": round(elapsed / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic 1080p road frames generated on device (resident in HBM); "
                "synthetic calibrated YOLOv8n weights (no checkpoint available)",
        "config": {"workload": "full chain 1920x1080, 32 camera streams x 1 frame per step per GPU: "
                               "CLAHE+Median (fused) -> letterbox -> YOLOv8n -> NMS -> "
                               "SORT+homography -> result hand-back to pinned host memory",
                   "streams_per_gpu": S, "frame": [H, W],
                   "detector_input": [job.eng.detector.in_h, job.eng.detector.in_w],
                   "parallelism": f"streams sharded {S}/GPU, no collective",
                   "forward_batch": S * job.eng.pair,
                   "conv_autotune": ("loaded" if args.tune_load else
                                     (not args.no_autotune)),
                   "conv_grid": args.conv_grid,
                   "execution": "eager" if args.eager else
                                ("graph per step" if args.no_pipeline else
                                 ("graphs, 4-stage software pipeline: stage k runs the second "
                                  "half of unit k-1's forward || preprocess of unit k+1 || the "
                                  "first half of unit k's forward || NMS+SORT+hand-back of unit "
                                  f"k-2 (two forward workspaces; a unit = {job.eng.pair} step(s), "
                                  f"one forward over their {S * job.eng.pair} frames), "
                                  f"{chunk_desc} units per graph"
                                  if args.depth == 4 else
                                  f"graphs, dependency-graph pipeline with {args.lanes} concurrent "
                                  "YOLO forwards (preprocess runs ahead, NMS+SORT+hand-back "
                                  f"follows in step order), {chunk_desc} steps per graph"
                                  if args.lanes > 1 else
                                  f"graphs, {args.depth}-stage software pipeline over steps "
                                  "(preprocess / YOLO / NMS+SORT+hand-back of consecutive steps "
                                  f"overlap), {chunk_desc} steps per graph"))},
        "roofline": roof,
        "end_to_end_roofline_frac": round(value / world * (BYTES_PER_FRAME / (PEAK_HBM * 1e9) +
                                                           FLOP_PER_FRAME / (PEAK_BF16 * 1e12)), 5),
        "sort": sort_rep,
        "handback": handback,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_frames > 0:
        nfr = args.cpu_frames
        host = job.frames[:nfr, 0].cpu().numpy()
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        res["cpu_baseline"] = cpu_baseline(host, np.arange(nfr) / 30.0, job.cfg, threads)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
