"""End-to-end benchmark of the MI355X road-vision hot path.

Metric (BASELINE.json): end-to-end frames/sec @1080p (preproc + YOLOv8n +
SORT).  Workload at N=1: configs[2] -- "Full chain 1920x1080 batch=32 on one
MI355X: CLAHE+Median+YOLOv8n+NMS+SORT IoU".  A step = one pass of the hot path
over one stream-major batch (32 camera streams x 1 frame): fused CLAHE+median
(proc frames written to HBM), letterbox, YOLOv8n forward (bf16 MFMA), NMS +
scale_boxes + class filter, SORT (KF + IoU + greedy association) with
ground-plane homography metrics, the hand-back of the step's detections,
track ids and metrics to pinned host memory, and -- on a consumer thread
inside the timed region -- the reference's List[Detection] of every stream
(src/detect/yolo_ultralytics.py:44-52, src/track/sort_tracker.py:278).
Inputs are synthetic road frames generated on the device before the timed
region (resident in HBM).

The K steps run as the 4-stage software pipeline of rvs_amd.schedule
(PipelinedRun: native launch list over four HIP streams, no graph capture).

Multi-GPU: one process per GPU.  Under torchrun the rank comes from the
environment; ``--gpus N`` without it spawns the N ranks itself (fresh child
processes, before this process touches the GPU).  Camera streams are
sharded (stream s -> rank s // 32), no collective on the data path (weak
scaling); rank timings are reduced with a MAX (rvs_amd.shard.timed_job).

Prints ONE JSON line (rank 0).
"""
import argparse
import gc
import hashlib
import importlib
import json
import os
import socket
import subprocess
import sys
import threading
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
PMC_TRAFFIC = os.path.join(REPO, "profiles", "r06", "pmc_traffic.json")
LIB = os.path.join(REPO, "road-vision-system_amd", "rvs_amd", "librvhip.so")


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
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--streams", type=int, default=32, help="camera streams per GPU")
    ap.add_argument("--tmax", type=int, default=int(os.environ.get("RV_TMAX", 1024)),
                    help="SORT track capacity per stream")
    ap.add_argument("--exec", dest="exec_mode", choices=["native", "eager", "sequential"],
                    default=os.environ.get("RV_EXEC", "native"),
                    help="the pipelined schedule issued by the native launch list (one C call "
                         "per run) or eagerly from Python; or plain sequential step() calls")
    ap.add_argument("--sync", choices=["flow", "stage"], default=os.environ.get("RV_SYNC", "flow"),
                    help="pipeline dependencies: per-dependency events (flow) or lock-stepped "
                         "stages (stage)")
    ap.add_argument("--pair", type=int, default=int(os.environ.get("RV_PAIR", 4)),
                    help="steps per pipeline unit (one forward over pair x streams frames); the "
                         "largest divisor of --steps not above it is used")
    ap.add_argument("--units", default=os.environ.get("RV_UNITS", "ends"),
                    help="pipeline unit sizes: 'ends' (default: half units of pair / 2 steps "
                         "first and last, pair steps between -- at --steps 20, 2,4,4,4,4,2), "
                         "'even' (--steps / pair units of pair steps), 'ramp' (units of 1 and 2 "
                         "steps at both ends of the run, pair steps between), or an explicit "
                         "comma-separated list summing to --steps")
    ap.add_argument("--warm-runs", type=int, default=int(os.environ.get("RV_WARM_RUNS", 3)),
                    help="untimed runs of the recorded schedule over the timed frames before the "
                         "timed region (warm-up of the schedule itself)")
    ap.add_argument("--no-consumer", action="store_true",
                    help="do not build the Detection lists inside the timed region")
    ap.add_argument("--no-autotune", action="store_true",
                    help="skip the per-layer conv kernel autotuning before the timed region")
    ap.add_argument("--conv-grid", choices=["persistent", "tuned"],
                    default=os.environ.get("RV_CONV_GRID", "persistent"),
                    help="keep the autotuned tile of every conv launch but run it on a "
                         "persistent grid (default), or keep the autotuner's grid choice")
    ap.add_argument("--tune-save", default=None, help="write the autotuned conv configs (JSON)")
    ap.add_argument("--tune-load", default=None,
                    help="load conv configs saved by --tune-save instead of autotuning")
    ap.add_argument("--conv-timing", choices=["both", "overlap", "eager", "none"], default="both",
                    help="per-launch conv timing after the timed region (HIP events around every "
                         "conv launch): the timed region's schedule issued eagerly (overlap), one "
                         "unit at a time with each launch alone (eager), both, or none")
    ap.add_argument("--cpu-frames", type=int, default=int(os.environ.get("RV_CPU_FRAMES", 12)),
                    help="CPU baseline: frames per worker (one camera stream per worker)")
    ap.add_argument("--cpu-workers", type=int, default=int(os.environ.get("RV_CPU_WORKERS", 0)),
                    help="CPU baseline workers (0: the CPUs this process may use: its affinity "
                         "mask capped by the cgroup CPU quota, host_cpu_budget)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the pair-1 rate and the secondary legs (configs[1], configs[4], "
                         "host-fed NV12; bench_extra.py)")
    ap.add_argument("--job", default=None,
                    help="module:Class of a stand-in rank job (CPU rehearsal of the rank logic "
                         "with gloo; tests/test_shard_gloo.py)")
    return ap.parse_args(argv)


def pick_pair(steps: int, pair: int) -> int:
    """Steps per pipeline unit: the largest p <= pair that divides `steps`
    (a driver may pass any --steps)."""
    return max(p for p in range(1, max(1, pair) + 1) if steps % p == 0)


def unit_sizes(steps: int, pair: int, spec: str) -> list:
    """Steps per pipeline unit, in order (rvs_amd.schedule.PipelinedRun
    units).  'even': steps / p units of p = pick_pair(steps, pair); 'ends':
    the same with the first and the last unit split in halves; 'ramp':
    1- and 2-step units at both ends (the first unit's preprocess and the
    last unit's forward + tracking run with little beside them, so small end
    units shorten the fill and the drain), units of `pair` between, any
    remainder as one unit in the middle; else an explicit list."""
    if spec == "even":
        p = pick_pair(steps, pair)
        return [p] * (steps // p)
    if spec == "ends":
        # the first unit's preprocess runs with nothing beside it (the fill)
        # and the last unit's forward + tracking with little beside it (the
        # drain); half-size units there shorten both (r06: 2,4,4,4,4,2 vs
        # even at --steps 20, three interleaved rounds on one box: 47.2k vs
        # 46.5k frames/s, profiles/r06/unit_layout_ab.txt)
        p = pick_pair(steps, pair)
        if p % 2 or steps // p < 2:
            return [p] * (steps // p)
        return [p // 2] + [p] * (steps // p - 1) + [p // 2]
    if spec == "ramp":
        head = [h for h in (1, 2) if h < pair]
        if 2 * sum(head) + pair > steps:
            p = pick_pair(steps, pair)
            return [p] * (steps // p)
        mid = steps - 2 * sum(head)
        body = [pair] * (mid // pair)
        if mid % pair:
            body.insert(len(body) // 2, mid % pair)
        return head + body + head[::-1]
    units = [int(x) for x in spec.split(",") if x.strip()]
    if sum(units) != steps or min(units) < 1:
        raise SystemExit(f"--units {spec}: sizes must be >= 1 and sum to --steps {steps}")
    return units


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv) -> int:
    """`--gpus N` without a torchrun environment: start N fresh ranks of this
    script (rank r on GPU r, torchrun's variables), wait for all of them and
    return the worst exit code.  Called before anything touches the GPU."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    codes = [p.wait() for p in procs]
    return max(codes, key=abs)


class BenchJob:
    """What one rank runs: its 32 camera streams through the full chain."""

    def __init__(self, args, rank: int, dev, frames=None):
        from rvs_amd.engine import RoadVisionEngine
        from rvs_amd.shard import rank_streams
        from rvs_amd.synth import road_frames
        self.args, self.dev = args, dev
        self.cfg = bench_config()
        self.S, self.K, self.Wm = args.streams, args.steps, args.warmup
        seq = args.exec_mode == "sequential"
        self.unit_sizes = None if seq else unit_sizes(args.steps, args.pair, args.units)
        lanes, pair = (1, 1) if seq else (2, max(self.unit_sizes))
        self.eng = RoadVisionEngine(self.cfg, self.S, (H, W), device=dev, tmax=args.tmax,
                                    lanes=lanes, pair=pair)
        self.frames = frames if frames is not None else road_frames(
            self.S, self.Wm + self.K, H, W, device=dev, stream_offset=rank_streams(self.S, rank).start)
        self.ts = torch.tensor([[f / 30.0] * self.S for f in range(self.Wm + self.K)],
                               dtype=torch.float64, device=dev)
        self.units = self.S * self.K
        self.runner = None
        # host thread during the timed region: "consume" builds every step's
        # Detection lists, "watch" only notes when each step was handed back
        self.consume = "off" if args.no_consumer else "consume"
        self._consumer = None
        self.cons = {}
        self.records = None
        self.device_end = 0.0
        self.issue_s = 0.0
        self.tags = (1, 2)       # rv_trace_marker tags around the timed region
        self.t_device_only = None  # local time of the device-only rerun
        self.sort_saved = None   # SORT state the timed region starts from
        torch.cuda.synchronize()

    def warmup(self):
        for f in range(self.Wm):
            out = self.eng.step(self.frames[f], self.ts[f])
        if self.Wm:
            self.eng.results(out)
        torch.cuda.synchronize()

    def prepare(self):
        a, eng = self.args, self.eng
        if a.tune_load:
            with open(a.tune_load) as f:
                eng.detector.load_tuned([tuple(c) for c in json.load(f)["configs"]])
        elif not a.no_autotune:  # per-layer conv kernel choice, on real activations
            eng.autotune(self.frames[0], reps=int(os.environ.get("RV_AUTOTUNE_REPS", "10")))
            if a.conv_grid == "persistent" and a.exec_mode != "sequential":
                # every conv on a persistent grid: the autotuner times each
                # launch alone, but beside the other pipeline stages persistent
                # grids share the chip better
                eng.detector.load_tuned([tuple(c[:4]) + (1,) + tuple(c[5:])
                                         for c in eng.detector.tuned_configs()])
            if a.tune_save:
                with open(a.tune_save, "w") as f:
                    json.dump({"configs": eng.detector.tuned_configs()}, f)
        torch.cuda.synchronize()
        K, Wm = self.K, self.Wm
        if a.exec_mode == "sequential":
            from rvs_amd.handback import Record
            self.records = [Record(self.S, eng.detector.max_det, self.dev) for _ in range(K)]
        else:
            from rvs_amd.schedule import PipelinedRun
            self.runner = PipelinedRun(eng, [self.frames[Wm + k] for k in range(K)],
                                       [self.ts[Wm + k] for k in range(K)], mode=a.exec_mode,
                                       sync=a.sync, units=self.unit_sizes)
            self.records = self.runner.records
            # the SORT state is restored after the warm runs (and before the
            # device-only rerun), so every timed run sees exactly the tracks
            # the warm-up steps left
            self.sort_saved = eng.tracker.state[0].clone()
            # everything allocated so far (torch, the engine, the plans) is
            # long-lived: move it out of the collector's generations, so a
            # full collection triggered by the consumer's Detection objects
            # does not traverse it inside a timed region (a 75 ms stall in
            # one of six runs without this, tools/consumer_ab.py); done
            # before the warm runs, so the device is busy up to the region
            gc.collect()
            gc.freeze()
            # the warm runs are the timed region's code path (schedule, the
            # consumer or watcher thread, its hand-back waits and Detection
            # lists), under their own marker tags 9/10: without the host
            # thread in them, its first-run costs landed in the timed region
            # (first run 40.0-40.3k against 41.7-41.8k frames/s after one
            # more untimed run with the thread, tools/consumer_ab.py, r04)
            tags, self.tags = self.tags, (9, 10)
            for _ in range(a.warm_runs):
                self.run()
                self.sync()
            self.tags = tags
            eng.tracker.state[0].copy_(self.sort_saved)
        torch.cuda.synchronize()

    def _consume(self, wait_step, materialise: bool, ready=None):
        """The consumer: every step's List[Detection] per stream, built as
        soon as that step's record has been handed back (materialise=False:
        only the host time each step became available)."""
        from rvs_amd.handback import DetectionPool
        names, n_det, busy, done = self.eng.names, 0, 0.0, []
        # Detection shells made while waiting for the next hand-back (the
        # allocations move out of the step's critical tail)
        # (made only while the next step is not ready yet: in a burst of
        # hand-backs the lists are built from what the pool holds)
        use_pool = os.environ.get("RV_CONSUMER_POOL", "1") != "0"  # A/B probe
        pool = DetectionPool() if materialise and ready is not None and use_pool else None
        want = 8192
        # RV_CONSUMER_DEFER=1 (A/B probe) builds every list after the last
        # step's hand-back (still inside the timed region).  The cyclic
        # garbage collector is off while the lists are built (the Detection
        # objects hold no cycles: reference counting frees them): a
        # collection triggered by the ~30k new objects of a run stalled the
        # consumer's last steps by up to 0.6 ms (r06: 4 interleaved rounds,
        # 46.8k -> 47.4k frames/s, profiles/r06/session_ab/r06ze;
        # RV_CONSUMER_NOGC=0 leaves it on)
        defer = os.environ.get("RV_CONSUMER_DEFER", "0") != "0"
        nogc = os.environ.get("RV_CONSUMER_NOGC", "1") != "0"
        if nogc:
            import gc
            gc.disable()
        if defer:
            wait_step(len(self.records) - 1)
        for k, rec in enumerate(self.records):
            if pool is not None:
                while len(pool.items) < want and not ready(k):
                    pool.top_up(min(want, len(pool.items) + 512))
            wait_step(k)
            t = time.perf_counter()
            done.append(t)
            if materialise:
                nk = sum(len(x) for x in rec.detections(names, pool))
                n_det += nk
                want = max(want, 5 * nk)
                busy += time.perf_counter() - t
        if nogc:
            gc.enable()
        self.cons = {"detections": n_det, "busy_s": busy, "end": time.perf_counter(),
                     "done": done}

    def run(self):
        from rvs_amd import _lib
        st = _lib.stream_ptr()
        _lib.call("rv_trace_marker", self.tags[0], st)  # brackets the region in a kernel trace
        t0 = time.perf_counter()
        if self.runner is not None:
            self.runner.run()
            wait = self.runner.wait_step
            ready = self.runner.step_ready
        else:
            evs = []
            for k in range(self.K):
                self.eng.step(self.frames[self.Wm + k], self.ts[self.Wm + k], self.records[k])
                e = torch.cuda.Event()
                e.record()
                evs.append(e)
            wait = lambda k: evs[k].synchronize()  # noqa: E731
            ready = lambda k: evs[k].query()  # noqa: E731
        self.issue_s = time.perf_counter() - t0
        _lib.call("rv_trace_marker", self.tags[1], st)
        if self.consume != "off":
            self._consumer = threading.Thread(target=self._consume,
                                              args=(wait, self.consume == "consume", ready))
            self._consumer.start()

    def sync(self):
        torch.cuda.synchronize()
        self.device_end = time.perf_counter()
        if self._consumer is not None:
            self._consumer.join()
            self._consumer = None

    def track_report(self) -> dict:
        st = self.eng.track_stats()
        return {"tmax": self.args.tmax, "tracks_mean": round(float(st["T"].mean()), 1),
                "tracks_max": int(st["T"].max()), "overflow_streams": int(st["overflow"].sum())}


def rank_job(job, device) -> dict:
    """warm-up, preparation (autotune + the recorded schedule), then the
    timed region (rvs_amd.shard.timed_job: barrier, sync, K steps, sync, max
    over ranks)."""
    from rvs_amd.shard import timed_job
    job.warmup()
    job.prepare()
    return timed_job(job.run, job.sync, job.units, device)


def rank_job_again(job, device) -> dict:
    """A second timed region over the same recorded schedule, without the
    Detection lists (a watcher thread only notes each step's completion),
    from the same SORT state as the first (the same timestamps replayed on
    continued tracks would run time backwards), bracketed by marker tags 7/8."""
    from rvs_amd.shard import timed_job
    consume, job.consume = job.consume, "watch"
    tags, job.tags = job.tags, (7, 8)
    if job.sort_saved is not None:
        job.eng.tracker.state[0].copy_(job.sort_saved)
    try:
        return timed_job(job.run, job.sync, job.units, device)
    finally:
        job.consume = consume
        job.tags = tags


def _union_ms(t0, t1) -> float:
    """Total length of the union of the intervals [t0[i], t1[i])."""
    tot, cs, ce = 0.0, None, None
    for a, b in sorted(zip(t0, t1)):
        if ce is None or a > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    return tot + (ce - cs if ce is not None else 0.0)


def _conv_pass(job, mode: str, tags):
    """One profiled pass over the K steps: HIP events around every conv
    launch of every forward context (rv_yolo_profile on each lane's handle),
    bracketed by trace markers `tags` so tools/trace_window.py can cut the
    same window out of a rocprofv3 trace.  Returns per step: (summed launch
    ms, FLOPs, bytes, launches, chip-union ms of the conv launches)."""
    from rvs_amd import _lib
    from rvs_amd.schedule import PipelinedRun
    eng, K, Wm = job.eng, job.K, job.Wm
    lib = _lib.load()
    hs = list(eng.detector._hs)
    # eager: each conv launched 5x back to back between its events, so an
    # event pair times kernels, not the dispatch gap in front of one kernel
    for h in hs:
        _lib.check(lib.rv_yolo_profile_reps(h, K, 5 if mode == "eager" else 1), "rv_yolo_profile")
    st = _lib.stream_ptr()
    _lib.call("rv_trace_marker", tags[0], st)
    if mode == "overlap":  # the timed region's schedule, issued eagerly with the events
        if job.sort_saved is not None:
            eng.tracker.state[0].copy_(job.sort_saved)
        prof = PipelinedRun(eng, [job.frames[Wm + k] for k in range(K)],
                            [job.ts[Wm + k] for k in range(K)], mode="eager", sync=job.args.sync,
                            units=job.unit_sizes)
        prof.run()
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
    ms_tot, nf_tot = np.zeros(n), 0
    fl, by, cv = np.zeros(n), np.zeros(n), np.zeros(n, np.int32)
    t0s, t1s = [], []
    for h in hs:
        ms, f1, c1, b1 = np.zeros(n), np.zeros(n), np.zeros(n, np.int32), np.zeros(n)
        nf = lib.rv_yolo_profile_read(h, ms.ctypes.data, f1.ctypes.data, c1.ctypes.data, n)
        if nf <= 0:  # a lane that ran no forward in this pass
            continue
        lib.rv_yolo_profile_bytes(h, b1.ctypes.data, n)
        fl, cv, by = f1, c1, b1  # the same plan on every lane
        ms_tot += ms
        nf_tot += nf
        cnt = lib.rv_yolo_profile_times(h, hs[0], None, None, 0) \
            if hasattr(lib, "rv_yolo_profile_times") else 0  # (an older A/B build lacks it)
        if cnt > 0:
            a, b = np.zeros(cnt), np.zeros(cnt)
            lib.rv_yolo_profile_times(h, hs[0], a.ctypes.data, b.ctypes.data, cnt)
            t0s += a.tolist()
            t1s += b.tolist()
    torch.cuda.synchronize()
    for h in hs:
        lib.rv_yolo_profile(h, 0)
    valid = cv >= 0
    # every profiled forward covers `pair` steps -> per step
    per = eng.pair
    steps = max(nf_tot, 1) * per
    union = _union_ms(t0s, t1s) / steps if mode == "overlap" else None
    table = os.environ.get("RV_CONV_TABLE")
    if table:  # per-launch table of this pass (tools: per-layer roofline)
        from rvs_amd.detect.weights import conv_list
        names = [c[0] for c in conv_list(eng.variant)]
        names[0] = "stem (model.0 + model.1 + model.2.cv1)"  # slot n - 1: the fused stem
        with open(f"{table}_{mode}.json", "w") as f:
            json.dump({"mode": mode, "forwards": int(nf_tot), "batch": eng.S * eng.pair,
                       "launches": [{"conv": names[int(cv[i])], "us": ms_tot[i] / max(nf_tot, 1) * 1e3,
                                     "gflop": fl[i] / 1e9, "mb": by[i] / 1e6}
                                    for i in range(n) if cv[i] >= 0]}, f, indent=0)
    return (float(ms_tot[valid].sum()) / steps, float(fl[valid].sum()) / per,
            float(by[valid].sum()) / per, int(valid.sum()) / per, union)


def _sort_phase_report():
    """Per-phase time of the fused SORT kernel averaged over every block of
    the run (a -DRV_SORT_PHASE build, RV_LIB_VARIANT=sph: tools/sort_phase.py);
    None for the production build."""
    from rvs_amd import _lib
    lib = _lib.load()
    if not hasattr(lib, "rv_sort_phase_read"):
        return None
    import ctypes
    buf = (ctypes.c_ulonglong * 8)()
    lib.rv_sort_phase_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.rv_sort_phase_read(buf, 0)
    n = max(1, buf[7])
    names = ["predict+load", "iou pairs", "sort", "greedy", "bookkeeping", "kf update+metrics"]
    return {"blocks": int(buf[7]), **{k: round(buf[i] / n / 100.0, 2) for i, k in enumerate(names)},
            "unit": "us per block (wall clock, 100 MHz)"}


def _lib_sha256() -> str:
    with open(LIB, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_traffic() -> dict:
    """HBM bytes per step of the conv family from rocprofv3 PMC passes
    (tools/gpu_pmc.sh -> profiles/r06/pmc_traffic.json), reported only when
    they were collected on the library this run loaded (same sha256)."""
    if not os.path.exists(PMC_TRAFFIC):
        return {"traffic": None, "traffic_note": "no PMC pass of this round's library"}
    d = json.load(open(PMC_TRAFFIC))
    if d.get("librvhip_sha256") != _lib_sha256():
        return {"traffic": None,
                "traffic_note": "the PMC passes in profiles/r06/pmc_traffic.json were collected "
                                "on another build of librvhip.so: not reported"}
    return {"traffic": d.get("conv_bytes_per_step"),
            "traffic_unit": "HBM bytes per step, all conv launches (rocprofv3 PMC: 2 x "
                            "FETCH_SIZE + WRITE_SIZE, separate passes, this build; "
                            "profiles/r06/pmc_traffic.json)"}


def conv_roofline(job, mode: str) -> dict:
    """Roofline of the conv family (every conv launch of a step:
    conv_patch_kernel, conv1x1_direct_kernel, c2f_chain_kernel, and the fused
    stem_kernel = model.0 + model.1 + model.2.cv1) against
    SURVEY §8(d)'s MFMA bound: achieved = the family's algorithmic FLOPs per
    step / its HIP-event-timed duration per step (rv_yolo_profile: events on
    the launch stream around every conv launch).
      "eager": one pipeline unit at a time, each launch alone, five times
               back to back between its events -- the kernels' own speed
               (the headline; rocprofv3 cross-check: trace window between
               the rv_trace_marker tags 5 and 6);
      "overlap": the timed region's schedule issued eagerly (tags 3 and 4),
               so each launch sees the concurrency it has in the timed
               region (`in_pipeline`): achieved = FLOPs / the chip-union
               busy time of the conv launches of both forward lanes (the
               time at least one conv launch is in flight), which can never
               exceed the step time; the summed launch durations (2-3
               streams run conv launches at once) are reported beside it.
    The bytes view (algorithmic activation + weight bytes of the launches at
    8 TB/s) is reported beside it."""
    job.runner = None
    torch.cuda.synchronize()
    res = {}
    for m, tags in (("overlap", (3, 4)), ("eager", (5, 6))):
        if mode in (m, "both"):
            res[m] = _conv_pass(job, m, tags)

    def view(conv_ms, flop, byts, nl, union=None):
        t = union if union else conv_ms
        tflops = flop / (t * 1e-3) / 1e12
        gbs = byts / (t * 1e-3) / 1e9
        v = {"bound": "mfma", "achieved": round(tflops, 2), "peak": PEAK_BF16,
             "unit": "TFLOP/s", "frac": round(tflops / PEAK_BF16, 5),
             "bytes_view": {"achieved_gbs": round(gbs, 1), "peak_gbs": PEAK_HBM,
                            "frac": round(gbs / PEAK_HBM, 5),
                            "algorithmic_bytes_per_step": round(byts)},
             "launches_per_step": nl, "conv_ms_per_step": round(t, 4),
             "algorithmic_gflop_per_step": round(flop / 1e9, 2)}
        if union:
            v["summed_launch_ms_per_step"] = round(conv_ms, 4)
        return v
    if not res or any(v[0] <= 0 for v in res.values()):
        return {"error": "no event timings"}
    # the line leads with what the timed region achieves: the in-pipeline
    # (chip-union) view when it was measured; the eager view -- each launch
    # alone, its inputs warm in L2 / MALL from the back-to-back repetitions --
    # is the kernels' own speed, reported beside it
    main = "overlap" if "overlap" in res else "eager"
    notes = {"eager": ("eager: one pipeline unit at a time, each launch alone, 5 back-to-back "
                       "repetitions between its events (repetitions 2-5 find their inputs in L2 / "
                       "MALL), on the timed region's forward batch; trace window: marker tags 5-6"),
             "overlap": ("in the pipeline: the timed region's schedule issued eagerly (trace "
                         "window: marker tags 3-4); conv_ms_per_step = the chip-union busy time "
                         "of the conv launches of both forward lanes (HIP events on each launch "
                         "stream), summed_launch_ms_per_step = their summed durations")}
    out = {"kernel": "conv family: conv_patch_kernel + conv1x1_direct_kernel + c2f_chain_kernel "
                     "+ stem_kernel "
                     "(all YOLOv8n conv launches of a step; HIP events on the launch stream)",
           "timing": notes[main]}
    out.update(view(*res[main]))
    out.update(pmc_traffic())
    if main == "overlap" and "eager" in res:
        out["eager"] = dict(view(*res["eager"]), timing=notes["eager"])
    return out


def host_cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpu_budget() -> dict:
    """The CPUs this process can actually use: its affinity mask, capped by
    the cgroup CPU quota when one is set (cgroup v2 cpu.max, or v1
    cpu.cfs_quota_us / cfs_period_us).  On the GPU box the mask lists all
    256 host CPUs but cpu.max grants 16 CPUs' worth of time, so more than 16
    single-threaded workers would only time-share those 16."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None and int(quota) < aff:
        n = max(1, int(quota))
        return {"cpus": n, "quota_cpus": round(quota, 2),
                "reason": f"cgroup CPU quota = {quota:g} CPUs of the {aff} in the affinity mask: "
                          f"one single-threaded worker per quota CPU"}
    return {"cpus": aff, "quota_cpus": None if quota is None else round(quota, 2),
            "reason": f"all {aff} CPUs of the affinity mask (no tighter cgroup CPU quota)"}


def _cpu_worker(wid: int, nfr: int, cfg: dict, start, q):
    """One camera stream on one core: the oracle port of the reference chain
    frame by frame, single-threaded, as main_preview.py:94-109 runs it: C
    restatement of CLAHE/median/letterbox, torch-CPU fp32 YOLOv8n, restated
    NMS, reference-semantics Python SORT + homography."""
    os.environ["OMP_NUM_THREADS"] = "1"
    torch.set_num_threads(1)
    from oracle import cpu, sort_ref, yolo_ref
    from rvs_amd.detect.weights import synthetic_weights
    from rvs_amd.geometry import find_homography
    from rvs_amd.synth import road_frames
    frames = road_frames(1, nfr, H, W, device="cpu", stream_offset=wid)[:, 0].numpy()
    model = yolo_ref.YoloRef(0, synthetic_weights(0, 0))
    proj = sort_ref.HomographyProjector(find_homography(np.array(IMAGE_POINTS, np.float32),
                                                        np.array(WORLD_POINTS, np.float32)),
                                        (0.0, 0.0), 1000.0)
    trk = sort_ref.SortTracker(cfg["tracking"])
    geo = cpu.letterbox_geometry(H, W)
    keep = cfg["detect"]["classes_keep"]
    stage = np.zeros(4)
    start.wait()
    t0 = time.perf_counter()
    for f, img in enumerate(frames):
        a = time.perf_counter()
        proc = cpu.median(cpu.clahe_ycrcb(img, 8, 2.0), 3)
        lb = cpu.letterbox(proc, geo)[None]
        b = time.perf_counter()
        raw = model.forward(yolo_ref.preprocess(lb)).numpy()
        c = time.perf_counter()
        dets = yolo_ref.postprocess(raw, geo[:2], (H, W), classes_keep=keep)[0]
        d = time.perf_counter()
        trk.update([sort_ref.Det(*map(float, r[:5]), int(r[5])) for r in dets], f / 30.0, proj)
        e = time.perf_counter()
        stage += [b - a, c - b, d - c, e - d]
    q.put((wid, len(frames), time.perf_counter() - t0, stage.tolist()))


def cpu_baseline(cfg: dict, nfr: int, workers: int) -> dict:
    """The CPU oracle port of the reference path on this host: `workers`
    processes, one camera stream each on one core (streams are independent,
    SURVEY §8(e)), released together after each has built its frames and
    model; value = all frames / the slowest worker's time.  Plus the
    reference's SORT association alone (_iou_matrix Python double loop +
    greedy, sort_tracker.py:182-210) at T = D = 100."""
    import multiprocessing as mp
    from oracle import sort_ref
    ctx = mp.get_context("spawn")  # fresh interpreters: nothing GPU-side is inherited
    start, q = ctx.Event(), ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker, args=(w, nfr, cfg, start, q)) for w in range(workers)]
    for p in procs:
        p.start()
    start.set()  # each worker times only its own frame loop (after its setup)
    res = [q.get(timeout=900) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    frames = sum(r[1] for r in res)
    slowest = max(r[2] for r in res)
    stage = np.sum([r[3] for r in res], axis=0) / frames
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
    return {"value": frames / slowest, "unit": "frames/s", "cores": workers, "kind": "port",
            "host_cpus": os.cpu_count(), "cpus_allowed": len(os.sched_getaffinity(0)),
            "cpu_model": host_cpu_model(),
            "per_core_frames_per_s": round(frames / sum(r[2] for r in res), 3),
            "stage_ms_per_frame": {k: round(v * 1e3, 2) for k, v in
                                   zip(["preprocess+letterbox", "yolov8n_fp32", "nms",
                                        "sort+homography"], stage)},
            "sort_associate_ms_T100_D100": round(assoc_ms, 2),
            "sample": f"{workers} camera streams x {nfr} consecutive 1080p frames, one stream "
                      f"per worker process on one core (C oracle CLAHE+median+letterbox, "
                      f"torch-CPU fp32 YOLOv8n, restated NMS, Python SORT+homography; 1 thread "
                      f"each); slowest worker {slowest:.1f} s"}


def steady_state(job, mult: int = 3) -> dict:
    """The pipeline's steady-state rate, free of its fill and drain: the same
    schedule recorded over mult x K steps (the K timed frames cycled, fresh
    timestamps), timed device-only like the rerun; the marginal rate of the
    extra (mult - 1) K steps, (mult - 1) K S / (t(mult K) - t(K)), is the rate
    of a pipeline that never fills or drains.  (r03 took hand-back
    completion times inside one K-step run, which units of 4 steps complete
    in bursts -- not a rate.)"""
    from rvs_amd.schedule import PipelinedRun
    from rvs_amd.shard import timed_job
    if job.runner is None or job.unit_sizes is None:
        return {}
    K, S, Wm = job.K, job.S, job.Wm
    n = mult * K
    ts = [torch.full((S,), (Wm + k) / 30.0, dtype=torch.float64, device=job.dev) for k in range(n)]
    units = job.unit_sizes * mult
    long_run = PipelinedRun(job.eng, [job.frames[Wm + (k % K)] for k in range(n)], ts,
                            mode=job.args.exec_mode, sync=job.args.sync, units=units)
    saved = job.eng.tracker.state[0].clone()
    long_run.run()  # warm
    torch.cuda.synchronize()
    # both lengths timed twice back to back from the same SORT state, the
    # faster of each kept: the estimator is a difference of two times, so
    # one slow run of either would move it by its whole delay
    tl, ts_ = [], []
    for _ in range(2):
        for run, out in ((job.runner, ts_), (long_run, tl)):
            job.eng.tracker.state[0].copy_(saved)
            out.append(timed_job(run.run, torch.cuda.synchronize, S, job.dev)["local_s"])
    job.eng.tracker.state[0].copy_(saved)
    long_run.close()
    t = {"local_s": min(tl)}
    t1 = min(ts_)
    if t["local_s"] <= t1:
        return {}
    per = (t["local_s"] - t1) / ((mult - 1) * K)
    return {"steady_state_ms_per_step": round(per * 1e3, 4),
            "steady_state_frames_per_s": round(S / per, 1),
            "steady_state_window": f"marginal rate of a {n}-step run of the same schedule (the K "
                                   f"timed frames cycled) over the {K}-step run, both device-only "
                                   f"and the faster of two runs each: "
                                   f"({n} - {K}) steps / (t({n}) - t({K}))",
            f"device_only_{n}_steps_frames_per_s": round(n * S / t["local_s"], 1)}


def _cpu_baseline_leg(args, rank: int, world: int, cfg) -> dict:
    """The CPU baseline, on rank 0 only, after the ranks' last barrier (the
    other ranks are done with the GPU by then): at N > 1 the scaling line
    keeps its baseline too.  {} when disabled or not rank 0."""
    if rank != 0 or args.no_cpu_baseline or args.cpu_frames <= 0:
        return {}
    budget = host_cpu_budget()
    workers = args.cpu_workers or budget["cpus"]
    res = cpu_baseline(cfg, args.cpu_frames, workers)
    res.update({"cpu_quota_cpus": budget["quota_cpus"], "cores_reason": budget["reason"]})
    return {"cpu_baseline": res}


def _rank_fields(t: dict, world: int, device) -> dict:
    """Per-rank fields of the line: the process group's size and backend,
    every rank's own timed-region seconds and every rank's device identity
    (PCI bus id; rvs_amd.shard.device_identity), both in rank order.  Every
    rank must call this (the device ids are all-gathered)."""
    from rvs_amd.shard import device_identity, gather_strings
    init = torch.distributed.is_initialized()
    return {"world_size": torch.distributed.get_world_size() if init else 1,
            "process_group_backend": torch.distributed.get_backend() if init else None,
            "per_rank_local_s": [round(x, 6) for x in t["per_rank_s"]],
            "per_rank_device": gather_strings(device_identity(device)),
            "local_s": round(t["local_s"], 6), "elapsed_s": round(t["elapsed_s"], 6)}


def _stub_main(args, rank, world) -> None:
    """Rank logic with a stand-in job (CPU rehearsal with gloo)."""
    mod, cls = args.job.split(":")
    job = getattr(importlib.import_module(mod), cls)(args, rank, "cpu")
    t = rank_job(job, "cpu")
    fields = _rank_fields(t, world, "cpu")
    if rank == 0:
        res = {"metric": METRIC, "value": t["value"], "unit": "frames/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": t["elapsed_s"] / args.steps * 1e3}
        res.update(fields)
        res.update(_cpu_baseline_leg(args, rank, world, bench_config()))
        print(json.dumps(res), flush=True)


def pair1_rate(job, rank: int, dev) -> dict:
    """The config's literal batch: one YOLOv8n forward per 32-stream step
    (pipeline units of 1 step, autotuned at batch 32, the same K steps,
    synthetic frames and consumer), timed like the headline -- in a fresh
    child process (not exec'd: started as a child, its JSON line read back).
    In this process a second engine's pipeline streams would share the
    hardware queues with the first engine's (GPU_MAX_HW_QUEUES = 4): that
    leg measured 27.8-33.6k frames/s against 36.5-37.1k for the same
    configuration run alone (r04)."""
    a = job.args
    cmd = [sys.executable, os.path.abspath(__file__), "--steps", str(job.K), "--warmup", str(job.Wm),
           "--pair", "1", "--units", "even", "--no-secondary", "--no-cpu-baseline",
           "--conv-timing", "none", "--streams", str(job.S), "--gpus", "1"]
    if a.exec_mode != "native":
        cmd += ["--exec", a.exec_mode]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT", "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID")}
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"pair-1 child exited {r.returncode}: {r.stderr[-800:]}")
    d = json.loads(r.stdout.strip().splitlines()[-1])
    return {"value": d["value"], "ms_per_step": d["ms_per_step"],
            "device_only": (d.get("device_only") or {}).get("value"),
            "forward_batch": job.S,
            "note": "pipeline units of 1 step: one forward over the step's 32 frames (the "
                    "config's batch=32), conv kernels autotuned at batch 32; same K steps, "
                    "synthetic frames and consumer as the headline; a fresh child process"}


def secondary_legs(job, dev) -> dict:
    """BASELINE configs[1] and configs[4], and the host-fed rate of
    configs[2] (bench_extra.py): a few seconds each; errors are reported,
    not raised (the headline stands on its own)."""
    import bench_extra
    out = {}
    for key, fn in (("config2_b1_latency", lambda: bench_extra.config2_latency(dev)),
                    ("config5_fp8", lambda: bench_extra.config5_fp8(dev)),
                    ("hostfed_nv12", lambda: bench_extra.hostfed_nv12(job))):
        t0 = time.perf_counter()
        try:
            out[key] = fn()
        except Exception as e:  # noqa: BLE001 -- a failed leg must not hide the headline
            out[key] = {"error": f"{type(e).__name__}: {e}"}
        out[key]["leg_wall_s"] = round(time.perf_counter() - t0, 2)
        torch.cuda.synchronize()
    return out


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus, argv)
    from rvs_amd.shard import init_from_env
    rank, world, local = init_from_env("gloo" if args.job else "nccl")
    if args.job:
        _stub_main(args, rank, world)
        if world > 1:
            torch.distributed.destroy_process_group()
        return 0
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    job = BenchJob(args, rank, dev)
    t = rank_job(job, dev)
    elapsed, value = t["elapsed_s"], t["value"]
    K, S = job.K, job.S
    sort_rep = job.track_report()  # the tracks the timed region left
    cons = job.cons
    handback = {"consumer": ("in the timed region: a host thread builds every step's "
                             "List[Detection] per stream (rvs_amd.handback.Record.detections) as "
                             "soon as the step's record is handed back"
                             if job.consume == "consume" else "off"),
                "record_bytes_per_step": job.records[0].nbytes}
    handback["host_issue_ms"] = round(job.issue_s * 1e3, 3)
    if job.consume == "consume" and cons:
        handback["detections_per_step"] = round(cons["detections"] / K, 1)
        handback["materialise_ms_per_step"] = round(cons["busy_s"] / K * 1e3, 3)
        handback["consumer_done_after_device_ms"] = round((cons["end"] - job.device_end) * 1e3, 3)
    # the same K steps again without the consumer, from the same SORT state:
    # the device-only rate, and the steady state from its per-step completions
    t2 = rank_job_again(job, dev) if job.consume == "consume" else None
    sort_phase = _sort_phase_report()
    job.t_device_only = t2["local_s"] if t2 is not None else None
    steady = steady_state(job) if world == 1 else {}
    roof = conv_roofline(job, args.conv_timing) if args.conv_timing != "none" else None
    if roof and "algorithmic_gflop_per_step" in roof:
        # the conv family's FLOPs over the whole step of the timed region (every
        # other stage included): the chip-level rate the bench delivers
        tf = roof["algorithmic_gflop_per_step"] / (elapsed / K) / 1e3
        roof["chip_level"] = {"achieved": round(tf, 2), "peak": PEAK_BF16, "unit": "TFLOP/s",
                              "frac": round(tf / PEAK_BF16, 5),
                              "note": "conv-family algorithmic FLOPs per step / ms_per_step"}
    P = job.eng.pair
    execution = ("sequential step() calls (no pipelining)" if args.exec_mode == "sequential" else
                 f"{args.exec_mode} launch list (rvs_amd.schedule.PipelinedRun, sync={args.sync}):"
                 f" 4-stage software pipeline over units of {job.unit_sizes} steps -- second half of unit "
                 "u-1's forward || preprocess of unit u+1 || first half of unit u's forward || "
                 "NMS+SORT+hand-back of unit u-2 -- on 4 HIP streams, one C call per run")
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
                               "SORT+homography -> result hand-back to pinned host memory -> "
                               "List[Detection] per stream",
                   "streams_per_gpu": S, "frame": [H, W],
                   "detector_input": [job.eng.detector.in_h, job.eng.detector.in_w],
                   "parallelism": f"streams sharded {S}/GPU, no collective",
                   "forward_batch": S * P,
                   "conv_autotune": ("loaded" if args.tune_load else (not args.no_autotune)),
                   "conv_grid": args.conv_grid,
                   "execution": execution},
        "roofline": roof,
        "end_to_end_roofline_frac": round(value / world * (BYTES_PER_FRAME / (PEAK_HBM * 1e9) +
                                                           FLOP_PER_FRAME / (PEAK_BF16 * 1e12)), 5),
        "sort": sort_rep,
        "handback": handback,
    }
    res.update(_rank_fields(t, world, dev))
    if t2 is not None:
        if sort_phase is not None:
            res["sort_phase"] = sort_phase
        res["device_only"] = {"value": round(t2["value"], 2),
                              "ms_per_step": round(t2["elapsed_s"] / K * 1e3, 4),
                              "note": "the same K steps timed again without the Detection "
                                      "consumer, from the same SORT state (trace window: marker "
                                      "tags 7-8)"}
    res.update(steady)
    if world == 1 and not args.no_secondary:
        if args.exec_mode != "sequential" and P > 1:
            try:
                res["pair1"] = pair1_rate(job, rank, dev)
            except Exception as e:  # noqa: BLE001
                res["pair1"] = {"error": f"{type(e).__name__}: {e}"}
        res["secondary"] = secondary_legs(job, dev)
    if world > 1:
        torch.distributed.barrier()
    res.update(_cpu_baseline_leg(args, rank, world, job.cfg))
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
