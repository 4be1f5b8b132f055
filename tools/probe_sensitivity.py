"""Critical-path sensitivity of the pipelined bench step: the timed region
(OverlappedSteps depth 4, 8 steps per graph, autotuned convs) re-captured with
one stage made (nearly) free at a time -- P = the fused CLAHE + median +
letterbox (replaced by the letterbox alone), T = NMS + SORT + hand-back
(NMS alone), Y1 / Y2 = the two halves of the forward (skipped).  The step
time with a stage removed bounds what speeding that stage up can buy.
Timing only: results of the modified steps are meaningless."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def timed(job, K):
    from rvs_amd.engine import OverlappedSteps
    eng = job.eng
    r = OverlappedSteps(eng, [job.frames[job.Wm + k] for k in range(K)],
                        [job.ts[job.Wm + k] for k in range(K)], depth=4, chunk=8)
    torch.cuda.synchronize()
    r.run()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        r.run()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    del r
    return best / K * 1e3


def main():
    args = bench.parse_args(["--steps", os.environ.get("K", "60")])
    dev = torch.device("cuda:0")
    job = bench.BenchJob(args, 0, dev)
    job.warmup()
    eng = job.eng
    eng.autotune(job.frames[0], reps=10)
    torch.cuda.synchronize()
    K = job.K
    orig_p, orig_y, orig_t = eng.preprocess_stage, eng.yolo_stage, eng.track_stage

    def p_letterbox(frames, lb_slot=0, lb_off=0):
        lb = eng.detector.letterbox(frames, lb_slot, lb_off)
        return frames, lb

    def y_skip(skip):
        def f(lb, slot=0, lane=0, part=0):
            if part != skip:
                orig_y(lb, slot, lane, part=part)
        return f

    def t_nms(ts, slot=0, record=None):
        dets, det_n = eng.detector.nms(ts.shape[0], slot)
        return {"dets": dets, "det_n": det_n, "record": record}

    def t_nms_pair(ts_list, slot, records):
        eng.detector.nms(eng.S * len(ts_list), slot)
        return [{"record": r} for r in records]
    orig_tp = eng.track_pair_stage

    out = {}
    out["base"] = timed(job, K)
    eng.preprocess_stage = p_letterbox
    out["P_letterbox_only"] = timed(job, K)
    eng.preprocess_stage = orig_p
    eng.track_stage, eng.track_pair_stage = t_nms, t_nms_pair
    out["T_nms_only"] = timed(job, K)
    eng.track_stage, eng.track_pair_stage = orig_t, orig_tp
    eng.yolo_stage = y_skip(2)
    out["no_Y2"] = timed(job, K)
    eng.yolo_stage = y_skip(1)
    out["no_Y1"] = timed(job, K)
    eng.yolo_stage = orig_y
    out["base_again"] = timed(job, K)
    print(json.dumps({k: round(v, 4) for k, v in out.items()} |
                     {"unit": "ms per 32-frame step", "pair": eng.pair}))


if __name__ == "__main__":
    main()
