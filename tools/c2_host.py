"""Config-2 (YOLOv8n 640x640 b=1) call anatomy: host submission time of one
native launch-list call (rv_sched) against the call's end-to-end latency and
its device span (HIP events around it), per variant (env RV_*)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    from rvs_amd.schedule import Schedule
    from rvs_amd.synth import road_frames
    dev = torch.device("cuda:0")
    frame = road_frames(1, 1, 640, 640, device=dev)[0].contiguous()
    eng = YoloEngine(0, weights.synthetic_weights(0, seed=0), 1, (640, 640), imgsz=640, device=dev,
                     classes_keep=[0, 2, 3, 5, 7])
    eng.autotune(eng.letterbox(frame), reps=5)
    det = Schedule()
    with det.recording():
        eng.run(frame)
    for _ in range(30):
        det.run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    sub, tot, span = [], [], []
    for _ in range(int(os.environ.get("ITERS", 300))):
        t0 = time.perf_counter()
        e0.record()
        det.run()
        t1 = time.perf_counter()
        e1.record()
        e1.synchronize()
        t2 = time.perf_counter()
        sub.append(t1 - t0)
        tot.append(t2 - t0)
        span.append(e0.elapsed_time(e1) * 1e-3)
    med = lambda a: float(np.median(a)) * 1e6  # noqa: E731
    print(f"{os.environ.get('NAME', 'base')}: launches {det.num_nodes()} "
          f"submit {med(sub):.1f} us, device span {med(span):.1f} us, call {med(tot):.1f} us")
    det.close()
    eng.close()


if __name__ == "__main__":
    main()
