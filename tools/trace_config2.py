"""Kernel trace of BASELINE configs[1] (YOLOv8n 640x640, batch 1: letterbox +
forward + NMS, the recorded launch list bench_extra.config2_latency times).
Run under rocprofv3 --kernel-trace; marker tags 11 / 12 bracket N calls.
  rocprofv3 --kernel-trace --output-format csv -d D -o t -- python tools/trace_config2.py
  python tools/trace_config2.py --report D/.../t_kernel_trace.csv"""
import csv
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]


def report(path, n):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    mk = [i for i, r in enumerate(rows) if "trace_marker" in r["Kernel_Name"]]
    a, b = mk[-2], mk[-1]
    win = rows[a + 1:b]
    t0 = int(rows[a]["End_Timestamp"])
    t1 = int(rows[b]["Start_Timestamp"])
    per = {}
    busy = 0
    last_end = None
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = r["Kernel_Name"].split("(")[0].replace("void rv::", "").split("<")[0]
        d = per.setdefault(k, [0, 0.0])
        d[0] += 1
        d[1] += (e - s) / 1e3
        busy += (e - s) / 1e3 if last_end is None or s >= last_end else max(0, e - last_end) / 1e3
        last_end = e if last_end is None else max(last_end, e)
    wall = (t1 - t0) / 1e3
    print(f"{n} calls: wall {wall / n:.1f} us per call, kernels busy {busy / n:.1f} us, "
          f"{len(win) / n:.1f} dispatches per call")
    for k, (c, us) in sorted(per.items(), key=lambda x: -x[1][1]):
        print(f"  {k:32s} {c / n:5.1f}/call {us / n:7.1f} us/call {us / c:6.2f} us avg")
    # the last call, dispatch by dispatch (duration, gap to the previous end, grid)
    per_call = len(win) // n
    prev = None
    print("last call:")
    for r in win[-per_call:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        prev = e
        k = r["Kernel_Name"].split("(")[0].replace("void rv::", "").split("<")[0]
        grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
        wg = r.get("Workgroup_Size_X", r.get("Workgroup_Size", "?"))
        print(f"  {(e - s) / 1e3:7.2f} us  gap {gap:6.2f}  grid {grid:>7} wg {wg:>5}  {k}")


def main():
    if sys.argv[1:2] == ["--report"]:
        report(sys.argv[2], int(os.environ.get("N", 20)))
        return
    import torch
    from rvs_amd import _lib
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
    for _ in range(20):
        det.run()
    torch.cuda.synchronize()
    n = int(os.environ.get("N", 20))
    _lib.call("rv_trace_marker", 11, _lib.stream_ptr())
    for _ in range(n):
        det.run()
        torch.cuda.synchronize()
    _lib.call("rv_trace_marker", 12, _lib.stream_ptr())
    torch.cuda.synchronize()
    det.close()
    eng.close()
    print("trace_config2 done")


if __name__ == "__main__":
    main()
