"""YOLOv8n forward (+ decode) time per frame against the batch size at 1080p
(384 x 640 letterbox): graph-replayed forwards after autotuning each batch
size.  The small P4 / P5 layers sit near a per-launch floor at B = 32, so a
larger batch amortises it -- the case for running two consecutive steps'
forwards as one B = 64 launch sequence (the per-stream SORT order does not
depend on it)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch  # noqa: E402
from rvs_amd.detect import weights  # noqa: E402
from rvs_amd.detect.yolo_hip import YoloEngine  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    flat = weights.synthetic_weights(0)
    out = {}
    for B in [int(x) for x in os.environ.get("BS", "32,64,96").split(",")]:
        eng = YoloEngine(0, flat, B, (1080, 1920), device=dev, classes_keep=[0, 2, 3, 5, 7])
        x = (torch.rand((B, 1080, 1920, 3), device=dev) * 255).to(torch.uint8)
        lb = eng.letterbox(x)
        eng.autotune(lb, reps=10)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            eng.forward_raw(lb)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(4):
                eng.forward_raw(lb)
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 40 * 1e3
        out[B] = {"ms_per_forward": round(ms, 4), "us_per_frame": round(ms * 1e3 / B, 3)}
        eng.close()
        del x, lb
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
