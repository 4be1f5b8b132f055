"""Eager bench work (autotuned convs, 32 streams x 1080p, full chain) for
rocprofv3 --pmc passes: one warm-up step, then one pipeline unit as the timed
region runs it (PAIR = 4 steps: four preprocess passes, ONE forward over their
128 frames, NMS, four SORT + hand-back) -- every dispatch is one row per
counter in counter_collection.csv (tools/pmc_report.py summarises the window
from the last LUT pass; tools/pmc_traffic.py divides the unit's conv bytes
by PAIR)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from rvs_amd.engine import RoadVisionEngine  # noqa: E402
from rvs_amd.synth import road_frames  # noqa: E402

S = int(os.environ.get("S", 32))
P = int(os.environ.get("PAIR", 4))
dev = torch.device("cuda:0")
eng = RoadVisionEngine(bench.bench_config(), S, (1080, 1920), device=dev, pair=P)
frames = road_frames(S, 1 + P, 1080, 1920, device=dev)
ts = torch.tensor([[f / 30.0] * S for f in range(1 + P)], dtype=torch.float64, device=dev)
eng.step(frames[0], ts[0])
if os.environ.get("TUNE"):  # the configurations a bench run saved (--tune-save)
    import json
    eng.detector.load_tuned([tuple(c) for c in json.load(open(os.environ["TUNE"]))["configs"]])
else:  # the bench's kernel configurations (at the unit's batch, persistent grids)
    eng.autotune(frames[0])
    eng.detector.load_tuned([tuple(c[:4]) + (1,) + tuple(c[5:])
                             for c in eng.detector.tuned_configs()])
if P > 1:
    from rvs_amd.handback import Record
    recs = [Record(S, eng.detector.max_det, dev) for _ in range(P)]
    eng.step_unit([frames[1 + h] for h in range(P)], [ts[1 + h] for h in range(P)], recs)
else:
    eng.step(frames[1], ts[1])
torch.cuda.synchronize()
print("pmc_step done")
