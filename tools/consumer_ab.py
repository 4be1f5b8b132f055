"""Is the consumer-vs-device-only gap of bench.py the consumer, or the order
of the runs?  Builds bench.py's job once (same args), then times the K-step
region alternately with the Detection consumer ("consume") and with the
watcher only ("watch"), every run from the same SORT state, and prints each
run's frames/s in order.
usage: python tools/consumer_ab.py [ROUNDS] [bench.py args ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

import bench  # noqa: E402
from rvs_amd.shard import timed_job  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    args = bench.parse_args(["--steps", "20", "--no-secondary", "--no-cpu-baseline"] + sys.argv[2:])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    job = bench.BenchJob(args, 0, dev)
    job.warmup()
    job.prepare()
    # PRELUDE=consume / watch: one more untimed run in that mode right before
    # the first timed one (allocator / device warm-up hypotheses)
    prelude = os.environ.get("PRELUDE", "none")
    if prelude != "none":
        job.consume = prelude
        job.run()
        job.sync()
        job.eng.tracker.state[0].copy_(job.sort_saved)
    out = []
    for r in range(rounds):
        for mode in (("consume", "watch") if r % 2 == 0 else ("watch", "consume")):
            job.consume = mode
            job.eng.tracker.state[0].copy_(job.sort_saved)
            t = timed_job(job.run, job.sync, job.units, dev)
            out.append((mode, round(t["value"], 1)))
            print(mode, round(t["value"], 1), flush=True)
    res = {m: [v for mm, v in out if mm == m] for m in ("consume", "watch")}
    print(json.dumps({"prelude": prelude, "order": out, **res}))


if __name__ == "__main__":
    main()
