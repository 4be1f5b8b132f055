"""Multi-GPU sharding rehearsed on the CPU with gloo,
world_size 2: each rank owns a disjoint block of camera streams, generates
exactly the frames a single process would for those streams, runs the
per-stream chain (oracle preprocess + SORT) with no data exchange, and the
timed region is reduced with a max over ranks.  The ranks run bench.py's
own rank logic -- rvs_amd.shard.init_from_env + bench.rank_job (warm-up,
prepare, shard.timed_job: barrier, sync, run, sync, barrier, MAX over
ranks, whole-job rate) -- with a CPU stub job in place of the GPU engine
and real perf_counter timing, so the code torchrun runs on the GPUs (with
the nccl = RCCL backend) is the code under test here."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _CpuJob:
    """bench.BenchJob's interface (constructor (args, rank, device); warmup /
    prepare / run / sync / units) over the oracle chain of this rank's
    streams: args.streams streams, args.steps frames each.  With RV_STUB_OUT
    set, a rank writes its per-stream results to RV_STUB_OUT/rank<r>.json."""

    def __init__(self, args, rank, dev="cpu"):
        from rvs_amd.shard import rank_streams
        from rvs_amd.synth import road_frames
        S, F = args.streams, args.steps
        self.rank = rank
        self.ids = rank_streams(S, rank)
        self.fr = road_frames(S, F, 48, 64, device="cpu", stream_offset=self.ids.start).numpy()
        self.S, self.F = S, F
        self.units = S * F
        self.out = {}
        self.calls = []

    def warmup(self):
        self.calls.append("warmup")

    def prepare(self):
        self.calls.append("prepare")

    def run(self):
        from oracle import cpu, sort_ref
        from rvs_amd.config import load_config
        self.calls.append("run")
        cfg = load_config()["tracking"]
        for j, sid in enumerate(self.ids):
            trk = sort_ref.SortTracker(cfg)
            rng = np.random.default_rng(sid)
            base = rng.uniform(0, 40, (3, 2))
            tracks = []
            for f in range(self.F):
                proc = cpu.median(cpu.clahe_ycrcb(self.fr[f, j]), 3)
                dets = [sort_ref.Det(x + 2 * f, y, x + 2 * f + 8, y + 8, 0.9, 2) for x, y in base]
                trk.update(dets, f / 30.0)
                tracks.append(([d.track_id for d in dets], int(proc.sum())))
            self.out[sid] = tracks
        if os.environ.get("RV_STUB_OUT"):
            import json
            with open(os.path.join(os.environ["RV_STUB_OUT"], f"rank{self.rank}.json"), "w") as f:
                json.dump({str(k): v for k, v in self.out.items()}, f)

    def sync(self):
        self.calls.append("sync")


def _worker(rank, world, port, S, F, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here),
                                                          "road-vision-system_amd"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank), OMP_NUM_THREADS="2")
    import torch.distributed as dist
    import bench
    from rvs_amd.shard import init_from_env
    r, w, _ = init_from_env("gloo")
    assert (r, w) == (rank, world) and dist.is_initialized()
    import argparse
    job = _CpuJob(argparse.Namespace(streams=S, steps=F), rank)
    t = bench.rank_job(job, "cpu")
    q.put((rank, list(job.ids), job.out, t, job.calls))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_matches_single_process():
    from rvs_amd.shard import partition
    S, F, world = 2, 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, S, F, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    # disjoint, covering stream blocks, as partition() lays them out
    assert [r[1] for r in res] == [list(x) for x in partition(S * world, world)]
    # bench.rank_job's order of operations on every rank
    assert all(r[4] == ["warmup", "prepare", "sync", "run", "sync"] for r in res)
    # the reported time is the MAX of the ranks' measured times, and the
    # whole-job rate is every rank's frames over it
    mx = max(r[3]["local_s"] for r in res)
    assert all(r[3]["local_s"] > 0 for r in res)
    assert all(r[3]["elapsed_s"] == mx for r in res)
    assert all(r[3]["per_rank_s"] == [x[3]["local_s"] for x in res] for r in res)
    assert all(abs(r[3]["value"] - S * F * world / mx) < 1e-9 * r[3]["value"] for r in res)
    # each rank's per-stream results equal a single process running all streams
    import sys
    merged = {}
    for r in res:
        merged.update(r[2])
    _check_single_process(merged, S * world, F)
    assert sys.modules.get("torch.distributed") is not None


def _check_single_process(merged, n_streams, F):
    from oracle import cpu, sort_ref
    from rvs_amd.config import load_config
    from rvs_amd.synth import road_frames
    fr = road_frames(n_streams, F, 48, 64, device="cpu").numpy()
    cfg = load_config()["tracking"]
    for sid in range(n_streams):
        trk = sort_ref.SortTracker(cfg)
        rng = np.random.default_rng(sid)
        base = rng.uniform(0, 40, (3, 2))
        for f in range(F):
            proc = cpu.median(cpu.clahe_ycrcb(fr[f, sid]), 3)
            dets = [sort_ref.Det(x + 2 * f, y, x + 2 * f + 8, y + 8, 0.9, 2) for x, y in base]
            trk.update(dets, f / 30.0)
            assert merged[sid][f] == ([d.track_id for d in dets], int(proc.sum()))


def test_bench_gpus_flag_spawns_the_ranks(tmp_path, capfd, monkeypatch):
    """`bench.py --gpus 2` without torchrun's environment starts the 2 ranks
    itself (fresh child processes with RANK / WORLD_SIZE / MASTER_*), each
    joins the process group (gloo here, RCCL on the GPUs) and runs its own
    stream block; rank 0 prints ONE JSON line with n_gpus = world_size = 2
    and the whole-job rate over the slowest rank."""
    import json
    import bench
    here = os.path.dirname(os.path.abspath(__file__))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("PYTHONPATH", here + os.pathsep + os.environ.get("PYTHONPATH", ""))
    monkeypatch.setenv("RV_STUB_OUT", str(tmp_path))
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    S, F = 2, 3
    rc = bench.main(["--gpus", "2", "--streams", str(S), "--steps", str(F), "--warmup", "0",
                     "--cpu-frames", "1", "--cpu-workers", "1",
                     "--job", "test_shard_gloo:_CpuJob"])
    assert rc == 0
    lines = [ln for ln in capfd.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["steps"] == F
    assert abs(d["value"] - S * F * 2 / d["elapsed_s"]) < 1e-4 * d["value"]  # elapsed_s rounded to 1 us
    assert d["elapsed_s"] >= d["local_s"] > 0
    # every rank's own timed-region time, and the reported time is their max
    assert len(d["per_rank_local_s"]) == 2 and all(x > 0 for x in d["per_rank_local_s"])
    assert abs(max(d["per_rank_local_s"]) - d["elapsed_s"]) < 1e-5
    # one device identity per rank, all distinct (on the GPU: PCI bus ids),
    # and the process group's backend
    assert len(d["per_rank_device"]) == 2 and len(set(d["per_rank_device"])) == 2
    assert d["process_group_backend"] == "gloo" and d["world_size"] == 2
    # the CPU baseline rides in the N > 1 line too (rank 0, after the barrier)
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["value"] > 0
    merged = {}
    for r in range(2):
        merged.update({int(k): [(a, b) for a, b in v] for k, v in
                       json.load(open(tmp_path / f"rank{r}.json")).items()})
    assert sorted(merged) == list(range(S * 2))
    _check_single_process(merged, S * 2, F)


def test_partition_rejects_uneven_split():
    from rvs_amd.shard import partition, rank_streams
    assert [len(r) for r in partition(256, 8)] == [32] * 8
    assert rank_streams(32, 3) == range(96, 128)
    with pytest.raises(ValueError):
        partition(10, 4)


def test_pick_pair_divides_the_step_count():
    """bench.py's pipeline unit: the largest pair <= --pair dividing --steps,
    so any driver step count runs (pair mode needs whole units)."""
    import bench
    assert bench.pick_pair(60, 4) == 4 and bench.pick_pair(20, 4) == 4
    assert bench.pick_pair(10, 4) == 2 and bench.pick_pair(9, 4) == 3
    assert bench.pick_pair(7, 4) == 1 and bench.pick_pair(5, 1) == 1 and bench.pick_pair(3, 0) == 1
    assert bench.parse_args([]).pair == 4
