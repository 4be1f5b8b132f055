"""Multi-GPU sharding rehearsed on the CPU with gloo,
world_size 2: each rank owns a disjoint block of camera streams, generates
exactly the frames a single process would for those streams, runs the
per-stream chain (oracle preprocess + SORT) with no data exchange, and the
timed region is reduced with a max over ranks.  The GPU bench uses the same
functions (bench.py -> rvs_amd.shard) with the nccl (RCCL) backend."""
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


def _worker(rank, world, port, S, F, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here),
                                                          "road-vision-system_amd"), here]
    import torch.distributed as dist
    from oracle import cpu, sort_ref
    from rvs_amd.config import load_config
    from rvs_amd.shard import job_throughput, max_over_ranks, rank_streams
    from rvs_amd.synth import road_frames
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = rank_streams(S, rank)
    fr = road_frames(S, F, 48, 64, device="cpu", stream_offset=ids.start).numpy()
    cfg = load_config()["tracking"]
    out = {}
    for j, sid in enumerate(ids):
        trk = sort_ref.SortTracker(cfg)
        rng = np.random.default_rng(sid)
        base = rng.uniform(0, 40, (3, 2))
        tracks = []
        for f in range(F):
            proc = cpu.median(cpu.clahe_ycrcb(fr[f, j]), 3)
            dets = [sort_ref.Det(x + 2 * f, y, x + 2 * f + 8, y + 8, 0.9, 2) for x, y in base]
            trk.update(dets, f / 30.0)
            tracks.append(([d.track_id for d in dets], int(proc.sum())))
        out[sid] = tracks
    elapsed = 0.1 * (rank + 1)
    mx = max_over_ranks(elapsed)
    q.put((rank, list(ids), out, mx, job_throughput(S * F, world, mx)))
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
    res.sort()
    # disjoint, covering stream blocks, as partition() lays them out
    assert [r[1] for r in res] == [list(x) for x in partition(S * world, world)]
    # max over ranks and whole-job throughput
    assert all(abs(r[3] - 0.2) < 1e-12 for r in res)
    assert all(abs(r[4] - S * F * world / 0.2) < 1e-6 for r in res)
    # each rank's per-stream results equal a single process running all streams
    import sys
    from oracle import cpu, sort_ref
    from rvs_amd.config import load_config
    from rvs_amd.synth import road_frames
    fr = road_frames(S * world, F, 48, 64, device="cpu").numpy()
    cfg = load_config()["tracking"]
    merged = {}
    for r in res:
        merged.update(r[2])
    for sid in range(S * world):
        trk = sort_ref.SortTracker(cfg)
        rng = np.random.default_rng(sid)
        base = rng.uniform(0, 40, (3, 2))
        for f in range(F):
            proc = cpu.median(cpu.clahe_ycrcb(fr[f, sid]), 3)
            dets = [sort_ref.Det(x + 2 * f, y, x + 2 * f + 8, y + 8, 0.9, 2) for x, y in base]
            trk.update(dets, f / 30.0)
            assert merged[sid][f] == ([d.track_id for d in dets], int(proc.sum()))
    assert sys.modules.get("torch.distributed") is not None


def test_partition_rejects_uneven_split():
    from rvs_amd.shard import partition, rank_streams
    assert [len(r) for r in partition(256, 8)] == [32] * 8
    assert rank_streams(32, 3) == range(96, 128)
    with pytest.raises(ValueError):
        partition(10, 4)
