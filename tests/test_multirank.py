"""world_size-2 gloo test of the sharded bench path (CPU, no GPU).

Each rank takes its static shard of the synthetic streams (bench.shard_streams),
composes them with the CPU oracle (the checker) and all-gathers digests; the
union must equal the single-process composition of all streams, with no stream
composed twice, and bench.max_over_ranks must return the slowest rank's time.
"""
import ctypes
import hashlib
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

W, H, PER_GPU, F = 64, 48, 3, 40


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _compose_digests(oracle_so, first, count):
    import bench
    lib = ctypes.CDLL(oracle_so)

    class OrCfg(ctypes.Structure):
        _fields_ = [(n, ctypes.c_int) for n in
                    ("w", "h", "log2_mfn", "poc_type", "log2_poc", "num_ref_default_m1",
                     "deblock", "frame_num", "idr_pic_id", "nwp")] + [
            ("wp_off", ctypes.c_int * 8), ("wp_lt", ctypes.c_int * 8), ("wp_valid", ctypes.c_int * 8)]

    offs = bench.synthetic_offsets(first, count, F, H)
    buf = (ctypes.c_uint8 * (1 << 16))()
    out = {}
    for k in range(count):
        cfg = OrCfg()
        lib.or_cfg_init(ctypes.byref(cfg), W, H)
        cfg.frame_num = 2
        h = hashlib.sha256()
        for off in offs[k]:
            n = lib.or_compose(buf, len(buf), ctypes.byref(cfg), int(off), 0, None)
            h.update(bytes(buf[:n]))
        out[first + k] = h.hexdigest()
    return out


def _rank(rank, world, port, oracle_so, q):
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = bench.shard_streams(rank, world, PER_GPU)
    dig = _compose_digests(oracle_so, first, count)
    got = [None] * world
    dist.all_gather_object(got, dig)
    slowest = bench.max_over_ranks(0.5 + rank, dist)
    dist.destroy_process_group()
    if rank == 0:
        q.put((got, slowest))


@pytest.mark.timeout(300)
def test_two_rank_static_shard(oracle):
    oracle_so = oracle._name
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, oracle_so, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, slowest = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    merged = {}
    for d in got:
        assert not (set(d) & set(merged)), "a stream was composed by two ranks"
        merged.update(d)
    assert sorted(merged) == list(range(world * PER_GPU))
    assert merged == _compose_digests(oracle_so, 0, world * PER_GPU)
    assert slowest == 1.5
