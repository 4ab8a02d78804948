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


def _gpu_rank(rank, world, port, q):
    """one rank of the sharded GPU path: its shard composed by libh264scroll
    (every rank on device 0 when only one GPU is visible), checked against
    the oracle, digests all-gathered"""
    import torch.distributed as dist
    import bench
    import h264scroll as hs
    sys.path.insert(0, HERE)
    import stepcheck
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wl = dict(bench.WORKLOADS["p720dyn"], streams=8, frames=4)
    first, count = bench.shard_streams(rank, world, wl["streams"])
    dev = rank % max(1, hs.device_count())
    b = bench.build_compose_batch(hs, wl, first, dev)
    b.compose(wl["frames"], rewind=True)
    rc = b.sync()
    ok, d = bench.verify_last_step(b, wl, first, 1) if rc == 0 else (False, hs.last_error())
    dig = {first + s: hashlib.sha256(b.output(s)).hexdigest() for s in range(count)}
    b.close()
    got = [None] * world
    dist.all_gather_object(got, (ok, d, dig))
    dist.destroy_process_group()
    if rank == 0:
        q.put(got)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_rank_gpu_shards_through_the_library():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_gpu_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    merged = {}
    for ok, d, dig in got:
        assert ok, d
        assert not (set(dig) & set(merged))
        merged.update(dig)
    assert sorted(merged) == list(range(16))


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_gpus_2_launches_two_ranks():
    """python bench.py --gpus 2 with no launcher starts two ranks itself and
    prints one line with n_gpus 2 and the verified last step"""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--streams", "16", "--no-cpu"], capture_output=True, text=True,
                       timeout=240, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = lines[0]
    assert out["n_gpus"] == 2 and out["verified"] is True, out
    assert out["verify"]["streams"] == 16
