"""GPU parity at the benchmarked scale: the exact batches bench.py times
(bench.build_compose_batch), composed several times with rewound arenas as
the bench does, and EVERY byte of the last step of every stream compared
with the CPU oracle (tests/stepcheck.py -> oracle/verify_oracle.c on the
host's cores).  These launches run the full grids the bench runs -- config
3's 102,400 k_dyn_row workgroups with the epoch-tagged TotalCoeff hand-off
between rect rows at full residency, the XCD frame rotation, the EP fix-up
and the gather -- which the small tests of test_gpu_dyn.py do not reach.
Dynamic-rect bits: oracle/dyn_oracle.c (parity unpinned);
P-only bits: pinned to the reference.  Run on an MI355X:
-m gpu."""
import os
import sys

import pytest

import stepcheck

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(scroll):
    if scroll.device_count() < 1:
        pytest.fail("no gfx950 device: " + scroll.last_error())
    return scroll


def _run(gpu, workload, passes, first=0, streams=None):
    wl = dict(bench.WORKLOADS[workload])
    if streams:
        wl["streams"] = streams
    b = bench.build_compose_batch(gpu, wl, first, 0)
    for _ in range(passes):
        b.compose(wl["frames"], rewind=True)
    assert b.sync() == 0, gpu.last_error()
    ok, d = bench.verify_last_step(b, wl, first, passes)
    b.close()
    assert ok, d
    return d


def test_config3_full_step(gpu):
    """BASELINE config 3 as benched: 256 streams x 16 frames of 1280x720 +
    the 360x360 rect, per-stream reference copies, device source generator;
    3 composes (state carried, arenas rewound) -- all 4,096 NALs of the last"""
    d = _run(gpu, "p720dyn", 3)
    assert d["streams"] == 256 and d["bytes"] > 200e6


def test_config4_shard(gpu):
    """BASELINE config 4, the last GPU's shard: streams 7,168 .. 8,191 (1,024
    per GPU) x 16 frames, source generator on the global stream ids"""
    d = _run(gpu, "p720dyn", 2, first=7 * 1024, streams=1024)
    assert d["streams"] == 1024


def test_config5_shard(gpu):
    """BASELINE config 5, the second GPU's shard: streams 128 .. 255 of
    3840x2160 with the 720x720 rect, scroll through 496 / 992 / 1488 / 1984
    (up to 6 references)"""
    d = _run(gpu, "p4kdyn", 2, first=128)
    assert d["streams"] == 128


def test_config2_full_step(gpu):
    """BASELINE config 2 as benched: 256 streams x 1024 P-only frames"""
    d = _run(gpu, "p720", 2)
    assert d["streams"] == 256


def test_hint_workload_step(gpu):
    """the UI-hint bench workload (P_Skip mode), every stream checked"""
    _run(gpu, "p720hint", 3)
