"""Host delivery (scroll_batch_output_to_host_async): the bytes each compose
appended to every stream, packed by the device into pinned host memory, must
equal the arena bytes (themselves checked against the oracle by the other
GPU tests) -- P-only and dynamic-rect batches, unaligned arena starts, an
append compose delivering only its new bytes, an undersized buffer writing
nothing, and a delivery on another stream.  Run on an MI355X: -m gpu."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(scroll):
    if scroll.device_count() < 1:
        pytest.fail("no gfx950 device: " + scroll.last_error())
    return scroll


def _check(hs, b, hb, prev):
    S = len(prev)
    assert b.sync() == 0, hs.last_error()
    assert hb.total() is not None, (hb.cap, [len(b.output(s)) - prev[s] for s in range(S)],
                                    [hb.table[2 + 2 * s] for s in range(S)])
    tot = 0
    for s in range(S):
        full = b.output(s)
        new = full[prev[s]:]
        assert hb.stream(s) == new, s
        assert hb.table[1 + 2 * s] % 16 == 0
        tot = max(tot, hb.table[1 + 2 * s] + ((len(new) + 15) & ~15))
        prev[s] = len(full)
    assert hb.total() == tot


def test_host_delivery_p_only(gpu):
    hs = gpu
    S, F = 24, 40
    rng = np.random.default_rng(3)
    b = hs.Batch(S, F, 1 << 20, device=0)
    for _ in range(S):
        b.add_stream(hs.make_config(1280, 720))
    hb = hs.HostBuffer(S * F * 4096, S)
    prev = [0] * S
    for it in range(3):                       # appends: arena starts at arbitrary bytes
        offs = rng.integers(0, 1400, (S, F)).astype(np.int32)
        b.set_offsets(offs)
        b.compose(F if it != 1 else 7)
        b.output_to_host_async(hb)
        _check(hs, b, hb, prev)
    hb.close()
    b.close()


def test_host_delivery_dyn(gpu):
    """the benched config-3 batch, 8 streams, two rewound composes (the
    delivery on another HIP stream is exercised by bench.py's host leg)"""
    hs = gpu
    wl = dict(bench.WORKLOADS["p720dyn"])
    wl["streams"] = 8
    b = bench.build_compose_batch(hs, wl, 0, 0)
    hb = hs.HostBuffer(8 * wl["frames"] * 200000, 8)
    for _ in range(2):
        b.compose(wl["frames"], rewind=True)
        b.output_to_host_async(hb)
        _check(hs, b, hb, [0] * 8)
    hb.close()
    b.close()


def test_host_delivery_after_sync_waits_for_the_copy(gpu):
    """compose -> sync -> deliver -> sync: the second sync must wait for the
    copy (and refresh the host mirror of undelivered); then deliver ->
    set_config -> compose -> deliver must not send the old bytes again"""
    hs = gpu
    S, F = 6, 24
    b = hs.Batch(S, F, 1 << 20, device=0)
    for _ in range(S):
        b.add_stream(hs.make_config(1280, 720))
    hb = hs.HostBuffer(S * F * 4096, S)
    prev = [0] * S
    offs = np.tile(np.arange(F, dtype=np.int32) * 11, (S, 1))
    b.set_offsets(offs)
    b.compose(F)
    assert b.sync() == 0
    for i in range(hb.cap):
        hb.data[i] = 0
    b.output_to_host_async(hb)
    _check(hs, b, hb, prev)
    # a config upload after the delivery: the host mirror must already hold
    # undelivered = 0, or the next delivery resends the bytes above
    for s in range(S):
        b.set_config(s, b.config(s))
    b.set_offsets(offs + 3)
    b.compose(F)
    b.output_to_host_async(hb)
    _check(hs, b, hb, prev)
    hb.close()
    b.close()


def test_host_delivery_of_ingested_streams(gpu, oracle):
    """an ingested stream's first delivery carries its header (SPS, PPS, A,
    B) and then the composed frames, like b.output(s)"""
    import ctypes
    hs = gpu
    S, F = 3, 10
    files = []
    for _ in range(S):
        pair = []
        for which in (0, 1):
            buf = (ctypes.c_uint8 * (320 * 240 * 3 + 4096))()
            n = oracle.or_ipcm_ref_file(buf, len(buf), 320, 240, which)
            pair.append(bytes(buf[:n]))
        files.append(tuple(pair))
    b = hs.Batch(S, F, 1 << 20, device=0)
    assert b.ingest(files) == 0
    hb = hs.HostBuffer(S * (1 << 19), S)
    prev = [0] * S
    b.output_to_host_async(hb)
    _check(hs, b, hb, prev)
    assert all(p > 200000 for p in prev)          # the I_PCM header went out
    b.set_offsets(np.tile(np.arange(F, dtype=np.int32) * 8, (S, 1)))
    b.compose(F)
    b.output_to_host_async(hb)
    _check(hs, b, hb, prev)
    hb.close()
    b.close()


def test_host_delivery_too_small_writes_nothing(gpu):
    hs = gpu
    S, F = 4, 20
    b = hs.Batch(S, F, 1 << 20, device=0)
    for _ in range(S):
        b.add_stream(hs.make_config(1280, 720))
    b.set_offsets(np.tile(np.arange(F, dtype=np.int32) * 9, (S, 1)))
    b.compose(F)
    hb = hs.HostBuffer(4096, S)
    for i in range(hb.cap):
        hb.data[i] = 0xA5
    b.output_to_host_async(hb)
    assert b.sync() == 0
    assert hb.total() is None
    assert all(hb.data[i] == 0xA5 for i in range(hb.cap))
    hb.close()
    b.close()
