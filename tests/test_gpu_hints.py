"""GPU parity of the UI-hint P slices:
k_plan (state) -> k_hint_stage -> k_plan (size) -> k_emit -> k_dyn_emit_gather,
through the C ABI, against the CPU restatement oracle/hint_oracle.c
(or_compose_hint) byte for byte.  Frames without hints, in the EXACT mode,
must equal the reference's scroll frames (or_compose, pinned by the
reference's golden vectors); tests/test_hint_oracle.py pins the hinted
layouts by decoding their MV fields from the standard.  Run on an MI355X:
-m gpu."""
import ctypes
import random

import numpy as np
import pytest

from conftest import synthetic_offsets
from dynhelp import OrCfg, hint_array, random_hints, split_nals

pytestmark = pytest.mark.gpu

EXACT, PSKIP, SPEC = 0, 1, 2


@pytest.fixture(scope="module")
def gpu(scroll):
    if scroll.device_count() < 1:
        pytest.fail("no gfx950 device: " + scroll.last_error())
    return scroll


def _cfg(oracle, w, h, waypoints=()):
    c = OrCfg()
    oracle.or_cfg_init(ctypes.byref(c), w, h)
    c.frame_num = 2
    for i, (o, lt, v) in enumerate(waypoints):
        c.wp_off[i], c.wp_lt[i], c.wp_valid[i] = o, lt, v
    c.nwp = len(waypoints)
    return c


def plan_hints(oracle, w, h, offsets, seed, modes=(EXACT, PSKIP, SPEC), p=0.8, waypoints=(),
               compose_mode=0, nmax=6):
    """random hints per (stream, frame) whose refs are valid in that frame,
    and the oracle's streams for them: -> (hints dict, [bytes per stream])"""
    rng = random.Random(seed)
    S, F = offsets.shape
    buf = (ctypes.c_uint8 * (8 << 20))()
    err = ctypes.c_int()
    hints, outs = {}, []
    for s in range(S):
        c = _cfg(oracle, w, h, waypoints)
        o = bytearray()
        for t in range(F):
            refs = [0, 1] + [2 + i for i in range(c.nwp) if c.wp_valid[i]]
            rects = random_hints(rng, w // 16, h // 16, refs, nmax) if rng.random() < p else []
            hm = rng.choice(modes)
            hints[(s, t)] = (rects, hm)
            arr, n = hint_array(rects)
            k = oracle.or_compose_hint(buf, len(buf), ctypes.byref(c), int(offsets[s, t]),
                                       compose_mode, arr, n, hm, ctypes.byref(err))
            assert err.value == 0 and k > 0
            o += bytes(buf[:k])
        outs.append(bytes(o))
    return hints, outs


def oracle_plain(oracle, w, h, offsets, compose_mode=0, waypoints=()):
    S, F = offsets.shape
    buf = (ctypes.c_uint8 * (8 << 20))()
    outs = []
    for s in range(S):
        c = _cfg(oracle, w, h, waypoints)
        o = bytearray()
        for t in range(F):
            k = oracle.or_compose(buf, len(buf), ctypes.byref(c), int(offsets[s, t]), compose_mode,
                                  None)
            o += bytes(buf[:k])
        outs.append(bytes(o))
    return outs


def gpu_hint_streams(gpu, w, h, offsets, hints, compose_mode=0, waypoints=(), arena=8 << 20):
    S, F = offsets.shape
    b = gpu.Batch(S, F, arena, mode=compose_mode)
    for _ in range(S):
        b.add_stream(gpu.make_config(w, h, waypoints=waypoints))
    for (s, f), (rects, hm) in hints.items():
        b.set_hints(s, f, rects, hm)
    b.set_offsets(offsets)
    b.compose(F)
    return b, b.sync()


def check_equal(b, want, streams=None):
    for s in (streams if streams is not None else range(len(want))):
        got, ws = b.output(s), want[s]
        if got != ws:
            gn, wn = split_nals(got), split_nals(ws)
            bad = next((i for i, (x, y) in enumerate(zip(gn, wn)) if x != y), min(len(gn), len(wn)))
            raise AssertionError(f"stream {s}: {len(got)} vs {len(ws)} bytes, {len(gn)} vs "
                                 f"{len(wn)} NALs, first differing NAL {bad}")


def test_hints_without_rects_equal_the_reference(gpu, oracle):
    """hinted pipeline, no rects, EXACT: the reference's scroll frames"""
    w, h = 1280, 720
    offs = synthetic_offsets(8, 40, h)
    offs[0] = np.arange(470, 510)                      # through the 496 waypoint
    want = oracle_plain(oracle, w, h, offs)
    b, rc = gpu_hint_streams(gpu, w, h, offs, {(0, 0): ([], EXACT)})
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


@pytest.mark.parametrize("w,h,seed", [(256, 720, 1), (640, 480, 2), (1280, 720, 3)])
def test_random_hints_both_modes(gpu, oracle, w, h, seed):
    offs = synthetic_offsets(6, 24, h, first_stream=seed)
    offs[1] = np.clip(np.arange(480, 504), 0, h)       # waypoints: refs 2 + i appear
    hints, want = plan_hints(oracle, w, h, offs, seed)
    b, rc = gpu_hint_streams(gpu, w, h, offs, hints)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


def test_hints_4k_many_rects(gpu, oracle):
    """3840x2160, up to SCROLL_HINT_MAX_RECTS rects, waypoint refs, both modes"""
    w, h = 3840, 2160
    offs = np.array([[490, 496, 500, 992, 1000, 1488], [1984, 1990, 2000, 1500, 700, 20]],
                    np.int32)
    hints, _ = plan_hints(oracle, w, h, offs, 7, nmax=64)
    hints[(0, 3)] = ([(k % 240, k // 240, k % 240 + 3, k // 240 + 70, k % 2, k - 32, -k)
                      for k in range(64)], PSKIP)
    _, want = _replan(oracle, w, h, offs, hints)
    b, rc = gpu_hint_streams(gpu, w, h, offs, hints, arena=32 << 20)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


def _replan(oracle, w, h, offs, hints, compose_mode=0):
    S, F = offs.shape
    buf = (ctypes.c_uint8 * (8 << 20))()
    err = ctypes.c_int()
    outs = []
    for s in range(S):
        c = _cfg(oracle, w, h)
        o = bytearray()
        for t in range(F):
            rects, hm = hints.get((s, t), ([], EXACT))
            arr, n = hint_array(rects)
            k = oracle.or_compose_hint(buf, len(buf), ctypes.byref(c), int(offs[s, t]),
                                       compose_mode, arr, n, hm, ctypes.byref(err))
            assert err.value == 0
            o += bytes(buf[:k])
        outs.append(bytes(o))
    return hints, outs


def test_static_frame_is_all_skips(gpu, oracle):
    w, h = 1280, 720
    offs = np.array([[100, 200, 300]], np.int32)
    hints = {(0, f): ([(0, 0, 80, 45, 0, 0, 0)], PSKIP) for f in range(3)}
    _, want = _replan(oracle, w, h, offs, hints)
    b, rc = gpu_hint_streams(gpu, w, h, offs, hints)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    assert b.output_size(0) < 3 * 30
    b.close()


def test_experiment_mode(gpu, oracle):
    """waypoint NAL instead of the scroll NAL: those frames stage nothing"""
    w, h = 640, 480
    offs = synthetic_offsets(4, 30, h, first_stream=5)
    offs[2] = np.arange(480, 510)
    hints, want = plan_hints(oracle, w, h, offs, 9, compose_mode=1)
    b, rc = gpu_hint_streams(gpu, w, h, offs, hints, compose_mode=1)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


def test_invalid_reference_fails_only_its_stream(gpu, oracle, scroll):
    w, h = 256, 256
    offs = synthetic_offsets(3, 8, h)
    hints = {(1, 2): ([(0, 0, 4, 4, 3, 0, 0)], EXACT)}      # waypoint 1: never valid here
    _, want = _replan(oracle, w, h, offs, {})
    b, rc = gpu_hint_streams(gpu, w, h, offs, hints)
    assert rc == scroll.SCROLL_ERR_CONFIG, rc
    assert "hint" in gpu.last_error()
    assert b.output_size(1) == 0                             # nothing committed
    check_equal(b, want, streams=[0, 2])
    b.close()


def test_chunks_clear_and_exclusivity(gpu, oracle, scroll):
    """hints persist across composes (frame f of each compose); clearing them
    returns to the k_emit path"""
    w, h = 512, 512
    offs = synthetic_offsets(3, 30, h, first_stream=2)
    F1 = 10
    rng = random.Random(5)
    per_f = {f: (random_hints(rng, w // 16, h // 16, [0, 1], 4), PSKIP) for f in range(F1)}
    hints = {(s, t): per_f[t % F1] for s in range(3) for t in range(20)}
    _, want = _replan(oracle, w, h, offs, hints)
    b = gpu.Batch(3, F1, 8 << 20)
    for _ in range(3):
        b.add_stream(gpu.make_config(w, h))
    for s in range(3):
        for f in range(F1):
            b.set_hints(s, f, *per_f[f])
    for c0 in (0, 10):
        b.set_offsets(np.ascontiguousarray(offs[:, c0:c0 + F1]))
        b.compose(F1)
        assert b.sync() == 0, gpu.last_error()
    b.clear_hints()
    b.set_offsets(np.ascontiguousarray(offs[:, 20:30]))
    b.compose(F1)
    assert b.sync() == 0, gpu.last_error()
    for s in range(3):                 # frames 20.. carry no hints: plain scroll frames
        assert b.output(s) == want[s], s
    b.close()
