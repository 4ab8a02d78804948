"""GPU parity of the dynamic rect under UI hints (SURVEY §8f row 1 x BASELINE
configs 3-5): k_plan (state) -> k_hdyn_code -> k_hint_stage / k_splice_stage
-> k_plan (size) -> k_emit -> k_dyn_emit_gather, through the C ABI, against
the CPU restatement oracle/splice_oracle.c (or_compose_hint_dyn) byte for
byte, with the rect placed per stream and per frame
(scroll_batch_set_dyn_rect_at).  The reference has no implementation of this
combination (docs/MASTER_DESIGN.md:58-64,109-146 describe it): parity is
UNPINNED beyond tests/test_hintdyn_oracle.py, which pins the restatement to
the plain dynamic-rect NAL when there are no hints and decodes +
reconstructs the hinted rects from the standard.  Run on an MI355X: -m gpu."""
import ctypes
import random

import numpy as np
import pytest

from conftest import synthetic_offsets
from dynhelp import OrCfg, Rect, hint_array, qp_field, random_hints, split_nals
from test_gpu_dyn import oracle_streams, random_refs, striped_refs, synth_source

pytestmark = pytest.mark.gpu

EXACT, PSKIP, SPEC = 0, 1, 2


@pytest.fixture(scope="module")
def gpu(scroll):
    if scroll.device_count() < 1:
        pytest.fail("no gfx950 device: " + scroll.last_error())
    return scroll


def plan(oracle, w, h, offsets, rw, rh, seed, p_hint=0.8, p_none=0.15, modes=(EXACT, PSKIP, SPEC),
         waypoints=(), fixed=None):
    """random hints and rect positions per (stream, frame):
    {(s, f): (rects, mode, (x0, y0) or None)}"""
    rng = random.Random(seed)
    S, F = offsets.shape
    mbw, mbh = w // 16, h // 16
    plan_ = {}
    for s in range(S):
        for f in range(F):
            rects = random_hints(rng, mbw, mbh, [0, 1], 5) if rng.random() < p_hint else []
            pos = fixed or (rng.randint(0, mbw - rw), rng.randint(0, mbh - rh))
            if rng.random() < p_none:
                pos = None
            plan_[(s, f)] = (rects, rng.choice(modes), pos)
    return plan_


def oracle_hintdyn(oracle, w, h, offsets, rw, rh, plan_, src, R, compose_mode=0, waypoints=(),
                   t0=0, qp_of=None):
    S, F = offsets.shape
    oracle.or_compose_hint_dyn.restype = ctypes.c_size_t
    buf = (ctypes.c_uint8 * (16 << 20))()
    err = ctypes.c_int()
    outs = []
    for s in range(S):
        c = OrCfg()
        oracle.or_cfg_init(ctypes.byref(c), w, h)
        c.frame_num = 2
        for i, (o, lt, v) in enumerate(waypoints):
            c.wp_off[i], c.wp_lt[i], c.wp_valid[i] = o, lt, v
        c.nwp = len(waypoints)
        o = bytearray()
        for f in range(F):
            rects, hm, pos = plan_[(s, f)]
            arr, n = hint_array(rects)
            rc = Rect(pos[0], pos[1], rw, rh, qp_field(qp_of(s, f)) if qp_of else 0) if pos else None
            sp = np.ascontiguousarray(src[s, t0 + f])
            k = oracle.or_compose_hint_dyn(buf, len(buf), ctypes.byref(c), int(offsets[s, f]),
                                           compose_mode, arr, n, hm,
                                           ctypes.byref(rc) if rc else None,
                                           sp.ctypes.data_as(ctypes.c_void_p), ctypes.byref(R.refs),
                                           ctypes.byref(err))
            assert err.value == 0 and k > 0, (s, f, err.value)
            o += bytes(buf[:k])
        outs.append(bytes(o))
    return outs


def gpu_batch(gpu, w, h, S, F, rect, R, slot=0, compose_mode=0, waypoints=(), arena=16 << 20):
    b = gpu.Batch(S, F, arena, mode=compose_mode)
    for _ in range(S):
        b.add_stream(gpu.make_config(w, h, waypoints=waypoints))
    b.set_dyn_rect(rect[0], rect[1], rect[2], rect[3], slot)
    b.set_dyn_refs(R.i420(0), R.i420(1))
    return b


def apply_plan(b, plan_, F, f0=0):
    for (s, f), (rects, hm, pos) in plan_.items():
        if not f0 <= f < f0 + F:
            continue
        b.set_hints(s, f - f0, rects, hm)
        b.set_dyn_rect_at(s, f - f0, *(pos if pos else (-1, -1)))


def check_equal(b, want):
    for s, ws in enumerate(want):
        got = b.output(s)
        if got != ws:
            gn, wn = split_nals(got), split_nals(ws)
            bad = next((i for i, (x, y) in enumerate(zip(gn, wn)) if x != y), min(len(gn), len(wn)))
            detail = ""
            if bad < min(len(gn), len(wn)):
                x, y = gn[bad], wn[bad]
                k = next((i for i, (p, q) in enumerate(zip(x, y)) if p != q), min(len(x), len(y)))
                detail = f"NAL {bad}: sizes {len(x)} vs {len(y)}, first diff at byte {k}"
            raise AssertionError(f"stream {s}: {len(got)} vs {len(ws)} bytes, "
                                 f"{len(gn)} vs {len(wn)} NALs; {detail}")


def test_no_hint_rects_exact_is_the_dynamic_rect(gpu, oracle):
    """hints on, no rects, EXACT, the batch rect everywhere: the plain
    dynamic-rect stream (or_compose_dyn, the k_dyn_row path's oracle)"""
    w, h = 640, 720
    offs = synthetic_offsets(3, 16, h)
    offs[1] = np.arange(486, 502)                          # through the 496 waypoint
    rc = Rect(5, 9, 7, 5)
    R = striped_refs(oracle, w, h)
    src = synth_source(oracle, 3, 16, rc)
    want = oracle_streams(oracle, w, h, offs, rc, src, R)
    b = gpu_batch(gpu, w, h, 3, 16, (rc.x0, rc.y0, rc.w, rc.h), R)
    b.set_hints(0, 0, [], EXACT)
    b.set_offsets(offs)
    b.set_dyn_source(src.tobytes(), 16)
    b.compose(16)
    assert b.sync() == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


@pytest.mark.parametrize("w,h,rw,rh,seed", [(256, 720, 4, 3, 1), (640, 480, 9, 6, 2),
                                             (1280, 720, 12, 8, 3)])
def test_moving_rect_random_hints(gpu, oracle, w, h, rw, rh, seed):
    S, F = 4, 12
    offs = synthetic_offsets(S, F, h, first_stream=seed)
    offs[1] = np.clip(np.arange(490, 490 + F), 0, h)
    rc = Rect(0, 0, rw, rh)
    R = striped_refs(oracle, w, h)
    src = synth_source(oracle, S, F, rc, t0=seed)
    pl = plan(oracle, w, h, offs, rw, rh, seed)
    want = oracle_hintdyn(oracle, w, h, offs, rw, rh, pl, src, R)
    b = gpu_batch(gpu, w, h, S, F, (0, 0, rw, rh), R)
    apply_plan(b, pl, F)
    b.set_offsets(offs)
    b.set_dyn_source(src.tobytes(), F)
    b.compose(F)
    assert b.sync() == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


def test_noise_source_random_refs_large_regions(gpu, oracle):
    """residual-heavy MBs (noise source against noise references, sub-pel
    chroma from odd hint motion) with the largest per-MB regions"""
    w, h, rw, rh, S, F = 512, 384, 6, 5, 3, 8
    offs = synthetic_offsets(S, F, h, first_stream=4)
    R = random_refs(w, h, 11)
    src = np.random.default_rng(12).integers(0, 256, (S, F, 384 * rw * rh), dtype=np.uint8)
    pl = plan(oracle, w, h, offs, rw, rh, 13, p_hint=1.0, p_none=0.1)
    want = oracle_hintdyn(oracle, w, h, offs, rw, rh, pl, src, R)
    b = gpu_batch(gpu, w, h, S, F, (0, 0, rw, rh), R, slot=2048 * rw * rh)
    apply_plan(b, pl, F)
    b.set_offsets(offs)
    b.set_dyn_source(src.tobytes(), F)
    b.compose(F)
    assert b.sync() == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


def test_small_regions_overflow_then_clear(gpu, oracle, scroll):
    """64-byte regions cannot hold noise MBs: SCROLL_ERR_OVERFLOW, nothing
    committed; clear_hints -> the plain dynamic rect (k_dyn_row path) again"""
    w, h, rw, rh, S, F = 256, 256, 3, 3, 2, 4
    offs = synthetic_offsets(S, 2 * F, h, first_stream=6)
    R = random_refs(w, h, 21)
    src = np.random.default_rng(22).integers(0, 256, (S, 2 * F, 384 * rw * rh), dtype=np.uint8)
    b = gpu_batch(gpu, w, h, S, F, (1, 1, rw, rh), R, slot=64 * rw * rh)
    b.set_hints(0, 0, [(0, 0, 16, 16, 0, 3, -5)], SPEC)
    b.set_offsets(np.ascontiguousarray(offs[:, :F]))
    b.set_dyn_source(np.ascontiguousarray(src[:, :F]).tobytes(), F)
    b.compose(F)
    assert b.sync() == scroll.SCROLL_ERR_OVERFLOW
    assert "region" in gpu.last_error()
    assert b.output_size(0) == 0
    b.clear_hints()
    b.set_dyn_rect(1, 1, rw, rh, 0)        # slot_bytes: the plain rect's staging cap again
    b.set_dyn_refs(R.i420(0), R.i420(1))
    rc = Rect(1, 1, rw, rh)
    want = oracle_streams(oracle, w, h, np.ascontiguousarray(offs[:, F:]), rc,
                          np.ascontiguousarray(src[:, F:]), R)
    b.reset_output()
    b.set_offsets(np.ascontiguousarray(offs[:, F:]))
    b.set_dyn_source(np.ascontiguousarray(src[:, F:]).tobytes(), F)
    b.compose(F)
    assert b.sync() == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


def test_chunks_experiment_mode_and_waypoint_refs(gpu, oracle):
    """hint rects naming a waypoint reference once it is valid, experiment
    mode (waypoint NAL instead of the scroll NAL), two composes"""
    w, h, rw, rh, S, F = 512, 512, 5, 4, 3, 10
    offs = synthetic_offsets(S, 2 * F, h, first_stream=8)
    offs[0] = np.arange(484, 484 + 2 * F)              # waypoint 0 (496) valid from t = 12
    rc = Rect(0, 0, rw, rh)
    R = striped_refs(oracle, w, h)
    src = synth_source(oracle, S, 2 * F, rc)
    rng = random.Random(9)
    pl = {}
    for s in range(S):
        for t in range(2 * F):
            if s == 0 and t >= 12 and t % 3 == 0:
                rects = [(0, 0, w // 16, 3, 2, 0, 0)]
            else:
                rects = random_hints(rng, w // 16, h // 16, [0, 1], 4)
            pos = (rng.randint(0, w // 16 - rw), rng.randint(0, h // 16 - rh)) if t % 4 else None
            pl[(s, t)] = (rects, rng.choice((EXACT, PSKIP, SPEC)), pos)
    want = oracle_hintdyn(oracle, w, h, offs, rw, rh, pl, src, R, compose_mode=1)
    b = gpu_batch(gpu, w, h, S, F, (0, 0, rw, rh), R, compose_mode=1)
    for c0 in (0, F):
        apply_plan(b, pl, F, f0=c0)
        b.set_offsets(np.ascontiguousarray(offs[:, c0:c0 + F]))
        b.set_dyn_source(np.ascontiguousarray(src[:, c0:c0 + F]).tobytes(), F)
        b.compose(F)
        assert b.sync() == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


def test_arguments(gpu, oracle, scroll):
    w, h = 256, 256
    R = striped_refs(oracle, w, h)
    b = gpu_batch(gpu, w, h, 1, 2, (0, 0, 4, 4), R)
    with pytest.raises(RuntimeError):
        b.set_dyn_rect_at(0, 0, 13, 0)                 # leaves the picture
    with pytest.raises(RuntimeError):
        b.set_dyn_rect_at(0, 2, 0, 0)                  # frame out of range
    b.set_dyn_rect_at(0, 1, 3, 3)                      # moved: needs hints
    b.set_offsets(np.array([[10, 20]], np.int32))
    b.dyn_source_synth(2, 0, 0)
    with pytest.raises(RuntimeError, match="hints"):
        b.compose(2)
    b.set_hints(0, 0, [], SPEC)
    with pytest.raises(RuntimeError):                  # one rect per frame
        b.set_splice(0, 0, 0, 0, 1, 1, b"\x00\x00\x00\x01\x21\x00")
    b.compose(2)
    assert b.sync() == 0, gpu.last_error()
    b.close()


def test_hinted_rect_qp_per_stream_and_frame(gpu, oracle):
    """the rect under hints at per-stream QPs (scroll_batch_set_dyn_qp_stream)
    with per-frame overrides (scroll_batch_set_dyn_qp_at), QP 0 included:
    k_hdyn_code quantises at the frame's QP, the rect's first coded MB
    carries mb_qp_delta QP - 26 (k_splice_stage), equal to the oracle"""
    w, h = 640, 480
    rw, rh = 9, 7
    S, F = 3, 5
    offs = synthetic_offsets(S, F, h)
    plan_ = plan(oracle, w, h, offs, rw, rh, seed=41)
    R = random_refs(w, h, 13)
    src = synth_source(oracle, S, F, Rect(0, 0, rw, rh))
    sq = [12, 40, 26]
    fq = {(0, 1): 0, (1, 3): 18, (2, 2): 51}
    qp_of = lambda s_, f_: fq.get((s_, f_), sq[s_])   # noqa: E731
    want = oracle_hintdyn(oracle, w, h, offs, rw, rh, plan_, src, R, qp_of=qp_of)
    b = gpu_batch(gpu, w, h, S, F, (0, 0, rw, rh), R, slot=2048 * rw * rh)   # QP 0: larger MB regions
    apply_plan(b, plan_, F)
    for s_, q in enumerate(sq):
        b.set_dyn_qp(q, stream=s_)
    for (s_, f_), q in fq.items():
        b.set_dyn_qp_at(s_, f_, q)
    b.set_offsets(np.ascontiguousarray(offs))
    b.set_dyn_source(np.ascontiguousarray(src).tobytes(), F)
    b.compose(F)
    assert b.sync() == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


def test_fallback_whole_frame_on_inconsistent_hints(gpu, oracle, scroll):
    """scroll_batch_set_fallback (docs/MASTER_DESIGN.md:220: hints
    inconsistent -> full conventional encode): the rect is the whole picture;
    streams 1 and 3 get frames whose topmost hint rect names a waypoint the
    frame lacks.  Those frames -- the ones that fail the stream without the
    flag -- come out as or_compose_hint_dyn with no hint rects and the
    whole-picture rect; every other frame (with or without the rect placed,
    all three hint modes) is the oracle's hinted frame; streams 0 and 2 are
    untouched.  Without the flag the same batch fails."""
    w, h, S, F = 320, 240, 4, 8
    mbw, mbh = w // 16, h // 16
    offs = synthetic_offsets(S, F, h, first_stream=2)
    offs[1] = np.clip(np.arange(490, 490 + F), 0, h)        # through the 496 waypoint
    rc = Rect(0, 0, mbw, mbh)
    R = striped_refs(oracle, w, h)
    src = synth_source(oracle, S, F, rc)
    rng = random.Random(9)
    pl, bad = {}, set()
    for s in range(S):
        for f in range(F):
            rects = random_hints(rng, mbw, mbh, [0, 1], 4)
            if s in (1, 3) and f % 3 != 1:
                rects = rects + [(2, 2, 9, 7, 2 + 6, 16, -32)]   # waypoint 6: never valid here
                bad.add((s, f))
            pl[(s, f)] = (rects, rng.choice((EXACT, PSKIP, SPEC)), (0, 0) if rng.random() < 0.35 else None)
    oracle.or_compose_hint_dyn.restype = ctypes.c_size_t
    buf = (ctypes.c_uint8 * (16 << 20))()
    err = ctypes.c_int()
    want, fell = [], set()
    for s in range(S):
        c = OrCfg()
        oracle.or_cfg_init(ctypes.byref(c), w, h)
        c.frame_num = 2
        o = bytearray()
        for f in range(F):
            rects, hm, pos = pl[(s, f)]
            sp = np.ascontiguousarray(src[s, f])
            arr, n = hint_array(rects)
            c2 = OrCfg.from_buffer_copy(c)
            r1 = Rect(0, 0, mbw, mbh) if pos else None
            k = oracle.or_compose_hint_dyn(buf, len(buf), ctypes.byref(c2), int(offs[s, f]), 0, arr, n, hm,
                                           ctypes.byref(r1) if r1 else None, sp.ctypes.data_as(ctypes.c_void_p),
                                           ctypes.byref(R.refs), ctypes.byref(err))
            if err.value != 0:                                 # inconsistent: the whole frame instead
                fell.add((s, f))
                c2 = OrCfg.from_buffer_copy(c)
                k = oracle.or_compose_hint_dyn(buf, len(buf), ctypes.byref(c2), int(offs[s, f]), 0, None, 0,
                                               hm, ctypes.byref(Rect(0, 0, mbw, mbh)),
                                               sp.ctypes.data_as(ctypes.c_void_p), ctypes.byref(R.refs),
                                               ctypes.byref(err))
            assert err.value == 0 and k > 0, (s, f)
            o += bytes(buf[:k])
            c = c2
        want.append(bytes(o))
    assert fell == bad, "the test's invalid rects must be the ones the oracle refuses"
    b = gpu_batch(gpu, w, h, S, F, (0, 0, mbw, mbh), R)
    b.set_fallback(True)
    apply_plan(b, pl, F)
    b.set_offsets(offs)
    b.set_dyn_source(src.tobytes(), F)
    b.compose(F)
    assert b.sync() == 0, gpu.last_error()
    check_equal(b, want)
    for s in range(S):
        for f in range(F):
            assert b.fallback_frame(s, f) == ((s, f) in fell), (s, f)
    b.close()
    b = gpu_batch(gpu, w, h, S, F, (0, 0, mbw, mbh), R)        # without the flag: the stream fails
    apply_plan(b, pl, F)
    b.set_offsets(offs)
    b.set_dyn_source(src.tobytes(), F)
    b.compose(F)
    assert b.sync() == scroll.SCROLL_ERR_CONFIG
    b.close()
    b = gpu_batch(gpu, w, h, S, F, (2, 2, 5, 4), R)             # not the whole picture
    with pytest.raises(RuntimeError):
        b.set_fallback(True)
    b.close()
