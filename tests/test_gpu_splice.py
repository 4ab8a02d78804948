"""GPU parity of the pre-encoded MB splice:
k_plan (state) -> k_splice_parse -> k_hint_stage / k_splice_stage ->
k_plan (size) -> k_emit -> k_dyn_emit_gather / k_dyn_emit, through the C ABI,
against the CPU restatement oracle/splice_oracle.c (or_compose_splice) byte
for byte.  tests/test_splice_oracle.py pins the restatement by decoding the
composed NALs from the standard.  External slices come from the oracle's
stand-in encoder (or_ext_slice).  Run on an MI355X: -m gpu."""
import ctypes
import random

import numpy as np
import pytest

from conftest import synthetic_offsets
from dynhelp import OrCfg, hint_array, random_hints, split_nals, ext_slice, splice_of

pytestmark = pytest.mark.gpu

EXACT, PSKIP, SPEC = 0, 1, 2


@pytest.fixture(scope="module")
def gpu(scroll):
    if scroll.device_count() < 1:
        pytest.fail("no gfx950 device: " + scroll.last_error())
    return scroll


def _cfg(oracle, w, h):
    c = OrCfg()
    oracle.or_cfg_init(ctypes.byref(c), w, h)
    c.frame_num = 2
    return c


def plan(oracle, w, h, offsets, seed, p_splice=0.7, p_hint=0.3, modes=(EXACT, PSKIP, SPEC),
         max_rect=(10, 8), compose_mode=0, ext_kw=None):
    """random splices (+ hints) per (stream, frame) whose refs are valid in
    that frame; -> (frames dict, oracle bytes per stream)"""
    rng = random.Random(seed)
    S, F = offsets.shape
    mbw, mbh = w // 16, h // 16
    buf = (ctypes.c_uint8 * (16 << 20))()
    err = ctypes.c_int()
    frames, outs = {}, []
    for s in range(S):
        c = _cfg(oracle, w, h)
        o = bytearray()
        for t in range(F):
            refs = [0, 1] + [2 + i for i in range(c.nwp) if c.wp_valid[i]]
            rects = random_hints(rng, mbw, mbh, refs, 3) if rng.random() < p_hint else []
            mode = rng.choice(modes)
            sp = None
            if rng.random() < p_splice:
                sw, sh = rng.randint(1, min(max_rect[0], mbw)), rng.randint(1, min(max_rect[1], mbh))
                x0, y0 = rng.randint(0, mbw - sw), rng.randint(0, mbh - sh)
                kw = dict(nrefs=len(refs), max_ref=len(refs) - 1,
                          skip_pm=rng.choice([0, 200, 600]), cbp_pm=rng.choice([300, 800, 1000]),
                          big_pm=rng.choice([0, 30]), mv_range=rng.choice([8, 200]),
                          slice_qp_delta=rng.randint(-4, 4), qp_jitter=rng.choice([0, 3]),
                          ref_idc=rng.choice([0, 1]), part_pm=rng.choice([0, 300, 1000]))
                kw.update(ext_kw or {})
                sp = (x0, y0, sw, sh, ext_slice(oracle, c, sw, sh, seed * 100003 + s * 1009 + t, **kw))
            frames[(s, t)] = (rects, mode, sp)
            arr, n = hint_array(rects)
            spc = splice_of(*sp) if sp else None
            k = oracle.or_compose_splice(buf, len(buf), ctypes.byref(c), int(offsets[s, t]),
                                         compose_mode, arr, n, mode,
                                         ctypes.byref(spc) if spc else None, ctypes.byref(err))
            assert err.value == 0 and k > 0, (s, t, err.value)
            o += bytes(buf[:k])
        outs.append(bytes(o))
    return frames, outs


def gpu_streams(gpu, w, h, offsets, frames, compose_mode=0, arena=16 << 20, debug=0):
    S, F = offsets.shape
    b = gpu.Batch(S, F, arena, mode=compose_mode)
    for _ in range(S):
        b.add_stream(gpu.make_config(w, h))
    if debug:
        b.set_debug(debug)
    for (s, f), (rects, mode, sp) in frames.items():
        if rects or sp or mode != EXACT:          # a splice alone would default to SPEC
            b.set_hints(s, f, rects, mode)
        if sp:
            b.set_splice(s, f, *sp)
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


@pytest.mark.parametrize("w,h,seed", [(320, 256, 1), (640, 480, 2), (1280, 720, 3)])
def test_random_splices(gpu, oracle, w, h, seed):
    offs = synthetic_offsets(5, 16, h, first_stream=seed)
    offs[1] = np.clip(np.arange(484, 500), 0, h)       # waypoints: refs 2 + i appear
    frames, want = plan(oracle, w, h, offs, seed)
    b, rc = gpu_streams(gpu, w, h, offs, frames)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    for (s, f), (_, _, sp) in frames.items():
        assert b.splice_status(s, f) == 0
    b.close()


def test_partitioned_splices(gpu, oracle):
    """every external MB partitioned (P_L0_L0_16x8 / 8x16, P_8x8 with random
    sub_mb_types, P_8x8ref0) or skipped, waypoint references, hints, all
    three modes: the composed 16x16 MBs around them predict from their 4x4
    blocks"""
    w, h = 640, 480
    offs = synthetic_offsets(4, 16, h, first_stream=9)
    offs[2] = np.arange(486, 502)
    frames, want = plan(oracle, w, h, offs, 31, p_splice=0.9, p_hint=0.4, max_rect=(12, 9),
                        ext_kw=dict(part_pm=1000, skip_pm=150, mv_range=300))
    b, rc = gpu_streams(gpu, w, h, offs, frames)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


def test_large_rect_4k_and_ep_path(gpu, oracle, scroll):
    """3840x2160, up to 25x25 MB splices with large levels; again with the
    dynamic emit's EP list capped at 4 (every NAL through k_dyn_emit)"""
    w, h = 3840, 2160
    offs = np.array([[490, 496, 500, 992], [1984, 1990, 2000, 700]], np.int32)
    frames, want = plan(oracle, w, h, offs, 11, p_splice=1.0, max_rect=(25, 25),
                        ext_kw=dict(cbp_pm=1000, big_pm=100, mv_range=2000, part_pm=500))
    for debug in (0, scroll.SCROLL_DEBUG_DYN_EPCAP4):
        b, rc = gpu_streams(gpu, w, h, offs, frames, arena=64 << 20, debug=debug)
        assert rc == 0, gpu.last_error()
        check_equal(b, want)
        b.close()


def test_whole_picture_and_corner_splices(gpu, oracle):
    w, h = 192, 128
    mbw, mbh = w // 16, h // 16
    offs = np.array([[40, 41, 42, 43, 44, 45]], np.int32)
    c = _cfg(oracle, w, h)
    rects = [(0, 0, mbw, mbh), (mbw - 3, 0, 3, 3), (0, mbh - 2, 4, 2), (mbw - 2, mbh - 2, 2, 2),
             (5, 3, 1, 1), (0, 0, 1, mbh)]
    frames = {}
    buf = (ctypes.c_uint8 * (4 << 20))()
    err = ctypes.c_int()
    o = bytearray()
    for t, (x0, y0, sw, sh) in enumerate(rects):
        mode = (EXACT, PSKIP, SPEC)[t % 3]
        sp = (x0, y0, sw, sh, ext_slice(oracle, c, sw, sh, 500 + t, cbp_pm=900, skip_pm=300))
        frames[(0, t)] = ([], mode, sp)
        k = oracle.or_compose_splice(buf, len(buf), ctypes.byref(c), int(offs[0, t]), 0, None, 0,
                                     mode, ctypes.byref(splice_of(*sp)), ctypes.byref(err))
        assert err.value == 0
        o += bytes(buf[:k])
    b, rc = gpu_streams(gpu, w, h, offs, frames)
    assert rc == 0, gpu.last_error()
    check_equal(b, [bytes(o)])
    b.close()


def test_experiment_mode(gpu, oracle):
    w, h = 640, 480
    offs = synthetic_offsets(3, 20, h, first_stream=4)
    offs[2] = np.arange(480, 500)
    frames, want = plan(oracle, w, h, offs, 21, compose_mode=1)
    b, rc = gpu_streams(gpu, w, h, offs, frames, compose_mode=1)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


def test_errors_fail_only_their_stream(gpu, oracle, scroll):
    w, h = 256, 256
    offs = synthetic_offsets(6, 6, h)
    c = _cfg(oracle, w, h)
    good = ext_slice(oracle, c, 4, 3, 1)
    G = 5                                                   # the stream without an error
    cases = {
        0: (scroll.SCROLL_SPLICE_ERR_MBTYPE, ext_slice(oracle, c, 4, 3, 1, bad_mb=0, bad_type=5)),
        1: (scroll.SCROLL_SPLICE_ERR_NAL, good[:4] + bytes([0x66]) + good[5:]),      # an SEI
        2: (scroll.SCROLL_SPLICE_ERR_SYNTAX, good[:len(good) // 2]),
        3: (scroll.SCROLL_SPLICE_ERR_REF, ext_slice(oracle, c, 4, 3, 2, nrefs=4, max_ref=3,
                                                    skip_pm=0)),
        4: (scroll.SCROLL_SPLICE_ERR_HEADER, good[:4] + bytes([0x65]) + good[5:]),   # IDR, P slice
    }
    b = gpu.Batch(6, 6, 8 << 20)
    for _ in range(6):
        b.add_stream(gpu.make_config(w, h))
    for s, (_, nal) in cases.items():
        b.set_splice(s, 2, 2, 2, 4, 3, nal)
    b.set_splice(G, 1, 2, 2, 4, 3, good)
    b.set_offsets(offs)
    b.compose(6)
    assert b.sync() == scroll.SCROLL_ERR_CONFIG
    assert "splice" in gpu.last_error()
    for s, (code, _) in cases.items():
        assert b.splice_status(s, 2) == code, s
        assert b.output_size(s) == 0, s                     # nothing committed
    buf = (ctypes.c_uint8 * (1 << 20))()
    err = ctypes.c_int()
    c4 = _cfg(oracle, w, h)
    o = bytearray()
    for t in range(6):
        sp = splice_of(2, 2, 4, 3, good) if t == 1 else None
        k = oracle.or_compose_splice(buf, len(buf), ctypes.byref(c4), int(offs[G, t]), 0, None, 0,
                                     SPEC, ctypes.byref(sp) if sp else None, ctypes.byref(err))
        o += bytes(buf[:k])
    assert b.output(G) == bytes(o)
    b.close()


def test_persist_remove_and_clear(gpu, oracle):
    """splices persist across composes; removing one / clearing all returns
    those frames to plain scroll frames"""
    w, h = 512, 512
    offs = synthetic_offsets(2, 30, h, first_stream=7)
    F1 = 10
    c = _cfg(oracle, w, h)
    sps = {f: (f % 5, f % 7, 3 + f % 4, 2 + f % 3, ext_slice(oracle, c, 3 + f % 4, 2 + f % 3, 900 + f))
           for f in range(F1)}
    b = gpu.Batch(2, F1, 8 << 20)
    for _ in range(2):
        b.add_stream(gpu.make_config(w, h))
    for s in range(2):
        for f in range(F1):
            b.set_splice(s, f, *sps[f])
    b.set_splice(1, 3, 0, 0, 0, 0, b"")                  # removed again
    buf = (ctypes.c_uint8 * (4 << 20))()
    err = ctypes.c_int()
    want = []
    for s in range(2):
        cs = _cfg(oracle, w, h)
        o = bytearray()
        for t in range(30):
            f = t % F1
            sp = splice_of(*sps[f]) if t < 20 and not (s == 1 and f == 3) else None
            k = oracle.or_compose_splice(buf, len(buf), ctypes.byref(cs), int(offs[s, t]), 0, None,
                                         0, SPEC, ctypes.byref(sp) if sp else None,
                                         ctypes.byref(err))
            assert err.value == 0
            o += bytes(buf[:k])
        want.append(bytes(o))
    for c0 in (0, 10, 20):
        if c0 == 20:
            b.clear_splices()
        b.set_offsets(np.ascontiguousarray(offs[:, c0:c0 + F1]))
        b.compose(F1)
        assert b.sync() == 0, gpu.last_error()
    for s in range(2):
        assert b.output(s) == want[s], s
    b.close()


def test_dynamic_coder_output_spliced_from_device(gpu, oracle):
    """MASTER_DESIGN 4.2 on one GPU: the dynamic rect coder encodes 400x400
    pictures (rect = the whole picture); its scroll NALs, left in its device
    arena, are spliced by device pointer into 1280x720 scroll frames"""
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    S, F, W, H = 3, 6, 1280, 720
    e, ptrs = bench.external_slices(gpu, S, F, 25, 25, 0, 0)
    offs = synthetic_offsets(S, F, H, first_stream=2)
    offs[1] = np.arange(492, 498)                         # a waypoint on the way
    b = gpu.Batch(S, F, 16 << 20)
    for _ in range(S):
        b.add_stream(gpu.make_config(W, H))
    b.set_splices_device([(s, f, 28, 10, 25, 25, p, n) for (s, f), (p, n) in ptrs.items()])
    b.set_offsets(offs)
    b.compose(F)
    assert b.sync() == 0, gpu.last_error()
    buf = (ctypes.c_uint8 * (16 << 20))()
    err = ctypes.c_int()
    for s in range(S):
        host, pos = e.output(s), 0
        c = _cfg(oracle, W, H)
        o = bytearray()
        for f in range(F):
            n = ptrs[(s, f)][1]
            sp = splice_of(28, 10, 25, 25, host[pos:pos + n])
            pos += n
            k = oracle.or_compose_splice(buf, len(buf), ctypes.byref(c), int(offs[s, f]), 0, None,
                                         0, SPEC, ctypes.byref(sp), ctypes.byref(err))
            assert err.value == 0
            o += bytes(buf[:k])
        assert b.output(s) == bytes(o), s
    b.close()
    e.close()


def test_startcode_less_odd_length_adjacent_frames(gpu, oracle):
    """NALs handed over without an Annex-B start code (optional in the API)
    whose lengths are not multiples of 4, in adjacent frames of a stream: the
    RBSP pool regions of neighbouring frames must not overlap (k_splice_unesc
    writes whole words, the last one zero-padded)"""
    w, h = 320, 256
    S, F = 2, 8
    offs = synthetic_offsets(S, F, h, first_stream=3)
    c = _cfg(oracle, w, h)
    frames = {}
    lens = set()
    for s in range(S):
        for t in range(F):
            seed = 3000 + 17 * s + t
            while True:
                nal = ext_slice(oracle, c, 5, 4, seed, cbp_pm=800, skip_pm=100)[4:]   # no start code
                if len(nal) % 4:
                    break
                seed += 1000
            lens.add(len(nal) % 4)
            frames[(s, t)] = ([], SPEC, (3, 2, 5, 4, nal))
    _, want = plan_from(oracle, w, h, offs, frames)
    b, rc = gpu_streams(gpu, w, h, offs, frames)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    assert lens <= {1, 2, 3}
    b.close()


def test_device_slices_at_every_alignment(gpu, oracle):
    """slices handed over by device pointer at every byte offset modulo 16
    (k_splice_units / k_splice_unesc read the aligned 16-byte lines around
    them, the bytes outside the slice masked): the oracle's bytes"""
    from test_gpu_ipcm import Hip             # device memory through libh264scroll's own HIP runtime
    w, h = 320, 256
    S, F = 2, 8
    offs = synthetic_offsets(S, F, h, first_stream=5)
    c = _cfg(oracle, w, h)
    frames = {}
    for s in range(S):
        for t in range(F):
            nal = ext_slice(oracle, c, 5, 4, 5000 + 31 * s + t, cbp_pm=800, skip_pm=100)
            frames[(s, t)] = ([], SPEC, (3, 2, 5, 4, nal))
    _, want = plan_from(oracle, w, h, offs, frames)
    total = sum(len(sp[4]) + 32 for (_, _, sp) in frames.values())
    dev = Hip().buf(total + 64, fill=0xA5)                   # non-zero bytes around the slices
    pos, specs = 0, []
    for k, ((s, t), (_, _, sp)) in enumerate(sorted(frames.items())):
        nal = bytes(sp[4])
        pos = ((pos + 15) & ~15) + k % 16
        dev.write(pos, nal)
        specs.append((s, t, 3, 2, 5, 4, dev.p + pos, len(nal)))
        pos += len(nal)
    b = gpu.Batch(S, F, 16 << 20)
    for _ in range(S):
        b.add_stream(gpu.make_config(w, h))
    b.set_splices_device(specs)
    b.set_offsets(offs)
    b.compose(F)
    assert b.sync() == 0, gpu.last_error()
    check_equal(b, want)
    assert {sp[6] % 16 for sp in specs} == set(range(16))
    b.close()
    dev.free()


def plan_from(oracle, w, h, offsets, frames, compose_mode=0):
    """oracle bytes per stream for a given frames dict (as plan() returns)"""
    S, F = offsets.shape
    buf = (ctypes.c_uint8 * (16 << 20))()
    err = ctypes.c_int()
    outs = []
    for s in range(S):
        c = _cfg(oracle, w, h)
        o = bytearray()
        for t in range(F):
            rects, mode, sp = frames.get((s, t), ([], SPEC, None))
            arr, n = hint_array(rects)
            spc = splice_of(*sp) if sp else None
            k = oracle.or_compose_splice(buf, len(buf), ctypes.byref(c), int(offsets[s, t]),
                                         compose_mode, arr, n, mode,
                                         ctypes.byref(spc) if spc else None, ctypes.byref(err))
            assert err.value == 0 and k > 0, (s, t, err.value)
            o += bytes(buf[:k])
        outs.append(bytes(o))
    return frames, outs


def test_intra_and_multislice_splices(gpu, oracle):
    """external pictures with I_4x4 / I_16x16 / I_PCM MBs (samples all zero
    in some: emulation prevention inside I_PCM), in one slice or a slice per
    one / two / three MB rows, spliced in all three modes over waypoints:
    k_splice_units finds the slices, one wave parses each, k_splice_fix
    chains them; I_PCM realigned at its composed position"""
    w, h = 640, 480
    offs = synthetic_offsets(4, 12, h, first_stream=5)
    offs[1] = np.arange(488, 500)
    for seed, rows in ((41, 0), (42, 1), (43, 2), (44, 3)):
        frames, want = plan(oracle, w, h, offs, seed, p_splice=0.9, p_hint=0.3, max_rect=(12, 9),
                            ext_kw=dict(intra_pm=500, slice_rows=rows, pcm_zero=seed % 2,
                                        part_pm=200, qp_jitter=5))
        b, rc = gpu_streams(gpu, w, h, offs, frames)
        assert rc == 0, gpu.last_error()
        check_equal(b, want)
        for (s, f), (_, _, sp) in frames.items():
            assert b.splice_status(s, f) == 0
        b.close()


def test_pcm_only_and_intra_types(gpu, oracle):
    """every coded MB intra of one type (I_PCM only: many alignments in one
    staging window; I_4x4 only; I_16x16 only), 4K rects"""
    w, h = 1920, 1088
    offs = synthetic_offsets(3, 6, h, first_stream=1)
    for types in (4, 1, 2):
        frames, want = plan(oracle, w, h, offs, 50 + types, p_splice=1.0, p_hint=0.2, max_rect=(30, 20),
                            ext_kw=dict(intra_pm=1000, intra_types=types, skip_pm=100,
                                        slice_rows=types - 1))
        b, rc = gpu_streams(gpu, w, h, offs, frames, arena=64 << 20)
        assert rc == 0, gpu.last_error()
        check_equal(b, want)
        b.close()


def test_intra_on_rect_edges(gpu, oracle, scroll):
    """I_4x4 / I_16x16 on the rect's top / left edge: refused inside the
    picture (SCROLL_SPLICE_ERR_MBTYPE, the stream fails alone), accepted with
    the rect in the picture's corner; I_PCM anywhere"""
    w, h = 256, 256
    offs = synthetic_offsets(4, 4, h, first_stream=2)
    c = _cfg(oracle, w, h)
    frames = {}
    for i, (mb, t) in enumerate(((0, 5), (1, 12), (4, 30), (0, 30))):
        nal = ext_slice(oracle, c, 4, 3, 1, bad_mb=mb, bad_type=t)
        frames[(i, 0)] = ([], SPEC, (0, 0, 4, 3, nal))                 # corner: accepted
        frames[(i, 2)] = ([], SPEC, (2, 2, 4, 3, nal))
    b, rc = gpu_streams(gpu, w, h, offs, frames)
    assert rc == scroll.SCROLL_ERR_CONFIG
    oracle.or_splice_refused.restype = ctypes.c_int
    for i, (mb, t) in enumerate(((0, 5), (1, 12), (4, 30), (0, 30))):
        want = 0 if t == 30 else scroll.SCROLL_SPLICE_ERR_MBTYPE
        assert b.splice_status(i, 2) == want, (i, b.splice_status(i, 2))
        if want == 0:
            assert b.splice_status(i, 0) == 0
        else:
            # the refused MB, as the oracle's parse names it (scroll_batch_splice_refusal)
            rb = (ctypes.c_uint8 * (len(frames[(i, 2)][2][4]) + 8))()
            mbs = (ctypes.c_uint8 * (4 * 12 * 2048))()
            rn = ctypes.c_size_t()
            sp = splice_of(*frames[(i, 2)][2])
            assert oracle.or_splice_parse(ctypes.byref(c), ctypes.byref(sp), mbs, rb, ctypes.byref(rn)) == want
            ref = oracle.or_splice_refused()
            assert b.splice_refusal(i, 2) == (want, (ref & 0xffff) % 4, (ref & 0xffff) // 4, ref >> 16)
            assert (ref & 0xffff, ref >> 16) == (mb, t)
    good = {k: v for k, v in frames.items() if k[0] >= 2}
    _, want = plan_from(oracle, w, h, offs[2:], {(s - 2, f): v for (s, f), v in good.items()})
    check_equal(b, [None, None] + want, streams=[2, 3])
    b.close()


def test_multislice_rules(gpu, oracle, scroll):
    """slices out of order (HEADER), a row missing (SYNTAX), trailing zero
    bytes after each slice (accepted), more than 1,024 slices (NAL)"""
    import h264_pslice as P
    w, h = 256, 256
    offs = synthetic_offsets(5, 3, h, first_stream=6)
    c = _cfg(oracle, w, h)
    nal = ext_slice(oracle, c, 4, 4, 5, slice_rows=1, intra_pm=300)
    units = P.nal_units(nal)
    assert len(units) == 4
    sc = b"\x00\x00\x00\x01"
    cases = [
        (scroll.SCROLL_SPLICE_ERR_SYNTAX, b"".join(sc + u for u in units[:3])),
        (scroll.SCROLL_SPLICE_ERR_HEADER, b"".join(sc + u for u in (units[0], units[2], units[1], units[3]))),
        (0, b"".join(sc + u + b"\x00\x00" for u in units)),
        (scroll.SCROLL_SPLICE_ERR_NAL, b"".join(sc + units[0] for _ in range(1025))),
        (0, nal),
    ]
    frames = {(s, 1): ([], SPEC, (2, 2, 4, 4, d)) for s, (_, d) in enumerate(cases)}
    b, rc = gpu_streams(gpu, w, h, offs, frames)
    assert rc == scroll.SCROLL_ERR_CONFIG
    for s, (code, _) in enumerate(cases):
        assert b.splice_status(s, 1) == code, (s, b.splice_status(s, 1))
    ok = [s for s, (code, _) in enumerate(cases) if code == 0]
    _, want = plan_from(oracle, w, h, offs[ok], {(i, f): frames[(s, f)] for i, s in enumerate(ok) for f in (1,)})
    for i, s in enumerate(ok):
        assert b.output(s) == want[i], s
    b.close()


@pytest.mark.parametrize("islice,rows", [(1, 0), (2, 0), (1, 1), (2, 2)])
def test_i_and_idr_pictures(gpu, oracle, islice, rows):
    """a conventional encoder's first frame / scene cut: I slices (islice 1)
    and IDR pictures (islice 2, nal_unit_type 5), one slice or one per 1-2
    MB rows, every MB intra with an I_PCM edge ring, spliced at random
    places in all three modes: k_splice_lanes / k_splice_parse read the I /
    IDR header and the MBs without mb_skip_run, equal to the oracle"""
    w, h = 640, 480
    offs = synthetic_offsets(3, 8, h, first_stream=7)
    frames, want = plan(oracle, w, h, offs, 60 + 3 * islice + rows, p_splice=0.9, p_hint=0.3,
                        max_rect=(14, 10), ext_kw=dict(islice=islice, slice_rows=rows, cbp_pm=800,
                                                       big_pm=20, qp_jitter=4))
    b, rc = gpu_streams(gpu, w, h, offs, frames)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    for (s, f), (_, _, sp) in frames.items():
        assert b.splice_status(s, f) == 0
    b.close()


def test_all_intra_25x25_in_the_rect_interior(gpu, oracle):
    """the verdict's case: a 25x25-MB all-intra picture (I_4x4 / I_16x16
    inside, I_PCM edge ring), as an I and as an IDR picture, spliced at the
    config-3 rect (28, 10) of a 1280x720 stream"""
    w, h = 1280, 720
    offs = synthetic_offsets(2, 4, h, first_stream=3)
    c = _cfg(oracle, w, h)
    frames = {}
    for s in range(2):
        for f in range(4):
            nal = ext_slice(oracle, c, 25, 25, 90 + 4 * s + f, islice=1 + (f & 1), cbp_pm=900, big_pm=10,
                            qp_jitter=2, intra_types=3 if s else 0)
            frames[(s, f)] = ([], SPEC if f % 3 else EXACT, (28, 10, 25, 25, nal))
    _, want = plan_from(oracle, w, h, offs, frames)
    b, rc = gpu_streams(gpu, w, h, offs, frames)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    b.close()
