"""The UI-hint P-slice restatement (oracle/hint_oracle.c), CPU only.

Pins: (1) without hints, and with hints that restate the scroll layout, a
hinted frame is byte-identical to the reference's scroll frame
(or_scroll_nal / or_compose, themselves pinned by the reference's golden
vectors); (2) decoding a hinted NAL's MV field from the standard
(tests/h264_pslice.py: mb_skip_run, P_Skip 8.4.1.1, median 8.4.1.3 -- or the
reference's predictor for the EXACT mode) gives back the hinted layout."""
import ctypes
import random

from dynhelp import OrCfg, hint_array, random_hints
import h264_pslice as P

EXACT, PSKIP, SPEC = 0, 1, 2


def _cfg(oracle, w, h):
    c = OrCfg()
    oracle.or_cfg_init(ctypes.byref(c), w, h)
    return c


def _offsets(s, n, h, oracle):
    return [oracle.or_synthetic_offset(s, i, h) for i in range(n)]


def _refs(c):
    return [0, 1] + [2 + i for i in range(c.nwp) if c.wp_valid[i]]


def _field(oracle, c, off, rects):
    mbw, mbh = c.w // 16, c.h // 16
    arr, n = hint_array(rects)
    out = (ctypes.c_int32 * (3 * mbw * mbh))()
    rc = oracle.or_hint_field(ctypes.byref(c), off, arr, n, out)
    return rc, [[(out[3 * (y * mbw + x)], 4 * out[3 * (y * mbw + x) + 1], 4 * out[3 * (y * mbw + x) + 2])
                 for x in range(mbw)] for y in range(mbh)]


def _split(buf):
    """Annex-B bytes -> NALs"""
    idx = [i for i in range(len(buf) - 3) if buf[i:i + 4] == b"\x00\x00\x00\x01"]
    return [bytes(buf[a:b]) for a, b in zip(idx, idx[1:] + [len(buf)])]


def test_no_hints_and_restated_layout_equal_scroll_frames(oracle):
    w, h = 320, 720
    buf_a = (ctypes.c_uint8 * (1 << 16))()
    buf_b = (ctypes.c_uint8 * (1 << 16))()
    err = ctypes.c_int()
    for s in range(6):
        ca, cb, cc = _cfg(oracle, w, h), _cfg(oracle, w, h), _cfg(oracle, w, h)
        for off in _offsets(s, 90, h, oracle):
            na = oracle.or_compose(buf_a, len(buf_a), ctypes.byref(ca), off, 0, None)
            nb = oracle.or_compose_hint(buf_b, len(buf_b), ctypes.byref(cb), off, 0, None, 0, EXACT,
                                        ctypes.byref(err))
            assert err.value == 0 and bytes(buf_a[:na]) == bytes(buf_b[:nb]), (s, off)
            # SPEC (standard predictor, no skips) gives the same bytes for the
            # plain layout: a row-uniform field never meets median3's quirk
            cs = OrCfg.from_buffer_copy(cb)
            cs.frame_num -= 1
            ks = oracle.or_hint_scroll_nal(buf_b, len(buf_b), ctypes.byref(cs), off, None, 0, SPEC,
                                           ctypes.byref(err))
            assert err.value == 0 and bytes(buf_b[:ks]) == _split(bytes(buf_a[:na]))[-1], (s, off)
            # the scroll layout restated as two rects (A rows, B rows)
            if oracle.or_needs_waypoint(ctypes.byref(cc), off):
                oracle.or_waypoint_nal(buf_b, len(buf_b), ctypes.byref(cc), off)
            a_end, ra, mva, rb, mvb = (ctypes.c_int() for _ in range(5))
            oracle.or_scroll_regions(ctypes.byref(cc), off, *(ctypes.byref(v) for v in
                                                              (a_end, ra, mva, rb, mvb)))
            rects = [(0, 0, w // 16, a_end.value, ra.value, 0, mva.value),
                     (0, a_end.value, w // 16, h // 16, rb.value, 0, mvb.value)]
            arr, n = hint_array(rects)
            k = oracle.or_hint_scroll_nal(buf_b, len(buf_b), ctypes.byref(cc), off, arr, n, EXACT,
                                          ctypes.byref(err))
            assert err.value == 0
            assert bytes(buf_b[:k]) == _split(bytes(buf_a[:na]))[-1], (s, off)


def _check_modes(oracle, w, h, seed, nframes):
    rng = random.Random(seed)
    buf = (ctypes.c_uint8 * (1 << 18))()
    err = ctypes.c_int()
    nskip_total = 0
    for s in range(3):
        c = _cfg(oracle, w, h)
        for off in _offsets(s + seed, nframes, h, oracle):
            if oracle.or_needs_waypoint(ctypes.byref(c), off):
                oracle.or_waypoint_nal(buf, len(buf), ctypes.byref(c), off)
            rects = random_hints(rng, w // 16, h // 16, _refs(c))
            rc, field = _field(oracle, c, off, rects)
            assert rc == 0
            for mode, pred in ((EXACT, "ref"), (PSKIP, "spec"), (SPEC, "spec")):
                c2 = OrCfg.from_buffer_copy(c)
                arr, n = hint_array(rects)
                k = oracle.or_hint_scroll_nal(buf, len(buf), ctypes.byref(c2), off, arr, n, mode,
                                              ctypes.byref(err))
                assert err.value == 0 and k > 0
                H, got, nskip = P.decode_mv_field(bytes(buf[:k]), w, h, predictor=pred)
                assert got == field, (s, off, mode, rects)
                assert H["nrefs"] == 2 + c.nwp
                if mode != PSKIP:
                    assert nskip == 0
                nskip_total += nskip
            oracle.or_hint_scroll_nal(buf, len(buf), ctypes.byref(c), off, None, 0, EXACT,
                                      ctypes.byref(err))     # advance frame_num
    return nskip_total


def test_hinted_nals_decode_to_the_hinted_field(oracle):
    """EXACT decodes with the reference's predictor, PSKIP with the
    standard's; both give back the layout.  P_Skip runs do occur."""
    assert _check_modes(oracle, 256, 720, 3, 60) > 0
    assert _check_modes(oracle, 640, 480, 11, 40) > 0


def test_chrome_only_frame_is_mostly_skips(oracle):
    w, h = 1280, 720
    c = _cfg(oracle, w, h)
    buf = (ctypes.c_uint8 * (1 << 18))()
    err = ctypes.c_int()
    rects = [(0, 0, 80, 45, 0, 0, 0)]           # the whole picture static on ref A
    arr, n = hint_array(rects)
    k = oracle.or_hint_scroll_nal(buf, len(buf), ctypes.byref(c), 100, arr, n, PSKIP,
                                  ctypes.byref(err))
    H, field, nskip = P.decode_mv_field(bytes(buf[:k]), w, h, predictor="spec")
    assert nskip == 80 * 45 and k < 20
    assert all(f == (0, 0, 0) for row in field for f in row)


def test_invalid_reference_is_an_error(oracle):
    w, h = 256, 256
    c = _cfg(oracle, w, h)
    buf = (ctypes.c_uint8 * (1 << 16))()
    err = ctypes.c_int()
    fn = c.frame_num
    for ref in (2, 5, -1):
        arr, n = hint_array([(1, 1, 3, 3, ref, 0, 0)])
        assert oracle.or_hint_scroll_nal(buf, len(buf), ctypes.byref(c), 40, arr, n, EXACT,
                                         ctypes.byref(err)) == 0
        assert err.value == 1 and c.frame_num == fn
    # a rect outside the picture names nothing
    arr, n = hint_array([(50, 50, 60, 60, 7, 0, 0)])
    assert oracle.or_hint_scroll_nal(buf, len(buf), ctypes.byref(c), 40, arr, n, EXACT,
                                     ctypes.byref(err)) > 0 and err.value == 0
