"""GPU parity of the dynamic-rect residual coder (BASELINE configs 3-5):
k_plan (state) -> k_dyn_rows -> k_dyn_code_general -> k_dyn_row -> k_dyn_static -> k_dyn_epfix /
k_dyn_epscan -> k_plan (size) -> k_emit -> k_dyn_emit_gather / k_dyn_emit,
through the C ABI, against the CPU restatement oracle/dyn_oracle.c
(or_compose_dyn), byte for byte.  The reference has no implementation of
this path, so these bits are pinned only by the restatement, which
tests/test_dyn_oracle.py checks with an independent decoder and the
reference's own CAVLC parser ("parity unpinned").
Run on an MI355X: -m gpu."""
import ctypes

import numpy as np
import pytest

from conftest import synthetic_offsets
from dynhelp import qp_field, OrCfg, Pic, Rect, Refs, StripedRefs, rect_source, split_nals

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(scroll):
    if scroll.device_count() < 1:
        pytest.fail("no gfx950 device: " + scroll.last_error())
    return scroll


class ArrayRefs:
    """Reference pictures A, B from numpy planes (I420 bytes for the GPU,
    or_refs for the oracle)."""

    def __init__(self, planes):               # planes: [(y, u, v), (y, u, v)] uint8 arrays
        self.planes = [tuple(np.ascontiguousarray(p, dtype=np.uint8) for p in pic) for pic in planes]
        h, w = self.planes[0][0].shape
        self.pics = [Pic(w, h, p[0].ctypes.data, p[1].ctypes.data, p[2].ctypes.data)
                     for p in self.planes]
        self.refs = Refs()
        self.refs.ab[0] = ctypes.pointer(self.pics[0])
        self.refs.ab[1] = ctypes.pointer(self.pics[1])

    def i420(self, k):
        return b"".join(p.tobytes() for p in self.planes[k])


def striped_refs(oracle, w, h):
    sr = StripedRefs(oracle, w, h)
    planes = []
    for y, u, v in sr.planes:
        planes.append((np.frombuffer(bytes(y), np.uint8).reshape(h, w),
                       np.frombuffer(bytes(u), np.uint8).reshape(h // 2, w // 2),
                       np.frombuffer(bytes(v), np.uint8).reshape(h // 2, w // 2)))
    return ArrayRefs(planes)


def random_refs(w, h, seed):
    rng = np.random.default_rng(seed)
    return ArrayRefs([(rng.integers(0, 256, (h, w)), rng.integers(0, 256, (h // 2, w // 2)),
                       rng.integers(0, 256, (h // 2, w // 2))) for _ in range(2)])


def synth_source(oracle, S, F, rect, t0=0):
    """[S][F][384 w h] of the documented synthetic source (dyn_oracle.h)"""
    n = 384 * rect.w * rect.h
    out = np.zeros((S, F, n), np.uint8)
    for s in range(S):
        for t in range(F):
            out[s, t] = np.frombuffer(bytes(rect_source(oracle, s, t0 + t, rect)), np.uint8)
    return out


def oracle_streams(oracle, w, h, offsets, rect, src, R, mode=0, frame_num=2, waypoints=()):
    S, F = offsets.shape
    oracle.or_compose_dyn.restype = ctypes.c_size_t
    buf = (ctypes.c_uint8 * (16 << 20))()
    nwp = ctypes.c_int()
    outs = []
    for s in range(S):
        cfg = OrCfg()
        oracle.or_cfg_init(ctypes.byref(cfg), w, h)
        cfg.frame_num = frame_num
        for i, (o, lt, v) in enumerate(waypoints):
            cfg.wp_off[i], cfg.wp_lt[i], cfg.wp_valid[i] = o, lt, v
        cfg.nwp = len(waypoints)
        o = bytearray()
        for t in range(F):
            sp = np.ascontiguousarray(src[s, t])
            n = oracle.or_compose_dyn(buf, len(buf), ctypes.byref(cfg), int(offsets[s, t]), mode,
                                      ctypes.byref(rect), sp.ctypes.data_as(ctypes.c_void_p),
                                      ctypes.byref(R.refs), ctypes.byref(nwp))
            assert n > 0
            o += bytes(buf[:n])
        outs.append(bytes(o))
    return outs


def gpu_streams(gpu, w, h, offsets, rect, R, src=None, synth=False, mode=0, chunks=None,
                arena=None, slot=0, waypoints=(), shared_refs=True, per_stream_refs=None, debug=0,
                stream_qp=None):
    S, F = offsets.shape
    b = gpu.Batch(S, F, arena or (8 << 20), mode=mode)
    if debug:
        b.set_debug(debug)
    for _ in range(S):
        b.add_stream(gpu.make_config(w, h, waypoints=waypoints))
    b.set_dyn_rect(rect.x0, rect.y0, rect.w, rect.h, slot)
    if rect.qp:
        b.set_dyn_qp(0 if rect.qp == -1 else rect.qp)
    for s, q in (stream_qp or {}).items():
        b.set_dyn_qp(q, stream=s)
    if shared_refs:
        b.set_dyn_refs(R.i420(0), R.i420(1))
    for s, Rs in (per_stream_refs or {}).items():
        b.set_dyn_refs(Rs.i420(0), Rs.i420(1), stream=s)
    pos = 0
    for n in (chunks or [F]):
        b.set_offsets(np.ascontiguousarray(offsets[:, pos:pos + n]))
        if synth:
            b.dyn_source_synth(n, 0, pos)
        else:
            b.set_dyn_source(np.ascontiguousarray(src[:, pos:pos + n]).tobytes(), n)
        b.compose(n)
        rc = b.sync()
        if rc != 0:
            return b, rc
        pos += n
    return b, 0


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


def test_dyn_small_with_waypoints(gpu, oracle):
    w, h = 64, 512
    rect = Rect(1, 3, 2, 20)
    offs = synthetic_offsets(3, 40, h)
    offs[0] = np.arange(480, 520)                     # crosses 496: a waypoint
    offs[1] = np.arange(1010, 970, -1)                # crosses 992: a second one
    R = striped_refs(oracle, w, h)
    src = synth_source(oracle, 3, 40, rect)
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, src)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    for s in (0, 1):
        nals = b.nals(s)
        assert any(k == 1 and sl == 0 for k, _, _, sl in nals)   # waypoints: run layout
        assert sum(sl == 2 for _, _, _, sl in nals) == 40         # every scroll NAL dynamic


def test_dyn_full_frame_random_pixels(gpu, oracle):
    """rect = whole picture (no left/top neighbours at the edges), random
    reference and source pixels (large residuals, long level codes)"""
    w, h = 96, 96
    rect = Rect(0, 0, 6, 6)
    rng = np.random.default_rng(7)
    S, F = 2, 12
    offs = rng.integers(-200, 300, (S, F)).astype(np.int32)
    R = random_refs(w, h, 1)
    src = rng.integers(0, 256, (S, F, 384 * 36)).astype(np.uint8)
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, src)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)


@pytest.mark.parametrize("rect", [(0, 0, 1, 20), (3, 4, 13, 3), (7, 0, 12, 20), (19, 19, 1, 1)])
def test_dyn_rect_shapes(gpu, oracle, rect):
    """window splits across rows, rect width 1 (TotalCoeff row ring), rects
    touching every picture edge"""
    w, h = 320, 320
    rc_ = Rect(*rect)
    S, F = 2, 6
    offs = synthetic_offsets(S, F, h, first_stream=5)
    R = random_refs(w, h, 3)
    src = synth_source(oracle, S, F, rc_)
    want = oracle_streams(oracle, w, h, offs, rc_, src, R)
    b, rc = gpu_streams(gpu, w, h, offs, rc_, R, src)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)


def test_dyn_720p_config3_device_synth(gpu, oracle):
    """BASELINE config 3 geometry: 1280x720, 360x360 rect at MB (28, 10);
    the source generated on the device (k_dyn_synth) must equal the
    documented generator, and the NALs the oracle's"""
    w, h = 1280, 720
    rect = Rect(28, 10, 25, 25)
    S, F = 2, 6
    offs = synthetic_offsets(S, F, h)
    R = striped_refs(oracle, w, h)
    src = synth_source(oracle, S, F, rect)
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, synth=True)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    eps = []
    for s in range(S):
        for t in range(F):
            rb, ep = b.dyn_frame_info(s, t)
            assert rb > 20000
            eps.append(ep)
    assert any(eps)                                   # emulation prevention exercised
    sizes = [sz for k, _, sz, sl in b.nals(0) if sl == 2]
    assert len(sizes) == F


def test_dyn_4k_config5_many_refs(gpu, oracle):
    """BASELINE config 5 geometry: 3840x2160 with the 720x720 rect (47x47 MBs);
    offsets walk past 496 / 992 / 1488 / 1984, so the slice carries up to 6
    reference pictures (ue(ref_idx)) and region-A rows predict through
    waypoint chains"""
    w, h = 3840, 2160
    rect = Rect(96, 44, 47, 47)
    offs = np.array([[400, 496, 700, 992, 1300, 1488, 1900, 1984, 2100]], np.int32)
    R = random_refs(w, h, 8)
    src = synth_source(oracle, 1, offs.shape[1], rect)
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, src, arena=64 << 20)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    assert sum(k == 1 for k, _, _, _ in b.nals(0)) == 4          # four waypoint NALs


def test_dyn_chunked_composes_and_experiment_mode(gpu, oracle):
    w, h = 64, 512
    rect = Rect(0, 5, 4, 9)
    S, F = 3, 30
    offs = synthetic_offsets(S, F, h, first_stream=1)
    R = random_refs(w, h, 11)
    src = synth_source(oracle, S, F, rect)
    for mode in (0, 1):
        want = oracle_streams(oracle, w, h, offs, rect, src, R, mode=mode)
        b, rc = gpu_streams(gpu, w, h, offs, rect, R, synth=True, mode=mode, chunks=[7, 1, 22])
        assert rc == 0, gpu.last_error()
        check_equal(b, want)
        b.close()


def test_dyn_half_pel_waypoint_chain(gpu, oracle):
    """a resumed config with a waypoint at an odd offset: its rows predict at
    half-pel chroma positions, which only the general path (k_dyn_code_general
    -> k_dyn_row<true>) does"""
    w, h = 64, 1024
    rect = Rect(1, 0, 2, 48)
    wps = [(501, 2, 1)]
    S, F = 1, 6
    offs = np.array([[600, 610, 777, 900, 505, 996]], np.int32)
    R = random_refs(w, h, 5)
    src = synth_source(oracle, S, F, rect)
    want = oracle_streams(oracle, w, h, offs, rect, src, R, waypoints=wps)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, src, waypoints=wps)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)


def test_dyn_per_stream_refs(gpu, oracle):
    w, h = 96, 64
    rect = Rect(1, 1, 3, 2)
    S, F = 3, 5
    offs = synthetic_offsets(S, F, h)
    Rs = [random_refs(w, h, 20 + s) for s in range(S)]
    src = synth_source(oracle, S, F, rect)
    want = [oracle_streams(oracle, w, h, offs[s:s + 1], rect, src[s:s + 1], Rs[s])[0]
            for s in range(S)]
    b, rc = gpu_streams(gpu, w, h, offs, rect, Rs[0], src, shared_refs=True,
                        per_stream_refs={1: Rs[1], 2: Rs[2]})
    assert rc == 0, gpu.last_error()
    check_equal(b, want)


def test_dyn_staging_overflow_commits_nothing(gpu, oracle):
    w, h = 96, 96
    rect = Rect(0, 0, 6, 6)
    rng = np.random.default_rng(3)
    offs = np.zeros((1, 2), np.int32)
    R = random_refs(w, h, 2)
    src = rng.integers(0, 256, (1, 2, 384 * 36)).astype(np.uint8)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, src, slot=1024)
    assert rc == gpu.SCROLL_ERR_OVERFLOW
    assert b.output_size(0) == 0


def test_dyn_large_nal_emit_path(gpu, oracle):
    """k_dyn_emit, the path for NALs with more EP bytes than the gather's
    list holds (2,048; no bench NAL reaches it): SCROLL_DEBUG_DYN_EPCAP4
    caps the list at 4, so every NAL with more EP bytes -- most config-3
    NALs, and the random-pixel ones -- goes through k_dyn_emit's LDS line
    buffer and scans, and the bytes must not change"""
    w, h = 1280, 720
    rect = Rect(28, 10, 25, 25)
    S, F = 2, 6
    offs = synthetic_offsets(S, F, h)
    R = striped_refs(oracle, w, h)
    src = synth_source(oracle, S, F, rect)
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, synth=True, debug=gpu.SCROLL_DEBUG_DYN_EPCAP4)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    eps = [b.dyn_frame_info(s, t)[1] for s in range(S) for t in range(F)]
    assert sum(e > 4 for e in eps) >= 2, eps          # the large-NAL path ran

    w, h = 96, 96
    rect = Rect(0, 0, 6, 6)
    rng = np.random.default_rng(17)
    S, F = 2, 10
    offs = rng.integers(-200, 300, (S, F)).astype(np.int32)
    R = random_refs(w, h, 4)
    src = rng.integers(0, 256, (S, F, 384 * 36)).astype(np.uint8)
    src[:, ::3] = 0                                   # zero pictures: long zero-bit runs
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, src, debug=gpu.SCROLL_DEBUG_DYN_EPCAP4)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)


def test_dyn_ep_windows(gpu, oracle):
    """the EP-position path of the whole-picture rects (round 6: their
    heaviest NALs hold more EP bytes than 2,048 -- a third of p720full's
    frames, ~2,200): k_dyn_epfix's 8,192-entry set and list, and
    k_dyn_gather taking the sorted list window by window into LDS.
    SCROLL_DEBUG_DYN_EPWIN puts any rect on that path with 7 positions per
    window, so every NAL with more EP bytes is gathered in several windows
    (and split over several workgroups the windows cross); bytes unchanged"""
    w, h = 1280, 720
    rect = Rect(28, 10, 25, 25)
    S, F = 2, 6
    offs = synthetic_offsets(S, F, h)
    R = striped_refs(oracle, w, h)
    src = synth_source(oracle, S, F, rect)
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, synth=True, debug=gpu.SCROLL_DEBUG_DYN_EPWIN)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    eps = [b.dyn_frame_info(s, t)[1] for s in range(S) for t in range(F)]
    assert sum(e > 7 for e in eps) >= 2, eps          # the window path ran

    w, h = 96, 96
    rect = Rect(0, 0, 6, 6)
    rng = np.random.default_rng(23)
    S, F = 2, 10
    offs = rng.integers(-200, 300, (S, F)).astype(np.int32)
    R = random_refs(w, h, 4)
    src = rng.integers(0, 256, (S, F, 384 * 36)).astype(np.uint8)
    src[:, ::3] = 0                                   # zero pictures: long zero-bit runs
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, src, debug=gpu.SCROLL_DEBUG_DYN_EPWIN)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)


def test_dyn_spill_pool_runs_out_and_grows(gpu, oracle):
    """the row stage is sized for typical rows (SCROLL_DYN_ROW_KBITS per MB);
    a row past its slot takes a spill slot (k_dyn_row), and the pool holds
    1/32 of the rect rows.  Random reference pictures make EVERY row spill:
    a 16 x 40-frame config-3 batch runs the pool out -- the compose fails
    with SCROLL_ERR_OVERFLOW and no stream commits anything (also those whose
    own rows all got slots), the batch grows its pools, and the same compose
    again is bit-exact (every row through a spill slot)"""
    w, h = 1280, 720
    rect = Rect(28, 10, 25, 25)
    S, F = 16, 40
    offs = synthetic_offsets(S, F, h)
    R = random_refs(w, h, 12)
    b = gpu.Batch(S, F, 16 << 20)
    for _ in range(S):
        b.add_stream(gpu.make_config(w, h))
    b.set_dyn_rect(rect.x0, rect.y0, rect.w, rect.h)
    b.set_dyn_refs(R.i420(0), R.i420(1))
    b.set_offsets(offs)
    b.dyn_source_synth(F, 0, 0)
    b.compose(F)
    rc = b.sync()
    assert rc == -4, gpu.last_error()                               # SCROLL_ERR_OVERFLOW
    assert "grown" in gpu.last_error()
    assert all(b.output_size(s) == 0 for s in range(S))             # nothing committed
    b.compose(F)
    assert b.sync() == 0, gpu.last_error()
    src = synth_source(oracle, S, F, rect)
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    check_equal(b, want)
    b.close()


def test_dyn_row_handoff_wait_is_bounded(gpu, oracle):
    """k_dyn_row's wait for the row above's TotalCoeffs is bounded: with
    SCROLL_DEBUG_DYN_NOPUBLISH rect row 0 of stream 0, frame 0 never
    publishes, row 1's wait expires (50 ms), stream 0 fails with
    SCROLL_ERR_DEVICE and commits nothing, and the other streams stay
    bit-exact; the next compose without the flag succeeds"""
    w, h = 1280, 720
    rect = Rect(28, 10, 25, 25)
    S, F = 3, 4
    offs = synthetic_offsets(S, F, h)
    R = striped_refs(oracle, w, h)
    src = synth_source(oracle, S, F, rect)
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, synth=True, debug=gpu.SCROLL_DEBUG_DYN_NOPUBLISH)
    assert rc == gpu.SCROLL_ERR_DEVICE, (rc, gpu.last_error())
    assert "stream 0" in gpu.last_error()
    assert b.output_size(0) == 0
    for s in (1, 2):
        assert b.output(s) == want[s], s
    b.set_debug(0)                                    # recovers: stream 0 composes again
    b.set_offsets(np.ascontiguousarray(offs[:, :1]))
    b.dyn_source_synth(1, 0, 0)
    b.compose(1)
    assert b.sync() == 0, gpu.last_error()
    assert len(b.output(0)) > 20000
    b.close()


@pytest.mark.parametrize("geom", [((1280, 720), (28, 10, 25, 25)), ((320, 320), (0, 0, 1, 20)),
                                  ((96, 96), (0, 0, 6, 6))])
def test_dyn_round3_gather_still_exact(gpu, oracle, geom):
    """SCROLL_DEBUG_DYN_GATHER1: the round-3 gather (k_dyn_emit_gather) in
    place of k_dyn_gather gives the same bytes (config-3 geometry, a width-1
    rect with tiny row groups, EP-dense random pixels)"""
    (w, h), r = geom
    rect = Rect(*r)
    S, F = 2, 5
    offs = synthetic_offsets(S, F, h)
    if w == 96:
        R = random_refs(w, h, 1)
        src = np.random.default_rng(5).integers(0, 256, (S, F, 384 * rect.w * rect.h)).astype(np.uint8)
    else:
        R = striped_refs(oracle, w, h)
        src = synth_source(oracle, S, F, rect)
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, src, debug=gpu.SCROLL_DEBUG_DYN_GATHER1)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)


@pytest.mark.parametrize("qp", [0, 12, 18, 22, 30, 37, 51])
def test_dyn_rect_qp(gpu, oracle, scroll, qp):
    """scroll_batch_set_dyn_qp: luma at qp, chroma at QPc, slice_qp_delta qp -
    26 in the dynamic NALs (waypoints on the way stay the reference's), at
    the config-3 geometry with random references (the largest levels) and
    through the general path's half-pel chroma waypoints; below 22 every NAL
    takes the general path with 16-bit levels"""
    w, h = 1280, 720
    rect = Rect(28, 10, 25, 25, qp_field(qp))
    S, F = 2, 8
    offs = synthetic_offsets(S, F, h, first_stream=3)
    offs[1] = np.arange(490, 498)
    R = random_refs(w, h, 7 + qp)
    src = synth_source(oracle, S, F, rect)
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    b, rc = gpu_streams(gpu, w, h, offs, rect, R, src)
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    with pytest.raises(Exception):
        b.set_dyn_qp(52)
    b.close()


def test_dyn_rect_qp_per_stream(gpu, oracle, scroll):
    """scroll_batch_set_dyn_qp_stream: one batch, each stream at its own QP
    (16-bit general path and int8 k_dyn_row path side by side), each equal
    to the oracle at that QP; a later batch-wide QP overrides them all"""
    w, h = 1280, 720
    S, F = 5, 6
    qps = [12, 40, 18, 26, 0]
    base = Rect(28, 10, 25, 25)
    offs = synthetic_offsets(S, F, h, first_stream=1)
    R = striped_refs(oracle, w, h)
    src = synth_source(oracle, S, F, base)
    want = []
    for s, q in enumerate(qps):
        rs = Rect(28, 10, 25, 25, qp_field(q))
        want += oracle_streams(oracle, w, h, offs[s:s + 1], rs, src[s:s + 1], R)
    b, rc = gpu_streams(gpu, w, h, offs, base, R, src, stream_qp=dict(enumerate(qps)))
    assert rc == 0, gpu.last_error()
    check_equal(b, want)
    b.close()


def test_dyn_qp_with_hints_and_deblocking(gpu, scroll):
    """QP is accepted under hints (per frame too); a stream with the
    deblocking filter on keeps QP 26"""
    b = gpu.Batch(2, 2, 1 << 20)
    b.add_stream(gpu.make_config(320, 320))
    b.add_stream(gpu.make_config(320, 320, deblock=0))
    b.set_dyn_rect(1, 1, 2, 2)
    b.set_dyn_qp(30, stream=0)
    with pytest.raises(Exception):
        b.set_dyn_qp(30, stream=1)
    with pytest.raises(Exception):
        b.set_dyn_qp(30)
    b.set_hints(0, 0, [], 1)
    b.set_dyn_qp_at(0, 1, 12)
    with pytest.raises(Exception):
        b.set_dyn_qp_at(1, 1, 12)
    b.set_dyn_qp_at(1, 1, 26)
    b.close()


def test_dyn_lite_timing_bytes_and_pairs(gpu, oracle):
    """scroll_batch_enable_timing(b, 2): only the dominant kernel's event
    pair (dyn code, also reported as dyn stage) is recorded; the composed
    bytes are the same as with full timing and with none"""
    w, h = 128, 256
    rect = Rect(2, 3, 4, 6)
    S, F = 4, 6
    offs = synthetic_offsets(S, F, h)
    R = striped_refs(oracle, w, h)
    src = synth_source(oracle, S, F, rect)
    want = oracle_streams(oracle, w, h, offs, rect, src, R)
    for mode in (0, 1, 2):
        b = gpu.Batch(S, F, 8 << 20)
        for _ in range(S):
            b.add_stream(gpu.make_config(w, h))
        b.set_dyn_rect(rect.x0, rect.y0, rect.w, rect.h, 0)
        b.set_dyn_refs(R.i420(0), R.i420(1))
        b.set_offsets(np.ascontiguousarray(offs))
        b.set_dyn_source(np.ascontiguousarray(src).tobytes(), F)
        if mode:
            b.enable_timing(True, lite=mode == 2)
            b.kernel_stats_ex()
        b.compose(F)
        assert b.sync() == 0, gpu.last_error()
        check_equal(b, want)
        if mode:
            ms, n = b.kernel_stats_ex()
            assert n == 1
            plan, emit, stage, demit, code, pack = ms
            assert code > 0 and stage > 0
            if mode == 2:
                assert plan == 0 and emit == 0 and demit == 0 and pack == 0 and stage == code
                assert b.kernel_ms(4) == -1.0           # lite: no per-kernel pairs
            else:
                assert plan > 0 and demit > 0
        b.close()


@pytest.mark.parametrize("w,h,rect,S,F,refs", [
    (1280, 720, (0, 0, 80, 45), 3, 6, "striped"),     # a whole 720p frame (ngroups 47)
    (1280, 720, (0, 0, 80, 45), 2, 3, "random"),      # noise: spill slots, multi-pass bit windows
    (3840, 2160, (0, 0, 240, 135), 1, 3, "striped"),  # a whole 4K frame: 137 row groups, 142 KB LDS rows
])
def test_dyn_rect_whole_frame(gpu, oracle, scroll, w, h, rect, S, F, refs):
    """the rect cap lifted to the whole frame (MASTER_DESIGN.md:220's full
    conventional encode as the hint fallback): every MB dynamic, rows of 80
    / 240 MBs through k_dyn_row (several bit-window passes, dynamic LDS past
    64 KB), more than 64 row groups through k_dyn_epfix / k_dyn_gather,
    equal to oracle/dyn_oracle.c"""
    rc = Rect(*rect)
    offs = synthetic_offsets(S, F, h, first_stream=2)
    R = striped_refs(oracle, w, h) if refs == "striped" else random_refs(w, h, 5)
    src = synth_source(oracle, S, F, rc)
    want = oracle_streams(oracle, w, h, offs, rc, src, R)
    b, rcode = gpu_streams(gpu, w, h, offs, rc, R, src, arena=(64 << 20) * F)
    assert rcode == 0, gpu.last_error()
    check_equal(b, want)
    b.close()
