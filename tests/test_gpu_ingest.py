"""GPU stream ingest: batched composer_init +
composer_write_header through scroll_batch_ingest, against the CPU
restatement or_composer_run (oracle/scroll_oracle.c, pinned to the
reference composer's golden outputs) byte for byte -- the header (SPS, PPS,
IDR A rewritten, B rewritten as a non-IDR I frame) and the scroll frames
composed after it.  Reference files vary what the parser must handle: the
reference-style I_PCM refs, POC type 0 / other log2 fields / no deblocking
control / High-profile SPS, emulation-prevention-heavy pixel data (zero
stripes), 3-byte start codes, extra NAL units, trailing zeros, and the
error rules (missing NAL units, an empty NAL unit stopping the parser, size
mismatch).  Run on an MI355X: -m gpu."""
import ctypes

import numpy as np
import pytest

from dynhelp import OrCfg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(scroll):
    if scroll.device_count() < 1:
        pytest.fail("no gfx950 device: " + scroll.last_error())
    return scroll


class BW:
    """MSB-first bit writer (test-side SPS / PPS)"""

    def __init__(self):
        self.b = []

    def u(self, v, n):
        self.b += [(v >> (n - 1 - i)) & 1 for i in range(n)]

    def ue(self, v):
        v += 1
        n = v.bit_length()
        self.u(0, n - 1)
        self.u(v, n)

    def se(self, v):
        self.ue(2 * v - 1 if v > 0 else -2 * v)

    def rbsp(self):
        b = self.b + [1]
        b += [0] * (-len(b) % 8)
        return bytes(int("".join(map(str, b[i:i + 8])), 2) for i in range(0, len(b), 8))


def ebsp(rbsp):
    out, z = bytearray(), 0
    for v in rbsp:
        if z >= 2 and v <= 3:
            out.append(3)
            z = 0
        out.append(v)
        z = z + 1 if v == 0 else 0
    return bytes(out)


def nal(ref_idc, typ, rbsp, sc4=True):
    return (b"\0\0\0\1" if sc4 else b"\0\0\1") + bytes([(ref_idc << 5) | typ]) + ebsp(rbsp)


def sps(w, h, log2_mfn=4, poc_type=2, log2_poc=4, profile=66):
    b = BW()
    b.u(profile, 8); b.u(0xc0, 8); b.u(40, 8); b.ue(0)
    if profile == 100:
        b.ue(1); b.ue(0); b.ue(0); b.u(0, 1); b.u(0, 1)
    b.ue(log2_mfn - 4); b.ue(poc_type)
    if poc_type == 0:
        b.ue(log2_poc - 4)
    b.ue(4); b.u(0, 1); b.ue(w // 16 - 1); b.ue(h // 16 - 1)
    b.u(1, 1); b.u(1, 1); b.u(0, 1); b.u(0, 1)
    return b.rbsp()


def pps(deblock=1, nref_m1=0, qp_off=0):
    b = BW()
    b.ue(0); b.ue(0); b.u(0, 1); b.u(0, 1); b.ue(0); b.ue(nref_m1); b.ue(0); b.u(0, 1); b.u(0, 2)
    b.se(qp_off); b.se(0); b.se(0); b.u(deblock, 1); b.u(0, 1); b.u(0, 1)
    return b.rbsp()


def idr_nal(oracle, w, h, yuv, log2_mfn=4, poc_type=2, log2_poc=4, deblock=1, idr_id=0):
    """an I_PCM IDR slice (experiment's writer, oracle/scroll_oracle.c) with
    the given parse parameters, 3 stripes of yuv[0:3], [3:6], [6:9]"""
    c = OrCfg()
    oracle.or_cfg_init(ctypes.byref(c), w, h)
    c.log2_mfn, c.poc_type, c.log2_poc, c.deblock, c.idr_pic_id = log2_mfn, poc_type, log2_poc, deblock, idr_id
    buf = (ctypes.c_uint8 * (w * h * 3 + 4096))()
    n = oracle.or_ipcm_striped(buf, len(buf), ctypes.byref(c), 0, (ctypes.c_uint8 * 9)(*yuv))
    return bytes(buf[:n])


def ref_file(oracle, w, h, which):
    buf = (ctypes.c_uint8 * (w * h * 3 + 4096))()
    n = oracle.or_ipcm_ref_file(buf, len(buf), w, h, which)
    return bytes(buf[:n])


def expected(oracle, a, b, nframes=0, speed=4):
    cap = 2 * (len(a) + len(b)) + 4096 + nframes * 64 * (1 + len(a) // 4096)
    buf = (ctypes.c_uint8 * cap)()
    n = oracle.or_composer_run(buf, cap, a, len(a), b, len(b), nframes, speed)
    return bytes(buf[:n])


def variant_files(oracle, w, h, k):
    """reference files exercising the parser; k picks the variant"""
    v = k % 5
    if v == 0:
        return ref_file(oracle, w, h, 0), ref_file(oracle, w, h, 1)
    if v == 1:        # POC type 0, log2 fields, no deblocking control, idr_pic_id, EP-heavy
        pa = dict(log2_mfn=6, poc_type=0, log2_poc=7, deblock=0, idr_id=5)
        head = nal(3, 7, sps(w, h, 6, 0, 7)) + nal(3, 8, pps(0))
        a = head + idr_nal(oracle, w, h, [0, 0, 0, 0, 1, 2, 3, 0, 0], **pa)
        b = head + idr_nal(oracle, w, h, [1, 0, 0, 0, 0, 0, 2, 3, 1], **pa)
        return a, b
    if v == 2:        # High profile SPS, 3-byte start codes, AUD + SEI first, trailing zeros
        aud = b"\0\0\1\x09\xf0"
        sei = nal(0, 6, bytes([5, 1, 0x80]), sc4=False)
        head = aud + sei + nal(3, 7, sps(w, h, profile=100), sc4=False) + b"\0\0" + \
            nal(3, 8, pps(1, qp_off=-2), sc4=False)
        a = head + idr_nal(oracle, w, h, [16, 128, 128, 235, 128, 128, 0, 0, 0]) + b"\0\0\0"
        b = head + idr_nal(oracle, w, h, [0, 0, 3, 200, 50, 60, 0, 3, 0])
        return a, b
    if v == 3:        # a second IDR and a second SPS later in the file are ignored
        a = ref_file(oracle, w, h, 0) + nal(3, 7, sps(w, h, 5)) + idr_nal(oracle, w, h, [9] * 9)
        b = ref_file(oracle, w, h, 1) + ref_file(oracle, w, h, 0)
        return a, b
    a = ref_file(oracle, w, h, 1)   # A and B swapped
    b = ref_file(oracle, w, h, 0)
    return a, b


def check_ingest(gpu, oracle, pairs, nframes=0, speed=4, arena=8 << 20):
    S = len(pairs)
    b = gpu.Batch(S, max(nframes, 1), arena)
    first = b.ingest(pairs)
    assert first == 0
    if nframes:
        offs = np.array([[oracle.or_tri(i * speed, int(b.config(s).height)) for i in range(nframes)]
                         for s in range(S)], np.int32)
        b.set_offsets(offs)
        b.compose(nframes)
        assert b.sync() == 0, gpu.last_error()
    for s, (ra, rb) in enumerate(pairs):
        want = expected(oracle, ra, rb, nframes, speed)
        assert want, "oracle refused the files"
        got = b.output(s)
        assert got == want, (s, len(got), len(want),
                             next((i for i, (x, y) in enumerate(zip(got, want)) if x != y), None))
    return b


def test_ingest_reference_refs_then_compose(gpu, oracle):
    """the reference-style I_PCM refs at three sizes; header + 60 composed frames"""
    pairs = [(ref_file(oracle, w, h, 0), ref_file(oracle, w, h, 1))
             for w, h in ((1280, 720), (640, 480), (320, 240), (1280, 720))]
    b = check_ingest(gpu, oracle, pairs, nframes=60, arena=16 << 20)
    c = b.config(2)
    assert (c.width, c.height, c.log2_max_frame_num, c.pic_order_cnt_type) == (320, 240, 4, 2)
    b.close()


@pytest.mark.parametrize("w,h", [(320, 240), (1280, 720)])
def test_ingest_parser_variants(gpu, oracle, w, h):
    pairs = [variant_files(oracle, w, h, k) for k in range(10)]
    b = check_ingest(gpu, oracle, pairs, nframes=8, arena=8 << 20)
    b.close()


def test_ingest_appends_after_existing_streams(gpu, oracle):
    w, h = 320, 240
    b = gpu.Batch(6, 4, 1 << 20)
    b.add_stream(gpu.make_config(w, h))
    first = b.ingest([variant_files(oracle, w, h, k) for k in (0, 1)])
    assert first == 1 and b.num_streams == 3
    for k, s in enumerate((1, 2)):
        assert b.output(s) == expected(oracle, *variant_files(oracle, w, h, k))
    first = b.ingest([variant_files(oracle, w, h, 2)])
    assert first == 3
    assert b.output(3) == expected(oracle, *variant_files(oracle, w, h, 2))
    b.close()


def test_ingest_errors_add_no_stream(gpu, oracle, scroll):
    w, h = 320, 240
    a, bb = ref_file(oracle, w, h, 0), ref_file(oracle, w, h, 1)
    sps_pps = nal(3, 7, sps(w, h)) + nal(3, 8, pps())
    bad = [
        (sps_pps, bb),                                       # no IDR in A
        (a, ref_file(oracle, 640, 480, 1)),                  # sizes differ
        (nal(3, 7, sps(w, h)) + b"\0\0\1\0\0\1" + a, bb),    # an empty NAL stops the parser
        (nal(3, 7, sps(w, h, poc_type=1)) + a, bb),          # POC type 1 refused
    ]
    for ra, rb in bad:
        assert expected(oracle, ra, rb) == b""               # the reference refuses too
        b = gpu.Batch(2, 1, 1 << 20)
        with pytest.raises(RuntimeError):
            b.ingest([(a, bb), (ra, rb)])
        assert "new stream 1" in gpu.last_error()
        assert b.num_streams == 0
        b.close()
    b = gpu.Batch(1, 1, 4096)                                # arena too small for the header
    with pytest.raises(RuntimeError):
        b.ingest([(a, bb)])
    b.close()


def test_ingest_segmented_matches_one_workgroup_path(gpu, oracle, monkeypatch):
    """the segmented path -- by default one pass (each 16 KB EBSP segment
    summarised, placed by look-back over the segments before it and written
    by one workgroup), or round 4's three passes with the write pass reading
    the summary pass's bytes (SCROLL_INGEST_THREEPASS) or decoding again
    (SCROLL_INGEST_RECOMPUTE) -- and the one-workgroup-per-stream path
    (SCROLL_INGEST_SERIAL) write the same bytes; EP-heavy 1280x720 files put
    zero runs of both parities across segment boundaries"""
    w, h = 1280, 720
    pairs = [variant_files(oracle, w, h, k) for k in (1, 2, 3, 6, 7)]
    outs = []
    for env in (None, "SCROLL_INGEST_THREEPASS", "SCROLL_INGEST_RECOMPUTE", "SCROLL_INGEST_SERIAL"):
        for e in ("SCROLL_INGEST_THREEPASS", "SCROLL_INGEST_RECOMPUTE", "SCROLL_INGEST_SERIAL"):
            monkeypatch.delenv(e, raising=False)
        if env:
            monkeypatch.setenv(env, "1")
        b = check_ingest(gpu, oracle, pairs, nframes=0, arena=8 << 20)
        outs.append([b.output(s) for s in range(len(pairs))])
        b.close()
    assert outs[0] == outs[1] == outs[2] == outs[3]


def test_ingest_one_pass_many_streams(gpu, oracle):
    """the one-pass path's look-back under load: 48 new streams of 1280x720
    files (about 90 segments each, A's chain continuing into B's), every
    header byte-identical to the oracle's"""
    w, h = 1280, 720
    pairs = [variant_files(oracle, w, h, k % 8) for k in range(48)]
    b = check_ingest(gpu, oracle, pairs, nframes=0, arena=8 << 20)
    b.close()


def _striped_i420(oracle, w, h, which):
    from dynhelp import StripedRefs
    sr = StripedRefs(oracle, w, h)
    return b"".join(bytes(p) for p in sr.planes[which]), sr


def test_ingest_then_dynamic_rect_at_default_qp(gpu, oracle):
    """ingested streams carry the batch's rect QP (26 by default): composed
    with the dynamic rect -- ingested before and after scroll_batch_set_dyn_rect
    -- their bytes are the header the oracle's composer_init +
    composer_write_header writes, then the oracle's dynamic-rect NALs
    (oracle/dyn_oracle.c) at QP 26.  (Round 5 left an ingested stream's QP
    at 0: slice_qp_delta -26 on the general path.)"""
    from dynhelp import Rect, rect_source
    from test_gpu_dyn import oracle_streams, synth_source
    w, h, F = 320, 240, 6
    rect = Rect(3, 2, 6, 5)
    a, bb = ref_file(oracle, w, h, 0), ref_file(oracle, w, h, 1)
    ia, sr = _striped_i420(oracle, w, h, 0)
    ib, _ = _striped_i420(oracle, w, h, 1)
    b = gpu.Batch(4, F, 8 << 20)
    try:
        assert b.ingest([(a, bb)]) == 0                  # before the rect exists
        b.set_dyn_rect(rect.x0, rect.y0, rect.w, rect.h)
        b.set_dyn_refs(ia, ib)
        assert b.ingest([(a, bb), (a, bb)]) == 1          # after it
        S = b.num_streams
        offs = np.array([[oracle.or_tri(i * 4 + 13 * s, h) for i in range(F)] for s in range(S)], np.int32)
        src = synth_source(oracle, S, F, rect)
        b.set_offsets(offs)
        b.set_dyn_source(np.ascontiguousarray(src).tobytes(), F)
        b.compose(F)
        assert b.sync() == 0, gpu.last_error()
        head = expected(oracle, a, bb, 0)
        want = oracle_streams(oracle, w, h, offs, rect, src, sr)
        for s in range(S):
            got = b.output(s)
            assert got[:len(head)] == head, s
            assert got[len(head):] == want[s], (s, len(got) - len(head), len(want[s]))
    finally:
        b.close()


def test_ingest_deblocking_stream_keeps_rect_qp_26(gpu, oracle, scroll):
    """a file whose PPS lacks deblocking_filter_control_present_flag (the
    loop filter on) cannot join a batch whose rect QP is not 26 (the rule
    add_stream enforces); nothing is added.  scroll_batch_set_config cannot
    turn the filter on for a stream whose rect QP is not 26."""
    w, h = 320, 240
    good = (ref_file(oracle, w, h, 0), ref_file(oracle, w, h, 1))
    nodb = variant_files(oracle, w, h, 1)                # deblock 0 in its PPS
    b = gpu.Batch(4, 2, 8 << 20)
    try:
        assert b.ingest([good]) == 0
        b.set_dyn_rect(1, 1, 2, 2)
        b.set_dyn_qp(30)
        with pytest.raises(RuntimeError):
            b.ingest([good, nodb])
        assert "deblocking" in gpu.last_error() and b.num_streams == 1
        assert b.ingest([good]) == 1                      # a file with the flag joins at QP 30
        c = b.config(1)
        c.deblocking_filter_control_present_flag = 0
        with pytest.raises(RuntimeError):
            b.set_config(1, c)
        assert "deblocking" in gpu.last_error()
        b.set_dyn_qp(26)
        b.set_config(1, c)                                # at QP 26 it may
        assert b.config(1).deblocking_filter_control_present_flag == 0
    finally:
        b.close()
