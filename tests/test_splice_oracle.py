"""The pre-encoded MB splice restatement (oracle/splice_oracle.c), CPU only.

The reference designs the splice (docs/MASTER_DESIGN.md:39-40,142-146,171)
but has no implementation, so the oracle DEFINES the bits ("parity
unpinned").  What pins it:
  (1) the external slices the stand-in encoder writes decode with the
      test-only standard decoder (tests/h264_pslice.py, written from the
      standard and independent of the oracle's tables) to the same motion,
      cbp and QP the oracle's parse reports;
  (2) a composed NAL decodes (the reference's predictor for EXACT, the
      standard's for PSKIP) so that every spliced MB has the external MB's
      ref, mv, cbp, QP and coefficient levels, and every other MB the
      UI-hint field of its frame;
  (3) without a splice the composed NAL equals the UI-hint NAL (itself equal
      to the reference's scroll frame without hints);
  (4) unsupported or malformed slices and invalid references are errors.
"""
import ctypes
import random

from dynhelp import OrCfg, hint_array, random_hints, ext_slice, splice_of, Splice
import h264_pslice as P

EXACT, PSKIP, SPEC = 0, 1, 2
ERR_NAL, ERR_HEADER, ERR_MBTYPE, ERR_SYNTAX, ERR_REF = 1, 2, 3, 4, 5


class SpliceMb(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("ref", "mx", "my", "cbp", "qp", "qpd", "skip")] + [
        ("tc", ctypes.c_uint8 * 27), ("t1", ctypes.c_uint8 * 27),
        ("boff", ctypes.c_uint32 * 27), ("blen", ctypes.c_uint32 * 27),
        ("part", ctypes.c_int), ("sub", ctypes.c_int), ("bref", ctypes.c_int * 16),
        ("bmx", ctypes.c_int * 16), ("bmy", ctypes.c_int * 16),
        ("intra", ctypes.c_int), ("mbt", ctypes.c_int), ("poff", ctypes.c_uint32), ("plen", ctypes.c_uint32),
        ("cbp_code", ctypes.c_int), ("pcm", ctypes.c_uint32), ("hasqpd", ctypes.c_int)]


def _cfg(oracle, w, h):
    c = OrCfg()
    oracle.or_cfg_init(ctypes.byref(c), w, h)
    return c


def _refs(c):
    return [0, 1] + [2 + i for i in range(c.nwp) if c.wp_valid[i]]


def _parse(oracle, c, sp):
    mbs = (SpliceMb * (sp.w * sp.h))()
    rb = (ctypes.c_uint8 * (sp.n + 8))()
    rn = ctypes.c_size_t()
    e = oracle.or_splice_parse(ctypes.byref(c), ctypes.byref(sp), mbs, rb, ctypes.byref(rn))
    return e, mbs


def _field(oracle, c, off, rects):
    mbw, mbh = c.w // 16, c.h // 16
    arr, n = hint_array(rects)
    out = (ctypes.c_int32 * (3 * mbw * mbh))()
    assert oracle.or_hint_field(ctypes.byref(c), off, arr, n, out) == 0
    return [[(out[3 * (y * mbw + x)], 4 * out[3 * (y * mbw + x) + 1], 4 * out[3 * (y * mbw + x) + 2])
             for x in range(mbw)] for y in range(mbh)]


def test_ext_slices_parse_like_the_standard_decoder(oracle):
    c = _cfg(oracle, 640, 368)
    cov = [0] * 5
    for seed, kw in enumerate([{}, dict(nrefs=1, max_ref=0), dict(nrefs=5, max_ref=4),
                               dict(skip_pm=900), dict(cbp_pm=1000, big_pm=300),
                               dict(slice_qp_delta=-7, qp_jitter=12), dict(ref_idc=2),
                               dict(mv_range=4000), dict(list_mod=1, nrefs=2, max_ref=1),
                               dict(part_pm=500), dict(part_pm=1000, nrefs=5, max_ref=4, skip_pm=100),
                               dict(part_pm=800, nrefs=1, max_ref=0, mv_range=3000),
                               dict(part_pm=600, skip_pm=600, cbp_pm=900),
                               dict(intra_pm=400, cbp_pm=900), dict(intra_pm=300, slice_rows=1, skip_pm=300),
                               dict(intra_pm=500, slice_rows=2, part_pm=300, qp_jitter=6)]):
        w, h = 5 + seed % 3, 4 + seed % 4
        nal = ext_slice(oracle, c, w, h, 100 + seed, **kw)
        e, mbs = _parse(oracle, c, splice_of(0, 0, w, h, nal))
        assert e == 0, (seed, kw)
        H, dec = P.decode_p_slice(nal, 16 * w, 16 * h, "spec")
        for y in range(h):
            for x in range(w):
                d, m = dec[y][x], mbs[y * w + x]
                assert (m.ref, m.mx, m.my, m.cbp, bool(m.skip)) == \
                    (d["ref"], d["mx"], d["my"], d["cbp"], d["skip"]), (seed, x, y)
                assert m.intra == d["intra"], (seed, x, y)
                if m.intra:
                    assert m.mbt == d["mbt"]
                    if m.hasqpd:
                        assert m.qp == d["qp"]
                    continue
                assert m.part == min(d["mbt"], 3), (seed, x, y)
                if m.part == 3:
                    assert [(m.sub >> (2 * i)) & 3 for i in range(4)] == d["sub"]
                assert [(m.bref[k], m.bmx[k], m.bmy[k]) for k in range(16)] == d["blocks"]
                cov[min(d["mbt"], 3)] += 1
                cov[4] += d["mbt"] == 4
                if m.cbp:
                    assert m.qp == d["qp"]
    assert all(cov), cov                       # every MB partitioning, P_8x8ref0 too


def _check_frame(oracle, c, off, rects, mode, sp, buf):
    """compose, decode, compare; returns the decoded composed and external MBs"""
    err = ctypes.c_int()
    c2 = OrCfg.from_buffer_copy(c)
    arr, n = hint_array(rects)
    k = oracle.or_splice_scroll_nal(buf, len(buf), ctypes.byref(c2), off, arr, n, mode,
                                    ctypes.byref(sp), ctypes.byref(err))
    assert err.value == 0 and k > 0
    nal = bytes(buf[:k])
    field = _field(oracle, c, off, rects)
    ext_nal = sp.data
    _, ext = P.decode_p_slice(ext_nal, 16 * sp.w, 16 * sp.h, "spec")
    H, got = P.decode_p_slice(nal, c.w, c.h, "ref" if mode == EXACT else "spec")
    assert H["nrefs"] == 2 + c.nwp and H["qp"] == 26
    for y in range(c.h // 16):
        for x in range(c.w // 16):
            g = got[y][x]
            if sp.x0 <= x < sp.x0 + sp.w and sp.y0 <= y < sp.y0 + sp.h:
                e = ext[y - sp.y0][x - sp.x0]
                assert (g["ref"], g["mx"], g["my"], g["cbp"]) == (e["ref"], e["mx"], e["my"], e["cbp"]), \
                    (off, mode, x, y)
                if e["intra"]:
                    # the same intra MB: type, every prediction mode, residual or samples
                    assert (g["intra"], g["mbt"], g["modes"], g["cmode"], g["dc16"], g["pcm"]) == \
                        (e["intra"], e["mbt"], e["modes"], e["cmode"], e["dc16"], e["pcm"]), (off, mode, x, y)
                    if e["intra"] == 2 or e["cbp"]:
                        assert g["qp"] == e["qp"]
                    assert (g["luma"], g["cdc"], g["cac"]) == (e["luma"], e["cdc"], e["cac"])
                    continue
                # partitionings kept (P_8x8ref0 -> P_8x8), every 4x4 block's motion
                assert (g["mbt"], g["sub"]) == (min(e["mbt"], 3), e["sub"]) or \
                    (e["skip"] and g["mbt"] == 0), (off, mode, x, y)
                assert g["blocks"] == e["blocks"], (off, mode, x, y)
                if e["cbp"]:
                    assert g["qp"] == e["qp"]
                    assert (g["luma"], g["cdc"], g["cac"]) == (e["luma"], e["cdc"], e["cac"])
            else:
                assert (g["ref"], g["mx"], g["my"]) == field[y][x] and g["cbp"] == 0, (off, mode, x, y)
    return got, ext


def test_spliced_mbs_decode_to_the_external_mbs(oracle):
    """random rects, external slices and hints over a scroll that crosses the
    496-px waypoint, so spliced MBs use waypoint references too"""
    rng = random.Random(5)
    buf = (ctypes.c_uint8 * (1 << 20))()
    err = ctypes.c_int()
    w, h = 256, 720
    c = _cfg(oracle, w, h)
    cov = dict(ref2=0, ext_skip=0, skipped=0, part=0)
    for i in range(20):
        off = 488 + i                              # 496: a waypoint
        if oracle.or_needs_waypoint(ctypes.byref(c), off):
            oracle.or_waypoint_nal(buf, len(buf), ctypes.byref(c), off)
        refs = _refs(c)
        sw, sh = rng.randint(1, 8), rng.randint(1, 6)
        x0, y0 = rng.randint(0, w // 16 - sw), rng.randint(0, h // 16 - sh)
        kw = dict(nrefs=len(refs), max_ref=len(refs) - 1, skip_pm=rng.choice([0, 200, 700]),
                  cbp_pm=rng.choice([0, 500, 1000]), big_pm=rng.choice([0, 50]),
                  mv_range=rng.choice([8, 300]), slice_qp_delta=rng.randint(-5, 5),
                  qp_jitter=rng.choice([0, 4]), ref_idc=rng.choice([0, 1]),
                  part_pm=rng.choice([0, 300, 900]))
        nal = ext_slice(oracle, c, sw, sh, 1000 + i, **kw)
        sp = splice_of(x0, y0, sw, sh, nal)
        rects = random_hints(rng, w // 16, h // 16, refs, nmax=3) if i % 3 == 0 else []
        for mode in (EXACT, PSKIP, SPEC):
            got, ext = _check_frame(oracle, c, off, rects, mode, sp, buf)
            cov["ref2"] += sum(m["ref"] >= 2 for row in ext for m in row) * (mode == EXACT)
            cov["ext_skip"] += sum(m["skip"] for row in ext for m in row) * (mode == EXACT)
            cov["part"] += sum(m["mbt"] > 0 for row in ext for m in row) * (mode == EXACT)
            if mode == PSKIP:
                cov["skipped"] += sum(got[y][x]["skip"] for y in range(y0, y0 + sh)
                                      for x in range(x0, x0 + sw))
        k = oracle.or_splice_scroll_nal(buf, len(buf), ctypes.byref(c), off, None, 0, EXACT,
                                        ctypes.byref(sp), ctypes.byref(err))
        assert k > 0
    # waypoint references, external P_Skip MBs, spliced MBs skipped again
    assert all(v > 0 for v in cov.values()), cov


def test_intra_and_multislice_splices(oracle):
    """external pictures with I_4x4 / I_16x16 / I_PCM MBs, in one slice or a
    slice per one or two MB rows (neighbours in another slice unavailable:
    motion, P_Skip, nC, intra mode prediction), spliced in all three modes;
    every spliced MB decodes to its external MB, every other MB to the hint
    field; over the 496 waypoint"""
    rng = random.Random(11)
    buf = (ctypes.c_uint8 * (1 << 21))()
    err = ctypes.c_int()
    w, h = 320, 720
    c = _cfg(oracle, w, h)
    cov = dict(i4=0, i16=0, pcm=0, slices=0)
    for i in range(16):
        off = 488 + i
        if oracle.or_needs_waypoint(ctypes.byref(c), off):
            oracle.or_waypoint_nal(buf, len(buf), ctypes.byref(c), off)
        refs = _refs(c)
        sw, sh = rng.randint(3, 9), rng.randint(3, 7)
        x0, y0 = rng.randint(0, w // 16 - sw), rng.randint(0, h // 16 - sh)
        rows = rng.choice([0, 1, 2])
        kw = dict(nrefs=len(refs), max_ref=len(refs) - 1, skip_pm=rng.choice([0, 200, 500]),
                  cbp_pm=rng.choice([500, 1000]), big_pm=rng.choice([0, 50]), mv_range=rng.choice([8, 300]),
                  slice_qp_delta=rng.randint(-5, 5), qp_jitter=rng.choice([0, 4]),
                  part_pm=rng.choice([0, 300]), intra_pm=rng.choice([300, 700]), slice_rows=rows,
                  pcm_zero=i % 4 == 3)
        nal = ext_slice(oracle, c, sw, sh, 2000 + i, **kw)
        sp = splice_of(x0, y0, sw, sh, nal)
        e, _ = _parse(oracle, c, sp)
        assert e == 0, (i, e)
        rects = random_hints(rng, w // 16, h // 16, refs, nmax=3) if i % 3 == 0 else []
        for mode in (EXACT, PSKIP, SPEC):
            got, ext = _check_frame(oracle, c, off, rects, mode, sp, buf)
        cov["i4"] += sum(m["intra"] == 1 for row in ext for m in row)
        cov["i16"] += sum(m["intra"] == 2 for row in ext for m in row)
        cov["pcm"] += sum(m["intra"] == 3 for row in ext for m in row)
        cov["slices"] += rows > 0 and sh > rows
        k = oracle.or_splice_scroll_nal(buf, len(buf), ctypes.byref(c), off, None, 0, EXACT,
                                        ctypes.byref(sp), ctypes.byref(err))
        assert k > 0
    assert all(v > 0 for v in cov.values()), cov


def test_multislice_rules(oracle):
    """slices must start where the previous one ended and cover the picture"""
    buf = (ctypes.c_uint8 * (1 << 18))()
    err = ctypes.c_int()
    c = _cfg(oracle, 256, 256)
    nal = ext_slice(oracle, c, 4, 4, 5, slice_rows=1)
    units = P.nal_units(nal)
    assert len(units) == 4

    def compose(data):
        c2 = OrCfg.from_buffer_copy(c)
        oracle.or_splice_scroll_nal(buf, len(buf), ctypes.byref(c2), 40, None, 0, EXACT,
                                    ctypes.byref(splice_of(2, 2, 4, 4, data)), ctypes.byref(err))
        return err.value

    sc = b"\x00\x00\x00\x01"
    assert compose(nal) == 0
    assert compose(b"".join(sc + u for u in units[:3])) == ERR_SYNTAX            # a row missing
    assert compose(b"".join(sc + u for u in (units[0], units[2], units[1], units[3]))) == ERR_HEADER
    assert compose(b"".join(sc + u + b"\x00\x00" for u in units)) == 0       # trailing zero bytes


def test_splice_at_picture_corners_and_whole_picture(oracle):
    buf = (ctypes.c_uint8 * (1 << 20))()
    w, h = 192, 128
    c = _cfg(oracle, w, h)
    mbw, mbh = w // 16, h // 16
    for j, (x0, y0, sw, sh) in enumerate([(0, 0, 3, 2), (mbw - 3, 0, 3, 3), (0, mbh - 2, 4, 2),
                                          (mbw - 2, mbh - 2, 2, 2), (0, 0, mbw, mbh),
                                          (5, 3, 1, 1)]):
        nal = ext_slice(oracle, c, sw, sh, 77 + j, cbp_pm=900, skip_pm=300, part_pm=400 * (j % 2))
        for mode in (EXACT, PSKIP, SPEC):
            _check_frame(oracle, c, 40, [], mode, splice_of(x0, y0, sw, sh, nal), buf)


def test_no_splice_equals_hint_nal(oracle):
    rng = random.Random(9)
    w, h = 256, 256
    a = (ctypes.c_uint8 * (1 << 18))()
    b = (ctypes.c_uint8 * (1 << 18))()
    err = ctypes.c_int()
    for mode in (EXACT, PSKIP, SPEC):
        c1, c2 = _cfg(oracle, w, h), _cfg(oracle, w, h)
        for i in range(30):
            off = oracle.or_synthetic_offset(1, i, h)
            rects = random_hints(rng, w // 16, h // 16, _refs(c1), nmax=3)
            arr, n = hint_array(rects)
            ka = oracle.or_compose_hint(a, len(a), ctypes.byref(c1), off, 0, arr, n, mode,
                                        ctypes.byref(err))
            assert err.value == 0
            kb = oracle.or_compose_splice(b, len(b), ctypes.byref(c2), off, 0, arr, n, mode, None,
                                          ctypes.byref(err))
            assert err.value == 0 and bytes(a[:ka]) == bytes(b[:kb])
            empty = Splice(0, 0, 0, 0, None, 0)
            c3 = OrCfg.from_buffer_copy(c1)
            c3.frame_num -= 1
            kc = oracle.or_splice_scroll_nal(b, len(b), ctypes.byref(c3), off, arr, n, mode,
                                             ctypes.byref(empty), ctypes.byref(err))
            assert err.value == 0 and bytes(b[:kc]) == bytes(a[ka - kc:ka])


def test_errors(oracle):
    buf = (ctypes.c_uint8 * (1 << 18))()
    err = ctypes.c_int()
    w, h = 256, 256
    c = _cfg(oracle, w, h)

    def compose(sp):
        c2 = OrCfg.from_buffer_copy(c)
        k = oracle.or_splice_scroll_nal(buf, len(buf), ctypes.byref(c2), 40, None, 0, EXACT,
                                        ctypes.byref(sp), ctypes.byref(err))
        assert (k == 0) == (err.value != 0) and c2.frame_num == c.frame_num + (k > 0)
        return err.value

    good = ext_slice(oracle, c, 4, 3, 1)
    assert compose(splice_of(2, 2, 4, 3, good)) == 0
    # intra MBs (5 = I_NxN in P, 12 = I_16x16 DC, 30 = I_PCM): spliced inside the rect
    for t in (5, 12, 30):
        ok = ext_slice(oracle, c, 4, 3, 1, bad_mb=5, bad_type=t)
        assert compose(splice_of(2, 2, 4, 3, ok)) == 0, t
    # on the rect's top / left edge an I_4x4 / I_16x16 DC would predict from
    # other samples in the composed picture (refused); I_PCM anywhere; with the
    # rect in the picture's corner those edges are the picture's (accepted)
    for mb in (0, 1, 4):
        for t in (5, 12):
            bad = ext_slice(oracle, c, 4, 3, 1, bad_mb=mb, bad_type=t)
            assert compose(splice_of(2, 2, 4, 3, bad)) == ERR_MBTYPE, (mb, t)
            assert compose(splice_of(0, 0, 4, 3, bad)) == 0, (mb, t)
        ok = ext_slice(oracle, c, 4, 3, 1, bad_mb=mb, bad_type=30)
        assert compose(splice_of(2, 2, 4, 3, ok)) == 0, mb
    # I_16x16 vertical prediction (mb_type 6) on the left edge reads no left samples
    ok = ext_slice(oracle, c, 4, 3, 1, bad_mb=4, bad_type=6)
    e, mbs = _parse(oracle, c, splice_of(2, 2, 4, 3, ok))
    assert e == 0 or e == ERR_MBTYPE                # the chroma mode decides (random)
    # mb_type past the P-slice range
    bad = ext_slice(oracle, c, 4, 3, 1, bad_mb=5, bad_type=31)
    assert compose(splice_of(2, 2, 4, 3, bad)) == ERR_SYNTAX
    # not a non-IDR slice: an IDR NAL header, an SPS
    # an IDR NAL header on a P slice: IDR pictures are I slices only
    assert compose(splice_of(2, 2, 4, 3, good[:4] + bytes([0x65]) + good[5:])) == ERR_HEADER
    assert compose(splice_of(2, 2, 4, 3, good[:4] + bytes([0x66]) + good[5:])) == ERR_NAL      # SEI
    assert compose(splice_of(2, 2, 4, 3, good[:4] + bytes([0x67]) + good[5:])) == ERR_NAL
    # a rect whose MB count differs from the slice's: too many MBs / too few
    assert compose(splice_of(2, 2, 4, 2, good)) == ERR_SYNTAX
    assert compose(splice_of(2, 2, 4, 4, good)) == ERR_SYNTAX
    # truncated
    assert compose(splice_of(2, 2, 4, 3, good[:len(good) // 2])) in (ERR_SYNTAX,)
    # a reference the frame does not have (waypoint 0 before any waypoint)
    assert c.nwp == 0
    bad = ext_slice(oracle, c, 4, 3, 2, nrefs=4, max_ref=3, skip_pm=0)
    assert compose(splice_of(2, 2, 4, 3, bad)) == ERR_REF
    # reference list: restating the composed list is fine, reordering is not
    ok = ext_slice(oracle, c, 4, 3, 3, list_mod=1)
    assert compose(splice_of(2, 2, 4, 3, ok)) == 0
    bad = ext_slice(oracle, c, 4, 3, 3, list_mod=2)
    assert compose(splice_of(2, 2, 4, 3, bad)) == ERR_HEADER
    # rect outside the picture
    assert compose(splice_of(14, 2, 4, 3, good)) == ERR_HEADER


def test_reference_parser_accepts_spliced_nals(oracle):
    """tests/golden/splice_ref.json: the reference's CAVLC P-slice parser
    (trans_resizer process_p_slice, built from /root/reference by
    oracle/Makefile `ref`) consumed the MB layer of every fixture NAL --
    external slices of the stand-in encoder and composed 320x320 NALs with a
    spliced rect, both modes, 2 and 3 references -- and its I-slice walker
    (process_i_slice) the stand-in encoder's I pictures, exactly up to the
    rbsp_stop_one_bit.  The oracle must still produce those NALs bit for bit;
    where the reference build exists the parse is repeated live."""
    import json
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "golden"))
    import make_golden_splice as mg
    fx = json.load(open(os.path.join(here, "golden", "splice_ref.json")))
    assert all(c["ref_status"] == 0 and c["ref_end_bit"] == c["stop_bit"] for c in fx)
    assert {c["kind"] for c in fx} == {"external", "external-i", "composed", "composed-intra"}
    refso = os.path.join(os.path.dirname(here), "oracle", "_ref", "libref_cavlc.so")
    ref = ctypes.CDLL(refso) if os.path.exists(refso) else None
    got = list(mg.cases(oracle))
    assert len(got) == len(fx)
    for (c, nal, rbsp), f in zip(got, fx):
        assert c["sha256"] == f["sha256"] and c["mb_start_bit"] == f["mb_start_bit"]
        if ref is not None:
            end = ctypes.c_size_t()
            if c["kind"] == "external-i":                 # the reference's I-slice walker
                assert ref.ref_cavlc_parse_i(rbsp, len(rbsp), c["mb_start_bit"], ctypes.byref(end)) == 0
            else:
                assert ref.ref_cavlc_parse(rbsp, len(rbsp), c["mb_start_bit"], c["nrefs"],
                                           ctypes.byref(end)) == 0
            assert end.value == c["stop_bit"]


def test_i_and_idr_slices_splice(oracle):
    """a conventional encoder's first frame and scene cuts are I / IDR
    pictures (MASTER_DESIGN.md:39-40,85-90): I slices (nal_unit_type 1) and
    IDR slices (5), one slice or one per MB row, every MB intra with an
    I_PCM edge ring (I_4x4 / I_16x16 inside), spliced into the rect's
    interior: they parse (no mb_skip_run, mb_type k = the P slice's 5 + k),
    compose as P-slice intra MBs and decode to the external MBs in all three
    modes; the same picture on the rect's left edge inside the composed
    picture keeps the edge ring's I_PCM and still splices; an all-I_4x4
    picture there is refused (SCROLL_SPLICE_ERR_MBTYPE)"""
    rng = random.Random(5)
    buf = (ctypes.c_uint8 * (1 << 21))()
    w, h = 640, 480
    c = _cfg(oracle, w, h)
    cov = dict(i4=0, i16=0, pcm=0)
    for i, (islice, rows) in enumerate([(1, 0), (2, 0), (1, 1), (2, 2), (2, 0), (1, 0)]):
        sw, sh = 25 if i == 0 else rng.randint(4, 12), 25 if i == 0 else rng.randint(4, 9)
        sw, sh = min(sw, w // 16 - 2), min(sh, h // 16 - 2)
        x0, y0 = rng.randint(1, w // 16 - sw - 1), rng.randint(1, h // 16 - sh - 1)
        nal = ext_slice(oracle, c, sw, sh, 700 + i, islice=islice, slice_rows=rows, cbp_pm=800,
                        big_pm=30, qp_jitter=3, intra_types=3 if i % 2 else 0, slice_qp_delta=rng.randint(-4, 4))
        nu = nal[4] & 31
        assert nu == (5 if islice == 2 else 1)
        sp = splice_of(x0, y0, sw, sh, nal)
        e, mbs = _parse(oracle, c, sp)
        assert e == 0, (i, e)
        for mode in (EXACT, PSKIP, SPEC):
            got, ext = _check_frame(oracle, c, 100 + i, [], mode, sp, buf)
        assert all(m["intra"] for row in ext for m in row)
        cov["i4"] += sum(m["intra"] == 1 for row in ext for m in row)
        cov["i16"] += sum(m["intra"] == 2 for row in ext for m in row)
        cov["pcm"] += sum(m["intra"] == 3 for row in ext for m in row)
        e2, _ = _parse(oracle, c, splice_of(0, y0, sw, sh, nal))          # the picture's left edge
        assert e2 == 0
    assert all(v > 0 for v in cov.values()), cov
    # an I_4x4 on the rect's top-left corner, inside the composed picture
    nal = ext_slice(oracle, c, 4, 4, 9, islice=1, bad_mb=0, bad_type=5)
    e, _ = _parse(oracle, c, splice_of(3, 3, 4, 4, nal))
    assert e == 3
