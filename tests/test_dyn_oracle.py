"""Dynamic-rect residual coder (oracle/dyn_oracle.c), CPU only.

No reference implementation exists: parity is UNPINNED.  These
tests check the restatement against the H.264 decoding process instead: every
emitted slice parses with an independent CAVLC parser (tests/h264_pslice.py),
the dynamic MBs reconstruct (dequant + inverse transform + prediction) to
within quantisation error of the synthetic source, and the scroll MBs are
unchanged from the reference path."""
import ctypes
import math
import sys
import os

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import h264_pslice as hp  # noqa: E402
from dynhelp import FlatRefs, OrCfg, Rect, StripedRefs, qp_field, rect_source, split_nals  # noqa: E402


def _pred(lib, cfg, R, ref, mv, mbx, mby):
    py = [[lib.or_ref_sample(ctypes.byref(cfg), ctypes.byref(R.refs), ref, 0, 16 * mbx + j, 16 * mby + i + mv)
           for j in range(16)] for i in range(16)]
    pc = []
    for p in (1, 2):
        q = 4 * mv
        o, f = q >> 3, q & 7
        rows = []
        for i in range(8):
            row = []
            for j in range(8):
                X, Y = 8 * mbx + j, 8 * mby + i
                a = lib.or_ref_sample(ctypes.byref(cfg), ctypes.byref(R.refs), ref, p, X, Y + o)
                b = lib.or_ref_sample(ctypes.byref(cfg), ctypes.byref(R.refs), ref, p, X, Y + o + 1)
                row.append(((8 - f) * a + f * b + 4) >> 3)
            rows.append(row)
        pc.append(rows)
    return py, pc[0], pc[1]


def _regions(cfg, off):
    """(a_end, ra, mva, rb, mvb) of a scroll frame, src/h264_writer.c:555-588"""
    h = cfg.h
    wa, woa, wb, wob = -1, 0, -1, 0
    if off > 496 and cfg.nwp > 0:
        for i in range(cfg.nwp):
            wo = cfg.wp_off[i]
            if cfg.wp_valid[i] and wo <= off and wo > woa and off - wo <= 496:
                wa, woa = i, wo
    if off - h < -496 and cfg.nwp > 0:
        for i in range(cfg.nwp):
            wo = cfg.wp_off[i]
            if cfg.wp_valid[i] and wo > off and off - wo >= -496:
                wb, wob = i, wo
                break
    ra, mva = (2 + wa, off - woa) if wa >= 0 else (0, off)
    rb, mvb = (2 + wb, off - wob) if wb >= 0 else (1, off - h)
    return (h - off) // 16, ra, mva, rb, mvb


def _psnr(a, b):
    mse = sum((x - y) ** 2 for x, y in zip(a, b)) / len(a)
    return 99.0 if mse == 0 else 10 * math.log10(255 * 255 / mse)


@pytest.mark.parametrize("w,h,rect,offs", [
    (64, 512, (1, 20, 2, 6), [0, 17, 496, 500, 505, 400, 300]),   # waypoint refs in the rect
    (96, 96, (1, 1, 4, 4), [0, 5, 40, 96]),                        # rect touching the edges
])
def test_dyn_slices_parse_and_reconstruct(oracle, w, h, rect, offs):
    lib = oracle
    R = StripedRefs(lib, w, h)
    rc = Rect(*rect)
    cfg = OrCfg()
    lib.or_cfg_init(ctypes.byref(cfg), w, h)
    cfg.frame_num = 2
    buf = (ctypes.c_uint8 * (1 << 21))()
    worst = 99.0
    for t, off in enumerate(offs):
        src = rect_source(lib, 3, t, rc)
        before = OrCfg.from_buffer_copy(cfg)
        n = lib.or_compose_dyn(buf, len(buf), ctypes.byref(cfg), off, 0, ctypes.byref(rc), src,
                               ctypes.byref(R.refs), None)
        nals = split_nals(bytes(buf[:n]))
        scroll = nals[-1]
        # the waypoint NAL (if any) is exactly the reference's
        state = OrCfg.from_buffer_copy(before)
        if len(nals) == 2:
            n0 = lib.or_waypoint_nal(buf, len(buf), ctypes.byref(state), off)
            assert bytes(buf[:n0]) == nals[0]
        a_end, ra, mva, rb, mvb = _regions(state, off)
        got = {}

        def on_mb(x, y, ref, mvd, cbp, luma, cdc, cac):
            inside = rc.x0 <= x < rc.x0 + rc.w and rc.y0 <= y < rc.y0 + rc.h
            assert ref == (ra if y < a_end else rb)
            if not inside:
                assert cbp == 0
            else:
                got[(x, y)] = (luma, cdc, cac)

        H, nmb = hp.parse_p_slice(scroll, w, h, on_mb=on_mb)
        assert nmb == (w // 16) * (h // 16)
        # reconstruction of every dynamic MB vs the source
        lw, cw = 16 * rc.w, 8 * rc.w
        rec, org = [], []
        for (x, y), (luma, cdc, cac) in got.items():
            mv = mva if y < a_end else mvb
            ref = ra if y < a_end else rb
            py, pu, pv = _pred(lib, state, R, ref, mv, x, y)
            ry, ru, rv = hp.reconstruct_mb(luma, cdc, cac, py, pu, pv)
            lx, ly = 16 * (x - rc.x0), 16 * (y - rc.y0)
            for i in range(16):
                for j in range(16):
                    rec.append(ry[i][j])
                    org.append(src[(ly + i) * lw + lx + j])
            cbase = lw * 16 * rc.h
            for p, rr in enumerate((ru, rv)):
                base = cbase + p * cw * 8 * rc.h
                for i in range(8):
                    for j in range(8):
                        rec.append(rr[i][j])
                        org.append(src[base + (8 * (y - rc.y0) + i) * cw + 8 * (x - rc.x0) + j])
        assert len(got) == rc.w * rc.h
        psnr = _psnr(rec, org)
        worst = min(worst, psnr)
        assert psnr > 34.0, (off, psnr)
        assert max(abs(a - b) for a, b in zip(rec, org)) <= 40          # QP 26: Qstep 13
    print("worst PSNR", worst)


def test_empty_rect_is_reference_path(oracle):
    lib = oracle
    w, h = 1280, 720
    R = StripedRefs(lib, w, h)
    c1, c2 = OrCfg(), OrCfg()
    lib.or_cfg_init(ctypes.byref(c1), w, h)
    lib.or_cfg_init(ctypes.byref(c2), w, h)
    empty = Rect(0, 0, 0, 0)
    b1 = (ctypes.c_uint8 * (1 << 20))()
    b2 = (ctypes.c_uint8 * (1 << 20))()
    for off in (0, 33, 496, 720):
        n1 = lib.or_compose(b1, len(b1), ctypes.byref(c1), off, 0, None)
        n2 = lib.or_compose_dyn(b2, len(b2), ctypes.byref(c2), off, 0, ctypes.byref(empty), None,
                                ctypes.byref(R.refs), None)
        assert bytes(b1[:n1]) == bytes(b2[:n2])


def test_forward_transform_matches_matrix(oracle):
    import random
    rng = random.Random(1)
    Cf = [[1, 1, 1, 1], [2, 1, -1, -2], [1, -1, -1, 1], [1, -2, 2, -1]]
    for _ in range(200):
        x = [rng.randint(-255, 255) for _ in range(16)]
        W = (ctypes.c_int * 16)()
        oracle.or_fwd4x4((ctypes.c_int * 16)(*x), W)
        X = [x[4 * i:4 * i + 4] for i in range(4)]
        T = [[sum(Cf[i][k] * X[k][j] for k in range(4)) for j in range(4)] for i in range(4)]
        Y = [[sum(T[i][k] * Cf[j][k] for k in range(4)) for j in range(4)] for i in range(4)]
        assert list(W) == [Y[i][j] for i in range(4) for j in range(4)]


def test_reference_cavlc_parser_accepts(oracle):
    """tests/golden/cavlc_ref.json: the reference's CAVLC parser (trans_resizer,
    built from /root/reference by oracle/Makefile `ref`) consumed the MB layer
    of every fixture NAL exactly up to its rbsp_stop_one_bit.  The oracle must
    still produce those NALs bit for bit; where the reference build exists the
    parse is repeated live."""
    import json
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_golden_cavlc as mg
    fx = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                     "cavlc_ref.json")))
    assert all(c["ref_status"] == 0 and c["ref_end_bit"] == c["stop_bit"] for c in fx)
    refso = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle",
                         "_ref", "libref_cavlc.so")
    ref = ctypes.CDLL(refso) if os.path.exists(refso) else None
    got = list(mg.cases(oracle))
    assert len(got) == len(fx)
    for (c, nal, rbsp), f in zip(got, fx):
        assert c["sha256"] == f["sha256"] and c["mb_start_bit"] == f["mb_start_bit"]
        if ref is not None:
            end = ctypes.c_size_t()
            assert ref.ref_cavlc_parse(rbsp, len(rbsp), c["mb_start_bit"], c["nrefs"],
                                       ctypes.byref(end)) == 0
            assert end.value == c["stop_bit"]


def test_cavlc_values_pinned_by_reference_decoder(oracle):
    """Value-level pin (tests/golden/make_golden_cavlc_values.py): every coded
    block of every dynamic MB of the cavlc_ref.json NALs (real levels and
    neighbour contexts) plus 600 synthetic MBs with escape-range levels is
    decoded by the REFERENCE's CAVLC functions (trans_resizer.c: cbp_inter_table
    + read_ue/se, compute_luma_nC / compute_chroma_nC, read_coeff_token,
    copy_cavlc_block's level parser, decode_total_zeros, decode_run_before);
    the coefficient vector rebuilt from those fields must equal the oracle's
    quantised coefficients, and nC, token and block lengths must agree.  The
    committed SHA-256 of those records pins the oracle where the reference
    build is absent.  Transform and quantiser: no reference (unpinned)."""
    import json
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_golden_cavlc_values as mv
    fx = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                     "cavlc_values.json")))
    refso = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle",
                         "_ref", "libref_cavlc.so")
    ref = ctypes.CDLL(refso) if os.path.exists(refso) else None
    mine, live, esc = [], [], [0, 0, 0]
    for case in mv.all_mbs(oracle):
        lv = case[7]
        _, exp = mv.expected(oracle, lv, case[3], case[4], case[5], case[6])
        mine += mv.oracle_records(lv, exp)
        esc = [a + b for a, b in zip(esc, mv.escapes(lv))]
        if ref is not None:
            live += mv.check_mb(oracle, ref, case)
    assert len(mine) == fx["blocks"]
    assert mv.digest(mine) == fx["sha256"]
    if ref is not None:
        assert live == mine
    # level_prefix 14 at suffixLength 0, prefix 15 at 0 and at > 0 all occur
    assert min(esc) > 1000, esc


# Table 8-15 (chroma_qp_index_offset 0): QPc for QP 30..51
_QPC = [29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39]


def test_dyn_rect_qp_decodes(oracle):
    """scroll_batch_set_dyn_qp's bits (or_dyn_rect.qp): the dynamic NAL's
    slice_qp_delta is qp - 26 and its MBs decode -- luma at qp, chroma at QPc
    -- to the source within what the quantiser step allows (PSNR falls as
    QP rises); waypoint NALs and the rect-free path are unchanged"""
    lib = oracle
    w, h = 96, 96
    R = StripedRefs(lib, w, h)
    buf = (ctypes.c_uint8 * (1 << 21))()
    psnrs = []
    qps = (0, 5, 12, 18, 22, 26, 30, 39, 51)
    for qp in qps:
        rc = Rect(1, 1, 4, 4, qp_field(qp))
        cfg = OrCfg()
        lib.or_cfg_init(ctypes.byref(cfg), w, h)
        cfg.frame_num = 2
        rec, org = [], []
        for t, off in enumerate([0, 5, 40, 96]):
            src = rect_source(lib, 3, t, rc)
            state = OrCfg.from_buffer_copy(cfg)
            n = lib.or_compose_dyn(buf, len(buf), ctypes.byref(cfg), off, 0, ctypes.byref(rc), src,
                                   ctypes.byref(R.refs), None)
            scroll = split_nals(bytes(buf[:n]))[-1]
            a_end, ra, mva, rb, mvb = _regions(state, off)
            got = {}

            def on_mb(x, y, ref, mvd, cbp, luma, cdc, cac):
                if rc.x0 <= x < rc.x0 + rc.w and rc.y0 <= y < rc.y0 + rc.h:
                    got[(x, y)] = (luma, cdc, cac)

            H, nmb = hp.parse_p_slice(scroll, w, h, on_mb=on_mb)
            assert H["qp_delta"] == qp - 26 and nmb == (w // 16) * (h // 16)
            qpc = qp if qp < 30 else _QPC[qp - 30]
            lw, cw = 16 * rc.w, 8 * rc.w
            for (x, y), (luma, cdc, cac) in got.items():
                mv = mva if y < a_end else mvb
                ref = ra if y < a_end else rb
                py, pu, pv = _pred(lib, state, R, ref, mv, x, y)
                ry, ru, rv = hp.reconstruct_mb(luma, cdc, cac, py, pu, pv, qp=qp, qpc=qpc)
                lx, ly = 16 * (x - rc.x0), 16 * (y - rc.y0)
                for i in range(16):
                    for j in range(16):
                        rec.append(ry[i][j])
                        org.append(src[(ly + i) * lw + lx + j])
                cbase = lw * 16 * rc.h
                for p, rr in enumerate((ru, rv)):
                    base = cbase + p * cw * 8 * rc.h
                    for i in range(8):
                        for j in range(8):
                            rec.append(rr[i][j])
                            org.append(src[base + (8 * (y - rc.y0) + i) * cw + 8 * (x - rc.x0) + j])
            assert len(got) == rc.w * rc.h
        psnrs.append(_psnr(rec, org))
    assert psnrs[qps.index(22)] > 38.0 and psnrs[qps.index(26)] > 34.0 and psnrs[0] > 50.0, psnrs
    assert all(a > b for a, b in zip(psnrs, psnrs[1:])), psnrs
    # qp 26 written out is the default's bytes
    c1, c2 = OrCfg(), OrCfg()
    lib.or_cfg_init(ctypes.byref(c1), w, h)
    lib.or_cfg_init(ctypes.byref(c2), w, h)
    b2 = (ctypes.c_uint8 * (1 << 20))()
    src = rect_source(lib, 3, 0, Rect(1, 1, 4, 4))
    n1 = lib.or_compose_dyn(buf, len(buf), ctypes.byref(c1), 40, 0, ctypes.byref(Rect(1, 1, 4, 4)), src,
                            ctypes.byref(R.refs), None)
    n2 = lib.or_compose_dyn(b2, len(b2), ctypes.byref(c2), 40, 0, ctypes.byref(Rect(1, 1, 4, 4, 26)), src,
                            ctypes.byref(R.refs), None)
    assert bytes(buf[:n1]) == bytes(b2[:n2])


def test_dyn_rect_low_qp_levels_clamped_and_parsed(oracle):
    """QP 0 on saturated residuals (black references, white chroma, +-255
    luma noise): the chroma DC levels reach OR_LEVEL_MAX (2063, the clamp;
    luma levels stay <= 1632 at any QP) and are coded with level_prefix 15
    (the escape every context accepts); the NAL parses in the test decoder
    to exactly those levels"""
    lib = oracle
    w, h = 64, 64
    R = FlatRefs(w, h, 0)
    rc = Rect(1, 1, 2, 2, qp_field(0))
    n = 384 * rc.w * rc.h
    rng = __import__("random").Random(5)
    src = (ctypes.c_uint8 * n)(*([rng.choice((0, 255)) for _ in range(256 * rc.w * rc.h)] +
                                 [255] * (128 * rc.w * rc.h)))
    cfg = OrCfg()
    lib.or_cfg_init(ctypes.byref(cfg), w, h)
    cfg.frame_num = 2
    buf = (ctypes.c_uint8 * (1 << 20))()
    nb = lib.or_compose_dyn(buf, len(buf), ctypes.byref(cfg), 3, 0, ctypes.byref(rc), src,
                            ctypes.byref(R.refs), None)
    scroll = split_nals(bytes(buf[:nb]))[-1]
    big = []

    def on_mb(x, y, ref, mvd, cbp, luma, cdc, cac):
        for b in luma:
            big.extend(abs(v) for v in b)
        for b in cdc:
            big.extend(abs(v) for v in b)

    H, nmb = hp.parse_p_slice(scroll, w, h, on_mb=on_mb)
    assert H["qp_delta"] == -26 and nmb == (w // 16) * (h // 16)
    assert max(big) == 2063                     # the clamp was reached and coded
