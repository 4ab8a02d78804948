"""The dynamic rect under UI hints (oracle/splice_oracle.c
or_hint_dyn_scroll_nal), CPU only.  No reference implementation exists
(docs/MASTER_DESIGN.md:58-64,109-146 describe a per-frame hint record with
motion regions AND the dynamic rect): parity is UNPINNED.  Anchors:
  - without hint rects, in EXACT mode, the NAL is the plain dynamic-rect NAL
    (or_scroll_nal_dyn, the restatement the GPU's k_dyn_row path matches);
  - every NAL decodes from the standard (tests/h264_pslice.py, median
    prediction for SPEC / PSKIP, the reference's for EXACT) to the hinted MV
    field, and the rect MBs reconstruct -- prediction at THEIR hinted motion
    (full-pel luma, 2-D 1/8-pel chroma) + dequantised residual -- to within
    quantisation error of the source, for rects moving from frame to frame."""
import ctypes
import math
import random

import pytest

import h264_pslice as hp
from dynhelp import OrCfg, Rect, StripedRefs, hint_array, random_hints, rect_source, split_nals

EXACT, PSKIP, SPEC = 0, 1, 2


def _cfg(oracle, w, h):
    c = OrCfg()
    oracle.or_cfg_init(ctypes.byref(c), w, h)
    c.frame_num = 2
    return c


def _refs(c):
    return [0, 1] + [2 + i for i in range(c.nwp) if c.wp_valid[i]]


def test_no_hints_exact_is_the_plain_dynamic_nal(oracle):
    w, h = 320, 720
    R = StripedRefs(oracle, w, h)
    oracle.or_compose_dyn.restype = ctypes.c_size_t
    a = (ctypes.c_uint8 * (1 << 21))()
    b = (ctypes.c_uint8 * (1 << 21))()
    err = ctypes.c_int()
    c1, c2 = _cfg(oracle, w, h), _cfg(oracle, w, h)
    for t, off in enumerate([0, 37, 480, 496, 497, 600, 700, 250]):
        rc = Rect(t % 5, 10 + t, 6, 4)
        src = rect_source(oracle, 5, t, rc)
        na = oracle.or_compose_dyn(a, len(a), ctypes.byref(c1), off, 0, ctypes.byref(rc), src,
                                   ctypes.byref(R.refs), None)
        nb = oracle.or_compose_hint_dyn(b, len(b), ctypes.byref(c2), off, 0, None, 0, EXACT,
                                        ctypes.byref(rc), src, ctypes.byref(R.refs), ctypes.byref(err))
        assert err.value == 0
        assert bytes(a[:na]) == bytes(b[:nb]), (t, off)


def _pred(lib, cfg, R, ref, mvx, mvy, mbx, mby):
    s = lambda p, x, y: lib.or_ref_sample(ctypes.byref(cfg), ctypes.byref(R.refs), ref, p, x, y)
    py = [[s(0, 16 * mbx + j + mvx, 16 * mby + i + mvy) for j in range(16)] for i in range(16)]
    qx, qy = 4 * mvx, 4 * mvy
    fx, fy = qx & 7, qy & 7
    pc = []
    for p in (1, 2):
        rows = []
        for i in range(8):
            row = []
            for j in range(8):
                xi, yi = 8 * mbx + j + (qx >> 3), 8 * mby + i + (qy >> 3)
                A, B = s(p, xi, yi), s(p, xi + 1, yi)
                C, D = s(p, xi, yi + 1), s(p, xi + 1, yi + 1)
                row.append(((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C
                            + fx * fy * D + 32) >> 6)
            rows.append(row)
        pc.append(rows)
    return py, pc[0], pc[1]


def _psnr(a, b):
    mse = sum((x - y) ** 2 for x, y in zip(a, b)) / len(a)
    return 99.0 if mse == 0 else 10 * math.log10(255 * 255 / mse)


@pytest.mark.parametrize("w,h,seed", [(256, 720, 1), (320, 256, 2)])
def test_hinted_rect_decodes_and_reconstructs(oracle, w, h, seed):
    rng = random.Random(seed)
    lib = oracle
    R = StripedRefs(lib, w, h)
    buf = (ctypes.c_uint8 * (1 << 22))()
    err = ctypes.c_int()
    c = _cfg(lib, w, h)
    mbw, mbh = w // 16, h // 16
    worst, nskip = 99.0, 0
    offs = [rng.randint(0, h) for _ in range(10)] + list(range(490, 500))
    for t, off in enumerate(offs):
        if lib.or_needs_waypoint(ctypes.byref(c), off):
            lib.or_waypoint_nal(buf, len(buf), ctypes.byref(c), off)
        rects = random_hints(rng, mbw, mbh, _refs(c), nmax=4)
        rw, rh = rng.randint(1, 5), rng.randint(1, 4)
        rc = Rect(rng.randint(0, mbw - rw), rng.randint(0, mbh - rh), rw, rh)
        src = rect_source(lib, seed, t, rc)
        mode = (EXACT, PSKIP, SPEC)[t % 3]
        arr, n = hint_array(rects)
        field = (ctypes.c_int32 * (3 * mbw * mbh))()
        assert lib.or_hint_field(ctypes.byref(c), off, arr, n, field) == 0
        c2 = OrCfg.from_buffer_copy(c)
        k = lib.or_hint_dyn_scroll_nal(buf, len(buf), ctypes.byref(c2), off, arr, n, mode,
                                       ctypes.byref(rc), src, ctypes.byref(R.refs), ctypes.byref(err))
        assert err.value == 0 and k > 0
        H, mbs = hp.decode_p_slice(bytes(buf[:k]), w, h, "ref" if mode == EXACT else "spec")
        rec, org = [], []
        lw, cw = 16 * rc.w, 8 * rc.w
        for y in range(mbh):
            for x in range(mbw):
                ref, mvx, mvy = field[3 * (y * mbw + x):3 * (y * mbw + x) + 3]
                g = mbs[y][x]
                assert (g["ref"], g["mx"], g["my"]) == (ref, 4 * mvx, 4 * mvy), (t, x, y)
                inside = rc.x0 <= x < rc.x0 + rc.w and rc.y0 <= y < rc.y0 + rc.h
                if not inside:
                    assert g["cbp"] == 0
                    continue
                nskip += g["skip"]
                py, pu, pv = _pred(lib, c, R, ref, mvx, mvy, x, y)
                ry, ru, rv = hp.reconstruct_mb(g["luma"], g["cdc"], g["cac"], py, pu, pv)
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
        psnr = _psnr(rec, org)
        worst = min(worst, psnr)
        assert psnr > 30.0, (t, off, psnr)
        lib.or_hint_dyn_scroll_nal(buf, len(buf), ctypes.byref(c), off, arr, n, mode,
                                   ctypes.byref(rc), src, ctypes.byref(R.refs), ctypes.byref(err))
    print("worst PSNR", worst, "skipped rect MBs", nskip)
