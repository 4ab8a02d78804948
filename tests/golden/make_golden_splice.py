#!/usr/bin/env python3
"""Fixtures anchoring the pre-encoded MB splice to the reference's parser.

The splice has no reference implementation; the reference does contain a
CAVLC P-slice PARSER that walks mb_skip_run, P macroblocks and their
residual blocks with the standard's nC rules (experiments/trans-resizer/
trans_resizer.c process_p_slice :1486-1787, copy_cavlc_block :612-755),
compiled from the reference sources by `make -C oracle ref`
(oracle/ref_cavlc.c -> oracle/_ref/libref_cavlc.so; its geometry is fixed
at 20x20 MBs).  This script writes, through the CPU oracle
(oracle/splice_oracle.c):
  * external slices of the oracle's stand-in encoder for 20x20-MB pictures
    (P_Skip runs, several references, QP changes, escape-coded levels), and
    I pictures through the reference's I-slice walker (process_i_slice);
  * composed 320x320 scroll NALs with a spliced rect (both modes, through
    the 496 waypoint so the composed list has 3 references);
and records, per NAL, the reference parser's verdict on its MB layer (status,
the bit where it stopped) next to the NAL's SHA-256 -> tests/golden/
splice_ref.json.

    python tests/golden/make_golden_splice.py
"""
import ctypes
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import h264_pslice as hp  # noqa: E402
from dynhelp import OrCfg, ext_slice, splice_of  # noqa: E402

EXT = [  # stand-in encoder parameters for 20x20-MB external slices
    dict(),
    dict(skip_pm=700, cbp_pm=300),
    dict(nrefs=1, max_ref=0, cbp_pm=1000, big_pm=200),
    dict(nrefs=4, max_ref=3, mv_range=600, qp_jitter=10, slice_qp_delta=-6),
    dict(ref_idc=1, skip_pm=0, cbp_pm=1000),
    dict(list_mod=1, skip_pm=400),
    # partitioned MBs: P_L0_L0_16x8 / 8x16, P_8x8 (every sub_mb_type), P_8x8ref0
    dict(part_pm=600),
    dict(part_pm=1000, nrefs=3, max_ref=2, skip_pm=0, cbp_pm=800, mv_range=900),
    dict(part_pm=700, nrefs=1, max_ref=0, skip_pm=300),
    # intra MBs in P slices (the walker's I_4x4 / I_16x16 paths, :1668-1735;
    # no I_PCM: the walker resets an I_PCM MB's TotalCoeffs to 0, :1745,
    # where 9.2.1 counts 16, so it would misread the nC of its neighbours)
    dict(intra_pm=400, intra_types=3, cbp_pm=800),
    dict(intra_pm=250, intra_types=3, skip_pm=300, part_pm=300, qp_jitter=6),
]
# I pictures for the reference's I-slice walker (process_i_slice :1063-1360;
# a whole 20x20-MB picture, one slice; I_4x4 / I_16x16 everywhere -- the
# walker counts an I_PCM MB's TotalCoeffs as 0, see above): a conventional
# encoder's first frame / scene cut, spliced as P-slice intra MBs (islice 3:
# the stand-in encoder's I-slice mode with the edge ring of intra_types)
EXT_I = [
    dict(islice=3, intra_types=3, cbp_pm=800),
    dict(islice=3, intra_types=1, cbp_pm=1000, big_pm=100, qp_jitter=8),
    dict(islice=3, intra_types=2, slice_qp_delta=-5),
]
# composed frames: (offset, mode, rect) on a 320x320 stream scrolling 490..500
SPLICED = [(490 + i, i % 2, rect) for i, rect in enumerate(
    [(3, 4, 8, 6), (0, 0, 20, 20), (19, 19, 1, 1), (5, 0, 10, 3), (0, 12, 7, 8), (12, 5, 8, 9),
     (2, 2, 16, 16), (9, 9, 2, 2), (0, 0, 1, 20), (1, 18, 19, 2), (4, 4, 12, 12)])]
# the same with partitioned external MBs (scrolling on past the waypoint)
SPLICED_PART = [(501 + i, i % 2, rect) for i, rect in enumerate(
    [(3, 4, 8, 6), (0, 0, 20, 20), (19, 0, 1, 20), (6, 6, 9, 9)])]


# composed frames with intra MBs spliced from one-slice and multi-slice
# external pictures (scrolling on)
SPLICED_INTRA = [(505 + i, i % 2, rect, rows) for i, (rect, rows) in enumerate(
    [((3, 4, 8, 6), 0), ((0, 0, 20, 20), 2), ((5, 5, 10, 10), 1), ((2, 12, 16, 8), 3)])]


def _stop_bit(rbsp):
    last1 = 8 * len(rbsp) - 1
    while not (rbsp[last1 >> 3] >> (7 - (last1 & 7))) & 1:
        last1 -= 1
    return last1


def cases(oracle):
    w = h = 320
    c = OrCfg()
    oracle.or_cfg_init(ctypes.byref(c), w, h)
    c.frame_num = 2
    for k, kw in enumerate(EXT):
        nal = ext_slice(oracle, c, 20, 20, 7000 + k, **kw)
        H, b, rbsp = hp.slice_header(nal, nrefs_default=2)      # the composer's PPS
        yield dict(kind="external", case=k, nrefs=H["nrefs"], sha256=hashlib.sha256(nal).hexdigest(),
                   nal_bytes=len(nal), mb_start_bit=b.p, stop_bit=_stop_bit(rbsp)), nal, rbsp
    for k, kw in enumerate(EXT_I):
        nal = ext_slice(oracle, c, 20, 20, 7500 + k, **kw)
        H, b, rbsp = hp.slice_header(nal, nrefs_default=2)
        yield dict(kind="external-i", case=k, nrefs=H["nrefs"], sha256=hashlib.sha256(nal).hexdigest(),
                   nal_bytes=len(nal), mb_start_bit=b.p, stop_bit=_stop_bit(rbsp)), nal, rbsp
    buf = (ctypes.c_uint8 * (1 << 21))()
    err = ctypes.c_int()
    for k, (off, mode, rect) in enumerate(SPLICED + SPLICED_PART):
        if oracle.or_needs_waypoint(ctypes.byref(c), off):
            oracle.or_waypoint_nal(buf, len(buf), ctypes.byref(c), off)
        nrefs = 2 + c.nwp
        part = dict(part_pm=600) if k >= len(SPLICED) else {}
        ext = ext_slice(oracle, c, rect[2], rect[3], 8000 + k, nrefs=nrefs, max_ref=nrefs - 1,
                        skip_pm=300, cbp_pm=700, big_pm=30, qp_jitter=4, **part)
        sp = splice_of(*rect, ext)
        n = oracle.or_splice_scroll_nal(buf, len(buf), ctypes.byref(c), off, None, 0, mode,
                                        ctypes.byref(sp), ctypes.byref(err))
        assert err.value == 0 and n > 0
        nal = bytes(buf[:n])
        H, b, rbsp = hp.slice_header(nal)
        yield dict(kind="composed", case=k, off=off, mode=mode, rect=list(rect), nrefs=H["nrefs"],
                   ext_sha256=hashlib.sha256(ext).hexdigest(), sha256=hashlib.sha256(nal).hexdigest(),
                   nal_bytes=len(nal), mb_start_bit=b.p, stop_bit=_stop_bit(rbsp)), nal, rbsp
    for k, (off, mode, rect, rows) in enumerate(SPLICED_INTRA):
        if oracle.or_needs_waypoint(ctypes.byref(c), off):
            oracle.or_waypoint_nal(buf, len(buf), ctypes.byref(c), off)
        nrefs = 2 + c.nwp
        ext = ext_slice(oracle, c, rect[2], rect[3], 9000 + k, nrefs=nrefs, max_ref=nrefs - 1,
                        skip_pm=300, cbp_pm=700, big_pm=30, qp_jitter=4, intra_pm=350, intra_types=3,
                        slice_rows=rows)
        sp = splice_of(*rect, ext)
        n = oracle.or_splice_scroll_nal(buf, len(buf), ctypes.byref(c), off, None, 0, mode,
                                        ctypes.byref(sp), ctypes.byref(err))
        assert err.value == 0 and n > 0
        nal = bytes(buf[:n])
        H, b, rbsp = hp.slice_header(nal)
        yield dict(kind="composed-intra", case=k, off=off, mode=mode, rect=list(rect), slice_rows=rows,
                   nrefs=H["nrefs"], ext_sha256=hashlib.sha256(ext).hexdigest(),
                   sha256=hashlib.sha256(nal).hexdigest(), nal_bytes=len(nal), mb_start_bit=b.p,
                   stop_bit=_stop_bit(rbsp)), nal, rbsp


def main():
    oracle = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "liboracle.so"))
    ref = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref_cavlc.so"))
    out = []
    for c, nal, rbsp in cases(oracle):
        end = ctypes.c_size_t()
        if c["kind"] == "external-i":
            rc = ref.ref_cavlc_parse_i(rbsp, len(rbsp), c["mb_start_bit"], ctypes.byref(end))
        else:
            rc = ref.ref_cavlc_parse(rbsp, len(rbsp), c["mb_start_bit"], c["nrefs"], ctypes.byref(end))
        c["ref_status"], c["ref_end_bit"] = rc, end.value
        out.append(c)
    json.dump(out, open(os.path.join(HERE, "splice_ref.json"), "w"), indent=1)
    ok = sum(c["ref_status"] == 0 and c["ref_end_bit"] == c["stop_bit"] for c in out)
    print(f"splice_ref.json: {len(out)} NALs, {ok} parsed exactly by the reference")


if __name__ == "__main__":
    main()
