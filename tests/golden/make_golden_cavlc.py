#!/usr/bin/env python3
"""Fixtures for the dynamic-rect residual coder's CAVLC syntax.

The dynamic rect has no reference implementation; the reference does contain
a CAVLC P-slice PARSER (experiments/trans-resizer/trans_resizer.c
process_p_slice / copy_inter_residual / copy_cavlc_block), compiled from the
reference sources by `make -C oracle ref` (oracle/ref_cavlc.c ->
oracle/_ref/libref_cavlc.so).  This script composes 320x320 frames with a
dynamic rect through the CPU oracle (oracle/dyn_oracle.c) and records, per
NAL, the reference parser's verdict on the MB layer: its status and the bit
where it stopped, next to the NAL's SHA-256 -> tests/golden/cavlc_ref.json.

    python tests/golden/make_golden_cavlc.py
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
from dynhelp import OrCfg, Rect, StripedRefs, rect_source, split_nals  # noqa: E402

CASES = [  # (rect, stream, offsets)
    ((3, 4, 12, 10), 0, [0, 1, 17, 160, 319, 320]),
    ((0, 0, 20, 20), 5, [0, 40, 300]),                 # the whole picture is dynamic
    ((19, 19, 1, 1), 9, [7]),                          # one corner MB
    ((2, 6, 5, 3), 11, list(range(0, 320, 37))),
]


def cases(oracle):
    w = h = 320
    R = StripedRefs(oracle, w, h)
    buf = (ctypes.c_uint8 * (1 << 21))()
    for rect, s, offs in CASES:
        rc = Rect(*rect)
        cfg = OrCfg()
        oracle.or_cfg_init(ctypes.byref(cfg), w, h)
        cfg.frame_num = 2
        for t, off in enumerate(offs):
            src = rect_source(oracle, s, t, rc)
            n = oracle.or_compose_dyn(buf, len(buf), ctypes.byref(cfg), off, 0, ctypes.byref(rc), src,
                                      ctypes.byref(R.refs), None)
            nal = split_nals(bytes(buf[:n]))[-1]
            H, b, rbsp = hp.slice_header(nal)
            last1 = 8 * len(rbsp) - 1
            while not (rbsp[last1 >> 3] >> (7 - (last1 & 7))) & 1:
                last1 -= 1
            yield dict(rect=list(rect), stream=s, frame=t, off=off, nrefs=H["nrefs"],
                       sha256=hashlib.sha256(nal).hexdigest(), nal_bytes=len(nal),
                       mb_start_bit=b.p, stop_bit=last1), nal, rbsp


def main():
    oracle = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "liboracle.so"))
    ref = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref_cavlc.so"))
    out = []
    for c, nal, rbsp in cases(oracle):
        end = ctypes.c_size_t()
        rc = ref.ref_cavlc_parse(rbsp, len(rbsp), c["mb_start_bit"], c["nrefs"], ctypes.byref(end))
        c["ref_status"], c["ref_end_bit"] = rc, end.value
        out.append(c)
    json.dump(out, open(os.path.join(HERE, "cavlc_ref.json"), "w"), indent=1)
    ok = sum(c["ref_status"] == 0 and c["ref_end_bit"] == c["stop_bit"] for c in out)
    print(f"cavlc_ref.json: {len(out)} NALs, {ok} parsed exactly by the reference")


if __name__ == "__main__":
    main()
