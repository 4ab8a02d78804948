#!/usr/bin/env python3
"""Value-level pin of the dynamic-rect CAVLC coder against the reference's
own CAVLC decode functions.

The dynamic rect has no reference encoder.  The reference does hold a CAVLC
P-slice parser (experiments/trans-resizer/trans_resizer.c), compiled from the
reference sources by `make -C oracle ref` into oracle/_ref/libref_cavlc.so
(oracle/ref_cavlc.c).  For every coded block of an MB residual written by the
CPU oracle (oracle/dyn_oracle.c or_mb_residual), the reference functions
decode:
  * coded_block_pattern (bitreader_read_ue + cbp_inter_table, :284) and
    mb_qp_delta (bitreader_read_se);
  * nC (compute_luma_nC :782, compute_chroma_nC :841) from the neighbours'
    TotalCoeffs;
  * TotalCoeff, TrailingOnes and the token length (read_coeff_token :549);
  * the whole block incl. its levels (copy_cavlc_block :612) -> its end;
  * total_zeros (decode_total_zeros :467) and every run_before
    (decode_run_before :514), read from where the oracle's levels end.
Each must equal what the oracle's quantised coefficients imply.  MB sets:
every dynamic MB of the tests/golden/cavlc_ref.json NALs (real levels and
contexts, caught by the oracle's or_dyn_set_trace hook) and synthetic MBs with
escape-range levels (level_prefix 14 and 15), every suffixLength, all nC
classes.  The transform and the quantiser have no reference and stay
unpinned.

    python tests/golden/make_golden_cavlc_values.py   -> cavlc_values.json
(the SHA-256 of the reference-decoded records, so tests/test_dyn_oracle.py can
check the oracle against them where the reference build is absent).
"""
import ctypes
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import h264_pslice as hp  # noqa: E402
import make_golden_cavlc as mg  # noqa: E402
from dynhelp import OrCfg, Rect, StripedRefs, rect_source, split_nals  # noqa: E402

TRACE = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.POINTER(ctypes.c_int),
                         ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                         ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int))


class OrBits(ctypes.Structure):
    _fields_ = [("buf", ctypes.c_void_p), ("cap", ctypes.c_size_t), ("nbits", ctypes.c_size_t)]


def _nc(nA, nB):
    if nA >= 0 and nB >= 0:
        return (nA + nB + 1) >> 1
    return nA if nA >= 0 else (nB if nB >= 0 else 0)


def block_of(lv, bid):
    """coefficients (scan order) and maxNumCoeff of block bid: luma raster
    0-15, 16 / 17 chroma DC Cb / Cr, 18 + 4 p + k chroma AC"""
    luma, cdc, cac = lv
    if bid < 16:
        return luma[bid], 16
    if bid < 18:
        return cdc[bid - 16], 4
    return cac[(bid - 18) >> 2][(bid - 18) & 3], 15


def expected(oracle, lv, avail_l, avail_t, tcl, tct):
    """the oracle's side of one MB: (cbp, [per coded block in coding order:
    dict id, nC, tc, t1, tz, runs, token_len, level_end (relative to the
    block start), len])"""
    luma, cdc, cac = lv
    cbp_l = 0
    for r in range(16):
        if any(luma[r]):
            cbp_l |= 1 << ((r // 4 // 2) * 2 + (r % 4) // 2)
    any_dc = any(any(cdc[p]) for p in range(2))
    any_ac = any(any(cac[p][k]) for p in range(2) for k in range(4))
    cbp_c = 2 if any_ac else (1 if any_dc else 0)
    cbp = cbp_l | cbp_c << 4
    order = []
    if cbp:
        for blk in range(16):
            q8, q4 = blk // 4, blk % 4
            x, y = (q8 % 2) * 2 + q4 % 2, (q8 // 2) * 2 + q4 // 2
            if cbp_l >> q8 & 1:
                order.append(4 * y + x)
        if cbp_c:
            order += [16, 17]
        if cbp_c == 2:
            order += list(range(18, 26))
    cur = [0] * 24
    ob = (ctypes.c_uint8 * 1024)()
    out = []
    for bid in order:
        coef, maxc = block_of(lv, bid)
        if bid < 16:
            x, y = bid % 4, bid // 4
            nA = cur[bid - 1] if x > 0 else (tcl[bid + 3] if avail_l else -1)
            nB = cur[bid - 4] if y > 0 else (tct[bid + 12] if avail_t else -1)
            nC = _nc(nA, nB)
        elif bid < 18:
            nC = -1
        else:
            i = bid - 2                                   # index into the 24 TotalCoeffs
            k = (bid - 18) & 3
            x, y = k % 2, k // 2
            nA = cur[i - 1] if x > 0 else (tcl[i + 1] if avail_l else -1)
            nB = cur[i - 2] if y > 0 else (tct[i + 2] if avail_t else -1)
            nC = _nc(nA, nB)
        nz = [p for p in range(maxc) if coef[p]]
        tc = len(nz)
        t1 = 0
        for p in reversed(nz):
            if t1 == 3 or coef[p] not in (1, -1):
                break
            t1 += 1
        tz = (nz[-1] + 1 - tc) if tc and tc < maxc else 0
        runs, zl = [], tz
        for j in range(tc - 1, 0, -1):
            if zl <= 0:
                break
            run = nz[j] - nz[j - 1] - 1
            runs.append(run)
            zl -= run
        b = OrBits()
        oracle.or_bits_init(ctypes.byref(b), ob, len(ob))
        got = oracle.or_cavlc_block(ctypes.byref(b), (ctypes.c_int * 16)(*coef, *([0] * (16 - len(coef)))), maxc, nC)
        assert got == tc
        code = ctypes.c_uint32()
        tl = oracle.or_ct_code(tc, t1, nC, ctypes.byref(code))
        zlen = oracle.or_tz_code(tc, tz, maxc, ctypes.byref(code)) if tc and tc < maxc else 0
        rl, zl = 0, tz
        for run in runs:
            rl += oracle.or_rb_code(zl, run, ctypes.byref(code))
            zl -= run
        n = b.nbits
        lev_end = n - zlen - rl
        if bid < 16:
            cur[bid] = tc
        elif bid >= 18:
            cur[bid - 2] = tc
        out.append(dict(id=bid, nC=nC, tc=tc, t1=t1, tz=tz, runs=runs, token_len=tl, level_end=lev_end, len=n))
    return cbp, out


def ref_decode(ref, rbsp, start, avail_l, avail_t, tcl, tct, exp):
    """the reference's side: ref_cavlc_mb, then ref_cavlc_tail at the oracle's
    level end of each block -> (cbp, qp_delta, [per block dict])"""
    data = bytes(rbsp[start >> 3:]) + b"\x00" * 8
    s0 = start & 7
    rec = ((ctypes.c_longlong * 7) * 26)()
    cbp, qpd = ctypes.c_int(), ctypes.c_int()
    nb = ref.ref_cavlc_mb(data, len(data), s0, avail_l, avail_t, (ctypes.c_int * 24)(*tcl),
                          (ctypes.c_int * 24)(*tct), ctypes.byref(cbp), ctypes.byref(qpd), rec)
    assert nb >= 0, "reference decode failed"
    out = []
    for i in range(nb):
        bid, nC, tc, t1, bs, te, be = (int(v) for v in rec[i])
        d = dict(id=bid, nC=nC, tc=tc, t1=t1, token_len=te - bs, len=be - bs, tz=None, runs=None)
        if i < len(exp) and tc:
            tz, runs, end = ctypes.c_int(), (ctypes.c_int * 16)(), ctypes.c_size_t()
            nr = ref.ref_cavlc_tail(data, len(data), bs + exp[i]["level_end"], tc, block_max(bid),
                                    ctypes.byref(tz), runs, ctypes.byref(end))
            assert nr >= 0, "reference total_zeros / run_before decode failed"
            d["tz"], d["runs"] = tz.value, list(runs[:nr])
            d["tail_end"] = int(end.value) - bs
            codes, sg, tcl2 = (ctypes.c_int * 16)(), ctypes.c_int(), ctypes.c_int()
            nl = ref.ref_cavlc_levels(data, len(data), bs, nC, block_max(bid), codes, ctypes.byref(sg),
                                      ctypes.byref(tcl2))
            assert nl == tc - t1 and tcl2.value == tc, "reference level decode failed"
            d["levels"] = [level_of(c) for c in codes[:nl]]
            d["signs"] = sg.value
        elif tc == 0:
            d["tz"], d["runs"], d["tail_end"] = 0, [], d["len"]
        out.append(d)
    return cbp.value, qpd.value, out


def level_of(code):
    """levelVal of a levelCode (9.2.2.1; the reference's formula,
    trans_resizer.c:696-697)"""
    v = (code + 2) >> 1
    return -v if code & 1 else v


def coefficients(d, maxc):
    """the block's coefficient vector (scan order) from the reference-decoded
    fields: trailing ones (signs), levels, total_zeros, runs (9.2.4)"""
    tc, t1 = d["tc"], d["t1"]
    if tc == 0:
        return [0] * maxc
    lev = [-1 if d["signs"] >> (t1 - 1 - i) & 1 else 1 for i in range(t1)] + d["levels"]
    runs = list(d["runs"]) + [0] * tc
    zl = d["tz"]
    coef = [0] * maxc
    p = tc + d["tz"] - 1                               # scan index of the highest level
    for i in range(tc):
        coef[p] = lev[i]
        r = runs[i] if i < tc - 1 and zl > 0 else (zl if i == tc - 1 else 0)
        if i < tc - 1:
            zl -= r
            p -= r + 1
    return coef


def block_max(bid):
    return 16 if bid < 16 else (4 if bid < 18 else 15)


def _read_levels(luma_p, cdc_p, cac_p):
    luma = [[luma_p[16 * r + k] for k in range(16)] for r in range(16)]
    cdc = [[cdc_p[4 * p + k] for k in range(4)] for p in range(2)]
    cac = [[[cac_p[60 * p + 15 * k + i] for i in range(15)] for k in range(4)] for p in range(2)]
    return luma, cdc, cac


def nal_mbs(oracle):
    """every dynamic MB of the cavlc_ref.json NALs: (tag, rbsp, start bit,
    avail_l, avail_t, tcl, tct, levels)"""
    w = h = 320
    R = StripedRefs(oracle, w, h)
    buf = (ctypes.c_uint8 * (1 << 21))()
    for rect, s, offs in mg.CASES:
        rc = Rect(*rect)
        cfg = OrCfg()
        oracle.or_cfg_init(ctypes.byref(cfg), w, h)
        cfg.frame_num = 2
        for t, off in enumerate(offs):
            src = rect_source(oracle, s, t, rc)
            got = []

            def cb(x, y, bit, lp, dp, ap, tl, tt):
                got.append((x, y, int(bit), _read_levels(lp, dp, ap),
                            [tl[i] for i in range(24)] if tl else [0] * 24,
                            [tt[i] for i in range(24)] if tt else [0] * 24, bool(tl), bool(tt)))

            fn = TRACE(cb)
            oracle.or_dyn_set_trace(fn)
            try:
                n = oracle.or_compose_dyn(buf, len(buf), ctypes.byref(cfg), off, 0, ctypes.byref(rc), src,
                                          ctypes.byref(R.refs), None)
            finally:
                oracle.or_dyn_set_trace(None)
            nal = split_nals(bytes(buf[:n]))[-1]
            _, _, rbsp = hp.slice_header(nal)
            for x, y, bit, lv, tcl, tct, al, at in got:
                yield (f"nal {rect} s{s} t{t} mb({x},{y})", rbsp, bit, int(al), int(at), tcl, tct, lv)


def _synth_block(rng, maxc):
    """levels: empty, sparse / dense, trailing ones, and magnitudes up to the
    12-bit escape (|level| <= 2000 stays inside level_prefix 15)"""
    c = [0] * maxc
    kind = rng.random()
    if kind < 0.12:
        return c
    nnz = rng.randint(1, maxc)
    for p in rng.sample(range(maxc), nnz):
        r = rng.random()
        if r < 0.35:
            c[p] = rng.choice([-1, 1])
        elif r < 0.55:
            c[p] = rng.choice([-1, 1]) * rng.randint(2, 9)          # sl 0 codes 14..29: prefix 14
        elif r < 0.75:
            c[p] = rng.choice([-1, 1]) * rng.randint(8, 60)
        elif r < 0.9:
            c[p] = rng.choice([-1, 1]) * rng.randint(60, 400)
        else:
            c[p] = rng.choice([-1, 1]) * rng.randint(400, 2000)     # prefix 15 at every suffixLength
    return c


def synth_mbs(oracle, n=600, seed=4):
    """synthetic MBs written by or_dyn_mb_levels_bits (the oracle's MB residual
    writer) with random neighbour TotalCoeffs (every nC class incl. >= 8)"""
    rng = random.Random(seed)
    buf = (ctypes.c_uint8 * (1 << 16))()
    for i in range(n):
        dens = rng.random()

        def blk(maxc):
            return _synth_block(rng, maxc) if rng.random() < dens + 0.2 else [0] * maxc

        luma = [blk(16) for _ in range(16)]
        cdc = [blk(4) for _ in range(2)]
        cac = [[blk(15) for _ in range(4)] for _ in range(2)]
        al, at = rng.random() < 0.8, rng.random() < 0.8
        tcl = [rng.choice([0, 0, 1, 2, 3, 4, 5, 7, 8, 11, 16]) if k < 16 else rng.randint(0, 15) for k in range(24)]
        tct = [rng.choice([0, 1, 2, 3, 4, 6, 8, 9, 13, 16]) if k < 16 else rng.randint(0, 15) for k in range(24)]
        L = ((ctypes.c_int * 16) * 16)(*[(ctypes.c_int * 16)(*r) for r in luma])
        D = ((ctypes.c_int * 4) * 2)(*[(ctypes.c_int * 4)(*r) for r in cdc])
        A = (((ctypes.c_int * 15) * 4) * 2)(*[((ctypes.c_int * 15) * 4)(*[(ctypes.c_int * 15)(*b) for b in p])
                                               for p in cac])
        cbp, tco, nbits = ctypes.c_int(), (ctypes.c_int * 24)(), ctypes.c_size_t()
        nby = oracle.or_dyn_mb_levels_bits(buf, len(buf), L, D, A, (ctypes.c_int * 24)(*tcl),
                                           (ctypes.c_int * 24)(*tct), int(al), int(at), ctypes.byref(cbp), tco,
                                           ctypes.byref(nbits))
        yield (f"synth {i}", bytes(buf[:nby]), 0, int(al), int(at), tcl, tct, (luma, cdc, cac))


def all_mbs(oracle):
    yield from nal_mbs(oracle)
    yield from synth_mbs(oracle)


def oracle_records(lv, exp):
    """per-block records of the oracle's side (the same form as check_mb's)"""
    return [[e["id"], e["nC"], e["token_len"], e["len"], list(block_of(lv, e["id"])[0])] for e in exp]


def check_mb(oracle, ref, case):
    """decode one MB with the reference functions and assert every value
    equals the oracle's; returns the reference's per-block records"""
    tag, rbsp, start, al, at, tcl, tct, lv = case
    cbp, exp = expected(oracle, lv, al, at, tcl, tct)
    rcbp, qpd, got = ref_decode(ref, rbsp, start, al, at, tcl, tct, exp)
    assert (rcbp, qpd) == (cbp, 0), tag
    assert [g["id"] for g in got] == [e["id"] for e in exp], tag
    recs = []
    for g, e in zip(got, exp):
        where = f"{tag} block {e['id']}"
        assert g["nC"] == e["nC"], where
        assert (g["tc"], g["t1"], g["token_len"]) == (e["tc"], e["t1"], e["token_len"]), where
        assert (g["tz"], g["runs"]) == (e["tz"], e["runs"]), where
        assert g["tail_end"] == g["len"] == e["len"], where
        coef, maxc = block_of(lv, e["id"])
        assert coefficients(g, maxc) == list(coef), where
        recs.append([g["id"], g["nC"], g["token_len"], g["len"], coefficients(g, maxc)])
    return recs


def escapes(lv):
    """level_prefix 14 / 15 events of an MB's levels as the oracle codes them
    (9.2.2.1): (prefix 14 at suffixLength 0, prefix 15 at 0, prefix 15 at > 0)"""
    e14 = e15a = e15b = 0
    luma, cdc, cac = lv
    blocks = list(luma) + list(cdc) + [b for p in cac for b in p]
    for coef in blocks:
        nz = [p for p in range(len(coef)) if coef[p]]
        tc = len(nz)
        t1 = 0
        for p in reversed(nz):
            if t1 == 3 or coef[p] not in (1, -1):
                break
            t1 += 1
        sl = 1 if tc > 10 and t1 < 3 else 0
        for j, p in enumerate(reversed(nz[:tc - t1])):
            v = coef[p]
            code = 2 * abs(v) - 2 + (v < 0) - (2 if j == 0 and t1 < 3 else 0)
            if sl == 0:
                e14 += 14 <= code < 30
                e15a += code >= 30
            else:
                e15b += code >= (15 << sl)
            sl = max(sl, 1)
            if abs(v) > (3 << (sl - 1)) and sl < 6:
                sl += 1
    return e14, e15a, e15b


def digest(records):
    return hashlib.sha256(json.dumps(records, separators=(",", ":")).encode()).hexdigest()


def main():
    oracle = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "liboracle.so"))
    ref = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref_cavlc.so"))
    recs, nmb = [], 0
    for case in all_mbs(oracle):
        recs += check_mb(oracle, ref, case)
        nmb += 1
    out = dict(mbs=nmb, blocks=len(recs), sha256=digest(recs),
               note="SHA-256 of the reference-decoded per-block records "
                    "[id, nC, coeff_token bits, block bits, coefficients decoded from TotalCoeff / "
                    "TrailingOnes / sign bits / levels / total_zeros / run_before], each asserted equal to "
                    "the oracle's")
    json.dump(out, open(os.path.join(HERE, "cavlc_values.json"), "w"), indent=1)
    print(f"cavlc_values.json: {nmb} MBs, {len(recs)} blocks decoded by the reference")


if __name__ == "__main__":
    main()
