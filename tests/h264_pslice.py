"""TEST-ONLY H.264 P-slice parser / reconstructor for the composer's NALs.

Parses the slices this repository emits (CAVLC, P_L0_16x16 MBs, no skips) --
slice header (7.3.3), mb layer (7.3.5), residual (7.3.5.3, CAVLC 9.2) -- and
reconstructs the dynamic MBs (dequantisation 8.5.12.1, inverse transform
8.5.12.2, chroma DC 8.5.11) on top of their inter prediction, so tests can
check the residual coder end to end against the source pixels.  Written from
the standard; its CAVLC tables are independent of the encoder's (oracle and
device code) and of the reference's parser.
"""

# ---------------------------------------------------------------- bits -------

def ebsp_to_rbsp(b):
    out, zeros = bytearray(), 0
    for x in b:
        if zeros >= 2 and x == 3:
            zeros = 0
            continue
        out.append(x)
        zeros = zeros + 1 if x == 0 else 0
    return bytes(out)


class Bits:
    def __init__(self, data, pos=0):
        self.d, self.p = data, pos

    def u(self, n):
        v = 0
        for _ in range(n):
            v = (v << 1) | ((self.d[self.p >> 3] >> (7 - (self.p & 7))) & 1)
            self.p += 1
        return v

    def ue(self):
        z = 0
        while self.u(1) == 0:
            z += 1
        return (1 << z) - 1 + (self.u(z) if z else 0)

    def se(self):
        k = self.ue()
        return (k + 1) // 2 if k & 1 else -(k // 2)


# ------------------------------------------------------------ CAVLC ---------
# Table 9-5: code -> (TotalCoeff, TrailingOnes) per nC class (0: 0<=nC<2, 2: 2<=nC<4,
# 4: 4<=nC<8, -1: chroma DC); nC >= 8 is a 6-bit FLC.
CT_TABLES = {}


def _init_tables():
    # explicit (tc, t1) -> code per class (Table 9-5), written out to avoid
    # ambiguity with fillers
    rows = {
        0: [["1"], ["000101", "01"], ["00000111", "000100", "001"],
            ["000000111", "00000110", "0000101", "00011"],
            ["0000000111", "000000110", "00000101", "000011"],
            ["00000000111", "0000000110", "000000101", "0000100"],
            ["0000000001111", "00000000110", "0000000101", "00000100"],
            ["0000000001011", "0000000001110", "00000000101", "000000100"],
            ["0000000001000", "0000000001010", "0000000001101", "0000000100"],
            ["00000000001111", "00000000001110", "0000000001001", "00000000100"],
            ["00000000001011", "00000000001010", "00000000001101", "0000000001100"],
            ["000000000001111", "000000000001110", "00000000001001", "00000000001100"],
            ["000000000001011", "000000000001010", "000000000001101", "00000000001000"],
            ["0000000000001111", "000000000000001", "000000000001001", "000000000001100"],
            ["0000000000001011", "0000000000001110", "0000000000001101", "000000000001000"],
            ["0000000000000111", "0000000000001010", "0000000000001001", "0000000000001100"],
            ["0000000000000100", "0000000000000110", "0000000000000101", "0000000000001000"]],
        2: [["11"], ["001011", "10"], ["000111", "00111", "011"],
            ["0000111", "001010", "001001", "0101"],
            ["00000111", "000110", "000101", "0100"],
            ["00000100", "0000110", "0000101", "00110"],
            ["000000111", "00000110", "00000101", "001000"],
            ["00000001111", "000000110", "000000101", "000100"],
            ["00000001011", "00000001110", "00000001101", "0000100"],
            ["000000001111", "00000001010", "00000001001", "000000100"],
            ["000000001011", "000000001110", "000000001101", "00000001100"],
            ["000000001000", "000000001010", "000000001001", "00000001000"],
            ["0000000001111", "0000000001110", "0000000001101", "000000001100"],
            ["0000000001011", "0000000001010", "0000000001001", "0000000001100"],
            ["0000000000111", "00000000001011", "0000000000110", "0000000001000"],
            ["00000000001001", "00000000001000", "00000000001010", "0000000000001"],
            ["00000000000111", "00000000000110", "00000000000101", "00000000000100"]],
        4: [["1111"], ["001111", "1110"], ["001011", "01111", "1101"],
            ["001000", "01100", "01110", "1100"],
            ["0001111", "01010", "01011", "1011"],
            ["0001011", "01000", "01001", "1010"],
            ["0001001", "001110", "001101", "1001"],
            ["0001000", "001010", "001001", "1000"],
            ["00001111", "0001110", "0001101", "01101"],
            ["00001011", "00001110", "0001010", "001100"],
            ["000001111", "00001010", "00001101", "0001100"],
            ["000001011", "000001110", "00001001", "00001100"],
            ["000001000", "000001010", "000001101", "00001000"],
            ["0000001101", "000000111", "000001001", "000001100"],
            ["0000001001", "0000001100", "0000001011", "0000001010"],
            ["0000000101", "0000001000", "0000000111", "0000000110"],
            ["0000000001", "0000000100", "0000000011", "0000000010"]],
    }
    for nc, rr in rows.items():
        d = {}
        for tc, row in enumerate(rr):
            for t1, code in enumerate(row):
                d[code] = (tc, t1)
        CT_TABLES[nc] = d
    dc = [["01"], ["000111", "1"], ["000100", "000110", "001"],
          ["000011", "0000011", "0000010", "000101"],
          ["000010", "00000011", "00000010", "0000000"]]
    d = {}
    for tc, row in enumerate(dc):
        for t1, code in enumerate(row):
            d[code] = (tc, t1)
    CT_TABLES[-1] = d


_init_tables()

# total_zeros, Tables 9-7 / 9-8: TZ[tc] = list of codes for total_zeros 0..16-tc
TZ = {
    1: "1 011 010 0011 0010 00011 00010 000011 000010 0000011 0000010 00000011 00000010 000000011 000000010 000000001",
    2: "111 110 101 100 011 0101 0100 0011 0010 00011 00010 000011 000010 000001 000000",
    3: "0101 111 110 101 0100 0011 100 011 0010 00011 00010 000001 00001 000000",
    4: "00011 111 0101 0100 110 101 100 0011 011 0010 00010 00001 00000",
    5: "0101 0100 0011 111 110 101 100 011 0010 00001 0001 00000",
    6: "000001 00001 111 110 101 100 011 010 0001 001 000000",
    7: "000001 00001 101 100 011 11 010 0001 001 000000",
    8: "000001 0001 00001 011 11 10 010 001 000000",
    9: "000001 000000 0001 11 10 001 01 00001",
    10: "00001 00000 001 11 10 01 0001",
    11: "0000 0001 001 010 1 011",
    12: "0000 0001 01 1 001",
    13: "000 001 1 01",
    14: "00 01 1",
    15: "0 1",
}
TZ = {k: {c: i for i, c in enumerate(v.split())} for k, v in TZ.items()}
TZDC = {1: {"1": 0, "01": 1, "001": 2, "000": 3}, 2: {"1": 0, "01": 1, "00": 2}, 3: {"1": 0, "0": 1}}
RB = {
    1: {"1": 0, "0": 1}, 2: {"1": 0, "01": 1, "00": 2}, 3: {"11": 0, "10": 1, "01": 2, "00": 3},
    4: {"11": 0, "10": 1, "01": 2, "001": 3, "000": 4},
    5: {"11": 0, "10": 1, "011": 2, "010": 3, "001": 4, "000": 5},
    6: {"11": 0, "000": 1, "001": 2, "011": 3, "010": 4, "101": 5, "100": 6},
    7: {"111": 0, "110": 1, "101": 2, "100": 3, "011": 4, "010": 5, "001": 6, "0001": 7,
        "00001": 8, "000001": 9, "0000001": 10, "00000001": 11, "000000001": 12,
        "0000000001": 13, "00000000001": 14},
}


def _match(bits, table, maxlen=16):
    s = ""
    for _ in range(maxlen):
        s += str(bits.u(1))
        if s in table:
            return table[s]
    raise ValueError("no VLC match: " + s)


def cavlc_block(bits, nC, maxc):
    """-> (coefficients in scan order [maxc], TotalCoeff)"""
    if nC == -1:
        tc, t1 = _match(bits, CT_TABLES[-1])
    elif nC >= 8:
        code = bits.u(6)
        tc, t1 = (0, 0) if code == 3 else ((code >> 2) + 1, code & 3)
    else:
        tc, t1 = _match(bits, CT_TABLES[0 if nC < 2 else (2 if nC < 4 else 4)])
    coef = [0] * maxc
    if tc == 0:
        return coef, 0
    lv = []
    for _ in range(t1):
        lv.append(-1 if bits.u(1) else 1)
    sl = 1 if (tc > 10 and t1 < 3) else 0
    for i in range(tc - t1):
        prefix = 0
        while bits.u(1) == 0:
            prefix += 1
        code = (min(15, prefix) << sl)
        if sl > 0 or prefix >= 14:
            ssize = sl
            if prefix == 14 and sl == 0:
                ssize = 4
            if prefix >= 15:
                ssize = prefix - 3
            if ssize:
                code += bits.u(ssize)
        if prefix >= 15 and sl == 0:
            code += 15
        if i == 0 and t1 < 3:
            code += 2
        level = (code + 2) >> 1 if code % 2 == 0 else -((code + 1) >> 1)
        lv.append(level)
        if sl == 0:
            sl = 1
        if abs(level) > (3 << (sl - 1)) and sl < 6:
            sl += 1
    tz = 0
    if tc < maxc:
        tz = _match(bits, TZDC[tc] if maxc == 4 else TZ[tc])
    runs, zl = [], tz
    for i in range(tc - 1):
        r = _match(bits, RB[min(zl, 7)]) if zl > 0 else 0
        runs.append(r)
        zl -= r
    runs.append(zl)
    pos = tc + tz - 1
    for i in range(tc):
        coef[pos] = lv[i]
        pos -= 1 + runs[i]
    return coef, tc


# ------------------------------------------------------- reconstruction ----
ZZ = [0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15]
V = [[10, 16, 13], [11, 18, 14], [13, 20, 16], [14, 23, 18], [16, 25, 20], [18, 29, 23]]
GOLOMB_TO_INTER_CBP = [0, 16, 1, 2, 4, 8, 32, 3, 5, 10, 12, 15, 47, 7, 11, 13, 14, 6, 9, 31, 35,
                       37, 42, 44, 33, 34, 36, 40, 39, 43, 45, 46, 17, 18, 20, 24, 19, 21, 26, 28,
                       23, 27, 29, 30, 22, 25, 38, 41]


def _cls(i, j):
    return 0 if (i % 2 == 0 and j % 2 == 0) else (1 if (i % 2 and j % 2) else 2)


def dequant4x4(scan, qp, dc=None):
    c = [0] * 16
    for k in range(16):
        c[ZZ[k]] = scan[k]
    d = [0] * 16
    for p in range(16):
        i, j = divmod(p, 4)
        d[p] = (c[p] * V[qp % 6][_cls(i, j)]) << (qp // 6)
    if dc is not None:
        d[0] = dc
    return d


def idct4x4(d):
    t = [0] * 16
    for i in range(4):
        r = d[4 * i:4 * i + 4]
        e0, e1 = r[0] + r[2], r[0] - r[2]
        e2, e3 = (r[1] >> 1) - r[3], r[1] + (r[3] >> 1)
        t[4 * i:4 * i + 4] = [e0 + e3, e1 + e2, e1 - e2, e0 - e3]
    out = [0] * 16
    for j in range(4):
        c = [t[j], t[4 + j], t[8 + j], t[12 + j]]
        e0, e1 = c[0] + c[2], c[0] - c[2]
        e2, e3 = (c[1] >> 1) - c[3], c[1] + (c[3] >> 1)
        for i, v in enumerate([e0 + e3, e1 + e2, e1 - e2, e0 - e3]):
            out[4 * i + j] = (v + 32) >> 6
    return out


def slice_header(nal, log2_mfn=4, poc_type=2, log2_poc=4, deblock=1, nrefs_default=1):
    """-> (header dict, Bits positioned at the first MB, RBSP bytes);
    nrefs_default: num_ref_idx_l0_active without an override (the composer's
    PPS: 2)"""
    assert nal[:4] == b"\x00\x00\x00\x01"
    ref_idc, nut = nal[4] >> 5, nal[4] & 31
    b = Bits(ebsp_to_rbsp(nal[5:]))
    H = {"first_mb": b.ue(), "slice_type": b.ue(), "pps": b.ue(), "frame_num": b.u(log2_mfn)}
    islice = H["slice_type"] in (2, 7)
    if nut == 5:
        H["idr_pic_id"] = b.ue()
    if poc_type == 0:
        H["poc"] = b.u(log2_poc)
    nrefs = nrefs_default
    if not islice and b.u(1):
        nrefs = b.ue() + 1
    H["nrefs"] = nrefs
    if not islice and b.u(1):
        while True:
            idc = b.ue()
            if idc == 3:
                break
            b.ue()
    if ref_idc and nut == 5:
        b.u(2)                                   # no_output_of_prior_pics, long_term_reference
    elif ref_idc:
        if b.u(1):
            while True:
                op = b.ue()
                if op == 0:
                    break
                if op in (1, 3):
                    b.ue()
                if op in (2, 3, 6):
                    b.ue()
                if op == 4:
                    b.ue()
    H["qp_delta"] = b.se()
    if deblock:
        if b.ue() != 1:
            b.se(); b.se()
    return H, b, b.d


def parse_p_slice(nal, w, h, log2_mfn=4, poc_type=2, log2_poc=4, deblock=1, on_mb=None):
    """Parse one P-slice NAL (Annex-B bytes).  on_mb(x, y, ref, mvd, cbp,
    luma, cdc, cac) is called per MB with the decoded levels.  Returns the
    header dict and the MB count."""
    assert nal[:4] == b"\x00\x00\x00\x01"
    hdr = nal[4]
    ref_idc, nut = hdr >> 5, hdr & 31
    b = Bits(ebsp_to_rbsp(nal[5:]))
    H = {"first_mb": b.ue(), "slice_type": b.ue(), "pps": b.ue(), "frame_num": b.u(log2_mfn)}
    if poc_type == 0:
        H["poc"] = b.u(log2_poc)
    nrefs = 1
    if b.u(1):
        nrefs = b.ue() + 1
    H["nrefs"] = nrefs
    if b.u(1):                                   # ref_pic_list_modification
        while True:
            idc = b.ue()
            if idc == 3:
                break
            b.ue()
    if ref_idc:
        if b.u(1):                               # adaptive ref pic marking
            while True:
                op = b.ue()
                if op == 0:
                    break
                if op in (1, 3):
                    b.ue()
                if op in (2, 3, 6):
                    b.ue()
                if op == 4:
                    b.ue()
    H["qp_delta"] = b.se()
    if deblock:
        if b.ue() != 1:
            b.se(); b.se()
    mbw, mbh = w // 16, h // 16
    tc_above = [None] * mbw
    n = 0
    for y in range(mbh):
        left = None
        for x in range(mbw):
            assert b.ue() == 0, "mb_skip_run"
            assert b.ue() == 0, "mb_type"
            if nrefs == 2:
                ref = 1 - b.u(1)
            elif nrefs > 2:
                ref = b.ue()
            else:
                ref = 0
            mvd = (b.se(), b.se())
            cbp = GOLOMB_TO_INTER_CBP[b.ue()]
            tcs = [0] * 24
            luma = [[0] * 16 for _ in range(16)]
            cdc = [[0] * 4 for _ in range(2)]
            cac = [[[0] * 15 for _ in range(4)] for _ in range(2)]
            if cbp:
                b.se()                           # mb_qp_delta
                top = tc_above[x]
                for blk in range(16):
                    q8, q4 = divmod(blk, 4)
                    bx, by = (q8 % 2) * 2 + q4 % 2, (q8 // 2) * 2 + q4 // 2
                    r = 4 * by + bx
                    if not cbp & (1 << q8):
                        continue
                    nA = tcs[r - 1] if bx > 0 else (left[r + 3] if left else -1)
                    nB = tcs[r - 4] if by > 0 else (top[r + 12] if top else -1)
                    nc = (nA + nB + 1) >> 1 if nA >= 0 and nB >= 0 else (nA if nA >= 0 else (nB if nB >= 0 else 0))
                    luma[r], tcs[r] = cavlc_block(b, nc, 16)
                if cbp >> 4:
                    for p in range(2):
                        cdc[p], _ = cavlc_block(b, -1, 4)
                    if (cbp >> 4) == 2:
                        for p in range(2):
                            for k in range(4):
                                bx, by = k % 2, k // 2
                                i = 16 + 4 * p + k
                                nA = tcs[i - 1] if bx > 0 else (left[i + 1] if left else -1)
                                nB = tcs[i - 2] if by > 0 else (top[i + 2] if top else -1)
                                nc = (nA + nB + 1) >> 1 if nA >= 0 and nB >= 0 else (nA if nA >= 0 else (nB if nB >= 0 else 0))
                                cac[p][k], tcs[i] = cavlc_block(b, nc, 15)
            if on_mb:
                on_mb(x, y, ref, mvd, cbp, luma, cdc, cac)
            tc_above[x] = tcs
            left = tcs
            n += 1
    # rbsp_stop_one_bit + alignment
    assert b.u(1) == 1, "stop bit"
    while b.p & 7:
        assert b.u(1) == 0
    assert b.p == 8 * len(b.d), (b.p, 8 * len(b.d))
    return H, n


def reconstruct_mb(luma, cdc, cac, pred_y, pred_u, pred_v, qp=26, qpc=26):
    """Residual + prediction of one MB: pred_* are 16x16 / 8x8 lists (rows)."""
    ry = [[0] * 16 for _ in range(16)]
    for r in range(16):
        res = idct4x4(dequant4x4(luma[r], qp))
        bx, by = 4 * (r % 4), 4 * (r // 4)
        for i in range(4):
            for j in range(4):
                ry[by + i][bx + j] = min(255, max(0, pred_y[by + i][bx + j] + res[4 * i + j]))
    out_c = []
    for p, pred in enumerate((pred_u, pred_v)):
        c = cdc[p]
        f = [c[0] + c[1] + c[2] + c[3], c[0] - c[1] + c[2] - c[3],
             c[0] + c[1] - c[2] - c[3], c[0] - c[1] - c[2] + c[3]]
        # 8.5.11.2: dcC = ((f * LevelScale4x4(qPc % 6, 0, 0)) << (qPc / 6)) >> 5 with
        # LevelScale4x4 = 16 * V for flat weights
        dcs = [((v * 16 * V[qpc % 6][0]) << (qpc // 6)) >> 5 for v in f]
        rc = [[0] * 8 for _ in range(8)]
        for k in range(4):
            scan = [0] + cac[p][k]
            res = idct4x4(dequant4x4(scan, qpc, dc=dcs[k]))
            bx, by = 4 * (k % 2), 4 * (k // 2)
            for i in range(4):
                for j in range(4):
                    rc[by + i][bx + j] = min(255, max(0, pred[by + i][bx + j] + res[4 * i + j]))
        out_c.append(rc)
    return ry, out_c[0], out_c[1]


# --------------------------------------------------- MV field (UI hints) -----
# Decodes the motion of a residual-free P slice: mb_skip_run (7.3.4), P_Skip
# motion (8.4.1.1), P_L0_16x16 with mvd + prediction.  predictor="spec" is
# the standard's median prediction (8.4.1.3); "ref" is the reference
# composer's get_mv_prediction (src/h264_writer.c:369-432, median3 :362-367),
# which its P slices (and the hint EXACT mode) are written with.

def _med(a, b, c):
    return sorted((a, b, c))[1]


def _ref_median3(a, b, c):
    if a > b:
        a, b = b, a
    if b > c:
        b = c
    if a > b:
        a = b
    return max(a, b)


def _neigh(field, x, y, mbw):
    """A, B, C-or-D as (ref, mx, my) or None"""
    A = field[y][x - 1] if x > 0 else None
    B = field[y - 1][x] if y > 0 else None
    if y > 0 and x + 1 < mbw:
        C = field[y - 1][x + 1]
    elif y > 0 and x > 0:
        C = field[y - 1][x - 1]
    else:
        C = None
    return A, B, C


def mvp_spec(A, B, C, ref):
    if B is None and C is None and A is not None:
        B = C = A
    nb = [n for n in (A, B, C)]
    match = [n is not None and n[0] == ref for n in nb]
    if sum(match) == 1:
        n = nb[match.index(True)]
        return n[1], n[2]
    v = [(0, 0) if n is None else (n[1], n[2]) for n in nb]
    return _med(v[0][0], v[1][0], v[2][0]), _med(v[0][1], v[1][1], v[2][1])


def mvp_ref(A, B, C, ref):
    nb = (A, B, C)
    avail = [n is not None for n in nb]
    match = [n is not None and n[0] == ref for n in nb]
    if sum(avail) == 0:
        return 0, 0
    if sum(avail) == 1:
        n = nb[avail.index(True)]
        return (n[1], n[2]) if n[0] == ref else (0, 0)
    if sum(match) == 1:
        n = nb[match.index(True)]
        return n[1], n[2]
    v = [(0, 0) if n is None else (n[1], n[2]) for n in nb]
    return _ref_median3(v[0][0], v[1][0], v[2][0]), _ref_median3(v[0][1], v[1][1], v[2][1])


def pskip_mv(A, B, C):
    if A is None or B is None or (A[0] == 0 and A[1] == 0 and A[2] == 0) or \
            (B[0] == 0 and B[1] == 0 and B[2] == 0):
        return 0, 0
    return mvp_spec(A, B, C, 0)


def decode_mv_field(nal, w, h, predictor="spec", **hdr_kw):
    """-> (header, field[y][x] = (ref, mx, my) in quarter pels, skipped MBs)"""
    H, b, data = slice_header(nal, **hdr_kw)
    pred = mvp_spec if predictor == "spec" else mvp_ref
    mbw, mbh = w // 16, h // 16
    field = [[None] * mbw for _ in range(mbh)]
    m, nskip, nrefs = 0, 0, H["nrefs"]
    while m < mbw * mbh:
        run = b.ue()
        for _ in range(run):
            y, x = divmod(m, mbw)
            assert y < mbh, "mb_skip_run past the picture"
            field[y][x] = (0,) + pskip_mv(*_neigh(field, x, y, mbw))
            m += 1
            nskip += 1
        if m >= mbw * mbh:
            break
        y, x = divmod(m, mbw)
        assert b.ue() == 0, "mb_type P_L0_16x16"
        ref = (1 - b.u(1)) if nrefs == 2 else (b.ue() if nrefs > 2 else 0)
        dx, dy = b.se(), b.se()
        assert b.ue() == 0, "coded_block_pattern"
        px, py = pred(*_neigh(field, x, y, mbw), ref)
        field[y][x] = (ref, px + dx, py + dy)
        m += 1
    assert b.u(1) == 1, "stop bit"
    while b.p & 7:
        assert b.u(1) == 0
    assert b.p == 8 * len(data), (b.p, 8 * len(data))
    return H, field, nskip


# ------------------------------------------- general P slice (splice) --------
# Any CAVLC P slice of inter MBs (P_L0_16x16, P_L0_L0_16x8 / 8x16, P_8x8 with
# sub_mb_types, P_8x8ref0) and P_Skip: mb_skip_run, motion per 4x4 block with
# the chosen predictor (partitions always with the standard's: 8.4.1.3 with the
# directional 16x8 / 8x16 rules and the 6.4.11.7 neighbour blocks),
# coded_block_pattern, mb_qp_delta (QP chain from the slice QP) and the
# residual levels.  Used to check that a spliced MB of a composed NAL decodes
# to the same syntax elements as in its external slice.

def _nc(nA, nB):
    if nA >= 0 and nB >= 0:
        return (nA + nB + 1) >> 1
    return nA if nA >= 0 else (nB if nB >= 0 else 0)


def _parts(mbt, sub):
    """(sub-)partitions in decoding order: (bx, by, bw, bh, mbPartIdx) in 4x4 units"""
    if mbt == 0:
        return [(0, 0, 4, 4, 0)]
    if mbt == 1:
        return [(0, 0, 4, 2, 0), (0, 2, 4, 2, 1)]
    if mbt == 2:
        return [(0, 0, 2, 4, 0), (2, 0, 2, 4, 1)]
    out = []
    for i in range(4):
        sx, sy = (i % 2) * 2, (i // 2) * 2
        st = sub[i]
        if st == 0:
            out.append((sx, sy, 2, 2, i))
        elif st == 1:
            out += [(sx, sy, 2, 1, i), (sx, sy + 1, 2, 1, i)]
        elif st == 2:
            out += [(sx, sy, 1, 2, i), (sx + 1, sy, 1, 2, i)]
        else:
            out += [(sx + k % 2, sy + k // 2, 1, 1, i) for k in range(4)]
    return out


GOLOMB_TO_INTRA_CBP = [47, 31, 15, 0, 23, 27, 29, 30, 7, 11, 13, 14, 39, 43, 45, 46, 16, 3, 5, 10, 12, 19,
                       21, 26, 28, 35, 37, 42, 44, 1, 2, 4, 8, 17, 18, 20, 24, 6, 9, 22, 25, 32, 33, 34,
                       36, 40, 38, 41]


class _BlockField:
    """motion (ref, mx, my) per 4x4 block of a picture of mbw x mbh MBs;
    sid[m]: the slice of MB m (another slice's MB is unavailable); an intra
    MB's blocks are (-1, 0, 0)"""

    def __init__(self, mbw, mbh):
        self.mbw = mbw
        self.f = [[None] * (4 * mbw) for _ in range(4 * mbh)]
        self.sid = [None] * (mbw * mbh)
        self.cur = 0

    def avail(self, nx, ny):
        return 0 <= nx < self.mbw and ny >= 0 and self.sid[ny * self.mbw + nx] == self.cur

    def nb(self, x, y, cx, cy, done):
        """block (cx, cy) relative to MB (x, y); inside the MB only once decoded"""
        if cy >= 0 and cx >= 4:
            return None
        if cy >= 0 and cx >= 0:
            return self.f[4 * y + cy][4 * x + cx] if (4 * cy + cx) in done else None
        nx, ny = x + (-1 if cx < 0 else (1 if cx >= 4 else 0)), y + (-1 if cy < 0 else 0)
        if not self.avail(nx, ny):
            return None
        return self.f[4 * ny + (cy % 4)][4 * nx + (cx % 4)]

    def set(self, x, y, bx, by, bw, bh, v, done):
        for j in range(bh):
            for i in range(bw):
                self.f[4 * y + by + j][4 * x + bx + i] = v
                done.add(4 * (by + j) + bx + i)

    def mb16(self, x, y):
        A, B = self.nb(x, y, -1, 0, ()), self.nb(x, y, 0, -1, ())
        C = self.nb(x, y, 4, -1, ())
        if C is None:
            C = self.nb(x, y, -1, -1, ())
        return A, B, C


def mvp_part(F, x, y, done, mbt, p, ref):
    bx, by, bw, _, mp = p
    A, B = F.nb(x, y, bx - 1, by, done), F.nb(x, y, bx, by - 1, done)
    C = F.nb(x, y, bx + bw, by - 1, done)
    if C is None:
        C = F.nb(x, y, bx - 1, by - 1, done)
    d = None
    if mbt == 1:
        d = B if mp == 0 else A
    elif mbt == 2:
        d = A if mp == 0 else C
    if d is not None and d[0] == ref:
        return d[1], d[2]
    return mvp_spec(A, B, C, ref)


def nal_units(data):
    """the NAL units of an Annex-B buffer (start codes dropped, trailing zero
    bytes trimmed); a buffer without a start code is one NAL"""
    if not (data[:3] == b"\x00\x00\x01" or data[:4] == b"\x00\x00\x00\x01"):
        return [bytes(data)]
    out, i, starts = [], 0, []
    while True:
        j = data.find(b"\x00\x00\x01", i)
        if j < 0:
            break
        starts.append(j + 3)
        i = j + 3
    for k, a in enumerate(starts):
        e = starts[k + 1] - 3 if k + 1 < len(starts) else len(data)
        u = data[a:e]
        out.append(u.rstrip(b"\x00") if k + 1 < len(starts) else u)
    return out


def _rbsp_stop(d):
    for i in range(len(d) - 1, -1, -1):
        if d[i]:
            return 8 * i + 7 - ((d[i] & -d[i]).bit_length() - 1)
    return -1


def decode_p_slice(nal, w, h, predictor="spec", log2_mfn=4, poc_type=2, log2_poc=4, deblock=1,
                   nrefs_default=2, trace=None):
    """-> (header, mbs[y][x] = dict(ref, mx, my, skip, cbp, qp, luma, cdc, cac,
    mbt, sub, blocks, intra, modes, cmode, dc16, pcm))

    nal: the picture's slices as Annex-B bytes (several NAL units one after
    the other; a single NAL may come without a start code).  An MB of another
    slice, or past the picture's edge, is unavailable.  mbt: the mb_type
    (0..4 inter, 5..30 intra), blocks: (ref, mx, my) per 4x4 block in raster
    order (intra: (-1, 0, 0)); ref / mx / my are block 0's.  intra: 0, 1
    I_4x4 (modes: Intra4x4PredMode per raster block), 2 I_16x16 (modes[0]:
    its luma mode, dc16: the DC levels; luma holds the AC levels from scan
    index 1), 3 I_PCM (pcm: its 384 sample bytes); cmode:
    intra_chroma_pred_mode."""
    mbw, mbh = w // 16, h // 16
    F = _BlockField(mbw, mbh)
    mbs = [[None] * mbw for _ in range(mbh)]
    tcs = [[None] * mbw for _ in range(mbh)]
    im = [[None] * mbw for _ in range(mbh)]          # Intra4x4PredModes (raster) of I_4x4 MBs
    pred = mvp_spec if predictor == "spec" else mvp_ref
    m, nmb, H0 = 0, mbw * mbh, None
    for si, unit in enumerate(nal_units(nal)):
        ref_idc, nut = unit[0] >> 5, unit[0] & 31
        assert nut in (1, 5), "coded slice of a non-IDR or IDR picture"
        rb = ebsp_to_rbsp(unit[1:])
        stop = _rbsp_stop(rb)
        b = Bits(rb)
        H = {"first_mb": b.ue(), "slice_type": b.ue(), "pps": b.ue(), "frame_num": b.u(log2_mfn)}
        assert H["first_mb"] == m, "slices in MB order"
        islice = H["slice_type"] in (2, 7)
        assert islice or H["slice_type"] in (0, 5), "a P or I slice"
        assert nut == 1 or islice, "an IDR picture has I slices"
        if nut == 5:
            H["idr_pic_id"] = b.ue()
        if poc_type == 0:
            H["poc"] = b.u(log2_poc)
        nrefs = nrefs_default
        if not islice and b.u(1):
            nrefs = b.ue() + 1
        H["nrefs"] = nrefs
        H["list_mod"] = 0 if islice else b.u(1)
        if H["list_mod"]:                        # ref_pic_list_modification (waypoints)
            while True:
                idc = b.ue()
                if idc == 3:
                    break
                b.ue()
        if ref_idc and nut == 5:
            b.u(2)                               # no_output_of_prior_pics, long_term_reference
        elif ref_idc and b.u(1):
            while True:
                op = b.ue()
                if op == 0:
                    break
                if op in (1, 3):
                    b.ue()
                if op in (2, 3, 6):
                    b.ue()
                if op == 4:
                    b.ue()
        qp = 26 + b.se()
        H["qp"] = qp
        if deblock:
            H["deblock_idc"] = b.ue()
            if H["deblock_idc"] != 1:
                b.se(); b.se()
        if H0 is None:
            H0 = H
        F.cur = si

        def te():
            return (1 - b.u(1)) if nrefs == 2 else (b.ue() if nrefs > 2 else 0)

        first = True
        while first or b.p < stop:
            first = False
            run = 0 if islice else b.ue()        # I slices: no mb_skip_run
            for _ in range(run):
                y, x = divmod(m, mbw)
                assert y < mbh, "mb_skip_run past the picture"
                F.sid[m] = si
                A, B_, C = F.mb16(x, y)
                if A is None or B_ is None or (A[0] == 0 and A[1:] == (0, 0)) or (B_[0] == 0 and B_[1:] == (0, 0)):
                    mv = (0, 0)
                else:
                    mv = mvp_spec(A, B_, C, 0)
                F.set(x, y, 0, 0, 4, 4, (0,) + mv, set())
                tcs[y][x] = [0] * 24
                mbs[y][x] = dict(ref=0, mx=mv[0], my=mv[1], skip=True, cbp=0, qp=qp, mbt=0, sub=None,
                                 blocks=[(0,) + mv] * 16, intra=0,
                                 luma=[[0] * 16 for _ in range(16)], cdc=[[0] * 4] * 2,
                                 cac=[[[0] * 15 for _ in range(4)] for _ in range(2)])
                m += 1
            if b.p >= stop:
                break
            y, x = divmod(m, mbw)
            F.sid[m] = si
            if trace is not None:
                trace.append((m, b.p))
            left = tcs[y][x - 1] if F.avail(x - 1, y) else None
            top = tcs[y - 1][x] if F.avail(x, y - 1) else None
            mbt = b.ue() + (5 if islice else 0)  # an I slice's mb_type k is the P slice's 5 + k
            assert mbt <= 30, "a P-slice mb_type"
            t = [0] * 24
            luma = [[0] * 16 for _ in range(16)]
            cdc = [[0] * 4 for _ in range(2)]
            cac = [[[0] * 15 for _ in range(4)] for _ in range(2)]

            def luma_nc(r):
                bx, by = r % 4, r // 4
                nA = t[r - 1] if bx > 0 else (left[r + 3] if left else -1)
                nB = t[r - 4] if by > 0 else (top[r + 12] if top else -1)
                return _nc(nA, nB)

            def chroma(cbpc):
                if cbpc:
                    for p in range(2):
                        cdc[p], _ = cavlc_block(b, -1, 4)
                    if cbpc == 2:
                        for p in range(2):
                            for k in range(4):
                                bx, by = k % 2, k // 2
                                i = 16 + 4 * p + k
                                nA = t[i - 1] if bx > 0 else (left[i + 1] if left else -1)
                                nB = t[i - 2] if by > 0 else (top[i + 2] if top else -1)
                                cac[p][k], t[i] = cavlc_block(b, _nc(nA, nB), 15)

            if mbt >= 5:                         # intra in a P slice (7.3.5)
                it = mbt - 5
                d = dict(ref=-1, mx=0, my=0, skip=False, mbt=mbt, sub=None, blocks=[(-1, 0, 0)] * 16,
                         intra=1 if it == 0 else (3 if it == 25 else 2), modes=None, cmode=None, dc16=None,
                         pcm=None, cbp=0)
                F.set(x, y, 0, 0, 4, 4, (-1, 0, 0), set())
                if it == 25:
                    while b.p & 7:
                        assert b.u(1) == 0, "pcm_alignment_zero_bit"
                    d["pcm"] = bytes(b.u(8) for _ in range(384))
                    t = [16] * 24
                    d.update(qp=qp, luma=luma, cdc=cdc, cac=cac)
                else:
                    if it == 0:
                        modes = [None] * 16
                        for blk in range(16):
                            q8, q4 = divmod(blk, 4)
                            bx, by = (q8 % 2) * 2 + q4 % 2, (q8 // 2) * 2 + q4 // 2
                            r = 4 * by + bx

                            def nmode(nx, ny, rr):
                                if not F.avail(nx, ny):
                                    return None
                                mm = im[ny][nx]
                                return 2 if mm is None else mm[rr]
                            mA = modes[r - 1] if bx else nmode(x - 1, y, r + 3)
                            mB = modes[r - 4] if by else nmode(x, y - 1, r + 12)
                            pm = 2 if mA is None or mB is None else min(mA, mB)
                            if b.u(1):
                                modes[r] = pm
                            else:
                                rem = b.u(3)
                                modes[r] = rem if rem < pm else rem + 1
                        im[y][x] = modes
                        d["modes"] = modes
                    else:
                        d["modes"] = [(it - 1) % 4]
                    d["cmode"] = b.ue()
                    if it == 0:
                        cbp = GOLOMB_TO_INTRA_CBP[b.ue()]
                    else:
                        cbp = (15 if it - 1 >= 12 else 0) | (((it - 1) // 4) % 3) << 4
                    d["cbp"] = cbp
                    if cbp or it != 0:
                        qp = (qp + b.se() + 52) % 52
                        if it != 0:
                            d["dc16"], _ = cavlc_block(b, luma_nc(0), 16)
                        for blk in range(16):
                            q8, q4 = divmod(blk, 4)
                            bx, by = (q8 % 2) * 2 + q4 % 2, (q8 // 2) * 2 + q4 // 2
                            r = 4 * by + bx
                            if not cbp & (1 << q8):
                                continue
                            if it == 0:
                                luma[r], t[r] = cavlc_block(b, luma_nc(r), 16)
                            else:
                                ac, t[r] = cavlc_block(b, luma_nc(r), 15)
                                luma[r] = [0] + ac
                        chroma(cbp >> 4)
                    d.update(qp=qp, luma=luma, cdc=cdc, cac=cac)
                tcs[y][x] = t
                mbs[y][x] = d
                m += 1
                continue
            sub = [b.ue() for _ in range(4)] if mbt >= 3 else None
            assert sub is None or max(sub) <= 3
            nref = 1 if mbt == 0 else (4 if mbt >= 3 else 2)
            refs = [0] * 4 if mbt == 4 else [te() for _ in range(nref)]
            done = set()
            if mbt == 0:
                dx, dy = b.se(), b.se()
                px, py = pred(*F.mb16(x, y), refs[0])
                F.set(x, y, 0, 0, 4, 4, (refs[0], px + dx, py + dy), done)
            else:
                for p in _parts(mbt, sub):
                    dx, dy = b.se(), b.se()
                    rf = refs[p[4]]
                    px, py = mvp_part(F, x, y, done, mbt, p, rf)
                    F.set(x, y, p[0], p[1], p[2], p[3], (rf, px + dx, py + dy), done)
            blocks = [F.f[4 * y + k // 4][4 * x + k % 4] for k in range(16)]
            cbp = GOLOMB_TO_INTER_CBP[b.ue()]
            if cbp:
                qp = (qp + b.se() + 52) % 52
                for blk in range(16):
                    q8, q4 = divmod(blk, 4)
                    bx, by = (q8 % 2) * 2 + q4 % 2, (q8 // 2) * 2 + q4 // 2
                    r = 4 * by + bx
                    if not cbp & (1 << q8):
                        continue
                    luma[r], t[r] = cavlc_block(b, luma_nc(r), 16)
                chroma(cbp >> 4)
            tcs[y][x] = t
            mbs[y][x] = dict(ref=blocks[0][0], mx=blocks[0][1], my=blocks[0][2], skip=False, cbp=cbp, qp=qp,
                             mbt=mbt, sub=sub, blocks=blocks, luma=luma, cdc=cdc, cac=cac, intra=0)
            m += 1
        assert b.p == stop, "slice data up to the stop bit"
        assert b.u(1) == 1, "stop bit"
        while b.p & 7:
            assert b.u(1) == 0
        while b.p < 8 * len(b.d):
            assert b.u(8) == 0, "trailing bytes"
    assert m == nmb, "the slices cover the picture"
    return H0, mbs
