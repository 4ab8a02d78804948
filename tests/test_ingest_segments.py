"""CPU model of the segmented ingest's emulation-prevention bookkeeping
(h264-scroll-encoder_amd/csrc/ingest_kernels.hip: k_ing_seg<SUMMARY>,
k_ing_fix, k_ing_seg<WRITE_*>), checked against the sequential rule of
nal.c:33-38 (insert 03 before a byte <= 3 after two zero bytes, the count
restarting after the insertion) on random byte strings cut into random
segments.  It pins the closed forms the kernels use:
  * an insertion goes before byte o iff o <= 3 and the zero run since the last
    non-zero byte, o - 1 - lnz, is even and >= 2;
  * a segment's summary (first / last non-zero byte, its value, the insertions
    after its first non-zero byte) does not depend on the segments before;
  * k_ing_fix: the insertions before a segment's first non-zero byte are the
    even runs >= 2 over its leading zeros (evens_ge2) plus the one at the
    first non-zero byte;
  * the write pass's last-non-zero clamp to -4 / -5 keeps the parity.
No GPU."""
import random

import pytest


def ebsp_sequential(rbsp):
    out, z = bytearray(), 0
    for v in rbsp:
        if z >= 2 and v <= 3:
            out.append(3)
            z = 0
        out.append(v)
        z = z + 1 if v == 0 else 0
    return bytes(out)


def insert_before(x, run):
    return x <= 3 and run >= 2 and run % 2 == 0


def summary(seg):
    """k_ing_seg<SUMMARY>: positions relative to the segment; the last
    non-zero byte before it unknown (a far sentinel)"""
    f = next((i for i, v in enumerate(seg) if v), -1)
    last = max((i for i, v in enumerate(seg) if v), default=-1)
    prev, cafter = -(1 << 40), 0
    for u, x in enumerate(seg):
        if insert_before(x, u - 1 - prev) and prev >= 0:
            cafter += 1
        if x:
            prev = u
    return dict(nout=len(seg), f=f, vf=seg[f] if f >= 0 else 0, last=last, cafter=cafter)


def evens_ge2(a, b):
    a = max(a, 2)
    f = a + (a & 1)
    return 0 if b < f else (b - f) // 2 + 1


def fix(sums):
    """k_ing_fix: each segment's output offset and incoming last non-zero
    byte (relative to its first byte); the total length"""
    pos, lnz, o0, res = 0, -1, 0, []
    for g in sums:
        res.append((pos, lnz - o0))
        of = o0 + g["f"] if g["f"] >= 0 else o0 + g["nout"]
        ins = evens_ge2(o0 - 1 - lnz, of - 2 - lnz) if g["nout"] else 0
        if g["f"] >= 0:
            run = of - 1 - lnz
            if insert_before(g["vf"], run):
                ins += 1
            ins += g["cafter"]
            lnz = o0 + g["last"]
        pos += g["nout"] + ins
        o0 += g["nout"]
    return res, pos


def clamp_parity(b):
    return b if b >= -4 else -4 - (b & 1)


def write(seg, lnz_rel):
    """k_ing_seg<WRITE_*>: the segment's bytes with their 03s, from the
    clamped incoming last non-zero byte"""
    prev, out = clamp_parity(lnz_rel), bytearray()
    for u, x in enumerate(seg):
        if insert_before(x, u - 1 - prev):
            out.append(3)
        out.append(x)
        if x:
            prev = u
    return bytes(out)


def random_rbsp(rng, n):
    kind = rng.randrange(4)
    if kind == 0:
        return bytes(rng.randrange(256) for _ in range(n))
    if kind == 1:                                   # zero-heavy with small values
        return bytes(rng.choice((0, 0, 0, 0, 1, 2, 3, 0x80)) for _ in range(n))
    if kind == 2:                                   # long zero runs of every parity
        out = bytearray()
        while len(out) < n:
            out += bytes(rng.randrange(0, 9)) + bytes([rng.choice((1, 2, 3, 4, 0xff))])
        return bytes(out[:n])
    return bytes(n)                                 # all zero


@pytest.mark.parametrize("seed", range(40))
def test_segmented_ep_matches_sequential(seed):
    rng = random.Random(seed)
    data = random_rbsp(rng, rng.randrange(0, 400))
    cuts = sorted(rng.sample(range(len(data) + 1), min(len(data) + 1, rng.randrange(1, 12))))
    bounds = [0] + [c for c in cuts if 0 < c < len(data)] + [len(data)]
    segs = [data[a:b] for a, b in zip(bounds, bounds[1:])]
    res, total = fix([summary(s) for s in segs])
    want = ebsp_sequential(data)
    assert total == len(want)
    got = bytearray(total)
    for s, (pos, lnz_rel) in zip(segs, res):
        w = write(s, lnz_rel)
        got[pos:pos + len(w)] = w
    assert bytes(got) == want


def test_evens_ge2():
    for a in range(-6, 12):
        for b in range(-6, 14):
            assert evens_ge2(a, b) == sum(1 for r in range(a, b + 1) if r >= 2 and r % 2 == 0)
