"""The dynamic-rect device functions (h264-scroll-encoder_amd/csrc/dyn_device.h),
compiled for the CPU by tests/hostsim, against the CPU restatement
oracle/dyn_oracle.c: CAVLC bit strings, reference-sample chains (waypoint
recursion, clamping, half-pel chroma), transform + quantiser, and the
closed-form emulation-prevention rule against the byte automaton of nal.c."""
import ctypes
import random

import numpy as np

from dynhelp import OrCfg, Pic, Refs


class OrBits(ctypes.Structure):
    _fields_ = [("buf", ctypes.c_void_p), ("cap", ctypes.c_size_t), ("nbits", ctypes.c_size_t)]


def _bits(buf, start, n):
    out = []
    for i in range(start, start + n):
        out.append((buf[i >> 3] >> (7 - (i & 7))) & 1)
    return out


def _word_bits(words, start, n):
    return [(words[i >> 5] >> (31 - (i & 31))) & 1 for i in range(start, start + n)]


def _random_block(rng, mx):
    kind = rng.random()
    c = [0] * mx
    if kind < 0.15:
        return c
    nnz = rng.randint(1, mx)
    pos = rng.sample(range(mx), nnz)
    for p in pos:
        r = rng.random()
        if kind < 0.5:
            c[p] = rng.choice([-1, 1]) if r < 0.7 else rng.randint(-4, 4) or 1
        elif kind < 0.85:
            c[p] = rng.randint(-40, 40) or -1
        else:
            c[p] = rng.randint(-160, 160) or 2
    return c


def test_cavlc_blocks_vs_oracle(hostsim, oracle):
    """every coeff_token table (nC -1, 0-1, 2-3, 4-7, >= 8), trailing ones,
    suffixLength escalation, level escapes, total_zeros / run_before"""
    rng = random.Random(12)
    ob = (ctypes.c_uint8 * 4096)()
    words = (ctypes.c_uint32 * 1024)()
    tc = ctypes.c_int()
    for it in range(4000):
        mx = rng.choice([16, 15, 4])
        nC = -1 if mx == 4 else rng.choice([0, 1, 2, 3, 4, 5, 7, 8, 9, 16])
        coef = _random_block(rng, mx)
        ca = (ctypes.c_int * 16)(*coef)
        bits = OrBits()
        oracle.or_bits_init(ctypes.byref(bits), ob, len(ob))
        ctypes.memset(ob, 0, len(ob))
        tco = oracle.or_cavlc_block(ctypes.byref(bits), ca, mx, nC)
        start = rng.randint(0, 63)
        ctypes.memset(words, 0, ctypes.sizeof(words))
        n = hostsim.sim_cavlc(ca, mx, nC, start, words, ctypes.byref(tc))
        assert n == bits.nbits, (it, coef, nC)
        assert tc.value == tco
        assert _word_bits(words, start, n) == _bits(ob, 0, n), (it, coef, nC)
        assert all(words[i] == 0 for i in range((start + n + 31) // 32, 1024))
        ctypes.memset(words, 0, ctypes.sizeof(words))          # the kernels' split form
        n2 = hostsim.sim_cavlc_split(ca, mx, nC, start, words, ctypes.byref(tc))
        assert n2 == n and tc.value == tco, (it, coef, nC)
        assert _word_bits(words, start, n) == _bits(ob, 0, n), (it, coef, nC)
        if mx != 4:                                    # k_dyn_row's form (tzrb table)
            ctypes.memset(words, 0, ctypes.sizeof(words))
            n4 = hostsim.sim_cavlc_split_t(ca, mx, nC, start, words, ctypes.byref(tc))
            assert n4 == n and tc.value == tco, (it, coef, nC)
            assert _word_bits(words, start, n) == _bits(ob, 0, n), (it, coef, nC)
        if mx == 4:                                    # the kernels' chroma-DC encoder
            ctypes.memset(words, 0, ctypes.sizeof(words))
            n3 = hostsim.sim_cavlc_dc4(ca, start, words, ctypes.byref(tc))
            assert n3 == n and tc.value == tco, (it, coef)
            assert _word_bits(words, start, n) == _bits(ob, 0, n), (it, coef)


def test_tzrb_table_lengths(hostsim):
    """k_dyn_row's total_zeros + run_before entries fit their 32-bit form
    (code + sentinel): at most 30 bits for 16 coefficients, 25 for 15"""
    assert hostsim.sim_tzrb_maxlen(16) == 30
    assert hostsim.sim_tzrb_maxlen(15) == 25


def test_packed_levels_vs_scalar(hostsim):
    """k_dyn_row's transform + quant on packed 16-bit pairs (levels_pk, host
    emulation of its dataflow) equals fwd4x4 + quant on random and extreme
    residual blocks, luma and chroma AC (the GPU parity tests check the
    instructions themselves)"""
    hostsim.sim_levels_pk.restype = ctypes.c_long
    assert hostsim.sim_levels_pk(ctypes.c_long(200000), 7) == 0


def _planes(rng, w, h):
    return [rng.integers(0, 256, (h, w), dtype=np.uint8), rng.integers(0, 256, (h // 2, w // 2), dtype=np.uint8),
            rng.integers(0, 256, (h // 2, w // 2), dtype=np.uint8)]


def test_reference_samples_vs_oracle(hostsim, oracle):
    """luma_row / chroma_row / chroma_px_any against or_ref_sample: waypoint
    chains as the composer creates them (multiples of 496: full-pel) and
    resumed tables with odd offsets (half-pel chroma steps), clamping at
    both picture edges"""
    rng = np.random.default_rng(4)
    prng = random.Random(4)
    w, h = 64, 1024
    pics = [_planes(rng, w, h) for _ in range(2)]
    arrs = [p for pic in pics for p in pic]
    pl = (ctypes.c_void_p * 6)(*[a.ctypes.data for a in arrs])
    P = [Pic(w, h, *[a.ctypes.data for a in pic]) for pic in pics]
    R = Refs()
    R.ab[0] = ctypes.pointer(P[0])
    R.ab[1] = ctypes.pointer(P[1])
    fast = ctypes.c_int()
    n_slow = 0
    for table in range(60):
        cfg = OrCfg()
        oracle.or_cfg_init(ctypes.byref(cfg), w, h)
        n = prng.randint(1, 8)
        if table % 2 == 0:
            offs = [496 * (k + 1) for k in range(n)]
        else:
            offs = sorted(prng.sample(range(-300, 2600), n))
        for k in range(n):
            cfg.wp_off[k], cfg.wp_lt[k], cfg.wp_valid[k] = offs[k], 2 + k, 1 if prng.random() > 0.1 else 0
        cfg.nwp = n
        wo = (ctypes.c_int * 8)(*cfg.wp_off)
        wv = (ctypes.c_int * 8)(*cfg.wp_valid)
        for _ in range(200):
            ri = prng.randint(0, 1 + n)
            p = prng.randint(0, 2)
            pw, ph = (w, h) if p == 0 else (w // 2, h // 2)
            x = prng.randint(0, pw - 1)
            y = prng.randint(-40, ph + 40)
            want = oracle.or_ref_sample(ctypes.byref(cfg), ctypes.byref(R), ri, p, x, y)
            got = hostsim.sim_ref_sample(w, h, wo, wv, ri, p, x, y, pl, ctypes.byref(fast))
            assert got == want, (table, ri, p, x, y, offs)
            n_slow += fast.value == 0
            if table % 2 == 0:
                assert fast.value == 1             # composer waypoints never need the tree
    assert n_slow > 0


def test_transform_quant_vs_oracle(hostsim, oracle):
    rng = np.random.default_rng(9)
    res = (ctypes.c_int * 16)()
    W = (ctypes.c_int * 16)()
    lv = (ctypes.c_int * 16)()
    for it in range(3000):
        r = rng.integers(-255, 256, 16) if it % 3 else rng.integers(-20, 21, 16)
        for i in range(16):
            res[i] = int(r[i])
        oracle.or_fwd4x4(res, W)
        hostsim.sim_fwd_quant(res, lv)
        for k in range(16):
            assert lv[k] == oracle.or_quant(W[k], 26, k, 0)
    for v in list(range(-17000, 17001, 97)) + [-16320, 16320, 0]:
        assert hostsim.sim_quant_dc(v) == oracle.or_quant(v, 26, 0, 1)


def _ep_automaton(b):
    zeros, n = 0, 0
    for v in b:
        if zeros >= 2 and v <= 3:
            n += 1
            zeros = 0
        zeros = 0 if v else zeros + 1
    return n


def test_ep_closed_form_vs_automaton(hostsim):
    """insert before byte i iff b_i <= 3 and the zero run before i (in the
    original RBSP) has even length >= 2 -- the form both dyn kernels use"""
    rng = np.random.default_rng(1)
    for it in range(3000):
        n = int(rng.integers(1, 200))
        p0 = rng.random()
        b = np.where(rng.random(n) < p0, 0, rng.integers(0, 6, n)).astype(np.uint8)
        buf = (ctypes.c_uint8 * n).from_buffer_copy(b.tobytes())
        assert hostsim.sim_ep_count(buf, n) == _ep_automaton(b.tolist()), b.tolist()


def test_compile_time_tables_match(hostsim):
    """the kernels copy CAVLC tables packed at compile time (make_ptabs);
    they must equal the runtime packing the host simulation checks against
    the oracle"""
    assert hostsim.sim_ptabs_match() == 1
