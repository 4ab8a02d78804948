"""TEST-ONLY: the device header's run-layout / bit-extraction / serial logic,
compiled for the CPU by tests/hostsim, against the reference's golden vectors.
This checks the algorithm of the GPU kernels without a GPU; the parity
evidence for the kernels themselves is tests/test_gpu_parity.py."""
import ctypes
import hashlib
import random

I8 = ctypes.c_int * 8
BUF = 16 << 20


def _run(sim, c, force, buf):
    wo = I8(*[t[0] for t in c["wp"]])
    wl = I8(*[t[1] for t in c["wp"]])
    wv = I8(*[t[2] for t in c["wp"]])
    fast, nr = ctypes.c_int(), ctypes.c_int()
    n = sim.sim_nal(c["w"], c["h"], c["log2_mfn"], c["poc_type"], c["log2_poc"], c["deblock"],
                    c["kind"], c["off"], c["frame_num"], c["nwp"], wo, wl, wv, force, buf, BUF,
                    ctypes.byref(fast), ctypes.byref(nr))
    assert n >= 0, (n, c)
    return bytes(buf[:n]), fast.value, nr.value


def test_fast_and_serial_paths_vs_golden(hostsim, golden_frames):
    buf = (ctypes.c_uint8 * BUF)()
    nfast = nslow = 0
    for c in golden_frames:
        if c["kind"] == 2:
            continue
        got, fast, nr = _run(hostsim, c, 0, buf)
        assert hashlib.sha256(got).hexdigest() == c["sha256"], c
        nfast += fast
        nslow += not fast
        if fast:
            assert 1 <= nr <= 12
            assert not c["has_ep"]          # EP frames must never take the fast path
        got2, _, _ = _run(hostsim, c, 1, buf)
        assert got2 == got
    assert nfast > 400 and nslow > 10


def test_len_lut_modulo(hostsim):
    assert hostsim.sim_check_lut() == 0


def test_stream_whole_lines(hostsim):
    """k_emit's store plan (shared device code) over whole streams: tiles of
    1..7 NALs, appends after a previous compose (head line merged from
    memory), tiny NALs (16x16) that exceed the neighbour layouts; bytes must
    equal the per-NAL reference, the previous bytes survive, the tail of the
    last line is zero and duplicate seam writes agree."""
    buf = (ctypes.c_uint8 * BUF)()
    out = (ctypes.c_uint8 * BUF)()
    rng = random.Random(7)
    wo, wl, wv = I8(*[496 * (k + 1) for k in range(8)]), I8(*[2 + k for k in range(8)]), I8(*[1] * 8)
    for it in range(160):
        w, h = 16 * rng.choice([1, 1, 2, 4, rng.randint(1, 40)]), 16 * rng.choice([1, 3, rng.randint(1, 30)])
        n = rng.randint(1, 40)
        kinds = [rng.choice([0, 0, 0, 1]) for _ in range(n)]
        offs = [rng.randint(0, h) for _ in range(n)]
        fns = [rng.randint(0, 50) for _ in range(n)]
        nwps = [rng.randint(0, 8) for _ in range(n)]
        ref = b""
        for i in range(n):
            c = dict(w=w, h=h, log2_mfn=4, poc_type=2, log2_poc=4, deblock=1, kind=kinds[i],
                     off=offs[i], frame_num=fns[i], nwp=nwps[i],
                     wp=[(496 * (k + 1), 2 + k, 1) for k in range(8)])
            b, fast, _ = _run(hostsim, c, 0, buf)
            assert fast
            ref += b
        A = lambda v: (ctypes.c_int * n)(*v)
        base = rng.choice([0, rng.randint(0, 300)])
        tile = rng.randint(1, 7)
        m = hostsim.sim_stream(w, h, 4, 2, 4, 1, n, A(kinds), A(offs), A(fns), A(nwps), wo, wl, wv,
                               base, tile, out, BUF)
        assert m == len(ref), (it, m)
        got = bytes(out[:base + m + 128])
        assert got[:base] == bytes((i * 37 + 11) & 255 for i in range(base))
        assert got[base:base + m] == ref, it
        end = base + m
        le = (end + 127) & ~127
        assert got[end:le] == bytes(le - end)
