"""CPU tests of the C-ABI library: it loads, exports every symbol the headers
declare, keeps the reference struct layouts, and its host-side (cold path)
entry points match the oracle.  No GPU compute is called here."""
import ctypes
import os
import random
import subprocess
import sys

import pytest

from conftest import PKG, REPO, golden_file

# reference struct sizes / offsets (measured from /root/reference/include with
# gcc 11.4 x86_64: sizeof Composer, ComposerConfig, NALWriter, BitWriter,
# BitReader, NALUnit, NALParser, offsetof(Composer, nw),
# offsetof(Composer, frames_written), offsetof(ComposerConfig, num_waypoints))
REF_LAYOUT = [432, 144, 40, 32, 32, 32, 24, 352, 424, 140]


def test_exports_every_header_symbol(scroll):
    syms = scroll.header_symbols()
    assert len(syms) >= 70
    out = subprocess.run(["nm", "-D", "--defined-only", scroll.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in syms if s not in exported]
    assert not missing, missing


def test_struct_layouts_match_reference(tmp_path):
    src = tmp_path / "abi.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "composer.h"\n'
                   '#include "nal_parser.h"\nint main(){printf("%zu %zu %zu %zu %zu %zu %zu '
                   '%zu %zu %zu", sizeof(Composer), sizeof(ComposerConfig), sizeof(NALWriter),'
                   ' sizeof(BitWriter), sizeof(BitReader), sizeof(NALUnit), sizeof(NALParser),'
                   ' offsetof(Composer,nw), offsetof(Composer,frames_written),'
                   ' offsetof(ComposerConfig,num_waypoints));}\n')
    exe = tmp_path / "abi"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)],
                   check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    assert got == REF_LAYOUT
    import h264scroll
    assert ctypes.sizeof(h264scroll.Composer) == REF_LAYOUT[0]
    assert ctypes.sizeof(h264scroll.ComposerConfig) == REF_LAYOUT[1]


def _py_ue(bits, v):
    if v == 0:
        bits.append(1)
        return
    x = (v + 1) & 0xFFFFFFFF
    m = x.bit_length() - 1 if x else 0
    bits.extend([0] * m)
    bits.extend((x >> (m - i)) & 1 for i in range(m + 1)) if x else bits.append(0)


def test_bitwriter_random_ops(scroll):
    """bitwriter_* against a bit-list model of src/bitwriter.c."""
    rng = random.Random(3)
    lib = scroll.lib
    for trial in range(200):
        buf = scroll.u8buf(4096)
        bw = scroll.BitWriter()
        lib.bitwriter_init(ctypes.byref(bw), buf, 4096)
        bits = []
        for _ in range(rng.randint(1, 60)):
            op = rng.randint(0, 3)
            if op == 0:
                n = rng.randint(1, 32)
                v = rng.getrandbits(32)
                lib.bitwriter_write_bits(ctypes.byref(bw), v, n)
                bits.extend((v >> (n - 1 - i)) & 1 for i in range(n))
            elif op == 1:
                v = rng.choice([0, 1, 2, 3, 7, rng.getrandbits(rng.randint(1, 31))])
                lib.bitwriter_write_ue(ctypes.byref(bw), v)
                _py_ue(bits, v)
            elif op == 2:
                v = rng.randint(-(1 << 20), 1 << 20)
                lib.bitwriter_write_se(ctypes.byref(bw), v)
                _py_ue(bits, 2 * v - 1 if v > 0 else -2 * v)
            else:
                b = rng.randint(0, 1)
                lib.bitwriter_write_bit(ctypes.byref(bw), b)
                bits.append(b)
        assert lib.bitwriter_get_bit_position(ctypes.byref(bw)) == len(bits)
        if trial % 2:
            lib.bitwriter_write_trailing_bits(ctypes.byref(bw))
            bits.append(1)
            while len(bits) % 8:
                bits.append(0)
        n = lib.bitwriter_get_size(ctypes.byref(bw))
        pad = bits + [0] * (-len(bits) % 8)
        want = bytes(int("".join(map(str, pad[i:i + 8])), 2) for i in range(0, len(pad), 8))
        assert n == len(want) and bytes(buf[:n]) == want


def test_bitreader_roundtrip(scroll):
    lib = scroll.lib
    buf = scroll.u8buf(256)
    bw = scroll.BitWriter()
    lib.bitwriter_init(ctypes.byref(bw), buf, 256)
    vals = [0, 1, 5, 1000, 65535]
    for v in vals:
        lib.bitwriter_write_ue(ctypes.byref(bw), v)
        lib.bitwriter_write_se(ctypes.byref(bw), -v)
    n = lib.bitwriter_get_size(ctypes.byref(bw))
    br = scroll.BitReader()
    lib.bitreader_init(ctypes.byref(br), buf, n)
    for v in vals:
        assert lib.bitreader_read_ue(ctypes.byref(br)) == v
        assert lib.bitreader_read_se(ctypes.byref(br)) == -v


def test_rbsp_to_ebsp_vs_oracle(scroll, oracle):
    rng = random.Random(9)
    for _ in range(300):
        n = rng.randint(0, 300)
        data = bytes(rng.choice([0, 0, 0, 1, 2, 3, 4, 0xff, rng.getrandbits(8)]) for _ in range(n))
        src = scroll.u8buf(data if data else b"\0")
        a, b = scroll.u8buf(2 * n + 8), (ctypes.c_uint8 * (2 * n + 8))()
        na = scroll.lib.rbsp_to_ebsp(a, len(a), src, n)
        nb = oracle.or_rbsp_to_ebsp(b, len(b), bytes(data) if data else b"\0", n)
        assert bytes(a[:na]) == bytes(b[:nb])
        back = scroll.u8buf(na + 1)
        nr = scroll.lib.ebsp_to_rbsp(back, a, na)
        assert bytes(back[:nr]) == data


def test_sps_pps(scroll, oracle):
    for w, h in [(64, 48), (1280, 720), (3840, 2160), (16, 16)]:
        a, b = scroll.u8buf(64), (ctypes.c_uint8 * 64)()
        assert bytes(a[:scroll.lib.h264_generate_sps(a, 64, w, h)]) == \
            bytes(b[:oracle.or_sps(b, 64, w, h)])
    a, b = scroll.u8buf(64), (ctypes.c_uint8 * 64)()
    assert bytes(a[:scroll.lib.h264_generate_pps(a, 64)]) == bytes(b[:oracle.or_pps(b, 64)])


def test_parser_on_golden_ref(scroll):
    data = golden_file("ipcm_64x48_a.h264")
    lib = scroll.lib
    buf = scroll.u8buf(data)
    p, u = scroll.NALParser(), scroll.NALUnit()
    lib.nal_parser_init(ctypes.byref(p), buf, len(data))
    types = []
    while lib.nal_parser_next(ctypes.byref(p), ctypes.byref(u)):
        types.append(u.nal_unit_type)
        if u.nal_unit_type == 7:
            r = scroll.u8buf(u.size + 1)
            rn = lib.ebsp_to_rbsp(r, u.data, u.size)
            vals = [ctypes.c_int() for _ in range(5)]
            assert lib.parse_sps(r, rn, *[ctypes.byref(v) for v in vals]) == 0
            assert [v.value for v in vals] == [64, 48, 4, 2, 0]
        if u.nal_unit_type == 8:
            r = scroll.u8buf(u.size + 1)
            rn = lib.ebsp_to_rbsp(r, u.data, u.size)
            a, b = ctypes.c_int(), ctypes.c_int()
            assert lib.parse_pps(r, rn, ctypes.byref(a), ctypes.byref(b)) == 0
            assert (a.value, b.value) == (1, 1)
    assert types == [7, 8, 5]


def test_composer_header_cold_path(scroll, oracle, tmp_path):
    """composer_init + composer_write_header (host) == reference header bytes."""
    pa, pb = tmp_path / "a.h264", tmp_path / "b.h264"
    pa.write_bytes(golden_file("ipcm_64x48_a.h264"))
    pb.write_bytes(golden_file("ipcm_64x48_b.h264"))
    c = scroll.Composer()
    assert scroll.lib.composer_init(ctypes.byref(c), str(pa).encode(), str(pb).encode()) == 0
    assert (scroll.lib.composer_get_width(ctypes.byref(c)),
            scroll.lib.composer_get_height(ctypes.byref(c))) == (64, 48)
    scroll.lib.composer_write_header(ctypes.byref(c))
    n = scroll.lib.composer_get_output_size(ctypes.byref(c))     # no frames queued: no GPU
    out = bytes(scroll.lib.composer_get_output(ctypes.byref(c))[:n])
    full = golden_file("composer_64x48_n40_s1.h264")
    a, b = pa.read_bytes(), pb.read_bytes()
    hb = (ctypes.c_uint8 * 65536)()
    hn = oracle.or_composer_run(hb, 65536, a, len(a), b, len(b), 0, 1)
    assert out == bytes(hb[:hn]) == full[:hn]
    assert c.cfg.frame_num == 2
    scroll.lib.composer_finish(ctypes.byref(c))


def test_composer_init_errors(scroll, tmp_path):
    c = scroll.Composer()
    assert scroll.lib.composer_init(ctypes.byref(c), b"/nonexistent/a", b"/nonexistent/b") == -1
    bad = tmp_path / "bad.h264"
    bad.write_bytes(b"\x00\x00\x00\x01\x67garbage")
    assert scroll.lib.composer_init(ctypes.byref(c), str(bad).encode(), str(bad).encode()) == -1


def test_no_device_fails_loudly(scroll):
    """Without a gfx950 GPU the hot path must refuse, never fall back."""
    if scroll.device_count() > 0:
        pytest.skip("GPU present")
    d = scroll.ScrollBatchDesc(0, 1, 1, 1 << 20, 0)
    h = ctypes.c_void_p()
    assert scroll.lib.scroll_batch_create(ctypes.byref(h), ctypes.byref(d)) == \
        scroll.SCROLL_ERR_NO_DEVICE
    code = ("import sys,ctypes; sys.path.insert(0,%r); import h264scroll as s;"
            "c=s.make_config(64,48); nw=s.NALWriter(); o=s.u8buf(1<<16); r=s.u8buf(1<<16);"
            "s.lib.nal_writer_init(ctypes.byref(nw),o,1<<16,r,1<<16);"
            "s.lib.h264_write_scroll_p_frame(ctypes.byref(nw),ctypes.byref(c),5)") % PKG
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
    assert p.returncode != 0
    assert "failed on the GPU path" in p.stderr


def test_needs_waypoint_host(scroll):
    c = scroll.make_config(1280, 2160)
    assert scroll.lib.h264_needs_waypoint(ctypes.byref(c), 0) == 0
    assert scroll.lib.h264_needs_waypoint(ctypes.byref(c), 496) == 1
    assert scroll.lib.h264_needs_waypoint(ctypes.byref(c), -496) == 1
    assert scroll.lib.h264_needs_waypoint(ctypes.byref(c), 497) == 0
    c2 = scroll.make_config(1280, 2160, waypoints=[(496, 2, 1)])
    assert scroll.lib.h264_needs_waypoint(ctypes.byref(c2), 496) == 0
    c3 = scroll.make_config(1280, 2160, waypoints=[(496, 2, 0)])
    assert scroll.lib.h264_needs_waypoint(ctypes.byref(c3), 496) == 1
