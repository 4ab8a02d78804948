"""Mid-stream long-term reference ("atlas") update, CPU side: the oracle's
or_update_ref (oracle/scroll_oracle.c) with index 1 at frame_num 1 is the
reference composer's own B-frame rewrite (h264_rewrite_as_non_idr_i_frame,
src/h264_writer.c:296-350, via or_composer_run, pinned to the reference's
golden composer outputs); index 0 differs only in the MMCO 6 index; the
config loses its waypoints and advances frame_num; refused files leave it
unchanged.  The GPU kernel is checked against this in test_gpu_refupdate.py."""
import ctypes

import numpy as np

from dynhelp import OrCfg, ipcm_file
from test_gpu_ingest import expected, ref_file


def split(data):
    pos = [i for i in range(len(data) - 3) if data[i:i + 4] == b"\0\0\0\1"]
    return [data[a:b] for a, b in zip(pos, pos[1:] + [len(data)])]


def upd(oracle, cfg, f, which):
    buf = (ctypes.c_uint8 * (len(f) * 2 + 4096))()
    n = oracle.or_update_ref(buf, len(buf), ctypes.byref(cfg), f, len(f), which)
    return bytes(buf[:n])


def unescape(b):
    out, z = bytearray(), 0
    for v in b:
        if z >= 2 and v == 3:
            z = 0
            continue
        out.append(v)
        z = z + 1 if v == 0 else 0
    return bytes(out)


class BR:
    def __init__(self, b):
        self.bits = "".join(f"{x:08b}" for x in b)
        self.p = 0

    def u(self, n):
        v = int(self.bits[self.p:self.p + n] or "0", 2)
        self.p += n
        return v

    def ue(self):
        z = 0
        while self.u(1) == 0:
            z += 1
        return (1 << z) - 1 + self.u(z)


def test_index1_is_the_reference_b_rewrite(oracle):
    for w, h in ((64, 48), (1280, 720)):
        a, b = ref_file(oracle, w, h, 0), ref_file(oracle, w, h, 1)
        header = expected(oracle, a, b, 0)
        want = split(header)[-1]                    # B as a non-IDR I frame (composer_write_header)
        cfg = OrCfg()
        oracle.or_cfg_init(ctypes.byref(cfg), w, h)
        cfg.frame_num = 1                           # after the IDR A (h264_rewrite_idr_frame)
        got = upd(oracle, cfg, b, 1)
        assert got == want
        assert cfg.frame_num == 2 and cfg.nwp == 0


def test_index0_header_and_state(oracle):
    w, h = 320, 240
    rng = np.random.default_rng(5)
    pic = rng.integers(0, 256, w * h * 3 // 2, dtype=np.uint8).tobytes()
    f = ipcm_file(oracle, w, h, pic)
    cfg = OrCfg()
    oracle.or_cfg_init(ctypes.byref(cfg), w, h)
    cfg.frame_num = 21                              # 21 mod 16 = 5
    cfg.nwp = 3
    for k in range(3):
        cfg.wp_valid[k] = 1
    n0 = upd(oracle, cfg, f, 0)
    assert cfg.frame_num == 22 and cfg.nwp == 0 and not any(cfg.wp_valid)
    assert n0[4] == 0x61                            # nal_ref_idc 3, non-IDR slice
    r = BR(unescape(n0[5:]))
    assert (r.ue(), r.ue(), r.ue()) == (0, 7, 0)    # first_mb, I (all), pps
    assert r.u(4) == 5                              # frame_num mod 2^4
    assert r.u(1) == 1                              # adaptive_ref_pic_marking_mode_flag
    assert [r.ue() for _ in range(5)] == [4, 2, 6, 0, 0]   # MMCO 4 -> 2, MMCO 6 -> idx 0, end
    cfg2 = OrCfg()
    oracle.or_cfg_init(ctypes.byref(cfg2), w, h)
    cfg2.frame_num = 21
    n1 = upd(oracle, cfg2, f, 1)
    assert len(n1) >= len(n0) - 1 and n1 != n0


def test_refused_files_leave_the_config(oracle):
    w, h = 64, 48
    cfg = OrCfg()
    oracle.or_cfg_init(ctypes.byref(cfg), w, h)
    cfg.frame_num = 7
    other = ref_file(oracle, 128, 48, 0)            # another picture size
    assert upd(oracle, cfg, other, 0) == b""
    assert upd(oracle, cfg, b"\0\0\0\1\x67", 1) == b""   # no PPS / IDR
    assert cfg.frame_num == 7
