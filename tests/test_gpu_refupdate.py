"""Mid-stream long-term reference ("atlas") updates on the GPU
(scroll_batch_update_refs -> k_ing_update) against the CPU restatement
or_update_ref (oracle/scroll_oracle.c; its index-1 form is the reference's
own B rewrite, test_refupdate_oracle.py): live streams compose through
waypoints, some get a new A or B picture (I_PCM files of random pictures),
then compose on -- every byte of every stream equals the oracle sequence
(or_compose ... or_update_ref ... or_compose).  Also: a size mismatch
refused with nothing appended, repeated streams refused, and a
dynamic-rect batch predicting from the new pictures after the update.
Run on an MI355X: -m gpu."""
import ctypes

import numpy as np
import pytest

from dynhelp import OrCfg, Pic, Rect, Refs, StripedRefs, ipcm_file, rect_source

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(scroll):
    if scroll.device_count() < 1:
        pytest.fail("no gfx950 device: " + scroll.last_error())
    return scroll


def _pic(rng, w, h):
    return rng.integers(0, 256, w * h * 3 // 2, dtype=np.uint8).tobytes()


def test_update_refs_through_waypoints(gpu, oracle):
    hs = gpu
    W, H, S, F1, F2 = 1280, 720, 6, 24, 20
    rng = np.random.default_rng(11)
    # up through 496 (a waypoint) and beyond; then back down and up again
    offs1 = (np.arange(F1)[None, :] * 12 + 420 + 3 * np.arange(S)[:, None]).astype(np.int32)
    offs1[:, 6] = 496                              # waypoints are written at multiples of 496
    offs2 = ((np.arange(F2)[None, :] * 37 + 100 + 11 * np.arange(S)[:, None]) % 700).astype(np.int32)
    b = hs.Batch(S, max(F1, F2), 16 << 20, device=0)
    for _ in range(S):
        b.add_stream(hs.make_config(W, H))
    b.set_offsets(offs1)
    b.compose(F1)
    ups = {0: 0, 2: 1, 5: 0}                       # stream -> which
    files = {s: ipcm_file(oracle, W, H, _pic(rng, W, H)) for s in ups}
    rc, st = b.update_refs(list(ups), list(ups.values()), [files[s] for s in ups])
    assert rc == 0 and st == [0, 0, 0]
    b.set_offsets(offs2)
    b.compose(F2)
    assert b.sync() == 0, hs.last_error()
    buf = (ctypes.c_uint8 * (8 << 20))()
    for s in range(S):
        cfg = OrCfg()
        oracle.or_cfg_init(ctypes.byref(cfg), W, H)
        cfg.frame_num = 2
        want = bytearray()
        for off in offs1[s]:
            n = oracle.or_compose(buf, len(buf), ctypes.byref(cfg), int(off), 0, None)
            want += bytes(buf[:n])
        if s in ups:
            assert cfg.nwp > 0                      # the update drops real waypoints
            f = files[s]
            n = oracle.or_update_ref(buf, len(buf), ctypes.byref(cfg), f, len(f), ups[s])
            assert n > 0
            want += bytes(buf[:n])
        for off in offs2[s]:
            n = oracle.or_compose(buf, len(buf), ctypes.byref(cfg), int(off), 0, None)
            want += bytes(buf[:n])
        assert b.output(s) == bytes(want), s
        got = b.config(s)
        assert got.frame_num == cfg.frame_num and got.num_waypoints == cfg.nwp, s
    b.close()


def test_update_refs_errors(gpu, oracle):
    hs = gpu
    W, H = 640, 352
    rng = np.random.default_rng(2)
    b = hs.Batch(2, 8, 4 << 20, device=0)
    for _ in range(2):
        b.add_stream(hs.make_config(W, H))
    b.set_offsets(np.tile(np.arange(8, dtype=np.int32) * 5, (2, 1)))
    b.compose(8)
    assert b.sync() == 0
    before = [b.output(s) for s in range(2)]
    wrong = ipcm_file(oracle, 1280, 720, _pic(rng, 1280, 720))
    good = ipcm_file(oracle, W, H, _pic(rng, W, H))
    rc, st = b.update_refs([0, 1], [1, 0], [good, wrong], check=False)
    assert rc < 0 and st[1] == 3                    # size mismatch: nothing appended
    assert st[0] == 0
    assert b.output(1) == before[1]
    assert len(b.output(0)) > len(before[0])
    rc, _ = b.update_refs([0, 0], [0, 1], [good, good], check=False)
    assert rc < 0                                   # a stream twice in one call
    rc, st = b.update_refs([1], [0], [b"\0\0\0\1\x09\xf0"], check=False)
    assert rc < 0 and st[0] == 1                    # no SPS / PPS / IDR
    b.close()


def test_update_refs_dynamic_rect(gpu, oracle):
    """config-3 geometry, 2 streams: stream 1 gets a new B (file + decoded
    planes via set_dyn_refs); the rect after the update predicts from it"""
    hs = gpu
    W, H, S, F1, F2 = 1280, 720, 2, 4, 4
    rect = Rect(28, 10, 25, 25)
    rng = np.random.default_rng(9)
    old = StripedRefs(oracle, W, H)
    newb = _pic(rng, W, H)
    offs1 = np.array([[470, 480, 490, 500], [100, 200, 300, 420]], np.int32)
    offs2 = np.array([[510, 520, 100, 90], [430, 440, 450, 460]], np.int32)
    b = hs.Batch(S, 4, 8 << 20, device=0)
    for _ in range(S):
        b.add_stream(hs.make_config(W, H))
    b.set_dyn_rect(rect.x0, rect.y0, rect.w, rect.h)
    pa = b"".join(bytes(p) for p in old.planes[0])
    pb = b"".join(bytes(p) for p in old.planes[1])
    for s in range(S):
        b.set_dyn_refs(pa, pb, stream=s)
    b.set_offsets(offs1)
    b.dyn_source_synth(F1, stream_base=0, t0=0)
    b.compose(F1)
    rc, st = b.update_refs([1], [1], [ipcm_file(oracle, W, H, newb)])
    assert rc == 0
    b.set_dyn_refs(pa, newb, stream=1)
    b.set_offsets(offs2)
    b.dyn_source_synth(F2, stream_base=0, t0=F1)
    b.compose(F2)
    assert b.sync() == 0, hs.last_error()
    nb = np.frombuffer(newb, np.uint8)
    ny, nu, nv = [(ctypes.c_uint8 * len(x)).from_buffer_copy(x.tobytes())
                  for x in (nb[:W * H], nb[W * H:W * H * 5 // 4], nb[W * H * 5 // 4:])]
    pic_b = Pic(W, H, ctypes.addressof(ny), ctypes.addressof(nu), ctypes.addressof(nv))
    R2 = Refs()
    R2.ab[0] = ctypes.pointer(old.pics[0])
    R2.ab[1] = ctypes.pointer(pic_b)
    oracle.or_compose_dyn.restype = ctypes.c_size_t
    buf = (ctypes.c_uint8 * (8 << 20))()
    for s in range(S):
        cfg = OrCfg()
        oracle.or_cfg_init(ctypes.byref(cfg), W, H)
        cfg.frame_num = 2
        want = bytearray()
        for t, off in enumerate(offs1[s]):
            src = rect_source(oracle, s, t, rect)
            n = oracle.or_compose_dyn(buf, len(buf), ctypes.byref(cfg), int(off), 0, ctypes.byref(rect), src,
                                      ctypes.byref(old.refs), None)
            want += bytes(buf[:n])
        R = old.refs
        if s == 1:
            f = ipcm_file(oracle, W, H, newb)
            n = oracle.or_update_ref(buf, len(buf), ctypes.byref(cfg), f, len(f), 1)
            want += bytes(buf[:n])
            R = R2
        for t, off in enumerate(offs2[s]):
            src = rect_source(oracle, s, F1 + t, rect)
            n = oracle.or_compose_dyn(buf, len(buf), ctypes.byref(cfg), int(off), 0, ctypes.byref(rect), src,
                                      ctypes.byref(R), None)
            want += bytes(buf[:n])
        assert b.output(s) == bytes(want), s
    b.close()
