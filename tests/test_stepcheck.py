"""The whole-step checker itself (CPU): or_compose_state advances the stream
state exactly as or_compose does, and oracle_step's last pass equals
composing every pass with the byte-writing oracle."""
import ctypes
import random

import numpy as np

import stepcheck
from conftest import synthetic_offsets
from dynhelp import OrCfg, Rect, StripedRefs, rect_source


def _cfg(oracle, w, h):
    c = OrCfg()
    oracle.or_cfg_init(ctypes.byref(c), w, h)
    c.frame_num = 2
    return c


def test_compose_state_matches_compose(oracle):
    rng = random.Random(4)
    buf = (ctypes.c_uint8 * (1 << 20))()
    for w, h in ((64, 2160), (320, 720)):
        for mode in (0, 1):
            a, b = _cfg(oracle, w, h), _cfg(oracle, w, h)
            for i in range(3000):
                off = rng.choice([rng.randint(-h, 2 * h), 496 * rng.randint(-4, 4)])
                oracle.or_compose(buf, len(buf), ctypes.byref(a), off, mode, None)
                oracle.or_compose_state(ctypes.byref(b), off, mode)
                assert bytes(a) == bytes(b), (w, h, mode, i, off)
            assert a.nwp == 8 or h < 2000           # the waypoint cap is reached


def test_oracle_step_equals_repeated_composes(oracle):
    w, h = 320, 720
    offs = synthetic_offsets(3, 40, h, first_stream=60)
    offs[0] = np.arange(470, 510)                # a waypoint in the first pass
    rect = (3, 20, 6, 5)
    got = stepcheck.oracle_step(oracle, w, h, offs, 3, rect=rect, stream_base=60, nthreads=3)
    R = StripedRefs(oracle, w, h)
    rc = Rect(*rect)
    oracle.or_compose_dyn.restype = ctypes.c_size_t
    buf = (ctypes.c_uint8 * (1 << 22))()
    for s in range(3):
        c = _cfg(oracle, w, h)
        for _ in range(3):
            o = bytearray()
            for t in range(40):
                src = rect_source(oracle, 60 + s, t, rc)
                n = oracle.or_compose_dyn(buf, len(buf), ctypes.byref(c), int(offs[s, t]), 0,
                                          ctypes.byref(rc), src, ctypes.byref(R.refs), None)
                o += bytes(buf[:n])
        assert got[s] == bytes(o), s
    p_only = stepcheck.oracle_step(oracle, w, h, offs, 2)
    for s in range(3):
        c = _cfg(oracle, w, h)
        for _ in range(2):
            o = bytearray()
            for t in range(40):
                n = oracle.or_compose(buf, len(buf), ctypes.byref(c), int(offs[s, t]), 0, None)
                o += bytes(buf[:n])
        assert p_only[s] == bytes(o), s
