"""Whole-step checker (test infrastructure): the bytes of one composed step of
every stream of a Batch against the CPU oracle (oracle/verify_oracle.h,
or_verify_compose on host threads).  Used by the scale parity tests
(tests/test_gpu_scale.py) and by bench.py after its timed region.

A bench step composes the same offsets again and again with rewound arenas;
`passes` = how many times the batch has composed them (the stream state --
frame_num, waypoint table -- carries from pass to pass), the arena holds the
last pass.
"""
import ctypes
import os
import subprocess

import numpy as np

from dynhelp import OrCfg, Rect, StripedRefs, hint_array

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_oracle():
    d = os.path.join(REPO, "oracle")
    so = os.path.join(d, "_build", "liboracle.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-C", d], check=True, stdout=subprocess.DEVNULL)
    lib = ctypes.CDLL(so)
    lib.or_verify_compose.restype = ctypes.c_int
    return lib


def oracle_step(oracle, W, H, offs, passes, rect=None, stream_base=0, t0=0, mode=0,
                nthreads=8, frame_num=2):
    """-> list of the oracle's bytes per stream for the last of `passes`
    compositions of offs[S][F] (config: make_config(W, H) defaults)"""
    offs = np.ascontiguousarray(offs, dtype=np.int32)
    S, F = offs.shape
    cfgs = (OrCfg * S)()
    for s in range(S):
        oracle.or_cfg_init(ctypes.byref(cfgs[s]), W, H)
        cfgs[s].frame_num = frame_num
    mbs = (W // 16) * (H // 16)
    rc_ = None
    refs = None
    if rect:
        rc_ = Rect(*rect)
        refs = StripedRefs(oracle, W, H)
    scale = 1                                   # grown on overflow
    while True:
        stride = scale * F * (2 * (256 + mbs) + (256 * rect[2] * rect[3] if rect else 0))
        out = np.empty(S * stride, np.uint8)
        sizes = (ctypes.c_size_t * S)()
        c2 = (OrCfg * S)()
        ctypes.memmove(c2, cfgs, ctypes.sizeof(cfgs))
        rc = oracle.or_verify_compose(
            S, F, c2, offs.ctypes.data_as(ctypes.c_void_p), mode,
            ctypes.byref(rc_) if rc_ else None, stream_base, t0, None,
            ctypes.byref(refs.refs) if refs else None, passes,
            out.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(stride), sizes, nthreads)
        if rc == 0:
            return [out[s * stride:s * stride + sizes[s]].tobytes() for s in range(S)]
        if scale >= 16:
            raise RuntimeError("or_verify_compose: a stream's bytes exceed the buffer")
        scale *= 4


def compare_streams(batch, want, streams=None):
    """-> (ok, detail): each stream's arena vs the oracle's bytes"""
    bad = []
    total = 0
    for s in (range(len(want)) if streams is None else streams):
        got = batch.output(s)
        total += len(got)
        if got != want[s]:
            a = np.frombuffer(got, np.uint8)
            b = np.frombuffer(want[s], np.uint8)
            n = min(len(a), len(b))
            first = int(np.argmax(a[:n] != b[:n])) if n and np.any(a[:n] != b[:n]) else n
            bad.append(f"stream {s}: {len(got)} vs {len(want[s])} bytes, first diff at {first}")
    return not bad, {"streams": len(want) if streams is None else len(list(streams)),
                     "bytes": total, "mismatches": bad[:8], "n_bad": len(bad)}


def oracle_hint_step(oracle, W, H, offs, passes, hints_of, mode, frame_num=2):
    """-> (bytes per stream, streams) of the last of `passes` compositions
    of offs[S][F] with the UI overlay hints_of(s, f) in hint mode `mode`
    (oracle/hint_oracle.c, one thread)"""
    S, F = offs.shape
    buf = (ctypes.c_uint8 * (4 << 20))()
    err = ctypes.c_int()
    outs = []
    for s in range(S):
        c = OrCfg()
        oracle.or_cfg_init(ctypes.byref(c), W, H)
        c.frame_num = frame_num
        for _ in range(passes - 1):
            for f in range(F):
                oracle.or_compose_state(ctypes.byref(c), int(offs[s, f]), 0)
        o = bytearray()
        for f in range(F):
            arr, n = hint_array(hints_of(s, f))
            k = oracle.or_compose_hint(buf, len(buf), ctypes.byref(c), int(offs[s, f]), 0, arr, n,
                                       mode, ctypes.byref(err))
            if err.value or not k:
                raise RuntimeError(f"hint oracle refused stream {s} frame {f}")
            o += bytes(buf[:k])
        outs.append(bytes(o))
    return outs, S
