#!/usr/bin/env python3
"""dyn_stamps.py -- profiling aid: where k_dyn_stage's time goes.

Runs the bench's config-3 workload (bench.py p720dyn) once with
SCROLL_DEBUG_DYN_STAMPS and prints, per dynamic NAL (one workgroup), the
s_memtime cycles spent in each window phase:
  A  residual -> transform -> quant -> levels / TotalCoeff
  B  nC + CAVLC encode into registers, chroma DC
  C  MB heads, piece offsets, window scan
  D  bits -> LDS buffer
  E  flush to the staging slot + EP count
plus the number of windows and the workgroup's total.  Then times the
workload without stamps (HIP events).

    python h264-scroll-encoder_amd/tools/dyn_stamps.py [--streams 256 --frames 16]
"""
import argparse
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ablate", action="store_true", help="also time the SCROLL_DEBUG_DYN_* ablations")
    args = ap.parse_args()
    import numpy as np
    import h264scroll as hs
    import bench

    wl = bench.WORKLOADS["p720dyn"]
    W, H, rect = wl["w"], wl["h"], wl["rect"]
    S, F = args.streams, args.frames
    b = hs.Batch(S, F, F * (2 * (64 + 3600) + 192 * 625) + (1 << 20))
    for _ in range(S):
        b.add_stream(hs.make_config(W, H))
    b.set_offsets(bench.synthetic_offsets(0, S, F, H))
    b.set_dyn_rect(*rect)
    ra, rb = bench.striped_i420(W, H, 0), bench.striped_i420(W, H, 1)
    for s in range(S):
        b.set_dyn_refs(ra, rb, stream=s)
    b.dyn_source_synth(F)
    b.compose(F, rewind=True)
    assert b.sync() == 0, hs.last_error()

    b.enable_timing(True)
    b.kernel_stats_ex()
    for _ in range(args.reps):
        b.compose(F, rewind=True)
    assert b.sync() == 0, hs.last_error()
    ms, n = b.kernel_stats_ex()
    print("kernel ms per compose: plan %.4f  emit %.4f  dyn_stage %.4f  dyn_emit %.4f"
          % tuple(x / n for x in ms))
    b.enable_timing(False)

    if args.ablate:
        for name, fl in (("no pixel loads", hs.SCROLL_DEBUG_DYN_NOLOAD),
                         ("no block CAVLC", hs.SCROLL_DEBUG_DYN_NOCAVLC),
                         ("no MB heads", hs.SCROLL_DEBUG_DYN_NOHEAD),
                         ("no bit writes", hs.SCROLL_DEBUG_DYN_NOWRITE),
                         ("none of these", hs.SCROLL_DEBUG_DYN_NOLOAD | hs.SCROLL_DEBUG_DYN_NOCAVLC |
                          hs.SCROLL_DEBUG_DYN_NOHEAD | hs.SCROLL_DEBUG_DYN_NOWRITE)):
            b.set_debug(fl)
            b.enable_timing(True)
            b.kernel_stats_ex()
            for _ in range(args.reps):
                b.compose(F, rewind=True)
            b.sync()
            ms, n = b.kernel_stats_ex()
            b.enable_timing(False)
            print("ablation %-16s dyn_stage %.4f ms" % (name, ms[2] / n))
    b.set_debug(hs.SCROLL_DEBUG_DYN_STAMPS)
    b.compose(F, rewind=True)
    assert b.sync() == 0, hs.last_error()
    buf = (ctypes.c_uint64 * (2 * S * F * 8))()
    got = hs.lib.scroll_batch_debug_stamps(b.h, buf, 2 * S * F)
    allst = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)[:got]
    a = allst[:S * F].astype(np.float64)
    names = ["A levels", "B cavlc", "C offsets", "D bits", "E flush"]
    tot = a[:, 6].mean()
    print(f"{S * F} NALs, windows/NAL {a[:, 5].mean():.1f}, cycles/NAL {tot:.0f} "
          f"(min {a[:, 6].min():.0f} max {a[:, 6].max():.0f})")
    for k, nm in enumerate(names):
        m = a[:, k].mean()
        print(f"  {nm:10s} {m:10.0f} cycles/NAL  {m / a[:, 5].mean():8.0f} /window  {100 * m / tot:5.1f} %")
    rest = tot - a[:, :5].sum(1).mean()
    print(f"  {'setup+tail':10s} {rest:10.0f} cycles/NAL  {100 * rest / tot:5.1f} %")
    e = allst[S * F:].astype(np.int64)          # k_dyn_emit_gather: realtime (100 MHz)
    e = e[e[:, 0] > 0]
    if len(e):
        t0 = e[:, 0].min()
        span = (e[:, 2].max() - t0) / 100.0
        dur = (e[:, 2] - e[:, 0]) / 100.0
        srt = (e[:, 1] - e[:, 0]) / 100.0
        print(f"k_dyn_emit_gather: {len(e)} WGs, span {span:.1f} us, WG duration mean {dur.mean():.1f} "
              f"p50 {np.percentile(dur, 50):.1f} p99 {np.percentile(dur, 99):.1f} max {dur.max():.1f} us, "
              f"prologue+sort mean {srt.mean():.1f} us")
        st0 = (e[:, 0] - t0) / 100.0
        print("  WG start times (us) p0/25/50/75/100:", np.percentile(st0, [0, 25, 50, 75, 100]).round(1))
        conc = [(np.sum((e[:, 0] <= x) & (e[:, 2] > x))) for x in np.linspace(t0, e[:, 2].max(), 12)]
        print("  resident WGs over time:", conc)
    b.close()


if __name__ == "__main__":
    main()
