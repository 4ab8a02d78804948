#!/usr/bin/env python3
"""dyn_stamps.py -- profiling aid: where k_dyn_row's time goes.

Runs a dynamic-rect workload of the bench (default p720dyn = config 3) once with
SCROLL_DEBUG_DYN_STAMPS and prints, per k_dyn_row workgroup (one rect row),
the s_memrealtime span (100 MHz, microseconds) of each phase:
  levels       pixels -> residual -> transform -> quant, TotalCoeff ranks
  cavlc+poll   CAVLC bodies; the last wave polls the row above's TotalCoeffs
  tokens       coeff_token and length of every piece
  mb+scan      cbp, piece offsets per MB; the row's MB offsets
  write        bits -> LDS window -> the row's row-stage words
plus the k_dyn_epfix steps and the k_dyn_gather workgroup spans.  Then times the workload
without stamps (HIP events).

    python h264-scroll-encoder_amd/tools/dyn_stamps.py [--workload p4kdyn]
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
    ap.add_argument("--workload", default="p720dyn", help="a dynamic-rect workload of bench.py")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import h264scroll as hs
    import bench

    wl = bench.WORKLOADS[args.workload]
    W, H, rect = wl["w"], wl["h"], wl["rect"]
    S, F = wl["streams"], wl["frames"]
    b = bench.build_compose_batch(hs, wl, 0, 0)         # the benched batch
    b.compose(F, rewind=True)
    assert b.sync() == 0, hs.last_error()

    b.enable_timing(True)
    b.kernel_stats_ex()
    for _ in range(args.reps):
        b.compose(F, rewind=True)
    assert b.sync() == 0, hs.last_error()
    ms, n = b.kernel_stats_ex()
    print("kernel ms per compose: plan %.4f  emit %.4f  dyn_stage %.4f  dyn_emit %.4f  dyn_code %.4f  dyn_pack %.4f"
          % tuple(x / n for x in ms))
    b.enable_timing(False)

    b.set_debug(hs.SCROLL_DEBUG_DYN_STAMPS)
    b.compose(F, rewind=True)
    assert b.sync() == 0, hs.last_error()
    mbh = H // 16
    na = max(1, -(-rect[1] // 64))                 # DYN_STATIC_ROWS = 64
    ng = na + rect[3] + max(1, -(-(mbh - rect[1] - rect[3]) // 64))
    nslot = (2 + ng) * S * F
    buf = (ctypes.c_uint64 * (nslot * 8))()
    got = hs.lib.scroll_batch_debug_stamps(b.h, buf, nslot)
    allst = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)[:got]
    grp = allst[2 * S * F:].astype(np.int64).reshape(S * F, ng, 8)
    rnames = ["levels", "cavlc+poll", "tokens", "mb+scan+lb", "write"]     # k_dyn_row
    for label, sel in (("rect rows (k_dyn_row)", slice(na, na + rect[3])),):
        names = rnames
        gsel = grp[:, sel].reshape(-1, 8)
        gsel = gsel[gsel[:, 5] > 0]
        if not len(gsel):                          # k_dyn_static records no stamps
            continue
        st = gsel[:, :6].astype(np.float64)
        tot = (st[:, 5] - st[:, 0]) / 100.0
        print(f"{label}: {len(gsel)} WGs, duration mean {tot.mean():.2f} us p50 {np.percentile(tot, 50):.2f} "
              f"p99 {np.percentile(tot, 99):.2f}, bits mean {gsel[:, 6].mean():.0f}")
        prev = st[:, 0]
        for k, nm in enumerate(names):
            cur = st[:, k + 1]
            cur = np.where(cur > 0, cur, prev)
            d = (cur - prev) / 100.0
            print(f"  {nm:9s} mean {d.mean():7.2f} us  p99 {np.percentile(d, 99):7.2f}")
            prev = cur
    for label, sel in (("k_dyn_row", slice(na, na + rect[3])),):
        gg = grp[:, sel]
        g0 = gg[:, :, 0][gg[:, :, 5] > 0]
        t0, t1 = g0.min(), gg[:, :, 5].max()
        print(f"{label} span {(t1 - t0) / 100.0:.1f} us")
        ends = gg[:, :, 5][gg[:, :, 5] > 0]
        conc = [int(np.sum((g0 <= x) & (ends > x))) for x in np.linspace(t0, t1, 12)]
        print("  resident WGs over time:", conc)
    x = allst[:S * F].astype(np.int64)           # k_dyn_epfix: entry, table+counts, work, sort, end
    x = x[x[:, 5] > 0]
    if len(x):
        t0 = x[:, 0].min()
        print(f"k_dyn_epfix: {len(x)} WGs, span {(x[:, 5].max() - t0) / 100.0:.1f} us, WG duration mean "
              f"{((x[:, 5] - x[:, 0]) / 100.0).mean():.1f} us, candidate words mean {(x[:, 6] & 0xffffffff).mean():.1f}, "
              f"EP positions mean {(x[:, 6] >> 32).mean():.1f}")
        # slots: 0 entry, 1 table+counts, 2 seams+cands (barrier), 3 sort, 4 wave 0's
        # candidates, 5 end, 6 counts, 7 the seam wave's end
        for nm, a, b_ in (("table+counts", 0, 1), ("seams+cands", 1, 2), ("  seam wave", 1, 7),
                          ("  cand wave0", 1, 4), ("sort", 2, 3), ("compact+out", 3, 5)):
            ok = x[:, b_] > 0
            d = (x[ok, b_] - x[ok, a]) / 100.0
            if len(d):
                print(f"  {nm:12s} mean {d.mean():7.2f} us  p99 {np.percentile(d, 99):7.2f}")
        nc = (x[:, 6] & 0xffffffff).astype(np.float64)
        dur = (x[:, 5] - x[:, 0]) / 100.0
        q = np.percentile(nc, [25, 50, 75])
        for lo, hi in ((0, q[0]), (q[0], q[1]), (q[1], q[2]), (q[2], np.inf)):
            m = (nc >= lo) & (nc < hi)
            if m.any():
                print(f"  candidates [{lo:.0f}, {hi:.0f}): {int(m.sum())} WGs, duration mean {dur[m].mean():.1f} us")
        conc = [int(np.sum((x[:, 0] <= v) & (x[:, 5] > v))) for v in np.linspace(t0, x[:, 5].max(), 12)]
        print("  resident WGs over time:", conc)
    e = allst[S * F:2 * S * F].astype(np.int64)  # k_dyn_gather: realtime (100 MHz)
    e = e[e[:, 0] > 0]
    if len(e):
        t0 = e[:, 0].min()
        span = (e[:, 2].max() - t0) / 100.0
        dur = (e[:, 2] - e[:, 0]) / 100.0
        srt = (e[:, 1] - e[:, 0]) / 100.0
        print(f"k_dyn_gather: {len(e)} WGs, span {span:.1f} us, WG duration mean {dur.mean():.1f} "
              f"p50 {np.percentile(dur, 50):.1f} p99 {np.percentile(dur, 99):.1f} max {dur.max():.1f} us, "
              f"prologue+sort mean {srt.mean():.1f} us")
        st0 = (e[:, 0] - t0) / 100.0
        print("  WG start times (us) p0/25/50/75/100:", np.percentile(st0, [0, 25, 50, 75, 100]).round(1))
        conc = [(np.sum((e[:, 0] <= x) & (e[:, 2] > x))) for x in np.linspace(t0, e[:, 2].max(), 12)]
        print("  resident WGs over time:", conc)
    b.close()


if __name__ == "__main__":
    main()
