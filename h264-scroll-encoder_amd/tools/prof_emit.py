#!/usr/bin/env python3
"""Ablation timing of the emit kernel (profiling aid, outputs of the ablated
variants are intentionally wrong).  Interleaves variants in one process.

    python h264-scroll-encoder_amd/tools/prof_emit.py [--streams 256] [--frames 1024]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--w", type=int, default=1280)
    ap.add_argument("--h", type=int, default=720)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variant", default="", help="run only this variant (for rocprofv3)")
    args = ap.parse_args()
    import h264scroll as hs
    from bench import synthetic_offsets

    S, F, W, H = args.streams, args.frames, args.w, args.h
    b = hs.Batch(S, F, F * 2 * (64 + (W // 16) * (H // 16)) + (1 << 16))
    for _ in range(S):
        b.add_stream(hs.make_config(W, H))
    b.set_offsets(synthetic_offsets(0, S, F, H))
    variants = {"full": 0, "nostore": hs.SCROLL_DEBUG_EMIT_NOSTORE,
                "zeros": hs.SCROLL_DEBUG_EMIT_ZEROS, "build": hs.SCROLL_DEBUG_EMIT_BUILD,
                "nopure": hs.SCROLL_DEBUG_EMIT_NOPURE, "nomixed": hs.SCROLL_DEBUG_EMIT_NOMIXED,
                "classify": hs.SCROLL_DEBUG_EMIT_NOPURE | hs.SCROLL_DEBUG_EMIT_NOMIXED,
                "nobytes": hs.SCROLL_DEBUG_EMIT_NOBYTES}
    if args.variant:
        variants = {args.variant: variants[args.variant]}
    res = {k: [] for k in variants}
    b.compose(F, rewind=True)
    b.sync()
    nbytes = b.last_bytes()
    b.enable_timing(True)
    for r in range(args.rounds):
        for name, fl in variants.items():
            b.set_debug(fl)
            b.kernel_stats()
            for _ in range(3):
                b.compose(F, rewind=True)
            assert b.sync() == 0, hs.last_error()
            p, e, n = b.kernel_stats()
            res[name].append((p / n, e / n))
    out = {"bytes_per_step": nbytes, "frames_per_step": S * F}
    for k, v in res.items():
        em = sorted(x[1] for x in v)[len(v) // 2]
        pm = sorted(x[0] for x in v)[len(v) // 2]
        out[k] = {"emit_ms_median": round(em, 4), "plan_ms_median": round(pm, 4),
                  "emit_GBps": round(nbytes / em / 1e6, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
