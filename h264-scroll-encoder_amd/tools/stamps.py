#!/usr/bin/env python3
"""Per-phase cycle stamps of k_emit (diagnostic build mode; SCROLL_DEBUG_EMIT_STAMPS)."""
import json, os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE)); sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import h264scroll as hs
from bench import synthetic_offsets
S, F, W, H = 256, 1024, 1280, 720
b = hs.Batch(S, F, F * 2 * (64 + (W // 16) * (H // 16)) + (1 << 16))
for _ in range(S):
    b.add_stream(hs.make_config(W, H))
b.set_offsets(synthetic_offsets(0, S, F, H))
b.compose(F, rewind=True); b.sync()
extra = 0
for a in sys.argv[1:]:
    if a.startswith("--flags="):
        extra = int(a.split("=", 1)[1])
b.set_debug(hs.SCROLL_DEBUG_EMIT_STAMPS | extra)
b.compose(F, rewind=True); assert b.sync() == 0
buf = (hs.ctypes.c_uint64 * (8 * 16384 * 2))()
n = hs.lib.scroll_batch_debug_stamps(b.h, buf, 16384 * 2)
a = np.frombuffer(buf, dtype=np.uint64)[: n * 8].reshape(n, 8).astype(np.int64)
act = a[a[:, 0] > 0]
t0 = act[:, 0].min()
d = {"waves": int(len(act)),
     "build": float(np.mean(act[:, 1] - act[:, 0])), "classify": float(np.mean(act[:, 2] - act[:, 1])),
     "mixed": float(np.mean(act[:, 3] - act[:, 2])), "stream": float(np.mean(act[:, 4] - act[:, 3])),
     "total_per_wave": float(np.mean(act[:, 4] - act[:, 0])),
     "span": float(act[:, 4].max() - t0),
     "start_spread": float(np.percentile(act[:, 0] - t0, [50, 90, 99]).tolist()[1]),
     "tot_chunks_mean": float(np.mean((act[:, 6] >> 32) & 0xffffff)), "tot_mx_mean": float(np.mean(act[:, 6] & 0xffffffff))}
rs = act[:, 5] & 0xffffffff; re_ = act[:, 7] & 0xffffffff
hw = (act[:, 7] >> 32) & 0xffffffff; xcc = (act[:, 6] >> 56) & 0xff
cu = (hw >> 8) & 0xf; se = (hw >> 13) & 0x7; sh = (hw >> 12) & 1; simd = (hw >> 4) & 3
r0 = rs.min()
d["realtime_span_us"] = float((re_.max() - r0) / 100.0)
d["wave_realtime_us_mean"] = float(np.mean(re_ - rs) / 100.0)
d["start_us_pct"] = [float(x) for x in np.percentile((rs - r0) / 100.0, [0, 25, 50, 75, 100])]
d["end_us_pct"] = [float(x) for x in np.percentile((re_ - r0) / 100.0, [0, 25, 50, 75, 100])]
key = xcc * 1000 + se * 100 + sh * 16 + cu
uk, cnts = np.unique(key, return_counts=True)
d["distinct_cus"] = int(len(uk)); d["waves_per_cu_min_max"] = [int(cnts.min()), int(cnts.max())]
# average concurrency over the span
T = np.arange(0, (re_.max() - r0), 5)
conc = [int(np.sum((rs - r0 <= t) & (re_ - r0 > t))) for t in T]
d["concurrency_samples"] = conc[:: max(1, len(conc) // 20)]
d["stream_cycles_per_64_chunks"] = d["stream"] / (d["tot_chunks_mean"] / 64)
print(json.dumps(d, indent=1))

# timeline: map each wave's memtime phase stamps onto its realtime span
# (constant clock per wave) and count waves per phase / bytes stored per bucket
if "--timeline" in sys.argv:
    m0 = act[:, 0].astype(np.float64); m4 = act[:, 4].astype(np.float64)
    scale = (re_ - rs).astype(np.float64) / np.maximum(m4 - m0, 1)
    ph = [(rs - r0) + (act[:, k] - m0) * scale for k in range(5)]   # 10-ns units
    pure_b = ((act[:, 6] >> 32) & 0xffffff).astype(np.float64) * 16   # all stored chunks
    mx_b = np.zeros_like(pure_b)
    step = 200                                                    # 2 us buckets
    rows = []
    for t in np.arange(0, ph[4].max(), step):
        t1 = t + step
        cnt = [int(np.sum((ph[k] <= t + step / 2) & (ph[k + 1] > t + step / 2))) for k in range(4)]
        def ov(a, b):
            return np.clip(np.minimum(b, t1) - np.maximum(a, t), 0, None) / np.maximum(b - a, 1e-9)
        by = float(np.sum(pure_b * ov(ph[3], ph[4])))
        rows.append([round(t / 100.0, 1)] + cnt + [round(by / (step * 10e-9) / 1e9, 0)])
    print("t_us build classify mixed stream GB/s")
    for r in rows:
        print(*r)
