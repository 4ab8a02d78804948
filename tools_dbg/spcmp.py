"""compare the dumped GPU splice bytes with the oracle's, MB by MB (debugging, CPU)"""
import ctypes, os, sys
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, R)
import numpy as np
from conftest import synthetic_offsets
from test_gpu_splice import plan
from dynhelp import split_nals
import h264_pslice as P
oracle = ctypes.CDLL(os.path.join(R, "oracle", "_build", "liboracle.so"))
oracle.or_bench_compose.restype = ctypes.c_double
w, h = 640, 480
offs = synthetic_offsets(4, 12, h, first_stream=5)
offs[1] = np.arange(488, 500)
seed = int(sys.argv[1]); rows = {41: 0, 42: 1, 43: 2, 44: 3}[seed]
frames, want = plan(oracle, w, h, offs, seed, p_splice=0.9, p_hint=0.3, max_rect=(12, 9),
                    ext_kw=dict(intra_pm=500, slice_rows=rows, pcm_zero=seed % 2, part_pm=200, qp_jitter=5))
for s in range(4):
    got = open(os.path.join(R, "gpurun_out", "spdbg", f"out_{seed}_{s}.bin"), "rb").read()
    if got == want[s]:
        print(s, "equal"); continue
    gn, wn = split_nals(got), split_nals(want[s])
    k = next(i for i, (x, y) in enumerate(zip(gn, wn)) if x != y)
    print("stream", s, "nal", k, len(gn[k]), len(wn[k]))
    # which frame: count scroll NALs
    print([ (t, frames[(s, t)][1], frames[(s, t)][2][:4] if frames[(s, t)][2] else None) for t in range(12)])
    for t in range(12):
        pass
    bg, bw = gn[k], wn[k]
    i = next(i for i in range(min(len(bg), len(bw))) if bg[i] != bw[i])
    print("first differing byte", i)
    for pred in ("spec", "ref"):
        try:
            Hg, mg = P.decode_p_slice(bg, w, h, predictor=pred)
            Hw, mw = P.decode_p_slice(bw, w, h, predictor=pred)
        except Exception as e:
            print(pred, "decode failed", repr(e)); continue
        for y in range(h // 16):
            for x in range(w // 16):
                a, b = mg[y][x], mw[y][x]
                if a != b:
                    print(pred, "MB", x, y, {kk: (a[kk], b[kk]) for kk in a if a[kk] != b[kk] and kk not in ("luma", "cac")})
                    break
            else:
                continue
            break
