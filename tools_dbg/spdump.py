"""dump the GPU bytes of the intra / multi-slice splice cases (debugging)"""
import ctypes, os, sys
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, os.path.join(R, "h264-scroll-encoder_amd"))
sys.path.insert(0, R)
import numpy as np
import h264scroll as gpu
from conftest import synthetic_offsets
from test_gpu_splice import plan, gpu_streams
oracle = ctypes.CDLL(os.path.join(R, "oracle", "_build", "liboracle.so"))
oracle.or_bench_compose.restype = ctypes.c_double
O = os.path.join(R, "gpurun_out", "spdbg")
os.makedirs(O, exist_ok=True)
w, h = 640, 480
offs = synthetic_offsets(4, 12, h, first_stream=5)
offs[1] = np.arange(488, 500)
for seed, rows in ((41, 0), (42, 1), (43, 2), (44, 3)):
    frames, want = plan(oracle, w, h, offs, seed, p_splice=0.9, p_hint=0.3, max_rect=(12, 9),
                        ext_kw=dict(intra_pm=500, slice_rows=rows, pcm_zero=seed % 2, part_pm=200, qp_jitter=5))
    b, rc = gpu_streams(gpu, w, h, offs, frames)
    print(seed, "rc", rc, gpu.last_error() if rc else "")
    for s in range(4):
        open(os.path.join(O, f"out_{seed}_{s}.bin"), "wb").write(bytes(b.output(s)))
        print(seed, s, "equal" if bytes(b.output(s)) == want[s] else "DIFF",
              [b.splice_status(s, f) for f in range(12)])
    b.close()
