#!/usr/bin/env python3
"""row_occupancy.py -- profiling aid: resident k_dyn_row workgroups per CU
(the HIP occupancy calculator, scroll_debug_row_occupancy) for the benched
rects and around config 5's LDS size, on the GPU box.

    python h264-scroll-encoder_amd/tools/row_occupancy.py
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import h264scroll as hs
    f = hs.lib.scroll_debug_row_occupancy
    f.restype = ctypes.c_int
    for name, w, mbw in (("config 3", 25, 80), ("config 5", 47, 240)):
        print(name, "w", w, "mbw", mbw, "WGs/CU", f(w, mbw, 0))
    for d in range(0, -2600, -128):
        print("config 5 with", d, "bytes:", f(47, 240, d))


if __name__ == "__main__":
    main()
