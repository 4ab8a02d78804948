/*
 * hint_device.h -- motion of a hinted / spliced frame, shared by k_hint_stage
 * (hint_kernels.hip) and k_splice_stage (splice_kernels.hip): the MV field
 * of the UI hints over the scroll layout, the reference's predictor
 * (h264_writer.c:369-432), the standard's (H.264 8.4.1.3) and P_Skip motion
 * (8.4.1.1).  Bits: oracle/hint_oracle.c.
 */
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "composer_batch.h"
#include "scroll_device.h"

namespace scroll {
namespace hint {

/* (ref, mv) of an MB, mv in quarter pels; ref -1 = not available, -2 = an
 * intra MB (available with refIdx -1, mv 0: it matches no reference) */
struct Mv {
    int ref, mx, my;
};

/* scroll layout of the frame (h264_writer.c:555-620) */
struct Layout {
    int a_end, ra, mva4, rb, mvb4;
};

/* the MB's own motion: the topmost rect holding it, else its scroll row;
 * bad = the rect names no valid reference of the frame */
__device__ inline Mv field(const ScrollHintRect *rc, const int32_t *wv, int nr, int x, int y,
                           const Layout &lay, int nwp, bool &bad)
{
    for (int i = nr - 1; i >= 0; --i) {
        const ScrollHintRect r = rc[i];
        if (x >= r.x0 && x < r.x1 && y >= r.y0 && y < r.y1) {
            const int k = r.ref - 2;
            bad = !(r.ref == 0 || r.ref == 1 || (k >= 0 && k < nwp && wv[k]));
            return Mv{r.ref, 4 * r.mv_x, 4 * r.mv_y};
        }
    }
    bad = false;
    return y < lay.a_end ? Mv{lay.ra, 0, lay.mva4} : Mv{lay.rb, 0, lay.mvb4};
}

/* get_mv_prediction (h264_writer.c:369-432): C is above-right, else
 * above-left; 0 available -> 0; 1 available -> its mv if its ref matches;
 * exactly one ref match -> that mv; else median3 (:362-367) */
__device__ inline void predict_ref(const Mv &A, const Mv &B, const Mv &C, int ref, int &px,
                                   int &py)
{
    const bool aA = A.ref != -1, aB = B.ref != -1, aC = C.ref != -1;
    const bool mA = aA && A.ref == ref, mB = aB && B.ref == ref, mC = aC && C.ref == ref;
    const int na = (int)aA + (int)aB + (int)aC, nm = (int)mA + (int)mB + (int)mC;
    if (na == 0) {
        px = py = 0;
    } else if (na == 1) {
        const Mv &k = aA ? A : (aB ? B : C);
        const bool m = k.ref == ref;
        px = m ? k.mx : 0;
        py = m ? k.my : 0;
    } else if (nm == 1) {
        const Mv &k = mA ? A : (mB ? B : C);
        px = k.mx;
        py = k.my;
    } else {
        px = median3(aA ? A.mx : 0, aB ? B.mx : 0, aC ? C.mx : 0);
        py = median3(aA ? A.my : 0, aB ? B.my : 0, aC ? C.my : 0);
    }
}

__device__ inline int med3(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }

/* H.264 8.4.1.3 for a 16x16 partition (unavailable: ref -1, mv 0) */
__device__ inline void predict_spec(Mv A, Mv B, Mv C, int ref, int &px, int &py)
{
    if (B.ref == -1 && C.ref == -1 && A.ref != -1) {     /* 8.4.1.3.1 */
        B = A;
        C = A;
    }
    const bool mA = A.ref == ref, mB = B.ref == ref, mC = C.ref == ref;
    if ((int)mA + (int)mB + (int)mC == 1) {
        const Mv &k = mA ? A : (mB ? B : C);
        px = k.mx;
        py = k.my;
    } else {
        px = med3(A.mx, B.mx, C.mx);
        py = med3(A.my, B.my, C.my);
    }
}

/* H.264 8.4.1.1: motion of a P_Skip MB whose left / top neighbour MBs are
 * available (aA, aB: inside the picture and, in a multi-slice picture, the
 * same slice) */
__device__ inline void pskip_mv(bool aA, bool aB, const Mv &A, const Mv &B, const Mv &C, int &px,
                                int &py)
{
    if (!aA || !aB || (A.ref == 0 && A.mx == 0 && A.my == 0) ||
        (B.ref == 0 && B.mx == 0 && B.my == 0)) {
        px = py = 0;
        return;
    }
    predict_spec(A, B, C, 0, px, py);
}

}  // namespace hint
}  // namespace scroll
