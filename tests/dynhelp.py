"""ctypes views of the dynamic-rect oracle (oracle/dyn_oracle.h) for tests."""
import ctypes


class OrCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("w", "h", "log2_mfn", "poc_type", "log2_poc", "num_ref_default_m1",
                 "deblock", "frame_num", "idr_pic_id", "nwp")] + [
        ("wp_off", ctypes.c_int * 8), ("wp_lt", ctypes.c_int * 8), ("wp_valid", ctypes.c_int * 8)]


class Rect(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("x0", "y0", "w", "h")]


class Pic(ctypes.Structure):
    _fields_ = [("w", ctypes.c_int), ("h", ctypes.c_int), ("y", ctypes.c_void_p),
                ("u", ctypes.c_void_p), ("v", ctypes.c_void_p)]


class Refs(ctypes.Structure):
    _fields_ = [("ab", ctypes.POINTER(Pic) * 2)]


class StripedRefs:
    """decoded I_PCM striped pictures A, B (the composer's synthetic refs)"""

    def __init__(self, lib, w, h):
        self.planes, self.pics = [], []
        for which in (0, 1):
            y = (ctypes.c_uint8 * (w * h))()
            u = (ctypes.c_uint8 * (w * h // 4))()
            v = (ctypes.c_uint8 * (w * h // 4))()
            lib.or_striped_planes(y, u, v, w, h, which)
            self.planes.append((y, u, v))
            self.pics.append(Pic(w, h, ctypes.addressof(y), ctypes.addressof(u), ctypes.addressof(v)))
        self.refs = Refs()
        self.refs.ab[0] = ctypes.pointer(self.pics[0])
        self.refs.ab[1] = ctypes.pointer(self.pics[1])


def rect_source(lib, s, t, rect):
    src = (ctypes.c_uint8 * (384 * rect.w * rect.h))()
    lib.or_dyn_source(src, s, t, ctypes.byref(rect))
    return src


def split_nals(data):
    """Annex-B stream -> list of NAL units (each with its 4-byte start code)"""
    out, i = [], 0
    starts = []
    while True:
        j = data.find(b"\x00\x00\x00\x01", i)
        if j < 0:
            break
        starts.append(j)
        i = j + 4
    for k, a in enumerate(starts):
        out.append(data[a:starts[k + 1] if k + 1 < len(starts) else len(data)])
    return out
