"""ctypes views of the dynamic-rect oracle (oracle/dyn_oracle.h) for tests."""
import ctypes


class OrCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("w", "h", "log2_mfn", "poc_type", "log2_poc", "num_ref_default_m1",
                 "deblock", "frame_num", "idr_pic_id", "nwp")] + [
        ("wp_off", ctypes.c_int * 8), ("wp_lt", ctypes.c_int * 8), ("wp_valid", ctypes.c_int * 8)]


class Rect(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("x0", "y0", "w", "h", "qp")]   # qp 0 = 26, -1 = QP 0


def qp_field(qp):
    """or_dyn_rect.qp for a QP 0..51 (0 = 26 there, OR_DYN_QP0 = -1 is QP 0)"""
    return -1 if qp == 0 else qp


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


class FlatRefs:
    """pictures A, B of one sample value everywhere"""

    def __init__(self, w, h, value=0):
        self.planes, self.pics = [], []
        for _ in (0, 1):
            y = (ctypes.c_uint8 * (w * h))(*([value] * (w * h)))
            u = (ctypes.c_uint8 * (w * h // 4))(*([value] * (w * h // 4)))
            v = (ctypes.c_uint8 * (w * h // 4))(*([value] * (w * h // 4)))
            self.planes.append((y, u, v))
            self.pics.append(Pic(w, h, ctypes.addressof(y), ctypes.addressof(u), ctypes.addressof(v)))
        self.refs = Refs()
        self.refs.ab[0] = ctypes.pointer(self.pics[0])
        self.refs.ab[1] = ctypes.pointer(self.pics[1])

    def i420(self, which):
        return b"".join(bytes(p) for p in self.planes[which])


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


class HintRect(ctypes.Structure):
    """or_hint_rect / ScrollHintRect (include/composer_batch.h)"""
    _fields_ = [(n, ctypes.c_int16) for n in ("x0", "y0", "x1", "y1", "ref", "reserved")] + [
        ("mv_x", ctypes.c_int32), ("mv_y", ctypes.c_int32)]


def hint_array(rects):
    """[(x0, y0, x1, y1, ref, mv_x, mv_y), ...] -> ctypes array (or None)"""
    if not rects:
        return None, 0
    arr = (HintRect * len(rects))()
    for i, (x0, y0, x1, y1, ref, mx, my) in enumerate(rects):
        arr[i] = HintRect(x0, y0, x1, y1, ref, 0, mx, my)
    return arr, len(rects)


def random_hints(rng, mbw, mbh, refs, nmax=6):
    """a UI-like overlay: static chrome (ref 0, mv 0), horizontally scrolling
    rows, second panes, random rects; refs = the valid reference indices"""
    out = []
    for _ in range(rng.randint(0, nmax)):
        kind = rng.random()
        if kind < 0.3:                                     # static chrome bar
            y0 = rng.choice([0, max(0, mbh - 2)])
            out.append((0, y0, mbw, y0 + rng.randint(1, 2), 0, 0, 0))
        elif kind < 0.55:                                  # horizontally scrolling row(s)
            y0 = rng.randint(0, mbh - 1)
            out.append((0, y0, mbw, y0 + rng.randint(1, 3), rng.choice(refs),
                        rng.choice([-37, -16, -5, 3, 16, 64]), rng.choice([0, 0, 16, -32])))
        else:                                              # pane / popup
            x0, y0 = rng.randint(-2, mbw - 1), rng.randint(-2, mbh - 1)
            out.append((x0, y0, x0 + rng.randint(1, mbw), y0 + rng.randint(1, mbh),
                        rng.choice(refs), rng.randint(-80, 80), rng.randint(-300, 300)))
    return out


def striped_i420(w, h, which):
    """The experiment's striped I_PCM picture (experiments/scroll-encoder/src/
    main.c:234-243 colours, h264_encoder.c:816-829 bands) as I420 bytes."""
    import numpy as np
    cols = ([81, 90, 240, 145, 54, 34, 41, 240, 110], [210, 16, 146, 170, 166, 16, 106, 202, 222])[which]
    third = (h // 16) // 3
    band = np.where(np.arange(h // 16) < third, 0, np.where(np.arange(h // 16) < 2 * third, 1, 2))
    yrow = np.repeat(band, 16)
    crow = yrow[::2]
    Y = np.repeat(np.array([cols[3 * b] for b in yrow], np.uint8)[:, None], w, 1)
    U = np.repeat(np.array([cols[3 * b + 1] for b in crow], np.uint8)[:, None], w // 2, 1)
    V = np.repeat(np.array([cols[3 * b + 2] for b in crow], np.uint8)[:, None], w // 2, 1)
    return Y.tobytes() + U.tobytes() + V.tobytes()


def ipcm_file(oracle, w, h, pic):
    """oracle: SPS + PPS + I_PCM IDR of an I420 picture"""
    import ctypes
    cap = w * h * 3 + 4096
    buf = (ctypes.c_uint8 * cap)()
    src = (ctypes.c_uint8 * len(pic)).from_buffer_copy(pic)
    n = oracle.or_ipcm_picture_file(buf, cap, w, h, src)
    return bytes(buf[:n])


# ---------------------------------------------------- splice (splice_oracle.h)
class Splice(ctypes.Structure):
    _fields_ = [("x0", ctypes.c_int), ("y0", ctypes.c_int), ("w", ctypes.c_int),
                ("h", ctypes.c_int), ("nal", ctypes.c_void_p), ("n", ctypes.c_size_t)]


class ExtParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("nrefs", "max_ref", "skip_pm", "cbp_pm", "big_pm", "mv_range",
                 "slice_qp_delta", "qp_jitter", "ref_idc", "bad_mb", "bad_type", "list_mod",
                 "part_pm", "intra_pm", "slice_rows", "pcm_zero", "intra_types", "islice")]


EXT_DEFAULT = dict(nrefs=0, max_ref=1, skip_pm=250, cbp_pm=600, big_pm=20, mv_range=64,
                   slice_qp_delta=0, qp_jitter=3, ref_idc=0, bad_mb=-1, bad_type=0,
                   list_mod=0, part_pm=0, intra_pm=0, slice_rows=0, pcm_zero=0, intra_types=0, islice=0)


def ext_slice(oracle, cfg, w, h, seed, **kw):
    """a standard P slice of a w x h MB picture from the oracle's stand-in
    dynamic encoder (or_ext_slice), as Annex-B bytes"""
    p = ExtParams(**{**EXT_DEFAULT, **kw})
    cap = 4096 + w * h * 4096
    buf = (ctypes.c_uint8 * cap)()
    n = oracle.or_ext_slice(buf, cap, ctypes.byref(cfg), w, h, seed, ctypes.byref(p))
    return bytes(buf[:n])


def splice_of(x0, y0, w, h, nal):
    buf = ctypes.create_string_buffer(bytes(nal), max(1, len(nal)))
    sp = Splice(x0, y0, w, h, ctypes.cast(buf, ctypes.c_void_p), len(nal))
    sp._buf, sp.data = buf, bytes(nal)       # keep the bytes alive with the struct
    return sp
