"""ctypes binding of libh264scroll.so (the C ABI in include/*.h).

Python is only the test/bench harness here: the product is the C-ABI
library.  This module loads lib/libh264scroll.so from this directory and
raises immediately if it is missing -- there is no Python or CPU fallback.

Mirrors the reference interface names (include/composer.h, h264_writer.h,
nal.h, bitwriter.h, nal_parser.h) plus the additive batch API of
include/composer_batch.h.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("H264SCROLL_LIB") or os.path.join(HERE, "lib", "libh264scroll.so")

SCROLL_OK = 0
SCROLL_ERR_NO_DEVICE = -1
SCROLL_ERR_ARG = -2
SCROLL_ERR_OOM = -3
SCROLL_ERR_OVERFLOW = -4
SCROLL_ERR_HIP = -5
SCROLL_ERR_CONFIG = -6
SCROLL_ERR_DEVICE = -7
SCROLL_MODE_COMPOSER = 0
SCROLL_MODE_EXPERIMENT = 1
SCROLL_DEBUG_FORCE_SERIAL = 1
SCROLL_DEBUG_EMIT_NOSTORE = 2
SCROLL_DEBUG_EMIT_ZEROS = 4
SCROLL_DEBUG_EMIT_BUILD = 8
SCROLL_DEBUG_EMIT_NOPURE = 16
SCROLL_DEBUG_EMIT_NOMIXED = 32
SCROLL_DEBUG_EMIT_STAMPS = 64
SCROLL_DEBUG_EMIT_NOBYTES = 128
SCROLL_DEBUG_DYN_STAMPS = 256
SCROLL_DEBUG_DYN_NOLOAD = 512
SCROLL_DEBUG_DYN_NOCAVLC = 1024
SCROLL_DEBUG_DYN_NOHEAD = 2048
SCROLL_DEBUG_DYN_NOWRITE = 4096
SCROLL_DEBUG_DYN_EPCAP4 = 8192
SCROLL_DEBUG_DYN_NOPUBLISH = 16384
SCROLL_DEBUG_DYN_GATHER1 = 32768
SCROLL_DEBUG_DYN_EPWIN = 65536
SCROLL_COMPOSE_REWIND = 1
MAX_WAYPOINTS = 8
MV_LIMIT_PX = 496


class WaypointInfo(ctypes.Structure):
    _fields_ = [("offset_px", ctypes.c_int), ("long_term_idx", ctypes.c_int),
                ("valid", ctypes.c_int)]


class ComposerConfig(ctypes.Structure):
    """include/h264_writer.h ComposerConfig (reference :37-59)."""
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int),
                ("mb_width", ctypes.c_int), ("mb_height", ctypes.c_int),
                ("log2_max_frame_num", ctypes.c_int), ("pic_order_cnt_type", ctypes.c_int),
                ("log2_max_pic_order_cnt_lsb", ctypes.c_int),
                ("num_ref_idx_l0_default_minus1", ctypes.c_int),
                ("deblocking_filter_control_present_flag", ctypes.c_int),
                ("frame_num", ctypes.c_int), ("idr_pic_id", ctypes.c_int),
                ("waypoints", WaypointInfo * MAX_WAYPOINTS), ("num_waypoints", ctypes.c_int)]


class NALWriter(ctypes.Structure):
    _fields_ = [("output", ctypes.POINTER(ctypes.c_uint8)), ("output_capacity", ctypes.c_size_t),
                ("output_pos", ctypes.c_size_t), ("rbsp", ctypes.POINTER(ctypes.c_uint8)),
                ("rbsp_capacity", ctypes.c_size_t)]


class BitWriter(ctypes.Structure):
    _fields_ = [("buffer", ctypes.POINTER(ctypes.c_uint8)), ("capacity", ctypes.c_size_t),
                ("byte_pos", ctypes.c_size_t), ("bit_pos", ctypes.c_int),
                ("current_byte", ctypes.c_uint8)]


class BitReader(ctypes.Structure):
    _fields_ = [("buffer", ctypes.POINTER(ctypes.c_uint8)), ("size", ctypes.c_size_t),
                ("byte_pos", ctypes.c_size_t), ("bit_pos", ctypes.c_int)]


class NALUnit(ctypes.Structure):
    _fields_ = [("nal_ref_idc", ctypes.c_int), ("nal_unit_type", ctypes.c_int),
                ("data", ctypes.POINTER(ctypes.c_uint8)), ("size", ctypes.c_size_t),
                ("rbsp_size", ctypes.c_size_t)]


class NALParser(ctypes.Structure):
    _fields_ = [("data", ctypes.POINTER(ctypes.c_uint8)), ("size", ctypes.c_size_t),
                ("pos", ctypes.c_size_t)]


class Composer(ctypes.Structure):
    """include/composer.h Composer (reference :23-49), caller-allocated."""
    _fields_ = [("cfg", ComposerConfig), ("parse_cfg", ComposerConfig),
                ("ref_a_rbsp", ctypes.c_void_p), ("ref_a_size", ctypes.c_size_t),
                ("ref_b_rbsp", ctypes.c_void_p), ("ref_b_size", ctypes.c_size_t),
                ("orig_sps", ctypes.c_void_p), ("orig_sps_size", ctypes.c_size_t),
                ("orig_pps", ctypes.c_void_p), ("orig_pps_size", ctypes.c_size_t),
                ("nw", NALWriter), ("output_buffer", ctypes.c_void_p),
                ("output_capacity", ctypes.c_size_t), ("rbsp_temp", ctypes.c_void_p),
                ("rbsp_capacity", ctypes.c_size_t), ("frames_written", ctypes.c_int)]


class ScrollBatchDesc(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("max_streams", ctypes.c_int),
                ("max_frames", ctypes.c_int), ("arena_bytes", ctypes.c_size_t),
                ("mode", ctypes.c_int)]


class ScrollSpliceDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("s", "f", "x0", "y0", "w", "h")] + [
        ("nal", ctypes.c_void_p), ("n", ctypes.c_uint64)]


class ScrollHintRect(ctypes.Structure):
    """include/composer_batch.h: MBs [x0, x1) x [y0, y1) take reference
    `ref` (0 = A, 1 = B, 2 + i = waypoint i) and displacement (mv_x, mv_y) px"""
    _fields_ = [(n, ctypes.c_int16) for n in ("x0", "y0", "x1", "y1", "ref", "reserved")] + [
        ("mv_x", ctypes.c_int32), ("mv_y", ctypes.c_int32)]


SCROLL_HINT_EXACT, SCROLL_HINT_PSKIP, SCROLL_HINT_SPEC, SCROLL_HINT_MAX_RECTS = 0, 1, 2, 64
(SCROLL_SPLICE_OK, SCROLL_SPLICE_ERR_NAL, SCROLL_SPLICE_ERR_HEADER, SCROLL_SPLICE_ERR_MBTYPE,
 SCROLL_SPLICE_ERR_SYNTAX, SCROLL_SPLICE_ERR_REF) = range(6)


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `make -C h264-scroll-encoder_amd` "
                          "(there is no fallback implementation)")
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    u8p = P(ctypes.c_uint8)
    sig = {
        "scroll_last_error": (ctypes.c_char_p, []),
        "scroll_device_count": (ctypes.c_int, []),
        "scroll_version": (ctypes.c_char_p, []),
        "scroll_batch_create": (ctypes.c_int, [P(ctypes.c_void_p), P(ScrollBatchDesc)]),
        "scroll_batch_destroy": (None, [ctypes.c_void_p]),
        "scroll_batch_add_stream": (ctypes.c_int, [ctypes.c_void_p, P(ComposerConfig)]),
        "scroll_batch_num_streams": (ctypes.c_int, [ctypes.c_void_p]),
        "scroll_batch_set_debug": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
        "scroll_batch_set_offsets": (ctypes.c_int, [ctypes.c_void_p, P(ctypes.c_int32),
                                                    ctypes.c_int]),
        "scroll_batch_offsets_device": (ctypes.c_void_p, [ctypes.c_void_p]),
        "scroll_batch_compose": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
        "scroll_batch_sync": (ctypes.c_int, [ctypes.c_void_p]),
        "scroll_batch_compose_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                   ctypes.c_int]),
        "scroll_batch_kernel_stats": (ctypes.c_int, [ctypes.c_void_p, P(ctypes.c_double),
                                                     P(ctypes.c_double), P(ctypes.c_int)]),
        "scroll_batch_last_bytes": (ctypes.c_ulonglong, [ctypes.c_void_p]),
        "scroll_batch_debug_stamps": (ctypes.c_longlong, [ctypes.c_void_p, P(ctypes.c_uint64),
                                                          ctypes.c_longlong]),
        "scroll_batch_last_nals": (ctypes.c_longlong, [ctypes.c_void_p]),
        "scroll_batch_get_config": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int,
                                                   P(ComposerConfig)]),
        "scroll_batch_set_config": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int,
                                                   P(ComposerConfig)]),
        "scroll_batch_output_size": (ctypes.c_size_t, [ctypes.c_void_p, ctypes.c_int]),
        "scroll_batch_copy_output": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int,
                                                    ctypes.c_size_t, u8p, ctypes.c_size_t]),
        "scroll_batch_output_device": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_int]),
        "scroll_host_alloc": (ctypes.c_int, [P(ctypes.c_void_p), ctypes.c_size_t]),
        "scroll_host_free": (None, [ctypes.c_void_p]),
        "scroll_batch_output_to_host_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p,
                                                             ctypes.c_size_t, ctypes.c_void_p,
                                                             ctypes.c_void_p]),
        "scroll_batch_reset_output": (ctypes.c_int, [ctypes.c_void_p]),
        "scroll_batch_nal_count": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
        "scroll_batch_nal_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                 P(ctypes.c_int), P(ctypes.c_int),
                                                 P(ctypes.c_uint32), P(ctypes.c_int)]),
        "scroll_batch_enable_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
        "scroll_batch_kernel_ms": (ctypes.c_float, [ctypes.c_void_p, ctypes.c_int]),
        "scroll_batch_set_dyn_rect": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_int] * 4 +
                                      [ctypes.c_size_t]),
        "scroll_batch_set_dyn_refs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, u8p, u8p]),
        "scroll_batch_set_dyn_qp": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
        "scroll_batch_set_dyn_qp_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
        "scroll_batch_set_dyn_qp_at": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                      ctypes.c_int]),
        "scroll_batch_set_dyn_source": (ctypes.c_int, [ctypes.c_void_p, u8p, ctypes.c_int]),
        "scroll_batch_set_dyn_rect_at": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_int] * 4),
        "scroll_batch_set_fallback": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
        "scroll_batch_fallback_frame": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                       ctypes.POINTER(ctypes.c_int)]),
        "scroll_batch_dyn_source_device": (ctypes.c_void_p, [ctypes.c_void_p, P(ctypes.c_size_t),
                                                             P(ctypes.c_size_t)]),
        "scroll_batch_dyn_source_synth": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int,
                                                         ctypes.c_int, ctypes.c_int]),
        "scroll_batch_dyn_frame_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                       P(ctypes.c_uint32), P(ctypes.c_uint32)]),
        "scroll_batch_dyn_totals": (ctypes.c_int, [ctypes.c_void_p, P(ctypes.c_ulonglong),
                                                   P(ctypes.c_ulonglong), P(ctypes.c_longlong)]),
        "scroll_batch_kernel_stats_ex": (ctypes.c_int, [ctypes.c_void_p, P(ctypes.c_double),
                                                        P(ctypes.c_int)]),
        "scroll_batch_set_hints": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                  P(ScrollHintRect), ctypes.c_int, ctypes.c_int]),
        "scroll_batch_clear_hints": (ctypes.c_int, [ctypes.c_void_p]),
        "scroll_batch_set_splice": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]),
        "scroll_batch_clear_splices": (ctypes.c_int, [ctypes.c_void_p]),
        "scroll_batch_set_splices_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int,
                                                           P(ScrollSpliceDesc)]),
        "scroll_batch_splice_status": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                      P(ctypes.c_int)]),
        "scroll_batch_splice_refusal": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                       P(ctypes.c_int), P(ctypes.c_int), P(ctypes.c_int),
                                                       P(ctypes.c_int)]),
        "scroll_batch_ingest": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, P(u8p),
                                               P(ctypes.c_size_t), P(u8p), P(ctypes.c_size_t),
                                               P(ctypes.c_int)]),
        "scroll_batch_update_refs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, P(ctypes.c_int),
                                                    P(ctypes.c_int), P(u8p), P(ctypes.c_size_t),
                                                    P(ctypes.c_int)]),
        "scroll_batch_update_refs_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, P(ctypes.c_int),
                                                           P(ctypes.c_int), ctypes.c_void_p,
                                                           P(ctypes.c_uint64), P(ctypes.c_int)]),
        "scroll_batch_ingest_stats": (ctypes.c_int, [ctypes.c_void_p, P(ctypes.c_double),
                                                     P(ctypes.c_int)]),
        "scroll_batch_ingest_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int,
                                                      ctypes.c_void_p, P(ctypes.c_uint64),
                                                      P(ctypes.c_int)]),
        "scroll_batch_ipcm_files_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                                          ctypes.c_void_p, ctypes.c_size_t,
                                                          P(ctypes.c_uint64)]),
        "scroll_batch_ipcm_files_device_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                                ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                                                ctypes.c_void_p, ctypes.c_size_t,
                                                                ctypes.c_void_p]),
        "scroll_batch_ipcm_stats": (ctypes.c_int, [ctypes.c_void_p, P(ctypes.c_double),
                                                   P(ctypes.c_int)]),
        "composer_batch_write_scroll_frames": (ctypes.c_int, [P(P(Composer)), P(ctypes.c_int),
                                                              ctypes.c_int, ctypes.c_int]),
        "composer_flush": (ctypes.c_int, [P(Composer)]),
        # reference ABI
        "composer_init": (ctypes.c_int, [P(Composer), ctypes.c_char_p, ctypes.c_char_p]),
        "composer_get_width": (ctypes.c_int, [P(Composer)]),
        "composer_get_height": (ctypes.c_int, [P(Composer)]),
        "composer_write_header": (None, [P(Composer)]),
        "composer_write_scroll_frame": (None, [P(Composer), ctypes.c_int]),
        "composer_get_output_size": (ctypes.c_size_t, [P(Composer)]),
        "composer_get_output": (u8p, [P(Composer)]),
        "composer_write_to_file": (ctypes.c_int, [P(Composer), ctypes.c_char_p]),
        "composer_finish": (None, [P(Composer)]),
        "composer_config_init": (None, [P(ComposerConfig), ctypes.c_int, ctypes.c_int]),
        "composer_config_set_sps_params": (None, [P(ComposerConfig), ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_int]),
        "composer_config_set_pps_params": (None, [P(ComposerConfig), ctypes.c_int,
                                                  ctypes.c_int]),
        "h264_generate_sps": (ctypes.c_size_t, [u8p, ctypes.c_size_t, ctypes.c_int,
                                                ctypes.c_int]),
        "h264_generate_pps": (ctypes.c_size_t, [u8p, ctypes.c_size_t]),
        "h264_rewrite_idr_frame": (ctypes.c_size_t, [P(NALWriter), P(ComposerConfig),
                                                     P(ComposerConfig), u8p, ctypes.c_size_t]),
        "h264_rewrite_as_non_idr_i_frame": (ctypes.c_size_t, [P(NALWriter), P(ComposerConfig),
                                                              P(ComposerConfig), u8p,
                                                              ctypes.c_size_t, ctypes.c_int]),
        "h264_write_scroll_p_frame": (ctypes.c_size_t, [P(NALWriter), P(ComposerConfig),
                                                        ctypes.c_int]),
        "h264_needs_waypoint": (ctypes.c_int, [P(ComposerConfig), ctypes.c_int]),
        "h264_write_waypoint_p_frame": (ctypes.c_size_t, [P(NALWriter), P(ComposerConfig),
                                                          ctypes.c_int]),
        "nal_writer_init": (None, [P(NALWriter), u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]),
        "nal_write_unit": (ctypes.c_size_t, [P(NALWriter), ctypes.c_int, ctypes.c_int, u8p,
                                             ctypes.c_size_t, ctypes.c_int]),
        "nal_writer_get_size": (ctypes.c_size_t, [P(NALWriter)]),
        "nal_writer_get_output": (u8p, [P(NALWriter)]),
        "rbsp_to_ebsp": (ctypes.c_size_t, [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]),
        "nal_parser_init": (None, [P(NALParser), u8p, ctypes.c_size_t]),
        "nal_parser_next": (ctypes.c_int, [P(NALParser), P(NALUnit)]),
        "ebsp_to_rbsp": (ctypes.c_size_t, [u8p, u8p, ctypes.c_size_t]),
        "parse_sps": (ctypes.c_int, [u8p, ctypes.c_size_t] + [P(ctypes.c_int)] * 5),
        "parse_pps": (ctypes.c_int, [u8p, ctypes.c_size_t] + [P(ctypes.c_int)] * 2),
        "bitwriter_init": (None, [P(BitWriter), u8p, ctypes.c_size_t]),
        "bitwriter_write_bits": (None, [P(BitWriter), ctypes.c_uint32, ctypes.c_int]),
        "bitwriter_write_bit": (None, [P(BitWriter), ctypes.c_int]),
        "bitwriter_write_ue": (None, [P(BitWriter), ctypes.c_uint32]),
        "bitwriter_write_se": (None, [P(BitWriter), ctypes.c_int32]),
        "bitwriter_write_trailing_bits": (None, [P(BitWriter)]),
        "bitwriter_flush": (None, [P(BitWriter)]),
        "bitwriter_get_size": (ctypes.c_size_t, [P(BitWriter)]),
        "bitwriter_get_bit_position": (ctypes.c_size_t, [P(BitWriter)]),
        "bitwriter_is_byte_aligned": (ctypes.c_int, [P(BitWriter)]),
        "bitreader_init": (None, [P(BitReader), u8p, ctypes.c_size_t]),
        "bitreader_read_bits": (ctypes.c_uint32, [P(BitReader), ctypes.c_int]),
        "bitreader_read_bit": (ctypes.c_int, [P(BitReader)]),
        "bitreader_read_ue": (ctypes.c_uint32, [P(BitReader)]),
        "bitreader_read_se": (ctypes.c_int32, [P(BitReader)]),
        "bitreader_get_bit_position": (ctypes.c_size_t, [P(BitReader)]),
        "bitreader_is_byte_aligned": (ctypes.c_int, [P(BitReader)]),
        "bitreader_get_remaining_bytes": (ctypes.c_size_t, [P(BitReader)]),
        "bitreader_get_pointer": (u8p, [P(BitReader)]),
    }
    # an A/B variant library from an earlier revision (H264SCROLL_LIB) may
    # lack the newest entry points: those stay unbound there (a call fails
    # loudly); the tree's own library must export every one
    variant = bool(os.environ.get("H264SCROLL_LIB"))
    for name, (res, args) in sig.items():
        try:
            f = getattr(lib, name)
        except AttributeError:
            if variant:
                continue
            raise
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def last_error():
    return (lib.scroll_last_error() or b"").decode()


def device_count():
    return lib.scroll_device_count()


def u8buf(data_or_size):
    if isinstance(data_or_size, int):
        return (ctypes.c_uint8 * data_or_size)()
    b = (ctypes.c_uint8 * len(data_or_size)).from_buffer_copy(data_or_size)
    return b


class HostBuffer:
    """Pinned host memory the device writes into (scroll_host_alloc): the
    packed bytes of Batch.output_to_host_async and its (offset, size) table."""

    def __init__(self, nbytes, nstreams):
        self.cap = (nbytes + 15) & ~15
        self.ns = nstreams
        self.p = ctypes.c_void_p()
        self.t = ctypes.c_void_p()
        if lib.scroll_host_alloc(ctypes.byref(self.p), self.cap) or \
                lib.scroll_host_alloc(ctypes.byref(self.t), 8 * (1 + 2 * nstreams)):
            raise RuntimeError("scroll_host_alloc: " + last_error())
        self.table = (ctypes.c_uint64 * (1 + 2 * nstreams)).from_address(self.t.value)
        self.data = (ctypes.c_uint8 * self.cap).from_address(self.p.value)

    def total(self):
        """packed bytes of the last delivery (None: it did not fit)"""
        v = self.table[0]
        return None if v == (1 << 64) - 1 else v

    def stream(self, s):
        """stream s's bytes of the last delivery; raises when that delivery did
        not fit (nothing was written, the table rows are stale)"""
        if self.total() is None:
            raise RuntimeError("the last delivery did not fit the host buffer: nothing was written")
        o, n = self.table[1 + 2 * s], self.table[2 + 2 * s]
        return ctypes.string_at(self.p.value + o, n)

    def close(self):
        if self.p:
            lib.scroll_host_free(self.p)
            lib.scroll_host_free(self.t)
            self.p = self.t = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def make_config(w, h, frame_num=2, log2_mfn=4, poc_type=2, log2_poc=4, deblock=1,
                waypoints=()):
    """ComposerConfig in the state composer_init + composer_write_header leave it
    (reference src/composer.c:199-203: frame_num 2 after the two I frames)."""
    c = ComposerConfig()
    lib.composer_config_init(ctypes.byref(c), w, h)
    lib.composer_config_set_sps_params(ctypes.byref(c), log2_mfn, poc_type, log2_poc)
    lib.composer_config_set_pps_params(ctypes.byref(c), 1, deblock)
    c.frame_num = frame_num
    for i, (off, lt, valid) in enumerate(waypoints):
        c.waypoints[i].offset_px, c.waypoints[i].long_term_idx, c.waypoints[i].valid = off, lt, valid
    c.num_waypoints = len(waypoints)
    return c


class Batch:
    """Many-stream batch on one GPU (include/composer_batch.h)."""

    def __init__(self, max_streams, max_frames, arena_bytes, device=0,
                 mode=SCROLL_MODE_COMPOSER):
        d = ScrollBatchDesc(device, max_streams, max_frames, arena_bytes, mode)
        h = ctypes.c_void_p()
        rc = lib.scroll_batch_create(ctypes.byref(h), ctypes.byref(d))
        if rc != SCROLL_OK:
            raise RuntimeError(f"scroll_batch_create failed ({rc}): {last_error()}")
        self.h = h
        self.max_frames = max_frames

    def close(self):
        if self.h:
            lib.scroll_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc < 0:
            raise RuntimeError(f"{what} failed ({rc}): {last_error()}")
        return rc

    def add_stream(self, cfg):
        return self._chk(lib.scroll_batch_add_stream(self.h, ctypes.byref(cfg)), "add_stream")

    @property
    def num_streams(self):
        return lib.scroll_batch_num_streams(self.h)

    def set_debug(self, flags):
        self._chk(lib.scroll_batch_set_debug(self.h, flags), "set_debug")

    def set_offsets(self, offsets):
        """offsets: numpy int32 array [num_streams, nframes]"""
        import numpy as np
        a = np.ascontiguousarray(offsets, dtype=np.int32)
        self._chk(lib.scroll_batch_set_offsets(
            self.h, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), a.shape[1]), "set_offsets")

    def offsets_device_ptr(self):
        return lib.scroll_batch_offsets_device(self.h)

    def compose(self, nframes, stream=None, rewind=False):
        self._chk(lib.scroll_batch_compose_ex(self.h, nframes, stream,
                                              SCROLL_COMPOSE_REWIND if rewind else 0), "compose")

    def sync(self):
        return lib.scroll_batch_sync(self.h)

    def config(self, s):
        c = ComposerConfig()
        self._chk(lib.scroll_batch_get_config(self.h, s, ctypes.byref(c)), "get_config")
        return c

    def set_config(self, s, cfg):
        self._chk(lib.scroll_batch_set_config(self.h, s, ctypes.byref(cfg)), "set_config")

    def output_size(self, s):
        return lib.scroll_batch_output_size(self.h, s)

    def output(self, s, start=0, n=None):
        if n is None:
            n = self.output_size(s) - start
        b = u8buf(max(n, 1))
        self._chk(lib.scroll_batch_copy_output(self.h, s, start, b, n), "copy_output")
        return bytes(b[:n])

    def output_to_host_async(self, hb, stream=None):
        """the bytes the last compose appended to every stream -> HostBuffer
        hb (packed, device-written, asynchronous: valid after sync())"""
        self._chk(lib.scroll_batch_output_to_host_async(self.h, hb.p, hb.cap, hb.t, stream),
                  "output_to_host_async")

    def output_device_ptr(self, s):
        """device address of stream s's arena (scroll_batch_output_device)"""
        return lib.scroll_batch_output_device(self.h, s)

    def reset_output(self):
        self._chk(lib.scroll_batch_reset_output(self.h), "reset_output")

    def nals(self, s):
        n = self._chk(lib.scroll_batch_nal_count(self.h, s), "nal_count")
        out = []
        k, o, sl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        sz = ctypes.c_uint32()
        for i in range(n):
            self._chk(lib.scroll_batch_nal_info(self.h, s, i, ctypes.byref(k), ctypes.byref(o),
                                                ctypes.byref(sz), ctypes.byref(sl)), "nal_info")
            out.append((k.value, o.value, sz.value, sl.value))
        return out

    def enable_timing(self, on=True, lite=False):
        """HIP-event timing of the composes that follow: every kernel pair, or
        (lite) only the dominant kernel's -- dyn code or emit -- with fewer
        event markers between the kernels (scroll_batch_enable_timing)."""
        self._chk(lib.scroll_batch_enable_timing(self.h, (2 if lite else 1) if on else 0), "enable_timing")

    def kernel_ms(self, which):
        return lib.scroll_batch_kernel_ms(self.h, which)

    def kernel_stats(self):
        """(plan ms, emit ms, composes) summed since the last call"""
        a, e, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        self._chk(lib.scroll_batch_kernel_stats(self.h, ctypes.byref(a), ctypes.byref(e),
                                                ctypes.byref(n)), "kernel_stats")
        return a.value, e.value, n.value

    def kernel_stats_ex(self):
        """(plan, emit, dyn stage, dyn emit, dyn code, dyn pack) ms summed since
        the last call, composes"""
        ms, n = (ctypes.c_double * 6)(), ctypes.c_int()
        self._chk(lib.scroll_batch_kernel_stats_ex(self.h, ms, ctypes.byref(n)), "kernel_stats_ex")
        return tuple(ms), n.value

    # ---- stream ingest ----
    def ingest(self, refs):
        """refs: [(ref_a_bytes, ref_b_bytes), ...] -> id of the first new stream
        (batched composer_init + composer_write_header on the GPU)"""
        n = len(refs)
        bufs = [(u8buf(bytes(a) or b"\0"), u8buf(bytes(b) or b"\0")) for a, b in refs]
        u8p = ctypes.POINTER(ctypes.c_uint8)
        pa = (u8p * max(n, 1))(*[ctypes.cast(x[0], u8p) for x in bufs])
        pb = (u8p * max(n, 1))(*[ctypes.cast(x[1], u8p) for x in bufs])
        na = (ctypes.c_size_t * max(n, 1))(*[len(a) for a, _ in refs])
        nb = (ctypes.c_size_t * max(n, 1))(*[len(b) for _, b in refs])
        first = ctypes.c_int()
        self._chk(lib.scroll_batch_ingest(self.h, n, pa, na, pb, nb, ctypes.byref(first)), "ingest")
        return first.value

    def ingest_device(self, n, d_files, desc):
        """files already on the device: desc = 4 n uint64 (offset, size of A, of B)"""
        arr = (ctypes.c_uint64 * max(1, len(desc)))(*desc)
        first = ctypes.c_int()
        self._chk(lib.scroll_batch_ingest_device(self.h, n, ctypes.c_void_p(d_files), arr,
                                                 ctypes.byref(first)), "ingest_device")
        return first.value

    def update_refs(self, streams, which, files, check=True):
        """mid-stream long-term reference updates: files[k] (Annex-B bytes with
        an IDR) -> a non-IDR I frame of stream streams[k] marked which[k]
        (0 = A, 1 = B); -> (rc, statuses)"""
        n = len(streams)
        st = (ctypes.c_int * n)(*streams)
        wh = (ctypes.c_int * n)(*which)
        bufs = [u8buf(f) for f in files]
        fp = (ctypes.POINTER(ctypes.c_uint8) * n)(*[ctypes.cast(x, ctypes.POINTER(ctypes.c_uint8)) for x in bufs])
        sz = (ctypes.c_size_t * n)(*[len(f) for f in files])
        stat = (ctypes.c_int * n)()
        rc = lib.scroll_batch_update_refs(self.h, n, st, wh, fp, sz, stat)
        if check:
            self._chk(rc, "update_refs")
        return rc, list(stat)

    def ingest_stats(self):
        ms, n = ctypes.c_double(), ctypes.c_int()
        self._chk(lib.scroll_batch_ingest_stats(self.h, ctypes.byref(ms), ctypes.byref(n)),
                  "ingest_stats")
        return ms.value, n.value

    # ---- reference files from pictures ----
    def ipcm_files_device(self, n, w, h, d_pics, pic_stride, d_out, out_stride):
        """n I420 pictures (device) -> n SPS+PPS+I_PCM IDR files (device);
        returns the file sizes"""
        sizes = (ctypes.c_uint64 * max(1, n))()
        self._chk(lib.scroll_batch_ipcm_files_device(self.h, n, w, h, ctypes.c_void_p(d_pics),
                                                     pic_stride, ctypes.c_void_p(d_out),
                                                     out_stride, sizes), "ipcm_files_device")
        return [int(sizes[i]) for i in range(n)]

    def ipcm_files_device_async(self, n, w, h, d_pics, pic_stride, d_out, out_stride, d_sizes):
        """the same, sizes to d_sizes (device, n u64), no host step: an
        overflow surfaces at the next sync()"""
        self._chk(lib.scroll_batch_ipcm_files_device_async(self.h, n, w, h, ctypes.c_void_p(d_pics), pic_stride,
                                                           ctypes.c_void_p(d_out), out_stride,
                                                           ctypes.c_void_p(d_sizes)), "ipcm_files_device_async")

    def ipcm_stats(self):
        ms, n = ctypes.c_double(), ctypes.c_int()
        self._chk(lib.scroll_batch_ipcm_stats(self.h, ctypes.byref(ms), ctypes.byref(n)),
                  "ipcm_stats")
        return ms.value, n.value

    # ---- UI hints ----
    def set_hints(self, s, f, rects, mode=SCROLL_HINT_EXACT):
        """rects: [(x0, y0, x1, y1, ref, mv_x, mv_y), ...] for frame f of stream s"""
        arr = (ScrollHintRect * max(1, len(rects)))()
        for i, (x0, y0, x1, y1, ref, mx, my) in enumerate(rects):
            arr[i] = ScrollHintRect(x0, y0, x1, y1, ref, 0, mx, my)
        self._chk(lib.scroll_batch_set_hints(self.h, s, f, arr, len(rects), mode), "set_hints")

    def clear_hints(self):
        self._chk(lib.scroll_batch_clear_hints(self.h), "clear_hints")

    # ---- pre-encoded MB splice ----
    def set_splice(self, s, f, x0, y0, w, h, nal):
        """the external P slice `nal` (bytes) into MB rect (x0, y0, w, h) of
        frame f of stream s; nal = b"" removes it"""
        nal = bytes(nal)
        self._chk(lib.scroll_batch_set_splice(self.h, s, f, x0, y0, w, h, nal, len(nal)),
                  "set_splice")

    def set_splices_device(self, entries):
        """entries: [(s, f, x0, y0, w, h, device_ptr, nbytes), ...]"""
        arr = (ScrollSpliceDesc * max(1, len(entries)))()
        for i, e in enumerate(entries):
            arr[i] = ScrollSpliceDesc(*e)
        self._chk(lib.scroll_batch_set_splices_device(self.h, len(entries), arr),
                  "set_splices_device")

    def clear_splices(self):
        self._chk(lib.scroll_batch_clear_splices(self.h), "clear_splices")

    def splice_status(self, s, f):
        st = ctypes.c_int()
        self._chk(lib.scroll_batch_splice_status(self.h, s, f, ctypes.byref(st)), "splice_status")
        return st.value

    def splice_refusal(self, s, f):
        """(status, mb_x, mb_y, mb_type): for SCROLL_SPLICE_ERR_MBTYPE the
        refused MB of the external picture and its P-slice mb_type"""
        v = [ctypes.c_int() for _ in range(4)]
        self._chk(lib.scroll_batch_splice_refusal(self.h, s, f, *[ctypes.byref(x) for x in v]),
                  "splice_refusal")
        return tuple(x.value for x in v)

    # ---- dynamic rect (configs 3-5) ----
    def set_dyn_rect(self, x0, y0, w, h, slot_bytes=0):
        self._chk(lib.scroll_batch_set_dyn_rect(self.h, x0, y0, w, h, slot_bytes), "set_dyn_rect")

    def set_dyn_qp(self, qp, stream=None):
        """the dynamic rect's QP (0..51) of every stream, or of one: its
        scroll NALs carry slice_qp_delta qp - 26 (scroll_batch_set_dyn_qp /
        _stream)"""
        if stream is None:
            self._chk(lib.scroll_batch_set_dyn_qp(self.h, qp), "set_dyn_qp")
        else:
            self._chk(lib.scroll_batch_set_dyn_qp_stream(self.h, stream, qp), "set_dyn_qp_stream")

    def set_dyn_qp_at(self, s, f, qp):
        """under UI hints: frame f of stream s at QP qp (-1: the stream's)"""
        self._chk(lib.scroll_batch_set_dyn_qp_at(self.h, s, f, qp), "set_dyn_qp_at")

    def set_dyn_refs(self, ref_a, ref_b, stream=-1):
        """ref_a / ref_b: I420 bytes (w*h*3/2) of reference pictures A and B"""
        self._chk(lib.scroll_batch_set_dyn_refs(self.h, stream, u8buf(bytes(ref_a)),
                                                u8buf(bytes(ref_b))), "set_dyn_refs")

    def set_dyn_rect_at(self, s, f, x0, y0):
        """Frame f of stream s puts the dynamic rect at MB (x0, y0); x0 = -1:
        no rect in that frame.  Positions other than set_dyn_rect's need UI
        hints (set_hints) at compose time."""
        self._chk(lib.scroll_batch_set_dyn_rect_at(self.h, s, f, x0, y0), "set_dyn_rect_at")

    def set_fallback(self, on=True):
        """the conventional-encode fallback (scroll_batch_set_fallback): frames
        whose hints name a reference they lack are coded as whole P frames"""
        self._chk(lib.scroll_batch_set_fallback(self.h, 1 if on else 0), "set_fallback")

    def fallback_frame(self, s, f):
        """1 when frame f of stream s fell back in the last compose"""
        v = ctypes.c_int()
        self._chk(lib.scroll_batch_fallback_frame(self.h, s, f, ctypes.byref(v)), "fallback_frame")
        return v.value

    def set_dyn_source(self, src, nframes):
        """src: bytes of [num_streams][nframes][384*w*h]"""
        self._chk(lib.scroll_batch_set_dyn_source(self.h, u8buf(bytes(src)), nframes),
                  "set_dyn_source")

    def dyn_source_device(self):
        ls, lf = ctypes.c_size_t(), ctypes.c_size_t()
        p = lib.scroll_batch_dyn_source_device(self.h, ctypes.byref(ls), ctypes.byref(lf))
        return p, ls.value, lf.value

    def dyn_source_synth(self, nframes, stream_base=0, t0=0):
        self._chk(lib.scroll_batch_dyn_source_synth(self.h, nframes, stream_base, t0),
                  "dyn_source_synth")

    def dyn_frame_info(self, s, f):
        """(rbsp bytes, EP bytes) of frame f's dynamic NAL, None if it has none"""
        r, e = ctypes.c_uint32(), ctypes.c_uint32()
        rc = self._chk(lib.scroll_batch_dyn_frame_info(self.h, s, f, ctypes.byref(r),
                                                       ctypes.byref(e)), "dyn_frame_info")
        return None if rc == 1 else (r.value, e.value)

    def dyn_totals(self):
        """last compose: (staged RBSP bytes, EP bytes, dynamic NALs) over all streams"""
        r, e, n = ctypes.c_ulonglong(), ctypes.c_ulonglong(), ctypes.c_longlong()
        self._chk(lib.scroll_batch_dyn_totals(self.h, ctypes.byref(r), ctypes.byref(e),
                                              ctypes.byref(n)), "dyn_totals")
        return r.value, e.value, n.value

    def last_bytes(self):
        return lib.scroll_batch_last_bytes(self.h)

    def last_nals(self):
        return lib.scroll_batch_last_nals(self.h)


def header_symbols():
    """Every function declared in include/*.h (the C-ABI contract)."""
    import re
    inc = os.path.join(os.path.dirname(HERE), "include")
    names = []
    for fn in sorted(os.listdir(inc)):
        if not fn.endswith(".h"):
            continue
        txt = open(os.path.join(inc, fn)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b([a-z_][a-z0-9_]*)\s*\(", txt, flags=re.M):
            if m.group(1) not in ("if", "while", "for", "sizeof", "return"):
                names.append(m.group(1))
    return sorted(set(names))
