"""GPU reference-file writer: scroll_batch_ipcm_files_device
turns I420 pictures in HBM into SPS + PPS + I_PCM IDR files, byte for byte
what the CPU restatement or_ipcm_picture_file writes (oracle/scroll_oracle.c;
pinned to the reference's striped I_PCM files by tests/test_oracle_golden.py).
Pictures vary what the kernels must handle: the reference's stripes, random
samples, all-zero pictures (an emulation-prevention byte every third RBSP
byte of each MB, zero runs longer than a workgroup's look-back), samples
0..3 only, chunk edges at every size.  The files then feed
scroll_batch_ingest_device and the composed streams are checked against the
reference composer's restatement.  Run on an MI355X: -m gpu."""
import ctypes
import hashlib

import numpy as np
import pytest

from dynhelp import ipcm_file, striped_i420

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(scroll):
    if scroll.device_count() < 1:
        pytest.fail("no gfx950 device: " + scroll.last_error())
    return scroll


class Hip:
    """Device buffers through the HIP runtime libh264scroll itself links (so
    the process holds one runtime, not torch's bundled one beside it)."""

    def __init__(self):
        self.lib = ctypes.CDLL("libamdhip64.so.7")
        L = self.lib
        L.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        L.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
        L.hipFree.argtypes = [ctypes.c_void_p]
        for f in (L.hipMalloc, L.hipMemcpy, L.hipMemset, L.hipFree, L.hipDeviceSynchronize):
            f.restype = ctypes.c_int

    def buf(self, n, fill=0):
        return DevBuf(self, n, fill)


class DevBuf:
    def __init__(self, hip, n, fill):
        self.hip, self.n, p = hip, n, ctypes.c_void_p()
        assert hip.lib.hipMalloc(ctypes.byref(p), n) == 0
        self.p = p.value
        assert hip.lib.hipMemset(self.p, fill, n) == 0

    def write(self, off, data):
        data = bytes(data)
        assert self.hip.lib.hipMemcpy(self.p + off, data, len(data), 1) == 0      # host -> device

    def read(self):
        host = np.empty(self.n, np.uint8)
        assert self.hip.lib.hipMemcpy(host.ctypes.data, self.p, self.n, 2) == 0  # device -> host
        return host

    def free(self):
        if self.p:
            self.hip.lib.hipFree(self.p)
            self.p = None


@pytest.fixture(scope="module")
def hip(gpu):
    return Hip()


def pictures(w, h, kinds, seed=7):
    rng = np.random.default_rng(seed)
    n = w * h * 3 // 2
    out = []
    for k in kinds:
        if k == "a" or k == "b":
            out.append(striped_i420(w, h, "ab".index(k)))
        elif k == "rand":
            out.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        elif k == "zero":
            out.append(bytes(n))
        elif k == "low":
            out.append(rng.integers(0, 4, n, dtype=np.uint8).tobytes())
        elif k == "sparse":              # mostly zero with isolated small values
            p = np.zeros(n, np.uint8)
            idx = rng.integers(0, n, n // 50)
            p[idx] = rng.integers(1, 4, idx.size, dtype=np.uint8)
            out.append(p.tobytes())
        else:
            raise ValueError(k)
    return out


def gpu_files(gpu, hip, w, h, pics, out_stride=None, b=None):
    n = len(pics)
    psz = w * h * 3 // 2
    stride = (psz + 255) // 256 * 256
    dev = hip.buf(n * stride)
    if out_stride is None:
        out_stride = (psz * 3 // 2 + psz + 4096 + 255) // 256 * 256
    out = hip.buf(n * out_stride, 0xAB)
    own = b is None
    if own:
        b = gpu.Batch(1, 1, 1 << 20, device=0)
    try:
        for i, p in enumerate(pics):
            dev.write(i * stride, p)
        sizes = b.ipcm_files_device(n, w, h, dev.p, stride, out.p, out_stride)
        assert hip.lib.hipDeviceSynchronize() == 0
        host = out.read()
        files = [host[i * out_stride:i * out_stride + sizes[i]].tobytes() for i in range(n)]
        tails = [host[i * out_stride + sizes[i]:(i + 1) * out_stride] for i in range(n)]
    finally:
        if own:
            b.close()
        dev.free()
        out.free()
    return files, tails


@pytest.mark.parametrize("w,h", [(64, 48), (1280, 720)])
def test_striped_refs_match_reference(gpu, hip, oracle, golden_md5, w, h):
    files, _ = gpu_files(gpu, hip, w, h, pictures(w, h, ["a", "b"]))
    for which, f in enumerate(files):
        g = golden_md5[f"ipcm_{w}x{h}_{'ab'[which]}.h264"]
        assert len(f) == g["bytes"] and hashlib.md5(f).hexdigest() == g["md5"]


@pytest.mark.parametrize("w,h", [(16, 16), (48, 32), (176, 144), (640, 480), (1280, 720)])
def test_pictures_match_oracle(gpu, hip, oracle, w, h):
    kinds = ["rand", "zero", "low", "sparse", "a"]
    pics = pictures(w, h, kinds, seed=w + h)
    files, tails = gpu_files(gpu, hip, w, h, pics)
    for k, (p, f, t) in enumerate(zip(pics, files, tails)):
        want = ipcm_file(oracle, w, h, p)
        assert f == want, f"{kinds[k]} {w}x{h}: {len(f)} vs {len(want)} bytes"
        assert (t == 0xAB).all(), "bytes written past the file"


@pytest.mark.parametrize("w,h", [(48, 32), (640, 480)])
def test_generating_write_pass_matches(gpu, hip, oracle, monkeypatch, w, h):
    """SCROLL_IPCM_RECOMPUTE: the write pass generates the RBSP again instead
    of reading the count pass's bytes; same files"""
    kinds = ["rand", "zero", "low", "sparse", "a"]
    pics = pictures(w, h, kinds, seed=3 * w + h)
    monkeypatch.setenv("SCROLL_IPCM_RECOMPUTE", "1")
    files, tails = gpu_files(gpu, hip, w, h, pics)
    for k, (p, f, t) in enumerate(zip(pics, files, tails)):
        assert f == ipcm_file(oracle, w, h, p), f"{kinds[k]} {w}x{h}"
        assert (t == 0xAB).all(), "bytes written past the file"


@pytest.mark.parametrize("w,h", [(16, 16), (176, 144), (1280, 720)])
def test_onepass_matches(gpu, hip, oracle, monkeypatch, w, h):
    """SCROLL_IPCM_ONEPASS (round 6, opt-in): count and write in one
    workgroup, the file offsets by a decoupled look-back over the chunks'
    hand-off words; same files, nothing past them -- twice on one batch, so
    the second call's words carry a new epoch over the first's"""
    kinds = ["rand", "zero", "low", "sparse", "a"]
    pics = pictures(w, h, kinds, seed=5 * w + h)
    monkeypatch.setenv("SCROLL_IPCM_ONEPASS", "1")
    b = gpu.Batch(1, 1, 1 << 20, device=0)
    try:
        for rep in range(2):
            files, tails = gpu_files(gpu, hip, w, h, pics[rep:] + pics[:rep], b=b)
            for k, (p, f, t) in enumerate(zip(pics[rep:] + pics[:rep], files, tails)):
                assert f == ipcm_file(oracle, w, h, p), f"{k} {w}x{h} call {rep}"
                assert (t == 0xAB).all(), "bytes written past the file"
    finally:
        b.close()


def test_4k_pictures(gpu, hip, oracle, golden_md5):
    w, h = 3840, 2160
    pics = pictures(w, h, ["a", "zero"])
    files, _ = gpu_files(gpu, hip, w, h, pics)
    g = golden_md5["ipcm_3840x2160_a.h264"]
    assert len(files[0]) == g["bytes"] and hashlib.md5(files[0]).hexdigest() == g["md5"]
    assert files[1] == ipcm_file(oracle, w, h, pics[1])


def test_overflow_reports_sizes(gpu, hip, oracle):
    w, h = 64, 48
    pics = pictures(w, h, ["zero"])
    want = ipcm_file(oracle, w, h, pics[0])
    b = gpu.Batch(1, 1, 1 << 20, device=0)
    try:
        with pytest.raises(RuntimeError):
            gpu_files(gpu, hip, w, h, pics, out_stride=len(want) - 1, b=b)
        files, _ = gpu_files(gpu, hip, w, h, pics, out_stride=len(want), b=b)
        assert files[0] == want
    finally:
        b.close()


def test_files_feed_ingest_and_compose(gpu, hip, oracle):
    """pixels -> reference files -> new streams -> scroll frames without
    leaving the GPU (scroll_batch_ingest_device on the files in place);
    equal to the reference composer's restatement run on the oracle's files"""
    w, h, nfr, speed = 176, 144, 30, 4
    pics = pictures(w, h, ["rand", "sparse", "a", "b"], seed=3)
    psz = w * h * 3 // 2
    stride = (psz + 255) // 256 * 256
    dev = hip.buf(4 * stride)
    for i, p in enumerate(pics):
        dev.write(i * stride, p)
    ostride = 2 * stride + 4096
    out = hip.buf(4 * ostride)
    b = gpu.Batch(2, nfr, 4 << 20, device=0)
    try:
        sizes = b.ipcm_files_device(4, w, h, dev.p, stride, out.p, ostride)
        desc = []
        for k in range(2):
            desc += [2 * k * ostride, sizes[2 * k], (2 * k + 1) * ostride, sizes[2 * k + 1]]
        assert b.ingest_device(2, out.p, desc) == 0
        offs = np.array([[oracle.or_tri(i * speed, h) for i in range(nfr)] for _ in range(2)], np.int32)
        b.set_offsets(offs)
        b.compose(nfr)
        assert b.sync() == 0, gpu.last_error()
        for k in range(2):
            a_, b_ = ipcm_file(oracle, w, h, pics[2 * k]), ipcm_file(oracle, w, h, pics[2 * k + 1])
            cap = 2 * (len(a_) + len(b_)) + 65536
            buf = (ctypes.c_uint8 * cap)()
            n = oracle.or_composer_run(buf, cap, a_, len(a_), b_, len(b_), nfr, speed)
            assert n and b.output(k) == bytes(buf[:n])
    finally:
        b.close()
        dev.free()
        out.free()


def test_async_entry_matches_and_reports_overflow_at_sync(gpu, hip, oracle, scroll):
    """scroll_batch_ipcm_files_device_async: sizes to a device array, no host
    step per call; back-to-back calls give the oracle's files, and a call
    past out_stride surfaces at the next sync as SCROLL_ERR_OVERFLOW (that
    call writes no file), the following calls unaffected once synced"""
    w, h = 176, 144
    pics = pictures(w, h, ["rand", "zero", "sparse", "a"], seed=11)
    n, psz = len(pics), w * h * 3 // 2
    stride = (psz + 255) // 256 * 256
    want = [ipcm_file(oracle, w, h, p) for p in pics]
    ostride = (max(len(f) for f in want) + 255) // 256 * 256
    dev, out, dsz = hip.buf(n * stride), hip.buf(n * ostride, 0xAB), hip.buf(8 * n)
    b = gpu.Batch(1, 1, 1 << 20, device=0)
    try:
        for i, p in enumerate(pics):
            dev.write(i * stride, p)
        for _ in range(3):                               # stream-ordered reuse of the batch scratch
            b.ipcm_files_device_async(n, w, h, dev.p, stride, out.p, ostride, dsz.p)
        assert b.sync() == 0, gpu.last_error()
        sizes = np.frombuffer(dsz.read().tobytes(), np.uint64)
        host = out.read()
        for i in range(n):
            assert int(sizes[i]) == len(want[i])
            assert host[i * ostride:i * ostride + len(want[i])].tobytes() == want[i]
        small = min(len(f) for f in want) - 1              # every file over
        out2 = hip.buf(n * ostride, 0xAB)
        b.ipcm_files_device_async(n, w, h, dev.p, stride, out2.p, small, dsz.p)
        assert b.sync() == scroll.SCROLL_ERR_OVERFLOW
        assert "out_stride" in gpu.last_error()
        assert (out2.read() == 0xAB).all(), "an over-size call wrote bytes"
        out2.free()
        b.ipcm_files_device_async(n, w, h, dev.p, stride, out.p, ostride, dsz.p)
        assert b.sync() == 0, gpu.last_error()
    finally:
        b.close()
        dev.free()
        out.free()
        dsz.free()


def test_async_after_compose_on_caller_stream(gpu, hip, oracle):
    """a compose queued on the caller's (non-blocking) HIP stream, then the
    asynchronous I_PCM entry on the batch's own stream, then one sync: the
    sync covers the compose too (own waits for it), so every stream's output
    is the oracle's whole, and the files are the oracle's"""
    import random
    from test_gpu_parity import _oracle_stream
    L = hip.lib
    L.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    L.hipStreamCreateWithFlags.restype = ctypes.c_int
    L.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    cs = ctypes.c_void_p()
    assert L.hipStreamCreateWithFlags(ctypes.byref(cs), 1) == 0        # hipStreamNonBlocking
    w, h, S, F = 1280, 720, 64, 256
    rng = random.Random(5)
    offs = np.array([[rng.randint(0, h) for _ in range(F)] for _ in range(S)], np.int32)
    pw, ph = 176, 144
    pics = pictures(pw, ph, ["rand", "sparse"], seed=2)
    n, psz = len(pics), pw * ph * 3 // 2
    stride = (psz + 255) // 256 * 256
    want_f = [ipcm_file(oracle, pw, ph, p) for p in pics]
    ostride = (max(len(f) for f in want_f) + 255) // 256 * 256
    dev, out, dsz = hip.buf(n * stride), hip.buf(n * ostride, 0xAB), hip.buf(8 * n)
    b = gpu.Batch(S, F, 4 << 20, device=0)
    try:
        for i, p in enumerate(pics):
            dev.write(i * stride, p)
        for _ in range(S):
            b.add_stream(gpu.make_config(w, h))
        b.set_offsets(offs)
        b.compose(F, stream=cs.value)
        b.ipcm_files_device_async(n, pw, ph, dev.p, stride, out.p, ostride, dsz.p)
        assert b.sync() == 0, gpu.last_error()
        for s in range(S):
            assert b.output_size(s) == len(_oracle_stream(oracle, w, h, offs[s])[0]), s
        for s in (0, S // 2, S - 1):
            assert b.output(s) == _oracle_stream(oracle, w, h, offs[s])[0], s
        host = out.read()
        for i in range(n):
            assert host[i * ostride:i * ostride + len(want_f[i])].tobytes() == want_f[i]
    finally:
        b.close()
        dev.free()
        out.free()
        dsz.free()
        L.hipStreamDestroy(cs)
