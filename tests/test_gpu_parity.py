"""GPU parity: the HIP path (through the C ABI) vs the reference's golden
vectors and vs the CPU oracle, byte for byte.  Run on an MI355X: -m gpu."""
import ctypes
import hashlib
import random

import numpy as np
import pytest

from conftest import golden_file, synthetic_offsets

pytestmark = pytest.mark.gpu

BUF = 64 << 20


@pytest.fixture(scope="module")
def gpu(scroll):
    if scroll.device_count() < 1:
        pytest.fail("no gfx950 device: " + scroll.last_error())
    return scroll


def _cfg_from_case(s, c):
    cfg = s.make_config(c["w"], c["h"], frame_num=c["frame_num"], log2_mfn=c["log2_mfn"],
                        poc_type=c["poc_type"], log2_poc=c["log2_poc"], deblock=c["deblock"])
    for i, (o, lt, v) in enumerate(c["wp"]):
        cfg.waypoints[i].offset_px, cfg.waypoints[i].long_term_idx, cfg.waypoints[i].valid = o, lt, v
    cfg.num_waypoints = c["nwp"]
    return cfg


def test_single_frame_api_vs_reference(gpu, golden_frames):
    """h264_write_scroll_p_frame / h264_write_waypoint_p_frame (drop-in, GPU)
    on arbitrary ComposerConfigs, including emulation-prevention cases."""
    lib = gpu.lib
    out, rb = gpu.u8buf(BUF), gpu.u8buf(1 << 20)
    for c in golden_frames:
        cfg = _cfg_from_case(gpu, c)
        nw = gpu.NALWriter()
        lib.nal_writer_init(ctypes.byref(nw), out, BUF, rb, 1 << 20)
        if c["kind"] == 0:
            n = lib.h264_write_scroll_p_frame(ctypes.byref(nw), ctypes.byref(cfg), c["off"])
        elif c["kind"] == 1:
            n = lib.h264_write_waypoint_p_frame(ctypes.byref(nw), ctypes.byref(cfg), c["off"])
        else:
            n = 0
            if lib.h264_needs_waypoint(ctypes.byref(cfg), c["off"]):
                n += lib.h264_write_waypoint_p_frame(ctypes.byref(nw), ctypes.byref(cfg), c["off"])
            n += lib.h264_write_scroll_p_frame(ctypes.byref(nw), ctypes.byref(cfg), c["off"])
        got = bytes(out[:nw.output_pos])
        assert n == nw.output_pos == c["bytes"], c
        assert hashlib.sha256(got).hexdigest() == c["sha256"], {k: c[k] for k in c if k != "hex"}
        assert cfg.frame_num == c["frame_num_after"] and cfg.num_waypoints == c["nwp_after"]


def _run_batch(gpu, w, h, offsets, chunks=None, debug=0, mode=0, frame_num=2, arena=None):
    S, F = offsets.shape
    per_frame = 2 * (64 + (w // 16) * (h // 16) * 2)
    b = gpu.Batch(S, F, arena or max(1 << 20, F * per_frame), mode=mode)
    for s in range(S):
        b.add_stream(gpu.make_config(w, h, frame_num=frame_num))
    if debug:
        b.set_debug(debug)
    done = 0
    nal_lists = [[] for _ in range(S)]
    for k in (chunks or [F]):
        b.set_offsets(offsets[:, done:done + k])
        b.compose(k)
        assert b.sync() == gpu.SCROLL_OK, gpu.last_error()
        for s in range(S):
            nal_lists[s].extend(b.nals(s))
        done += k
    assert done == F
    outs = [b.output(s) for s in range(S)]
    cfgs = [b.config(s) for s in range(S)]
    b.close()
    return outs, nal_lists, cfgs


def _frame_sizes(nals, nframes):
    # composer mode: a waypoint NAL belongs to the scroll NAL that follows it
    sizes, acc = [], 0
    for kind, off, size, slow in nals:
        acc += size
        if kind == 0:
            sizes.append(acc)
            acc = 0
    assert len(sizes) == nframes
    return sizes


@pytest.mark.parametrize("wh", [(1280, 720), (3840, 2160), (64, 48), (352, 288)])
def test_batch_synthetic_streams_vs_reference(gpu, golden_streams, wh):
    gs = [g for g in golden_streams if (g["w"], g["h"]) == wh]
    F = gs[0]["nframes"]
    sids = [g["stream"] for g in gs]
    offs = np.stack([synthetic_offsets(1, F, wh[1], first_stream=s)[0] for s in sids])
    chunks = [1, 63, 64, 65, F - 193] if F > 193 else None
    outs, nals, cfgs = _run_batch(gpu, wh[0], wh[1], offs, chunks=chunks)
    for g, out, nl in zip(gs, outs, nals):
        assert _frame_sizes(nl, F) == g["sizes"], (wh, g["stream"])
        assert hashlib.sha256(out).hexdigest() == g["sha256"], (wh, g["stream"])


def test_batch_forced_serial_path(gpu, golden_streams):
    gs = [g for g in golden_streams if (g["w"], g["h"]) == (352, 288)][:4]
    F = gs[0]["nframes"]
    offs = np.stack([synthetic_offsets(1, F, 288, first_stream=g["stream"])[0] for g in gs])
    outs, nals, _ = _run_batch(gpu, 352, 288, offs, debug=gpu.SCROLL_DEBUG_FORCE_SERIAL)
    for g, out, nl in zip(gs, outs, nals):
        assert all(n[3] == 1 for n in nl)
        assert hashlib.sha256(out).hexdigest() == g["sha256"]


class OrCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("w", "h", "log2_mfn", "poc_type", "log2_poc", "num_ref_default_m1", "deblock",
                 "frame_num", "idr_pic_id", "nwp")] + [
        ("wp_off", ctypes.c_int * 8), ("wp_lt", ctypes.c_int * 8), ("wp_valid", ctypes.c_int * 8)]


def _oracle_stream(oracle, w, h, offsets, mode=0, frame_num=2):
    cfg = OrCfg()
    oracle.or_cfg_init(ctypes.byref(cfg), w, h)
    cfg.frame_num = frame_num
    buf = (ctypes.c_uint8 * (4 << 20))()
    out = bytearray()
    for off in offsets:
        n = oracle.or_compose(buf, len(buf), ctypes.byref(cfg), int(off), mode, None)
        out += bytes(buf[:n])
    return bytes(out), cfg


@pytest.mark.parametrize("mode", [0, 1])
def test_batch_random_offsets_vs_oracle(gpu, oracle, mode):
    """Waypoint-heavy random offset sequences (incl. the 8-waypoint cap, negative
    and out-of-frame offsets) through the GPU state machine, vs the oracle."""
    rng = random.Random(100 + mode)
    for trial in range(6):
        w, h = 16 * rng.randint(1, 40), 16 * rng.randint(1, 300)
        S, F = rng.randint(1, 9), rng.randint(1, 300)
        offs = np.zeros((S, F), dtype=np.int32)
        for s in range(S):
            for i in range(F):
                r = rng.random()
                if r < 0.3:
                    offs[s, i] = 496 * rng.randint(-2, 12)
                elif r < 0.9:
                    offs[s, i] = rng.randint(0, h)
                else:
                    offs[s, i] = rng.randint(-3 * h, 3 * h)
        outs, nals, cfgs = _run_batch(gpu, w, h, offs, mode=mode,
                                      chunks=[F // 2, F - F // 2] if F > 1 else None)
        for s in range(S):
            want, oc = _oracle_stream(oracle, w, h, offs[s], mode=mode)
            assert outs[s] == want, (trial, s, w, h)
            assert cfgs[s].frame_num == oc.frame_num and cfgs[s].num_waypoints == oc.nwp
            for k in range(oc.nwp):
                assert (cfgs[s].waypoints[k].offset_px, cfgs[s].waypoints[k].long_term_idx) == \
                    (oc.wp_off[k], oc.wp_lt[k])


def test_experiment_mode_config1(gpu, oracle, golden_md5):
    """BASELINE config 1 (run.sh): 1280x720, 248 frames, start 496, waypoint
    instead of scroll.  I-frame header from the I_PCM writer; P frames on GPU."""
    g = golden_md5["experiment_1280x720_n248_S1"]
    hb = (ctypes.c_uint8 * (4 << 20))()
    hn = oracle.or_experiment_run(hb, len(hb), 1280, 720, 0, 1)     # SPS+PPS+2 I_PCM frames
    m = 720 - 16
    x = np.arange(248) + 496
    p = x % (2 * m)
    offs = np.where(p < m, p, 2 * m - p).astype(np.int32)[None, :]
    outs, _, _ = _run_batch(gpu, 1280, 720, offs, mode=gpu.SCROLL_MODE_EXPERIMENT)
    full = bytes(hb[:hn]) + outs[0]
    assert len(full) == g["bytes"]
    assert hashlib.md5(full).hexdigest() == g["md5"] == "8fd7eb782eb679ebef95da7fb718c7a4"


def test_composer_dropin_end_to_end(gpu, tmp_path):
    """composer_init/header/write_scroll_frame/write_to_file == reference CLI bytes."""
    pa, pb = tmp_path / "a.h264", tmp_path / "b.h264"
    pa.write_bytes(golden_file("ipcm_64x48_a.h264"))
    pb.write_bytes(golden_file("ipcm_64x48_b.h264"))
    lib = gpu.lib
    c = gpu.Composer()
    assert lib.composer_init(ctypes.byref(c), str(pa).encode(), str(pb).encode()) == 0
    lib.composer_write_header(ctypes.byref(c))
    for i in range(40):
        p = i % 96
        lib.composer_write_scroll_frame(ctypes.byref(c), p if p < 48 else 96 - p)
    out = tmp_path / "o.h264"
    assert lib.composer_write_to_file(ctypes.byref(c), str(out).encode()) == 0
    got, want = out.read_bytes(), golden_file("composer_64x48_n40_s1.h264")
    assert c.frames_written == 40, (c.frames_written, len(got), len(want), gpu.last_error())
    assert got == want, (len(got), len(want), gpu.last_error())
    lib.composer_finish(ctypes.byref(c))


def test_composer_dropin_720p_md5(gpu, oracle, golden_md5, tmp_path):
    g = golden_md5["composer_1280x720_n360_s4"]
    refs = []
    for which in (0, 1):
        b = (ctypes.c_uint8 * (2 << 20))()
        n = oracle.or_ipcm_ref_file(b, len(b), 1280, 720, which)
        p = tmp_path / f"r{which}.h264"
        p.write_bytes(bytes(b[:n]))
        refs.append(str(p).encode())
    lib = gpu.lib
    c = gpu.Composer()
    assert lib.composer_init(ctypes.byref(c), refs[0], refs[1]) == 0
    lib.composer_write_header(ctypes.byref(c))
    for i in range(360):
        p = (i * 4) % 1440
        lib.composer_write_scroll_frame(ctypes.byref(c), p if p < 720 else 1440 - p)
    n = lib.composer_get_output_size(ctypes.byref(c))
    data = bytes(lib.composer_get_output(ctypes.byref(c))[:n])
    assert n == g["bytes"] and hashlib.md5(data).hexdigest() == g["md5"]
    lib.composer_finish(ctypes.byref(c))


def test_composer_level_batch(gpu, golden_streams, tmp_path):
    """composer_batch_write_scroll_frames over several Composers at once."""
    gs = [g for g in golden_streams if (g["w"], g["h"]) == (64, 48)][:4]
    pa, pb = tmp_path / "a.h264", tmp_path / "b.h264"
    pa.write_bytes(golden_file("ipcm_64x48_a.h264"))
    pb.write_bytes(golden_file("ipcm_64x48_b.h264"))
    lib = gpu.lib
    cs = [gpu.Composer() for _ in gs]
    for c in cs:
        assert lib.composer_init(ctypes.byref(c), str(pa).encode(), str(pb).encode()) == 0
        lib.composer_write_header(ctypes.byref(c))
    hdr = lib.composer_get_output_size(ctypes.byref(cs[0]))
    F = gs[0]["nframes"]
    offs = np.stack([synthetic_offsets(1, F, 48, first_stream=g["stream"])[0] for g in gs])
    ptrs = (ctypes.POINTER(gpu.Composer) * (len(gs) * F))()
    vals = (ctypes.c_int * (len(gs) * F))()
    k = 0
    for i in range(F):                      # interleaved order, per-Composer order kept
        for s in range(len(gs)):
            ptrs[k] = ctypes.pointer(cs[s])
            vals[k] = int(offs[s, i])
            k += 1
    assert lib.composer_batch_write_scroll_frames(ptrs, vals, k, 0) == 0
    for g, c in zip(gs, cs):
        n = lib.composer_get_output_size(ctypes.byref(c))
        data = bytes(lib.composer_get_output(ctypes.byref(c))[:n])
        assert hashlib.sha256(data[hdr:]).hexdigest() == g["sha256"]
        lib.composer_finish(ctypes.byref(c))


def test_overflow_is_reported_and_not_committed(gpu):
    offs = synthetic_offsets(2, 50, 720)
    b = gpu.Batch(2, 50, 64 << 10)               # 64 KB arena: ~20 frames fit
    for _ in range(2):
        b.add_stream(gpu.make_config(1280, 720))
    b.set_offsets(offs)
    b.compose(50)
    assert b.sync() == gpu.SCROLL_ERR_OVERFLOW
    assert b.output_size(0) == 0 and b.config(0).frame_num == 2
    b.set_offsets(offs[:, :10])
    b.compose(10)
    assert b.sync() == gpu.SCROLL_OK and b.output_size(0) > 0
    b.close()


def test_state_checkpoint_resume(gpu, oracle):
    """get_config/set_config move a stream between batches mid-sequence."""
    offs = synthetic_offsets(1, 400, 2160, first_stream=3)
    b1 = gpu.Batch(1, 400, 32 << 20)
    b1.add_stream(gpu.make_config(3840, 2160))
    b1.set_offsets(offs[:, :250])
    b1.compose(250)
    assert b1.sync() == 0
    part1 = b1.output(0)
    cfg = b1.config(0)
    b1.close()
    b2 = gpu.Batch(1, 400, 32 << 20)
    b2.add_stream(cfg)
    b2.set_offsets(offs[:, 250:])
    b2.compose(150)
    assert b2.sync() == 0
    want, _ = _oracle_stream(oracle, 3840, 2160, offs[0])
    assert part1 + b2.output(0) == want
    b2.close()
