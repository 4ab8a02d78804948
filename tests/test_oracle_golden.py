"""Pin the CPU oracle against the reference's own outputs (golden vectors made
by tests/golden/make_golden.py from the reference compiled in oracle/_ref)."""
import ctypes
import hashlib

import pytest

from conftest import golden_file

BUF = 80 << 20


@pytest.fixture(scope="module")
def buf():
    return (ctypes.c_uint8 * BUF)()


def _md5(b, n):
    return hashlib.md5(bytes(b[:n])).hexdigest()


@pytest.mark.parametrize("w,h", [(64, 48), (1280, 720), (3840, 2160)])
@pytest.mark.parametrize("which", [0, 1])
def test_ipcm_refs(oracle, buf, golden_md5, w, h, which):
    n = oracle.or_ipcm_ref_file(buf, BUF, w, h, which)
    g = golden_md5[f"ipcm_{w}x{h}_{'ab'[which]}.h264"]
    assert n == g["bytes"] and _md5(buf, n) == g["md5"]


def test_ipcm_small_files_bytes(oracle, buf):
    for which, name in ((0, "ipcm_64x48_a.h264"), (1, "ipcm_64x48_b.h264")):
        n = oracle.or_ipcm_ref_file(buf, BUF, 64, 48, which)
        assert bytes(buf[:n]) == golden_file(name)


def _refs(oracle, w, h):
    out = []
    for which in (0, 1):
        b = (ctypes.c_uint8 * (w * h * 2 + 4096))()
        n = oracle.or_ipcm_ref_file(b, len(b), w, h, which)
        out.append(bytes(b[:n]))
    return out


@pytest.mark.parametrize("name", ["composer_64x48_n40_s1", "composer_64x48_n200_s3",
                                  "composer_1280x720_n250_s4", "composer_1280x720_n360_s4",
                                  "composer_1280x720_n500_s3", "composer_3840x2160_n1200_s4"])
def test_composer_runs(oracle, buf, golden_md5, name):
    g = golden_md5[name]
    a, b = _refs(oracle, g["w"], g["h"])
    n = oracle.or_composer_run(buf, BUF, a, len(a), b, len(b), g["n"], g["s"])
    assert n == g["bytes"]
    assert _md5(buf, n) == g["md5"]
    if name == "composer_64x48_n40_s1":
        assert bytes(buf[:n]) == golden_file(name + ".h264")


@pytest.mark.parametrize("name", ["experiment_1280x720_n248_S1", "experiment_640x480_n900_S1",
                                  "experiment_1280x720_n900_S1", "experiment_3840x2160_n300_S8"])
def test_experiment_runs(oracle, buf, golden_md5, name):
    g = golden_md5[name]
    n = oracle.or_experiment_run(buf, BUF, g["w"], g["h"], g["n"], g["S"])
    assert n == g["bytes"] and _md5(buf, n) == g["md5"]


def test_config1_known_answer(golden_md5):
    # run.sh's config-1 output hash
    assert golden_md5["experiment_1280x720_n248_S1"]["md5"] == "8fd7eb782eb679ebef95da7fb718c7a4"


class OrCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("w", "h", "log2_mfn", "poc_type", "log2_poc", "num_ref_default_m1", "deblock",
                 "frame_num", "idr_pic_id", "nwp")] + [
        ("wp_off", ctypes.c_int * 8), ("wp_lt", ctypes.c_int * 8), ("wp_valid", ctypes.c_int * 8)]


def or_cfg_from_case(oracle, c):
    cfg = OrCfg()
    oracle.or_cfg_init(ctypes.byref(cfg), c["w"], c["h"])
    cfg.log2_mfn, cfg.poc_type, cfg.log2_poc = c["log2_mfn"], c["poc_type"], c["log2_poc"]
    cfg.deblock, cfg.frame_num, cfg.nwp = c["deblock"], c["frame_num"], c["nwp"]
    for i, (o, lt, v) in enumerate(c["wp"]):
        cfg.wp_off[i], cfg.wp_lt[i], cfg.wp_valid[i] = o, lt, v
    return cfg


def test_single_frame_cases(oracle, buf, golden_frames):
    """Arbitrary ComposerConfig x offset x kind vs the reference's h264_write_*."""
    for c in golden_frames:
        cfg = or_cfg_from_case(oracle, c)
        if c["kind"] == 0:
            n = oracle.or_scroll_nal(buf, BUF, ctypes.byref(cfg), c["off"])
        elif c["kind"] == 1:
            n = oracle.or_waypoint_nal(buf, BUF, ctypes.byref(cfg), c["off"])
        else:
            n = oracle.or_compose(buf, BUF, ctypes.byref(cfg), c["off"], 0, None)
        got = bytes(buf[:n])
        assert hashlib.sha256(got).hexdigest() == c["sha256"], c
        assert cfg.frame_num == c["frame_num_after"] and cfg.nwp == c["nwp_after"]
        if "hex" in c:
            assert got.hex() == c["hex"]


def test_emulation_prevention_cases_present(golden_frames):
    # the fixture set must exercise 0x03 insertion (huge MVs, long zero fields)
    assert sum(c["has_ep"] for c in golden_frames) >= 20


def test_synthetic_streams(oracle, buf, golden_streams):
    for g in golden_streams:
        if g["w"] == 3840 and g["stream"] not in (0, 7):
            continue                      # keep the CPU suite fast
        cfg = OrCfg()
        oracle.or_cfg_init(ctypes.byref(cfg), g["w"], g["h"])
        cfg.frame_num = 2
        h = hashlib.sha256()
        for i in range(g["nframes"]):
            off = oracle.or_synthetic_offset(g["stream"], i, g["h"])
            n = oracle.or_compose(buf, BUF, ctypes.byref(cfg), off, 0, None)
            assert n == g["sizes"][i], (g["w"], g["stream"], i)
            h.update(bytes(buf[:n]))
        assert h.hexdigest() == g["sha256"]


def test_median3_quirk_and_bench_smoke(oracle):
    # bench's CPU leg must run: a tiny multi-thread sample
    b = ctypes.c_ulonglong()
    fps = oracle.or_bench_compose(4, 20, 1280, 720, 2, 2, ctypes.byref(b))
    assert fps > 0 and b.value > 4 * 20 * 2000


@pytest.mark.parametrize("w,h", [(64, 48), (1280, 720)])
@pytest.mark.parametrize("which", [0, 1])
def test_ipcm_picture_file_pinned(oracle, golden_md5, w, h, which):
    """or_ipcm_picture_file (any I420 picture, the GPU reference-file
    writer's checker) reproduces the reference's striped I_PCM files when
    given the striped pictures"""
    from dynhelp import ipcm_file, striped_i420
    got = ipcm_file(oracle, w, h, striped_i420(w, h, which))
    g = golden_md5[f"ipcm_{w}x{h}_{'ab'[which]}.h264"]
    assert len(got) == g["bytes"] and hashlib.md5(got).hexdigest() == g["md5"]
