#!/usr/bin/env python3
"""bench.py -- composed frames/s of the MI355X scroll composer.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload p720dyn|p720|p4kdyn|p720hint|p720splice|ingest720|ipcm720]

One process per GPU (torch.distributed.run for N > 1; RANK / LOCAL_RANK /
WORLD_SIZE from the env).  Streams are independent, so each rank owns a static
shard (its own streams; weak scaling, no collective in the data path; gloo is
used only for the timing barrier / max-over-ranks).

A step = one scroll_batch_compose over every stream of the rank:
  workload p720dyn (default, BASELINE config 3 -- the metric's "1280x720,
  360x360 dyn"): 256 streams x 16 composed 1280x720 frames, each scroll NAL
  with the 360x360 dynamic rect at MB (28, 10) coded by the 4x4 transform +
  quant + CAVLC path; source pixels = the SURVEY 8(d) synthetic generator
  (k_dyn_synth), reference pictures A / B = the experiment's striped I_PCM
  pictures, one copy per stream; all resident in HBM before timing.
  workload p720 (BASELINE config 2): 256 streams x 1024 composed frames,
  P-only (no dynamic rect).
  workload p4kdyn (BASELINE config 5 per GPU): 128 streams x 16 composed
  3840x2160 frames with a 720x720 rect (47x47 MBs); config 4 = p720dyn with
  --streams 1024 per GPU on 8 GPUs.
  workload p720hint (UI hints; no BASELINE number): 256
  streams x 16 composed 1280x720 frames whose scroll NALs carry a UI overlay
  (static chrome and side panel, a horizontally scrolling carousel) in the
  P_Skip mode, coded per MB by k_hint_stage.
  workload p720splice (pre-encoded MB splice; no BASELINE
  number): 256 streams x 16 composed 1280x720 frames, each scroll NAL with a
  25x25-MB external P slice spliced in; the slices are produced on the GPU by
  the dynamic rect coder for 400x400 pictures (the "dynamic encoder"), stay
  in HBM and are handed over by device pointer and parsed again every step.
  workload ipcm720 (metric: reference files/s): a step =
  scroll_batch_ipcm_files_device of 256 random 1280x720 I420 pictures in HBM
  -> 256 SPS+PPS+I_PCM IDR files in HBM (the files ingest720 reads).
  workload ingest720 (metric: ingested streams/s): a
  step = scroll_batch_ingest_device of 256 new streams whose 1280x720 I_PCM
  reference files (A, B; one copy per stream) are resident in HBM --
  composer_init + composer_write_header on the GPU.
  Offsets = SURVEY 8(d) synthetic scroll (speed 1+(s%8), phase 97 s mod 1440)
  in HBM; output arenas are rewound on device at every step (the bytes of a
  step are the product).
Prints ONE JSON line (rank 0) with the dominant kernel's roofline (k_dyn_row
for the dynamic rect, k_hint_stage, k_emit; HIP events on its launch stream),
the CPU oracle on host cores (rank 0, N = 1) and, after the timed region, the
check of the last step's bytes against the oracle ("verified"; a mismatch
exits with status 3).  --gpus N without a launcher starts N ranks itself.
"""
import argparse
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "h264-scroll-encoder_amd"))

METRIC = "composed frames/sec (1280x720, 360x360 dyn) at 1/2/4/8 GPU; bit-exact vs CPU"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
NAL_DESC_BYTES = 32            # NalDesc read per NAL by k_emit

WORKLOADS = {
    "p720dyn": dict(w=1280, h=720, streams=256, frames=16, rect=(28, 10, 25, 25), rect_px=360,
                    desc="BASELINE config 3: 256 concurrent 1280x720 streams + 360x360 "
                         "synthetic dynamic rect (4x4 int transform + quant + CAVLC), "
                         "composer_write_scroll_frame semantics"),
    "p4kdyn": dict(w=3840, h=2160, streams=128, frames=16, rect=(96, 44, 47, 47), rect_px=720,
                   desc="BASELINE config 5 per GPU: 128 concurrent 3840x2160 streams (1024 over 8 "
                        "GPUs) + 720x720 dynamic rect (47x47 MBs, +16 px margin); the scroll passes "
                        "496/992/1488/1984 -> up to 6 reference pictures"),
    "p720full": dict(w=1280, h=720, streams=256, frames=4, rect=(0, 0, 80, 45), rect_px="1280x720",
                     metric="composed frames/sec (1280x720, whole-frame residual: the conventional-encode "
                            "fallback); bit-exact vs CPU",
                     desc="the conventional-encode fallback (docs/MASTER_DESIGN.md:220): 256 concurrent "
                          "1280x720 streams, every scroll frame's whole picture (80x45 MBs) through the "
                          "residual coder (4x4 int transform + quant + CAVLC) over the scroll motion"),
    "p720": dict(w=1280, h=720, streams=256, frames=1024, rect=None,
                 desc="BASELINE config 2: 256 concurrent 1280x720 streams, P-only "
                      "(no dynamic rect), composer_write_scroll_frame semantics"),
    "ingest720": dict(w=1280, h=720, streams=256, frames=1, rect=None, ingest=True,
                      desc="stream ingest (SURVEY 8f rows 3-4): 256 new 1280x720 streams per step, "
                           "composer_init + composer_write_header from I_PCM reference files in HBM"),
    "ipcm720": dict(w=1280, h=720, streams=256, frames=1, rect=None, ipcm=True,
                    desc="reference files from pictures (SURVEY 8f row 3): 256 1280x720 I420 "
                         "pictures in HBM -> 256 SPS+PPS+I_PCM IDR Annex-B files in HBM per step"),
    "p720splice": dict(w=1280, h=720, streams=256, frames=16, rect=None, splice=(28, 10, 25, 25),
                       desc="pre-encoded MB splice (SURVEY 8f row 2): 256 concurrent 1280x720 "
                            "streams, every scroll NAL carries a 25x25-MB external P slice "
                            "(400x400 px: a 360x360 preview + margin) spliced at MB (28, 10); "
                            "the slices are the dynamic rect coder's output for 400x400 "
                            "pictures, resident in HBM, parsed again every step"),
    "p720splicerows": dict(w=1280, h=720, streams=256, frames=16, rect=None, splice=(28, 10, 25, 25),
                           slice_rows=True,
                           desc="pre-encoded MB splice, one slice per MB row (SURVEY 8f row 2): as "
                                "p720splice, the 25x25-MB external picture as 25 Annex-B slices "
                                "(first_mb_in_slice 25 r), one parse wave per slice"),
    "p720hint": dict(w=1280, h=720, streams=256, frames=16, rect=None, hints=True,
                     desc="UI hints (SURVEY 8f row 1): 256 concurrent 1280x720 streams, scroll "
                          "frames with a static chrome / side panel / horizontal carousel "
                          "overlay, P_Skip mode"),
}


def _bits_to_bytes(bits):
    import numpy as np
    bits = np.asarray(bits, np.uint8)
    return np.packbits(bits).tobytes()


def _ue(v):
    v += 1
    n = v.bit_length()
    return [0] * (n - 1) + [(v >> (n - 1 - i)) & 1 for i in range(n)]


def _u(v, n):
    return [(v >> (n - 1 - i)) & 1 for i in range(n)]


def _escape(rbsp):
    """nal.c:24-50 emulation prevention (vectorised check, loop only if needed)"""
    import numpy as np
    a = np.frombuffer(rbsp, np.uint8)
    if len(a) < 3 or not np.any((a[:-2] == 0) & (a[1:-1] == 0) & (a[2:] <= 3)):
        return rbsp
    out, z = bytearray(), 0
    for v in rbsp:
        if z >= 2 and v <= 3:
            out.append(3)
            z = 0
        out.append(v)
        z = z + 1 if v == 0 else 0
    return bytes(out)


def ipcm_ref_file(w, h, which):
    """an Annex-B reference file as a harness would write it (SURVEY Appendix
    B): SPS + PPS + IDR of striped I_PCM MBs in the experiment's colours"""
    import numpy as np
    trail = lambda b: b + [1] + [0] * (-(len(b) + 1) % 8)
    sps = trail(_u(66, 8) + _u(0xc0, 8) + _u(40, 8) + _ue(0) + _ue(0) + _ue(2) + _ue(10) + [0] +
                _ue(w // 16 - 1) + _ue(h // 16 - 1) + [1, 1, 0, 0])
    pps = trail(_ue(0) + _ue(0) + [0, 0] + _ue(0) + _ue(1) + _ue(0) + [0, 0, 0] + _ue(0) * 3 +
                [1, 0, 0])
    hdr = _ue(0) + _ue(7) + _ue(0) + _u(0, 4) + _ue(0) + [0, 1] + _ue(0) + _ue(1) + _ue(25)
    hdr += [0] * (-len(hdr) % 8)
    cols = ([81, 90, 240, 145, 54, 34, 41, 240, 110], [210, 16, 146, 170, 166, 16, 106, 202, 222])[which]
    mbw, mbh = w // 16, h // 16
    third = mbh // 3
    body = bytearray(_bits_to_bytes(hdr))
    for y in range(mbh):
        st = 0 if y < third else (1 if y < 2 * third else 2)
        mb = bytes([cols[3 * st]] * 256 + [cols[3 * st + 1]] * 64 + [cols[3 * st + 2]] * 64)
        row = (mb + b"\x0d\x00") * mbw
        body += row if y < mbh - 1 else row[:-2]
    body += b"\x80"
    nal = lambda hb, r: b"\0\0\0\1" + bytes([hb]) + _escape(r)
    return nal(0x67, _bits_to_bytes(sps)) + nal(0x68, _bits_to_bytes(pps)) + nal(0x65, bytes(body))


def oracle_lib():
    """CHECKER / CPU baseline only: oracle/_build/liboracle.so (built on demand)"""
    repo_oracle = os.path.join(HERE, "oracle")
    so = os.path.join(repo_oracle, "_build", "liboracle.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-s", "-C", repo_oracle], check=True)
    lib = ctypes.CDLL(so)
    lib.or_composer_run.restype = ctypes.c_size_t
    lib.or_ipcm_picture_file.restype = ctypes.c_size_t
    return lib


def verify_ingest_step(b, files, first, S):
    """CHECKER (after timing): the first and the last stream ingested by the
    last timed step against or_composer_run (oracle/scroll_oracle.c)"""
    lib = oracle_lib()
    a, bb = files
    cap = 2 * (len(a) + len(bb)) + 4096
    buf = (ctypes.c_uint8 * cap)()
    n = lib.or_composer_run(buf, cap, a, len(a), bb, len(bb), 0, 1)
    want = bytes(buf[:n])
    bad = [k for k in (first, first + S - 1) if b.output(k) != want]
    return (not bad), {"streams_checked": 2, "mismatch": bad}


def verify_ipcm_step(pics, out, sizes, ostride, W, H):
    """CHECKER (after timing): the first and the last file of the last timed
    step against or_ipcm_picture_file (oracle/scroll_oracle.c)"""
    import numpy as np
    lib = oracle_lib()
    cap = 2 * W * H + (1 << 16)
    buf = (ctypes.c_uint8 * cap)()
    S = len(sizes)
    bad = []
    for k in (0, S - 1):
        p = np.ascontiguousarray(pics[k].cpu().numpy())
        n = lib.or_ipcm_picture_file(buf, cap, W, H, p.ctypes.data_as(ctypes.c_void_p))
        got = out[k * ostride:k * ostride + sizes[k]].cpu().numpy().tobytes()
        if got != bytes(buf[:n]):
            bad.append(k)
    return (not bad), {"files_checked": 2, "mismatch": bad}


def cpu_baseline_ingest(files, nstreams=8):
    """composer_init + composer_write_header restated (oracle/scroll_oracle.c
    or_composer_run, no frames) on one host core"""
    repo_oracle = os.path.join(HERE, "oracle")
    so = os.path.join(repo_oracle, "_build", "liboracle.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-s", "-C", repo_oracle], check=True)
    lib = ctypes.CDLL(so)
    lib.or_composer_run.restype = ctypes.c_size_t
    a, b = files
    cap = 2 * (len(a) + len(b)) + 4096
    buf = (ctypes.c_uint8 * cap)()
    t0 = time.perf_counter()
    for _ in range(nstreams):
        if not lib.or_composer_run(buf, cap, a, len(a), b, len(b), 0, 1):
            raise RuntimeError("oracle refused the reference files")
    sps = nstreams / (time.perf_counter() - t0)
    return dict(value=round(sps, 2), unit="streams/s", cores=1, kind="port",
                sample=f"{nstreams} streams, the same 1280x720 I_PCM reference pair, 1 thread, "
                       f"oracle/scroll_oracle.c or_composer_run -O2")


def run_ingest(args, wl, rank, world, local, dist):
    import numpy as np
    import torch
    import h264scroll as hs
    torch.cuda.set_device(local)
    W, H, S = wl["w"], wl["h"], wl["streams"]
    fa, fb = ipcm_ref_file(W, H, 0), ipcm_ref_file(W, H, 1)
    la, lb = (len(fa) + 255) & ~255, (len(fb) + 255) & ~255
    pair = la + lb
    host = np.zeros(S * pair, np.uint8)
    for k in range(S):                        # one copy per stream (own HBM traffic)
        host[k * pair:k * pair + len(fa)] = np.frombuffer(fa, np.uint8)
        host[k * pair + la:k * pair + la + len(fb)] = np.frombuffer(fb, np.uint8)
    dev = torch.from_numpy(host).to(f"cuda:{local}")
    desc = []
    for k in range(S):
        desc += [k * pair, len(fa), k * pair + la, len(fb)]
    nsteps = args.warmup + args.steps
    arena = (2 * pair + (1 << 20) + 4095) & ~4095
    b = hs.Batch(S * nsteps, 1, arena, device=local)
    torch.cuda.synchronize()

    def barrier():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()

    for _ in range(args.warmup):
        b.ingest_device(S, dev.data_ptr(), desc)
    b.enable_timing(True)
    b.ingest_stats()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.ingest_device(S, dev.data_ptr(), desc)
    barrier()
    t1 = time.perf_counter()
    kms, kn = b.ingest_stats()
    out_bytes = b.output_size(S * nsteps - 1)
    b.enable_timing(False)
    el = max_over_ranks(t1 - t0, dist)
    verified, vdetail = (None, None) if args.no_verify else verify_ingest_step(b, (fa, fb), S * (nsteps - 1), S)
    if rank == 0:
        k_ms = kms / max(kn, 1)
        alg = S * (len(fa) + len(fb) + out_bytes)          # files in, header NALs out
        achieved = alg / (k_ms * 1e-3) / 1e9
        out = {
            "metric": "ingested streams/s (composer_init + composer_write_header, 1280x720 "
                      "I_PCM reference pair per stream); bit-exact vs CPU",
            "value": round(S * args.steps * world / el, 1),
            "unit": "streams/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * el / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": wl["desc"], "resolution": f"{W}x{H}", "streams_per_step": S,
                       "parallelism": f"static stream shard x{world}, no RCCL"},
            "bytes_per_stream": {"in": len(fa) + len(fb), "out": out_bytes},
            "verified": verified, "verify": vdetail,
            "roofline": {"bound": "hbm", "kernel": ING_KERNEL,
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic_of(args.workload, ING_KERNEL, alg),
                         "alg_bytes_per_launch": alg, "kernel_ms_avg": round(k_ms, 4)},
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline_ingest((fa, fb))
        print(json.dumps(out), flush=True)
    b.close()
    if verified is False:
        sys.exit(3)


def cpu_baseline_ipcm(pics, w, h):
    """or_ipcm_picture_file (oracle/scroll_oracle.c) on one host core over the
    given pictures"""
    repo_oracle = os.path.join(HERE, "oracle")
    so = os.path.join(repo_oracle, "_build", "liboracle.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-s", "-C", repo_oracle], check=True)
    lib = ctypes.CDLL(so)
    lib.or_ipcm_picture_file.restype = ctypes.c_size_t
    cap = 2 * w * h + (1 << 16)
    buf = (ctypes.c_uint8 * cap)()
    t0 = time.perf_counter()
    for p in pics:
        if not lib.or_ipcm_picture_file(buf, cap, w, h, p.ctypes.data_as(ctypes.c_void_p)):
            raise RuntimeError("oracle I_PCM writer failed")
    fps = len(pics) / (time.perf_counter() - t0)
    return dict(value=round(fps, 2), unit="files/s", cores=1, kind="port",
                sample=f"{len(pics)} random {w}x{h} I420 pictures, 1 thread, "
                       f"oracle/scroll_oracle.c or_ipcm_picture_file -O2")


def run_ipcm(args, wl, rank, world, local, dist):
    import numpy as np
    import torch
    import h264scroll as hs
    torch.cuda.set_device(local)
    W, H, S = wl["w"], wl["h"], wl["streams"]
    pic = W * H * 3 // 2
    g = torch.Generator(device=f"cuda:{local}").manual_seed(1234 + rank)
    pics = torch.randint(0, 256, (S, pic), dtype=torch.uint8, device=f"cuda:{local}", generator=g)
    ostride = ((3 * (W * H * 193 // 128)) // 2 + 128 + 255) & ~255
    out = torch.empty(S * ostride, dtype=torch.uint8, device=f"cuda:{local}")
    b = hs.Batch(1, 1, 1 << 16, device=local)
    torch.cuda.synchronize()

    def barrier():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()

    # the asynchronous entry (sizes stay on the device, overflow reported at
    # the sync): a step is the two passes' launches, no host round trip
    d_sizes = torch.zeros(S, dtype=torch.int64, device=f"cuda:{local}")
    for _ in range(args.warmup):
        b.ipcm_files_device_async(S, W, H, pics.data_ptr(), pic, out.data_ptr(), ostride, d_sizes.data_ptr())
    if b.sync() != 0:
        raise RuntimeError(hs.last_error())
    b.enable_timing(True)
    b.ipcm_stats()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.ipcm_files_device_async(S, W, H, pics.data_ptr(), pic, out.data_ptr(), ostride, d_sizes.data_ptr())
    barrier()
    t1 = time.perf_counter()
    if b.sync() != 0:
        raise RuntimeError(hs.last_error())
    sizes = [int(v) for v in d_sizes.cpu().tolist()]
    kms, kn = b.ipcm_stats()
    b.enable_timing(False)
    el = max_over_ranks(t1 - t0, dist)
    verified, vdetail = (None, None) if args.no_verify else verify_ipcm_step(pics, out, sizes, ostride, W, H)
    if rank == 0:
        k_ms = kms / max(kn, 1)
        alg = S * pic + sum(sizes)                       # pictures in, files out
        achieved = alg / (k_ms * 1e-3) / 1e9
        res = {
            "metric": "reference files/s (1280x720 I420 picture -> SPS+PPS+I_PCM IDR Annex-B file); "
                      "bit-exact vs CPU",
            "value": round(S * args.steps * world / el, 1),
            "unit": "files/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * el / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": wl["desc"], "resolution": f"{W}x{H}", "files_per_step": S,
                       "parallelism": f"static shard x{world}, no RCCL"},
            "bytes_per_file": {"in": pic, "out": round(sum(sizes) / S, 1)},
            "api": "scroll_batch_ipcm_files_device_async (sizes on the device, no host step per call)",
            "verified": verified, "verify": vdetail,
            "roofline": {"bound": "hbm", "kernel": IPCM_KERNEL,
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic_of(args.workload, IPCM_KERNEL, alg),
                         "alg_bytes_per_launch": alg, "kernel_ms_avg": round(k_ms, 4)},
        }
        if world == 1 and not args.no_cpu:
            host = pics[:8].cpu().numpy()
            res["cpu_baseline"] = cpu_baseline_ipcm([np.ascontiguousarray(p) for p in host], W, H)
        print(json.dumps(res), flush=True)
    b.close()
    if verified is False:
        sys.exit(3)


def ui_hints(s, f, w, h):
    """the UI overlay of frame f of stream s (MB rects, include/composer_batch.h):
    static top / bottom chrome and a side panel (reference A, no motion), a
    carousel band scrolling horizontally on reference B"""
    mbw, mbh = w // 16, h // 16
    side = mbw // 7
    return [(0, 0, mbw, 2, 0, 0, 0),                                  # top chrome
            (0, mbh - 2, mbw, mbh, 0, 0, 0),                          # bottom bar
            (0, 2, side, mbh - 2, 0, 0, 0),                           # side panel
            (side, mbh // 2 - 3, mbw, mbh // 2 + 3, 1, -((3 * f + s) % 256), 0)]   # carousel


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


def synthetic_offsets(first, nstreams, nframes, h):
    import numpy as np
    s = np.arange(first, first + nstreams, dtype=np.int64)[:, None]
    i = np.arange(nframes, dtype=np.int64)[None, :]
    p = (i * (1 + s % 8) + (97 * s) % (2 * h)) % (2 * h)
    return np.where(p < h, p, 2 * h - p).astype(np.int32)


def shard_streams(rank, world, per_gpu):
    """Static contiguous stream shard of rank (weak scaling): [first, first + per_gpu)."""
    if not (0 <= rank < world) or per_gpu <= 0:
        raise ValueError("bad shard")
    return rank * per_gpu, per_gpu


def max_over_ranks(x, dist):
    """Elapsed time of the slowest rank (gloo all-reduce MAX; identity for one rank)."""
    if dist is None:
        return float(x)
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def rect_label(wl):
    """'360x360' for a square rect of rect_px pixels, else rect_px itself"""
    r = wl.get("rect_px")
    return f"{r}x{r}" if isinstance(r, int) else str(r)


def cpu_baseline(wl, threads):
    """Oracle (C restatement, bit-exact to the reference) on host cores."""
    repo_oracle = os.path.join(HERE, "oracle")
    so = os.path.join(repo_oracle, "_build", "liboracle.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-s", "-C", repo_oracle], check=True)
    lib = ctypes.CDLL(so)
    lib.or_bench_compose.restype = ctypes.c_double
    lib.or_bench_compose_dyn.restype = ctypes.c_double
    if wl["rect"]:
        x0, y0, rw, rh = wl["rect"]
        nstreams, nframes = 4 * threads, max(8, 64 * 625 // (rw * rh))
        nbytes = ctypes.c_ulonglong()
        fps = lib.or_bench_compose_dyn(nstreams, nframes, wl["w"], wl["h"], x0, y0, rw, rh,
                                       threads, ctypes.byref(nbytes))
        fps1 = lib.or_bench_compose_dyn(1, 48, wl["w"], wl["h"], x0, y0, rw, rh, 1,
                                        ctypes.byref(nbytes))
        return dict(value=round(fps, 1), unit="frames/s", cores=threads, kind="port",
                    sample=f"{nstreams} streams x {nframes} frames {wl['w']}x{wl['h']} + "
                           f"{rect_label(wl)} dynamic rect ({rw}x{rh} MBs; same synthetic offsets, 4 source "
                           f"frames cycled per stream), {threads} pthreads, "
                           f"oracle/dyn_oracle.c -O2",
                    single_core_fps=round(fps1, 1))
    nstreams, nframes = 256, 512
    nbytes = ctypes.c_ulonglong()
    fps = lib.or_bench_compose(nstreams, nframes, wl["w"], wl["h"], threads, 200,
                               ctypes.byref(nbytes))
    fps1 = lib.or_bench_compose(8, 512, wl["w"], wl["h"], 1, 100, ctypes.byref(nbytes))
    return dict(value=round(fps, 1), unit="frames/s", cores=threads, kind="port",
                sample=f"{nstreams} streams x {nframes} frames {wl['w']}x{wl['h']} (same "
                       f"synthetic offsets), {threads} pthreads, oracle/scroll_oracle.c -O2",
                single_core_fps=round(fps1, 1))


def cpu_baseline_hint(wl, nstreams=128, nframes=256):
    """Oracle (oracle/hint_oracle.c) on one host core over a bounded sample
    of the same workload."""
    import numpy as np
    repo_oracle = os.path.join(HERE, "oracle")
    so = os.path.join(repo_oracle, "_build", "liboracle.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-s", "-C", repo_oracle], check=True)
    lib = ctypes.CDLL(so)
    sys.path.insert(0, os.path.join(HERE, "tests"))
    from dynhelp import OrCfg, hint_array
    W, H = wl["w"], wl["h"]
    offs = synthetic_offsets(0, nstreams, nframes, H)
    buf = (ctypes.c_uint8 * (1 << 20))()
    err = ctypes.c_int()
    arrs = {}
    t0 = time.perf_counter()
    for s in range(nstreams):
        c = OrCfg()
        lib.or_cfg_init(ctypes.byref(c), W, H)
        c.frame_num = 2
        for f in range(nframes):
            key = (s, f % wl["frames"])
            if key not in arrs:
                arrs[key] = hint_array(ui_hints(s, key[1], W, H))
            arr, n = arrs[key]
            lib.or_compose_hint(buf, len(buf), ctypes.byref(c), int(offs[s, f]), 0, arr, n, 1,
                                ctypes.byref(err))
    fps = nstreams * nframes / (time.perf_counter() - t0)
    return dict(value=round(fps, 1), unit="frames/s", cores=1, kind="port",
                sample=f"{nstreams} streams x {nframes} frames {W}x{H}, same offsets and UI "
                       f"overlay, P_Skip mode, 1 thread, oracle/hint_oracle.c -O2")


def external_slices(hs, S, F, sw, sh, first, device):
    """the "dynamic encoder" of MASTER_DESIGN 4.2 on the GPU: a batch of
    sw*16 x sh*16 pictures whose dynamic rect covers the whole picture, so
    each scroll NAL is a P slice of sw x sh residual MBs.  Returns the batch
    (its arenas hold the NALs) and per (s, f) the NAL's device pointer and
    size."""
    import numpy as np
    ew, eh = 16 * sw, 16 * sh
    e = hs.Batch(S, F, F * (2048 + 1024 * sw * sh) + (1 << 20), device=device)
    for _ in range(S):
        e.add_stream(hs.make_config(ew, eh))
    offs = synthetic_offsets(first, S, F, eh)              # < 496: no waypoints
    e.set_offsets(offs)
    e.set_dyn_rect(0, 0, sw, sh)
    e.set_dyn_refs(striped_i420(ew, eh, 0), striped_i420(ew, eh, 1))
    e.dyn_source_synth(F, stream_base=first, t0=0)
    e.compose(F, rewind=True)
    if e.sync() != 0:
        raise RuntimeError(hs.last_error())
    ptrs = {}
    for s in range(S):
        base, pos = e.output_device_ptr(s), 0
        nals = e.nals(s)
        assert len(nals) == F, "one scroll NAL per frame (no waypoints)"
        for f, (kind, _, size, _) in enumerate(nals):
            ptrs[(s, f)] = (base + pos, size)
            pos += size
    return e, ptrs


def _set_first_mb(nal, k):
    """an Annex-B slice NAL whose first_mb_in_slice is 0 with it set to k:
    the RBSP's bits after that ue(0) shifted behind ue(k), re-aligned and
    re-escaped (input preparation, outside the timed region)"""
    import re
    if k == 0:
        return nal
    i = nal.index(b"\x00\x00\x01") + 3
    rbsp = nal[i + 1:].replace(b"\x00\x00\x03", b"\x00\x00")
    v = int.from_bytes(rbsp, "big")
    tz = (v & -v).bit_length() - 1
    v >>= tz
    nb = 8 * len(rbsp) - tz                          # through rbsp_stop_one_bit
    assert (v >> (nb - 1)) & 1, "first_mb_in_slice must be 0"
    x = k + 1
    L = 2 * x.bit_length() - 1
    v = (x << (nb - 1)) | (v & ((1 << (nb - 1)) - 1))
    nb += L - 1
    pad = (-nb) % 8
    out = (v << pad).to_bytes((nb + pad) // 8, "big")
    out = re.sub(rb"\x00\x00(?=[\x00-\x03])", b"\x00\x00\x03", out)
    return b"\x00\x00\x00\x01" + nal[i:i + 1] + out


def external_row_slices(hs, torch, S, F, sw, sh, first, device):
    """external pictures of sw x sh MBs coded as one slice per MB row: row r
    of frame (s, f) is the dynamic rect coder's NAL for an sw x 1-MB picture
    (stream s * sh + r) -- a slice predicts nothing across its boundary, so a
    one-row picture's slice data is that row's slice -- with its
    first_mb_in_slice set to r * sw.  The pictures sit in one device buffer.
    Returns (keep-alive objects, per (s, f) device pointer and size, per (s,
    f) host bytes)."""
    import numpy as np
    e, ptrs = external_slices(hs, S * sh, F, sw, 1, first * sh, device)
    rows = {}
    for ss in range(S * sh):
        out, pos = e.output(ss), 0
        for f in range(F):
            n = ptrs[(ss, f)][1]
            rows[(ss, f)] = bytes(out[pos:pos + n])
            pos += n
    e.close()
    host, pool, offs = {}, bytearray(), {}
    for s in range(S):
        for f in range(F):
            pic = b"".join(_set_first_mb(rows[(s * sh + r, f)], r * sw) for r in range(sh))
            host[(s, f)] = pic
            offs[(s, f)] = len(pool)
            pool += pic
            pool += bytes((-len(pool)) % 16)
    dev = torch.from_numpy(np.frombuffer(bytes(pool), np.uint8).copy()).to(f"cuda:{device}")
    base = dev.data_ptr()
    return dev, {k: (base + offs[k], len(host[k])) for k in host}, host


def cpu_baseline_splice(wl, slices, nframes=64, threads=None):
    """oracle/splice_oracle.c on the host cores over a bounded sample: the
    same external slices (copied to the host) into 4 streams per thread x
    nframes frames, one stream at a time per thread (ctypes releases the GIL
    for the whole call: the threads run the C code in parallel, like config
    3's pthreads)"""
    from concurrent.futures import ThreadPoolExecutor
    repo_oracle = os.path.join(HERE, "oracle")
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import subprocess
    subprocess.run(["make", "-s", "-C", repo_oracle], check=True, stdout=subprocess.DEVNULL)
    lib = ctypes.CDLL(os.path.join(repo_oracle, "_build", "liboracle.so"))
    from dynhelp import OrCfg, splice_of
    W, H = wl["w"], wl["h"]
    x0, y0, sw, sh = wl["splice"]
    threads = threads or usable_cores()
    nstreams = 4 * threads
    offs = synthetic_offsets(0, nstreams, nframes, H)
    sps = [splice_of(x0, y0, sw, sh, slices[k % len(slices)]) for k in range(nstreams * nframes)]

    def one_stream(s):
        buf = (ctypes.c_uint8 * (4 << 20))()
        err = ctypes.c_int()
        c = OrCfg()
        lib.or_cfg_init(ctypes.byref(c), W, H)
        c.frame_num = 2
        for f in range(nframes):
            lib.or_compose_splice(buf, len(buf), ctypes.byref(c), int(offs[s, f]), 0, None, 0,
                                  2, ctypes.byref(sps[s * nframes + f]), ctypes.byref(err))

    def run(n, nthr):
        t0 = time.perf_counter()
        with ThreadPoolExecutor(nthr) as ex:
            list(ex.map(one_stream, range(n)))
        return n * nframes / (time.perf_counter() - t0)

    fps1 = run(1, 1)
    fps = run(nstreams, threads)
    return {"value": round(fps, 1), "unit": "frames/s", "cores": threads,
            "kind": "port", "sample": f"{nstreams} streams x {nframes} frames, {W}x{H} with a "
                                      f"{sw}x{sh}-MB spliced slice, {threads} threads, "
                                      f"oracle/splice_oracle.c -O2 (parse + compose)",
            "single_core_fps": round(fps1, 1)}


def run_splice(args, wl, rank, world, local, dist):
    import numpy as np
    import torch
    import h264scroll as hs

    torch.cuda.set_device(local)
    stream = torch.cuda.current_stream()
    S, F, W, H = wl["streams"], wl["frames"], wl["w"], wl["h"]
    x0, y0, sw, sh = wl["splice"]
    first, _ = shard_streams(rank, world, S)
    if wl.get("slice_rows"):
        e, ptrs, ext_host = external_row_slices(hs, torch, S, F, sw, sh, first, local)
    else:
        e, ptrs = external_slices(hs, S, F, sw, sh, first, local)
        ext_host = {}
        for s in range(S):
            out, pos = e.output(s), 0
            for f in range(F):
                n = ptrs[(s, f)][1]
                ext_host[(s, f)] = bytes(out[pos:pos + n])
                pos += n
    ext_bytes = sum(n for _, n in ptrs.values())
    entries = [(s, f, x0, y0, sw, sh, p, n) for (s, f), (p, n) in ptrs.items()]
    per_frame = 2 * (64 + (W // 16) * (H // 16)) + 2 * ext_bytes // (S * F) + 4096
    b = hs.Batch(S, F, F * per_frame + (1 << 20), device=local)
    for _ in range(S):
        b.add_stream(hs.make_config(W, H))
    b.set_offsets(synthetic_offsets(first, S, F, H))

    def barrier():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()

    def step():
        b.set_splices_device(entries)            # new content in place: parsed again
        b.compose(F, stream=stream.cuda_stream, rewind=True)

    for _ in range(args.warmup):
        step()
    barrier()
    if b.sync() != 0:
        raise RuntimeError(hs.last_error())
    b.enable_timing(True)
    b.kernel_stats_ex()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    t1 = time.perf_counter()
    if b.sync() != 0:
        raise RuntimeError(hs.last_error())
    (plan_ms, emit_ms, stage_ms, demit_ms, _, _), n_launch = b.kernel_stats_ex()
    step_bytes = b.last_bytes()
    rbsp_tot, ep_tot, dyn_nals = b.dyn_totals()
    b.enable_timing(False)
    el = max_over_ranks(t1 - t0, dist)
    value = S * F * args.steps * world / el
    verified, vdetail = (None, None) if args.no_verify else \
        verify_splice_step(b, ext_host, wl, first, args.warmup + args.steps)
    if rank == 0:
        n = max(n_launch, 1)
        kms = {"plan": plan_ms / n, "emit": emit_ms / n, "splice_stage": stage_ms / n,
               "dyn_emit": demit_ms / n}
        # k_splice_parse + k_splice_stage per launch: the external slices read
        # (twice: the parse and the body copy), the staged RBSP written
        alg_bytes = 2 * ext_bytes + rbsp_tot
        achieved = alg_bytes / (kms["splice_stage"] * 1e-3) / 1e9
        out = {
            "metric": "spliced composed frames/sec (1280x720 + 25x25-MB external " +
                      ("picture, one slice per MB row)" if wl.get("slice_rows") else "slice)"),
            "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * el / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": wl["desc"], "resolution": f"{W}x{H}",
                       "streams_per_gpu": S, "frames_per_step": F, "splice_rect_mb": [x0, y0, sw, sh],
                       "parallelism": f"static stream shard x{world}, no RCCL"},
            "bytes_per_frame": round(step_bytes / (S * F), 1),
            "external_slice_bytes_per_frame": round(ext_bytes / (S * F), 1),
            "roofline": {"bound": "hbm", "kernel": SPLICE_KERNEL,
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic_of(args.workload, SPLICE_KERNEL, alg_bytes),
                         "alg_bytes_per_launch": alg_bytes,
                         "kernel_ms_avg": {k: round(v, 4) for k, v in kms.items() if v > 0},
                         "timing": "HIP events around this kernel only, on its launch stream, over the "
                                   "timed steps (the other kernels: rocprofv3 stats in profiles/)"},
            "verified": verified, "verify": vdetail, "revision": revision(),
        }
        if world == 1 and not args.no_cpu:
            slices = [ext_host[(s, f)] for s in range(min(S, 4)) for f in range(F)]
            out["cpu_baseline"] = cpu_baseline_splice(wl, slices)
        print(json.dumps(out), flush=True)
    b.close()
    if not wl.get("slice_rows"):
        e.close()
    if verified is False:
        sys.exit(3)


def verify_splice_step(b, ext_host, wl, first, passes, nstreams=None):
    """CHECKER (after timing): the last step's bytes of every stream (or the
    first nstreams) against oracle/splice_oracle.c (the external slices
    copied back from the encoder's arena; the splice path's default
    SCROLL_HINT_SPEC)"""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import stepcheck
    from dynhelp import OrCfg, splice_of
    t0 = time.perf_counter()
    oracle = stepcheck.load_oracle()
    S, F, W, H = wl["streams"], wl["frames"], wl["w"], wl["h"]
    x0, y0, sw, sh = wl["splice"]
    ns = S if nstreams is None else min(S, nstreams)
    offs = synthetic_offsets(first, ns, F, H)
    buf = (ctypes.c_uint8 * (8 << 20))()
    err = ctypes.c_int()
    want = []
    for s in range(ns):
        c = OrCfg()
        oracle.or_cfg_init(ctypes.byref(c), W, H)
        c.frame_num = 2
        for _ in range(passes - 1):
            for f in range(F):
                oracle.or_compose_state(ctypes.byref(c), int(offs[s, f]), 0)
        o = bytearray()
        for f in range(F):
            sp = splice_of(x0, y0, sw, sh, ext_host[(s, f)])
            k = oracle.or_compose_splice(buf, len(buf), ctypes.byref(c), int(offs[s, f]), 0, None, 0,
                                         2, ctypes.byref(sp), ctypes.byref(err))
            if err.value or not k:
                return False, {"error": f"oracle refused stream {s} frame {f}"}
            o += bytes(buf[:k])
        want.append(bytes(o))
    ok, d = stepcheck.compare_streams(b, want)
    d.update(sample=f"first {ns} of {S} streams", passes=passes,
             seconds=round(time.perf_counter() - t0, 2), checker="oracle/splice_oracle.c")
    return ok, d


ING_KERNEL = "ingest call: k_ing_scan, k_ing_head, k_ing_seg<FUSED>"
IPCM_KERNEL = "k_ipcm (count + write passes)"
# the splice workloads' timed launches (one HIP event pair: parse, then stage)
SPLICE_KERNEL = ("k_splice_units+k_splice_unesc+k_splice_lanes+k_splice_parse+k_splice_fix"
                 "+k_hint_stage+k_splice_stage")
SPLICE_KERNELS = SPLICE_KERNEL.split("+")


def traffic_of(workload, kernel, alg_bytes):
    """HBM bytes per call from profiles/traffic_<workload>.json when it was
    measured on this very configuration (load_traffic), else None"""
    t = load_traffic(workload, kernel, alg_bytes)
    return t.get("hbm_bytes_per_launch") if t else None


def load_traffic(workload, kernel, alg_bytes):
    """PMC traffic of the dominant kernel (profiles/traffic_<workload>.json,
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes, tools/traffic.py) -- only when
    it was measured on this very launch: same kernel and the same algorithmic
    bytes per launch (i.e. the same streams x frames x rect).  Otherwise None:
    PMC counters need their own rocprofv3 runs, they cannot be read inside
    this process."""
    p = os.path.join(HERE, "profiles", f"traffic_{workload}.json")
    try:
        t = json.load(open(p))
    except (OSError, ValueError):
        return None
    if t.get("kernel") != kernel or abs(float(t.get("alg_bytes_per_launch", -1)) - alg_bytes) > 0.5:
        return None
    return t


def usable_cores():
    """host cores this process may use: the CPU affinity set, capped by the
    cgroup CPU quota (the GPU box grants a 16-CPU quota on a many-core host,
    where os.cpu_count() shows every core of the machine)"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(-(-int(quota) // int(period)))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def revision():
    """the source revision of this tree: git's HEAD (+ "-dirty" with
    uncommitted changes to tracked files) where the tree has its .git, else
    the .revision file written on the build host before a GPU run (the
    snapshot on the GPU box has no .git).  A stale .revision never shadows
    git."""
    if os.path.isdir(os.path.join(HERE, ".git")):
        try:
            import subprocess
            head = subprocess.run(["git", "-C", HERE, "rev-parse", "HEAD"], capture_output=True,
                                  text=True, timeout=10).stdout.strip()
            dirty = subprocess.run(["git", "-C", HERE, "status", "--porcelain", "--untracked-files=no"],
                                   capture_output=True, text=True, timeout=10).stdout.strip()
            if head:
                return head + ("-dirty" if dirty else "")
        except Exception:
            pass
    p = os.path.join(HERE, ".revision")
    if os.path.exists(p):
        w = open(p).read().split()
        return (w[0] + ("-dirty" if "dirty" in w[1:] else "")) if w else None
    return None


def launch_ranks(n):
    """--gpus N without a launcher: start N ranks (torch.distributed.run, one
    process per GPU, rendezvous on 127.0.0.1) as children and exit with their
    status.  Runs before anything touches the GPU in this process."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="p720dyn", choices=sorted(WORKLOADS))
    ap.add_argument("--streams", type=int, default=0, help="override streams per GPU")
    ap.add_argument("--frames", type=int, default=0, help="override frames per step")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--time-every", type=int, default=4,
                    help="HIP events around the dominant kernel on every k-th timed compose step")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the post-timing oracle check of the last step")
    ap.add_argument("--no-host", action="store_true",
                    help="skip the host-delivery (PCIe-inclusive) and single-frame latency legs")
    args = ap.parse_args()

    wl = dict(WORKLOADS[args.workload])
    if args.streams:
        wl["streams"] = args.streams
    if args.frames:
        wl["frames"] = args.frames

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}")
    import torch
    ndev = torch.cuda.device_count()            # counts without initialising the GPU
    if ndev and local >= ndev:                  # more ranks than GPUs (a rehearsal): share them
        local %= ndev
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    if wl.get("splice"):
        run_splice(args, wl, rank, world, local, dist)
        if dist:
            dist.destroy_process_group()
        return
    if wl.get("ingest") or wl.get("ipcm"):
        (run_ingest if wl.get("ingest") else run_ipcm)(args, wl, rank, world, local, dist)
        if dist:
            dist.destroy_process_group()
        return

    import torch
    import h264scroll as hs

    torch.cuda.set_device(local)
    stream = torch.cuda.current_stream()
    S, F, W, H = wl["streams"], wl["frames"], wl["w"], wl["h"]
    first, _ = shard_streams(rank, world, S)       # static contiguous shard
    rect = wl["rect"]
    hints = wl.get("hints", False)
    b = build_compose_batch(hs, wl, first, local)

    def barrier():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()

    for _ in range(args.warmup):
        b.compose(F, stream=stream.cuda_stream, rewind=True)
    barrier()
    if b.sync() != 0:
        raise RuntimeError(hs.last_error())
    # lite: HIP events around the dominant kernel only (every event record
    # is a marker packet between the kernels; the full set adds ~40 us of
    # queue gaps to a step).  The other kernels' times come from rocprofv3
    b.enable_timing(True, lite=True)
    b.kernel_stats_ex()                             # reset accumulators
    barrier()
    # the event pair on every --time-every-th timed step only (its two marker
    # packets hold the queue ~5 us each: 5 % of a one-frame step); the
    # kernel's average is over the steps that carried it
    te = max(1, args.time_every)
    t0 = time.perf_counter()
    for i in range(args.steps):
        if te > 1:
            b.enable_timing(i % te == 0, lite=True)
        b.compose(F, stream=stream.cuda_stream, rewind=True)
    barrier()
    t1 = time.perf_counter()
    if b.sync() != 0:
        raise RuntimeError(hs.last_error())
    (plan_ms, emit_ms, stage_ms, demit_ms, code_ms, pack_ms), n_launch = b.kernel_stats_ex()
    step_bytes = b.last_bytes()                     # per step, all streams of this rank
    step_nals = b.last_nals()
    if rect or hints:
        rbsp_tot, ep_tot, dyn_nals = b.dyn_totals()
    b.enable_timing(False)

    el = max_over_ranks(t1 - t0, dist)
    frames_total = S * F * args.steps * world
    value = frames_total / el
    ms_step = 1000.0 * el / args.steps

    # after the timed region: the last step's bytes of this rank's streams
    # against the CPU oracle (the checker), every rank its own shard
    verified, vdetail = (None, None) if args.no_verify else \
        verify_last_step(b, wl, first, args.warmup + args.steps)
    all_ok = verified is not False
    if dist:
        import torch as _t
        flag = _t.tensor([0.0 if verified is False else 1.0], dtype=_t.float64)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        all_ok = flag.item() > 0.5

    # after the timed region and the check: the same workload delivered to
    # pinned host memory (never `value`), and the single-frame API latency
    host_leg = None
    if world == 1 and not args.no_host:
        host_leg = host_delivery(hs, wl, first, local, min(args.steps, 10), b)

    if rank == 0:
        n = max(n_launch, 1)
        kms = {"plan": plan_ms / n, "emit": emit_ms / n, "dyn_stage": stage_ms / n,
               "dyn_emit": demit_ms / n}
        if rect:
            kms["dyn_code"] = code_ms / n
            kms["dyn_pack"] = pack_ms / n
        if rect:
            # k_dyn_rows + k_dyn_row per launch (k_dyn_code_general: no
            # frame here): the source and prediction samples of every
            # dynamic MB (384 B each) read.  The row-stage bits the rect rows
            # write are intermediate and not counted (a lower bound)
            kern = "k_dyn_row"
            alg_bytes = dyn_nals * 2 * 384 * rect[2] * rect[3]
            kern_ms = kms["dyn_code"]
        elif hints:
            # k_hint_stage per launch: the staged RBSP written, the rects read
            kern = "k_hint_stage"
            alg_bytes = rbsp_tot + dyn_nals * (8 + 20 * 4)
            kern_ms = kms["dyn_stage"]
        else:
            kern = "k_emit"
            alg_bytes = step_bytes + NAL_DESC_BYTES * step_nals   # per k_emit launch
            kern_ms = kms["emit"]
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        traffic = load_traffic(args.workload, kern, alg_bytes)
        out = {
            "metric": wl.get("metric", METRIC),
            "value": round(value, 1),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": wl["desc"], "resolution": f"{W}x{H}",
                       "streams_per_gpu": S, "frames_per_step": F,
                       "parallelism": f"static stream shard x{world}, no RCCL"},
            "bytes_per_frame": round(step_bytes / (S * F), 1),
            "roofline": {"bound": "hbm", "kernel": kern,
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
                         "traffic_source": (f"profiles/traffic_{args.workload}.json (rocprofv3 "
                                            f"FETCH_SIZE/WRITE_SIZE passes of this launch)")
                         if traffic else "not measured for this launch",
                         "alg_bytes_per_launch": alg_bytes,
                         "kernel_ms_avg": {k: round(v, 4) for k, v in kms.items() if v > 0},
                         "timing": "HIP events around this kernel only, on its launch stream, on every "
                                   "%d-th timed step (the other kernels: rocprofv3 stats in profiles/)" % te},
            "verified": None if verified is None else bool(all_ok),
            "verify": vdetail,
            "revision": revision(),
        }
        if rect:
            out["config"]["dyn_rect_mb"] = list(rect)
            out["dyn"] = {"rbsp_bytes_per_frame": round(rbsp_tot / max(dyn_nals, 1), 1),
                          "ep_bytes_per_frame": round(ep_tot / max(dyn_nals, 1), 2)}
        if hints:
            out["hint"] = {"rbsp_bytes_per_frame": round(rbsp_tot / max(dyn_nals, 1), 1),
                           "ep_bytes_per_frame": round(ep_tot / max(dyn_nals, 1), 2)}
        if host_leg:
            out["host_delivery"] = host_leg
        if world == 1 and not args.no_cpu:
            cores = usable_cores()
            out["cpu_baseline"] = cpu_baseline_hint(wl) if hints else cpu_baseline(wl, cores)
            out["cpu_baseline"]["host"] = {"os_cpu_count": os.cpu_count(), "usable_cores": cores}
        print(json.dumps(out), flush=True)
    b.close()
    if dist:
        dist.destroy_process_group()
    if not all_ok:
        sys.exit(3)


def host_delivery(hs, wl, first, device, steps, b0):
    """PCIe-inclusive throughput (the reference hands its bytes over in host
    memory, composer.c:255-291): every step's bytes of every stream packed by
    the device into pinned host memory (scroll_batch_output_to_host_async).
    Two batches alternate on two HIP streams, so one's compose overlaps the
    other's copy.  Also the single-frame drop-in latency: h264_write_scroll_p_frame
    (one 1280x720 P NAL per call, host bytes back) against the reference's
    86-90 us per frame on one CPU core."""
    import ctypes
    import torch
    S, F = wl["streams"], wl["frames"]
    per_step = b0.last_bytes()
    cap = int(per_step * 1.25 + 16 * S + (1 << 20))
    b1 = build_compose_batch(hs, wl, first, device)
    bats = [b0, b1]
    hbs = [hs.HostBuffer(cap, S), hs.HostBuffer(cap, S)]
    sts = [torch.cuda.Stream(device=device), torch.cuda.Stream(device=device)]
    for i in range(2):                              # warm both
        bats[i].compose(F, stream=sts[i].cuda_stream, rewind=True)
        bats[i].output_to_host_async(hbs[i], stream=ctypes.c_void_p(sts[i].cuda_stream))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        i = k & 1
        bats[i].compose(F, stream=sts[i].cuda_stream, rewind=True)
        bats[i].output_to_host_async(hbs[i], stream=ctypes.c_void_p(sts[i].cuda_stream))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ok = all(h.total() is not None for h in hbs)
    # the delivered bytes of the last step equal the arena bytes (checked above against the oracle)
    i = (steps - 1) & 1
    bats[i].sync()
    same = all(hbs[i].stream(s) == bats[i].output(s) for s in range(0, S, max(1, S // 8)))
    delivered = sum(hbs[i].table[2 + 2 * s] for s in range(S))
    for h in hbs:
        h.close()
    b1.close()
    # single-frame latency through the reference ABI (one P NAL per call)
    lib = hs.lib
    cfg = hs.make_config(1280, 720)
    buf = (ctypes.c_uint8 * (1 << 20))()
    rb = (ctypes.c_uint8 * (1 << 20))()
    nw = hs.NALWriter()
    lat = []
    for k in range(60):
        lib.nal_writer_init(ctypes.byref(nw), buf, len(buf), rb, len(rb))
        ta = time.perf_counter()
        lib.h264_write_scroll_p_frame(ctypes.byref(nw), ctypes.byref(cfg), 4 * (k % 100))
        lat.append(time.perf_counter() - ta)
    lat = sorted(lat[10:])
    return {"value": round(S * F * steps / el, 1), "unit": "frames/s (PCIe-inclusive, pinned host memory)",
            "gb_per_s": round(delivered * steps / el / 1e9, 2), "bytes_per_step": int(delivered),
            "steps": steps, "ok": bool(ok and same),
            "how": "scroll_batch_output_to_host_async after each compose; two batches on two HIP streams",
            "single_frame_us": {"p50": round(1e6 * lat[len(lat) // 2], 1), "min": round(1e6 * lat[0], 1),
                                "api": "h264_write_scroll_p_frame 1280x720 (GPU round trip per call)",
                                "reference_cpu_us": "86-90 (BASELINE.md section 2, one core)"}}


def build_compose_batch(hs, wl, first, device):
    """the benched batch of a compose workload (p720dyn / p4kdyn / p720 /
    p720hint): streams first .. first + S - 1, SURVEY 8(d) offsets, the rect
    with one copy of the striped reference pictures per stream and the
    synthetic source on device, or the UI overlay"""
    S, F, W, H = wl["streams"], wl["frames"], wl["w"], wl["h"]
    rect = wl["rect"]
    per_frame_bound = 2 * (64 + (W // 16) * (H // 16))
    if rect:
        per_frame_bound += 192 * rect[2] * rect[3]      # ~75 B per dynamic MB measured
        per_frame_bound += 8 * (W // 16) * (H // 16)     # waypoint-heavy headers at 4K
    b = hs.Batch(S, F, F * per_frame_bound + (1 << 20), device=device)
    for _ in range(S):
        b.add_stream(hs.make_config(W, H))
    b.set_offsets(synthetic_offsets(first, S, F, H))
    if rect:
        b.set_dyn_rect(*rect)
        ra, rb = striped_i420(W, H, 0), striped_i420(W, H, 1)
        for s in range(S):                               # one copy per stream (own traffic)
            b.set_dyn_refs(ra, rb, stream=s)
        b.dyn_source_synth(F, stream_base=first, t0=0)
    if wl.get("hints"):
        for s in range(S):
            for f in range(F):
                b.set_hints(s, f, ui_hints(first + s, f, W, H), hs.SCROLL_HINT_PSKIP)
    return b


def verify_last_step(b, wl, first, passes, hint_streams=None):
    """CHECKER (runs after timing): the bytes of the last composed step
    against the CPU oracle (tests/stepcheck.py -> oracle/verify_oracle.c on
    all usable host cores).  Every stream (the UI overlay: every stream, or
    the first `hint_streams`, through the single-threaded hint oracle).
    -> (ok, detail)"""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import stepcheck
    t0 = time.perf_counter()
    S, F, W, H = wl["streams"], wl["frames"], wl["w"], wl["h"]
    offs = synthetic_offsets(first, S, F, H)
    oracle = stepcheck.load_oracle()
    if wl.get("hints"):
        want, ns = stepcheck.oracle_hint_step(oracle, W, H, offs[:hint_streams or S], passes,
                                              lambda s, f: ui_hints(first + s, f, W, H), 1)
        ok, d = stepcheck.compare_streams(b, want)
        d["sample"] = f"first {ns} of {S} streams"
    else:
        want = stepcheck.oracle_step(oracle, W, H, offs, passes, rect=wl["rect"],
                                     stream_base=first, t0=0, nthreads=usable_cores())
        ok, d = stepcheck.compare_streams(b, want)
        d["sample"] = f"all {S} streams of the rank"
    d["passes"] = passes
    d["seconds"] = round(time.perf_counter() - t0, 2)
    d["checker"] = "oracle/verify_oracle.c" if not wl.get("hints") else "oracle/hint_oracle.c"
    return ok, d



if __name__ == "__main__":
    main()
