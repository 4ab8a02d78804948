#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ from the REFERENCE itself.

Run HERE (needs /root/reference):   make -C oracle ref && python tests/golden/make_golden.py

Everything written is data (inputs + expected outputs) produced by running the
reference C compiled from its own sources (oracle/_ref/).  The reference is
never copied into the repo and never travels to the GPU box; only these files do.

Outputs
  files/ipcm_64x48_{a,b}.h264        I_PCM striped refs (SURVEY App. B harness)
  files/composer_64x48_n40_s1.h264   reference `composer` CLI output
  md5.json                           md5 + size of larger whole-run outputs
  frames.jsonl                       single-frame cases: cfg + kind + offset -> NAL bytes
  streams.json                       synthetic streams: per-frame sizes + sha256
"""
import hashlib
import json
import os
import random
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref")


def run(*args, **kw):
    return subprocess.run(args, check=True, capture_output=True, **kw)


def md5(b):
    return hashlib.md5(b).hexdigest()


def main():
    if not os.path.exists(os.path.join(REF, "composer")):
        sys.exit("build the reference first: make -C oracle ref")
    os.makedirs(os.path.join(HERE, "files"), exist_ok=True)
    tmp = tempfile.mkdtemp()
    md5s = {}

    def ipcm(w, h, which):
        p = os.path.join(tmp, f"ipcm_{w}x{h}_{'ab'[which]}.h264")
        run(os.path.join(REF, "ref_ipcm"), str(w), str(h), str(which), p)
        return p

    # --- I_PCM refs + composer CLI runs ---
    for (w, h) in [(64, 48), (1280, 720), (3840, 2160)]:
        pa, pb = ipcm(w, h, 0), ipcm(w, h, 1)
        for p in (pa, pb):
            d = open(p, "rb").read()
            md5s[os.path.basename(p)] = {"bytes": len(d), "md5": md5(d)}
            if w == 64:
                open(os.path.join(HERE, "files", os.path.basename(p)), "wb").write(d)
        runs = {(64, 48): [(40, 1), (200, 3)], (1280, 720): [(250, 4), (360, 4), (500, 3)],
                (3840, 2160): [(1200, 4)]}[(w, h)]
        for (n, s) in runs:
            o = os.path.join(tmp, "out.h264")
            run(os.path.join(REF, "composer"), "--ref-a", pa, "--ref-b", pb,
                "-n", str(n), "-s", str(s), "-o", o)
            d = open(o, "rb").read()
            name = f"composer_{w}x{h}_n{n}_s{s}"
            md5s[name] = {"bytes": len(d), "md5": md5(d), "w": w, "h": h, "n": n, "s": s}
            if w == 64 and n == 40:
                open(os.path.join(HERE, "files", name + ".h264"), "wb").write(d)

    # --- experiment test-mode runs (config 1 and friends) ---
    for (w, h, n, sp) in [(1280, 720, 248, 1), (640, 480, 900, 1), (1280, 720, 900, 1),
                          (3840, 2160, 300, 8)]:
        o = os.path.join(tmp, "exp.h264")
        run(os.path.join(REF, "h264_scroll_encoder"), "-t", "-w", str(w), "-H", str(h),
            "-n", str(n), "-S", str(sp), "-o", o)
        d = open(o, "rb").read()
        md5s[f"experiment_{w}x{h}_n{n}_S{sp}"] = {"bytes": len(d), "md5": md5(d), "w": w,
                                                 "h": h, "n": n, "S": sp}
    json.dump(md5s, open(os.path.join(HERE, "md5.json"), "w"), indent=1, sort_keys=True)

    # --- single-frame cases through h264_write_* with arbitrary ComposerConfig ---
    rng = random.Random(20261015)
    cases = []

    def add_case(w, h, l2f, poct, l2p, dbf, fn, nwp, wps, kind, off):
        cases.append(dict(w=w, h=h, log2_mfn=l2f, poc_type=poct, log2_poc=l2p, deblock=dbf,
                          frame_num=fn, nwp=nwp, wp=wps, kind=kind, off=off))

    def rand_wps(h, nwp):
        wps = []
        for i in range(8):
            if rng.random() < 0.6:
                wo = 496 * rng.randint(1, max(1, (h + 600) // 496 + 1))
            else:
                wo = rng.randint(-200, h + 700)
            lt = 2 + i if rng.random() < 0.8 else rng.randint(0, 40)
            valid = 1 if (i < nwp and rng.random() < 0.85) else rng.randint(0, 1)
            wps.append([wo, lt, valid])
        return wps

    for k in range(900):
        if k < 700:
            mbw, mbh = rng.randint(1, 24), rng.randint(1, 20)
            w, h = 16 * mbw, 16 * mbh
            if rng.random() < 0.05:
                h += rng.randint(1, 15)         # non-multiple-of-16 cfg.height
        else:
            w, h = rng.choice([(1280, 720), (640, 480), (3840, 2160), (1920, 1088)])
        l2f = 4 if rng.random() < 0.7 else rng.randint(4, 16)
        poct = 2 if rng.random() < 0.7 else 0
        l2p = 4 if rng.random() < 0.6 else rng.randint(4, 16)
        dbf = 1 if rng.random() < 0.8 else 0
        fn = rng.randint(0, 40) if rng.random() < 0.8 else rng.randint(0, 10 ** 6)
        nwp = rng.choice([0, 0, 0, 1, 1, 2, 3, 4, 5, 6, 7, 8])
        wps = rand_wps(h, nwp)
        r = rng.random()
        if r < 0.25:
            off = 496 * rng.randint(0, max(1, h // 496 + 1))
        elif r < 0.85:
            off = rng.randint(0, h)
        elif r < 0.95:
            off = rng.randint(-h - 600, 2 * h + 600)
        else:
            off = rng.randint(-(1 << 26), 1 << 26)   # huge MVs: long Exp-Golomb codes
        kind = rng.choice([0, 0, 1, 2, 2])
        add_case(w, h, l2f, poct, l2p, dbf, fn, nwp, wps, kind, off)
    # emulation-prevention forcing cases: long zero runs in frame_num/poc fields
    for fn in (0, 1 << 16, 1 << 15):
        for kind in (0, 1, 2):
            add_case(48, 32, 16, 0, 16, 1, fn, 0, rand_wps(32, 0), kind, 5)
            add_case(160, 96, 16, 0, 16, 0, fn, 2, rand_wps(96, 2), kind, 600)

    inp = "\n".join(
        " ".join(str(v) for v in [c["w"], c["h"], c["log2_mfn"], c["poc_type"], c["log2_poc"],
                                   c["deblock"], c["frame_num"], c["nwp"]]
                 + [x for t in c["wp"] for x in t] + [c["kind"], c["off"]])
        for c in cases) + "\n"
    out = run(os.path.join(REF, "ref_frames"), input=inp.encode()).stdout.decode().split("\n")
    n_ep = 0
    with open(os.path.join(HERE, "frames.jsonl"), "w") as f:
        for c, line in zip(cases, out):
            hx, fn_after, nwp_after = line.split()
            b = bytes.fromhex(hx)
            c["frame_num_after"], c["nwp_after"] = int(fn_after), int(nwp_after)
            c["bytes"] = len(b)
            c["sha256"] = hashlib.sha256(b).hexdigest()
            if len(b) <= 2048:
                c["hex"] = hx
            # does the reference output contain emulation-prevention bytes?
            c["has_ep"] = any(b[i] == 0 and b[i + 1] == 0 and b[i + 2] == 3
                              for i in range(5, len(b) - 2))
            n_ep += c["has_ep"]
            f.write(json.dumps(c) + "\n")
    print(f"frames.jsonl: {len(cases)} cases, {n_ep} with emulation prevention")

    # --- synthetic streams through composer_write_scroll_frame semantics ---
    streams = []
    for (w, h, sids, nf) in [(1280, 720, range(0, 24), 1500), (3840, 2160, [0, 3, 7, 13], 900),
                             (64, 48, range(0, 8), 300), (352, 288, range(0, 8), 700)]:
        for s in sids:
            lines = run(os.path.join(REF, "ref_stream"), str(w), str(h), str(s),
                        str(nf)).stdout.decode().split()
            frames = [bytes.fromhex(x) for x in lines]
            hsh = hashlib.sha256(b"".join(frames)).hexdigest()
            streams.append(dict(w=w, h=h, stream=s, nframes=nf, sizes=[len(x) for x in frames],
                                sha256=hsh))
    json.dump(streams, open(os.path.join(HERE, "streams.json"), "w"))
    print(f"streams.json: {len(streams)} streams")


if __name__ == "__main__":
    main()
