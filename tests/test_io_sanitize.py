"""Host AddressSanitizer + UndefinedBehaviorSanitizer run of the native audio decoder (SURVEY.md §5:
libkdfm_io parses untrusted FLAC / WAV bit streams).  CPU only.

tests/sanitize/io_fuzz.cpp is compiled together with csrc/audio_io.cpp (the library source, not the
shipped .so) under -fsanitize=address,undefined -fno-sanitize-recover=all and fed:
  - a corpus written here with tests/flac_writer.py (every subframe kind, Rice2 + escapes, all four
    stereo decorrelations, wasted bits, 8..24-bit samples) plus RIFF WAV in every encoding the
    decoder takes and the real recording tests/golden/default_ipa.wav;
  - seeded corruptions of each file (bit flips, stomps, truncations, extreme length fields).
Pass = every valid file decodes, short output buffers are refused, the 4-thread collate zero-pads,
and no sanitizer report (any report aborts the driver with a non-zero status).
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from flac_writer import encode

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(ROOT, "kd-via-fm-in-asr_amd", "csrc", "audio_io.cpp")
DRIVER = os.path.join(HERE, "sanitize", "io_fuzz.cpp")


def _signal(n, bps, seed, ch=1):
    g = np.random.default_rng(seed)
    t = np.arange(n)
    lim = (1 << (bps - 1)) - 1
    x = [0.4 * np.sin(2 * np.pi * (220 + 110 * c) * t / 16000) + 0.05 * g.standard_normal(n) for c in range(ch)]
    return np.stack([np.clip(np.round(v * lim), -lim - 1, lim).astype(np.int64) for v in x])


def _corpus(d):
    from test_data import _wav_bytes
    files = []

    def put(name, blob):
        p = os.path.join(d, name)
        with open(p, "wb") as fh:
            fh.write(blob)
        files.append(p)
    for i, (kind, order) in enumerate([("verbatim", 0), ("fixed", 2), ("lpc", 8), ("lpc", 32)]):
        put(f"k{i}.flac", encode(_signal(2000, 16, i), 16000, 16, 576,
                                 plan=lambda f, c, k=kind, o=order: {"kind": k, "order": o, "porder": 2}))
    for bps in (8, 12, 24):
        put(f"b{bps}.flac", encode(_signal(1500, bps, bps), 16000, bps, 512,
                                   plan=lambda f, c: {"kind": "lpc", "order": 4, "porder": f % 4, "rice2": True}))
    for st in ("indep", "left_side", "side_right", "mid_side"):
        put(f"s_{st}.flac", encode(_signal(1800, 16, 3, ch=2), 16000, 16, 1024, stereo=st,
                                   plan=lambda f, c: {"kind": ["fixed", "lpc", "verbatim"][(f + c) % 3],
                                                      "order": 3, "porder": 1}))
    x = _signal(3000, 16, 9)
    x[0, :1000] = 77
    x[0, 1000:2000] = (x[0, 1000:2000] >> 2) << 2   # 2 wasted bits in the second block

    def plan(f, c):
        if f == 0:
            return {"kind": "constant"}
        if f == 1:
            return {"kind": "fixed", "order": 2, "wasted": 2, "porder": 0}
        return {"kind": "fixed", "order": 1, "porder": 3, "escape_part": f % 8}
    put("cwe.flac", encode(x, 16000, 16, 1000, plan=plan))
    for fmt, bits, ext in [(1, 8, False), (1, 16, False), (1, 24, False), (1, 32, False), (3, 32, False),
                           (3, 64, False), (1, 16, True)]:
        s = (np.random.default_rng(bits).uniform(-0.9, 0.9, (2, 900)) if fmt == 3 else _signal(900, bits, bits, 2))
        put(f"w{fmt}_{bits}_{int(ext)}.wav", _wav_bytes(s, 16000, fmt, bits, ext))
    files.append(os.path.join(HERE, "golden", "default_ipa.wav"))
    return files


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_audio_io_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "io_fuzz")
    inc = os.path.join(ROOT, "include")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all", f"-I{inc}", DRIVER, SRC, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    files = _corpus(str(tmp_path))
    scratch = tmp_path / "scratch"
    scratch.mkdir()
    # verify_asan_link_order=0: the environment may preload a library ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, "150", "20261016", str(scratch), *files], capture_output=True, text=True, env=env,
                       timeout=600)
    report = (r.stdout + r.stderr)[-6000:]
    assert r.returncode == 0, report
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, report
    assert r.stdout.startswith(f"files {len(files)} "), report
    # the corruptions must actually exercise the error paths
    rejected = int(r.stdout.split("mutated-rejected")[1])
    assert rejected > 100, r.stdout
