"""Data path (kdfm/data.py + libkdfm_io.so): native FLAC/WAV decode, manifest reading, GigaSpeech text
rules, SentencePiece ids, NeMo collate and DistributedSampler sharding.  CPU only.

Pins: FLAC round trips through tests/flac_writer.py (every subframe / residual / stereo construct,
bit-exact samples, CRCs verified by the decoder); WAV against Python's ``wave`` module on a real
recording held by the reference (tests/golden/default_ipa.wav, from NeMo/tutorials/tts/
audio_samples/); the sampler against torch's own DistributedSampler.
"""
import json
import os
import struct
import wave

import numpy as np
import pytest
import torch

from kdfm import data as D

from flac_writer import encode, expected_mono

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from kdfm import _build
    _build.build_io()
    D.io_lib()


def _signal(n, bps, seed, ch=1):
    g = np.random.default_rng(seed)
    t = np.arange(n)
    lim = (1 << (bps - 1)) - 1
    out = []
    for c in range(ch):
        x = 0.4 * np.sin(2 * np.pi * (220 + 110 * c) * t / 16000) + 0.05 * g.standard_normal(n)
        out.append(np.clip(np.round(x * lim), -lim - 1, lim).astype(np.int64))
    return np.stack(out)


def _write(tmp_path, name, blob):
    p = tmp_path / name
    p.write_bytes(blob)
    return str(p)


def test_io_library_exports_every_symbol():
    lib = D.io_lib()
    for s in D.IO_SYMBOLS:
        assert hasattr(lib, s), s
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "kdfm_io.h")).read()
    for s in D.IO_SYMBOLS:
        assert s in hdr
    assert lib.kdfm_io_version().decode().startswith("kdfm_io")


@pytest.mark.parametrize("kind,order", [("verbatim", 0), ("fixed", 0), ("fixed", 1), ("fixed", 2), ("fixed", 3),
                                        ("fixed", 4), ("lpc", 1), ("lpc", 8), ("lpc", 12), ("lpc", 32)])
def test_flac_subframe_kinds_bit_exact(tmp_path, kind, order):
    x = _signal(3000, 16, order + 7)
    blob = encode(x, 16000, 16, 1152, plan=lambda f, c: {"kind": kind, "order": order, "porder": 2})
    p = _write(tmp_path, "a.flac", blob)
    got = D.load_audio(p)
    np.testing.assert_array_equal(got, expected_mono(x, 16))
    info = D.probe(p)
    assert (info.sample_rate, info.channels, info.bits_per_sample, info.frames) == (16000, 1, 16, 3000)


@pytest.mark.parametrize("bps", [8, 12, 16, 20, 24])
@pytest.mark.parametrize("rice2", [False, True])
def test_flac_sample_sizes_and_rice2(tmp_path, bps, rice2):
    x = _signal(2500, bps, bps)
    blob = encode(x, 16000, bps, 576, plan=lambda f, c: {"kind": "lpc" if f % 2 else "fixed", "order": 4,
                                                         "porder": f % 4, "rice2": rice2})
    got = D.load_audio(_write(tmp_path, "b.flac", blob))
    np.testing.assert_array_equal(got, expected_mono(x, bps))


@pytest.mark.parametrize("stereo", ["indep", "left_side", "side_right", "mid_side"])
def test_flac_stereo_modes_mono_mix(tmp_path, stereo):
    x = _signal(4100, 16, 3, ch=2)
    blob = encode(x, 16000, 16, 1024, stereo=stereo,
                  plan=lambda f, c: {"kind": ["fixed", "lpc", "verbatim"][(f + c) % 3], "order": 3, "porder": 1})
    got = D.load_audio(_write(tmp_path, "s.flac", blob))
    np.testing.assert_array_equal(got, expected_mono(x, 16))


def test_flac_constant_wasted_escape_and_explicit_blocksizes(tmp_path):
    x = _signal(5000, 16, 9)
    x[0, :1000] = 1234                      # constant frames
    x[0, 1000:2000] = (x[0, 1000:2000] >> 3) << 3   # 3 wasted bits
    blocks = {0: "constant"}

    def plan(f, c):
        if f == 0:
            return {"kind": "constant"}
        if f == 1:
            return {"kind": "fixed", "order": 2, "wasted": 3, "porder": 0}
        return {"kind": "fixed", "order": 1, "porder": 3, "escape_part": f % 8}
    # 1000-sample blocks: explicit 16-bit block size codes; the last block (1000) too; and an
    # 8-bit explicit code via a 200-sample stream
    blob = encode(x, 16000, 16, 1000, plan=plan)
    got = D.load_audio(_write(tmp_path, "c.flac", blob))
    np.testing.assert_array_equal(got, expected_mono(x, 16))
    y = _signal(700, 16, 10)
    blob = encode(y, 16000, 16, 200, plan=lambda f, c: {"kind": "fixed", "order": 2, "porder": 3},
                  header_ss_from_streaminfo=True)
    np.testing.assert_array_equal(D.load_audio(_write(tmp_path, "d.flac", blob)), expected_mono(y, 16))
    assert blocks


def test_flac_offset_duration_and_corruption(tmp_path):
    x = _signal(8000, 16, 11)
    blob = encode(x, 16000, 16, 1152, plan=lambda f, c: {"kind": "lpc", "order": 6, "porder": 2})
    p = _write(tmp_path, "o.flac", blob)
    full = expected_mono(x, 16)
    np.testing.assert_array_equal(D.load_audio(p, offset=0.1, duration=0.2), full[1600:4800])
    np.testing.assert_array_equal(D.load_audio(p, offset=0.45), full[7200:])
    bad = bytearray(blob)
    bad[len(bad) // 2] ^= 0x40
    q = _write(tmp_path, "bad.flac", bytes(bad))
    with pytest.raises(D.AudioIOError, match="CRC|corrupt|residual|subframe|reserved|mismatch"):
        D.load_audio(q)
    with pytest.raises(D.AudioIOError, match="cannot read"):
        D.load_audio(str(tmp_path / "missing.flac"))
    with pytest.raises(D.AudioIOError, match="not a RIFF"):
        D.load_audio(_write(tmp_path, "junk.wav", b"hello world, not audio"))


def test_wav_real_recording_matches_wave_module():
    p = os.path.join(GOLD, "default_ipa.wav")
    with wave.open(p) as w:
        raw = np.frombuffer(w.readframes(w.getnframes()), "<i2")
        sr = w.getframerate()
    got = D.load_audio(p)
    np.testing.assert_array_equal(got, raw.astype(np.float32) / np.float32(32768))
    info = D.probe(p)
    assert (info.sample_rate, info.channels, info.frames) == (sr, 1, raw.size)


def _wav_bytes(samples: np.ndarray, sr: int, fmt: int, bits: int, extensible=False) -> bytes:
    ch = samples.shape[0]
    inter = samples.T.reshape(-1)
    if fmt == 3:
        body = inter.astype("<f4" if bits == 32 else "<f8").tobytes()
    elif bits == 8:
        body = (inter + 128).astype(np.uint8).tobytes()
    elif bits == 24:
        v = inter.astype("<i4").tobytes()
        body = b"".join(v[i:i + 3] for i in range(0, len(v), 4))
    else:
        body = inter.astype("<i2" if bits == 16 else "<i4").tobytes()
    ba = ch * bits // 8
    if extensible:
        fmtc = struct.pack("<HHIIHHHHI", 0xFFFE, ch, sr, sr * ba, ba, bits, 22, bits, 0) + \
            struct.pack("<H", fmt) + b"\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
    else:
        fmtc = struct.pack("<HHIIHH", fmt, ch, sr, sr * ba, ba, bits)
    chunks = b"LIST" + struct.pack("<I", 3) + b"abc\x00"  # odd-sized chunk + pad byte
    chunks += b"fmt " + struct.pack("<I", len(fmtc)) + fmtc + b"data" + struct.pack("<I", len(body)) + body
    return b"RIFF" + struct.pack("<I", 4 + len(chunks)) + b"WAVE" + chunks


@pytest.mark.parametrize("fmt,bits,ext", [(1, 8, False), (1, 16, False), (1, 24, False), (1, 32, False),
                                          (3, 32, False), (3, 64, False), (1, 16, True), (3, 32, True)])
def test_wav_encodings_stereo(tmp_path, fmt, bits, ext):
    n = 1500
    if fmt == 3:
        x = np.random.default_rng(bits).uniform(-0.9, 0.9, (2, n))
        chans = [(x[c].astype(np.float32) if bits == 32 else x[c]).astype(np.float32) for c in range(2)]
    else:
        x = _signal(n, bits, bits, ch=2)
        scale = np.float32(1.0 / (1 << (bits - 1)))
        chans = [((x[c] - 0) .astype(np.float32) * scale) for c in range(2)]
    p = _write(tmp_path, "w.wav", _wav_bytes(x, 16000, fmt, bits, ext))
    want = (chans[0] + chans[1]) / np.float32(2)
    np.testing.assert_array_equal(D.load_audio(p), want)


def test_manifest_filters_relative_paths_and_text_rules(tmp_path):
    (tmp_path / "aud").mkdir()
    lines = [{"audio_filepath": "aud/a.flac", "duration": 0.05, "text": "too short"},
             {"audio_filepath": "aud/b.flac", "duration": 3.0, "text": "kept one"},
             {"audio_filepath": "/abs/c.flac", "duration": 20.0, "text": "too long"},
             {"audio_filepath": "aud/d.flac", "duration": 10.0, "text": "kept two", "offset": 1.5}]
    mp = tmp_path / "m.json"
    mp.write_text("\n".join(json.dumps(e) for e in lines) + "\n\n")
    es = D.read_manifest(str(mp), min_duration=0.1, max_duration=16.7)
    assert [e["text"] for e in es] == ["kept one", "kept two"]
    assert es[0]["audio_filepath"] == str(tmp_path / "aud" / "b.flac")
    assert es[1]["offset"] == 1.5
    assert len(D.read_manifest(f"{mp},{mp}", max_number=3)) == 3
    assert D.strip_special_tags("<COMMA> hello <music>  world <PERIOD>") == ("hello world", False)
    assert D.strip_special_tags("<NOISE> <SIL>") == ("", True)
    assert D.normalize_text_cv("Hello, World!  It's  OK.") == "hello world it's ok"
    assert D.normalize_librispeech("  HELLO World ") == "hello world"


def _toy_corpus(tmp_path, n=7, sr=16000):
    import sentencepiece as spm
    words = "the quick brown fox jumps over a lazy dog while seven wizards quietly hex bold jumping zebras".split()
    g = np.random.default_rng(0)
    texts = [" ".join(g.choice(words, size=int(g.integers(3, 9)))) for _ in range(n)]
    (tmp_path / "sp.txt").write_text("\n".join(texts * 20) + "\n")
    spm.SentencePieceTrainer.train(input=str(tmp_path / "sp.txt"), model_prefix=str(tmp_path / "sp"),
                                   vocab_size=40, model_type="bpe", character_coverage=1.0, minloglevel=2)
    paths, sigs = [], []
    for i in range(n):
        x = _signal(int(sr * (0.3 + 0.1 * i)), 16, 100 + i)
        sigs.append(expected_mono(x, 16))
        paths.append(_write(tmp_path, f"u{i}.flac", encode(x, sr, 16, 4096 if i % 2 else 1152)))
    mp = str(tmp_path / "train.json")
    assert D.manifest_from_audio(paths, texts, mp) == n
    return mp, D.SentencePieceTokenizer(str(tmp_path / "sp.model")), texts, sigs


def test_dataset_collate_and_native_batch_agree(tmp_path):
    mp, tok, texts, sigs = _toy_corpus(tmp_path)
    ds = D.AudioToBPEDataset(mp, tok, sample_rate=16000, max_duration=16.7, min_duration=0.1)
    assert len(ds) == len(texts)
    a, al, t, tl = ds[2]
    np.testing.assert_array_equal(a.numpy(), sigs[2])
    assert tok.ids_to_text(t.tolist()) == texts[2]
    ref = D.speech_collate_fn([ds[i] for i in (0, 3, 5)], pad_id=0)
    ld = D.ManifestBatchLoader(ds, 3, shuffle=False, threads=3)
    got = ld.load_host([0, 3, 5])
    for r, g in zip(ref, got):
        assert torch.equal(r, g)
    fixed = D.ManifestBatchLoader(ds, 3, shuffle=False, pad_to_samples=16000 * 2).load_host([0, 3, 5])
    assert fixed[0].shape == (3, 32000) and torch.equal(fixed[0][:, : ref[0].shape[1]], ref[0])
    assert float(fixed[0][:, ref[0].shape[1]:].abs().sum()) == 0.0
    with pytest.raises(D.AudioIOError, match="pad_to_samples"):
        D.ManifestBatchLoader(ds, 3, pad_to_samples=100).load_host([0])


@pytest.mark.parametrize("n,world,drop_last", [(10, 2, False), (11, 4, False), (11, 4, True), (3, 8, False)])
def test_distributed_indices_match_torch_sampler(n, world, drop_last):
    from torch.utils.data.distributed import DistributedSampler
    for rank in range(world):
        for shuffle in (False, True):
            s = DistributedSampler(list(range(n)), num_replicas=world, rank=rank, shuffle=shuffle, seed=7,
                                   drop_last=drop_last)
            s.set_epoch(3)
            assert D.distributed_indices(n, rank, world, shuffle, 7, 3, drop_last) == list(iter(s))


def test_loader_iterates_shards_and_surfaces_errors(tmp_path):
    mp, tok, texts, sigs = _toy_corpus(tmp_path)
    ds = D.AudioToBPEDataset(mp, tok)
    seen = []
    for rank in range(2):
        ld = D.ManifestBatchLoader(ds, 2, rank=rank, world_size=2, shuffle=True, seed=1, threads=2, prefetch=2)
        ld.set_epoch(1)
        for audio, al, tk, tl in ld:
            assert audio.shape[0] == tk.shape[0] == al.shape[0]
            for r in range(audio.shape[0]):
                L = int(al[r])
                hit = [i for i, s in enumerate(sigs) if s.size == L and np.array_equal(audio[r, :L].numpy(), s)]
                assert len(hit) == 1
                seen.append(hit[0])
                assert tok.ids_to_text(tk[r, : int(tl[r])].tolist()) == texts[hit[0]]
    assert sorted(set(seen)) == list(range(len(texts)))  # padded sampler may repeat one utterance
    os.remove(ds.entries[4]["audio_filepath"])
    ld = D.ManifestBatchLoader(ds, 7, shuffle=False)
    with pytest.raises(D.AudioIOError):
        for _ in ld:
            pass
