"""Manifest data path for the ver5 step: JSONL manifest -> native FLAC/WAV decode -> SentencePiece
ids -> padded batch in pinned memory -> device.

The reference trains from NeMo manifests (one JSON object per line with ``audio_filepath``,
``duration``, ``text``) that it writes itself:

* LibriSpeech: ``build_manifest_from_hf`` (asr_train_diffm.py:31-88) — text ``lower().strip()``.
* GigaSpeech: ``build_manifest_from_hf_gigaspeech`` (asr_train_diffm_GS.py:35-178) — special tags
  (``<COMMA>``, ``<MUSIC>`` ...) stripped, tag-only utterances and clips < 1 s skipped, then
  ``normalize_text_cv(text, keep_punct=False)``.

and feeds them to NeMo's ``AudioToBPEDataset`` (built by ctc_bpe_models.py:96-165; the dataset and
collate sources are absent from the reference) through a ``torch.utils.data.DataLoader``
(ctc_models.py:370-380; ``num_workers`` 8, ``pin_memory``, ``max_duration`` 16.7,
``min_duration`` 0.1, conformer_ctc_bpe.yaml:33-43).

Here the decode + pad of a whole batch is ONE native call (libkdfm_io.so, include/kdfm_io.h) that
runs B decodes on host threads straight into a pinned staging buffer (no per-sample tensors, no
worker processes, ctypes drops the GIL for the call); a prefetch thread keeps ``prefetch`` batches
ahead and the H2D copy is issued on its own HIP stream so it overlaps the previous step.
Rank sharding follows ``torch.utils.data.DistributedSampler`` (seeded per-epoch permutation, padded
to a multiple of world size, strided by rank) — the sampler Lightning installs under DDP.

Module API (NeMo names): ``read_manifest``, ``AudioToBPEDataset`` (``__getitem__`` ->
``(signal, signal_len, tokens, tokens_len)``), ``speech_collate_fn``, ``SentencePieceTokenizer``;
the production loader is ``ManifestBatchLoader``.  Nothing here imports ``oracle/``.
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
import queue
import re
import threading
from dataclasses import dataclass
from typing import Iterator, List, Optional, Sequence

import numpy as np
import torch

IO_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libkdfm_io.so")

_io = None
_io_lock = threading.Lock()


class AudioIOError(RuntimeError):
    """A native decode failed (status + the library's message)."""


def io_lib() -> C.CDLL:
    """Load libkdfm_io.so (built by ``kdfm._build.build_io``).  No fallback: missing -> raises."""
    global _io
    with _io_lock:
        if _io is None:
            if not os.path.exists(IO_LIB_PATH):
                raise AudioIOError(f"{IO_LIB_PATH} is missing: run __graft_entry__.build()")
            lib = C.CDLL(IO_LIB_PATH)
            P, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
            lib.kdfm_audio_probe.argtypes = [C.c_char_p, P, P, P, P]
            lib.kdfm_audio_decode.argtypes = [C.c_char_p, i64, i64, P, i64, P, P]
            lib.kdfm_audio_load_batch.argtypes = [P, i32, P, P, P, i64, P, i32, i32]
            for f in ("kdfm_audio_probe", "kdfm_audio_decode", "kdfm_audio_load_batch"):
                getattr(lib, f).restype = C.c_int
            lib.kdfm_io_last_error.restype = C.c_char_p
            lib.kdfm_io_last_error.argtypes = []
            lib.kdfm_io_version.restype = C.c_char_p
            lib.kdfm_io_version.argtypes = []
            _io = lib
    return _io


IO_SYMBOLS = ("kdfm_audio_probe", "kdfm_audio_decode", "kdfm_audio_load_batch", "kdfm_io_last_error",
              "kdfm_io_version")


def _check(rc: int) -> None:
    if rc != 0:
        raise AudioIOError(f"kdfm_io status {rc}: {io_lib().kdfm_io_last_error().decode(errors='replace')}")


@dataclass
class AudioInfo:
    sample_rate: int
    channels: int
    bits_per_sample: int
    frames: int

    @property
    def duration(self) -> float:
        return self.frames / float(self.sample_rate)


def probe(path: str) -> AudioInfo:
    """soundfile.info equivalent (asr_train_diffm_GS.py:85-87)."""
    sr, ch, bits, n = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
    _check(io_lib().kdfm_audio_probe(os.fsencode(path), C.byref(sr), C.byref(ch), C.byref(bits), C.byref(n)))
    return AudioInfo(sr.value, ch.value, bits.value, n.value)


def load_audio(path: str, offset: float = 0.0, duration: Optional[float] = None,
               target_sr: Optional[int] = None) -> np.ndarray:
    """Mono float32 samples of one file: NeMo ``AudioSegment.from_file(path, offset, duration)``
    (soundfile float32 read, channel mean).  ``target_sr`` must equal the file's rate — resampling
    is not part of this path (the reference trains on 16 kHz corpora, asr_train_diffm.py:1443)."""
    info = probe(path)
    if target_sr is not None and info.sample_rate != target_sr:
        raise AudioIOError(f"{path}: sample rate {info.sample_rate} != {target_sr} (no resampling)")
    off = int(round(offset * info.sample_rate))
    nmax = -1 if duration is None else int(round(duration * info.sample_rate))
    cap = max(0, info.frames - off) if nmax < 0 else max(0, min(nmax, info.frames - off))
    out = np.zeros(cap, np.float32)
    n = C.c_int64()
    _check(io_lib().kdfm_audio_decode(os.fsencode(path), off, nmax, out.ctypes.data if cap else None, cap,
                                      C.byref(n), None))
    return out[: n.value]


# ------------------------------------------------------------------------------------------------
# text normalisation used by the reference's manifest writers

BANNED_TAGS = ("<MUSIC>", "<COMMA>", "<NOISE>", "<VOCALIZED_NOISE>", "<LAUGHTER>", "<SPOKEN_NOISE>",
               "<PERIOD>", "<QUESTION_MARK>", "<EXCLAMATION_MARK>", "<SEMICOLON>", "<COLON>", "<DASH>",
               "<ELLIPSIS>", "<SIL>", "<OTHER>")  # asr_train_diffm_GS.py:50-54
_TAGS_RE = re.compile("(?:%s)" % "|".join(re.escape(t) for t in BANNED_TAGS), re.IGNORECASE)


def strip_special_tags(text: str) -> tuple:
    """``_strip_special_tags`` (asr_train_diffm_GS.py:60-71): remove GigaSpeech tags, collapse
    whitespace; returns ``(text, is_tag_only)``."""
    if not text:
        return "", True
    no_tags = re.sub(r"\s+", " ", _TAGS_RE.sub(" ", text)).strip()
    return no_tags, len(no_tags) == 0


def normalize_text_cv(text: str, keep_punct: bool = False) -> str:
    """The reference CALLS ``normalize_text_cv`` (asr_train_diffm_GS.py:167) but never defines it
    (latent NameError).  Restated as the CommonVoice-style normaliser its name and
    call describe: lower-case, drop punctuation except apostrophes unless ``keep_punct``, collapse
    whitespace.  Parity unpinned (no definition exists to pin against)."""
    t = text.lower()
    if not keep_punct:
        t = re.sub(r"[^\w\s']", " ", t)
        t = t.replace("_", " ")
    return re.sub(r"\s+", " ", t).strip()


def normalize_librispeech(text: str) -> str:
    """``sample["text"].lower().strip()`` (asr_train_diffm.py:85)."""
    return text.lower().strip()


# ------------------------------------------------------------------------------------------------
# manifests

def read_manifest(manifest_filepath, min_duration: Optional[float] = None, max_duration: Optional[float] = None,
                  max_number: int = -1) -> List[dict]:
    """NeMo manifest reading (``collections.ASRAudioText`` over ``manifest.item_iter``): one JSON object
    per line, comma-separated or list of manifest paths, relative ``audio_filepath`` resolved
    against the manifest's directory, entries outside [min_duration, max_duration] dropped,
    at most ``max_number`` kept (``max_utts``)."""
    paths = manifest_filepath.split(",") if isinstance(manifest_filepath, str) else list(manifest_filepath)
    out: List[dict] = []
    for mp in paths:
        base = os.path.dirname(os.path.abspath(mp))
        with open(mp, encoding="utf-8") as f:
            for ln, line in enumerate(f, 1):
                line = line.strip()
                if not line:
                    continue
                try:
                    e = json.loads(line)
                except json.JSONDecodeError as ex:
                    raise ValueError(f"{mp}:{ln}: not JSON: {ex}") from None
                if "audio_filepath" not in e or "duration" not in e:
                    raise ValueError(f"{mp}:{ln}: manifest entry needs audio_filepath and duration")
                dur = float(e["duration"])
                if min_duration is not None and dur < min_duration:
                    continue
                if max_duration is not None and dur > max_duration:
                    continue
                ap = os.path.expanduser(e["audio_filepath"])
                if not os.path.isabs(ap):
                    ap = os.path.join(base, ap)
                out.append({"audio_filepath": ap, "duration": dur, "text": e.get("text", ""),
                            "offset": float(e.get("offset", 0.0) or 0.0)})
                if 0 < max_number <= len(out):
                    return out
    return out


def write_manifest(manifest_path: str, entries: Sequence[dict]) -> None:
    """JSONL writer with the reference's keys (asr_train_diffm.py:81-86)."""
    d = os.path.dirname(manifest_path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(manifest_path, "w", encoding="utf-8") as f:
        for e in entries:
            f.write(json.dumps({"audio_filepath": e["audio_filepath"], "duration": float(e["duration"]),
                                "text": e["text"]}, ensure_ascii=False) + "\n")


def manifest_from_audio(paths: Sequence[str], texts: Sequence[str], manifest_path: str,
                        normalize=normalize_librispeech, min_sec: float = 0.0) -> int:
    """Write a manifest for local audio files, durations from the native probe (the offline
    analogue of build_manifest_from_hf / _gigaspeech: no HF download).  Returns lines written."""
    entries = []
    for p, t in zip(paths, texts):
        info = probe(p)
        if info.duration < min_sec:
            continue
        entries.append({"audio_filepath": p, "duration": info.duration, "text": normalize(t)})
    write_manifest(manifest_path, entries)
    return len(entries)


# ------------------------------------------------------------------------------------------------
# tokenizer

class SentencePieceTokenizer:
    """NeMo ``SentencePieceTokenizer`` surface used by the BPE CTC path: ``text_to_ids``,
    ``ids_to_text``, ``vocab_size``, ``pad_id`` (the CTC blank is ``vocab_size``, losses/ctc.py:46)."""

    def __init__(self, model_path: str):
        import sentencepiece as spm
        self.model_path = model_path
        self.tokenizer = spm.SentencePieceProcessor(model_file=model_path)
        self.vocab_size = self.tokenizer.get_piece_size()
        self.pad_id = self.tokenizer.pad_id()

    def text_to_ids(self, text: str) -> List[int]:
        return list(self.tokenizer.encode_as_ids(text))

    def ids_to_text(self, ids) -> str:
        return self.tokenizer.decode_ids([int(i) for i in ids])

    def text_to_tokens(self, text: str) -> List[str]:
        return list(self.tokenizer.encode_as_pieces(text))


# ------------------------------------------------------------------------------------------------
# dataset + collate (module API)

class AudioToBPEDataset:
    """NeMo ``AudioToBPEDataset`` contract: ``__getitem__(i) -> (f32[N], i64 len, i64[U], i64 U)``."""

    def __init__(self, manifest_filepath, tokenizer, sample_rate: int = 16000, max_duration: Optional[float] = None,
                 min_duration: Optional[float] = None, max_utts: int = 0, use_start_end_token: bool = False,
                 trim: bool = False):
        if trim:
            raise NotImplementedError("trim_silence is off in every reference config (conformer_ctc_bpe.yaml:41)")
        self.sample_rate = sample_rate
        self.tokenizer = tokenizer
        self.entries = read_manifest(manifest_filepath, min_duration, max_duration, max_utts if max_utts > 0 else -1)
        self.use_start_end_token = use_start_end_token
        self._tok_cache: dict = {}

    def __len__(self) -> int:
        return len(self.entries)

    def tokens(self, i: int) -> List[int]:
        t = self._tok_cache.get(i)
        if t is None:
            t = self.tokenizer.text_to_ids(self.entries[i]["text"])
            if self.use_start_end_token:
                t = [self.tokenizer.tokenizer.bos_id()] + t + [self.tokenizer.tokenizer.eos_id()]
            self._tok_cache[i] = t
        return t

    def __getitem__(self, i: int):
        e = self.entries[i]
        dur = e["duration"] if e["offset"] > 0 else None
        a = torch.from_numpy(load_audio(e["audio_filepath"], e["offset"], dur, self.sample_rate))
        t = torch.tensor(self.tokens(i), dtype=torch.int64)
        return a, torch.tensor(a.numel(), dtype=torch.int64), t, torch.tensor(t.numel(), dtype=torch.int64)


def speech_collate_fn(batch, pad_id: int = 0):
    """NeMo ``_speech_collate_fn``: zero-pad audio to the longest signal, pad tokens with
    ``pad_id`` to the longest transcript; returns ``(audio, audio_len, tokens, tokens_len)``."""
    a_len = torch.stack([b[1] for b in batch])
    t_len = torch.stack([b[3] for b in batch])
    N = int(a_len.max()) if len(batch) else 0
    U = int(t_len.max()) if len(batch) else 0
    audio = torch.zeros(len(batch), N, dtype=torch.float32)
    toks = torch.full((len(batch), U), pad_id, dtype=torch.int64)
    for i, b in enumerate(batch):
        audio[i, : b[0].numel()] = b[0]
        toks[i, : b[2].numel()] = b[2]
    return audio, a_len, toks, t_len


# ------------------------------------------------------------------------------------------------
# production loader

def distributed_indices(n: int, rank: int, world_size: int, shuffle: bool, seed: int, epoch: int,
                        drop_last: bool = False) -> List[int]:
    """``torch.utils.data.DistributedSampler.__iter__`` semantics."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g).tolist()
    else:
        idx = list(range(n))
    if drop_last and n % world_size:
        num = math.ceil((n - world_size) / world_size)
    else:
        num = math.ceil(n / world_size)
    total = num * world_size
    if not drop_last:
        pad = total - len(idx)
        if pad > 0:
            idx += (idx * math.ceil(pad / max(1, len(idx))))[:pad]
    else:
        idx = idx[:total]
    return idx[rank:total:world_size]


class ManifestBatchLoader:
    """Sharded, prefetching batch loader: ``for audio, audio_len, tokens, tokens_len in loader``.

    Per batch: one ``kdfm_audio_load_batch`` call decodes the B files on ``threads`` host threads
    into a pinned (B, N) staging buffer; tokens come from the (cached) SentencePiece ids; the
    tensors are copied to ``device`` with ``non_blocking`` on a dedicated copy stream and the
    consumer's current stream waits on that copy.  ``pad_to_samples`` fixes N (static shapes for
    HIP-graph capture; e.g. ``max_duration * sample_rate``); otherwise N = longest in the batch,
    as NeMo's collate does.  ``drop_last`` defaults to the DataLoader's False."""

    def __init__(self, dataset: AudioToBPEDataset, batch_size: int, rank: int = 0, world_size: int = 1,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False, threads: int = 8,
                 device: Optional[str] = None, prefetch: int = 2, pad_to_samples: Optional[int] = None,
                 pad_id: int = 0):
        if batch_size <= 0:
            raise ValueError("batch_size must be positive")
        self.ds = dataset
        self.batch_size = batch_size
        self.rank, self.world_size = rank, world_size
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.threads = threads
        self.device = torch.device(device) if device is not None else None
        self.prefetch = max(1, prefetch)
        self.pad_to = pad_to_samples
        self.pad_id = pad_id
        self.epoch = 0
        self._frames = [None] * len(dataset)
        self._copy_stream = None

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def _batches(self) -> List[List[int]]:
        idx = distributed_indices(len(self.ds), self.rank, self.world_size, self.shuffle, self.seed, self.epoch)
        bs = [idx[i:i + self.batch_size] for i in range(0, len(idx), self.batch_size)]
        if self.drop_last and bs and len(bs[-1]) < self.batch_size:
            bs.pop()
        return bs

    def __len__(self) -> int:
        return len(self._batches())

    def _span(self, i: int):
        """(offset frames, max frames, frames) of entry i, from the native probe (cached)."""
        f = self._frames[i]
        if f is None:
            e = self.ds.entries[i]
            info = probe(e["audio_filepath"])
            if info.sample_rate != self.ds.sample_rate:
                raise AudioIOError(f"{e['audio_filepath']}: sample rate {info.sample_rate} != {self.ds.sample_rate}")
            off = int(round(e["offset"] * info.sample_rate))
            nmax = int(round(e["duration"] * info.sample_rate)) if e["offset"] > 0 else -1
            n = max(0, info.frames - off) if nmax < 0 else max(0, min(nmax, info.frames - off))
            f = (off, nmax, n)
            self._frames[i] = f
        return f

    def load_host(self, ids: Sequence[int]):
        """Decode + collate one batch into pinned host tensors (no device work)."""
        spans = [self._span(i) for i in ids]
        N = max((s[2] for s in spans), default=0)
        if self.pad_to is not None:
            if N > self.pad_to:
                raise AudioIOError(f"utterance of {N} samples exceeds pad_to_samples={self.pad_to}")
            N = self.pad_to
        B = len(ids)
        pin = torch.cuda.is_available()
        audio = torch.empty(B, N, dtype=torch.float32, pin_memory=pin)
        a_len = torch.empty(B, dtype=torch.int64, pin_memory=pin)
        paths = (C.c_char_p * B)(*[os.fsencode(self.ds.entries[i]["audio_filepath"]) for i in ids])
        offs = np.array([s[0] for s in spans], np.int64)
        nmax = np.array([s[1] for s in spans], np.int64)
        _check(io_lib().kdfm_audio_load_batch(C.cast(paths, C.c_void_p), B, offs.ctypes.data, nmax.ctypes.data,
                                              audio.data_ptr(), N, a_len.data_ptr(), self.ds.sample_rate,
                                              self.threads))
        toks = [self.ds.tokens(i) for i in ids]
        U = max((len(t) for t in toks), default=0)
        tk = torch.full((B, U), self.pad_id, dtype=torch.int64)
        for r, t in enumerate(toks):
            if t:
                tk[r, : len(t)] = torch.tensor(t, dtype=torch.int64)
        t_len = torch.tensor([len(t) for t in toks], dtype=torch.int64)
        if pin:
            tk, t_len = tk.pin_memory(), t_len.pin_memory()
        return audio, a_len, tk, t_len

    def _to_device(self, host):
        if self.device is None or self.device.type != "cuda":
            return host
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(device=self.device)
        with torch.cuda.stream(self._copy_stream):
            dev = tuple(t.to(self.device, non_blocking=True) for t in host)
        ev = torch.cuda.Event()
        ev.record(self._copy_stream)
        return dev, ev, host

    def __iter__(self) -> Iterator:
        batches = self._batches()
        q: "queue.Queue" = queue.Queue(maxsize=self.prefetch)
        stop = threading.Event()

        def producer():
            try:
                for ids in batches:
                    if stop.is_set():
                        return
                    q.put(("ok", self.load_host(ids)))
                q.put(("end", None))
            except BaseException as ex:  # surfaced in the consumer
                q.put(("err", ex))

        th = threading.Thread(target=producer, name="kdfm-data", daemon=True)
        th.start()
        try:
            while True:
                kind, item = q.get()
                if kind == "end":
                    return
                if kind == "err":
                    raise item
                out = self._to_device(item)
                if isinstance(out, tuple) and len(out) == 3 and isinstance(out[1], torch.cuda.Event):
                    dev, ev, host = out
                    torch.cuda.current_stream(self.device).wait_event(ev)
                    for t in dev:  # the pinned source must outlive the async copy
                        t.record_stream(torch.cuda.current_stream(self.device))
                    yield dev
                else:
                    yield out
        finally:
            stop.set()
            while th.is_alive():
                try:
                    q.get_nowait()
                except queue.Empty:
                    th.join(timeout=0.05)
