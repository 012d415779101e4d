"""Test infrastructure: a small FLAC *encoder* (pure Python + numpy) that emits every construct the
native decoder (csrc/audio_io.cpp) must handle — CONSTANT / VERBATIM / FIXED(0..4) / LPC subframes,
Rice and Rice2 residuals with several partition orders and escape partitions, wasted bits, the
four channel assignments, explicit 8/16-bit block-size codes, 8/12/16/20/24-bit samples.

There is no FLAC encoder or decoder in this image (no soundfile/libFLAC/ffmpeg), so the decoder is
pinned by round trips through this writer, whose output is the format's published bitstream layout
(frame header with CRC-8, CRC-16 footer) — parity against libFLAC itself is unpinned.
"""
from __future__ import annotations

import numpy as np


class BitWriter:
    def __init__(self):
        self.acc = 0
        self.n = 0

    def put(self, v: int, k: int) -> None:
        if k:
            self.acc = (self.acc << k) | (int(v) & ((1 << k) - 1))
            self.n += k

    def sput(self, v: int, k: int) -> None:
        self.put(int(v) & ((1 << k) - 1), k)

    def unary(self, q: int) -> None:
        self.put(1, q + 1)

    def align(self) -> None:
        if self.n % 8:
            self.put(0, 8 - self.n % 8)

    def bytes(self) -> bytes:
        assert self.n % 8 == 0
        return self.acc.to_bytes(self.n // 8, "big") if self.n else b""


def crc8(data: bytes) -> int:
    c = 0
    for b in data:
        c ^= b
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(data: bytes) -> int:
    c = 0
    for b in data:
        c ^= b << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def _utf8_num(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    for extra, lim in ((1, 1 << 11), (2, 1 << 16), (3, 1 << 21), (4, 1 << 26), (5, 1 << 31)):
        if n < lim:
            out = []
            for _ in range(extra):
                out.append(0x80 | (n & 0x3F))
                n >>= 6
            lead = ((0xFF << (7 - extra)) & 0xFF) | n
            return bytes([lead] + out[::-1])
    raise ValueError(n)


def _residual(bw: BitWriter, res: np.ndarray, order: int, bs: int, porder: int, rice2: bool, escape_part: int):
    bw.put(1 if rice2 else 0, 2)
    bw.put(porder, 4)
    pbits, esc = (5, 31) if rice2 else (4, 15)
    psize = bs >> porder
    pos = 0
    for p in range(1 << porder):
        n = psize - order if p == 0 else psize
        part = [int(x) for x in res[pos:pos + n]]
        pos += n
        if p == escape_part:
            mx = max((abs(x) for x in part), default=0)
            nb = (mx.bit_length() + 1) if mx else 0
            bw.put(esc, pbits)
            bw.put(nb, 5)
            for x in part:
                bw.sput(x, nb)
            continue
        us = [(x << 1) if x >= 0 else ((-x) << 1) - 1 for x in part]
        mean = (sum(us) / len(us)) if us else 0
        k = max(0, min(esc - 1, int(mean).bit_length() - 1 if mean >= 1 else 0))
        bw.put(k, pbits)
        for u in us:
            bw.unary(u >> k)
            bw.put(u & ((1 << k) - 1), k)


FIXED = {0: [], 1: [1], 2: [2, -1], 3: [3, -3, 1], 4: [4, -6, 4, -1]}


def _subframe(bw: BitWriter, x: np.ndarray, bps: int, kind: str, order: int, porder: int, rice2: bool,
              escape_part: int, wasted: int, lpc_prec: int, lpc_shift: int):
    x = [int(v) for v in x]
    bs = len(x)
    if wasted:
        assert all(v % (1 << wasted) == 0 for v in x)
        x = [v >> wasted for v in x]
    sb = bps - wasted
    bw.put(0, 1)
    if kind == "constant":
        assert all(v == x[0] for v in x)
        bw.put(0, 6)
    elif kind == "verbatim":
        bw.put(1, 6)
    elif kind == "fixed":
        bw.put(8 + order, 6)
    elif kind == "lpc":
        bw.put(32 + order - 1, 6)
    else:
        raise ValueError(kind)
    if wasted:
        bw.put(1, 1)
        bw.unary(wasted - 1)
    else:
        bw.put(0, 1)
    if kind == "constant":
        bw.sput(x[0], sb)
        return
    if kind == "verbatim":
        for v in x:
            bw.sput(v, sb)
        return
    for v in x[:order]:
        bw.sput(v, sb)
    if kind == "fixed":
        c = FIXED[order]
        res = [x[i] - sum(c[j] * x[i - 1 - j] for j in range(order)) for i in range(order, bs)]
    else:
        xf = np.asarray(x, np.float64)
        A = np.stack([xf[order - 1 - j: bs - 1 - j] for j in range(order)], 1)
        coef, *_ = np.linalg.lstsq(A, xf[order:], rcond=None)
        lim = (1 << (lpc_prec - 1)) - 1
        qc = [int(max(-lim - 1, min(lim, round(c * (1 << lpc_shift))))) for c in coef]
        bw.put(lpc_prec - 1, 4)
        bw.sput(lpc_shift, 5)
        for c in qc:
            bw.sput(c, lpc_prec)
        res = [x[i] - (sum(qc[j] * x[i - 1 - j] for j in range(order)) >> lpc_shift) for i in range(order, bs)]
    _residual(bw, np.asarray(res, dtype=object), order, bs, porder, rice2, escape_part)


_BS_CODES = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12}
_SS_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6}


def encode(chans: np.ndarray, rate: int, bps: int, block: int, plan=None, stereo: str = "indep",
           header_ss_from_streaminfo: bool = False) -> bytes:
    """chans: (C, N) int array.  ``plan(frame_index, channel) -> dict`` of subframe options
    (kind, order, porder, rice2, escape_part, wasted, lpc_prec, lpc_shift)."""
    chans = np.asarray(chans, np.int64)
    C, N = chans.shape
    out = bytearray(b"fLaC")
    si = BitWriter()
    si.put(block, 16)
    si.put(block, 16)
    si.put(0, 24)
    si.put(0, 24)
    si.put(rate, 20)
    si.put(C - 1, 3)
    si.put(bps - 1, 5)
    si.put(N, 36)
    si.put(0, 128)
    body = si.bytes()
    out += bytes([0x80 | 0]) + len(body).to_bytes(3, "big") + body
    plan = plan or (lambda f, c: {"kind": "fixed", "order": 2})
    for fi, s in enumerate(range(0, N, block)):
        x = chans[:, s:s + block]
        bs = x.shape[1]
        hw = BitWriter()
        hw.put(0x3FFE, 14)
        hw.put(0, 1)
        hw.put(0, 1)
        if bs in _BS_CODES and bs == block:
            bcode, extra = _BS_CODES[bs], None
        elif bs <= 256:
            bcode, extra = 6, (bs - 1, 8)
        else:
            bcode, extra = 7, (bs - 1, 16)
        hw.put(bcode, 4)
        hw.put(0, 4)  # sample rate from STREAMINFO
        mode = {"indep": C - 1, "left_side": 8, "side_right": 9, "mid_side": 10}[stereo]
        hw.put(mode, 4)
        hw.put(0 if header_ss_from_streaminfo else _SS_CODES[bps], 3)
        hw.put(0, 1)
        hdr = hw.bytes() + _utf8_num(fi)
        hw2 = BitWriter()
        if extra:
            hw2.put(extra[0], extra[1])
        hdr += hw2.bytes()
        hdr += bytes([crc8(hdr)])
        if stereo == "indep":
            subs = [(x[c], bps) for c in range(C)]
        else:
            l, r = x[0], x[1]
            side = l - r
            if stereo == "left_side":
                subs = [(l, bps), (side, bps + 1)]
            elif stereo == "side_right":
                subs = [(side, bps + 1), (r, bps)]
            else:
                subs = [((l + r) >> 1, bps), (side, bps + 1)]
        bw = BitWriter()
        for c, (v, b) in enumerate(subs):
            o = {"kind": "fixed", "order": 2, "porder": 0, "rice2": False, "escape_part": -1, "wasted": 0,
                 "lpc_prec": 12, "lpc_shift": 10}
            o.update(plan(fi, c))
            if o["kind"] == "constant" and not np.all(v == v[0]):
                o["kind"] = "verbatim"
            if o["kind"] in ("fixed", "lpc"):
                o["order"] = min(o["order"], bs)
                while o["porder"] and ((bs >> o["porder"]) << o["porder"] != bs or (bs >> o["porder"]) < o["order"]):
                    o["porder"] -= 1
            _subframe(bw, v, b, o["kind"], o["order"], o["porder"], o["rice2"], o["escape_part"], o["wasted"],
                      o["lpc_prec"], o["lpc_shift"])
        bw.align()
        frame = hdr + bw.bytes()
        frame += crc16(frame).to_bytes(2, "big")
        out += frame
    return bytes(out)


def expected_mono(chans: np.ndarray, bps: int) -> np.ndarray:
    """soundfile float32 scaling + NeMo channel mean, in the decoder's float32 order."""
    chans = np.asarray(chans, np.int64)
    scale = np.float32(1.0 / (1 << (bps - 1)))
    f = [c.astype(np.float32) * scale for c in chans]
    if len(f) == 1:
        return f[0]
    s = np.zeros_like(f[0])
    for c in f:
        s = s + c
    return s / np.float32(len(f))
