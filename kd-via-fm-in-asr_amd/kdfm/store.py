"""Flat device buffers for parameters, gradients and optimizer state.

Every trainable tensor of the step is a view into ONE contiguous fp32 buffer (and its gradient a
view into one gradient buffer).  This is the MI355X layout choice that makes the data-parallel
exchange a single large RCCL all-reduce and the optimizer a single fused AdamW launch, and it lets
the fused q|k|v projection read three NeMo parameters as one (3d, d) matrix.
"""
from __future__ import annotations

import math

import torch

from . import kernels as K
from .config import fused_groups

ALIGN = 4  # floats (16 bytes): every tensor starts 16-B aligned for dwordx4 loads
# start of every parameter (fused q|k|v group: of the group) in floats.  Fixed: the flat layout (and
# with it the saved AdamW moments, checkpoint.py) must not depend on the environment
GROUP_ALIGN = ALIGN


def _numel(shape):
    return int(math.prod(shape)) if shape else 1


class FlatStore:
    def __init__(self, specs: list, device, with_grad: bool = True, with_adam: bool = False):
        self.specs = list(specs)
        self.device = torch.device(device)
        self.offsets = {}
        inner = set()
        names = [n for n, _ in self.specs]
        for fname, (first, count, fshape) in fused_groups(self.specs).items():
            i = names.index(first)
            inner.update(names[i + 1:i + count])
        off = 0
        for name, shape in self.specs:
            if name not in inner:
                off = -(-off // GROUP_ALIGN) * GROUP_ALIGN
            self.offsets[name] = off
            n = _numel(shape)
            off += -(-n // ALIGN) * ALIGN
        off = -(-off // GROUP_ALIGN) * GROUP_ALIGN
        self.numel = off
        self.data = torch.zeros(self.numel, device=self.device, dtype=torch.float32)
        # bumped by load(): a frozen store's derived weight copies (kernels.register_frozen) are rebuilt after it
        self.version = 0
        self.grad = torch.zeros(self.numel, device=self.device, dtype=torch.float32) if with_grad else None
        self.exp_avg = torch.zeros_like(self.data) if with_adam else None
        self.exp_avg_sq = torch.zeros_like(self.data) if with_adam else None
        self.P = {}
        self.G = {}
        shapes = dict(self.specs)
        for name, shape in self.specs:
            o, n = self.offsets[name], _numel(shape)
            self.P[name] = self.data[o:o + n].view(shape)
            if self.grad is not None:
                self.G[name] = self.grad[o:o + n].view(shape)
        for fname, (first, count, fshape) in fused_groups(self.specs).items():
            o = self.offsets[first]
            n = _numel(fshape)
            # members must be adjacent and unpadded for the fused view to be exact
            assert _numel(shapes[first]) % ALIGN == 0, fname
            self.P[fname] = self.data[o:o + n].view(fshape)
            if self.grad is not None:
                self.G[fname] = self.grad[o:o + n].view(fshape)

    # ---- bf16 twins for the bf16 GEMM path (kernels.bf16_twin) ----
    def enable_bf16_twins(self) -> None:
        """Allocate and register the bf16 copy of the buffer and the per-weight transposed copy
        (2-D weights and fused groups as units); refresh_bf16() fills them."""
        if getattr(self, "h", None) is not None:
            return
        shapes = dict(self.specs)
        fused = fused_groups(self.specs)
        members = set()
        entries = []
        for fname, (first, count, fshape) in fused.items():
            names = [n for n, _ in self.specs]
            i0 = names.index(first)
            members.update(names[i0:i0 + count])
            if len(fshape) == 2:
                entries.append((self.offsets[first], fshape[0], fshape[1]))
        for name, shape in self.specs:
            if name in members or not name.endswith(".weight") or len(shape) < 2:
                continue
            if _numel(shape[2:]) != 1 or shape[0] * shape[1] < 64:
                continue
            entries.append((self.offsets[name], int(shape[0]), int(shape[1])))
        entries.sort()
        tab = []
        blk = 0
        for off, r, c in entries:
            tab.append((off, r, c, blk))
            blk += -(-(r * c) // 256)
        self.h = torch.zeros(self.numel, device=self.device, dtype=torch.bfloat16)
        self.ht = torch.zeros(self.numel, device=self.device, dtype=torch.bfloat16)
        self._ttab = torch.tensor(tab, dtype=torch.int64, device=self.device)
        self._tblocks = blk
        K.register_bf16_twin(self.data, self.h, self.ht, entries)

    def enable_bf16_mirror(self) -> None:
        """A bf16 mirror of the whole buffer (same layout) for the large-tile GEMM's weight operands, kept current by
        load() / refresh_bf16() and by the optimizer (kdfm_adamw_noam_bf16 writes it in the same pass)."""
        if getattr(self, "mirror", None) is not None:
            return
        self.mirror = torch.empty(self.numel, device=self.device, dtype=torch.bfloat16)
        K.cast_bf16(self.data, self.mirror)
        K.register_bf16_mirror(self.data, self.mirror)

    def refresh_bf16(self) -> None:
        if getattr(self, "mirror", None) is not None:
            K.cast_bf16(self.data, self.mirror)
        if getattr(self, "h", None) is None:
            return
        K.cast_bf16(self.data, self.h)
        if self._tblocks:
            K.cast_bf16_t(self.data, self.ht, self._ttab, self._ttab.shape[0], self._tblocks)

    @property
    def trainable_count(self) -> int:
        return sum(_numel(s) for _, s in self.specs)

    def load(self, state: dict, strict: bool = True) -> None:
        """Copy a {name: tensor} dict (NeMo names) into the buffer (host->device upload)."""
        missing = []
        for name, shape in self.specs:
            if name not in state:
                missing.append(name)
                continue
            t = state[name]
            if tuple(t.shape) != tuple(shape):
                raise ValueError(f"{name}: shape {tuple(t.shape)} != {tuple(shape)}")
            self.P[name].copy_(t.detach().to(torch.float32))
        self.version += 1
        if getattr(self, "mirror", None) is not None:
            K.cast_bf16(self.data, self.mirror)
        if strict and missing:
            raise KeyError(f"missing parameters: {missing[:5]}{'...' if len(missing) > 5 else ''}")

    def state_dict(self) -> dict:
        return {name: self.P[name].detach().clone().cpu() for name, _ in self.specs}

    def grads(self) -> dict:
        return {name: self.G[name].detach().clone().cpu() for name, _ in self.specs}

    def zero_grad(self) -> None:
        if self.grad is not None:
            K.fill(self.grad, 0.0)


def init_uniform(specs: list, seed: int) -> dict:
    """Seeded host-side init: U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for weights/biases, ~1 for norm
    scales, small normal for the relative-position biases (random-init weights for the benchmark;
    the real teacher checkpoint needs a remote fetch)."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    shapes = dict(specs)
    for name, shape in specs:
        if (".norm_" in name or "batch_norm" in name) and name.endswith(".weight"):
            t = 1.0 + 0.1 * (torch.rand(shape, generator=g) * 2 - 1)
        elif (".norm_" in name or "batch_norm" in name) and name.endswith(".bias"):
            t = 0.1 * (torch.rand(shape, generator=g) * 2 - 1)
        elif "pos_bias" in name:
            t = 0.1 * torch.randn(shape, generator=g)
        else:
            wname = name[: -len("bias")] + "weight" if name.endswith(".bias") else name
            ws = shapes.get(wname, shape)
            fan_in = _numel(ws[1:]) if len(ws) > 1 else ws[0]
            s = 1.0 / math.sqrt(max(1, fan_in))
            t = (torch.rand(shape, generator=g) * 2 - 1) * s
        out[name] = t.float()
    return out
