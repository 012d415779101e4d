"""Which operand slots does each lane's e8m0 scale byte multiply in v_mfma_scale_f32_16x16x128_f8f6f4 (gfx950)?
For every lane L and operand X in {A, B}: one MFMA with all scales 2^0 except lane L's X-scale 2^1, on 8 random
operand sets (small integers, exact in e4m3; tools/fp8_probe.hip's batched kernel).  The difference to the all-unit
MFMA is the sum of the contributions of the slots lane L's scale covers; per output row (A) or column (B) that is a
128-unknown linear system (slot on / off) over 8 x 16 equations, solved by least squares and rounded.
Prints, per lane, the (lane, byte) slots its scale byte covers."""
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def e4m3(x):
    return torch.from_numpy(x.astype(np.float32)).to(torch.float8_e4m3fn).view(torch.uint8).numpy()


def main():
    lib = C.CDLL(os.path.join(HERE, "fp8_probe.so"))
    dev = torch.device("cuda")
    rng = np.random.default_rng(3)
    ND = 8
    A = rng.choice([-2.0, -1.0, 1.0, 2.0], size=(ND, 64, 32))
    B = rng.choice([-2.0, -1.0, 1.0, 2.0], size=(ND, 64, 32))
    blocks = [("base", -1, d) for d in range(ND)] + [(op, L, d) for op in ("A", "B") for L in range(64) for d in range(ND)]
    nb = len(blocks)
    a = np.zeros((nb, 64, 32), np.uint8)
    b = np.zeros((nb, 64, 32), np.uint8)
    lsa = np.full((nb, 64), 127, np.int32)
    lsb = np.full((nb, 64), 127, np.int32)
    Aq, Bq = e4m3(A), e4m3(B)
    for t, (op, L, d) in enumerate(blocks):
        a[t], b[t] = Aq[d], Bq[d]
        if op == "A":
            lsa[t, L] = 128
        elif op == "B":
            lsb[t, L] = 128
    dc = torch.zeros(nb, 64, 4, device=dev)
    keep = [torch.from_numpy(x.view(np.int32).reshape(nb, -1).copy()).to(dev) for x in (a, b)] + \
        [torch.from_numpy(x.copy()).to(dev) for x in (lsa, lsb)]
    rc = lib.fp8_probe_batch(*[C.c_void_p(k.data_ptr()) for k in keep[:2]], C.c_void_p(dc.data_ptr()),
                             *[C.c_void_p(k.data_ptr()) for k in keep[2:]], C.c_int(-nb))
    assert rc == 0, rc
    cc = dc.cpu().numpy()
    full = np.zeros((nb, 16, 16))
    for l in range(64):
        for r in range(4):
            full[:, 4 * (l >> 4) + r, l & 15] = cc[:, l, r]
    base = full[:ND]
    ref = np.einsum("dgrj,dgcj->drc", A.reshape(ND, 4, 16, 32), B.reshape(ND, 4, 16, 32))
    print(f"unit-scale MFMA vs exact (same-map pairing): max err {np.abs(base - ref).max():g}", flush=True)
    t = ND
    for op in ("A", "B"):
        print(f"--- {op} scale lanes", flush=True)
        for L in range(64):
            delta = np.stack([full[t + d] - base[d] for d in range(ND)])   # [d, r, c]
            t += ND
            cover = []
            for line in range(16):   # row of C for A, column for B
                # unknowns: slots (g, j) of this row / column, x[g, j]; contribution of slot (g, j) to C[line, c]
                # (A) = A[d, 16 g + line, j] * B[d, 16 g + c, j]
                if op == "A":
                    M = np.einsum("dgj,dgcj->dcgj", A.reshape(ND, 4, 16, 32)[:, :, line, :],
                                  B.reshape(ND, 4, 16, 32)).reshape(ND * 16, 128)
                    y = delta[:, line, :].reshape(-1)
                else:
                    M = np.einsum("dgrj,dgj->drgj", A.reshape(ND, 4, 16, 32),
                                  B.reshape(ND, 4, 16, 32)[:, :, line, :]).reshape(ND * 16, 128)
                    y = delta[:, :, line].reshape(-1)
                if not np.any(y):
                    continue
                x, *_ = np.linalg.lstsq(M, y, rcond=None)
                xr = np.round(x)
                resid = np.abs(M @ xr - y).max()
                for s in np.nonzero(xr)[0]:
                    g, j = divmod(int(s), 32)
                    cover.append((16 * g + line, j, int(xr[s])))
                if resid > 0:
                    cover.append(("resid", resid))
            lanes = sorted({c[0] for c in cover if c[0] != "resid"})
            desc = {ln: [c[1] for c in cover if c[0] == ln] for ln in lanes}
            summ = "; ".join(f"lane {ln} bytes {min(v)}..{max(v)} ({len(v)})" + ("" if len(set(c[2] for c in cover if c[0] == ln)) == 1 else " mixed") for ln, v in desc.items())
            bad = [c for c in cover if c[0] == "resid"]
            print(f"{op} scale lane {L:2d}: {summ}{' RESID ' + str(bad) if bad else ''}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
