"""Debug: which rows of the prepared-operand attention forward differ from the register-staged one."""
import math
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "kd-via-fm-in-asr_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch
from kdfm import kernels as K
from test_attn_fwd3_gpu import _inputs

for (B, H, T, d, p) in [(1, 1, 64, 44, 0.0), (1, 1, 130, 44, 0.0), (1, 2, 64, 88, 0.0), (2, 2, 77, 88, 0.1)]:
    qkv, qu, qv, ppos, lens = _inputs(B, H, T, d, 7)
    seed = torch.tensor([321], dtype=torch.int64, device="cuda")
    sc = 1.0 / math.sqrt(d // H)
    o1 = torch.empty(B * T, d, device="cuda")
    lse1 = torch.empty(B, H, T, device="cuda")
    K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o1, None, None, B, H, T, sc, p, seed, 17, lse=lse1)
    o2 = torch.zeros(B * T, d, device="cuda")
    lse2 = torch.zeros(B, H, T, device="cuda")
    prep = K.attn_kv_prep(qkv, lens, B, H, T)
    pb = K.attn_band_prep(ppos, H, T)[0]
    K.relpos_attn_fwd3(qu, qv, prep, pb, lens, o2, B, H, T, sc, p, seed, 17, lse=lse2)
    torch.cuda.synchronize()
    dr = (o1 - o2).abs().amax(1).cpu()
    bad = (dr > 0).nonzero().flatten().tolist()
    print(B, H, T, d, p, "rows differing:", len(bad), bad[:40])
    dl = (lse1 - lse2).abs().cpu()
    print("  lse rows differing:", (dl > 0).nonzero()[:20].tolist())
