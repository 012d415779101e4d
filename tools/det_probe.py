"""Probe: which reduction differs between two identical runs in deterministic mode."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kd-via-fm-in-asr_amd"))
import torch
from kdfm import kernels as K

torch.manual_seed(0)
dev = "cuda"
for math in ("bf16", "f32"):
    K.set_math(math)
    K.set_deterministic(True)
    for (M, N, Kd) in [(25664, 96, 96), (25664, 96, 128), (12832, 352, 88), (12832, 88, 352), (32080, 88, 792)]:
        dy = torch.randn(M, N, device=dev)
        x = torch.randn(M, Kd, device=dev)
        outs = []
        for _ in range(3):
            dW = torch.zeros(N, Kd, device=dev)
            db = torch.zeros(N, device=dev)
            K.linear_dw(dy, x, dW, db=db)
            torch.cuda.synchronize()
            outs.append((dW.clone(), db.clone()))
        same = all(torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1]) for o in outs[1:])
        ref = dy.double().t() @ x.double()
        err = ((outs[0][0].double() - ref).norm() / ref.norm()).item()
        print(math, "linear_dw", (M, N, Kd), "sk", K._splitk_for(N, Kd + 1, M), "bitwise-same", same, "rel err", f"{err:.2e}")
    T = 401
    M = 64 * T
    dy = torch.randn(M, 96, device=dev)
    x = torch.randn(M, 96, device=dev)
    outs = []
    for _ in range(3):
        G = torch.zeros(96, 288, device=dev)
        db = torch.zeros(96, device=dev)
        K.conv3_dw(dy, x, G, T, db=db)
        torch.cuda.synchronize()
        outs.append((G.clone(), db.clone()))
    same = all(torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1]) for o in outs[1:])
    print(math, "conv3_dw bitwise-same", same)
