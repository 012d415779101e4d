"""Probe: find main/side-stream kernel calls that may run concurrently (no fork/join between them)
and touch overlapping device memory."""
import sys, os, functools
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kd-via-fm-in-asr_amd"))
from dataclasses import replace
import torch
from kdfm import kernels as K
from kdfm.config import DEFAULT
from kdfm.engine import Ver5Engine
from kdfm import overlap

EVENTS = []   # ("call", name, side?, ranges) | ("fork",) | ("join",)
ACTIVE = [False]


def span(t):
    if t.numel() == 0:
        return None
    n = sum((s - 1) * st for s, st in zip(t.shape, t.stride())) + 1
    p = t.data_ptr()
    return (p, p + n * t.element_size())


OUT = {"layernorm_bwd": (5, 6, 7), "dropout": (1,), "axpby": (2,), "colsum": (1,), "relpos_softmax_bwd": (2, 3),
       "bn_silu_bwd": (6, 7, 8, 9), "dwconv_bwd": (3, 4, 5), "glu_mask_bwd": (3,), "col2im_3x3s2": (3,),
       "im2col_3x3s2": (2,), "fill": (0,), "convw_prep": (1, 2), "convw_grad": (1,), "adapter_bwd": (6, 7, 8, 9),
       "fm_time_bwd": (3, 4, 5, 6), "gemm": (2,)}
OUT_KW = {"Cpre", "ones_out", "fwd", "bwd"}


def wrap(name):
    fn = getattr(K, name)
    @functools.wraps(fn)
    def w(*a, **k):
        r = fn(*a, **k)
        if ACTIVE[0]:
            rs = []
            for i, x in enumerate(a):
                if isinstance(x, torch.Tensor) and span(x):
                    rs.append((span(x), i in OUT.get(name, ())))
            for kk, x in k.items():
                if isinstance(x, torch.Tensor) and span(x):
                    rs.append((span(x), kk in OUT_KW))
            if name == "scratch" and isinstance(r, torch.Tensor):
                rs = [(span(r), True)]
            EVENTS.append(("call", name, torch.cuda.current_stream().cuda_stream != 0, rs))
        return r
    setattr(K, name, w)


for n in ["gemm", "layernorm_bwd", "dropout", "axpby", "colsum", "relpos_softmax_bwd", "bn_silu_bwd", "dwconv_bwd",
          "glu_mask_bwd", "col2im_3x3s2", "im2col_3x3s2", "fill", "convw_prep", "convw_grad", "adapter_bwd",
          "fm_time_bwd", "scratch"]:
    wrap(n)

orig_run, orig_join = overlap.WGRAD.run, overlap.WGRAD.join


def run(fn, *keep):
    if ACTIVE[0]:
        EVENTS.append(("fork",))
    return orig_run(fn, *keep)


def join():
    if ACTIVE[0]:
        EVENTS.append(("join",))
    return orig_join()


overlap.WGRAD.run = run
overlap.WGRAD.join = join

cfg = replace(DEFAULT, n_layers=16, deterministic=True)
g = torch.Generator().manual_seed(21)
B, N = 4, 256000
wav = (0.1 * torch.randn(B, N, generator=g)).cuda()
wl = torch.tensor([256000, 256000, 230000, 256000], dtype=torch.int64).cuda()
tg = torch.randint(0, 128, (B, 60), generator=g).cuda()
tl = torch.full((B,), 60, dtype=torch.int64).cuda()
eng = Ver5Engine(cfg, "cuda")
Gbase = eng.student.grad.data_ptr()
Gend = Gbase + 4 * eng.student.grad.numel()
for it in range(2):
    eng.set_seed(77)
    eng.advance_rng()
    ctx = eng.forward(wav, wl, tg, tl, train=True)
    if it == 1:
        ACTIVE[0] = True
    eng.backward(ctx)
    ACTIVE[0] = False
    del ctx
    torch.cuda.synchronize()

# reconstruct concurrency: side call S (issued after fork f) is ordered after all main calls issued before f;
# main call M is ordered after all side calls issued before the last join preceding M.
calls = []
last_fork_main_idx = None
last_join = -1
main_seen = 0
for i, e in enumerate(EVENTS):
    if e[0] == "fork":
        last_fork_main_idx = i
    elif e[0] == "join":
        last_join = i
    else:
        calls.append((i, e[1], e[2], e[3], last_fork_main_idx, last_join))
conflicts = 0
for (i, n1, side1, r1, f1, j1) in calls:
    if not side1:
        continue
    # main calls after this side call's fork that are not behind a join issued after this side call
    for (k, n2, side2, r2, f2, j2) in calls:
        if side2 or k < f1:
            continue
        if j2 > i:      # a join after the side call precedes this main call -> ordered
            continue
        for a, wa in r1:
            for b, wb in r2:
                if (wa or wb) and a[0] < b[1] and b[0] < a[1]:
                    inG = Gbase <= a[0] < Gend and Gbase <= b[0] < Gend
                    if conflicts < 40:
                        print(f"overlap: side#{i} {n1}{'(W)' if wa else ''} [{a[0]:#x},{a[1]:#x}) vs main#{k} {n2}{'(W)' if wb else ''} [{b[0]:#x},{b[1]:#x}) inG={inG}")
                    conflicts += 1
print("events", len(EVENTS), "calls", len(calls), "overlaps", conflicts)
