"""Per-phase timing of one eager ver5 step with HIP events (phases serialised on one stream so each
is measured alone; the production step overlaps the teacher on a second stream).
usage: python tools/phase_timing.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402
from kdfm.config import DEFAULT  # noqa: E402
from kdfm.conformer import EncoderShapes, encoder_backward, encoder_forward  # noqa: E402
from kdfm.engine import Ver5Engine, synthetic_batch  # noqa: E402
from kdfm.overlap import WGRAD  # noqa: E402
from kdfm.frontend import frontend_forward, mel_frames  # noqa: E402
from kdfm.heads import heads_backward, heads_forward  # noqa: E402

cfg = DEFAULT
K.set_math(cfg.math)
eng = Ver5Engine(cfg, "cuda")
B, N, U = 32, 256000, 100
wav, wl, tg, tl = synthetic_batch(cfg, B, N, U, "cuda")
for _ in range(2):
    eng.train_step(wav, wl, tg, tl)
torch.cuda.synchronize()

ev = {}


def mark(name):
    WGRAD.join()   # side-stream weight gradients of the phase count in the phase
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    ev[name] = e


for rep in range(2):
    ev.clear()
    dev = eng.device
    Tm = mel_frames(cfg, N)
    Ss = EncoderShapes(cfg, B, Tm, cfg.d_student, cfg.heads_student)
    St = EncoderShapes(cfg, B, Tm, cfg.d_teacher, cfg.heads_teacher)
    T = Ss.T
    mel_len = torch.empty(B, dtype=torch.int64, device=dev)
    len1, len2 = torch.empty_like(mel_len), torch.empty_like(mel_len)
    torch.cuda.synchronize()
    mark("start")
    K.subsample_lengths(wl, mel_len, len1, len2, cfg.hop)
    mel_t = frontend_forward(cfg, eng.fe, wav, wl, mel_len, dither=0.0)
    mel_s = frontend_forward(cfg, eng.fe, wav, wl, mel_len, dither=cfg.dither, seed=eng.seed, rng_stream=3)
    mark("frontend x2")
    sfeats = torch.empty(cfg.n_layers, Ss.rows, Ss.d, device=dev)
    pos_s = eng._pos_emb(T, Ss.d)
    srun = encoder_forward(cfg, Ss, eng.student.P, "encoder.", mel_s, mel_len, len1, len2, sfeats, pos_s,
                           train=True, seed=eng.seed, salt=1, save=True, bn_running=eng.bn.P, use_batch_stats=True,
                           ws=eng._enc_ws(Ss))
    mark("student_fwd")
    tfeats = torch.empty(cfg.n_layers, St.rows, St.d, device=dev)
    encoder_forward(cfg, St, eng.teacher.P, "teacher.encoder.", mel_t, mel_len, len1, len2, tfeats,
                    eng._pos_emb(T, St.d), train=False, seed=eng.seed, salt=2, save=False, bn_running=eng.bn.P,
                    use_batch_stats=False, ws=eng._enc_ws(St))
    mark("teacher_fwd")
    n = cfg.n_layers * Ss.rows
    acc = torch.zeros(7, device=dev)
    hctx = heads_forward(cfg, eng.student.P, sfeats.view(n, Ss.d), tfeats.view(n, St.d), T, eng.hws, acc[1:6],
                         seed=eng.seed)
    mark("heads_fwd")
    eng.student.zero_grad()
    dfeats = torch.empty(cfg.n_layers, Ss.rows, Ss.d, device=dev)
    heads_backward(cfg, eng.student.P, eng.student.G, hctx, eng.hws, dfeats.view(n, Ss.d), seed=eng.seed)
    mark("heads_bwd")
    encoder_backward(cfg, Ss, eng.student.P, eng.student.G, "encoder.", srun, dfeats, pos_s, len1, len2,
                     seed=eng.seed, salt=1, ws=eng._enc_ws(Ss))
    mark("student_bwd")
    eng.optimizer_step()
    mark("optimizer")
    torch.cuda.synchronize()
names = list(ev)
tot = 0.0
for a, b in zip(names, names[1:]):
    ms = ev[a].elapsed_time(ev[b])
    tot += ms
    print(f"{b:14s} {ms:8.3f} ms")
print(f"{'sum':14s} {tot:8.3f} ms")
