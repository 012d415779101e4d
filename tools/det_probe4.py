"""Probe: gradient determinism over repeated forward+backward in one process (WGRAD on/off)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kd-via-fm-in-asr_amd"))
from dataclasses import replace
import torch
from kdfm.config import DEFAULT
from kdfm.engine import Ver5Engine
from kdfm.overlap import WGRAD

mode = sys.argv[1] if len(sys.argv) > 1 else "on"
WGRAD.enabled = mode != "off"
if mode == "serial2q":   # two queues, but every side launch is joined immediately
    _run = WGRAD.run
    def run_join(fn, *keep):
        _run(fn, *keep)
        torch.cuda.current_stream().wait_stream(WGRAD._stream(torch.cuda.current_stream().device))
    WGRAD.run = run_join
cfg = replace(DEFAULT, n_layers=16, deterministic=True)
g = torch.Generator().manual_seed(21)
B, N = 4, 256000
wav = (0.1 * torch.randn(B, N, generator=g)).cuda()
wl = torch.tensor([256000, 256000, 230000, 256000], dtype=torch.int64).cuda()
tg = torch.randint(0, 128, (B, 60), generator=g).cuda()
tl = torch.full((B,), 60, dtype=torch.int64).cuda()
eng = Ver5Engine(cfg, "cuda")
ref = None
order = list(eng.student.grads().keys())
for it in range(8):
    eng.set_seed(77)
    eng.advance_rng()
    ctx = eng.forward(wav, wl, tg, tl, train=True)
    eng.backward(ctx)
    del ctx
    torch.cuda.synchronize()
    gr = eng.student.grads()
    gr = {k: v.clone() for k, v in gr.items()}
    if ref is None:
        ref = gr
        continue
    bad = [k for k in order if not torch.equal(ref[k], gr[k])]
    # report the LAST-in-backward-order first: backward walks heads, decoder, layers 15..0, subsampling
    heads = [k for k in bad if not k.startswith(("encoder.", "decoder."))]
    print(mode, it, "differing:", len(bad), "heads:", heads[:6], "first enc:", [k for k in bad if k.startswith("encoder.layers.15")][:4], "dec", [k for k in bad if k.startswith("decoder")])
