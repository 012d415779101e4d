"""Which Python call sites issue the compute-stream kdfm_gemm launches of one bench step, with their
shapes: one eager train step with K.call patched to log each kdfm_gemm descriptor (M, N, K, batch, modes,
epilogue), its stream and the calling frames.  usage: python tools/gemm_calls.py [out.txt] [xl]
(xl: the FastConformer-XL shapes of bench.py's xl_shape_sensitivity line)"""
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402
from kdfm.config import DEFAULT  # noqa: E402
from kdfm.engine import Ver5Engine, synthetic_batch  # noqa: E402

dev = torch.device("cuda", 0)
CFG = DEFAULT
if len(sys.argv) > 2 and sys.argv[2] == "xl":
    from dataclasses import replace
    sys.path.insert(0, ROOT)
    from bench import XL_SHAPES
    CFG = replace(DEFAULT, **XL_SHAPES)
K.set_math(CFG.math)
eng = Ver5Engine(CFG, dev)
wav, wl, tg, tl = synthetic_batch(CFG, 32, 256000, 100, dev, seed=1234)
eng.train_step(wav, wl, tg, tl, None)
torch.cuda.synchronize()
names = {eng.compute_stream.cuda_stream: "compute", eng._side_stream().cuda_stream: "teacher"}
from kdfm.overlap import WGRAD  # noqa: E402
for st in WGRAD._side.values():
    names[st.cuda_stream] = "wgrad"
log = []
orig = K.call


CASTS = {}


def call(name, *args):
    if name in ("kdfm_cast_bf16_2d", "kdfm_fp8_quant_mx"):
        fr = [f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in traceback.extract_stack()[-7:-2]]
        rows, cols = (args[4], args[5]) if name == "kdfm_cast_bf16_2d" else (args[2], args[3])
        key = f"{name} {rows}x{cols} " + " < ".join(reversed(fr))
        CASTS[key] = CASTS.get(key, 0) + 1
    if name == "kdfm_gemm":
        d = K._GEMM_DESC.contents
        s = args[-1]
        s = s.value if hasattr(s, "value") else s
        fr = [f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in traceback.extract_stack()[-6:-2]]
        route = None
    orig(name, *args)
    if name == "kdfm_gemm":
        route = K.ROUTES[int(K._lib.lib().kdfm_gemm_last_route())]
        log.append(f"{names.get(s, s):8s} route={route} M={d.M} N={d.N} K={d.K} batch={d.batch1}x{d.batch2} amode={d.amode} "
                   f"bmode={d.bmode} epi={d.epi} math={d.math} grid~({-(-d.M // 64)},{-(-d.N // 64)})  " + " < ".join(reversed(fr)))


K.call = call
eng.train_step(wav, wl, tg, tl, None)
torch.cuda.synchronize()
K.call = orig
log += [f"{n:5d} x {k}" for k, n in sorted(CASTS.items(), key=lambda kv: -kv[1])]
txt = "\n".join(log)
out = sys.argv[1] if len(sys.argv) > 1 else None
if out:
    open(out, "w").write(txt + "\n")
print(txt)
