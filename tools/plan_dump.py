"""Dump the bench step plan's op list: kernel launches with their stream, event records / waits with the
event's index (a wait names the stream that recorded it), host callbacks -- to trace which cross-stream
wait a compute-stream gap sits behind.  usage: python tools/plan_dump.py [out.txt]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402
from kdfm.config import DEFAULT  # noqa: E402
from kdfm.engine import Ver5Engine, synthetic_batch  # noqa: E402
from kdfm.overlap import WGRAD  # noqa: E402

dev = torch.device("cuda", 0)
K.set_math(DEFAULT.math)
eng = Ver5Engine(DEFAULT, dev)
wav, wl, tg, tl = synthetic_batch(DEFAULT, 32, 256000, 100, dev, seed=1234)
eng.train_step(wav, wl, tg, tl, None)
plan = eng.make_plan(wav, wl, tg, tl)
torch.cuda.synchronize()
streams = {eng.compute_stream.cuda_stream: "compute", eng._side_stream().cuda_stream: "teacher"}
for st in WGRAD._side.values():
    streams[st.cuda_stream] = "wgrad"
try:
    streams[eng._aux_stream().cuda_stream] = "aux"
except Exception:
    pass


def sname(s):
    s = s.value if hasattr(s, "value") else s
    return streams.get(s, str(s))


evs, rec_by = {}, {}
lines = []
for i, op in enumerate(plan.ops):
    if op[0] == "k" and getattr(op[1], "__name__", "") == "kdfm_event_record":   # K.LinkEvent (event, stream)
        e = evs.setdefault(op[2][0], len(evs))
        rec_by[e] = sname(op[2][1])
        lines.append(f"{i:5d} R {sname(op[2][1]):8s} ev{e}")
    elif op[0] == "k" and getattr(op[1], "__name__", "") == "kdfm_stream_wait_event":   # (stream, event)
        e = evs.setdefault(op[2][1], len(evs))
        lines.append(f"{i:5d} W {sname(op[2][0]):8s} ev{e} (recorded on {rec_by.get(e, '?')})")
    elif op[0] == "k":
        nm = getattr(op[1], "__name__", "?")
        s = op[2][-1] if op[2] else None
        lines.append(f"{i:5d} K {sname(s):8s} {nm}")
    elif op[0] in ("er", "ew"):
        e = evs.setdefault(op[1].value, len(evs))
        if op[0] == "er":
            rec_by[e] = sname(op[2])
            lines.append(f"{i:5d} R {sname(op[2]):8s} ev{e}")
        else:
            lines.append(f"{i:5d} W {sname(op[2]):8s} ev{e} (recorded on {rec_by.get(e, '?')})")
    else:
        lines.append(f"{i:5d} H          {getattr(op[1], '__name__', op[1])}")
out = sys.argv[1] if len(sys.argv) > 1 else None
txt = "\n".join(lines)
if out:
    open(out, "w").write(txt + "\n")
else:
    print(txt)
