"""The happens-before race checker (tools/race_check.py) over the real multi-stream step on the GPU:
the benchmark's default overlapped schedule -- KD heads in two layer halves (KDFM_HEADS_SPLIT=1, the
first half's forward on the weight-gradient stream, its backward on the teacher stream), weight
gradients on their own stream, CTC/KL on the teacher stream, the 4-bucket all-reduce of a world of 2
issued from the weight-gradient stream -- with use_diffkd off and on.  Any conflicting access pair fails
(the NoiseAdapter gradient fold of the two halves raced until it moved to the weight-gradient
stream).  Each case runs in its own process: the checker patches torch's event / stream / collective
entry points."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("diffkd", [False, True], ids=["ver5", "ver5+diffkd"])
def test_overlapped_step_has_no_race(diffkd):
    env = dict(os.environ, KDFM_HEADS_SPLIT="1")
    cmd = [sys.executable, os.path.join(ROOT, "tools", "race_check.py"), "--layers", "4", "--batch", "4",
           "--seconds", "4", "--steps", "2"] + (["--diffkd"] if diffkd else [])
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    assert "heads_split=True" in r.stdout, r.stdout + r.stderr[-3000:]
    assert r.returncode == 0, "races:\n" + r.stdout[-6000:] + r.stderr[-2000:]
