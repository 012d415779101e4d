"""kdfm's kernel-argument placement (HIP_FORCE_DEV_KERNARG, read once by the HIP runtime at start-up):
imported first it sets the variable and reports it in effect; imported after torch has started the
runtime it reports it NOT in effect and warns (a silent dependency on import order);
an explicit setting wins either way.  Each case runs in a fresh interpreter; no GPU is touched (on CPU
torch.cuda.is_initialized() stays False, so the late-import case fakes an initialised runtime)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kd-via-fm-in-asr_amd")


def _run(code, env_extra=None, drop=True):
    env = dict(os.environ)
    if drop:
        env.pop("HIP_FORCE_DEV_KERNARG", None)
    env.update(env_extra or {})
    env["PYTHONPATH"] = PKG + os.pathsep + env.get("PYTHONPATH", "")
    return subprocess.run([sys.executable, "-W", "always", "-c", code], env=env, capture_output=True, text=True,
                          timeout=300)


def test_import_first_sets_it():
    r = _run("import kdfm, os; print(kdfm.KERNARG_IN_DEVICE_MEMORY, os.environ['HIP_FORCE_DEV_KERNARG'])")
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["True", "1"] and "RuntimeWarning" not in r.stderr


def test_late_import_warns():
    code = ("import torch; torch.cuda.is_initialized = lambda: True\n"
            "import kdfm; print(kdfm.KERNARG_IN_DEVICE_MEMORY)")
    r = _run(code)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "False" and "imported after the HIP runtime started" in r.stderr


def test_explicit_setting_wins():
    code = ("import torch; torch.cuda.is_initialized = lambda: True\n"
            "import kdfm; print(kdfm.KERNARG_IN_DEVICE_MEMORY)")
    r = _run(code, {"HIP_FORCE_DEV_KERNARG": "1"})
    assert r.stdout.strip() == "True" and "RuntimeWarning" not in r.stderr
    r = _run("import kdfm; print(kdfm.KERNARG_IN_DEVICE_MEMORY)", {"HIP_FORCE_DEV_KERNARG": "0"})
    assert r.stdout.strip() == "False"
