"""Checkpoint interop for the fused engine.

* Lightning `.ckpt` — what `trainer.fit` writes through ModelCheckpoint(save_last=True)
  (asr_train_diffm.py:1745-1759) and what asr_inference_diffm.py:486-492 reads back:
  `ckpt["state_dict"]` holds the DistilFlowMatchingCTCModelBPE keys — student `preprocessor.*`,
  `encoder.*`, `decoder.*`, the ver5 heads (`tae.*`, `sproj.*`, `adapter.*`, `denoiser.*`,
  `fm_latent.*`) and the frozen teacher under `teacher.*` — loaded with strict=False.
* `.nemo` — NeMo's SaveRestoreConnector archive (a tar, optionally gzip'd, entries optionally
  prefixed "./") with `model_config.yaml` and `model_weights.ckpt` (a bare state dict).  The
  teacher `stt_en_conformer_ctc_small` arrives this way (asr_train_diffm.py:91-102); its
  `encoder.*` / `decoder.*` / `preprocessor.*` keys map to the engine's `teacher.*` store.

Every file is read with loaders that execute nothing: torch.load(weights_only=True) (classes the
weights-only allowlist rejects, e.g. the OmegaConf DictConfig NeMo stores as hyper_parameters, are
replaced by inert stand-ins for that load) and yaml.safe_load.  Optimizer moments are kept in the engine's own flat layout under
`optimizer_states[0]["kdfm_flat"]` (Lightning's per-parameter index depends on NeMo's module
registration order, which does not exist here); resume restores them bit-exactly.
"""
from __future__ import annotations

import io
import os
import tarfile
from collections import OrderedDict

import torch
import yaml

TEACHER_MAP = (("encoder.", "teacher.encoder."), ("decoder.", "teacher.decoder."),
               ("preprocessor.", "teacher.preprocessor."))
_IGNORED_SUFFIXES = ("num_batches_tracked",)
_HEAD_PREFIXES = ("tae.", "sproj.", "adapter.", "denoiser.", "fm_latent.", "fm_latent_2.", "diffkd.", "flow_matching.", "router.")


def _fb_nemo(fb: torch.Tensor) -> torch.Tensor:
    return fb.detach().cpu().reshape(1, *fb.shape)


def engine_state_dict(eng, *, teacher: bool = True, frontend: bool = True) -> "OrderedDict[str, torch.Tensor]":
    """Reference-named state dict of the engine (CPU tensors): student + heads, BatchNorm running
    statistics (+ num_batches_tracked), frontend buffers, and the teacher under `teacher.*`."""
    sd = OrderedDict()
    if frontend:
        sd["preprocessor.featurizer.window"] = eng.fe.window.detach().cpu().clone()
        sd["preprocessor.featurizer.fb"] = _fb_nemo(eng.fe.fb)
    # the student's BatchNorm layers saw one batch-statistics update per optimizer step; the frozen
    # teacher's counters are whatever was loaded (its BN runs on running statistics and never counts)
    nbt = torch.tensor(int(eng.step.item()), dtype=torch.int64)
    # the conformer FM meta-encoder's BatchNorms run once per meta-encoder CALL: sum(S_i) calls per step
    # (asr_train.py:1320-1336 loops the meta-encoder over every sampling step of every hooked layer), so the
    # reference's counter advances by that much per optimizer step
    meta_calls = 1
    cfg = getattr(eng, "cfg", None)
    if cfg is not None and getattr(cfg, "kd_model", None) == "encfm" and getattr(cfg, "encfm_meta", None) == "conformer":
        from .config import encfm_fixed_steps
        meta_calls = int(sum(encfm_fixed_steps(cfg)))
    loaded_nbt = getattr(eng, "bn_batches_tracked", {})
    for name, _ in eng.student.specs:
        sd[name] = eng.student.P[name].detach().cpu().clone()
    # heads this version never trains (kept so the reference module can load the dict strictly)
    for name, t in getattr(eng, "frozen_heads", {}).items():
        sd[name] = t.detach().cpu().clone()
    fixed = getattr(eng, "fixed", None)
    for name, _ in (fixed.specs if fixed is not None else []):   # used, never trained (DiffKD's encoder)
        sd[name] = fixed.P[name].detach().cpu().clone()
    for name, _ in eng.bn.specs:
        if teacher or not name.startswith("teacher."):
            sd[name] = eng.bn.P[name].detach().cpu().clone()
            if name.endswith("running_var"):
                key = name[:-len("running_var")] + "num_batches_tracked"
                if name.startswith("teacher."):
                    sd[key] = loaded_nbt.get(key, torch.tensor(0, dtype=torch.int64)).clone()
                elif name.startswith("flow_matching.meta_encoder."):
                    sd[key] = nbt * meta_calls
                else:
                    sd[key] = nbt.clone()
    if teacher:
        if frontend:
            sd["teacher.preprocessor.featurizer.window"] = eng.fe.window.detach().cpu().clone()
            sd["teacher.preprocessor.featurizer.fb"] = _fb_nemo(eng.fe.fb)
        for name, _ in eng.teacher.specs:
            sd[name] = eng.teacher.P[name].detach().cpu().clone()
    return sd


def load_engine_state(eng, sd: dict, *, strict: bool = False, fb_atol: float = 1e-5) -> dict:
    """Copy every known key of `sd` into the engine's device stores (shapes must match exactly).
    Returns {"missing": [...], "unexpected": [...], "frontend_mismatch": [...]}; strict=True raises
    on missing or unexpected keys (num_batches_tracked and the KD heads the version does not use
    excepted: the reference builds every head for every version)."""
    stores = [eng.student, eng.teacher, eng.bn] + ([eng.fixed] if getattr(eng, "fixed", None) is not None else [])
    known = {}
    for st in stores:
        for name, _ in st.specs:
            known[name] = st
    loaded, unexpected, fe_bad = set(), [], []
    with torch.no_grad():
        for k, v in sd.items():
            if not torch.is_tensor(v):
                continue
            if k in known:
                dst = known[k].P[k]
                if tuple(v.shape) != tuple(dst.shape):
                    raise ValueError(f"{k}: checkpoint shape {tuple(v.shape)} != engine shape {tuple(dst.shape)}")
                dst.copy_(v.to(dtype=dst.dtype, device=dst.device))
                loaded.add(k)
            elif k.endswith(("featurizer.window", "featurizer.fb")):
                mine = eng.fe.window if k.endswith("window") else eng.fe.fb
                ref = v.reshape(mine.shape).to(torch.float32).cpu()
                if ref.shape != mine.shape or (ref - mine.detach().cpu()).abs().max().item() > fb_atol:
                    fe_bad.append(k)
            elif k in getattr(eng, "frozen_heads", {}):
                # a head the configured version does not train (kdfm.config.head_modules): kept
                # host-side and written back by engine_state_dict
                dst = eng.frozen_heads[k]
                if tuple(v.shape) != tuple(dst.shape):
                    raise ValueError(f"{k}: checkpoint shape {tuple(v.shape)} != reference head shape {tuple(dst.shape)}")
                eng.frozen_heads[k] = v.detach().to("cpu", torch.float32).clone()
            elif k.endswith(_IGNORED_SUFFIXES) or k.startswith(_HEAD_PREFIXES):
                if k.startswith("teacher.") and k.endswith("num_batches_tracked"):
                    if not hasattr(eng, "bn_batches_tracked"):
                        eng.bn_batches_tracked = {}
                    eng.bn_batches_tracked[k] = v.detach().to("cpu", torch.int64).reshape(())
                continue
            else:
                unexpected.append(k)
    missing = [k for k in known if k not in loaded]
    if strict and (missing or unexpected):
        raise KeyError(f"state dict mismatch: missing {missing[:8]}..., unexpected {unexpected[:8]}...")
    for st in (eng.student, eng.teacher):   # bf16 weight twins (opt-in direct-B GEMM path)
        st.version += 1                     # the frozen teacher's large-tile copies (kernels.register_frozen)
        if st.data.is_cuda:
            st.refresh_bf16()
    return {"missing": missing, "unexpected": unexpected, "frontend_mismatch": fe_bad}


# ---- Lightning .ckpt ------------------------------------------------------------------------------

class InertGlobal:
    """Stand-in for a class the checkpoint names but torch's weights-only unpickler does not allow
    (NeMo's ModelPT.save_hyperparameters stores an OmegaConf DictConfig under 'hyper_parameters').
    It records its construction arguments and pickled state and runs nothing."""

    def __init__(self, *args, **kwargs):
        self._args, self._kwargs = args, kwargs

    def __setstate__(self, state):
        self.__dict__["_state"] = state

    def __repr__(self):
        return f"<inert {type(self).__module__}.{type(self).__qualname__}>"


def _inert(module: str, name: str):
    cls = type(name, (InertGlobal,), {"__module__": module})
    cls.__qualname__ = name
    return cls


def _load_weights_only(src, *, max_globals: int = 64):
    """torch.load(weights_only=True) that tolerates classes outside the allowlist: each global the
    weights-only unpickler rejects is re-declared as an InertGlobal subclass of the same qualified
    name and allowlisted for this load only, so the file still executes nothing."""
    import pickle
    import re
    extra = []
    data = src if isinstance(src, (bytes, bytearray)) else None
    for _ in range(max_globals):
        try:
            with torch.serialization.safe_globals(extra):
                return torch.load(io.BytesIO(data) if data is not None else src, map_location="cpu",
                                  weights_only=True)
        except pickle.UnpicklingError as e:
            m = re.search(r"GLOBAL ([\w.]+)\.(\w+) was not an allowed global", str(e))
            if m is None:
                raise
            extra.append(_inert(m.group(1), m.group(2)))
    raise ValueError(f"checkpoint names more than {max_globals} classes outside the weights-only allowlist")


def read_lightning_ckpt(path: str) -> dict:
    ck = _load_weights_only(path)
    if not isinstance(ck, dict) or "state_dict" not in ck:
        raise ValueError(f"{path}: not a Lightning checkpoint (no 'state_dict')")
    return ck


def save_lightning_ckpt(eng, path: str, *, epoch: int = 0, global_step: int | None = None,
                        hyper_parameters: dict | None = None) -> None:
    step = int(eng.step.item()) if global_step is None else int(global_step)
    ck = {
        "epoch": int(epoch),
        "global_step": step,
        "pytorch-lightning_version": "2.x (kdfm)",
        "state_dict": engine_state_dict(eng),
        "optimizer_states": [{"kdfm_flat": {
            "exp_avg": eng.student.exp_avg.detach().cpu().clone(),
            "exp_avg_sq": eng.student.exp_avg_sq.detach().cpu().clone(),
            "step": torch.tensor(step, dtype=torch.int64),
            # optimizer steps taken before the moments started (AdamW bias correction counts from here)
            "adam_base": torch.tensor(int(eng.adam_base.item()), dtype=torch.int64),
            "names": [n for n, _ in eng.student.specs],
            "offsets": torch.tensor([eng.student.offsets[n] for n, _ in eng.student.specs], dtype=torch.int64),
        }}],
        "lr_schedulers": [{"last_epoch": step}],
        "hyper_parameters": dict(hyper_parameters or {}),
    }
    tmp = path + ".tmp"
    torch.save(ck, tmp)
    os.replace(tmp, path)


def restore_lightning_ckpt(eng, path: str, *, optimizer: bool = True, strict: bool = False) -> dict:
    """Load weights (and, when present, the flat AdamW moments + step counter) for resume."""
    ck = read_lightning_ckpt(path)
    info = load_engine_state(eng, ck["state_dict"], strict=strict)
    info["resumed_optimizer"] = False
    opt = (ck.get("optimizer_states") or [{}])[0].get("kdfm_flat") if optimizer else None
    if opt is not None:
        names = [n for n, _ in eng.student.specs]
        if list(opt["names"]) != names or opt["exp_avg"].numel() != eng.student.numel:
            raise ValueError(f"{path}: optimizer layout does not match this engine's parameter set")
        with torch.no_grad():
            eng.student.exp_avg.copy_(opt["exp_avg"].to(eng.student.exp_avg.device))
            eng.student.exp_avg_sq.copy_(opt["exp_avg_sq"].to(eng.student.exp_avg_sq.device))
            eng.step.fill_(int(opt["step"]))
            eng.adam_base.fill_(int(opt.get("adam_base", 0)))
        info["resumed_optimizer"] = True
    elif optimizer and "global_step" in ck:
        # a reference (Lightning/NeMo) checkpoint: its AdamW moments are keyed by NeMo's module
        # registration order and are not restored, but the Noam schedule resumes at its step
        import warnings
        warnings.warn(f"{path}: no kdfm flat optimizer state; AdamW moments restart from zero, "
                      f"the schedule resumes at global_step {int(ck['global_step'])}")
        with torch.no_grad():
            eng.step.fill_(int(ck["global_step"]))
            # fresh moments: AdamW's bias correction restarts (torch's per-parameter state 'step'
            # would be 0), only the Noam schedule continues at global_step
            eng.adam_base.fill_(int(ck["global_step"]))
    info["epoch"] = int(ck.get("epoch", 0))
    info["global_step"] = int(ck.get("global_step", 0))
    return info


# ---- .nemo ----------------------------------------------------------------------------------------

def _tar_member(tf: tarfile.TarFile, basename: str):
    for m in tf.getmembers():
        if m.isfile() and os.path.basename(m.name) == basename:
            return tf.extractfile(m).read()
    return None


def read_nemo(path: str):
    """(config dict, state dict) of a .nemo archive; nothing is extracted to disk."""
    with tarfile.open(path, "r:*") as tf:
        raw_cfg = _tar_member(tf, "model_config.yaml")
        raw_w = _tar_member(tf, "model_weights.ckpt")
    if raw_w is None:
        raise ValueError(f"{path}: no model_weights.ckpt in the archive")
    cfg = yaml.safe_load(raw_cfg.decode()) if raw_cfg is not None else {}
    sd = _load_weights_only(raw_w)
    if isinstance(sd, dict) and "state_dict" in sd and not any(k.startswith("encoder.") for k in sd):
        sd = sd["state_dict"]
    return cfg, sd


def teacher_keys(sd: dict) -> dict:
    """Map a stand-alone EncDecCTCModelBPE state dict onto the distillation model's `teacher.*`."""
    out = {}
    for k, v in sd.items():
        for src, dst in TEACHER_MAP:
            if k.startswith(src):
                out[dst + k[len(src):]] = v
                break
    return out


def load_teacher_nemo(eng, path: str, *, strict: bool = True) -> dict:
    """Initialise the frozen teacher from a Conformer-CTC .nemo (e.g. stt_en_conformer_ctc_small)."""
    cfg, sd = read_nemo(path)
    info = load_engine_state(eng, teacher_keys(sd), strict=False)
    info["missing"] = [k for k in info["missing"] if k.startswith("teacher.")]
    if strict and info["missing"]:
        raise KeyError(f"{path}: teacher keys missing: {info['missing'][:8]}")
    info["config"] = cfg
    return info


def save_nemo(eng, path: str, model_config: dict) -> None:
    """Write the student (+ heads) as a .nemo archive: model_config.yaml + model_weights.ckpt."""
    sd = engine_state_dict(eng, teacher=False)
    wbuf = io.BytesIO()
    torch.save(sd, wbuf)
    cbuf = yaml.safe_dump(model_config, sort_keys=False).encode()
    tmp = path + ".tmp"
    with tarfile.open(tmp, "w:") as tf:
        for name, data in (("./model_config.yaml", cbuf), ("./model_weights.ckpt", wbuf.getvalue())):
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            tf.addfile(ti, io.BytesIO(data))
    os.replace(tmp, path)


__all__ = ["engine_state_dict", "load_engine_state", "read_lightning_ckpt", "save_lightning_ckpt",
           "restore_lightning_ckpt", "read_nemo", "teacher_keys", "load_teacher_nemo", "save_nemo"]
