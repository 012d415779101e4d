"""Checkpoint interop (kdfm/checkpoint.py) on CPU stores: reference key
names, Lightning .ckpt round trip with the flat AdamW moments (resume), .nemo archive round trip,
teacher initialisation from a stand-alone Conformer-CTC .nemo (encoder./decoder. -> teacher.*),
and the inference script's strict=False contract (asr_inference_diffm.py:486-492)."""
import io
import os
import tarfile
from dataclasses import replace

import pytest
import torch

from kdfm import checkpoint as C
from kdfm.config import DEFAULT
from kdfm.engine import Ver5Engine


@pytest.fixture()
def eng():
    cfg = replace(DEFAULT, n_layers=2)
    e = Ver5Engine(cfg, "cpu", init=False)
    g = torch.Generator().manual_seed(3)
    for st in (e.student, e.teacher, e.bn):
        st.data.copy_(torch.randn(st.data.shape, generator=g))
    e.student.exp_avg.copy_(torch.randn(e.student.numel, generator=g))
    e.student.exp_avg_sq.copy_(torch.rand(e.student.numel, generator=g))
    e.step.fill_(123)
    return e


def _same(a, b):
    """per-parameter equality of two FlatStores (the alignment padding is not state)"""
    return all(torch.equal(a.P[n], b.P[n]) for n, _ in a.specs)


def _fresh():
    return Ver5Engine(replace(DEFAULT, n_layers=2), "cpu", init=False)


def test_state_dict_reference_names(eng):
    sd = C.engine_state_dict(eng)
    for k in ("encoder.pre_encode.conv.0.weight", "encoder.layers.1.self_attn.pos_bias_u",
              "encoder.layers.0.conv.batch_norm.running_var", "encoder.layers.0.conv.batch_norm.num_batches_tracked",
              "decoder.decoder_layers.0.weight", "denoiser.net.0.weight", "fm_latent.fm.meta_encoder.0.weight",
              "teacher.encoder.layers.1.feed_forward2.linear2.weight", "teacher.decoder.decoder_layers.0.bias",
              "preprocessor.featurizer.fb", "teacher.preprocessor.featurizer.window"):
        assert k in sd, k
    assert sd["preprocessor.featurizer.fb"].shape[0] == 1
    assert sd["decoder.decoder_layers.0.weight"].shape == (DEFAULT.classes, DEFAULT.d_student, 1)


def test_lightning_roundtrip_and_resume(eng, tmp_path):
    p = str(tmp_path / "last.ckpt")
    C.save_lightning_ckpt(eng, p, epoch=4)
    e2 = _fresh()
    info = C.restore_lightning_ckpt(e2, p, strict=True)
    assert info["resumed_optimizer"] and info["epoch"] == 4 and info["global_step"] == 123
    assert info["frontend_mismatch"] == [] and info["unexpected"] == []
    assert _same(eng.student, e2.student) and _same(eng.teacher, e2.teacher) and _same(eng.bn, e2.bn)
    assert torch.equal(eng.student.exp_avg, e2.student.exp_avg)
    assert torch.equal(eng.student.exp_avg_sq, e2.student.exp_avg_sq)
    assert int(e2.step) == 123 and int(e2.adam_base) == 0
    # the inference script's load: ckpt["state_dict"], strict=False, on a model without the teacher
    ck = C.read_lightning_ckpt(p)
    sd = {k: v for k, v in ck["state_dict"].items() if not k.startswith("teacher.")}
    e3 = _fresh()
    info = C.load_engine_state(e3, sd, strict=False)
    assert all(k.startswith("teacher.") for k in info["missing"])
    assert _same(e3.student, eng.student)


def test_shape_mismatch_raises(eng):
    sd = C.engine_state_dict(eng)
    sd["decoder.decoder_layers.0.bias"] = torch.zeros(7)
    with pytest.raises(ValueError):
        C.load_engine_state(_fresh(), sd)


def test_unexpected_keys_strict(eng):
    sd = C.engine_state_dict(eng)
    sd["layer_proj.0.weight"] = torch.zeros(1)
    assert C.load_engine_state(_fresh(), sd)["unexpected"] == ["layer_proj.0.weight"]
    with pytest.raises(KeyError):
        C.load_engine_state(_fresh(), sd, strict=True)


def test_untrained_heads_round_trip(eng):
    """the heads a version never trains (fm_latent_2 for ver5) are kept as loaded and
    written back, so a kdfm state dict carries the reference module's full key set
    (asr_train_diffm.py:559-564 builds every head for every version)."""
    from kdfm.config import all_head_specs
    sd = C.engine_state_dict(eng)
    for name, shape in all_head_specs(eng.cfg):
        assert name in sd and tuple(sd[name].shape) == tuple(shape), name
    w = torch.arange(32, dtype=torch.float32).view(32, 1)
    sd["fm_latent_2.fm.time_embed.weight"] = w
    e2 = _fresh()
    info = C.load_engine_state(e2, sd, strict=True)
    assert info["unexpected"] == []
    assert torch.equal(C.engine_state_dict(e2)["fm_latent_2.fm.time_embed.weight"], w)
    sd["fm_latent_2.fm.time_embed.weight"] = torch.zeros(1)
    with pytest.raises(ValueError):
        C.load_engine_state(_fresh(), sd)


def test_nemo_roundtrip(eng, tmp_path):
    p = str(tmp_path / "student.nemo")
    C.save_nemo(eng, p, {"encoder": {"d_model": 88, "n_layers": 2}, "target": "kdfm"})
    cfg, sd = C.read_nemo(p)
    assert cfg["encoder"]["d_model"] == 88
    assert not any(k.startswith("teacher.") for k in sd)
    e2 = _fresh()
    C.load_engine_state(e2, sd)
    assert _same(e2.student, eng.student)


def test_teacher_from_nemo_gz(eng, tmp_path):
    """A stand-alone EncDecCTCModelBPE .nemo (gzip'd tar, './'-prefixed names, tokenizer files)."""
    sd = {k[len("teacher."):]: v for k, v in C.engine_state_dict(eng).items() if k.startswith("teacher.")}
    wbuf = io.BytesIO()
    torch.save(sd, wbuf)
    p = str(tmp_path / "stt_en_conformer_ctc_small.nemo")
    with tarfile.open(p, "w:gz") as tf:
        for name, data in (("./model_config.yaml", b"encoder:\n  d_model: 176\n"),
                           ("./model_weights.ckpt", wbuf.getvalue()), ("./tokenizer.model", b"\x00")):
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            tf.addfile(ti, io.BytesIO(data))
    e2 = _fresh()
    info = C.load_teacher_nemo(e2, p)
    assert info["config"]["encoder"]["d_model"] == 176
    assert _same(e2.teacher, eng.teacher)
    tb = [n for n, _ in e2.bn.specs if n.startswith("teacher.")]
    assert all(torch.equal(e2.bn.P[n], eng.bn.P[n]) for n in tb)


class DictConfigStandIn:
    """Stands for omegaconf.DictConfig (not importable here), which NeMo's ModelPT stores as
    ckpt["hyper_parameters"] through save_hyperparameters(cfg): a class outside torch's
    weights-only allowlist.  Instantiating it would record the side effect below."""
    constructed = 0

    def __init__(self, content):
        type(self).constructed += 1
        self._content = content


def test_reference_style_ckpt_with_foreign_hyperparameters(eng, tmp_path):
    """A Lightning checkpoint as the reference writes it: hyper_parameters hold a non-allowlisted
    class and there is no kdfm flat optimizer entry.  The state dict loads, the foreign
    object comes back as an inert stand-in (its code never runs), and the Noam schedule resumes at
    global_step."""
    sd = C.engine_state_dict(eng)
    sd["teacher.encoder.layers.0.conv.batch_norm.num_batches_tracked"] = torch.tensor(777)
    p = str(tmp_path / "reference.ckpt")
    torch.save({"epoch": 2, "global_step": 4567, "state_dict": sd,
                "optimizer_states": [{"state": {}, "param_groups": []}],
                "hyper_parameters": {"cfg": DictConfigStandIn({"encoder": {"d_model": 88}})}}, p)
    DictConfigStandIn.constructed = 0
    e2 = _fresh()
    with pytest.warns(UserWarning, match="schedule resumes"):
        info = C.restore_lightning_ckpt(e2, p)
    assert DictConfigStandIn.constructed == 0
    assert not info["resumed_optimizer"] and info["global_step"] == 4567 and int(e2.step) == 4567
    # fresh moments: AdamW's bias correction restarts while the schedule continues
    assert int(e2.adam_base) == 4567
    assert _same(e2.student, eng.student) and _same(e2.teacher, eng.teacher)
    hp = C.read_lightning_ckpt(p)["hyper_parameters"]["cfg"]
    assert isinstance(hp, C.InertGlobal) and not isinstance(hp, DictConfigStandIn)
    assert hp._state == {"_content": {"encoder": {"d_model": 88}}}
    # teacher BatchNorm counters pass through; the student's count its optimizer steps
    out = C.engine_state_dict(e2)
    assert int(out["teacher.encoder.layers.0.conv.batch_norm.num_batches_tracked"]) == 777
    assert int(out["encoder.layers.0.conv.batch_norm.num_batches_tracked"]) == 4567


def test_conformer_meta_bn_counter_counts_module_calls():
    """The conformer FM meta-encoder's BatchNorms run once per meta-encoder call, sum(S_i) times per step
    (asr_train.py:1320-1336), so their num_batches_tracked is step x sum(S_i); the encoder's
    BatchNorms still count optimizer steps."""
    from kdfm.config import encfm_fixed_steps
    cfg = replace(DEFAULT, n_layers=2, kd_model="encfm", encfm_dynamic=False, encfm_meta="conformer",
                  encfm_steps_per_layer=(2, 3))
    e = Ver5Engine(cfg, "cpu", init=False)
    e.step.fill_(10)
    sd = C.engine_state_dict(e, teacher=False)
    meta = [k for k in sd if k.startswith("flow_matching.meta_encoder.") and k.endswith("num_batches_tracked")]
    assert meta, "no meta-encoder BatchNorm in the state dict"
    assert sum(encfm_fixed_steps(cfg)) == 5
    for k in meta:
        assert int(sd[k]) == 50, k
    assert int(sd["encoder.layers.0.conv.batch_norm.num_batches_tracked"]) == 10
