"""Invariants NeMo's own tests pin for the (source-absent) leaf modules, checked on the oracle.

NeMo/tests/collections/asr/test_asr_filterbankfeatures_seq_len.py:22-32 (seq_len = frames - 1),
test_padding_and_batch_size_invariance.py:23-45 (mel invariant to trailing zero padding, atol 5e-2)
and :133-145 (encoder invariant to batch size); conformer_ctc_bpe.yaml:10 (Small = 13M params).
"""
import math

import pytest
import torch

from oracle import ver5

CFG = ver5.StepConfig()


def _fe():
    b = ver5.frontend_buffers(CFG)
    return b["preprocessor.featurizer.window"], b["preprocessor.featurizer.fb"][0]


@pytest.mark.parametrize("L", [800, 16000, 16123, 256000])
def test_seq_len_is_frames_minus_one(L):
    w, fb = _fe()
    x = torch.randn(1, L)
    mel, ln = ver5.preprocess(x, torch.tensor([L]), w, fb, CFG)
    assert mel.shape[2] - 1 == int(ln[0]) == L // CFG.hop


@pytest.mark.parametrize("length", [15950, 15999, 16049])
def test_mel_invariant_to_padding(length):
    w, fb = _fe()
    a1 = torch.arange(0, length).unsqueeze(0) / 16000
    a2 = torch.cat([a1, torch.zeros(1, 16000)], dim=1)
    l = torch.tensor([length])
    m1, n1 = ver5.preprocess(a1, l, w, fb, CFG)
    m2, _ = ver5.preprocess(a2, l, w, fb, CFG)
    torch.testing.assert_close(m1[..., : int(n1)], m2[..., : int(n1)], atol=5e-2, rtol=0)


def test_rel_shift_index_form():
    T = 13
    x = torch.randn(2, 3, T, 2 * T - 1)
    y = ver5.rel_shift(x)[..., :T]
    i = torch.arange(T).view(T, 1)
    j = torch.arange(T).view(1, T)
    ref = x[:, :, i, T - 1 - i + j]
    torch.testing.assert_close(y, ref)


def test_small_teacher_param_count():
    p = ver5.init_encoder(CFG, CFG.d_teacher, CFG.heads_teacher, 0, "")
    p.update(ver5.init_decoder(CFG, CFG.d_teacher, 0, "dec."))
    n = sum(v.numel() for k, v in p.items() if "running" not in k and "num_batches" not in k)
    assert abs(n / 1e6 - 13.0) < 0.05, n
    s = ver5.init_encoder(CFG, CFG.d_student, CFG.heads_student, 0, "")
    ns = sum(v.numel() for k, v in s.items() if "running" not in k and "num_batches" not in k)
    assert 3.2e6 < ns < 3.4e6


def test_encoder_batch_size_invariance():
    cfg = ver5.StepConfig(n_layers=2)
    p = ver5.init_encoder(cfg, 88, 2, 3, "enc.")
    bn = {k: v.clone() for k, v in p.items() if "running" in k}
    mel = torch.randn(1, 80, 101)
    l = torch.tensor([101])
    y1, _, _ = ver5.encoder(mel, l, p, "enc.", 88, 2, cfg, False, bn)
    y2, _, _ = ver5.encoder(mel.repeat(2, 1, 1), l.repeat(2), p, "enc.", 88, 2, cfg, False, bn)
    torch.testing.assert_close(y1, y2[:1], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(y1, y2[1:], rtol=1e-5, atol=1e-5)


def test_logitkd_oracle_is_ctc_plus_alpha_kl():
    """kd_model "logitkd" (DistilEncDecCTCModelBPE, asr_train_diffm.py:243-321): the same student / teacher
    forward as the FM step, total = CTC + kd_alpha * KL, no latent heads; only encoder / decoder train."""
    import torch
    from oracle import ver5 as O
    cfg = O.StepConfig(n_layers=1)
    p = O.init_all(cfg)
    g = torch.Generator().manual_seed(2)
    B, N = 2, 8000
    wav = 0.1 * torch.randn(B, N, generator=g)
    wl = torch.tensor([N, 6000])
    tg = torch.randint(0, cfg.vocab, (B, 5), generator=g)
    tl = torch.tensor([5, 3])
    T = ((N // cfg.hop) // 2) // 2 + 1
    eps = torch.randn(1, B, cfg.latent, T, generator=g)
    full = O.ver5_step(p, wav, wl, tg, tl, cfg, eps)
    lk = O.ver5_step(p, wav, wl, tg, tl, O.StepConfig(n_layers=1, kd_model="logitkd"), None)
    torch.testing.assert_close(lk["ctc"], full["ctc"])
    torch.testing.assert_close(lk["kl"], full["kl"])
    torch.testing.assert_close(lk["loss"], full["ctc"] + cfg.kd_alpha * full["kl"])
    names = O.trainable_names(p, kd_model="logitkd")
    assert names and all(k.startswith(("encoder.", "decoder.")) for k in names)
