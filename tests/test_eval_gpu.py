"""GPU evaluation path: the CTC greedy kernel is bit-identical to the oracle's decode (argmax ->
collapse -> drop blank, oracle/ver5.py greedy_ctc) on random log-probs with ragged lengths and
forced repeats; the WER metric through the device kernel reproduces NeMo's known answers; and the
engine's eval forward (Ver5Engine.infer, f32 parity mode) matches the oracle's eval-mode encoder +
decoder with bit-identical greedy transcripts."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_greedy_kernel_matches_oracle_decode():
    from kdfm import eval as E
    from oracle import ver5 as O
    g = torch.Generator().manual_seed(0)
    B, T, C = 7, 401, 129
    lp = torch.log_softmax(torch.randn(B, T, C, generator=g) * 3, dim=-1)
    # force long runs of repeats and blanks so collapsing matters
    lab = torch.randint(0, C, (B, T // 4), generator=g).repeat_interleave(4, dim=1)
    lab = torch.cat([lab, torch.full((B, T - lab.shape[1]), C - 1)], dim=1)
    lp = lp + 20.0 * torch.nn.functional.one_hot(lab, C)
    lens = torch.tensor([T, 400, 1, 0, 37, 256, 399])
    got = E.ctc_greedy_decode(lp.cuda(), lens.cuda(), blank=C - 1)
    ref = O.greedy_ctc(lp, lens, blank=C - 1)
    assert got == ref
    # exact ties -> first index, like torch.argmax
    tie = torch.zeros(1, 5, C)
    assert E.ctc_greedy_decode(tie.cuda(), None, blank=C - 1) == [[0]]


def test_wer_metric_device_decoding():
    from kdfm import eval as E
    vocab = [" "] + [chr(ord('a') + i) for i in range(26)] + ["'"]
    idx = {c: i for i, c in enumerate(vocab)}
    blank = len(vocab)

    def run(pred, ref):
        ids, prev = [], -1
        for c in (idx[ch] for ch in pred):
            if c == prev:
                ids.append(blank)
            ids.append(c)
            prev = c
        logp = torch.log(torch.nn.functional.one_hot(torch.tensor(ids), blank + 1).float() * 0.99 + 0.01 / blank)
        wer = E.WER(E.CTCGreedyDecoding(E.CharVocabulary(vocab)))
        wer.update(predictions=logp.unsqueeze(0).cuda(), predictions_lengths=None,
                   targets=torch.tensor([[idx[c] for c in ref]]), targets_lengths=torch.tensor([len(ref)]))
        return wer.compute()[0]

    assert run('cat', 'cot') == 1.0
    assert run('g p u', 'gpu') == 3.0
    assert run('ducati motorcycle', 'ducuti motorcycle') == 0.5


def test_engine_infer_matches_oracle_eval_forward():
    from dataclasses import replace

    from kdfm import eval as E
    from kdfm import kernels as K
    from kdfm.config import PARITY
    from kdfm.engine import Ver5Engine
    from oracle import ver5 as O
    cfg = replace(PARITY, n_layers=2)
    prev = K.get_math()
    K.set_math("f32")
    try:
        _infer_check(cfg, E, O)
    finally:
        K.set_math(prev)


def _infer_check(cfg, E, O):
    from kdfm.engine import Ver5Engine
    eng = Ver5Engine(cfg, "cuda:0")
    g = torch.Generator().manual_seed(3)
    B, N = 3, 19200
    wav = 0.1 * torch.randn(B, N, generator=g)
    wl = torch.tensor([N, 16000, 9001])
    lp, enc_len = eng.infer(wav.cuda(), wl.cuda())
    ocfg = O.StepConfig(n_layers=cfg.n_layers)
    p = {}
    p.update(O.frontend_buffers(ocfg))
    p.update(eng.student.state_dict())
    bn = {name: eng.bn.P[name].detach().cpu().clone() for name, _ in eng.bn.specs}
    p.update(bn)
    mel, mel_len = O.preprocess(wav, wl, p["preprocessor.featurizer.window"], p["preprocessor.featurizer.fb"][0], ocfg)
    enc, olen, _ = O.encoder(mel, mel_len, p, "encoder.", ocfg.d_student, ocfg.heads_student, ocfg, False,
                             {k: v.clone() for k, v in bn.items()})
    ref = O.decoder(enc, p, "decoder.")
    assert torch.equal(enc_len.cpu(), olen)
    err = (lp.cpu() - ref).abs().max().item()
    assert err <= 2e-3 * ref.abs().max().item(), err
    got = E.ctc_greedy_decode(lp, enc_len, blank=cfg.vocab)
    assert got == O.greedy_ctc(ref, olen, blank=cfg.vocab)
    # validation pass: loss finite, WER in [0, inf)
    tg = torch.randint(0, cfg.vocab, (B, 6), generator=g)
    tl = torch.tensor([6, 5, 3])
    vocab = E.CharVocabulary([chr(0x4e00 + i) for i in range(cfg.vocab)])
    wer = E.WER(E.CTCGreedyDecoding(vocab, blank_id=cfg.vocab))
    m = E.validation_pass(eng, (wav.cuda(), wl.cuda(), tg.cuda(), tl.cuda()), wer)
    assert m["val_loss"] == m["val_loss"] and m["val_wer_denom"] >= 3
