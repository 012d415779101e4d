"""Evaluation-path host logic: word_error_rate and the WER metric against
the known answers of NeMo's own tests (NeMo/tests/collections/asr/test_asr_metrics.py:57-199), the
native edit distance against a Python Levenshtein, and CTC label collapsing.  No GPU needed: label
tensors are decoded on the host; log-prob tensors go to the device kernel (tests/test_eval_gpu.py)."""
import random
import string

import pytest
import torch


def _ev():
    from kdfm import eval as E
    return E


VOCAB = [" "] + list(string.ascii_lowercase) + ["'"]


def _py_lev(a, b):
    prev = list(range(len(b) + 1))
    for i in range(1, len(a) + 1):
        cur = [i] + [0] * len(b)
        for j in range(1, len(b) + 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (a[i - 1] != b[j - 1]))
        prev = cur
    return prev[-1]


def test_word_error_rate_known_answers():
    # test_asr_metrics.py:119-124
    E = _ev()
    assert E.word_error_rate(hypotheses=['cat'], references=['cot']) == 1.0
    assert E.word_error_rate(hypotheses=['GPU'], references=['G P U']) == 1.0
    assert E.word_error_rate(hypotheses=['G P U'], references=['GPU']) == 3.0
    assert E.word_error_rate(hypotheses=['ducati motorcycle'], references=['motorcycle']) == 1.0
    assert E.word_error_rate(hypotheses=['ducati motorcycle'], references=['ducuti motorcycle']) == 0.5
    assert E.word_error_rate(hypotheses=['a B c'], references=['a b c']) == 1.0 / 3.0
    assert E.word_error_rate(hypotheses=['cat'], references=['']) == float("inf")
    with pytest.raises(ValueError):
        E.word_error_rate(hypotheses=['a'], references=['a', 'b'])


def test_edit_distance_matches_python_levenshtein():
    E = _ev()
    rng = random.Random(0)
    for _ in range(300):
        a = [rng.choice("abcd") for _ in range(rng.randint(0, 30))]
        b = [rng.choice("abcd") for _ in range(rng.randint(0, 30))]
        assert E.edit_distance(a, b) == _py_lev(a, b)
    assert E.edit_distance("kitten".split(), "sitting".split()) == 1
    assert E.edit_distance(list("kitten"), list("sitting")) == 3


def _string_to_ctc(txt):
    """test_asr_metrics.py:62-89: a CTC label sequence emitting txt (blank between repeats)."""
    blank = len(VOCAB)
    idx = {c: i for i, c in enumerate(VOCAB)}
    out, prev = [], -1
    for c in (idx[ch] for ch in txt):
        if c == prev:
            out.append(blank)
        out.append(c)
        prev = c
    return torch.tensor(out).unsqueeze(0)


def _wer_ctc(E, prediction, reference):
    wer = E.WER(E.CTCGreedyDecoding(E.CharVocabulary(VOCAB)), use_cer=False)
    idx = {c: i for i, c in enumerate(VOCAB)}
    tgt = torch.tensor([idx[c] for c in reference]).unsqueeze(0)
    wer.update(predictions=_string_to_ctc(prediction), predictions_lengths=None, targets=tgt,
               targets_lengths=torch.tensor([len(reference)]))
    return wer.compute()[0]


def test_wer_metric_simple():
    # test_asr_metrics.py:169-175
    E = _ev()
    assert _wer_ctc(E, 'cat', 'cot') == 1.0
    assert _wer_ctc(E, 'gpu', 'g p u') == 1.0
    assert _wer_ctc(E, 'g p u', 'gpu') == 3.0
    assert _wer_ctc(E, 'ducati motorcycle', 'motorcycle') == 1.0
    assert _wer_ctc(E, 'ducati motorcycle', 'ducuti motorcycle') == 0.5
    assert abs(_wer_ctc(E, 'a f c', 'a b c') - 1.0 / 3.0) < 1e-6


def test_wer_metric_randomized():
    # test_asr_metrics.py:177-198: the metric equals word_error_rate on the decoded strings
    E = _ev()
    rng = random.Random(1)
    for _ in range(64):
        s1 = ''.join(rng.choice(''.join(VOCAB)) for _ in range(rng.randint(1, 200)))
        s2 = ''.join(rng.choice(''.join(VOCAB)) for _ in range(rng.randint(1, 200)))
        if s2.strip():
            assert abs(_wer_ctc(E, s1, s2) - E.word_error_rate([s1], [s2])) < 1e-6


def test_label_collapse_rule():
    """fold repeats, drop blank (= 5 here), a blank separates a repeated token (App. A.9)"""
    E = _ev()
    lab = torch.tensor([[1, 1, 5, 1, 2, 2, 5, 5, 3, 1]])
    d = E.CTCGreedyDecoding(E.CharVocabulary("abcde"))
    assert d.ctc_decoder_predictions_tensor(lab)[0].y_sequence == [1, 1, 2, 3, 1]
    assert d.ctc_decoder_predictions_tensor(lab, torch.tensor([4]))[0].y_sequence == [1, 1]
    assert d.ctc_decoder_predictions_tensor(lab, fold_consecutive=False)[0].y_sequence == [1, 1, 1, 2, 2, 3, 1]
