"""Evaluation path: the reference's validation / test pass.

Reference: NeMo EncDecCTCModel.validation_pass / test_step (ctc_models.py:625-692) as driven by
asr_inference_diffm.py:541-562 (trainer.test -> test_wer, test_loss) and the distillation model's
eval forward (asr_train_diffm.py:606-643, which returns (log_probs, enc_len, greedy) in eval mode):

  log_probs, enc_len, greedy = model.forward(input_signal, input_signal_length)
  loss = CTCLoss(log_probs, targets, enc_len, target_len)            # mean over the batch
  WER.update(predictions=log_probs, ...)  -> CTC greedy decode -> text -> editdistance
  metrics = {val_loss, val_wer_num, val_wer_denom, val_wer}           # test_* for test_step

Pieces:
  * ctc_greedy_decode — the device kernel kdfm_ctc_greedy (argmax, collapse repeats, drop blank;
    SURVEY.md Appendix A.9);
  * edit_distance — native Levenshtein distance (kdfm_edit_distance, the `editdistance` package's role);
  * word_error_rate — metrics/wer.py:35-73;
  * WER — the torchmetrics-style accumulator of metrics/wer.py:249-359 (scores, words);
  * CTCGreedyDecoding — ctc_decoder_predictions_tensor + decode_tokens_to_str over a character
    vocabulary or a SentencePiece model (the .nemo tokenizer, when one is available locally);
  * validation_pass / test_step — the metric dict of ctc_models.py:625-692 for a kdfm model or a
    Ver5Engine.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from . import kernels as K


# ------------------------------------------------------------------------------------------------
# native pieces
# ------------------------------------------------------------------------------------------------

def ctc_greedy_decode(log_probs: torch.Tensor, lengths: torch.Tensor | None, blank: int, fold: bool = True):
    """log_probs (B, T, C) device f32 -> list of B token-id lists (GPU kernel, one copy to host)."""
    if log_probs.dim() != 3:
        raise ValueError("log_probs must be (B, T, C)")
    B, T, Cn = log_probs.shape
    lp = log_probs.detach()
    if lp.stride(2) != 1 or lp.stride(1) != Cn or lp.stride(0) != T * Cn:
        lp = lp.contiguous()
    dev = lp.device
    tok = torch.empty(B, T, dtype=torch.int32, device=dev)
    ntok = torch.empty(B, dtype=torch.int32, device=dev)
    lens = None if lengths is None else lengths.to(device=dev, dtype=torch.int64).contiguous()
    K.call("kdfm_ctc_greedy", K.ptr(K._f32(lp)), Cn, K.ptr(lens), K.ptr(tok), K.ptr(ntok), None, B, T, Cn, int(blank),
           int(bool(fold)), K.stream_ptr())
    tok_h, n_h = tok.cpu().numpy(), ntok.cpu().numpy()
    return [tok_h[b, :n_h[b]].tolist() for b in range(B)]


def _collapse_labels(labels: np.ndarray, length: int, blank: int, fold: bool) -> list:
    """Host form of the same rule for integer label tensors (NeMo accepts label predictions too)."""
    out, prev = [], None
    for t in range(length):
        a = int(labels[t])
        if a != blank and (not fold or a != prev):
            out.append(a)
        prev = a
    return out


def edit_distance(a, b) -> int:
    """Levenshtein distance between two sequences of hashable items (editdistance.eval)."""
    if len(a) == 0:
        return len(b)
    if len(b) == 0:
        return len(a)
    codes: dict = {}
    ia = np.fromiter((codes.setdefault(x, len(codes)) for x in a), dtype=np.int32, count=len(a))
    ib = np.fromiter((codes.setdefault(x, len(codes)) for x in b), dtype=np.int32, count=len(b))
    d = _lib.lib().kdfm_edit_distance(ia.ctypes.data_as(C.c_void_p), len(ia), ib.ctypes.data_as(C.c_void_p), len(ib))
    if d < 0:
        raise _lib.KdfmError("kdfm_edit_distance: bad arguments")
    return int(d)


def word_error_rate(hypotheses, references, use_cer: bool = False) -> float:
    """metrics/wer.py:35-73: sum of word (or character) edit distances / sum of reference lengths."""
    if len(hypotheses) != len(references):
        raise ValueError("In word error rate calculation, hypotheses and reference lists must have the same "
                         f"number of elements. But I got:{len(hypotheses)} and {len(references)} correspondingly")
    scores = 0
    words = 0
    for h, r in zip(hypotheses, references):
        h_list, r_list = (list(h), list(r)) if use_cer else (h.split(), r.split())
        words += len(r_list)
        scores += edit_distance(h_list, r_list)
    return 1.0 * scores / words if words != 0 else float("inf")


# ------------------------------------------------------------------------------------------------
# decoding + metric objects (NeMo CTCDecoding 'greedy' / WER contract)
# ------------------------------------------------------------------------------------------------

@dataclass
class Hypothesis:
    text: str
    y_sequence: list = field(default_factory=list)


class CharVocabulary:
    """Character vocabulary (NeMo CTCDecoding with a label list): text = concatenated labels."""

    def __init__(self, labels):
        self.labels = list(labels)

    @property
    def vocab_size(self) -> int:
        return len(self.labels)

    def ids_to_text(self, ids) -> str:
        return "".join(self.labels[i] for i in ids)

    def text_to_ids(self, text: str):
        idx = {c: i for i, c in enumerate(self.labels)}
        return [idx[c] for c in text]


class SentencePieceTokenizer:
    """The .nemo model's SentencePiece tokenizer (ids -> text), loaded from a local model file."""

    def __init__(self, model_path: str):
        import sentencepiece as spm
        self.sp = spm.SentencePieceProcessor(model_file=model_path)

    @property
    def vocab_size(self) -> int:
        return int(self.sp.get_piece_size())

    def ids_to_text(self, ids) -> str:
        return self.sp.decode_ids([int(i) for i in ids])

    def text_to_ids(self, text: str):
        return list(self.sp.encode_as_ids(text))


class CTCGreedyDecoding:
    """Greedy CTC decoding; blank = vocabulary size (losses/ctc.py:46)."""

    def __init__(self, tokenizer, blank_id: int | None = None):
        self.tokenizer = tokenizer
        self.blank_id = tokenizer.vocab_size if blank_id is None else blank_id

    def decode_tokens_to_str(self, ids) -> str:
        return self.tokenizer.ids_to_text(ids)

    def ctc_decoder_predictions_tensor(self, decoder_outputs, decoder_lengths=None, fold_consecutive=True):
        """decoder_outputs: (B, T, C) float log-probs (device kernel) or (B, T) integer labels."""
        if decoder_outputs.dim() == 3 and decoder_outputs.is_floating_point():
            if not decoder_outputs.is_cuda:
                raise _lib.KdfmError("CTC greedy decoding of log-probs runs on the device; got a CPU tensor")
            seqs = ctc_greedy_decode(decoder_outputs, decoder_lengths, self.blank_id, fold_consecutive)
        else:
            lab = decoder_outputs.detach().long().cpu().numpy()
            if lab.ndim == 3:
                lab = lab.argmax(-1)
            lens = [lab.shape[1]] * lab.shape[0] if decoder_lengths is None else \
                decoder_lengths.detach().long().cpu().tolist()
            seqs = [_collapse_labels(lab[b], int(lens[b]), self.blank_id, fold_consecutive) for b in range(lab.shape[0])]
        return [Hypothesis(text=self.decode_tokens_to_str(s), y_sequence=s) for s in seqs]


class WER:
    """metrics/wer.py:249-359 (CTC decoding): update() accumulates word edit distances and reference
    word counts of one batch; compute() -> (wer, scores, words)."""

    def __init__(self, decoding: CTCGreedyDecoding, use_cer: bool = False, fold_consecutive: bool = True,
                 batch_dim_index: int = 0):
        self.decoding = decoding
        self.use_cer = use_cer
        self.fold_consecutive = fold_consecutive
        self.batch_dim_index = batch_dim_index
        self.reset()

    def reset(self):
        self.scores = 0
        self.words = 0

    def update(self, predictions, predictions_lengths, targets, targets_lengths, **_):
        if self.batch_dim_index != 0:
            targets = targets.transpose(0, self.batch_dim_index)
            predictions = predictions.transpose(0, self.batch_dim_index)
        tl = targets_lengths.long().cpu().tolist()
        tg = targets.long().cpu()
        references = [self.decoding.decode_tokens_to_str(tg[i, :tl[i]].tolist()) for i in range(tg.shape[0])]
        hyps = self.decoding.ctc_decoder_predictions_tensor(predictions, predictions_lengths,
                                                             fold_consecutive=self.fold_consecutive)
        scores = words = 0
        for h, r in zip(hyps, references):
            h_list, r_list = (list(h.text), list(r)) if self.use_cer else (h.text.split(), r.split())
            words += len(r_list)
            scores += edit_distance(h_list, r_list)
        self.scores, self.words = scores, words   # per-batch state, as the reference's update() sets it
        return hyps, references

    def compute(self):
        s, w = float(self.scores), float(self.words)
        return (s / w if w else float("inf")), s, w

    def __call__(self, **kw):
        return self.update(**kw)


# ------------------------------------------------------------------------------------------------
# validation / test pass
# ------------------------------------------------------------------------------------------------

def validation_pass(model, batch, wer: WER, ctc_blank: int | None = None) -> dict:
    """ctc_models.py:625-665 for a kdfm model (EncDecCTCModelBPE / DistilFlowMatchingCTCModelBPE in
    eval mode) or a Ver5Engine (its student: Ver5Engine.infer).  batch = (signal, signal_len,
    transcript, transcript_len)."""
    from .engine import Ver5Engine
    signal, signal_len, transcript, transcript_len = batch
    if isinstance(model, Ver5Engine):
        log_probs, enc_len = model.infer(signal, signal_len)
        loss = model.ctc_mean(log_probs, enc_len, transcript, transcript_len)
    else:
        with torch.no_grad():
            out = model.forward(input_signal=signal, input_signal_length=signal_len)
            log_probs, enc_len = out[0], out[1]
            loss = model.loss(log_probs=log_probs, targets=transcript, input_lengths=enc_len,
                              target_lengths=transcript_len)
    wer.update(predictions=log_probs, predictions_lengths=enc_len, targets=transcript, targets_lengths=transcript_len)
    w, num, den = wer.compute()
    wer.reset()
    return {"val_loss": float(loss), "val_wer_num": num, "val_wer_denom": den, "val_wer": w}


def test_step(model, batch, wer: WER) -> dict:
    """ctc_models.py:685-692: the validation pass with val_ -> test_ keys."""
    return {k.replace("val_", "test_"): v for k, v in validation_pass(model, batch, wer).items()}


def epoch_wer(outputs, prefix="val_") -> float:
    """Corpus WER of a list of step outputs: sum(num) / sum(denom) (multi_validation_epoch_end)."""
    num = sum(o[prefix + "wer_num"] for o in outputs)
    den = sum(o[prefix + "wer_denom"] for o in outputs)
    return num / den if den else float("inf")


__all__ = ["ctc_greedy_decode", "edit_distance", "word_error_rate", "Hypothesis", "CharVocabulary",
           "SentencePieceTokenizer", "CTCGreedyDecoding", "WER", "validation_pass", "test_step", "epoch_wer"]
