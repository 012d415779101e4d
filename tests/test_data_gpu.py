"""Manifest loader -> ver5 step on the GPU: the batches ManifestBatchLoader lands on cuda:0 (copy
stream + event) equal the host collate, and one training step of the HIP engine runs on them."""
import pytest
import torch

from kdfm import data as D

from test_data import _toy_corpus

pytestmark = pytest.mark.gpu


def test_loader_feeds_engine_train_step(tmp_path):
    from dataclasses import replace

    from kdfm.config import PARITY
    from kdfm.engine import Ver5Engine

    assert torch.cuda.is_available()
    mp, tok, texts, sigs = _toy_corpus(tmp_path)
    ds = D.AudioToBPEDataset(mp, tok, max_duration=16.7, min_duration=0.1)
    cfg = replace(PARITY, n_layers=2)
    assert tok.vocab_size <= cfg.vocab
    ld = D.ManifestBatchLoader(ds, 3, shuffle=False, threads=4, device="cuda:0", pad_to_samples=32000)
    host = D.ManifestBatchLoader(ds, 3, shuffle=False, pad_to_samples=32000)
    eng = Ver5Engine(cfg, "cuda:0")
    batches = ld._batches()
    n = 0
    for (audio, al, tk, tl), ids in zip(ld, batches):
        assert audio.is_cuda and tk.is_cuda
        ref = host.load_host(ids)
        for g, r in zip((audio, al, tk, tl), ref):
            assert torch.equal(g.cpu(), r)
        ctx = eng.forward(audio, al, tk, tl, train=True)
        eng.backward(ctx)
        eng.optimizer_step()
        torch.cuda.synchronize()
        assert torch.isfinite(eng.losses).all()
        n += 1
    assert n == len(batches) == 3
