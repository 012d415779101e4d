"""CTC loss kernels (kdfm_ctc_loss: concurrent alpha / beta recursion blocks + per-frame posterior
/ gradient blocks, csrc/loss.hip) against torch.nn.functional.ctc_loss in float64 on the CPU
(NeMo CTCLoss -> torch CTCLoss, losses/ctc.py:68-82: blank = C-1, zero_infinity=True).

Cases: ragged input and target lengths, repeated labels (forced blanks), an infeasible utterance
(target longer than the frames: zero loss and zero gradient under zero_infinity), and target
lengths that take each states-per-thread instantiation (S = 2U+1 up to 1201).
Tolerances, float32 yardstick: alpha and beta are running log-space sums (|alpha| ~ 1e3 after 400
frames of random log-probs), so float32 rounding alone moves a posterior by ~1e-3 relative.  The
kernel's max error against float64 (nll and gradient, scale * (exp(lp) - posterior): the gradient
torch returns for normalised log-probs) must stay within 4x torch's OWN float32 CTC error on the same
inputs (+1e-6).  Two runs are bitwise identical.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _case(B, T, C, Umax, seed):
    g = torch.Generator().manual_seed(seed)
    lp = torch.log_softmax(torch.randn(B, T, C, generator=g, dtype=torch.float64) * 2, -1)
    in_len = torch.randint(max(1, T // 2), T + 1, (B,), generator=g)
    in_len[0] = T
    tgt_len = torch.minimum(torch.randint(1, Umax + 1, (B,), generator=g), (in_len - 1) // 2 + 1)
    tgt_len[0] = min(Umax, (T - 1) // 2 + 1)
    tg = torch.randint(0, C - 1, (B, Umax), generator=g)
    tg[0, 1::3] = tg[0, 0::3][: tg[0, 1::3].numel()]   # repeats: consecutive equal labels
    if B > 2:                                            # infeasible: more labels than frames
        in_len[2] = 3
        tgt_len[2] = min(Umax, 5)
    return lp, tg, in_len, tgt_len


def _run(K, lp, tg, in_len, tgt_len, scale):
    B, T, C = lp.shape
    Umax = tg.shape[1]
    dev = "cuda"
    lpf = lp.float().to(dev)
    S = 2 * Umax + 1
    a = torch.empty(B * T * S, device=dev)
    b = torch.empty_like(a)
    nll = torch.empty(B, device=dev)
    grad = torch.full((B, T, C), 7.0, device=dev)   # every cell must be written
    K.ctc_loss(lpf, tg.to(dev), in_len.to(dev), tgt_len.to(dev), a, b, nll, grad, B, T, C, C - 1, scale, True)
    torch.cuda.synchronize()
    return nll.cpu(), grad.cpu()


@pytest.mark.parametrize("B,T,C,Umax", [(6, 401, 129, 100), (3, 700, 129, 300), (2, 1300, 33, 600),
                                        (4, 7, 5, 3), (4, 401, 1025, 100)])
def test_ctc_matches_torch_float64(B, T, C, Umax):
    from kdfm import kernels as K
    lp, tg, in_len, tgt_len = _case(B, T, C, Umax, T + Umax)
    scale = 1.0 / B
    nll, grad = _run(K, lp, tg, in_len, tgt_len, scale)
    x = lp.float().double().clone().requires_grad_(True)   # the same fp32-rounded inputs
    ref = F.ctc_loss(x.transpose(0, 1), tg, in_len, tgt_len, blank=C - 1, reduction="none", zero_infinity=True)
    (gref,) = torch.autograd.grad(ref.sum() * scale, x)
    x32 = lp.float().clone().requires_grad_(True)
    r32 = F.ctc_loss(x32.transpose(0, 1), tg, in_len, tgt_len, blank=C - 1, reduction="none", zero_infinity=True)
    (g32,) = torch.autograd.grad(r32.sum() * scale, x32)
    yard_n = (r32.detach().double() - ref.detach()).abs().max().item()
    yard_g = (g32.double() - gref).abs().max().item()
    err_n = (nll.double() - ref.detach()).abs().max().item()
    err_g = (grad.double() - gref).abs().max().item()
    assert err_n <= 4 * yard_n + 1e-6 * ref.detach().abs().max().item(), (err_n, yard_n)
    assert err_g <= 4 * yard_g + 1e-6, (err_g, yard_g)
    for bi in range(B):   # frames past the input length get exactly zero gradient
        if int(in_len[bi]) < T:
            assert grad[bi, int(in_len[bi]):].abs().max().item() == 0.0
    if B > 2 and C > 5:
        assert nll[2].item() == 0.0 and grad[2].abs().max().item() == 0.0
    nll2, grad2 = _run(K, lp, tg, in_len, tgt_len, scale)
    assert torch.equal(nll, nll2) and torch.equal(grad, grad2)


@pytest.mark.parametrize("C", [129, 300, 1025, 3001])
def test_log_softmax_and_logit_kd_wide_vocab(C):
    """kdfm_log_softmax / kdfm_kl_div_logits beyond 256 classes (V = 1024 BPE: 1025 decoder outputs,
    conformer_ctc_bpe.yaml:87; SURVEY §8 V sensitivity) against float64 torch: log_softmax, and the
    logit KD of asr_train_diffm.py:751-756 (kl_div(log_softmax(s/T), softmax(t/T), 'batchmean') * T^2)
    with its gradient wrt the student log-probs' logits."""
    from kdfm import kernels as K
    g = torch.Generator().manual_seed(C)
    rows, Tk = 37, 2.0
    x = torch.randn(rows, C, generator=g, dtype=torch.float64) * 3
    t = torch.randn(rows, C, generator=g, dtype=torch.float64) * 3
    lp = torch.empty(rows, C, device="cuda")
    K.log_softmax(x.float().cuda(), lp)
    ref = torch.log_softmax(x.float().double(), -1)
    assert (lp.double().cpu() - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()
    grad = torch.zeros(rows, C, device="cuda")
    acc = torch.zeros(1, device="cuda")
    B = 3
    K.kl_div_logits(lp, t.float().cuda(), grad, acc, Tk, 0.1 * Tk / B, Tk * Tk / B)
    torch.cuda.synchronize()
    s_ = lp.double().cpu().clone().requires_grad_(True)
    kl = torch.nn.functional.kl_div(torch.log_softmax(s_ / Tk, -1), torch.softmax(torch.log_softmax(t.float().double(), -1)
                                                                                   / Tk, -1), reduction="sum") * Tk * Tk / B
    (gs,) = torch.autograd.grad(kl, s_)
    assert abs(acc.item() - kl.item()) <= 1e-4 * abs(kl.item()) + 1e-6, (acc.item(), kl.item())
    # the kernel returns d(0.1 * kl)/d(logits): the student log-probs' own log_softmax backward folded in
    # (sum of the per-row gradient is zero), so compare against dkl/ds projected onto the zero-sum space
    want = 0.1 * (gs - torch.exp(s_.detach()) * gs.sum(-1, keepdim=True))
    assert (grad.double().cpu() - want).abs().max().item() <= 1e-4 * want.abs().max().item() + 1e-7
