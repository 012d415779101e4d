"""Where the striding conv0 weight gradient of the logit-KD module step departs from the float64 oracle:
per-tap and per-channel error, with the weight-gradient stream overlapped and serialised."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kd-via-fm-in-asr_amd")]
from oracle import ver5 as O  # noqa: E402


def run(overlap):
    from kdfm import kernels as K
    from kdfm.distill import DistilEncDecCTCModelBPE, EncDecCTCModelBPE
    from kdfm.overlap import WGRAD
    WGRAD.enabled = overlap
    K.set_math("f32")
    K.set_deterministic(True)
    n_layers, B, N = 2, 2, 16000
    kw = dict(n_layers=n_layers, dither=0.0, spec_augment=False, dropout=0.0, dropout_pre_encoder=0.0, dropout_att=0.0)
    torch.manual_seed(int(os.environ.get("DIAG_SEED", "0")))   # the decoders' default init
    teacher = EncDecCTCModelBPE(d_model=176, n_heads=4, device="cuda", init_seed=0, **kw)
    model = DistilEncDecCTCModelBPE(teacher, kd_alpha=0.1, kd_temperature=1.0, device="cuda", init_seed=1, **kw)
    g = torch.Generator().manual_seed(14)
    for name, buf in teacher.named_buffers():
        if name.endswith("running_var"):
            buf.copy_(1.0 + 0.3 * torch.rand(buf.shape, generator=g))
        elif name.endswith("running_mean"):
            buf.copy_(0.2 * torch.randn(buf.shape, generator=g))
    model.train()
    wav = 0.1 * torch.randn(B, N, generator=g)
    wl = torch.tensor([N, 12345], dtype=torch.int64)
    U = 9
    tg = torch.randint(0, 128, (B, U), generator=g)
    tl = torch.tensor([U, 4], dtype=torch.int64)
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    loss = model.training_step((wav.cuda(), wl.cuda(), tg.cuda(), tl.cuda()), 0)
    loss.backward()
    torch.cuda.synchronize()
    ocfg = O.StepConfig(n_layers=n_layers, kd_model="logitkd")
    p = dict(O.frontend_buffers(ocfg))
    p.update(O.frontend_buffers(ocfg, "teacher.preprocessor.featurizer."))
    for k, v in sd.items():
        if k.startswith(("encoder.", "decoder.", "teacher.encoder.", "teacher.decoder.")):
            p[k] = v
    names = O.trainable_names(p, kd_model="logitkd")
    p64 = {k: (v.double() if v.is_floating_point() else v) for k, v in p.items()}
    for k in names:
        p64[k] = p64[k].clone().requires_grad_(True)
    out = O.ver5_step(p64, wav.double(), wl, tg, tl, ocfg, None)
    og = dict(zip(names, torch.autograd.grad(out["loss"], [p64[k] for k in names], allow_unused=True)))
    params = dict(model.named_parameters())
    for k in ("encoder.pre_encode.conv.0.weight", "encoder.pre_encode.conv.0.bias", "encoder.pre_encode.conv.2.weight",
              "encoder.pre_encode.out.weight"):
        mine = params[k].grad.detach().cpu().double()
        ref = og[k]
        d = (mine - ref).abs()
        print(f"overlap={overlap} {k}: max err {d.max().item():.3e} of max {ref.abs().max().item():.3e}")
        if k.endswith("conv.0.weight"):
            dd = d.view(-1, 9)
            print("   per tap max err:", [f"{v:.2e}" for v in dd.max(0).values.tolist()])
            ch = dd.max(1).values
            top = torch.topk(ch, 6)
            print("   worst channels:", [(int(i), f"{v:.2e}", f"{ref.view(-1, 9)[i].abs().max().item():.2e}")
                                        for v, i in zip(top.values.tolist(), top.indices.tolist())])
            ratio = (mine.view(-1, 9) / ref.view(-1, 9))
            print("   mine/ref (channel 0):", [f"{v:.5f}" for v in ratio[0].tolist()])
    # the student's mel vs the oracle's
    if "mel" in out:
        print("oracle mel shape", tuple(out["mel"].shape))
        # the oracle's conv0 pre-activations nearest zero (a ReLU the GPU's f32 log-mel can flip)
        mel = out["mel"].detach().double().transpose(1, 2).unsqueeze(1)   # (B, 1, T, F)
        w0 = p64["encoder.pre_encode.conv.0.weight"].detach()
        b0 = p64["encoder.pre_encode.conv.0.bias"].detach()
        pre = torch.nn.functional.conv2d(mel, w0, b0, stride=2, padding=1)
        flat = pre.abs().flatten()
        idx = torch.topk(-flat, 4).indices
        for i in idx.tolist():
            b, rem = divmod(i, pre[0].numel())
            c, rem = divmod(rem, pre.shape[2] * pre.shape[3])
            t, f = divmod(rem, pre.shape[3])
            print(f"   near-zero conv0 pre-activation: b={b} ch={c} t={t} f={f} value={pre[b, c, t, f].item():.3e}")


if __name__ == "__main__":
    run(True)
    run(False)
