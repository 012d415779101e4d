import sys, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/kd-via-fm-in-asr_amd"); sys.path.insert(0, "/root/repo/tests")
import test_nemo_api_gpu as T
from oracle import ver5 as O
for rep in range(2):
    n_layers, B, N = 2, 2, 16000
    teacher, model = T._models(n_layers)
    model.train()
    g = torch.Generator().manual_seed(9)
    wav = 0.1 * torch.randn(B, N, generator=g)
    wl = torch.tensor([N, 13000], dtype=torch.int64)
    U = 9
    tg = torch.randint(0, 128, (B, U), generator=g)
    tl = torch.tensor([U, 5], dtype=torch.int64)
    Tt = ((N // 160) // 2) // 2 + 1
    eps = [torch.randn(B * Tt, 96, generator=g) for _ in range(n_layers)]
    model.adapter.eps_override = [e.cuda() for e in eps]
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    loss = model.training_step((wav.cuda(), wl.cuda(), tg.cuda(), tl.cuda()), 0)
    loss.backward(); torch.cuda.synchronize()
    ocfg = O.StepConfig(n_layers=n_layers)
    p = dict(O.frontend_buffers(ocfg)); p.update(O.frontend_buffers(ocfg, "teacher.preprocessor.featurizer."))
    for k, v in sd.items():
        if k.startswith(("encoder.", "decoder.", "teacher.encoder.", "teacher.decoder.", "tae.", "sproj.", "adapter.", "denoiser.", "fm_latent.")):
            p[k] = v
    names = O.trainable_names(p)
    for k in names: p[k] = p[k].clone().requires_grad_(True)
    eps_o = torch.stack([e.view(B, Tt, 96).permute(0, 2, 1) for e in eps])
    out = O.ver5_step(p, wav, wl, tg, tl, ocfg, eps_o)
    print("loss", loss.item(), out["loss"].item())
    og = torch.autograd.grad(out["loss"], [p[k] for k in names], allow_unused=True)
    params = dict(model.named_parameters())
    rows = []
    for k, gr in zip(names, og):
        if gr is None: continue
        mine = params[k].grad.detach().cpu()
        rows.append(((mine - gr).abs().max().item() / (gr.abs().max().item() + 1e-12), k))
    rows.sort(reverse=True)
    for r, k in rows[:8]: print(f"  {r:.2e} {k}")
