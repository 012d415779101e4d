"""Batched pos projection (conformer.pos_proj_all) vs the per-layer projection: bitwise repeatability of
the batched GEMM and its agreement with K.linear per layer, and the kdfm_gemm route it takes."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kd-via-fm-in-asr_amd"))


def main():
    from kdfm import kernels as K, _lib
    from kdfm.conformer import pos_proj_all
    from types import SimpleNamespace
    for det in (False, True):
        K.set_deterministic(det) if hasattr(K, "set_deterministic") else None
        for d, nl in ((88, 16), (176, 4)):
            npos, blk = 801, 88 * 88 * 13
            g = torch.Generator(device="cuda").manual_seed(0)
            flat = torch.randn(nl * blk, device="cuda", generator=g) * 0.1
            P = {f"layers.{i}.self_attn.linear_pos.weight": flat[i * blk:i * blk + d * d].view(d, d) for i in range(nl)}
            pos = torch.randn(npos, d, device="cuda", generator=g)
            cfg = SimpleNamespace(n_layers=nl)
            a = pos_proj_all(cfg, P, "", pos)
            route = int(_lib.lib().kdfm_gemm_last_route())
            b = pos_proj_all(cfg, P, "", pos)
            ref = torch.empty(nl, npos, d, device="cuda")
            for i in range(nl):
                K.linear(pos, P[f"layers.{i}.self_attn.linear_pos.weight"], None, ref[i])
            torch.cuda.synchronize()
            print(f"det={det} d={d} nl={nl} route={K.ROUTES.get(route, route)} repeat_equal={torch.equal(a, b)} "
                  f"vs_linear_maxdiff={(a - ref).abs().max().item():.3e} ref_scale={ref.abs().max().item():.3e}", flush=True)


if __name__ == "__main__":
    main()
