"""Benchmark: utterances/sec of the ver5 FM-distillation training step (BASELINE.json metric) on
N MI355X GPUs, one process per GPU (torch.distributed.run), weak scaling B=32 per GPU.

Workload (BASELINE.json configs[1] shape, synthetic): Conformer-CTC-small teacher (d176/h4/16L,
frozen, eval) -> halved student (d88/h2/16L) FM distillation, ver5 heads, 16 kHz audio of 16.0 s
(256000 samples) per utterance, U=100 target tokens, bf16 MFMA operands with fp32 accumulation and
fp32 storage, dropout 0.1, SpecAugment and dither on, AdamW + Noam.  A step is one full
forward + backward + (RCCL all-reduce) + optimizer update over one batch.

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

B_PER_GPU = 32
N_SAMPLES = 256000
U_TOKENS = 100
# attention + FFN dense contractions per utterance (student fwd+bwd + teacher fwd)
FFN_FLOPS_NOTE = "ffn_up GEMMs: 2*M*N*K per launch (M=B*T' rows, N=4d, K=d)"
MI355X_BF16_DENSE_TFLOPS = 2500.0   # /opt/skills/guides/MI355X_MICROARCH.md chip table (dense)
MI355X_F32_MFMA_TFLOPS = 157.3
MI355X_HBM_GBPS = 8000.0            # MI355X_MICROARCH.md §HBM (8 TB/s spec peak)
# PMC traffic of the roofline kernel (tools/pmc_traffic.sh -> tools/pmc_summary.py, 2 separate --pmc
# passes, FETCH_SIZE doubled per the gfx950 correction); committed under profiles/
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r01_s10_pmc_traffic.json")
ROOF_KERNEL = "kdfm::skc_fwd_kernel<3>"


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the committed PMC summary; template instantiations of
    the same kernel (e.g. the compile-time epilogue variants skc_fwd_kernel<3, E>) are pooled,
    launch-weighted, since the bench's timing tag covers all of them."""
    try:
        with open(PMC_TRAFFIC) as fh:
            rows = json.load(fh)
    except (OSError, ValueError):
        return None
    stem = kernel[:-1] if kernel.endswith(">") else kernel
    hit = [r for r in rows if r["kernel"] == kernel or r["kernel"].startswith(stem + ",")]
    n = sum(r["launches"] for r in hit)
    return sum(r["bytes_total"] for r in hit) / n if n else None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=B_PER_GPU)
    ap.add_argument("--samples", type=int, default=N_SAMPLES)
    ap.add_argument("--math", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as one captured HIP graph (measured slower: hipGraph replay ran the "
                         "teacher / weight-gradient / CTC streams serially, 43.9 vs 40.1 ms/step eager)")
    return ap.parse_args()


def cpu_baseline(threads: int, samples: int):
    """Oracle (pure-PyTorch CPU restatement of the same step, fp32) on a bounded sample:
    B=2 utterances of the same 16 s shape, 1 warm-up + 2 timed steps (forward + backward)."""
    from oracle import ver5 as O
    torch.set_num_threads(threads)
    ocfg = O.StepConfig()
    p = O.init_all(ocfg)
    names = O.trainable_names(p)
    for k in names:
        p[k].requires_grad_(True)
    Bc = 2
    g = torch.Generator().manual_seed(1234)
    wav = 0.1 * torch.randn(Bc, samples, generator=g)
    wl = torch.full((Bc,), samples, dtype=torch.int64)
    tg = torch.randint(0, ocfg.vocab, (Bc, U_TOKENS), generator=g)
    tl = torch.full((Bc,), U_TOKENS, dtype=torch.int64)
    T = ((samples // ocfg.hop) // 2) // 2 + 1
    eps = torch.randn(ocfg.n_layers, Bc, ocfg.latent, T, generator=g)
    times = []
    for i in range(3):
        t0 = time.perf_counter()
        out = O.ver5_step(p, wav, wl, tg, tl, ocfg, eps)
        torch.autograd.grad(out["loss"], [p[k] for k in names], allow_unused=True)
        times.append(time.perf_counter() - t0)
    per_step = sum(times[1:]) / len(times[1:])
    return {"value": round(Bc / per_step, 4), "unit": "utterances/sec", "cores": threads, "kind": "port",
            "sample": f"oracle/ver5.py fp32 forward+backward, B={Bc} x {samples / 16000:.1f} s utterances, "
                      f"mean of {len(times) - 1} steps after 1 warm-up ({per_step:.2f} s/step), "
                      f"torch.set_num_threads({threads})"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("KDFM_DIST_BACKEND", "nccl")   # gloo only for 1-GPU rehearsals
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from dataclasses import replace

    from kdfm import kernels as K
    from kdfm.config import DEFAULT
    from kdfm.engine import GraphedTrainStep, Ver5Engine, synthetic_batch

    cfg = replace(DEFAULT, math=args.math)
    K.set_math(cfg.math)
    eng = Ver5Engine(cfg, dev)
    eng.set_seed(1000 + rank)
    wav, wl, tg, tl = synthetic_batch(cfg, args.batch, args.samples, U_TOKENS, dev, seed=1234 + rank)

    from kdfm.ddp import BucketedGradAllReduce, max_over_ranks
    # RCCL over xGMI: the flat 13.8 MB gradient buffer in 4 buckets, each all-reduced on a comm
    # stream as soon as the backward has finalised it (heads, decoder, layers 15..0)
    ar = BucketedGradAllReduce(eng.student.numel, buckets=4) if world > 1 else None
    # warm-up: one eager step (lazy buffers, allocator pools), graph capture, then replays
    eng.train_step(wav, wl, tg, tl, ar)
    if not args.graph:
        # eager multi-stream issue: teacher encoder, weight-gradient GEMMs and CTC/KL overlap the
        # student / head chain on their own HIP streams
        run = lambda: eng.train_step(wav, wl, tg, tl, ar)  # noqa: E731
    else:
        graphed = GraphedTrainStep(eng, wav, wl, tg, tl, ar, world)
        run = graphed.step
    for _ in range(max(0, args.warmup - 1)):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    # dominant-kernel timing: one instrumented eager step right after the timed replays, every
    # ffn_up launch bracketed by HIP events on the stream it runs on (main or teacher stream)
    trace = K.Trace(["ffn_up", "deno_conv"])
    with trace:
        eng.train_step(wav, wl, tg, tl, ar)
    torch.cuda.synchronize()
    losses = eng.losses.detach().cpu().tolist()
    tsum = trace.summary()
    empty = {"launches": 0, "ms_total": 0.0, "flops_total": 0.0, "bytes_total": 0.0}
    summ = tsum.get("ffn_up", empty)
    deno = tsum.get("deno_conv", empty)
    if rank == 0:
        utt = world * args.batch * args.steps / elapsed
        n_l = max(1, summ["launches"])
        avg_ms = summ["ms_total"] / n_l
        flops_per_launch = summ["flops_total"] / n_l
        achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
        peak = MI355X_BF16_DENSE_TFLOPS if cfg.math == "bf16" else MI355X_F32_MFMA_TFLOPS
        # roofline subject: the dominant kernel of the step (rocprof: the denoiser k=3 conv products,
        # kdfm_gemm skinny CONV mode) - HBM-bound (72 flop/B at f32 storage << the bf16 ridge)
        d_l = max(1, deno["launches"])
        d_ms = deno["ms_total"] / d_l
        d_bytes = deno["bytes_total"] / d_l
        d_gbps = d_bytes / (d_ms * 1e-3) / 1e9 if d_ms > 0 else 0.0
        d_traffic = pmc_traffic(ROOF_KERNEL)
        cpu = None
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_threads, args.samples)
        line = {
            "metric": "utterances/sec (FM-distill train step, Conformer-CTC-small) at 1/2/4/8 MI355X",
            "value": round(utt, 3),
            "unit": "utterances/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": cfg.math,
            "data": "synthetic (0.1*N(0,1) 16 kHz audio, random-init weights; no network for corpora/checkpoints)",
            "config": {"workload": "ver5 FM-distill step, Conformer-CTC-small teacher (d176 h4 L16) -> student "
                                   "(d88 h2 L16), BASELINE.json configs[1] shape",
                       "global_batch": world * args.batch, "seq_len": args.samples,
                       "frames_subsampled": (args.samples // 160) // 4 + 1, "parallelism": f"dp{world}"},
            "roofline": {"bound": "hbm",
                         "kernel": "kdfm_gemm CONV (denoiser Conv1d k=3 over 16 stacked layers, 205312 x 96 x 288, "
                                   "LDS-slab skc_fwd_kernel<3>)",
                         "achieved": round(d_gbps, 1), "peak": MI355X_HBM_GBPS, "unit": "GB/s",
                         "frac": round(d_gbps / MI355X_HBM_GBPS, 4), "traffic": d_traffic,
                         "traffic_source": "profiles/r01_s10_pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE)",
                         "launches": deno["launches"], "avg_ms": round(d_ms, 5), "bytes_per_launch": d_bytes},
            "roofline_mfma_ffn": {"bound": "mfma", "kernel": "kdfm_gemm ffn_up (Conformer FFN d->4d, SiLU+dropout)",
                                  "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s",
                                  "frac": round(achieved / peak, 5), "launches": summ["launches"],
                                  "avg_ms": round(avg_ms, 5), "flops_per_launch": flops_per_launch},
            "cpu_baseline": cpu,
            "losses_last_step": [round(x, 5) for x in losses],
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
