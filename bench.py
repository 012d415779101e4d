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
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
sys.path.insert(0, ROOT)

import kdfm  # noqa: E402,F401  (sets HIP_FORCE_DEV_KERNARG before the HIP runtime initialises)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

B_PER_GPU = 32
N_SAMPLES = 256000
U_TOKENS = 100
# attention + FFN dense contractions per utterance (student fwd+bwd + teacher fwd)
MI355X_BF16_DENSE_TFLOPS = 2500.0   # /opt/skills/guides/MI355X_MICROARCH.md chip table (dense)
MI355X_F32_MFMA_TFLOPS = 157.3
MI355X_HBM_GBPS = 8000.0            # MI355X_MICROARCH.md §HBM (8 TB/s spec peak)
# PMC traffic per kernel (tools/pmc_traffic.sh -> tools/pmc_summary.py: separate --pmc FETCH_SIZE and
# WRITE_SIZE passes, FETCH_SIZE doubled per the gfx950 correction), committed under profiles/
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r06_pmc_traffic.json")
# the committed rocprofv3 kernel summary of this bench command (tools/prof_summary.py over a kernel trace, whole
# steps): each family's kernel ms/step from it is printed beside the HIP-event timing (tools/roofline_check.py)
KERNEL_SUMMARY = [os.path.join(ROOT, "profiles", "r06", n) for n in ("final_kernel_summary.txt",
                                                                        "close1_kernel_summary.txt")]
# kdfm_gemm kernel family (kernels.ROUTES) -> kernel-name stems in the rocprofv3 / PMC summaries
ROUTE_KERNELS = {"generic": ("gemm_kernel",), "skinny": ("sk_fwd_kernel", "skd_fwd_kernel"),
                 "rowstream_fwd": ("rs_fwd_kernel",), "wide_wgrad": ("rs_wgrad_kernel", "rs_fold_kernel"),
                 "split_fold": ("gemm_kernel", "rs_fold_kernel"), "slab_conv": ("skc_fwd_kernel",),
                 "wgrad_rows": ("wgr_kernel", "wgd_kernel", "wgr_fold_kernel", "wgr_fold4_kernel", "wgr_fold_batch_kernel")}
# the fused kernels traced outside kdfm_gemm (kernels._traced tags) -> kernel-name stems
FAMILY_KERNELS = {"ffn_fwd": ("ffn_fwd_kernel",), "ffn_bwd": ("ffn_bwd_kernel",),
                  "wgrad_bf16": ("wgr_kernel", "wgd_kernel", "wgr_fold_kernel", "wgr_fold4_kernel",
                                 "wgr_fold_batch_kernel"),
                  "attn_fwd": ("relpos_attn_fwd_kernel", "relpos_attn_fwd3_kernel"),
                  "attn_prep": ("attn_kv_prep_kernel", "attn_band_prep_kernel"),
                  "attn_bwd": ("attn_bwd_dq_kernel", "attn_bwd_dkv_kernel", "attn_bwd_dpos_kernel",
                               "attn_bwd_dkv2_kernel", "attn_bwd_dpos2_kernel", "attn_rowdot_kernel",
                               "attn_dpos_fold_kernel")}
# FLOPs per utterance of one training step (B=32, 16.0 s) and of its attention +
# FFN dense contractions (student fwd+bwd + teacher fwd), the north-star MFMA roofline subject
STEP_GFLOP_PER_UTT = 62.6
ATTN_FFN_GFLOP_PER_UTT = 23.0


def _is_call_kernel(stem):
    """Kernels that start a traced call; folds / row-dot prologues run inside a call and add bytes, not calls."""
    return "fold" not in stem and "rowdot" not in stem


def pmc_traffic(stems):
    """HBM bytes per CALL of a kernel family from the committed PMC summary: every family kernel's
    bytes (main kernels, their folds) divided by the launches of the main kernels only, i.e. the same
    unit as `bytes_per_launch` (one traced call = one main launch + its fold); None if absent."""
    try:
        with open(PMC_TRAFFIC) as fh:
            rows = json.load(fh)
    except (OSError, ValueError):
        return None
    name = lambda r: r["kernel"].split(" ")[0].split("<")[0]  # noqa: E731
    hit = [r for r in rows if any(name(r).endswith(st) for st in stems)]
    n = sum(r["launches"] for r in hit if _is_call_kernel(name(r)))
    return round(sum(r["bytes_total"] for r in hit) / n, 1) if n else None


def _summary_path():
    return next((pth for pth in KERNEL_SUMMARY if os.path.exists(pth)), None)


def profile_ms(stems):
    """A family's kernel ms/step in the committed kernel summary (None if absent): its lines
    '<ms> ms/step <n>/step avg <us> us <kernel name>' whose kernel base name is one of `stems`."""
    pth = _summary_path()
    if pth is None:
        return None
    tot, hit = 0.0, False
    with open(pth) as fh:
        for ln in fh:
            parts = ln.split()
            if len(parts) < 7 or parts[1] != "ms/step":
                continue
            name = " ".join(parts[6:]).replace("void ", "").split("<")[0].split("(")[0].strip()
            if name.split("::")[-1] in stems:
                tot += float(parts[0])
                hit = True
    return round(tot, 3) if hit else None


def _family_stems(fam):
    if fam == "wgrad_rows":
        return tuple(set(ROUTE_KERNELS["wgrad_rows"]) | set(FAMILY_KERNELS["wgrad_bf16"]))
    return FAMILY_KERNELS.get(fam) or ROUTE_KERNELS.get(fam, (fam,))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=B_PER_GPU)
    ap.add_argument("--samples", type=int, default=N_SAMPLES)
    ap.add_argument("--math", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads for the CPU baseline (default: every core this process may use, its "
                         "affinity set capped by the cgroup CPU quota; os.cpu_count() is reported beside it)")
    ap.add_argument("--no-f32-sensitivity", action="store_true",
                    help="skip the --math f32 sensitivity measurement (the reference trains fp32)")
    ap.add_argument("--deterministic", action="store_true",
                    help="ordered reductions everywhere (bitwise-reproducible steps; kdfm_set_deterministic)")
    ap.add_argument("--eager", action="store_true",
                    help="issue every timed step through the Python wrappers instead of replaying the recorded "
                         "step plan (kdfm/plan.py)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as one captured HIP graph (measured slower: hipGraph replay ran the "
                         "teacher / weight-gradient / CTC streams serially, 43.9 vs 40.1 ms/step eager)")
    return ap.parse_args()


def attn_ffn_gflop_per_utt(cfg, samples):
    """SURVEY.md §8(d)'s MFMA-bound contractions per utterance, from the layer dimensions: per ConformerLayer
    and utterance of T frames, the two FFNs (32 T d^2) + q|k|v and out projections (8 T d^2) + scores,
    rel-pos band and P V (8 T^2 d); student forward + backward (x3) + teacher forward.  23.0 GFLOP/utt at the
    Conformer-CTC-small bench shape (d 88 / 176, T 401)."""
    from kdfm.config import sub_dims
    T = sub_dims(cfg, samples // cfg.hop + 1)[-1][0]
    per = lambda d: 40.0 * T * d * d + 8.0 * T * T * d  # noqa: E731
    return (3 * cfg.n_layers * per(cfg.d_student) + cfg.n_layers * per(cfg.d_teacher)) / 1e9


# FastConformer-XL layer shapes (BASELINE.json configs[4]; fast-conformer_ctc_bpe.yaml:29 XLarge row: d_model 1024,
# 8 heads -> head dim 128, 24 layers, conv kernel 9, xscaling False; dw_striding x8 with 256 channels, :113-125)
# for student and teacher: the one config change of the xl_shape_sensitivity line
XL_SHAPES = dict(d_student=1024, heads_student=8, d_teacher=1024, heads_teacher=8, n_layers=24,
                 subsampling="dw_striding", subsampling_factor=8, subsampling_conv_channels=256, conv_kernel=9,
                 xscaling=False, sched_d_model=1024)


def sensitivity(dev, samples, steps=3, **overrides):
    """utt/s of the same step with one configuration change (1 warm-up + `steps` timed eager steps on a
    separate engine): math="f32" -- exact-f32 MFMA arithmetic, the reference trains fp32
    (asr_train_diffm.py:1762-1769); vocab=1024 -- a 1024-token BPE tokenizer, 1025 decoder classes
    (conformer_ctc_bpe.yaml:87, SURVEY.md §8 V sensitivity)."""
    from dataclasses import replace

    from kdfm import kernels as K
    from kdfm.config import DEFAULT
    from kdfm.engine import Ver5Engine, synthetic_batch
    cfg = replace(DEFAULT, **overrides)
    eng = Ver5Engine(cfg, dev)
    eng.set_seed(1000)
    wav, wl, tg, tl = synthetic_batch(cfg, B_PER_GPU, samples, U_TOKENS, dev, seed=1234)
    with K.mode(cfg.math, fp8=cfg.linear_fp8):
        eng.train_step(wav, wl, tg, tl)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.train_step(wav, wl, tg, tl)
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    del eng
    torch.cuda.empty_cache()
    utt = B_PER_GPU * steps / el
    peak = MI355X_BF16_DENSE_TFLOPS if cfg.math == "bf16" else MI355X_F32_MFMA_TFLOPS
    gf = attn_ffn_gflop_per_utt(cfg, samples)
    return {"value": round(utt, 3), "unit": "utterances/sec", "ms_per_step": round(1e3 * el / steps, 3),
            "steps": steps, "issue": "eager", "config_change": overrides,
            "attn_ffn_gflop_per_utt": round(gf, 2),
            "attn_ffn_mfma_frac": round(gf * 1e9 * utt / (peak * 1e12), 5),
            "note": "same workload with this one change; sensitivity only, not the headline value"}


def _cgroup_cpu_max():
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            return fh.read().strip()
    except OSError:
        return None


def _usable_cpus():
    n = len(os.sched_getaffinity(0))
    q = _cgroup_cpu_max()
    if q and not q.startswith("max"):
        quota, period = (int(v) for v in q.split()[:2])
        n = min(n, max(1, quota // period))
    return n


def _progress(msg):
    # the GPU pool's watchdog kills a command that prints nothing for 3 minutes: long CPU phases report
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(threads: int, samples: int, batches=(2, 32), steps: int = 5, budget_s: float = 25.0):
    """Oracle (pure-PyTorch CPU restatement of the same step, fp32: frontend x2, teacher + student
    encoders, decoders, CTC, logit KD, ver5 heads, autograd backward) on the host cores, per
    BASELINE.md: B=2 (config 1) and B=32 (the bench batch) utterances of the same 16 s shape,
    1 warm-up + up to `steps` timed forward+backward steps each (fewer once a batch size has used
    `budget_s` seconds, at least 2), median.  `value` is the B=32 rate."""
    import platform
    import statistics
    from oracle import ver5 as O
    torch.set_num_threads(threads)
    ocfg = O.StepConfig()
    p = O.init_all(ocfg)
    names = O.trainable_names(p)
    for k in names:
        p[k].requires_grad_(True)
    T = ((samples // ocfg.hop) // 2) // 2 + 1
    res = {}
    for Bc in batches:
        g = torch.Generator().manual_seed(1234)
        wav = 0.1 * torch.randn(Bc, samples, generator=g)
        wl = torch.full((Bc,), samples, dtype=torch.int64)
        tg = torch.randint(0, ocfg.vocab, (Bc, U_TOKENS), generator=g)
        tl = torch.full((Bc,), U_TOKENS, dtype=torch.int64)
        eps = torch.randn(ocfg.n_layers, Bc, ocfg.latent, T, generator=g)
        times = []
        t_start = time.perf_counter()
        for i in range(steps + 1):
            t0 = time.perf_counter()
            out = O.ver5_step(p, wav, wl, tg, tl, ocfg, eps)
            torch.autograd.grad(out["loss"], [p[k] for k in names], allow_unused=True)
            times.append(time.perf_counter() - t0)
            del out
            _progress(f"cpu_baseline threads={threads} B={Bc} step {i} ({'warm-up' if i == 0 else 'timed'}): "
                      f"{times[-1]:.2f} s")
            if i >= 2 and time.perf_counter() - t_start > budget_s:
                break
        med = statistics.median(times[1:])
        res[Bc] = {"utt_per_s": round(Bc / med, 4), "s_per_step_median": round(med, 3),
                   "s_per_step": [round(t, 3) for t in times[1:]]}
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            cpu = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), cpu)
    except OSError:
        cpu = platform.processor() or cpu
    big = max(batches)
    nt = len(res[big]["s_per_step"])
    return {"value": res[big]["utt_per_s"], "unit": "utterances/sec", "cores": threads, "kind": "port",
            "cpu_model": cpu, "host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "by_batch": {str(b): v for b, v in res.items()},
            "sample": f"oracle/ver5.py fp32 forward+backward of the same step, B={list(batches)} x "
                      f"{samples / 16000:.1f} s utterances, median of {nt} timed steps (B={big}) after 1 warm-up, "
                      f"torch.set_num_threads({threads}); value = B={big}"}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def rank_launch_cmd(argv, gpus: int, port: int) -> list:
    """The command that runs this benchmark as `gpus` ranks on one node (one process per GPU,
    torch.distributed.run over 127.0.0.1), forwarding this process's own arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def visible_gpu_count(environ=None, kfd_nodes="/sys/class/kfd/kfd/topology/nodes"):
    """GPUs this process could use, without initialising any GPU runtime (the launcher parent forks and
    execs the ranks, so it must stay GPU-free by construction): the device list of HIP_VISIBLE_DEVICES /
    ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when one is set (the innermost mask HIP applies), else the
    KFD topology nodes with a non-zero simd_count (CPU nodes report 0).  None when neither says."""
    env = os.environ if environ is None else environ
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            return len([t for t in v.split(",") if t.strip() and t.strip() != "-1"])
    try:
        nodes = os.listdir(kfd_nodes)
    except OSError:
        return None
    n = 0
    for node in nodes:
        try:
            with open(os.path.join(kfd_nodes, node, "properties")) as fh:
                props = dict(ln.split(None, 1) for ln in fh.read().splitlines() if ln.strip())
        except (OSError, ValueError):
            continue
        if int(props.get("simd_count", "0").strip() or 0) > 0:
            n += 1
    return n


def launch_ranks(args, argv, run=None) -> int | None:
    """`bench.py --gpus N` outside a launcher (no WORLD_SIZE in the environment) with N > 1: start the N
    ranks as child processes and return their exit code (the reference trains with Lightning's
    `devices=args.gpus`, asr_train_diffm.py:1762-1769).  This process never touches the GPU (nothing here
    initialises HIP; the children are fresh processes, not an exec).  Inside a launcher (WORLD_SIZE set)
    each rank checks that the launcher's world size is the one asked for.  Returns None when this process
    is itself the (only) rank to run."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks")
        return None
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus == 1:
        return None
    backend = os.environ.get("KDFM_DIST_BACKEND", "nccl")
    n_dev = visible_gpu_count()   # environment / sysfs only: nothing in the parent touches torch.cuda or HIP
    if backend == "nccl" and n_dev and n_dev < args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {n_dev} "
                         f"(KDFM_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs)")
    cmd = rank_launch_cmd(argv, args.gpus, _free_port())
    _progress("launching " + " ".join(cmd))
    import subprocess
    return (run or subprocess.call)(cmd)


def main():
    args = parse()
    rc = launch_ranks(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
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

    cfg = replace(DEFAULT, math=args.math, deterministic=args.deterministic)
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
    issue = "eager"
    if args.graph:
        issue = "hip_graph"
    elif args.eager:
        # eager multi-stream issue: teacher encoder, weight-gradient GEMMs and CTC/KL overlap the
        # student / head chain on their own HIP streams
        run = lambda: eng.train_step(wav, wl, tg, tl, ar)  # noqa: E731
    else:
        # the same four-stream schedule replayed from a recorded step plan: the launches, cross-stream
        # edges and all-reduce callbacks of one step, re-issued without the Python wrappers (the
        # recording is itself a full training step)
        plan = eng.make_plan(wav, wl, tg, tl, ar)
        run = plan.replay
        issue = f"step plan ({len(plan)} recorded ops)"
    if args.graph:
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
    if os.environ.get("KDFM_PLAN_KNOCKOUT") and rank == 0:   # what-if probe (kdfm/plan.py): not a bench line
        print(f"KNOCKOUT {os.environ['KDFM_PLAN_KNOCKOUT']} ms_per_step {1e3 * elapsed / args.steps:.3f}", flush=True)
        return
    # live per-kernel timing over the schedule that was timed: a second step plan recorded with
    # every traced launch -- each kdfm_gemm launch (keyed by the kernel family libkdfm routed it to), the fused
    # kernels, the frontend, the depthwise convs -- bracketed by HIP events on the stream it runs on.  The events
    # are part of that plan (each replay re-records them in place), so the durations come from a REPLAYED step with
    # the same four-stream overlap and contention as the timed ones (the round-5 line took them from an eager
    # instrumented step: 1.3x more optimistic than the rocprof summary of the replayed step).  Eager / graph issue:
    # one instrumented eager step.
    trace = K.Trace(["*", "frontend", "dwconv", "ffn_fwd", "ffn_bwd", "wgrad_bf16", "wgrad_fold", "attn_fwd", "attn_prep",
                     "attn_bwd"])
    trace_issue = "eager instrumented step"
    if not args.eager and not args.graph:
        with trace:
            tplan = eng.make_plan(wav, wl, tg, tl, ar)
        tplan.replay()   # one warm replay; the events keep the timestamps of the last one
        torch.cuda.synchronize()
        tplan.replay()
        trace_issue = f"replayed step plan with per-launch HIP events ({len(tplan)} ops)"
    else:
        with trace:
            eng.train_step(wav, wl, tg, tl, ar)
    torch.cuda.synchronize()
    losses = eng.losses.detach().cpu().tolist()
    if not all(math.isfinite(x) for x in losses):
        raise RuntimeError(f"non-finite losses after the timed steps: {losses}")
    tsum = trace.summary()
    # the plans keep their steps' activations alive: release them before the sensitivity engines are built
    tplan = plan = run = None
    torch.cuda.empty_cache()
    empty = {"launches": 0, "ms_total": 0.0, "flops_total": 0.0, "bytes_total": 0.0}
    if rank == 0:
        utt = world * args.batch * args.steps / elapsed
        utt_gpu = utt / world
        bf16_peak = MI355X_BF16_DENSE_TFLOPS if cfg.math == "bf16" else MI355X_F32_MFMA_TFLOPS

        def rate(t):
            n = max(1, t["launches"])
            ms = t["ms_total"] / n
            gbps = (t["bytes_total"] / n) / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
            tfl = (t["flops_total"] / n) / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
            return n, ms, gbps, tfl

        routes = {k[5:]: v for k, v in tsum.items() if k.startswith("gemm:")}
        # the row-parallel weight gradients run both inside kdfm_gemm (f32 operands) and as kdfm_wgrad_bf16
        # (bf16 operands): one kernel family
        if "wgrad_bf16" in tsum:
            w = dict(routes.get("wgrad_rows", empty))
            for k in ("launches", "ms_total", "flops_total", "bytes_total"):
                w[k] = w.get(k, 0) + tsum["wgrad_bf16"][k]
            # deferred folds (kdfm_wgrad_fold_flush: one batched launch per encoder layer) run outside the
            # products' traced calls: their time joins the family, not their launch count (a call stays one
            # product + its fold)
            if "wgrad_fold" in tsum:
                w["ms_total"] += tsum["wgrad_fold"]["ms_total"]
            routes["wgrad_rows"] = w
        for fam in ("ffn_fwd", "ffn_bwd", "attn_fwd", "attn_prep", "attn_bwd"):
            if fam in tsum:
                routes[fam] = tsum[fam]
        by_route = {}
        for r, t in sorted(routes.items(), key=lambda kv: -kv[1]["ms_total"]):
            n, ms, gbps, tfl = rate(t)
            by_route[r] = {"launches": n, "ms_per_step": round(t["ms_total"], 3), "avg_ms": round(ms, 5),
                           "GB_per_s": round(gbps, 1), "TFLOP_per_s": round(tfl, 2),
                           "bytes_per_launch": round(t["bytes_total"] / n, 1),
                           "flops_per_launch": round(t["flops_total"] / n, 1),
                           "profile_ms_per_step": profile_ms(_family_stems(r))}
        dom = next(iter(by_route)) if by_route else "generic"
        dt = routes.get(dom, empty)
        n, ms, gbps, tfl = rate(dt)
        intensity = dt["flops_total"] / max(1.0, dt["bytes_total"])
        ridge = bf16_peak * 1e12 / (MI355X_HBM_GBPS * 1e9)
        if intensity < ridge:
            roof = {"bound": "hbm", "achieved": round(gbps, 1), "peak": MI355X_HBM_GBPS, "unit": "GB/s",
                    "frac": round(gbps / MI355X_HBM_GBPS, 4)}
        else:
            roof = {"bound": "mfma", "achieved": round(tfl, 2), "peak": bf16_peak, "unit": "TFLOP/s",
                    "frac": round(tfl / bf16_peak, 4)}
        stems = FAMILY_KERNELS.get(dom) or ROUTE_KERNELS.get(dom, (dom,))
        roof.update({"traffic": pmc_traffic(stems),
                     "traffic_source": os.path.relpath(PMC_TRAFFIC, ROOT) + " (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, "
                                       "all of the family's kernels incl. folds, per call = per main-kernel launch)",
                     "kernel": f"{dom} family ({', '.join(stems)}): the kernel family with the largest aggregated "
                               f"time of the step (kdfm_gemm routes + the fused kernels, HIP events on their streams)",
                     "timing_source": trace_issue,
                     "profile_ms_per_step": profile_ms(_family_stems(dom)),
                     "profile_source": (os.path.relpath(_summary_path(), ROOT) + " (rocprofv3 --kernel-trace of this "
                                        "bench command, whole steps; tools/roofline_check.py)") if _summary_path() else None,
                     "launches": n, "avg_ms": round(ms, 5), "bytes_per_launch": round(dt["bytes_total"] / n, 1),
                     "flops_per_launch": round(dt["flops_total"] / n, 1),
                     "arith_intensity_flop_per_byte": round(intensity, 2)})
        # the critical path: the compute stream carries the student chain and the whole backward's data
        # gradients (the teacher, weight gradients and CTC/KL overlap it on their own streams)
        csum = trace.summary(stream=eng.compute_stream.cuda_stream)
        croutes = {k[5:]: v for k, v in csum.items() if k.startswith("gemm:")}
        for fam in ("ffn_fwd", "ffn_bwd", "attn_fwd", "attn_prep", "attn_bwd", "wgrad_bf16"):
            if fam in csum:
                croutes[fam] = csum[fam]
        crit = None
        if croutes:
            cdom, ct = max(croutes.items(), key=lambda kv: kv[1]["ms_total"])
            cn, cms, cgbps, ctfl = rate(ct)
            cint = ct["flops_total"] / max(1.0, ct["bytes_total"])
            cb = "hbm" if cint < ridge else "mfma"
            crit = {"bound": cb, "achieved": round(cgbps if cb == "hbm" else ctfl, 2),
                    "peak": MI355X_HBM_GBPS if cb == "hbm" else bf16_peak, "unit": "GB/s" if cb == "hbm" else "TFLOP/s",
                    "frac": round((cgbps / MI355X_HBM_GBPS) if cb == "hbm" else (ctfl / bf16_peak), 4),
                    "kernel": f"{cdom} family: the most time on the compute (critical-path) stream",
                    "ms_per_step_on_stream": round(ct["ms_total"], 3), "launches": cn, "avg_ms": round(cms, 5),
                    "traffic": pmc_traffic(FAMILY_KERNELS.get(cdom) or ROUTE_KERNELS.get(cdom, (cdom,))),
                    "by_family_ms": {k: round(v["ms_total"], 3) for k, v in
                                     sorted(croutes.items(), key=lambda kv: -kv[1]["ms_total"])}}
        # MFMA rate of the attention / FFN kernels (the north-star MFMA subject) per family
        mfma_fams = {}
        for fam in ("ffn_fwd", "ffn_bwd", "attn_fwd", "attn_bwd"):
            if fam in tsum:
                n_, ms_, _, tfl_ = rate(tsum[fam])
                mfma_fams[fam] = {"TFLOP_per_s": round(tfl_, 2), "frac_bf16_peak": round(tfl_ / bf16_peak, 5),
                                  "launches": n_, "avg_ms": round(ms_, 5),
                                  "flops_per_launch": round(tsum[fam]["flops_total"] / n_, 1)}
        fe = rate(tsum.get("frontend", empty))
        dw = rate(tsum.get("dwconv", empty))
        cpu = None
        _progress(f"timed {args.steps} steps: {1e3 * elapsed / args.steps:.3f} ms/step ({utt:.1f} utt/s)")
        if not args.no_cpu_baseline and world == 1:
            # every core this process may use: its affinity set capped by the cgroup CPU quota (the GPU
            # box: 256 CPUs visible, cpu.max = 16 CPUs; 256 threads under that quota stall for minutes).
            # os.cpu_count() (the whole machine) is reported beside it
            threads = args.cpu_threads or _usable_cpus()
            cpu = cpu_baseline(threads, args.samples)
            cpu["cgroup_cpu_max"] = _cgroup_cpu_max()
        f32 = v1024 = encfm = xl = xl8 = None
        if not args.no_f32_sensitivity and cfg.math == "bf16" and world == 1:
            _progress("f32 sensitivity")
            f32 = sensitivity(dev, args.samples, math="f32")
            f32["dtype"] = "f32"
            _progress("V=1024 sensitivity")
            v1024 = sensitivity(dev, args.samples, vocab=1024)
            _progress("encoder-level FM + router sensitivity")
            encfm = sensitivity(dev, args.samples, kd_model="encfm")
            encfm["note"] = ("the asr_train.py model family on the same workload: router + flow matching on every "
                             "hooked layer pair instead of the ver5 latent heads; not the headline value")
            _progress("FastConformer-XL shape sensitivity")
            xl = sensitivity(dev, args.samples, **XL_SHAPES)
            xl["note"] = ("BASELINE.json configs[4]'s layer shapes (FastConformer-XL: d_model 1024, 8 heads, head dim "
                          "128, 24 layers, dw_striding x8, kernel 9, no xscaling) for student and teacher on the same "
                          "16 s x B=32 workload, bf16 (the wide Linear products on the large-tile route, "
                          "csrc/biggemm.hip); not the headline value")
            _progress("FastConformer-XL fp8 sensitivity")
            xl8 = sensitivity(dev, args.samples, linear_fp8=True, **XL_SHAPES)
            xl8["note"] = ("configs[4] at its stated precision: the same XL step with the wide Linear products' forward "
                           "and data gradients on MX fp8 operands (e4m3 with an e8m0 scale per 32 contraction "
                           "elements, applied by the block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4); attention "
                           "core and weight gradients bf16; not the headline value")
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
                       "global_batch": world * args.batch, "seq_len": args.samples, "issue": issue,
                       "deterministic": cfg.deterministic,
                       "kernarg_device_memory": bool(getattr(__import__("kdfm"), "KERNARG_IN_DEVICE_MEMORY", False)),
                       "frames_subsampled": (args.samples // 160) // 4 + 1, "parallelism": f"dp{world}"},
            "roofline": roof,
            "roofline_by_family": by_route,
            "roofline_critical_path": crit,
            "mfma_attn_ffn_by_family": mfma_fams,
            "attn_ffn_mfma_frac": {"value": round(ATTN_FFN_GFLOP_PER_UTT * 1e9 * utt_gpu / (bf16_peak * 1e12), 5),
                                   "formula": "23.0 GFLOP/utt (SURVEY §8(d)) x utt/s per GPU / dense bf16 peak"},
            "whole_step": {"tflops": round(STEP_GFLOP_PER_UTT * 1e9 * utt_gpu / 1e12, 2),
                           "frac_bf16_peak": round(STEP_GFLOP_PER_UTT * 1e9 * utt_gpu / (bf16_peak * 1e12), 5),
                           "formula": "62.6 GFLOP/utt (SURVEY §8(d)) x utt/s per GPU"},
            "mel_frontend_hbm": {"achieved": round(fe[2], 1), "unit": "GB/s", "peak": MI355X_HBM_GBPS,
                                 "frac": round(fe[2] / MI355X_HBM_GBPS, 4), "launches": fe[0], "avg_ms": round(fe[1], 5),
                                 "bytes": "4 B x (N samples + T x 80 mel) per utterance (1.54 MB at 16 s)"},
            "dwconv_hbm": {"achieved": round(dw[2], 1), "unit": "GB/s", "peak": MI355X_HBM_GBPS,
                           "frac": round(dw[2] / MI355X_HBM_GBPS, 4), "launches": dw[0], "avg_ms": round(dw[1], 5),
                           "bytes": "read g + write y, 4 B x rows x d per launch"},
            "cpu_baseline": cpu,
            "f32_sensitivity": f32,
            "vocab_1024_sensitivity": v1024,
            "encoder_fm_router_sensitivity": encfm,
            "xl_shape_sensitivity": xl,
            "xl_fp8_sensitivity": xl8,
            "losses_last_step": [round(x, 5) for x in losses],
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
