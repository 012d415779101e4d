"""The ver5 FM-distillation training step as an explicit forward/backward schedule of libkdfm
kernels (no autograd graph, no per-op Python autograd overhead, capturable as one HIP graph).

Reference call stack: DistilFlowMatchingCTCModelBPE.training_step
(asr_train_diffm.py:731-828) -> forward (:606-643) [student preprocessor + SpecAugment + encoder,
teacher preprocessor + encoder under no_grad, decoder] -> CTC (:740-746) -> logit KD (:751-756)
-> per-layer ver5 heads (:773-792) -> total (:803-811) -> Lightning backward -> AdamW + Noam.
"""
from __future__ import annotations

import contextlib

import math

import torch

from . import _lib
from . import kernels as K
from .config import (Ver5Config, all_head_specs, bn_buffer_specs, diffkd_specs, meta_bn_specs, student_specs,
                     teacher_specs)
from .conformer import EncoderRun, EncoderShapes, compute_lengths, encoder_backward, encoder_forward, fold_arena, \
    encoder_forward_steps, layer_images, make_workspace
from .frontend import FrontendConsts, frontend_forward, mel_frames, specaugment_
from .encfm import EncFMWorkspace, encfm_backward, encfm_forward
from .heads import SALT_HEADS, HeadsWorkspace, heads_backward, heads_forward, tae_forward
from .overlap import WGRAD

# Stream priorities (KDFM_STREAM_PRIO=1): the critical-path streams (the compute stream that carries
# the student chain and the backward, the teacher stream that bounds the forward, the CTC/KL stream the
# heads join on) are created high-priority, the weight-gradient stream keeps the default low one, so
# the dispatcher hands freed CUs to the critical path first when both have workgroups waiting.
# Off by default: measured 19.2 -> 25.8 ms per step on ROCm 7 (profiles/r02/prio_bench_*.log) --
# the high-priority streams lose their overlap with each other.
# KDFM_STREAM_PRIO=compute[,side][,aux]: only the named roles high-priority (the round-6 A/B: the compute stream alone,
# so the student chain takes freed CUs ahead of the teacher and the weight gradients)
_PRIO_ENV = __import__("os").environ.get("KDFM_STREAM_PRIO", "0")
_STEP_BRACKET = __import__("os").environ.get("KDFM_STEP_BRACKET", "1") == "1"
# the frozen teacher's bf16 weight twins and fused-kernel images are rebuilt on the teacher stream after it forks
# (KDFM_TEACHER_PREP_SIDE=0: on the compute stream before the fork, delaying both chains)
_TEACHER_PREP_SIDE = __import__("os").environ.get("KDFM_TEACHER_PREP_SIDE", "1") == "1"
_PRIO = {"compute", "side", "aux"} if _PRIO_ENV == "1" else {r for r in _PRIO_ENV.split(",") if r not in ("", "0")}


# One stream per (device, role), shared by every engine of the process: torch hands out pool streams round-robin
# and HIP maps streams onto the GPU_MAX_HW_QUEUES = 4 hardware queues in creation order, so a second engine's
# fresh streams could share a queue with the weight-gradient stream (module-level, made once) and serialise
# behind it -- measured: the same XL step 81.5 ms on a process's first engine, 91 ms on its second
# (tools/xl_cmp.py, profiles/r06/xl_cmp_*.log).  Engines of one process run one after the other.
_STREAMS = {}


def _crit_stream(dev, role):
    key = (str(torch.device(dev)), role)
    s = _STREAMS.get(key)
    if s is None:
        s = _STREAMS[key] = torch.cuda.Stream(dev, priority=-1) if role in _PRIO else torch.cuda.Stream(dev)
    return s
from .store import FlatStore, init_uniform

SALT_STUDENT, SALT_TEACHER, SALT_FRONT = 1, 2, 3


# KDFM_DEC_SIDE=1: the decoder weight gradient on the weight-gradient stream (A/B switch; default 0, the compute
# stream: 2122 / 2124 vs 2115 / 2104 utt/s, profiles/r04/r4w)
_DEC_SIDE = __import__("os").environ.get("KDFM_DEC_SIDE", "0") == "1"


class _OnStream:
    """Run a block on the engine's compute stream: it first waits for the caller's current stream,
    and the caller's stream waits for it afterwards (no-op when already on it, e.g. while capturing)."""

    def __init__(self, eng):
        self.eng = eng
        self.ctx = None

    def __enter__(self):
        cs = self.eng.compute_stream
        if cs is None:
            return self
        if K.stream_ptr() == cs.cuda_stream:
            return self
        self.eng._link_in.after_current(cs)
        self.ctx = K.on_stream(cs)
        self.ctx.__enter__()
        return self

    def __exit__(self, *a):
        if self.ctx is not None:
            self.ctx.__exit__(*a)
            self.eng._link_out.current_after(self.eng.compute_stream)
            self.ctx = None


class Ver5Engine:
    """Owns the student (trainable, flat buffer + AdamW state), the frozen teacher and all step
    buffers on one device."""

    def __init__(self, cfg: Ver5Config, device="cuda", *, teacher_seed=0, student_seed=1, heads_seed=2,
                 init=True):
        self.cfg = cfg
        self.device = torch.device(device)
        dev = self.device
        self.student = FlatStore(student_specs(cfg), dev, with_grad=True, with_adam=True)
        self.teacher = FlatStore(teacher_specs(cfg), dev, with_grad=False)
        K.register_frozen(self.teacher.data, self.teacher)   # the frozen teacher's large-tile weight copies persist
        # used but never-trained student-side parameters: DiffKD's encoder (its output is detached
        # before every use, asr_train_diffm.py:382-383, so AdamW never touches it)
        self.fixed = FlatStore(diffkd_specs(cfg, False) if cfg.use_diffkd else [], dev, with_grad=False)
        self.bn = FlatStore(bn_buffer_specs(cfg, cfg.d_student, "encoder.")
                            + bn_buffer_specs(cfg, cfg.d_teacher, "teacher.encoder.") + meta_bn_specs(cfg), dev,
                            with_grad=False)
        self.fe = FrontendConsts(cfg, dev)
        self.seed = torch.zeros(1, dtype=torch.int64, device=dev)     # uint64 bits, advanced on device
        self.step = torch.zeros(1, dtype=torch.int64, device=dev)
        # optimizer steps taken before the AdamW moments were (re)started: AdamW's bias correction
        # counts from here while the Noam schedule counts from 0 (a resume whose moments could not
        # be restored, checkpoint.restore_lightning_ckpt)
        self.adam_base = torch.zeros(1, dtype=torch.int64, device=dev)
        self.lr = torch.zeros(1, device=dev)
        # total, ctc, kl, recon, layer KD (kd/fm pre+post, ver5: fm_post; + the DiffKD term with use_diffkd)
        self.losses = torch.zeros(5, device=dev)
        # [sum g^2 of the (all-reduced, mean) gradient, #non-finite entries] when cfg.grad_check
        self.grad_stats = torch.zeros(2, device=dev) if cfg.grad_check else None
        self.hws = HeadsWorkspace(cfg, dev)
        # the ver5 heads run in two layer halves: layers [0, L/2) as soon as both encoders have issued layer
        # L/2 - 1 (beside the encoders' second half), backward beside the encoder backward's first half;
        # the halves have their own workspaces (per-step weight layouts, bias-gradient accumulators)
        self.heads_split = __import__("os").environ.get("KDFM_HEADS_SPLIT", "1") == "1"
        self.hws_b = HeadsWorkspace(cfg, dev)
        if K.twins_enabled():   # opt-in direct-B skinny path (KDFM_SKINNY_DIRECT_MIN_M)
            self.student.enable_bf16_twins()
            self.teacher.enable_bf16_twins()
        # KDFM_BF16_MIRROR=1 (wide models, d_model >= 512): the student's weights also live as a bf16 mirror the
        # optimizer writes in its own pass (kdfm_adamw_noam_bf16), read by the large-tile products without a cast
        # per weight per step.  Off by default: measured neutral on the XL bf16 step (82.0-82.2 vs 82.0-82.9 ms,
        # interleaved, profiles/r06/r6ac_bf16_mirror_ab.log) -- the casts it removes were not on the critical path
        if (dev.type == "cuda" and max(cfg.d_student, cfg.d_teacher) >= 512
                and __import__("os").environ.get("KDFM_BF16_MIRROR", "0") == "1"):
            self.student.enable_bf16_mirror()
        self._pos = {}
        self._imgs = None   # kernels.WeightImages of the student and the teacher encoders (bf16 math)
        self._ws = {}
        # the step runs on a created (non-null) stream: ROCm makes the legacy null stream wait for a
        # HIP graph replayed on any other stream (tools/graph_probe.py), which serialised the whole-step
        # graph's branches behind the main stream
        self.compute_stream = _crit_stream(dev, "compute") if dev.type == "cuda" else None
        self._link_in, self._link_out = K.StreamLink(), K.StreamLink()   # caller <-> compute stream
        # weight gradients on the side stream (the benchmark's schedule) or in line: None follows the
        # config (in line exactly when deterministic); the overlapped-vs-serialised determinism test
        # forces both with ordered reductions
        self.overlap_wgrad = None
        # encoder-level FM (kd_model "encfm"): optional injected router Gumbel noise (L*B, K) for parity
        # runs, the per-(B, T) workspaces, and the last step's [flow, router, total, mean steps] stats
        self.encfm_gumbel = None
        self._encfm = {}
        self.encfm_stats = None
        if init:
            st = init_uniform(student_specs(cfg), student_seed)
            hd = init_uniform([s for s in student_specs(cfg) if not s[0].startswith(("encoder.", "decoder."))],
                              heads_seed)
            st.update(hd)
            self.student.load(st)
            self.teacher.load(init_uniform(teacher_specs(cfg), teacher_seed))
            if self.fixed.specs:
                self.fixed.load(init_uniform(self.fixed.specs, heads_seed + 2000))
            self.reset_bn()
        # heads the reference module builds but this version never trains (asr_train_diffm.py:559-564):
        # kept host-side (seeded init, or whatever a checkpoint held) so saved state dicts carry the
        # reference's full key set
        trained = {n for n, _ in student_specs(cfg)}
        frozen = [s for s in all_head_specs(cfg) if s[0] not in trained]
        self.frozen_heads = init_uniform(frozen, heads_seed + 1000) if frozen else {}

    # ---------------------------------------------------------------------------------------------
    def reset_bn(self):
        for name, _ in self.bn.specs:
            K.fill(self.bn.P[name], 1.0 if name.endswith("running_var") else 0.0)

    def set_seed(self, seed: int):
        self.seed.fill_(int(seed) & 0x7FFFFFFFFFFFFFFF)

    @property
    def seed_u64(self):
        return self.seed  # passed as const uint64_t* (bit pattern)

    def _pos_emb(self, T, d):
        key = (T, d)
        if key not in self._pos:
            pe = torch.empty(2 * T - 1, d, device=self.device)
            K.relpos_table(T, d, pe)
            self._pos[key] = pe
        return self._pos[key]

    def _encfm_ws(self, B, T):
        """The encoder-level FM workspace for this batch shape.  Only the CURRENT shape is cached: a meta-encoder
        workspace holds every step's saved activations (GBs at the bench shape), so one per padded length would
        grow without bound over a real run; a new (B, T) drops the previous one (the allocator
        reuses its blocks: the previous step's streams were joined before this forward)."""
        ws = self._encfm.get((B, T))
        if ws is None:
            self._encfm.clear()
            if self.cfg.encfm_meta != "mlp":
                from .fmmeta import MetaFMWorkspace
                ws = self._encfm[(B, T)] = MetaFMWorkspace(self.cfg, B, T, self.device)
            else:
                ws = self._encfm[(B, T)] = EncFMWorkspace(self.cfg, B, T, self.device)
        return ws

    def _side_stream(self):
        if getattr(self, "_side", None) is None:
            self._side = _crit_stream(self.device, "side")
        return self._side

    def _teacher_forward(self, mel_t, mel_len, len1, len2, tfeats, tlogits, St, T):
        cfg = self.cfg
        Cn = cfg.classes
        encoder_forward(cfg, St, self.teacher.P, "teacher.encoder.", mel_t, mel_len, len1, len2, tfeats,
                        self._pos_emb(T, St.d), train=False, seed=self.seed, salt=SALT_TEACHER, save=False,
                        bn_running=self.bn.P, use_batch_stats=False, ws=self._enc_ws(St, "teacher.encoder."))
        K.linear(tfeats[-1], self.teacher.P["teacher.decoder.decoder_layers.0.weight"].view(Cn, St.d),
                 self.teacher.P["teacher.decoder.decoder_layers.0.bias"], tlogits)

    def _enc_ws(self, S, prefix):
        # one workspace per encoder: the teacher and the student run concurrently on two streams and
        # each writes its own re-laid-out weights here (equal widths shared one)
        key = (prefix, S.d, S.F2)
        if key not in self._ws:
            self._ws[key] = make_workspace(S, self.device)
        return self._ws[key]

    # ---------------------------------------------------------------------------------------------
    def _on_stream(self):
        return _OnStream(self)

    def _mode(self):
        """The config's MFMA arithmetic and reduction mode for the duration of a call (restored
        afterwards: the kernels' modes are process-global)."""
        return K.mode(self.cfg.math, self.cfg.deterministic, fp8=self.cfg.linear_fp8,
                      wide=max(self.cfg.d_student, self.cfg.d_teacher) >= 512)

    def forward(self, wav, wav_len, targets, tgt_len, *, train=True, eps=None, save=True):
        """One forward pass; returns the context backward() consumes.  eps: optional injected
        NoiseAdapter noise (n_layers*B*T', latent) for parity runs."""
        with self._on_stream(), self._mode(), K.weight_epoch(), K.region("forward"):
            return self._forward(wav, wav_len, targets, tgt_len, train=train, eps=eps, save=save)

    def _forward(self, wav, wav_len, targets, tgt_len, *, train, eps, save):
        cfg = self.cfg
        dev = self.device
        B, N = wav.shape
        Tm = mel_frames(cfg, N)
        Ss = EncoderShapes(cfg, B, Tm, cfg.d_student, cfg.heads_student)
        St = EncoderShapes(cfg, B, Tm, cfg.d_teacher, cfg.heads_teacher)
        T = Ss.T
        mel_len = torch.empty(B, dtype=torch.int64, device=dev)
        len1 = torch.empty_like(mel_len)
        len2 = torch.empty_like(mel_len)
        len1, len2 = compute_lengths(cfg, wav_len, mel_len, len1, len2, cfg.hop)
        seed = self.seed
        encfm = cfg.kd_model == "encfm"
        heads = cfg.kd_model == "diffm"     # "logitkd": CTC + logit KD only, no latent heads
        # kl | recon, kd_pre, fm_pre, kd_post, fm_post (heads.RECON..FM_POST) | diffkd | sum of the layer-KD
        # terms and diffkd (zeroed before the teacher stream forks: its auto-encoder adds the recon term)
        acc = torch.zeros(8, device=dev)
        teacher_prep = None
        if K.get_math() == "bf16":   # bf16 twins of the weights the skinny products stream
            self.student.refresh_bf16()
            # fragment images of the fused Conformer kernels (ffn / lnproj / rowgemm): one launch each
            if self._imgs is None:
                self._imgs = (layer_images(cfg, self.student.P, "encoder.", cfg.d_student, train=True, dev=dev),
                              layer_images(cfg, self.teacher.P, "teacher.encoder.", cfg.d_teacher, train=False,
                                           dev=dev))
            for im in self._imgs:
                im.register()
            self._imgs[0].refresh()

            def teacher_prep():
                self.teacher.refresh_bf16()
                self._imgs[1].refresh()
            if not _TEACHER_PREP_SIDE:   # KDFM_TEACHER_PREP_SIDE=0: on this stream, before the teacher forks
                teacher_prep()
                teacher_prep = None
        # ---- frontends (teacher preprocessor is in eval mode: no dither) ----
        dither = cfg.dither if train else 0.0
        own_mel = train and (dither > 0.0 or not cfg.share_frontend)   # the student computes its own mel
        Cn = cfg.classes
        rows = Ss.rows
        main = torch.cuda.current_stream(dev)
        side = self._side_stream()
        tfeats = torch.empty(cfg.n_layers, St.rows, St.d, device=dev)
        tlogits = torch.empty(rows, Cn, device=dev)
        n_st = cfg.n_layers * Ss.rows
        # the teacher auto-encoder's outputs are written on the teacher stream: allocated BEFORE the teacher
        # stream's join below, so a block the caching allocator hands over here cannot be one this stream
        # frees later in the step (the student frontend's temporaries) and the teacher stream then overwrites
        # while this stream still reads it (tools/race_check.py: preemph_pad.xp vs tae_forward's zt)
        tae = None
        if heads:
            tae = (torch.empty(n_st, cfg.latent, device=dev), torch.empty(n_st, St.d, device=dev))
        if own_mel:
            # the teacher's own (undithered) frontend goes to the teacher stream with its encoder (and the
            # teacher's weight twins / images: read by teacher-stream kernels only)
            K.wait_stream(side, main)
            with torch.cuda.stream(side), K.region("teacher_frontend"):
                if teacher_prep is not None:
                    teacher_prep()
                mel_t = frontend_forward(cfg, self.fe, wav, wav_len, mel_len, dither=0.0)
        else:
            mel_t = frontend_forward(cfg, self.fe, wav, wav_len, mel_len, dither=0.0)
            K.wait_stream(side, main)
            if teacher_prep is not None:
                with torch.cuda.stream(side):
                    teacher_prep()
        tgen = encoder_forward_steps(cfg, St, self.teacher.P, "teacher.encoder.", mel_t, mel_len, len1, len2,
                                     tfeats, self._pos_emb(T, St.d), train=False, seed=seed, salt=SALT_TEACHER,
                                     save=False, bn_running=self.bn.P, use_batch_stats=False, ws=self._enc_ws(St, "teacher.encoder."))
        if own_mel:
            mel_s = frontend_forward(cfg, self.fe, wav, wav_len, mel_len, dither=dither, seed=seed,
                                     rng_stream=SALT_FRONT)
        elif train and cfg.specaug:
            mel_s = torch.empty_like(mel_t)
            K.axpby(mel_t.view(B * Tm, -1), None, mel_s.view(B * Tm, -1), 1.0, 0.0)
        else:
            mel_s = mel_t
        if train and cfg.specaug:
            specaugment_(cfg, mel_s, mel_len, seed, SALT_FRONT + 1)
        # ---- the frozen teacher encoder (eval mode, nothing saved) on the teacher stream and the
        # student encoder (saved for backward) on this one, issued layer by layer in alternation so
        # the two encoders overlap on the CUs while the host is still issuing ----
        sfeats = torch.empty(cfg.n_layers, Ss.rows, Ss.d, device=dev)
        pos_s = self._pos_emb(T, Ss.d)
        srun = EncoderRun() if save else None
        sgen = encoder_forward_steps(cfg, Ss, self.student.P, "encoder.", mel_s, mel_len, len1, len2, sfeats, pos_s,
                                     train=train, seed=seed, salt=SALT_STUDENT, save=save, bn_running=self.bn.P,
                                     use_batch_stats=train, ws=self._enc_ws(Ss, "encoder."), run=srun)
        h = self._heads_half(train, save) if heads else 0
        nb = h * Ss.rows
        hctx_b = None
        # the first heads half accumulates its loss terms into slots of its own (it runs on another stream
        # beside the second half: no two streams add into one scalar), folded into acc after the join
        acc_h = torch.zeros(8, device=dev) if h else None
        with K.region("encoders"):
            for k in range(cfg.n_layers + 1):
                with K.on_stream(side):
                    next(tgen)
                next(sgen)
                if h and k == h:
                    # both encoders have issued layers [0, h): the auto-encoder of those teacher layers on the
                    # teacher stream, then the heads of those layers on the heads stream, beside layers [h, L)
                    with torch.cuda.stream(side):
                        tae_forward(cfg, self.student.P, tfeats[:h].view(nb, St.d), tae[0][:nb], tae[1][:nb], acc[1:2],
                                    layers=h)
                    hctx_b = self._heads_first_half(cfg, Ss, St, T, h, sfeats, tfeats, tae, acc_h, eps, seed, save,
                                                    main, side)
        with torch.cuda.stream(side):
            K.linear(tfeats[-1], self.teacher.P["teacher.decoder.decoder_layers.0.weight"].view(Cn, St.d),
                     self.teacher.P["teacher.decoder.decoder_layers.0.bias"], tlogits)
        for t in (tfeats, tlogits, mel_t, mel_len, len1, len2):
            t.record_stream(side)
        # ---- the ver5 heads' TeacherAutoEncoder reads only the teacher: on the teacher stream, right after
        # the teacher encoder (the second layer half; the first went out after teacher layer h - 1), off the
        # student's chain (the main stream joins the teacher stream below) ----
        if tae is not None:
            with torch.cuda.stream(side):
                tae_forward(cfg, self.student.P, tfeats[h:].view(n_st - nb, St.d), tae[0][nb:], tae[1][nb:], acc[1:2],
                            layers=cfg.n_layers - h)
            for t in (*tae, acc, tfeats):
                t.record_stream(side)
        # ---- decoders, CTC, logit KD ----
        dec_in = sfeats[-1]
        if encfm:
            # asr_train.py: the router + flow matching over every hooked layer pair (it needs the teacher's
            # features), and the decoder reads the last layer's FM output (:595-666)
            K.wait_stream(main, side)
            ews = self._encfm_ws(B, T)
            with K.region("encfm_forward"):
                dec_in = encfm_forward(cfg, self.student.P, sfeats, tfeats, ews, seed=seed, train=train,
                                       gumbel=self.encfm_gumbel, bn_running=self.bn.P)
            self.encfm_stats = ews.stats
        logits = torch.empty(rows, Cn, device=dev)
        K.linear(dec_in, self.student.P["decoder.decoder_layers.0.weight"].view(Cn, Ss.d),
                 self.student.P["decoder.decoder_layers.0.bias"], logits)
        lp = torch.empty(rows, Cn, device=dev)
        K.log_softmax(logits, lp)
        if not encfm:
            K.wait_stream(main, side)
        # ---- CTC + logit KD on a third stream: they only need the two logit tensors, and their
        # result is first needed after the KD heads' forward, so the serial CTC recursion overlaps it ----
        aux = self._aux_stream()
        K.wait_stream(aux, main)
        Umax = targets.shape[1]
        nll = torch.empty(B, device=dev)
        glogits = torch.empty(rows, Cn, device=dev)
        with torch.cuda.stream(aux), K.region("ctc_kl"):
            alpha_ws = torch.empty(B * T * (2 * Umax + 1), device=dev)
            beta_ws = torch.empty_like(alpha_ws)
            K.ctc_loss(lp, targets, len2, tgt_len, alpha_ws, beta_ws, nll, glogits, B, T, Cn, cfg.vocab, 1.0 / B)
            del alpha_ws, beta_ws
            Tk = cfg.kd_temperature
            K.kl_div_logits(lp, tlogits, glogits, acc[0:1], Tk, cfg.kd_alpha * Tk / B, Tk * Tk / B)
        for t in (lp, tlogits, targets, len2, tgt_len, nll, glogits, acc):
            t.record_stream(aux)
        # ---- ver5 heads over all layers at once ----
        n = cfg.n_layers * rows
        if encfm:
            hctx = None
            K.axpby(ews.stats[2:3].view(1, 1), None, acc[7:8].view(1, 1), 1.0, 0.0)   # forward's total_loss
        elif not heads:
            hctx = None   # logit KD only: acc[1:8] stay 0, the total is CTC + kd_alpha * KL
        else:
            with K.region("heads_forward"):
                na = n - nb
                hctx_a = heads_forward(cfg, self.student.P, sfeats[h:].view(na, Ss.d), tfeats[h:].view(na, St.d), T,
                                       self.hws, acc[1:6], seed=seed, eps=None if eps is None else eps[nb:],
                                       save=save, Pfix=self.fixed.P, acc_diffkd=acc[6:7], tae=(tae[0][nb:], tae[1][nb:]),
                                       layers=cfg.n_layers - h)
                if h:
                    K.wait_stream(main, self._heads_stream(main))   # the first half's loss terms
                    K.axpby(acc_h[2:7].view(1, 5), acc[2:7].view(1, 5), acc[2:7].view(1, 5), 1.0, 1.0)
                hctx = (hctx_b, hctx_a, h) if save else None
                K.colsum(acc[2:7].view(5, 1), acc[7:8], accumulate=False)
        # device (recon, kd_pre, fm_pre, kd_post, fm_post, diffkd): the v/* log keys
        self.kd_terms = acc[1:7]
        ctx = dict(B=B, T=T, Ss=Ss, St=St, mel_len=mel_len, len1=len1, len2=len2, srun=srun, sfeats=sfeats,
                   glogits=glogits, hctx=hctx, lp=lp, nll=nll, pos_s=pos_s, acc=acc, dec_in=dec_in,
                   ews=ews if encfm else None)
        self._join_losses(ctx)   # CTC/KL overlapped the heads forward; losses valid after forward()
        return ctx

    # ---------------------------------------------------------------------------------------------
    def infer(self, wav, wav_len):
        """Eval-mode student forward (asr_train_diffm.py:606-643 with self.training False; the
        validation pass of ctc_models.py:625-665): frontend without dither or SpecAugment, encoder
        with BatchNorm running statistics and no dropout, decoder + log_softmax.  The reference's eval
        forward also runs the teacher encoder (:629-631) and discards it (only training_step reads
        the hooks), so it is skipped.  Returns log_probs (B, T', V+1) and enc_len (B,)."""
        with self._on_stream(), self._mode(), K.weight_epoch():
            return self._infer(wav, wav_len)

    def _infer(self, wav, wav_len):
        cfg = self.cfg
        dev = self.device
        B, N = wav.shape
        Tm = mel_frames(cfg, N)
        Ss = EncoderShapes(cfg, B, Tm, cfg.d_student, cfg.heads_student)
        mel_len = torch.empty(B, dtype=torch.int64, device=dev)
        len1 = torch.empty_like(mel_len)
        len2 = torch.empty_like(mel_len)
        len1, len2 = compute_lengths(cfg, wav_len.to(device=dev, dtype=torch.int64), mel_len, len1, len2, cfg.hop)
        mel = frontend_forward(cfg, self.fe, wav.to(dev), wav_len.to(dev), mel_len, dither=0.0)
        feats = torch.empty(cfg.n_layers, Ss.rows, Ss.d, device=dev)
        encoder_forward(cfg, Ss, self.student.P, "encoder.", mel, mel_len, len1, len2, feats,
                        self._pos_emb(Ss.T, Ss.d), train=False, seed=self.seed, salt=SALT_STUDENT, save=False,
                        bn_running=self.bn.P, use_batch_stats=False, ws=self._enc_ws(Ss, "encoder."))
        Cn = cfg.classes
        logits = torch.empty(Ss.rows, Cn, device=dev)
        K.linear(feats[-1], self.student.P["decoder.decoder_layers.0.weight"].view(Cn, Ss.d),
                 self.student.P["decoder.decoder_layers.0.bias"], logits)
        lp = torch.empty(Ss.rows, Cn, device=dev)
        K.log_softmax(logits, lp)
        return lp.view(B, Ss.T, Cn), len2

    def ctc_mean(self, log_probs, enc_len, targets, tgt_len):
        """CTCLoss(reduction='mean_batch', zero_infinity=True) of eval log-probs (ctc_models.py:637)."""
        B, T, Cn = log_probs.shape
        dev = log_probs.device
        targets = targets.to(device=dev, dtype=torch.int64).contiguous()
        tgt_len = tgt_len.to(device=dev, dtype=torch.int64)
        Umax = max(1, targets.shape[1])
        a = torch.empty(B * T * (2 * Umax + 1), device=dev)
        bta = torch.empty_like(a)
        nll = torch.empty(B, device=dev)
        g = torch.empty(B * T, Cn, device=dev)
        K.ctc_loss(log_probs.reshape(B * T, Cn), targets, enc_len, tgt_len, a, bta, nll, g, B, T, Cn, self.cfg.vocab,
                   1.0 / B)
        return nll.mean()

    def _aux_stream(self):
        """The CTC/KL stream.  By default it IS the teacher stream: the main stream has just joined the
        teacher there (the heads need its features), so the teacher stream is idle for exactly the span
        CTC/KL run beside the heads forward, and the step keeps to three compute streams -- with RCCL's
        own stream under DDP, four, within the GPU_MAX_HW_QUEUES=4 hardware queues, so no two streams
        share a queue (a shared queue serialises its streams).  KDFM_AUX_STREAM=1: a stream of its own."""
        if getattr(self, "_aux", None) is None:
            own = __import__("os").environ.get("KDFM_AUX_STREAM", "0") == "1"
            self._aux = _crit_stream(self.device, "aux") if own else self._side_stream()
        return self._aux

    def _serial(self):
        """Weight gradients (and the heads' second stream) in line: deterministic mode unless overlap_wgrad
        says otherwise."""
        return self.cfg.deterministic if self.overlap_wgrad is None else not self.overlap_wgrad

    def _heads_half(self, train, save):
        """h > 0: the heads run as layers [0, h) and [h, L) (KDFM_HEADS_SPLIT=0: one call over all)."""
        return self.cfg.n_layers // 2 if self.heads_split and self.cfg.n_layers >= 2 else 0

    def _heads_stream(self, main):
        """Where the first heads half runs in the forward: the weight-gradient stream (idle until the
        backward), or in line when the schedule is serialised."""
        return main if self._serial() else WGRAD.stream()

    def _heads_first_half(self, cfg, Ss, St, T, h, sfeats, tfeats, tae, acc, eps, seed, save, main, side):
        """acc: the half's own loss slots (same layout as the step's accumulator; recon stays with the teacher
        auto-encoder on the teacher stream)."""
        nb = h * Ss.rows
        hs = self._heads_stream(main)
        # the teacher features / auto-encoder outputs of layers [0, h) come from the teacher stream: wait for it
        # in line too (the serialised schedule once read them unjoined -- profiles/r05/r5zz*)
        K.wait_stream(hs, side)
        if hs is not main:
            K.wait_stream(hs, main)
            for t in (sfeats, tfeats, *tae, acc) + (() if eps is None else (eps,)):
                t.record_stream(hs)
        with K.on_stream(hs), K.region("heads_forward_first_half"):
            return heads_forward(cfg, self.student.P, sfeats[:h].view(nb, Ss.d), tfeats[:h].view(nb, St.d), T,
                                 self.hws_b, acc[1:6], seed=seed, eps=None if eps is None else eps[:nb], save=save,
                                 Pfix=self.fixed.P, acc_diffkd=acc[6:7], tae=(tae[0][:nb], tae[1][:nb]), layers=h,
                                 salt=SALT_HEADS + 100)

    def _join_losses(self, ctx):
        """Join the CTC/KL stream and assemble the loss vector (total, ctc, kl, recon, fm)."""
        K.wait_stream(torch.cuda.current_stream(self.device), self._aux_stream())
        acc = ctx["acc"]
        K.loss_combine(ctx["nll"], acc[0:1], acc[1:2], acc[7:8], self.cfg.kd_alpha, self.losses)

    def backward(self, ctx, grad_ready=None):
        """grad_ready(offset): optional callback, called whenever every student gradient at flat
        index >= offset is final (BucketedGradAllReduce.ready overlap)."""
        # deterministic mode keeps the weight-gradient products on the issuing stream unless
        # overlap_wgrad says otherwise
        serial = self.cfg.deterministic if self.overlap_wgrad is None else not self.overlap_wgrad
        with self._on_stream(), self._mode(), WGRAD.serialized(serial), K.weight_epoch(), K.region("backward"):
            try:
                self._backward(ctx, grad_ready)
            except BaseException:
                # a backward that raises between setting the deferred-fold arena and ending deferral leaves
                # queued folds pointing into the arena: drop them so the next backward starts clean
                K.wgrad_fold_discard_all()
                raise

    def _backward(self, ctx, grad_ready):
        cfg = self.cfg
        P, G = self.student.P, self.student.G
        off = self.student.offsets
        Ss = ctx["Ss"]
        n = cfg.n_layers * Ss.rows
        self.student.zero_grad()
        dfeats = torch.empty(cfg.n_layers, Ss.rows, Ss.d, device=self.device)
        # the heads' / decoder's weight-gradient folds join the encoder's deferred ones (conformer.fold_arena): one
        # batched fold launch before each gradient-ready point
        arena = fold_arena(self._enc_ws(Ss, "encoder."), self.device)
        if arena is not None:
            WGRAD.run(lambda: K.wgrad_set_fold_arena(arena), arena)
            _ready = grad_ready

            def grad_ready_flushed(offset):
                WGRAD.run(K.wgrad_fold_flush)
                if _ready is not None:
                    _ready(offset)
            grad_ready = grad_ready_flushed if grad_ready is not None else None
        dec0 = off["decoder.decoder_layers.0.weight"]
        g = ctx.pop("glogits")
        Cn = cfg.classes
        Wd = P["decoder.decoder_layers.0.weight"].view(Cn, Ss.d)
        if cfg.kd_model == "encfm":
            # decoder first: its input is the last layer's FM output, whose gradient the FM backward needs
            ews = ctx.pop("ews")
            self._decoder_dw(g, ctx["dec_in"])
            K.linear_dx(g, Wd, ews.gxS)
            del g
            with K.region("encfm_backward"):
                encfm_backward(cfg, P, G, ews, dfeats.view(n, Ss.d), ews.gxS, WGRAD.run, seed=self.seed)
            if grad_ready is not None:
                grad_ready(min(o for k, o in off.items() if not k.startswith(("encoder.", "decoder."))))
        elif ctx.get("hctx") is None:
            # logit KD only (kd_model "logitkd"): the decoder's gradient is the encoder's only input gradient
            ctx.pop("hctx", None)
            self._decoder_dw(g, ctx["sfeats"][-1])
            K.fill(dfeats, 0.0)
            K.linear_dx(g, Wd, dfeats[-1])
            del g
        else:
            hctx_b, hctx_a, h = ctx.pop("hctx")
            nb = h * Ss.rows
            dfv = dfeats.view(n, Ss.d)
            if h:
                # the first layer half's heads backward: in line, or on the teacher stream (idle since CTC/KL)
                # beside this half and the encoder backward of layers [h, L); the encoder backward joins it
                # before it reads dfeats[h - 1].  Its weight gradients are issued first either way, so the
                # weight-gradient stream sees the same launch order as the serialised schedule.
                side = main = torch.cuda.current_stream(self.device)
                if not self._serial():
                    side = self._side_stream()
                    K.wait_stream(side, main)
                    dfeats.record_stream(side)
                with K.on_stream(side), K.region("heads_backward_first_half"):
                    heads_backward(cfg, P, G, hctx_b, self.hws_b, dfv[:nb], seed=self.seed)
                if side is not main:
                    ctx["heads_join"] = (h - 1, side)
            with K.region("heads_backward"):
                heads_backward(cfg, P, G, hctx_a, self.hws, dfv[nb:], seed=self.seed)
            if grad_ready is not None:
                grad_ready(min(o for k, o in off.items() if not k.startswith(("encoder.", "decoder."))))
            # decoder: logits = W enc + b ; grad wrt logits from CTC + KL
            self._decoder_dw(g, ctx["sfeats"][-1])
            K.linear_dx(g, Wd, dfeats[-1], R=dfeats[-1], rscale=1.0)
            del g
        layer_done = None
        if grad_ready is not None:
            grad_ready(min(dec0, off["decoder.decoder_layers.0.bias"]))
            firsts = {i: min(o for k, o in off.items() if k.startswith(f"encoder.layers.{i}."))
                      for i in range(cfg.n_layers)}
            layer_done = lambda i: grad_ready(firsts[i])  # noqa: E731
        join = ctx.pop("heads_join", None)
        with K.region("encoder_backward"):
            encoder_backward(cfg, Ss, P, G, "encoder.", ctx.pop("srun"), dfeats, ctx["pos_s"], ctx["len1"],
                             ctx["len2"], seed=self.seed, salt=SALT_STUDENT, ws=self._enc_ws(Ss, "encoder."),
                             on_layer_done=layer_done,
                             before_read=None if join is None else {join[0]: lambda: K.wait_stream(
                                 torch.cuda.current_stream(self.device), join[1])}, arena_set=arena is not None)

    def _decoder_dw(self, g, x):
        """The decoder's weight / bias gradient from the logits gradient g and its input x, on the
        weight-gradient stream (a parameter gradient only: off the compute stream's path)."""
        G = self.student.G
        Cn, d = g.shape[1], x.shape[1]
        if _DEC_SIDE:
            WGRAD.run(lambda: K.linear_dw(g, x, G["decoder.decoder_layers.0.weight"].view(Cn, d),
                                          db=G["decoder.decoder_layers.0.bias"]), g, x)
        else:
            K.linear_dw(g, x, G["decoder.decoder_layers.0.weight"].view(Cn, d), db=G["decoder.decoder_layers.0.bias"])

    def optimizer_step(self, grad_scale: float = 1.0):
        with self._on_stream(), self._mode(), K.region("optimizer"):
            self._optimizer_step(grad_scale)

    def _optimizer_step(self, grad_scale):
        cfg = self.cfg
        st = self.student
        K.step_advance(self.step, None)
        if self.grad_stats is not None:
            K.grad_stats(st.grad, grad_scale, self.grad_stats)
        K.adamw_noam(st.data, st.grad, st.exp_avg, st.exp_avg_sq, self.step, cfg.lr, cfg.sched_d_model,
                     cfg.warmup_steps, cfg.min_lr, cfg.betas[0], cfg.betas[1], cfg.adam_eps, cfg.weight_decay,
                     grad_scale, self.lr, adam_base=self.adam_base, gstats=self.grad_stats,
                     p16=getattr(st, "mirror", None))

    def advance_rng(self):
        with self._on_stream():
            K.step_advance(None, self.seed)

    def allreduce_grads(self, allreduce) -> float:
        """allreduce(flat gradient) -- the buckets the backward has not launched yet, then the waits -- issued on
        the engine's compute stream, so the last buckets' collectives are ordered after the backward's last
        gradient writes and AdamW after the collectives by stream order.  (Issuing it from the caller's stream is
        ordered too -- backward() makes that stream wait for the compute stream -- the round-5 intermittent DDP
        mismatch was the first heads half reading unjoined teacher outputs, fixed in _heads_first_half: DESIGN.md
        §10, profiles/r05/r5zz7; tools/race_check.py models both issue points.)  Returns the gradient scale
        (1 / world)."""
        with self._on_stream(), K.region("allreduce"):
            return allreduce(self.student.grad)

    def train_step(self, wav, wav_len, targets, tgt_len, allreduce=None):
        """forward + backward + (all-reduce) + AdamW.  Returns the device loss vector."""
        ready = getattr(allreduce, "ready", None)
        grad = self.student.grad
        # one caller <-> compute-stream bracket for the whole step (the inner calls' brackets are then no-ops):
        # the forward -> backward -> optimizer hand-overs stay on the compute stream instead of each making a
        # round trip through the caller's stream (KDFM_STEP_BRACKET=0: per-call brackets)
        with (self._on_stream() if _STEP_BRACKET else contextlib.nullcontext()):
            self.advance_rng()
            with K.weight_epoch():   # one epoch for forward + backward: the large-tile route converts each weight once
                ctx = self.forward(wav, wav_len, targets, tgt_len, train=True)
                self.backward(ctx, grad_ready=(lambda o: ready(grad, o)) if ready is not None else None)
                del ctx
            scale = 1.0
            if allreduce is not None:
                scale = self.allreduce_grads(allreduce)
            self.optimizer_step(scale)
        return self.losses


    def make_plan(self, wav, wav_len, targets, tgt_len, allreduce=None):
        """Record one training step (RNG advance, forward, backward, all-reduce, AdamW) as a StepPlan
        (kdfm/plan.py) whose replay() is the same step issued without the Python wrappers, on the same
        four streams.  The inputs are the plan's static buffers (copy each new batch into them).  Run
        one eager train_step first so every lazily created workspace exists.  The all-reduce's ready()
        callbacks and its final wait run as host callbacks in their recorded places."""
        from .plan import StepPlan
        plan = StepPlan()
        ready = getattr(allreduce, "ready", None)
        grad = self.student.grad
        box = {}

        def finish():
            box["scale"] = self.allreduce_grads(allreduce) if allreduce is not None else 1.0

        def step():
            with (self._on_stream() if _STEP_BRACKET else contextlib.nullcontext()):   # as train_step
                self.advance_rng()
                with K.weight_epoch():
                    ctx = self.forward(wav, wav_len, targets, tgt_len, train=True)
                    self.backward(ctx, grad_ready=(lambda o: plan.host(ready, grad, o)) if ready is not None else None)
                    del ctx
                if allreduce is not None:
                    with K.region("allreduce"):
                        plan.host(finish)
                self.optimizer_step(box.get("scale", 1.0))

        plan.record(step)
        plan.inputs = (wav, wav_len, targets, tgt_len)
        # the recorded launches address the engine's cached workspaces too (encoder workspaces with the fold
        # arena, the encoder-level FM workspace, the heads' workspaces): keep those tensors alive with the plan, so
        # a later forward at another shape (which drops the encoder-FM workspace) or a grown fold arena cannot
        # free memory a replay still writes
        plan.keep.append(self._workspace_tensors())
        return plan

    def _workspace_tensors(self):
        """Every tensor reachable from the engine's lazily created workspaces."""
        out, seen = [], set()

        def walk(o, depth=0):
            if depth > 4 or id(o) in seen:
                return
            seen.add(id(o))
            if isinstance(o, torch.Tensor):
                out.append(o)
            elif isinstance(o, dict):
                for v in o.values():
                    walk(v, depth + 1)
            elif isinstance(o, (list, tuple)):
                for v in o:
                    walk(v, depth + 1)
            elif hasattr(o, "__dict__") and not isinstance(o, type):
                for v in vars(o).values():
                    walk(v, depth + 1)
        for o in (self._ws, self._encfm, self._pos, self.hws, self.hws_b):
            walk(o)
        return out


class GraphedTrainStep:
    """The whole training step captured as HIP graphs (fixed shapes, static input buffers):
    graph A = RNG advance + forward + backward (both streams), then the optional eager RCCL
    all-reduce of the flat gradient buffer, then graph B = fused AdamW.  Replays launch the ~3k
    kernels of a step with no Python or per-launch host cost."""

    def __init__(self, eng: Ver5Engine, wav, wav_len, targets, tgt_len, allreduce=None, world: int = 1):
        self.eng = eng
        self.inputs = (wav, wav_len, targets, tgt_len)
        self.allreduce = allreduce
        scale = 1.0 / world
        self.g_step = torch.cuda.CUDAGraph()
        self.g_opt = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        cs = eng.compute_stream
        with torch.cuda.graph(self.g_step, stream=cs):
            eng.advance_rng()
            ctx = eng.forward(*self.inputs, train=True)
            eng.backward(ctx)
            del ctx
        with torch.cuda.graph(self.g_opt, pool=self.g_step.pool(), stream=cs):
            eng.optimizer_step(scale)
        torch.cuda.synchronize()

    def step(self):
        with self.eng._on_stream():
            self.g_step.replay()
            if self.allreduce is not None:
                self.allreduce(self.eng.student.grad)
            self.g_opt.replay()
        return self.eng.losses


def synthetic_batch(cfg: Ver5Config, B: int, n_samples: int, U: int, device, seed: int = 1234, tgt_seed: int = 4321):
    """wav = 0.1*N(0,1), all lengths N; U tokens uniform in [0, vocab)."""
    g = torch.Generator().manual_seed(seed)
    wav = (0.1 * torch.randn(B, n_samples, generator=g)).to(device)
    wav_len = torch.full((B,), n_samples, dtype=torch.int64, device=device)
    gt = torch.Generator().manual_seed(tgt_seed)
    targets = torch.randint(0, cfg.vocab, (B, U), generator=gt, dtype=torch.int64).to(device)
    tgt_len = torch.full((B,), U, dtype=torch.int64, device=device)
    return wav, wav_len, targets, tgt_len


__all__ = ["Ver5Engine", "synthetic_batch", "math", "_lib"]
