#!/usr/bin/env python3
"""Benchmark of the ContextUnet DDPM hot path on MI355X (driver contract, one JSON line on rank 0).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--sample-steps S] [--no-cpu]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...   (N > 1)

Metric (BASELINE.json): train-step images/s + T=1500 sample images/s, 64x64x1, bs=256 per GPU.
  value   = whole-job train-step throughput: N * 256 images / (max over ranks of the time of K steps)
            one step = Philox noise/t + perturb + ContextUnet fwd (train BN) + mse + bwd + Adam
            (+ bucketed RCCL gradient all-reduce when N > 1), n_feat=128, 6 params, fp32, synthetic data.
  sample  = T=1500 reverse diffusion of 256 images per GPU (w=0, hipGraph-captured steps, on-device
            snapshots): images / wall time; replicas only when N > 1 (no collective).
            + CFG (w=1, 3: cond + uncond halves in one batched forward) over --cfg-sample-steps, extrapolated.
  roofline: the dominant kernel (conv3x3 128->128 @64x64) timed live with HIP events on its stream.
  configs (N=1 only): C4 = bf16 mixed-precision train + CFG w in {0,1,3} sampling; C5 = 256x256,
            n_feat=256, T=2000 at --c5-batch (shortened runs, step counts in the output).
  cpu_baseline: the CPU oracle restatement (torch CPU fp32, the reference algorithm) on the host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "train-step images/sec + T=1500 sample images/sec, 64×64×1, bs=256, 1/2/4/8 GPU"
NF, NCF, H, T = 128, 6, 64, 1500
CONV_GFLOP_PER_IMG = 1.2079596          # conv3x3 128->128 @ 64x64
FWD_GFLOP_PER_IMG = 19.178788
PEAK_FP32_TFLOPS = 157.3                # MI355X dense fp32 MFMA (MI355X_MICROARCH.md)
PEAK_BF16_TFLOPS = 2500.0               # MI355X dense bf16 MFMA (no sparsity)
# conv arithmetic -> (bf16 MFMA products per fp32 MAC, description); peak = fp32-equivalent FLOP/s ceiling
CONV_MATH_INFO = {"fp32": (0, "fp32 MFMA v_mfma_f32_32x32x2_f32"),
                  "x6": (6, "fp32-accurate split-bf16: 3-term bf16 operands, 6 cross products on "
                            "v_mfma_f32_32x32x16_bf16, fp32 accumulate"),
                  "h3": (3, "fp32-class split-fp16: operands scaled by a per-tensor power of two, 2-term fp16 "
                            "(11+11 bits), 3 cross products on v_mfma_f32_32x32x16_f16, fp32 accumulate")}
NT_CODE = {"fp32": 0, "x6": 6, "h3": 4}   # engine / C-ABI arithmetic code


_T0 = time.perf_counter()


def _progress(msg: str):
    """One progress line per leg / CPU step on stderr (the run writes its JSON only at the end; a long silent run
    reads as hung to the GPU harness)."""
    print(f"[bench {time.perf_counter() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def _dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def conv_peak(math: str) -> float:
    nprod = CONV_MATH_INFO[math][0]
    return PEAK_FP32_TFLOPS if nprod == 0 else PEAK_BF16_TFLOPS / nprod


def time_dominant_conv_probe(B: int, math: str, relu: bool, reps: int = 20):
    """Synthetic probe of the same kernel on its own: launch time (HIP events on its stream) on random operands,
    relu(randn) (the forward's post-BN-ReLU inputs) or randn (sign-symmetric, dgrad-like; lower clocks)."""
    import cdm_amd
    L = cdm_amd.lib()
    s = torch.cuda.current_stream()
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(B * H * H, NF, device="cuda", generator=g)
    if relu:
        x.relu_()
    W = torch.randn(NF, NF, 3, 3, device="cuda", generator=g) * 0.05
    b = torch.zeros(NF, device="cuda")
    wpk = torch.empty(9 * NF, NF, device="cuda")
    L.cdm_pack_conv3x3(W.data_ptr(), b.data_ptr(), NF, NF, None, None, None, None, 0.0, wpk.data_ptr(), None, None,
                       16, s.cuda_stream)
    y = torch.empty(B * H * H, NF, device="cuda")
    stats = torch.empty((B * H * H + 127) // 128, 2, NF, device="cuda")
    nterm = NT_CODE[math]
    wx = torch.empty(9 * NF // 16 * 3 * NF * 16, dtype=torch.bfloat16, device="cuda")
    am = torch.empty(2, device="cuda")
    if nterm == 4:
        L.cdm_amax_f32(wpk.data_ptr(), 9 * NF, NF, NF, am.data_ptr() + 4, 0, s.cuda_stream)
        L.cdm_split_f16x2(wpk.data_ptr(), NF, 9 * NF, NF, am.data_ptr() + 4, wx.data_ptr(), s.cuda_stream)
    else:
        L.cdm_split_bf16x3(wpk.data_ptr(), NF, 9 * NF, NF, wx.data_ptr(), s.cuda_stream)
    L.cdm_amax_f32(x.data_ptr(), B * H * H, NF, NF, am.data_ptr(), 0, s.cuda_stream)

    def launch():
        if nterm == 4:
            L.cdm_conv3x3_fwd_h3(x.data_ptr(), B, H, H, NF, NF, wx.data_ptr(), am.data_ptr(), am.data_ptr() + 4,
                                 b.data_ptr(), y.data_ptr(), NF, NF, 0, stats.data_ptr(), NF, 16, None, s.cuda_stream)
        elif nterm:
            L.cdm_conv3x3_fwd_x3(x.data_ptr(), B, H, H, NF, NF, wx.data_ptr(), b.data_ptr(), y.data_ptr(), NF, NF, 0,
                                 stats.data_ptr(), NF, 16, nterm, s.cuda_stream)
        else:
            L.cdm_conv3x3_fwd(x.data_ptr(), B, H, H, NF, NF, wpk.data_ptr(), b.data_ptr(), y.data_ptr(), NF, NF, 0,
                              stats.data_ptr(), NF, 16, s.cuda_stream)

    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        launch()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def time_dominant_conv_in_step(trainer, x0, c, rounds: int = 5):
    """The dominant kernel on the operands it gets in training: one more (eager) training step after the timed region
    records the arguments of its 3x3-conv launches of the roofline shape (128 -> 128 @64x64 forward, batch 256:
    init_conv.conv2, down1 x4, up2 x4 — the real activations, BatchNorm transforms and weights of that step); those
    launches are then re-issued back to back (rounds x 9) between two HIP events on their stream, so no host gap is
    timed.  Re-issuing a forward conv rewrites the same values (its outputs / stats / maxima are idempotent).
    Returns (mean ms per launch, launches per round)."""
    eng = trainer.eng
    calls = []

    def probe(args):
        key, _, B, S, cin, *_rest = args
        cout = args[9]
        if key.endswith(".wpk") and cin == NF and cout == NF and S == H:
            calls.append(args)

    eng.launch_probe = probe
    try:
        trainer.step(x0, c, inject=None, eager=True)
    finally:
        eng.launch_probe = None
    torch.cuda.synchronize()
    st = torch.cuda.Stream()              # re-issued on a stream of our own (the step may run on the null stream)
    calls = [a[:14] + (st.cuda_stream,) + a[15:] for a in calls]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for a in calls:                      # one untimed pass
        eng._conv3x3(*a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(st)
    for _ in range(rounds):
        for a in calls:
            eng._conv3x3(*a)
    e1.record(st)
    e1.synchronize()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    ev = e0.elapsed_time(e1)
    print(f"[conv replay] {len(calls)} launches x {rounds}: events {ev:.3f} ms, wall {wall:.3f} ms, stream {calls[0][14]}",
          file=sys.stderr, flush=True)
    return ev / (rounds * len(calls)), len(calls)


# FETCH_SIZE per byte read in the LDS-halo conv's staging pattern (4 lanes x 16 B = 64 B of a pixel's channel row per
# chunk): 0.6706, measured on a 537 MB tensor read once in exactly that pattern (tools/fetch_calib.hip,
# profiles/r3_fetch_calibration.txt); wide 16-B-per-lane streaming reads give the guide's 0.5 (measured 0.5000)
HALO_FETCH_PER_BYTE = 0.6706


def pmc_traffic(math: str):
    """HBM bytes per launch of the dominant kernel from the committed PMC passes (tools/gpu_profile.sh), or None.

    The 0.6706 FETCH_SIZE calibration holds for the LDS-halo conv's staging pattern only: it is applied to profiles of
    a halo-kernel arithmetic (h3 / x6 / bf16) that carry FETCH_SIZE and WRITE_SIZE (KiB).  A profile with a plain
    ``traffic_bytes`` (the round-1 fp32 gemm_f32_kernel pass) is reported as recorded; anything else gives None, so a
    profile file of another shape never aborts the bench after its timed legs."""
    import glob
    suffix = "" if math == "fp32" else "_" + math
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc_conv128{suffix}.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if math != "fp32" and "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        return int((d["FETCH_SIZE"] / HALO_FETCH_PER_BYTE + d["WRITE_SIZE"]) * 1024)
    if "traffic_bytes" in d:
        return int(d["traffic_bytes"])
    return None


def _cpu_train_rate(R, nf: int, T: int, bs: int, steps: int, warmup: int):
    """Train steps (perturb + fwd + mse + bwd + Adam) of the CPU oracle at batch bs -> seconds per step."""
    from cdm_amd.model import ContextUnet
    torch.manual_seed(0)
    m = ContextUnet(1, nf, NCF, H)                  # only for the reference-identical seeded parameter init
    sd = R.clone_sd(m.state_dict())
    del m
    tr = R.OracleTrainer(sd, n_feat=nf, n_cfeat=NCF, height=H, lr=1e-5)
    _, _, ab = R.make_schedule(T)
    g = torch.Generator().manual_seed(1234)
    x = torch.rand(bs, 1, H, H, generator=g); c = torch.rand(bs, NCF, generator=g)

    def one():
        noise = torch.randn(bs, 1, H, H, generator=g)
        t = torch.randint(1, T + 1, (bs,), generator=g)
        tr.step(x, c, noise, t, T, ab, lambda: R.draw_shortcut(1, nf))
        _progress(f"cpu train step n_feat={nf} bs={bs}")

    for _ in range(warmup):
        one()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    return (time.perf_counter() - t0) / max(steps, 1), tr.sd


def _cpu_sample_rate(R, sd, nf: int, T: int, n: int, w: float, steps: int):
    """`steps` reverse-diffusion steps of the reference sampler (code/train_diffusion_condition.py:312-329: z draw,
    cond (+ uncond) eval forward with its fresh shortcut, CFG combine, denoise_add_noise) -> seconds per step."""
    b, a, ab = R.make_schedule(T)
    fn = R.make_model_fn(sd, n_feat=nf, n_cfeat=NCF, height=H)
    g = torch.Generator().manual_seed(99)
    x = torch.randn(n, 1, H, H, generator=g)
    params = torch.rand(n, NCF, generator=g)
    uncond = torch.zeros_like(params)
    t0 = time.perf_counter()
    for i in range(T, T - steps, -1):
        t = torch.tensor([i / T])
        z = torch.randn(x.shape, generator=g)
        if w > 0:
            ec = fn(x, t, params); eu = fn(x, t, uncond)
            eps = eu + w * (ec - eu)
        else:
            eps = fn(x, t, params)
        x = R.denoise_add_noise(x, i, eps, z, b, a, ab)
        if n >= 32:
            _progress(f"cpu sample step n={n} w={w:g}")
    return (time.perf_counter() - t0) / steps


def host_cpus():
    """(os.cpu_count(), CPUs in this process's affinity mask, cgroup CPU quota or None)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    return os.cpu_count(), aff, quota


def usable_cpus() -> int:
    """os.cpu_count(), capped by the affinity mask and the cgroup CPU quota: on the GPU box
    os.cpu_count() reports the machine's 256 CPUs while the cgroup grants 16, and the oracle's train step runs 1.75x
    slower on 32 threads than on 16 (profiles/r3_host_probe.txt), so more threads than the quota understate the host."""
    cores, aff, quota = host_cpus()
    n = min(cores, aff)
    if quota:
        n = min(n, max(1, int(quota)))
    return n


def cpu_baseline(threads: int):
    """The reference algorithm (CPU oracle = torch CPU fp32 restatement, pinned bit-exact to the reference's own
    outputs) on the host cores, per BASELINE.md §3 (torch.set_num_threads(os.cpu_count()) unless --cpu-threads caps
    it), a bounded sample of ~30 s of CPU work: the C2 train step at bs=256 timed directly (one step, after a bs=8
    warm-up step), 2 sampling steps at n=32 for w=0 and w=1 extrapolated to T=1500 (per image), and config C1
    (n_feat=64, bs=8, T=1000)."""
    from oracle import ref_cpu as R
    cores, aff, quota = host_cpus()
    torch.set_num_threads(threads)
    bs, ns, S = 256, 32, 2
    _cpu_train_rate(R, NF, T, 8, steps=0, warmup=1)                 # load the kernels / allocator at a small batch
    dt, sd = _cpu_train_rate(R, NF, T, bs, steps=1, warmup=0)
    s0 = _cpu_sample_rate(R, sd, NF, T, ns, 0.0, S)
    s1 = _cpu_sample_rate(R, sd, NF, T, ns, 1.0, S)
    del sd
    # C1 (BASELINE.json configs[0]): n_feat=64, bs=8, T=1000
    T1 = 1000
    dt1, sd1 = _cpu_train_rate(R, 64, T1, 8, steps=5, warmup=1)
    s01 = _cpu_sample_rate(R, sd1, 64, T1, 8, 0.0, 10)
    return {
        "value": bs / dt, "unit": "images/s", "cores": threads, "threads": threads, "host_cpus": cores,
        "affinity_cpus": aff,
        "cgroup_cpu_quota": quota, "kind": "port",
        "sample": f"C2 shape: 1 train step (perturb + fwd + mse + bwd + Adam) at bs={bs}, n_feat=128, 64x64, timed "
                  f"directly after a bs=8 warm-up step; CPU oracle = torch CPU fp32 restatement of the reference path on "
                  f"{threads} threads (os.cpu_count() = {cores}, affinity {aff}, cgroup quota {quota})",
        "ms_per_step": round(dt * 1e3, 1),
        "sample_img_per_s_extrapolated": {"w=0": ns / (s0 * T), "w=1": ns / (s1 * T)},
        "sample_note": f"{S} reverse-diffusion steps at n={ns} timed per guide weight ({s0 * 1e3:.0f} / "
                       f"{s1 * 1e3:.0f} ms per step for w=0 / w=1) and extrapolated x{T} steps",
        "c1": {"workload": "C1: n_feat=64, 6 params, 64x64, T=1000, bs=8 (BASELINE configs[0], the reference's CPU "
                           "case)", "train_img_per_s": round(8 / dt1, 3), "train_ms_per_step": round(dt1 * 1e3, 1),
               "train_steps": 5, "sample_ms_per_step": round(s01 * 1e3, 1),
               "sample_img_per_s_extrapolated": 8 / (s01 * T1), "sample_steps_run": 10},
    }


def sample_rate(model, T: int, n: int, w: float, steps: int, rank: int, barrier, dist=None):
    """Time `steps` hipGraph-replayed denoise steps (n images, guide weight w) -> (ms/step, steps run)."""
    from cdm_amd.diffusion import GraphSampler, Schedule
    H, ncf = model.h, model.n_cfeat
    S = min(steps, T)
    sched = Schedule(T, "cuda")
    params = torch.rand(n, ncf, generator=torch.Generator().manual_seed(77 + rank))
    smp = GraphSampler(model, sched, n, w, params, save_rate=20, z_source="device", seed=4321 + rank)
    smp.prepare_rng(host_z=False)
    x_T = torch.randn(n, 1, H, H, generator=torch.Generator().manual_seed(99 + rank))
    smp.prepare()                               # weight pack + hipGraph capture outside the timed region
    barrier()
    ts = time.perf_counter()
    smp.run(x_T, steps=S)                       # S < T: time S steps, extrapolate to T (reported as such)
    barrier()
    dts = time.perf_counter() - ts
    if dist is not None:
        tt = torch.tensor([dts], device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dts = float(tt.item())
    del smp
    return dts / S * 1e3, S


def train_rate(nf: int, H: int, T: int, B: int, math: str, steps: int, warmup: int, rank: int, barrier,
               use_graph: bool = True, dist=None, conv_probe: bool = False):
    """Train steps/s of a fresh seeded ContextUnet on synthetic data -> (model, ms/step, final loss[, conv timing])."""
    from cdm_amd import ContextUnet, Trainer
    torch.manual_seed(0)
    model = ContextUnet(1, nf, NCF, H, shortcut_source="device", conv_math=math).cuda()
    trainer = Trainer(model, 1e-5, T, B, seed=rank, use_graph=use_graph)
    g = torch.Generator(device="cuda").manual_seed(1234 + rank)
    x0 = torch.rand(B, 1, H, H, device="cuda", generator=g)   # synthetic maps in [0,1) (min-max range)
    c = torch.rand(B, NCF, device="cuda", generator=g)        # synthetic normalised parameters
    for _ in range(warmup):
        trainer.step(x0, c)
    # one HIP event after every step on the launch stream (recording one does not synchronise): the per-step GPU times
    # whose median BASELINE.md §3 names; the contract's value stays the barrier-bracketed K-step span
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    barrier()
    t0 = time.perf_counter()
    evs[0].record()
    for k in range(steps):
        trainer.step(x0, c)
        evs[k + 1].record()
    barrier()
    dt = time.perf_counter() - t0
    step_ms = [evs[k].elapsed_time(evs[k + 1]) for k in range(steps)]
    loss = float(trainer.loss.item())
    if dist is not None:
        tt = torch.tensor([dt], device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    conv = time_dominant_conv_in_step(trainer, x0, c) if conv_probe else None
    del trainer
    model.eval()
    train_rate.last_step_ms = step_ms
    if conv_probe:
        return model, dt / steps * 1e3, loss, conv
    return model, dt / steps * 1e3, loss


def step_stats(step_ms):
    """Median / min / max of the per-step GPU times (HIP events), ms."""
    if not step_ms:
        return None
    v = sorted(step_ms)
    n = len(v)
    med = v[n // 2] if n % 2 else 0.5 * (v[n // 2 - 1] + v[n // 2])
    return {"median_ms": round(med, 3), "min_ms": round(v[0], 3), "max_ms": round(v[-1], 3), "steps": n,
            "measured": "HIP events recorded after every timed step on the launch stream"}


def whole_path_rooflines(math: str, B: int, ms_step: float, n: int, sample_ms: dict):
    """Whole-path fractions of the conv arithmetic's ceiling (north_star: training-step and T=1500 sampling throughput
    as achieved roofline fractions): the algorithmic fp32-equivalent FLOPs (forward 19.178788 GFLOP/img,
    train step 3x) over the measured time, against the ceiling of the arithmetic the 3x3 convs run in (h3: 2.5 PF/s / 3
    products; bf16: 2.5 PF/s; fp32: the fp32 MFMA peak).  sample_ms: {"w=0": ms per denoise step, "w=1": ..., ...}; a
    CFG step runs the 2n-image forward.  The non-conv FLOPs (~1 %) count as if they ran at that ceiling too."""
    peak = PEAK_BF16_TFLOPS if math == "bf16" else conv_peak(math)
    tr = 3 * FWD_GFLOP_PER_IMG * B / (ms_step * 1e-3) / 1e3
    out = {"train_step": {"achieved": round(tr, 2), "peak": round(peak, 2), "unit": "TFLOP/s",
                          "frac": round(tr / peak, 4), "gflop_per_img": round(3 * FWD_GFLOP_PER_IMG, 4)}}
    for k, ms in sample_ms.items():
        imgs = n if k == "w=0" else 2 * n
        a = FWD_GFLOP_PER_IMG * imgs / (ms * 1e-3) / 1e3
        out[f"sample_{k}"] = {"achieved": round(a, 2), "peak": round(peak, 2), "unit": "TFLOP/s",
                              "frac": round(a / peak, 4), "forward_images_per_step": imgs}
    return out


def extra_configs(args, barrier):
    """BASELINE configs C4 (bf16 mixed-precision train + CFG sampling) and C5 (256x256, n_feat=256, T=2000),
    single GPU, shortened runs (step counts stated in the output)."""
    out = {}
    # C4: bf16 MFMA operands, fp32 accumulate / master weights / activations; CFG w in {0,1,3}
    model, ms, loss, (cms4, cn4) = train_rate(NF, H, T, args.batch, "bf16", 10, 3, 0, barrier, conv_probe=True)
    c4_steps = step_stats(getattr(train_rate, "last_step_ms", None))
    _progress(f"C4 train {ms:.3f} ms/step")
    c4_tf = CONV_GFLOP_PER_IMG * args.batch / (cms4 * 1e-3) / 1e3
    c4 = {"workload": "C4: ContextUnet n_feat=128 64x64, bf16 mixed-precision convs (bf16 operands, fp32 "
                      "accumulate, fp32 master weights / activations / norms), T=1500",
          "batch": args.batch, "train_img_per_s": round(args.batch / (ms * 1e-3), 2), "train_ms_per_step": round(ms, 3),
          "train_steps": 10, "final_loss": loss,
          "roofline": {"bound": "mfma", "kernel": "conv3x3 128->128 @64x64 fwd (conv3x3_halo_x3_kernel<1,64>, bf16)",
                       "achieved": round(c4_tf, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                       "frac": round(c4_tf / PEAK_BF16_TFLOPS, 4), "launch_ms": round(cms4, 4),
                       "measured": f"mean over the {cn4} forward launches of this shape of a C4 training step, "
                                   "re-issued back to back between HIP events (as the C2 roofline)"},
          "train_tflops": round(3 * FWD_GFLOP_PER_IMG * args.batch / ms, 2), "sample": {}}
    for w in (0.0, 1.0, 3.0):
        sms, S = sample_rate(model, T, args.sample_batch, w, args.extra_sample_steps, 0, barrier)
        _progress(f"C4 sample w={w:g} {sms:.3f} ms/step")
        c4["sample"][f"w={w:g}"] = {"ms_per_denoise_step": round(sms, 3), "steps_run": S,
                                   "img_per_s": round(args.sample_batch / (sms * 1e-3 * T), 4),
                                   "extrapolated_to_T": S < T}
    c4["train_step_stats"] = c4_steps
    c4["whole_path_roofline"] = whole_path_rooflines(
        "bf16", args.batch, ms, args.sample_batch, {k: v["ms_per_denoise_step"] for k, v in c4["sample"].items()})
    out["c4_bf16_cfg"] = c4
    del model
    torch.cuda.empty_cache()
    # C5: 256x256 maps, n_feat=256 (1.093 B params; up0 alone 1.07 B), T=2000, split-bf16 fp32-accurate convs
    B5, T5 = args.c5_batch, 2000
    C5_TRAIN, C5_SAMPLE = 6, 300
    model, ms, loss = train_rate(256, 256, T5, B5, args.conv_math, C5_TRAIN, 2, 0, barrier)
    _progress(f"C5 train {ms:.3f} ms/step")
    sms, S = sample_rate(model, T5, B5, 0.0, C5_SAMPLE, 0, barrier)
    _progress(f"C5 sample {sms:.3f} ms/step")
    out["c5_256"] = {"workload": "C5: ContextUnet n_feat=256, 256x256x1, 6 params, T=2000, train-mode BatchNorm",
                     "conv_math": args.conv_math, "batch": B5, "train_img_per_s": round(B5 / (ms * 1e-3), 3),
                     "train_ms_per_step": round(ms, 3), "train_steps": C5_TRAIN, "final_loss": loss,
                     "train_tflops": round(3 * 1226.82 * B5 / ms, 2),
                     "sample": {"w=0": {"ms_per_denoise_step": round(sms, 3), "steps_run": S,
                                        "img_per_s": round(B5 / (sms * 1e-3 * T5), 5), "extrapolated_to_T": True}}}
    del model
    torch.cuda.empty_cache()
    out["stats_pk_pdf"] = stats_rate(args.sample_batch)
    return out


def reference_logged_workloads(model, barrier):
    """The reference's own logged GPU workloads on this path (…params_6/…/timing_and_performance.log):
    NLL evaluation of 200 images x T=1500 no-grad forwards at bs=32 (calculate_likelihood, code/train_diffusion_elbo.py:
    108-149; logged 364.16 s, :267) and T=1500 sampling of n=10 / n=25 images at w=0 (logged 19.38 s / 45.77 s,
    :280-289) — full runs, nothing extrapolated; the C2 model (h3) on synthetic maps / parameters."""
    from cdm_amd.likelihood import LikelihoodEvaluator
    out = {}
    g = torch.Generator().manual_seed(2024)
    N, bs = 200, 32
    x = torch.rand(N, 1, H, H, generator=g).cuda(); c = torch.rand(N, NCF, generator=g).cuda()
    batches = [(x[i:i + bs], c[i:i + bs]) for i in range(0, N, bs)]
    ev = LikelihoodEvaluator(model, T, "device")
    ev._refresh()
    for xb, cb in (batches[0], batches[-1]):          # capture the B=32 and the ragged B=8 graphs outside the timing
        r = ev._run(xb.shape[0])
        r.load(xb, cb)
        r.capture(ev.K)
    barrier()
    t0 = time.perf_counter()
    nll = ev.likelihood(batches)
    barrier()
    dt = time.perf_counter() - t0
    _progress(f"NLL 200 x T=1500 {dt:.2f} s")
    out["nll_200_T1500"] = {"workload": "calculate_likelihood of 200 maps (bs=32: 6 batches + 8), T=1500 eval forwards "
                                        "each (code/train_diffusion_elbo.py:108-149)", "seconds": round(dt, 3),
                            "img_fwd_per_s": round(N * T / dt, 1), "nll": nll, "reference_logged_s": 364.16,
                            "reference_source": "graphs/conditional_lr_1e-05_epochs_100_timesteps_1500_params_6/"
                                                "spectrum_lr_1e-05_epochs_100_timesteps_1500_params_6/"
                                                "timing_and_performance.log:267 (one NVIDIA GPU, model unrecorded)"}
    for n, logged, line in ((10, 19.38, 280), (25, 45.77, 289)):
        ms, S = sample_rate(model, T, n, 0.0, T, 0, barrier)
        _progress(f"sample n={n} T=1500 {ms:.3f} ms/step")
        out[f"sample_n{n}_T1500"] = {"workload": f"sample_ddpm of {n} maps, T=1500, w=0 (full run)",
                                     "seconds": round(ms * S * 1e-3, 3), "ms_per_denoise_step": round(ms, 3),
                                     "img_per_s": round(n / (ms * S * 1e-3), 3), "steps_run": S,
                                     "reference_logged_s": logged,
                                     "reference_source": f"same log :{line}"}
    return out


def stats_rate(n: int):
    """Sample-statistics row: P(k) (power_spectrum, ortho DFT + radial bins) and per-map PDF
    (0.01 bins) of n 64x64 maps on the HIP kernels, next to the reference algorithm on the CPU (oracle, 8 maps)."""
    import cdm_amd
    from oracle import stats_ref as R
    g = torch.Generator(device="cuda").manual_seed(5)
    maps = torch.rand(n, 1, H, H, device="cuda", generator=g)
    edges = torch.arange(0.0, 1.0 + 0.01, 0.01, dtype=torch.float64).numpy()
    cdm_amd.power_spectra(maps); cdm_amd.pdfs(maps, edges)            # warm-up (bin geometry cached)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        cdm_amd.power_spectra(maps)
    torch.cuda.synchronize()
    pk_ms = (time.perf_counter() - t0) / reps * 1e3
    t0 = time.perf_counter()
    for _ in range(reps):
        cdm_amd.pdfs(maps, edges)
    torch.cuda.synchronize()
    pdf_ms = (time.perf_counter() - t0) / reps * 1e3
    host = maps[:8, 0].cpu().numpy()
    t0 = time.perf_counter()
    for m in host:
        R.power_spectrum(m, 1.0)
        import numpy as np
        np.histogram(m.ravel(), edges, density=True)
    cpu_ms = (time.perf_counter() - t0) / len(host) * 1e3
    return {"workload": f"P(k) (diffusion_utilities.py:302) + PDF (train_diffusion.py:205) of {n} maps 64x64",
            "power_spectra_ms": round(pk_ms, 3), "pdf_ms": round(pdf_ms, 3),
            "maps_per_s": round(n / ((pk_ms + pdf_ms) * 1e-3), 1),
            "cpu_reference_ms_per_map": round(cpu_ms, 3), "cpu_sample": "8 maps, numpy (1 thread, the reference loop)"}


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` with no rank environment (WORLD_SIZE unset): run the N ranks as ONE child process tree,
    `python -m torch.distributed.run --nproc-per-node N ... bench.py <same args>`, inheriting stdout (rank 0 prints the
    JSON line) and stderr, and return its exit status.  Called before anything touches the GPU, and never replaces this
    process (no exec): the parent only waits."""
    import socket
    import subprocess
    with socket.socket() as sk:                      # a free rendezvous port on the loopback interface
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    _progress(f"--gpus {n}: launching {n} ranks (torch.distributed.run, rendezvous 127.0.0.1:{port})")
    return subprocess.call(cmd, env=dict(os.environ))


def plumbing_check(args, world: int, rank: int):
    """CPU rehearsal of the N-rank harness (--plumbing-check; tests/test_bench_cpu.py): gloo process group, the world
    size check, barrier-bracketed timing of K steps with the max over ranks, rank-0 JSON — with a stand-in CPU step (a
    small matmul) instead of the GPU workload.  Not a measurement: the line says so in `metric` and `plumbing_only`."""
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    a = torch.randn(64, 64)

    def barrier():
        if dist is not None:
            dist.barrier()
    for _ in range(args.warmup):
        a = torch.tanh(a @ a)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = torch.tanh(a @ a)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    if rank == 0:
        print(json.dumps({"metric": "plumbing check (no measurement)", "plumbing_only": True, "value": None,
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(dt / max(args.steps, 1) * 1e3, 4),
                          "config": {"parallelism": f"dp{world}", "batch_per_gpu": args.batch,
                                     "global_batch": args.batch * world}}), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--sample-steps", type=int, default=T, help="sampling steps actually run (T=1500 = full)")
    ap.add_argument("--sample-batch", type=int, default=256)
    ap.add_argument("--cfg-sample-steps", type=int, default=T,
                    help="steps run for the C2 CFG (w=1,3) sampling rates (T = full runs)")
    ap.add_argument("--extra-sample-steps", type=int, default=T, help="sampling steps of the C4 legs (T = full runs)")
    ap.add_argument("--c5-batch", type=int, default=16)
    ap.add_argument("--no-extra", action="store_true", help="skip the C4 / C5 legs")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0 = the CPUs this process may use: os.cpu_count() within the affinity "
                         "mask and the cgroup CPU quota)")
    ap.add_argument("--conv-math", choices=sorted(CONV_MATH_INFO), default="h3",
                    help="3x3 conv arithmetic of the C2 / C5 legs (fp32-accurate; see DESIGN.md §3)")
    ap.add_argument("--plumbing-check", action="store_true",
                    help="CPU-only rehearsal of the N-rank launch / timing / JSON path (gloo, stand-in step; no GPU)")
    args = ap.parse_args()

    # --gpus N: the ranks come from the environment of torch.distributed.run; without one, this process launches them
    # (before any GPU call) and relays their exit status
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = _dist_env()
    if world != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}")
    if args.plumbing_check:
        plumbing_check(args, world, rank)
        return
    # rehearsal of the N>1 path on a one-GPU box: CDM_BENCH_REHEARSE=1 puts every rank on cuda:0 and runs the
    # collectives over gloo (RCCL refuses two ranks on one device); never set by the driver's runs
    rehearse = os.environ.get("CDM_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    import cdm_amd  # noqa: F401

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    B = args.batch
    model, ms_step, loss, (conv_ms, conv_n) = train_rate(NF, H, T, B, args.conv_math, args.steps, args.warmup, rank,
                                                         barrier, use_graph=not args.no_graph, dist=dist,
                                                         conv_probe=True)
    train_ips = world * B / (ms_step * 1e-3)
    c2_steps = step_stats(getattr(train_rate, "last_step_ms", None))
    _progress(f"C2 train {ms_step:.3f} ms/step")

    # ---------------- sampling (replicas) ----------------
    n = args.sample_batch
    sms, S = sample_rate(model, T, n, 0.0, args.sample_steps, rank, barrier, dist)
    sample_ips = world * n / (sms * 1e-3 * T)
    _progress(f"C2 sample w=0 {sms:.3f} ms/step")
    cfg = {}
    for w in ((1.0, 3.0) if args.cfg_sample_steps > 0 else ()):   # 0: no CFG legs (profiling runs)
        cms, CS = sample_rate(model, T, n, w, args.cfg_sample_steps, rank, barrier, dist)
        _progress(f"C2 sample w={w:g} {cms:.3f} ms/step")
        cfg[f"w={w:g}"] = {"ms_per_denoise_step": round(cms, 3), "steps_run": CS,
                           "img_per_s": round(world * n / (cms * 1e-3 * T), 4), "extrapolated_to_T": CS < T}
    logged = reference_logged_workloads(model, barrier) if (world == 1 and not args.no_extra) else None
    del model
    torch.cuda.empty_cache()

    # ---------------- roofline of the dominant kernel ----------------
    conv_tflops = CONV_GFLOP_PER_IMG * B / (conv_ms * 1e-3) / 1e3
    probe_relu = time_dominant_conv_probe(B, args.conv_math, relu=True)
    probe_randn = time_dominant_conv_probe(B, args.conv_math, relu=False)
    peak = conv_peak(args.conv_math)

    extra = extra_configs(args, barrier) if (world == 1 and not args.no_extra) else None

    wp = whole_path_rooflines(args.conv_math, B, ms_step, n,
                              {"w=0": sms, **{k: v["ms_per_denoise_step"] for k, v in cfg.items()}})
    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(train_ips, 3),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic",
            "config": {"workload": "ContextUnet DDPM train step (fwd+bwd+Adam), n_feat=128, 6 params, 64x64x1, "
                                   "T=1500, train-mode BatchNorm",
                       "batch_per_gpu": B, "global_batch": B * world, "n_feat": NF, "n_cfeat": NCF, "T": T,
                       "parallelism": f"dp{world}", "conv_math": args.conv_math},
            "sample": {"img_per_s": round(sample_ips, 4), "T": T, "steps_run": S, "extrapolated": S < T,
                       "n_per_gpu": n, "guide_w": 0.0, "ms_per_denoise_step": round(sms, 3),
                       "scaling": "replicas", "cfg": cfg},
            "roofline": {"bound": "mfma",
                         "kernel": "conv3x3 128->128 @64x64 fwd (" + (
                             f"conv3x3_halo_x3_kernel<{NT_CODE[args.conv_math]},64> (PreBnRelu / PreNone staging)"
                             if NT_CODE[args.conv_math] else "gemm_f32_kernel<LdIm2colA<128,16,64>>") + ")",
                         "arithmetic": CONV_MATH_INFO[args.conv_math][1],
                         "achieved": round(conv_tflops, 2), "peak": round(peak, 2), "unit": "TFLOP/s",
                         "frac": round(conv_tflops / peak, 4), "traffic": pmc_traffic(args.conv_math),
                         "launch_ms": round(conv_ms, 4),
                         "measured": f"mean over the {conv_n} forward launches of this shape of a training step (their "
                                     f"real operands, recorded in one extra step after the timed region), re-issued "
                                     f"back to back between HIP events on the launch stream",
                         "probe_ms": {"relu_randn": round(probe_relu, 4), "randn": round(probe_randn, 4),
                                      "note": "the kernel alone on synthetic operands, same launch"},
                         "algorithmic": f"{CONV_GFLOP_PER_IMG} GFLOP/img x {B} img per launch (fp32 FLOPs); peak = "
                                        + ("fp32 MFMA dense" if peak == PEAK_FP32_TFLOPS else
                                           f"bf16/fp16 MFMA dense {PEAK_BF16_TFLOPS:.0f} / "
                                           f"{CONV_MATH_INFO[args.conv_math][0]} products per fp32 MAC"),
                         "vs_fp32_mfma_peak": round(conv_tflops / PEAK_FP32_TFLOPS, 4)},
            "train_tflops_per_gpu": round(3 * FWD_GFLOP_PER_IMG * B / (ms_step * 1e-3) / 1e3, 2),
            "train_step_stats": c2_steps,
            "whole_path_roofline": wp,
            "final_loss": loss,
        }
        out["sample"]["roofline"] = {k[len("sample_"):]: v for k, v in wp.items() if k.startswith("sample_")}
        if extra:
            out["configs"] = extra
        if logged:
            out["reference_logged_workloads"] = logged
        if not args.no_cpu and world == 1:      # the CPU baseline is an N=1 leg (rank 0)
            out["cpu_baseline"] = cpu_baseline(args.cpu_threads or usable_cpus())
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
