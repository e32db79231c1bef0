#!/usr/bin/env python
"""Benchmark: UNet denoising steps/sec on 1x128x512 mel-latents (BASELINE.json metric), config 2:
50-step DDIM reverse sample (49 UNet + scheduler iterations), batch 8 per GPU, latent [8,32,16,64],
fp32, style maps from a 1x128x512 style spectrogram.

One bench "step" = one complete 49-iteration reverse loop over the batch (replayed from one hipGraph,
including the reference's per-step pred_x0 / noise_pred log copies).  value = denoising iterations
(UNet forward + DDIM update over a batch-8 latent) per second summed over all ranks.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (weak scaling: 8 latents per GPU)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "music-style-transfer-ldm_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

METRIC = "UNet denoising steps/sec on 1×128×512 mel-latents, 1/2/4/8 MI355X"
FP32_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_*_f32) = FP32 vector peak
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
UNET_GFLOP_PER_SAMPLE = 0.4494   # SURVEY.md §8(d), torch FlopCounterMode-verified


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("sample", "transfer", "train"), default="sample",
                    help="sample = config 2 (the BASELINE metric, default); transfer = config 5 (content/style "
                         "transfer loop, T'=100, eta=1.0); train = configs 3/4 (encode -> UNet train step -> decode, "
                         "batch 32/GPU, RCCL grad all-reduce when N>1)")
    ap.add_argument("--batch", type=int, default=None, help="latents per GPU (8 sample/transfer, 32 train)")
    ap.add_argument("--timesteps", type=int, default=None, help="50 for sample, T'=100 for transfer")
    ap.add_argument("--eta", type=float, default=None, help="0.0 for sample, 1.0 for transfer")
    ap.add_argument("--split", type=int, default=1,
                    help="run the per-GPU batch as this many sub-batch chains on separate streams (one graph)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bound on the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="per-kernel HBM traffic summary produced from a rocprofv3 --pmc pass")
    a = ap.parse_args()
    if a.batch is None:
        a.batch = 32 if a.workload == "train" else 8
    if a.timesteps is None:
        a.timesteps = 100 if a.workload == "transfer" else 50
    if a.eta is None:
        a.eta = 1.0 if a.workload == "transfer" else 0.0
    return a


def layer_flops(d):
    """Algorithmic FLOPs of one conv launch: 2 * B * Cout * Hout * Wout * Cin * (taps hitting each output)."""
    if d.transposed:
        # each output parity sees kh*kw/4 taps on average (exact for k even; k3: (1+2+2+4)/4)
        taps = d.kh * d.kw / 4.0
    else:
        taps = d.kh * d.kw
    return 2.0 * d.B * d.Cout * d.Hout * d.Wout * d.Cin * taps


def layer_bytes(d):
    """Algorithmic HBM bytes of one conv launch: weights + input + output (fp32, unique)."""
    w = d.Cout * d.Cin * d.kh * d.kw
    return 4.0 * (w + d.B * d.Cin * d.Hin * d.Win + d.B * d.Cout * d.Hout * d.Wout)


def _graph_time_us(fn, reps):
    """Average device time per call of fn() in a dependent chain: reps calls captured in one hipGraph,
    replayed, bracketed by HIP events on the replay stream (host launch cost excluded)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    g.replay()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def time_layers(engine, shape, dev, reps=50):
    """Average launch duration of each UNet GEMM-shaped kernel, HIP events on the launching stream."""
    import ctypes
    from ldm_amd import _lib as L
    from ldm_amd import ops
    w = engine.weights(shape)
    names = ["enc1", "enc2", "enc3", "enc4", "bottleneck", "dec4", "dec3", "dec2", "dec1",
             "ca2.q", "ca2.kv", "ca2.out", "ca1.q", "ca1.kv", "ca1.out"]
    plans = list(w.conv_plan) + [w.ca_plan_q[0], w.ca_plan_kv[0], w.ca_plan_o[0],
                                 w.ca_plan_q[1], w.ca_plan_kv[1], w.ca_plan_o[1]]
    wptr = list(w.conv_w) + [w.ca_wq[0], w.ca_wkv[0], w.ca_wo[0], w.ca_wq[1], w.ca_wkv[1], w.ca_wo[1]]
    bptr = list(w.conv_b) + [w.ca_bq[0], w.ca_bkv[0], w.ca_bo[0], w.ca_bq[1], w.ca_bkv[1], w.ca_bo[1]]
    out = {}
    st = torch.cuda.current_stream()
    for i, name in enumerate(names):
        d = L.ConvDesc()
        L.call("ldm_unet_layer_desc", ctypes.byref(shape), i, ctypes.byref(d))
        x = torch.randn(d.B, d.Cin, d.Hin, d.Win, device=dev)
        y = torch.empty(d.B, d.Cout, d.Hout, d.Wout, device=dev)
        ep = L.Epilogue()
        ep.bias = bptr[i]
        ep.act = 1 if i < 8 else 0
        plan = plans[i]
        ws = torch.zeros(max(1, int(plan.ws_floats)), device=dev)     # split-K counters + partials
        args = (ctypes.byref(d), ctypes.byref(plan), x.data_ptr(), wptr[i], ctypes.byref(ep), y.data_ptr(),
                ws.data_ptr())
        lib = L.load()
        L.check(lib.ldm_conv_forward_ws(*args, st.cuda_stream), name)
        us = _graph_time_us(lambda: lib.ldm_conv_forward_ws(*args, torch.cuda.current_stream().cuda_stream), reps)
        fl, by = layer_flops(d), layer_bytes(d)
        out[name] = {"us": round(us, 3), "tflops": round(fl / us / 1e6, 2), "gbs": round(by / us / 1e3, 1),
                     "flops": fl, "bytes": by, "plan": list(plan.key())}
    # attention cores
    for name, E, Lt in (("attn2", 256, shape.H * shape.W // 16), ("attn1", 512, shape.H * shape.W // 64)):
        q = torch.randn(shape.B, E, Lt, device=dev)
        kv = torch.randn(shape.B, 2 * E, Lt, device=dev)
        o = torch.empty_like(q)
        scale = float((1.0 / (E // 4)) ** 0.5)
        lib = L.load()
        us = _graph_time_us(lambda: lib.ldm_attention_core(q.data_ptr(), kv.data_ptr(), o.data_ptr(), shape.B, E, 4,
                                                           Lt, Lt, scale, torch.cuda.current_stream().cuda_stream),
                            reps)
        fl = 4.0 * shape.B * E * Lt * Lt
        by = 4.0 * shape.B * 4 * E * Lt
        out[name] = {"us": round(us, 3), "tflops": round(fl / us / 1e6, 2), "gbs": round(by / us / 1e3, 1),
                     "flops": fl, "bytes": by}
        # the reverse loop's folded form: scores from the projection input z against scale*Wq^T K
        z = torch.randn(shape.B, Lt, E, device=dev)
        kf = torch.randn(shape.B, 4, Lt, E, device=dev)
        bf = torch.randn(shape.B, 4, Lt, device=dev)
        us = _graph_time_us(lambda: lib.ldm_attention_folded(z.data_ptr(), kv.data_ptr(), kf.data_ptr(), bf.data_ptr(),
                                                             o.data_ptr(), shape.B, E, 4, Lt, Lt,
                                                             torch.cuda.current_stream().cuda_stream), reps)
        fl = 2.0 * shape.B * 4 * Lt * Lt * E + 2.0 * shape.B * E * Lt * Lt
        by = 4.0 * shape.B * (Lt * E * 2 + 4 * E * Lt + 2 * E * Lt)
        out[name + "f"] = {"us": round(us, 3), "tflops": round(fl / us / 1e6, 2), "gbs": round(by / us / 1e3, 1),
                           "flops": fl, "bytes": by}
    return out


def cpu_baseline(ldm, batch, times, eta, seconds):
    """The oracle's torch-CPU restatement of the reference loop (oracle/ldm_torch_cpu.py), fp32, on this
    box's host cores, over a bounded number of denoising iterations of the same workload."""
    from oracle import ldm_torch_cpu as TC
    try:
        ncores = len(os.sched_getaffinity(0))
    except AttributeError:
        ncores = os.cpu_count() or 1
    ncores = max(1, min(ncores, 16))   # the GPU box's CPU share per GPU (16)
    torch.set_num_threads(ncores)
    sd = {k: v.detach().float().cpu() for k, v in ldm.state_dict().items()}
    ab = TC.schedule(200)[2]
    g = torch.Generator().manual_seed(5)
    style = torch.rand(batch, 1, 128, 512, generator=g)
    x = torch.randn(batch, 32, 16, 64, generator=g)
    with torch.no_grad():
        emb = TC.style_encoder(sd, style)
        s5, s6 = emb["s5"], emb["s6"]
        TC.reverse_loop(sd, ab, x, s5, s6, times[:2], eta)        # warm-up (1 iteration)
        n, t0 = 0, time.perf_counter()
        while True:
            i = n % (len(times) - 1)
            TC.reverse_loop(sd, ab, x, s5, s6, times[i:i + 2], eta)
            n += 1
            if time.perf_counter() - t0 >= seconds and n >= 3:
                break
        dt = time.perf_counter() - t0
    return {"value": round(n / dt, 3), "unit": "steps/s", "cores": ncores, "kind": "port",
            "sample": f"{n} DDIM iterations (UNet fwd + update, batch {batch}, [{batch},32,16,64] latents, fp32) "
                      f"of the same 50-step schedule, torch-CPU restatement oracle/ldm_torch_cpu.py, {dt:.1f}s"}


TRAIN_GFLOP_PER_SAMPLE = 10.7   # frozen VAE enc fwd 0.698 + 3 x (style enc 1.642 + UNet 0.449 + dec 1.242)


def run_train(args, world, rank, dev, M):
    """Configs 3/4: LDMTrainer.train_step (reference train.py:163-208) = VAE encode -> style encode ->
    q_sample -> UNet -> predict_start -> VAE decode -> losses -> backward -> (RCCL bucketed grad
    all-reduce when N>1) -> GradScaler + Adam.  Eager (the step ends in the reference's .item() syncs).
    value = samples/s over all ranks; weak scaling (batch per GPU fixed)."""
    import torch.distributed as dist
    from models.train import LDMTrainer
    torch.manual_seed(0)
    ldm = M.LDM(32, pretrained_path="").to(dev)               # random-init weights of the architecture
    if world > 1:
        from ldm_amd import dist as hdist                      # same initial weights on every rank
        hdist.broadcast_parameters(ldm)
    trainer = LDMTrainer(ldm, None, dev, lr=1e-4)                 # LDMTrainer default (train.py:142)
    ldm.train()
    B = args.batch
    g = torch.Generator().manual_seed(11 + rank)
    content = torch.rand(B, 1, 128, 512, generator=g).to(dev)
    style = torch.rand(B, 1, 128, 512, generator=g).to(dev)
    torch.manual_seed(7 + rank)
    for _ in range(args.warmup):
        trainer.train_step(content, style)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        losses = trainer.train_step(content, style)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if not all(map(lambda v: v == v and abs(v) != float("inf"), losses.values())):
        raise SystemExit(f"non-finite losses {losses}")
    ms_step = elapsed / args.steps * 1e3
    value = B * world * args.steps / elapsed
    flops = TRAIN_GFLOP_PER_SAMPLE * 1e9 * B
    achieved = flops / (ms_step * 1e-3) / 1e12
    return {
        "metric": "LDM train samples/sec (encode -> UNet train step -> decode), 1/2/4/8 MI355X",
        "value": round(value, 2), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (U[0,1) content/style mels; random-init weights; t ~ randint on device)",
        "config": {"workload": f"configs 3/4: LDMTrainer.train_step, batch {B}/GPU, 1x128x512 mels, fp32 kernels "
                               f"inside the reference's autocast region, Adam + GradScaler"
                               + (f", RCCL bucketed grad all-reduce over {world} ranks" if world > 1 else ""),
                   "global_batch": B * world, "parallelism": f"dp{world}"},
        "roofline": {"kernel": "whole train step (composite)", "bound": "mfma", "achieved": round(achieved, 2),
                     "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
                     "traffic": None, "flops_per_step": flops},
        "last_losses": {k: round(v, 6) for k, v in losses.items()},
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    import models.model as M
    from ldm_amd.engine import GraphedDDIM

    if args.workload == "train":
        result = run_train(args, world, rank, dev, M)
        if rank == 0:
            print(json.dumps(result), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    torch.manual_seed(0)
    ldm = M.LDM(32, pretrained_path="").to(dev).eval()     # random-init weights of the architecture
    B = args.batch
    g = torch.Generator().manual_seed(1 + rank)
    style = torch.rand(B, 1, 128, 512, generator=g).to(dev)   # synthetic 1x128x512 style mel, U[0,1)
    if args.workload == "transfer":
        # config 5: encode a content mel, q_sample it at T'-1, then the T'-step loop (model.py:468-559)
        content = torch.rand(B, 1, 128, 512, generator=torch.Generator().manual_seed(101 + rank)).to(dev)
        with torch.no_grad():
            z0 = ldm.encoder(content)
            t_start = torch.full((B,), args.timesteps - 1, dtype=torch.long, device=dev)
            z_T, _ = ldm.noise_scheduler(z0, t_start)
        times = torch.linspace(args.timesteps - 1, 0, args.timesteps).long()          # (model.py:514)
    else:
        torch.manual_seed(1234 + rank)
        z_T = torch.randn((B, 32, 16, 64)).to(dev)                 # CPU generator like model.py:394
        times = torch.linspace(ldm.num_timesteps - 1, 0, args.timesteps).long()
    n_iter = len(times) - 1
    coefs = ldm.noise_scheduler.reverse_coefs(times).to(dev)
    t_table = times[:-1].view(-1, 1).expand(-1, B).contiguous().to(dev)
    with torch.no_grad():
        emb = ldm.style_encoder(style)
        eng = M.engine_for(ldm.unet)
        gd = GraphedDDIM(eng, z_T, emb["s5"], emb["s6"], t_table, coefs, args.eta, logs=True, split=args.split)
        for _ in range(args.warmup):
            gd.replay()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            gd.replay()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    if not torch.isfinite(gd.x).all():
        raise SystemExit("non-finite sample")
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    iters = n_iter * args.steps * world
    value = iters / elapsed
    ms_step = elapsed / args.steps * 1e3
    us_iter = elapsed / (n_iter * args.steps) * 1e6

    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32", "data": "synthetic (U[0,1) style mel, N(0,1) z_T; random-init weights)",
        "config": {"workload": (f"config 2: {args.timesteps}-step DDIM reverse sample ({n_iter} UNet+update "
                                f"iterations per step), batch {B}/GPU, 1x128x512 mel -> [{B},32,16,64] latents, "
                                f"eta={args.eta}, hipGraph replay of {args.split} concurrent sub-batch chains")
                   if args.workload == "sample" else
                   (f"config 5: content/style transfer loop, T'={args.timesteps} ({n_iter} UNet+update iterations "
                    f"per step, content encoded and q_sampled at T'-1 before timing), batch {B}/GPU, "
                    f"eta={args.eta}, fp32 compute and accumulators (>= the config's fp16), hipGraph replay"),
                   "global_batch": B * world,
                   "latent": [B, 32, 16, 64], "parallelism": f"dp{world} (independent batch shards)"},
        "us_per_denoise_iteration": round(us_iter, 2),
    }
    # whole-step composite roofline
    flops_iter = UNET_GFLOP_PER_SAMPLE * 1e9 * B
    bytes_iter = 27.37e6 + B * (2.52e6 + 0.655e6)
    t_roof = max(flops_iter / (FP32_PEAK_TFLOPS * 1e12), bytes_iter / (HBM_PEAK_GBS * 1e9))
    result["step_roofline"] = {"t_roof_us": round(t_roof * 1e6, 2), "t_measured_us": round(us_iter, 2),
                               "frac": round(t_roof * 1e6 / us_iter, 4),
                               "achieved_tflops": round(flops_iter / (us_iter * 1e-6) / 1e12, 2)}

    if rank == 0 and not args.no_kernel_timing:
        with torch.no_grad():
            kt = time_layers(eng, eng.shape(B, 32, 16, 64), dev)
        convs = {k: v for k, v in kt.items() if "plan" in v}
        dom = max(convs, key=lambda k: convs[k]["us"])
        dk = kt[dom]
        traffic = None
        if os.path.exists(args.pmc):
            try:
                with open(args.pmc) as f:
                    pmc = json.load(f)
                traffic = pmc.get("per_launch_bytes", {}).get(dom)
            except (OSError, ValueError):
                traffic = None
        result["roofline"] = {"kernel": f"conv_mfma ({dom})", "bound": "mfma",
                              "achieved": dk["tflops"], "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                              "frac": round(dk["tflops"] / FP32_PEAK_TFLOPS, 4), "traffic": traffic,
                              "flops_per_launch": dk["flops"], "avg_launch_us": dk["us"]}
        result["kernels"] = {k: {kk: vv for kk, vv in v.items() if kk not in ("flops", "bytes")} for k, v in kt.items()}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(ldm, B, times, args.eta, args.cpu_seconds)
        result["gpu_over_cpu"] = round(value / result["cpu_baseline"]["value"], 1)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
