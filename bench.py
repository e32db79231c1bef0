#!/usr/bin/env python
"""Benchmark: UNet denoising steps/sec on 1x128x512 mel-latents (BASELINE.json metric), config 2:
50-step DDIM reverse sample (49 UNet + scheduler iterations), batch 8 per GPU, latent [8,32,16,64],
fp32, style maps from a 1x128x512 style spectrogram.

One bench "step" = one complete 49-iteration reverse loop over the batch (replayed from one hipGraph,
including the reference's per-step pred_x0 / noise_pred log copies).  value = denoising iterations
(UNet forward + DDIM update over a batch-8 latent) per second summed over all ranks.

    python bench.py [--gpus N --steps K --warmup W]       (N > 1: bench.py starts its own N ranks)
    torchrun --nproc-per-node N bench.py --gpus N ...      (weak scaling: 8 latents per GPU)

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py is its own launcher: before any GPU call it
checks that N HIP devices are visible, starts N fresh worker processes of itself (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, the same env:// rendezvous and init_process_group("nccl")
path torchrun gives them), waits for them and exits with the first failing rank's code.  Under torchrun
(WORLD_SIZE set) --gpus must equal WORLD_SIZE.
"""
import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "music-style-transfer-ldm_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

METRIC = "UNet denoising steps/sec on 1×128×512 mel-latents, 1/2/4/8 MI355X"
FP32_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_*_f32) = FP32 vector peak
LOWP_PEAK_TFLOPS = 2500.0     # MI355X_MICROARCH.md: BF16 / F16 dense MFMA peak
DT_CODE = {"fp32": 0, "fp16": 1, "bf16": 2}
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
UNET_GFLOP_PER_SAMPLE = 0.4494   # SURVEY.md §8(d), torch FlopCounterMode-verified


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("sample", "transfer", "train", "stress"), default="sample",
                    help="sample = config 2 (the BASELINE metric, default); transfer = config 5 (content/style "
                         "transfer loop, T'=100, eta=1.0); train = configs 3/4 (encode -> UNet train step -> decode, "
                         "batch 32/GPU, RCCL grad all-reduce when N>1); stress = SURVEY's secondary shape S "
                         "(UNet(1, 1) on the raw [1,1,128,512] mel, 50-step DDIM, batch 1/GPU)")
    ap.add_argument("--batch", type=int, default=None, help="latents per GPU (8 sample/transfer, 32 train)")
    ap.add_argument("--timesteps", type=int, default=None, help="50 for sample, T'=100 for transfer")
    ap.add_argument("--eta", type=float, default=None, help="0.0 for sample, 1.0 for transfer")
    ap.add_argument("--dtype", choices=("fp32", "fp16", "bf16"), default=None,
                    help="step-kernel operand precision (fp32 accumulation and sampler state): fp32 for sample "
                         "(config 2), fp16 for transfer (config 5)")
    ap.add_argument("--split", type=int, default=1,
                    help="run the per-GPU batch as this many sub-batch chains on separate streams (one graph)")
    ap.add_argument("--train-eager", action="store_true", help="train workload: no hipGraph capture of the step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cpu-legs", action="store_true", help="skip the config-1 / config-3 CPU legs")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r06", "pmc_traffic_step.json"),
                    help="per-kernel HBM traffic summary produced from a rocprofv3 --pmc pass (fp32 step kernels)")
    ap.add_argument("--pmc-lowp", default=os.path.join(ROOT, "profiles", "r06", "pmc_traffic_step_fp16.json"),
                    help="the same for the fp16 step kernels (config 5, DTYPE=fp16 tools/pmc_step_traffic.sh)")
    a = ap.parse_args()
    if a.batch is None:
        a.batch = {"train": 32, "stress": 1}.get(a.workload, 8)
    if a.timesteps is None:
        a.timesteps = 100 if a.workload == "transfer" else 50
    if a.eta is None:
        a.eta = 1.0 if a.workload == "transfer" else 0.0
    if a.dtype is None:
        a.dtype = {"transfer": "fp16", "train": "bf16"}.get(a.workload, "fp32")
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
    from ldm_amd.graphs import capture
    with capture(g):
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


STEP_LAYERS = [  # (name, Cin, Cout, mode 0 conv s1 / 1 conv s2 / 2 convT s2, input scale divisor)
    ("enc1", 32, 64, 0, 1), ("enc2", 64, 128, 1, 1), ("enc3", 128, 256, 1, 2), ("enc4", 256, 512, 1, 4),
    ("bottleneck", 512, 512, 0, 8), ("dec4", 512, 256, 2, 8), ("dec3", 256, 128, 2, 4), ("dec2", 128, 64, 2, 2)]
def _layer_forms():
    """KS_LAYERS: the layers the loop runs on uconv.hip's K-split form, as the library reports them
    (ldm_step_layer_forms; LDM_UCONV_KS overrides its default)."""
    from ldm_amd import _lib as L
    k = L.step_layer_forms()
    return tuple(l for l in range(9) if (k >> l) & 1)


def time_step_layers(engine, B, H, W, dev, reps=50):
    """Average launch duration of each kernel of the reverse loop's UNet step, launched exactly as the loop
    launches it (the engine's packed step weights and folded biases on uconv.hip), timed as a dependent chain of `reps` launches in one hipGraph with HIP
    events on the launching stream.  dec1 runs fused with the DDIM update and is not timed alone."""
    from ldm_amd import _lib as L
    lib = L.load()
    KS_LAYERS = _layer_forms()
    shape = engine.shape(B, 32, H, W)
    w = engine.weights(shape)
    out = {}
    # the bottleneck on CA1's folded values (bfold.hip) replaces CA1's P V and the uconv bottleneck in the loop
    bfold = int(w.use_step) != 0 and bool(lib.ldm_bneck_fold_supported(B, H, W))
    for layer, (name, cin, cout, mode, div) in enumerate(STEP_LAYERS):
        if bfold and name == "bottleneck":
            u = torch.randn(B, 512, 576, device=dev)
            pr = torch.softmax(torch.randn(B, 4, 16, 16, device=dev), -1).contiguous()
            pbias = torch.randn(16, 512, device=dev)
            yb = torch.empty(B, 16, 512, device=dev)
            dt = int(w.step_dtype)
            fn = lambda: lib.ldm_bneck_pv(u.data_ptr(), pr.data_ptr(), pbias.data_ptr(), yb.data_ptr(), B, dt,  # noqa: E731
                                          torch.cuda.current_stream().cuda_stream)
            L.check(fn(), name)
            us = _graph_time_us(fn, reps)
            fl = 2.0 * B * 16 * 512 * 576
            by = 4.0 * (B * 512 * 576 + B * 4 * 256 + 16 * 512 + B * 16 * 512)
            out[name] = {"us": round(us, 3), "tflops": round(fl / us / 1e6, 2), "gbs": round(by / us / 1e3, 1),
                         "flops": fl, "bytes": by, "bound": "hbm",
                         "kernel": "bneck_pv_kernel (CA1 values folded into the bottleneck, K = 576 per sample)"}
            continue
        hin, win = H // div, W // div
        hout, wout = (hin, win) if mode == 0 else ((hin // 2, win // 2) if mode == 1 else (2 * hin, 2 * win))
        x = torch.randn(B, hin, win, cin, device=dev)
        y = torch.empty(B, hout, wout, cout, device=dev)
        bias = w.step_pb[layer - 3] if layer in (3, 4) else w.conv_b[layer]
        bc = torch.randn(B, cout, device=dev) if layer == 1 else None
        sk = torch.randn(B, hout, wout, cout, device=dev) if mode == 2 else None
        dt = int(w.step_dtype)
        nws = int(lib.ldm_step_workspace_floats(B, H, W))
        ws = torch.zeros(max(1, nws), device=dev)
        args = (x.data_ptr(), w.step_w[layer], bias, None if bc is None else bc.data_ptr(),
                None if sk is None else sk.data_ptr(), y.data_ptr())

        def run():
            stp = torch.cuda.current_stream().cuda_stream
            return lib.ldm_step_conv_ws(layer, B, H, W, *args, dt, ws.data_ptr() if nws else None, stp)

        L.check(run(), name)
        us = _graph_time_us(run, reps)
        taps = 9 if mode < 2 else 2.25
        fl = 2.0 * B * cout * hout * wout * cin * taps
        by = (2.0 if dt else 4.0) * cin * cout * 9 + 4.0 * (B * cin * hin * win + B * cout * hout * wout)
        out[name] = {"us": round(us, 3), "tflops": round(fl / us / 1e6, 2), "gbs": round(by / us / 1e3, 1),
                     "flops": fl, "bytes": by, "kernel": ("uconv_kernel (K split)" if layer in KS_LAYERS else "uconv_kernel")
                     + ("" if dt == 0 else (" fp16 operands" if dt == 1 else " bf16 operands"))}
    # the folded cross-attentions of the loop (CA1: its probabilities only when the bottleneck takes the values)
    for name, E, Lt in (("attn2_folded", 256, H * W // 16), ("attn1_folded", 512, H * W // 64)):
        z = torch.randn(B, Lt, E, device=dev)
        kv = torch.randn(B, 2 * E, Lt, device=dev)
        kf = torch.randn(B, 4, Lt, E, device=dev)
        bf = torch.randn(B, 4, Lt, device=dev)
        o = torch.empty(B, Lt, E, device=dev)
        probs = bfold and name == "attn1_folded"
        own = probs and bool(lib.ldm_ca1_probs_form())   # the loop's CA1 launch: ca1_probs_kernel (the default)
        if own:
            us = _graph_time_us(lambda: lib.ldm_ca1_probs(z.data_ptr(), kf.data_ptr(), bf.data_ptr(), o.data_ptr(), B,
                                                          torch.cuda.current_stream().cuda_stream), reps)
            fl = 2.0 * B * 4 * Lt * Lt * E
            by = 4.0 * B * (Lt * E + 4 * E * Lt + 4 * Lt * Lt)
        elif probs:
            us = _graph_time_us(lambda: lib.ldm_attention_folded_probs(z.data_ptr(), kf.data_ptr(), bf.data_ptr(),
                                                                       o.data_ptr(), B, E, 4, Lt, Lt,
                                                                       torch.cuda.current_stream().cuda_stream), reps)
            fl = 2.0 * B * 4 * Lt * Lt * E
            by = 4.0 * B * (Lt * E + 4 * E * Lt + 4 * Lt * Lt)
        else:
            us = _graph_time_us(lambda: lib.ldm_attention_folded(z.data_ptr(), kv.data_ptr(), kf.data_ptr(),
                                                                 bf.data_ptr(), o.data_ptr(), B, E, 4, Lt, Lt,
                                                                 torch.cuda.current_stream().cuda_stream), reps)
            fl = 2.0 * B * 4 * Lt * Lt * E + 2.0 * B * E * Lt * Lt
            by = 4.0 * B * (Lt * E * 2 + 4 * E * Lt + 2 * E * Lt)
        out[name] = {"us": round(us, 3), "tflops": round(fl / us / 1e6, 2), "gbs": round(by / us / 1e3, 1),
                     "flops": fl, "bytes": by, "bound": "hbm",
                     "kernel": "ca1_probs_kernel (folded, probabilities only)" if own else
                               "attention_mfma_kernel (folded" + (", probabilities only)" if probs else ")")}
    return out


def cpu_env():
    """Host cores for the CPU baseline: every core of this process's affinity mask, capped by the CPU share
    the box declares for one GPU (OMP_NUM_THREADS; the GPU box sets 16), and the CPU model name."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(aff, share) if share > 0 else aff)
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"affinity_cores": aff, "threads": threads, "model": model}


def _median_s(fn, warmups=3, runs=10):
    """3 warm-up runs, then the median of >= 10 timed runs (seconds)."""
    for _ in range(warmups):
        fn()
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2], ts


def _cpu_model(ldm):
    return {k: v.detach().float().cpu().clone() for k, v in ldm.state_dict().items()}


def cpu_baseline(ldm, batch, times, eta):
    """Configs 2 / 5 on the host: one denoising iteration (UNet forward + DDIM update) of the same workload
    in the oracle's torch-CPU restatement of the reference loop (oracle/ldm_torch_cpu.py), fp32."""
    from oracle import ldm_torch_cpu as TC
    env = cpu_env()
    torch.set_num_threads(env["threads"])
    sd = _cpu_model(ldm)
    ab = TC.schedule(200)[2]
    g = torch.Generator().manual_seed(1)
    style = torch.rand(batch, 1, 128, 512, generator=g)
    torch.manual_seed(1234)
    x = torch.randn(batch, 32, 16, 64)
    with torch.no_grad():
        emb = TC.style_encoder(sd, style)
        s5, s6 = emb["s5"], emb["s6"]
        k = [0]

        def one():   # one iteration, walking the schedule like the loop does
            i = k[0] % (len(times) - 1)
            TC.reverse_loop(sd, ab, x, s5, s6, times[i:i + 2], eta)
            k[0] += 1
        med, ts = _median_s(one)
    return {"value": round(1.0 / med, 3), "unit": "steps/s", "cores": env["threads"], "kind": "port",
            "cpu_model": env["model"], "affinity_cores": env["affinity_cores"],
            "sample": f"median of {len(ts)} single DDIM iterations after 3 warm-ups (UNet forward + update, batch "
                      f"{batch}, [{batch},32,16,64] latents, eta={eta}, fp32), torch-CPU restatement "
                      f"oracle/ldm_torch_cpu.py; runs {min(ts):.3f}-{max(ts):.3f} s"}


def cpu_leg_forward(ldm):
    """Config 1 on the host: LDM.forward (encode -> q_sample -> UNet -> predict_start -> decode) + the
    diffusion / compression (MSE + KL) losses, batch 1, oracle/ldm_torch_cpu.py, fp32."""
    from oracle import ldm_torch_cpu as TC
    env = cpu_env()
    torch.set_num_threads(env["threads"])
    sd = _cpu_model(ldm)
    ab = TC.schedule(200)[2]
    g = torch.Generator().manual_seed(0)
    content = torch.rand(1, 1, 128, 512, generator=g)
    style = torch.rand(1, 1, 128, 512, generator=torch.Generator().manual_seed(1))
    t = torch.randint(0, 200, (1,), generator=torch.Generator().manual_seed(7))
    eps = torch.randn(1, 32, 16, 64, generator=torch.Generator().manual_seed(11))

    def one():
        with torch.no_grad():
            o = TC.ldm_forward(sd, content, style, t, eps, ab)
            loss = torch.mean((o["noise_pred"] - o["noise"]) ** 2) + torch.mean((o["reconstructed"] - content) ** 2) \
                + TC.kl_loss(o["z_0"])
        return float(loss)
    med, ts = _median_s(one)
    return {"value": round(1.0 / med, 3), "unit": "forward+loss/s", "cores": env["threads"], "kind": "port",
            "cpu_model": env["model"],
            "sample": f"config 1: median of {len(ts)} LDM.forward + loss at batch 1 after 3 warm-ups, "
                      f"oracle/ldm_torch_cpu.py; {med * 1e3:.1f} ms each"}


def cpu_leg_train(ldm, batch=8):
    """Config 3 on the host: the train step's arithmetic (frozen VAE encode, style encode, q_sample, UNet,
    decode, diffusion + compression losses, backward through the trained modules, Adam) in the oracle's
    torch-CPU restatement under autograd, fp32, on a small batch (samples/s scales ~linearly)."""
    from oracle import ldm_torch_cpu as TC
    env = cpu_env()
    torch.set_num_threads(env["threads"])
    sd = _cpu_model(ldm)
    trained = [k for k in sd if not k.startswith("encoder.") and sd[k].is_floating_point()
               and "running_" not in k and "num_batches" not in k]
    for k in trained:
        sd[k].requires_grad_(True)
    opt = torch.optim.Adam([sd[k] for k in trained], lr=1e-4)
    ab = TC.schedule(200)[2]
    g = torch.Generator().manual_seed(0)
    content = torch.rand(batch, 1, 128, 512, generator=g)
    style = torch.rand(batch, 1, 128, 512, generator=torch.Generator().manual_seed(1))
    t = torch.randint(0, 200, (batch,), generator=torch.Generator().manual_seed(7))
    eps = torch.randn(batch, 32, 16, 64, generator=torch.Generator().manual_seed(11))

    def one():
        opt.zero_grad()
        o = TC.ldm_forward(sd, content, style, t, eps, ab, train_decoder=True)
        loss = torch.mean((o["noise_pred"] - o["noise"]) ** 2) + torch.mean((o["reconstructed"] - content) ** 2) \
            + TC.kl_loss(o["z_0"])
        loss.backward()
        opt.step()
    med, ts = _median_s(one, warmups=3, runs=10)
    return {"value": round(batch / med, 3), "unit": "samples/s", "cores": env["threads"], "kind": "port",
            "cpu_model": env["model"],
            "sample": f"config 3: median of {len(ts)} train steps at batch {batch} after 3 warm-ups (fwd + bwd + "
                      f"Adam, fp32), oracle/ldm_torch_cpu.py under autograd; {med:.2f} s each"}


TRAIN_GFLOP_PER_SAMPLE = 10.7   # frozen VAE enc fwd 0.698 + 3 x (style enc 1.642 + UNet 0.449 + dec 1.242)


def run_train(args, world, rank, dev, M):
    """Configs 3/4: LDMTrainer.train_step (reference train.py:163-208) = VAE encode -> style encode ->
    q_sample -> UNet -> predict_start -> VAE decode -> losses -> backward -> (RCCL bucketed grad
    all-reduce when N>1) -> GradScaler + Adam, replayed from one hipGraph (LDMTrainer.graph_step; the RCCL
    all-reduces and SyncBN's statistic all-reduces are graph nodes when N > 1; --train-eager for the eager step).
    value = samples/s over all ranks; weak scaling (batch per GPU fixed)."""
    import torch.distributed as dist
    from models.train import LDMTrainer
    torch.manual_seed(0)
    ldm = M.LDM(32, pretrained_path="").to(dev)               # random-init weights of the architecture
    if world > 1:
        from ldm_amd import dist as hdist                      # same initial weights on every rank
        hdist.broadcast_parameters(ldm)
    trainer = LDMTrainer(ldm, None, dev, lr=1e-4)                 # LDMTrainer default (train.py:142)
    trainer.autocast_dtype = {"fp32": None, "fp16": torch.float16, "bf16": torch.bfloat16}[args.dtype]
    # the whole step replayed from a hipGraph (LDMTrainer.graph_step; warm-up covers the 2 eager steps and the
    # capture); with N > 1 the capture holds the bucketed RCCL gradient all-reduces and SyncBN's collectives
    trainer.graph_step = not args.train_eager
    if args.dtype == "fp32":
        os.environ["LDM_AMD_DTYPE"] = "fp32"                      # autocast region present, fp32 operands
    ldm.train()
    B = args.batch
    g = torch.Generator().manual_seed(11 + rank)
    content = torch.rand(B, 1, 128, 512, generator=g).to(dev)
    style = torch.rand(B, 1, 128, 512, generator=g).to(dev)
    torch.manual_seed(7 + rank)
    for _ in range(args.warmup):
        trainer.train_step(content, style)
    # the batch resident in the captured step's input buffers (filled in place once): a replay then copies
    # nothing into them (LDMTrainer.graph_inputs; the eager step reads content / style as given)
    gin = trainer.graph_inputs() if trainer.graph_step else None
    if gin is not None and gin[0] is not None and gin[1] is not None:
        gin[0].copy_(content)
        gin[1].copy_(style)
        content, style = gin[0], gin[1]
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
    peak = FP32_PEAK_TFLOPS if args.dtype == "fp32" else LOWP_PEAK_TFLOPS
    # HBM bytes per step from the newest committed PMC passes of this line (tools/pmc_train.sh: FETCH_SIZE x2 +
    # WRITE_SIZE summed over the step's dispatches), bf16 only (the passes profile the default line)
    traffic = None
    if args.dtype == "bf16" and world == 1:
        for rnd in ("r06", "r05", "r04", "r03"):
            pth = os.path.join(ROOT, "profiles", rnd, "train_pmc.json")
            if os.path.exists(pth):
                try:
                    with open(pth) as f:
                        traffic = json.load(f).get("step_hbm_bytes")
                    traffic = {"bytes_per_step": traffic, "source": f"profiles/{rnd}/train_pmc.json",
                               "achieved_gbs": round(traffic / (ms_step * 1e-3) / 1e9, 1)}
                except (OSError, ValueError, TypeError):
                    traffic = None
                break
    return {
        "metric": "LDM train samples/sec (encode -> UNet train step -> decode), 1/2/4/8 MI355X",
        "value": round(value, 2), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32" if args.dtype == "fp32" else f"{args.dtype} (conv / weight-gradient operands inside the autocast "
                                                     f"region; fp32 accumulation, BN, attention, optimizer)",
        "data": "synthetic (U[0,1) content/style mels; random-init weights; t ~ randint on device)",
        "config": {"workload": f"configs 3/4: LDMTrainer.train_step, batch {B}/GPU, 1x128x512 mels, "
                               f"torch.autocast({args.dtype}) region of train.py:174, Adam + GradScaler"
                               + (f", RCCL bucketed grad all-reduce over {world} ranks" if world > 1 else "")
                               + (", step replayed from one hipGraph (LDMTrainer.graph_step)"
                                  if trainer._graph is not None else ", eager step"),
                   "global_batch": B * world, "parallelism": f"dp{world}"},
        "roofline": {"kernel": "whole train step (composite)", "bound": "mfma", "achieved": round(achieved, 2),
                     "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                     "traffic": traffic, "flops_per_step": flops},
        "last_losses": {k: round(v, 6) for k, v in losses.items()},
    }


# SURVEY.md §8(d) shape S: UNet(1, 1) on [B,1,128,512], s5 [B,256,32,128], s6 [B,512,16,64] — per sample-step
# FLOPs by layer (2 * MACs; the convT layers over their input grid): enc1 / dec1 75.5 M each, enc2-4 and dec4-2
# 2.416 G each, CA2 (L = S = 4096 tokens, E = 256) 19.33 G of which the attention core is 4 E L S = 17.18 G, CA1
# (1024 tokens, E = 512) 4.29 G (core 2.15 G), bottleneck 4.83 G: 43.10 GFLOP
STRESS_GFLOP_PER_SAMPLE = 43.10


def run_stress(args, world, rank, dev, M):
    """Shape S: a DDIM reverse loop (args.timesteps - 1 UNet + update iterations, the
    reference's update of model.py:442-458) with the denoiser a UNet(1, 1) on the raw [B,1,128,512] mel and
    synthetic style maps s5 [B,256,32,128], s6 [B,512,16,64].  The UNet's latent width (1) is one the fused
    engine does not take, so every iteration is the per-layer path (NCHW conv kernels, the KV-tiled flash
    attention over 4096 / 1024 tokens) + the DDIM update kernel; the whole loop is one hipGraph."""
    from ldm_amd import ops
    from ldm_amd.graphs import capture
    B = args.batch
    torch.manual_seed(0)
    unet = M.UNet(1, 1, 64).to(dev).eval()                 # random-init weights of the architecture
    sched = M.ForwardDiffusion()
    g = torch.Generator().manual_seed(1 + rank)
    z_T = torch.randn((B, 1, 128, 512), generator=g).to(dev)
    s5 = torch.rand((B, 256, 32, 128), generator=g).to(dev)
    s6 = torch.rand((B, 512, 16, 64), generator=g).to(dev)
    emb = {"s5": s5, "s6": s6}
    times = torch.linspace(sched.num_timesteps - 1, 0, args.timesteps).long()
    n_iter = len(times) - 1
    coefs = sched.reverse_coefs(times).to(dev)
    coef_rows = [coefs[i].contiguous() for i in range(n_iter)]
    t_table = times[:-1].view(-1, 1).expand(-1, B).contiguous().to(dev)
    x = torch.empty_like(z_T)
    x0_logs = torch.empty((n_iter,) + tuple(z_T.shape), device=dev)
    eps_logs = torch.empty_like(x0_logs)

    def loop():
        x.copy_(z_T)
        for i in range(n_iter):
            eps = unet(x, t_table[i], emb)
            ops.ddim_step_(x, eps, coef_rows[i], float(args.eta), x0_logs[i], eps_logs[i])

    with torch.no_grad():
        loop()                                              # packs weights, plans, allocations: outside capture
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with capture(graph):
            loop()
        for _ in range(args.warmup):
            graph.replay()
        torch.cuda.synchronize()
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            graph.replay()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    if not torch.isfinite(x).all():
        raise SystemExit("non-finite sample")
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    us_iter = elapsed / (n_iter * args.steps) * 1e6
    flops_iter = STRESS_GFLOP_PER_SAMPLE * 1e9 * B
    t_roof = flops_iter / (FP32_PEAK_TFLOPS * 1e12)
    result = {
        "metric": METRIC, "value": round(n_iter * args.steps * world / elapsed, 2), "unit": "steps/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (N(0,1) z_T, U[0,1) style maps; random-init weights)",
        "config": {"workload": f"shape S (SURVEY §8(d), secondary): {args.timesteps}-step DDIM reverse sample ({n_iter} "
                               f"iterations per step) with UNet(1, 1) on the raw [{B},1,128,512] mel, s5 [{B},256,32,128], "
                               f"s6 [{B},512,16,64], eta={args.eta}, per-layer kernels + flash attention, hipGraph replay",
                   "global_batch": B * world, "latent": [B, 1, 128, 512], "parallelism": f"dp{world} (batch shards)"},
        "us_per_denoise_iteration": round(us_iter, 2),
        "step_roofline": {"t_roof_us": round(t_roof * 1e6, 2), "t_measured_us": round(us_iter, 2),
                          "frac": round(t_roof * 1e6 / us_iter, 4),
                          "achieved_tflops": round(flops_iter / (us_iter * 1e-6) / 1e12, 2)},
    }
    if rank == 0 and not args.no_kernel_timing:
        # the dominant kernel: CA2's attention core over 4096 x 4096 tokens (KV-tiled flash forward), timed as
        # the loop launches it (q [B,256,4096], kv [B,512,4096] of the projections), HIP events around a graph
        E, Lq = 256, 32 * 128
        q = torch.randn(B, E, Lq, device=dev)
        kv = torch.randn(B, 2 * E, Lq, device=dev)
        assert ops.attention_uses_flash(E, 4, Lq, Lq)
        us = _graph_time_us(lambda: ops.attention_core(q, kv, 4), 10)
        fl = 4.0 * B * E * Lq * Lq
        result["roofline"] = {"kernel": "fa::flash_fwd_kernel (CA2 attention core, L = S = 4096, E = 256)",
                              "bound": "mfma", "achieved": round(fl / us / 1e6, 2), "peak": FP32_PEAK_TFLOPS,
                              "unit": "TFLOP/s", "frac": round(fl / us / 1e6 / FP32_PEAK_TFLOPS, 4), "traffic": None,
                              "flops_per_launch": fl, "avg_launch_us": round(us, 3)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import ldm_torch_cpu as TC
        env = cpu_env()
        torch.set_num_threads(env["threads"])
        sd = {k: v.detach().float().cpu().clone() for k, v in unet.state_dict().items()}
        ab = TC.schedule(200)[2]
        xc = z_T.cpu().clone()
        s5c, s6c = s5.cpu(), s6.cpu()
        with torch.no_grad():
            med, ts = _median_s(lambda: TC.reverse_loop(sd, ab, xc, s5c, s6c, times[:2], args.eta, p=""),
                                warmups=1, runs=3)
        result["cpu_baseline"] = {"value": round(1.0 / med, 4), "unit": "steps/s", "cores": env["threads"],
                                  "kind": "port", "cpu_model": env["model"], "affinity_cores": env["affinity_cores"],
                                  "sample": f"median of {len(ts)} single DDIM iterations after 1 warm-up (UNet(1, 1) "
                                            f"forward at shape S + update, batch {B}, fp32), torch-CPU restatement "
                                            f"oracle/ldm_torch_cpu.py; runs {min(ts):.2f}-{max(ts):.2f} s"}
        result["gpu_over_cpu"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
    return result


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, cmd, env=None, poll_s=0.2, grace_s=30.0):
    """Start `cmd` as n worker processes, rank r with RANK = LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE = n,
    MASTER_ADDR = 127.0.0.1 and one free MASTER_PORT (an inherited MASTER_PORT is kept), every other variable
    inherited (HSA_ENABLE_IPC_MODE_LEGACY=0 among them).  The workers share this process's stdout / stderr (rank 0
    prints the JSON line).  Waits for all of them; when one fails, the others get SIGTERM after `grace_s` seconds
    (they are usually blocked in a collective with the dead rank) and SIGKILL if they ignore it.  Returns 0 or the
    exit code of the first rank that failed.  The workers stay in this process's process group (a `timeout` or
    job-control signal to the group reaches them too); this function signals only the PIDs it started, and a
    SIGTERM to this process is forwarded to them."""
    base = dict(os.environ if env is None else env)
    base["MASTER_ADDR"] = "127.0.0.1"
    base.setdefault("MASTER_PORT", str(_free_port()))
    base["WORLD_SIZE"] = base["LOCAL_WORLD_SIZE"] = str(n)
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
        procs.append(subprocess.Popen(cmd, env=e))
    first_bad, t_bad = 0, None

    def _forward(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
        raise SystemExit(128 + signum)
    old = signal.signal(signal.SIGTERM, _forward)
    try:
        while True:
            codes = [p.poll() for p in procs]
            for c in codes:
                if c not in (None, 0) and first_bad == 0:
                    first_bad, t_bad = c, time.monotonic()
            if all(c is not None for c in codes):
                break
            if t_bad is not None and time.monotonic() - t_bad > grace_s:
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
                t_bad = float("inf")
                deadline = time.monotonic() + 10.0
                while any(p.poll() is None for p in procs) and time.monotonic() < deadline:
                    time.sleep(poll_s)
                for p in procs:
                    if p.poll() is None:
                        p.kill()
            time.sleep(poll_s)
    finally:
        signal.signal(signal.SIGTERM, old)
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    if first_bad < 0:                       # killed by a signal: report it the way a shell does
        first_bad = 128 - first_bad
    return first_bad


def self_launch(n):
    """bench.py --gpus n > 1 without torchrun: n fresh ranks of this script, started before this process makes
    any GPU call (torch.cuda.device_count() does not initialise the runtime on this image)."""
    visible = torch.cuda.device_count()
    if visible < n:
        raise SystemExit(f"bench.py --gpus {n}: only {visible} HIP device(s) visible; one rank per GPU needs {n}")
    return launch_ranks(n, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:])


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(self_launch(args.gpus))
        if args.gpus < 1:
            raise SystemExit(f"--gpus {args.gpus}: need at least one GPU")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU, the two must agree")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    import models.model as M
    from ldm_amd.engine import GraphedDDIM

    if args.workload in ("train", "stress"):
        if args.workload == "stress":
            result = run_stress(args, world, rank, dev, M)
            if rank == 0:
                print(json.dumps(result), flush=True)
            if world > 1:
                dist.destroy_process_group()
            return
        result = run_train(args, world, rank, dev, M)
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            torch.manual_seed(0)
            result["cpu_baseline"] = cpu_leg_train(M.LDM(32, pretrained_path="").eval())
            result["gpu_over_cpu"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
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
        eng.dtype = args.dtype
        gd = GraphedDDIM(eng, z_T, emb["s5"], emb["s6"], t_table, coefs, args.eta, logs=True, split=args.split)
        # N > 1: every step ends with the sample all-gather of dist.sharded_style_sample (RCCL over xGMI),
        # so the timed region holds the job's only collective
        gathered = torch.empty((world,) + tuple(gd.x.shape), device=dev) if world > 1 else None

        def one_step():
            gd.replay()
            if gathered is not None:
                dist.all_gather_into_tensor(gathered, gd.x)
        for _ in range(args.warmup):
            one_step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            one_step()
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
        "vs_baseline": None,
        "dtype": "fp32" if args.dtype == "fp32" else f"{args.dtype} (conv operands; fp32 accumulation, epilogue, "
                                                     f"attention and sampler state)",
        "data": "synthetic (U[0,1) style mel, N(0,1) z_T; random-init weights)",
        "config": {"workload": (f"config 2: {args.timesteps}-step DDIM reverse sample ({n_iter} UNet+update "
                                f"iterations per step), batch {B}/GPU, 1x128x512 mel -> [{B},32,16,64] latents, "
                                f"eta={args.eta}, hipGraph replay of {args.split} concurrent sub-batch chains")
                   if args.workload == "sample" else
                   (f"config 5: content/style transfer loop, T'={args.timesteps} ({n_iter} UNet+update iterations "
                    f"per step, content encoded and q_sampled at T'-1 before timing), batch {B}/GPU, "
                    f"eta={args.eta}, {args.dtype} step-kernel operands with fp32 accumulators, hipGraph replay"),
                   "global_batch": B * world,
                   "latent": [B, 32, 16, 64],
                   "parallelism": f"dp{world} (batch shards" + (", all-gather of the samples every step)" if world > 1
                                                                 else ")")},
        "us_per_denoise_iteration": round(us_iter, 2),
    }
    # whole-step composite roofline
    flops_iter = UNET_GFLOP_PER_SAMPLE * 1e9 * B
    bytes_iter = 27.37e6 + B * (2.52e6 + 0.655e6)
    peak_c = FP32_PEAK_TFLOPS if args.dtype == "fp32" else LOWP_PEAK_TFLOPS
    t_roof = max(flops_iter / (peak_c * 1e12), bytes_iter / (HBM_PEAK_GBS * 1e9))
    result["step_roofline"] = {"t_roof_us": round(t_roof * 1e6, 2), "t_measured_us": round(us_iter, 2),
                               "frac": round(t_roof * 1e6 / us_iter, 4),
                               "achieved_tflops": round(flops_iter / (us_iter * 1e-6) / 1e12, 2)}

    if rank == 0 and not args.no_kernel_timing:
        with torch.no_grad():
            kt = time_step_layers(eng, B, 16, 64, dev)
        dom = max(kt, key=lambda k: kt[k]["us"])      # the longest launch of the step
        dk = kt[dom]
        traffic = None
        pmc_file = args.pmc if args.dtype == "fp32" else (args.pmc_lowp if args.dtype == "fp16" else None)
        if pmc_file and os.path.exists(pmc_file):   # (bf16 step kernels: no PMC pass recorded)
            try:
                with open(pmc_file) as f:
                    pmc = json.load(f)
                traffic = pmc.get("per_launch_bytes", {}).get(dom)
            except (OSError, ValueError):
                traffic = None
        peak = FP32_PEAK_TFLOPS if args.dtype == "fp32" else LOWP_PEAK_TFLOPS
        if dk.get("bound") == "hbm":   # a byte-bound launch (the folded-value bottleneck, the attentions)
            result["roofline"] = {"kernel": f"{dk['kernel']} ({dom})", "bound": "hbm",
                                  "achieved": dk["gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(dk["gbs"] / HBM_PEAK_GBS, 4), "traffic": traffic,
                                  "bytes_per_launch": dk["bytes"], "avg_launch_us": dk["us"]}
        else:
            result["roofline"] = {"kernel": f"{dk['kernel']} ({dom})", "bound": "mfma",
                                  "achieved": dk["tflops"], "peak": peak, "unit": "TFLOP/s",
                                  "frac": round(dk["tflops"] / peak, 4), "traffic": traffic,
                                  "flops_per_launch": dk["flops"], "avg_launch_us": dk["us"]}
        result["kernels"] = {k: {kk: vv for kk, vv in v.items() if kk not in ("flops", "bytes")} for k, v in kt.items()}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(ldm, B, times, args.eta)
        result["gpu_over_cpu"] = round(value / result["cpu_baseline"]["value"], 1)
        if args.workload == "sample" and not args.no_cpu_legs:
            result["cpu_legs"] = {"config1": cpu_leg_forward(ldm), "config3": cpu_leg_train(ldm)}

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
