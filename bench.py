"""Benchmark: CRNN training step (SE-ResNet31 -> 2x512 BiLSTM -> CTC head, fwd + CTC bwd +
AdamW) in bf16 at B=256 per GPU on 32x256 synthetic crops — BASELINE.json configs[2]
(1 GPU) / configs[3] (data parallel, RCCL all-reduce of gradients).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU)

`python bench.py --gpus N` (N > 1) with no launcher env starts the N ranks itself (a torch.distributed.run
child, before any GPU call in this process). A run whose rank count differs from --gpus exits non-zero.
Rank 0 prints ONE JSON line (metric/value/...); value = lines/s over all ranks.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for sub in ("rcnn-ocr_amd", "oracle"):
    p = os.path.join(REPO, sub)
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "text-lines/sec (train step incl. CTC bwd) at B=256, 32×256 crops; 1/2/4/8 MI355X"
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (spec, MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0       # HBM3E spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--height", type=int, default=32)
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sub", action="store_true",
                    help="default train line only: skip the configs[1] inference and configs[4] long-line "
                         "sub-measurements that a 1-GPU run attaches as sub_measurements")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="batch of the CPU baseline sample (default: the bench batch, B=256, as BASELINE.md)")
    ap.add_argument("--cpu-steps", type=int, default=1, help="timed CPU steps (after one warm-up at B=32)")
    ap.add_argument("--path", default="api", choices=["api", "engine"],
                    help="train mode: api = the reference user's path (RCNN forward -> crnn_hip.ctc_loss -> "
                         "loss.backward() -> optimizer.step(), model/model.py:223-227, training/train.py:493-518); "
                         "engine = CRNNEngine forward / ctc / backward called directly (A/B of the API overhead)")
    ap.add_argument("--mode", default="train", choices=["train", "infer", "attn", "attn_train", "preprocess"],
                    help="train: BASELINE configs[2]/[3] (the headline); infer: configs[1] (eval forward + greedy "
                         "CTC decode on device); attn: eval encode + the reference's attention head, 26-step greedy "
                         "decode (SURVEY 8f next-1); attn_train: the reference's own training step (encoder + "
                         "teacher-forced attention decoder, 26 steps, cross-entropy, backward, AdamW); preprocess: "
                         "the input pipeline (ResizeAndPadA + Normalize of ragged uint8 crops into the encoder "
                         "layout, SURVEY 8f next-2)")
    ap.add_argument("--kernel-timing", default="last", choices=["all", "last", "off"],
                    help="HIP events around every conv / BiLSTM launch (the roofline's per-launch durations) in "
                         "all timed steps, only the last timed step (default: the ~170 event records of an "
                         "instrumented step cost 0.5 ms of GPU time, profiles/r02s_infer_fuse_and_timing_ab.log), "
                         "or none")
    ap.add_argument("--config", default=None, choices=["long"],
                    help="long: BASELINE configs[4] shapes (32x1024 crops, 4x768 BiLSTM, batch 64/GPU)")
    a = ap.parse_args()
    if a.config == "long":
        a.width, a.hidden, a.layers, a.batch = 1024, 768, 4, 64
    return a


def usable_cpus():
    """host cores this process may use: the affinity mask, capped by a cgroup CPU quota (on the GPU
    box os.cpu_count() reports the whole machine, while the job gets a share of it)"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(args, threads, shapes, attn_params=None):
    """oracle (CPU fp32 restatement, 'port') train step / inference on a bounded sample: the bench's
    own batch (B=256 by default) after one B=32 warm-up step; the CTC loss is torch's
    F.ctc_loss (CPU) as the reference path would call it."""
    import crnn_oracle as O
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    torch.set_num_threads(threads)
    C = 194
    T = args.width // 8
    B = args.cpu_sample or args.batch
    sd = recipe_state_dict(shapes, 0)
    p = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v)
         for k, v in sd.items()}
    ap = None
    if attn_params is not None:
        ap = {k: v.clone().requires_grad_(args.mode == "attn_train") for k, v in attn_params.items()}
    params = [v for v in p.values() if getattr(v, "requires_grad", False)]
    params += [v for v in (ap or {}).values() if v.requires_grad]
    opt = torch.optim.AdamW(params, lr=1e-4)

    def ctc(logits, tg, tl):
        lp = torch.nn.functional.log_softmax(logits, -1).permute(1, 0, 2)
        il = torch.full((logits.shape[0],), logits.shape[1], dtype=torch.long)
        return torch.nn.functional.ctc_loss(lp, tg, il, tl, blank=0, reduction="mean", zero_infinity=True)

    def step(x, tg, tl, text, ty):
        if args.mode == "attn":
            with torch.no_grad():
                O.attn_greedy(attn_params, O.encode(x, p, O.Ctx(train=False), args.layers), 26, 1, 3, C)
            return
        if args.mode == "attn_train":
            opt.zero_grad(set_to_none=True)
            lg = O.attn_teacher(ap, O.encode(x, p, O.Ctx(train=True), args.layers), text, 26, 3, C)
            torch.nn.functional.cross_entropy(lg.reshape(-1, C), ty.reshape(-1), ignore_index=0).backward()
            opt.step()
            return
        if args.mode == "infer":
            with torch.no_grad():
                O.head(O.encode(x, p, O.Ctx(train=False), args.layers), p).argmax(-1)
            return
        opt.zero_grad(set_to_none=True)
        logits = O.head(O.encode(x, p, O.Ctx(train=True), args.layers), p)
        ctc(logits, tg, tl).backward()
        opt.step()

    def batch(n, seed):
        x, _, tg, tl = synthetic_batch(n, args.height, args.width, T, C, seed=seed)
        return (x, tg, tl) + attn_text(tg, tl, n)

    step(*batch(min(32, B), 98))  # warm-up
    data = batch(B, 99)
    t0 = time.perf_counter()
    for _ in range(args.cpu_steps):
        step(*data)
    dt = time.perf_counter() - t0
    what = ("train step (fwd + teacher-forced attention decode + CE + bwd + AdamW)" if args.mode == "attn_train"
            else "eval encode + 26-step greedy attention decode" if args.mode == "attn"
            else "eval forward + argmax" if args.mode == "infer"
            else "train step (fwd + F.ctc_loss + bwd + AdamW)")
    return {"value": round(B * args.cpu_steps / dt, 3), "unit": "text-lines/s", "cores": threads,
            "cpu_model": cpu_model(), "kind": "port",
            "sample": f"oracle/crnn_oracle.py fp32 torch-CPU {what}, B={B} x {args.cpu_steps} timed step(s) "
                      f"(+1 warm-up step at B={min(32, B)}) at {args.height}x{args.width}, hidden {args.hidden}, "
                      f"{args.layers} BiLSTM layers; {dt:.1f} s; torch.set_num_threads({threads}) = the cores "
                      f"this process may use (os.cpu_count() = {os.cpu_count()} on this host)"}


def attn_text(tg, tl, B, steps=26, sos=1, eos=2):
    """teacher-forcing inputs / targets from the synthetic labels, as the reference packs them
    (data/transforms.py:123-157): text_in = [SOS, y[:L], PAD...], target_y = [y[:L], EOS, PAD...],
    L = min(len, steps - 1); label ids (synthetic_batch: [B, Lmax] zero-padded) are moved past the
    reserved ids (PAD 0, SOS 1, EOS 2, blank 3)."""
    text = torch.zeros(B, steps, dtype=torch.long)
    ty = torch.zeros(B, steps, dtype=torch.long)
    for b in range(B):
        n = min(int(tl[b]), steps - 1)
        y = ((tg[b, :n].long() - 3) % 190) + 4
        text[b, 0] = sos
        text[b, 1:n + 1] = y
        ty[b, :n] = y
        ty[b, n] = eos
    return text, ty


def pmc_traffic():
    """the committed PMC summary (tools/gpu_pmc.sh + tools/pmc_traffic.py -> profiles/*_pmc_traffic.json)
    taken on THIS source tree: measured HBM bytes per launch of the hot kernels. A summary whose
    source_hash differs from the running tree's (crnn_hip._lib.source_hash) is stale and not used:
    -> (None, reason)."""
    import glob
    from crnn_hip._lib import source_hash
    want = source_hash()
    fs = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")))
    for f in reversed(fs):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("source_hash") == want:
            return d, os.path.relpath(f, REPO)
    return None, f"no profiles/*_pmc_traffic.json taken on this tree (source_hash {want})"


def lstm_roofline(lstm, args, eng, tsteps):
    """HBM roofline of the BiLSTM recurrence (north star: >= 40% on the step at B=256): algorithmic
    bytes per step (CRNNEngine.lstm_step_bytes) x steps / measured sweep time."""
    out = {}
    for k, (n, ms, byt) in lstm.items():
        gbs = byt / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        out[k] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                  "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": None,
                  "sweeps_per_step": n // tsteps, "us_per_sweep": round(ms / n * 1e3, 2),
                  "us_per_timestep": round(ms / n / (args.width // 8) * 1e3, 3),
                  "algorithmic_bytes_per_timestep": byt / n / (args.width // 8)}
    seq = eng._seq_ok(args.batch)
    out["kernel"] = ("persistent whole-sequence BiLSTM (lstm_seq.hip)" if seq else "per-step BiLSTM launches (lstm.hip)")
    pmc, src = pmc_traffic()
    if pmc and seq and args.mode == "train" and args.batch == 256 and args.hidden == 512:   # the PMC pass's config
        for k in ("lstm_fwd", "lstm_bwd"):
            if k in out and k in pmc:
                out[k]["traffic"] = pmc[k]["hbm_bytes_per_launch"]
                out[k]["traffic_note"] = f"HBM bytes per sweep launch, {src}"
    return out


def synthetic_crops(n, seed):
    """ragged uint8 RGB text-line crops: height U{24..96}, aspect U[2, 16] (wider ones are fit by
    width), random pixels — the shapes ResizeAndPadA sees on real datasets."""
    import numpy as np
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        h = int(rng.integers(24, 97))
        w = max(1, int(h * rng.uniform(2.0, 16.0)))
        out.append(rng.integers(0, 256, (h, w, 3), dtype=np.uint8))
    return out


def bench_preprocess(args, world, rank, dev):
    """crnn_preprocess over a device-resident ragged batch -> encoder input."""
    from crnn_hip.preprocess import CropBatch, preprocess
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    crops = synthetic_crops(args.batch, 4321 + rank)
    batch = CropBatch.upload(crops, dev)
    H, W = args.height, args.width

    def step():
        return preprocess(batch, H, W, out="encoder", dtype=dtype)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for e0, e1 in ev:
        e0.record()
        step()
        e1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    src_bytes = int(batch.data.numel())
    out_bytes = args.batch * H * W * 8 * (2 if dtype == torch.bfloat16 else 4)
    algo = src_bytes + out_bytes
    gbs = algo / (kern_ms * 1e-3) / 1e9
    if rank == 0:
        out = {
            "metric": f"text-lines/sec (input pipeline: ResizeAndPadA + Normalize of ragged uint8 crops into the "
                      f"encoder layout), B={args.batch}, {H}x{W} canvas, 1 MI355X",
            "value": round(args.batch * world * args.steps / elapsed, 1), "unit": "text-lines/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic ragged uint8 RGB crops (height U{24..96}, aspect U[2,16]), device-resident",
            "config": {"workload": f"crnn_preprocess -> [B,{H},{W},8] {args.dtype} (SURVEY 8f next-2)",
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch, "canvas": f"{H}x{W}",
                       "parallelism": f"dp{world}" if world > 1 else "single"},
            "roofline": {"bound": "hbm", "kernel": "preprocess_kernel", "achieved": round(gbs, 1),
                         "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": None,
                         "algorithmic_bytes_per_launch": algo, "src_bytes": src_bytes, "out_bytes": out_bytes,
                         "kernel_us": round(kern_ms * 1e3, 2),
                         "timing": "HIP events around each launch on the launch stream, timed region"},
        }
        if world == 1 and not args.no_cpu_baseline:
            import preprocess_oracle as P
            sample = crops[: max(1, (args.cpu_sample or 32) // 4)]
            t1 = time.perf_counter()
            for im in sample:
                P.preprocess(im, H, W)
            dt = time.perf_counter() - t1
            out["cpu_baseline"] = {"value": round(len(sample) / dt, 3), "unit": "text-lines/s", "cores": 1,
                                   "kind": "port", "sample": f"oracle/preprocess_oracle.py (numpy, scalar loops) on "
                                                             f"{len(sample)} of the crops; {dt:.1f} s"}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """`python bench.py --gpus N` without a launcher: start N fresh ranks (one process per GPU) under
    torch.distributed.run as a CHILD process and return its exit code. This process has not touched the
    GPU (no HIP call before this point), and it never execs: it only waits and relays (rank 0 prints the
    JSON line straight to the inherited stdout)."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["CRNN_BENCH_SPAWNED"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    from crnn_hip import dist as D
    world = D.env_world()[0]
    if world != args.gpus:   # never report an N-GPU line measured on another rank count
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s) (WORLD_SIZE); refusing to "
                 f"report a line whose n_gpus differs from --gpus")
    world, rank, local = D.init_from_env()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if args.mode == "preprocess":
        return bench_preprocess(args, world, rank, dev)
    out = measure(args, world, rank, dev)
    if rank == 0 and world == 1 and args.mode == "train" and args.config is None and not args.no_sub:
        # BASELINE configs[1] (inference) and configs[4] (long lines) as sub-measurements of the default line,
        # so that the driver's own run observes them; each with its own rooflines and a
        # bounded CPU-oracle sample
        import copy
        subs = {}
        for key, mode, cfg, steps, cpu_b in (("configs1_infer", "infer", None, 20, 256),
                                              ("configs4_long", "train", "long", 10, 8)):
            a = copy.copy(args)
            a.mode, a.config, a.steps, a.warmup, a.cpu_sample = mode, cfg, steps, 3, cpu_b
            if cfg == "long":
                a.width, a.hidden, a.layers, a.batch = 1024, 768, 4, 64
            t0 = time.perf_counter()
            r = measure(a, world, rank, dev)
            r["wall_s"] = round(time.perf_counter() - t0, 1)
            subs[key] = {k: r[k] for k in ("metric", "value", "unit", "ms_per_step", "steps", "warmup", "dtype",
                                           "config", "roofline", "roofline_lstm", "cpu_baseline", "wall_s")
                         if k in r}
            torch.cuda.empty_cache()
        out["sub_measurements"] = subs
    if world > 1 and args.mode == "train" and args.config is None and not args.no_sub:
        # BASELINE configs[4] in its own multi-GPU form (32x1024 crops, 4x768 BiLSTM, batch 64 per GPU, DP over the
        # same ranks) as a sub-measurement of the N-rank line, so that the driver's scaling runs observe it. Every
        # rank takes part (the timed region is collective); rank 0 attaches the result
        import copy
        a = copy.copy(args)
        a.mode, a.config, a.steps, a.warmup = "train", "long", min(args.steps, 10), min(args.warmup, 3)
        a.width, a.hidden, a.layers, a.batch = 1024, 768, 4, 64
        torch.cuda.empty_cache()
        t0 = time.perf_counter()
        r = measure(a, world, rank, dev)
        if rank == 0:
            r["wall_s"] = round(time.perf_counter() - t0, 1)
            out["sub_measurements"] = {"configs4_long_dp": {k: r[k] for k in (
                "metric", "value", "unit", "n_gpus", "ms_per_step", "steps", "warmup", "dtype", "config", "roofline",
                "roofline_lstm", "dp", "wall_s") if k in r}}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def measure(args, world, rank, dev):
    """build the model for args, time args.steps steps after args.warmup (barrier + synchronize around the
    timed region, max over ranks) -> the bench line's dict on rank 0 (None on the other ranks)"""
    from crnn_hip import dist as D
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.optim import FusedAdamW
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN

    C = 194
    T = args.width // 8
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    attn = args.mode in ("attn", "attn_train")
    model = RCNN(num_classes=C, hidden_size=args.hidden, blank_id=3 if attn else None, num_rnn_layers=args.layers,
                 compute_dtype=dtype, decoder="attn" if attn else "ctc")
    shapes = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]   # the model's own parameter table
    model.load_state_dict(recipe_state_dict(shapes, 0), strict=False)
    model = model.to(dev).train(args.mode in ("train", "attn_train"))
    x, _, tg, tl = synthetic_batch(args.batch, args.height, args.width, T, C, seed=1234 + rank)
    x = x.to(dev)
    tg = tg.to(dev, torch.int32)
    tl = tl.to(dev, torch.int32)
    eng = model._engine_for(x)
    model.flatten_parameters_()
    if world > 1:
        D.broadcast_params(model._flat_param)
        model.mark_params_changed()
    grads, _, _ = model._grad_views()
    opt = FusedAdamW(model, lr=1e-4, weight_decay=1e-2)
    inv_world = 1.0 / world
    # DP: bucketed RCCL all-reduce of the flat gradient, issued stage by stage during the backward
    # (head / BiLSTM first, stem last) so it overlaps the remaining backward kernels
    reducer = D.OverlappedAllReduce(model._flat_grad, model.flat_offsets(), timing=True) if world > 1 else None
    model.stage_done = reducer.ready if reducer is not None else None   # the API path's backward hook

    ids = torch.empty(args.batch, T, dtype=torch.int32, device=dev)
    lens = torch.empty(args.batch, dtype=torch.int32, device=dev)
    from crnn_hip._lib import call, stream_ptr
    # A/B switches (include/crnn_hip.h CRNN_OPT_*): CRNN_OPTS="key=value,key=value"
    opts = {int(k): int(v) for k, v in (kv.split("=") for kv in os.environ.get("CRNN_OPTS", "").split(",") if kv)}
    for k, v in opts.items():
        call("crnn_set_option", k, v)

    def infer_step():
        eng.forward(x, train=False, save_for_backward=False)
        lg = eng.logits_padded()
        call("crnn_ctc_greedy", lg.data_ptr(), lg.shape[-1], args.batch, T, C, ids.data_ptr(), lens.data_ptr(),
             stream_ptr())
        return lens

    def attn_step():
        with torch.no_grad():
            return model(x, is_train=False, batch_max_length=25)

    from crnn_hip.attn import cross_entropy
    text_in, target_y = attn_text(tg.cpu(), tl.cpu(), args.batch)
    text_in, target_y = text_in.to(dev), target_y.to(dev)

    def attn_train_step():
        opt.zero_grad(set_to_none=True)
        logits = model(x, text=text_in, is_train=True, batch_max_length=25)
        loss = cross_entropy(logits, target_y, ignore_index=0)
        loss.backward()
        opt.step(grad_scale=inv_world)
        return loss

    def step():
        if args.mode == "attn":
            return attn_step()
        if args.mode == "attn_train":
            if world > 1:
                raise NotImplementedError("attn_train is a 1-GPU bench line")
            return attn_train_step()
        if args.mode == "infer":
            return infer_step()
        if args.path == "api":   # the reference user's step (training/train.py:493-518) on the drop-in API
            opt.zero_grad(set_to_none=True)
            loss = ctc_loss(model(x), tg, tl)
            loss.backward()
            if reducer is not None:
                reducer.finish()
            opt.step(grad_scale=inv_world)
            return loss
        eng.forward(x, train=True, save_for_backward=True, dropout_p=model.enc_dropout.p)
        loss, dl = eng.ctc(eng.logits_padded(), tg, tl)
        eng.backward(dl, grads, accumulate=False, stage_done=reducer.ready if reducer else None)
        if reducer is not None:
            reducer.finish()
        opt.step(grad_scale=inv_world)
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if reducer is not None:
        reducer.wait_events.clear()   # the exposed-wait events of the timed steps only
    eng.enable_timing(args.kernel_timing == "all")
    # the BiLSTM sweeps' kernel-only events in every timed step (4 event pairs per step): their per-sweep
    # mean is the one a profiler averages, where the last step alone varies with the sweep's placement
    eng.enable_lstm_timing(args.kernel_timing != "off")
    t0 = time.perf_counter()
    for i in range(args.steps):
        if args.kernel_timing == "last" and i == args.steps - 1:
            eng.enable_timing(True)
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timing = eng.conv_timing()
    tsteps = {"all": args.steps, "last": 1, "off": 1}[args.kernel_timing]   # steps the conv events covered
    lsteps = args.steps if args.kernel_timing != "off" else 1                # ... and the BiLSTM events
    eng.enable_timing(False)
    eng.enable_lstm_timing(False)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    divergence = None
    if world > 1:   # replicas must hold identical weights after the timed steps (same reduced grads)
        c = model._flat_param.double().sum().reshape(1)
        cmax, cmin = c.clone(), c.clone()
        dist.all_reduce(cmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(cmin, op=dist.ReduceOp.MIN)
        divergence = float((cmax - cmin).item())
    dp_overlap = None
    if reducer is not None:   # per-step exposed all-reduce wait of the compute stream, max over ranks
        ex = torch.tensor([reducer.exposed_ms_per_step()], dtype=torch.float64, device=dev)
        dist.all_reduce(ex, op=dist.ReduceOp.MAX)
        nb, nbytes = reducer.buckets_per_step()
        dp_overlap = {"exposed_allreduce_ms_per_step_max_rank": round(float(ex.item()), 4),
                      "buckets_per_step": nb, "allreduce_bytes_per_step": nbytes,
                      "bucket_mb": [round(b / 2 ** 20, 2) for b in reducer.last_bucket_bytes()],
                      "exposed_note": "HIP events on the compute stream around finish()'s wait for the collective "
                                      "stream (the all-reduce time NOT hidden under the backward), mean over the "
                                      "timed steps"}
    lines = args.batch * world * args.steps
    value = lines / elapsed
    final_loss = float(loss.float().mean().item()) if args.mode in ("train", "attn_train") else 0.0

    if rank == 0:
        lstm = {k: timing.pop(k) for k in ("lstm_fwd", "lstm_bwd") if k in timing}
        conv_launches = sum(v[0] for v in timing.values())
        conv_ms = sum(v[1] for v in timing.values())
        conv_flop = sum(v[2] for v in timing.values())
        achieved = conv_flop / (conv_ms * 1e-3) / 1e12 if conv_ms > 0 else 0.0
        pmc, src = pmc_traffic()
        conv_traffic = conv_mfma_busy = None
        conv_traffic_note = None if pmc else src
        if pmc and "conv" in pmc and args.mode == "train" and args.batch == 256 and args.width == 256 \
                and dtype == torch.bfloat16:
            conv_traffic = pmc["conv"]["hbm_bytes_per_launch"]
            conv_mfma_busy = pmc["conv"].get("mfma_busy_frac")
            conv_traffic_note = (f"measured HBM bytes per conv launch (mean over fwd/dgrad/wgrad launches, "
                                 f"2*FETCH_SIZE + WRITE_SIZE), {src}; algorithmic per-launch FLOPs above")
        per_kind = {k: {"launches_per_step": v[0] // tsteps, "ms_per_step": round(v[1] / tsteps, 3),
                        "tflops": round(v[2] / (v[1] * 1e-3) / 1e12, 1) if v[1] > 0 else None}
                    for k, v in timing.items()}
        out = {
            "metric": (METRIC if args.mode == "train" and args.config is None else
                       "text-lines/sec (train step incl. CTC bwd), long lines: B=64/GPU, 32x1024 crops, 4x768 BiLSTM"
                       if args.mode == "train" else
                       "text-lines/sec (inference: eval forward + greedy CTC decode), B=256, 32x256 crops, 1 MI355X"
                       if args.mode == "infer" else
                       "text-lines/sec (inference with the attention head: eval encode + 26-step greedy attention "
                       "decode), B=256, 32x256 crops, 1 MI355X" if args.mode == "attn" else
                       "text-lines/sec (the reference's attention training step: encoder + 26-step teacher-forced "
                       "attention decoder + cross-entropy, bwd, AdamW), B=256, 32x256 crops, 1 MI355X"),
            "value": round(value, 2),
            "unit": "text-lines/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
            "data": "synthetic (seeded 32xW uint8 crops with white padding, random labels; recipe-init weights)",
            "config": {"workload": (f"train step: SE-ResNet31 + {args.layers}x{args.hidden} BiLSTM + CTC head, fwd + "
                                    f"CTC bwd + AdamW (BASELINE " + ("configs[4])" if args.config == "long" else
                                                                    "configs[2]/[3])")
                                    if args.mode == "train" else
                                    f"inference: SE-ResNet31 + {args.layers}x{args.hidden} BiLSTM + CTC head, eval "
                                    f"forward + on-device greedy decode (BASELINE configs[1])"
                                    if args.mode == "infer" else
                                    f"inference: SE-ResNet31 + {args.layers}x{args.hidden} BiLSTM encode + the "
                                    f"reference's attention decoder (fp32), 26 greedy steps (SURVEY 8f next-1)"
                                    if args.mode == "attn" else
                                    f"train step: SE-ResNet31 + {args.layers}x{args.hidden} BiLSTM encoder ({args.dtype}) "
                                    f"+ the reference's attention decoder (fp32), 26 teacher-forced steps, "
                                    f"cross-entropy (ignore PAD), fwd + bwd + AdamW (SURVEY 8f next-1)"),
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                       "crop": f"{args.height}x{args.width}", "seq_len": T, "hidden": args.hidden,
                       "rnn_layers": args.layers, "num_classes": C,
                       **({"path": ("RCNN API: model(x) -> crnn_hip.ctc_loss -> loss.backward() -> "
                                    "FusedAdamW.step()" if args.path == "api" else
                                    "CRNNEngine forward / ctc / backward called directly")}
                          if args.mode == "train" else {}),
                       "parallelism": f"dp{world}" if world > 1 else "single"},
            "roofline": {"bound": "mfma", "kernel": "implicit-GEMM conv (fwd+dgrad+wgrad, all 28 convs)",
                         "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": conv_traffic,
                         "traffic_note": conv_traffic_note, "mfma_busy_frac_pmc": conv_mfma_busy,
                         "algorithmic_flop_per_step": conv_flop / tsteps,
                         "launches_per_step": conv_launches // tsteps,
                         "kernel_ms_per_step": round(conv_ms / tsteps, 3),
                         "timing": ("HIP events around every conv launch on the launch stream, "
                                    + {"all": "every timed step", "last": "the last timed step",
                                       "off": "off (no figures)"}[args.kernel_timing])},
            "kernels": per_kind,
            "roofline_lstm": lstm_roofline(lstm, args, eng, lsteps),
            "final_loss": round(final_loss, 4),
            **({"options": opts} if opts else {}),
            "dp": ({"allreduce": ("RCCL" if dist.get_backend() == "nccl" else dist.get_backend())
                    + " sum of the flat fp32 gradient, bucketed and overlapped with the backward",
                    "param_checksum_spread": divergence, **(dp_overlap or {})} if world > 1 else None),
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                threads = usable_cpus()
                ap_cpu = ({k[5:]: v.detach().float().cpu() for k, v in model.state_dict().items()
                           if k.startswith("attn.")} if attn else None)
                out["cpu_baseline"] = cpu_baseline(args, threads, shapes, ap_cpu)
            except Exception as e:  # report, never fake
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        return out
    return None


if __name__ == "__main__":
    main()
