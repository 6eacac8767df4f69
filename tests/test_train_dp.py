"""run_training with world_size 2 (SURVEY §5 "Config" world_size, §8e): two
processes on the box's one GPU (gloo over device tensors, per-step BiLSTM launches: the persistent
sweeps need the whole chip), launched the way torchrun would (RANK / WORLD_SIZE / MASTER_* in the
env). With CRNN_SHARE_DEVICE=1 every rank uses device 0; the two ranks compute concurrently (r05: no
turn-taking) and the overlapped all-reduce runs as in deployment. Checked against a single-process
emulation of the same job: the same batches dealt to the two "ranks", each step's two shard gradients
accumulated in one process and applied as their mean. BN keeps per-shard batch statistics in both, so
the emulation is the DP step's definition: measured |dp - emulation| / |update| = 1.5e-10 after two
epochs (profiles/r04o_dp.log). The emulation also keeps one copy of the BN running statistics per rank and
averages them at each epoch end, as sync_bn_stats does; rank 0's checkpoint must hold that average. Reference: training/train.py:179-235, :493-518.

Both sides run the conv weight gradients with fp32 split-K slabs (CRNN_OPT_WGRAD_SLAB_BF16 = 0): the default
bf16 slabs round each partial once, which turns the all-reduce's last-ulp differences from the emulation's
in-place accumulation (the 1.5e-10 above) into bf16-ulp jumps of whole partials, measured 2.8e-4 after two
epochs (r06f6). The bf16-slab kernel itself is pinned by tests/test_gpu_kernels.py (one-rounding bound,
accumulate mode)."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from helpers import GOLDEN

LINES = os.path.join(GOLDEN, "lines")
CHARSET = os.path.join(GOLDEN, "charset.txt")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg_dict(exp_dir, **kw):
    c = {"train_csvs": [os.path.join(LINES, "a", "labels.csv"), os.path.join(LINES, "b", "train", "labels.csv")],
         "train_roots": [os.path.join(LINES, "a"), os.path.join(LINES, "b", "train")],
         "val_csvs": [None, os.path.join(LINES, "b", "val", "labels.csv")],
         "val_roots": [None, os.path.join(LINES, "b", "val")],
         "charset_path": CHARSET, "img_h": 32, "img_w": 128, "max_len": 16, "hidden_size": 64, "batch_size": 8,
         "epochs": 2, "lr": 0.05, "optimizer": "SGD", "momentum": 0.9, "scheduler": "None",
         "weight_decay": 0.0, "val_size": 8, "seed": 7, "eval_every": 1, "exp_dir": exp_dir, "enc_dropout_p": 0.0}
    c.update(kw)
    return c


def _worker(rank, world, port, cfg_path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), CRNN_SHARE_DEVICE="1", CRNN_LSTM_PER_STEP="1",
                      CRNN_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for sub in ("../rcnn-ocr_amd", "../oracle"):
        sys.path.insert(0, os.path.join(here, sub))
    try:
        from crnn_hip import _lib as L
        L.call("crnn_set_option", L.OPT_WGRAD_SLAB_BF16, 0)
        from training.train import Config, run_training
        out = run_training(Config(cfg_path), device="cuda")
        q.put((rank, out, None))
    except Exception:
        import traceback
        q.put((rank, None, traceback.format_exc()))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def _emulate(cfg, world):
    """the DP job in one process: the same model init, splits and batch dealing as run_training; per
    step the `world` shards' gradients accumulate, then the optimizer applies their mean"""
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.optim import make_optimizer
    from data.dataset import batches
    from data.transforms import ctc_targets, load_charset, preprocess_batch
    from model.model import RCNN
    from training.train import build_splits
    from training.utils import set_seed
    set_seed(cfg.seed)
    dev = torch.device("cuda", 0)
    itos, stoi = load_charset(cfg.charset_path)
    model = RCNN(num_classes=len(itos), hidden_size=cfg.hidden_size, sos_id=stoi["<SOS>"], eos_id=stoi["<EOS>"],
                 pad_id=stoi["<PAD>"], blank_id=None, enc_dropout_p=0.0, compute_dtype=torch.bfloat16).to(dev)
    model.flatten_parameters_()
    p0 = model._flat_param.detach().clone()
    opt = make_optimizer(cfg.optimizer, model, cfg.lr, cfg.weight_decay, cfg.momentum)
    train_sets, _ = build_splits(cfg, stoi, cfg.img_h, cfg.img_w, cfg.max_len, "utf-8", cfg.val_size, cfg.seed)
    flat = [(d, i) for d, s in enumerate(train_sets) for i in range(len(s))]
    # BN running statistics: one copy per "rank", updated only by that rank's shards, replaced by their
    # fp64 mean at the end of every epoch (training/train.py sync_bn_stats, before eval and checkpoint)
    bufs = {n: b for n, b in model.named_buffers() if n.endswith(("running_mean", "running_var"))}
    per_rank = [{n: b.detach().clone() for n, b in bufs.items()} for _ in range(world)]
    model.train()

    @torch.no_grad()
    def load(r):
        for n, b in bufs.items():
            b.copy_(per_rank[r][n])

    @torch.no_grad()
    def save(r):
        for n, b in bufs.items():
            per_rank[r][n].copy_(b)
    for epoch in range(1, cfg.epochs + 1):
        eb = [[flat[i] for i in b] for b in batches(range(len(flat)), cfg.batch_size, True, cfg.seed + epoch)]
        for k in range(len(eb) // world):
            opt.zero_grad(set_to_none=True)
            for r in range(world):
                load(r)
                crops, labels = zip(*[train_sets[d][i] for d, i in eb[r + world * k]])
                x = preprocess_batch(list(crops), cfg.img_h, cfg.img_w, out="encoder", dtype=torch.bfloat16,
                                     device=dev)
                ids, lens = ctc_targets(list(labels), stoi, cfg.max_len)
                ctc_loss(model(x), ids, lens).backward()
                save(r)
            opt.step(grad_scale=1.0 / world)
        with torch.no_grad():
            for n, b in bufs.items():
                m = sum(per_rank[r][n].double() for r in range(world)) / world
                for r in range(world):
                    per_rank[r][n].copy_(m.to(b.dtype))
        load(0)
    torch.cuda.synchronize()
    return p0, model


@pytest.mark.gpu
def test_run_training_world2_matches_single_process_emulation(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from training.train import Config
    exp = str(tmp_path / "exp")
    cfg_path = tmp_path / "dp.json"
    cfg_path.write_text(json.dumps(_cfg_dict(exp, world_size=2)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, str(cfg_path), q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=240) for _ in ps), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    for rank, out, err in res:
        assert err is None, f"rank {rank}: {err}"
        assert set(out) == {"val_acc", "val_loss", "exp_dir"} and out["exp_dir"] == exp
    assert res[0][1] == res[1][1], "ranks disagree on the gathered validation metrics"
    rows = open(os.path.join(exp, "metrics_epoch.csv"), encoding="utf-8").read().strip().splitlines()
    assert len(rows) == 3, rows                    # header + 2 epochs, written by rank 0 only
    log = open(os.path.join(exp, "train.log"), encoding="utf-8").read()
    assert "world_size=2" in log
    spreads = [float(l.rsplit(" ", 1)[1]) for l in log.splitlines() if "replica parameter checksum spread" in l]
    assert len(spreads) == 2 and all(s == 0.0 for s in spreads), spreads
    # rank 0's weights vs the single-process emulation of the same DP job
    cfg = Config(str(cfg_path))
    from crnn_hip import _lib as L
    L.call("crnn_set_option", L.OPT_WGRAD_SLAB_BF16, 0)
    try:
        p0, model = _emulate(cfg, 2)
    finally:
        L.call("crnn_set_option", L.OPT_WGRAD_SLAB_BF16, 1)
    sd = torch.load(os.path.join(exp, "last_weights.pth"), map_location="cpu", weights_only=True)
    dp = torch.cat([sd[k].float().reshape(-1) for k, _ in model.named_parameters()])
    em = model._flat_param.detach().float().cpu()
    upd = float((em - p0.cpu()).norm())
    rel = float((dp - em).norm()) / upd
    print(f"DP vs emulation: |dp - emu| / |update| = {rel:.3e} (update norm {upd:.3e})")
    assert upd > 0 and rel < 1e-6, rel
    # BN running statistics: rank 0 saves the ranks' mean, as the emulation computes it. Each rank's
    # statistics come from its own shards' forward passes; the weights they see differ from the emulation's by
    # the rel above, so the buffers agree to a tolerance of the same kind
    names = [n for n, _ in model.named_buffers() if n.endswith(("running_mean", "running_var"))]
    assert names
    worst = 0.0
    for n in names:
        a, b = sd[n].float(), dict(model.named_buffers())[n].detach().float().cpu()
        worst = max(worst, float((a - b).abs().max()) / (float(b.abs().max()) + 1e-12))
    print(f"BN running statistics: max relative |dp - emu| = {worst:.3e} over {len(names)} buffers")
    assert worst < 1e-4, worst
