"""training/train.py of the reference (sherstpasha/RCNN-OCR training/train.py:59-137, :179-782) on
the MI355X HIP path:

    cfg = Config("configs/config.json")        # JSON -> attributes, resume merge, exp_dir
    run_training(cfg, device="cuda")           # -> {"val_acc", "val_loss", "exp_dir"}

Same config keys and `getattr` defaults (img_h 64, img_w 256, hidden_size 256, batch_size 32,
lr 1e-3, optimizer "Adam", scheduler "ReduceLROnPlateau", eval_every, val_size 3000, ...), the same
train / val split rules (separate val CSV per dataset, else a seeded random split of val_size), the
proportional multi-dataset batch sampler, the epoch loop with eval_every, validation loss + greedy
decode + accuracy / CER / WER, metrics_epoch.csv, the three checkpoints + weight files per
evaluation, resume from a checkpoint, and the scheduler step rules.

New keys of this path (SURVEY §5 "Config"): `decoder` ("ctc", this path's default: CTC head +
CTC loss; "attn": the reference's attention head + cross-entropy), `num_rnn_layers`
(2), `dtype` ("bf16" | "fp32"), `enc_dropout_p` (0.1), `world_size` (data parallel).

Data parallel (`world_size` > 1, one process per GPU under `torchrun --nproc-per-node N`): every
rank builds the same model and takes rank 0's weights (broadcast of the flat parameter buffer);
each epoch's batches (`batch_size` samples each, per rank) are dealt round-robin to the ranks, the
same count to every rank (the remainder is dropped and logged); the backward's stage hooks drive the
overlapped bucketed gradient all-reduce (crnn_hip.dist.OverlappedAllReduce, RCCL over xGMI) and the
optimizer applies the rank mean. BatchNorm keeps per-rank batch statistics (the reference's plain
BatchNorm2d); rank 0's running statistics are the ones saved. Validation batches are dealt the same
way and the losses, references and hypotheses gathered, so every rank sees the same metrics and
scheduler decisions; only rank 0 writes logs, metrics_epoch.csv and checkpoints.

Each step: one HIP preprocess launch for the ragged batch (ResizeAndPadA + Normalize straight into
the encoder layout) -> RCNN forward on the engine -> CTC (or cross-entropy) loss -> backward ->
fused optimizer; one loss.item() per step as the reference (:510). bf16 compute replaces the
reference's fp16 autocast + GradScaler (no loss scaling needed). Out of scope:
albumentations augmentation (train and val both use the val transform; the reference's
random_split shares one transform anyway) and TensorBoard (not installed).
"""
from __future__ import annotations

import csv
import json
import logging
import os
import random
from pathlib import Path
from typing import Dict, List, Optional

import torch

from crnn_hip.ctc import ctc_greedy_decode, ctc_loss
from crnn_hip.optim import make_optimizer
from data.dataset import OCRDatasetAttn, batches, random_split_indices
from data.transforms import ctc_targets, decode_tokens, load_charset, pack_attention_targets, preprocess_batch
from model.model import RCNN
from training.metrics import character_error_rate, compute_accuracy, word_error_rate
from training.utils import load_checkpoint, save_checkpoint, save_weights, set_seed


def setup_logger(exp_dir: str) -> logging.Logger:
    """training/train.py:35-56: console + exp_dir/train.log"""
    logger = logging.getLogger(f"crnn_hip.train.{os.path.abspath(exp_dir)}")
    logger.setLevel(logging.INFO)
    logger.propagate = False
    if not logger.handlers:
        fmt = logging.Formatter("%(asctime)s | %(levelname)s | %(message)s")
        fh = logging.FileHandler(os.path.join(exp_dir, "train.log"), encoding="utf-8")
        fh.setFormatter(fmt)
        logger.addHandler(fh)
        sh = logging.StreamHandler()
        sh.setFormatter(fmt)
        logger.addHandler(sh)
    return logger


class Config:
    """training/train.py:59-137: every JSON key becomes an attribute; a `resume_path` (checkpoint
    file or experiment directory) merges the experiment's saved config.json under the user's
    non-null keys and points exp_dir at the experiment; exp_dir defaults to the first free expN."""

    _RESUME_CKPT_CANDIDATES = ["last_ckpt.pth", "best_loss_ckpt.pth", "best_acc_ckpt.pth"]

    def __init__(self, path: str):
        with open(path, "r", encoding="utf-8") as f:
            user_data = json.load(f)
        for k, v in self._maybe_apply_resume(user_data).items():
            setattr(self, k, v)
        if not getattr(self, "exp_dir", None):
            i = 1
            while os.path.exists(f"exp{i}"):
                i += 1
            self.exp_dir = f"exp{i}"

    def save(self, out_path: Optional[str] = None):
        if out_path is None:
            out_path = os.path.join(self.exp_dir, "config.json")
        os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
        with open(out_path, "w", encoding="utf-8") as f:
            json.dump(self.__dict__, f, indent=4, ensure_ascii=False)

    def __getitem__(self, key):
        return getattr(self, key)

    def _maybe_apply_resume(self, user_data: dict) -> dict:
        resume_path = user_data.get("resume_path")
        if not resume_path:
            return dict(user_data)
        resume_path = Path(resume_path).expanduser().resolve()
        if not resume_path.exists():
            raise FileNotFoundError(f"resume path not found: {resume_path}")
        if resume_path.is_dir():
            resume_dir = resume_path
            resume_ckpt = next((resume_dir / n for n in self._RESUME_CKPT_CANDIDATES if (resume_dir / n).is_file()),
                               None)
            if resume_ckpt is None:
                raise FileNotFoundError(f"no checkpoint of {self._RESUME_CKPT_CANDIDATES} in {resume_dir}")
        else:
            resume_ckpt, resume_dir = resume_path, resume_path.parent
        merged = {}
        cfg_path = resume_dir / "config.json"
        if cfg_path.is_file():
            try:
                with open(cfg_path, "r", encoding="utf-8") as f:
                    merged = json.load(f)
            except Exception as e:   # the reference only reports it (:123-124)
                print(f"[Config] could not read {cfg_path}: {e}")
        for k, v in user_data.items():
            if v is not None:
                merged[k] = v
        merged["resume_path"] = str(resume_ckpt)
        merged["exp_dir"] = str(resume_dir)
        return merged


class ProportionalBatchSampler:
    """data/dataset.py:295-331: each batch takes round(batch_size * p_i) samples of dataset i
    (re-shuffled when exhausted); len = the fewest whole batches any dataset supports."""

    def __init__(self, sizes: List[int], batch_size: int, proportions: List[float], rng: random.Random):
        assert abs(sum(proportions) - 1.0) < 1e-6, "proportions must sum to 1"
        self.sizes, self.batch_size, self.proportions, self.rng = sizes, batch_size, proportions, rng
        self.idxs = [self._fresh(n) for n in sizes]

    def _fresh(self, n):
        ix = list(range(n))
        self.rng.shuffle(ix)
        return ix

    def __len__(self):
        return min(n // max(1, int(round(self.batch_size * p))) for n, p in zip(self.sizes, self.proportions)
                   if p > 0)

    def __iter__(self):
        for _ in range(len(self)):
            batch = []
            for d, p in enumerate(self.proportions):
                k = int(round(self.batch_size * p))
                if k == 0:
                    continue
                if len(self.idxs[d]) < k:
                    self.idxs[d] = self._fresh(self.sizes[d])
                batch.extend((d, self.idxs[d].pop()) for _ in range(k))
            self.rng.shuffle(batch)
            yield batch


class _Split:
    """a dataset and the indices of one split of it (random_split's Subset)"""

    def __init__(self, ds: OCRDatasetAttn, idx: List[int]):
        self.ds, self.idx = ds, list(idx)

    def __len__(self):
        return len(self.idx)

    def __getitem__(self, i):
        return self.ds[self.idx[i]]


def build_splits(cfg, stoi, img_h, img_w, max_len, encoding, val_size, seed):
    """training/train.py:320-392: per training CSV its own val CSV if given, else a seeded random
    split of min(val_size, n) samples (split_train_val :141-176)."""
    train_csvs, train_roots = cfg.train_csvs, cfg.train_roots
    val_csvs, val_roots = getattr(cfg, "val_csvs", None), getattr(cfg, "val_roots", None)
    train_sets, val_sets = [], []
    any_val = bool(val_csvs and val_roots)
    for i, (c, r) in enumerate(zip(train_csvs, train_roots)):
        sep = bool(any_val and i < len(val_csvs) and i < len(val_roots)
                   and val_csvs[i] is not None and val_roots[i] is not None)
        if any_val:
            kw = dict(img_height=img_h, img_max_width=img_w, encoding=encoding, max_len=max_len, strict_max_len=True)
        else:   # split_train_val (:141-176): no max_len filter, long labels are cut by the collate
            kw = dict(img_height=img_h, img_max_width=img_w, encoding=encoding)
        full = OCRDatasetAttn(c, r, stoi, **kw)
        if sep:
            train_sets.append(_Split(full, range(len(full))))
            vds = OCRDatasetAttn(val_csvs[i], val_roots[i], stoi, **kw)
            val_sets.append(_Split(vds, range(len(vds))))
            continue
        n_val = min(val_size if val_size else 3000, len(full)) if any_val else min(val_size, len(full))
        if len(full) - n_val <= 0:
            raise ValueError(f"dataset {c} has {len(full)} samples, not more than val_size {n_val}")
        tr, va = random_split_indices(len(full), n_val, seed + i)
        train_sets.append(_Split(full, tr))
        val_sets.append(_Split(full, va))
    return train_sets, val_sets


def _null_logger() -> logging.Logger:
    """ranks > 0: no console / file output"""
    lg = logging.getLogger("crnn_hip.train.silent")
    lg.propagate = False
    if not lg.handlers:
        lg.addHandler(logging.NullHandler())
    return lg


def _dp_setup(cfg, device: str):
    """-> (world, rank, torch.device): torchrun's env when world_size (config or WORLD_SIZE) > 1"""
    from crnn_hip import dist as D
    world_env, rank, local = D.env_world()
    want = getattr(cfg, "world_size", None)
    world = int(want) if want is not None else world_env
    if world < 1:
        raise ValueError("world_size must be >= 1")
    if world != world_env:
        raise RuntimeError(f"world_size {world} needs one process per GPU: launch with torchrun --nproc-per-node "
                           f"{world} (WORLD_SIZE is {world_env})")
    dev = torch.device(device)
    if dev.type != "cuda" or not torch.cuda.is_available():
        raise RuntimeError("run_training needs the HIP device (the CRNN path has no CPU fallback)")
    if world > 1:
        world, rank, local = D.init_from_env()
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
    return world, rank, dev


_BN_STATS = ("running_mean", "running_var")


def sync_bn_stats(model, world: int) -> None:
    """data parallel: every rank normalises with its own batch statistics (BatchNorm2d, no SyncBN), so the
    ranks' running_mean / running_var drift apart while the replicas' weights stay identical. Before eval
    and checkpointing they are replaced by their mean over the ranks (all-reduce in fp64), so every rank
    evaluates the same model and rank 0 saves the job's statistics."""
    if world <= 1:
        return
    import torch.distributed as tdist
    bufs = [b for n, b in model.named_buffers() if n.endswith(_BN_STATS)]
    if not bufs:
        return
    flat = torch.cat([b.detach().reshape(-1).double() for b in bufs])
    tdist.all_reduce(flat)
    flat /= world
    off = 0
    with torch.no_grad():
        for b in bufs:
            n = b.numel()
            b.copy_(flat[off:off + n].view_as(b).to(b.dtype))
            off += n


def ctc_infeasible(ids: torch.Tensor, lens: torch.Tensor, T: int) -> int:
    """samples whose CTC alignment cannot exist at T frames: label length + repeated neighbours > T
    (torch's ctc_loss gives +inf there and zero_infinity zeroes the sample's loss and gradient).
    Vectorised: equal neighbours (k, k+1) counted where k + 1 < len."""
    ids = torch.as_tensor(ids)
    lens = torch.as_tensor(lens).reshape(-1).to(ids.device)
    if ids.ndim != 2 or ids.shape[1] < 2:
        return int((lens > T).sum())
    k = torch.arange(1, ids.shape[1], device=ids.device)
    rep = ((ids[:, 1:] == ids[:, :-1]) & (k[None, :] < lens[:, None])).sum(1)
    return int(((lens + rep) > T).sum())


def run_training(cfg: Config, device: str = "cuda") -> Dict[str, object]:
    seed = getattr(cfg, "seed", 42)
    set_seed(seed)
    world, rank, dev = _dp_setup(cfg, device)
    import torch.distributed as tdist
    exp_dir = getattr(cfg, "exp_dir", None)
    if world > 1:   # one experiment directory for the job: rank 0's
        box = [exp_dir]
        tdist.broadcast_object_list(box, src=0)
        exp_dir = cfg.exp_dir = box[0]
    lead = rank == 0
    if lead:
        os.makedirs(exp_dir, exist_ok=True)
        logger = setup_logger(exp_dir)
    else:
        logger = _null_logger()
    logger.info(f"Start training | exp_dir={exp_dir} | seed={seed} | world_size={world}")
    if lead:
        try:
            cfg.save()
        except Exception as e:
            logger.info(f"Config save skipped: {e}")

    charset_path = cfg.charset_path
    encoding = getattr(cfg, "encoding", "utf-8")
    img_h, img_w = getattr(cfg, "img_h", 64), getattr(cfg, "img_w", 256)
    max_len = getattr(cfg, "max_len", 25)
    hidden_size = getattr(cfg, "hidden_size", 256)
    batch_size = getattr(cfg, "batch_size", 32)
    epochs = getattr(cfg, "epochs", 20)
    lr = getattr(cfg, "lr", 1e-3)
    optimizer_name = getattr(cfg, "optimizer", "Adam")
    scheduler_name = getattr(cfg, "scheduler", "ReduceLROnPlateau")
    weight_decay = getattr(cfg, "weight_decay", 0.0)
    momentum = getattr(cfg, "momentum", 0.9)
    resume_path = getattr(cfg, "resume_path", None)
    eval_every = getattr(cfg, "eval_every", getattr(cfg, "save_every", 1))
    try:
        eval_every = int(eval_every)
    except (TypeError, ValueError):
        raise ValueError("eval_every must be a positive integer")
    if eval_every < 1:
        raise ValueError("eval_every must be >= 1")
    train_proportions = getattr(cfg, "train_proportions", None)
    val_size = getattr(cfg, "val_size", 3000)
    decoder = getattr(cfg, "decoder", "ctc")
    num_rnn_layers = getattr(cfg, "num_rnn_layers", 2)
    dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[getattr(cfg, "dtype", "bf16")]
    enc_dropout_p = getattr(cfg, "enc_dropout_p", 0.1)

    if resume_path:
        exp_dir = os.path.dirname(resume_path)
        if lead:
            os.makedirs(exp_dir, exist_ok=True)
            logger = setup_logger(exp_dir)
    log_dir = os.path.join(exp_dir, "logs")
    metrics_csv_path = os.path.join(exp_dir, "metrics_epoch.csv")
    if lead:
        os.makedirs(log_dir, exist_ok=True)
        if not os.path.exists(metrics_csv_path):
            with open(metrics_csv_path, "w", newline="", encoding="utf-8") as f:
                csv.writer(f).writerow(["epoch", "train_loss", "val_loss", "val_acc", "val_cer", "val_wer", "lr"])
    paths = {k: os.path.join(exp_dir, f"{k}_ckpt.pth") for k in ("best_loss", "best_acc", "last")}
    wpaths = {k: os.path.join(exp_dir, f"{k}_weights.pth") for k in ("best_loss", "best_acc", "last")}

    itos, stoi = load_charset(charset_path)
    PAD, SOS, EOS = stoi["<PAD>"], stoi["<SOS>"], stoi["<EOS>"]
    BLANK = stoi.get("<BLANK>", None)
    logger.info(f"Charset loaded: {len(itos)} tokens")
    model = RCNN(num_classes=len(itos), hidden_size=hidden_size, sos_id=SOS, eos_id=EOS, pad_id=PAD, blank_id=BLANK,
                 enc_dropout_p=enc_dropout_p, decoder=decoder, num_rnn_layers=num_rnn_layers,
                 compute_dtype=dtype).to(dev)
    reducer = None
    if world > 1:
        from crnn_hip import dist as D
        # one flat parameter buffer (the optimizer's and the all-reduce's unit), rank 0's values
        model.flatten_parameters_()
        D.broadcast_params(model._flat_param)
        for b in model.buffers():
            tdist.broadcast(b, 0)
        model.mark_params_changed()
        reducer = D.OverlappedAllReduce(model._flat_grad, model.flat_offsets())
        model.stage_done = reducer.ready
    optimizer = make_optimizer(optimizer_name, model, lr, weight_decay, momentum)
    if scheduler_name == "ReduceLROnPlateau":
        scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, mode="min", factor=0.5, patience=3,
                                                               min_lr=1e-7)
    elif scheduler_name == "CosineAnnealingLR":
        scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=epochs)
    elif scheduler_name in ("None", None):
        scheduler = None
    else:
        raise ValueError(f"Unknown scheduler: {scheduler_name}")

    train_sets, val_sets = build_splits(cfg, stoi, img_h, img_w, max_len, encoding, val_size, seed)
    rng = random.Random(seed)
    if train_proportions is not None:
        tot = sum(train_proportions)
        props = [p / tot for p in train_proportions]
        assert len(props) == len(train_sets), "train_proportions != num train_sets"
        sampler = ProportionalBatchSampler([len(s) for s in train_sets], batch_size, props, rng)
        n_train_batches = len(sampler)
    else:
        flat = [(d, i) for d, s in enumerate(train_sets) for i in range(len(s))]
        n_train_batches = (len(flat) + batch_size - 1) // batch_size
    logger.info(f"Datasets: train={sum(len(s) for s in train_sets)} val={sum(len(s) for s in val_sets)}; "
                f"train_batches/epoch={n_train_batches}; batch_size={batch_size}; decoder={decoder}")

    def load_batch(items):
        crops, labels = zip(*items)
        x = preprocess_batch(list(crops), img_h, img_w, out="encoder", dtype=dtype, device=dev)
        return x, list(labels)

    def ctc_refs(labels):
        ids, lens = ctc_targets(labels, stoi, max_len)
        return ids, lens, ["".join(itos[t] for t in row[:n]) for row, n in zip(ids.tolist(), lens.tolist())]

    infeasible = [0]

    def train_loss(x, labels):
        if decoder == "ctc":
            ids, lens = ctc_targets(labels, stoi, max_len)
            logits = model(x)
            infeasible[0] += ctc_infeasible(ids, lens, logits.shape[1])
            return ctc_loss(logits, ids, lens)
        from crnn_hip.attn import cross_entropy
        text_in, target_y, _ = pack_attention_targets(labels, stoi, max_len, drop_blank=True)
        logits = model(x, text=text_in.to(dev), is_train=True, batch_max_length=max_len)
        return cross_entropy(logits.reshape(-1, logits.shape[-1]), target_y.to(dev).reshape(-1), ignore_index=PAD)

    @torch.no_grad()
    def val_batch(x, labels):
        """(loss, refs, hyps) of one validation batch (training/train.py:548-577)"""
        if decoder == "ctc":
            ids, lens, refs = ctc_refs(labels)
            logits = model(x)
            loss = float(ctc_loss(logits, ids, lens))
            hyps = ["".join(itos[t] for t in s) for s in ctc_greedy_decode(logits)]
            return loss, refs, hyps
        from crnn_hip.attn import cross_entropy
        text_in, target_y, _ = pack_attention_targets(labels, stoi, max_len, drop_blank=True)
        tf = model(x, text=text_in.to(dev), is_train=True, batch_max_length=max_len)
        loss = float(cross_entropy(tf.reshape(-1, tf.shape[-1]), target_y.to(dev).reshape(-1), ignore_index=PAD))
        pred = model(x, is_train=False, batch_max_length=max_len).argmax(-1).cpu()
        hyps = [decode_tokens(r, itos, pad_id=PAD, eos_id=EOS, blank_id=BLANK) for r in pred]
        refs = [decode_tokens(r, itos, pad_id=PAD, eos_id=EOS, blank_id=BLANK) for r in target_y]
        return loss, refs, hyps

    start_epoch, global_step = 1, 0
    best_val_loss, best_val_acc = float("inf"), -1.0
    if resume_path and os.path.isfile(resume_path):
        # the optimizer state is copied into the flat buffers at its first step (crnn_hip/optim.py);
        # every rank reads the same (rank 0's) checkpoint
        ck = load_checkpoint(resume_path, model, optimizer=optimizer, scheduler=scheduler, map_location=str(dev))
        start_epoch = int(ck.get("epoch", 0)) + 1
        global_step = int(ck.get("global_step", 0))
        best_val_loss = float(ck.get("best_val_loss", best_val_loss))
        best_val_acc = float(ck.get("best_val_acc", best_val_acc))
        logger.info(f"Resumed from: {resume_path} (epoch={start_epoch - 1}, step={global_step})")

    ck_config = {"batch_size": batch_size, "epochs": epochs, "lr": lr, "optimizer": optimizer_name,
                 "scheduler": scheduler_name, "weight_decay": weight_decay, "momentum": momentum, "img_h": img_h,
                 "img_w": img_w, "encoding": encoding, "max_len": max_len, "charset_path": charset_path,
                 "train_csvs": cfg.train_csvs, "train_roots": cfg.train_roots,
                 "val_csvs": getattr(cfg, "val_csvs", None), "val_roots": getattr(cfg, "val_roots", None),
                 "hidden_size": hidden_size, "decoder": decoder, "num_rnn_layers": num_rnn_layers}

    def deal(items):
        """this rank's share: every world-th item from its rank, the same count on every rank"""
        if world == 1:
            return list(items)
        n = len(items) // world
        return [items[rank + world * k] for k in range(n)]

    for epoch in range(start_epoch, epochs + 1):
        model.train()
        total, nb = 0.0, 0
        infeasible[0] = 0
        if train_proportions is not None:
            epoch_batches = list(iter(sampler))
        else:
            epoch_batches = [[flat[i] for i in b] for b in batches(range(len(flat)), batch_size, True, seed + epoch)]
        mine = deal(epoch_batches)
        if world > 1 and len(epoch_batches) % world:
            logger.info(f"epoch {epoch}: {len(epoch_batches) % world} of {len(epoch_batches)} batches dropped "
                        f"(the same batch count on every rank)")
        for b in mine:
            x, labels = load_batch([train_sets[d][i] for d, i in b])

            def fwd_bwd():
                optimizer.zero_grad(set_to_none=True)
                lo = train_loss(x, labels)
                lo.backward()
                return lo

            loss = fwd_bwd()
            if reducer is not None:
                reducer.finish()
                optimizer.step(grad_scale=1.0 / world)
            else:
                optimizer.step()
            total += float(loss.item())
            nb += 1
            global_step += 1
        if world > 1:   # the job's mean train loss and infeasible count
            t = torch.tensor([total, float(nb), float(infeasible[0])], dtype=torch.float64, device=dev)
            tdist.all_reduce(t)
            total, nb, infeasible[0] = float(t[0]), int(t[1]), int(t[2])
        avg_train_loss = total / max(1, nb)
        if infeasible[0]:
            logger.info(f"epoch {epoch}: {infeasible[0]} training samples have no CTC alignment at the model's "
                        f"frame count (label + repeats > T); zero_infinity zeroed their loss and gradient")
        sync_bn_stats(model, world)   # before eval / checkpoints: one set of running statistics for the job
        should_eval = ((epoch - start_epoch) % eval_every == 0) or (epoch == epochs)
        avg_val_loss = val_acc = val_cer = val_wer = None
        if should_eval:
            model.eval()
            tot_loss, tot_batches, refs_all, hyps_all = 0.0, 0, [], []
            vb = [(vs, b) for vs in val_sets for b in batches(range(len(vs)), batch_size, False, 0)]
            if world > 1:   # every batch once: round-robin over the ranks (no drop)
                vb = vb[rank::world]
            for vs, b in vb:
                x, labels = load_batch([vs[i] for i in b])
                l, refs, hyps = val_batch(x, labels)
                tot_loss += l
                tot_batches += 1
                refs_all += refs
                hyps_all += hyps
            if world > 1:
                box = [None] * world
                tdist.all_gather_object(box, (tot_loss, tot_batches, refs_all, hyps_all))
                tot_loss = sum(v[0] for v in box)
                tot_batches = sum(v[1] for v in box)
                refs_all = [r for v in box for r in v[2]]
                hyps_all = [h for v in box for h in v[3]]
            n = max(1, len(refs_all))
            avg_val_loss = tot_loss / max(1, tot_batches)
            val_acc = compute_accuracy(refs_all, hyps_all)
            val_cer = sum(character_error_rate(r, h) for r, h in zip(refs_all, hyps_all)) / n
            val_wer = sum(word_error_rate(r, h) for r, h in zip(refs_all, hyps_all)) / n
        if world > 1:   # the replicas must hold the same weights: report the spread of their checksums
            c = (model._flat_param.detach().double().sum() + sum(
                b.detach().double().sum() for n, b in model.named_buffers() if n.endswith(_BN_STATS))).reshape(1)
            cmax, cmin = c.clone(), c.clone()
            tdist.all_reduce(cmax, op=tdist.ReduceOp.MAX)
            tdist.all_reduce(cmin, op=tdist.ReduceOp.MIN)
            logger.info(f"epoch {epoch}: replica parameter checksum spread {float(cmax - cmin):.3e}")
        lr_now = optimizer.param_groups[0]["lr"]
        if lead:
            with open(metrics_csv_path, "a", newline="", encoding="utf-8") as f:
                row = ([f"{avg_val_loss:.6f}", f"{val_acc:.6f}", f"{val_cer:.6f}", f"{val_wer:.6f}"] if should_eval
                       else ["skipped"] * 4)
                csv.writer(f).writerow([epoch, f"{avg_train_loss:.6f}"] + row + [f"{lr_now:.6e}"])
        msg = f"Epoch {epoch:03d}/{epochs} | train_loss={avg_train_loss:.4f}"
        if should_eval:
            msg += f" | val_loss={avg_val_loss:.4f} | acc={val_acc:.4f} | CER={val_cer:.4f} | WER={val_wer:.4f}"
        logger.info(msg + f" | lr={lr_now:.2e}")
        if should_eval:
            def ck(path, vl, va):
                if lead:
                    save_checkpoint(path, model, optimizer, scheduler, None, epoch, global_step, vl, va, itos, stoi,
                                    ck_config, log_dir)

            def sw(path):
                if lead:
                    save_weights(path, model)
            ck(paths["last"], avg_val_loss, val_acc)
            sw(wpaths["last"])
            if avg_val_loss < best_val_loss:
                best_val_loss = avg_val_loss
                ck(paths["best_loss"], best_val_loss, val_acc)
                sw(wpaths["best_loss"])
            if val_acc >= best_val_acc:
                best_val_acc = val_acc
                ck(paths["best_acc"], best_val_loss, best_val_acc)
                sw(wpaths["best_acc"])
        if scheduler is not None:
            if isinstance(scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
                if should_eval and avg_val_loss is not None:
                    scheduler.step(avg_val_loss)
            else:
                scheduler.step()
    if reducer is not None:
        model.stage_done = None
        tdist.barrier()   # rank 0's checkpoints are on disk before any rank returns
    logger.info("Training finished.")
    return {"val_acc": best_val_acc, "val_loss": best_val_loss, "exp_dir": exp_dir}
