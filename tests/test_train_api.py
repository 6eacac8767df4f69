"""training.train boundary (reference training/train.py:59-137, :179-782): Config, the CSV dataset
reader, the split / sampler rules on the host (CPU tests), and run_training end to end on the HIP
path on the committed tiny line sets (tests/golden/lines, tests/golden/make_lines.py; GPU tests)."""
import csv
import json
import os
import random

import pytest
import torch

from helpers import GOLDEN

LINES = os.path.join(GOLDEN, "lines")
CHARSET = os.path.join(GOLDEN, "charset.txt")


def _stoi():
    from data.transforms import load_charset
    return load_charset(CHARSET)[1]


def test_config_attributes_and_resume_merge(tmp_path, monkeypatch):
    from training.train import Config
    monkeypatch.chdir(tmp_path)
    p = tmp_path / "c.json"
    p.write_text(json.dumps({"lr": 0.5, "batch_size": 4, "resume_path": None}))
    cfg = Config(str(p))
    assert cfg.lr == 0.5 and cfg["batch_size"] == 4 and cfg.exp_dir == "exp1"
    cfg.save()
    assert json.loads((tmp_path / "exp1" / "config.json").read_text())["lr"] == 0.5
    os.makedirs(tmp_path / "exp2")
    (tmp_path / "exp2" / "config.json").write_text(json.dumps({"lr": 0.1, "epochs": 7, "img_h": 32}))
    (tmp_path / "exp2" / "best_acc_ckpt.pth").write_bytes(b"x")
    p.write_text(json.dumps({"lr": 0.25, "epochs": None, "resume_path": str(tmp_path / "exp2")}))
    cfg = Config(str(p))
    # user keys win unless null; the experiment's config fills the rest (train.py:120-136)
    assert cfg.lr == 0.25 and cfg.epochs == 7 and cfg.img_h == 32
    assert cfg.resume_path.endswith("best_acc_ckpt.pth") and cfg.exp_dir == str(tmp_path / "exp2")
    p.write_text(json.dumps({"resume_path": str(tmp_path / "nope")}))
    with pytest.raises(FileNotFoundError):
        Config(str(p))


def test_dataset_reader_rules(tmp_path):
    """header detection, label normalisation, charset / max_len / missing-path skips, basename
    index resolution (data/dataset.py:163-261)"""
    from data.dataset import OCRDatasetAttn
    stoi = _stoi()
    root = os.path.join(LINES, "a")
    ds = OCRDatasetAttn(os.path.join(root, "labels.csv"), root, stoi, max_len=40)
    assert len(ds) == 40 and ds.reasons == {}
    img, label = ds[0]
    assert img.dtype.name == "uint8" and img.ndim == 3 and img.shape[2] == 3 and img.shape[0] == 32
    rows = list(csv.reader(open(os.path.join(root, "labels.csv"), encoding="utf-8")))[1:]
    assert label == rows[0][1]
    bad = tmp_path / "bad.csv"
    with open(bad, "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(["img_000.png", "  ok  "])          # normalised to "ok"
        w.writerow(["only_one_column"])                    # bad_row
        w.writerow(["", "x"])                              # empty_fname
        w.writerow(["img_001.png", ""])                    # empty_label
        w.writerow(["img_002.png", "a☃b"])            # charset
        w.writerow(["img_003.png", "abcdefghijk"])         # too_long (max_len 10)
        w.writerow(["missing.png", "abc"])                 # missing_path
        w.writerow(["sub/IMG_004.PNG", "abc"])             # resolved through the basename index
    ds = OCRDatasetAttn(str(bad), root, stoi, max_len=10)
    assert [s[1] for s in ds.samples] == ["ok", "abc"]
    assert dict(ds.reasons) == {"bad_row": 1, "empty_fname": 1, "empty_label": 1, "charset": 1, "too_long": 1,
                                "missing_path": 1}
    assert ds.samples[1][0].endswith("img_004.png")


def test_evaluate_dataset_loader(tmp_path):
    """evaluate_dataset.load_dataset (evaluate_dataset.py:18-56): filename / text columns, missing
    extensions tried, missing images skipped"""
    from evaluate_dataset import load_dataset
    root = os.path.join(LINES, "b", "val")
    p = tmp_path / "e.csv"
    p.write_text("filename,text\nva_000.png,abc\nva_001,007\nnope.png,x\n", encoding="utf-8")
    paths, texts = load_dataset(str(p), root)
    assert [os.path.basename(q) for q in paths] == ["va_000.png", "va_001.png"] and texts == ["abc", "007"]
    with pytest.raises(ValueError):
        (tmp_path / "bad.csv").write_text("file,label\na,b\n")
        load_dataset(str(tmp_path / "bad.csv"), root)


def test_split_and_proportional_sampler():
    from data.dataset import batches, random_split_indices
    from training.train import ProportionalBatchSampler
    tr, va = random_split_indices(40, 10, 42)
    assert len(tr) == 30 and len(va) == 10 and sorted(tr + va) == list(range(40))
    assert random_split_indices(40, 10, 42) == (tr, va)
    bs = list(batches(range(10), 4, False, 0))
    assert bs == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]
    s = ProportionalBatchSampler([30, 12], 8, [0.5, 0.5], random.Random(0))
    assert len(s) == 3       # min(30 // 4, 12 // 4)
    out = list(s)
    assert len(out) == 3 and all(sum(1 for d, _ in b if d == 0) == 4 for b in out)


def _cfg(tmp_path, **kw):
    from training.train import Config
    c = {"train_csvs": [os.path.join(LINES, "a", "labels.csv"), os.path.join(LINES, "b", "train", "labels.csv")],
         "train_roots": [os.path.join(LINES, "a"), os.path.join(LINES, "b", "train")],
         "val_csvs": [None, os.path.join(LINES, "b", "val", "labels.csv")],
         "val_roots": [None, os.path.join(LINES, "b", "val")],
         "charset_path": CHARSET, "img_h": 32, "img_w": 128, "max_len": 16, "hidden_size": 64, "batch_size": 16,
         "epochs": 3, "lr": 2e-3, "optimizer": "Adam", "scheduler": "CosineAnnealingLR", "weight_decay": 1e-5,
         "val_size": 8, "seed": 7, "eval_every": 1, "exp_dir": str(tmp_path / "exp"), "enc_dropout_p": 0.0}
    c.update(kw)
    p = tmp_path / f"cfg_{len(os.listdir(tmp_path))}.json"
    p.write_text(json.dumps(c))
    return Config(str(p))


@pytest.mark.gpu
@pytest.mark.parametrize("decoder", ["ctc", "attn"])
def test_run_training_end_to_end(tmp_path, decoder):
    """run_training on the HIP path: returns the reference's dict, writes the three checkpoints +
    weights and metrics_epoch.csv, the training loss falls, and a resume continues the epoch count
    with the optimizer state (training/train.py:475-485, :617-771)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from training.train import run_training
    cfg = _cfg(tmp_path, decoder=decoder)
    out = run_training(cfg, device="cuda")
    assert set(out) == {"val_acc", "val_loss", "exp_dir"} and out["exp_dir"] == cfg.exp_dir
    assert 0.0 <= out["val_acc"] <= 1.0 and out["val_loss"] < float("inf")
    for n in ("last_ckpt.pth", "best_loss_ckpt.pth", "best_acc_ckpt.pth", "last_weights.pth", "train.log",
              "config.json", "metrics_epoch.csv"):
        assert os.path.isfile(os.path.join(cfg.exp_dir, n)), n
    rows = list(csv.reader(open(os.path.join(cfg.exp_dir, "metrics_epoch.csv"), encoding="utf-8")))
    assert rows[0] == ["epoch", "train_loss", "val_loss", "val_acc", "val_cer", "val_wer", "lr"]
    assert [r[0] for r in rows[1:]] == ["1", "2", "3"]
    tl = [float(r[1]) for r in rows[1:]]
    assert all(t == t for t in tl) and tl[-1] < tl[0], tl
    ck = torch.load(os.path.join(cfg.exp_dir, "last_ckpt.pth"), map_location="cpu", weights_only=True)
    assert ck["epoch"] == 3 and ck["config"]["decoder"] == decoder
    assert ck["optimizer_state"]["state"][0]["exp_avg"].abs().sum() > 0
    # resume: one more epoch from the last checkpoint (epochs = 4)
    cfg2 = _cfg(tmp_path, decoder=decoder, epochs=4, resume_path=os.path.join(cfg.exp_dir, "last_ckpt.pth"))
    run_training(cfg2, device="cuda")
    rows = list(csv.reader(open(os.path.join(cfg.exp_dir, "metrics_epoch.csv"), encoding="utf-8")))
    assert [r[0] for r in rows[1:]] == ["1", "2", "3", "4"]
    ck = torch.load(os.path.join(cfg.exp_dir, "last_ckpt.pth"), map_location="cpu", weights_only=True)
    assert ck["epoch"] == 4 and ck["global_step"] > 0
    # evaluate_dataset.py on the trained checkpoint (evaluate_dataset.py:59-158)
    from evaluate_dataset import evaluate_model
    vroot = os.path.join(LINES, "b", "val")
    r = evaluate_model(os.path.join(cfg.exp_dir, "last_ckpt.pth"), CHARSET, os.path.join(vroot, "labels.csv"), vroot,
                       batch_size=4, img_h=32, img_w=128, report_path=str(tmp_path / "report.csv"), verbose=False)
    assert r["samples"] == 8 and 0.0 <= r["accuracy"] <= 1.0 and r["cer"] >= 0.0
    rows = list(csv.reader(open(r["report"], encoding="utf-8")))
    assert rows[0] == ["image_path", "true_text", "predicted_text", "cer", "wer", "exact_match"] and len(rows) == 9


def test_ctc_infeasible_count():
    """label + repeated neighbours > T has no CTC alignment (zero_infinity zeroes it): counted"""
    from training.train import ctc_infeasible
    ids = torch.tensor([[5, 5, 6, 0], [5, 6, 7, 8], [9, 9, 9, 0]])
    lens = torch.tensor([3, 4, 3])
    # needs: 3 + 1 = 4, 4 + 0 = 4, 3 + 2 = 5
    assert ctc_infeasible(ids, lens, 4) == 1
    assert ctc_infeasible(ids, lens, 3) == 3
    assert ctc_infeasible(ids, lens, 5) == 0
    # repeats past the label length do not count
    assert ctc_infeasible(torch.tensor([[5, 6, 6, 6]]), torch.tensor([2]), 2) == 0
    assert ctc_infeasible(torch.tensor([[5, 6, 6, 6]]), torch.tensor([4]), 5) == 1


def test_split_without_val_csvs_keeps_long_labels(tmp_path):
    """no val_csvs / val_roots at all: the reference's split_train_val (training/train.py:141-176)
    builds the datasets WITHOUT max_len (no too-long filter) and takes min(val_size, n) for val"""
    from training.train import build_splits
    stoi = _stoi()
    root = os.path.join(LINES, "a")
    cfg = type("C", (), {"train_csvs": [os.path.join(root, "labels.csv")], "train_roots": [root]})()
    tr, va = build_splits(cfg, stoi, 32, 128, 2, "utf-8", 5, 7)   # max_len 2 would drop every label
    assert len(tr[0]) + len(va[0]) == 40 and len(va[0]) == 5
    cfg.val_csvs, cfg.val_roots = [None], [None]
    with pytest.raises(ValueError):       # with a val list given, max_len filters (train.py:356-366)
        build_splits(cfg, stoi, 32, 128, 2, "utf-8", 5, 7)
