"""training/utils.py API of sherstpasha/RCNN-OCR (training/utils.py:9-162) for the CTC path.

Checkpoint dict keys are the reference's (training/utils.py:24-37), so `model_state` holds
reference-named encoder weights plus ctc_head.* (CTC) or the reference's attn.* (attention). Loading uses torch.load(weights_only=True):
the dict holds only tensors, numbers, strings, lists and dicts.
"""
from __future__ import annotations

import random

import torch

from crnn_hip.ctc import ctc_greedy_decoder as _hip_greedy
from model.model import RCNN


def save_checkpoint(path, model, optimizer, scheduler, scaler, epoch, global_step, best_val_loss, best_val_acc,
                    itos, stoi, config, log_dir):
    ckpt = {
        "epoch": epoch,
        "global_step": global_step,
        "model_state": model.state_dict(),
        "optimizer_state": optimizer.state_dict() if optimizer is not None else None,
        "scheduler_state": scheduler.state_dict() if scheduler is not None else None,
        "scaler_state": scaler.state_dict() if scaler is not None else None,
        "best_val_loss": best_val_loss,
        "best_val_acc": best_val_acc,
        "itos": itos,
        "stoi": stoi,
        "config": config,
        "log_dir": log_dir,
    }
    torch.save(ckpt, path)


def save_weights(path, model):
    torch.save(model.state_dict(), path)


def load_checkpoint(path, model, optimizer=None, scheduler=None, scaler=None, map_location="auto"):
    if map_location == "auto":
        map_location = "cuda" if torch.cuda.is_available() else "cpu"
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    model.load_state_dict(ckpt["model_state"])
    if optimizer is not None and ckpt.get("optimizer_state") is not None:
        optimizer.load_state_dict(ckpt["optimizer_state"])
    if scheduler is not None and ckpt.get("scheduler_state") is not None:
        scheduler.load_state_dict(ckpt["scheduler_state"])
    if scaler is not None and ckpt.get("scaler_state") is not None:
        scaler.load_state_dict(ckpt["scaler_state"])
    return ckpt


def set_seed(seed: int = 42):
    random.seed(seed)
    torch.manual_seed(seed)


def rcnn_from_state(model_state, num_classes, hidden_size, sos_id, eos_id, pad_id, blank_id,
                    compute_dtype=torch.bfloat16) -> RCNN:
    """An RCNN whose decoder matches the checkpoint, loaded strictly: ctc_head.* -> the CTC model;
    attn.* (every checkpoint the reference trains, model/model.py:203-213) -> decoder="attn" (the
    reference's exact key set); neither -> ValueError (no head to decode with)."""
    if any(k.startswith("ctc_head.") for k in model_state):
        decoder = "ctc"
    elif any(k.startswith("attn.") for k in model_state):
        decoder = "attn"
    else:
        raise ValueError("checkpoint has neither ctc_head.* nor attn.* weights: no decoder to load")
    n_rnn = len({k.split(".")[1] for k in model_state if k.startswith("enc_rnn.") and k.endswith("linear.bias")})
    model = RCNN(num_classes=num_classes, hidden_size=hidden_size, sos_id=sos_id, eos_id=eos_id, pad_id=pad_id,
                 blank_id=blank_id, decoder=decoder, num_rnn_layers=max(1, n_rnn), compute_dtype=compute_dtype)
    model.load_state_dict(model_state, strict=True)
    return model


def load_crnn(checkpoint_path, itos=None, stoi=None, hidden_size=256, sos_token="<SOS>", eos_token="<EOS>",
              pad_token="<PAD>", blank_token="<BLANK>", device=None, eval_mode=True,
              compute_dtype=torch.bfloat16) -> RCNN:
    """training/utils.py:70-119: strict load (the reference's own contract) into the decoder the
    checkpoint holds — CTC (ctc_head.*) or the reference's attention decoder (attn.*)."""
    if device is None:
        device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    state = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    if isinstance(state, dict) and "model_state" in state:
        model_state = state["model_state"]
        itos = itos if itos is not None else state.get("itos")
        stoi = stoi if stoi is not None else state.get("stoi")
    else:
        model_state = state
    assert itos is not None and stoi is not None, "itos/stoi required (pass them or use a full checkpoint)"
    blank = stoi.get(blank_token, None) if blank_token is not None else None
    model = rcnn_from_state(model_state, len(itos), hidden_size, stoi[sos_token], stoi[eos_token], stoi[pad_token],
                            blank, compute_dtype)
    model = model.to(device)
    if eval_mode:
        model.eval()
    return model


def ctc_greedy_decoder(logits: torch.Tensor, alphabet, blank: int = 0, layout: str = "BTC"):
    """training/utils.py:122-150 contract (texts, seqs) with an explicit layout."""
    return _hip_greedy(logits, alphabet, blank=blank, layout=layout)


def decode(ctc_out, alphabet, method: str = "greedy", layout: str = "BTC"):
    """training/utils.py:153-162 (log_softmax is monotone per row: argmax on logits is identical)."""
    if isinstance(ctc_out, tuple):
        ctc_out = ctc_out[0]
    if method != "greedy":
        raise ValueError(f"Unsupported decode method: {method}")
    return ctc_greedy_decoder(ctc_out, alphabet, layout=layout)
