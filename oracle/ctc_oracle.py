"""ORACLE — test infrastructure only (see oracle/crnn_oracle.py header).

Log-space CTC forward/backward restated in numpy float64.

The reference never calls a CTC loss; the north star's CTC is
torch.nn.functional.ctc_loss (third-party PyTorch; reference requirements.txt:5
pins torchvision 0.15.2 => torch 2.0.1; this container has torch 2.10.0).
Semantics restated (Graves et al. 2006 alpha/beta over the blank-extended label
l' of length S = 2L+1):
  * inputs are logits [B,T,C]; log_softmax over C is applied here;
  * blank = 0; every sample uses input_length = T (crops are padded to a fixed
    width, data/transforms.py:100-120);
  * loss_b = -log p(l_b | x_b); reduction 'mean' = mean_b(loss_b / max(L_b,1)),
    'sum' = sum_b loss_b, 'none' = per-sample vector;
  * zero_infinity: an infeasible alignment (loss = +inf) contributes 0 loss and 0 grad;
  * gradient wrt the LOGITS = softmax - occupancy/p (the log_softmax Jacobian folded
    in, exactly what autograd through log_softmax + ctc_loss yields).
Pinned by tests/golden/ctc_cases.npz (F.ctc_loss values/grads generated in-container).
"""
from __future__ import annotations

import numpy as np

NEG = -np.inf


def _lse(a, b):
    m = np.maximum(a, b)
    with np.errstate(invalid="ignore"):
        r = m + np.log(np.exp(a - m) + np.exp(b - m))
    return np.where(np.isneginf(m), NEG, r)


def _lse3(a, b, c):
    return _lse(_lse(a, b), c)


def ctc_single(lp, label):
    """lp: [T,C] log-probs (float64); label: list of ids. Returns (nll, occupancy[T,C])."""
    T, C = lp.shape
    L = len(label)
    S = 2 * L + 1
    ext = np.zeros(S, dtype=np.int64)
    ext[1::2] = label
    alpha = np.full((T, S), NEG)
    alpha[0, 0] = lp[0, ext[0]]
    if S > 1:
        alpha[0, 1] = lp[0, ext[1]]
    for t in range(1, T):
        for s in range(S):
            a = alpha[t - 1, s]
            if s >= 1:
                a = _lse(a, alpha[t - 1, s - 1])
            if s >= 2 and ext[s] != 0 and ext[s] != ext[s - 2]:
                a = _lse(a, alpha[t - 1, s - 2])
            alpha[t, s] = a + lp[t, ext[s]]
    beta = np.full((T, S), NEG)
    beta[T - 1, S - 1] = lp[T - 1, ext[S - 1]]
    if S > 1:
        beta[T - 1, S - 2] = lp[T - 1, ext[S - 2]]
    for t in range(T - 2, -1, -1):
        for s in range(S):
            b = beta[t + 1, s]
            if s + 1 < S:
                b = _lse(b, beta[t + 1, s + 1])
            if s + 2 < S and ext[s] != 0 and ext[s] != ext[s + 2]:
                b = _lse(b, beta[t + 1, s + 2])
            beta[t, s] = b + lp[t, ext[s]]
    ll = alpha[T - 1, S - 1]
    if S > 1:
        ll = _lse(ll, alpha[T - 1, S - 2])
    nll = -ll
    occ = np.full((T, C), NEG)
    ab = alpha + beta
    for s in range(S):
        occ[:, ext[s]] = _lse(occ[:, ext[s]], ab[:, s])
    # alpha and beta both include lp[t, ext[s]]: divide it out once
    with np.errstate(invalid="ignore"):
        post = np.exp(occ - lp - ll) if np.isfinite(ll) else np.zeros_like(lp)
    post = np.nan_to_num(post, nan=0.0)
    return nll, post


def log_softmax(x, axis=-1):
    m = x.max(axis=axis, keepdims=True)
    y = x - m
    return y - np.log(np.exp(y).sum(axis=axis, keepdims=True))


def ctc_loss_and_grad(logits_btc, targets, lengths, reduction="mean", zero_infinity=True):
    """logits [B,T,C] -> (loss, dloss/dlogits [B,T,C]) in float64."""
    logits_btc = np.asarray(logits_btc, dtype=np.float64)
    B, T, C = logits_btc.shape
    lp = log_softmax(logits_btc)
    sm = np.exp(lp)
    losses = np.zeros(B)
    grads = np.zeros_like(lp)
    for b in range(B):
        L = int(lengths[b])
        label = [int(v) for v in np.asarray(targets[b])[:L]]
        nll, post = ctc_single(lp[b], label)
        g = sm[b] - post
        if np.isinf(nll) and zero_infinity:    # torch zeroes only +inf (infeasible); NaN stays NaN
            nll, g = 0.0, np.zeros_like(g)
        elif not np.isfinite(nll):
            g = np.full_like(g, np.nan)
        losses[b] = nll
        grads[b] = g
    if reduction == "mean":
        w = 1.0 / (np.maximum(np.asarray(lengths, dtype=np.float64), 1.0) * B)
        return float((losses * w * B).mean()), grads * w[:, None, None]
    if reduction == "sum":
        return float(losses.sum()), grads
    return losses, grads
