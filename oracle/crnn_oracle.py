"""ORACLE — test infrastructure only. NOT part of the product path.

CPU fp32 restatement of the reference CRNN hot path (sherstpasha/RCNN-OCR),
written from scratch in functional form so every intermediate is reachable.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline, never as the thing measured
or shipped. The HIP product path (rcnn-ocr_amd/crnn_hip) never imports it.

Pinned against tests/golden/*.npz, which were produced by running the reference
itself (tests/golden/make_goldens.py): eval-mode encode + CTC-head logits,
train-mode loss + gradients, CTC loss/grad values, greedy-decode strings and a
4-layer 768-hidden BiLSTM stack.

Citations are /root/reference/<file>:<line>.
Parameters are a dict keyed by the reference's state_dict names
(model/model.py:166-213, model/seresnet31.py:70-187) + `ctc_head.{weight,bias}`.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from ctc_oracle import ctc_loss_and_grad  # noqa: E402  (oracle/ on sys.path)

BN_EPS = 1e-5
BN_MOMENTUM = 0.1

# (layer name, blocks, stride, inplanes, planes) — model/seresnet31.py:92-127
STAGES = [("layer1", 1, 2, 128, 256), ("layer2", 2, 1, 256, 256),
          ("layer3", 5, 2, 256, 512), ("layer4", 3, 1, 512, 512)]


class Ctx:
    """train flag + BN running-stat updates + recorded intermediates.

    `force` (test use): ReLU masks / 2x2 max-pool window indices, by decision-site name, that
    replace the oracle's own decisions. An fp64 evaluation that takes an fp32 path's decisions
    is that path's exact reference: fp32 ties (|pre-activation| within rounding of 0) no longer
    decide which side of a ReLU kink the two evaluations land on.

    `store` (test use): applied to every tensor the HIP path keeps in its compute dtype between
    kernels (conv outputs before BN, BN-ReLU outputs, pooled / block outputs, the sequence, the
    LSTM input projections and hidden states, the BiLSTM outputs); e.g. bf16 round-to-nearest
    makes this the bf16-storage model of the computation, the error bar of a bf16 HIP run.
    BN statistics are taken before `store`, as the HIP conv epilogue sums its fp32 accumulators.
    `momentum`: BN running-statistics momentum (1.0: running stats := this batch's)."""

    def __init__(self, train: bool, record: bool = False, force: Optional[Dict[str, torch.Tensor]] = None,
                 store=None, momentum: float = BN_MOMENTUM):
        self.train = train
        self.record = record
        self.acts: Dict[str, torch.Tensor] = {}
        self.running: Dict[str, torch.Tensor] = {}
        self.force = force or {}
        self.store = store if store is not None else (lambda t: t)
        self.momentum = momentum

    def rec(self, name, t):
        if self.record:
            if t.requires_grad:
                t.retain_grad()
            self.acts[name] = t


def relu(ctx: Ctx, site: str, u):
    m = ctx.force.get(site)
    return torch.relu(u) if m is None else u * m.to(u.dtype)


def maxpool2(ctx: Ctx, site: str, x):
    """F.max_pool2d(x, 2, 2); forced: window element t = 2*dh + dw per output."""
    idx = ctx.force.get(site)
    if idx is None:
        return F.max_pool2d(x, 2, 2)
    B, C, H, W = x.shape
    win = x.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
    return win.gather(-1, idx.long()[..., None]).squeeze(-1)


def batchnorm(x, p, prefix, ctx: Ctx):
    """nn.BatchNorm2d (torch defaults eps=1e-5, momentum=0.1): train mode normalises
    with the biased batch variance and folds the unbiased one into running_var."""
    w, b = p[prefix + ".weight"], p[prefix + ".bias"]
    xs = ctx.store(x)
    if ctx.train:
        n = x.numel() // x.shape[1]
        mean = x.mean(dim=(0, 2, 3))
        var = ((x - mean.view(1, -1, 1, 1)) ** 2).mean(dim=(0, 2, 3))
        with torch.no_grad():
            rm = p[prefix + ".running_mean"]
            rv = p[prefix + ".running_var"]
            m = ctx.momentum
            ctx.running[prefix + ".running_mean"] = (1 - m) * rm + m * mean.detach()
            ctx.running[prefix + ".running_var"] = (1 - m) * rv + m * var.detach() * n / max(1, n - 1)
    else:
        mean, var = p[prefix + ".running_mean"], p[prefix + ".running_var"]
    inv = torch.rsqrt(var + BN_EPS)
    return (xs - mean.view(1, -1, 1, 1)) * (inv * w).view(1, -1, 1, 1) + b.view(1, -1, 1, 1)


def se_layer(x, p, prefix, ctx: Optional[Ctx] = None):
    """SELayer.forward, model/seresnet31.py:16-20 (reduction 16, no biases)."""
    y = x.mean(dim=(2, 3))
    y = y @ p[prefix + ".fc.0.weight"].t()
    y = relu(ctx, prefix, y) if ctx is not None else torch.relu(y)
    y = torch.sigmoid(y @ p[prefix + ".fc.2.weight"].t())
    return x * y[:, :, None, None]


def se_block(x, p, prefix, stride, has_ds, ctx):
    """SEBasicBlock.forward, model/seresnet31.py:55-67 (dropblock: identity at p=0, else the
    multiplier forced under "<prefix>.dropblock", see dropblock_keep)."""
    out = F.conv2d(x, p[prefix + ".conv1.weight"], stride=stride, padding=1)
    out = ctx.store(relu(ctx, prefix + ".bn1", batchnorm(out, p, prefix + ".bn1", ctx)))
    out = F.conv2d(out, p[prefix + ".conv2.weight"], stride=1, padding=1)
    out = batchnorm(out, p, prefix + ".bn2", ctx)
    out = se_layer(out, p, prefix + ".se", ctx)
    drop = ctx.force.get(prefix + ".dropblock")   # DropBlock2d (:62) as keep * scale, dropblock_mult
    if drop is not None:
        out = out * drop.to(out.dtype)
    if has_ds:
        idn = F.conv2d(x, p[prefix + ".downsample.0.weight"], stride=stride)
        idn = batchnorm(idn, p, prefix + ".downsample.1", ctx)
    else:
        idn = x
    return ctx.store(relu(ctx, prefix + ".out", out + idn))


def backbone(x, p, ctx):
    """SEResNet31.forward, model/seresnet31.py:180-187."""
    x = F.conv2d(ctx.store(x), p["cnn.conv0.0.weight"], padding=1)
    x = ctx.store(relu(ctx, "cnn.conv0.1", batchnorm(x, p, "cnn.conv0.1", ctx)))
    x = F.conv2d(x, p["cnn.conv0.3.weight"], padding=1)
    x = relu(ctx, "cnn.conv0.4", batchnorm(x, p, "cnn.conv0.4", ctx))
    x = ctx.store(maxpool2(ctx, "stem.pool", x))
    ctx.rec("stem", x)
    for name, blocks, stride, inp, planes in STAGES:
        for i in range(blocks):
            s = stride if i == 0 else 1
            has_ds = i == 0 and (stride != 1 or inp != planes)
            x = se_block(x, p, f"cnn.{name}.{i}", s, has_ds, ctx)
            ctx.rec(f"{name}.{i}", x)
        ctx.rec(name, x)
    # conv_out, model/seresnet31.py:129-136
    x = F.conv2d(x, p["cnn.conv_out.0.weight"], stride=(2, 1), padding=(0, 1))
    x = ctx.store(relu(ctx, "cnn.conv_out.1", batchnorm(x, p, "cnn.conv_out.1", ctx)))
    x = F.conv2d(x, p["cnn.conv_out.3.weight"], stride=1, padding=0)
    x = relu(ctx, "cnn.conv_out.4", batchnorm(x, p, "cnn.conv_out.4", ctx))
    ctx.rec("cnn_out", x)
    return x


def lstm_direction(x, w_ih, w_hh, b_ih, b_hh, reverse, store=None):
    """nn.LSTM single direction, gate order i,f,g,o; h0 = c0 = 0.
    Reverse direction runs over the flipped sequence (model/model.py:152-163).
    store: applied to the input projections and to each h_t (Ctx.store)."""
    B, T, _ = x.shape
    H = w_hh.shape[1]
    st = store if store is not None else (lambda t: t)
    xg = st(x @ w_ih.t() + b_ih + b_hh)
    h = x.new_zeros(B, H)
    c = x.new_zeros(B, H)
    outs = [None] * T
    order = range(T - 1, -1, -1) if reverse else range(T)
    for t in order:
        g = xg[:, t] + h @ w_hh.t()
        i, f, gg, o = g.split(H, dim=1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = st(torch.sigmoid(o) * torch.tanh(c))
        outs[t] = h
    return torch.stack(outs, dim=1)


def bilstm(x, p, prefix, store=None):
    """BidirectionalLSTM.forward, model/model.py:159-163."""
    r = prefix + ".rnn."
    hf = lstm_direction(x, p[r + "weight_ih_l0"], p[r + "weight_hh_l0"], p[r + "bias_ih_l0"],
                        p[r + "bias_hh_l0"], False, store)
    hb = lstm_direction(x, p[r + "weight_ih_l0_reverse"], p[r + "weight_hh_l0_reverse"],
                        p[r + "bias_ih_l0_reverse"], p[r + "bias_hh_l0_reverse"], True, store)
    h = torch.cat([hf, hb], dim=2)
    out = h @ p[prefix + ".linear.weight"].t() + p[prefix + ".linear.bias"]
    return store(out) if store is not None else out


def encode(x, p, ctx, num_rnn_layers=2):
    """RCNN.encode, model/model.py:215-221 (enc_dropout identity: eval or p=0)."""
    f = backbone(x, p, ctx)
    seq = ctx.store(f.mean(dim=2).permute(0, 2, 1))   # AdaptiveAvgPool2d((1,None)) + squeeze + permute
    ctx.rec("seq", seq)
    for i in range(num_rnn_layers):
        seq = bilstm(seq, p, f"enc_rnn.{i}", ctx.store)
        ctx.rec(f"rnn{i}", seq)
    return seq


def head(enc, p):
    """CTC head: Linear(H -> num_classes)."""
    return enc @ p["ctc_head.weight"].t() + p["ctc_head.bias"]


class _CTC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits_btc, targets, lengths, reduction, zero_infinity):
        loss, grad = ctc_loss_and_grad(logits_btc.detach().double().numpy(), targets.numpy(),
                                       lengths.numpy(), reduction=reduction,
                                       zero_infinity=zero_infinity)
        ctx.save_for_backward(torch.from_numpy(grad).to(logits_btc.dtype))
        return torch.tensor(loss, dtype=logits_btc.dtype)

    @staticmethod
    def backward(ctx, go):
        (g,) = ctx.saved_tensors
        return g * go, None, None, None, None


# ---------------------------------------------------------------- attention decoder
# Parameters keyed by the reference's Attention state_dict (model/model.py:23-79):
# attention_cell.{i2h.weight, h2h.weight, h2h.bias, score.weight, rnn.weight_ih, rnn.weight_hh,
# rnn.bias_ih, rnn.bias_hh}, generator.{weight, bias}. Eval mode (dropout = identity).
def attn_cell(p, enc, h, c, char, num_classes, alpha_mask=None):
    """AttentionCell.forward (model/model.py:33-45): additive attention over the encoder
    sequence, then LSTMCell([context, onehot(char)], (h, c)) (gate order i, f, g, o).
    alpha_mask [B, T]: the training-mode F.dropout(alpha) (:40) as an explicit scaled keep-mask."""
    pre = "attention_cell."
    proj_H = enc @ p[pre + "i2h.weight"].t()                                   # :35
    proj_h = (h @ p[pre + "h2h.weight"].t() + p[pre + "h2h.bias"]).unsqueeze(1)  # :36
    e = torch.tanh(proj_H + proj_h) @ p[pre + "score.weight"].t()             # :37 [B,T,1]
    alpha = torch.softmax(e, dim=1)                                           # :39
    if alpha_mask is not None:                                                # :40
        alpha = alpha * alpha_mask.to(alpha.dtype).unsqueeze(2)
    context = (alpha.transpose(1, 2) @ enc).squeeze(1)                        # :42
    onehot = F.one_hot(char, num_classes).to(enc.dtype)                       # :81-85
    x = torch.cat([context, onehot], 1)                                       # :43
    gates = x @ p[pre + "rnn.weight_ih"].t() + p[pre + "rnn.bias_ih"] + h @ p[pre + "rnn.weight_hh"].t() \
        + p[pre + "rnn.bias_hh"]
    i, f, g, o = gates.chunk(4, 1)
    c2 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
    h2 = torch.sigmoid(o) * torch.tanh(c2)
    return h2, c2


def attn_greedy(p, enc, steps, sos_id, blank_id, num_classes):
    """Attention._greedy_decode (model/model.py:91-112): logits per step with the blank column
    masked to -1e4 (:87-89), next input = argmax. -> [B, steps, V]"""
    B, H = enc.shape[0], p["attention_cell.h2h.weight"].shape[0]
    h = torch.zeros(B, H, dtype=enc.dtype)
    c = torch.zeros(B, H, dtype=enc.dtype)
    ch = torch.full((B,), sos_id, dtype=torch.long)
    out = []
    for _ in range(steps):
        h, c = attn_cell(p, enc, h, c, ch, num_classes)
        lg = h @ p["generator.weight"].t() + p["generator.bias"]
        if blank_id is not None:
            lg[:, blank_id] = -1e4
        out.append(lg)
        ch = lg.argmax(1)
    return torch.stack(out, 1)


def attn_teacher(p, enc, text, steps, blank_id, num_classes, alpha_masks=None):
    """Attention.forward with teacher forcing (model/model.py:114-148, sampling_prob = 0):
    input at step t is text[:, t]; logits = generator(all h), blank masked. -> [B, steps, V].
    alpha_masks[t] [B, T]: step t's attention-weight dropout mask (attn_drop_masks), or None."""
    B, H = enc.shape[0], p["attention_cell.h2h.weight"].shape[0]
    h = torch.zeros(B, H, dtype=enc.dtype)
    c = torch.zeros(B, H, dtype=enc.dtype)
    hs = []
    for t in range(steps):
        h, c = attn_cell(p, enc, h, c, text[:, t], num_classes,
                         None if alpha_masks is None else alpha_masks[t])
        hs.append(h)
    lg = torch.stack(hs, 1) @ p["generator.weight"].t() + p["generator.bias"]
    if blank_id is not None:
        lg[:, :, blank_id] = -1e4
    return lg


def drop_keep_mask(seed: int, n: int, p: float) -> np.ndarray:
    """The HIP path's counter-based dropout mask (csrc/common.hpp drop_hash): element i kept iff
    splitmix64-finalizer(seed ^ i * golden) >> 32 >= p * 2^32; -> float64 keep / (1 - p). The
    reference uses torch's Philox stream, which is not reproduced: masks agree in distribution,
    so parity with dropout on is checked against this restatement of the mask."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ (i * np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        h = ((z ^ (z >> np.uint64(31))) & M) >> np.uint64(32)
    t = p * 4294967296.0
    thr = 0xFFFFFFFF if t >= 4294967295.0 else int(t)
    return (h >= np.uint64(thr)).astype(np.float64) / (1.0 - p)


def _splitmix_hash(seed: int, idx: np.ndarray) -> np.ndarray:
    """csrc/common.hpp drop_hash: splitmix64's finalizer on seed ^ idx * golden, high 32 bits."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ (idx.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return (z ^ (z >> np.uint64(31))) >> np.uint64(32)


def dropblock_keep(seed: int, B: int, C: int, H: int, W: int, p: float, block_size: int) -> np.ndarray:
    """torchvision.ops.drop_block2d (training) as SEBasicBlock applies it (model/seresnet31.py:49-53,
    62), with the HIP path's seed draw -> keep [B, C, H, W] uint8 (1 = kept). The published algorithm:
    bs = min(block_size, H, W); gamma = p*H*W / (bs^2 (H-bs+1)(W-bs+1)); seeds ~ Bernoulli(gamma) on
    [B, C, H-bs+1, W-bs+1]; pad by bs//2; bs x bs stride-1 max-pool with padding bs//2; keep =
    1 - pooled. Seed (n, c, i, j) = 1 iff drop_hash(seed, flat NCHW index) < gamma * 2^32 (torch's
    Philox stream is not reproduced: masks agree in distribution, parity is checked against this)."""
    bs = min(block_size, H, W)
    if bs % 2 == 0:
        raise ValueError("drop_block2d: the mask of an even block is (H+2) x (W+2) and does not broadcast")
    Hs, Ws = H - bs + 1, W - bs + 1
    gamma = p * H * W / (bs * bs * Hs * Ws)
    t = gamma * 4294967296.0
    thr = 0xFFFFFFFF if t >= 4294967295.0 else int(t)
    seeds = (_splitmix_hash(seed, np.arange(B * C * Hs * Ws)) < np.uint64(thr)).astype(np.float32)
    noise = F.pad(torch.from_numpy(seeds.reshape(B, C, Hs, Ws)), [bs // 2] * 4, value=0.0)
    noise = F.max_pool2d(noise, stride=(1, 1), kernel_size=(bs, bs), padding=bs // 2)
    return (1.0 - noise).numpy().astype(np.uint8)


def dropblock_mult(keep: np.ndarray) -> torch.Tensor:
    """keep * numel / (1e-6 + kept) in fp32 (drop_block2d's normalize_scale)"""
    k = torch.from_numpy(keep.astype(np.float32))
    scale = np.float32(k.numel()) / (np.float32(1e-6) + np.float32(int(keep.sum())))
    return k * float(scale)


def attn_drop_masks(seed: int, steps: int, B: int, T: int, p: float):
    """per-step attention-weight masks of crnn_hip/attn.py run_train (step t uses seed + t,
    element (b, t') = index b*T + t') -> list of [B, T] tensors (None when p == 0)"""
    if p == 0.0:
        return None
    return [torch.from_numpy(drop_keep_mask(seed + t, B * T, p).reshape(B, T)) for t in range(steps)]


def ctc_loss(logits_btc, targets, lengths, reduction="mean", zero_infinity=True):
    """F.ctc_loss(log_softmax(logits), blank=0) restated (numpy, float64)."""
    return _CTC.apply(logits_btc, targets, lengths, reduction, zero_infinity)


def greedy_decode(logits_btc) -> List[List[int]]:
    """training/utils.py:122-150 semantics with an explicit (B,T,C) layout:
    argmax over C, drop repeats (prev tracks every t, blank included), drop blank 0."""
    preds = np.asarray(logits_btc).argmax(axis=2)
    out = []
    for row in preds:
        prev, seq = 0, []
        for p in row:
            p = int(p)
            if p != 0 and p != prev:
                seq.append(p)
            prev = p
        out.append(seq)
    return out


def ids_to_text(seqs, itos):
    """alphabet[p-1] with alphabet = itos[1:] (training/utils.py:146)."""
    return ["".join(itos[1:][p - 1] for p in s) for s in seqs]


def adamw_step(p, g, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, wd=1e-2):
    """torch.optim.AdamW update (training/train.py:294-295 option), numpy float64."""
    p = p * (1 - lr * wd)
    m = beta1 * m + (1 - beta1) * g
    v = beta2 * v + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = np.sqrt(v) / math.sqrt(bc2) + eps
    p = p - (lr / bc1) * m / denom
    return p, m, v


def param_shapes(hidden: int, num_classes: int, num_rnn_layers: int = 2, enc_dim: int = 512
                 ) -> List[Tuple[str, Tuple[int, ...]]]:
    """Ordered (name, shape) of the CTC model's state dict (reference key order)."""
    out = []

    def conv(n, co, ci, kh, kw):
        out.append((n + ".weight", (co, ci, kh, kw)))

    def bn(n, c):
        out.extend([(n + ".weight", (c,)), (n + ".bias", (c,)), (n + ".running_mean", (c,)),
                    (n + ".running_var", (c,)), (n + ".num_batches_tracked", ())])

    conv("cnn.conv0.0", 64, 3, 3, 3); bn("cnn.conv0.1", 64)
    conv("cnn.conv0.3", 128, 64, 3, 3); bn("cnn.conv0.4", 128)
    for name, blocks, stride, inp, planes in STAGES:
        for i in range(blocks):
            pre = f"cnn.{name}.{i}"
            ci = inp if i == 0 else planes
            conv(pre + ".conv1", planes, ci, 3, 3); bn(pre + ".bn1", planes)
            conv(pre + ".conv2", planes, planes, 3, 3); bn(pre + ".bn2", planes)
            out.append((pre + ".se.fc.0.weight", (planes // 16, planes)))
            out.append((pre + ".se.fc.2.weight", (planes, planes // 16)))
            if i == 0 and (stride != 1 or inp != planes):
                conv(pre + ".downsample.0", planes, ci, 1, 1); bn(pre + ".downsample.1", planes)
    conv("cnn.conv_out.0", 512, 512, 2, 2); bn("cnn.conv_out.1", 512)
    conv("cnn.conv_out.3", 512, 512, 2, 2); bn("cnn.conv_out.4", 512)
    for l in range(num_rnn_layers):
        ind = enc_dim if l == 0 else hidden
        pre = f"enc_rnn.{l}"
        for sfx in ["", "_reverse"]:
            out.append((f"{pre}.rnn.weight_ih_l0{sfx}", (4 * hidden, ind)))
            out.append((f"{pre}.rnn.weight_hh_l0{sfx}", (4 * hidden, hidden)))
            out.append((f"{pre}.rnn.bias_ih_l0{sfx}", (4 * hidden,)))
            out.append((f"{pre}.rnn.bias_hh_l0{sfx}", (4 * hidden,)))
        out.append((f"{pre}.linear.weight", (hidden, 2 * hidden)))
        out.append((f"{pre}.linear.bias", (hidden,)))
    out.append(("ctc_head.weight", (num_classes, hidden)))
    out.append(("ctc_head.bias", (num_classes,)))
    return out
