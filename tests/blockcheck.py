"""Decision-consistent local parity for the HIP residual stages (test infrastructure).

Each SE-residual block (model/seresnet31.py:35-60 of the reference) is recomputed in fp64 from
the HIP path's OWN saved input tensor and upstream gradient, so ReLU / SE decisions are the HIP
path's and fp32 coin-flip ties (|pre-activation| ~ 1e-7, unavoidable in millions of decisions)
cannot move the comparison. What is left is each kernel's own rounding, ~1e-6 relative.

forward:  conv1 -> BN1(batch stats) -> ReLU -> conv2 -> BN2 -> SE -> (+ identity | BN(ds conv)) -> ReLU
backward: every parameter gradient of the block and d(block input).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _nchw(t, B, h, w, c):
    return t.reshape(B, h, w, c).double().cpu().permute(0, 3, 1, 2)


def _chan(t):
    return t.double().cpu()[None, :, None, None]


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-30))


def _bn_bwd(g, z, mean, inv, sc):
    xh = (z - _chan(mean)) * _chan(inv)
    db, dgm = g.sum(dim=(0, 2, 3)), (g * xh).sum(dim=(0, 2, 3))
    n = g.numel() / g.shape[1]
    dz = _chan(sc) * (g - (db / n)[None, :, None, None] - xh * (dgm / n)[None, :, None, None])
    return dz, dgm, db


def _bn_fwd(z, gamma, beta, eps=1e-5):
    mu, var = z.mean(dim=(0, 2, 3)), z.var(dim=(0, 2, 3), unbiased=False)
    return (z - mu[None, :, None, None]) / torch.sqrt(var + eps)[None, :, None, None] * _chan(gamma) + _chan(beta)


def block_errors(eng, params, grads):
    """-> list of (block index, {quantity: relative error}) for every residual block.

    eng: the CRNNEngine after forward(save_for_backward) + backward with eng.debug = True;
    params / grads: reference-named fp32 tensors (model parameters and their .grad)."""
    sv, dbg = eng._saved, eng.dbg
    P64 = {k: v.detach().double().cpu() for k, v in params.items()}
    G = {k: v.detach().double().cpu() for k, v in grads.items()}
    B = sv["B"]
    out = []
    for bi in reversed(range(len(eng.blocks))):
        blk, sb = eng.blocks[bi], sv["blocks"][bi]
        P, ho, wo, h, w = blk.planes, sb["ho"], sb["wo"], sb["h"], sb["w"]
        HW = ho * wo
        c1, c2 = blk.conv1, blk.conv2
        st, pd = (c1.sh, c1.sw), (c1.ph, c1.pw)
        xin = _nchw(sb["x"], B, h, w, c1.ci)[:, : c1.ci_real]
        y = _nchw(sb["y"], B, ho, wo, P)
        z1, z2 = _nchw(sb["z1"], B, ho, wo, P), _nchw(sb["z2"], B, ho, wo, P)
        a1 = _nchw(sb["a1"], B, ho, wo, P)
        s, hid, pooled = (sb[k].double().cpu() for k in ("s", "hid", "pooled"))
        w1, w2 = P64[blk.prefix + ".se.fc.0.weight"], P64[blk.prefix + ".se.fc.2.weight"]
        cw1, cw2 = P64[c1.name], P64[c2.name]
        e = {}
        # ---- forward, each stage from the HIP tensor feeding it
        e["fwd.z1"] = rel(z1, F.conv2d(xin, cw1, stride=st, padding=pd))
        a1r = torch.relu(_bn_fwd(z1, P64[c1.bn + ".weight"], P64[c1.bn + ".bias"]))
        e["fwd.a1"] = rel(a1, a1r)
        e["fwd.z2"] = rel(z2, F.conv2d(a1, cw2, padding=1))
        u2 = _bn_fwd(z2, P64[c2.bn + ".weight"], P64[c2.bn + ".bias"])
        sr = torch.sigmoid(torch.relu(u2.mean(dim=(2, 3)) @ w1.t()) @ w2.t())
        e["fwd.se"] = rel(s, sr)
        if blk.ds is None:
            idn = xin
        else:
            ds = blk.ds
            zd = _nchw(sb["ds"]["zd"], B, ho, wo, P)
            idn = _bn_fwd(zd, P64[ds.bn + ".weight"], P64[ds.bn + ".bias"])
        e["fwd.y"] = rel(y, torch.relu(u2 * s[:, :, None, None] + idn))
        # ---- backward from the HIP upstream gradient
        gy = _nchw(dbg[f"dy.b{bi}"], B, ho, wo, P) * (y > 0)
        u2h = z2 * _chan(sb["sc2"]) + _chan(sb["sh2"])
        dsig = (gy * u2h).sum(dim=(2, 3)) * s * (1 - s)
        dh = (dsig @ w2) * (hid > 0)
        e["se.fc.2"] = rel(G[blk.prefix + ".se.fc.2.weight"], dsig.t() @ hid)
        e["se.fc.0"] = rel(G[blk.prefix + ".se.fc.0.weight"], dh.t() @ pooled)
        g2 = gy * s[:, :, None, None] + ((dh @ w1) / HW)[:, :, None, None]
        dz2, dg2, db2 = _bn_bwd(g2, z2, sb["m2"], sb["i2"], sb["sc2"])
        e["bn2.weight"], e["bn2.bias"] = rel(G[c2.bn + ".weight"], dg2), rel(G[c2.bn + ".bias"], db2)
        e["conv2"] = rel(G[c2.name], torch.nn.grad.conv2d_weight(a1, cw2.shape, dz2, stride=1, padding=1))
        da1 = torch.nn.grad.conv2d_input(a1.shape, cw2, dz2, stride=1, padding=1)
        dz1, dg1, db1 = _bn_bwd(da1 * (a1 > 0), z1, sb["m1"], sb["i1"], sb["sc1"])
        e["bn1.weight"], e["bn1.bias"] = rel(G[c1.bn + ".weight"], dg1), rel(G[c1.bn + ".bias"], db1)
        e["conv1"] = rel(G[c1.name], torch.nn.grad.conv2d_weight(xin, cw1.shape, dz1, stride=st, padding=pd))
        dx = torch.nn.grad.conv2d_input(xin.shape, cw1, dz1, stride=st, padding=pd)
        if blk.ds is None:
            dx = dx + gy
        else:
            dsv = sb["ds"]
            dzd, dgd, dbd = _bn_bwd(gy, zd, dsv["m"], dsv["i"], dsv["sc"])
            sd_, pd_ = (ds.sh, ds.sw), (ds.ph, ds.pw)
            cwd = P64[ds.name]
            e["ds.bn.weight"], e["ds.bn.bias"] = rel(G[ds.bn + ".weight"], dgd), rel(G[ds.bn + ".bias"], dbd)
            e["ds.conv"] = rel(G[ds.name], torch.nn.grad.conv2d_weight(xin, cwd.shape, dzd, stride=sd_, padding=pd_))
            dx = dx + torch.nn.grad.conv2d_input(xin.shape, cwd, dzd, stride=sd_, padding=pd_)
        if bi > 0:
            e["dx"] = rel(_nchw(dbg[f"dy.b{bi - 1}"], B, h, w, c1.ci)[:, : c1.ci_real], dx)
        out.append((bi, e))
    return out


def _fma_pos(z, sc, sh):
    """sign of the kernels' fp32 fma(z, sc, sh): z*sc is exact in fp64 and rounding keeps signs."""
    return (z.double() * sc.double() + sh.double()) > 0


def hip_decisions(eng):
    """The HIP forward's ReLU / max-pool decisions, NCHW, by oracle decision-site name
    (crnn_oracle.relu / maxpool2), from the engine's saved forward tensors."""
    sv = eng._saved
    B = sv["B"]
    cpu = lambda t: t.detach().cpu()
    perm = lambda t: t.permute(0, 3, 1, 2)
    f = {}
    st = sv["stem"]
    f["cnn.conv0.1"] = perm(cpu(st["a0"]) > 0)
    z1 = cpu(st["z1"]).reshape(B, st["h1"], st["w1"], -1)
    sc1, sh1 = cpu(st["sc1"]), cpu(st["sh1"])
    pos = _fma_pos(z1, sc1, sh1)
    f["cnn.conv0.4"] = perm(pos)
    # the pool kernel: first strict max of relu(fp32 fma) over t = 2*dh + dw
    v = torch.where(pos, (z1.double() * sc1.double() + sh1.double()).float(), torch.zeros(()))
    Hh, Wh = st["h1"] // 2, st["w1"] // 2
    win = v.reshape(B, Hh, 2, Wh, 2, -1).permute(0, 1, 3, 2, 4, 5).reshape(B, Hh, Wh, 4, -1)
    best = torch.full(win[:, :, :, 0].shape, -float("inf"))
    arg = torch.zeros(best.shape, dtype=torch.long)
    for t in range(4):
        gt = win[:, :, :, t] > best
        best = torch.where(gt, win[:, :, :, t], best)
        arg = torch.where(gt, torch.full_like(arg, t), arg)
    f["stem.pool"] = perm(arg)
    for blk, sb in zip(eng.blocks, sv["blocks"]):
        f[blk.prefix + ".bn1"] = perm(cpu(sb["a1"]).reshape(B, sb["ho"], sb["wo"], -1) > 0)
        f[blk.prefix + ".se"] = cpu(sb["hid"]) > 0
        f[blk.prefix + ".out"] = perm(cpu(sb["y"]).reshape(B, sb["ho"], sb["wo"], -1) > 0)
        if sb.get("drop") is not None:   # DropBlock2d's multiplier (crnn_oracle.se_block)
            import crnn_oracle as O
            f[blk.prefix + ".dropblock"] = O.dropblock_mult(perm(cpu(sb["drop"]["keep"])).numpy())
    co = sv["co"]
    f["cnn.conv_out.1"] = perm(cpu(co["a0"]).reshape(B, co["h2"], co["w2"], -1) > 0)
    zc = cpu(co["z1"]).reshape(B, co["h3"], co["w3"], -1)
    f["cnn.conv_out.4"] = perm(_fma_pos(zc, cpu(co["sc1"]), cpu(co["sh1"])))
    return f
