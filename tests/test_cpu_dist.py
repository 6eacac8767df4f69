"""world_size-2 and -4 gloo tests of the data-parallel glue (crnn_hip/dist.py) on CPU.

The HIP compute path has no CPU fallback, so these exercise what DP adds on top of it:
the bucketed gradient all-reduce and the parameter broadcast, and check the DP identity on
the oracle's train step: averaging per-rank gradients of a BN-free sub-network equals the
single-process gradient of the concatenated batch."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for sub in ("../rcnn-ocr_amd", "../oracle"):
        sys.path.insert(0, os.path.join(here, sub))
    from crnn_hip import dist as D
    D.init_from_env("gloo")
    try:
        # bucketed all-reduce: tiny buckets force many collectives in flight
        tri = world * (world + 1) // 2   # sum over ranks of (rank + 1)
        g = torch.arange(1000, dtype=torch.float32) * (rank + 1)
        D.allreduce_grads(g, bucket_bytes=4 * 37)
        ok_sum = torch.allclose(g, torch.arange(1000, dtype=torch.float32) * tri)
        # broadcast from rank 0
        p = torch.full((17,), float(rank + 5))
        D.broadcast_params(p)
        ok_bc = bool((p == 5).all())
        # DP identity on the oracle's BiLSTM + head (no BN): mean of rank grads == full-batch grad
        import crnn_oracle as O
        from crnn_hip.recipe import recipe_state_dict
        torch.manual_seed(0)
        shapes = [(k, s) for k, s in O.param_shapes(16, 10, 1, enc_dim=24) if k.startswith(("enc_rnn", "ctc_head"))]
        sd = recipe_state_dict(shapes, 7)
        gen = torch.Generator().manual_seed(3)
        x = torch.randn(2 * world, 6, 24, generator=gen)
        tg = torch.randint(1, 10, (2 * world, 3), generator=gen)
        tl = torch.tensor([3, 2, 1, 3] * ((world + 1) // 2))[: 2 * world]

        def grads(xs, ts, ls):
            p = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
            lg = O.head(O.bilstm(xs, p, "enc_rnn.0"), p)
            # sum-reduction makes the per-sample decomposition exact
            O.ctc_loss(lg, ts, ls, reduction="sum").backward()
            return torch.cat([p[k].grad.reshape(-1) for k, _ in shapes])

        full = grads(x, tg, tl)
        part = grads(x[2 * rank:2 * rank + 2], tg[2 * rank:2 * rank + 2], tl[2 * rank:2 * rank + 2])
        D.allreduce_grads(part)
        ok_dp = torch.allclose(part, full, rtol=1e-4, atol=1e-5)
        # overlapped reducer: stage-wise readiness in backward order, every element reduced exactly once
        offs = {"cnn.conv0.0.weight": (0, 100), "cnn.layer1.0.conv1.weight": (100, 300),
                "cnn.conv_out.0.weight": (400, 200), "enc_rnn.0.linear.weight": (600, 300),
                "ctc_head.weight": (900, 100)}
        ok_ov = True
        for mb in (4, 4 * 250, 4 * 5000):   # every stage its own bucket / merged / all at finish()
            g2 = torch.arange(1000, dtype=torch.float32) * (rank + 1)
            red = D.OverlappedAllReduce(g2, offs, min_bucket_bytes=mb)
            for pre in (["ctc_head.", "enc_rnn."], ["cnn.conv_out."], ["cnn.layer1.0."], ["cnn.conv0."]):
                red.ready(pre)
            red.finish()
            ok_ov = ok_ov and torch.allclose(g2, torch.arange(1000, dtype=torch.float32) * tri)
        # the REAL layout and stage order: RCNN.flat_offsets() and CRNNEngine.backward_stages() (the
        # sequence backward() reports), in order and shuffled; buckets must tile the buffer exactly
        # once, each issued only once all of its parameters were reported final
        from crnn_hip.engine import CRNNEngine
        from model.model import RCNN
        offs = RCNN(num_classes=10, hidden_size=16).flat_offsets()
        n = sum(k for _, k in offs.values())
        stages = CRNNEngine.backward_stages()
        covered = set()
        for st in stages:
            covered |= {k for k in offs if any(k.startswith(p) for p in st)}
        ok_real = covered == set(offs)
        orders = [stages, list(reversed(stages)), stages[:3] + stages[5:] + stages[3:5]]
        for order in orders:
            for mb in (4, 4 << 20, 1 << 40):
                g3 = torch.ones(n) * (rank + 1)
                red = D.OverlappedAllReduce(g3, offs, min_bucket_bytes=mb)
                seen = []
                for st in order:
                    red.ready(st)
                    seen += [k for k in offs if any(k.startswith(p) for p in st)]
                    for lo, hi in red.issued:   # every bucket so far holds only reported parameters
                        ok_real = ok_real and all(k in seen for k, (s0, c) in offs.items() if s0 < hi and s0 + c > lo)
                red.finish()
                spans = sorted(red.last_issued)
                ok_real = ok_real and spans[0][0] == 0 and spans[-1][1] == n and all(
                    a[1] == b[0] for a, b in zip(spans, spans[1:]))
                ok_real = ok_real and bool((g3 == tri).all())
        # per-replica dropout streams: the engine's mask seed differs across ranks for the same torch seed
        from crnn_hip.engine import dropout_seed
        seeds = [None] * world
        dist.all_gather_object(seeds, dropout_seed(1234))
        ok_drop = len(set(seeds)) == world
        q.put((rank, ok_sum, ok_bc, ok_dp and ok_ov and ok_real and ok_drop))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_allreduce_broadcast_and_dp_identity(world):
    """world 2 and world 4: bucketed sum, broadcast, the DP identity on the oracle's
    BiLSTM + head, and the overlapped reducer's bucket tiling on the model's real layout and stage order"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] and r[2] and r[3] for r in res), res


def test_buckets_cover_buffer():
    from crnn_hip.dist import buckets
    bs = buckets(1003, 4, 40)
    assert bs[0] == slice(0, 10) and bs[-1].stop == 1003
    assert sum(s.stop - s.start for s in bs) == 1003


def test_dropout_seed_single_process_is_torch_seed():
    """without a process group the enc_dropout mask seed is torch's initial seed (masks unchanged)"""
    from crnn_hip.engine import dropout_seed
    assert dropout_seed(1234) == 1234
    assert dropout_seed(-1) == 0xFFFFFFFFFFFFFFFF
