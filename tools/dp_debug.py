"""Bisect a data-parallel gradient mismatch (tests/test_gpu_dp.py): two ranks share the one GPU
(gloo over device tensors). Per rank: the local gradient of the same step three times (plain,
plain, plain after a reducer-driven step), and the reduced gradient with the overlapped reducer
driven by the stage hooks, with a device sync inside each hook, and with everything issued at
finish() only. Prints, per variant, the max relative difference against the host-summed local
gradient and the parameters it falls in.
    python tools/dp_debug.py"""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _where(diff, offsets, ref=None, top=4):
    """(count, top params by max |diff| relative to the reference gradient's max)"""
    out = []
    for k, (s, n) in offsets.items():
        d = float(diff[s:s + n].abs().max())
        if d > 0:
            den = float(ref[s:s + n].abs().max()) if ref is not None else 1.0
            out.append((round(d / (den + 1e-30), 6), k))
    return len(out), sorted(out, reverse=True)[:top]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), CRNN_SHARE_DEVICE="1", CRNN_LSTM_PER_STEP="1",
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    for sub in ("rcnn-ocr_amd", "oracle"):
        sys.path.insert(0, os.path.join(REPO, sub))
    import torch.distributed as dist
    lines = []
    try:
        import crnn_oracle as O
        from crnn_hip import dist as D
        from crnn_hip.ctc import ctc_loss
        from crnn_hip.optim import FusedAdamW
        from crnn_hip.recipe import recipe_state_dict, synthetic_batch
        from model.model import RCNN
        D.init_from_env("gloo")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        m = RCNN(num_classes=194, hidden_size=64, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
        m.load_state_dict(recipe_state_dict(O.param_shapes(64, 194), 5 + rank), strict=False)
        m = m.to(dev).train()
        x, _, tg, tl = synthetic_batch(16, 32, 128, 16, 194, seed=100 + rank)
        x = x.to(dev)
        m(x)
        D.broadcast_params(m._flat_param)
        m.mark_params_changed()
        opt = FusedAdamW(m, lr=1e-3)
        offs = m.flat_offsets()

        def local():
            m.stage_done = None
            opt.zero_grad()
            ctc_loss(m(x), tg, tl).backward()
            torch.cuda.synchronize()
            return m._flat_grad.detach().cpu().clone()

        g1 = local()
        for i in range(6):
            g2 = local()
            lines.append(f"rank {rank}: local step {i + 2} vs 1: {_where(g2 - g1, offs, g1)}")
        want = g1.clone()
        dist.all_reduce(want)
        scale = float(want.abs().max()) + 1e-30

        def reduced(mode):
            red = D.OverlappedAllReduce(m._flat_grad, offs,
                                        min_bucket_bytes=(1 << 40) if mode == "finish_only" else 1 << 20)

            def hook(prefixes):
                if mode == "sync_hook":
                    torch.cuda.synchronize()
                red.ready(prefixes)
            m.stage_done = hook
            opt.zero_grad()
            ctc_loss(m(x), tg, tl).backward()
            red.finish()
            torch.cuda.synchronize()
            m.stage_done = None
            got = m._flat_grad.detach().cpu().clone()
            d = got - want
            return (f"rank {rank}: {mode:12s} buckets {len(red.last_issued):2d} rel err {float(d.abs().max()) / scale:.3e} "
                    f"{_where(d, offs)}")

        for mode in ("overlap", "sync_hook", "finish_only", "overlap"):
            lines.append(reduced(mode))
        for i in range(4):
            g3 = local()
            lines.append(f"rank {rank}: local step after reducer steps vs 1: {_where(g3 - g1, offs, g1)}")
        q.put((rank, lines, None))
    except Exception:
        import traceback
        q.put((rank, lines, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def main():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=200) for _ in ps), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=30)
    for rank, lines, err in res:
        for ln in lines:
            print(ln, flush=True)
        if err:
            print(err, flush=True)


if __name__ == "__main__":
    main()
