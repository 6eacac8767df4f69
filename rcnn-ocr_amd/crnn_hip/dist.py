"""Data parallelism for the CRNN step: one process per GPU, RCCL over xGMI.

The path shards by sample: every rank runs the full train step on its own
batch shard; BatchNorm uses per-rank batch statistics (the reference's plain BatchNorm2d,
no SyncBN). The only exchange is a sum all-reduce of the flat fp32 gradient buffer; the
optimizer then scales by 1/world. Parameters are broadcast from rank 0 once at start.

Overlap (OverlappedAllReduce): the flat buffer is laid out in parameter order (stem first, CTC
head last) and the backward finalises gradients from the end of it towards the start, stage by
stage (CRNNEngine.backward's stage_done hook). Each time the final region grows by at least
min_bucket bytes its new part is all-reduced asynchronously on RCCL's stream while the backward
kernels of the earlier layers keep running; finish() issues the remainder and makes the compute
stream wait for every collective before the optimizer step.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

BUCKET_BYTES = 32 << 20


def env_world():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_from_env(backend: Optional[str] = None):
    """init_process_group from torchrun's env (MASTER_ADDR/PORT, RANK, WORLD_SIZE);
    backend 'nccl' (= RCCL on ROCm) for HIP devices, 'gloo' for CPU tests."""
    world, rank, local = env_world()
    if os.environ.get("CRNN_SHARE_DEVICE") == "1":   # rehearsal only: every rank on device 0
        local = 0
    if world <= 1 or dist.is_initialized():
        return world, rank, local
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if backend is None:
        backend = os.environ.get("CRNN_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return world, rank, local


def buckets(n: int, elem_bytes: int = 4, bucket_bytes: int = BUCKET_BYTES) -> List[slice]:
    per = max(1, bucket_bytes // elem_bytes)
    return [slice(i, min(n, i + per)) for i in range(0, n, per)]


def broadcast_params(flat: torch.Tensor, src: int = 0):
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(flat, src)


def allreduce_grads(flat_grad: torch.Tensor, bucket_bytes: int = BUCKET_BYTES):
    """sum all-reduce of a flat gradient buffer in reverse-order buckets (the head / LSTM
    gradients live at the end of the buffer and are final first), all in flight together."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return
    works = [dist.all_reduce(flat_grad[s], async_op=True)
             for s in reversed(buckets(flat_grad.numel(), flat_grad.element_size(), bucket_bytes))]
    for w in works:
        w.wait()


class OverlappedAllReduce:
    """bucketed sum all-reduce of a flat gradient buffer, overlapped with the backward: call
    ready(prefixes) from CRNNEngine.backward's stage_done hook, then finish().

    Readiness is tracked per parameter: the issuable region is the longest SUFFIX of the buffer
    whose parameters have all been reported final, whatever order the stages report in (a stage
    that finishes out of layout order just waits until everything after it is final). Each issued
    bucket is recorded in `issued` as (lo, hi) for tests."""

    def __init__(self, flat_grad: torch.Tensor, offsets, min_bucket_bytes: int = 8 << 20, timing: bool = False):
        """offsets: {param name: (start, numel)} into flat_grad (the model's flat layout).
        timing: finish() brackets the compute stream's wait for the collectives with HIP events
        (exposed_ms_per_step(): the all-reduce time the backward did not hide)."""
        self.flat = flat_grad
        self.offsets = offsets
        spans = sorted((s, s + n, k) for k, (s, n) in offsets.items())
        pos = 0
        for s, e, k in spans:
            if s != pos:
                raise ValueError(f"offsets must tile the flat buffer contiguously (gap / overlap at {k})")
            pos = e
        if pos != flat_grad.numel():
            raise ValueError("offsets do not cover the flat buffer")
        self.spans = spans
        self.min_elems = max(1, min_bucket_bytes // flat_grad.element_size())
        self.active = dist.is_initialized() and dist.get_world_size() > 1
        self.issued = []
        self.last_issued = []
        self.stream = None   # the collective stream (HIP tensors)
        self.timing = timing and flat_grad.is_cuda
        self.wait_events = []   # (start, end) per finish() with timing
        self.reset()

    def reset(self):
        self.last_issued, self.issued = self.issued, []
        self.done = set()                # parameter names reported final
        self.cursor = len(self.spans)    # spans[cursor:] are final (a suffix)
        self.hi = self.flat.numel()      # [hi, end) already issued
        self.works = []

    @property
    def lo(self) -> int:
        """start of the final suffix"""
        return self.spans[self.cursor][0] if self.cursor < len(self.spans) else self.flat.numel()

    def ready(self, prefixes):
        for k in self.offsets:
            if any(k.startswith(p) for p in prefixes):
                self.done.add(k)
        while self.cursor > 0 and self.spans[self.cursor - 1][2] in self.done:
            self.cursor -= 1
        if self.active and self.hi - self.lo >= self.min_elems:
            self._issue(self.lo, self.hi)

    def _issue(self, lo, hi):
        """all-reduce flat[lo:hi] on the collective stream, after the work the caller's (compute)
        stream has enqueued so far: an explicit event edge, not the process group's notion of the
        calling thread's current stream (the hooks run on the autograd thread; without the edge a
        bucket was occasionally read before its last gradient kernel had finished,
        tests/test_gpu_dp.py)"""
        self.issued.append((lo, hi))
        if self.flat.is_cuda:
            cur = torch.cuda.current_stream(self.flat.device)
            if self.stream is None:
                self.stream = torch.cuda.Stream(self.flat.device)
            ev = torch.cuda.Event()
            ev.record(cur)
            self.stream.wait_event(ev)
            with torch.cuda.stream(self.stream):
                self.works.append(dist.all_reduce(self.flat[lo:hi], async_op=True))
        else:
            self.works.append(dist.all_reduce(self.flat[lo:hi], async_op=True))
        self.hi = lo

    def finish(self):
        """issue what is left (everything must be final by now) and make the caller's stream wait"""
        if self.active:
            if self.hi > 0:
                missing = [k for _, _, k in self.spans[:self.cursor] if k not in self.done]
                if missing:
                    raise RuntimeError(f"finish(): gradients never reported final: {missing[:4]}")
                self._issue(0, self.hi)
            ev = None
            if self.timing:   # before the waits: a wait() may already order the caller's stream
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(torch.cuda.current_stream(self.flat.device))
            for w in self.works:
                w.wait()   # makes the collective stream wait for the collectives' completion
            if self.stream is not None:   # and the caller's stream for the collective stream
                torch.cuda.current_stream(self.flat.device).wait_stream(self.stream)
            if ev is not None:
                ev[1].record(torch.cuda.current_stream(self.flat.device))
                self.wait_events.append(ev)
        self.reset()

    def exposed_ms_per_step(self) -> float:
        """mean over the recorded finish() calls of the compute stream's wait for the collectives (ms);
        synchronise first"""
        if not self.wait_events:
            return 0.0
        return sum(a.elapsed_time(b) for a, b in self.wait_events) / len(self.wait_events)

    def last_bucket_bytes(self):
        return [(hi - lo) * self.flat.element_size() for lo, hi in self.last_issued]

    def buckets_per_step(self):
        """(bucket count, bytes) of the last completed step"""
        b = self.last_bucket_bytes()
        return len(b), sum(b)
