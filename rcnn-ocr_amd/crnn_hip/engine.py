"""CRNN hot-path engine: forward / backward of SE-ResNet31 -> BiLSTM -> CTC head
over libcrnn_hip.so. PyTorch supplies device memory and the stream only.

Reference path (sherstpasha/RCNN-OCR):
  SEResNet31.forward          model/seresnet31.py:180-187
  SEBasicBlock.forward        model/seresnet31.py:55-67
  RCNN.encode                 model/model.py:215-221
  BidirectionalLSTM.forward   model/model.py:159-163
  + CTC head Linear(H -> C)

Data layout in HBM (all activations NHWC, compute dtype T = bf16 | fp32):
  input crop  [B][H][W][8]   (3 channels zero-padded to 8)
  conv output z (pre-BN)     saved for BN backward; BN+ReLU outputs are
                             recomputed from z wherever a kernel can fuse it
  sequence    [B][T][512]    == conv_out output [B][1][T][512] (no permute)
  LSTM        xg [B][T][2][4H], hseq [B][T][2H], gates [2][T][B][4H], c [2][T][B][H] fp32
  logits      [B*T][Cpad] fp32 (Cpad = C rounded up to 8, zero columns)
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from . import _lib as L
from ._lib import BnBwdDesc, ConvDesc, call, ptr

BN_EPS = 1e-5
BN_MOMENTUM = 0.1

# (stage, blocks, stride, inplanes, planes) — model/seresnet31.py:92-127
STAGES = [("layer1", 1, 2, 128, 256), ("layer2", 2, 1, 256, 256),
          ("layer3", 5, 2, 256, 512), ("layer4", 3, 1, 512, 512)]


def dropout_seed(base: int) -> int:
    """the engine's dropout mask stream seed: torch's initial seed, with the data-parallel rank mixed in
    when a process group of more than one rank is up (run_training seeds every rank alike, so without the
    rank the replicas would draw identical masks, unlike independent per-replica dropout)"""
    seed = base & 0xFFFFFFFFFFFFFFFF
    import torch.distributed as tdist
    if tdist.is_available() and tdist.is_initialized() and tdist.get_world_size() > 1:
        seed ^= ((tdist.get_rank() + 1) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return seed


def round8(n: int) -> int:
    return (n + 7) // 8 * 8


@dataclass
class ConvSpec:
    name: str          # weight key
    bn: str            # BN prefix
    ci: int            # stored input channels
    ci_real: int
    co: int
    kh: int
    kw: int
    sh: int
    sw: int
    ph: int
    pw: int

    def out_hw(self, h, w):
        return (h + 2 * self.ph - self.kh) // self.sh + 1, (w + 2 * self.pw - self.kw) // self.sw + 1

    def desc(self, b, h, w) -> ConvDesc:
        ho, wo = self.out_hw(h, w)
        return ConvDesc(b, h, w, self.ci, ho, wo, self.co, self.kh, self.kw, self.sh, self.sw,
                        self.ph, self.pw, self.ci_real)


@dataclass
class BlockSpec:
    prefix: str
    conv1: ConvSpec
    conv2: ConvSpec
    ds: Optional[ConvSpec]
    planes: int


def backbone_specs():
    stem0 = ConvSpec("cnn.conv0.0.weight", "cnn.conv0.1", 8, 3, 64, 3, 3, 1, 1, 1, 1)
    stem1 = ConvSpec("cnn.conv0.3.weight", "cnn.conv0.4", 64, 64, 128, 3, 3, 1, 1, 1, 1)
    blocks: List[BlockSpec] = []
    for name, nblk, stride, inp, planes in STAGES:
        for i in range(nblk):
            s = stride if i == 0 else 1
            ci = inp if i == 0 else planes
            pre = f"cnn.{name}.{i}"
            c1 = ConvSpec(pre + ".conv1.weight", pre + ".bn1", ci, ci, planes, 3, 3, s, s, 1, 1)
            c2 = ConvSpec(pre + ".conv2.weight", pre + ".bn2", planes, planes, planes, 3, 3, 1, 1, 1, 1)
            ds = None
            if i == 0 and (stride != 1 or inp != planes):
                ds = ConvSpec(pre + ".downsample.0.weight", pre + ".downsample.1", ci, ci, planes, 1, 1,
                              s, s, 0, 0)
            blocks.append(BlockSpec(pre, c1, c2, ds, planes))
    co0 = ConvSpec("cnn.conv_out.0.weight", "cnn.conv_out.1", 512, 512, 512, 2, 2, 2, 1, 0, 1)
    co1 = ConvSpec("cnn.conv_out.3.weight", "cnn.conv_out.4", 512, 512, 512, 2, 2, 1, 1, 0, 0)
    return stem0, stem1, blocks, co0, co1


def gate_perm(H: int) -> List[int]:
    """packed row 4j+q <- reference row q*H+j (i,f,g,o interleaved per unit)."""
    return [q * H + j for j in range(H) for q in range(4)]


class Workspace:
    """Named device buffers, (re)allocated only when a shape changes: a step
    at a fixed batch geometry allocates nothing (hipGraph-capturable)."""

    def __init__(self, device):
        self.device = device
        self.bufs: Dict[str, torch.Tensor] = {}

    def get(self, name, shape, dtype) -> torch.Tensor:
        shape = tuple(int(s) for s in shape)
        t = self.bufs.get(name)
        if t is None or t.shape != shape or t.dtype != dtype:
            t = torch.empty(shape, dtype=dtype, device=self.device)
            self.bufs[name] = t
        return t

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in self.bufs.values())


_SEQ_TIMEOUT_MSG = ("persistent BiLSTM sweep timed out waiting for a co-resident workgroup (error word set; "
                    "its outputs are NaN): the grid was not fully resident on the device")


class CRNNEngine:
    def __init__(self, params: Dict[str, torch.Tensor], buffers: Dict[str, torch.Tensor], hidden: int,
                 num_classes: int, num_rnn_layers: int = 2, dtype: torch.dtype = torch.bfloat16,
                 enc_dim: int = 512, version_source=None):
        self.p = params
        self.buf = buffers
        self.H = hidden
        self.C = num_classes
        self.Cpad = round8(num_classes)
        # RCNN(decoder="attn") has no CTC head (the reference's parameter set): the encoder ends at
        # enc_dropout and forward() returns None
        self.has_head = "ctc_head.weight" in params
        self.nl = num_rnn_layers
        self.enc_dim = enc_dim
        self.dtype = dtype
        self.dt = L.dtype_code(dtype)
        any_p = next(iter(params.values()))
        self.device = any_p.device
        L.require_device(any_p)
        L.lib()
        self.stem0, self.stem1, self.blocks, self.co0, self.co1 = backbone_specs()
        self.ws = Workspace(self.device)
        self.packed: Dict[str, torch.Tensor] = {}
        self.perm = torch.tensor(gate_perm(hidden), dtype=torch.int32, device=self.device)
        self.packed_version = None
        self._pack_jobs = None
        self.version = 0
        # in-place edits of the parameters (torch optimizers, load_state_dict) bump the
        # flat buffer's version counter; kernel-side updates call mark_params_changed()
        self.version_source = version_source
        self._saved = None
        # forward generation: the engine keeps ONE set of saved activations, so a backward must
        # belong to the latest grad-enabled forward (checked by saved_generation())
        self.fwd_gen = 0
        # persistent BiLSTM status (see poll_status)
        self._seq_used = False
        self._sticky_carry = 0
        self._sticky_index = 0      # int32 index of the status word in rnn.seq_ws (set with the buffer)
        self._status_host = None
        self._status_evt = None
        self._cur_ver = None
        self._eval_affine: Dict[str, tuple] = {}   # BN tag -> version key of its cached eval affine
        self._side = None           # side stream of the running backward (wgrad_stream)
        self._rside = None          # ... or of its conv wgrad slab reduces (wgrad_reduce_stream)
        self._slab_i, self._slab_ev = 0, [None, None]
        self._side_stream = None
        self.debug = False      # when set, backward keeps copies of block-boundary gradients
        self._last_partials = None  # (psum, rows, rows_per_partial) of the latest training-mode conv
        self._drop_seed = dropout_seed(int(torch.initial_seed()))  # enc_dropout mask stream (per replica)
        self._drop_calls = 0
        self.dbg: Dict[str, torch.Tensor] = {}

    # ------------------------------------------------------------------ weights
    def mark_params_changed(self):
        """call after editing parameters or BN buffers in a way torch's version counters do not see
        (kernel-side updates, writes through `.data`): the packed weights and the cached eval
        affines are rebuilt at the next forward."""
        self.version += 1
        self._eval_affine.clear()

    def convs(self):
        yield self.stem0
        yield self.stem1
        for b in self.blocks:
            yield b.conv1
            yield b.conv2
            if b.ds is not None:
                yield b.ds
        yield self.co0
        yield self.co1

    def tw_convs(self):
        """the convs whose input gradient can run on the forward path (crnn_conv_dgrad_tw): bf16,
        stride 1, KH*KW in (1, 4, 9), Co % 64 == 0, unpadded Ci % 16 == 0; not the stem (halo kernels)"""
        if not self.dgrad_tw or self.dtype != torch.bfloat16:
            return []
        return [cs for cs in self.convs() if cs not in (self.stem0, self.stem1) and cs.sh == 1 and cs.sw == 1
                and cs.kh * cs.kw in (1, 4, 9) and cs.co % 64 == 0 and cs.ci % 16 == 0 and cs.ci == cs.ci_real]

    def _dgrad(self, cs: "ConvSpec", b, h, w, dy, dx, dres=None, yres=None, accumulate=0):
        """input gradient of conv `cs` (input map h x w): the forward-path form where packed and
        supported, else the native dgrad kernels"""
        d = cs.desc(b, h, w)
        wt = self.packed.get(cs.name + ".t")
        fl = self.conv_flops(cs, b, h, w)
        if wt is not None and L.lib().crnn_conv_dgrad_tw_rows(self.dt, d) > 0:
            self._conv_call("dgrad", fl, "crnn_conv_dgrad_tw", self.dt, d, ptr(dy), ptr(wt), ptr(dx), ptr(dres),
                            ptr(yres), accumulate, L.stream_ptr())
        else:
            self._conv_call("dgrad", fl, "crnn_conv_dgrad", self.dt, d, ptr(dy), ptr(self.packed[cs.name]), ptr(dx),
                            ptr(dres), ptr(yres), accumulate, L.stream_ptr())

    def pack(self):
        """fp32 reference-layout parameters -> compute-dtype kernel layouts: every weight in one
        crnn_pack_batch launch (job table built once; all pointers are persistent views)."""
        ver = (self.version, self.version_source() if self.version_source is not None else 0)
        self._cur_ver = ver
        if self.packed_version == ver:
            return
        if self._pack_jobs is None:
            self._build_pack_jobs()
        (cjobs, cn, crows, cslab), (jobs, n, total), (tjobs, tn, ttiles) = self._pack_jobs
        call("crnn_pack_conv_batch", self.dt, ptr(cjobs), cn, crows, cslab, L.stream_ptr())
        call("crnn_pack_batch", self.dt, ptr(jobs), n, total, L.stream_ptr())
        if tn:
            call("crnn_pack_conv_t_batch", self.dt, ptr(tjobs), tn, ttiles, L.stream_ptr())
        self.packed_version = ver

    def _build_pack_jobs(self):
        T, H = self.dtype, self.H
        jobs = []

        def job(kind, src, dst, a, b, c, d=0, e=0, out_f32=False, perm=None, src2=None):
            jobs.append(L.PackJob(kind, 1 if out_f32 else 0, a, b, c, d, e, 0, 0, ptr(src), ptr(src2), ptr(perm),
                                  ptr(dst)))
            return dst.numel()

        sizes = []
        # a strided block's conv1 and downsample weights back to back (crnn_conv_dgrad_ds reads the
        # downsample's [Co][Ci] rows right after conv1's)
        for blk in self.blocks:
            if blk.ds is not None and blk.conv1.name not in self.packed:
                c1, ds = blk.conv1, blk.ds
                n1 = c1.co * c1.kh * c1.kw * c1.ci
                cat = torch.empty(n1 + ds.co * ds.kh * ds.kw * ds.ci, dtype=T, device=self.device)
                self.packed[c1.name] = cat[:n1].view(c1.co, c1.kh, c1.kw, c1.ci)
                self.packed[ds.name] = cat[n1:].view(ds.co, ds.kh, ds.kw, ds.ci)
        # conv weights: their own launch, one block per output channel (crnn_pack_conv_batch); the
        # convs with a transposed pack get their OHWI pack from that kernel's tiles (dst2, below)
        tw = self.tw_convs()
        rows, slab = 0, 0
        for cs in self.convs():
            if any(cs is t for t in tw):
                continue
            out = self._pbuf(cs.name, (cs.co, cs.kh, cs.kw, cs.ci), T)
            job(L.PACK_CONV, self.p[cs.name], out, cs.co, cs.ci_real, cs.kh, cs.kw, cs.ci)
            jobs[-1].start = rows
            rows += cs.co
            slab = max(slab, cs.ci_real * cs.kh * cs.kw)
        carr = (L.PackJob * len(jobs))(*jobs)
        craw = torch.frombuffer(bytearray(bytes(carr)), dtype=torch.uint8).to(self.device)
        conv_tab = (craw, len(jobs), rows, slab)
        jobs.clear()
        # transposed, flipped kernels [Ci][KH][KW][Co] of the stride-1 convs (crnn_conv_dgrad_tw)
        tiles = 0
        for cs in tw:
            out = self._pbuf(cs.name + ".t", (cs.ci, cs.kh, cs.kw, cs.co), T)
            job(L.PACK_CONV_T, self.p[cs.name], out, cs.co, cs.ci, cs.kh, cs.kw)
            jobs[-1].dst2 = ptr(self._pbuf(cs.name, (cs.co, cs.kh, cs.kw, cs.ci), T))
            jobs[-1].start = tiles
            tiles += L.lib().crnn_pack_conv_t_tiles(cs.co, cs.ci)
        # the BiLSTM's W_hh'^T (BPTT B operand, K-contiguous): a gathered transpose on the same tiled
        # kernel (KH = KW = 1, perm = the gate interleave) when its 16-B source rows allow, else an
        # element gather in crnn_pack_batch (below)
        whh_names = [f"enc_rnn.{l}.rnn.weight_hh_l0{sfx}" for l in range(self.nl) for sfx in ("", "_reverse")]
        tiled_t = H % 16 == 0 and all(self.p[n].data_ptr() % 16 == 0 for n in whh_names)
        for l in range(self.nl if tiled_t else 0):
            pre = f"enc_rnn.{l}"
            whh_t = self._pbuf(pre + ".whh_t", (2, H, 4 * H), T)
            for d, sfx in enumerate(["", "_reverse"]):
                job(L.PACK_CONV_T, self.p[pre + ".rnn.weight_hh_l0" + sfx], whh_t[d], 4 * H, H, 1, 1, perm=self.perm)
                jobs[-1].start = tiles
                tiles += L.lib().crnn_pack_conv_t_tiles(4 * H, H)
        if jobs:
            tarr = (L.PackJob * len(jobs))(*jobs)
            traw = torch.frombuffer(bytearray(bytes(tarr)), dtype=torch.uint8).to(self.device)
        else:
            traw = None
        tw_tab = (traw, len(jobs), tiles)
        jobs.clear()
        for l in range(self.nl):
            pre = f"enc_rnn.{l}"
            ind = self.enc_dim if l == 0 else H
            wih = self._pbuf(pre + ".wih", (2, 4 * H, ind), T)
            whh = self._pbuf(pre + ".whh", (2, 4 * H, H), T)
            bias = self._pbuf(pre + ".bias", (2, 4 * H), torch.float32)
            whh_t = self._pbuf(pre + ".whh_t", (2, H, 4 * H), T)
            for d, sfx in enumerate(["", "_reverse"]):
                r = pre + ".rnn."
                if not tiled_t:
                    sizes.append(job(L.PACK_TRANSPOSE, self.p[r + "weight_hh_l0" + sfx], whh_t[d], 4 * H, 4 * H, H,
                                     perm=self.perm))
                sizes.append(job(L.PACK_ROWS, self.p[r + "weight_ih_l0" + sfx], wih[d], 4 * H, 4 * H, ind,
                                 perm=self.perm))
                sizes.append(job(L.PACK_ROWS, self.p[r + "weight_hh_l0" + sfx], whh[d], 4 * H, 4 * H, H,
                                 perm=self.perm))
                sizes.append(job(L.PACK_ROWS_SUM, self.p[r + "bias_ih_l0" + sfx], bias[d], 4 * H, 4 * H, 1,
                                 out_f32=True, perm=self.perm, src2=self.p[r + "bias_hh_l0" + sfx]))
            lw = self._pbuf(pre + ".lin", (H, 2 * H), T)
            sizes.append(job(L.PACK_ROWS, self.p[pre + ".linear.weight"], lw, H, H, 2 * H))
        if self.has_head:
            hw = self._pbuf("head.w", (self.Cpad, H), T)
            sizes.append(job(L.PACK_ROWS, self.p["ctc_head.weight"], hw, self.Cpad, self.C, H))
            hb = self._pbuf("head.b", (self.Cpad,), torch.float32)
            sizes.append(job(L.PACK_ROWS, self.p["ctc_head.bias"], hb, self.Cpad, self.C, 1, out_f32=True))
        start = 0
        for jb, n in zip(jobs, sizes):
            jb.start = start
            start += n
        arr = (L.PackJob * len(jobs))(*jobs)
        raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.device)
        self._pack_jobs = (conv_tab, (raw, len(jobs), start), tw_tab)

    # ------------------------------------------------------------------ instrumentation
    def enable_timing(self, on: bool = True):
        """record HIP events around every implicit-GEMM conv launch (fwd / dgrad / wgrad)
        on the launch stream; conv_time_ms() sums them after a synchronize."""
        self.timers = [] if on else None

    def enable_lstm_timing(self, on: bool = True):
        """record the persistent BiLSTM sweeps' kernel-only events in every step, also when the conv events
        are off (four event pairs per step: the per-sweep mean over many steps, comparable to a profiler's)"""
        self.lstm_timers = [] if on else None

    def _timer_list(self):
        return self.timers if getattr(self, "timers", None) is not None else self.lstm_timers

    def _conv_call(self, kind, flops, name, *args):
        t0 = self._mark()
        call(name, *args)
        self._record(kind, flops, t0)

    def _mark(self):
        """start event on the current (launch) stream when timing is on, else None"""
        if getattr(self, "timers", None) is None:
            return None
        a = torch.cuda.Event(enable_timing=True)
        a.record()
        return a

    def _seq_marks(self):
        """(start, end) events the library records around the next persistent BiLSTM kernel alone
        (crnn_lstm_seq_time_next), when timing is on; else None"""
        if getattr(self, "timers", None) is None and getattr(self, "lstm_timers", None) is None:
            return None
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()   # creates the HIP events; the library re-records both on the launch stream
        b.record()
        call("crnn_lstm_seq_time_next", a.cuda_event, b.cuda_event)
        return a, b

    def _record(self, kind, work, start):
        if start is None:
            return
        b = torch.cuda.Event(enable_timing=True)
        b.record()
        self.timers.append((kind, work, start, b))

    @staticmethod
    def lstm_step_bytes(B, H, T):
        """algorithmic HBM bytes of ONE forward recurrence step of one layer, both directions
        (SURVEY.md §8d): W_hh + precomputed x-gates + h_{t-1} read / h_t write + c read/write (fp32)."""
        s = 2 if T == torch.bfloat16 else 4
        return 2 * (4 * H * H * s + B * 4 * H * s + 2 * B * H * s + 2 * B * H * 4)

    @staticmethod
    def lstm_bptt_step_bytes(B, H, T):
        """the BPTT step's counterpart: W_hh + dgates_{t'} read + dgates_t write + saved gates read +
        dh read + c_t, c_{t-1} read (fp32), both directions."""
        s = 2 if T == torch.bfloat16 else 4
        return 2 * (4 * H * H * s + 3 * B * 4 * H * s + B * H * s + 2 * B * H * 4)

    def conv_timing(self):
        """{kind: (launches, total_ms, total_work)} since enable_timing(); clears the list. Kinds:
        conv fwd / dgrad / wgrad (work = FLOP) and lstm_fwd / lstm_bwd (recurrence sweeps, work =
        algorithmic bytes)."""
        out = {}
        lt = getattr(self, "lstm_timers", None)
        for kind, flops, a, b in (self.timers or []) + (lt or []):
            n, ms, fl = out.get(kind, (0, 0.0, 0.0))
            out[kind] = (n + 1, ms + a.elapsed_time(b), fl + flops)
        if self.timers is not None:
            self.timers.clear()
        if lt is not None:
            lt.clear()
        return out

    @staticmethod
    def conv_flops(cs: "ConvSpec", b, h, w):
        ho, wo = cs.out_hw(h, w)
        return 2.0 * b * ho * wo * cs.co * cs.ci_real * cs.kh * cs.kw

    def _pbuf(self, name, shape, dtype, zero=False):
        t = self.packed.get(name)
        if t is None:
            t = (torch.zeros if zero else torch.empty)(shape, dtype=dtype, device=self.device)
            self.packed[name] = t
        return t

    # ------------------------------------------------------------------ helpers
    # persistent whole-sequence BiLSTM kernels (lstm_seq.hip): bf16, supported shapes only;
    # CRNN_LSTM_PER_STEP=1 forces the per-step launches (A/B and fallback coverage)
    use_seq = os.environ.get("CRNN_LSTM_PER_STEP", "0") != "1"
    # conv weight gradients on a second stream (CRNN_WGRAD_STREAM, default 0): the wgrad GEMMs are
    # off the dgrad chain's critical path, so they overlap the chain's HBM-bound BN / SE backward
    # passes and fill its GEMMs' last rounds of tiles. Each wgrad's input gradient then gets a
    # buffer of its own (no rotation), and the compute stream joins the side stream before
    # backward() returns. Measured (profiles/r02t_wgrad_side_stream_ab.log): the two streams
    # time-share the CUs, the wgrad launches take twice as long, and the step gains 0.4 %, so off.
    wgrad_stream = os.environ.get("CRNN_WGRAD_STREAM", "0") == "1"
    # only the conv wgrads' split-K slab REDUCES on a second stream (CRNN_WGRAD_REDUCE_STREAM, default 0):
    # a memory-bound pass whose output (the fp32 weight gradient) nothing reads before the optimizer, run
    # beside the next dgrad GEMM instead of in the chain; the slabs alternate between two buffers, and a
    # GEMM waits only for the reduce that last read its buffer. Measured (r04, same box, alternating):
    # 17.24k vs 17.39k lines/s — the reduces stretch and the dgrads they overlap slow down by more than
    # the 0.35 ms taken off the chain (profiles/r04c_reduce_stream_ab.log), so off
    wgrad_reduce_stream = os.environ.get("CRNN_WGRAD_REDUCE_STREAM", "0") == "1"
    # forward without saved activations: eval conv -> BN -> ReLU pairs as one conv launch with the
    # running-stat affine + ReLU in the epilogue, and the BiLSTM sweeps store no gates / cell
    # states (CRNN_EVAL_FUSE, default 1)
    eval_fuse = os.environ.get("CRNN_EVAL_FUSE", "1") == "1"
    # strided blocks: conv1's and the downsample's dgrads as one launch (CRNN_DS_FUSE, default 1)
    ds_fuse = os.environ.get("CRNN_DS_FUSE", "1") == "1"
    # stride-1 conv dgrads on the FORWARD conv path with a transposed, flipped weight pack
    # (crnn_conv_dgrad_tw; CRNN_DGRAD_TW, default 1): the forward's K-contiguous B operand, tiles and
    # padding-row skip instead of the dgrad loader's transposed LDS reads
    dgrad_tw = os.environ.get("CRNN_DGRAD_TW", "1") == "1"
    # the stem's BN-backward sums from the pooled forward output and gradient (CRNN_BNG_POOL_OUT:
    # a quarter of the bytes of the full-resolution z; CRNN_POOL_OUT_REDUCE, default 1)
    pool_out_reduce = os.environ.get("CRNN_POOL_OUT_REDUCE", "1") == "1"

    def _seq_ok(self, B):
        return self.use_seq and bool(L.lib().crnn_lstm_seq_supported(self.dt, B, self.H))

    def _seq_ws(self, B):
        n = (L.lib().crnn_lstm_seq_workspace(B) + 3) // 4
        t = self.ws.bufs.get("rnn.seq_ws")
        if t is None or t.numel() != n:
            if t is not None:
                self._fold_sticky(t)
            # zeroed at allocation: the sticky status word (after the ring) is never zeroed again
            t = self.ws.bufs["rnn.seq_ws"] = torch.zeros(n, dtype=torch.int32, device=self.device)
            # the library's own layout (include/crnn_hip.h crnn_lstm_seq_status_offset), kept with the buffer
            self._sticky_index = int(L.lib().crnn_lstm_seq_status_offset(B)) // 4
        self._seq_used = True
        return t

    def _fold_sticky(self, old):
        self._sticky_carry |= int(old[self._sticky_index].item())

    def status_word(self) -> Optional[torch.Tensor]:
        """the persistent BiLSTM's sticky status word (int32 device view, 0 = ok), or None when no
        persistent sweep has run: FusedAdamW passes it to its kernel, which skips the update when it
        is set (a timed-out sweep leaves NaN gradients that must not reach the weights)."""
        t = self.ws.bufs.get("rnn.seq_ws") if self._seq_used else None
        return None if t is None else t[self._sticky_index:self._sticky_index + 1]

    def seq_status(self) -> int:
        """OR of the error words of every persistent BiLSTM launch so far (0 = ok; non-zero: a
        bounded wait timed out and that sweep's outputs are NaN). Synchronises."""
        t = self.ws.bufs.get("rnn.seq_ws")
        return self._sticky_carry | (0 if t is None else int(t[self._sticky_index].item()))

    def check_status(self):
        """raise if any persistent BiLSTM sweep has timed out (synchronises)"""
        if self.seq_status():
            raise RuntimeError(_SEQ_TIMEOUT_MSG)

    def poll_status(self):
        """non-blocking check, called once per forward / backward: raise if a status copy enqueued
        by an earlier call has landed and shows a timed-out sweep; enqueue the next copy (4 bytes
        into pinned host memory, ordered after this call's kernels on the current stream)."""
        if not self._seq_used:
            return
        if self._status_evt is not None and self._status_evt.query():
            if int(self._status_host[0]) or self._sticky_carry:
                raise RuntimeError(_SEQ_TIMEOUT_MSG)
            self._status_evt = None
        if self._status_evt is None:
            t = self.ws.bufs["rnn.seq_ws"]
            if self._status_host is None:
                self._status_host = torch.zeros(1, dtype=torch.int32).pin_memory()
            i = self._sticky_index
            self._status_host.copy_(t[i:i + 1], non_blocking=True)
            self._status_evt = torch.cuda.Event()
            self._status_evt.record()

    def _bn_finalize(self, prefix, psum, psq, rows, count, train, tag, rpp=1):
        C = psum.shape[-1] if psum is not None else self.p[prefix + ".weight"].numel()
        ws = self.ws
        mean = ws.get(tag + ".mean", (C,), torch.float32)
        inv = ws.get(tag + ".inv", (C,), torch.float32)
        sc = ws.get(tag + ".scale", (C,), torch.float32)
        sh = ws.get(tag + ".shift", (C,), torch.float32)
        rm = self.buf[prefix + ".running_mean"]
        rv = self.buf[prefix + ".running_var"]
        if not train:
            # eval affine from the running statistics: recomputed only when the parameters or the
            # running statistics have changed since (train forwards clear the cache: their kernels
            # update the statistics and these buffers without bumping a torch version counter).
            # Writes through `.data` bump no version counter: mark_params_changed() clears the cache
            # (a replaced `.data` tensor is caught by its storage pointer)
            key = (self._cur_ver, rm._version, rv._version, rm.data_ptr(), rv.data_ptr())
            if self._eval_affine.get(tag) == key:
                return mean, inv, sc, sh
            self._eval_affine[tag] = key
        else:
            self._eval_affine.clear()
        call("crnn_bn_finalize", ptr(psum) if train else None, ptr(psq) if train else None, rows, rpp, C, count,
             ptr(self.p[prefix + ".weight"]), ptr(self.p[prefix + ".bias"]),
             ptr(rm), ptr(rv), BN_MOMENTUM if self.update_running else 0.0, BN_EPS, 1 if train else 0,
             ptr(mean), ptr(inv), ptr(sc), ptr(sh), ptr(self._fin_ws()), L.stream_ptr())
        if train and self.update_running:
            nbt = self.buf.get(prefix + ".num_batches_tracked")
            if nbt is not None:
                self._nbt.append(nbt)
        return mean, inv, sc, sh

    def _fin_ws(self):
        t = self.ws.bufs.get("bn.fin_ws")
        if t is None:   # zeroed once: the finalize kernels keep their ticket counters re-armed
            n = (L.lib().crnn_bn_finalize_workspace(512) + 3) // 4
            t = self.ws.bufs["bn.fin_ws"] = torch.zeros(n, dtype=torch.float32, device=self.device)
        return t

    def _conv_bn(self, cs: ConvSpec, x, b, h, w, train, tag, partials=False):
        """z = conv(x); BN statistics (train) or running stats (eval) -> (z, mean, inv, scale, shift, ho, wo)."""
        d = cs.desc(b, h, w)
        ho, wo = d.Ho, d.Wo
        z = self.ws.get(tag + ".z", (b, ho, wo, cs.co), self.dtype)
        s = L.stream_ptr()
        if train:
            rows = L.lib().crnn_conv_stat_rows(self.dt, d)
            psum = self.ws.get("stat.sum", (self._stat_cap,), torch.float32)[: rows * cs.co].view(rows, cs.co)
            psq = self.ws.get("stat.sq", (self._stat_cap,), torch.float32)[: rows * cs.co].view(rows, cs.co)
            self._conv_call("fwd", self.conv_flops(cs, b, h, w), "crnn_conv_fwd", self.dt, d, ptr(x),
                            ptr(self.packed[cs.name]), ptr(z), ptr(psum), ptr(psq), s)
            rpp = L.lib().crnn_conv_stat_rows_per_partial(self.dt, d)
            stats = self._bn_finalize(cs.bn, psum, psq, rows, b * ho * wo, True, tag, rpp)
            self._last_partials = (psum, rows, rpp)
        elif partials:
            # eval, but the conv's per-tile sums are wanted (the SE squeeze reads them instead of
            # making a pass over z: mean over HW of the running-stat affine is affine in mean(z))
            rows = L.lib().crnn_conv_stat_rows(self.dt, d)
            psum = self.ws.get("stat.sum", (self._stat_cap,), torch.float32)[: rows * cs.co].view(rows, cs.co)
            psq = self.ws.get("stat.sq", (self._stat_cap,), torch.float32)[: rows * cs.co].view(rows, cs.co)
            self._conv_call("fwd", self.conv_flops(cs, b, h, w), "crnn_conv_fwd", self.dt, d, ptr(x),
                            ptr(self.packed[cs.name]), ptr(z), ptr(psum), ptr(psq), s)
            stats = self._bn_finalize(cs.bn, None, None, 0, b * ho * wo, False, tag)
            self._last_partials = (psum, rows, L.lib().crnn_conv_stat_rows_per_partial(self.dt, d))
        else:
            self._conv_call("fwd", self.conv_flops(cs, b, h, w), "crnn_conv_fwd", self.dt, d, ptr(x),
                            ptr(self.packed[cs.name]), ptr(z), None, None, s)
            stats = self._bn_finalize(cs.bn, None, None, 0, b * ho * wo, False, tag)
        return (z,) + stats + (ho, wo)

    def _conv_bn_relu_eval(self, cs: ConvSpec, x, b, h, w, tag, out_name):
        """eval-mode conv -> BN (running statistics) -> ReLU as ONE conv launch (crnn_conv_fwd_bnrelu:
        the affine + ReLU on the fp32 accumulators of the implicit-GEMM or halo kernel, no z tensor,
        no bn_act pass); None when unsupported (the caller runs conv, finalize, bn_act)."""
        d = cs.desc(b, h, w)
        if not self.eval_fuse or not L.lib().crnn_conv_fwd_bnrelu_supported(self.dt, d):
            return None
        _, _, sc, sh = self._bn_finalize(cs.bn, None, None, 0, b * d.Ho * d.Wo, False, tag)
        a = self.ws.get(out_name, (b, d.Ho, d.Wo, cs.co), self.dtype)
        self._conv_call("fwd", self.conv_flops(cs, b, h, w), "crnn_conv_fwd_bnrelu", self.dt, d, ptr(x),
                        ptr(self.packed[cs.name]), ptr(a), ptr(sc), ptr(sh), L.stream_ptr())
        return a, d.Ho, d.Wo

    def _stat_capacity(self, B, H, W):
        cap = 0
        lib = L.lib()

        def upd(cs, h, w):
            nonlocal cap
            d = cs.desc(B, h, w)
            cap = max(cap, lib.crnn_conv_stat_rows(self.dt, d) * cs.co)
            return d.Ho, d.Wo

        h, w = upd(self.stem0, H, W)
        h, w = upd(self.stem1, h, w)
        h, w = h // 2, w // 2
        for blk in self.blocks:
            h1, w1 = upd(blk.conv1, h, w)
            upd(blk.conv2, h1, w1)
            if blk.ds is not None:
                upd(blk.ds, h, w)
            h, w = h1, w1
        h, w = upd(self.co0, h, w)
        upd(self.co1, h, w)
        return cap

    # ------------------------------------------------------------------ forward
    def forward(self, images: torch.Tensor, train: bool, update_running: bool = True,
                save_for_backward: bool = False, dropout_p: float = 0.0, dropblock_p: float = 0.0,
                dropblock_block_size: int = 5) -> torch.Tensor:
        """images [B,3,H,W] fp32 (reference NCHW input), or the encoder layout [B,H,W,8] in the
        compute dtype (crnn_hip.preprocess out="encoder") -> logits [B,T,C] fp32 (view).
        dropout_p: enc_dropout probability applied to the encoder output in training
        (model/model.py:201,220); counter-based mask, regenerated in backward (crnn_dropout).
        dropblock_p / dropblock_block_size: every SE block's DropBlock2d in training
        (model/seresnet31.py:49-53,62); keep bytes per block (crnn_dropblock_mask), applied inside
        the SE-residual kernel and to the SE side of the block's gradient in backward."""
        L.require_device(images)
        self.pack()
        self.update_running = update_running
        ws, dt, T = self.ws, self.dt, self.dtype
        packed = images.dim() == 4 and images.shape[-1] == 8 and images.shape[1] != 3 and images.dtype == T
        if packed:
            images = images.contiguous()
            B, H, W = images.shape[:3]
        else:
            images = images.contiguous().float()
            B, Cin, H, W = images.shape
            if Cin != 3:
                raise ValueError("expected 3-channel crops")
        s = L.stream_ptr()
        if train and (dropout_p > 0.0 or dropblock_p > 0.0):
            self._drop_calls += 1   # one mask draw per training forward (enc_dropout, DropBlock2d)
        fuse = not train and not save_for_backward and self.eval_fuse   # eval inference fusions
        self._stat_cap = self._stat_capacity(B, H, W) if train or fuse else 0
        self._nbt = []
        sv = {}

        if packed:
            x0 = images
        else:
            x0 = ws.get("in", (B, H, W, 8), T)
            call("crnn_nchw_to_nhwc", dt, ptr(images), ptr(x0), B, 3, H, W, 8, s)
        # stem (model/seresnet31.py:81-89)
        fused = self._conv_bn_relu_eval(self.stem0, x0, B, H, W, "s0", "s0.a") if fuse else None
        if fused is not None:
            a0, h, w = fused
            z0 = m0 = i0 = sc0 = sh0 = None
        else:
            z0, m0, i0, sc0, sh0, h, w = self._conv_bn(self.stem0, x0, B, H, W, train, "s0")
            a0 = ws.get("s0.a", (B, h, w, 64), T)
            call("crnn_bn_act", dt, ptr(z0), ptr(sc0), ptr(sh0), ptr(a0), B * h * w, 64, 1, s)
        d1 = self.stem1.desc(B, h, w)
        if d1.Ho % 2 or d1.Wo % 2:
            raise ValueError("stem maxpool expects even H and W")
        if fuse and L.lib().crnn_conv_fwd_bnrelu_pool_supported(dt, d1):
            # eval inference: conv -> BN -> ReLU -> max-pool in the halo kernel's epilogue
            _, _, sc1, sh1 = self._bn_finalize(self.stem1.bn, None, None, 0, B * d1.Ho * d1.Wo, False, "s1")
            xp = ws.get("s1.pool", (B, d1.Ho // 2, d1.Wo // 2, 128), T)
            self._conv_call("fwd", self.conv_flops(self.stem1, B, h, w), "crnn_conv_fwd_bnrelu_pool", dt, d1,
                            ptr(a0), ptr(self.packed[self.stem1.name]), ptr(xp), ptr(sc1), ptr(sh1), s)
            h, w = d1.Ho, d1.Wo
            z1 = m1 = i1 = None
        else:
            z1, m1, i1, sc1, sh1, h, w = self._conv_bn(self.stem1, a0, B, h, w, train, "s1")
            xp = ws.get("s1.pool", (B, h // 2, w // 2, 128), T)
            call("crnn_bn_relu_maxpool", dt, ptr(z1), ptr(sc1), ptr(sh1), ptr(xp), B, h, w, 128, s)
        sv["stem"] = dict(x0=x0, z0=z0, m0=m0, i0=i0, sc0=sc0, sh0=sh0, a0=a0, z1=z1, m1=m1, i1=i1, sc1=sc1,
                          sh1=sh1, H=H, W=W, h1=h, w1=w)
        x, h, w = xp, h // 2, w // 2
        # residual stages
        blk_saved = []
        for bi, blk in enumerate(self.blocks):
            tag = f"b{bi}"
            P = blk.planes
            fused = self._conv_bn_relu_eval(blk.conv1, x, B, h, w, tag + ".c1", tag + ".a1") if fuse else None
            if fused is not None:
                a1, ho, wo = fused
                z1b = bm1 = bi1 = bs1 = bh1 = None
            else:
                z1b, bm1, bi1, bs1, bh1, ho, wo = self._conv_bn(blk.conv1, x, B, h, w, train, tag + ".c1")
                a1 = ws.get(tag + ".a1", (B, ho, wo, P), T)
                call("crnn_bn_act", dt, ptr(z1b), ptr(bs1), ptr(bh1), ptr(a1), B * ho * wo, P, 1, s)
            self._last_partials = None
            z2, bm2, bi2, bs2, bh2, _, _ = self._conv_bn(blk.conv2, a1, B, ho, wo, train, tag + ".c2", partials=fuse)
            HW = ho * wo
            Cr = P // 16
            pooled = ws.get(tag + ".pooled", (B, P), torch.float32)
            hid = ws.get(tag + ".hid", (B, Cr), torch.float32)
            se = ws.get(tag + ".s", (B, P), torch.float32)
            lp = self._last_partials if train or fuse else None
            w1, w2 = self.p[blk.prefix + ".se.fc.0.weight"], self.p[blk.prefix + ".se.fc.2.weight"]
            if lp is not None and HW % lp[2] == 0 and lp[1] * lp[2] == B * HW:
                # squeeze from conv2's BN partial sums (no pass over z2), fused into the excitation launch
                call("crnn_se_pool_mlp_fwd", ptr(lp[0]), lp[1], lp[2], ptr(bs2), ptr(bh2), ptr(pooled), ptr(w1),
                     ptr(w2), ptr(hid), ptr(se), B, HW, P, Cr, s)
            else:
                call("crnn_se_pool", dt, ptr(z2), ptr(bs2), ptr(bh2), ptr(pooled), B, HW, P, s)
                call("crnn_se_mlp_fwd", ptr(pooled), ptr(w1), ptr(w2), ptr(hid), ptr(se), B, P, Cr, s)
            dsv = None
            if blk.ds is not None:
                zd, dm, di, dsc, dsh, _, _ = self._conv_bn(blk.ds, x, B, h, w, train, tag + ".ds")
                dsv = dict(zd=zd, m=dm, i=di, sc=dsc, sh=dsh)
                idn, isc, ish = zd, dsc, dsh
            else:
                idn, isc, ish = x, None, None
            y = ws.get(tag + ".y", (B, ho, wo, P), T)
            drop = None
            if train and dropblock_p > 0.0:
                # DropBlock2d between the SE gate and the residual add (model/seresnet31.py:61-62)
                seed = ((self._drop_seed ^ 0xD1B54A32D192ED03)
                        + 0x9E3779B97F4A7C15 * (self._drop_calls * 64 + bi + 1)) & 0xFFFFFFFFFFFFFFFF
                keep = ws.get(tag + ".keep", (B, ho, wo, P), torch.uint8)
                kept = ws.get(tag + ".kept", (1,), torch.int64)
                call("crnn_dropblock_mask", ptr(keep), ptr(kept), B, ho, wo, P, float(dropblock_p),
                     int(dropblock_block_size), seed, s)
                call("crnn_se_residual_drop_fwd", dt, ptr(z2), ptr(bs2), ptr(bh2), ptr(se), ptr(idn), ptr(isc),
                     ptr(ish), ptr(y), B, HW, P, ptr(keep), ptr(kept), s)
                drop = dict(keep=keep, kept=kept, seed=seed)
            else:
                call("crnn_se_residual_fwd", dt, ptr(z2), ptr(bs2), ptr(bh2), ptr(se), ptr(idn), ptr(isc), ptr(ish),
                     ptr(y), B, HW, P, s)
            blk_saved.append(dict(x=x, h=h, w=w, ho=ho, wo=wo, z1=z1b, m1=bm1, i1=bi1, sc1=bs1, sh1=bh1, a1=a1,
                                  z2=z2, m2=bm2, i2=bi2, sc2=bs2, sh2=bh2, pooled=pooled, hid=hid, s=se, ds=dsv,
                                  y=y, drop=drop))
            x, h, w = y, ho, wo
        sv["blocks"] = blk_saved
        # conv_out (model/seresnet31.py:129-136) + height collapse (model/model.py:191,216-218)
        fused = self._conv_bn_relu_eval(self.co0, x, B, h, w, "co0", "co0.a") if fuse else None
        if fused is not None:
            ac0, h2, w2 = fused
            zc0 = cm0 = ci0 = cs0 = ch0 = None
        else:
            zc0, cm0, ci0, cs0, ch0, h2, w2 = self._conv_bn(self.co0, x, B, h, w, train, "co0")
            ac0 = ws.get("co0.a", (B, h2, w2, 512), T)
            call("crnn_bn_act", dt, ptr(zc0), ptr(cs0), ptr(ch0), ptr(ac0), B * h2 * w2, 512, 1, s)
        zc1, cm1, ci1, cs1, ch1, h3, w3 = self._conv_bn(self.co1, ac0, B, h2, w2, train, "co1")
        Tn = w3
        seq = ws.get("seq", (B, Tn, 512), T)
        call("crnn_hpool_fwd", dt, ptr(zc1), ptr(cs1), ptr(ch1), ptr(seq), B, h3, w3, 512, s)
        sv["co"] = dict(x=x, h=h, w=w, z0=zc0, m0=cm0, i0=ci0, sc0=cs0, sh0=ch0, a0=ac0, h2=h2, w2=w2, z1=zc1,
                        m1=cm1, i1=ci1, sc1=cs1, sh1=ch1, h3=h3, w3=w3)
        if self._nbt:
            torch._foreach_add_(self._nbt, 1)   # BN num_batches_tracked, one launch
        # BiLSTM stack (model/model.py:195-198)
        xin, rnn_saved = self._rnn_forward(seq, B, Tn, save_for_backward)
        sv["rnn"] = rnn_saved
        Hd = self.H
        # enc_dropout (model/model.py:201,220): identity in eval; in training a counter-based mask
        # (crnn_dropout) whose seed is saved so the backward regenerates it
        sv["drop"] = None
        if train and dropout_p > 0.0:
            seed = (self._drop_seed + 0x9E3779B97F4A7C15 * self._drop_calls) & 0xFFFFFFFFFFFFFFFF
            xdr = ws.get("enc.drop", (B, Tn, Hd), T)
            call("crnn_dropout", dt, ptr(xin), ptr(xdr), B * Tn * Hd, float(dropout_p), seed, s)
            sv["drop"] = (float(dropout_p), seed)
            xin = xdr
        sv["enc"] = xin
        sv["B"], sv["T"] = B, Tn
        logits = None
        if self.has_head:   # CTC head
            logits = ws.get("logits", (B, Tn, self.Cpad), torch.float32)
            call("crnn_gemm_nt", dt, ptr(xin), Hd, ptr(self.packed["head.w"]), Hd, ptr(logits), self.Cpad,
                 ptr(self.packed["head.b"]), B * Tn, self.Cpad, Hd, 1, 0, s)
        self.poll_status()
        if save_for_backward:
            self.fwd_gen += 1
            sv["gen"] = self.fwd_gen
        self._saved = sv if save_for_backward else None
        return logits[:, :, : self.C] if logits is not None else None

    def _rnn_forward(self, seq, B, Tn, save_for_backward):
        """the BiLSTM stack (model/model.py:151-163, 195-198) over seq [B, T, enc_dim] (compute dtype)
        -> (output [B, T, hidden], per-layer saved tensors)"""
        ws, dt, T, s = self.ws, self.dt, self.dtype, L.stream_ptr()
        Hd = self.H
        xin = seq
        rnn_saved = []
        for l in range(self.nl):
            pre = f"enc_rnn.{l}"
            ind = xin.shape[-1]
            xg = ws.get(f"r{l}.xg", (B, Tn, 2, 4 * Hd), T)
            call("crnn_gemm_nt", dt, ptr(xin), ind, ptr(self.packed[pre + ".wih"]), ind, ptr(xg), 8 * Hd,
                 ptr(self.packed[pre + ".bias"]), B * Tn, 8 * Hd, ind, 0, 0, s)
            hseq = ws.get(f"r{l}.hseq", (B, Tn, 2 * Hd), T)
            gsv = ws.get(f"r{l}.gates", (2, Tn, B, 4 * Hd), T)
            csv = ws.get(f"r{l}.c", (2, Tn, B, Hd), torch.float32)
            whh = self.packed[pre + ".whh"]
            if self._seq_ok(B):
                ev = self._seq_marks()
                # without saved activations the sweep stores no gates / cell states (inference)
                keep = save_for_backward or not self.eval_fuse
                call("crnn_lstm_seq_fwd", ptr(xg), ptr(whh), ptr(hseq), ptr(gsv) if keep else None,
                     ptr(csv) if keep else None, ptr(self._seq_ws(B)), B, Tn, Hd, s)
                if ev is not None:
                    self._timer_list().append(("lstm_fwd", Tn * self.lstm_step_bytes(B, Hd, T), ev[0], ev[1]))
            else:
                t0 = self._mark()
                for st in range(Tn):
                    call("crnn_lstm_step_fwd", dt, ptr(xg), ptr(whh), ptr(hseq), ptr(gsv), ptr(csv), B, Tn, Hd, st, s)
                self._record("lstm_fwd", Tn * self.lstm_step_bytes(B, Hd, T), t0)
            out = ws.get(f"r{l}.out", (B, Tn, Hd), T)
            call("crnn_gemm_nt", dt, ptr(hseq), 2 * Hd, ptr(self.packed[pre + ".lin"]), 2 * Hd, ptr(out), Hd,
                 ptr(self.p[pre + ".linear.bias"]), B * Tn, Hd, 2 * Hd, 0, 0, s)
            rnn_saved.append(dict(x=xin, hseq=hseq, gates=gsv, c=csv, out=out))
            xin = out
        return xin, rnn_saved

    def bilstm_stack(self, seq: torch.Tensor, dout: Optional[torch.Tensor] = None, grads=None):
        """The BiLSTM stack alone (model/model.py:195-198) on seq [B, T, enc_dim] fp32: -> output
        [B, T, hidden] fp32; with dout (d loss / d output, fp32) also the BiLSTM parameter gradients
        into `grads` (overwritten) and -> (output, d seq fp32). The same kernels and workspace as the
        full forward / backward (tests: the 4 x 768 stack golden, tests/golden/bilstm_stack.npz)."""
        L.require_device(seq)
        self.pack()
        B, Tn, _ = seq.shape
        s = L.stream_ptr()
        xs = self.ws.get("stack.in", tuple(seq.shape), self.dtype)
        xs.copy_(seq)
        out, saved = self._rnn_forward(xs, B, Tn, dout is not None)
        self.poll_status()
        y = out.float().clone()
        if dout is None:
            return y
        self.g = grads
        self.accumulate = False
        dx = self.ws.get("stack.dout", (B, Tn, self.H), self.dtype)
        dx.copy_(dout)
        dseq = self._rnn_backward(dx, saved, B, Tn, 0)
        self.poll_status()
        return y, dseq.float().clone()

    def check_generation(self, gen: int):
        """raise unless the saved activations are those of forward generation `gen`: a second
        grad-enabled forward (loss = f(m(x1)) + f(m(x2)), activation checkpointing) before the
        first one's backward would otherwise silently differentiate the wrong batch."""
        cur = self._saved["gen"] if self._saved is not None else None
        if cur != gen:
            raise RuntimeError(
                "RCNN HIP engine: this backward belongs to forward #%d, but the engine holds the saved "
                "activations of %s; it keeps one forward's activations, so run backward before the next "
                "grad-enabled forward (or run the other forwards under torch.no_grad())"
                % (gen, "forward #%d" % cur if cur is not None else "no forward"))

    # ------------------------------------------------------------------ CTC
    def ctc(self, logits_padded: torch.Tensor, targets: torch.Tensor, lengths: torch.Tensor,
            want_grad: bool = True, zero_infinity: bool = True):
        """mean-reduced CTC loss (device scalar) and d loss / d logits [B,T,Cpad] (fp32)."""
        B, Tn, _ = logits_padded.shape
        ws = self.ws
        s = L.stream_ptr()
        tg = targets.to(device=self.device, dtype=torch.int32).contiguous()
        ln = lengths.to(device=self.device, dtype=torch.int32).contiguous()
        Lmax = tg.shape[1]
        loss_b = ws.get("ctc.loss_b", (B,), torch.float32)
        dlog = ws.get("ctc.dlogits", (B, Tn, self.Cpad), torch.float32) if want_grad else None
        call("crnn_ctc_loss", ptr(logits_padded), self.Cpad, B, Tn, self.C, ptr(tg), Lmax, ptr(ln), ptr(loss_b),
             ptr(dlog), 1 if zero_infinity else 0, s)
        loss = ws.get("ctc.loss", (1,), torch.float32)
        call("crnn_ctc_reduce_mean", ptr(loss_b), ptr(ln), B, ptr(loss), s)
        return loss, dlog

    def logits_padded(self):
        return self.ws.bufs["logits"]

    # ------------------------------------------------------------------ backward
    def _bn_bwd(self, mode, dy, z, stats, prefix, M, C, HW=1, y=None, se=None, dpool=None, out=None,
                accumulate_params=False, se_abc=None, sums=None, reduce_y=None):
        """BN backward: per-channel sums of g (mode, crnn_hip.h CRNN_BNG_*) -> finalize -> apply.
        se_abc = (abc, B): the SE mode's sums come from crnn_se_bn_bwd_reduce's per-sample terms
        (no second pass over the tensor); sums = (pg, pgx, rows): given by the producing dgrad;
        reduce_y (pool mode): the pooled forward output, whose sums (CRNN_BNG_POOL_OUT) read the
        pooled tensors instead of the full-resolution z."""
        mean, inv, sc, sh = stats
        ws = self.ws
        s = L.stream_ptr()
        d = BnBwdDesc(ptr(dy), ptr(z), ptr(mean), ptr(inv), ptr(sc), ptr(sh), ptr(y), ptr(se), ptr(dpool), mode,
                      M, C, HW)
        if sums is not None:   # (pg, pgx, rows) already produced (crnn_conv_dgrad_bnrelu)
            pg, pgx, rows = sums
        elif se_abc is not None:
            abc, B = se_abc
            rows = B
            pg = self._bnb_ws("bnb.pg")[: rows * C]
            pgx = self._bnb_ws("bnb.pgx")[: rows * C]
            call("crnn_se_bn_partials", ptr(abc), ptr(se), ptr(dpool), ptr(pg), ptr(pgx), B, HW, C, s)
        else:
            rows = L.lib().crnn_bn_rows(M)
            pg = self._bnb_ws("bnb.pg")[: rows * C]
            pgx = self._bnb_ws("bnb.pgx")[: rows * C]
            rd = d
            if reduce_y is not None:
                rd = BnBwdDesc(ptr(dy), ptr(z), ptr(mean), ptr(inv), ptr(sc), ptr(sh), ptr(reduce_y), None, None,
                               5, M, C, HW)   # CRNN_BNG_POOL_OUT
            call("crnn_bn_bwd_reduce", self.dt, rd, ptr(pg), ptr(pgx), rows, s)
        mg = ws.get("bnb.mg", (512,), torch.float32)
        mgx = ws.get("bnb.mgx", (512,), torch.float32)
        call("crnn_bn_bwd_finalize", ptr(pg), ptr(pgx), rows, C, M, ptr(self.g[prefix + ".weight"]),
             ptr(self.g[prefix + ".bias"]), ptr(mg), ptr(mgx), 1 if accumulate_params else 0, ptr(self._fin_ws()), s)
        call("crnn_bn_bwd_apply", self.dt, d, ptr(mg), ptr(mgx), ptr(out), s)
        return out

    def _bnb_ws(self, name):
        """the BN-backward per-channel partial rows (pg / pgx): room for 1024 rows of 512 channels
        (the reduce and dgrad-epilogue row caps) and for the SE mode's one row per sample"""
        B = self._saved["B"] if self._saved is not None else 0
        return self.ws.get(name, (max(1024 * 512, B * 512),), torch.float32)

    def _dz(self, tag, scratch, n):
        """the BN-backward output that a conv's dgrad AND wgrad read: a view of the rotating scratch
        buffer, or (wgrads on the side stream) a buffer of its own, so the dgrad chain cannot
        overwrite it before the side stream has read it"""
        if self._side is None:
            return scratch[:n]
        return self.ws.get("g.dz." + tag, (n,), self.dtype)

    def _wgrad(self, cs: ConvSpec, dz, x, b, h, w):
        if self._rside is not None:
            return self._wgrad_split(cs, dz, x, b, h, w)
        if self._side is not None:
            # ordered after everything the compute stream has enqueued so far (dz's producer)
            self._side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self._side):
                return self._wgrad_launch(cs, dz, x, b, h, w)
        return self._wgrad_launch(cs, dz, x, b, h, w)

    def _wgrad_launch(self, cs: ConvSpec, dz, x, b, h, w):
        d = cs.desc(b, h, w)
        need = L.lib().crnn_conv_wgrad_workspace(self.dt, d)
        wsb = self.ws.get("wgrad.ws", (self._wg_cap,), torch.float32)
        if need > wsb.numel() * 4:
            raise RuntimeError("wgrad workspace too small")
        beta = 1.0 if self.accumulate else 0.0
        self._conv_call("wgrad", self.conv_flops(cs, b, h, w), "crnn_conv_wgrad", self.dt, d, ptr(dz), ptr(x),
                        ptr(self.g[cs.name]), ptr(wsb), wsb.numel() * 4, beta, L.stream_ptr())

    def _wgrad_split(self, cs: ConvSpec, dz, x, b, h, w):
        """the split-K GEMM on the compute stream, its slab reduce on the reduce stream"""
        d = cs.desc(b, h, w)
        need = L.lib().crnn_conv_wgrad_workspace(self.dt, d)
        i = self._slab_i
        self._slab_i ^= 1
        wsb = self.ws.get(f"wgrad.ws{i}", (self._wg_cap,), torch.float32)
        if need > wsb.numel() * 4:
            raise RuntimeError("wgrad workspace too small")
        cur = torch.cuda.current_stream(self.device)
        if self._slab_ev[i] is not None:       # the reduce that last read this buffer
            cur.wait_event(self._slab_ev[i])
        self._conv_call("wgrad", self.conv_flops(cs, b, h, w), "crnn_conv_wgrad_gemm", self.dt, d, ptr(dz), ptr(x),
                        ptr(wsb), wsb.numel() * 4, L.stream_ptr())
        ev = torch.cuda.Event()
        ev.record(cur)
        self._rside.wait_event(ev)
        with torch.cuda.stream(self._rside):
            t0 = self._mark()
            call("crnn_conv_wgrad_reduce", self.dt, d, ptr(self.g[cs.name]), ptr(wsb), wsb.numel() * 4,
                 1.0 if self.accumulate else 0.0, L.stream_ptr())
            self._record("wgrad", 0.0, t0)
            done = torch.cuda.Event()
            done.record(self._rside)
        self._slab_ev[i] = done

    def _wgrad_capacity(self, B, H, W):
        lib = L.lib()
        cap = 0

        def upd(cs, h, w):
            nonlocal cap
            d = cs.desc(B, h, w)
            cap = max(cap, lib.crnn_conv_wgrad_workspace(self.dt, d) // 4)
            return d.Ho, d.Wo

        h, w = upd(self.stem0, H, W)
        h, w = upd(self.stem1, h, w)
        h, w = h // 2, w // 2
        for blk in self.blocks:
            h1, w1 = upd(blk.conv1, h, w)
            upd(blk.conv2, h1, w1)
            if blk.ds is not None:
                upd(blk.ds, h, w)
            h, w = h1, w1
        h, w = upd(self.co0, h, w)
        upd(self.co1, h, w)
        return cap

    @staticmethod
    def backward_stages() -> List[List[str]]:
        """the parameter-name prefixes backward() reports final through stage_done, in its order"""
        blocks = backbone_specs()[2]
        return ([["ctc_head.", "enc_rnn."], ["cnn.conv_out."]] + [[b.prefix + "."] for b in reversed(blocks)]
                + [["cnn.conv0."]])

    def backward(self, dlogits: Optional[torch.Tensor], grads: Dict[str, torch.Tensor], accumulate: bool = False,
                 stage_done=None, denc: Optional[torch.Tensor] = None):
        """Full backward from d loss / d logits [B,T,Cpad] fp32 into `grads` (fp32, reference layouts).
        stage_done(prefixes): called (host side, after the stage's kernels are enqueued) each time the
        gradients of every parameter under the given name prefixes are final — CTC head + BiLSTM, then
        conv_out, each residual block (last to first), the stem — so a data-parallel caller can start
        their all-reduce while the rest of the backward runs.
        denc: instead of dlogits, d loss / d encoder output [B,T,hidden] (fp32; the attention
        decoder's backward, crnn_hip/attn.py) — the CTC head is skipped (its grads are zeroed
        unless accumulating)."""
        sv = self._saved
        self._side = None
        self._rside = None
        if self.wgrad_stream:
            if self._side_stream is None:
                self._side_stream = torch.cuda.Stream(self.device)
            self._side = self._side_stream
        elif self.wgrad_reduce_stream:
            if self._side_stream is None:
                self._side_stream = torch.cuda.Stream(self.device)
            self._rside = self._side_stream
            self._slab_i, self._slab_ev = 0, [None, None]
        side = self._side if self._side is not None else self._rside
        if stage_done is None:
            done = lambda prefixes: None  # noqa: E731
        elif side is None:
            done = stage_done
        else:
            def done(prefixes):
                # the stage's weight gradients come from the side stream, its BN / SE ones from
                # the compute stream: issue the hook (an all-reduce orders itself after the
                # caller's current stream) on the side stream once it has caught up with both
                side.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(side):
                    stage_done(prefixes)
        if sv is None:
            raise RuntimeError("forward(save_for_backward=True) must precede backward")
        self.g = grads
        self.accumulate = accumulate
        ws, dt, T = self.ws, self.dt, self.dtype
        s = L.stream_ptr()
        B, Tn, Hd = sv["B"], sv["T"], self.H
        st = sv["stem"]
        self._wg_cap = self._wgrad_capacity(B, st["H"], st["W"])
        acc = 1 if accumulate else 0
        M = B * Tn
        dx = ws.get("rnn.dx_head", (B, Tn, Hd), T)
        if denc is not None:   # attention decoder: the gradient enters at the encoder output
            if tuple(denc.shape) != (B, Tn, Hd) or denc.dtype != torch.float32 or not denc.is_contiguous():
                raise ValueError("denc must be contiguous fp32 [B, T, hidden]")
            call("crnn_cast_f32", dt, ptr(denc), ptr(dx), M * Hd, s)
            if not accumulate and self.has_head:
                grads["ctc_head.weight"].zero_()
                grads["ctc_head.bias"].zero_()
        else:
            self._head_backward(dlogits, grads, acc, dx)
        if sv["drop"] is not None:  # enc_dropout backward: the forward's mask, from its seed
            call("crnn_dropout", dt, ptr(dx), ptr(dx), M * Hd, sv["drop"][0], sv["drop"][1], s)
        try:
            self._backward_encoder(dx, grads, acc, done)
        finally:
            if side is not None:
                torch.cuda.current_stream(self.device).wait_stream(side)
                self._side = None
                self._rside = None
        self.poll_status()

    def _head_backward(self, dlogits, grads, acc, dx):
        sv, ws, dt, T, s = self._saved, self.ws, self.dt, self.dtype, L.stream_ptr()
        B, Tn, Hd = sv["B"], sv["T"], self.H
        M = B * Tn
        # ---- CTC head
        dlT = ws.get("head.dlT", (B, Tn, self.Cpad), T)
        call("crnn_cast_f32", dt, ptr(dlogits), ptr(dlT), M * self.Cpad, s)
        hw_g = ws.get("head.dw", (self.Cpad, Hd), torch.float32)
        self._gemm_tn(dlT, self.Cpad, sv["enc"], Hd, hw_g, Hd, self.Cpad, Hd, M, 0)
        self._store_grad("ctc_head.weight", hw_g[: self.C], bool(acc))
        call("crnn_colsum", L.F32, ptr(dlogits), self.Cpad, M, self.C, ptr(grads["ctc_head.bias"]), acc, 1, s)
        call("crnn_gemm_nn", dt, ptr(dlT), self.Cpad, ptr(self.packed["head.w"]), Hd, ptr(dx), Hd, M, Hd,
             self.Cpad, 0, 0, s)

    def _rnn_backward(self, dx, rnn_saved, B, Tn, acc):
        """BPTT through the BiLSTM stack: d output [B, T, hidden] -> d input [B, T, enc_dim]; the
        parameter gradients straight into self.g (reference layouts)"""
        ws, dt, T, s = self.ws, self.dt, self.dtype, L.stream_ptr()
        Hd = self.H
        M = B * Tn
        grads = self.g
        for l in reversed(range(self.nl)):
            pre = f"enc_rnn.{l}"
            r = rnn_saved[l]
            ind = r["x"].shape[-1]
            dh = ws.get("rnn.dhseq", (B, Tn, 2 * Hd), T)
            call("crnn_gemm_nn", dt, ptr(dx), Hd, ptr(self.packed[pre + ".lin"]), 2 * Hd, ptr(dh), 2 * Hd, M,
                 2 * Hd, Hd, 0, 0, s)
            self._gemm_tn(dx, Hd, r["hseq"], 2 * Hd, grads[pre + ".linear.weight"], 2 * Hd, Hd, 2 * Hd, M, acc)
            call("crnn_colsum", dt, ptr(dx), Hd, M, Hd, ptr(grads[pre + ".linear.bias"]), acc, 0, s)
            dg = ws.get("rnn.dgates", (2, Tn, B, 4 * Hd), T)
            dc = ws.get("rnn.dc", (2, B, Hd), torch.float32)
            whh, whh_t = self.packed[pre + ".whh"], self.packed[pre + ".whh_t"]
            if self._seq_ok(B):
                ev = self._seq_marks()
                call("crnn_lstm_seq_bwd", ptr(dh), ptr(whh_t), ptr(r["gates"]), ptr(r["c"]), ptr(dg),
                     ptr(self._seq_ws(B)), B, Tn, Hd, s)
                if ev is not None:
                    self._timer_list().append(("lstm_bwd", Tn * self.lstm_bptt_step_bytes(B, Hd, T), ev[0], ev[1]))
            else:
                t0 = self._mark()
                bws = ws.get("rnn.bptt_ws", (L.lib().crnn_lstm_bptt_workspace(B, Hd) // 4,), torch.float32)
                for stp in range(Tn):
                    call("crnn_lstm_step_bwd", dt, ptr(dh), ptr(whh), ptr(whh_t), ptr(r["gates"]), ptr(r["c"]),
                         ptr(dg), ptr(dc), ptr(bws), B, Tn, Hd, stp, s)
                self._record("lstm_bwd", Tn * self.lstm_bptt_step_bytes(B, Hd, T), t0)
            rr = pre + ".rnn."
            gq = lambda n: ptr(self._gview(rr + n))  # noqa: E731
            # gradients straight into the parameters' .grad views (reference row order)
            if T == torch.bfloat16:   # all four in one batched split-K launch + slab reduce
                need = L.lib().crnn_lstm_wgrad_workspace(B, Tn, Hd, ind)
                wgw = ws.get("rnn.wgrad_ws", ((need + 3) // 4,), torch.float32)
                call("crnn_lstm_wgrad", ptr(dg), ptr(r["x"]), ptr(r["hseq"]), gq("weight_ih_l0"),
                     gq("weight_ih_l0_reverse"), gq("weight_hh_l0"), gq("weight_hh_l0_reverse"), ptr(wgw),
                     wgw.numel() * 4, B, Tn, Hd, ind, acc, s)
            else:
                call("crnn_lstm_dwhh", dt, ptr(dg), ptr(r["hseq"]), gq("weight_hh_l0"), gq("weight_hh_l0_reverse"),
                     B, Tn, Hd, acc, s)
                call("crnn_lstm_dwih", dt, ptr(dg), ptr(r["x"]), gq("weight_ih_l0"), gq("weight_ih_l0_reverse"),
                     B, Tn, Hd, ind, acc, s)
            dbws = ws.get("rnn.dbws", (L.lib().crnn_lstm_dbias_workspace(Hd) // 4,), torch.float32)
            call("crnn_lstm_dbias", dt, ptr(dg), gq("bias_ih_l0"), gq("bias_hh_l0"), gq("bias_ih_l0_reverse"),
                 gq("bias_hh_l0_reverse"), ptr(dbws), B, Tn, Hd, acc, s)
            nxt = ws.get(f"rnn.dx_l{l}", (B, Tn, ind), T)
            call("crnn_lstm_dx", dt, ptr(dg), ptr(self.packed[pre + ".wih"]), ptr(nxt), B, Tn, Hd, ind, s)
            dx = nxt
        return dx

    def _backward_encoder(self, dx, grads, acc, done):
        sv, ws, dt, T, s = self._saved, self.ws, self.dt, self.dtype, L.stream_ptr()
        B, Tn, Hd = sv["B"], sv["T"], self.H
        M = B * Tn
        accumulate = self.accumulate
        st = sv["stem"]
        # ---- BiLSTM stack, reverse
        dx = self._rnn_backward(dx, sv["rnn"], B, Tn, acc)
        dseq = dx  # [B, T, 512]
        if self.debug:
            self.dbg["dseq"] = dseq.clone()
        done(["ctc_head.", "enc_rnn."])
        # ---- conv_out + height collapse
        co = sv["co"]
        big = self._scratch_elems(sv)
        bufA = ws.get("g.A", (big,), T)
        bufB = ws.get("g.B", (big,), T)
        bufC = ws.get("g.C", (big,), T)
        h3, w3 = co["h3"], co["w3"]
        if h3 == 1:
            dyf = dseq
        else:
            dyf = bufA[: B * h3 * w3 * 512].view(B, h3, w3, 512)
            call("crnn_hpool_bwd", dt, ptr(dseq), ptr(dyf), B, h3, w3, 512, s)
        dz = self._dz("co1", bufB, B * h3 * w3 * 512)
        self._bn_bwd(1, dyf, co["z1"], (co["m1"], co["i1"], co["sc1"], co["sh1"]), self.co1.bn, B * h3 * w3, 512,
                     out=dz, accumulate_params=accumulate)
        self._wgrad(self.co1, dz, co["a0"], B, co["h2"], co["w2"])
        da = bufC[: B * co["h2"] * co["w2"] * 512]
        self._dgrad(self.co1, B, co["h2"], co["w2"], dz, da)
        dz0 = self._dz("co0", bufA, B * co["h2"] * co["w2"] * 512)
        self._bn_bwd(1, da, co["z0"], (co["m0"], co["i0"], co["sc0"], co["sh0"]), self.co0.bn,
                     B * co["h2"] * co["w2"], 512, out=dz0, accumulate_params=accumulate)
        self._wgrad(self.co0, dz0, co["x"], B, co["h"], co["w"])
        dy = bufB[: B * co["h"] * co["w"] * 512]
        self._dgrad(self.co0, B, co["h"], co["w"], dz0, dy)
        done(["cnn.conv_out."])
        # ---- residual blocks, reverse
        bufs = [bufA, bufB, bufC]
        cur = 1  # dy lives in bufB
        for bi in reversed(range(len(self.blocks))):
            blk = self.blocks[bi]
            sb = sv["blocks"][bi]
            P = blk.planes
            ho, wo, h, w = sb["ho"], sb["wo"], sb["h"], sb["w"]
            HW = ho * wo
            Mo = B * HW
            Cr = P // 16
            o1, o2 = [k for k in range(3) if k != cur]
            dyb = bufs[cur][: Mo * P]
            if self.debug:
                self.dbg[f"dy.b{bi}"] = dyb.clone().view(B, ho, wo, P)
            # the SE side's gradient: through the block's DropBlock2d when it ran (the residual side
            # below keeps dyb: the mask sits before the add, model/seresnet31.py:62-66)
            dyse = dyb
            if sb["drop"] is not None:
                dyse = ws.get(f"dropblock.dy.{Mo * P}", (Mo * P,), dyb.dtype)
                call("crnn_dropblock_apply", dt, ptr(dyb), ptr(dyse), ptr(sb["drop"]["keep"]),
                     ptr(sb["drop"]["kept"]), Mo * P, s)
            ds = ws.get(f"se.ds{P}", (B, P), torch.float32)
            abc = ws.get(f"se.abc{P}", (B, 3, P), torch.float32)
            bn2 = blk.conv2.bn
            # one pass over (dy, y, z2) for the SE gate gradient AND the BN2 sums (crnn_hip.h)
            call("crnn_se_bn_bwd_reduce", dt, ptr(dyse), ptr(sb["y"]), ptr(sb["z2"]), ptr(sb["m2"]), ptr(sb["i2"]),
                 ptr(self.p[bn2 + ".weight"]), ptr(self.p[bn2 + ".bias"]), ptr(ds), ptr(abc), B, HW, P, s)
            if self.debug:   # the SE chain kernel by kernel (tools/cohab_model.py localises differences)
                for k, v in (("y", sb["y"]), ("z2", sb["z2"]), ("m2", sb["m2"]), ("i2", sb["i2"]), ("s", sb["s"]),
                             ("hid", sb["hid"]), ("pooled", sb["pooled"]), ("1_ds", ds), ("1_abc", abc)):
                    self.dbg[f"se.b{bi}.{k}"] = v.clone()
            dsig = ws.get(f"se.dsig{P}", (B, P), torch.float32)
            dhid = ws.get(f"se.dhid{P}", (B, Cr), torch.float32)
            dpool = ws.get(f"se.dpool{P}", (B, P), torch.float32)
            # the SE MLP backward also writes BN2's per-sample backward sums (crnn_se_bn_partials' rows)
            pg2 = self._bnb_ws("bnb.pg")[: B * P]
            pgx2 = self._bnb_ws("bnb.pgx")[: B * P]
            call("crnn_se_mlp_bwd_partials", ptr(ds), ptr(sb["pooled"]), ptr(sb["hid"]), ptr(sb["s"]),
                 ptr(self.p[blk.prefix + ".se.fc.0.weight"]), ptr(self.p[blk.prefix + ".se.fc.2.weight"]),
                 ptr(dsig), ptr(dhid), ptr(dpool), ptr(self._gview(blk.prefix + ".se.fc.0.weight")),
                 ptr(self._gview(blk.prefix + ".se.fc.2.weight")), ptr(abc), ptr(pg2), ptr(pgx2), B, P, Cr, HW, acc,
                 s)
            if self.debug:
                for k, v in (("2_dsig", dsig), ("2_dhid", dhid), ("2_dpool", dpool), ("2_pg", pg2), ("2_pgx", pgx2),
                             ("2_dw1", self._gview(blk.prefix + ".se.fc.0.weight")),
                             ("2_dw2", self._gview(blk.prefix + ".se.fc.2.weight"))):
                    self.dbg[f"se.b{bi}.{k}"] = v.clone()
            dz2 = self._dz(f"b{bi}.c2", bufs[o1], Mo * P)
            self._bn_bwd(3, dyse, sb["z2"], (sb["m2"], sb["i2"], sb["sc2"], sb["sh2"]), blk.conv2.bn, Mo, P, HW=HW,
                         y=sb["y"], se=sb["s"], dpool=dpool, out=dz2, accumulate_params=accumulate,
                         sums=(pg2, pgx2, B))
            if self.debug:
                for k, v in (("3_mg", ws.get("bnb.mg", (512,), torch.float32)),
                             ("3_mgx", ws.get("bnb.mgx", (512,), torch.float32)),
                             ("3_dgamma", self.g[bn2 + ".weight"]), ("3_dz2", dz2)):
                    self.dbg[f"se.b{bi}.{k}"] = v.clone()
            self._wgrad(blk.conv2, dz2, sb["a1"], B, ho, wo)
            da1 = bufs[o2][: Mo * P]
            d2 = blk.conv2.desc(B, ho, wo)
            wt2 = self.packed.get(blk.conv2.name + ".t")
            frows = L.lib().crnn_conv_dgrad_tw_rows(dt, d2) if wt2 is not None else 0
            fname, fw = ("crnn_conv_dgrad_bnrelu_tw", wt2) if frows > 0 else \
                ("crnn_conv_dgrad_bnrelu", self.packed[blk.conv2.name])
            if frows == 0:
                frows = L.lib().crnn_conv_dgrad_bnrelu_rows(dt, d2)
            sums = None
            if frows > 0 and frows * P <= 1024 * 512:
                # dgrad + BN1's backward sums in the epilogue (no reduce pass over da1, z1)
                pg = self._bnb_ws("bnb.pg")[: frows * P]
                pgx = self._bnb_ws("bnb.pgx")[: frows * P]
                self._conv_call("dgrad", self.conv_flops(blk.conv2, B, ho, wo), fname, dt, d2,
                                ptr(dz2), ptr(fw), ptr(da1), ptr(sb["z1"]), ptr(sb["m1"]),
                                ptr(sb["i1"]), ptr(sb["sc1"]), ptr(sb["sh1"]), ptr(pg), ptr(pgx), s)
                sums = (pg, pgx, frows)
            else:
                self._dgrad(blk.conv2, B, ho, wo, dz2, da1)
            d1 = blk.conv1.desc(B, h, w)
            dds = blk.ds.desc(B, h, w) if blk.ds is not None else None
            # the downsample's dgrad as one more tap of conv1's parity class (0, 0): its input gradient
            # dzd follows dz1 in one buffer (crnn_conv_dgrad_ds's layout contract)
            fuse_ds = (dds is not None and self.ds_fuse and 2 * Mo * P <= bufs[o1].numel()
                       and L.lib().crnn_conv_dgrad_ds_supported(dt, d1, dds))
            if fuse_ds:
                dzcat = self._dz(f"b{bi}.c1ds", bufs[o1], 2 * Mo * P)
                dz1 = dzcat[: Mo * P]
            else:
                dz1 = self._dz(f"b{bi}.c1", bufs[o1], Mo * P)
            self._bn_bwd(1, da1, sb["z1"], (sb["m1"], sb["i1"], sb["sc1"], sb["sh1"]), blk.conv1.bn, Mo, P,
                         out=dz1, accumulate_params=accumulate, sums=sums)
            self._wgrad(blk.conv1, dz1, sb["x"], B, h, w)
            Ci = blk.conv1.ci
            dxb = bufs[o2][: B * h * w * Ci]
            if blk.ds is None:
                self._dgrad(blk.conv1, B, h, w, dz1, dxb, dres=dyb, yres=sb["y"])
                cur = o2
            elif fuse_ds:
                dsv = sb["ds"]
                dzd = dzcat[Mo * P:]
                self._bn_bwd(2, dyb, dsv["zd"], (dsv["m"], dsv["i"], dsv["sc"], dsv["sh"]), blk.ds.bn, Mo, P,
                             y=sb["y"], out=dzd, accumulate_params=accumulate)
                self._wgrad(blk.ds, dzd, sb["x"], B, h, w)
                self._conv_call("dgrad", self.conv_flops(blk.conv1, B, h, w) + self.conv_flops(blk.ds, B, h, w),
                                "crnn_conv_dgrad_ds", dt, d1, dds, ptr(dzcat), ptr(self.packed[blk.conv1.name]),
                                ptr(dxb), s)
                cur = o2
            else:
                self._conv_call("dgrad", self.conv_flops(blk.conv1, B, h, w), "crnn_conv_dgrad", dt, blk.conv1.desc(B, h, w), ptr(dz1), ptr(self.packed[blk.conv1.name]),
                     ptr(dxb), None, None, 0, s)
                dsv = sb["ds"]
                dzd = self._dz(f"b{bi}.ds", bufs[o1], Mo * P)
                self._bn_bwd(2, dyb, dsv["zd"], (dsv["m"], dsv["i"], dsv["sc"], dsv["sh"]), blk.ds.bn, Mo, P,
                             y=sb["y"], out=dzd, accumulate_params=accumulate)
                self._wgrad(blk.ds, dzd, sb["x"], B, h, w)
                self._conv_call("dgrad", self.conv_flops(blk.ds, B, h, w), "crnn_conv_dgrad", dt, blk.ds.desc(B, h, w), ptr(dzd), ptr(self.packed[blk.ds.name]),
                     ptr(dxb), None, None, 1, s)
                cur = o2
            done([blk.prefix + "."])
        # ---- stem
        o1, o2 = [k for k in range(3) if k != cur]
        dp = bufs[cur]
        if self.debug:
            self.dbg["dpool"] = dp[: B * (st["h1"] // 2) * (st["w1"] // 2) * 128].clone()
        h1, w1 = st["h1"], st["w1"]
        # BN -> ReLU -> MaxPool backward in one pass pair (CRNN_BNG_POOL: the pooled gradient is
        # routed to each window's first maximum inside the BN-backward reduce / apply kernels)
        dz1 = self._dz("s1", bufs[o2], B * h1 * w1 * 128)
        self._bn_bwd(4, dp, st["z1"], (st["m1"], st["i1"], st["sc1"], st["sh1"]), self.stem1.bn, B * h1 * w1, 128,
                     HW=w1, out=dz1, accumulate_params=accumulate,
                     reduce_y=sv["blocks"][0]["x"] if self.pool_out_reduce else None)
        self._wgrad(self.stem1, dz1, st["a0"], B, h1, w1)
        da0 = bufs[o1][: B * h1 * w1 * 64]
        self._conv_call("dgrad", self.conv_flops(self.stem1, B, h1, w1), "crnn_conv_dgrad", dt, self.stem1.desc(B, h1, w1), ptr(dz1), ptr(self.packed[self.stem1.name]),
             ptr(da0), None, None, 0, s)
        dz0 = self._dz("s0", bufs[cur], B * h1 * w1 * 64)
        self._bn_bwd(1, da0, st["z0"], (st["m0"], st["i0"], st["sc0"], st["sh0"]), self.stem0.bn, B * h1 * w1, 64,
                     out=dz0, accumulate_params=accumulate)
        self._wgrad(self.stem0, dz0, st["x0"], B, st["H"], st["W"])
        done(["cnn.conv0."])

    def _gemm_tn(self, A, lda, Bm, ldb, C, ldc, M, N, K, acc):
        """C (fp32) (+)= A^T B: bf16 through split-K slabs + reduce (crnn_gemm_tn_slab), fp32 direct."""
        if self.dtype == torch.bfloat16:
            need = L.lib().crnn_gemm_tn_workspace(M, N, K)
            w = self.ws.get(f"tn.ws.{need}", (need // 4 + 4,), torch.float32)
            call("crnn_gemm_tn_slab", ptr(A), lda, ptr(Bm), ldb, ptr(C), ldc, M, N, K, acc, ptr(w), w.numel() * 4,
                 L.stream_ptr())
        else:
            call("crnn_gemm_tn", self.dt, ptr(A), lda, ptr(Bm), ldb, ptr(C), ldc, M, N, K, acc, L.stream_ptr())

    def _scratch_elems(self, sv):
        st = sv["stem"]
        B = sv["B"]
        return B * st["h1"] * st["w1"] * 128

    def _gview(self, name):
        """the .grad tensor a kernel writes into directly (contiguous fp32 on the device)."""
        g = self.g[name]
        if g.dtype != torch.float32 or not g.is_contiguous() or g.device != self.device:
            raise ValueError(f"gradient buffer for {name} must be a contiguous fp32 tensor on {self.device}")
        return g

    def _store_grad(self, name, src, accumulate):
        g = self.g[name]
        src = src.reshape(g.shape)
        if accumulate:
            g.add_(src)
        else:
            g.copy_(src)
