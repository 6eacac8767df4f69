/*
 * crnn_hip.h — C ABI of the MI355X-native CRNN hot path (libcrnn_hip.so).
 *
 * SE-ResNet31 -> height-collapse -> BiLSTM -> CTC, forward and training step,
 * as hand-written HIP kernels for gfx950. This is the drop-in boundary: the
 * Python mirror of the reference API (rcnn-ocr_amd/model/model.py RCNN,
 * inference.py OCRInference, training/train.py run_training) binds these
 * entry points with ctypes; see INTEGRATION.md.
 *
 * Reference interfaces each group replaces (paths relative to the
 * sherstpasha/RCNN-OCR checkout):
 *   crnn_conv_*            nn.Conv2d(bias=False)       model/seresnet31.py:37-45, 82-86, 130-134, 153-154
 *   crnn_bn_*              nn.BatchNorm2d (+ReLU)      model/seresnet31.py:40-45, 83-88, 131-136, 154
 *   crnn_maxpool_*         nn.MaxPool2d(2,2)           model/seresnet31.py:88
 *   crnn_se_*              SELayer + residual + ReLU   model/seresnet31.py:5-20, 55-67
 *   crnn_hpool_*           AdaptiveAvgPool2d((1,None)) + squeeze + permute   model/model.py:191, 216-218
 *   crnn_lstm_*            nn.LSTM(bidirectional, batch_first)               model/model.py:152-163
 *   crnn_gemm_*            nn.Linear (BiLSTM output, CTC head)                model/model.py:157,162
 *   crnn_ctc_*             F.ctc_loss(blank=0) / ctc_greedy_decoder            training/utils.py:122-162
 *   crnn_adam_step         torch.optim.Adam (L2) / AdamW step                 training/train.py:292-295
 *   crnn_adamw             torch.optim.AdamW step                             training/train.py:294-295
 *   crnn_sgd_step          torch.optim.SGD(momentum) step                     training/train.py:296-299
 *
 * Conventions
 *   - dtype: CRNN_F32 (parity mode, exact-f32 MFMA) or CRNN_BF16 (perf mode,
 *     bf16 MFMA); accumulation is always fp32. Parameters, BN statistics,
 *     LSTM cell state, logits and CTC are fp32 in both modes.
 *   - Activations are NHWC ([B][H][W][C]); channel counts are multiples of 8.
 *   - Every buffer is allocated by the caller (device pointers); the library
 *     never allocates. `stream` is a hipStream_t passed as void*.
 *   - No host synchronisation inside any call: every entry point is safe to
 *     capture into a hipGraph.
 *   - Return value: 0 on success, else a hipError_t-compatible code;
 *     crnn_last_error_string() describes the last failure (thread-local).
 */
#ifndef CRNN_HIP_H
#define CRNN_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRNN_F32 0
#define CRNN_BF16 1
/* crnn_gemm_nt / nn / tn only: fp32 operands in memory, converted to bf16 while staged, bf16 MFMA, fp32
 * accumulation, fp32 C (c_f32 implied) — the attention decoder's training GEMMs (r06), the precision of the
 * reference's fp16 autocast (training/train.py:499) */
#define CRNN_F32_BF16MMA 2

int crnn_version(void);
const char* crnn_last_error_string(void);
/* tuning switches, process-wide (benchmark A/B only; defaults are the measured-best settings) */
enum { CRNN_OPT_GEMM_STAGGER = 0,    /* 256-row conv GEMM: waves 4-7 one barrier behind waves 0-3 */
       CRNN_OPT_GEMM_PERSISTENT = 1, /* retired in r06 (the persistent 256-row GEMM measured 20-50 % slower and
                                        was removed); the key is kept so option numbers stay stable: no effect */
       CRNN_OPT_DEEP_LINEAR = 2,     /* bf16 crnn_gemm_nt/nn on the 256-row kernel when its grid fills the chip (default 1) */
       CRNN_OPT_WGRAD_TILE = 3,      /* conv wgrad plan: 0 = 256x256, 1 = 256x128 tiles, n >= 2: ~128n blocks */
       CRNN_OPT_LSTM_TILE = 4,       /* persistent BiLSTM workgroup tile: 0 = auto, 1 = 32 samples x 32 units,
                                        2 = 16 x 32, 3 = 16 x 64 (when the grid fits the CUs) */
       CRNN_OPT_HALO_CONV = 5,       /* full-resolution 3x3 stride-1 convs (the stem's 64 -> 128) on the
                                        halo-tiled direct kernel (conv_halo.hip): 1 = on (default), 0 = GEMM,
                                        n >= 2: on, with n-row bands for the MFMA-bound instances */
       CRNN_OPT_LSTM_HANDOFF = 6,    /* persistent BiLSTM forward: 1 = K-split waves, data-tagged granule ring,
                                        0 = K-split waves, write-through payload + step counter, 2 = unit-complete
                                        waves (each wave owns whole units over the full K; h staged once per
                                        workgroup in LDS; granules published from registers), 3 (default) = the
                                        same with 8 waves of 8 units where the tile has 64 units (H <= 512),
                                        form 1 on the 32-unit tiles (4.03 vs 4.24 us per step
                                        inside the train step) */
       CRNN_OPT_WGRAD_REDUCE = 7,    /* conv wgrad split-K slab reduce: 1 = (co, 64-channel) tiles transposed
                                        through LDS, coalesced OIHW stores (default), 0 = flat, scattered stores */
       CRNN_OPT_WGRAD_FAST = 8,      /* conv wgrad on the 256-row kernel: 1 = per-tile scalar pixel decode for
                                        64-aligned pixel tiles (default), 0 = per-lane decode */
       CRNN_OPT_ROW_CLASS = 9,       /* conv dgrad of 1-2-row maps (conv_out[1]): 1 = one class per input row (only
                                        the taps that reach a real output row; default), 0 = generic */
       CRNN_OPT_QUANT_TILE = 10,     /* conv fwd / dgrad: 1 = a 256-row grid that fills its last round of tiles to
                                        < 70 % runs on the 128x128 kernel (default), 0 = off */
       CRNN_OPT_PAD_SKIP = 11,       /* 3x3 conv fwd / dgrad over 4-row maps on the 256-row kernel: 1 = skip the MFMAs
                                        of the fragment rows that read only zero padding (default) */
       CRNN_OPT_LSTM_BWD_PART = 12,  /* persistent BPTT: 1 = partial-sum form (own dgates x own W_hh rows, partials
                                        handed off as tagged granules), 0 = dgates + counter hand-off (default) */
       CRNN_OPT_LSTM_L2_HANDOFF = 13,  /* persistent BPTT (2: and forward): hand-off payload kept in the XCD's L2 (plain
                                          stores) for groups verified (HW_REG_XCC_ID) to run on one XCD (1, default);
                                          0 = always sc1 */
       CRNN_OPT_GEMM4W = 14,         /* 256-row GEMM family: 1 = the 4-wave form (one wave per SIMD, 128 x BN/2
                                        per wave, fragments double-buffered in registers), 0 = the 8-wave form;
                                        otherwise a mask of the families that take the 4-wave form: 2 = the conv
                                        weight gradients, 4 = the BN-fused conv input gradients, 8 = the BiLSTM
                                        weight gradients (default 2 since r06, when the asm-load register reuse
                                        behind r05's co-scheduled mismatch was found and fixed) */
       CRNN_OPT_DIAG = 15,           /* diagnostics only (default 0): bit 0 = conv fwd / plain dgrad / wgrad GEMMs
                                        skip their epilogue stores (the measured epilogue cost; results invalid) */
       CRNN_OPT_DGRAD_GROUP = 16,    /* strided conv dgrad on the 256-row kernel: 1 = all parity classes in ONE launch
                                        (grouped tile table, longest-K class first), 0 = a launch per class,
                                        2 = grouped with 256 x 256 tiles when Ci % 256 == 0 (default) */
       CRNN_OPT_FIN_TICKET = 17,     /* retired in r06 (the r01-r03 ticketed BN finalize was removed): no effect */
       CRNN_OPT_CONV_HALO_W = 18,    /* 3x3 / stride-1 conv fwd and stride-1 dgrad (forward path) over maps of a
                                        power-of-two width 32..256 on the 256-row kernel: 1 = one W-halo A image per
                                        (kernel row, 64-channel block) serves the three kw K-tiles (gemm256hw.hpp;
                                        default), 0 = an A image per K-tile (gemm256.hpp) */
       CRNN_OPT_LSTM_PIPE = 19,      /* retired in r06 (the pipelined two-group BiLSTM sweeps measured slower and
                                        were removed): no effect */
       CRNN_OPT_LINEAR_ROW8 = 20,    /* bf16 crnn_gemm_nt / nn on the 256-row kernel: 1 = 16-B row stores through the
                                        wave's LDS (8 columns per lane; default), 0 = 8-B stores from the MFMA layout */
       CRNN_OPT_HALO_ROW16 = 21,     /* the stem's input conv (3 -> 64, halo kernel): 1 = the output tile staged in LDS
                                        and stored as full 128-B lines (16 B per lane; default), 0 = 8-B stores from
                                        the MFMA layout */
       CRNN_OPT_HALO_WG2 = 22,       /* the stem input conv's weight gradient (halo kernel, streaming): 1 = one workgroup
                                        per band (two per CU, one slab each; default), 0 = min(bands, CUs) workgroups */
       CRNN_OPT_WGRAD_SLAB_BF16 = 23, /* bf16 conv weight gradients on the GEMM kernels: 1 (default) = split-K
                                        partial slabs stored as bf16 (half the slab bytes written and re-read by
                                        the reduce; each partial rounded once, fp32 sum), 0 = fp32 slabs. fp32
                                        convs and the halo stem kernels always use fp32 slabs */
       CRNN_OPT_COUNT = 24 };
int crnn_set_option(int key, int value);
/* current value of a tuning switch (0 for an unknown key) */
int crnn_get_option(int key);

/* ------------------------------------------------------------------ layout */
/* fp32 NCHW image batch -> dtype NHWC with channels zero-padded to Cp. */
int crnn_nchw_to_nhwc(int dtype, const float* x, void* y, int B, int C, int H, int W, int Cp, void* stream);
/* fp32 -> dtype cast of n contiguous elements. */
int crnn_cast_f32(int dtype, const float* src, void* dst, long n, void* stream);
/* dropout (reference: model/model.py:201,220 nn.Dropout(enc_dropout_p) on the encoder output):
 * y[i] = x[i] / (1 - p) if hash(seed, i) >= p * 2^32 else 0 (in place allowed). The mask is a
 * function of (seed, i) only, so the backward is the same call on dy with the same seed. Not
 * torch's Philox stream: masks agree in distribution, not bit for bit. p in [0, 1). */
int crnn_dropout(int dtype, const void* x, void* y, long n, float p, unsigned long long seed, void* stream);
/* DropBlock2d, training mode (replaces torchvision.ops.DropBlock2d as SEBasicBlock uses it,
   model/seresnet31.py:49-53 and :62; identity in eval or at p == 0, decided by the caller).
   crnn_dropblock_mask: keep u8 [B][H][W][C] (1 = kept) and *kept = number of kept elements
   (zeroed by the call); bs = min(block_size, H, W) must be odd (torchvision's mask for an even bs
   is (H+2) x (W+2) and the reference's multiply raises) and gamma = p*H*W / (bs^2 (H-bs+1)(W-bs+1))
   <= 1 (bernoulli_'s range). Seeds: drop_hash(seed, ((n*C + c)*(H-bs+1) + i)*(W-bs+1) + j) <
   gamma * 2^32 (not torch's Philox stream; oracle dropblock_keep restates it).
   crnn_dropblock_apply: y = x * keep * n / (1e-6 + *kept) (in place allowed; n % 8 == 0). */
int crnn_dropblock_mask(unsigned char* keep, unsigned long long* kept, int B, int H, int W, int C, float p,
                        int block_size, unsigned long long seed, void* stream);
int crnn_dropblock_apply(int dtype, const void* x, void* y, const unsigned char* keep,
                         const unsigned long long* kept, long n, void* stream);
/* conv weight OIHW fp32 -> OHWI dtype with Ci zero-padded to Cip. */
int crnn_pack_conv_weight(int dtype, const float* w, void* out, int Co, int Ci, int KH, int KW, int Cip, void* stream);
/* row gather + cast: out[r][c] = src[perm[r]][c] (perm == NULL: identity), rows >= rows_src are zero.
 * Used for LSTM gate interleave (row 4*j+gate <- gate*H+j) and padded heads. */
int crnn_pack_rows(int dtype, const float* src, void* out, const int* perm, int rows_out, int rows_src, int cols, void* stream);

/* Batched packing: every job of a DEVICE-resident table in one launch (the per-step re-pack of
 * all weights after an optimizer step). kind CRNN_PACK_CONV: src OIHW -> dst OHWI(Cip),
 * (a,b,c,d,e) = (Co,Ci,KH,KW,Cip); CRNN_PACK_ROWS: crnn_pack_rows with (a,b,c) = (rows_out,
 * rows_src, cols); CRNN_PACK_ROWS_SUM: the same with src2 added (LSTM b_ih + b_hh). out_f32
 * selects an fp32 destination instead of dtype. start = first element of the job in the
 * concatenation (jobs in order, start[0] = 0); total = all elements. */
#define CRNN_PACK_CONV 0
#define CRNN_PACK_ROWS 1
#define CRNN_PACK_ROWS_SUM 2
#define CRNN_PACK_TRANSPOSE 3 /* dst[c][r] = src[perm[r]][c], (a,b,c) = (rows, rows_src, cols) */
typedef struct {
  int kind, out_f32;
  int a, b, c, d, e, pad_;
  long start;
  const float* src;
  const float* src2;
  const int* perm;
  void* dst;
  void* dst2;  /* CRNN_PACK_CONV_T only (NULL: none): also the plain OHWI pack dst2[co][kh][kw][ci] of the same
                  weights from the same staged tile (Cip = Ci), so the source is read once */
} crnn_pack_job;
int crnn_pack_batch(int dtype, const crnn_pack_job* jobs, int njobs, long total, void* stream);
/* conv weights only (kind CRNN_PACK_CONV, a..e = Co, Ci, KH, KW, Cip), one block per output channel:
 * job.start = the job's first output channel in the concatenation (total_rows = sum of Co);
 * max_slab = the largest Ci*KH*KW (<= 16384). Same output as crnn_pack_batch for these jobs. */
int crnn_pack_conv_batch(int dtype, const crnn_pack_job* jobs, int njobs, long total_rows, int max_slab,
                         void* stream);
/* transposed, flipped conv kernels for crnn_conv_dgrad_tw (kind CRNN_PACK_CONV_T, a..d = Co, Ci, KH, KW;
 * Ci % 16 == 0, KH*KW in {1, 4, 9}): dst[ci][kh][kw][co] = src_OIHW[perm ? perm[co] : co][ci][KH-1-kh][KW-1-kw]
 * in dtype (KH = KW = 1 with perm: a gathered transpose, the BiLSTM's W_hh'^T). One workgroup per
 * 64 x 16 (co, ci) tile, coalesced both ways through LDS; job.start = the job's first tile in the
 * concatenation (a job has ceil(Co/64) * ceil(Ci/16) tiles, co-tile major); total_tiles = all. */
#define CRNN_PACK_CONV_T 4
int crnn_pack_conv_t_batch(int dtype, const crnn_pack_job* jobs, int njobs, long total_tiles, void* stream);
/* workgroup tiles of one CRNN_PACK_CONV_T job (the job.start increment) */
int crnn_pack_conv_t_tiles(int Co, int Ci);

/* ------------------------------------------------------------------ conv */
typedef struct {
  int B, Hi, Wi, Ci; /* Ci: stored (padded) input channels */
  int Ho, Wo, Co;
  int KH, KW, sh, sw, ph, pw;
  int Ci_real; /* true input channels (<= Ci); 0 means Ci */
} crnn_conv_desc;

/* y[B][Ho][Wo][Co] = conv(x[B][Hi][Wi][Ci], w[Co][KH][KW][Ci]).
 * psum/psq (may be NULL): per-channel partial statistics of y from the fp32 accumulators,
 * [crnn_conv_stat_rows(d)][Co]: psum = sum, psq = sum of squared deviations from the
 * partial's own mean, each partial covering crnn_conv_stat_rows_per_partial(d) rows;
 * consumed by crnn_bn_finalize. */
int crnn_conv_fwd(int dtype, const crnn_conv_desc* d, const void* x, const void* w, void* y, float* psum, float* psq, void* stream);
int crnn_conv_stat_rows(int dtype, const crnn_conv_desc* d);
int crnn_conv_stat_rows_per_partial(int dtype, const crnn_conv_desc* d);
/* eval-mode conv -> BatchNorm (running statistics) -> ReLU in one launch
 * (model/seresnet31.py:56-57, conv1 -> bn1 -> relu of BasicBlock; :129-131 conv_out):
 * y = max(conv(x, w) * scale[c] + shift[c], 0) from the fp32 accumulators (scale / shift:
 * crnn_bn_finalize with train = 0), on the implicit-GEMM and the halo (stem) kernels alike
 * (crnn_conv_fwd_bnrelu_supported: 1 / 0). */
int crnn_conv_fwd_bnrelu_supported(int dtype, const crnn_conv_desc* d);
/* the same with the stem's 2x2 / stride-2 max-pool after the ReLU (model/seresnet31.py:81-89,
 * conv0.3 -> conv0.4 -> relu -> maxpool): y[B][Ho/2][Wo/2][Co]; bf16, the halo stem geometry only */
int crnn_conv_fwd_bnrelu_pool_supported(int dtype, const crnn_conv_desc* d);
int crnn_conv_fwd_bnrelu_pool(int dtype, const crnn_conv_desc* d, const void* x, const void* w, void* y, const float* scale, const float* shift, void* stream);
int crnn_conv_fwd_bnrelu(int dtype, const crnn_conv_desc* d, const void* x, const void* w, void* y, const float* scale, const float* shift, void* stream);
/* dx[B][Hi][Wi][Ci] = dgrad(dy) (+= dx if accumulate) (+ dres*(yres>0) if dres != NULL). */
int crnn_conv_dgrad(int dtype, const crnn_conv_desc* d, const void* dy, const void* w, void* dx, const void* dres, const void* yres, int accumulate, void* stream);
/* dgrad of a residual block's strided pair in one pass (model/seresnet31.py:56 conv1 3x3 stride 2
 * and :64-67 downsample 1x1 stride 2, both reading the block input x): dx = dgrad_conv1(dy) +
 * dgrad_downsample(dy_ds), the downsample being one more tap of conv1's parity class (0, 0).
 * Layout contract: dy_ds follows dy in memory (dy + B*Ho*Wo*Co elements) and the downsample's
 * packed [Co][1][1][Ci] weights follow w (w + Co*9*Ci elements). d: conv1, dds: the downsample. */
int crnn_conv_dgrad_ds_supported(int dtype, const crnn_conv_desc* d, const crnn_conv_desc* dds);
int crnn_conv_dgrad_ds(int dtype, const crnn_conv_desc* d, const crnn_conv_desc* dds, const void* dy, const void* w, void* dx, void* stream);
/* dgrad fused with the BatchNorm backward sums of the layer before (conv input = ReLU(BN(z))):
 * dx as crnn_conv_dgrad (no accumulate / residual), plus per partial row r (128 rows of dx)
 * pg[r][c] = sum g, pgx[r][c] = sum g (z - mean) invstd with g = dx (z scale + shift > 0) — the
 * CRNN_BNG_RELU sums crnn_bn_bwd_reduce would compute, from the fp32 accumulators; feed them to
 * crnn_bn_bwd_finalize with rows = crnn_conv_dgrad_bnrelu_rows(). bf16, stride 1; rows = 0 means
 * the geometry is not supported (use crnn_conv_dgrad + crnn_bn_bwd_reduce). */
int crnn_conv_dgrad_bnrelu_rows(int dtype, const crnn_conv_desc* d);
int crnn_conv_dgrad_bnrelu(int dtype, const crnn_conv_desc* d, const void* dy, const void* w, void* dx, const void* z,
                           const float* mean, const float* invstd, const float* scale, const float* shift, float* pg,
                           float* pgx, void* stream);
/* stride-1 dgrad on the forward conv path: wt = the transposed, flipped kernel
 * wt[Ci][KH][KW][Co] = w[Co][KH-1-kh][KW-1-kw][Ci] (crnn_pack_conv_batch kind CRNN_PACK_CONV_T),
 * K-contiguous like a forward weight, so dgrad(dy) is the forward conv of dy with pad K-1-pad and
 * runs the forward's loaders, tiles and padding-row skip. Same outputs and epilogues as
 * crnn_conv_dgrad / crnn_conv_dgrad_bnrelu. bf16, stride 1, Co % 64 == 0, geometries on the 256-row
 * kernel: crnn_conv_dgrad_tw_rows = the pg / pgx partial rows of the bnrelu form (2 per 256 dx rows),
 * 0 when the geometry is not supported. */
int crnn_conv_dgrad_tw_rows(int dtype, const crnn_conv_desc* d);
int crnn_conv_dgrad_tw(int dtype, const crnn_conv_desc* d, const void* dy, const void* wt, void* dx, const void* dres,
                       const void* yres, int accumulate, void* stream);
int crnn_conv_dgrad_bnrelu_tw(int dtype, const crnn_conv_desc* d, const void* dy, const void* wt, void* dx,
                              const void* z, const float* mean, const float* invstd, const float* scale,
                              const float* shift, float* pg, float* pgx, void* stream);
/* dw_oihw (fp32, reference layout) = beta*dw + wgrad(dy, x); ws = split-K slabs. */
int crnn_conv_wgrad(int dtype, const crnn_conv_desc* d, const void* dy, const void* x, float* dw_oihw, float* ws, size_t ws_bytes, float beta, void* stream);
size_t crnn_conv_wgrad_workspace(int dtype, const crnn_conv_desc* d);
/* the two halves of crnn_conv_wgrad, so that the slab reduce can run on another stream (ordered by the
 * caller after the GEMM; the slab workspace must not be reused before the reduce has read it):
 * _gemm writes the split-K fp32 slabs into ws, _reduce sums them into dw_oihw (beta as above). */
int crnn_conv_wgrad_gemm(int dtype, const crnn_conv_desc* d, const void* dy, const void* x, float* ws, size_t ws_bytes,
                         void* stream);
int crnn_conv_wgrad_reduce(int dtype, const crnn_conv_desc* d, float* dw_oihw, const float* ws, size_t ws_bytes,
                           float beta, void* stream);
/* fwd tile (BM x BN) the library picks for (dtype, d): bf16 GEMM-sized convs run the 256-row
 * deep-pipelined kernel, fp32 (parity mode) and small ones the 128/64 kernels */
void crnn_conv_fwd_tile(int dtype, const crnn_conv_desc* d, int* bm, int* bn);
void crnn_conv_wgrad_plan(int dtype, const crnn_conv_desc* d, int* bm, int* bn, int* splits);

/* ------------------------------------------------------------------ batchnorm */
/* Combine (sum, M2) partials (Chan, in double) -> per-channel affine (scale = gamma*invstd,
 * shift = beta - mean*scale). train: batch statistics over `count` rows, partial r covering rows
 * [r*rows_per_partial, ...) (biased var to normalise, unbiased into running_var, momentum
 * update); eval: running statistics. mean/invstd saved for backward. */
int crnn_bn_finalize(const float* psum, const float* psq, int rows, long rows_per_partial, int C, long count,
                     const float* gamma, const float* beta,
                     float* running_mean, float* running_var, float momentum, float eps, int train,
                     float* mean, float* invstd, float* scale, float* shift, float* ws, void* stream);
/* bytes of `ws` crnn_bn_finalize / crnn_bn_bwd_finalize need for C channels: 64 ticket counters
 * then the chunk partials. ZERO it once before first use (the one-launch path's counters re-arm
 * themselves); calls sharing one workspace must be stream-ordered. */
size_t crnn_bn_finalize_workspace(int C);
/* per-channel (sum, M2) partials of an NHWC tensor [M][C] (for tensors not produced by a conv);
 * partial r covers ceil(M/rows) rows. */
int crnn_channel_stats(int dtype, const void* x, long M, int C, float* psum, float* psq, int rows, void* stream);
/* y = act(z*scale + shift), act = ReLU if relu. */
int crnn_bn_act(int dtype, const void* z, const float* scale, const float* shift, void* y, long M, int C, int relu, void* stream);
/* y = maxpool2x2(relu(z*scale+shift)), z [B][H][W][C] -> y [B][H/2][W/2][C]. */
int crnn_bn_relu_maxpool(int dtype, const void* z, const float* scale, const float* shift, void* y, int B, int H, int W, int C, void* stream);
/* dy_full[B][H][W][C] = gradient routed to the first max of each 2x2 window of relu(z*scale+shift). */
int crnn_maxpool_bwd(int dtype, const void* z, const float* scale, const float* shift, const void* dpool, void* dy_full, int B, int H, int W, int C, void* stream);

#define CRNN_BNG_PLAIN 0 /* g = dy                                   */
#define CRNN_BNG_RELU 1  /* g = dy * (z*scale+shift > 0)             */
#define CRNN_BNG_RESID 2 /* g = dy * (y > 0)                         */
#define CRNN_BNG_SE 3    /* g = dy * (y > 0) * s[b][c] + dpool[b][c] */
#define CRNN_BNG_POOL 4  /* BN -> ReLU -> MaxPool2d(2,2): dy = POOLED grad [B][H/2][W/2][C],   \
                            HW = full-res W (even H, W); g = dy at the window's first max of \
                            relu(z*scale+shift) when > 0, else 0 (crnn_maxpool_bwd fused)  */
#define CRNN_BNG_POOL_OUT 5 /* crnn_bn_bwd_reduce only: the CRNN_BNG_POOL sums from the POOLED output \
                            y [B][H/2][W/2][C] = maxpool(relu(z*scale+shift)) instead of z: a window \
                            contributes g = dy where y > 0, at xhat = ((y - shift)/scale - mean)*invstd \
                            (the max is one value of the window, so its z follows from y); z is read  \
                            only for channels with scale == 0 (all four tie: the first element). Reads \
                            the pooled tensors only: a quarter of the full-resolution z              */
typedef struct {
  const void* dy;
  const void* z;
  const float* mean;
  const float* invstd;
  const float* scale;
  const float* shift;
  const void* y;      /* RESID / SE */
  const float* s;     /* SE: [B][C] */
  const float* dpool; /* SE: [B][C], already divided by HW */
  int mode;
  long M; /* rows = B*HW */
  int C;
  int HW;
} crnn_bn_bwd_desc;
/* partials of sum(g), sum(g*xhat) -> [rows][C] each */
int crnn_bn_bwd_reduce(int dtype, const crnn_bn_bwd_desc* d, float* pg, float* pgx, int rows, void* stream);
/* -> dgamma, dbeta (written, or added if accumulate), mean_g = sum(g)/count, mean_gx = sum(g xhat)/count */
int crnn_bn_bwd_finalize(const float* pg, const float* pgx, int rows, int C, long count, float* dgamma, float* dbeta,
                         float* mean_g, float* mean_gx, int accumulate, float* ws, void* stream);
/* dz = scale * (g - mean_g - xhat*mean_gx) */
int crnn_bn_bwd_apply(int dtype, const crnn_bn_bwd_desc* d, const float* mean_g, const float* mean_gx, void* dz, void* stream);
int crnn_bn_rows(long M); /* partial rows used by the reduce kernels for M */

/* ------------------------------------------------------------------ SE + residual */
/* pooled[b][c] = mean_hw(z2*scale+shift) */
int crnn_se_pool(int dtype, const void* z2, const float* scale, const float* shift, float* pooled, int B, int HW, int C, void* stream);
/* the same pooled values in training mode from the SE conv's BN partial sums (crnn_conv_fwd psum,
 * `rows` partial rows of rows_per_partial data rows): requires HW % rows_per_partial == 0 and
 * rows * rows_per_partial == B * HW (partials tile each sample); no pass over z2 */
int crnn_se_pool_partials(const float* psum, int rows, long rows_per_partial, const float* scale,
                          const float* shift, float* pooled, int B, int HW, int C, void* stream);
/* hid = relu(pooled W1^T) [B][Cr]; s = sigmoid(hid W2^T) [B][C] (fp32; W1 [Cr][C], W2 [C][Cr]) */
int crnn_se_mlp_fwd(const float* pooled, const float* w1, const float* w2, float* hid, float* s, int B, int C, int Cr, void* stream);
/* crnn_se_pool_partials + crnn_se_mlp_fwd in ONE launch (the squeeze computed in the excitation
 * kernel's load stage, same arithmetic: pooled / hid / s bit-identical to the pair); pooled is
 * still written (the backward reads it). model/seresnet31.py:22-40 */
int crnn_se_pool_mlp_fwd(const float* psum, int rows, long rows_per_partial, const float* scale, const float* shift,
                         float* pooled, const float* w1, const float* w2, float* hid, float* s, int B, int HW, int C,
                         int Cr, void* stream);
/* y = relu((z2*scale+shift)*s[b][c] + idn'), idn' = idn*iscale+ishift if iscale else idn */
int crnn_se_residual_fwd(int dtype, const void* z2, const float* scale, const float* shift, const float* s,
                         const void* idn, const float* iscale, const float* ishift, void* y, int B, int HW, int C, void* stream);
/* crnn_se_residual_fwd with the block's DropBlock2d (model/seresnet31.py:61-62) between the SE gate
   and the residual add: y = relu((z2*scale+shift) * s * keep * B*HW*C / (1e-6 + *kept) + idn'). */
int crnn_se_residual_drop_fwd(int dtype, const void* z2, const float* scale, const float* shift, const float* s,
                              const void* idn, const float* iscale, const float* ishift, void* y, int B, int HW,
                              int C, const unsigned char* keep, const unsigned long long* kept, void* stream);
/* ds[b][c] = sum_hw dy*(y>0)*(z2*scale+shift) */
int crnn_se_bwd_reduce(int dtype, const void* dy, const void* y, const void* z2, const float* scale, const float* shift,
                       float* ds, int B, int HW, int C, void* stream);
/* SE block backward, one pass over (dy, y, z2) for both reductions (per sample b, channel c):
 *   dy_m = dy * (y > 0), xhat = (z2 - mean) * invstd
 *   abc[b][0][c] = sum_hw dy_m, abc[b][1][c] = sum_hw dy_m xhat, abc[b][2][c] = sum_hw xhat
 *   ds[b][c] = sum_hw dy_m (z2 scale + shift) = gamma abc[1] + beta abc[0]
 * crnn_se_bn_partials then gives the CRNN_BNG_SE BatchNorm sums as B partial rows for
 * crnn_bn_bwd_finalize (rows = B): pg = s abc[0] + HW dpool, pgx = s abc[1] + dpool abc[2] —
 * the same quantities crnn_bn_bwd_reduce computes with a second pass. */
int crnn_se_bn_bwd_reduce(int dtype, const void* dy, const void* y, const void* z2, const float* mean,
                          const float* invstd, const float* gamma, const float* beta, float* ds, float* abc, int B,
                          int HW, int C, void* stream);
int crnn_se_bn_partials(const float* abc, const float* s, const float* dpool, float* pg, float* pgx, int B, int HW,
                        int C, void* stream);
/* SE MLP backward: dsig, dhid (work [B][C] and [B][Cr]), dpool = W1^T dhid / HW; dw1/dw2 (fp32, written) */
int crnn_se_mlp_bwd(const float* ds, const float* pooled, const float* hid, const float* s, const float* w1, const float* w2,
                    float* dsig, float* dhid, float* dpool, float* dw1, float* dw2, int B, int C, int Cr, int HW, int accumulate,
                    void* stream);
/* the same, plus crnn_se_bn_partials' rows pg / pgx [B][C] from abc (crnn_se_bn_bwd_reduce) in the kernel that
 * produces dpool: one launch fewer per SE block (abc == NULL: no partials, = crnn_se_mlp_bwd) */
int crnn_se_mlp_bwd_partials(const float* ds, const float* pooled, const float* hid, const float* s, const float* w1,
                             const float* w2, float* dsig, float* dhid, float* dpool, float* dw1, float* dw2,
                             const float* abc, float* pg, float* pgx, int B, int C, int Cr, int HW, int accumulate,
                             void* stream);

/* ------------------------------------------------------------------ height collapse */
/* seq[b][w][c] = mean_h relu(z*scale+shift), z [B][Hh][W][C] */
int crnn_hpool_fwd(int dtype, const void* z, const float* scale, const float* shift, void* seq, int B, int Hh, int W, int C, void* stream);
/* dy_full[b][h][w][c] = dseq[b][w][c] / Hh */
int crnn_hpool_bwd(int dtype, const void* dseq, void* dy_full, int B, int Hh, int W, int C, void* stream);

/* ------------------------------------------------------------------ GEMM (linear layers) */
/* C[M][N] (ldc) = A[M][K] (lda) . B[N][K]^T (ldb) (+ bias[N]) (+= C if accumulate); C is fp32 if c_f32 else dtype */
int crnn_gemm_nt(int dtype, const void* A, int lda, const void* B, int ldb, void* C, int ldc, const float* bias,
                 int M, int N, int K, int c_f32, int accumulate, void* stream);
/* C[M][N] = A[M][K] . B[K][N] (ldb), N multiple of 8 */
int crnn_gemm_nn(int dtype, const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                 int M, int N, int K, int c_f32, int accumulate, void* stream);
/* C[M][N] fp32 (+)= A[K][M]^T . B[K][N]  (weight gradients; M, N multiples of 8) */
int crnn_gemm_tn(int dtype, const void* A, int lda, const void* B, int ldb, float* C, int ldc,
                 int M, int N, int K, int accumulate, void* stream);
/* out[n] (+)= sum_m X[m][n]  (bias gradients), X dtype or fp32 */
/* bf16 C (fp32, ldc) (+)= A^T B as above via split-K fp32 slabs + one reduce (deterministic);
 * ws: crnn_gemm_tn_workspace(M, N, K) bytes */
size_t crnn_gemm_tn_workspace(int M, int N, int K);
int crnn_gemm_tn_slab(const void* A, int lda, const void* B, int ldb, float* C, int ldc, int M, int N, int K,
                      int accumulate, float* ws, size_t ws_bytes, void* stream);
int crnn_colsum(int dtype, const void* X, int ld, long M, int N, float* out, int accumulate, int x_f32, void* stream);

/* ------------------------------------------------------------------ BiLSTM */
/* Gate-interleaved ("packed") layout: packed row 4*j+q <-> reference row q*H+j (q = i,f,g,o).
 * xg   [B][T][2][4H]  x W_ih'^T + b_ih' + b_hh' (dtype)
 * whh  [2][4H][H]     packed W_hh (dtype)
 * hseq [B][T][2H]     outputs, forward dir in [0,H), reverse dir in [H,2H) (dtype)
 * gsv  [2][T][B][4H]  saved post-activation gates (dtype); csv [2][T][B][H] saved cell state (fp32) */
int crnn_lstm_step_fwd(int dtype, const void* xg, const void* whh, void* hseq, void* gsv, float* csv, int B, int T, int H, int step, void* stream);
/* BPTT. dgates [2][T][B][4H] (dtype, pre-activation gate grads), dc [2][B][H] fp32 running cell grad.
 * step 0 initialises (dh_rec = 0, dc = 0); step s>0 runs dh_rec = dgates(step s-1) . W_hh with the
 * cell backward of step s fused into the GEMM epilogue. */
int crnn_lstm_step_bwd(int dtype, const void* dhseq, const void* whh, const void* whh_t, const void* gsv,
                       const float* csv, void* dgates, float* dc, float* ws, int B, int T, int H, int step, void* stream);
/* whh_t [2][H][4H] = packed W_hh transposed (bf16; CRNN_PACK_TRANSPOSE) and ws
 * (crnn_lstm_bptt_workspace bytes) enable the split-K one-shot step; NULL -> the staged kernel. */
size_t crnn_lstm_bptt_workspace(int B, int H);
/* dW_hh (reference row order, fp32 [2][4H][H]) (+)= sum_t dgates_t^T h_{t-1} */
int crnn_lstm_dwhh(int dtype, const void* dgates, const void* hseq, float* dwhh_fwd, float* dwhh_rev, int B, int T, int H, int accumulate, void* stream);
/* dW_ih (reference row order, fp32 [2][4H][In]) (+)= sum dgates^T x ; x [B][T][In] */
int crnn_lstm_dwih(int dtype, const void* dgates, const void* x, float* dwih_fwd, float* dwih_rev, int B, int T, int H, int In, int accumulate, void* stream);
/* db (reference order, fp32 [2][4H]) (+)= sum_{t,b} dgates */
/* bias gradient of each direction into both b_ih and b_hh (they receive the same gradient; b2_* may be NULL);
 * ws: crnn_lstm_dbias_workspace(H) bytes; deterministic (no atomics) */
int crnn_lstm_dbias(int dtype, const void* dgates, float* b_fwd, float* b2_fwd, float* b_rev, float* b2_rev, float* ws, int B, int T, int H, int accumulate, void* stream);
size_t crnn_lstm_dbias_workspace(int H);
/* dx [B][T][In] (dtype) = sum_dir dgates . W_ih'  (wih packed [2][4H][In]) */
int crnn_lstm_dx(int dtype, const void* dgates, const void* wih, void* dx, int B, int T, int H, int In, void* stream);
/* bf16: all four weight gradients of a layer (dW_ih and dW_hh, both directions, reference row
 * order, fp32, += if accumulate) in one batched split-K GEMM launch + one slab reduce. x [B][T][In],
 * hseq [B][T][2H], dgates [2][T][B][4H]; ws: crnn_lstm_wgrad_workspace bytes. */
size_t crnn_lstm_wgrad_workspace(int B, int T, int H, int In);
int crnn_lstm_wgrad(const void* dgates, const void* x, const void* hseq, float* dwih_f, float* dwih_r, float* dwhh_f,
                    float* dwhh_r, float* ws, size_t ws_bytes, int B, int T, int H, int In, int accumulate,
                    void* stream);
/* Persistent whole-sequence recurrence (bf16 only; replaces the T per-step launches of
 * crnn_lstm_step_fwd / crnn_lstm_step_bwd with ONE launch per layer and direction pair, same
 * buffers and results). One workgroup per (direction, S samples, U units), S x U chosen per
 * sweep by crnn_lstm_seq_config() among 16 x 32, 32 x 32 and 16 x 64 (H <= 512) such that the
 * grid 2*(B/S)*(H/U) fits the device's CU count (all resident); H in {256, 512, 768}.
 * ws: crnn_lstm_seq_workspace(B) bytes of device memory, the used part zeroed by the call itself:
 * [2*(B/16+1)] step counters (the first 2*B/S used; counter of slice (d, bs) = d*(B/S)+bs reaches
 * (H/U)*T) then one error word (non-zero after a bounded wait timed out, in which case the outputs
 * carry NaN), then (256-B aligned) the forward's hand-off ring of 2*B*H 8-byte granules
 * {2 bf16 of h_t, u32 tag}, then at crnn_lstm_seq_status_offset(B) a sticky status word that no
 * call zeroes (the caller zeroes it once, at allocation): every call ORs its error word into it,
 * so the host can poll one word for "any persistent sweep since allocation timed out". */
int crnn_lstm_seq_supported(int dtype, int B, int H);
size_t crnn_lstm_seq_status_offset(int B);
/* the (samples, units) workgroup tile the forward (bwd = 0) or BPTT (bwd = 1) sweep uses for
 * (B, H); 0 if unsupported */
int crnn_lstm_seq_config(int B, int H, int bwd, int* S, int* U);
/* diagnostics: record per-phase s_memrealtime stamps of the following persistent launches into a
 * device buffer of (grid * T * 8) u64 (NULL: off) */
int crnn_lstm_seq_debug_stamps(unsigned long long* buf);
/* measurement: record the two hipEvent_t right before and right after the NEXT persistent sweep's
 * kernel on its stream (not around the counter memset and the status kernel the call also
 * enqueues); one-shot, NULL pairs are ignored */
int crnn_lstm_seq_time_next(void* ev_start, void* ev_end);
size_t crnn_lstm_seq_workspace(int B);
/* gsv / csv: the gates and cell states BPTT reads, or both NULL (inference: not stored) */
int crnn_lstm_seq_fwd(const void* xg, const void* whh, void* hseq, void* gsv, float* csv, unsigned* ws, int B, int T,
                      int H, void* stream);
/* BPTT: dhseq [B][T][2H] upstream grad, whh_t [2][H][4H] -> dgates [2][T][B][4H] */
int crnn_lstm_seq_bwd(const void* dhseq, const void* whh_t, const void* gsv, const float* csv, void* dgates,
                      unsigned* ws, int B, int T, int H, void* stream);

/* ------------------------------------------------------------------ attention decoder (fp32)
 * The reference's attention head (model/model.py:23-148), one decoder step
 * per call sequence (host loop: crnn_hip/attn.py):
 *   crnn_gemm_nt  proj_h = h W_h2h^T + b_h2h            (proj_H = enc W_i2h^T once per decode)
 *   crnn_attn_context: alpha = softmax_t(score . tanh(proj_H[b,t] + proj_h[b])),
 *                      ctx[b][0..C) (row stride ldc) = sum_t alpha' enc[b,t]; alpha (optional
 *                      output) = the softmax; alpha' = alpha * mask / (1 - drop_p), the
 *                      training-mode F.dropout(alpha) of model/model.py:38, mask element (b, t) kept
 *                      iff splitmix64(seed ^ (b*T + t) * golden) >> 32 >= drop_p * 2^32 (0 = off)
 *   crnn_gemm_nt  gates = hx W_cat^T, hx = [ctx | h] rows, W_cat = [W_ih[:, :C] | W_hh]
 *   crnn_attn_cell: LSTMCell (i, f, g, o) with + b_ih + b_hh + W_ih[:, C + ch[b * ch_stride]]
 *                   (the one-hot input); writes h, c, hx[b][C + j] and hs (optional)
 *   crnn_gemm_nt  logits = h W_gen^T + b_gen
 *   crnn_attn_out: blank column masked to -1e4, logits -> probs_t (optional), argmax -> ch */
int crnn_attn_context(const float* projH, const float* projh, const float* score, const float* enc, float* ctx,
                      int ldc, float* alpha, int B, int T, int H, int C, float drop_p, unsigned long long seed,
                      void* stream);
/* the same with proj_H and enc stored as bf16 (the bf16 training pass, AttnDecoderHIP(train_bf16=True): the
 * reference's fp16 autocast runs this attention on fp16 tensors, training/train.py:499-505); fp32 arithmetic */
int crnn_attn_context_bf16(const void* projH, const float* projh, const float* score, const void* enc, float* ctx,
                           int ldc, float* alpha, int B, int T, int H, int C, float drop_p, unsigned long long seed,
                           void* stream);
int crnn_attn_cell(const float* gates, const float* b_ih, const float* b_hh, const float* w_ih, int ldw, const int* ch,
                   int ch_stride, float* h, float* c, float* hx, int ldx, float* hs, int ld_hs, float* gact, float* cs,
                   int B, int H, int C, void* stream);
/* the gate GEMM and the cell in one launch: gates = X[B][C+H] W^T (+ b_ih + b_hh + the one-hot column) -> LSTMCell,
 * with W [4H][C+H] (ldw), b_ih / b_hh [4H] and wv [V][4H] (wv[ch][r] = W_ih[r][C + ch]) in GATE-INTERLEAVED row order
 * (row 4u + q = the reference's row q*H + u, q = i f g o); writes h, c, hx[b][C + j] (row stride ldhx; must not be X),
 * hs (optional) and gact / cs (optional, the reference's gate-block order) as crnn_attn_cell does, bit for bit.
 * dtype CRNN_F32 or CRNN_F32_BF16MMA (the GEMM of crnn_gemm_nt with that dtype) */
int crnn_attn_gates_cell(int dtype, const float* X, int ldx, const float* W, int ldw, const float* b_ih,
                         const float* b_hh, const float* wv, const int* ch, int ch_stride, float* h, float* c,
                         float* hx, int ldhx, float* hs, int ld_hs, float* gact, float* cs, int B, int H, int C,
                         void* stream);
/* backward (teacher forcing; host loop in crnn_hip/attn.py): gact = the activated gates
 * (i f g o) and cs = c_t the forward saved (crnn_attn_cell's optional outputs), c_prev NULL at
 * t = 0; dh = dh1 + dh2 (row strides ld1, ld2; either NULL), dc NULL = 0 -> dgates
 * (pre-activation) and dc_prev */
int crnn_attn_cell_bwd(const float* gact, const float* c_t, const float* c_prev, const float* dh1, int ld1,
                       const float* dh2, int ld2, const float* dc, float* dgates, float* dc_prev, int B, int H,
                       void* stream);
/* attention backward for one step (block per sample): de[b][t'] = alpha (dalpha - sum alpha dalpha)
 * with dalpha_t' = mask/(1-p) dctx . enc_t'; dprojh[b] = score * sum_t' de (1 - tanh^2 u_t');
 * dscore_part[b] += sum_t' de tanh(u_t') (u = proj_H + proj_h; csrc/attn.hip). drop_p, seed = the
 * forward step's (the mask is regenerated, not stored). No [B][T][*] array is written per step: */
int crnn_attn_bwd(const float* dctx, int lddc, const float* alpha, const float* enc, const float* projH,
                  const float* projh, const float* score, float* de, float* dprojh, float* dscore_part, int B, int T,
                  int H, int C, float drop_p, unsigned long long seed, void* stream);
/* the same with enc and proj_H stored as bf16 (pairs with crnn_attn_context_bf16) */
int crnn_attn_bwd_bf16(const float* dctx, int lddc, const float* alpha, const void* enc, const void* projH,
                       const float* projh, const float* score, float* de, float* dprojh, float* dscore_part, int B,
                       int T, int H, int C, float drop_p, unsigned long long seed, void* stream);
/* after the step loop: denc[b][t'][c] = sum_t alpha'_t[b][t'] dctx_t[b][c] (written; dctx rows
 * [steps][B] of stride lddc, alpha [steps][B][T], step t's mask from seed + t) */
int crnn_attn_denc(const float* dctx, int lddc, const float* alpha, int steps, int B, int T, int C, float drop_p,
                   unsigned long long seed, float* denc, void* stream);
/* dprojH[b][t'][k] = score_k sum_t de_t[b][t'] (1 - tanh^2(proj_H[b][t'][k] + proj_h_t[b][k]))
 * (proj_h [steps][B][H], de [steps][B][T]; written) */
int crnn_attn_dproj_enc(const float* projh, const float* de, const float* projH, const float* score, int steps, int B,
                     int T, int H, float* dprojH, void* stream);
/* the same with proj_H stored as bf16 (pairs with crnn_attn_context_bf16) */
int crnn_attn_dproj_enc_bf16(const float* projh, const float* de, const void* projH, const float* score, int steps,
                             int B, int T, int H, float* dprojH, void* stream);
/* teacher-forcing one-hot rows: X[t][b][col0 + text[b][t]] = 1 (rows [steps][B] of stride ldx,
 * zeroed by the caller; ids outside [0, V) leave the row zero) — the saved [context | h | onehot]
 * rows make dW_ih (both parts) and dW_hh one GEMM in the backward */
int crnn_attn_onehot_rows(const int* text, int text_ld, int steps, int B, int V, float* X, int ldx, int col0,
                          void* stream);
int crnn_attn_out(const float* logits, int ldl, int B, int V, int blank, float* probs_t, int ldp, int* ch,
                  void* stream);
/* the attention head's training loss, nn.CrossEntropyLoss(ignore_index) (training/train.py:289,503):
 * logits [M][ldl] (V used), targets [M] -> loss[0] = mean over rows with target != ignore_index of
 * (logsumexp - logit[target]); dlogits [M][ldd] (may be NULL) = d loss / d logits.
 * ws: M + 1 floats of scratch. */
int crnn_attn_xent(const float* logits, int ldl, const int* targets, int M, int V, int ignore_index, float* loss,
                   float* dlogits, int ldd, float* ws, void* stream);

/* ------------------------------------------------------------------ input pipeline
 * ResizeAndPadA + A.Normalize(0.5, 0.5) + ToTensorV2 (data/transforms.py:62-120, :185-193) for a
 * ragged batch of uint8 HWC crops packed back to back in `src` (device memory). Per crop the
 * caller fills the reference's geometry (data/transforms.py:91-118: new size, alignment offsets,
 * interp 0 = INTER_LINEAR / 1 = INTER_AREA); c = 1 (gray, replicated), 3 (RGB) or 4 (RGBA, alpha
 * dropped). out_kind 0: fp32 NCHW [B][3][H][W] (the reference's tensor); 1: the encoder input
 * [B][H][W][8] in dtype (channels 3..7 zero; what crnn_nchw_to_nhwc makes of kind 0);
 * 2: the uint8 canvas [B][H][W][3] before normalisation. */
typedef struct {
  long long offset; /* byte offset of the crop in src */
  int h, w, c;      /* source size, channels */
  int new_h, new_w; /* resized size */
  int y0, x0;       /* placement on the white canvas */
  int interp;       /* 0 linear, 1 area (the reference's _interp) */
  int pad;
} crnn_crop_desc;
int crnn_preprocess(const unsigned char* src, const crnn_crop_desc* desc, int B, int H, int W, int out_kind,
                    int dtype, void* out, void* ws, long ws_bytes, void* stream);
/* bytes of device workspace crnn_preprocess needs (the per-column / per-row resampling taps) */
long crnn_preprocess_workspace(int B, int H, int W);

/* ------------------------------------------------------------------ CTC */
/* Per-sample log-space CTC over logits [B][T][ldc] (fp32, C classes, blank = 0, input length T).
 * loss[b] = -log p(target_b); dlogits (may be NULL) = grad of the 'mean' reduction
 * (mean_b loss_b/len_b) wrt logits, with zero_infinity semantics if zero_inf. */
int crnn_ctc_loss(const float* logits, int ldc, int B, int T, int C, const int* targets, int Lmax, const int* lengths,
                  float* loss, float* dlogits, int zero_inf, void* stream);
/* mean_b(loss_b / max(len_b,1)) -> out[0] */
int crnn_ctc_reduce_mean(const float* loss, const int* lengths, int B, float* out, void* stream);
/* greedy decode (training/utils.py:122-150 semantics, explicit [B][T] layout):
 * ids [B][T] collapsed labels (blank & repeats removed, zero past lens[b]), lens [B];
 * logits rows have stride ldc >= C; T <= 16384 (the per-sample argmax row lives in LDS) */
int crnn_ctc_greedy(const float* logits, int ldc, int B, int T, int C, int* ids, int* lens, void* stream);

/* ------------------------------------------------------------------ optimiser */
/* fused Adam / AdamW over a flat fp32 buffer (one launch; replaces torch.optim.Adam / AdamW,
 * training/train.py:292-295): g is multiplied by grad_scale first (DP averaging); coupled = 1 is
 * torch.optim.Adam's L2 decay (g += weight_decay * p before the moments, the reference's default
 * optimizer "Adam"), coupled = 0 AdamW's decoupled decay (p *= 1 - lr * weight_decay).
 * skip: null, or a device int32 status word (the persistent BiLSTM's sticky error word,
 * crnn_lstm_seq_status_offset): when it is non-zero the kernel leaves p, m and v untouched.
 * step counts from 1 (bias corrections 1 - beta^step). */
int crnn_adam_step(float* p, const float* g, float* m, float* v, long n, float lr, float beta1, float beta2,
                   float eps, float weight_decay, int step, float grad_scale, int coupled, const int* skip,
                   void* stream);
/* fused SGD (torch.optim.SGD with momentum, dampening 0, no Nesterov; training/train.py:296-299):
 * d = grad_scale*g + weight_decay*p; momentum_buf = d on the first step (first_step = 1), else
 * momentum*momentum_buf + d; p -= lr*momentum_buf (momentum = 0: p -= lr*d, buffer unused).
 * skip as crnn_adam_step. */
int crnn_sgd_step(float* p, const float* g, float* momentum_buf, long n, float lr, float momentum,
                  float weight_decay, float grad_scale, int first_step, const int* skip, void* stream);
/* AdamW without a status guard: crnn_adam_step(..., coupled = 0, skip = null) */
int crnn_adamw(float* p, const float* g, float* m, float* v, long n, float lr, float beta1, float beta2, float eps,
               float weight_decay, int step, float grad_scale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CRNN_HIP_H */
