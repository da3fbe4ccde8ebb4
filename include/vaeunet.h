/*
 * vaeunet.h — C-ABI of the MI355X-native VAE-U-Net training hot path.
 *
 * The reference (tmuird/VAEUNET) is pure Python on PyTorch: its "plugin API"
 * is torch.nn.Module + autograd, and the device work it reaches is ATen
 * (SURVEY.md §2b).  This library replaces those ATen calls on the hot path
 * (SURVEY.md §8a rows A-Q).  Every entry point takes plain device pointers,
 * sizes and a hipStream_t (passed as void*), launches asynchronously on that
 * stream and returns 0 or a hipError_t code.  No torch types cross this
 * boundary; the Python host side (vaeunet_amd/_lib.py) binds it with ctypes,
 * which is how a Python reference would bind any C library
 * (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   dtype   : 0 = fp32 (parity mode), 1 = bf16 (autocast / speed mode)
 *   layout  : activations are NHWC with a pixel stride (elements) so that a
 *             channel slice of a wider tensor can be addressed in place
 *             (torch channels_last tensors are exactly this).
 *   stats   : BatchNorm partial statistics are (sum, centered M2) per
 *             (row-tile, channel); they are combined in fp64 with Chan's
 *             formula, in a fixed order (bitwise reproducible).
 */
#ifndef VAEUNET_H
#define VAEUNET_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Implicit-GEMM operand: element [m][k] of a (virtual) im2col matrix.
 * m = (n*H + h)*W + w over the row grid, k = (r*S + s)*C + c over taps and
 * channels.  The source pixel is (h*sy + r*dy + oy, w*sx + s*dx + ox) in a
 * (Hs, Ws) image; out-of-range pixels read as 0 (zero padding).  Channel c
 * comes from source t where cend[t-1] <= c < cend[t] (channel concat,
 * unet_parts.py:94 / unet_resnet.py:98 never materialised).
 *   3x3 conv fwd (unet_parts.py:40,43): R=S=3, sy=sx=dy=dx=1, oy=ox=-1
 *   1x1 conv     (unet_parts.py:11,15,19,100): R=S=1, oy=ox=0
 *   ConvT 2x2 s2 input-grad gather (unet_parts.py:76): R=S=2, sy=sx=2 */
typedef struct VuGather {
  const void* src[3];
  int64_t stride[3];   /* pixel stride of each source, elements */
  int32_t cend[3];     /* cumulative channel end of each source */
  int32_t nsrc;
  int32_t C;           /* channels per tap (== cend[nsrc-1]) */
  int32_t N, H, W;     /* row grid */
  int32_t Hs, Ws;      /* source image */
  int32_t R, S;        /* taps */
  int32_t sy, sx, dy, dx, oy, ox;
} VuGather;

/* out[m][j] = sum_k A[m][k] * B[j][k] (+ bias), B dense [ncol][ldb].
 * out_mode 0: out[m*out_stride + out_coff + j]
 * out_mode 1: ConvTranspose 2x2/s2 pixel shuffle, j = (a*2+b)*cout + co ->
 *             out pixel (n, 2h+a+opy, 2w+b+opx) of an (oH, oW) image.
 * out_mode 2: stride-2 sub-lattice: row m -> out pixel (n, 2h+opy, 2w+opx)
 *             of an (oH, oW) image (one parity class of a stride-2 conv's
 *             input gradient, ResNet encoder of unet_resnet.py:131).
 * stat_sum/stat_m2 (optional): per (row tile, column) sum and centered M2 of
 * the stored (dtype-rounded) values, for BatchNorm (unet_parts.py:41,44). */
typedef struct VuGemmFwd {
  VuGather a;
  const void* b;
  int64_t ldb;
  int32_t ncol;
  int32_t out_mode;
  void* out;
  int64_t out_stride;
  int32_t out_coff;
  int32_t oH, oW, opy, opx, cout;
  const float* bias;
  float* stat_sum;
  float* stat_m2;
  int32_t accumulate;  /* out += result (gradient accumulation) */
  int32_t ksplit;      /* set by the library (split-K ways); callers pass 0 */
  float* workspace;    /* fp32 split-K slabs, vu_gemm_fwd_workspace_bytes() */
  /* Optional BatchNorm-backward partial sums of the OUTPUT (an input gradient
   * that feeds the backward of a train-mode BatchNorm(+ReLU) over bnb_x, the
   * BN's pre-normalisation input, same shape as the output, bnb_xstride
   * elements per pixel): for output row tile r of vu_gemm_fwd_bnb_tile()
   * pixels and channel c (ncol = C, out_coff 0, no accumulate),
   *   bnb_part[(2r + 0) * ncol + c] = sum dz,
   *   bnb_part[(2r + 1) * ncol + c] = sum dz * (x - bnb_mean[c]) * bnb_invstd[c],
   *   dz = stored output * (x * bnb_scale[c] + bnb_shift[c] > 0 if bnb_relu)
   * -- what vu_bn_bwd_reduce's first stage computes, finished by
   * vu_bn_bwd_finish.  bnb_part = NULL: not requested. */
  const void* bnb_x;
  int64_t bnb_xstride;
  const float* bnb_scale;
  const float* bnb_shift;
  const float* bnb_mean;
  const float* bnb_invstd;
  float* bnb_part;
  int32_t bnb_relu;
  /* epilogue ReLU: out = relu(acc + bias) before the storage rounding and the
   * statistics (an eval-mode BatchNorm folded into the weights and bias,
   * vaeunet_amd.engine.fold_bn_eval; with accumulate it applies to the new
   * term; not with bnb_part).  0 = none. */
  int32_t relu;
  /* Optional per-sample, per-border-class bias (round 5): the latent-broadcast
   * shortcut of a DecoderBlock's conv1 (unet/unet_resnet.py:37-41, 92-99).
   * The z_proj source of that conv is a per-sample constant map c_n, so its
   * share of the 3x3 conv is sum over the taps INSIDE the image of W_z c_n:
   * one of 9 vectors per sample by the pixel's border class.  Before the
   * storage rounding, the ReLU and the statistics:
   *   out[m][j] += zbias[(n * 9 + cls) * ncol + j],   m = (n, h, w),
   *   cls = 3 * rc(h, H) + rc(w, W),  rc(v, L) = v == 0 ? 0 : v == L - 1 ? 2 : 1
   * (vu_zbias_fwd builds the table).  out_mode 0, H >= 2, W >= 2, no
   * bnb_part; served by the ping-pong kernel (incl. its split-K finish) and
   * the generic kernel -- the dispatcher keeps such problems on those.
   * NULL: none. */
  const float* zbias;
} VuGemmFwd;

/* Weight-gradient GEMM: out[s][i][j] = sum_{m in split s} P[m][i] * Q[m][j]
 * (fp32 slabs, one per split of the m range; reduced by vu_slab_reduce). */
typedef struct VuGemmWgrad {
  VuGather p;
  VuGather q;
  int32_t ni, nj;
  int32_t splits;
  int64_t m_per_split;
  float* out;
} VuGemmWgrad;

/* ---- GEMM family ------------------------------------------------------ */
int vu_gemm_fwd(const VuGemmFwd* args, int dtype, void* stream);
int64_t vu_gemm_fwd_row_tile(const VuGemmFwd* args, int dtype);  /* BM used */
/* Pixels per BatchNorm-backward partial row tile when the kernel the
 * dispatcher picks for this problem can emit bnb_part (bf16, 3x3 stride-1
 * kernels: the resident-weight 64 -> 64 kernel and the ping-pong kernel incl.
 * its split-K finish), else 0 (the caller then runs vu_bn_bwd_reduce). */
int64_t vu_gemm_fwd_bnb_tile(const VuGemmFwd* args, int dtype);
/* bytes of args->workspace the dispatcher needs for this problem (0 = none):
 * the split-K slabs of the 3x3 kernel when its grid is under one block per CU */
int64_t vu_gemm_fwd_workspace_bytes(const VuGemmFwd* args, int dtype);
/* the kernel the dispatcher picks for this problem (tests): 1 generic, 2 v2
 * LDS-DMA tiles, 3 v3 halo, 4 v4 ping-pong, 5 v5 persistent short-K, 6 v6
 * resident weights, 7 v7 small-grid, 8 1x1 stream, 9 image conv, 10 7x7 stem,
 * 12 v2 small-grid mode, 13 v2 tail (small grids no other rule admits) */
int vu_gemm_fwd_kernel(const VuGemmFwd* args, int dtype);
int vu_gemm_wgrad(const VuGemmWgrad* args, int dtype, void* stream);
/* output tile (BI x BJ) the dispatcher picks for this problem (split-K sizing) */
int vu_gemm_wgrad_tile(const VuGemmWgrad* args, int dtype, int* bi, int* bj);
/* out[i*s_i + (j / C)*s_tap + (j % C)*s_c] (=|+=) sum_s slab[s][i][j],
 * skipping channels (j % C) >= cvalid (zero-padded input channels) */
int vu_slab_reduce(const float* slab, int splits, int ni, int nj, int C,
                   int cvalid, int64_t s_i, int64_t s_tap, int64_t s_c,
                   float* out, int accumulate, void* stream);

/* Dispatcher tuning (tests / experiments):
 *   VU_TUNE_V4_MIN_BLOCKS: smallest grid for which the ping-pong 3x3 kernel
 *     (gemm_fwd4.hip) is used without split-K (default 256 = one block per
 *     CU; 0 forces it);
 *   VU_TUNE_V4_SPLITK: 0 = no split-K, 1 = automatic (default: grids of
 *     16..255 256x256 tiles are split to reach one block per CU), k >= 2 =
 *     k-way split wherever the ping-pong kernel serves (tests);
 *   VU_TUNE_FP8_GRID: cap on the grid of the persistent fp8 kernel (default
 *     0 = CU count; tests use small caps so that every block walks several
 *     tiles);
 *   VU_TUNE_STREAM: 1 (default) lets the short-K 1x1 stream kernel
 *     (gemm_stream.hip) serve the problems it takes, 0 routes them to v2;
 *   VU_TUNE_V4_SPLIT_CHUNKS: fewest 32-channel chunks per automatic split-K
 *     slice (default 2);
 *   VU_TUNE_V2_SMALL: 1 (default) serves small grids (too few 256-row
 *     tiles) with 128x64 4-wave v2 tiles instead of split-K / v3;
 *   VU_TUNE_V5: 1 (default) serves the short-K 1x1 / ConvTranspose GEMMs
 *     with the persistent v5 kernel (gemm_fwd5.hip), 0 routes them to v2,
 *     k >= 2 caps its grid at k blocks (tests: several tiles per block);
 *   VU_TUNE_V6: 1 (default) serves 64 -> 64 3x3 convs (and their input
 *     gradients) with >= 1 tile of 16x32 pixels per CU with the
 *     resident-weight persistent kernel (gemm_fwd6.hip), 0 routes them to
 *     v3/v4, k >= 2 serves any grid with the grid capped at k (tests). */
#define VU_TUNE_V4_MIN_BLOCKS 0
#define VU_TUNE_FP8_GRID 4
#define VU_TUNE_STREAM 5
#define VU_TUNE_V4_SPLITK 6
#define VU_TUNE_V4_SPLIT_CHUNKS 8
#define VU_TUNE_V2_SMALL 9
#define VU_TUNE_V5 10
#define VU_TUNE_V6 11
/*   VU_TUNE_GEN: highest kernel generation the GEMM dispatchers may pick
 *     (1 = generic only ... 4 = all, the default);
 *   VU_TUNE_SLAB4: 0 = scalar split-K slab reduce (default 1 = vectorised);
 *   VU_TUNE_V2_CFG: tile configuration of short-K v2 GEMMs (0 default, 1, 2);
 *   VU_TUNE_BN_NT_MB: streamed-tensor size (MB) from which the BatchNorm
 *     passes use non-temporal loads (default 32; -1 = never).
 * The library reads no environment variables: these are the only knobs. */
#define VU_TUNE_GEN 12
#define VU_TUNE_SLAB4 13
#define VU_TUNE_V2_CFG 14
#define VU_TUNE_BN_NT_MB 15
/*   VU_TUNE_V7: small-grid 3x3 kernel (gemm_fwd7.hip): 0 = off (v4 split-K /
 *     v2 small-grid tiles), 1 = default (grids under one 256x256 tile per CU,
 *     except 32-pixel-wide ones with >= 512 input channels, which stay on the
 *     ping-pong split-K), 2 = every small grid. */
#define VU_TUNE_V7 16
/*   VU_TUNE_V7_NBW: weight-ring slots (tap rows) of the small-grid kernel (3 default, 4) */
#define VU_TUNE_V7_NBW 17
/*   VU_TUNE_V7_XM: experiment mode of the small-grid kernel (A/B timing runs
 *     only, results are wrong): 0 off, 2 no DMA inside the loop, 4 no loop */
#define VU_TUNE_V7_XM 18
/*   VU_TUNE_W3_SMALL: 1 (default) lets the halo weight-gradient kernel take
 *     16-pixel-wide images and use 64-channel tiles on small grids; 0 = the
 *     round-2 rules (A/B runs) */
#define VU_TUNE_W3_SMALL 19
/*   VU_TUNE_FP8_XM: experiment mode of the fp8 conv (A/B timing only, results
 *     wrong): 0 off, 1 no MFMAs, 2 no DMA inside the loop */
#define VU_TUNE_FP8_XM 20
/*   VU_TUNE_FP8_PP: fp8 conv schedule: 1 (default) one tile per block on the
 *     ping-pong step loop, 0 the persistent kernel (also used whenever
 *     VU_TUNE_FP8_GRID caps the grid) */
#define VU_TUNE_FP8_PP 21
/*   VU_TUNE_ATTN: 1 (default) batched attention-gate kernels (U pixel rows /
 *     vectors of loads in flight per lane), 0 = one row per iteration,
 *     2 = as 1 with the psi backward that emits the BatchNorm partials on
 *     two rows per lane (fewer VGPRs, one more wave per SIMD) */
#define VU_TUNE_ATTN 22
/*   VU_TUNE_FP8_C64: 1 (default) 64 -> 64 fp8 convs on the resident-weight
 *     tile-stream kernel (statistics row tile 64), 0 = the step-loop kernel */
#define VU_TUNE_FP8_C64 23
/*   VU_TUNE_FP8_SPLIT: 1 (default) split-K for fp8 grids under one block per
 *     CU (slabs in VuConvFp8.workspace + the split-K finish), 0 off */
#define VU_TUNE_FP8_SPLIT 24
/*   VU_TUNE_BN_MINBLK: fewest blocks of the BatchNorm streaming kernels on
 *     small tensors (default 256; 0 = ~16 pixel rows per thread only).
 *     (Was 23 until round 4, the same key as VU_TUNE_FP8_C64, which took it.) */
#define VU_TUNE_BN_MINBLK 25
/*   VU_TUNE_W3_FAST: 1 (default) the halo weight-gradient main loop with
 *     immediate-offset fragment reads and incremental tile addressing, 0 the
 *     round-3 loop, 2 the round-4 loop without s_setprio (A/B runs) */
#define VU_TUNE_W3_FAST 26
/*   VU_TUNE_PP_FULL: 1 (default) = the ping-pong 3x3 kernel runs one read
 *     segment and one 32-MFMA segment per step (2 barriers) instead of two
 *     halves (0; bit-identical outputs) */
#define VU_TUNE_PP_FULL 27
/*   VU_TUNE_W2_BIG: 1 = 256 x 256 output tiles for the 1x1 / ConvT weight
 *     gradients with both dimensions >= 256 (0 = 128 x 256) */
#define VU_TUNE_W2_BIG 28
/*   VU_TUNE_V6_XM: experiment modes of the resident-weight 64 -> 64 kernel
 *     (0 default; 1 = s_setprio around each tap's MFMAs; 2-4 = timing
 *     decompositions with wrong results: no in-loop halo DMA, no epilogue
 *     statistics / stores, fragments read once per group). */
#define VU_TUNE_V6_XM 29
/*   VU_TUNE_PP_PERSIST: 1 = the ping-pong kernel's 128/256-column tiles as a
 *     persistent walk (one block per CU; the next tile's first halo and
 *     weights stream in during the current tile's epilogue), 0 (default) =
 *     one tile per block. */
#define VU_TUNE_PP_PERSIST 30
/*   VU_TUNE_BN_ONEPASS: 1 = vu_bn_bwd_fused runs bf16 tensors of at most
 *     8192 pixels as ONE launch (a block per 8 channels reduces and
 *     applies); 0 (default) = the two-launch path (the one-launch form
 *     measured 12 % slower on config 3: uncoalesced channel slices). */
#define VU_TUNE_BN_ONEPASS 31
/*   VU_TUNE_STREAM_PD: tiles of operand loads each wave of the 1x1 stream
 *     kernel (gemm_stream.hip) keeps in flight beyond the one it computes:
 *     1 or 2. */
#define VU_TUNE_STREAM_PD 32
/*   VU_TUNE_UNSAFE: 1 = allow the experiment modes (VU_TUNE_V6_XM,
 *     VU_TUNE_V7_XM, VU_TUNE_FP8_XM) to be set non-zero; several of them
 *     produce wrong results by design (timing decompositions).  Without it a
 *     non-zero experiment mode is refused (hipErrorInvalidValue). */
#define VU_TUNE_UNSAFE 33
/*   VU_TUNE_V6_STAG: 1 (default) = the resident-weight 64 -> 64 kernel with
 *     the two wave halves' epilogues staggered into the next tile's first
 *     group (bit-identical results), 0 = the round-5 lock-step kernel. */
#define VU_TUNE_V6_STAG 34
/*   VU_TUNE_BN_STATS1: 1 = vu_bn_finalize as one launch (the last block of
 *     each channel group combines the group's partials, handed off through
 *     write-through stores and one agent-scope atomic per block; measured
 *     0.6-1.1 % slower per step than the two launches), 0 (default) = the
 *     two-launch path (stage 1 + stage 2).  Same fp64 combine up to the
 *     summation order. */
#define VU_TUNE_BN_STATS1 35
/*   VU_TUNE_V5_GRP: 1 = the persistent short-K 1x1 / ConvT GEMM walks its
 *     tiles in 4 x 8 blocks per 32 consecutive tiles (one XCD's share of a
 *     round) when the tile grid divides that way, 0 (default) = row-major
 *     (the grouping measured 5-8 % slower on the up1 / up2 ConvT GEMMs:
 *     per XCD, sharing A across 16 column tiles beats the smaller set). */
#define VU_TUNE_V5_GRP 36
/*   VU_TUNE_V5_WIDE: 1 = the persistent short-K 1x1 / ConvT GEMM takes
 *     256 x 256 output tiles on 32-wide K steps (half the operand bytes per
 *     MFMA of the 256 x 128 tiles, the same 96 KB in flight) for problems with
 *     a full round of such tiles and no accumulate; 0 (default) = 256 x 128
 *     (the wide tiles measured 3-15 % slower per shape: each step fetches
 *     half cache lines of every operand row). */
#define VU_TUNE_V5_WIDE 37
int vu_gemm_set_tuning(int key, int value);
/* Bit mask of the experiment modes currently non-zero (bit 0 V6_XM, 1 V7_XM,
 * 2 FP8_XM): 0 in production.  bench.py refuses to report while it is not. */
int vu_gemm_experiment_modes(void);
/* ABI check: out[0..7] = sizeof VuGather, VuGemmFwd, VuGemmWgrad, VuConvFp8,
 * VuPermJob, VuMtEntry, VuLatentJob, VuLatentHeads as this library was
 * compiled (bindings compare their own struct sizes against it;
 * tests/test_modules.py) */
void vu_abi_struct_sizes(int64_t* out);

/* ---- fp8 (OCP e4m3fn) 3x3 conv forward: BASELINE.json configs[4] ------- */
/* *amax (= or max=) max |x| over P pixels x C channels (C % 8 == 0); exact
 * and order-independent (integer max of the float bits) */
int vu_amax(const void* x, int64_t xs, int64_t P, int C, float* amax,
            int accumulate, int dtype, void* stream);
/* y = e4m3(clamp(x * s, +-448)) round-to-nearest-even, s = 448 / *amax (1 if
 * *amax == 0); *dq = 1/s, the dequantisation scale (dq may be NULL) */
int vu_quant_fp8(const void* x, int64_t xs, int64_t P, int C,
                 const float* amax, uint8_t* y, int64_t ys, float* dq,
                 int dtype, void* stream);
/* BatchNorm apply (+ReLU) fused with e4m3 quantisation, delayed scaling
 * (fp8 DoubleConv: BN1's output is conv2's fp8 input, and only that):
 *   z = relu?(x * scale[c] + shift[c])   (scale == NULL: z = relu?(x))
 *   y = e4m3(clamp(z * s, +-448)), s = 448 / amax_ring[slot] (1 if 0),
 *   *dq = 1/s; max|z| is max-accumulated into amax_ring[(slot+1)%3] (the
 *   next step's scale) and amax_ring[(slot+2)%3] is cleared.  calibrate != 0:
 *   only max-accumulate max|z| into amax_ring[slot] (first step), y unused.
 * C = 8 * 2^k <= 2048, strides multiples of 8.  Replaces the bf16 apply +
 * vu_amax + vu_quant_fp8 sequence (unet_parts.py:41-43 BN -> ReLU -> conv). */
int vu_bn_apply_fp8(const void* x, int64_t xs, uint8_t* y, int64_t ys,
                    int64_t P, int C, const float* scale, const float* shift,
                    int relu, float* amax_ring, int slot, int calibrate,
                    float* dq, int dtype, void* stream);
/* per-row version for weights: fp32 [rows][cols] -> e4m3 [rows][ldy] (zero
 * padded), dq[r] = 1/s_r with s_r = 448 / max_k |x[r][k]| */
int vu_quant_rows_fp8(const float* x, int rows, int64_t cols, uint8_t* y,
                      int64_t ldy, float* dq, void* stream);
/* out[m][co] = x_scale[0] * w_scale[co] * sum_k xq[m][k] wq[co][k]
 *              (+ bias[co]), bf16 NHWC at out[m*out_stride + out_coff + co].
 * a: 3x3 stride-1 pad-1 gather over 1-3 e4m3 NHWC sources (64-channel
 * aligned, pixel strides multiple of 16); wq: e4m3 [ncol][ldw], k = tap*C +
 * c (conv weights [Cout][Cin][r][s] in (r, s, c) order).  stat_sum/stat_m2
 * (optional) as in VuGemmFwd with the row tile vu_conv3x3_fp8_row_tile. */
typedef struct VuConvFp8 {
  VuGather a;
  const void* w;
  int64_t ldw;
  int32_t ncol;
  int32_t out_coff;
  const float* x_scale;
  const float* w_scale;
  const float* bias;
  void* out;
  int64_t out_stride;
  float* stat_sum;
  float* stat_m2;
  /* split-K over the input channels for grids under one block per CU:
   * vu_conv3x3_fp8_workspace_bytes() of fp32 slab space (NULL when 0) */
  float* workspace;
  /* optional (round 6): per statistics row tile and channel, the min / max of
   * the stored (bf16-rounded) output, laid out as stat_sum; only where
   * vu_conv3x3_fp8_minmax_ok() (else the launch is refused).  NULL: none. */
  float* stat_min;
  float* stat_max;
} VuConvFp8;
/* statistics row tile (128, or 64 on the 64 -> 64 resident-weight kernel)
 * when the kernel serves this problem, else 0 */
int64_t vu_conv3x3_fp8_row_tile(const VuConvFp8* args);
/* fp32 split-K slab bytes vu_conv3x3_fp8 needs in args->workspace (0 = none) */
int64_t vu_conv3x3_fp8_workspace_bytes(const VuConvFp8* args);
int vu_conv3x3_fp8(const VuConvFp8* args, void* stream);
/* 1 when the kernel serving *args can emit stat_min / stat_max, else 0 */
int vu_conv3x3_fp8_minmax_ok(const VuConvFp8* args);
/* amax[0] = max over rows x C of |relu?(y * scale[c] + shift[c])| for y in
 * {pmin, pmax} ([rows][C] per-tile min / max of a conv output): the
 * just-in-time e4m3 scale of relu(BN(y)) without a pass over y (the affine is
 * monotone per channel); the same two roundings as vu_bn_apply_fp8, so it
 * equals that kernel's calibration max exactly.  scale NULL: identity.
 * C % 4 == 0 and 16-byte aligned pmin / pmax / scale / shift. */
int vu_fp8_relu_amax(const float* pmin, const float* pmax, int64_t rows, int C, const float* scale,
                     const float* shift, int relu, float* amax, void* stream);

/* ---- weights ----------------------------------------------------------- */
/* out[i0][i1][i2][i3] (contiguous) = in[base + i0*s0 + i1*s1 + i2*s2 + i3*s3]
 * for i3 < d3v, 0 for d3v <= i3 < d3 (channel padding of the 3-channel input
 * layer); strides may be negative (flipped taps of the input-gradient
 * weights). */
int vu_permute4(const float* in, int64_t base, int64_t s0, int64_t s1,
                int64_t s2, int64_t s3, int d0, int d1, int d2, int d3,
                int d3v, void* out, int dtype, void* stream);

/* Batched vu_permute4 (one launch for all derived weight images of a step).
 * jobs: device array.  q = the input-fastest dim when it is not dim 3 (the
 * job is then a batched 2-D transpose in T x T tiles, T = vu_permute4_tile()
 * (64; 32 before round 4): one block per tile, prod(other dims) *
 * ceil(d_q/T) * ceil(d3/T) blocks), or 3 (streamed,
 * ceil(numel / vu_permute4_chunk()) blocks).  chunk0 = prefix block count,
 * nchunks = total blocks. */
typedef struct VuPermJob {
  const float* in;
  int64_t base, s0, s1, s2, s3;
  int32_t d0, d1, d2, d3, d3v, dtype;
  void* out;
  int64_t chunk0;
  int32_t q, pad_;
} VuPermJob;
int64_t vu_permute4_chunk(void);
int64_t vu_permute4_tile(void);
int vu_permute4_batch(const VuPermJob* jobs, int njobs, int64_t nchunks,
                      void* stream);
/* Round 4: the same with the 3x3 / 2x2 weight images (q = 4: dims 1, 2
 * merge into T = 9 or 4 taps that form one contiguous input run with dim 0
 * or dim 3; 32 x T x 32 tile transpose, ceil(d0/32) * ceil(d3/32) blocks) in
 * a launch of their own: jobs[0, ntap) are the q = 4 jobs (chunk0 prefix from
 * 0, tap_blocks in all), jobs[ntap, njobs) the others (chunk0 prefix from 0
 * again, rest_blocks in all). */
int vu_permute4_batch2(const VuPermJob* jobs, int njobs, int ntap,
                       int64_t tap_blocks, int64_t rest_blocks, void* stream);

/* ---- BatchNorm (nn.BatchNorm2d train mode, unet_parts.py:41,44) -------- */
/* combine per-tile (sum, M2) partials; counts: tile t has
 * min(tile_rows, rows - t*tile_rows) rows.  Writes scale/shift (y*scale+shift
 * is the affine-normalised value), save_mean/save_invstd and updates running
 * stats in place (momentum, unbiased variance), like F.batch_norm. */
int vu_bn_finalize(const float* psum, const float* pm2, int tiles,
                   int64_t tile_rows, int64_t rows, int C,
                   const float* gamma, const float* beta,
                   float* running_mean, float* running_var, float momentum,
                   float eps, float* scale, float* shift, float* save_mean,
                   float* save_invstd, int64_t* num_batches_tracked,
                   float* workspace, void* stream);
/* eval mode: scale/shift from running statistics; save_mean/save_invstd
 * (optional) receive running_mean and 1/sqrt(running_var + eps) */
int vu_bn_eval_coeffs(const float* gamma, const float* beta,
                      const float* running_mean, const float* running_var,
                      float eps, int C, float* scale, float* shift,
                      float* save_mean, float* save_invstd, void* stream);
/* y = max(0, x*scale[c] + shift[c]) (relu=1) or x*scale+shift (relu=0) */
/* Train-mode BatchNorm forward in ONE launch for small tensors (tiles <=
 * 256 partial-statistics tiles, C % 32 == 0, strides % 8 == 0:
 * vu_bn_fwd_fused_supported): vu_bn_finalize's statistics (same fp64 group-mean
 * combine, coef = [scale; shift; mean; invstd] rows of C floats, running
 * statistics, num_batches_tracked) and out = relu?(y*scale + shift
 * [+ res*rscale + rshift | + res]) (vu_bn_apply / vu_bn_add_relu). */
int vu_bn_fwd_fused_supported(int tiles, int C, int64_t ys, int64_t rs, int64_t os);
int vu_bn_fwd_fused(const float* psum, const float* pm2, int tiles, int64_t tile_rows, int64_t P, int C,
                    const float* gamma, const float* beta, float* running_mean, float* running_var,
                    int64_t* num_batches_tracked, float momentum, float eps, float* coef, const void* y,
                    int64_t ys, const void* res, int64_t rs, const float* rscale, const float* rshift,
                    void* out, int64_t os, int relu, int dtype, void* stream);
int vu_bn_apply(const void* x, int64_t x_stride, void* y, int64_t y_stride,
                int64_t P, int C, const float* scale, const float* shift,
                int relu, int dtype, void* stream);
/* Backward of y = relu(x*scale+shift): per-channel sums of dz and dz*xhat,
 * dz = dy * (z > 0).  Writes dgamma, dbeta (accumulate flag) and the
 * coefficients (k1, k2, k3) with dx = k1*dz + k2*(x - mean) + k3.
 * train = 1: mean/invstd are the batch statistics (differentiated through);
 * train = 0: eval mode, they are constants (k2 = k3 = 0). */
/* BatchNorm(+ReLU) backward of a small tensor (partial-sum blocks <= 128:
 * vu_bn_bwd_fused_supported) in two launches: vu_bn_bwd_reduce's partial pass,
 * then its fp64 finish (dgamma, dbeta written or accumulated) folded into
 * vu_bn_bwd_apply's pass.  workspace: vu_reduce_workspace_bytes(P, C). */
int vu_bn_bwd_fused_supported(int64_t P, int C, int64_t dys, int64_t xs, int64_t dxs);
int vu_bn_bwd_fused(const void* dy, int64_t dys, const void* x, int64_t xs, int64_t P, int C,
                    const float* scale, const float* shift, const float* mean, const float* invstd,
                    const float* gamma, int relu, int train, float* dgamma, float* dbeta,
                    int accumulate, void* dx, int64_t dxs, float* workspace, int dtype, void* stream);
int vu_bn_bwd_reduce(const void* dy, int64_t dy_stride, const void* x,
                     int64_t x_stride, int64_t P, int C, const float* scale,
                     const float* shift, const float* mean,
                     const float* invstd, const float* gamma, int relu,
                     int train, float* dgamma, float* dbeta, int accumulate,
                     float* coef, float* workspace, int dtype, void* stream);
/* dx = k1*dz + k2*(x-mean) + k3 (+ add) */
/* Second stage of vu_bn_bwd_reduce over partials a GEMM epilogue wrote
 * (VuGemmFwd.bnb_part, nblk row tiles): dgamma, dbeta and the apply
 * coefficients coef [3][C], exactly as vu_bn_bwd_reduce.  workspace:
 * vu_bn_bwd_finish_workspace_bytes(nblk, C) bytes (fp32 row folds). */
int64_t vu_bn_bwd_finish_workspace_bytes(int nblk, int C);
int vu_bn_bwd_finish(const float* part, int nblk, int64_t P, int C,
                     const float* gamma, const float* invstd, int train,
                     float* dgamma, float* dbeta, int accumulate, float* coef,
                     float* workspace, void* stream);
int vu_bn_bwd_apply(const void* dy, int64_t dy_stride, const void* x,
                    int64_t x_stride, int64_t P, int C, const float* scale,
                    const float* shift, const float* mean, const float* coef,
                    int relu, void* dx, int64_t dx_stride, int dtype,
                    void* stream);
/* the backward apply (no ReLU) of TWO BatchNorms fed by the same output
 * gradient dy (the attention gate's W_g / W_x BatchNorms, whose gradient is
 * the psi backward's ds): dx1 from (x1, mean1, coef1 = that BN's
 * vu_bn_bwd_finish coefficients), dx2 likewise, dy read once; per element
 * vu_bn_bwd_apply's arithmetic (round 6) */
int vu_bn_bwd_apply2_ok(int C, int64_t dys, int64_t x1s, int64_t x2s, int64_t dx1s, int64_t dx2s);
int vu_bn_bwd_apply2(const void* dy, int64_t dys, const void* x1, int64_t x1s, const void* x2, int64_t x2s,
                     int64_t P, int C, const float* mean1, const float* coef1, const float* mean2,
                     const float* coef2, void* dx1, int64_t dx1s, void* dx2, int64_t dx2s, int dtype,
                     void* stream);

/* ---- per-channel reductions / elementwise ------------------------------ */
/* out[c] (=|+=) sum over the pixels of the (Hr, Wr) window at (y0, x0) of
 * every (H, W) image of x[pix*stride + c]  (bias gradients) */
int vu_chan_sum(const void* x, int64_t stride, int N, int H, int W, int y0,
                int x0, int Hr, int Wr, int C, float* out, int accumulate,
                float* workspace, int dtype, void* stream);
int64_t vu_reduce_workspace_bytes(int64_t P, int C);
int64_t vu_bn_finalize_workspace_bytes(int tiles, int C);
/* y[p][0..C) = 0 for P pixels at pixel stride ys (channel-slice zero fill) */
int vu_zero(void* y, int64_t ys, int64_t P, int C, int dtype, void* stream);
/* one wave sleeping ~rounds x 3.4 us on the stream (0 <= rounds <= 1000):
 * bench.py's per-launch timing puts it in front of each timed launch so the
 * event pair brackets GPU time only (no memory access) */
int vu_gpu_delay(int rounds, void* stream);
/* zero insertion for a stride-2 conv's input gradient: up (N,H,W,C) holds
 * dy (N,h,w,C) at the even pixels, zeros elsewhere (C, strides % 8 == 0) */
int vu_zero_insert2(const void* dy, int64_t dys, int N, int h, int w, int C,
                    void* up, int64_t ups, int H, int W, int dtype, void* stream);
/* generic NHWC copy/cast: y[p*ys + c] = x[p*xs + c] (+ y if accumulate) */
int vu_copy(const void* x, int64_t xs, int xdtype, void* y, int64_t ys,
            int ydtype, int64_t P, int C, int accumulate, void* stream);
/* NCHW/NHWC fp32 input -> NHWC storage padded to Cp channels (zeros) */
int vu_input_pack(const float* x, int64_t sn, int64_t sc, int64_t sh,
                  int64_t sw, int N, int C, int H, int W, int Cp, void* y,
                  int dtype, void* stream);

/* ---- pooling / resampling (unet_parts.py:57,73,85-89) ------------------ */
int vu_maxpool2_fwd(const void* x, int64_t xs, int N, int H, int W, int C,
                    void* y, int64_t ys, int dtype, void* stream);
/* dx (over the full HxW input) = routed dy (first max wins) [+ add] */
int vu_maxpool2_bwd(const void* x, int64_t xs, const void* dy, int64_t dys,
                    int N, int H, int W, int C, void* dx, int64_t dxs,
                    const void* add, int64_t adds, int dtype, void* stream);
/* MaxPool2d(2) fused with the BatchNorm(+ReLU) of the DoubleConv that feeds it
 * (Down, unet_parts.py:51-63; H, W even, C = 8 * 2^k <= 2048, 8-element
 * strides, else hipErrorInvalidValue): a = relu(y*scale+shift) is stored AND
 * pooled in one pass (replaces vu_bn_apply + vu_maxpool2_fwd). */
int vu_bn_apply_maxpool2(const void* y, int64_t ys, void* a, int64_t as, void* pool, int64_t ps,
                         int N, int H, int W, int C, const float* scale, const float* shift,
                         int relu, int dtype, void* stream);
/* BatchNorm(+ReLU) backward THROUGH that 2x2 max-pool: y the BN input, dp
 * the gradient of the pooled output, add the skip gradient of a (or NULL);
 * recomputes a, its first-max argmax and a's gradient per window (as
 * vu_bn_apply_maxpool2 / vu_maxpool2_bwd store them) in a partial pass and an
 * apply pass -> dx (gradient of y); dgamma/dbeta as vu_bn_bwd_reduce, coef
 * [3][C] scratch, workspace vu_reduce_workspace_bytes(N*H*W, C). */
int vu_bn_bwd_pool_supported(int H, int W, int C, int64_t ys, int64_t dps, int64_t adds, int64_t dxs);
int vu_bn_bwd_pool(const void* y, int64_t ys, const void* dp, int64_t dps, const void* add, int64_t adds,
                   int N, int H, int W, int C, const float* scale, const float* shift, const float* mean,
                   const float* invstd, const float* gamma, int relu, int train, float* dgamma,
                   float* dbeta, int accumulate, float* coef, float* workspace, void* dx, int64_t dxs,
                   int dtype, void* stream);
/* bilinear, align_corners=True, (Hi,Wi) -> (Ho,Wo) placed at (py,px) inside
 * a zero (Hp,Wp) canvas (F.pad of unet_parts.py:88-89 folded in). */
int vu_upsample_fwd(const void* x, int64_t xs, int N, int Hi, int Wi, int C,
                    void* y, int64_t ys, int Ho, int Wo, int Hp, int Wp,
                    int py, int px, int dtype, void* stream);
/* transposed gather (no atomics): dx[n,i,j] = sum over the output pixels
 * whose stencil touches (i,j). */
int vu_upsample_bwd(const void* dy, int64_t dys, int N, int Hi, int Wi, int C,
                    void* dx, int64_t dxs, int Ho, int Wo, int Hp, int Wp,
                    int py, int px, int accumulate, int dtype, void* stream);

/* ---- attention gate (unet_parts.py:7-30) ------------------------------- */
/* pixels per statistics tile of vu_attn_psi_fwd */
int64_t vu_attn_tile_rows(void);
/* q[p] = bpsi + sum_c wpsi[c] * relu(ug[p,c]*sg[c]+tg[c] + ux[p,c]*sx[c]+tx[c])
 * plus per-tile (sum, M2) of q for BatchNorm2d(1). */
int vu_attn_psi_fwd(const void* ug, const void* ux, int64_t P, int F,
                    const float* sg, const float* tg, const float* sx,
                    const float* tx, const float* wpsi, const float* bpsi,
                    float* q, float* psum, float* pm2, int64_t tile_rows,
                    int dtype, void* stream);
/* p = sigmoid(q*st[0] + st[1]); out[p,c] = x[p,c] * p  (also stores p) */
int vu_attn_gate_fwd(const float* q, const float* st, const void* x,
                     int64_t xs, int64_t P, int C, float* pmap, void* out,
                     int64_t os, int dtype, void* stream);
/* backward of out = x*p: dx_direct = dout*p (written to dx), and
 * dq_pre[p] = (sum_c dout*x) * p * (1-p)  (grad w.r.t. the BN(1) output) */
int vu_attn_gate_bwd(const void* dout, int64_t dos, const void* x, int64_t xs,
                     const float* pmap, int64_t P, int C, void* dx,
                     int64_t dxs, float* dqpre, int dtype, void* stream);
/* backward through psi conv + relu: given dq[p] (grad of q), produce
 * ds[p,c] = dq[p]*wpsi[c]*(s>0) (the gradient of both BN branches), and
 * dwpsi[c], dbpsi (deterministic partial reduction). */
int64_t vu_attn_psi_bwd_workspace_bytes(int64_t P, int F);
int vu_attn_psi_bwd(const void* ug, const void* ux, int64_t P, int F,
                    const float* sg, const float* tg, const float* sx,
                    const float* tx, const float* wpsi, const float* dq,
                    void* ds, float* dwpsi, float* dbpsi, int accumulate,
                    float* workspace, int dtype, void* stream);
/* the same (batched kernels, VU_TUNE_ATTN 1) also emitting the first stage of
 * the backward reduction of the two BatchNorms ds flows into (W_g's over ug,
 * W_x's over ux, unet_parts.py:11-20; no ReLU between): per block b,
 *   bnb_?[(2b + 0) * F + c] = sum ds,  bnb_?[(2b + 1) * F + c] = sum ds * (u - mean) * invstd
 * over the stored ds -- VuGemmFwd.bnb_part's layout, finished by
 * vu_bn_bwd_finish with nblk = vu_attn_psi_bwd_blocks(P). */
int64_t vu_attn_psi_bwd_blocks(int64_t P);
int vu_attn_psi_bwd_bnb_ok(int F);   /* 1 when vu_attn_psi_bwd_bnb serves F */
int vu_attn_psi_bwd_bnb(const void* ug, const void* ux, int64_t P, int F,
                        const float* sg, const float* tg, const float* sx,
                        const float* tx, const float* wpsi, const float* dq,
                        void* ds, float* dwpsi, float* dbpsi, int accumulate,
                        float* workspace, const float* mean_g, const float* invstd_g,
                        const float* mean_x, const float* invstd_x, float* bnb_g,
                        float* bnb_x, int dtype, void* stream);

/* ---- 1x1 conv with a tiny output (OutConv unet_parts.py:97-103,
 *      final_conv unet_resnet.py:189) -------------------------------------- */
/* y[p*ys + j] = b[j] + sum_c x[p*xs+c] w[j*C+c], j < J <= 4, y fp32 */
int vu_pointwise_fwd(const void* x, int64_t xs, int64_t P, int C, int J,
                     const float* w, const float* b, float* y, int64_t ys,
                     int dtype, void* stream);
/* dx[p,c] = sum_j dy[p,j] w[j,c];  dw[j,c] (+)= sum_p dy x;  db[j] (+)= sum_p dy */
int64_t vu_pointwise_bwd_workspace_bytes(int64_t P, int C, int J);
int vu_pointwise_bwd(const void* x, int64_t xs, const float* dy, int64_t dys,
                     int64_t P, int C, int J, const float* w, void* dx,
                     int64_t dxs, float* dw, float* db, int accumulate,
                     float* workspace, int dtype, void* stream);
/* The same 1x1 conv over the producing BatchNorm + ReLU applied on the fly
 * (round 6: the UNet's last BN never materialised): x is the PRE-BN tensor
 * and the operand a = relu(x * bn_scale[c] + bn_shift[c]) rounded to the
 * storage dtype (the bytes vu_bn_apply would store).  C <= 512. */
int vu_pointwise_bn_fwd(const void* x, int64_t xs, int64_t P, int C, int J,
                        const float* bn_scale, const float* bn_shift, const float* w,
                        const float* b, float* y, int64_t ys, int dtype, void* stream);
/* Backward of vu_pointwise_bn_fwd: dx = gradient w.r.t. a (as
 * vu_pointwise_bwd), dw / db over the re-formed a, and bnb[blk][2][C] = the
 * first stage of the BatchNorm's backward reduction over block blk's pixels
 * (sum dz, sum dz * (x - mean) * invstd, dz = the stored dx masked by the
 * ReLU) -- VuGemmFwd.bnb_part's layout, finished by vu_bn_bwd_finish with
 * nblk = vu_pointwise_bn_bwd_blocks(P).  bn_coef: rows scale, shift, mean,
 * invstd at coef_stride floats apart.  workspace: vu_pointwise_bwd's. */
int64_t vu_pointwise_bn_bwd_blocks(int64_t P);
int vu_pointwise_bn_bwd(const void* x, int64_t xs, const float* bn_coef, int64_t coef_stride,
                        const float* dy, int64_t dys, int64_t P, int C, int J, const float* w,
                        void* dx, int64_t dxs, float* dw, float* db, int accumulate,
                        float* workspace, float* bnb, int dtype, void* stream);

/* ---- loss (utils/loss.py) ---------------------------------------------- */
int64_t vu_loss_workspace_bytes(void);
/* sums[0..3] = {sum BCE-with-logits, sum sigmoid*t, sum sigmoid, sum t} over
 * n elements (fp64, deterministic); loss[0] = w_bce*BCE_mean + w_dice*(1-dice)
 * (CombinedLoss, loss.py:44-63), parts = {BCE_mean, 1-dice} (optional). */
int vu_bce_dice_fwd2(const float* logits, const float* target, int64_t n,
                     double* sums, float smooth, float w_bce, float w_dice,
                     float* loss, float* parts, double* workspace,
                     void* stream);
int vu_bce_dice_fwd(const float* logits, const float* target, int64_t n,
                    double* sums, double* workspace, void* stream);
/* grad = g * d/dlogit (w_bce*BCE_mean + w_dice*(1-dice)), g = *gscale */
int vu_bce_dice_bwd(const float* logits, const float* target, int64_t n,
                    const double* sums, float smooth, float w_bce,
                    float w_dice, const float* gscale, float* grad,
                    void* stream);
/* kl_with_free_bits (loss.py:148-170), B x L: value and/or grads (scaled by
 * *gscale when given) */
int vu_kl_free_bits2(const float* mu, const float* logvar, int B, int L,
                     float free_bits, const float* gscale, float* value,
                     float* gmu, float* glogvar, void* stream);
int vu_kl_free_bits(const float* mu, const float* logvar, int B, int L,
                    float free_bits, float* value, float* gmu, float* glogvar,
                    void* stream);

/* dice_score (utils/metrics.py:8-35): a = x > 0.5, b = t > 0.5 over n
 * elements; *score = 1 if sum a + sum b == 0 else (2*sum(a*b) + epsilon) /
 * (sum a + sum b + epsilon), computed on the device (no host sync; the
 * reference's denominator.item() branch is a device select).  counts
 * (optional) = {sum a, sum b, sum a*b}.  workspace: vu_loss_workspace_bytes */
int vu_dice_score(const float* x, const float* t, int64_t n, float epsilon,
                  float* score, double* counts, double* workspace,
                  void* stream);

/* ---- optimizer (train.py:334,406-411) ---------------------------------- */
/* sum of squares of n fp32 values into out (fp64, deterministic) */
int vu_sumsq(const float* x, int64_t n, double* out, double* workspace,
             void* stream);

/* Multi-tensor table entry (device memory).  Replaces the foreach loops of
 * torch.nn.utils.clip_grad_norm_ (train.py:408) and torch.optim.AdamW.step
 * (train.py:409, optimizer built at train.py:334).  A tensor's param, grad
 * and moment buffers share strides and are processed as flat fp32 storage of
 * numel elements, cut into vu_mt_chunk_elems() chunks; chunk0 = number of
 * chunks of all previous entries (entries in chunk order).  step_size =
 * lr / (1 - beta1^step) and bc2_sqrt = sqrt(1 - beta2^step) per tensor. */
typedef struct VuMtEntry {
  void* param;
  void* grad;
  void* exp_avg;
  void* exp_avg_sq;
  int64_t numel;
  int64_t chunk0;
  float step_size;
  float bc2_sqrt;
} VuMtEntry;

int64_t vu_mt_chunk_elems(void);
/* ||grads||_2 over all entries (fp64 accumulation) -> *total_norm, and
 * *clip_coef = min(1, max_norm / (total_norm + 1e-6)) (either may be NULL);
 * workspace: nchunks doubles */
int vu_mt_grad_norm(const VuMtEntry* table, int ntensors, int64_t nchunks,
                    float max_norm, float* total_norm, float* clip_coef,
                    double* workspace, void* stream);
/* grads *= *coef (clip_grad_norm_'s in-place scaling) */
int vu_mt_scale_grads(const VuMtEntry* table, int ntensors, int64_t nchunks,
                      const float* coef, void* stream);
/* one AdamW step over all entries; grads multiplied by *grad_scale when
 * given (not written back); decay = 1 - lr*weight_decay */
int vu_mt_adamw(const VuMtEntry* table, int ntensors, int64_t nchunks,
                float decay, float one_minus_beta1, float beta2,
                float one_minus_beta2, float eps, const float* grad_scale,
                void* stream);

/* Graph-capturable AdamW: *step (device, shared by the table) is incremented
 * first and the bias corrections are derived from it on the device (double,
 * rounded to float once: the same values as the host path); zero_grad != 0
 * clears each gradient after use (persistent .grad buffers for replays). */
int vu_mt_adamw_dev(const VuMtEntry* table, int ntensors, int64_t nchunks,
                    double lr, double weight_decay, double beta1, double beta2,
                    double eps, float* step, int zero_grad, void* stream);
/* the same, each gradient multiplied by *grad_scale (the clip coefficient of
 * vu_mt_grad_norm) as it is read -- the bits of vu_mt_scale_grads followed by
 * vu_mt_adamw_dev, one pass over the gradients fewer; only with zero_grad
 * (the scaled gradient is never stored).  grad_scale NULL = 1. */
int vu_mt_adamw_dev_scaled(const VuMtEntry* table, int ntensors, int64_t nchunks,
                           double lr, double weight_decay, double beta1, double beta2,
                           double eps, float* step, int zero_grad, const float* grad_scale,
                           void* stream);

/* ---- VAE-U-Net (unet/unet_resnet.py) ----------------------------------- */
/* ResNet34 stem max-pool 3x3/s2/p1 (timm resnet34, unet_resnet.py:131):
 * idx receives the window argmax (0..8, first max wins) per output element */
int vu_maxpool3s2_fwd(const void* x, int64_t xs, int N, int H, int W, int C,
                      void* y, int64_t ys, uint8_t* idx, int dtype,
                      void* stream);
int vu_maxpool3s2_bwd(const void* dy, int64_t dys, const uint8_t* idx, int N,
                      int H, int W, int C, void* dx, int64_t dxs,
                      int accumulate, int dtype, void* stream);
/* BasicBlock tail: out = relu(y*sc+sh + (r*rsc+rsh | r)) */
int vu_bn_add_relu(const void* y, int64_t ys, const float* sc, const float* sh,
                   const void* r, int64_t rs, const float* rsc,
                   const float* rsh, int64_t P, int C, void* out, int64_t os,
                   int dtype, void* stream);
/* g = dout * (out > 0) */
int vu_relu_mask(const void* dout, int64_t ds, const void* out, int64_t os,
                 int64_t P, int C, void* g, int64_t gs, int dtype,
                 void* stream);
/* out[n][c] (+)= scale * sum over the HW pixels of sample n (avg-pool head,
 * latent-broadcast backward) */
int vu_sample_sum(const void* x, int64_t xs, int N, int HW, int C, float scale,
                  float* out, int accumulate, float* workspace, int dtype,
                  void* stream);
/* workspace bytes of vu_sample_sum (per-split partial sums) */
int64_t vu_sample_sum_workspace_bytes(int N, int C);
/* y[n,p,c] (+)= scale * v[n][c]: interpolate(z[...,None,None], align_corners)
 * as an exact broadcast (unet_resnet.py:217-221, 93) */
int vu_sample_broadcast(const float* v, int N, int HW, int C, float scale,
                        void* y, int64_t ys, int accumulate, int dtype,
                        void* stream);
/* mu/logvar heads after pooling: y[b][j] = bias[j] + sum_k x[b][k] w[j][k] */
int vu_linear_small_fwd(const float* x, int B, int K, const float* w,
                        const float* bias, int J, float* y, void* stream);
int vu_linear_small_bwd(const float* x, int B, int K, const float* w, int J,
                        const float* dy, float* dx, int dx_acc, float* dw,
                        float* db, int w_acc, void* stream);
/* reparameterize (unet_resnet.py:191-194): z = mu + eps*exp(0.5*logvar) */
int vu_reparam_fwd(const float* mu, const float* lv, const float* eps, int n,
                   float* z, void* stream);
int vu_reparam_bwd(const float* lv, const float* eps, const float* dz, int n,
                   float* dmu, float* dlv, int accumulate, void* stream);

/* ---- fused VAE bottleneck + latent injection (round 4) -------------------
 * Replaces, for a latent VECTOR z, the heads / reparameterize / broadcast /
 * z_initial / z_proj chain of unet_resnet.py:140-154,191-194,217-229 and
 * :37-41,93-94 (DecoderBlock).  Downstream of z every map is a per-sample
 * constant, so each 1x1 conv + BatchNorm2d + ReLU "consumer" is computed on
 * the N sample vectors (train-mode statistics over N*HW pixels == over the N
 * vectors, running_var unbiased with count N*HW) and its map is written once,
 * activated.  latent.hip. */

/* one block per sample: pooled[n][c] = mean_p f4[n,p,c]; mu / logvar[n][j] =
 * b[j] + sum_c w[j][c] pooled[n][c] (the conv1x1 + AdaptiveAvgPool2d heads,
 * pool and 1x1 conv commuted); z = mu + eps * exp(logvar / 2), or z = mu when
 * eps == NULL.  C = 8 * 2^k <= 2048, fs % 8 == 0. */
int vu_vae_heads_fwd(const void* f4, int64_t fs, int N, int HW, int C, const float* w_mu,
                     const float* b_mu, const float* w_lv, const float* b_lv, int L, const float* eps,
                     float* pooled, float* mu, float* logvar, float* z, int dtype, void* stream);

/* One latent consumer (device table entry): map[n, p, c] = relu(BN(W z[n] +
 * b))[c] for c < co, 0 for co <= c < cpad, at out + (n*HW + p)*out_stride.
 * Forward saves y[n][c] = W z[n] + b and coef [4][co] = scale, shift, mean,
 * invstd.  Backward: dmap (pixel stride dmap_stride, co channels) -> part
 * [N][splits][co] partial pixel sums -> weight / bias / gamma / beta
 * gradients (written, or added when grad_acc) and the consumer's share of
 * dz.  The entry points take a HOST array of at most 8 entries and pass it
 * by value in the kernel arguments (a captured graph replays it); block0,
 * sblock0 and cgroups are filled in by the library. */
typedef struct VuLatentJob {
  const float* w;              /* [co][L] */
  const float* bias;           /* [co] or NULL */
  const float* gamma;
  const float* beta;
  float* running_mean;         /* NULL: not tracked */
  float* running_var;
  int64_t* num_batches_tracked;
  float momentum, eps;
  int32_t train, co, cpad, HW;
  void* out;
  int64_t out_stride;
  float* y;                    /* [N][co] */
  float* coef;                 /* [4][co] */
  int64_t block0;
  int32_t cgroups, grad_acc;
  const void* dmap;            /* backward: d(map), co channels */
  int64_t dmap_stride;
  float* part;                 /* vu_latent_part_floats(N, co) */
  int64_t sblock0;
  float* dw;                   /* [co][L] or NULL */
  float* dbias;
  float* dgamma;
  float* dbeta;
  /* round 5: the consumer's activated vectors [N][co] (rounded to the
   * storage dtype, i.e. the values its map would hold) are written here when
   * non-NULL; out = NULL (the latent shortcut of a DecoderBlock: no map) then
   * skips the map stores (cpad = co, out_stride 0). */
  float* act;
} VuLatentJob;

/* the heads' backward inputs / outputs for vu_latent_bwd */
typedef struct VuLatentHeads {
  const float* z;              /* [N][L] */
  const float* eps;            /* NULL: z = mu */
  const float* logvar;
  const float* dmu_in;         /* incoming d/dmu, d/dlogvar (KL term) or NULL */
  const float* dlv_in;
  const float* dz_in;          /* incoming d/dz from outside the consumers, or NULL */
  const float* pooled;         /* [N][C] */
  const float* w_mu;
  const float* w_lv;           /* [L][C] */
  float* dw_mu;
  float* db_mu;
  float* dw_lv;
  float* db_lv;                /* written, or added when grad_acc */
  float* dpooled;              /* [N][C] (the caller broadcasts dpooled / HW into d f4) */
  int32_t C, grad_acc;
} VuLatentHeads;

int64_t vu_latent_fwd_blocks(int N, int HW, int cpad);
/* jobs: host array (<= 8); z [N][L] fp32 device (L <= 64, N <= 64) */
int vu_latent_fwd(const VuLatentJob* jobs, int njobs, const float* z, int N, int L, int dtype, void* stream);
int64_t vu_latent_part_floats(int N, int co);
int vu_latent_bwd_sums(const VuLatentJob* jobs, int njobs, int N, int dtype, void* stream);
int64_t vu_latent_bwd_workspace_bytes(int N, int L, int64_t sum_co);
/* 1 when vu_latent_bwd serves N samples, latent size L, consumers with
 * sum_co output channels in all and C encoder channels (N <= 64, L <= 64,
 * C % 8 == 0), else 0 (the caller takes the map path) */
int vu_latent_bwd_supported(int N, int L, int64_t sum_co, int C);
/* two launches: every consumer's BN / ReLU / conv backward on the vectors
 * (one block per 32 consumer channels; dz partials into the workspace of
 * vu_latent_bwd_workspace_bytes, required when njobs > 0), then dz,
 * reparameterize backward, both heads' backward -> dpooled (one block per 8
 * encoder channels) */
int vu_latent_bwd(const VuLatentJob* jobs, int njobs, const VuLatentHeads* heads, int N, int L,
                  float* workspace, void* stream);

/* ---- latent-broadcast shortcut of a DecoderBlock's conv1 (round 5) ------
 * unet/unet_resnet.py:37-41, 92-99: conv1 contracts over the concat
 * [x, skip, z_proj(z) broadcast]; the last source is a per-sample constant
 * map c_n (L channels at input channels [cz0, cz0 + L) of conv1.weight).  Its
 * contribution becomes VuGemmFwd.zbias (forward) and its backward reduces to
 * per-sample region sums of conv1's pre-BatchNorm output gradient dy:
 *   R[n][c][tap] = sum over the output pixels whose tap reads inside the image
 *                = T - [ky=0] Row0 - [ky=2] RowL - [kx=0] Col0 - [kx=2] ColL + corners
 *   dW[c][cz0 + l][tap] (+)= sum_n c_n[l] R[n][c][tap]
 *   dc[n][l]             = sum_c sum_tap W[c][cz0 + l][tap] R[n][c][tap]
 * dc (the pixel sum of d(map), what vu_latent_bwd_sums produced from the map
 * gradient) goes to the consumer's VuLatentJob.part split by 32-channel
 * chunk of c (vu_latent_bwd sums the splits).  Jobs travel by value
 * (at most 8); block0 is filled by the library. */
typedef struct VuZbJob {
  const float* w;              /* conv1.weight (fp32), element strides below */
  int64_t ws_co, ws_ci, ws_ky, ws_kx;
  int32_t cz0, L, co, H, W;    /* z channels [cz0, cz0 + L); co = conv1 outputs; output image H x W */
  const float* act;            /* [N][L] the z_proj vectors (VuLatentJob.act) */
  const float* row_scale;      /* [co] or NULL: eval-mode BN folded into conv1 (table rows scaled) */
  float* table;                /* forward: [N][9][co] */
  const void* dy;              /* backward: conv1's pre-BN output gradient, NHWC, co channels */
  int64_t dy_stride;
  float* rs;                   /* backward workspace, vu_zbias_rs_floats(N, co, H, W) floats */
  float* part;                 /* the consumer's VuLatentJob.part ([N][32][L]) */
  float* dw;                   /* conv1.weight.grad (strides of w): z columns written, or added when grad_acc */
  int32_t grad_acc;
  int32_t rs_ready;            /* 1: rs's region partials already written (vu_bn_bwd_apply_zrs): no region pass */
  int64_t block0;
} VuZbJob;
/* 1 when the shortcut serves N samples, L latent channels and co conv1 outputs */
int vu_zbias_supported(int N, int L, int co);
int64_t vu_zbias_rs_floats(int N, int co, int H, int W);
/* the [N][9][co] tables of every job (one launch) */
int vu_zbias_fwd(const VuZbJob* jobs, int njobs, int N, void* stream);
/* region sums of every job's dy (partials per ~64 KB pixel chunk -- skipped
 * for jobs with rs_ready -- then their sums), then dW's z columns and the dc
 * partials (three launches, two when every job has rs_ready); dtype: dy's
 * storage (VU_BF16 / VU_F32) */
int vu_zbias_bwd(const VuZbJob* jobs, int njobs, int N, int dtype, void* stream);
/* BatchNorm(+ReLU) backward apply (vu_bn_bwd_apply's arithmetic, coef from
 * vu_bn_bwd_reduce / vu_bn_bwd_finish) of a shortcut conv1's BatchNorm over
 * N x H x W x C, also writing the region partials of the dy it stores into rs
 * (the first N * nchunks * 5 * C floats of a vu_zbias_rs_floats buffer; the
 * job then passes rs_ready = 1): dy and rs bit-identical to vu_bn_bwd_apply
 * followed by vu_zbias_bwd's region pass.  Replaces the backward re-read of
 * dy for unet_resnet.py:92-99's z channels. */
int vu_bn_bwd_apply_zrs_ok(int H, int W, int C, int64_t dzs, int64_t xs, int64_t dys);
int vu_bn_bwd_apply_zrs(const void* dz, int64_t dzs, const void* x, int64_t xs, int N, int H, int W, int C,
                        const float* scale, const float* shift, const float* mean, const float* coef, int relu,
                        void* dy, int64_t dys, float* rs, int dtype, void* stream);
/* 0 when a consumer of this geometry is served (co = 8 * 2^k <= 2048, cpad % 8,
 * stride % 8), else hipErrorInvalidValue */
int vu_latent_check_job(int co, int cpad, int64_t out_stride, int dtype);

/* ---- inference sampling path (utils/vae_utils.py, visualize_vae.py) --- */
/* out[e] = (sum_{k < groups} x[k*n + e]) / groups  (stack(preds).mean(0)) */
int vu_mean_groups(const float* x, int groups, int64_t n, float* out,
                   void* stream);
/* y = 1 / (1 + exp(-x)) */
int vu_sigmoid(const float* x, int64_t n, float* y, void* stream);
/* Feathered sliding-window accumulation of one patch prediction
 * (visualize_vae.py:360-384): pred [B][ph][pw] (image stride pred_img_stride)
 * -> out/wsum [B][H][W] at (sh, sw), weight = ramp-tapered ones (ramp[ov] =
 * linspace(0, 1, ov); leading taper if top/left, trailing (1 - ramp) if
 * bottom/right, each only when the patch extent > 2*ov).  Launches of
 * overlapping patches accumulate in launch order (no atomics). */
int vu_patch_blend(const float* pred, int64_t pred_img_stride, int B, int ph,
                   int pw, float* out, float* wsum, int H, int W, int sh,
                   int sw, const float* ramp, int overlap, int top,
                   int bottom, int left, int right, void* stream);
/* out = out / (wsum + 1e-8) */
int vu_blend_finish(float* out, const float* wsum, int64_t n, void* stream);
/* calculate_uncertainty_metrics (visualize_vae.py:90-117) over the sample
 * axis of seg [samples][n]: mean, unbiased std, entropy of the mean,
 * mutual information, coefficient of variation (eps 1e-7) */
int vu_uncertainty(const float* seg, int samples, int64_t n, float* mean,
                   float* std, float* entropy, float* mutual_info,
                   float* coeff_var, void* stream);
/* Per-sample integer pixel map over NHWC images (flips and 90-degree
 * rotations of patch batches, utils/data_loading.py:116-120):
 * y[b, i, j, :] = x[b, m0*i + m1*j + m2, m3*i + m4*j + m5, :], map = int32
 * [B][6] in device memory; x (B, H, W, C) -> y (B, Ho, Wo, C). */
int vu_gather_affine(const void* x, int B, int H, int W, int C, const int* map,
                     void* y, int Ho, int Wo, int dtype, void* stream);

/* Patch-cache producer (IDRIDDataset.precompute_all_patches,
 * utils/data_loading.py:370-397, and is_valid_patch :287-300): for the
 * ny x nx windows of size P at `stride` over one scaled image img [C][H][W]
 * fp32 and its mask [H][W] fp32, black[w] = #pixels with channel mean < 0.1
 * (left-to-right fp32 sum / C) and lesion[w] = #mask pixels > 0.5 (int32,
 * window w = row-major (y/stride, x/stride)).  Every window must lie inside
 * the image (else hipErrorInvalidValue). */
int vu_patch_stats(const float* img, int C, int H, int W, const float* mask,
                   int P, int stride, int ny, int nx, int* black, int* lesion,
                   void* stream);

#ifdef __cplusplus
}
#endif
#endif
