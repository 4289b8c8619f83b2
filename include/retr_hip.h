/* C-ABI of libretr_hip.so — the MI355X (gfx950) kernels behind the RE⫶TR hot path.
 *
 * The reference (simeonjunker/retr) is pure Python/PyTorch: it has no native FFI of its own.
 * Each entry point below replaces the implicit PyTorch/cuDNN/cuBLAS work of one reference
 * call site (cited per function).  The Python host layer
 * (retr_amd/_lib.py) binds these with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - every pointer is a device pointer owned by the caller (torch caching allocator); kernels
 *     never allocate, free or synchronise, so every call is hipGraph-capturable;
 *   - `dtype` selects the operand type: RETR_F32 (exact-f32 MFMA, parity mode) or RETR_BF16;
 *   - `stream` is a hipStream_t (torch's current stream);
 *   - return 0 on success, non-zero on error; retr_last_error() returns the message.
 *   - activations of the ResNet are NHWC; transformer tokens are batch-major rows [B*L][C].
 */
#ifndef RETR_HIP_H
#define RETR_HIP_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

#define RETR_DTYPE_F32 0
#define RETR_DTYPE_BF16 1

const char* retr_last_error(void);
int retr_abi_version(void);
/* Dropout masks are keep(seed_op + *seed_base, index): seed_base is a device uint64 that the
 * training loop advances once per step (retr_seed_bump), so a captured hipGraph replays with
 * fresh masks.  NULL (default) -> the per-op seed alone. */
void retr_set_seed_base(const unsigned long long* device_ptr);
/* Deterministic mode (config.deterministic): 1 = every reduction runs in a fixed order, so two
 * runs on the same inputs are bitwise equal — linear weight-gradient GEMMs are not split over K
 * (no fp32 atomics) and bias gradients use an ordered column sum instead of the fused row sums.
 * 0 (default) = split-K with fp32 atomics for the linear weight gradients.  (Convolution weight
 * gradients, LayerNorm / embedding parameter gradients, attention backward, the loss and the
 * optimizer reductions are fixed-order in both modes.) */
void retr_set_deterministic(int on);
int retr_get_deterministic(void);
int retr_seed_bump(unsigned long long* device_ptr, unsigned long long delta, void* stream);
/* Measurement only (bench.py kernel probe; no reference counterpart): one wave busy-waits
 * `us` microseconds on the device clock, so a following event pair times device execution
 * without the host launch gap. */
int retr_spin_us(float us, void* stream);

/* ---- linear layers: nn.Linear / MHA in/out-proj / MLP head / feed_forward --------------------
 * replaces F.linear at models/transformer_modules.py:6-11, models/caption.py:161-174,
 * torch/nn/functional.py:5785-5850 (in-proj) and :6601 (out-proj).
 * y = relu2( residual + dropout( relu1( x W^T + b ) ) ); relu: 0 none, 1 relu1 */
int retr_linear_fwd(int dtype, const void* x, long ldx, const void* w, long ldw,
                    const float* bias, void* y, long ldy, int y_f32, int M, int N, int K, int relu,
                    const float* residual, long ldr, float drop_p, unsigned long long seed,
                    void* stream);
/* dx = gate( dy W [+ addend] ), gate(v) = v * (gate_src > 0); w_trans: w holds W^T [K][N] */
int retr_linear_dgrad(int dtype, const void* dy, long lddy, const void* w, long ldw, void* dx,
                      long lddx, int dx_f32, int M, int N, int K, const void* addend,
                      int addend_f32, long lda, const void* gate, long ldg, int w_trans,
                      void* stream);
/* Split-K variants for GEMMs with few output tiles and a long reduction (FFN down-projections,
 * FFN up-projection data gradients, the vocabulary head's data gradient): `splits` slices
 * write fp32 slabs ws[splits][M][N_out] with plain stores, a second kernel adds them in slice
 * order (deterministic) and applies the same epilogue as retr_linear_fwd / _dgrad.
 * retr_linear_splits(dtype, M, N_out, K_reduction): the slice count to use (1 = don't split). */
int retr_linear_splits(int dtype, int M, int N, int K);
int retr_linear_fwd_splitk(int dtype, const void* x, long ldx, const void* w, long ldw,
                           const float* bias, void* y, long ldy, int y_f32, int M, int N, int K,
                           int relu, const float* residual, long ldr, float drop_p,
                           unsigned long long seed, float* ws, int splits, void* stream);

/* LayerNorm of a residual-stream linear's output, produced by that linear's epilogue (the
 * following pre-norm block's LN, or the stack's final norm: models/ConcatTransformer.py's
 * norm -> attention / FFN order): y = LN(out) and y2 = LN(out) + pos[row % period] (either may be
 * null), row statistics mean / rstd for the backward. */
typedef struct retr_ln_out {
  const float* gamma;
  const float* beta;
  float eps;
  int y_bf16;           /* y / y2 element type: 1 bf16, 0 fp32 (the fused kernel takes bf16) */
  void* y;
  void* y2;
  long ldy;
  const float* pos;
  int period;
  float* mean;
  float* rstd;
} retr_ln_out;
/* retr_linear_fwd_splitk (fp32 out) + retr_layernorm_fwd of its output in one epilogue launch
 * after the slices (bf16, N 256 / 512); any other case runs the two calls.  Replaces the
 * FFResidual output -> next norm pair of models/ConcatTransformer.py:171-257. */
int retr_linear_fwd_splitk_ln(int dtype, const void* x, long ldx, const void* w, long ldw,
                              const float* bias, float* y, long ldy, int M, int N, int K, int relu,
                              const float* residual, long ldr, float drop_p,
                              unsigned long long seed, float* ws, int splits,
                              const retr_ln_out* ln, void* stream);
int retr_linear_dgrad_splitk(int dtype, const void* dy, long lddy, const void* w, long ldw,
                             void* dx, long lddx, int dx_f32, int M, int N, int K,
                             const void* addend, int addend_f32, long lda, const void* gate,
                             long ldg, int w_trans, float* ws, int splits, void* stream);
/* the slices of retr_linear_dgrad_splitk only (no epilogue): ws[splits][M][K] fp32 partial
 * products for a consumer that sums them (retr_layernorm_bwd_slabs); splits = a normalised
 * slice count (retr_linear_splits).  bf16 only. */
int retr_linear_dgrad_slabs(int dtype, const void* dy, long lddy, const void* w, long ldw, int M,
                            int N, int K, int w_trans, float* ws, int splits, void* stream);
/* dw[N][K] (=|+=) dy^T x (fp32); db[N] (=|+=) column sums of dy (fused; db may be NULL).
 * accumulate = 0: dw/db are overwritten (no pre-zeroing needed); 1: added to.
 * N may be ragged when lddy covers N rounded up to the 16-byte vector (padded dy rows). */
int retr_linear_wgrad(int dtype, const void* dy, long lddy, const void* x, long ldx, float* dw,
                      long lddw, int M, int N, int K, float* db, int accumulate, void* stream);
/* db[N] += column sums of dy[M][N] */
int retr_bias_grad(int dtype, const void* dy, long lddy, int M, int N, float* db, void* stream);

/* Launch-configuration overrides for on-GPU tuning sweeps (tools/group_micro.py); value 0 =
 * the built-in choice.  Returns the previous value (-1: unknown knob). */
enum {
  RETR_TUNE_GROUP_TILE = 0,     /* grouped fwd/dgrad GEMM tile: 64 or 128 */
  RETR_TUNE_GROUP_STAGES = 1,   /* its LDS ring depth: 64-tile 2|4, 128-tile 1|2|3 */
  RETR_TUNE_WGRAD_TILE = 2,     /* grouped weight-gradient tile: 64 or 128 */
  RETR_TUNE_WGRAD_STAGES = 3,   /* its ring depth: 2|4 (64), 2|3 (128) */
  RETR_TUNE_WGRAD_KC = 4,       /* weight-gradient K-slice length in tokens (multiple of 64) */
  RETR_TUNE_ATTN_MODE = 5,      /* bf16 attention: 1 streaming K/V tiles, 2 LDS-resident */
  RETR_TUNE_BIG_TILE = 6,       /* large bf16 GEMMs (convs): 1 128x128 S1, 2 128x128 S2,
                                   3 256x256, 4 128x64 S3, 5 reg-staged 64x64, 6 64x64 S2,
                                   7 128x128 S1 one epilogue band, 8 64x64 S4, 9 64x128 S3,
                                   10 / 11 / 12 32x64 S4 / S3 / S2, 13 64x64 S1, 14 64x128 S1,
                                   15 128x64 S1 */
  RETR_TUNE_NT_STORE = 7,       /* 1: non-temporal GEMM output stores */
  RETR_TUNE_CONV_WGRAD_SPLITS = 8, /* conv weight-gradient split-K: 1 legacy ceil(512 / tiles),
                                      >= 2 that many slices (capped by the K-steps) */
  RETR_TUNE_CONV_WGRAD_TILE = 9, /* conv weight-gradient tile (bf16): 1 always 64x64 LDS-DMA,
                                    2 never (0: the built-in shape rule) */
  RETR_TUNE_ATTN_SPLIT = 10,    /* resident attention backward, two waves per 32 rows (even / odd
                                   tiles): 1 never, 2 dq on every grid and dkdv on 2-wave
                                   grids, 0 (auto) / 3 both on 2-wave grids only, 4 both
                                   everywhere */
  RETR_TUNE_LIN_WGRAD = 11,     /* bf16 linear weight gradient with >= 256 128x128 tiles: 0 auto
                                   (LDS-DMA 128x128, 4 waves), 1 register-staged 128x128,
                                   2 LDS-DMA 256x256, 4 LDS-DMA 128x128 8 waves */
  RETR_TUNE_ATTN_FSPLIT = 12,   /* bf16 streaming attention forward, key split: 0 auto, 1 off,
                                   2 two parities x 64 queries, 3 four parities x 32 queries,
                                   4 two parities x 32 queries */
  RETR_TUNE_LIN_SMALL = 13,     /* 2: few-tile bf16 linears single-pass on the 32x64 LDS-DMA tile
                                   (no split-K up to K 2048; rejected: +0.1 ms/step in the graphed
                                   step, profiles/r3_ab_lin_small.txt); 0 / 1 split-K slabs */
  RETR_TUNE_SHORTK = 14,        /* short-K (K <= 256, N >= 256) bf16 GEMMs on the single-stage
                                   64x64 LDS-DMA tile: 0 auto (on), 1 off */
  RETR_TUNE_ADAMW_NT = 15,      /* AdamW update streams: 0 (auto) / 1 non-temporal loads and
                                   stores, 2 plain, 3 non-temporal with two groups in flight (A/B) */
  RETR_TUNE_WGRAD_B32 = 16,     /* 1: 3x3 / strided conv weight gradients on the 64-bit-cursor
                                   ConvWgradB loader instead of ConvWgradB32 */
  RETR_TUNE_WGRAD_FUSED = 17,   /* grouped bf16 linear weight gradients: 0 slabs + a separate
                                   slab_sum_group launch (default), 1 split-K reduced by each
                                   tile's last-arriving block inside the GEMM launch */
  RETR_TUNE_SPLITK_FUSED = 18,  /* split-K forward / data-gradient linears: 0 slabs + a separate
                                   slab-epilogue launch, 1 slice sum + epilogue by each tile's
                                   last-arriving block (csrc/splitk_fused.hpp) */
  RETR_TUNE_WB_CHUNK = 19,      /* retr_linear_wgrad_batch block order: runs of n > 0 logical
                                   blocks per XCD turn (0: 4).  (Round 5's problem-affine order was
                                   removed in round 6: DESIGN.md section 4) */
  RETR_TUNE_CW_CHUNK = 20,      /* retr_conv2d_wgrad_group block order: runs of n > 0 logical
                                   blocks per XCD turn (0: 4).  (The slice-affine order was
                                   removed in round 6) */
  RETR_TUNE_CONV3X3 = 21,       /* bf16 3x3 stride-1 convs (fwd / dgrad): 0 the direct kernel with
                                   the input halo in LDS on maps >= 32 wide (csrc/conv3x3.hip),
                                   1 the implicit GEMM, 2 the direct kernel on every map >= 16 */
  RETR_TUNE_C3_TILE = 22,       /* direct 3x3 kernel tile variant (sweeps; 0 auto) */
  RETR_TUNE_PANEL = 23,         /* bf16 linears with K <= 256 into N >= 1024 (FFN expansions and
                                   their gated data gradients): 0 the 64x64 gemm2 tile, 1 the
                                   resident-A panel kernel (csrc/panel.hpp; measured 0.39 ms/step
                                   slower, profiles/r4_ab_panel_rejected.txt) */
  RETR_TUNE_PANEL_GROUPS = 24,  /* column-tile runs per row panel (0: ~512 blocks) */
  RETR_TUNE_PANEL_CONV = 25,    /* 1: also the 1x1 stride-1 convs with K <= 256 into >= 1024
                                   channels on the panel kernel (A/B) */
  RETR_TUNE_ATTN_KEEPPRE = 26,  /* bf16 streaming attention forward with dropout and saved keep
                                   bits: 0 hashed inside the forward, 1 pregenerated by
                                   attn_keep_bits_kernel and read by the forward (0.036 ms/step
                                   slower, profiles/r4_ab_keep_bits.txt) */
  RETR_TUNE_LN_BWD = 27,        /* LayerNorm backward (C 256 / 512) rows / waves per block: 0 auto
                                   (32 / 16 at >= 4096 rows, else 8 / 4), 1 32/16, 2 16/8, 3 8/4,
                                   4 16/16, 5 64/16, 6 8/8 (tools/ln_micro.py) */
  RETR_TUNE_UNPACK_GRID = 28,   /* retr_conv_wgrad_unpack_group: 0 one block per output-channel
                                   row; -1 round 5's block per 64 chunks, > 0 that kernel with
                                   its grid capped (A/B) */
  RETR_TUNE_CW_WAVES = 29,      /* retr_conv2d_wgrad_group wave layout of the 128x128 tile (sweeps):
                                   0 kind 0 (1x1) 4 waves / kind 1 (3x3, strided) 8 waves, 1 both
                                   4 waves (64x64 per wave), 2 both 8 waves (32x64 per wave) */
  RETR_TUNE_DEC_ORDER = 30,     /* decode attention blocks (retr_dec_*_heads*): 0 a row's (or beam
                                   group's) head blocks on one XCD (its L2 holds the row's partial
                                   slabs and whole K / V cache lines), 1 block b = (b / H, b % H) */
  RETR_TUNE_DEC_WAVES = 31,     /* decode wave layouts (C 256): 0 four waves per (row, head)
                                   attention block (hd 32, <= 128 self / 256 memory keys), 16 per
                                   64-unit FFN block, 8 per 128-unit block; 1 two / four (round-5
                                   kernels as first built); 2 four / four; 3 16-wave FFN blocks
                                   of both widths; 4 eight-wave 64-unit FFN blocks */
  RETR_TUNE_ROWLN = 32,         /* retr_linear_fwd_splitk_ln at N = 256: 0 auto, 1 the split-K
                                   slabs + slab_epilogue_ln path, 2 / 3 / 4 the row-complete
                                   32 x 256 tile with the LayerNorm in its epilogue (2 / 3 / 4
                                   stage ring), 5 its 64 x 256 8-wave variant (csrc/linear.hip) */
  RETR_TUNE_LIN_K256 = 33,      /* bf16 linears with K = 256 on the register-staged tiles (few
                                   output tiles: M 2048 / 6400 x N 256): 0 / 2 every K-step
                                   fetched at once (gemm2.hpp gemm_short_kernel), 1 the
                                   double-buffered K loop (gemm.hpp gemm_kernel) */
  RETR_TUNE_COUNT = 40
};
int retr_tune(int knob, int value);

/* ---- grouped projections (csrc/linear_group.hip): up to 16 independent GEMMs of one block in
 * one launch -- the q|k and v in-projections of SelfAttResidual, q / k / v of CrossAttResidual
 * (models/transformer_modules.py:38,66 -> torch/nn/functional.py:5785-5850), their data
 * gradients, and the weight gradients of a whole block.  fp32 (dtype 0) runs the problems one
 * by one through the single-GEMM entry points. */
typedef struct {
  const void* x; long ldx;          /* [M][K] */
  const void* w; long ldw;          /* [N][K] */
  const float* bias;                /* [N] or NULL */
  void* y; long ldy;                /* [M][N] (dtype, or fp32 when y_f32) */
  const float* residual; long ldr;  /* [M][N] fp32 or NULL */
  float drop_p; unsigned long long seed;
  int M, N, K, relu;
} retr_linear_fwd_desc;
int retr_linear_fwd_group(int dtype, int y_f32, int n, const retr_linear_fwd_desc* d,
                          void* stream);

typedef struct {
  const void* dy; long lddy;        /* [M][N] */
  const void* w; long ldw;          /* W [N][K] (w_trans 0) or W^T [K][N] (w_trans 1) */
  void* dx; long lddx;              /* [M][K] */
  const void* addend; long lda;     /* or NULL */
  const void* gate; long ldg;       /* or NULL */
  int M, N, K, pad;
} retr_linear_dgrad_desc;
int retr_linear_dgrad_group(int dtype, int dx_f32, int addend_f32, int w_trans, int n,
                            const retr_linear_dgrad_desc* d, void* stream);

/* dw[N][K] (=|+=) dy^T x, db[N] (=|+=) colsum dy for up to 8 problems: token-split fp32 slabs
 * (plain stores) summed in slice order by a second launch -- deterministic, no atomics.
 * workspace: retr_linear_wgrad_group_workspace(n, d) bytes of device memory. */
typedef struct {
  const void* dy; long lddy;        /* [M][N] */
  const void* x; long ldx;          /* [M][K] */
  float* dw; long lddw;             /* [N][K] */
  float* db;                        /* [N] or NULL */
  int M, N, K, accumulate;
} retr_linear_wgrad_desc;
size_t retr_linear_wgrad_group_workspace(int n, const retr_linear_wgrad_desc* d);
int retr_linear_wgrad_group(int dtype, int n, const retr_linear_wgrad_desc* d, void* workspace,
                            void* stream);
/* extra fixed-order partial sums folded into the weight-gradient group's slab-sum launch:
 * dst[c] (=|+=) sum_{s < nparts} parts[s * stride + c], c < cols (e.g. a LayerNorm's
 * dgamma / dbeta partial rows from retr_layernorm_bwd2) */
typedef struct {
  const float* parts;
  long stride;
  int nparts, cols;
  float* dst;
  int accumulate;
} retr_slab_sum_desc;
int retr_linear_wgrad_group2(int dtype, int n, const retr_linear_wgrad_desc* d, void* workspace,
                             int nx, const retr_slab_sum_desc* x, void* stream);
/* Deferred weight-gradient batch (bf16): the weight gradients of many blocks -- e.g. every
 * projection of a whole transformer backward, models/transformer_modules.py:22-97 via
 * torch/nn/functional.py:5785-5850 -- in ONE launch, one K-slice per tile (no fp32 slabs, no
 * slab-sum launch); db[N] (=|+=) colsum dy rides along in the first column tile; the nx extra
 * partial-row sums (LayerNorm dgamma / dbeta) are summed by extra blocks of the same launch.
 * Every output element is one fp32 chain over all M tokens in order, whatever the batch.
 * table: device memory of retr_linear_wgrad_batch_table_bytes(n, nx) bytes (16-byte aligned),
 * written in stream order by this call; keep it alive until the launch has run. */
size_t retr_linear_wgrad_batch_table_bytes(int n, int nx);
int retr_linear_wgrad_batch(int n, const retr_linear_wgrad_desc* d, int nx,
                            const retr_slab_sum_desc* x, void* table, size_t table_bytes,
                            void* stream);

/* ---- fused feed-forward block (models/transformer_modules.py:6-11,77-97 feed_forward inside
 * FFResidual; replaces the linear_fwd (ReLU) + linear_fwd_splitk pair of the forward and the
 * linear_dgrad (ReLU gate) + linear_dgrad_splitk pair of the backward at d_model 256, bf16):
 *   retr_ffn_fwd       h = relu(n W1^T + b1) -> h [M][F] bf16;  y = res + drop(h W2^T + b2) fp32
 *   retr_ffn_bwd_data  dh = [h > 0] (dbr W2) -> dh [M][F] bf16;  dn = dh W1 -> dn [M][C] bf16
 * W1 [F][C], W2 [C][F] row-major bf16 (the backward reads them transposed in LDS).  ws: fp32
 * [splits][M][C] slabs; splits from retr_ffn_splits(M, C, F) (0 = shape not supported: C must
 * be 256, F a multiple of 64). */
int retr_ffn_splits(int M, int C, int F);
int retr_ffn_fwd(const void* n, long ldn, const void* w1, const float* b1, const void* w2,
                 const float* b2, void* h, long ldh, const float* residual, long ldr, float* y,
                 long ldy, int M, int C, int F, float drop_p, unsigned long long seed, float* ws,
                 int splits, void* stream);
int retr_ffn_bwd_data(const void* dbr, long lddbr, const void* w2, const void* h, long ldh,
                      const void* w1, void* dh, long lddh, void* dn, long lddn, int M, int C,
                      int F, float* ws, int splits, void* stream);

/* ---- ResNet convolutions (torchvision conv stack via models/backbone.py:65-69, FrozenBN
 * models/backbone.py:41-51 folded into the weights) --------------------------------------- */
int retr_conv_pack(int dtype, const float* w, const float* bn_w, const float* bn_b,
                   const float* bn_rm, const float* bn_rv, const float* conv_bias, int Co, int Ci,
                   int KH, int KW, int Cp, void* w_out, void* wt_out, float* bias_out,
                   float* scale_out, void* stream);
/* every conv's packing in one launch (up to 16 per kernel, more in further launches) */
typedef struct {
  const float *w, *bn_w, *bn_b, *bn_rm, *bn_rv, *conv_bias;   /* as retr_conv_pack */
  void *w_out, *wt_out;
  float *bias_out, *scale_out;
  int Co, Ci, KH, KW, Cp, pad;
} retr_conv_pack_desc;
int retr_conv_pack_group(int dtype, int n, const retr_conv_pack_desc* d, void* stream);
/* bf16 [W3eff | Wdseff] (rows x (ka + kb), ka, kb % 8 == 0) and b3 + bds of the fused bottleneck
   tails (retr_conv1x1_fwd_cat operands), up to 8 per launch */
typedef struct {
  const void *a, *b;
  void* dst;
  const float *bias_a, *bias_b;
  float* bias_dst;
  int rows, ka, kb;
} retr_cat_rows_desc;
int retr_cat_rows_group(int n, const retr_cat_rows_desc* d, void* stream);
int retr_conv2d_fwd(int dtype, const void* x, int Nb, int H, int W, int C, const void* w,
                    const float* bias, const void* residual, void* y, int Co, int KH, int KW,
                    int stride, int pad, int dil, int relu, void* stream);
/* retr_conv2d_fwd over an explicit output extent OH x OW (<= the conv's own; used by the
 * space-to-depth stem, a 4x4 pad-2 conv whose 321st row / column torchvision never computes) */
int retr_conv2d_fwd_out(int dtype, const void* x, int Nb, int H, int W, int C, const void* w,
                        const float* bias, const void* residual, void* y, int Co, int KH, int KW,
                        int stride, int pad, int dil, int OH, int OW, int relu, void* stream);
/* Bottleneck tail with its 1x1 downsample folded in (torchvision Bottleneck.forward:
 * relu(bn3(conv3(h)) + bn_ds(conv_ds(x))), models/backbone.py:65) as ONE 1x1 conv over the
 * channel concatenation [x1 | x2] (never materialised): y[Nb*OH*OW][Co] =
 * act([x1 x2'] . w^T + bias), x1 [Nb*OH*OW][C1] (h), x2 [Nb][H2][W2][C2] (the block input)
 * sampled at stride2 (x2' = x2[:, ::s, ::s]), w [Co][C1 + C2] = [W3eff | Wdseff],
 * bias = b3 + bds.  bf16 only. */
int retr_conv1x1_fwd_cat(int dtype, const void* x1, int C1, const void* x2, int C2, int Nb,
                         int OH, int OW, int H2, int W2, int stride2, const void* w,
                         const float* bias, void* y, int Co, int relu, void* stream);
/* dx[Nb][H][W][C] = gate(dgrad(dy, W) [+ addend]), gate = (gate > 0).  addend may be dx itself
 * (in place) when dx already holds gate(addend) at every pixel: a stride-2 conv then rewrites
 * only the pixels its taps reach (ResNet first blocks: the 1x1 stride-2 downsample's data
 * gradient added onto conv1's gated one, resnet.py) */
int retr_conv2d_dgrad(int dtype, const void* dy, int Nb, int H, int W, int C, const void* wt,
                      void* dx, int Co, int KH, int KW, int stride, int pad, int dil,
                      const void* addend, const void* gate, void* stream);
/* ws[splits][Co][KH*KW*C] = partial dWeff per slice of the pixel reduction (fp32, plain
 * stores, overwritten; NHWC tap order; no atomics).  splits = retr_conv2d_wgrad_splits(...) */
int retr_conv2d_wgrad(int dtype, const void* dy, const void* x, int Nb, int H, int W, int C,
                      float* ws, int Co, int KH, int KW, int stride, int pad, int dil,
                      void* stream);
int retr_conv2d_wgrad_splits(int dtype, int Nb, int H, int W, int C, int Co, int KH, int KW,
                             int stride, int pad, int dil);
/* Grouped bf16 weight gradients of many convolutions -- the whole backbone backward of
 * models/backbone.py:65,69,86-91 (torchvision Bottleneck convs) -- in two launches (dense 1x1
 * stride-1 convs; 3x3 / strided convs), one K-slice length for the whole group instead of each
 * conv's own split count.  Usage: fill the geometry, call _plan (sets kind: 0 dense 1x1, 1 3x3 /
 * strided, -1 not groupable -> retr_conv2d_wgrad; and splits), allocate ws[splits][Co][KH*KW*C]
 * fp32 per problem, call retr_conv2d_wgrad_group, then retr_conv_wgrad_unpack(..., splits) per
 * problem.  table: retr_conv2d_wgrad_group_table_bytes(n) + 512 bytes of device memory. */
typedef struct {
  const void* dy; const void* x;    /* dY [Nb*OH*OW][Co], X [Nb][H][W][C] (bf16, NHWC) */
  float* ws;                        /* [splits][Co][KH*KW*C] fp32 slabs */
  int Nb, H, W, C, Co, KH, KW, stride, pad, dil;
  int splits, kind;                 /* set by retr_conv2d_wgrad_group_plan */
} retr_conv_wgrad_desc;
size_t retr_conv2d_wgrad_group_table_bytes(int n);
int retr_conv2d_wgrad_group_plan(int dtype, int n, retr_conv_wgrad_desc* d);
int retr_conv2d_wgrad_group(int dtype, int n, const retr_conv_wgrad_desc* d, void* table,
                            size_t table_bytes, void* stream);
/* Every grouped conv's slab sum + OIHW re-layout (+ scale) in one launch:
 * grad[Co][Ci][KH][KW] (=|+=) scale[co] * sum_s ws[s][co][kh][kw][ci] (slices summed by four
 * waves in a fixed order).  table: retr_conv_wgrad_unpack_group_table_bytes(n) bytes of device
 * memory (16-byte aligned), written in stream order by the call. */
typedef struct {
  const float* ws; const float* scale;   /* scale [Co] or NULL */
  float* grad;
  int Co, Ci, Cp, KH, KW, splits, accumulate, pad;
} retr_conv_unpack_desc;
size_t retr_conv_wgrad_unpack_group_table_bytes(int n);
int retr_conv_wgrad_unpack_group(int n, const retr_conv_unpack_desc* d, void* table,
                                 size_t table_bytes, void* stream);
/* grad[Co][Ci][KH][KW] (=|+=) scale[co] * sum_s ws[s] (slices added in order: deterministic) */
int retr_conv_wgrad_unpack(const float* ws, const float* scale, float* grad, int Co, int Ci,
                           int Cp, int KH, int KW, int accumulate, int splits, void* stream);
/* Fused stride-1 bottleneck forward for the frozen layer1 (torchvision Bottleneck,
 * models/backbone.py:65; frozen by models/backbone.py:58-60, so backward needs none of its
 * activations): y = relu(conv1x1_64->256(relu(conv3x3(relu(conv1x1(x))))) + residual), all BN
 * folded.  ds = 0: identity residual (Cin = 256, w3 [256][64]); ds = 1: the 1x1 stride-1
 * downsample folded in (Cin = 64, w3 = [W3 | Wds] [256][128], b3 = b3 + bds).  w1 [64][Cin],
 * w2 [64][3][3][64] packed (retr_conv_pack layout), NHWC bf16, H % 8 == 0, W % 16 == 0.
 * Bitwise equal to retr_conv2d_fwd x 3 (or x 2 + retr_conv1x1_fwd_cat). */
int retr_bottleneck_s1_fwd(int dtype, const void* x, int N, int H, int W, int Cin,
                           const void* w1, const float* b1, const void* w2, const float* b2,
                           const void* w3, const float* b3, int ds, void* y, void* stream);
/* Fused frozen stem (retr_amd/csrc/stem.hip; torchvision conv1 + bn1 + relu + maxpool,
 * models/backbone.py:85-95, frozen by models/backbone.py:58-60): the space-to-depth conv
 * (x [N][H2][W2][16] from retr_nchw_to_s2d16, w [Co][4][4][16] from retr_stem_s2d_weights, bias
 * fp32, stride 1, pad 2, output H2 x W2) + bias + ReLU + MaxPool2d(3, 2, 1) in one launch;
 * y [N][(H2+1)/2][(W2+1)/2][Co] bf16, Co == 64.  The conv output never reaches HBM.  Bitwise
 * equal to retr_conv2d_fwd_out + retr_maxpool3x3s2. */
int retr_stem_pool_fwd(int dtype, const void* x, int N, int H2, int W2, const void* w,
                       const float* bias, void* y, int Co, void* stream);
/* NCHW fp32 image -> NHWC (channels zero-padded to Cp) */
int retr_nchw_to_nhwc(int dtype, const float* x, void* y, int N, int C, int H, int W, int Cp,
                      void* stream);
/* bf16 space-to-depth stem input (models/backbone.py:85-95 -> torchvision conv1, 7x7 stride 2
 * pad 3): y[n][Y][X][(dy*2+dx)*3+c] = x[n][c][2Y+dy][2X+dx], 12 channels + 4 zero (C == 3,
 * H and W even) */
int retr_nchw_to_s2d16(const float* x, void* y, int N, int C, int H, int W, void* stream);
/* the stem's packed [Co][7][7][Cp] bf16 weights re-laid for that input: [Co][4][4][16],
 * w2[co][i][j][(dy*2+dx)*3+c] = wp[co][2i+dy-1][2j+dx-1][c] (zero off the 7x7 taps); the conv
 * is then retr_conv2d_fwd_out(k 4, stride 1, pad 2, OH = H/2, OW = W/2) */
int retr_stem_s2d_weights(const void* wp, void* w2, int Co, int Cp, void* stream);
/* RefCOCO encoder-input pipeline (data_utils/refcoco.py:131-178, data_utils/utils.py:161-252):
 * one descriptor per item; coefficient / window tables computed on the host as Pillow /
 * torchvision do (retr_amd/data_pipeline.py). */
typedef struct {
  long long src_off;            /* byte offset of the item's HxWx3 uint8 image in src */
  long long tmp_off;            /* byte offset of its horizontal-pass buffer [D][S][3] in tmp */
  int H, W;                     /* source image size */
  int x0, y0, rw, rh;           /* pasted region: source origin and size */
  int bx, by, bw, bh;           /* context: zeroed / masked box in region coordinates (bw 0: none) */
  int D, ox, oy;                /* padded side, image paste offsets (ImageOps.pad rounding) */
  int mx, my;                   /* mask paste offsets (pad_mask_to_max: floor) */
  int coef_off, ksize;          /* ints into coef: bounds [S][2] (xmin, count), then [S][ksize] */
  int win_off;                  /* ints into win: mask tap windows [S][2] (lo, hi) */
  int ops;                      /* ColorJitter ops, 4 bits per slot in order: 1 brightness,
                                   2 contrast, 3 saturation, 0 end */
  float f[3];                   /* their factors */
  int pad_[2];
} retr_pipe_item;
/* crop/pad/resize (+ jitter) + normalise n items to fp32 [n][3][S][S] (u8: [n][S][S][3]
 * scratch, tmp: sum of D*S*3 bytes) and, when mask != null, their resized masks [n][S][S];
 * src, items, coef, win, tmp, u8, out, mask are device pointers, mean / std_ host float[3] */
int retr_pipe_run(const unsigned char* src, const retr_pipe_item* items, int n, const int* coef,
                  const int* win, unsigned char* tmp, int max_d, unsigned char* u8, float* out,
                  unsigned char* mask, int S, const float* mean, const float* std_,
                  void* stream);
/* MaxPool2d(3, 2, 1) on NHWC (torchvision stem) */
int retr_maxpool3x3s2(int dtype, const void* x, void* y, int N, int H, int W, int C, int OH,
                      int OW, void* stream);
/* F.interpolate(mask[None].float(), size=(h,w)) nearest -> bool (models/backbone.py:75) */
int retr_mask_nearest(const unsigned char* m, unsigned char* out, int N, int H, int W, int h,
                      int w, void* stream);

/* ---- LayerNorm (nn.LayerNorm in SelfAttResidual/CrossAttResidual/FFResidual, encoder/decoder
 * final norms: models/transformer_modules.py:31,58,89; models/ConcatTransformer.py:105,146) ---
 * y = LN(x) (type dtype), y2 = y + pos[row % period] (optional), saves mean/rstd */
int retr_layernorm_fwd(int dtype, const float* x, long ldx, const float* gamma,
                       const float* beta, float eps, int M, int C, void* y, long ldy, void* y2,
                       const float* pos, int period, float* mean, float* rstd, void* stream);
/* dx = [addend +] LN'(dy [+ dy2]); dgamma/dbeta accumulate (fp32) via per-block partials in
 * `workspace` (retr_layernorm_bwd_workspace bytes) reduced in a fixed order (deterministic) */
int retr_layernorm_bwd(int dtype, const void* dy, const void* dy2, long lddy, const float* x,
                       long ldx, const float* gamma, const float* mean, const float* rstd, int M,
                       int C, float* dx, long lddx, const float* addend, float* dgamma,
                       float* dbeta, float* workspace, void* stream);
size_t retr_layernorm_bwd_workspace(int M, int C);
/* retr_layernorm_bwd plus two fusions of the transformer blocks' backward (ops._ln_bwd):
 *  - dxd != NULL: also writes dxd = bf16(dropout(dx)) with the (drop_p, seed) mask of the
 *    residual dropout that PRODUCED this LayerNorm's input (the previous block's
 *    retr_dropout_apply of its incoming gradient, models/transformer_modules.py:44-46);
 *  - nparts != NULL: the dgamma/dbeta partial rows are left in `workspace` ([*nparts][2C]:
 *    dgamma partials in columns [0, C), dbeta in [C, 2C)) for the caller's slab sum
 *    (retr_linear_wgrad_group2) instead of a reduction launch. */
int retr_layernorm_bwd2(int dtype, const void* dy, const void* dy2, long lddy, const float* x,
                        long ldx, const float* gamma, const float* mean, const float* rstd, int M,
                        int C, float* dx, long lddx, const float* addend, float* dgamma,
                        float* dbeta, float* workspace, void* dxd, long lddxd, float drop_p,
                        unsigned long long seed, int* nparts, void* stream);
/* retr_layernorm_bwd2 whose incoming gradient is the fp32 split-K slabs of the producing bf16
 * data gradient (retr_linear_dgrad_slabs): dy = bf16(sum of ws[0..splits) in slice order) --
 * bitwise the retr_linear_dgrad_splitk + retr_layernorm_bwd2 pair, one launch and the bf16 dy
 * round trip fewer.  C 256 or 512, 16-byte aligned rows.  Replaces the LayerNorm backward of
 * the FFN block's pre-norm (models/transformer_modules.py:6-11) after the up-projection's data
 * gradient. */
int retr_layernorm_bwd_slabs(const float* ws, int splits, const float* x, long ldx,
                             const float* gamma, const float* mean, const float* rstd, int M,
                             int C, float* dx, long lddx, const float* addend, float* dgamma,
                             float* dbeta, float* workspace, void* dxd, long lddxd, float drop_p,
                             unsigned long long seed, int* nparts, void* stream);

/* ---- DecoderEmbeddings: word[caps] + pos[t] -> LayerNorm(eps) -> dropout
 * (models/transformer_modules.py:113-129) ------------------------------------------------- */
int retr_embed_ln_fwd(const long long* tokens, int B, int T, int C, const float* word,
                      const float* posw, const float* gamma, const float* beta, float eps,
                      float drop_p, unsigned long long seed, float* y, float* mean, float* rstd,
                      void* stream);
/* deterministic (no atomics): dword rows are summed in token-position order by one writer,
 * dposw over the batch in order, dgamma/dbeta from per-block partials in block order.
 * workspace: retr_embed_ln_bwd_workspace(B, T, C) bytes. */
int retr_embed_ln_bwd(const long long* tokens, int B, int T, int C, const float* word,
                      const float* posw, const float* gamma, const float* mean, const float* rstd,
                      const float* dy, float drop_p, unsigned long long seed, float* dword,
                      float* dposw, float* dgamma, float* dbeta, int padding_idx,
                      void* workspace, void* stream);
size_t retr_embed_ln_bwd_workspace(int B, int T, int C);

/* ---- multi-head attention core: softmax(q k^T * hd^-1/2 + mask) -> dropout -> @ v
 * (torch/nn/functional.py:6576-6606 need_weights path used by models/ConcatTransformer.py:160,
 * 204,210).  q: row (b*Lq+i) at q + row*ldq + h*hd; k/v likewise with Lk.  kpm: uint8 [B][Lk]
 * (1 = padded key).  lse: fp32 [B*H][Lq] saved for backward.  probs (optional): fp32
 * [B][Lq][Lk] head-averaged attention weights (att dicts of Caption.forward). */
int retr_attention_fwd(int dtype, const void* q, long ldq, const void* k, long ldk,
                       const void* v, long ldv, void* o, long ldo, int B, int H, int Lq, int Lk,
                       int hd, const unsigned char* kpm, int causal, float drop_p,
                       unsigned long long seed, float* lse, float* probs, void* stream);
int retr_attention_bwd(int dtype, const void* q, long ldq, const void* k, long ldk,
                       const void* v, long ldv, const void* o, long ldo, const void* dout,
                       long lddo, const float* lse, void* dq, long lddq, void* dk, long lddk,
                       void* dv, long lddv, int B, int H, int Lq, int Lk, int hd,
                       const unsigned char* kpm, int causal, float drop_p,
                       unsigned long long seed, float* workspace, void* stream);
size_t retr_attention_bwd_workspace(int B, int H, int Lq);
/* The same pair with the attention-dropout keep decisions saved by the forward: dmask
 * (retr_attention_dropout_mask_bytes) receives one bit per score ([B*H][ceil(Lk/32)][Lq]
 * uint32 words) from retr_attention_fwd_dm when drop_p > 0 on the bf16 head-dim 32/64 kernels,
 * and retr_attention_bwd_dm reads it instead of regenerating every decision from the hash --
 * the same bits, so the same results.  Paths that do not use it leave / ignore it. */
size_t retr_attention_dropout_mask_bytes(int B, int H, int Lq, int Lk);
int retr_attention_fwd_dm(int dtype, const void* q, long ldq, const void* k, long ldk,
                          const void* v, long ldv, void* o, long ldo, int B, int H, int Lq,
                          int Lk, int hd, const unsigned char* kpm, int causal, float drop_p,
                          unsigned long long seed, float* lse, float* probs, void* dmask,
                          void* stream);
int retr_attention_bwd_dm(int dtype, const void* q, long ldq, const void* k, long ldk,
                          const void* v, long ldv, const void* o, long ldo, const void* dout,
                          long lddo, const float* lse, void* dq, long lddq, void* dk, long lddk,
                          void* dv, long lddv, int B, int H, int Lq, int Lk, int hd,
                          const unsigned char* kpm, int causal, float drop_p,
                          unsigned long long seed, float* workspace, const void* dmask,
                          void* stream);
/* decode step: q [B][.] one query row per caption (or beam); k/v with Lmax rows per kv batch,
 * first Lk valid.  Query row r attends kv batch r / kv_group (kv_group = beams per image for
 * the shared cross-attention memory, else 1); with `anc` (int32 [B][Lmax], beam search) key j
 * of row r is cache row anc[r][j] * Lmax + j instead. */
int retr_attention_decode(int dtype, const void* q, long ldq, const void* k, long ldk,
                          const void* v, long ldv, void* o, long ldo, int B, int H, int Lk,
                          int Lmax, int hd, const unsigned char* kpm, int kv_group,
                          const int* anc, void* stream);

/* ---- CrossEntropyLoss (models/caption.py:210, engine.py:71) and argmax (decode.py:71) ----- */
int retr_ce_fwd(int dtype, const void* logits, long ld, int M, int V, const long long* targets,
                float* lse, float* loss_rows, float* loss, void* stream);
int retr_ce_bwd(int dtype, const void* logits, long ld, int M, int V, const long long* targets,
                const float* lse, const float* dloss, float inv_count, void* dlogits, long lddl,
                void* stream);
/* Training form of the pair above (bf16 logits, ld % 8 == 0, lddl % 8 == 0): one pass over the
   logits writes lse, the per-row losses, the mean and dlogits = (softmax - onehot) * inv_count
   as for dloss = 1 (what loss.backward() passes); retr_ce_bwd_rescale then rewrites dlogits with
   retr_ce_bwd's arithmetic only when *dloss != 1. */
int retr_ce_fwd_bwd(int dtype, const void* logits, long ld, int M, int V,
                    const long long* targets, float* lse, float* loss_rows, float* loss,
                    float inv_count, void* dlogits, long lddl, void* stream);
int retr_ce_bwd_rescale(int dtype, const void* logits, long ld, int M, int V,
                        const long long* targets, const float* lse, const float* dloss,
                        float inv_count, void* dlogits, long lddl, void* stream);
int retr_argmax_rows(int dtype, const void* x, long ld, int M, int V, long long* out,
                     void* stream);
/* the same first-index argmax for few long rows (decode logits): 16 segments per row in
 * parallel, partials reduced by a second kernel.  workspace: retr_argmax_workspace(M) bytes;
 * falls back to retr_argmax_rows for fp32 / short rows */
size_t retr_argmax_workspace(int M);
int retr_argmax_rows_ws(int dtype, const void* x, long ld, int M, int V, long long* out,
                        void* workspace, void* stream);

/* greedy bookkeeping for step i (eval_utils/decode.py:72-79) on device */
/* ---- beam search (new capability; reference decode.py has greedy only) -------------------
 * per row of x [M][ld]: the K best (index, log-softmax value), first index on ties (K <= 8) */
int retr_topk_rows(int dtype, const void* x, long ld, int M, int V, int K, int* idx,
                   float* logprob, void* stream);
/* one beam step for B images x K beams: select survivors from the retr_topk_rows candidates,
 * reorder hist [B*K][T] / anc [B*K][T], append step i's token, done = i once all finished */
int retr_beam_select(const int* cand_tok, const float* cand_lp, int B, int K, int i, int T,
                     long long eos, float* scores, unsigned char* finished, long long* hist,
                     int* anc, long long* tok, unsigned char* item_done, int* done,
                     void* stream);
int retr_greedy_update(const long long* pred, int B, int T, int i, long long eos,
                       long long* caption, unsigned char* finished, int* done, long long* tok,
                       void* stream);
/* retr_argmax_rows_ws + retr_greedy_update with the per-row reduction and the bookkeeping in
 * one launch (pred is written too); workspace: retr_argmax_workspace(B) bytes */
int retr_greedy_select(int dtype, const void* logits, long ld, int B, int V, void* workspace,
                       int T, int i, long long eos, long long* pred, long long* caption,
                       unsigned char* finished, int* done, long long* tok, void* stream);
/* retr_greedy_select for one row group of a batch decoded as independent groups (write_all = 1:
 * every column written, done = the group's first all-finished step; eval_utils/decode.py
 * DEC_SPLIT clears the columns after the last group's) */
int retr_greedy_select2(int dtype, const void* logits, long ld, int B, int V, void* workspace,
                        int T, int i, long long eos, long long* pred, long long* caption,
                        unsigned char* finished, int* done, long long* tok, int write_all,
                        void* stream);

/* ---- elementwise helpers --------------------------------------------------------------- */
/* Encoder output without a final LayerNorm (pre_norm=False; models/ConcatTransformer.py:24,
 * 105-106): y = cast(x), y2 = cast(x + pos[row % period]) (either output may be NULL) */
int retr_add_pos_fwd(int dtype, const float* x, long ldx, int M, int C, const float* pos,
                     int period, void* y, void* y2, long ldy, void* stream);
/* out[i] (fp32) = a[i] + b[i] (either input may be NULL): gradient of retr_add_pos_fwd */
int retr_sum2(int dtype, const void* a, const void* b, long n, float* out, void* stream);
/* y[m][n] = x[m][n] * keep(seed, m*N+n) * scale   (backward of the branch dropout) */
int retr_dropout_apply(int dtype_out, const float* x, long ldx, void* y, long ldy, int M, int N,
                       float drop_p, unsigned long long seed, void* stream);
/* y[c][r] = x[r][c] (fp32 -> dtype), rows R..R_pad-1 of y's inner dim zero-filled */
int retr_transpose_cast(int dtype, const float* x, void* y, int R, int C, int R_pad,
                        void* stream);
/* out (dtype) <- in (fp32), contiguous */
int retr_cast(int dtype, const float* x, void* y, long n, void* stream);
/* dpos[p][c] += sum_{m: m % period == p} d[m][c] */
int retr_pos_grad(int dtype, const void* d, long ld, int M, int C, int period, float* dpos,
                  void* stream);
/* retr_pos_grad with dpos overwritten (dpos = the sums): no zero fill before a fresh gradient */
int retr_pos_grad_set(int dtype, const void* d, long ld, int M, int C, int period, float* dpos,
                      void* stream);
/* Several contributions to one position-gradient buffer (the decoder blocks' query-position
 * gradients, models/ConcatTransformer.py's query_pos used by every decoder layer) in one launch:
 * dpos (+)= sum over items in order of sum_b d_i[b * period + t] -- bitwise the sequence of
 * retr_pos_grad calls (the first one retr_pos_grad_set when accumulate is 0). */
typedef struct retr_pos_item {
  const void* d;
  long ld;
  int M;
  int pad;
} retr_pos_item;
int retr_pos_grad_multi(int dtype, int n, const retr_pos_item* items, int C, int period,
                        float* dpos, int accumulate, void* stream);

/* ---- fused clip_grad_norm_ + AdamW over flat fp32 arenas --------------------------------
 * Replaces engine.py:80-83 (torch.nn.utils.clip_grad_norm_ + optimizer.step()) with the
 * optimizer built at main.py:39-41 (torch.optim.AdamW, two param groups).
 * retr_adamw_sumsq: partials[b] = sum of grad^2 over a grid-stride slice (b < nparts; grad may
 *   be NULL -> zeros); if step != NULL, *step += 1 (device-side step counter).
 * retr_adamw_update: coef = min(max_norm / (sqrt(sum partials) + 1e-6), 1) when max_norm > 0;
 *   g *= coef (written back only when coef < 1); AdamW (amsgrad=False, maximize=False) with
 *   hyper = {lr, weight_decay} read from device memory and bias corrections from the step count
 *   *step + step_offset (the offset covers parameters that skipped steps without a gradient).
 *   n % 4 == 0, all arrays 16-byte aligned. */
int retr_adamw_sumsq(const float* grad, long n, float* partials, int nparts, float* step,
                     void* stream);
/* param_bf16 (optional): bf16 copy of the updated parameters (the GEMM weight shadow) */
int retr_adamw_update(float* param, float* grad, float* exp_avg, float* exp_avg_sq, long n,
                      const float* hyper, double beta1, double beta2, float eps,
                      const float* step, float step_offset, const float* partials, int nparts,
                      float max_norm, void* param_bf16, void* stream);
/* retr_adamw_update with zero_grad = 1: the gradient arena range is zeroed by the update (the
 * clipped gradient is not written back) -- GraphedTrainStep's consume mode */
int retr_adamw_update2(float* param, float* grad, float* exp_avg, float* exp_avg_sq, long n,
                       const float* hyper, double beta1, double beta2, float eps,
                       const float* step, float step_offset, const float* partials, int nparts,
                       float max_norm, void* param_bf16, int zero_grad, void* stream);

/* ---- fused incremental-decode step (csrc/decode.hip; eval_utils/decode.py:53-81 in KV-cache
 * form, decoder layer models/ConcatTransformer.py:187-214 + transformer_modules.py:22-97).
 * bf16 weights [N][K] row-major, fp32 residual rows [R][C], bf16 activations.
 * dec_gemm: out = A W^T + b (opt. ReLU) over N columns; column n goes to segment s = n / segw:
 * row r -> d_s + r * rs_s + (n - s*segw) (bf16); pos_s selects A = a_pos, else a_plain. */
int retr_dec_gemm(const void* a_plain, const void* a_pos, int R, int C, const void* w,
                  const float* bias, int N, void* d0, long rs0, int pos0, void* d1, long rs1,
                  int pos1, void* d2, long rs2, int pos2, int segw, int relu, void* stream);
/* x = xin (+ b2 + sum_j slabs[j], in slab order); xout = x (optional); n = LN(x) (bf16),
 * npos = LN(x) + pos (bf16, optional) */
int retr_dec_rows(const float* xin, const float* slabs, int nslab, const float* b2, int R, int C,
                  float* xout, const float* gamma, const float* beta, float eps, const float* pos,
                  void* n, void* npos, void* stream);
/* decode-step input rows: x = LN_e(word[tok[r]] + qpos) (fp32, the retr_embed_ln_fwd
 * arithmetic, DecoderEmbeddings models/ConcatTransformer.py:224-243 at one position), then
 * n = LN1(x), npos = LN1(x) + qpos (bf16, the retr_dec_rows arithmetic) */
int retr_dec_embed_rows(const long long* tok, int R, int C, const float* word, const float* qpos,
                        const float* ge, const float* be, float epse, float* x, const float* g1,
                        const float* b1, float eps1, void* n, void* npos, void* stream);
/* per query row: multi-head attention over Lk cache/memory rows ((anc ? anc[r][j] : r/kv_group)
 * * Lmax + j; kpm [R/kv_group][Lk]), xo = x + o Wo^T + bo, then LN(xo) (+pos) -> q2 = (.) Wq^T
 * + bq, or q2 = LN(xo) when wq is NULL */
int retr_dec_attn_row(const void* q, const void* k, const void* v, int R, int C, int H, int Lk,
                      int Lmax, int kv_group, const int* anc, const unsigned char* kpm,
                      const float* x, const void* wo, const float* bo, float* xo,
                      const float* gamma, const float* beta, float eps, const float* pos,
                      const void* wq, const float* bq, void* q2, void* stream);
/* FFN over hidden units [32 j, 32 j + 32): slabs[j] = relu(n3 W1_j^T + b1_j) W2[:, j]^T (fp32) */
/* Decode-step attention sub-layers, one wave per (row, head) (csrc/decode_heads.hip; replace
 * retr_dec_gemm + retr_dec_attn_row x 2 of the fused step, eval_utils/decode.py:53-81 in
 * KV-cache form).  Self: the head's q|k|v from n / npos and W_in [3C][C], k / v written to the
 * cache row r * Lmax + i, attention over keys 0..i (beam ancestry anc), then the head's partial
 * out-projection into slab[h][R][C].  Cross: xo = x + (sum_h slab_in[h] + bo_in) (heads in
 * order), LN(xo) (+pos), the head's query from wq rows [h hd, (h+1) hd) + bq, attention over
 * the memory rows (r / kv_group) * Lk + j (kpm masks), the head's partial out-projection into
 * slab_out[h][R][C].  C 256 | 512, head dim 32 | 64. */
int retr_dec_self_heads(const void* n, const void* npos, int R, int C, int H, const void* win,
                        const float* bin, void* kc, void* vc, int i, int Lmax, const int* anc,
                        const void* wo, float* slab, void* stream);
/* retr_dec_self_heads with the layer's LN1 in its prologue (xin != NULL; n / npos ignored):
 * x = xin + (sum_j slabs[j] + b2) (the previous layer's FFN partials [nslab][R][C]), written to
 * xout, n = bf16(LN1(x)), npos = bf16(LN1(x) + qpos) -- the retr_dec_rows launch between decoder
 * layers folded in. */
int retr_dec_self_heads_ln(const void* n, const void* npos, int R, int C, int H, const void* win,
                           const float* bin, void* kc, void* vc, int i, int Lmax, const int* anc,
                           const void* wo, float* slab, const float* xin, const float* slabs,
                           int nslab, const float* b2, const float* gamma, const float* beta,
                           float eps, const float* qpos, float* xout, void* stream);
int retr_dec_cross_heads(const float* slab_in, const float* x, const float* bo_in, float* xo,
                         int R, int C, int H, const float* gamma, const float* beta, float eps,
                         const float* pos, const void* wq, const float* bq, const void* k,
                         const void* v, int Lk, int kv_group, const unsigned char* kpm,
                         const void* wo, float* slab_out, void* stream);
/* retr_dec_self_heads_ln for the first decoder layer with the DecoderEmbeddings in the prologue:
 * x = LN(word[tok[r]] + qpos; ge, be, epse) -> xout (models/transformer_modules.py:118-127), then
 * LN1 (gamma, beta, eps) and the self sub-layer -- replaces retr_dec_embed_rows +
 * retr_dec_self_heads.  Head dim 32, at most 128 keys. */
int retr_dec_self_heads_embed(const long long* tok, const float* word, const float* ge,
                              const float* be, float epse, int R, int C, int H, const void* win,
                              const float* bin, void* kc, void* vc, int i, int Lmax,
                              const int* anc, const void* wo, float* slab, const float* gamma,
                              const float* beta, float eps, const float* qpos, float* xout,
                              void* stream);
/* Multi-row variants (beam search): rb rows x one head per block, the head's weight slices (and
 * the memory keys / values when kv_group % rb == 0) staged in LDS once per block.  Same operands
 * and results as retr_dec_self_heads_ln / retr_dec_cross_heads; C = 256, H = 8, rb in {1, 2, 4,
 * 5} (1 = the per-(row, head) kernels), R % rb == 0, at most 128 self / 256 memory keys. */
int retr_dec_self_heads_mr(const void* n, const void* npos, int R, int C, int H, const void* win,
                           const float* bin, void* kc, void* vc, int i, int Lmax, const int* anc,
                           const void* wo, float* slab, const float* xin, const float* slabs,
                           int nslab, const float* b2, const float* gamma, const float* beta,
                           float eps, const float* qpos, float* xout, int rb, void* stream);
int retr_dec_cross_heads_mr(const float* slab_in, const float* x, const float* bo_in, float* xo,
                            int R, int C, int H, const float* gamma, const float* beta, float eps,
                            const float* pos, const void* wq, const float* bq, const void* k,
                            const void* v, int Lk, int kv_group, const unsigned char* kpm,
                            const void* wo, float* slab_out, int rb, void* stream);
int retr_dec_ffn(const void* n3, int R, int C, const void* w1, const float* b1, const void* w2,
                 int F, float* slabs, void* stream);
/* bf16 decode linear for few rows (the greedy step's MLP head): y = bf16(x W^T + bias) (ReLU),
 * the same 16 x 16 tiles with K split over 4 waves; M <= 4096, K % 32 == 0, 16-byte aligned rows. */
int retr_dec_linear_bf16(const void* x, long ldx, const void* w, long ldw, const float* bias,
                         void* y, long ldy, int M, int N, int K, int relu, void* stream);
/* fp32 parity-mode decode linear for few rows: y = x W^T (+ bias) (ReLU) (+ res), exact-f32 MFMA,
 * one 16 x 16 tile per block with K split over its 4 waves (summed in wave order); M <= 64,
 * K % 16 == 0, 16-byte aligned x / w rows. */
int retr_dec_linear_f32(const float* x, long ldx, const float* w, long ldw, const float* bias,
                        float* y, long ldy, int M, int N, int K, int relu, const float* res,
                        long ldr, void* stream);
/* up to three such linears with the same M and K in one launch (the q | k | v projections) */
int retr_dec_linear3_f32(int n, const float* x0, long ldx0, const float* w0, long ldw0,
                         const float* b0, float* y0, long ldy0, int N0, int relu0,
                         const float* r0, long ldr0, const float* x1, long ldx1, const float* w1,
                         long ldw1, const float* b1, float* y1, long ldy1, int N1, int relu1,
                         const float* r1, long ldr1, const float* x2, long ldx2, const float* w2,
                         long ldw2, const float* b2, float* y2, long ldy2, int N2, int relu2,
                         const float* r2, long ldr2, int M, int K, void* stream);
/* retr_dec_ffn with its input LayerNorm in the prologue: per row x = xin + (sum_j hslab[j] + bo)
 * (slabs [nslab][R][C] in order), written to xout, FFN input = bf16(LN(x; gamma, beta, eps)) --
 * the retr_dec_rows launch between the per-head cross-attention partials and the FFN folded in. */
int retr_dec_ffn_ln(const float* xin, const float* hslab, int nslab, const float* bo,
                    const float* gamma, const float* beta, float eps, float* xout, int R, int C,
                    const void* w1, const float* b1, const void* w2, int F, float* slabs,
                    void* stream);
/* retr_dec_ffn_ln over 64 hidden units per block: slabs [F / 64][R][C] */
int retr_dec_ffn_ln64(const float* xin, const float* hslab, int nslab, const float* bo,
                      const float* gamma, const float* beta, float eps, float* xout, int R, int C,
                      const void* w1, const float* b1, const void* w2, int F, float* slabs,
                      void* stream);
/* ... over 128 hidden units per block (C = 256): slabs [F / 128][R][C] -- half the blocks that
 * each re-derive their 16 rows' LayerNorm (beam rows) */
int retr_dec_ffn_ln128(const float* xin, const float* hslab, int nslab, const float* bo,
                       const float* gamma, const float* beta, float eps, float* xout, int R,
                       int C, const void* w1, const float* b1, const void* w2, int F,
                       float* slabs, void* stream);

/* ---- fused decode step of the fp32 parity mode (csrc/decode_f32.hip, round 6): the same
 * three launches per decoder layer as the bf16 step, every value fp32 (eval_utils/decode.py:53-81
 * greedy / beam steps; models/transformer_modules.py:22-97, ConcatTransformer.py:187-214,
 * 224-243).  d_model 256, 8 heads; all row / weight operands 16-byte aligned. */
/* block (row, head): prologue x = xin + (sum_j slabs[j] + b2) (slabs [nslab][R][C]) or, with
 * tok != NULL (layer 0), x = LN_e(word[tok] + qpos); x -> xout (h = 0 blocks); LN1(x) (+qpos)
 * -> the head's q | k | v (win [3C][C], bin [3C]), k / v -> cache row r * Lmax + i (fp32
 * caches), attention over keys 0..i (anc: beam ancestry [R][Lmax] or NULL), the head's partial
 * out-projection -> slab [H][R][C] */
int retr_dec_self_f32(int R, int C, int H, const float* win, const float* bin, float* kc,
                      float* vc, int i, int Lmax, const int* anc, const float* wo, float* slab,
                      const float* xin, const float* slabs, int nslab, const float* b2,
                      const long long* tok, const float* word, const float* ge, const float* be,
                      float epse, const float* gamma, const float* beta, float eps,
                      const float* qpos, float* xout, void* stream);
/* block (row, head): x' = x + (sum_h slab_in[h] + bo_in) -> xo; LN2(x') + pos -> the head's cross
 * query (wq rows 0..C, bq), attention over Lk memory rows (r / kv_group) * Lk + j (kpm
 * [R / kv_group][Lk] or NULL), the head's partial out-projection -> slab_out [H][R][C] */
int retr_dec_cross_f32(int R, int C, int H, const float* slab_in, const float* x,
                       const float* bo_in, float* xo, const float* gamma, const float* beta,
                       float eps, const float* pos, const float* wq, const float* bq,
                       const float* k, const float* v, int Lk, int kv_group,
                       const unsigned char* kpm, const float* wo, float* slab_out, void* stream);
/* x'' = xin + (sum_j hslab[j] + bo) -> xout; FFN partials of LN3(x'') over 64 hidden units per
 * block (exact-f32 MFMA) -> slabs [F / 64][R][C] */
int retr_dec_ffn_f32(const float* xin, const float* hslab, int nslab, const float* bo,
                     const float* gamma, const float* beta, float eps, float* xout, int R, int C,
                     const float* w1, const float* b1, const float* w2, int F, float* slabs,
                     void* stream);
/* x = xin + (sum_j slabs[j] + b2) -> xout (optional); n = LN(x) (fp32) */
int retr_dec_rows_f32(const float* xin, const float* slabs, int nslab, const float* b2, int R,
                      int C, float* xout, const float* gamma, const float* beta, float eps,
                      float* n, void* stream);

#ifdef __cplusplus
}
#endif
#endif
