/*
 * pmunet_hip.h — C ABI of libpmunet_hip.so, the MI355X (gfx950) hot path of the
 * Probabilistic Multi-Planar U-Net.
 *
 * The reference (qzs634/Probabilistic-Multiplanar-Unet) has no FFI: its hot path is
 * PyTorch module code.  Each entry point below replaces the PyTorch operator(s) the
 * reference calls at the cited line (PMU/ = Probabilistic-Multiplanar-Unet/):
 *
 *   pmu_conv3x3_fwd      nn.Conv2d(3x3,pad 1)+bias, with the producer's BatchNorm2d(train/eval)
 *                        + ReLU (+MaxPool2d(2) | AvgPool2d(2,ceil) | F.pad+torch.cat) fused
 *                        into the operand load     PMU/model/unet/unet_parts.py:15-20,33,52-66
 *                                                  PMU/model/probabilistic_unet/probabilistic_unet.py:36-44
 *   pmu_conv3x3_dgrad    autograd of the above w.r.t. its input (BN-backward fused in the load)
 *   pmu_conv3x3_wgrad    autograd of the above w.r.t. its weight (split-K, deterministic)
 *   pmu_conv_first_fwd / _wgrad   the Cin<=4 first layer of UNet / prior / posterior
 *   pmu_convT2x2_fwd/_dgrad/_wgrad  nn.ConvTranspose2d(k2,s2)        unet_parts.py:52
 *   pmu_bn_*             BatchNorm2d batch statistics, running-stat update, backward coefficients
 *   pmu_maxpool2_bwd / pmu_avgpool2_bwd                              unet_parts.py:33, probabilistic_unet.py:36
 *   pmu_head1x1_fwd/_bwd, pmu_wgrad1x1   OutConv + sigmoid           unet_parts.py:70-76, unet_model.py:48-49
 *   pmu_sgd_clip         clip_grad_value_(0.1) + SGD(momentum)        PMU/train.py:65,108-110
 *   pmu_bce_* / pmu_ce_* BCELoss / CrossEntropyLoss (+ grad)          trainer/unet_trainer.py:23,30-37
 *   pmu_dice_counts      dice_coeff + argmax/one-hot                  PMU/dice_loss.py:5-12, trainer/unet_trainer.py:39-58
 *   pmu_dice_sums        dice_coeff's three sums for arbitrary tensors PMU/dice_loss.py:5-12
 *   pmu_fcomb_*          Fcomb 1x1 chain with tiled z                 probabilistic_unet.py:116-181
 *   pmu_spatial_mean(_bwd) / pmu_linear_*   AxisAlignedConvGaussian head  probabilistic_unet.py:95-108
 *   pmu_slice_view_layout / pmu_slice_max / pmu_gather_slices
 *                        MRI_Dataset pad_dimensions/sample_slice/preprocess  PMU/utils/mri_dataset.py:70-112
 *   pmu_fuse3view        eval.py 3-view volume fusion + per-class Dice PMU/eval.py:42-65,157-203
 *
 * Conventions
 *   - All tensors are device pointers, fp32, activations stored channels-last (NHWC),
 *     weights in PyTorch's native layouts ([Cout][Cin][3][3], ConvT [Cin][Cout][2][2]).
 *   - Every call is asynchronous on the given hipStream_t (passed as void*), never
 *     allocates, never synchronises, and is safe to capture in a hipGraph.
 *   - Every call returns 0 on success, PMU_ERR_ARG for an invalid argument (checked
 *     on the host before any launch), or the hipError_t of a failed launch.
 *   - Reductions are deterministic: fixed-shape partial slabs, no float atomics — except the
 *     metric counters (pmu_dice_counts, pmu_fuse3view: fp64 atomics of integer values, exact) and
 *     pmu_dice_sums (fp64 atomics; exact for the 0/1 inputs the reference feeds it).
 */
#ifndef PMUNET_HIP_H
#define PMUNET_HIP_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

#define PMU_ABI_VERSION 1

enum { PMU_OK = 0, PMU_ERR_ARG = 1001 };

/* How one conv-input source turns stored values into operand values. */
enum {
  PMU_SRC_RAW = 0,    /* value = x                                                    */
  PMU_SRC_BNRELU = 1, /* value = max(0, x*scale[c] + shift[c])        coef = [scale|shift]          */
  PMU_SRC_BNBWD = 2   /* value = dL/dz of BN+ReLU: g=x*(z*scale+shift>0);
                         scale*g + kx*(z-mean) + kc                   coef = [scale|shift|mean|kx|kc] */
};
enum { PMU_POOL_NONE = 0, PMU_POOL_MAX2 = 1, PMU_POOL_AVG2CEIL = 2 };
/* Storage type of a source's tensors (pmu_src.dtype bits; 0 = both fp32).  bf16 storage is what
 * torch.autocast(bfloat16) keeps a conv output in (config c5): the pre-BN z of the bf16 path. */
enum { PMU_DT_X_BF16 = 1, PMU_DT_Z_BF16 = 2 };

typedef struct pmu_src {
  const float* x;    /* NHWC [N][H][W][C]: raw values, pre-BN z, or upstream gradient */
  const float* z;    /* PMU_SRC_BNBWD: pre-BN z, same shape as x; else NULL          */
  const float* coef; /* per-channel coefficient block (see modes)                     */
  int mode, pool;
  int C, H, W;       /* stored tensor dims                                            */
  int off_h, off_w;  /* top/left offset of the (pooled) source inside the frame (F.pad) */
  int dtype;         /* PMU_DT_* bits: x / z stored as bf16 (read as fp32 exactly).  Only the
                        materialising and streaming calls take bf16 sources (pmu_frame_to_bf16,
                        pmu_frame_to_f32, pmu_head1x1_fwd, pmu_wgrad1x1); the others refuse them */
} pmu_src;

/* A conv operand: one frame of N x H x W pixels whose channels are the concatenation
 * of up to two sources (torch.cat([skip, up], 1) of unet_parts.py:66). */
typedef struct pmu_frame {
  pmu_src src[2];
  int nsrc;
  int N, H, W;
} pmu_frame;

/* ---- 3x3 convolution: direct-sum weight gradient (channel counts the Winograd weight gradient
 * does not take: Cout % 32 or Cin % 64 != 0) ------------------------------------------------ */
/* dw[Cout][Cin][3][3] = dL/dw; ws must hold pmu_conv3x3_wgrad_ws() bytes. */
size_t pmu_conv3x3_wgrad_ws(int N, int H, int W, int Cin, int Cout);
int pmu_conv3x3_wgrad(const pmu_frame* dz, const pmu_frame* act, int Cout, float* dw,
                      float* ws, size_t ws_bytes, void* stream);

/* ---- fp32 Winograd F(2x2,3x3) variant (the c2 fp32 path) ------------------------------
 * The same operators as pmu_conv3x3_fwd / _dgrad in fp32, computed as 16 per-component GEMMs of
 * transformed operands (B^T d B) and weights (G g G^T), output A^T M A: fp32 rounding differs from
 * the direct sum by ~1e-6 relative.  Weights pre-transformed by pmu_conv3x3_pack_wino ([32 output
 * rows][16 channels] blocks); part rows = pmu_conv3x3_tiles_wino() (16 x 16 pixel tiles); tee as
 * pmu_conv3x3_fwd / _dgrad. */
size_t pmu_conv3x3_packed_size_wino(int Cout, int Cin, int dgrad);
int pmu_conv3x3_pack_wino(const float* w, int Cout, int Cin, int dgrad, float* wp, void* stream);
int pmu_conv3x3_tiles_wino(int N, int H, int W);
int pmu_conv3x3_fwd_wino(const pmu_frame* in, const float* wp, const float* bias, int Cout, float* z,
                         float* part, float* tee, void* stream);
int pmu_conv3x3_dgrad_wino(const pmu_frame* dz, const float* wp, int Cin, int Csplit, float* dx0, float* dx1,
                           float* tee, void* stream);
/* The same F(2x2,3x3) operators on a materialised operand in 1024-thread workgroups (16 waves, four per
 * SIMD; 64 output channels x 16 x 16 pixels per block; waves split the 16 components in halves).
 * C % 8 == 0; weights by pmu_conv3x3_pack_wino2h ([64 output rows][8 channels][16 components]);
 * part rows = pmu_conv3x3_tiles_wino2h() (16 x 16 pixel blocks). */
size_t pmu_conv3x3_packed_size_wino2h(int Cout, int Cin, int dgrad);
int pmu_conv3x3_pack_wino2h(const float* w, int Cout, int Cin, int dgrad, float* wp, void* stream);
int pmu_conv3x3_tiles_wino2h(int N, int H, int W);
int pmu_conv3x3_fwd_wino2h(const float* xt, int Cin, int N, int H, int W, const float* wp, const float* bias,
                           int Cout, float* z, float* part, void* stream);
int pmu_conv3x3_dgrad_wino2h(const float* dzt, int Cout, int N, int H, int W, const float* wp, int Cin,
                             int Csplit, float* dx0, float* dx1, void* stream);
/* The input gradient fused with the BatchNorm+ReLU backward reduction of the layer that produced this
 * conv's operand (dx is that layer's da, no concat split): part[pmu_conv3x3_tiles_wino2h rows][2][Cin]
 * = (sum g, sum g*xhat), g = dx * (z*coef[c]+coef[Cin+c] > 0), xhat = (z-mean)*invstd — the sums
 * pmu_bn_bwd_reduce(dx, z, ...) computes, without reading dx back (PMU/model/unet/unet_parts.py:16-17). */
int pmu_conv3x3_dgrad_wino2h_bnr(const float* dzt, int Cout, int N, int H, int W, const float* wp, int Cin,
                                 float* dx, const float* z, const float* coef, const float* mean,
                                 const float* invstd, float* part, void* stream);
/* ---- fp32 Winograd F(4x4,3x3) on a materialised operand (images >= 32 x 32: the c2 fp32 default) --
 * Replaces the same nn.Conv2d forward / input gradient (PMU/model/unet/unet_parts.py:15,18; autograd of
 * PMU/model/unet/unet_model.py:31-54) as pmu_conv3x3_*_wino_raw: 36 per-component GEMMs of
 * B^T d B (6x6 patches) and G g G^T, output A^T M A per 4x4 tile; fp32 rounding differs from the direct
 * sum by a few 1e-6 relative.  xt / dzt [N][H][W][C] fp32 with C % 8 == 0; weights pre-transformed by
 * pmu_conv3x3_pack_wino4 ([32 output rows][8 channels][36 components] blocks); part rows =
 * pmu_conv3x3_tiles_wino4() (32 x 32 pixel blocks). */
size_t pmu_conv3x3_packed_size_wino4(int Cout, int Cin, int dgrad);
int pmu_conv3x3_pack_wino4(const float* w, int Cout, int Cin, int dgrad, float* wp, void* stream);
int pmu_conv3x3_tiles_wino4(int N, int H, int W);
int pmu_conv3x3_dgrad_wino4(const float* dzt, int Cout, int N, int H, int W, const float* wp, int Cin,
                            int Csplit, float* dx0, float* dx1, void* stream);
/* as pmu_conv3x3_dgrad_wino2h_bnr (part rows = pmu_conv3x3_tiles_wino4) */
int pmu_conv3x3_dgrad_wino4_bnr(const float* dzt, int Cout, int N, int H, int W, const float* wp, int Cin,
                                float* dx, const float* z, const float* coef, const float* mean,
                                const float* invstd, float* part, void* stream);
/* dw[Cout][Cin][3][3] from the teed operands dzt [N][H][W][Cout] and xt [N][H][W][Cin] (fp32), by
 * Winograd F(2x2,3x3): dw = G^T [sum over 2x2 tiles of (A dY A^T) .* (B^T X B)] G.  Cout % 32 == 0,
 * Cin % 64 == 0 (pmu_conv3x3_wgrad_ws_wino returns 0 otherwise); ws must hold that many bytes. */
size_t pmu_conv3x3_wgrad_ws_wino(int N, int H, int W, int Cin, int Cout);
int pmu_conv3x3_wgrad_wino(const float* dzt, const float* xt, int N, int H, int W, int Cout, int Cin,
                           float* dw, float* ws, size_t ws_bytes, void* stream);

/* ---- bf16-MFMA variants (config c5, BASELINE.json configs[4]: "... bf16") --------------
 * torch.autocast(bfloat16) arithmetic for the same operators: the operand (after the fused fp32
 * BN/ReLU/pool/concat transform) and the weights are rounded to bf16 (RNE), products are summed in
 * fp32 on v_mfma_f32_32x32x16_bf16, and every output (z, BN partials, dx, dw) stays fp32, so all
 * the fp32 BN / pool / head / optimizer kernels above consume them unchanged.
 * Weights are always pre-packed (bf16, [row block of 64][chunk of 16][tap][64][16]). */
size_t pmu_conv3x3_packed_size_bf16(int Cout, int Cin, int dgrad);
int pmu_conv3x3_pack_bf16(const float* w, int Cout, int Cin, int dgrad, unsigned short* wp, void* stream);
/* rows of the fused-staging convs' BN partial sums (256-pixel tiles) */
int pmu_conv3x3_tiles(int N, int H, int W);
/* z = conv3x3(frame) + bias / dx as the direct-sum fp32 conv of pmu_hip_experiments.h (part rows =
 * pmu_conv3x3_tiles()).  tee (nullable):
 * receives the bf16 operand the kernel multiplied, [N][H][W][pad8(K channels)] as pmu_frame_to_bf16
 * would write it (padding channels untouched) — the input of pmu_conv3x3_wgrad_bf16, for free. */
int pmu_conv3x3_fwd_bf16(const pmu_frame* in, const unsigned short* wp, const float* bias, int Cout,
                         float* z, float* part, unsigned short* tee, void* stream);
int pmu_conv3x3_dgrad_bf16(const pmu_frame* dz, const unsigned short* wp, int Cin, int Csplit,
                           float* dx0, float* dx1, unsigned short* tee, void* stream);

/* The bf16-mode main path: a conv whose operand was materialised once by pmu_frame_to_bf16
 * (xt / dzt: [N][H][W][Cp] bf16, Cp % 8 == 0), weights packed per 64 output rows x 32 channels
 * (pmu_conv3x3_pack_raw).  Outputs as pmu_conv3x3_fwd / _dgrad; dgrad needs Csplit % 32 == 0 when
 * Csplit < Cin; N*H*W*Cp < 2^31. */
size_t pmu_conv3x3_packed_size_raw(int Cout, int Cin, int dgrad);
int pmu_conv3x3_pack_raw(const float* w, int Cout, int Cin, int dgrad, unsigned short* wp, void* stream);
int pmu_conv3x3_fwd_raw(const unsigned short* xt, int Cp, int N, int H, int W, const unsigned short* wp,
                        const float* bias, int Cout, float* z, float* part, void* stream);
/* rows of pmu_conv3x3_fwd_raw's part[tile][2][Cout] (its pixel tiles are 256 or 512 pixels) */
int pmu_conv3x3_tiles_raw(int N, int H, int W, int Cout);
int pmu_conv3x3_dgrad_raw(const unsigned short* dzt, int Cp, int N, int H, int W, const unsigned short* wp,
                          int Cin, int Csplit, float* dx0, float* dx1, void* stream);
/* The same convolutions with both operands staged by LDS-DMA (512-thread workgroups, 512- or
 * 1024-pixel tiles, 16-channel chunks), for maps at least 32 wide: Cp % 16 == 0, Csplit == Cin or
 * Csplit % 32 == 0 (pmu_conv3x3_dma_ok).  Weights packed by pmu_conv3x3_pack_dma (its own layout);
 * part rows = pmu_conv3x3_tiles_dma().  Launches whose operand reaches 4 GiB are split over images. */
int pmu_conv3x3_dma_ok(int H, int W, int Cp, int NOUT, int split);
int pmu_conv3x3_tiles_dma(int N, int H, int W, int Cout, int Cp);
size_t pmu_conv3x3_packed_size_dma(int Cout, int Cin, int dgrad);
int pmu_conv3x3_pack_dma(const float* w, int Cout, int Cin, int dgrad, unsigned short* wp, void* stream);
int pmu_conv3x3_fwd_dma(const unsigned short* xt, int Cp, int N, int H, int W, const unsigned short* wp,
                        const float* bias, int Cout, float* z, float* part, void* stream);
int pmu_conv3x3_dgrad_dma(const unsigned short* dzt, int Cp, int N, int H, int W, const unsigned short* wp,
                          int Cin, int Csplit, float* dx0, float* dx1, void* stream);
/* the same with a concat split (Csplit < Cin, (Cin - Csplit) % 8 == 0) that also writes dx1b, a bf16
 * (RNE) copy of dx1 [N][H][W][Cin-Csplit]: the up-sampled part's gradient is the transposed conv's
 * bf16 operand (unet_parts.py:52,66 under autocast) — no separate pmu_frame_to_bf16 pass over dx1 */
int pmu_conv3x3_dgrad_dma_x1b(const unsigned short* dzt, int Cp, int N, int H, int W, const unsigned short* wp,
                              int Cin, int Csplit, float* dx0, float* dx1, unsigned short* dx1b, void* stream);
/* the same without the fp32 dx1 (only dx1b), plus part[tile][0][Cin] = per-tile column sums of dx
 * (part[tile][1][*] = 0; tiles = pmu_conv3x3_tiles_dma(N, H, W, Cin, Cp)): the transposed conv's bias
 * gradient (unet_parts.py:52 backward) is the sum over tiles of channels [Csplit, Cin)
 * (pmu_convT2x2_dbias_rows). */
int pmu_conv3x3_dgrad_dma_x1b_sum(const unsigned short* dzt, int Cp, int N, int H, int W, const unsigned short* wp,
                                  int Cin, int Csplit, float* dx0, unsigned short* dx1b, float* part, void* stream);
/* dbias[c] = sum over r < R of part[r * ld + c], c < Cout, in a fixed order; ws holds
 * pmu_convT2x2_dbias_rows_ws(Cout) bytes. */
size_t pmu_convT2x2_dbias_rows_ws(int Cout);
int pmu_convT2x2_dbias_rows(const float* part, int R, long long ld, int Cout, float* dbias, float* ws, void* stream);
/* as pmu_conv3x3_dgrad_wino2h_bnr (part rows = pmu_conv3x3_tiles_dma(N, H, W, Cin, Cp)) */
int pmu_conv3x3_dgrad_dma_bnr(const unsigned short* dzt, int Cp, int N, int H, int W, const unsigned short* wp,
                              int Cin, float* dx, const float* z, const float* coef, const float* mean,
                              const float* invstd, float* part, void* stream);
/* bf16 activation gradients (config c5, unet_parts.py:15,18 backward under torch.autocast(bfloat16),
 * whose conv backward returns dx in bf16): the four input gradients above with dx / dx0 stored as
 * bf16 (RNE) and every other output (dx1 values, dx1b, column sums, BN-backward partials) formed from
 * the rounded values.  Cin % 8 == 0, Csplit % 8 == 0.  Consumers: pmu_frame_to_bf16 (BN-backward
 * frames with a bf16 da), pmu_maxpool2_bwd_bnr_dxb, pmu_bn_bwd_reduce_dxb, pmu_conv_first_wgrad. */
int pmu_conv3x3_dgrad_dma_dxb(const unsigned short* dzt, int Cp, int N, int H, int W, const unsigned short* wp,
                              int Cin, int Csplit, unsigned short* dx0, float* dx1, void* stream);
int pmu_conv3x3_dgrad_dma_x1b_dxb(const unsigned short* dzt, int Cp, int N, int H, int W, const unsigned short* wp,
                                  int Cin, int Csplit, unsigned short* dx0, float* dx1, unsigned short* dx1b,
                                  void* stream);
int pmu_conv3x3_dgrad_dma_x1b_sum_dxb(const unsigned short* dzt, int Cp, int N, int H, int W,
                                      const unsigned short* wp, int Cin, int Csplit, unsigned short* dx0,
                                      unsigned short* dx1b, float* part, void* stream);
int pmu_conv3x3_dgrad_dma_bnr_dxb(const unsigned short* dzt, int Cp, int N, int H, int W, const unsigned short* wp,
                                  int Cin, unsigned short* dx, const float* z, const float* coef, const float* mean,
                                  const float* invstd, float* part, void* stream);
/* The bf16 operand of a frame, materialised: out[N][H][W][Cpad] = bf16(frame value) (channels
 * >= C zero; Cpad % 4 == 0) — the BN+ReLU(+pool)(+concat) activation or the BN+ReLU backward dz
 * that pmu_conv3x3_wgrad_bf16 multiplies. */
int pmu_frame_to_bf16(const pmu_frame* f, int Cpad, unsigned short* out, void* stream);
/* out[N][H][W][C] = the frame's fp32 operand values (e.g. MaxPool2d of BN+ReLU, unet_parts.py:33). */
int pmu_frame_to_f32(const pmu_frame* f, float* out, void* stream);
/* the frame into the first channels of a wider NHWC tensor (output pixel stride ldo elements): the
 * skip half of an Up block's concat operand, whose other half pmu_convT2x2_fwd_ld /
 * pmu_convT2x2_fwd_dma_ldb write in place (unet_parts.py:66).  Channel counts of 4 (fp32) / 8 (bf16). */
int pmu_frame_to_f32_ld(const pmu_frame* f, float* out, int ldo, void* stream);
int pmu_frame_to_bf16_ld(const pmu_frame* f, int Cpad, unsigned short* out, int ldo, void* stream);
/* One pass over a level's BN+ReLU activation for both of its consumers (unet_parts.py:33 MaxPool2d
 * and :66 torch.cat): f is the max-pooled frame (one fp32 BNRELU source, even source dims, C a
 * power-of-two multiple of 8 up to 2048; pmu_frame_pool_skip_ok); out[N][H][W][C] receives the
 * pooled operand and skip (pixel stride ldo_skip >= C, a multiple of 8) the unpooled activation in
 * its first C channels.  Bit-identical to pmu_frame_to_* + pmu_frame_to_*_ld. */
int pmu_frame_pool_skip_ok(const pmu_frame* f);
int pmu_frame_to_bf16_pool_skip(const pmu_frame* f, unsigned short* out, unsigned short* skip, int ldo_skip,
                                void* stream);
int pmu_frame_to_f32_pool_skip(const pmu_frame* f, float* out, float* skip, int ldo_skip, void* stream);
/* dw[Cout][Cin][3][3] from dzt [N][H][W][pad8(Cout)] and xt [N][H][W][pad8(Cin)] (bf16, pad8(c) =
 * c rounded up to a multiple of 8); ws must hold pmu_conv3x3_wgrad_ws_bf16() bytes. */
size_t pmu_conv3x3_wgrad_ws_bf16(int N, int H, int W, int Cin, int Cout);
int pmu_conv3x3_wgrad_bf16(const unsigned short* dzt, const unsigned short* xt, int N, int H, int W,
                           int Cout, int Cin, float* dw, float* ws, size_t ws_bytes, void* stream);
/* The same weight gradient with both operands staged by LDS-DMA (csrc/wgrad3x3_bf16_dma.hip): a wave
 * owns a 32-co x 32-ci fragment pair and all nine taps, walks 16-pixel-wide image strips row by row
 * and keeps the three activation rows of a step in registers (one new row per step).  Maps at least
 * 16 wide (pmu_conv3x3_wgrad_dma_ok); ws holds pmu_conv3x3_wgrad_ws_bf16_dma() bytes. */
int pmu_conv3x3_wgrad_dma_ok(int N, int H, int W, int Cin, int Cout);
size_t pmu_conv3x3_wgrad_ws_bf16_dma(int N, int H, int W, int Cin, int Cout);
int pmu_conv3x3_wgrad_bf16_dma(const unsigned short* dzt, const unsigned short* xt, int N, int H, int W,
                               int Cout, int Cin, float* dw, float* ws, size_t ws_bytes, void* stream);

/* Weight gradient from materialised bf16 operands: xt [N][H][W][pad8(Cin)] (the convT input after BN+ReLU)
 * and dut [N][Hd][Wd][pad8(Cout)] (du); dbias (nullable) sums the fp32 du over the output region. */
/* The same forward / input gradient with both GEMM operands staged by LDS-DMA from materialised bf16
 * tensors: xt = the BN+ReLU operand [N][H][W][Cip] (pmu_frame_to_bf16), dut = du [N][Hd][Wd][Cop];
 * weights packed by pmu_convT2x2_pack_dma (2 * 4*Cin*Cout bytes).  Cin % 32 == 0, Cout % 32 == 0 and
 * the GEMM column count (forward 4*Cout, dgrad Cin) % 128 == 0 (pmu_convT2x2_dma_ok). */
int pmu_convT2x2_dma_ok(int Cin, int Cout, int dgrad);
size_t pmu_convT2x2_packed_size_dma(int Cin, int Cout);
int pmu_convT2x2_pack_dma(const float* w, int Cin, int Cout, int dgrad, unsigned short* wp, void* stream);
int pmu_convT2x2_fwd_dma(const unsigned short* xt, int Cip, int N, int H, int W, const unsigned short* wp,
                         const float* bias, int Cin, int Cout, float* u, void* stream);
/* the same written as bf16 into channels [0, Cout) of a wider NHWC bf16 tensor (pixel stride ldo):
 * the up-sampled half of the Up block's bf16 concat operand — no fp32 u (unet_parts.py:52,66) */
int pmu_convT2x2_fwd_dma_ldb(const unsigned short* xt, int Cip, int N, int H, int W, const unsigned short* wp,
                             const float* bias, int Cin, int Cout, unsigned short* ub, int ldo, void* stream);
int pmu_convT2x2_dgrad_dma(const unsigned short* dut, int Cop, int Hd, int Wd, int off_h, int off_w,
                           const unsigned short* wp, int N, int H, int W, int Cin, int Cout, float* dx,
                           void* stream);
/* the same with dx stored as bf16 (RNE; autocast's dtype for ConvTranspose2d's input gradient,
 * unet_parts.py:52 backward): its consumer's BN backward reads it (pmu_bn_bwd_reduce_dxb and the
 * BN-backward frames) */
int pmu_convT2x2_dgrad_dma_dxb(const unsigned short* dut, int Cop, int Hd, int Wd, int off_h, int off_w,
                               const unsigned short* wp, int N, int H, int W, int Cin, int Cout, unsigned short* dx,
                               void* stream);
size_t pmu_convT2x2_wgrad_ws_bf16(int N, int H, int W, int Cin, int Cout);
int pmu_convT2x2_wgrad_bf16(const unsigned short* xt, const unsigned short* dut, const float* du, int N, int H,
                            int W, int Hd, int Wd, int off_h, int off_w, int Cin, int Cout, float* dw,
                            float* dbias, float* ws, size_t ws_bytes, void* stream);

/* ---- first layer (Cin <= 4, planes given NCHW-style, one pointer per channel) ------ */
int pmu_conv_first_fwd(const float* const* planes, int Cin, int N, int H, int W,
                       const float* w, const float* bias, int Cout, float* z, float* part,
                       void* stream);
int pmu_conv_first_tiles(int N, int H, int W);
size_t pmu_conv_first_wgrad_ws(int N, int H, int W, int Cin, int Cout);
/* dz: one BN-backward (or raw) source; its da may be bf16-stored (a *_dxb input gradient's dx) */
int pmu_conv_first_wgrad(const pmu_frame* dz, const float* const* planes, int Cin, int Cout,
                         float* dw, float* ws, size_t ws_bytes, void* stream);

/* ---- BatchNorm2d ------------------------------------------------------------------- */
/* Column reduction of fp32 partials part[R][Wd] into fp64 partials out[G][Wd]. */
int pmu_colsum_f64(const float* part, int R, int Wd, double* out, int G, void* stream);
int pmu_colsum_groups(int R);
/* From fp64 sums acc[G][2][C] (sum, sumsq) over count elements: mean, invstd, coef=[scale|shift];
 * update running stats (unbiased var, momentum) when running_mean != NULL, and add 1 to
 * *num_batches_tracked when it is non-NULL (BatchNorm2d's counter, PMU/model/unet/unet_parts.py:16,19:
 * one launch instead of a separate increment per layer). */
int pmu_bn_fwd_finalize(const double* acc, int G, int C, double count, const float* gamma,
                        const float* beta, float eps, float momentum, float* running_mean,
                        float* running_var, long long* num_batches_tracked, float* mean, float* invstd,
                        float* coef, void* stream);
/* Eval mode: coef from running stats. */
int pmu_bn_eval_coef(const float* running_mean, const float* running_var, const float* gamma,
                     const float* beta, float eps, int C, float* coef, void* stream);
/* BN+ReLU backward reduction over da (NHWC) and z: part[tile][2][C] = (sum g, sum g*xhat). */
int pmu_bn_bwd_reduce(const float* da, const float* z, const float* coef, const float* mean,
                      const float* invstd, int P, int C, float* part, void* stream);
/* the same with da stored as bf16 (a *_dxb input gradient's dx); C % 4 == 0 */
int pmu_bn_bwd_reduce_dxb(const unsigned short* da, const float* z, const float* coef, const float* mean,
                          const float* invstd, int P, int C, float* part, void* stream);
int pmu_bn_bwd_tiles(int P, int C);
/* From acc[G][2][C]: dgamma, dbeta, dbias(conv bias feeding BN) and the BNBWD coef block
 * [scale|shift|mean|kx|kc]. */
int pmu_bn_bwd_finalize(const double* acc, int G, int C, double count, const float* gamma,
                        const float* coef, const float* mean, const float* invstd, float* dgamma,
                        float* dbeta, float* dbias, float* bcoef, void* stream);

/* out[P][C] = max(0, z*scale+shift) (NHWC), coef = [scale|shift]; any C (float4 path when C % 4 == 0). */
int pmu_bnrelu_apply(const float* z, const float* coef, long long P, int C, float* out, void* stream);

/* ---- pooling backward ------------------------------------------------------------ */
/* dx[N][H][W][C] += dpool routed to the first max (row-major) of each 2x2 window of
 * relu(z*scale+shift), or of z itself when coef is NULL (a standalone Down block's raw input).
 * accumulate=0 overwrites dx (zeros outside windows). */
int pmu_maxpool2_bwd(const float* dpool, const float* z, const float* coef, int N, int H, int W,
                     int C, float* dx, int accumulate, void* stream);
/* pmu_maxpool2_bwd (BN+ReLU coef, C % 4 == 0) fused with the BatchNorm+ReLU backward reduction of
 * the pooled layer over the resulting dx (= that layer's da; replaces pmu_bn_bwd_reduce for it):
 * part[pmu_maxpool2_bwd_bnr_tiles rows][2][C] = (sum g, sum g*xhat), g = dx*(z*scale+shift > 0),
 * xhat = (z-mean)*invstd.  MaxPool2d(2) backward, unet_parts.py:33; BN backward, unet_parts.py:16,19. */
int pmu_maxpool2_bwd_bnr_tiles(int N, int H, int W, int C);
int pmu_maxpool2_bwd_bnr(const float* dpool, const float* z, const float* coef, const float* mean,
                         const float* invstd, int N, int H, int W, int C, float* dx, int accumulate,
                         float* part, void* stream);
/* the same with dpool and the skip gradient stored as bf16 (the *_dxb input gradients' dx; skip
 * nullable = no accumulation): dx (fp32, a separate tensor) = skip + routed dpool, summed in fp32 as
 * autograd accumulates the skip activation's two gradients (unet_parts.py:33,66) */
int pmu_maxpool2_bwd_bnr_dxb(const unsigned short* dpool, const unsigned short* skip, const float* z,
                             const float* coef, const float* mean, const float* invstd, int N, int H, int W, int C,
                             float* dx, float* part, void* stream);
/* The pooled layer's da = skip + routed dpool kept in registers instead of stored (config c5's skip
 * levels): _stats_dxb forms only the partial sums above (bit-equal part); _bnbwd_dxb, given that
 * layer's BN-backward coefficients (pmu_bn_bwd_finalize's bcoef) and its forward coef (the routing's
 * argmax), writes dz = BN+ReLU backward of that da as the bf16 operand [N][H][W][ldo] of its input and
 * weight gradients — bit-equal to pmu_frame_to_bf16 of Src(da, BNBWD) over the stored da.  ldo == C;
 * C / 4 divides 256 or is a multiple of it. */
int pmu_maxpool2_bwd_bnr_stats_dxb(const unsigned short* dpool, const unsigned short* skip, const float* z,
                                   const float* coef, const float* mean, const float* invstd, int N, int H, int W,
                                   int C, float* part, void* stream);
int pmu_maxpool2_bwd_bnbwd_dxb(const unsigned short* dpool, const unsigned short* skip, const float* z,
                               const float* coef, const float* bcoef, int N, int H, int W, int C, int ldo,
                               unsigned short* dz, void* stream);
/* The same for fp32 dpool / skip gradients (config c2) with an fp32 dz: bit-equal to pmu_maxpool2_bwd_bnr
 * accumulating into skip and to pmu_frame_to_f32 of Src(that da, BNBWD, bcoef, z). */
int pmu_maxpool2_bwd_bnr_stats(const float* dpool, const float* skip, const float* z, const float* coef,
                               const float* mean, const float* invstd, int N, int H, int W, int C, float* part,
                               void* stream);
int pmu_maxpool2_bwd_bnbwd(const float* dpool, const float* skip, const float* z, const float* coef,
                           const float* bcoef, int N, int H, int W, int C, int ldo, float* dz, void* stream);
/* AvgPool2d(2,2,ceil_mode=True) backward: dx = dpool/count(window), overwrite. */
int pmu_avgpool2_bwd(const float* dpool, int N, int H, int W, int C, float* dx, void* stream);
/* The same (bit-equal dx, here da: N x H x W x C at the pooled layer's resolution) fused with the BN+ReLU
 * backward partial sums of the layer whose activation was pooled (probabilistic_unet.py:36 AvgPool2d,
 * :30-32 BN+ReLU): part[pmu_bn_bwd_tiles(N*H*W, C) rows][2][C] as pmu_bn_bwd_reduce forms them from
 * (da, z).  C % 4 == 0. */
int pmu_avgpool2_bwd_bnr(const float* dpool, const float* z, const float* coef, const float* mean,
                         const float* invstd, int N, int H, int W, int C, float* da, float* part, void* stream);

/* ---- ConvTranspose2d(k=2, s=2) ---------------------------------------------------- */
/* Optional packed weights (wp, pmu_convT2x2_packed_size bytes): k-contiguous B operands for the
 * pipelined GEMMs (dgrad=0: [ab][co][ci] for the forward, dgrad=1: [ci][ab][co] for dgrad). */
size_t pmu_convT2x2_packed_size(int Cin, int Cout);
int pmu_convT2x2_pack(const float* w, int Cin, int Cout, int dgrad, float* wp, void* stream);
/* u[N][2H][2W][Cout] = convT(act(frame)) + bias, frame is N x H x W x Cin.  wp (nullable) = packed
 * forward weights; used when the frame is one unpooled BN+ReLU source and Cin%16 == Cout%32 == 0. */
int pmu_convT2x2_fwd(const pmu_frame* in, const float* w, const float* wp, const float* bias, int Cout,
                     float* u, void* stream);
/* the same into channels [0, Cout) of a wider NHWC tensor (pixel stride ldo floats), the up-sampled
 * half of the Up block's fp32 concat operand; pipelined path only (wp given, pmu_convT2x2_fwd_ld_ok) */
int pmu_convT2x2_fwd_ld_ok(const pmu_frame* in, int Cout);
int pmu_convT2x2_fwd_ld(const pmu_frame* in, const float* w, const float* wp, const float* bias, int Cout,
                        float* u, int ldo, void* stream);
/* dx[N][H][W][Cin] from du (NHWC [N][Hd][Wd][Cout], convT output placed at (off_h,off_w)). */
int pmu_convT2x2_dgrad(const float* du, int Hd, int Wd, int off_h, int off_w, const float* w,
                       const float* wp, int N, int H, int W, int Cin, int Cout, float* dx, void* stream);
size_t pmu_convT2x2_wgrad_ws(int N, int H, int W, int Cin, int Cout);
int pmu_convT2x2_wgrad(const float* du, int Hd, int Wd, int off_h, int off_w,
                       const pmu_frame* act, int Cout, float* dw, float* dbias, float* ws,
                       size_t ws_bytes, void* stream);

/* ---- 1x1 head (OutConv) -------------------------------------------------------------- */
/* y[N][K][H][W] (NCHW) = w[K][C] . act(frame) + b; sigmoid applied when do_sigmoid. */
int pmu_head1x1_fwd(const pmu_frame* in, const float* w, const float* b, int K, int do_sigmoid,
                    float* y, void* stream);
/* dl = dy * s*(1-s) (do_sigmoid) or dy; da[N][H][W][C] = w^T dl (NHWC); dl written (NCHW). */
int pmu_head1x1_bwd(const float* dy, const float* y, int do_sigmoid, const float* w, int K, int C,
                    int N, int H, int W, float* dl, float* da, void* stream);
/* pmu_head1x1_bwd fused with the BatchNorm+ReLU backward reduction of the layer feeding the head
 * (da is its gradient; replaces pmu_bn_bwd_reduce for it): part[pmu_head1x1_bwd_tiles rows][2][C]
 * as pmu_maxpool2_bwd_bnr.  With dw non-NULL the same pass also forms the head's weight gradient
 * (pmu_wgrad1x1's dw[K][C] and db[K] from act = relu(z*scale+shift); ws of pmu_wgrad1x1_ws bytes) and
 * dl is not written (may be NULL).  Shapes: pmu_head1x1_bwd_bnr_ok (C = 4q, q a power of two <= 64).
 * OutConv backward, unet_parts.py:70-76; BN backward of the last DoubleConv, unet_parts.py:19. */
int pmu_head1x1_bwd_bnr_ok(int N, int H, int W, int C);
int pmu_head1x1_bwd_tiles(int N, int H, int W);
int pmu_head1x1_bwd_bnr(const float* dy, const float* y, int do_sigmoid, const float* w, int K, int C,
                        int N, int H, int W, float* dl, float* da, const float* z, const float* coef,
                        const float* mean, const float* invstd, float* part, float* dw, float* db, float* ws,
                        size_t ws_bytes, void* stream);
/* With dw non-NULL, da may be NULL too (not stored): pmu_head1x1_bwd_dz then writes the last layer's
 * dz straight from dy — da = sum_k g_k w[k] formed as the pass above forms it — as that layer's
 * BN+ReLU backward over bcoef (pmu_bn_bwd_finalize's 5 C coefficients): bf16 bits (out_bf16, C % 8
 * == 0; the bf16 convs' operand) or fp32, [N][H][W][C]; bit-equal to pmu_frame_to_bf16 / _f32 of
 * Src(stored da, BNBWD, bcoef, z).  Shapes as pmu_head1x1_bwd_bnr_ok, K <= 8. */
int pmu_head1x1_bwd_dz(const float* dy, const float* y, int do_sigmoid, const float* w, int K, int C,
                       int N, int H, int W, const float* z, const float* bcoef, int out_bf16, void* dz,
                       void* stream);
size_t pmu_wgrad1x1_ws(int P, int K, int C);
/* dw[K][C] = sum_p dl[p][k] act[p][c], db[k] = sum_p dl[p][k]; dl NCHW [N][K][H][W]. */
int pmu_wgrad1x1(const float* dl, const pmu_frame* act, int K, float* dw, float* db, float* ws,
                 size_t ws_bytes, void* stream);

/* ---- optimizer --------------------------------------------------------------------- */
/* Multi-tensor fused clip_grad_value_ + SGD(momentum, dampening 0, no nesterov):
 *   g = clamp(gscale*g, -clip, clip) (clip <= 0: no clipping); buf = momentum*buf + g; p -= lr*buf.
 * (buf starting at zero reproduces torch's first-step buf = g; gscale = 1/world_size turns an
 * all-reduced gradient sum into the data-parallel mean before clipping.)
 * ptrs: device array of 3*ntensors pointers (p, g, buf); chunks: device array, one block each. */
typedef struct pmu_sgd_chunk {
  int tensor; /* index into ptrs/3 */
  int len;    /* elements in this chunk (any; 16-B aligned chunks of 16384 stream float4) */
  long long start;
} pmu_sgd_chunk;
int pmu_sgd_clip(const pmu_sgd_chunk* chunks, int nchunks, void* const* ptrs, float gscale, float lr,
                 float momentum, float clip, void* stream);

/* ---- losses (row a6) -------------------------------------------------------------------
 * nn.BCELoss on the sigmoid head / nn.CrossEntropyLoss on the logits (PMU/trainer/unet_trainer.py:
 * 23,30-37) and the summed CE of ProbabilisticUnet.elbo (probabilistic_unet.py:286-304).
 * reduction: 0 none (loss[i] per element / pixel), 1 mean, 2 sum (loss[0]).  Forward partial sums
 * are fp64 in a fixed order (deterministic); ws: pmu_loss_ws(n) bytes (n = elements / pixels).
 * count_out (optional, device float): the mean's denominator (n for BCE, non-ignored pixels for
 * CE), read by pmu_ce_bwd for reduction 1.  Backward: gout is the upstream gradient on the device
 * (a scalar for mean/sum, per element for none); BCE dy = g (y - t) / max(y (1 - y), 1e-12) (torch's
 * formula; mean divides g by n); CE dx = g (softmax - onehot(t)), ignore_index pixels 0.
 * Logits x NCHW [N][K][HW], targets int64 [N][HW]. */
size_t pmu_loss_ws(long long n);
int pmu_bce_fwd(const float* y, const float* t, long long n, int reduction, float* loss, double* ws,
                float* count_out, void* stream);
int pmu_bce_bwd(const float* y, const float* t, long long n, int reduction, const float* gout, float* dy,
                void* stream);
int pmu_ce_fwd(const float* x, const long long* tgt, int N, int K, long long HW, int reduction,
               long long ignore_index, float* loss, double* ws, float* count_out, void* stream);
int pmu_ce_bwd(const float* x, const long long* tgt, int N, int K, long long HW, int reduction,
               long long ignore_index, const float* gout, const float* count, float* dx, void* stream);

/* ---- metrics ------------------------------------------------------------------------- */
/* counts[k][3] = (sum pred_k*t_k, sum pred_k, sum t_k) for k < K, exact (integer-valued fp64).
 * K==1: pred = (y > 0.5), t = mask.  K>1: pred = onehot(first argmax_c softmax(y)), t = (mask == k).
 * y NCHW [N][K][H][W], mask [N][H][W]. */
int pmu_dice_counts(const float* y, const float* mask, int N, int K, int H, int W,
                    double* counts, void* stream);
/* pmu_dice_counts of S predictions y[S][N][K][H][W] against one mask in one launch: counts[S][K][3],
 * the same integers as S pmu_dice_counts calls (the eval over several prior samples,
 * PMU/trainer/probunet_trainer.py:41-60). */
int pmu_dice_counts_many(const float* y, const float* mask, int S, int N, int K, int H, int W, double* counts,
                         void* stream);

/* (sum a*b, sum a, sum b) over n elements into out[3] (fp64): dice_coeff's three sums
 * (PMU/dice_loss.py:5-12) for arbitrary pred/target tensors. */
int pmu_dice_sums(const float* a, const float* b, long long n, double* out, void* stream);

/* ---- multi-planar slicer (PMU/utils/mri_dataset.py:11-143) --------------------------------
 * A scan vol [d0][d1][d2] (f64) is re-laid out per view into a padded p0 x p1 x p2 frame
 * (pad_dimensions :85-98 = zeros at the end of the argmin axis) so each slice is contiguous:
 *   view 0: out[i][j][k] (slice = image[i,:,:]),  view 1: out[j][i][k] (image[:,j,:]),
 *   view 2: out[k][i][j] (image[:,:,k])            (sample_slice :70-82). */
int pmu_slice_view_layout(const double* vol, int d0, int d1, int d2, int p0, int p1, int p2, int view,
                          double* out, void* stream);
/* out[s] = max over the px elements of slice s (preprocess' max :109-110, index-map filter :45-46). */
int pmu_slice_max(const double* slices, int nslices, long long px, double* out, void* stream);
/* Batch assembly from a device slice table: addr[g] = device address of f64 slice g (px elements),
 * maxv[g] its max.  out[b][:] = float(slice[ids[b]] / maxv[ids[b]]) when normalize and the max is
 * non-zero, else float(value) (preprocess :101-112 then .float() :142).  ids: device [B]. */
int pmu_gather_slices(const long long* addr, const double* maxv, const int* ids, int B, long long px,
                      int normalize, float* out, void* stream);

/* ---- 3-view volume fusion (PMU/eval.py:157-203) --------------------------------------------
 * v0 [D0][C][D1][D2], v1 [D1][C][D0][D2], v2 [D2][C][D0][D1]: the per-view stacks of slice
 * predictions (probabilities; logits=1 applies softmax over C first).  In the view-0 frame:
 * avg = (p0 + p1 + p2) / 3 (optional output, [D0][C][D1][D2]), label = first argmax of avg
 * (optional, int32 [D0][D1][D2]), and counts[4][C][3] = exact (intersection, |pred|, |truth|) of the
 * one-hot argmax of view 0, view 1, view 2 and avg vs truth [D0][D1][D2] == c.  C <= 8. */
int pmu_fuse3view(const float* v0, const float* v1, const float* v2, const float* truth, int D0, int D1,
                  int D2, int C, int logits, float* avg, int* label, double* counts, void* stream);

/* ---- probabilistic path: latent head of AxisAlignedConvGaussian ---------------------------
 * probabilistic_unet.py:95-108: encoding = mean_{h,w} relu(bn(z_last)); mu_log_sigma = conv1x1(encoding). */
/* out[N][C] = (1/(H*W)) sum_{h,w} max(0, z*scale+shift), z NHWC, coef = [scale|shift]. */
int pmu_spatial_mean(const float* z, const float* coef, int N, int H, int W, int C, float* out,
                     void* stream);
/* da[N][H][W][C] = dmean[N][C] / (H*W). */
int pmu_spatial_mean_bwd(const float* dmean, int N, int H, int W, int C, float* da, void* stream);
/* The same fused with the BN+ReLU backward partial sums of the averaged layer (:39 mean over the
 * encoder's last activation): part as pmu_avgpool2_bwd_bnr.  C % 4 == 0. */
int pmu_spatial_mean_bwd_bnr(const float* dmean, const float* z, const float* coef, const float* mean,
                             const float* invstd, int N, int H, int W, int C, float* da, float* part, void* stream);
/* y[N][M] = x[N][K] . w[M][K]^T + b  (a 1x1 conv on a 1x1 map, probabilistic_unet.py:72,101). */
int pmu_linear_fwd(const float* x, const float* w, const float* b, int N, int K, int M, float* y,
                   void* stream);
/* dx = dy.w (dx may be NULL), dw = dy^T.x, db = sum_n dy (db may be NULL); M <= 256. */
int pmu_linear_bwd(const float* x, const float* w, const float* dy, int N, int K, int M, float* dx,
                   float* dw, float* db, void* stream);

/* ---- probabilistic path: Fcomb (probabilistic_unet.py:116-181) ----------------------------
 * logits = W_last . relu(W_NH ... relu(W_1 . cat(f, tile(z)) + b_1) ...) + b_last per pixel,
 * NH = no_convs_fcomb - 1 hidden 1x1 convs (1..3), F = feature width (<= 64), L = latent dim,
 * K = classes (<= 32).  w[l], b[l]: PyTorch layouts (w[0] = W_1 [F][F+L], w[l>0] = [F][F]),
 * wl = W_last [K][F].  The tiled z is never built: zb = W_1z . z + b_1 is a per-(sample,image)
 * bias from pmu_fcomb_zbias. */
/* zb[SN][F] = w1[:, F:F+L] . z[SN][L] + b1. */
int pmu_fcomb_zbias(const float* z, const float* w1, const float* b1, int SN, int F, int L,
                    float* zb, void* stream);
/* feat NHWC [N][H][W][F]; zb [S][N][F]; y NCHW [S][N][K][H][W] (S samples in one pass). */
int pmu_fcomb_fwd(const float* feat, const float* zb, const float* const* w, const float* const* b,
                  const float* wl, const float* bl, int F, int L, int K, int NH, int S, int N, int H,
                  int W, float* y, void* stream);
size_t pmu_fcomb_bwd_ws(int N, int H, int W);
/* One sample: dl = dL/dlogits NCHW [N][K][H][W] -> dfeat NHWC, dz [N][L] (may be NULL),
 * dw[l], db[l] (PyTorch layouts, overwritten), dwl, dbl.  z [N][L] and zb [N][F] as in forward. */
int pmu_fcomb_bwd(const float* feat, const float* z, const float* zb, const float* dl,
                  const float* const* w, const float* const* b, const float* wl, const float* bl,
                  int F, int L, int K, int NH, int N, int H, int W, float* dfeat, float* dz,
                  float* const* dw, float* const* db, float* dwl, float* dbl, float* ws,
                  size_t ws_bytes, void* stream);

/* ---- diagnostics: resident blocks per CU of the main GEMM kernels (hipOccupancy API) ---- */
int pmu_occupancy_conv3x3_raw(int* blocks_per_cu);
int pmu_occupancy_wgrad3x3_bf16(int* blocks_per_cu);

/* ---- batched weight packing ------------------------------------------------------------------
 * One launch re-packs the weights of many layers into one layout after an optimizer step
 * (pmu_hip.optim.FusedSGD -> pmu_hip.engine.repack): jobs[] in DEVICE memory, job j = one tensor w
 * [Cout][Cin][3][3] (ConvTranspose2d: [Cin][Cout][2][2]) packed into dst as the single-tensor pack
 * function of that layout would, using workgroups [block0, block0 + nblocks) of a grid of `blocks`
 * (nblocks from the matching *_blocks query).  dgrad is uniform over the jobs of one call. */
typedef struct {
  const float* w;
  void* dst;
  int Cout, Cin, block0, nblocks;
} pmu_pack_job;
int pmu_conv3x3_pack_wino2h_blocks(int Cout, int Cin, int dgrad);
int pmu_conv3x3_pack_wino2h_multi(const pmu_pack_job* jobs, int njobs, int blocks, int dgrad, void* stream);
int pmu_conv3x3_pack_wino4_blocks(int Cout, int Cin, int dgrad);
int pmu_conv3x3_pack_wino4_multi(const pmu_pack_job* jobs, int njobs, int blocks, int dgrad, void* stream);
int pmu_convT2x2_pack_blocks(int Cin, int Cout, int dgrad);
int pmu_convT2x2_pack_multi(const pmu_pack_job* jobs, int njobs, int blocks, int dgrad, void* stream);
int pmu_conv3x3_pack_dma_blocks(int Cout, int Cin, int dgrad);
int pmu_conv3x3_pack_dma_multi(const pmu_pack_job* jobs, int njobs, int blocks, int dgrad, void* stream);
int pmu_convT2x2_pack_dma_blocks(int Cin, int Cout, int dgrad);
int pmu_convT2x2_pack_dma_multi(const pmu_pack_job* jobs, int njobs, int blocks, int dgrad, void* stream);

/* ---- build identity and the bounds-checked debug build ------------------------------------ */
/* Bit 0: experiments build (make EXPERIMENTS=1: kernel-variant A/B switches honoured); bit 1:
 * bounds-checked debug build (make DEBUG=1 -> libpmunet_hip_debug.so, PMU_DCHECK in the kernels). */
int pmu_build_flags(void);
/* Debug build: synchronises the device and returns the first recorded index-bound violation,
 * out[0..4] = {code (PMU_DBG_* in csrc/pmu_common.h; 0 = none), source line, workgroup, set,
 * translation unit}; *tu_name (may be NULL) receives the source file.  Release build: out all 0.
 * pmu_debug_reset clears the records. */
int pmu_debug_read(int* out, const char** tu_name);
int pmu_debug_reset(void);

#ifdef __cplusplus
}
#endif
#endif
