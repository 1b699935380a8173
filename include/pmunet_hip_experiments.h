/* libpmunet_hip EXPERIMENTS build only (csrc: make EXPERIMENTS=1 -> pmu_hip/libpmunet_hip_exp.so).
 *
 * Kernels that were built, tested against fp64 / the oracle and measured, but that the engine's
 * default dispatch does not reach: measured slower or equal, or breaking the parity contract.  They
 * stay buildable for A/B (PMU_LIB=exp, tools/kbench*.py, the engine's PMU_* switches, which the
 * shipped library ignores) and their tests run against the experiments library
 * (tests/conftest.py exp_lib).  Same types and conventions as include/pmunet_hip.h. */
#ifndef PMUNET_HIP_EXPERIMENTS_H
#define PMUNET_HIP_EXPERIMENTS_H

#include "pmunet_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- direct-sum fp32 3x3 convolution (implicit GEMM, fused staging): PMU_FP32_CONV=direct A/B */
/* z[N][H][W][Cout] = conv3x3(frame, w) + bias.  If part != NULL, per-tile BN partial
 * sums (sum z, sum z^2) are written to part[tile][2][Cout]; pmu_conv3x3_tiles() gives
 * the tile count.  tee (nullable): receives the operand the kernel multiplied (the frame after
 * BN+ReLU / pooling / concatenation), [N][H][W][Cin] fp32 — a RAW source for pmu_conv3x3_wgrad. */
int pmu_conv3x3_fwd(const pmu_frame* in, const float* w, const float* wp, const float* bias,
                    int Cout, float* z, float* part, float* tee, void* stream);
/* Optional pre-packed weights (wp != NULL replaces w): the per-block/chunk B tiles laid out
 * contiguously in LDS order, so staging is a straight copy.  dgrad=1 packs the flipped,
 * transposed operand of pmu_conv3x3_dgrad. */
size_t pmu_conv3x3_packed_size(int Cout, int Cin, int dgrad);
int pmu_conv3x3_pack(const float* w, int Cout, int Cin, int dgrad, float* wp, void* stream);
/* dx = dL/d(frame) for frame channels [0,Csplit) -> dx0 (NHWC, Csplit ch) and
 * [Csplit,Cin) -> dx1 (NHWC, Cin-Csplit ch).  dz is a frame whose single source is
 * normally PMU_SRC_BNBWD. */
int pmu_conv3x3_dgrad(const pmu_frame* dz, const float* w, const float* wp, int Cin, int Csplit,
                      float* dx0, float* dx1, float* tee, void* stream);  /* tee: dz after BN backward, [N][H][W][Cout] */

/* ---- 512-thread F(2x2,3x3) kernels on a materialised operand: PMU_WINO2H=0 A/B (the 1024-thread
 * pmu_conv3x3_*_wino2h kernels replace them on every shape) */
/* The F(2x2) operators on a materialised operand (pmu_frame_to_f32 of the frame): xt /
 * dzt [N][H][W][C] fp32 with C % 16 == 0, staged by LDS-DMA.  part rows = pmu_conv3x3_tiles_wino(). */
int pmu_conv3x3_fwd_wino_raw(const float* xt, int Cin, int N, int H, int W, const float* wp, const float* bias,
                             int Cout, float* z, float* part, void* stream);
int pmu_conv3x3_dgrad_wino_raw(const float* dzt, int Cout, int N, int H, int W, const float* wp, int Cin,
                               int Csplit, float* dx0, float* dx1, void* stream);

/* ---- F(4x4,3x3) forward: breaks the model-level 1e-3 / Dice contract through the BatchNorm statistics
 * (DESIGN.md §3a); PMU_WINO4=1 A/B */
int pmu_conv3x3_fwd_wino4(const float* xt, int Cin, int N, int H, int W, const float* wp, const float* bias,
                          int Cout, float* z, float* part, void* stream);

/* ---- F(4x4,3x3) weight gradient: measured equal to F(2x2) (LDS-read bound); PMU_WGRAD4=1 A/B */
/* The same weight gradient by Winograd F(4x4,3x3): 36 products per 4x4 tile and channel pair (2.25
 * per output pixel vs F(2x2)'s 4), output transform in fp64; fp32 rounding ~1.3e-6 of rms |dw|
 * (tools/wgrad_err.py).  Cout % 32 == 0, Cin % 64 == 0 (pmu_conv3x3_wgrad_ws_wino4 returns 0
 * otherwise); ws must hold that many bytes. */
size_t pmu_conv3x3_wgrad_ws_wino4(int N, int H, int W, int Cin, int Cout);
int pmu_conv3x3_wgrad_wino4(const float* dzt, const float* xt, int N, int H, int W, int Cout, int Cin,
                            float* dw, float* ws, size_t ws_bytes, void* stream);

/* ---- bf16-stored z: breaks the c5 eval Dice contract and is not faster; PMU_BF16_Z=1 */
/* bf16 storage of z (config c5: torch.autocast keeps a conv's output in bf16, unet_parts.py:15,18 under
 * autocast), centred: the forward stores bf16(z - zoff[c]) (RNE; zoff = the BN running mean, null: 0)
 * with the BN partial sums of stored + zoff; every consumer then applies the centred coefficients of
 * pmu_bn_center.  The input gradient's BN-backward partials read such a z. */
int pmu_conv3x3_fwd_dma_zb(const unsigned short* xt, int Cp, int N, int H, int W, const unsigned short* wp,
                           const float* bias, int Cout, unsigned short* z, const float* zoff, float* part,
                           void* stream);
/* coef_out = [scale | shift + off*scale], mean_out = mean - off (in place allowed; mean may be NULL) */
int pmu_bn_center(const float* coef, const float* mean, const float* off, int C, float* coef_out,
                  float* mean_out, void* stream);
int pmu_conv3x3_dgrad_dma_bnr_zb(const unsigned short* dzt, int Cp, int N, int H, int W, const unsigned short* wp,
                                 int Cin, float* dx, const unsigned short* z, const float* coef, const float* mean,
                                 const float* invstd, float* part, void* stream);

/* ---- register-staged bf16 ConvT forward / input gradient: the engine takes the LDS-DMA kernels on
 * exactly these shapes */
/* ConvTranspose2d(k2,s2) forward / input gradient with bf16 operands (fp32 sums and outputs), weights
 * packed as pmu_convT2x2_pack's layouts in bf16 (4*Cin*Cout elements).  The forward takes one unpooled
 * BN+ReLU source with Cin % 32 == 0, Cout % 32 == 0 (pmu_convT2x2_bf16_ok), dgrad Cin % 128 == 0 and
 * Cout % 32 == 0. */
int pmu_convT2x2_pack_bf16(const float* w, int Cin, int Cout, int dgrad, unsigned short* wp, void* stream);
int pmu_convT2x2_bf16_ok(const pmu_frame* in, int Cout);
int pmu_convT2x2_fwd_bf16(const pmu_frame* in, const unsigned short* wp, const float* bias, int Cout,
                          float* u, void* stream);
int pmu_convT2x2_dgrad_bf16(const float* du, int Hd, int Wd, int off_h, int off_w, const unsigned short* wp,
                            int N, int H, int W, int Cin, int Cout, float* dx, void* stream);

/* the same over a bf16-stored z (C % 4 == 0) */
int pmu_bn_bwd_reduce_zb(const float* da, const unsigned short* z, const float* coef, const float* mean,
                         const float* invstd, int P, int C, float* part, void* stream);

/* the same over a bf16-stored z (coef required, C % 4 == 0) */
int pmu_maxpool2_bwd_zb(const float* dpool, const unsigned short* z, const float* coef, int N, int H, int W,
                        int C, float* dx, int accumulate, void* stream);

/* ---- persistent tile schedule of the LDS-DMA convs (conv3x3_bf16_dma.hip PERS; PMU_DMA_PERS=1 turns
 * it on for the pmu_conv3x3_*_dma entries of this library): 1 when a conv of this shape (NOUT outputs
 * of a Cp-channel operand) would run it — one resident workgroup per slot walking a run of tiles, the
 * next tile's first chunk fetched under the current one's last — else 0.  Bit-identical to the
 * one-tile grid; measured slower. */
int pmu_conv3x3_dma_persistent(int N, int H, int W, int NOUT, int Cp);

/* ---- diagnostics of the direct-sum kernel */
int pmu_occupancy_conv3x3_pipe(int* blocks_per_cu);

#ifdef __cplusplus
}
#endif

#endif  /* PMUNET_HIP_EXPERIMENTS_H */
