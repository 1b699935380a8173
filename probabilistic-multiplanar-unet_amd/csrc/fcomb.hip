// Fcomb (PMU/model/probabilistic_unet/probabilistic_unet.py:116-181) and the latent head of
// AxisAlignedConvGaussian (probabilistic_unet.py:95-108) on gfx950.
//
// Fcomb: logits = W_last . relu(W_NH ... relu(W_1 . [f ; tile(z)] + b_1) ...) + b_last per pixel.
// The tiled z is never materialised: W_1 . [f ; z] = W_1f . f + (W_1z . z + b_1), the second term
// being a per-(sample, image) bias zb computed once (pmu_fcomb_zbias).  One launch evaluates S
// samples: the feature tile is staged and W_1f . f computed once, then each sample adds its own zb.
// Per-pixel layers are 64-wide GEMMs on f32 MFMA (32x32x2); activations stay in LDS.
// Backward recomputes the forward for its tile in LDS and back-propagates through the chain,
// accumulating weight gradients in registers across the tiles of a persistent block and writing
// one fp32 partial slab per block (fixed-order reduction, no atomics).
#include "pmu_common.h"

namespace {

constexpr int FW = 64;         // padded feature / hidden width
constexpr int KP = 32;         // padded output classes
constexpr int RS = FW + 1;     // LDS row stride (b32 reads: consecutive lanes -> distinct banks)
constexpr int MAXNH = 3;       // hidden layers supported (no_convs_fcomb <= 4)

struct FcombW {
  const float* w[MAXNH];  // w[0] = W_1 [F][F+L] (feature part used), w[l] = [F][F]
  const float* b[MAXNH];  // b[0] unused in-kernel (folded into zb)
  const float* wl;        // W_last [K][F]
  const float* bl;        // [K]
  int F, L, K, NH;
};

// stage all weights into LDS: Ws[l][o][c] (padded to 64x64, stride RS), Wl[o][c] (32 x 64)
__device__ __forceinline__ void stage_weights(const FcombW& p, float* Ws, float* Wl) {
  for (int e = threadIdx.x; e < MAXNH * FW * FW; e += blockDim.x) {
    const int l = e / (FW * FW), r = e % (FW * FW), o = r / FW, c = r % FW;
    float v = 0.f;
    if (l < p.NH && o < p.F && c < p.F) v = p.w[l][(long long)o * (l == 0 ? p.F + p.L : p.F) + c];
    Ws[(l * FW + o) * RS + c] = v;
  }
  for (int e = threadIdx.x; e < KP * FW; e += blockDim.x) {
    const int o = e / FW, c = e % FW;
    Wl[o * RS + c] = (o < p.K && c < p.F) ? p.wl[o * p.F + c] : 0.f;
  }
}

// acc[fn] (32 px x 32 out, out = fn*32 + lane&31) = sum_k A[px][k] * W[o][k] over k < 64.
// A rows are this wave's 32 pixels (row base pa), W rows o (stride RS).
template <int NF>
__device__ __forceinline__ void mm64(const float* A, const float* W, int lane, f32x16 (&acc)[NF]) {
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[f][r] = 0.f;
  const float* pa = A + (lane & 31) * RS + (lane >> 5);
#pragma unroll 4
  for (int k = 0; k < FW; k += 2) {
    const float av = pa[k];
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[f] = mfma_f32_32x32x2(av, W[(f * 32 + (lane & 31)) * RS + k + (lane >> 5)], acc[f]);
  }
}

// ------------------------------------------------------------------------------------------
// forward: y[s][n][k][h][w]; feat NHWC [P][F]; zb [S][N][F]
// Register-resident: a wave owns 32 pixels and computes every layer transposed,
//   out^T[o][px] = sum_k W[o][k] * in^T[k][px]     (MFMA A = weight rows, B = activations)
// so the accumulator of one layer IS the B operand of the next: lane (px = lane&31, half h) holds
// channels o = acc_row(r) = (r&3) + 8(r>>2) + 4h in register r, and k-step s of a 32-channel block
// feeds channel acc_row(s) of that block (the K order inside a block is free as long as A and B
// agree).  The matching weight values W[o][8q+4h .. 8q+4h+3] of 4 consecutive k-steps are one
// ds_read_b128 of the LDS weight row.  Activations never touch LDS; weights are staged once per
// block (persistent over 32-pixel groups).
// ------------------------------------------------------------------------------------------
constexpr int RRS = 68;  // LDS weight row stride: b128 reads of 8 rows hit distinct bank groups

// channels c0..c0+3 of a row of F floats: one float4 when rows are 16-B aligned (F % 4 == 0),
// else guarded scalar loads (any num_filters[0] <= 64 is legal in the reference)
__device__ __forceinline__ float4 ld4_row(const float* row, int c0, int F, bool f4) {
  if (f4) return c0 < F ? *reinterpret_cast<const float4*>(row + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
  return make_float4(c0 < F ? row[c0] : 0.f, c0 + 1 < F ? row[c0 + 1] : 0.f, c0 + 2 < F ? row[c0 + 2] : 0.f,
                     c0 + 3 < F ? row[c0 + 3] : 0.f);
}

template <bool FEWK>  // FEWK: K <= 4 classes, last layer on VALU
__global__ __launch_bounds__(256, 2) void fcomb_fwd_kernel(const float* __restrict__ feat, const float* __restrict__ zb,
                                                           FcombW p, int S, int N, long long HW, float* __restrict__ y,
                                                           long long ngroups) {
  __shared__ __attribute__((aligned(16))) float Wsh[(MAXNH * FW + KP) * RRS + MAXNH * FW + KP];
  float* Bsh = Wsh + (MAXNH * FW + KP) * RRS;  // biases: [l][64] for l >= 1, then last [32]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < MAXNH * FW * FW; e += 256) {
    const int l = e / (FW * FW), r = e % (FW * FW), o = r / FW, c = r % FW;
    float v = 0.f;
    if (l < p.NH && o < p.F && c < p.F) v = p.w[l][(long long)o * (l == 0 ? p.F + p.L : p.F) + c];
    Wsh[(l * FW + o) * RRS + c] = v;
  }
  for (int e = tid; e < KP * FW; e += 256) {
    const int o = e / FW, c = e % FW;
    Wsh[(MAXNH * FW + o) * RRS + c] = (o < p.K && c < p.F) ? p.wl[o * p.F + c] : 0.f;
  }
  for (int e = tid; e < MAXNH * FW + KP; e += 256) {
    float v = 0.f;
    if (e < MAXNH * FW) {
      const int l = e / FW, o = e % FW;
      if (l >= 1 && l < p.NH && o < p.F) v = p.b[l][o];
    } else if (e - MAXNH * FW < p.K) {
      v = p.bl[e - MAXNH * FW];
    }
    Bsh[e] = v;
  }
  __syncthreads();

  const int h = lane >> 5;
  const bool f4 = (p.F & 3) == 0;
  const long long P = (long long)N * HW;
  const float* wrow = Wsh + (lane & 31) * RRS + 4 * h;  // + (row block)*RRS + kb*32 + 8q
  for (long long g = (long long)blockIdx.x * 4 + wave; g < ngroups; g += (long long)gridDim.x * 4) {
    const long long px = g * 32 + (lane & 31);
    const bool valid = px < P;
    const long long pxc = valid ? px : P - 1;
    const long long n = pxc / HW, pix = pxc - n * HW;
    // ---- layer 1 feature part (sample independent): u[ob] = W_1f . f
    f32x16 u[2];
#pragma unroll
    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
      for (int r = 0; r < 16; ++r) u[ob][r] = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c0 = kb * 32 + 8 * q + 4 * h;
        float4 fv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (valid) fv = ld4_row(feat + pxc * p.F, c0, p.F, f4);
        const float fa[4] = {fv.x, fv.y, fv.z, fv.w};
        float4 w4[2];
#pragma unroll
        for (int ob = 0; ob < 2; ++ob) w4[ob] = *reinterpret_cast<const float4*>(wrow + (ob * 32) * RRS + kb * 32 + 8 * q);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
          for (int ob = 0; ob < 2; ++ob) {
            const float wa = s4 == 0 ? w4[ob].x : s4 == 1 ? w4[ob].y : s4 == 2 ? w4[ob].z : w4[ob].w;
            u[ob] = mfma_f32_32x32x2(wa, fa[s4], u[ob]);
          }
      }
    for (int s = 0; s < S; ++s) {
      // ---- h1 = relu(u + zb[s][n])
      f32x16 hc[2];
      const float* zr = zb + ((long long)s * N + n) * p.F;
#pragma unroll
      for (int ob = 0; ob < 2; ++ob)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c0 = ob * 32 + 8 * q + 4 * h;
          const float4 zv = ld4_row(zr, c0, p.F, f4);
          hc[ob][4 * q + 0] = fmaxf(0.f, u[ob][4 * q + 0] + zv.x);
          hc[ob][4 * q + 1] = fmaxf(0.f, u[ob][4 * q + 1] + zv.y);
          hc[ob][4 * q + 2] = fmaxf(0.f, u[ob][4 * q + 2] + zv.z);
          hc[ob][4 * q + 3] = fmaxf(0.f, u[ob][4 * q + 3] + zv.w);
        }
      // ---- hidden layers 2..NH
      for (int l = 1; l < p.NH; ++l) {
        f32x16 na[2];
#pragma unroll
        for (int ob = 0; ob < 2; ++ob)
#pragma unroll
          for (int r = 0; r < 16; ++r) na[ob][r] = 0.f;
        const float* wl = wrow + (l * FW) * RRS;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float4 w4[2];
#pragma unroll
            for (int ob = 0; ob < 2; ++ob) w4[ob] = *reinterpret_cast<const float4*>(wl + (ob * 32) * RRS + kb * 32 + 8 * q);
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
              for (int ob = 0; ob < 2; ++ob) {
                const float wa = s4 == 0 ? w4[ob].x : s4 == 1 ? w4[ob].y : s4 == 2 ? w4[ob].z : w4[ob].w;
                na[ob] = mfma_f32_32x32x2(wa, hc[kb][4 * q + s4], na[ob]);
              }
          }
#pragma unroll
        for (int ob = 0; ob < 2; ++ob)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 bv = *reinterpret_cast<const float4*>(Bsh + l * FW + ob * 32 + 8 * q + 4 * h);
            hc[ob][4 * q + 0] = fmaxf(0.f, na[ob][4 * q + 0] + bv.x);
            hc[ob][4 * q + 1] = fmaxf(0.f, na[ob][4 * q + 1] + bv.y);
            hc[ob][4 * q + 2] = fmaxf(0.f, na[ob][4 * q + 2] + bv.z);
            hc[ob][4 * q + 3] = fmaxf(0.f, na[ob][4 * q + 3] + bv.w);
          }
      }
      if (FEWK) {
        // ---- last layer for a few classes (the trainer's 3): VALU dot products instead of a
        // 32-row MFMA tile that would be 7/8 padding. Lane (px, h) holds half the channels of its
        // pixel: register 4q+s4 of block kb = channel kb*32 + 8q + 4h + s4.
        float yk[4] = {0.f, 0.f, 0.f, 0.f};
        const float* wlast = Wsh + (MAXNH * FW) * RRS + 4 * h;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k >= p.K) break;
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float4 w4 = *reinterpret_cast<const float4*>(wlast + k * RRS + kb * 32 + 8 * q);
              yk[k] = fmaf(w4.x, hc[kb][4 * q + 0], yk[k]);
              yk[k] = fmaf(w4.y, hc[kb][4 * q + 1], yk[k]);
              yk[k] = fmaf(w4.z, hc[kb][4 * q + 2], yk[k]);
              yk[k] = fmaf(w4.w, hc[kb][4 * q + 3], yk[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) yk[k] += __shfl_xor(yk[k], 32, 64);
        if (valid) {
          float* yo = y + ((long long)s * N + n) * p.K * HW + pix;
#pragma unroll
          for (int k = 0; k < 4; ++k)  // the two halves store alternate classes
            if (k < p.K && (k & 1) == h) yo[(long long)k * HW] = yk[k] + Bsh[MAXNH * FW + k];
        }
        continue;
      }
      // ---- last layer (K <= 32 rows); two accumulators (one per input block) to break the chain
      f32x16 la[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) la[kb][r] = 0.f;
      const float* wlast = wrow + (MAXNH * FW) * RRS;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const float4 w4 = *reinterpret_cast<const float4*>(wlast + kb * 32 + 8 * q);
          la[kb] = mfma_f32_32x32x2(w4.x, hc[kb][4 * q + 0], la[kb]);
          la[kb] = mfma_f32_32x32x2(w4.y, hc[kb][4 * q + 1], la[kb]);
          la[kb] = mfma_f32_32x32x2(w4.z, hc[kb][4 * q + 2], la[kb]);
          la[kb] = mfma_f32_32x32x2(w4.w, hc[kb][4 * q + 3], la[kb]);
        }
      if (valid) {
        float* yo = y + ((long long)s * N + n) * p.K * HW + pix;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int k = acc_row(r, lane);
          if (k < p.K) yo[(long long)k * HW] = la[0][r] + la[1][r] + Bsh[MAXNH * FW + k];
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward (one sample): given dl = dL/dy [N][K][HW], recompute the chain per 64-pixel tile
// and produce dfeat NHWC [P][F], per-block partial slabs of dW_l, db_l, dW_last, db_last and
// per-image dzb[n][F] (= dL/d(zb), summed over the image's pixels).
// block = 4 waves; GEMMs over 64 px x 64 out are split 2x2 over waves.
// ------------------------------------------------------------------------------------------
constexpr int BT = 64;

struct FcombG {
  float* dfeat;  // [P][F]
  float* ws;     // per block: NH*64*64 (dW_l, [o][c]) + 32*64 (dW_last) + NH*64 (db_l) + 32 (db_last)
  float* dzb;    // per block: [N][64]  (zeroed by the kernel, block-partial)
};

constexpr int WS_BLOCK = MAXNH * FW * FW + KP * FW + MAXNH * FW + KP;

// C[px][o] += sum_k A[px][k] * B[k][o]  for a 32x32 fragment: A row stride RS, B given as
// element accessor (k, o).  Lane supplies A[px = lane&31][k] and B[k][o = lane&31].
template <class BF>
__device__ __forceinline__ void frag_mm(const float* A, int arow0, int K, const BF& bf, int ocol0, int lane,
                                        f32x16& acc) {
  const float* pa = A + (arow0 + (lane & 31)) * RS + (lane >> 5);
#pragma unroll 4
  for (int k = 0; k < K; k += 2)
    acc = mfma_f32_32x32x2(pa[k], bf(k + (lane >> 5), ocol0 + (lane & 31)), acc);
}

__global__ __launch_bounds__(256) void fcomb_bwd_kernel(const float* __restrict__ feat, const float* __restrict__ zb,
                                                        const float* __restrict__ dl, FcombW p, int N, long long HW,
                                                        FcombG g, long long ntiles) {
  __shared__ __attribute__((aligned(16))) float sm[MAXNH * FW * RS + KP * RS + BT * RS + MAXNH * BT * RS + BT * RS + BT * 33];
  float* Ws = sm;                     // [NH][64 o][RS]
  float* Wl = Ws + MAXNH * FW * RS;   // [32][RS]
  float* Fb = Wl + KP * RS;           // features [64][RS]
  float* Hb = Fb + BT * RS;           // H1..H3 [3][64][RS]
  float* Xb = Hb + MAXNH * BT * RS;   // scratch dU [64][RS]
  float* Db = Xb + BT * RS;           // dl [64][33]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fm = wave >> 1, fn = wave & 1;  // 2x2 split of 64x64 GEMMs
  const int NH = p.NH;
  stage_weights(p, Ws, Wl);
  float* myws = g.ws + (long long)blockIdx.x * WS_BLOCK;
  float* mydzb = g.dzb + (long long)blockIdx.x * N * FW;
  for (int e = tid; e < N * FW; e += 256) mydzb[e] = 0.f;

  // weight-gradient accumulators (register-resident across tiles): dW_l[o][c] frag (fm, fn)
  f32x16 dW[MAXNH];
  f32x16 dWl;
#pragma unroll
  for (int l = 0; l < MAXNH; ++l)
#pragma unroll
    for (int r = 0; r < 16; ++r) dW[l][r] = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) dWl[r] = 0.f;
  float dbl = 0.f, db[MAXNH] = {0.f, 0.f, 0.f};  // thread tid < 64 owns column tid
  const long long P = (long long)N * HW;

  for (long long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long long p0 = tile * BT;
    __syncthreads();
    for (int e = tid; e < BT * FW; e += 256) {
      const int r = e / FW, c = e % FW;
      const long long px = p0 + r;
      Fb[r * RS + c] = (px < P && c < p.F) ? feat[px * p.F + c] : 0.f;
    }
    for (int e = tid; e < BT * KP; e += 256) {
      const int r = e / KP, k = e % KP;
      const long long px = p0 + r;
      float v = 0.f;
      if (px < P && k < p.K) {  // 32-bit decode (P < 2^31, host-checked)
        const unsigned n = (unsigned)px / (unsigned)HW, pix = (unsigned)px - n * (unsigned)HW;
        v = dl[((size_t)n * p.K + k) * (unsigned)HW + pix];
      }
      Db[r * 33 + k] = v;
    }
    __syncthreads();
    // ---- recompute H_l = relu(U_l)
    for (int l = 0; l < NH; ++l) {
      const float* A = l == 0 ? Fb : Hb + (l - 1) * BT * RS;
      const float* W = Ws + l * FW * RS;
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      frag_mm(A, fm * 32, FW, [&](int k, int o) { return W[o * RS + k]; }, fn * 32, lane, acc);
      float* H = Hb + l * BT * RS;
      const int o = fn * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = fm * 32 + acc_row(r, lane);
        float b;
        if (l == 0) {
          const long long px = p0 + rr;
          const unsigned n = (unsigned)(px < P ? px : P - 1) / (unsigned)HW;
          b = o < p.F ? zb[(size_t)n * p.F + o] : 0.f;
        } else {
          b = o < p.F ? p.b[l][o] : 0.f;
        }
        H[rr * RS + o] = fmaxf(0.f, acc[r] + b);
      }
      __syncthreads();
    }
    // ---- last layer: dU_NH = (dl . W_last) * [H_NH > 0];  dW_last += dl^T H_NH;  db_last += sum dl
    {
      const float* Hn = Hb + (NH - 1) * BT * RS;
      if (wave < 2) {  // dW_last [32 o][64 c]: frag (o 0..31, c = wave*32..)
        const float* pd = Db + (lane >> 5) * 33;
#pragma unroll 4
        for (int k = 0; k < BT; k += 2) {  // k = pixel
          const float av = pd[(k) * 33 + (lane & 31)];          // A[o][px] = dl[px][o]
          const float bv = Hn[(k + (lane >> 5)) * RS + wave * 32 + (lane & 31)];  // B[px][c]
          dWl = mfma_f32_32x32x2(av, bv, dWl);
        }
      }
      if (tid < KP) {
        float s = 0.f;
        for (int r = 0; r < BT; ++r) s += Db[r * 33 + tid];
        dbl += s;
      }
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      // dH[px][c] = sum_o dl[px][o] W_last[o][c]  (A = Db rows (stride 33), K = 32 classes)
      {
        const float* pa = Db + (fm * 32 + (lane & 31)) * 33 + (lane >> 5);
#pragma unroll 4
        for (int k = 0; k < KP; k += 2)
          acc = mfma_f32_32x32x2(pa[k], Wl[(k + (lane >> 5)) * RS + fn * 32 + (lane & 31)], acc);
      }
      const int c = fn * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = fm * 32 + acc_row(r, lane);
        Xb[rr * RS + c] = Hn[rr * RS + c] > 0.f ? acc[r] : 0.f;
      }
      __syncthreads();
    }
    // ---- hidden layers l = NH-1 .. 0:  dU_l in Xb
    for (int l = NH - 1; l >= 0; --l) {
      const float* Hin = l == 0 ? Fb : Hb + (l - 1) * BT * RS;  // input of layer l
      // dW_l[o][c] += sum_px dU[px][o] * Hin[px][c]   (frag: o = fm*32.., c = fn*32..)
      {
        const float* pa = Xb + (lane >> 5) * RS + fm * 32 + (lane & 31);  // A[o][px] = dU[px][o]
        const float* pb = Hin + (lane >> 5) * RS + fn * 32 + (lane & 31);
        f32x16 acc = dW[0];
        if (l == 1) acc = dW[1];
        if (l == 2) acc = dW[2];
#pragma unroll 4
        for (int k = 0; k < BT; k += 2) acc = mfma_f32_32x32x2(pa[k * RS], pb[k * RS], acc);
        if (l == 0) dW[0] = acc;
        if (l == 1) dW[1] = acc;
        if (l == 2) dW[2] = acc;
      }
      if (tid < FW) {  // db_l (l >= 1) or per-image dzb (l == 0)
        if (l > 0) {
          float s = 0.f;
          for (int r = 0; r < BT; ++r) s += Xb[r * RS + tid];
          if (l == 1) db[1] += s;
          if (l == 2) db[2] += s;
        } else {
          // group the tile's pixels by image
          int r = 0;
          while (r < BT && p0 + r < P) {
            const long long n = (p0 + r) / HW;
            const long long end = (n + 1) * HW - p0;
            const int r1 = (int)(end < BT ? end : BT);
            float s = 0.f;
            for (int q = r; q < r1 && p0 + q < P; ++q) s += Xb[q * RS + tid];
            mydzb[n * FW + tid] += s;
            r = r1;
          }
        }
      }
      // dX[px][c] = sum_o dU[px][o] W_l[o][c]
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const float* W = Ws + l * FW * RS;
      {
        const float* pa = Xb + (fm * 32 + (lane & 31)) * RS + (lane >> 5);
#pragma unroll 4
        for (int k = 0; k < FW; k += 2)
          acc = mfma_f32_32x32x2(pa[k], W[(k + (lane >> 5)) * RS + fn * 32 + (lane & 31)], acc);
      }
      __syncthreads();  // everyone done reading Xb / Hin
      const int c = fn * 32 + (lane & 31);
      if (l > 0) {
        const float* Hm = Hb + (l - 1) * BT * RS;  // relu mask of layer l-1's output
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rr = fm * 32 + acc_row(r, lane);
          Xb[rr * RS + c] = Hm[rr * RS + c] > 0.f ? acc[r] : 0.f;
        }
      } else if (c < p.F) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const long long px = p0 + fm * 32 + acc_row(r, lane);
          if (px < P) g.dfeat[px * p.F + c] = acc[r];
        }
      }
      __syncthreads();
    }
  }
  // ---- write the block's partial slab
#pragma unroll
  for (int l = 0; l < MAXNH; ++l) {
    if (l >= NH) break;
    const int c = fn * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) myws[(l * FW + fm * 32 + acc_row(r, lane)) * FW + c] = dW[l][r];
  }
  if (wave < 2) {
#pragma unroll
    for (int r = 0; r < 16; ++r) myws[MAXNH * FW * FW + acc_row(r, lane) * FW + wave * 32 + (lane & 31)] = dWl[r];
  }
  if (tid < FW) {
    for (int l = 1; l < MAXNH; ++l) myws[MAXNH * FW * FW + KP * FW + l * FW + tid] = db[l];
    myws[MAXNH * FW * FW + KP * FW + tid] = 0.f;
  }
  if (tid < KP) myws[MAXNH * FW * FW + KP * FW + MAXNH * FW + tid] = dbl;
}

// ------------------------------------------------------------------------------------------
// backward, register-resident (the default): a wave owns 32 pixels at a time, exactly like the
// forward, and keeps the recomputed chain f, H_1..H_NH transposed in registers.  Every layer of
// the backward is one MFMA chain:
//   dIn^T[c][px] = sum_o W[o][c] dU^T[o][px]   A = W column (b32 LDS reads), B = dU registers
//   dW[o][c]    += sum_px dU[px][o] Hin[px][c] A, B from a 32-px LDS scratch per wave,
//                                              accumulators register-resident across groups
// The scratch (dU and the layer input, [px][65]) is written once per layer from registers; the
// bias sums are its column sums.  Each wave walks a contiguous range of 32-px groups, so its
// per-image dzb partials touch at most IPW images; the four waves' weight-gradient fragments are
// summed in LDS in wave order and each block writes one slab (fixed-order reduction, no atomics).
// ------------------------------------------------------------------------------------------
constexpr int SRS = 65;               // scratch row stride
constexpr int SCR = 2 * 32 * SRS;     // per-wave scratch floats (A: dU / dy, B: layer input)
constexpr int WLDS = (MAXNH * FW + KP) * RRS + MAXNH * FW + KP;  // staged weights + biases

struct BwdGeom {
  long long G;  // 32-px groups
  int nb;       // blocks (4 waves each)
  int gpw;      // groups per wave
  int ipw;      // images a wave's range can touch
};

__host__ __device__ inline BwdGeom bwd_geom(int N, long long HW) {
  BwdGeom g;
  g.G = ((long long)N * HW + 31) / 32;
  long long nb = (g.G + 3) / 4;
  if (nb > 256) nb = 256;  // one block (a wave per SIMD) per CU
  if (nb < 1) nb = 1;
  g.nb = (int)nb;
  g.gpw = (int)((g.G + 4 * nb - 1) / (4 * nb));
  g.ipw = (int)(((long long)g.gpw * 32 - 1) / HW) + 2;
  return g;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void zero2(f32x16 (&a)[2]) {
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) a[b][r] = 0.f;
}

// out^T = W . in^T over 64 input channels (forward layer, weights via b128 as in the forward kernel)
__device__ __forceinline__ void bwd_layer_fwd(const float* wl, const f32x16 (&in)[2], f32x16 (&out)[2]) {
  zero2(out);
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 w4[2];
#pragma unroll
      for (int ob = 0; ob < 2; ++ob) w4[ob] = *reinterpret_cast<const float4*>(wl + (ob * 32) * RRS + kb * 32 + 8 * q);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int ob = 0; ob < 2; ++ob) {
          const float wa = s4 == 0 ? w4[ob].x : s4 == 1 ? w4[ob].y : s4 == 2 ? w4[ob].z : w4[ob].w;
          out[ob] = mfma_f32_32x32x2(wa, in[kb][4 * q + s4], out[ob]);
        }
    }
}

// dx^T[c][px] = sum_o W[o][c] du^T[o][px] over NKB 32-row blocks of o (rows o >= omax skipped)
template <int NKB>
__device__ __forceinline__ void bwd_layer_dx(const float* W, const f32x16 (&du)[NKB], int omax, int lane,
                                             f32x16 (&dx)[2]) {
  zero2(dx);
  const int h = lane >> 5;
  const float* wc = W + 4 * h * RRS + (lane & 31);
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int o0 = kb * 32 + (s & 3) + 8 * (s >> 2);  // row of the h = 0 half
      if (o0 >= omax) continue;                         // wave-uniform
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) dx[cb] = mfma_f32_32x32x2(wc[o0 * RRS + cb * 32], du[kb][s], dx[cb]);
    }
}

// scratch[px][ch] <- transposed activation block(s) held in registers
template <int NB>
__device__ __forceinline__ void put_act(float* S, const f32x16 (&a)[NB], int lane) {
  float* row = S + (lane & 31) * SRS;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) row[b * 32 + acc_row(r, lane)] = a[b][r];
}

// dW[ob][cb] += sum_px SA[px][ob*32+o] SB[px][cb*32+c]
template <int NOB>
__device__ __forceinline__ void bwd_layer_dw(const float* SA, const float* SB, int lane, f32x16 (&dw)[NOB][2]) {
  const float* pa = SA + (lane >> 5) * SRS + (lane & 31);
  const float* pb = SB + (lane >> 5) * SRS + (lane & 31);
#pragma unroll 4
  for (int t = 0; t < 16; ++t) {
    float a[NOB], b[2];
#pragma unroll
    for (int ob = 0; ob < NOB; ++ob) a[ob] = pa[2 * t * SRS + ob * 32];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) b[cb] = pb[2 * t * SRS + cb * 32];
#pragma unroll
    for (int ob = 0; ob < NOB; ++ob)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) dw[ob][cb] = mfma_f32_32x32x2(a[ob], b[cb], dw[ob][cb]);
  }
}

__device__ __forceinline__ void relu_mask(f32x16 (&d)[2], const f32x16 (&hval)[2]) {
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) d[b][r] = hval[b][r] > 0.f ? d[b][r] : 0.f;
}

template <int NH>
__global__ __launch_bounds__(256, 1) void fcomb_bwd_reg_kernel(const float* feat,
                                                               const float* __restrict__ zb,
                                                               const float* __restrict__ dl, FcombW p, int N,
                                                               long long HW, float* __restrict__ dfeat,
                                                               float* __restrict__ ws, float* __restrict__ dzb_slab,
                                                               BwdGeom geo) {
  __shared__ __attribute__((aligned(16))) float sm[WLDS + 4 * SCR];
  float* Bsh = sm + (MAXNH * FW + KP) * RRS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  for (int e = tid; e < MAXNH * FW * FW; e += 256) {
    const int l = e / (FW * FW), r = e % (FW * FW), o = r / FW, c = r % FW;
    float v = 0.f;
    if (l < p.NH && o < p.F && c < p.F) v = p.w[l][(long long)o * (l == 0 ? p.F + p.L : p.F) + c];
    sm[(l * FW + o) * RRS + c] = v;
  }
  for (int e = tid; e < KP * FW; e += 256) {
    const int o = e / FW, c = e % FW;
    sm[(MAXNH * FW + o) * RRS + c] = (o < p.K && c < p.F) ? p.wl[o * p.F + c] : 0.f;
  }
  for (int e = tid; e < MAXNH * FW + KP; e += 256) {
    float v = 0.f;
    if (e < MAXNH * FW) {
      const int l = e / FW, o = e % FW;
      if (l >= 1 && l < p.NH && o < p.F) v = p.b[l][o];
    } else if (e - MAXNH * FW < p.K) {
      v = p.bl[e - MAXNH * FW];
    }
    Bsh[e] = v;
  }
  __syncthreads();

  float* SA = sm + WLDS + wave * SCR;
  float* SB = SA + 32 * SRS;
  const float* wrow = sm + (lane & 31) * RRS + 4 * h;
  const bool f4 = (p.F & 3) == 0;
  const unsigned uHW = (unsigned)HW;
  const long long P = (long long)N * HW;
  const int gw = blockIdx.x * 4 + wave;
  const long long g0 = (long long)gw * geo.gpw;
  const long long g1 = g0 + geo.gpw < geo.G ? g0 + geo.gpw : geo.G;
  const int nlo = (int)((unsigned long long)(g0 * 32) / uHW);
  float* mydzb = dzb_slab + (long long)gw * geo.ipw * FW;
  for (int j = 0; j < geo.ipw; ++j) mydzb[j * FW + lane] = 0.f;

  f32x16 dW[NH][2][2], dWl[1][2];
#pragma unroll
  for (int l = 0; l < NH; ++l)
#pragma unroll
    for (int ob = 0; ob < 2; ++ob) zero2(dW[l][ob]);
  zero2(dWl[0]);
  float dbl = 0.f, dbh[NH > 1 ? NH : 1];  // lane = channel
#pragma unroll
  for (int l = 0; l < (NH > 1 ? NH : 1); ++l) dbh[l] = 0.f;

  for (long long g = g0; g < g1; ++g) {
    const long long px = g * 32 + (lane & 31);
    const bool valid = px < P;
    const unsigned pxc = (unsigned)(valid ? px : P - 1);
    const unsigned n = pxc / uHW, pix = pxc - n * uHW;
    // ---- recompute the chain: A[0] = f, A[l] = H_l
    // A[0] = f is re-read from HBM for dW_1 rather than held (its 32 registers would spill)
    auto load_f = [&](f32x16 (&fa)[2]) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float4 fv = make_float4(0.f, 0.f, 0.f, 0.f);
          if (valid) fv = ld4_row(feat + (size_t)pxc * p.F, kb * 32 + 8 * q + 4 * h, p.F, f4);
          fa[kb][4 * q + 0] = fv.x;
          fa[kb][4 * q + 1] = fv.y;
          fa[kb][4 * q + 2] = fv.z;
          fa[kb][4 * q + 3] = fv.w;
        }
    };
    f32x16 A[NH + 1][2];
    load_f(A[0]);
#pragma unroll
    for (int l = 0; l < NH; ++l) {
      f32x16 u[2];
      bwd_layer_fwd(wrow + (l * FW) * RRS, A[l], u);
#pragma unroll
      for (int ob = 0; ob < 2; ++ob)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c0 = ob * 32 + 8 * q + 4 * h;
          const float4 bv = l == 0 ? ld4_row(zb + (size_t)n * p.F, c0, p.F, f4)
                                   : *reinterpret_cast<const float4*>(Bsh + l * FW + c0);
          A[l + 1][ob][4 * q + 0] = fmaxf(0.f, u[ob][4 * q + 0] + bv.x);
          A[l + 1][ob][4 * q + 1] = fmaxf(0.f, u[ob][4 * q + 1] + bv.y);
          A[l + 1][ob][4 * q + 2] = fmaxf(0.f, u[ob][4 * q + 2] + bv.z);
          A[l + 1][ob][4 * q + 3] = fmaxf(0.f, u[ob][4 * q + 3] + bv.w);
        }
    }
    // ---- dy^T (classes in the acc layout of one 32-row block)
    f32x16 dy[1];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = acc_row(r, lane);
      dy[0][r] = (valid && k < p.K) ? dl[((size_t)n * p.K + k) * uHW + pix] : 0.f;
    }
    // ---- last layer: dWl += dy^T H_NH, dbl += sum dy, dH = Wl^T dy
    put_act(SA, dy, lane);
    put_act(SB, A[NH], lane);
    wave_sync();
    bwd_layer_dw<1>(SA, SB, lane, dWl);
    if (lane < KP) {
      float s = 0.f;
#pragma unroll 8
      for (int r = 0; r < 32; ++r) s += SA[r * SRS + lane];
      dbl += s;
    }
    f32x16 d[2];
    bwd_layer_dx<1>(sm + (MAXNH * FW) * RRS, dy, p.K, lane, d);
    relu_mask(d, A[NH]);
    // ---- hidden layers NH-1 .. 0: d = dU_{l+1}
#pragma unroll
    for (int l = NH - 1; l >= 0; --l) {
      wave_sync();  // previous scratch reads done (in-order LDS; fences keep the compiler honest)
      put_act(SA, d, lane);
      if (l == 0) {
        f32x16 fa[2];
        load_f(fa);
        put_act(SB, fa, lane);
      } else {
        put_act(SB, A[l], lane);
      }
      wave_sync();
      bwd_layer_dw<2>(SA, SB, lane, dW[l]);
      if (l > 0) {
        float s = 0.f;
#pragma unroll 8
        for (int r = 0; r < 32; ++r) s += SA[r * SRS + lane];
        dbh[l] += s;
      } else {
        // per-image sums of dU_1 over this group's valid pixels
        int r = 0;
        while (r < 32 && g * 32 + r < P) {
          const unsigned nn = (unsigned)(g * 32 + r) / uHW;
          long long end = (long long)(nn + 1) * HW - g * 32;
          if (end > 32) end = 32;
          if (end > P - g * 32) end = P - g * 32;
          float s = 0.f;
          for (int q = r; q < (int)end; ++q) s += SA[q * SRS + lane];
          mydzb[(nn - nlo) * FW + lane] += s;
          r = (int)end;
        }
      }
      f32x16 dx[2];
      bwd_layer_dx<2>(sm + (l * FW) * RRS, d, FW, lane, dx);
      if (l > 0) {
        relu_mask(dx, A[l]);
#pragma unroll
        for (int b = 0; b < 2; ++b) d[b] = dx[b];
      } else if (valid) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c0 = cb * 32 + 8 * q + 4 * h;
            float* out = dfeat + (size_t)pxc * p.F;
            if (f4) {
              if (c0 < p.F)
                *reinterpret_cast<float4*>(out + c0) =
                    make_float4(dx[cb][4 * q], dx[cb][4 * q + 1], dx[cb][4 * q + 2], dx[cb][4 * q + 3]);
            } else {
#pragma unroll
              for (int i = 0; i < 4; ++i)
                if (c0 + i < p.F) out[c0 + i] = dx[cb][4 * q + i];
            }
          }
      }
    }
  }

  // ---- block reduction of the four waves' partials (wave order), one slab per block
  __syncthreads();
  float* red = sm;  // WS_BLOCK floats, layout of the slab
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int l = 0; l < NH; ++l)
#pragma unroll
        for (int ob = 0; ob < 2; ++ob)
#pragma unroll
          for (int cb = 0; cb < 2; ++cb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              float* e = red + (l * FW + ob * 32 + acc_row(r, lane)) * FW + cb * 32 + (lane & 31);
              *e = w == 0 ? dW[l][ob][cb][r] : *e + dW[l][ob][cb][r];
            }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float* e = red + MAXNH * FW * FW + acc_row(r, lane) * FW + cb * 32 + (lane & 31);
          *e = w == 0 ? dWl[0][cb][r] : *e + dWl[0][cb][r];
        }
      float* rb = red + MAXNH * FW * FW + KP * FW;
#pragma unroll
      for (int l = 0; l < MAXNH; ++l) {
        const float v = (l >= 1 && l < NH) ? dbh[l < NH ? l : 0] : 0.f;
        rb[l * FW + lane] = w == 0 ? v : rb[l * FW + lane] + v;
      }
      if (lane < KP) rb[MAXNH * FW + lane] = w == 0 ? dbl : rb[MAXNH * FW + lane] + dbl;
    }
    __syncthreads();
  }
  float* myws = ws + (long long)blockIdx.x * WS_BLOCK;
  for (int e = tid; e < WS_BLOCK; e += 256) {
    const bool unused = e < MAXNH * FW * FW && e / (FW * FW) >= NH;
    myws[e] = unused ? 0.f : red[e];
  }
}

// dzb_out[n][c] = sum over the waves whose group range touches image n (wave order)
__global__ void fcomb_dzb_reduce_kernel(const float* __restrict__ slab, int N, long long HW, BwdGeom geo,
                                        float* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * FW) return;
  const int n = e / FW, c = e % FW;
  const long long gfirst = (long long)n * HW / 32, glast = ((long long)(n + 1) * HW - 1) / 32;
  const int nw = geo.nb * 4;
  const long long wlo = gfirst / geo.gpw;
  long long whi = glast / geo.gpw;
  if (whi > nw - 1) whi = nw - 1;
  float s = 0.f;
  for (long long w = wlo; w <= whi; ++w) {
    const long long nlo = w * geo.gpw * 32 / HW;
    s += slab[(w * geo.ipw + (n - nlo)) * FW + c];
  }
  out[e] = s;
}

struct FcombOut {
  float* dw[MAXNH];  // dw[0] = dW_1 [F][F+L]
  float* db[MAXNH];
  float* dwl;
  float* dbl;
  float* dz;  // [N][L] or null
};

// sum the per-block slabs (fixed order) and scatter to the PyTorch-layout gradients;
// entries past WS_BLOCK reduce the per-image dzb slabs into dzb_out [N][64]
__global__ void fcomb_reduce_kernel(const float* __restrict__ ws, const float* __restrict__ dzb_slab, int nblk, int N,
                                    FcombW p, FcombOut o, float* __restrict__ dzb_out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= WS_BLOCK) {
    const int q = e - WS_BLOCK;
    if (q >= N * FW) return;
    float s = 0.f;
    for (int b = 0; b < nblk; ++b) s += dzb_slab[(long long)b * N * FW + q];
    dzb_out[q] = s;
    return;
  }
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += ws[(long long)b * WS_BLOCK + e];
  if (e < MAXNH * FW * FW) {
    const int l = e / (FW * FW), r = e % (FW * FW), oo = r / FW, c = r % FW;
    if (l < p.NH && oo < p.F && c < p.F) o.dw[l][(long long)oo * (l == 0 ? p.F + p.L : p.F) + c] = s;
    return;
  }
  int r = e - MAXNH * FW * FW;
  if (r < KP * FW) {
    const int oo = r / FW, c = r % FW;
    if (oo < p.K && c < p.F) o.dwl[oo * p.F + c] = s;
    return;
  }
  r -= KP * FW;
  if (r < MAXNH * FW) {
    const int l = r / FW, c = r % FW;
    if (l >= 1 && l < p.NH && c < p.F) o.db[l][c] = s;
    return;
  }
  r -= MAXNH * FW;
  if (r < p.K) o.dbl[r] = s;
}

// the z side of layer 1 from dzb[n][o] = dL/d(zb[n][o]):
//   db_1[o] = sum_n dzb[n][o];  dW_1[o][F+l] = sum_n dzb[n][o] z[n][l];  dz[n][l] = sum_o dzb[n][o] W_1[o][F+l]
__global__ void fcomb_zgrad_kernel(const float* __restrict__ dzb, const float* __restrict__ z, int N, FcombW p,
                                   FcombOut o) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int F = p.F, L = p.L;
  if (e < F) {
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += dzb[n * FW + e];
    o.db[0][e] = s;
    return;
  }
  int r = e - F;
  if (r < F * L) {
    const int oo = r / L, l = r % L;
    float s = 0.f;
    for (int n = 0; n < N; ++n) s = fmaf(dzb[n * FW + oo], z[(long long)n * L + l], s);
    o.dw[0][(long long)oo * (F + L) + F + l] = s;
    return;
  }
  r -= F * L;
  if (o.dz && r < N * L) {
    const int n = r / L, l = r % L;
    float s = 0.f;
    for (int oo = 0; oo < F; ++oo) s = fmaf(dzb[n * FW + oo], p.w[0][(long long)oo * (F + L) + F + l], s);
    o.dz[r] = s;
  }
}

// zb[s][n][o] = sum_l W_1[o][F+l] z[s][n][l] + b_1[o]
__global__ void fcomb_zbias_kernel(const float* __restrict__ z, const float* __restrict__ w1, const float* __restrict__ b1,
                                   int SN, int F, int L, float* __restrict__ zb) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= SN * F) return;
  const int sn = e / F, o = e % F;
  float acc = b1 ? b1[o] : 0.f;
  for (int l = 0; l < L; ++l) acc = fmaf(w1[(long long)o * (F + L) + F + l], z[(long long)sn * L + l], acc);
  zb[e] = acc;
}

// ---------------- latent head of AxisAlignedConvGaussian ----------------
// mean[n][c] = (1/HW) sum_p relu(z*scale+shift)  (torch.mean over dim 2 then 3, :97-98)
__global__ __launch_bounds__(256) void spatial_mean_kernel(const float* __restrict__ z, const float* __restrict__ coef,
                                                           int N, int HW, int C, float* __restrict__ out) {
  __shared__ float red[256];
  const int n = blockIdx.y;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int pg = threadIdx.x >> 6;
  float s = 0.f;
  if (c < C) {
    const float sc = coef[c], sh = coef[C + c];
    for (int p = pg; p < HW; p += 4) s += fmaxf(0.f, fmaf(z[((long long)n * HW + p) * C + c], sc, sh));
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (pg == 0 && c < C) out[(long long)n * C + c] = (red[threadIdx.x] + red[threadIdx.x + 64] + red[threadIdx.x + 128] +
                                                      red[threadIdx.x + 192]) / (float)HW;
}

// da[n][p][c] = dmean[n][c] / HW  (backward of the spatial mean)
__global__ void spatial_mean_bwd_kernel(const float* __restrict__ dmean, int N, int HW, int C, float* __restrict__ da) {
  const long long total = (long long)N * HW * C;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    const long long n = e / ((long long)HW * C);
    da[e] = dmean[n * C + c] / (float)HW;
  }
}

// y[n][m] = sum_k x[n][k] w[m][k] + b[m]   (the 1x1 conv of a 1x1 map, :72,101)
__global__ void linear_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
                                  int N, int K, int M, float* __restrict__ y) {
  __shared__ float red[256];
  const int n = blockIdx.y, m = blockIdx.x;
  float s = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) s = fmaf(x[(long long)n * K + k], w[(long long)m * K + k], s);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) y[(long long)n * M + m] = red[0] + (b ? b[m] : 0.f);
}

// dx[n][k] = sum_m dy[n][m] w[m][k];  dw[m][k] = sum_n dy[n][m] x[n][k];  db[m] = sum_n dy[n][m]
__global__ void linear_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ dy,
                                  int N, int K, int M, float* __restrict__ dx, float* __restrict__ dw,
                                  float* __restrict__ db) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < K) {
    for (int n = 0; n < N; ++n) {
      float s = 0.f;
      for (int m = 0; m < M; ++m) s = fmaf(dy[(long long)n * M + m], w[(long long)m * K + k], s);
      if (dx) dx[(long long)n * K + k] = s;
    }
    for (int m = 0; m < M; ++m) {
      float s = 0.f;
      for (int n = 0; n < N; ++n) s = fmaf(dy[(long long)n * M + m], x[(long long)n * K + k], s);
      dw[(long long)m * K + k] = s;
    }
  }
  if (db && blockIdx.x == 0 && threadIdx.x < M) {
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += dy[(long long)n * M + threadIdx.x];
    db[threadIdx.x] = s;
  }
}

static int fcomb_bwd_blocks(long long ntiles) {
  long long b = ntiles < 512 ? ntiles : 512;
  return (int)(b < 1 ? 1 : b);
}

static bool make_w(FcombW& p, const float* const* w, const float* const* b, const float* wl, const float* bl, int F,
                   int L, int K, int NH) {
  if (F < 1 || F > FW || L < 0 || K < 1 || K > KP || NH < 1 || NH > MAXNH || !w || !b || !wl || !bl) return false;
  for (int l = 0; l < MAXNH; ++l) {
    p.w[l] = l < NH ? w[l] : nullptr;
    p.b[l] = l < NH ? b[l] : nullptr;
    if (l < NH && (!w[l] || !b[l])) return false;
  }
  p.wl = wl; p.bl = bl; p.F = F; p.L = L; p.K = K; p.NH = NH;
  return true;
}

}  // namespace

extern "C" int pmu_fcomb_zbias(const float* z, const float* w1, const float* b1, int SN, int F, int L, float* zb,
                               void* stream) {
  PMU_REQUIRE(z && w1 && b1 && zb && SN > 0 && F > 0 && F <= FW && L >= 0);
  hipLaunchKernelGGL(fcomb_zbias_kernel, dim3((unsigned)pmu_cdiv((long long)SN * F, 256)), dim3(256), 0,
                     (hipStream_t)stream, z, w1, b1, SN, F, L, zb);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_fcomb_fwd(const float* feat, const float* zb, const float* const* w, const float* const* b,
                             const float* wl, const float* bl, int F, int L, int K, int NH, int S, int N, int H, int W,
                             float* y, void* stream) {
  FcombW p;
  PMU_REQUIRE(feat && zb && y && S > 0 && N > 0 && H > 0 && W > 0 && make_w(p, w, b, wl, bl, F, L, K, NH));
  const long long HW = (long long)H * W;
  const long long ngroups = ((long long)N * HW + 31) / 32;
  long long g = (ngroups + 3) / 4;
  if (g > 512) g = 512;  // persistent: 2 blocks per CU
  if (K <= 4)
    hipLaunchKernelGGL(fcomb_fwd_kernel<true>, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, feat, zb, p, S, N,
                       HW, y, ngroups);
  else
    hipLaunchKernelGGL(fcomb_fwd_kernel<false>, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, feat, zb, p, S, N,
                       HW, y, ngroups);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" size_t pmu_fcomb_bwd_ws(int N, int H, int W) {
  if (N <= 0 || H <= 0 || W <= 0) return 0;
  const long long ntiles = ((long long)N * H * W + BT - 1) / BT;
  const int nb = fcomb_bwd_blocks(ntiles);
  const size_t lds = (size_t)nb * WS_BLOCK + (size_t)nb * N * FW;  // LDS-tile kernel
  const BwdGeom g = bwd_geom(N, (long long)H * W);
  const size_t reg = (size_t)g.nb * WS_BLOCK + (size_t)g.nb * 4 * g.ipw * FW;  // register-resident
  return ((lds > reg ? lds : reg) + (size_t)N * FW) * sizeof(float);
}

static int fcomb_bwd_impl() {  // PMU_FCOMB_BWD=tile selects the LDS-tile kernel (A/B)
  static int v = -1;
  if (v < 0) {
    const char* e = pmu_variant_env("PMU_FCOMB_BWD");
    v = (e && e[0] == 't') ? 0 : 1;
  }
  return v;
}

extern "C" int pmu_fcomb_bwd(const float* feat, const float* z, const float* zb, const float* dl,
                             const float* const* w, const float* const* b, const float* wl, const float* bl, int F,
                             int L, int K, int NH, int N, int H, int W, float* dfeat, float* dz, float* const* dw,
                             float* const* db, float* dwl, float* dbl, float* ws, size_t ws_bytes, void* stream) {
  FcombW p;
  PMU_REQUIRE(feat && z && zb && dl && dfeat && dw && db && dwl && dbl && ws);
  PMU_REQUIRE(N > 0 && H > 0 && W > 0 && make_w(p, w, b, wl, bl, F, L, K, NH));
  PMU_REQUIRE(ws_bytes >= pmu_fcomb_bwd_ws(N, H, W));
  PMU_REQUIRE((long long)N * H * W < (1LL << 31) && (long long)N * H * W * K < (1LL << 32));  // 32-bit decode
  FcombOut o;
  for (int l = 0; l < MAXNH; ++l) {
    o.dw[l] = l < NH ? dw[l] : nullptr;
    o.db[l] = l < NH ? db[l] : nullptr;
    if (l < NH) PMU_REQUIRE(dw[l] && db[l]);
  }
  o.dwl = dwl; o.dbl = dbl; o.dz = dz;
  const long long HW = (long long)H * W;
  hipStream_t st0 = (hipStream_t)stream;
  if (fcomb_bwd_impl() == 1) {
    const BwdGeom geo = bwd_geom(N, HW);
    float* slab = ws + (size_t)geo.nb * WS_BLOCK;
    float* dzb = slab + (size_t)geo.nb * 4 * geo.ipw * FW;
    if (NH == 1)
      hipLaunchKernelGGL(fcomb_bwd_reg_kernel<1>, dim3(geo.nb), dim3(256), 0, st0, feat, zb, dl, p, N, HW, dfeat, ws,
                         slab, geo);
    else if (NH == 2)
      hipLaunchKernelGGL(fcomb_bwd_reg_kernel<2>, dim3(geo.nb), dim3(256), 0, st0, feat, zb, dl, p, N, HW, dfeat, ws,
                         slab, geo);
    else
      hipLaunchKernelGGL(fcomb_bwd_reg_kernel<3>, dim3(geo.nb), dim3(256), 0, st0, feat, zb, dl, p, N, HW, dfeat, ws,
                         slab, geo);
    PMU_CHECK_LAUNCH();
    hipLaunchKernelGGL(fcomb_reduce_kernel, dim3((unsigned)pmu_cdiv(WS_BLOCK, 256)), dim3(256), 0, st0, ws, slab,
                       geo.nb, 0, p, o, dzb);
    PMU_CHECK_LAUNCH();
    hipLaunchKernelGGL(fcomb_dzb_reduce_kernel, dim3((unsigned)pmu_cdiv((long long)N * FW, 256)), dim3(256), 0, st0,
                       slab, N, HW, geo, dzb);
    PMU_CHECK_LAUNCH();
    hipLaunchKernelGGL(fcomb_zgrad_kernel, dim3((unsigned)pmu_cdiv(F + F * L + (long long)N * L, 256)), dim3(256), 0,
                       st0, dzb, z, N, p, o);
    PMU_CHECK_LAUNCH();
    return PMU_OK;
  }
  const long long ntiles = ((long long)N * HW + BT - 1) / BT;
  const int nb = fcomb_bwd_blocks(ntiles);
  FcombG gg;
  gg.dfeat = dfeat;
  gg.ws = ws;
  gg.dzb = ws + (size_t)nb * WS_BLOCK;
  float* dzb = gg.dzb + (size_t)nb * N * FW;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(fcomb_bwd_kernel, dim3((unsigned)nb), dim3(256), 0, st, feat, zb, dl, p, N, HW, gg, ntiles);
  PMU_CHECK_LAUNCH();
  hipLaunchKernelGGL(fcomb_reduce_kernel, dim3((unsigned)pmu_cdiv(WS_BLOCK + (long long)N * FW, 256)), dim3(256), 0, st,
                     ws, gg.dzb, nb, N, p, o, dzb);
  PMU_CHECK_LAUNCH();
  hipLaunchKernelGGL(fcomb_zgrad_kernel, dim3((unsigned)pmu_cdiv(F + F * L + (long long)N * L, 256)), dim3(256), 0, st,
                     dzb, z, N, p, o);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_spatial_mean(const float* z, const float* coef, int N, int H, int W, int C, float* out,
                                void* stream) {
  PMU_REQUIRE(z && coef && out && N > 0 && H > 0 && W > 0 && C > 0);
  hipLaunchKernelGGL(spatial_mean_kernel, dim3((unsigned)pmu_cdiv(C, 64), (unsigned)N), dim3(256), 0,
                     (hipStream_t)stream, z, coef, N, H * W, C, out);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_spatial_mean_bwd(const float* dmean, int N, int H, int W, int C, float* da, void* stream) {
  PMU_REQUIRE(dmean && da && N > 0 && H > 0 && W > 0 && C > 0);
  const long long total = (long long)N * H * W * C;
  const long long g = total / 256 + 1 < 4096 ? total / 256 + 1 : 4096;
  hipLaunchKernelGGL(spatial_mean_bwd_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, dmean, N, H * W, C,
                     da);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_linear_fwd(const float* x, const float* w, const float* b, int N, int K, int M, float* y,
                              void* stream) {
  PMU_REQUIRE(x && w && y && N > 0 && K > 0 && M > 0 && N <= 65535);
  hipLaunchKernelGGL(linear_fwd_kernel, dim3((unsigned)M, (unsigned)N), dim3(256), 0, (hipStream_t)stream, x, w, b, N,
                     K, M, y);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_linear_bwd(const float* x, const float* w, const float* dy, int N, int K, int M, float* dx, float* dw,
                              float* db, void* stream) {
  PMU_REQUIRE(x && w && dy && dw && N > 0 && K > 0 && M > 0 && M <= 256);
  hipLaunchKernelGGL(linear_bwd_kernel, dim3((unsigned)pmu_cdiv(K, 256)), dim3(256), 0, (hipStream_t)stream, x, w, dy,
                     N, K, M, dx, dw, db);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
