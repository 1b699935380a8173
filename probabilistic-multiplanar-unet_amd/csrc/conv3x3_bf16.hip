// 3x3 / pad 1 convolution on gfx950 bf16 MFMA (v_mfma_f32_32x32x16_bf16): config c5's precision
// (BASELINE.json configs[4]: "5-level U-Net base=64ch bf16").
//
// Same operator and fusion as conv3x3.hip (nn.Conv2d(k=3, padding=1) of DoubleConv / Encoder,
// PMU/model/unet/unet_parts.py:15,18, PMU/model/probabilistic_unet/probabilistic_unet.py:38,43,
// with the producer's BatchNorm2d + ReLU (+ MaxPool2d(2) | AvgPool2d(2, ceil) | F.pad + torch.cat)
// applied while the operand is staged), with the arithmetic split as torch.autocast(bfloat16) does
// it: operands rounded to bf16 (RNE) after the fp32 BN/ReLU/pool transform, products summed in
// fp32, outputs (pre-BN z, BN partial sums, dx) written in fp32.
//
// GEMM view as conv3x3.hip (M = pixels, N = output channels, K = 9 x input channels).
// Block: 256 threads = 4 waves, 2 blocks per CU (<= 72 KB LDS each).  Tile: 256 pixels (TH x TW)
// x BNT output channels (64 or 128); per chunk of BK = 16 input channels one (TH+2) x (TW+2) bf16
// halo tile and 9 taps x BNT x 16 bf16 weights are staged, then every tap is ONE k-step of 16:
// lane half h reads k = 8h..8h+7 of its row with one ds_read_b128 (48-B rows: conflict-free for
// any 16 consecutive rows).  Wave layout: BNT = 128 -> 2 (pixels) x 2 (channels) waves of 128 px x
// 64 ch = 4 x 2 accumulators; BNT = 64 -> 4 x 1 waves of 64 px x 64 ch = 2 x 2 accumulators.
#include <cstdlib>

#include "pmu_stage.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BM = 256;      // pixels per tile
constexpr int BK = 16;       // reduction channels per chunk (= one MFMA k-step per tap)
constexpr int LSB = 24;      // LDS row stride in bf16 (32 B of data + 16 B pad)
constexpr int MAX_HP = 340;  // max halo pixels: (8+2)*(32+2) = 340
constexpr int NI = 6;        // A items per thread: ceil(340*4 / 256)
constexpr int PJ = 64;       // packed-weight row block
constexpr int A_ELEMS = MAX_HP * LSB;

struct ConvArgsB {
  DevFrame in;
  const unsigned short* wp;  // packed bf16 weights [jb][ch][tap][PJ][BK]
  const float* bias;
  float* out0;
  float* out1;
  float* part;
  unsigned short* tee;       // optional bf16 copy of the operand [N][H][W][pad8(KC)] (blockIdx.y == 0 writes)
  int NOUT, KC, split, tiles_w, tiles_h;
};

// Copy the staged chunk's interior pixels (the operand itself, already transformed and rounded to
// bf16) from LDS to the tee tensor: the weight-gradient kernel reads these instead of
// re-materialising the operand (pmu_frame_to_bf16).  512 units of 8 channels per chunk.
template <int TWL>
__device__ __forceinline__ void tee_chunk(const ConvArgsB& a, const unsigned short* As, int k0, int n, int h0, int w0,
                                          int tid) {
  constexpr int TW = 1 << TWL, HW2 = TW + 2;
  const int Cp = (a.KC + 7) & ~7;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int u = tid + 256 * i;
    const int q = u >> 1, half = u & 1;
    const int r = q >> TWL, c = q & (TW - 1);
    const int h = h0 + r, w = w0 + c, ch = k0 + 8 * half;
    if (h < a.in.H && w < a.in.W && ch < a.KC) {
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = *reinterpret_cast<const u32x4*>(As + ((r + 1) * HW2 + c + 1) * LSB + 8 * half);
      // streamed past the caches: read back only by the backward's weight-gradient kernel
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(a.tee + (((long long)n * a.in.H + h) * a.in.W + w) * Cp + ch));
    }
  }
}

__device__ __forceinline__ unsigned short bf16_bits(float v) {
  return __builtin_bit_cast(unsigned short, (__bf16)v);
}

// wp[jb][ch][tap][jl][kl] = B[tap][j = jb*PJ + jl][k = ch*BK + kl] (zero padded), bf16 RNE.
//   forward: B[tap][co][ci] = w[co][ci][tap];  dgrad: B[tap][ci][co] = w[co][ci][8 - tap]
__global__ __launch_bounds__(256) void pack_w_bf16_kernel(const float* __restrict__ w, int Cout, int Cin, int dgrad,
                                                          int njb, unsigned short* __restrict__ wp) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  const int nch = (KC + BK - 1) / BK;
  const long long total = (long long)njb * nch * 9 * PJ * BK;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int kl = (int)(e % BK);
    long long r = e / BK;
    const int jl = (int)(r % PJ); r /= PJ;
    const int tap = (int)(r % 9); r /= 9;
    const int ch = (int)(r % nch);
    const int jb = (int)(r / nch);
    const int j = jb * PJ + jl, k = ch * BK + kl;
    float v = 0.f;
    if (j < NOUT && k < KC)
      v = dgrad ? w[((long long)k * Cin + j) * 9 + (8 - tap)] : w[((long long)j * Cin + k) * 9 + tap];
    wp[e] = bf16_bits(v);
  }
}

static int packed_row_blocks(int NOUT) { return 2 * pmu_cdiv(NOUT, 2 * PJ); }

template <int TWL, int BNT, bool DGRAD>
__global__ __launch_bounds__(256, 2) void conv3x3_bf16_kernel(ConvArgsB a) {
  constexpr int FM = (BNT == 128) ? 4 : 2;  // pixel fragments per wave
  constexpr int FN = 2;                     // channel fragments per wave
  constexpr int WM = BM / (32 * FM);        // waves along pixels
  constexpr int TW = 1 << TWL, TH = BM >> TWL, HW2 = TW + 2, HP = (TH + 2) * HW2;
  constexpr int B_ELEMS = 9 * BNT * LSB;
  __shared__ __attribute__((aligned(16))) unsigned short smem[A_ELEMS + B_ELEMS];
  unsigned short* As = smem;
  unsigned short* Bs = smem + A_ELEMS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  int t = blockIdx.x;
  const int tw = t % a.tiles_w; t /= a.tiles_w;
  const int th = t % a.tiles_h; t /= a.tiles_h;
  const int n = t;
  const int h0 = th * TH, w0 = tw * TW;
  const int j0 = blockIdx.y * BNT;
  const DevFrame& F = a.in;
  const int nch = (a.KC + BK - 1) / BK;

  int ih[NI], iw[NI], dst[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int it = tid + 256 * i;
    const int hp = it >> 2;
    const int hr = hp / HW2, hc = hp - hr * HW2;
    ih[i] = (it < HP * 4) ? h0 - 1 + hr : PMU_NO_ITEM;
    iw[i] = w0 - 1 + hc;
    dst[i] = hp * LSB + 4 * (it & 3);
  }
  const int hsel = (lane >> 5) * 8;
  int abase[FM], bbase[FN];
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    const int q = wm * 32 * FM + fm * 32 + (lane & 31);
    abase[fm] = ((q >> TWL) * HW2 + (q & (TW - 1))) * LSB + hsel;
  }
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) bbase[fn] = (wn * 64 + fn * 32 + (lane & 31)) * LSB + hsel;

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // packed B: this block's BNT/PJ row blocks of one chunk, 16-B units (2 per row)
  constexpr int UNITS = 9 * BNT * 2;
  const uint4* wsrc = reinterpret_cast<const uint4*>(a.wp);
  const long long tile_units = 9LL * PJ * BK / 8;
  const int jb0 = j0 / PJ;

  for (int ch = 0; ch < nch; ++ch) {
    stage_items<NI, true>(F, n, ch * BK, BK, tid & 3, ih, iw, dst, As);
#pragma unroll
    for (int i = 0; i < (UNITS + 255) / 256; ++i) {
      const int u = tid + 256 * i;
      if (UNITS % 256 == 0 || u < UNITS) {
        const int hh = u / (9 * PJ * 2);        // row block inside the block
        const int uu = u - hh * (9 * PJ * 2);
        const int row = uu >> 1, qq = uu & 1;   // row = tap*PJ + jl
        const int tap = row / PJ, jl = row - tap * PJ;
        const uint4 v = wsrc[((long long)(jb0 + hh) * nch + ch) * tile_units + uu];
        *reinterpret_cast<uint4*>(Bs + (tap * BNT + hh * PJ + jl) * LSB + 8 * qq) = v;
      }
    }
    __syncthreads();
    if (a.tee && blockIdx.y == 0) tee_chunk<TWL>(a, As, ch * BK, n, h0, w0, tid);

    // BNT = 64: the next tap's operands are read ahead of the current tap's MFMAs; BNT = 128 has
    // no registers for a second set (the partner wave on the SIMD covers the read latency)
    constexpr int NB = (BNT == 128) ? 1 : 2;
    bf16x8 op[NB][FM + FN];
    auto load_ops = [&](int tap, bf16x8 (&o)[FM + FN]) {
      const int toff = ((tap / 3) * HW2 + (tap % 3)) * LSB;
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) o[fm] = *reinterpret_cast<const bf16x8*>(As + abase[fm] + toff);
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) o[FM + fn] = *reinterpret_cast<const bf16x8*>(Bs + tap * BNT * LSB + bbase[fn]);
    };
    if (NB == 2) load_ops(0, op[0]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (NB == 1) load_ops(tap, op[0]);
      else if (tap + 1 < 9) load_ops(tap + 1, op[(tap + 1) % NB]);
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(op[tap % NB][fm], op[tap % NB][FM + fn], acc[fm][fn], 0, 0, 0);
    }
    __syncthreads();
  }

  // epilogue: fwd writes z (+bias) and per-tile BN partials; dgrad writes dx split in two
  float* red = reinterpret_cast<float*>(smem);  // [WM][BNT][2]
  float s1[FN], s2[FN];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    s1[fn] = 0.f; s2[fn] = 0.f;
    const int j = j0 + wn * 64 + fn * 32 + (lane & 31);
    const bool jok = j < a.NOUT;
    const float b = (!DGRAD && jok && a.bias) ? a.bias[j] : 0.f;
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = wm * 32 * FM + fm * 32 + acc_row(r, lane);
        const int h = h0 + (q >> TWL), w = w0 + (q & (TW - 1));
        if (!jok || h >= F.H || w >= F.W) continue;
        const long long pix = ((long long)n * F.H + h) * F.W + w;
        const float v = acc[fm][fn][r] + b;
        if (!DGRAD) {
          a.out0[pix * a.NOUT + j] = v;
          s1[fn] += v;
          s2[fn] = fmaf(v, v, s2[fn]);
        } else if (j < a.split) {
          a.out0[pix * a.split + j] = v;
        } else {
          a.out1[pix * (a.NOUT - a.split) + (j - a.split)] = v;
        }
      }
    }
  }
  if (!DGRAD && a.part) {
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      s1[fn] += __shfl_xor(s1[fn], 32, 64);
      s2[fn] += __shfl_xor(s2[fn], 32, 64);
      if (lane < 32) {
        const int jj = wn * 64 + fn * 32 + lane;
        red[(wm * BNT + jj) * 2 + 0] = s1[fn];
        red[(wm * BNT + jj) * 2 + 1] = s2[fn];
      }
    }
    __syncthreads();
    if (tid < BNT) {
      const int j = j0 + tid;
      if (j < a.NOUT) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int v = 0; v < WM; ++v) {
          t1 += red[(v * BNT + tid) * 2 + 0];
          t2 += red[(v * BNT + tid) * 2 + 1];
        }
        a.part[((long long)blockIdx.x * 2 + 0) * a.NOUT + j] = t1;
        a.part[((long long)blockIdx.x * 2 + 1) * a.NOUT + j] = t2;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Software-pipelined variant (2 blocks/CU, BNT = 64): chunk c+1's global loads (A items and the
// packed B tile) are issued into registers before chunk c's 9 x 4 MFMAs and transformed/written
// to LDS after them.  At bf16 rates a chunk's MFMAs last ~1 us, so the synchronous kernel above
// pays the full global-load latency per chunk; here it hides under the MFMAs, and the partner
// block's MFMAs cover this block's commit phase.  Operand modes are template parameters.
// ---------------------------------------------------------------------------------------------
constexpr int PB_UNITS = 9 * 64 * 2;               // 16-B units of a BNT = 64 B tile
constexpr int PB_N = (PB_UNITS + 255) / 256;       // 5 (the last one for tid < 128)

// Lean staging for the pipelined kernel: the items' pixel offsets inside the current source are
// tile constants, computed once per source (32-bit element offsets: the host routes tensors of
// >= 2^31 elements to the synchronous kernel), so a chunk's prefetch is NI (x2 for BN-backward)
// float4 loads at offset + channel and its commit one transform per item — no per-item 64-bit
// index arithmetic or divergent bounds branches in the pipelined loop.
template <int TWL>
__device__ __forceinline__ void item_offsets(const DevSrc& s, int n, int h0, int w0, int tid, int (&eo)[NI],
                                             unsigned& okm) {
  constexpr int TW = 1 << TWL, TH = BM >> TWL, HW2 = TW + 2, HP = (TH + 2) * HW2;
  okm = 0u;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int it = tid + 256 * i;
    const int hp = it >> 2;
    const int hr = hp / HW2, hc = hp - hr * HW2;
    const int hs = h0 - 1 + hr - s.off_h, ws = w0 - 1 + hc - s.off_w;
    const bool ok = it < HP * 4 && hs >= 0 && ws >= 0 && hs < s.H && ws < s.W;
    okm |= ok ? (1u << i) : 0u;
    eo[i] = ok ? ((n * s.H + hs) * s.W + ws) * s.C : 0;
  }
}

template <bool DGRAD, int POOL, int TWL>
__global__ __launch_bounds__(256, 2) void conv3x3_bf16_pipe_kernel(ConvArgsB a) {
  static_assert(POOL == PMU_POOL_NONE, "pooled sources are materialised (pmu_frame_to_f32) in bf16 mode");
  constexpr int BNT = 64, FM = 2, FN = 2, WM = 4;
  constexpr int TW = 1 << TWL, TH = BM >> TWL, HW2 = TW + 2, HP = (TH + 2) * HW2;
  __shared__ __attribute__((aligned(16))) unsigned short smem[A_ELEMS + 9 * BNT * LSB];
  unsigned short* As = smem;
  unsigned short* Bs = smem + A_ELEMS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave;
  int t = blockIdx.x;
  const int tw = t % a.tiles_w; t /= a.tiles_w;
  const int th = t % a.tiles_h; t /= a.tiles_h;
  const int n = t;
  const int h0 = th * TH, w0 = tw * TW;
  const int j0 = blockIdx.y * BNT;
  const DevFrame& F = a.in;
  const int nch = (a.KC + BK - 1) / BK;
  const int cq4 = 4 * (tid & 3);

  int dst[NI];
  unsigned vm = 0u;  // items this thread stages at all
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int it = tid + 256 * i;
    dst[i] = (it >> 2) * LSB + 4 * (it & 3);
    vm |= (it < HP * 4) ? (1u << i) : 0u;
  }
  const int hsel = (lane >> 5) * 8;
  int abase[FM], bbase[FN];
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    const int q = wm * 32 * FM + fm * 32 + (lane & 31);
    abase[fm] = ((q >> TWL) * HW2 + (q & (TW - 1))) * LSB + hsel;
  }
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) bbase[fn] = (fn * 32 + (lane & 31)) * LSB + hsel;

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // current source (s0 first, then s1 of a concat frame) and its tile-constant item offsets
  int eo[NI];
  unsigned okm;
  int second = 0;
  const float* sx = F.s0.x;
  const float* sz = F.s0.z;
  const float* sco = F.s0.coef;
  int sC = F.s0.C, sraw = F.s0.mode == PMU_SRC_RAW;
  item_offsets<TWL>(F.s0, n, h0, w0, tid, eo, okm);

  float4 px0, px1, px2, px3, px4, px5;  // prefetched operand items (plain locals: no scratch)
  float4 pz0, pz1, pz2, pz3, pz4, pz5;  // BN-backward: z of the same items
  float4 psc, psh, pmu, pkx, pkc;
  uint4 pb0, pb1, pb2, pb3, pb4;
  const uint4* wtile = reinterpret_cast<const uint4*>(a.wp) + (long long)(j0 / PJ) * nch * (9 * PJ * BK / 8);
  const bool b4 = tid < PB_UNITS - 4 * 256;
  static_assert(PB_N == 5 && NI == 6, "staging register layout");
#define PMU_X(I) (*reinterpret_cast<const float4*>(sx + (unsigned)(eo[I] + c_)))
#define PMU_Z(I) (*reinterpret_cast<const float4*>(sz + (unsigned)(eo[I] + c_)))
#define PMU_PREFETCH(CH)                                                                         \
  {                                                                                             \
    const int k0_ = (CH) * BK;                                                                  \
    if (F.nsrc > 1 && !second && k0_ >= F.C0) { /* uniform: switch to the concat's 2nd source */ \
      second = 1;                                                                               \
      sx = F.s1.x; sz = F.s1.z; sco = F.s1.coef; sC = F.s1.C; sraw = F.s1.mode == PMU_SRC_RAW;  \
      item_offsets<TWL>(F.s1, n, h0, w0, tid, eo, okm);                                         \
    }                                                                                           \
    const int c_ = k0_ - (second ? F.C0 : 0) + cq4;                                             \
    px0 = PMU_X(0); px1 = PMU_X(1); px2 = PMU_X(2); px3 = PMU_X(3); px4 = PMU_X(4); px5 = PMU_X(5); \
    if (DGRAD) {                                                                                \
      pz0 = PMU_Z(0); pz1 = PMU_Z(1); pz2 = PMU_Z(2); pz3 = PMU_Z(3); pz4 = PMU_Z(4); pz5 = PMU_Z(5); \
      pmu = *reinterpret_cast<const float4*>(sco + 2 * sC + c_);                                \
      pkx = *reinterpret_cast<const float4*>(sco + 3 * sC + c_);                                \
      pkc = *reinterpret_cast<const float4*>(sco + 4 * sC + c_);                                \
    }                                                                                           \
    if (DGRAD || !sraw) {                                                                       \
      psc = *reinterpret_cast<const float4*>(sco + c_);                                         \
      psh = *reinterpret_cast<const float4*>(sco + sC + c_);                                    \
    }                                                                                           \
    const uint4* src_ = wtile + (long long)(CH) * (9 * PJ * BK / 8) + tid;                      \
    pb0 = src_[0]; pb1 = src_[256]; pb2 = src_[512]; pb3 = src_[768];                           \
    pb4 = src_[b4 ? 1024 : 0];                                                                  \
  }
#define PMU_ITEM(I, X, Z)                                                                        \
  if ((vm >> (I)) & 1u) {                                                                       \
    float4 v_;                                                                                  \
    if (DGRAD) {                                                                                \
      v_ = make_float4(pmu_bnbwd1(X.x, Z.x, psc.x, psh.x, pmu.x, pkx.x, pkc.x),                 \
                       pmu_bnbwd1(X.y, Z.y, psc.y, psh.y, pmu.y, pkx.y, pkc.y),                 \
                       pmu_bnbwd1(X.z, Z.z, psc.z, psh.z, pmu.z, pkx.z, pkc.z),                 \
                       pmu_bnbwd1(X.w, Z.w, psc.w, psh.w, pmu.w, pkx.w, pkc.w));                \
    } else {                                                                                    \
      v_ = sraw ? X : pmu_bnrelu4(X, psc, psh);                                                 \
    }                                                                                           \
    if (!((okm >> (I)) & 1u)) v_ = make_float4(0.f, 0.f, 0.f, 0.f);                             \
    pmu_lds_store4<true>(As, dst[I], v_);                                                       \
  }
#define PMU_COMMIT()                                                                             \
  {                                                                                             \
    PMU_ITEM(0, px0, pz0) PMU_ITEM(1, px1, pz1) PMU_ITEM(2, px2, pz2)                           \
    PMU_ITEM(3, px3, pz3) PMU_ITEM(4, px4, pz4) PMU_ITEM(5, px5, pz5)                           \
    *reinterpret_cast<uint4*>(Bs + ((tid) >> 1) * LSB + 8 * ((tid) & 1)) = pb0;                 \
    *reinterpret_cast<uint4*>(Bs + ((tid + 256) >> 1) * LSB + 8 * ((tid) & 1)) = pb1;           \
    *reinterpret_cast<uint4*>(Bs + ((tid + 512) >> 1) * LSB + 8 * ((tid) & 1)) = pb2;           \
    *reinterpret_cast<uint4*>(Bs + ((tid + 768) >> 1) * LSB + 8 * ((tid) & 1)) = pb3;           \
    if (b4) *reinterpret_cast<uint4*>(Bs + ((tid + 1024) >> 1) * LSB + 8 * ((tid) & 1)) = pb4;  \
  }

  const bool tee = a.tee && blockIdx.y == 0;
  PMU_PREFETCH(0)
  PMU_COMMIT()
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const bool more = ch + 1 < nch;
    if (more) PMU_PREFETCH(ch + 1)  // in flight during the MFMAs below
    if (tee) tee_chunk<TWL>(a, As, ch * BK, n, h0, w0, tid);
    bf16x8 op[2][FM + FN];
    auto load_ops = [&](int tap, bf16x8 (&o)[FM + FN]) {
      const int toff = ((tap / 3) * HW2 + (tap % 3)) * LSB;
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) o[fm] = *reinterpret_cast<const bf16x8*>(As + abase[fm] + toff);
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) o[FM + fn] = *reinterpret_cast<const bf16x8*>(Bs + tap * BNT * LSB + bbase[fn]);
    };
    load_ops(0, op[0]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap + 1 < 9) load_ops(tap + 1, op[(tap + 1) & 1]);
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(op[tap & 1][fm], op[tap & 1][FM + fn], acc[fm][fn], 0, 0, 0);
    }
    __syncthreads();
    if (more) {
      PMU_COMMIT()
      __syncthreads();
    }
  }
#undef PMU_PREFETCH
#undef PMU_COMMIT
#undef PMU_ITEM
#undef PMU_X
#undef PMU_Z

  // epilogue (as conv3x3_bf16_kernel with WN = 1).  Per channel block of 32 the destination
  // (z, or the dx half the channels fall in: split % 32 == 0, host-checked) is uniform; in a full
  // tile every element is stored without bounds tests, addressed from one 32-bit pixel base per
  // fragment row plus compile-time pixel offsets.
  float* red = reinterpret_cast<float*>(smem);
  float s1[FN], s2[FN];
  const bool full = h0 + TH <= F.H && w0 + TW <= F.W && j0 + BNT <= a.NOUT;
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    s1[fn] = 0.f; s2[fn] = 0.f;
    const int jb = j0 + fn * 32;
    const int j = jb + (lane & 31);
    const bool jok = j < a.NOUT;
    const float b = (!DGRAD && jok && a.bias) ? a.bias[j] : 0.f;
    float* dstp;
    int ld;
    if (!DGRAD) { dstp = a.out0 + j; ld = a.NOUT; }
    else if (jb < a.split) { dstp = a.out0 + j; ld = a.split; }
    else { dstp = a.out1 + (j - a.split); ld = a.NOUT - a.split; }
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = wm * 32 * FM + fm * 32 + acc_row(r, lane);
        const int h = h0 + (q >> TWL), w = w0 + (q & (TW - 1));
        if (!full && (!jok || h >= F.H || w >= F.W)) continue;
        const unsigned pix = (unsigned)((n * F.H + h) * F.W + w);
        const float v = acc[fm][fn][r] + b;
        dstp[(size_t)pix * (unsigned)ld] = v;
        if (!DGRAD) {
          s1[fn] += v;
          s2[fn] = fmaf(v, v, s2[fn]);
        }
      }
    }
  }
  if (!DGRAD && a.part) {
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      s1[fn] += __shfl_xor(s1[fn], 32, 64);
      s2[fn] += __shfl_xor(s2[fn], 32, 64);
      if (lane < 32) {
        red[(wm * BNT + fn * 32 + lane) * 2 + 0] = s1[fn];
        red[(wm * BNT + fn * 32 + lane) * 2 + 1] = s2[fn];
      }
    }
    __syncthreads();
    if (tid < BNT) {
      const int j = j0 + tid;
      if (j < a.NOUT) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int v = 0; v < WM; ++v) {
          t1 += red[(v * BNT + tid) * 2 + 0];
          t2 += red[(v * BNT + tid) * 2 + 1];
        }
        a.part[((long long)blockIdx.x * 2 + 0) * a.NOUT + j] = t1;
        a.part[((long long)blockIdx.x * 2 + 1) * a.NOUT + j] = t2;
      }
    }
  }
}

// sources the pipelined staging handles: float4 channels, chunks never straddle sources
static bool pipe_src_ok(const pmu_src& s) {
  if (s.C % BK != 0) return false;
  if (s.pool == PMU_POOL_NONE) return true;
  return s.pool == PMU_POOL_MAX2 && s.mode == PMU_SRC_BNRELU;
}

static int pick_twl(int W) {
  if (W > 16) return 5;
  if (W > 8) return 4;
  return 3;
}

static int launch_bf16(const pmu_frame* in, const unsigned short* wp, const float* bias, int NOUT, int KC, float* out0,
                       float* out1, int split, float* part, unsigned short* tee, bool dgrad, void* stream) {
  ConvArgsB a;
  a.in = make_dev_frame(in);
  a.wp = wp; a.bias = bias; a.out0 = out0; a.out1 = out1; a.part = part; a.tee = tee;
  a.NOUT = NOUT; a.KC = KC; a.split = split;
  const int twl = pick_twl(in->W);
  const int TW = 1 << twl, TH = BM / TW;
  a.tiles_w = pmu_cdiv(in->W, TW);
  a.tiles_h = pmu_cdiv(in->H, TH);
  const int bnt = 64;  // BNT = 128 needs the 1-block/CU pipelined variant (register budget)
  dim3 grid((unsigned)(a.tiles_w * a.tiles_h * in->N), (unsigned)pmu_cdiv(NOUT, bnt));
  hipStream_t st = (hipStream_t)stream;
  {
    const pmu_src& s0 = in->src[0];
    const bool two = in->nsrc > 1;
    const pmu_src& s1 = in->src[1];
    const int pool = s0.pool;
    const bool ok = pipe_src_ok(s0) && (!two || (pipe_src_ok(s1) && s1.pool == pool));
    const bool modes_ok = dgrad ? (!two && s0.mode == PMU_SRC_BNBWD)
                                : (s0.mode != PMU_SRC_BNBWD && (!two || s1.mode != PMU_SRC_BNBWD));
    // 32-bit item offsets inside every source, 32-bit pixel indices of the output
    const bool small = (long long)s0.C * s0.H * s0.W * in->N < (1LL << 31) &&
                       (!two || (long long)s1.C * s1.H * s1.W * in->N < (1LL << 31)) &&
                       (long long)in->N * in->H * in->W < (1LL << 31);
    const bool split_ok = !dgrad || split % 32 == 0 || split == NOUT;
    if (ok && modes_ok && small && split_ok && pool == PMU_POOL_NONE && !pmu_variant_env("PMU_BF16_NOPIPE")) {
#define PMU_BP(D, P, T)                                                                    \
  if (dgrad == D && pool == P && twl == T) {                                               \
    hipLaunchKernelGGL((conv3x3_bf16_pipe_kernel<D, P, T>), grid, dim3(256), 0, st, a);    \
    PMU_CHECK_LAUNCH();                                                                    \
    return PMU_OK;                                                                         \
  }
      PMU_BP(false, PMU_POOL_NONE, 3) PMU_BP(false, PMU_POOL_NONE, 4) PMU_BP(false, PMU_POOL_NONE, 5)
      PMU_BP(true, PMU_POOL_NONE, 3) PMU_BP(true, PMU_POOL_NONE, 4) PMU_BP(true, PMU_POOL_NONE, 5)
#undef PMU_BP
    }
  }
#define PMU_BF(T, B, D)                                                              \
  if (twl == T && bnt == B && dgrad == D) {                                            \
    hipLaunchKernelGGL((conv3x3_bf16_kernel<T, B, D>), grid, dim3(256), 0, st, a);     \
    PMU_CHECK_LAUNCH();                                                                \
    return PMU_OK;                                                                     \
  }
  PMU_BF(3, 64, false) PMU_BF(4, 64, false) PMU_BF(5, 64, false)
  PMU_BF(3, 64, true) PMU_BF(4, 64, true) PMU_BF(5, 64, true)
#undef PMU_BF
  return PMU_ERR_ARG;
}

}  // namespace

// rows of the fused-staging convs' BN partial sums part[tile][2][Cout]: tiles of BM = 256 pixels, 32, 16 or
// 8 wide (pick_twl) — the bf16 kernels here, and the experiments build's fp32 direct-sum conv
extern "C" int pmu_conv3x3_tiles(int N, int H, int W) {
  const int twl = pick_twl(W);
  const int TW = 1 << twl, TH = BM / TW;
  return N * pmu_cdiv(H, TH) * pmu_cdiv(W, TW);
}

extern "C" size_t pmu_conv3x3_packed_size_bf16(int Cout, int Cin, int dgrad) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  return (size_t)packed_row_blocks(NOUT) * pmu_cdiv(KC, BK) * 9 * PJ * BK * sizeof(unsigned short);
}

extern "C" int pmu_conv3x3_pack_bf16(const float* w, int Cout, int Cin, int dgrad, unsigned short* wp, void* stream) {
  PMU_REQUIRE(w && wp && Cout > 0 && Cin > 0);
  const int NOUT = dgrad ? Cin : Cout;
  const long long total = (long long)(pmu_conv3x3_packed_size_bf16(Cout, Cin, dgrad) / sizeof(unsigned short));
  long long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(pack_w_bf16_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, dgrad,
                     packed_row_blocks(NOUT), wp);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_conv3x3_fwd_bf16(const pmu_frame* in, const unsigned short* wp, const float* bias, int Cout,
                                    float* z, float* part, unsigned short* tee, void* stream) {
  PMU_REQUIRE(valid_frame(in) && wp && z && Cout > 0);
  const int Cin = in->src[0].C + (in->nsrc > 1 ? in->src[1].C : 0);
  return launch_bf16(in, wp, bias, Cout, Cin, z, nullptr, Cout, part, tee, false, stream);
}

extern "C" int pmu_conv3x3_dgrad_bf16(const pmu_frame* dz, const unsigned short* wp, int Cin, int Csplit, float* dx0,
                                      float* dx1, unsigned short* tee, void* stream) {
  PMU_REQUIRE(valid_frame(dz) && dz->nsrc == 1 && wp && dx0 && Cin > 0);
  PMU_REQUIRE(Csplit > 0 && Csplit <= Cin && (Csplit == Cin || dx1));
  return launch_bf16(dz, wp, nullptr, Cin, dz->src[0].C, dx0, dx1, Csplit, nullptr, tee, true, stream);
}
