// 3x3 / pad 1 convolution as an implicit GEMM on gfx950 f32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces nn.Conv2d(k=3, padding=1) of DoubleConv / Encoder
// (PMU/model/unet/unet_parts.py:15,18; PMU/model/probabilistic_unet/probabilistic_unet.py:38,43)
// together with the producer's BatchNorm2d + ReLU (+ MaxPool2d(2) | AvgPool2d(2, ceil) |
// F.pad + torch.cat) applied while the operand is staged (unet_parts.py:16-20,33,58-66).
//
// GEMM view (forward):  M = output pixels, N = Cout, K = 9 * Cin.
//   Per K chunk of BK input channels ONE (TH+2) x (TW+2) halo tile of the transformed input is
//   staged in LDS; all 9 taps read shifted windows of it (im2col-free).  Weights of the chunk
//   are staged as B[tap][cout][k] from a pre-packed copy (pmu_conv3x3_pack) by straight copy.
// GEMM view (input gradient, "dgrad"): the same kernel with the roles of Cin/Cout swapped and
//   the taps flipped: dx[p][ci] = sum_{tap,co} dz[p + d(tap)][co] * w[co][ci][8 - tap].
//
// Block: 256 threads (4 waves), 2 blocks per CU (73 KB LDS each) so one block's staging overlaps
// the other's MFMAs.  Tile: 256 pixels (TH x TW, TW in {32,16,8}) x 64 output channels; wave w
// owns pixels [64w, 64w+64) x 64 channels = 2 x 2 32x32 accumulators.
// LDS rows are k-contiguous (BK = 16 floats + 4 pad): lane half h reads k = 8h..8h+7 with two
// ds_read_b128 and feeds one k per MFMA step (the K order inside a chunk is free as long as A
// and B agree), conflict-free for 16 consecutive rows.  The next tap's 8 reads are issued ahead
// of the current tap's 32 MFMAs.
#include <cstdlib>
#include <cstring>

#include "pmu_stage.h"

// The direct-sum fp32 conv is the engine's PMU_FP32_CONV=direct A/B only (the default fp32 path is
// Winograd on every shape: conv3x3_wino2h.hip, conv3x3_wino4.hip, and conv3x3_wino.hip's fused
// kernels for channel counts off the 16 grid): experiments build only.
#ifdef PMU_EXPERIMENTS

namespace {

constexpr int BM = 256;     // pixels per tile
constexpr int BN = 64;      // output channels per tile
constexpr int BK = 16;      // reduction channels per chunk
constexpr int LS = BK + 4;  // LDS row stride (floats)
constexpr int MAX_HP = 340; // max halo pixels: (8+2)*(32+2) = (32+2)*(8+2) = 340, (16+2)^2 = 324
constexpr int A_FLOATS = MAX_HP * LS;
constexpr int STAGE = A_FLOATS + 9 * BN * LS;
constexpr int NI = 6;       // A items per thread: ceil(340*4 / 256)

struct ConvArgs {
  DevFrame in;       // operand frame (fwd: activation; dgrad: dz)
  const float* w;    // [Cout][Cin][3][3] (PyTorch layout)
  const float* wp;   // packed weights (pack_w_kernel layout) or null
  const float* bias; // fwd only
  float* out0;       // fwd: z [N][H][W][NOUT]; dgrad: dx channels [0, split)
  float* out1;       // dgrad: dx channels [split, NOUT)
  float* part;       // fwd BN partials [tiles][2][NOUT] or null
  float* tee;        // optional copy of the staged operand [N][H][W][KC] (blockIdx.y == 0 writes)
  int NOUT, KC;      // GEMM N (output channels) and reduction channels
  int split;         // dgrad channel split
  int twl;           // log2(TW)
  int tiles_w, tiles_h;
};

// Packed weights: wp[jb][ch][tap][jl][kl] (jb = N block of BN, ch = K chunk of BK), zero padded,
// i.e. each block's B tile of one chunk is 9*BN*BK contiguous floats in LDS order.
//   forward: B[tap][j=co][k=ci] = w[co][ci][tap];  dgrad: B[tap][j=ci][k=co] = w[co][ci][8-tap]
__global__ __launch_bounds__(256) void pack_w_kernel(const float* __restrict__ w, int Cout, int Cin, int dgrad,
                                                     float* __restrict__ wp) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  const int nch = (KC + BK - 1) / BK;
  const long long tile = 9LL * BN * BK;
  const long long total = (long long)((NOUT + BN - 1) / BN) * nch * tile;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int kl = (int)(e % BK);
    long long r = e / BK;
    const int jl = (int)(r % BN); r /= BN;
    const int tap = (int)(r % 9); r /= 9;
    const int ch = (int)(r % nch);
    const int jb = (int)(r / nch);
    const int j = jb * BN + jl, k = ch * BK + kl;
    float v = 0.f;
    if (j < NOUT && k < KC)
      v = dgrad ? w[((long long)k * Cin + j) * 9 + (8 - tap)] : w[((long long)j * Cin + k) * 9 + tap];
    wp[e] = v;
  }
}

// stage chunk k0 of the B operand (9 taps x BN x BK) into Bs
template <bool DGRAD>
__device__ __forceinline__ void stage_B(const ConvArgs& a, int j0, int k0, float* Bs, int tid) {
  if (a.wp) {  // straight copy of the packed tile into padded rows
    const int nch = (a.KC + BK - 1) / BK;
    const float4* src = reinterpret_cast<const float4*>(a.wp + ((long long)(j0 / BN) * nch + k0 / BK) * (9 * BN * BK));
#pragma unroll 3
    for (int it = tid; it < 9 * BN * BK / 4; it += 256) {
      const int row = it >> 2, q = it & 3;
      *reinterpret_cast<float4*>(Bs + row * LS + 4 * q) = src[it];
    }
    return;
  }
  for (int it = tid; it < 9 * BN * BK; it += 256) {  // from the PyTorch layout (no pack)
    const int kl = it % BK;
    const int jl = (it / BK) % BN;
    const int tap = it / (BK * BN);
    const int j = j0 + jl, k = k0 + kl;
    float v = 0.f;
    if (j < a.NOUT && k < a.KC)
      v = DGRAD ? a.w[((long long)k * a.NOUT + j) * 9 + (8 - tap)] : a.w[((long long)j * a.KC + k) * 9 + tap];
    Bs[(tap * BN + jl) * LS + kl] = v;
  }
}

// Copy a staged chunk's interior pixels (the transformed operand: BN+ReLU, pooled, concatenated, or
// the BN+ReLU backward of dz) to the tee tensor, from which the weight gradient stages a plain copy
// instead of re-deriving it.  1024 float4 per chunk.
__device__ __forceinline__ void tee_chunk32(const ConvArgs& a, const float* As, int k0, int n, int h0, int w0, int twl,
                                            int tid) {
  const int TW = 1 << twl, HW2 = TW + 2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = tid + 256 * i;
    const int q = u >> 2, qq = u & 3;
    const int r = q >> twl, c = q & (TW - 1);
    const int h = h0 + r, w = w0 + c, ch = k0 + 4 * qq;
    if (h < a.in.H && w < a.in.W && ch < a.KC)
      *reinterpret_cast<float4*>(a.tee + (((long long)n * a.in.H + h) * a.in.W + w) * a.KC + ch) =
          *reinterpret_cast<const float4*>(As + ((r + 1) * HW2 + c + 1) * LS + 4 * qq);
  }
}

// Epilogue shared by both conv kernels: fwd writes z (+bias) and per-tile BN partial sums
// (sum, sum of squares per channel, reduced over the block through LDS); dgrad writes dx split
// into the two concat halves.
template <bool DGRAD>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x16 (&acc)[2][2], float* smem, int n, int h0,
                                              int w0, int j0, int TW) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const DevFrame& F = a.in;
  float* red = smem;  // [4 waves][64 ch][2]
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
#pragma unroll
  for (int fn = 0; fn < 2; ++fn) {
    const int j = j0 + fn * 32 + (lane & 31);
    const bool jok = j < a.NOUT;
    const float b = (!DGRAD && jok && a.bias) ? a.bias[j] : 0.f;
#pragma unroll
    for (int fm = 0; fm < 2; ++fm) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = wave * 64 + fm * 32 + acc_row(r, lane);
        const int h = h0 + (q >> a.twl), w = w0 + (q & (TW - 1));
        if (!jok || h >= F.H || w >= F.W) continue;
        const long long pix = ((long long)n * F.H + h) * F.W + w;
        const float v = acc[fm][fn][r] + b;
        if (!DGRAD) {
          a.out0[pix * a.NOUT + j] = v;
          s1[fn] += v;
          s2[fn] = fmaf(v, v, s2[fn]);
        } else {
          if (j < a.split) a.out0[pix * a.split + j] = v;
          else a.out1[pix * (a.NOUT - a.split) + (j - a.split)] = v;
        }
      }
    }
  }
  if (!DGRAD && a.part) {
#pragma unroll
    for (int fn = 0; fn < 2; ++fn) {
      s1[fn] += __shfl_xor(s1[fn], 32, 64);
      s2[fn] += __shfl_xor(s2[fn], 32, 64);
      if (lane < 32) {
        red[(wave * 64 + fn * 32 + lane) * 2 + 0] = s1[fn];
        red[(wave * 64 + fn * 32 + lane) * 2 + 1] = s2[fn];
      }
    }
    __syncthreads();
    if (tid < 64) {
      const int j = j0 + tid;
      if (j < a.NOUT) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int wv = 0; wv < 4; ++wv) {
          t1 += red[(wv * 64 + tid) * 2 + 0];
          t2 += red[(wv * 64 + tid) * 2 + 1];
        }
        a.part[((long long)blockIdx.x * 2 + 0) * a.NOUT + j] = t1;
        a.part[((long long)blockIdx.x * 2 + 1) * a.NOUT + j] = t2;
      }
    }
  }
}

// TWL = log2 of the tile width (compile-time, so every tap's LDS offset is an immediate)
template <bool DGRAD, int TWL>
__global__ __launch_bounds__(256, 2) void conv3x3_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[STAGE];
  float* As = smem;
  float* Bs = smem + A_FLOATS;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  constexpr int TW = 1 << TWL;
  constexpr int TH = BM >> TWL;
  constexpr int HW2 = TW + 2;
  constexpr int HP = (TH + 2) * HW2;

  int t = blockIdx.x;
  const int tw = t % a.tiles_w; t /= a.tiles_w;
  const int th = t % a.tiles_h; t /= a.tiles_h;
  const int n = t;
  const int h0 = th * TH, w0 = tw * TW;
  const int j0 = blockIdx.y * BN;
  const DevFrame& F = a.in;
  const int nchunks = (a.KC + BK - 1) / BK;

  // staging items (chunk-independent): halo pixel of item i and its LDS row; quad = tid & 3
  int ih[NI], iw[NI], dst[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int it = tid + 256 * i;
    const int hp = it >> 2;
    const int hr = hp / HW2, hc = hp - hr * HW2;
    ih[i] = (it < HP * 4) ? h0 - 1 + hr : PMU_NO_ITEM;
    iw[i] = w0 - 1 + hc;
    dst[i] = hp * LS + 4 * (it & 3);
  }

  // MFMA operand addressing
  const int hsel = (lane >> 5) * 8;
  int abase[2], bbase[2];
#pragma unroll
  for (int fm = 0; fm < 2; ++fm) {
    const int q = wave * 64 + fm * 32 + (lane & 31);
    const int r = q >> TWL, c = q & (TW - 1);
    abase[fm] = (r * HW2 + c) * LS + hsel;
  }
#pragma unroll
  for (int fn = 0; fn < 2; ++fn) bbase[fn] = (fn * 32 + (lane & 31)) * LS + hsel;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  for (int ch = 0; ch < nchunks; ++ch) {
    const int k0 = ch * BK;
    stage_items<NI>(F, n, k0, BK, tid & 3, ih, iw, dst, As);
    stage_B<DGRAD>(a, j0, k0, Bs, tid);
    __syncthreads();
    if (a.tee && blockIdx.y == 0) tee_chunk32(a, As, k0, n, h0, w0, TWL, tid);

    float4 op[2][8];  // operand registers double-buffered across taps
    auto load_ops = [&](int tap, float4 (&o)[8]) {
      const int toff = ((tap / 3) * HW2 + (tap % 3)) * LS;
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) {
        o[2 * fm + 0] = *reinterpret_cast<const float4*>(As + abase[fm] + toff);
        o[2 * fm + 1] = *reinterpret_cast<const float4*>(As + abase[fm] + toff + 4);
      }
#pragma unroll
      for (int fn = 0; fn < 2; ++fn) {
        o[4 + 2 * fn + 0] = *reinterpret_cast<const float4*>(Bs + tap * BN * LS + bbase[fn]);
        o[4 + 2 * fn + 1] = *reinterpret_cast<const float4*>(Bs + tap * BN * LS + bbase[fn] + 4);
      }
    };
    auto mfmas = [&](const float4 (&o)[8]) {
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
#pragma unroll
          for (int fn = 0; fn < 2; ++fn) {
            const float4 va = o[2 * fm + (s >> 2)], vb = o[4 + 2 * fn + (s >> 2)];
            const float x = (s & 3) == 0 ? va.x : (s & 3) == 1 ? va.y : (s & 3) == 2 ? va.z : va.w;
            const float y = (s & 3) == 0 ? vb.x : (s & 3) == 1 ? vb.y : (s & 3) == 2 ? vb.z : vb.w;
            acc[fm][fn] = mfma_f32_32x32x2(x, y, acc[fm][fn]);
          }
    };
    load_ops(0, op[0]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap + 1 < 9) load_ops(tap + 1, op[(tap + 1) & 1]);
      mfmas(op[tap & 1]);
    }
    __syncthreads();
  }

  conv_epilogue<DGRAD>(a, acc, smem, n, h0, w0, j0, TW);
}

// ---------------------------------------------------------------------------------------------
// Software-pipelined variant (1 block/CU, LDS double-buffered; the default): the next chunk's A
// items and B tile are loaded into registers before the current chunk's 9 x 32 MFMAs, transformed
// and written to the other LDS buffer after them, with one barrier per chunk.  The operand modes are template
// parameters (M1 < 0: single source), so the staging has no runtime dispatch.  Used when every
// source is a fast-path source whose channel count is a multiple of BK and packed weights exist.
// ---------------------------------------------------------------------------------------------
constexpr int PIPE_NB = 9 * BN * BK / 4 / 256;  // packed-B float4 per thread per chunk
static_assert(PIPE_NB == 9, "PipeB holds 9 float4");

// SB (single buffer): one LDS stage and 2 blocks per CU — the commit waits behind a barrier, but the
// partner block's MFMAs cover it.
template <bool DGRAD, int POOL, bool SB = false>
__global__ __launch_bounds__(256, SB ? 2 : 1) void conv3x3_pipe_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[(SB ? 1 : 2) * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int TW = 1 << a.twl;
  const int TH = BM >> a.twl;
  const int HW2 = TW + 2;
  const int HP = (TH + 2) * HW2;

  int t = blockIdx.x;
  const int tw = t % a.tiles_w; t /= a.tiles_w;
  const int th = t % a.tiles_h; t /= a.tiles_h;
  const int n = t;
  const int h0 = th * TH, w0 = tw * TW;
  const int j0 = blockIdx.y * BN;
  const DevFrame& F = a.in;
  const int nchunks = (a.KC + BK - 1) / BK;
  const int cq4 = 4 * (tid & 3);

  int ih[NI], iw[NI], dst[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int it = tid + 256 * i;
    const int hp = it >> 2;
    const int hr = hp / HW2, hc = hp - hr * HW2;
    ih[i] = (it < HP * 4) ? h0 - 1 + hr : PMU_NO_ITEM;
    iw[i] = w0 - 1 + hc;
    dst[i] = hp * LS + 4 * (it & 3);
  }
  const int hsel = (lane >> 5) * 8;
  int abase[2], bbase[2];
#pragma unroll
  for (int fm = 0; fm < 2; ++fm) {
    const int q = wave * 64 + fm * 32 + (lane & 31);
    const int r = q >> a.twl, c = q & (TW - 1);
    abase[fm] = (r * HW2 + c) * LS + hsel;
  }
#pragma unroll
  for (int fn = 0; fn < 2; ++fn) bbase[fn] = (fn * 32 + (lane & 31)) * LS + hsel;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  PmuPref<POOL, DGRAD, NI> pf;
  // packed-B prefetch as plain locals (a struct passed by reference or an array here is kept in scratch)
  float4 pb0, pb1, pb2, pb3, pb4, pb5, pb6, pb7, pb8;
  const float4* wpk = reinterpret_cast<const float4*>(a.wp + (long long)(j0 / BN) * nchunks * (9 * BN * BK));
#define PMU_PB_ST(R, V) *reinterpret_cast<float4*>(bs_ + ((tid + 256 * (R)) >> 2) * LS + 4 * (tid & 3)) = (V);
#define PMU_PREFETCH(CH)                                                                                    \
  {                                                                                                        \
    const int k0_ = (CH) * BK;                                                                             \
    const bool second_ = F.nsrc > 1 && k0_ >= F.C0;                                                        \
    pmu_prefetch<POOL, DGRAD, NI>(pmu_pick_src(F, second_), k0_ - (second_ ? F.C0 : 0) + cq4, n, ih, iw, pf); \
    const float4* src_ = wpk + (long long)(CH) * (9 * BN * BK / 4) + tid;                                  \
    pb0 = src_[0]; pb1 = src_[256]; pb2 = src_[512]; pb3 = src_[768]; pb4 = src_[1024];                    \
    pb5 = src_[1280]; pb6 = src_[1536]; pb7 = src_[1792]; pb8 = src_[2048];                                \
  }
#define PMU_COMMIT(BUF)                                                                                     \
  {                                                                                                        \
    pmu_commit<POOL, DGRAD, NI>(pf, ih, dst, (BUF));                                                       \
    float* bs_ = (BUF) + A_FLOATS;                                                                         \
    PMU_PB_ST(0, pb0) PMU_PB_ST(1, pb1) PMU_PB_ST(2, pb2) PMU_PB_ST(3, pb3) PMU_PB_ST(4, pb4)              \
    PMU_PB_ST(5, pb5) PMU_PB_ST(6, pb6) PMU_PB_ST(7, pb7) PMU_PB_ST(8, pb8)                                \
  }

  PMU_PREFETCH(0)
  PMU_COMMIT(smem)
  __syncthreads();
  for (int ch = 0; ch < nchunks; ++ch) {
    const float* As = smem + (SB ? 0 : (ch & 1) * STAGE);
    const float* Bs = As + A_FLOATS;
    if (ch + 1 < nchunks) PMU_PREFETCH(ch + 1)
    if (a.tee && blockIdx.y == 0) tee_chunk32(a, As, ch * BK, n, h0, w0, a.twl, tid);
    float4 op[2][8];
    auto load_ops = [&](int tap, float4 (&o)[8]) {
      const int toff = ((tap / 3) * HW2 + (tap % 3)) * LS;
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) {
        o[2 * fm + 0] = *reinterpret_cast<const float4*>(As + abase[fm] + toff);
        o[2 * fm + 1] = *reinterpret_cast<const float4*>(As + abase[fm] + toff + 4);
      }
#pragma unroll
      for (int fn = 0; fn < 2; ++fn) {
        o[4 + 2 * fn + 0] = *reinterpret_cast<const float4*>(Bs + tap * BN * LS + bbase[fn]);
        o[4 + 2 * fn + 1] = *reinterpret_cast<const float4*>(Bs + tap * BN * LS + bbase[fn] + 4);
      }
    };
    auto mfmas = [&](const float4 (&o)[8]) {
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
#pragma unroll
          for (int fn = 0; fn < 2; ++fn) {
            const float4 va = o[2 * fm + (s >> 2)], vb = o[4 + 2 * fn + (s >> 2)];
            const float x = (s & 3) == 0 ? va.x : (s & 3) == 1 ? va.y : (s & 3) == 2 ? va.z : va.w;
            const float y = (s & 3) == 0 ? vb.x : (s & 3) == 1 ? vb.y : (s & 3) == 2 ? vb.z : vb.w;
            acc[fm][fn] = mfma_f32_32x32x2(x, y, acc[fm][fn]);
          }
    };
    load_ops(0, op[0]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap + 1 < 9) load_ops(tap + 1, op[(tap + 1) & 1]);
      mfmas(op[tap & 1]);
    }
    if (SB) {
      __syncthreads();
      if (ch + 1 < nchunks) {
        PMU_COMMIT(smem)
        __syncthreads();
      }
    } else {
      if (ch + 1 < nchunks) PMU_COMMIT(smem + ((ch + 1) & 1) * STAGE)
      __syncthreads();
    }
  }
#undef PMU_PREFETCH
#undef PMU_COMMIT
#undef PMU_PB_ST
  conv_epilogue<DGRAD>(a, acc, smem, n, h0, w0, j0, TW);
}

static int pick_twl(int W) {
  if (W > 16) return 5;
  if (W > 8) return 4;
  return 3;
}

// 0: sync kernel, 1: pipelined double-buffered (1 block/CU), 2 (default): pipelined single-buffered,
// 2 blocks/CU — measured fwd 117 -> 128 TF, dgrad 113 -> 122 TF on the c2 shapes (the partner block's
// MFMAs cover each block's commit phase).  PMU_CONV_IMPL=sync|pipe1 selects the others.
static int pipe_mode() {
  static const int v = [] {
    const char* e = pmu_variant_env("PMU_CONV_IMPL");
    if (e && strcmp(e, "sync") == 0) return 0;
    if (e && strcmp(e, "pipe1") == 0) return 1;
    return 2;
  }();
  return v;
}
static bool use_pipe() { return pipe_mode() != 0; }

// a source the pipelined staging handles: float4 channels, chunks never straddle sources
static bool pipe_src_ok(const pmu_src& s) {
  if (s.C % BK != 0) return false;
  if (s.pool == PMU_POOL_NONE) return true;
  return s.pool == PMU_POOL_MAX2 && s.mode == PMU_SRC_BNRELU;
}

static int launch_conv(const pmu_frame* in, const float* w, const float* wp, const float* bias, int NOUT, int KC,
                       float* out0, float* out1, int split, float* part, float* tee, bool dgrad, void* stream) {
  ConvArgs a;
  a.in = make_dev_frame(in);
  a.w = w; a.wp = wp; a.bias = bias; a.out0 = out0; a.out1 = out1; a.part = part; a.tee = tee;
  a.NOUT = NOUT; a.KC = KC; a.split = split;
  a.twl = pick_twl(in->W);
  const int TW = 1 << a.twl, TH = BM / TW;
  a.tiles_w = pmu_cdiv(in->W, TW);
  a.tiles_h = pmu_cdiv(in->H, TH);
  dim3 grid((unsigned)(a.tiles_w * a.tiles_h * in->N), (unsigned)pmu_cdiv(NOUT, BN));
  hipStream_t st = (hipStream_t)stream;
  if (wp && use_pipe()) {
    const pmu_src& s0 = in->src[0];
    const bool two = in->nsrc > 1;
    const pmu_src& s1 = in->src[1];
    const bool ok = pipe_src_ok(s0) && (!two || pipe_src_ok(s1));
    // one pool mode for the whole frame; the BN-backward source only for dgrad (single source)
    const int pool = s0.pool;
    const bool same_pool = !two || s1.pool == pool;
    const bool modes_ok = dgrad ? (!two && s0.mode == PMU_SRC_BNBWD)
                                : (s0.mode != PMU_SRC_BNBWD && (!two || s1.mode != PMU_SRC_BNBWD));
    const bool c0_ok = !two || s0.C % BK == 0;
#define PMU_PIPE(DG, PL)                                                                           \
  if (dgrad == DG && pool == PL) {                                                                 \
    if (pipe_mode() == 2)                                                                          \
      hipLaunchKernelGGL((conv3x3_pipe_kernel<DG, PL, true>), grid, dim3(256), 0, st, a);          \
    else                                                                                           \
      hipLaunchKernelGGL((conv3x3_pipe_kernel<DG, PL, false>), grid, dim3(256), 0, st, a);         \
    PMU_CHECK_LAUNCH();                                                                            \
    return PMU_OK;                                                                                 \
  }
    if (ok && same_pool && modes_ok && c0_ok) {
      PMU_PIPE(false, PMU_POOL_NONE)
      PMU_PIPE(false, PMU_POOL_MAX2)
      PMU_PIPE(true, PMU_POOL_NONE)
    }
#undef PMU_PIPE
  }
#define PMU_CLASSIC(DG, T)                                                                         \
  if (dgrad == DG && a.twl == T) {                                                                 \
    hipLaunchKernelGGL((conv3x3_kernel<DG, T>), grid, dim3(256), 0, st, a);                        \
    PMU_CHECK_LAUNCH();                                                                            \
    return PMU_OK;                                                                                 \
  }
  PMU_CLASSIC(false, 3) PMU_CLASSIC(false, 4) PMU_CLASSIC(false, 5)
  PMU_CLASSIC(true, 3) PMU_CLASSIC(true, 4) PMU_CLASSIC(true, 5)
#undef PMU_CLASSIC
  return PMU_ERR_ARG;
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

}  // namespace

// (pmu_conv3x3_tiles: defined in conv3x3_bf16.hip, same 256-pixel tile geometry)

extern "C" size_t pmu_conv3x3_packed_size(int Cout, int Cin, int dgrad) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  return (size_t)pmu_cdiv(NOUT, BN) * pmu_cdiv(KC, BK) * 9 * BN * BK * sizeof(float);
}

extern "C" int pmu_conv3x3_pack(const float* w, int Cout, int Cin, int dgrad, float* wp, void* stream) {
  PMU_REQUIRE(w && wp && Cout > 0 && Cin > 0);
  const long long total = (long long)(pmu_conv3x3_packed_size(Cout, Cin, dgrad) / sizeof(float));
  long long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(pack_w_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, dgrad, wp);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_conv3x3_fwd(const pmu_frame* in, const float* w, const float* wp, const float* bias, int Cout,
                               float* z, float* part, float* tee, void* stream) {
  PMU_REQUIRE(valid_frame(in) && (w || wp) && z && Cout > 0);
  const int Cin = in->src[0].C + (in->nsrc > 1 ? in->src[1].C : 0);
  PMU_REQUIRE(!tee || Cin % 4 == 0);
  return launch_conv(in, w, wp, bias, Cout, Cin, z, nullptr, Cout, part, tee, false, stream);
}

extern "C" int pmu_conv3x3_dgrad(const pmu_frame* dz, const float* w, const float* wp, int Cin, int Csplit,
                                 float* dx0, float* dx1, float* tee, void* stream) {
  PMU_REQUIRE(valid_frame(dz) && dz->nsrc == 1 && (w || wp) && dx0 && Cin > 0);
  PMU_REQUIRE(Csplit > 0 && Csplit <= Cin && (Csplit == Cin || dx1));
  const int Cout = dz->src[0].C;
  PMU_REQUIRE(!tee || Cout % 4 == 0);
  return launch_conv(dz, w, wp, nullptr, Cin, Cout, dx0, dx1, Csplit, nullptr, tee, true, stream);
}

// Diagnostic: resident blocks per CU of the main kernel of this file (hipOccupancy API).
extern "C" int pmu_occupancy_conv3x3_pipe(int* blocks_per_cu) {
  PMU_REQUIRE(blocks_per_cu);
  int n = 0;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(conv3x3_pipe_kernel<false, PMU_POOL_NONE, false>), 256, 0);
  if (e != hipSuccess) return (int)e;
  *blocks_per_cu = n;
  return PMU_OK;
}
#endif  // PMU_EXPERIMENTS
