// 3x3 / pad 1 convolution as an implicit GEMM on gfx950 f32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces nn.Conv2d(k=3, padding=1) of DoubleConv / Encoder
// (PMU/model/unet/unet_parts.py:15,18; PMU/model/probabilistic_unet/probabilistic_unet.py:38,43)
// together with the producer's BatchNorm2d + ReLU (+ MaxPool2d(2) | AvgPool2d(2, ceil) |
// F.pad + torch.cat) applied while the operand is staged (unet_parts.py:16-20,33,58-66).
//
// GEMM view (forward):  M = output pixels, N = Cout, K = 9 * Cin.
//   A block stages, per K chunk of BK input channels, ONE (TH+2) x (TW+2) halo tile of the
//   transformed input into LDS; all 9 taps read shifted windows of it (im2col-free).
//   Weights of the chunk are staged as B[tap][cout][k].
// GEMM view (input gradient, "dgrad"): the same kernel with the roles of Cin/Cout swapped
//   and the taps flipped: dx[p][ci] = sum_{tap,co} dz[p + d(tap)][co] * w[co][ci][8 - tap].
//
// Tile: 256 pixels (TH x TW, TW in {32,16,8}) x 64 output channels, 4 waves; wave w owns
// pixels [64w, 64w+64) x all 64 channels = 2 x 2 32x32 accumulators.
// LDS rows are k-contiguous (BK = 16 floats + 4 pad): lane half h reads k = 8h..8h+7 with two
// ds_read_b128 and feeds one k per MFMA step (the K order inside a chunk is free as long as
// A and B agree), conflict-free for 16 consecutive rows.
#include "pmu_common.h"

namespace {

constexpr int BM = 256;   // pixels per tile
constexpr int BN = 64;    // output channels per tile
constexpr int BK = 16;    // reduction channels per chunk
constexpr int LS = BK + 4;  // LDS row stride (floats)
constexpr int MAX_HP = 340; // max halo pixels: (8+2)*(32+2) = (32+2)*(8+2) = 340, (16+2)^2 = 324

struct ConvArgs {
  DevFrame in;       // operand frame (fwd: activation; dgrad: dz)
  const float* w;    // [Cout][Cin][3][3] (PyTorch layout)
  const float* bias; // fwd only
  float* out0;       // fwd: z [N][H][W][NOUT]; dgrad: dx channels [0, split)
  float* out1;       // dgrad: dx channels [split, NOUT)
  float* part;       // fwd BN partials [tiles][2][NOUT] or null
  int NOUT, KC;      // GEMM N (output channels) and reduction channels
  int split;         // dgrad channel split
  int twl;           // log2(TW)
  int tiles_w, tiles_h;
  int dgrad;
};

template <bool DGRAD>
__global__ __launch_bounds__(256, 2) void conv3x3_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[MAX_HP * LS + 9 * BN * LS];
  float* As = smem;
  float* Bs = smem + MAX_HP * LS;

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

  // per-lane A/B LDS bases
  const int hsel = (lane >> 5) * 8;
  int abase[2];
#pragma unroll
  for (int fm = 0; fm < 2; ++fm) {
    const int q = wave * 64 + fm * 32 + (lane & 31);
    const int r = q >> a.twl, c = q & (TW - 1);
    abase[fm] = (r * HW2 + c) * LS + hsel;
  }
  int bbase[2];
#pragma unroll
  for (int fn = 0; fn < 2; ++fn) bbase[fn] = (fn * 32 + (lane & 31)) * LS + hsel;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nchunks = (a.KC + BK - 1) / BK;
  const bool bvec = ((a.KC % BK) == 0) && ((a.NOUT % 4) == 0) && (j0 + BN <= a.NOUT) &&
                    (DGRAD ? ((a.NOUT * 9) % 4 == 0) : true);

  for (int ch = 0; ch < nchunks; ++ch) {
    const int k0 = ch * BK;
    // ---- stage A: halo tile of the transformed operand, channels k0..k0+BK
    for (int it = tid; it < HP * (BK / 4); it += 256) {
      const int hp = it >> 2, cq = it & 3;
      const int hr = hp / HW2, hc = hp - hr * HW2;
      const float4 v = frame_value4(F, n, h0 - 1 + hr, w0 - 1 + hc, k0 + 4 * cq);
      *reinterpret_cast<float4*>(As + hp * LS + 4 * cq) = v;
    }
    // ---- stage B
    if (bvec) {
      if (!DGRAD) {
        // per output channel co: w[co][k0..k0+16][0..9) is 144 contiguous floats
        for (int it = tid; it < BN * 36; it += 256) {
          const int jl = it / 36, q = it - jl * 36;
          const float4 v = *reinterpret_cast<const float4*>(
              a.w + ((long long)(j0 + jl) * a.KC + k0) * 9 + 4 * q);
          const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int idx = 4 * q + e, kl = idx / 9, tap = idx - kl * 9;
            Bs[(tap * BN + jl) * LS + kl] = vv[e];
          }
        }
      } else {
        // per reduction channel co (= k): w[co][j0..j0+64][0..9) is 576 contiguous floats
        for (int it = tid; it < BK * 144; it += 256) {
          const int kl = it / 144, q = it - kl * 144;
          const float4 v = *reinterpret_cast<const float4*>(
              a.w + ((long long)(k0 + kl) * a.NOUT + j0) * 9 + 4 * q);
          const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int idx = 4 * q + e, jl = idx / 9, tap = idx - jl * 9;
            Bs[((8 - tap) * BN + jl) * LS + kl] = vv[e];
          }
        }
      }
    } else {
      for (int it = tid; it < 9 * BN * BK; it += 256) {
        const int kl = it % BK;
        const int jl = (it / BK) % BN;
        const int tap = it / (BK * BN);
        const int j = j0 + jl, k = k0 + kl;
        float v = 0.f;
        if (j < a.NOUT && k < a.KC) {
          v = DGRAD ? a.w[((long long)k * a.NOUT + j) * 9 + (8 - tap)]
                    : a.w[((long long)j * a.KC + k) * 9 + tap];
        }
        Bs[(tap * BN + jl) * LS + kl] = v;
      }
    }
    __syncthreads();

    // ---- 9 taps x 8 k-steps x (2x2) MFMAs
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = ((tap / 3) * HW2 + (tap % 3)) * LS;
      float av[2][8], bv[2][8];
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) {
        const float4 x0 = *reinterpret_cast<const float4*>(As + abase[fm] + toff);
        const float4 x1 = *reinterpret_cast<const float4*>(As + abase[fm] + toff + 4);
        av[fm][0] = x0.x; av[fm][1] = x0.y; av[fm][2] = x0.z; av[fm][3] = x0.w;
        av[fm][4] = x1.x; av[fm][5] = x1.y; av[fm][6] = x1.z; av[fm][7] = x1.w;
      }
#pragma unroll
      for (int fn = 0; fn < 2; ++fn) {
        const float4 y0 = *reinterpret_cast<const float4*>(Bs + tap * BN * LS + bbase[fn]);
        const float4 y1 = *reinterpret_cast<const float4*>(Bs + tap * BN * LS + bbase[fn] + 4);
        bv[fn][0] = y0.x; bv[fn][1] = y0.y; bv[fn][2] = y0.z; bv[fn][3] = y0.w;
        bv[fn][4] = y1.x; bv[fn][5] = y1.y; bv[fn][6] = y1.z; bv[fn][7] = y1.w;
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
#pragma unroll
          for (int fn = 0; fn < 2; ++fn) acc[fm][fn] = mfma_f32_32x32x2(av[fm][s], bv[fn][s], acc[fm][fn]);
    }
    __syncthreads();
  }

  // ---- epilogue
  float* red = smem;  // reuse LDS: [4 waves][64 ch][2]
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
    __syncthreads();
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

static int pick_twl(int W) {
  if (W > 16) return 5;
  if (W > 8) return 4;
  return 3;
}

static int launch_conv(const pmu_frame* in, const float* w, const float* bias, int NOUT, int KC,
                       float* out0, float* out1, int split, float* part, bool dgrad, void* stream) {
  ConvArgs a;
  a.in = make_dev_frame(in);
  a.w = w; a.bias = bias; a.out0 = out0; a.out1 = out1; a.part = part;
  a.NOUT = NOUT; a.KC = KC; a.split = split; a.dgrad = dgrad;
  a.twl = pick_twl(in->W);
  const int TW = 1 << a.twl, TH = BM / TW;
  a.tiles_w = pmu_cdiv(in->W, TW);
  a.tiles_h = pmu_cdiv(in->H, TH);
  dim3 grid((unsigned)(a.tiles_w * a.tiles_h * in->N), (unsigned)pmu_cdiv(NOUT, BN));
  if (dgrad)
    hipLaunchKernelGGL(conv3x3_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(conv3x3_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, a);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

}  // namespace

extern "C" int pmu_conv3x3_tiles(int N, int H, int W) {
  const int twl = pick_twl(W);
  const int TW = 1 << twl, TH = BM / TW;
  return N * pmu_cdiv(H, TH) * pmu_cdiv(W, TW);
}

extern "C" int pmu_conv3x3_fwd(const pmu_frame* in, const float* w, const float* bias, int Cout,
                               float* z, float* part, void* stream) {
  PMU_REQUIRE(valid_frame(in) && w && z && Cout > 0);
  const int Cin = in->src[0].C + (in->nsrc > 1 ? in->src[1].C : 0);
  return launch_conv(in, w, bias, Cout, Cin, z, nullptr, Cout, part, false, stream);
}

extern "C" int pmu_conv3x3_dgrad(const pmu_frame* dz, const float* w, int Cin, int Csplit,
                                 float* dx0, float* dx1, void* stream) {
  PMU_REQUIRE(valid_frame(dz) && dz->nsrc == 1 && w && dx0 && Cin > 0);
  PMU_REQUIRE(Csplit > 0 && Csplit <= Cin && (Csplit == Cin || dx1));
  const int Cout = dz->src[0].C;
  return launch_conv(dz, w, nullptr, Cin, Cout, dx0, dx1, Csplit, nullptr, true, stream);
}
