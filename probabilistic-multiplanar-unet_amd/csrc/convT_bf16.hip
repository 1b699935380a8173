// ConvTranspose2d(Cin, Cout, kernel 2, stride 2) of Up (PMU/model/unet/unet_parts.py:52), forward
// and input gradient on bf16 MFMA (config c5, torch.autocast(bfloat16) arithmetic: the BN+ReLU
// operand / du and the weights rounded to bf16, fp32 sums, fp32 outputs).
//
// GEMM views as convT.hip's pipelined kernel:
//   forward : C[pix][ab*Cout+co] = act(x)[pix][ci] . Bp[ab*Cout+co][ci]   (M=pixels, N=4Cout, K=Cin)
//   dgrad   : dx[pix][ci] = sum_k' du(pix, k') . Bp[ci][k' = ab*Cout+co]  (M=pixels, N=Cin, K=4Cout)
// Tile 128 x 128 x 32 (two 32x32x16 k-steps per chunk), 4 waves of 64 x 64 (2 x 2 accumulators),
// double-buffered bf16 LDS (80-B rows: ds_read_b128 conflict-free), the next chunk's global loads
// in registers under the current chunk's MFMAs, 2 blocks per CU.
#include "pmu_stage.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int TM = 128, TN = 128, TK = 32, TLS = 40;  // LDS row stride (bf16)

struct TArgs {
  const float* a;             // fwd: z [M][Cin] (pre-BN);  dgrad: du [N][Hd][Wd][Cout]
  const float* coef;          // fwd: [scale|shift]
  const unsigned short* bp;   // packed bf16 B [Ncols][K]
  const float* bias;
  float* out;                 // fwd: u [N][2H][2W][Cout];  dgrad: dx [M][Cin]
  long long M;
  int Ncols, K, H, W, Cin, Cout, Hd, Wd, off_h, off_w;
};

__global__ void convT_pack_bf16_kernel(const float* __restrict__ w, int Cin, int Cout, int dgrad,
                                       unsigned short* __restrict__ wp) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long E = 4LL * Cin * Cout;
  if (e >= E) return;
  const int ab = (int)(e & 3);  // e = (ci*Cout + co)*4 + ab
  const long long cc = e >> 2;
  const int co = (int)(cc % Cout), ci = (int)(cc / Cout);
  const unsigned short v = __builtin_bit_cast(unsigned short, (__bf16)w[e]);
  if (dgrad) wp[(long long)ci * 4 * Cout + ab * Cout + co] = v;
  else wp[((long long)ab * Cout + co) * Cin + ci] = v;
}

template <bool DGRAD>
__global__ __launch_bounds__(256, 2) void convT_bf16_kernel(TArgs p) {
  __shared__ __attribute__((aligned(16))) unsigned short As[2][TM * TLS];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2][TN * TLS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const long long m0 = (long long)blockIdx.x * TM;
  const int n0 = blockIdx.y * TN;
  const int hsel = (lane >> 5) * 8;
  // A: rows (tid>>3) + 32i, 4 consecutive k at 4*(tid&7); B: rows (tid>>2) + 64i, 8 k at 8*(tid&3)
  const int kq = 4 * (tid & 7), bq = 8 * (tid & 3);
  long long abase[4];
  bool aok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long long m = m0 + (tid >> 3) + 32 * i;
    aok[i] = m < p.M;
    const long long mm = aok[i] ? m : 0;
    if constexpr (DGRAD) {
      const int j = (int)(mm % p.W);
      const long long t = mm / p.W;
      const int ii = (int)(t % p.H);
      const long long n = t / p.H;
      abase[i] = ((n * p.Hd + p.off_h + 2 * ii) * p.Wd + p.off_w + 2 * j) * p.Cout;
    } else {
      abase[i] = mm * p.Cin;
    }
  }
  const unsigned short* br0 = p.bp + (long long)(n0 + (tid >> 2)) * p.K + bq;
  const unsigned short* br1 = br0 + 64LL * p.K;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float4 ra0, ra1, ra2, ra3;
  uint4 rb0, rb1;
#define PMU_TLOAD(K0)                                                                           \
  {                                                                                             \
    long long off_ = (K0) + kq;                                                                 \
    if (DGRAD) {                                                                                \
      const int ab_ = (K0) / p.Cout;                                                            \
      off_ = ((long long)(ab_ >> 1) * p.Wd + (ab_ & 1)) * p.Cout + ((K0) - ab_ * p.Cout) + kq;  \
    }                                                                                           \
    ra0 = *reinterpret_cast<const float4*>(p.a + abase[0] + off_);                              \
    ra1 = *reinterpret_cast<const float4*>(p.a + abase[1] + off_);                              \
    ra2 = *reinterpret_cast<const float4*>(p.a + abase[2] + off_);                              \
    ra3 = *reinterpret_cast<const float4*>(p.a + abase[3] + off_);                              \
    rb0 = *reinterpret_cast<const uint4*>(br0 + (K0));                                          \
    rb1 = *reinterpret_cast<const uint4*>(br1 + (K0));                                          \
  }
  auto xf = [](float4 v, bool ok, float4 sc, float4 sh) {
    if (!DGRAD) v = pmu_bnrelu4(v, sc, sh);
    return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  };
#define PMU_TSTORE(BUF, K0)                                                                     \
  {                                                                                             \
    float4 sc_ = make_float4(0.f, 0.f, 0.f, 0.f), sh_ = sc_;                                    \
    if (!DGRAD) {                                                                               \
      sc_ = *reinterpret_cast<const float4*>(p.coef + (K0) + kq);                               \
      sh_ = *reinterpret_cast<const float4*>(p.coef + p.Cin + (K0) + kq);                       \
    }                                                                                           \
    unsigned short* as_ = As[BUF] + (tid >> 3) * TLS + kq;                                      \
    pmu_lds_store4<true>(as_, 0, xf(ra0, aok[0], sc_, sh_));                                    \
    pmu_lds_store4<true>(as_, 32 * TLS, xf(ra1, aok[1], sc_, sh_));                             \
    pmu_lds_store4<true>(as_, 64 * TLS, xf(ra2, aok[2], sc_, sh_));                             \
    pmu_lds_store4<true>(as_, 96 * TLS, xf(ra3, aok[3], sc_, sh_));                             \
    *reinterpret_cast<uint4*>(Bs[BUF] + (tid >> 2) * TLS + bq) = rb0;                           \
    *reinterpret_cast<uint4*>(Bs[BUF] + ((tid >> 2) + 64) * TLS + bq) = rb1;                    \
  }

  const int nch = p.K / TK;
  PMU_TLOAD(0)
  PMU_TSTORE(0, 0)
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int cur = c & 1;
    const bool more = c + 1 < nch;
    if (more) PMU_TLOAD((c + 1) * TK)
#pragma unroll
    for (int s = 0; s < TK / 16; ++s) {
      bf16x8 av[2], bv[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        av[f] = *reinterpret_cast<const bf16x8*>(&As[cur][(wm * 64 + f * 32 + (lane & 31)) * TLS + 16 * s + hsel]);
        bv[f] = *reinterpret_cast<const bf16x8*>(&Bs[cur][(wn * 64 + f * 32 + (lane & 31)) * TLS + 16 * s + hsel]);
      }
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[fm], bv[fn], acc[fm][fn], 0, 0, 0);
    }
    if (more) PMU_TSTORE(cur ^ 1, (c + 1) * TK)
    __syncthreads();
  }
#undef PMU_TLOAD
#undef PMU_TSTORE

#pragma unroll
  for (int fn = 0; fn < 2; ++fn) {
    const int col = n0 + wn * 64 + fn * 32 + (lane & 31);
    if constexpr (DGRAD) {
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const long long m = m0 + wm * 64 + fm * 32 + acc_row(r, lane);
          if (m < p.M) p.out[m * p.Cin + col] = acc[fm][fn][r];
        }
    } else {
      const int ab = col / p.Cout, co = col - ab * p.Cout;
      const float b = p.bias ? p.bias[co] : 0.f;
      const unsigned Wu = (unsigned)p.W, Hu = (unsigned)p.H;  // 32-bit decode (M < 2^31, host-checked)
      float* outc = p.out + (long long)(ab >> 1) * 2 * p.W * p.Cout + (ab & 1) * p.Cout + co;
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const unsigned m = (unsigned)(m0 + wm * 64 + fm * 32 + acc_row(r, lane));
          if (m < (unsigned)p.M) {
            const unsigned t = m / Wu, j = m - t * Wu;
            const unsigned n = t / Hu, i = t - n * Hu;
            outc[((long long)(n * 2 * Hu + 2 * i) * (2 * Wu) + 2 * j) * p.Cout] = acc[fm][fn][r] + b;
          }
        }
    }
  }
}

}  // namespace

extern "C" int pmu_convT2x2_pack_bf16(const float* w, int Cin, int Cout, int dgrad, unsigned short* wp, void* stream) {
  PMU_REQUIRE(w && wp && Cin > 0 && Cout > 0);
  const long long E = 4LL * Cin * Cout;
  hipLaunchKernelGGL(convT_pack_bf16_kernel, dim3((unsigned)pmu_cdiv(E, 256)), dim3(256), 0, (hipStream_t)stream, w,
                     Cin, Cout, dgrad, wp);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_convT2x2_bf16_ok(const pmu_frame* in, int Cout) {
  if (!in || !valid_frame(in) || in->nsrc != 1) return 0;
  const pmu_src& s = in->src[0];
  const long long M = (long long)in->N * in->H * in->W;
  return s.mode == PMU_SRC_BNRELU && s.pool == PMU_POOL_NONE && s.off_h == 0 && s.off_w == 0 && s.H == in->H &&
         s.W == in->W && s.C % TK == 0 && Cout % TK == 0 && (4 * Cout) % TN == 0 && M < (1LL << 31);
}

extern "C" int pmu_convT2x2_fwd_bf16(const pmu_frame* in, const unsigned short* wp, const float* bias, int Cout,
                                     float* u, void* stream) {
  PMU_REQUIRE(wp && u && pmu_convT2x2_bf16_ok(in, Cout));
  TArgs p{};
  p.a = in->src[0].x; p.coef = in->src[0].coef; p.bp = wp; p.bias = bias; p.out = u;
  p.M = (long long)in->N * in->H * in->W; p.Ncols = 4 * Cout; p.K = in->src[0].C;
  p.H = in->H; p.W = in->W; p.Cin = in->src[0].C; p.Cout = Cout;
  dim3 grid((unsigned)pmu_cdiv(p.M, TM), (unsigned)(p.Ncols / TN));
  hipLaunchKernelGGL(convT_bf16_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, p);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_convT2x2_dgrad_bf16(const float* du, int Hd, int Wd, int off_h, int off_w, const unsigned short* wp,
                                       int N, int H, int W, int Cin, int Cout, float* dx, void* stream) {
  PMU_REQUIRE(du && wp && dx && N > 0 && H > 0 && W > 0 && Cin % TN == 0 && Cout % TK == 0);
  PMU_REQUIRE(off_h >= 0 && off_w >= 0 && off_h + 2 * H <= Hd && off_w + 2 * W <= Wd);
  TArgs p{};
  p.a = du; p.bp = wp; p.out = dx;
  p.M = (long long)N * H * W; p.Ncols = Cin; p.K = 4 * Cout;
  p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout; p.Hd = Hd; p.Wd = Wd; p.off_h = off_h; p.off_w = off_w;
  dim3 grid((unsigned)pmu_cdiv(p.M, TM), (unsigned)(Cin / TN));
  hipLaunchKernelGGL(convT_bf16_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, p);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
