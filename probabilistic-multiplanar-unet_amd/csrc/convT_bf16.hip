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
#include <cstdlib>
#include "pmu_stage.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#ifdef PMU_EXPERIMENTS
constexpr int TM = 128, TN = 128, TK = 32, TLS = 40;  // LDS row stride (bf16)
#endif

struct TArgs {
  const float* a;             // fwd: z [M][Cin] (pre-BN);  dgrad: du [N][Hd][Wd][Cout]
  const float* coef;          // fwd: [scale|shift]
  const unsigned short* bp;   // packed bf16 B [Ncols][K]
  const float* bias;
  float* out;                 // fwd: u [N][2H][2W][Cout];  dgrad: dx [M][Cin]
  long long M;
  int Ncols, K, H, W, Cin, Cout, Hd, Wd, off_h, off_w;
  int lw, lh;                 // fwd: log2 W, log2 H when powers of two (shift/mask epilogue), else -1
  int nnb, xcd;               // column blocks; 1: 1-D XCD-ordered grid, column blocks fastest
};

#ifdef PMU_EXPERIMENTS
// (register-staged ConvT forward / input gradient: their shapes are exactly the LDS-DMA kernels'
// (convT_bf16_dma.hip), which the engine always takes; experiments build only)
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
  // with p.xcd the column blocks of one row block run back to back on one XCD: the A rows (the
  // big operand) come from HBM once and are re-read from that XCD's L2
  long long mb;
  int nb_;
  if (p.xcd) {
    const int lb = pmu_xcd_block(blockIdx.x, gridDim.x);
    nb_ = lb % p.nnb;
    mb = lb / p.nnb;
  } else {
    mb = blockIdx.x;
    nb_ = blockIdx.y;
  }
  const long long m0 = mb * TM;
  const int n0 = nb_ * TN;
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
    if constexpr (DGRAD) {  // 32-bit decode (M < 2^31, host-checked)
      const unsigned t = (unsigned)mm / (unsigned)p.W, j = (unsigned)mm - t * (unsigned)p.W;
      const unsigned n = t / (unsigned)p.H, ii = t - n * (unsigned)p.H;
      abase[i] = ((long long)(n * p.Hd + p.off_h + 2 * ii) * p.Wd + p.off_w + 2 * j) * p.Cout;
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
      if (p.lw >= 0 && p.lh >= 0) {  // shift/mask decode: the divisions cost as much as a short K loop
        const bool full = m0 + TM <= p.M;
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const unsigned m = (unsigned)(m0 + wm * 64 + fm * 32 + acc_row(r, lane));
            if (full || m < (unsigned)p.M) {
              const unsigned j = m & (Wu - 1), t = m >> p.lw;
              const unsigned i = t & (Hu - 1), n = t >> p.lh;
              outc[(size_t)((n * 2 * Hu + 2 * i) * (2 * Wu) + 2 * j) * (unsigned)p.Cout] = acc[fm][fn][r] + b;
            }
          }
      } else {
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
}

#endif  // PMU_EXPERIMENTS

// ---------------------------------------------------------------------------------------------
// Weight gradient on bf16 MFMA: dW[ci][co][a][b] = sum_p xt[p][ci] * dut[pix_ab(p)][co]
// (xt = bf16 of the BN+ReLU input, dut = bf16 of du, both materialised by pmu_frame_to_bf16).
// K = convT-input pixels, 64 per tile in flat (n, i, j) order; the MFMA takes 8 consecutive pixels
// per lane half, so both operands are read with ds_read_b64_tr_b16 from channel-contiguous LDS rows
// (as wgrad3x3_bf16): the tap only changes which du pixel a row holds.  Block = 128 ci x 64 co x 4
// taps, 4 waves (one 32-ci fragment each) x (2 co fragments x 4 taps) = 8 accumulators; the next
// tile's 12 units per thread are in registers under the current tile's 32 MFMAs per wave.
// Split-K slabs ws[split][ab][ci][co] are reduced in a fixed order.
// ---------------------------------------------------------------------------------------------
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
constexpr int WCI = 128, WCO = 64, WPX = 64;
constexpr int XSW = WCI + 32;  // 320-B rows: 64 mod 256, transposed reads conflict-free
constexpr int DSW = WCO + 32;  // 192-B rows
constexpr int XU = WPX * WCI / 8 / 256;      // 4 X units per thread
constexpr int DU = 4 * WPX * WCO / 8 / 256;  // 8 D units per thread

struct TwbArgs {
  const unsigned short* xt;   // [N][H][W][Cip]
  const unsigned short* dut;  // [N][Hd][Wd][Cop]
  float* ws;
  int N, H, W, Hd, Wd, oh, ow, Cin, Cout, Cip, Cop, ntiles, nsplit;
};

__device__ __forceinline__ s16x4 tr_read(const unsigned short* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}
__device__ __forceinline__ uint4 keep_if(bool ok, uint4 v) {
  return make_uint4(ok ? v.x : 0u, ok ? v.y : 0u, ok ? v.z : 0u, ok ? v.w : 0u);
}

__global__ __launch_bounds__(256, 2) void convT_wgrad_bf16_kernel(TwbArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned short Xs[WPX * XSW];
  __shared__ __attribute__((aligned(16))) unsigned short Ds[4 * WPX * DSW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nco = pmu_cdiv_dev(a.Cout, WCO);
  // (channel block, split) in XCD order, channel blocks fastest: the blocks of one split read the same
  // pixel rows at the same time through one XCD's L2 (see wgrad3x3_bf16.hip)
  const int nblk = gridDim.x;
  const int lbk = pmu_xcd_block(blockIdx.y * nblk + blockIdx.x, nblk * gridDim.y);
  const int blk = lbk % nblk;
  const int co0 = (blk % nco) * WCO, ci0 = (blk / nco) * WCI;
  const int split = lbk / nblk;
  const long long P = (long long)a.N * a.H * a.W;
  const int t_beg = (int)(((long long)a.ntiles * split) / a.nsplit);
  const int t_end = (int)(((long long)a.ntiles * (split + 1)) / a.nsplit);

  f32x16 acc[2][4];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[f][t][r] = 0.f;

  uint4 rx0, rx1, rx2, rx3, rd0, rd1, rd2, rd3, rd4, rd5, rd6, rd7;  // plain locals (no scratch)
  static_assert(XU == 4 && DU == 8, "staging register layout");
  // X unit u = tid + 256 i: pixel u >> 4, 8-channel unit u & 15; D unit: tap u >> 9, pixel (u >> 3) & 63, unit u & 7
#define PMU_XL(I, R)                                                                                \
  {                                                                                                \
    const int u_ = tid + 256 * (I);                                                                \
    const long long p_ = (long long)tile_ * WPX + (u_ >> 4);                                       \
    const int c_ = ci0 + 8 * (u_ & 15);                                                            \
    const bool ok_ = p_ < P && c_ < a.Cip;                                                         \
    R = keep_if(ok_, *reinterpret_cast<const uint4*>(a.xt + (ok_ ? p_ * a.Cip + c_ : 0)));        \
  }
// D units of a thread cover two du pixel slots (I even / odd: tile pixel (tid >> 3) and +32) and 4
// taps; the slots are decoded once per tile in 32 bits (N*H*W < 2^30, host-checked).  Decoding each
// unit with 64-bit divisions made this kernel VALU-bound.
#define PMU_DL(I, R)                                                                                \
  {                                                                                                \
    const int tap_ = (I) >> 1;                                                                     \
    const int c_ = co0 + 8 * (tid & 7);                                                            \
    const bool ok_ = okd_[(I) & 1] && c_ < a.Cop;                                                  \
    const unsigned q_ = ok_ ? qd_[(I) & 1] + (unsigned)(((tap_ >> 1) * a.Wd + (tap_ & 1)) * a.Cop + c_) : 0u; \
    R = keep_if(ok_, *reinterpret_cast<const uint4*>(a.dut + q_));                                 \
  }
#define PMU_LOAD(T)                                                                                 \
  {                                                                                                \
    const int tile_ = (T);                                                                         \
    unsigned qd_[2];  /* 32-bit element offsets (du < 2^32 elements, host-checked) */            \
    bool okd_[2];                                                                                  \
    _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_) {                                             \
      const unsigned p_ = (unsigned)tile_ * WPX + (unsigned)(tid >> 3) + 32u * s_;                 \
      okd_[s_] = p_ < (unsigned)P;                                                                 \
      const unsigned t2_ = p_ / (unsigned)a.W, j_ = p_ - t2_ * (unsigned)a.W;                      \
      const unsigned n_ = t2_ / (unsigned)a.H, i_ = t2_ - n_ * (unsigned)a.H;                      \
      qd_[s_] = ((n_ * a.Hd + a.oh + 2 * i_) * a.Wd + a.ow + 2 * j_) * a.Cop;                       \
    }                                                                                              \
    PMU_XL(0, rx0) PMU_XL(1, rx1) PMU_XL(2, rx2) PMU_XL(3, rx3)                                    \
    PMU_DL(0, rd0) PMU_DL(1, rd1) PMU_DL(2, rd2) PMU_DL(3, rd3)                                    \
    PMU_DL(4, rd4) PMU_DL(5, rd5) PMU_DL(6, rd6) PMU_DL(7, rd7)                                    \
  }
#define PMU_XS(I, R) { const int u_ = tid + 256 * (I); *reinterpret_cast<uint4*>(Xs + (u_ >> 4) * XSW + 8 * (u_ & 15)) = R; }
#define PMU_DS(I, R) { const int u_ = tid + 256 * (I); *reinterpret_cast<uint4*>(Ds + ((u_ >> 9) * WPX + ((u_ >> 3) & 63)) * DSW + 8 * (u_ & 7)) = R; }
#define PMU_STORE()                                                                                 \
  {                                                                                                \
    PMU_XS(0, rx0) PMU_XS(1, rx1) PMU_XS(2, rx2) PMU_XS(3, rx3)                                    \
    PMU_DS(0, rd0) PMU_DS(1, rd1) PMU_DS(2, rd2) PMU_DS(3, rd3)                                    \
    PMU_DS(4, rd4) PMU_DS(5, rd5) PMU_DS(6, rd6) PMU_DS(7, rd7)                                    \
  }

  // transposed-read lane roles (see wgrad3x3_bf16.hip)
  const int h = lane >> 5, g = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
  const int xcol = wave * 32 + 16 * g + 4 * p;
  const int dcol = 16 * g + 4 * p;
  if (t_beg < t_end) {
    PMU_LOAD(t_beg)
    PMU_STORE()
  }
  __syncthreads();
  for (int tile = t_beg; tile < t_end; ++tile) {
    const bool more = tile + 1 < t_end;
    if (more) PMU_LOAD(tile + 1)  // in flight during the MFMAs
#pragma unroll
    for (int ks = 0; ks < WPX / 16; ++ks) {
      const int pk0 = 16 * ks + 8 * h + q, pk1 = pk0 + 4;
      const bf16x8 af = __builtin_bit_cast(bf16x8, __builtin_shufflevector(tr_read(Xs + pk0 * XSW + xcol),
                                                                             tr_read(Xs + pk1 * XSW + xcol), 0, 1, 2,
                                                                             3, 4, 5, 6, 7));
#pragma unroll
      for (int tap = 0; tap < 4; ++tap)
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const unsigned short* d = Ds + (tap * WPX) * DSW + 32 * f + dcol;
          const bf16x8 bfr = __builtin_bit_cast(bf16x8, __builtin_shufflevector(tr_read(d + pk0 * DSW),
                                                                                  tr_read(d + pk1 * DSW), 0, 1, 2, 3,
                                                                                  4, 5, 6, 7));
          acc[f][tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc[f][tap], 0, 0, 0);
        }
    }
    __syncthreads();
    if (more) {
      PMU_STORE()
      __syncthreads();
    }
  }
#undef PMU_XL
#undef PMU_DL
#undef PMU_LOAD
#undef PMU_XS
#undef PMU_DS
#undef PMU_STORE
  // slab ws[split][ab][ci][co]: accumulator rows = ci (A rows), columns = co (lanes)
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int co = co0 + 32 * f + (lane & 31);
    if (co >= a.Cout) continue;
#pragma unroll
    for (int tap = 0; tap < 4; ++tap)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ci = ci0 + wave * 32 + acc_row(r, lane);
        if (ci < a.Cin) a.ws[(((long long)split * 4 + tap) * a.Cin + ci) * a.Cout + co] = acc[f][tap][r];
      }
  }
}

// dW[ci][co][ab] = sum_s ws[s][ab][ci][co] (4 split groups per element, fixed order)
__global__ __launch_bounds__(256) void convT_wreduce_bf16_kernel(const float* __restrict__ ws, int nsplit, int Cin,
                                                                 int Cout, float* __restrict__ dw) {
  __shared__ float red[4][64];
  const long long CC = (long long)Cin * Cout, E = 4 * CC;
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const long long e = (long long)blockIdx.x * 64 + lane;  // (ab * Cin + ci) * Cout + co
  float s0 = 0.f, s1 = 0.f;
  if (e < E) {
    int sp = g;
    for (; sp + 4 < nsplit; sp += 8) {
      s0 += ws[(long long)sp * E + e];
      s1 += ws[(long long)(sp + 4) * E + e];
    }
    for (; sp < nsplit; sp += 4) s0 += ws[(long long)sp * E + e];
  }
  red[g][lane] = s0 + s1;
  __syncthreads();
  if (g == 0 && e < E) {
    const float t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    const int ab = (int)(e / CC);
    const long long cc = e - ab * CC;  // ci * Cout + co
    dw[cc * 4 + ab] = t;
  }
}

// dbias[co] = sum of du over the convT output region, fp32 (the unrounded gradient), fixed order.
// Block b: PL = 256 / (Cout/4) pixel lanes x Cout/4 channel quads; lane pl sums pixels
// b*PL + pl + k*G*PL as float4, the lanes are added in order through LDS into part[b][Cout].
__global__ __launch_bounds__(256) void convT_dbias_part_kernel(const float* __restrict__ du, int N, int H2, int W2,
                                                               int Hd, int Wd, int oh, int ow, int Cout,
                                                               float* __restrict__ part) {
  __shared__ float4 red[256];
  const int nq = Cout / 4, PL = 256 / nq;
  const int t = threadIdx.x, qd = t % nq, pl = t / nq;
  const unsigned npx = (unsigned)N * H2 * W2;  // < 2^32 (host-checked)
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (pl < PL) {
    const unsigned stride = gridDim.x * PL;
    // pixels r, r + stride, ... in order; 4 loads in flight per thread
#pragma unroll 4
    for (unsigned r = blockIdx.x * PL + pl; r < npx; r += stride) {
      const unsigned row = r / (unsigned)W2, x = r - row * W2;
      const unsigned n = row / (unsigned)H2, y = row - n * H2;
      const float4 v = *reinterpret_cast<const float4*>(
          du + (((long long)n * Hd + oh + y) * Wd + ow + x) * Cout + 4 * qd);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[t] = acc;
  __syncthreads();
  if (pl == 0) {
    float4 s = red[qd];
    for (int l = 1; l < PL; ++l) {
      const float4 v = red[l * nq + qd];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    *reinterpret_cast<float4*>(part + (long long)blockIdx.x * Cout + 4 * qd) = s;
  }
}
// scalar variant for Cout not a multiple of 4 (or > 1024)
__global__ __launch_bounds__(256) void convT_dbias_part1_kernel(const float* __restrict__ du, int N, int H2, int W2,
                                                                int Hd, int Wd, int oh, int ow, int Cout,
                                                                float* __restrict__ part) {
  const long long rows = (long long)N * H2;
  for (int c = threadIdx.x; c < Cout; c += 256) {
    float s = 0.f;
    for (long long r = blockIdx.x; r < rows; r += gridDim.x) {
      const long long n = r / H2;
      const int y = (int)(r - n * H2);
      const float* row = du + ((n * Hd + oh + y) * Wd + ow) * Cout + c;
      for (int x = 0; x < W2; ++x) s += row[(long long)x * Cout];
    }
    part[(long long)blockIdx.x * Cout + c] = s;
  }
}
// db[c] = sum of the G partial rows (row stride ld): 64 channels per block, 4 row groups summed in a
// fixed order
__global__ __launch_bounds__(256) void convT_dbias_sum_kernel(const float* __restrict__ part, int G, int Cout,
                                                              long long ld, float* __restrict__ db) {
  __shared__ float red[256];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), grp = threadIdx.x >> 6;
  float s = 0.f;
  if (c < Cout) {
    const int g0 = (G * grp) / 4, g1 = (G * (grp + 1)) / 4;
#pragma unroll 4
    for (int gidx = g0; gidx < g1; ++gidx) s += part[(long long)gidx * ld + c];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (grp == 0 && c < Cout) db[c] = ((red[threadIdx.x] + red[64 + threadIdx.x]) + red[128 + threadIdx.x]) + red[192 + threadIdx.x];
}

static void twb_geometry(int N, int H, int W, int Cin, int Cout, int* ntiles, int* nsplit) {
  *ntiles = (int)(((long long)N * H * W + WPX - 1) / WPX);
  const int bmn = pmu_cdiv(Cin, WCI) * pmu_cdiv(Cout, WCO);
  static const int target = [] {  // PMU_CONVT_BWBLOCKS: workgroups the split-K aims for (A/B)
    const char* e = getenv("PMU_CONVT_BWBLOCKS");
    return e ? atoi(e) : 512;
  }();
  int sp = target / bmn;
  if (sp < 1) sp = 1;
  if (sp > *ntiles) sp = *ntiles;
  *nsplit = sp;
}
constexpr int DB_G = 2048;  // dbias partial rows (blocks of the partial-sum pass: 8 per CU)

}  // namespace

#ifdef PMU_EXPERIMENTS
static void set_grid(TArgs& p, int nnb) {
  static const int xcd = [] {
    const char* e = pmu_variant_env("PMU_CONVT_XCD");
    return e ? atoi(e) : 1;
  }();
  p.nnb = nnb;
  p.xcd = xcd && (long long)pmu_cdiv(p.M, TM) * nnb < (1LL << 31);
}

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
  auto log2_or = [](int v) { return (v & (v - 1)) == 0 ? __builtin_ctz((unsigned)v) : -1; };
  p.lw = log2_or(in->W); p.lh = log2_or(in->H);
  if (4LL * p.M * Cout >= (1LL << 32)) p.lw = -1;  // the shift path's output index is 32-bit
  set_grid(p, p.Ncols / TN);
  const dim3 grid = p.xcd ? dim3((unsigned)(pmu_cdiv(p.M, TM) * p.nnb)) : dim3((unsigned)pmu_cdiv(p.M, TM), (unsigned)p.nnb);
  hipLaunchKernelGGL(convT_bf16_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, p);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_convT2x2_dgrad_bf16(const float* du, int Hd, int Wd, int off_h, int off_w, const unsigned short* wp,
                                       int N, int H, int W, int Cin, int Cout, float* dx, void* stream) {
  PMU_REQUIRE(du && wp && dx && N > 0 && H > 0 && W > 0 && Cin % TN == 0 && Cout % TK == 0);
  PMU_REQUIRE(off_h >= 0 && off_w >= 0 && off_h + 2 * H <= Hd && off_w + 2 * W <= Wd);
  PMU_REQUIRE((long long)N * H * W < (1LL << 31));  // 32-bit pixel decode
  TArgs p{};
  p.a = du; p.bp = wp; p.out = dx;
  p.M = (long long)N * H * W; p.Ncols = Cin; p.K = 4 * Cout;
  p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout; p.Hd = Hd; p.Wd = Wd; p.off_h = off_h; p.off_w = off_w;
  set_grid(p, Cin / TN);
  const dim3 grid = p.xcd ? dim3((unsigned)(pmu_cdiv(p.M, TM) * p.nnb)) : dim3((unsigned)pmu_cdiv(p.M, TM), (unsigned)p.nnb);
  hipLaunchKernelGGL(convT_bf16_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, p);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

#endif  // PMU_EXPERIMENTS

extern "C" size_t pmu_convT2x2_wgrad_ws_bf16(int N, int H, int W, int Cin, int Cout) {
  int nt, ns;
  twb_geometry(N, H, W, Cin, Cout, &nt, &ns);
  return ((size_t)ns * 4 * Cin * Cout + (size_t)DB_G * Cout) * sizeof(float);
}

extern "C" int pmu_convT2x2_wgrad_bf16(const unsigned short* xt, const unsigned short* dut, const float* du, int N, int H,
                                       int W, int Hd, int Wd, int off_h, int off_w, int Cin, int Cout, float* dw,
                                       float* dbias, float* ws, size_t ws_bytes, void* stream) {
  PMU_REQUIRE(xt && dut && dw && ws && N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0);
  PMU_REQUIRE(off_h >= 0 && off_w >= 0 && off_h + 2 * H <= Hd && off_w + 2 * W <= Wd && (!dbias || du));
  PMU_REQUIRE(ws_bytes >= pmu_convT2x2_wgrad_ws_bf16(N, H, W, Cin, Cout));
  PMU_REQUIRE((long long)N * 4 * H * W < (1LL << 32));  // the bias-sum pass decodes pixels in 32 bits
  PMU_REQUIRE((long long)N * Hd * Wd * pmu_cdiv(Cout, 8) * 8 < (1LL << 32));  // 32-bit du offsets
  TwbArgs a;
  a.xt = xt; a.dut = dut; a.ws = ws;
  a.N = N; a.H = H; a.W = W; a.Hd = Hd; a.Wd = Wd; a.oh = off_h; a.ow = off_w; a.Cin = Cin; a.Cout = Cout;
  a.Cip = (Cin + 7) & ~7; a.Cop = (Cout + 7) & ~7;
  twb_geometry(N, H, W, Cin, Cout, &a.ntiles, &a.nsplit);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)(pmu_cdiv(Cin, WCI) * pmu_cdiv(Cout, WCO)), (unsigned)a.nsplit);
  hipLaunchKernelGGL(convT_wgrad_bf16_kernel, grid, dim3(256), 0, st, a);
  PMU_CHECK_LAUNCH();
  const long long E = 4LL * Cin * Cout;
  hipLaunchKernelGGL(convT_wreduce_bf16_kernel, dim3((unsigned)pmu_cdiv(E, 64)), dim3(256), 0, st, (const float*)ws,
                     a.nsplit, Cin, Cout, dw);
  PMU_CHECK_LAUNCH();
  if (dbias) {
    float* part = ws + (size_t)a.nsplit * 4 * Cin * Cout;
    if (Cout % 4 == 0 && Cout <= 1024)
      hipLaunchKernelGGL(convT_dbias_part_kernel, dim3(DB_G), dim3(256), 0, st, du, N, 2 * H, 2 * W, Hd, Wd, off_h,
                         off_w, Cout, part);
    else
      hipLaunchKernelGGL(convT_dbias_part1_kernel, dim3(DB_G), dim3(256), 0, st, du, N, 2 * H, 2 * W, Hd, Wd, off_h,
                         off_w, Cout, part);
    PMU_CHECK_LAUNCH();
    hipLaunchKernelGGL(convT_dbias_sum_kernel, dim3((unsigned)pmu_cdiv(Cout, 64)), dim3(256), 0, st, (const float*)part,
                       DB_G, Cout, (long long)Cout, dbias);
    PMU_CHECK_LAUNCH();
  }
  return PMU_OK;
}

// dbias[c] = sum over r < R of part[r * ld + c] (c < Cout), fixed order: the bias gradient from the
// per-tile column sums of pmu_conv3x3_dgrad_dma_x1b_sum (part + Csplit, ld = 2 Cin).  Two passes: the
// rows in DB_RG contiguous groups (one block per 64 channels x group: thousands of rows per channel
// are a latency chain for one block) into ws[DB_RG][Cout], then those rows in order.
static constexpr int DB_RG = 64;
static __global__ __launch_bounds__(256) void dbias_rows_part_kernel(const float* __restrict__ part, int R, int Cout,
                                                              long long ld, float* __restrict__ ws) {
  const int g = blockIdx.y, r0 = (int)((long long)R * g / DB_RG), r1 = (int)((long long)R * (g + 1) / DB_RG);
  // (the one-block sum kernel over this group's rows, its 4 row sub-groups in order)
  __shared__ float red[256];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), grp = threadIdx.x >> 6;
  float s = 0.f;
  if (c < Cout) {
    const int a0 = r0 + ((r1 - r0) * grp) / 4, a1 = r0 + ((r1 - r0) * (grp + 1)) / 4;
#pragma unroll 4
    for (int r = a0; r < a1; ++r) s += part[(long long)r * ld + c];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (grp == 0 && c < Cout)
    ws[(long long)g * Cout + c] = ((red[threadIdx.x] + red[64 + threadIdx.x]) + red[128 + threadIdx.x]) + red[192 + threadIdx.x];
}

extern "C" size_t pmu_convT2x2_dbias_rows_ws(int Cout) { return (size_t)DB_RG * Cout * sizeof(float); }

extern "C" int pmu_convT2x2_dbias_rows(const float* part, int R, long long ld, int Cout, float* dbias, float* ws,
                                       void* stream) {
  PMU_REQUIRE(part && dbias && ws && R > 0 && Cout > 0 && ld >= Cout);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(dbias_rows_part_kernel, dim3((unsigned)pmu_cdiv(Cout, 64), DB_RG), dim3(256), 0, st, part, R,
                     Cout, ld, ws);
  PMU_CHECK_LAUNCH();
  hipLaunchKernelGGL(convT_dbias_sum_kernel, dim3((unsigned)pmu_cdiv(Cout, 64)), dim3(256), 0, st, (const float*)ws,
                     DB_RG, Cout, (long long)Cout, dbias);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
