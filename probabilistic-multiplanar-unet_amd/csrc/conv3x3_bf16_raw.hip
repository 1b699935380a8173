// 3x3 / pad 1 convolution of a materialised bf16 operand on bf16 MFMA (config c5's main path).
//
// nn.Conv2d(k=3, padding=1) of DoubleConv (PMU/model/unet/unet_parts.py:15,18) forward, and its
// input gradient, with torch.autocast(bfloat16) arithmetic.  In bf16 mode every conv operand is
// first written once as a dense bf16 NHWC tensor by one streaming pass (pmu_frame_to_bf16: the
// producer's BatchNorm + ReLU, the max-pool, the F.pad + torch.cat of the skip connection, or
// the BN+ReLU backward of dz), which the weight gradient needs anyway.  The GEMM kernel then only
// copies 16-B units into LDS: half the bytes of the fp32 sources (a quarter for dz), no transform
// arithmetic and half the prefetch registers of the fused-staging kernel (conv3x3_bf16.hip).
//
// GEMM view: M = 256 output pixels (TH x TW tile), N = 64 output channels, K = 9 taps x channels,
// chunks of 32 channels: the (TH+2) x (TW+2) halo tile (80-B rows) and 9 x 64 x 32 packed weights
// are staged per chunk, each tap is two 32x32x16 k-steps.  4 waves of 64 px x 64 ch (2 x 2
// accumulators), 2 blocks per CU (73 KB LDS), the next chunk's 15 units per thread in registers
// under the current chunk's 72 MFMAs per wave.
#include <cstdlib>

#include "pmu_stage.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BNT = 64, BK = 32;
constexpr int LS = 40;       // LDS row stride (bf16): 64 B of data + 16 B pad, ds_read_b128 conflict-free
constexpr int B_UNITS = 9 * BNT * BK / 8;  // 2304 16-B units of packed weights per chunk
constexpr int B_EL = 9 * BNT * LS;

// Tile of BMT pixels (= threads: one wave per 64 pixels).  BMT = 512 halves the weight bytes per
// FLOP of BMT = 256: the per-CU vector-memory path (64 B/clk) bounds the 256-pixel tile at ~1/3 of
// the MFMA rate (58 KB per chunk per block), the 512-pixel tile needs 16.5 B/clk at full rate.
template <int BMT>
struct RawGeo {
  static constexpr int MAX_HP = BMT == 512 ? 660 : 340;  // (TH+2)*(TW+2) over TW in {8,16,32}
  static constexpr int A_EL = MAX_HP * LS;
  static constexpr int NA = (MAX_HP * 4 + BMT - 1) / BMT;  // A units per thread
  static constexpr int NB = (B_UNITS + BMT - 1) / BMT;     // B units per thread
};

struct RawArgs {
  const unsigned short* x;   // operand [N][H][W][Cp] bf16
  const unsigned short* wp;  // packed [jb][ch][tap][64][32] bf16
  const float* bias;
  float* out0;
  float* out1;
  float* part;
  int N, H, W, Cp, NOUT, split, tiles_w, tiles_h, nch;
  int ncb, xcd;              // output-channel blocks; 1: 1-D XCD-ordered grid, channel blocks fastest
};

__device__ __forceinline__ unsigned short bf16_bits(float v) { return __builtin_bit_cast(unsigned short, (__bf16)v); }

// wp[jb][ch][tap][jl][kl] = B[tap][j = 64 jb + jl][k = 32 ch + kl], zero padded, bf16 RNE
//   forward: B[tap][co][ci] = w[co][ci][tap];  dgrad: B[tap][ci][co] = w[co][ci][8 - tap]
__global__ __launch_bounds__(256) void pack_raw_kernel(const float* __restrict__ w, int Cout, int Cin, int dgrad,
                                                       unsigned short* __restrict__ wp) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  const int nch = (KC + BK - 1) / BK, njb = (NOUT + BNT - 1) / BNT;
  const long long total = (long long)njb * nch * 9 * BNT * BK;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int kl = (int)(e % BK);
    long long r = e / BK;
    const int jl = (int)(r % BNT); r /= BNT;
    const int tap = (int)(r % 9); r /= 9;
    const int ch = (int)(r % nch);
    const int jb = (int)(r / nch);
    const int j = jb * BNT + jl, k = ch * BK + kl;
    float v = 0.f;
    if (j < NOUT && k < KC)
      v = dgrad ? w[((long long)k * Cin + j) * 9 + (8 - tap)] : w[((long long)j * Cin + k) * 9 + tap];
    wp[e] = bf16_bits(v);
  }
}

template <bool DGRAD, int TWL, int BMT>
__global__ __launch_bounds__(BMT, 2) void conv3x3_raw_kernel(RawArgs a) {
  using G = RawGeo<BMT>;
  constexpr int FM = 2, FN = 2, NA = G::NA, NB = G::NB, NWV = BMT / 64;
  constexpr int TW = 1 << TWL, TH = BMT >> TWL, HW2 = TW + 2, HP = (TH + 2) * HW2;
  static_assert(HP <= G::MAX_HP, "halo tile fits");
  __shared__ __attribute__((aligned(16))) unsigned short smem[G::A_EL + B_EL];
  unsigned short* As = smem;
  unsigned short* Bs = smem + G::A_EL;
  const int tid = threadIdx.x, lane = tid & 63, wm = tid >> 6;
  // (spatial tile, output-channel block): with a.xcd the channel blocks of one spatial tile run
  // back to back on one XCD, so its halo operand is fetched from HBM once and re-read from L2
  int t, cb;
  if (a.xcd) {
    const int lb = pmu_xcd_block(blockIdx.x, gridDim.x);
    cb = lb % a.ncb;
    t = lb / a.ncb;
  } else {
    t = blockIdx.x;
    cb = blockIdx.y;
  }
  const int tsp = t;
  const int tw = t % a.tiles_w; t /= a.tiles_w;
  const int th = t % a.tiles_h; t /= a.tiles_h;
  const int n = t;
  const int h0 = th * TH, w0 = tw * TW;
  const int j0 = cb * BNT;
  PMU_DCHECK(n < a.N && j0 < a.NOUT, PMU_DBG_GRID);

  // A units: halo pixel hp = it >> 2, 8-channel unit q = it & 3; tile-constant 32-bit offsets
  int eo[NA], dsta[NA];
  unsigned okm = 0u, vm = 0u;
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    // unit -> (halo pixel, 8-channel unit) so that each 8-lane ds_write_b128 group covers 8 rows of
    // one unit column: conflict-free on the 80-B rows (row-major pairs of rows would be 2-way)
    const int it = tid + BMT * i;
    const int hp = (it >> 5) * 8 + (it & 7), q = (it >> 3) & 3;
    const int hr = hp / HW2, hc = hp - hr * HW2;
    const int h = h0 - 1 + hr, w = w0 - 1 + hc;
    const bool v = hp < HP;
    const bool ok = v && h >= 0 && w >= 0 && h < a.H && w < a.W;
    vm |= v ? (1u << i) : 0u;
    okm |= ok ? (1u << i) : 0u;
    eo[i] = ok ? ((n * a.H + h) * a.W + w) * a.Cp + 8 * q : 0;
    PMU_DCHECK(!ok || ((long long)(n * a.H + h) * a.W + w) < (long long)a.N * a.H * a.W, PMU_DBG_OPERAND);
    dsta[i] = hp * LS + 8 * q;
  }
  const int hsel = (lane >> 5) * 8;
  int abase[FM], bbase[FN];
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    const int q = wm * 64 + fm * 32 + (lane & 31);
    abase[fm] = ((q >> TWL) * HW2 + (q & (TW - 1))) * LS + hsel;
  }
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) bbase[fn] = (fn * 32 + (lane & 31)) * LS + hsel;

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int bq = (tid >> 3) & 3;  // B unit of this thread within its row (BMT is a multiple of 32)
  const uint4* wt = reinterpret_cast<const uint4*>(a.wp) + (long long)(j0 / BNT) * a.nch * B_UNITS +
                    ((tid >> 5) * 8 + (tid & 7)) * 4 + bq;
  uint4 ra0, ra1, ra2, ra3, ra4, ra5;                     // plain locals (no scratch)
  unsigned kmask = 0u;                                    // A units in range (zeroed at commit)
  uint4 rb0, rb1, rb2, rb3, rb4, rb5, rb6, rb7, rb8;
  static_assert(NA <= 6 && NB <= 9, "staging register layout");
  // channel units past Cp (a partial last chunk) read as zero
#define PMU_RA(I, R)                                                                               \
  if ((I) < NA) {                                                                                 \
    const bool k_ = ((okm >> (I)) & 1u) && k0_ + 8 * ((tid >> 3) & 3) < a.Cp;              \
    R = *reinterpret_cast<const uint4*>(a.x + (k_ ? (unsigned)(eo[I] + k0_) : 0u));               \
    kmask = k_ ? (kmask | (1u << (I))) : (kmask & ~(1u << (I)));                                  \
  }
#define PMU_RB(I, R) \
  if ((I) < NB) R = s_[(B_UNITS % BMT == 0 || (I) + 1 < NB || tid + BMT * (I) < B_UNITS) ? BMT * (I) : 0];
  // (B units use the same row-interleaved order as A: see wt and PMU_WB)
#define PMU_PREFETCH(CH)                                                                           \
  {                                                                                               \
    const int k0_ = (CH) * BK;                                                                    \
    PMU_RA(0, ra0) PMU_RA(1, ra1) PMU_RA(2, ra2) PMU_RA(3, ra3) PMU_RA(4, ra4) PMU_RA(5, ra5)    \
    const uint4* s_ = wt + (long long)(CH) * B_UNITS;                                             \
    PMU_RB(0, rb0) PMU_RB(1, rb1) PMU_RB(2, rb2) PMU_RB(3, rb3) PMU_RB(4, rb4)                    \
    PMU_RB(5, rb5) PMU_RB(6, rb6) PMU_RB(7, rb7) PMU_RB(8, rb8)                                   \
  }
#define PMU_WA(I, R)                                                                               \
  if ((I) < NA && ((vm >> (I)) & 1u)) {                                                           \
    const bool k_ = (kmask >> (I)) & 1u; /* zeroed here, not at the load: no wait before the MFMAs */ \
    *reinterpret_cast<uint4*>(As + dsta[I]) =                                                     \
        make_uint4(k_ ? R.x : 0u, k_ ? R.y : 0u, k_ ? R.z : 0u, k_ ? R.w : 0u);                  \
  }
#define PMU_WB(I, R)                                                                               \
  if ((I) < NB && (B_UNITS % BMT == 0 || (I) + 1 < NB || tid + BMT * (I) < B_UNITS))               \
    *reinterpret_cast<uint4*>(Bs + (((tid + BMT * (I)) >> 5) * 8 + (tid & 7)) * LS + 8 * bq) = R;
#define PMU_COMMIT()                                                                               \
  {                                                                                               \
    PMU_WA(0, ra0) PMU_WA(1, ra1) PMU_WA(2, ra2) PMU_WA(3, ra3) PMU_WA(4, ra4) PMU_WA(5, ra5)    \
    PMU_WB(0, rb0) PMU_WB(1, rb1) PMU_WB(2, rb2) PMU_WB(3, rb3) PMU_WB(4, rb4)                    \
    PMU_WB(5, rb5) PMU_WB(6, rb6) PMU_WB(7, rb7) PMU_WB(8, rb8)                                   \
  }

  PMU_PREFETCH(0)
  PMU_COMMIT()
  __syncthreads();
  for (int ch = 0; ch < a.nch; ++ch) {
    const bool more = ch + 1 < a.nch;
    if (more) PMU_PREFETCH(ch + 1)  // in flight during the MFMAs below
    // Operands move a whole tap (both k-steps: 8 x ds_read_b128) ahead of its 8 MFMAs; the
    // scheduling barriers keep the compiler from sinking each read next to its first use (it did:
    // one LDS round trip exposed every two MFMAs).
    bf16x8 op[2][2][FM + FN];
    auto load_tap = [&](int tap, bf16x8 (&o)[2][FM + FN]) {
      const int toff = ((tap / 3) * HW2 + (tap % 3)) * LS;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) o[s][fm] = *reinterpret_cast<const bf16x8*>(As + abase[fm] + toff + 16 * s);
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          o[s][FM + fn] = *reinterpret_cast<const bf16x8*>(Bs + tap * BNT * LS + bbase[fn] + 16 * s);
      }
    };
    load_tap(0, op[0]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap + 1 < 9) load_tap(tap + 1, op[(tap + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn)
            acc[fm][fn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(op[tap & 1][s][fm], op[tap & 1][s][FM + fn],
                                                                   acc[fm][fn], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    if (more) {
      PMU_COMMIT()
      __syncthreads();
    }
  }
#undef PMU_RA
#undef PMU_RB
#undef PMU_PREFETCH
#undef PMU_WA
#undef PMU_WB
#undef PMU_COMMIT

  // epilogue: per 32-channel block the destination is uniform (split % 32 == 0, host-checked);
  // full tiles store without bounds tests
  float* red = reinterpret_cast<float*>(smem);  // [NWV][64][2]
  float s1[FN], s2[FN];
  const bool full = h0 + TH <= a.H && w0 + TW <= a.W && j0 + BNT <= a.NOUT;
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
        const int q = wm * 64 + fm * 32 + acc_row(r, lane);
        const int h = h0 + (q >> TWL), w = w0 + (q & (TW - 1));
        if (!full && (!jok || h >= a.H || w >= a.W)) continue;
        const unsigned pix = (unsigned)((n * a.H + h) * a.W + w);
        PMU_DCHECK(pix < (unsigned)(a.N * a.H * a.W) && j < a.NOUT, PMU_DBG_OUTPUT);
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
        for (int v = 0; v < NWV; ++v) {
          t1 += red[(v * BNT + tid) * 2 + 0];
          t2 += red[(v * BNT + tid) * 2 + 1];
        }
        PMU_DCHECK(tsp < a.N * a.tiles_h * a.tiles_w, PMU_DBG_WORKSPACE);
        a.part[((long long)tsp * 2 + 0) * a.NOUT + j] = t1;
        a.part[((long long)tsp * 2 + 1) * a.NOUT + j] = t2;
      }
    }
  }
}

static int pick_twl(int W) {
  if (W > 16) return 5;
  if (W > 8) return 4;
  return 3;
}

// pixels per tile: PMU_RAW_BMT=256|512 forces one (A/B measurements); default 256
static int raw_bmt(int N, int H, int W, int TW, int ncb) {
  static const int forced = [] {
    const char* e = pmu_variant_env("PMU_RAW_BMT");
    return e ? atoi(e) : 0;
  }();
  if (forced == 256 || forced == 512) return forced;
  (void)N; (void)H; (void)W; (void)TW; (void)ncb;
  return 256;
}

static int launch_raw(const unsigned short* x, int Cp, int N, int H, int W, const unsigned short* wp,
                      const float* bias, int NOUT, float* out0, float* out1, int split, float* part, bool dgrad,
                      void* stream) {
  PMU_REQUIRE(x && wp && out0 && N > 0 && H > 0 && W > 0 && Cp > 0 && Cp % 8 == 0 && NOUT > 0);
  PMU_REQUIRE((long long)N * H * W * Cp < (1LL << 31));
  PMU_REQUIRE(!dgrad || split == NOUT || (split % 32 == 0 && split < NOUT && out1));
  RawArgs a;
  a.x = x; a.wp = wp; a.bias = bias; a.out0 = out0; a.out1 = out1; a.part = part;
  a.N = N; a.H = H; a.W = W; a.Cp = Cp; a.NOUT = NOUT; a.split = dgrad ? split : NOUT;
  a.nch = pmu_cdiv(Cp, BK);
  const int twl = pick_twl(W);
  const int TW = 1 << twl;
  const int ncb = pmu_cdiv(NOUT, BNT);
  // 512-pixel tiles when they still give the chip >= 2 blocks per CU; part (BN partials) is then
  // indexed by the 512-pixel tile (pmu_conv3x3_tiles_raw)
  const int bmt = raw_bmt(N, H, W, TW, ncb);
  const int TH = bmt / TW;
  a.tiles_w = pmu_cdiv(W, TW);
  a.tiles_h = pmu_cdiv(H, TH);
  static const int xcd = [] {
    const char* e = pmu_variant_env("PMU_RAW_XCD");
    return e ? atoi(e) : 1;
  }();
  a.ncb = ncb;
  a.xcd = xcd;
  const dim3 grid = xcd ? dim3((unsigned)(a.tiles_w * a.tiles_h * N * ncb)) : dim3((unsigned)(a.tiles_w * a.tiles_h * N), (unsigned)ncb);
  hipStream_t st = (hipStream_t)stream;
#define PMU_RK(D, T, B)                                                                 \
  if (dgrad == D && twl == T && bmt == B) {                                             \
    hipLaunchKernelGGL((conv3x3_raw_kernel<D, T, B>), grid, dim3(B), 0, st, a);         \
    PMU_CHECK_LAUNCH();                                                                 \
    return PMU_OK;                                                                      \
  }
  PMU_RK(false, 3, 256) PMU_RK(false, 4, 256) PMU_RK(false, 5, 256)
  PMU_RK(true, 3, 256) PMU_RK(true, 4, 256) PMU_RK(true, 5, 256)
  PMU_RK(false, 3, 512) PMU_RK(false, 4, 512) PMU_RK(false, 5, 512)
  PMU_RK(true, 3, 512) PMU_RK(true, 4, 512) PMU_RK(true, 5, 512)
#undef PMU_RK
  return PMU_ERR_ARG;
}

static int raw_tiles(int N, int H, int W, int NOUT) {
  const int TW = 1 << pick_twl(W);
  const int ncb = pmu_cdiv(NOUT, BNT);
  const int bmt = raw_bmt(N, H, W, TW, ncb);
  return N * pmu_cdiv(H, bmt / TW) * pmu_cdiv(W, TW);
}

}  // namespace

extern "C" int pmu_conv3x3_tiles_raw(int N, int H, int W, int Cout) { return raw_tiles(N, H, W, Cout); }

extern "C" size_t pmu_conv3x3_packed_size_raw(int Cout, int Cin, int dgrad) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  return (size_t)pmu_cdiv(NOUT, BNT) * pmu_cdiv(KC, BK) * 9 * BNT * BK * sizeof(unsigned short);
}

extern "C" int pmu_conv3x3_pack_raw(const float* w, int Cout, int Cin, int dgrad, unsigned short* wp, void* stream) {
  PMU_REQUIRE(w && wp && Cout > 0 && Cin > 0);
  const long long total = (long long)(pmu_conv3x3_packed_size_raw(Cout, Cin, dgrad) / sizeof(unsigned short));
  long long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(pack_raw_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, dgrad, wp);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_conv3x3_fwd_raw(const unsigned short* xt, int Cp, int N, int H, int W, const unsigned short* wp,
                                   const float* bias, int Cout, float* z, float* part, void* stream) {
  return launch_raw(xt, Cp, N, H, W, wp, bias, Cout, z, nullptr, Cout, part, false, stream);
}

extern "C" int pmu_conv3x3_dgrad_raw(const unsigned short* dzt, int Cp, int N, int H, int W, const unsigned short* wp,
                                     int Cin, int Csplit, float* dx0, float* dx1, void* stream) {
  return launch_raw(dzt, Cp, N, H, W, wp, nullptr, Cin, dx0, dx1, Csplit, nullptr, true, stream);
}

// Diagnostic: resident blocks per CU of the main kernel of this file (hipOccupancy API).
extern "C" int pmu_occupancy_conv3x3_raw(int* blocks_per_cu) {
  PMU_REQUIRE(blocks_per_cu);
  int n = 0;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(conv3x3_raw_kernel<false, 5, 256>), 256, 0);
  if (e != hipSuccess) return (int)e;
  *blocks_per_cu = n;
  return PMU_OK;
}
