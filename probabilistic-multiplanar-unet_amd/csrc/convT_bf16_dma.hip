// ConvTranspose2d(Cin, Cout, kernel 2, stride 2) of Up (PMU/model/unet/unet_parts.py:52), forward and
// input gradient on bf16 MFMA with both GEMM operands staged by LDS-DMA (config c5, autocast arithmetic).
//
//   forward : u[n][2i+a][2j+b][co] = bias[co] + sum_ci xt[pix][ci] * W[ci][co][a][b]
//             GEMM M = input pixels, N = 4 Cout (column ab*Cout + co), K = Cin; A = xt, the bf16 BN+ReLU
//             operand materialised once (pmu_frame_to_bf16; the weight gradient reads it too)
//   dgrad   : dx[pix][ci] = sum_{ab,co} du[n][oh+2i+a][ow+2j+b][co] * W[ci][co][a][b]
//             GEMM M = input pixels, N = Cin, K = 4 Cout (k = ab*Cout + co); A gathered from dut, the
//             bf16 du materialised once (its F.pad offset oh/ow inside the skip frame)
//
// 512 threads = 8 waves, a wave owns 128 rows x 64 columns (4 x 2 accumulators of 32x32x16); tiles
// 256 x 256 (NSTAGE = 4) or 512 x 128 (NSTAGE = 3) with 32-deep K chunks.  Every chunk's A and B
// tiles arrive by global_load_lds (16 B per lane) NSTAGE - 1 chunks ahead: one barrier per chunk, no
// staging registers.  Each DMA instruction writes 1 KB contiguously, so the LDS layout is a unit
// permutation: (row, 16-B unit q) at 4 row + (q XOR bits 2..3 of row), conflict-free for the
// 32x32x16 fragment reads; B is packed in global memory in that order (a straight copy).
#include <cstdlib>

#include "pmu_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BK = 32, NT = 512, NWV = 8, FM = 4, FN = 2;

__device__ __forceinline__ int tpos(int row, int q) { return 4 * row + (q ^ ((row >> 2) & 3)); }

struct GArgs {
  const unsigned short* a;    // fwd: xt [M][lda];  dgrad: dut [N][Hd][Wd][lda]
  const unsigned short* bp;   // packed B [nb][kc][BN x 4 units]
  const float* bias;
  float* out;                 // fwd: u [N][2H][2W][Cout];  dgrad: dx [M][Ncols]
  int M, Ncols, K, lda;
  int H, W, Cout, Hd, Wd, oh, ow;
  int nnb;
  int ldo;                    // fwd: output pixel stride (Cout, or the concat operand's width)
  unsigned short* outb;       // fwd, nullable: write bf16(u) here (pixel stride ldo) instead of out
  int pair;                   // outb 4-byte aligned and ldo even: channel pairs stored as one 4-byte word
  int w32;                    // fwd: W % 32 == 0 (a 32-pixel fragment never wraps an image row)
};

template <int WN>
struct TG {
  static constexpr int WM = NWV / WN;
  static constexpr int BM = 128 * WM, BN = 64 * WN;
  static constexpr int NSTAGE = WN == 4 ? 4 : 3;
  static constexpr int A_BYTES = BM * BK * 2, STAGE = (BM + BN) * BK * 2;
  static constexpr int NUA = BM * 4 / NT, NUB = BN * 4 / NT;
  static_assert(NSTAGE * STAGE <= 160 * 1024, "LDS");
};

__device__ __forceinline__ void convT_pack_dma_body(const float* __restrict__ w, int Cin, int Cout, int dgrad, int BN,
                                                    unsigned short* __restrict__ wp, int bid, int nblk) {
  const int Ncols = dgrad ? Cin : 4 * Cout, K = dgrad ? 4 * Cout : Cin;
  const int nkc = K / BK;
  const long long total = (long long)Ncols * K;
  for (long long e = (long long)bid * blockDim.x + threadIdx.x; e < total; e += (long long)nblk * blockDim.x) {
    const int el = (int)(e & 7);
    long long r = e >> 3;
    const int p = (int)(r % (BN * 4));
    r /= BN * 4;
    const int kc = (int)(r % nkc), nb = (int)(r / nkc);
    const int row = p >> 2, q = (p & 3) ^ ((row >> 2) & 3);
    const int n = nb * BN + row, k = kc * BK + 8 * q + el;
    int ci, co, ab;
    if (dgrad) { ci = n; ab = k / Cout; co = k - ab * Cout; }
    else { ci = k; ab = n / Cout; co = n - ab * Cout; }
    wp[e] = __builtin_bit_cast(unsigned short, (__bf16)w[((long long)ci * Cout + co) * 4 + ab]);
  }
}
__host__ __device__ __forceinline__ int convT_dma_bn(int Ncols) { return Ncols % 256 == 0 ? 256 : 128; }
__global__ __launch_bounds__(256) void convT_pack_dma_kernel(const float* __restrict__ w, int Cin, int Cout, int dgrad,
                                                             int BN, unsigned short* __restrict__ wp) {
  convT_pack_dma_body(w, Cin, Cout, dgrad, BN, wp, blockIdx.x, gridDim.x);
}
// job: .Cout = the ConvTranspose2d's in_channels, .Cin = its out_channels (as pmu_convT2x2_pack_multi)
__global__ __launch_bounds__(256) void convT_pack_dma_multi_kernel(const pmu_pack_job* __restrict__ jobs, int njobs,
                                                                   int dgrad) {
  const pmu_pack_job& j = jobs[pmu_job_of(jobs, njobs, blockIdx.x)];
  const int cin = j.Cout, cout = j.Cin;
  convT_pack_dma_body(j.w, cin, cout, dgrad, convT_dma_bn(dgrad ? cin : 4 * cout), (unsigned short*)j.dst,
                      blockIdx.x - j.block0, j.nblocks);
}

template <bool DGRAD, int WN>
__global__ __launch_bounds__(NT, 1) void convT_dma_kernel(GArgs g) {
  using G = TG<WN>;
  constexpr int NS = G::NSTAGE, BN = G::BN, NUA = G::NUA, NUB = G::NUB, NDMA = NUA + NUB;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NS * G::STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lb = pmu_xcd_block(blockIdx.x, gridDim.x);
  const int nb = lb % g.nnb, mb = lb / g.nnb;
  const int m0 = mb * G::BM, n0 = nb * BN;
  const int nkc = g.K / BK;
  PMU_DCHECK(m0 < g.M && n0 < g.Ncols, PMU_DBG_GRID);

  // A units of this thread: row and 16-B unit of each DMA round, as element offsets (rows past M
  // read row M - 1: every DMA is issued, so the vmcnt accounting below is exact; never stored)
  long long aoff[NUA];
  int aq[NUA];
#pragma unroll
  for (int r = 0; r < NUA; ++r) {
    const int p = (r * NWV + wave) * 64 + lane;
    const int row = p >> 2, q = (p & 3) ^ ((row >> 2) & 3);
    int m = m0 + row;
    m = m < g.M ? m : g.M - 1;
    aq[r] = 8 * q;
    if constexpr (DGRAD) {
      const unsigned t = (unsigned)m / (unsigned)g.W, j = (unsigned)m - t * (unsigned)g.W;
      const unsigned n = t / (unsigned)g.H, i = t - n * (unsigned)g.H;
      aoff[r] = ((long long)(n * g.Hd + g.oh + 2 * i) * g.Wd + g.ow + 2 * j) * g.lda;
    } else {
      aoff[r] = (long long)m * g.lda;
    }
  }
  const unsigned short* bsrc = g.bp + ((long long)nb * nkc * BN * 4 + (long long)wave * 64 + lane) * 8;

#define PMU_GLDS(S, D)                                                                                      \
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(S),                     \
                                   (__attribute__((address_space(3))) void*)(D), 16, 0, 0);
  auto fetch = [&](int kc) {
    unsigned char* st = smem + (kc % NS) * G::STAGE;
    long long koff;
    if constexpr (DGRAD) {  // 32 | Cout: one chunk lies inside one tap ab
      const int ab = (kc * BK) / g.Cout, co0 = kc * BK - ab * g.Cout;
      koff = ((long long)(ab >> 1) * g.Wd + (ab & 1)) * g.lda + co0;
    } else {
      koff = (long long)kc * BK;
    }
#pragma unroll
    for (int r = 0; r < NUA; ++r) PMU_GLDS(g.a + aoff[r] + koff + aq[r], st + (r * NWV + wave) * 1024)
    const unsigned short* bs = bsrc + (long long)kc * BN * 4 * 8;
#pragma unroll
    for (int r = 0; r < NUB; ++r) PMU_GLDS(bs + r * NT * 8, st + G::A_BYTES + (r * NWV + wave) * 1024)
  };

  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int li = lane & 31, hq = lane >> 5;
  int aro[FM], bro[FN];
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) aro[fm] = wm * 128 + fm * 32 + li;
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) bro[fn] = wn * 64 + fn * 32 + li;

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nkc) fetch(s);
  // wait until chunk c has landed (this thread's DMAs: at most min(NS - 2, nkc - 1 - c) later chunks may
  // stay outstanding), then a plain barrier: everyone's have, and every read of the chunk before c is
  // done.  (__syncthreads()' release fence would wait for every DMA in flight, the later chunks' too.)
  auto chunk_ready = [&](int c) {
    const int later = (nkc - 1 - c) < (NS - 2) ? (nkc - 1 - c) : (NS - 2);
    if (later >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NDMA) : "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  bf16x8 op[2][FM + FN];
  auto load = [&](const unsigned char* cur, int s, bf16x8 (&o)[FM + FN]) {
    const int q = 2 * s + hq;
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) o[fm] = *reinterpret_cast<const bf16x8*>(cur + 16 * tpos(aro[fm], q));
#pragma unroll
    for (int fn = 0; fn < FN; ++fn)
      o[FM + fn] = *reinterpret_cast<const bf16x8*>(cur + G::A_BYTES + 16 * tpos(bro[fn], q));
  };
  auto mfmas = [&](const bf16x8 (&o)[FM + FN]) {
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn)
        acc[fm][fn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o[fm], o[FM + fn], acc[fm][fn], 0, 0, 0);
  };
  // Each k-step's operands are read during the previous k-step's MFMAs — the next chunk's first one
  // during this chunk's second, after the chunk barrier — so no LDS round trip sits between a barrier
  // and the MFMAs (with the reads of both k-steps issued after the barrier, every chunk paid one).
  chunk_ready(0);
  load(smem, 0, op[0]);
  for (int kc = 0; kc < nkc; ++kc) {
    if (kc + NS - 1 < nkc) fetch(kc + NS - 1);   // into chunk kc - 1's stage: read by everyone (barrier)
    const unsigned char* cur = smem + (kc % NS) * G::STAGE;
    __builtin_amdgcn_s_waitcnt(0xC07F);           // lgkmcnt(0): k-step 0's operands
    __builtin_amdgcn_sched_barrier(0);
    load(cur, 1, op[1]);
    __builtin_amdgcn_sched_barrier(0);
    mfmas(op[0]);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);           // k-step 1's operands: this chunk's last reads
    __builtin_amdgcn_sched_barrier(0);
    if (kc + 1 < nkc) {
      chunk_ready(kc + 1);
      __builtin_amdgcn_sched_barrier(0);
      load(smem + ((kc + 1) % NS) * G::STAGE, 0, op[0]);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfmas(op[1]);
    __builtin_amdgcn_sched_barrier(0);
  }
#undef PMU_GLDS

  // epilogue
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int col = n0 + bro[fn];
    if constexpr (DGRAD) {
      if (g.outb) {
        // bf16 dx (pmu_convT2x2_dgrad_dma_dxb; RNE) as 4-byte channel pairs, as the forward's bf16 output:
        // the even lane stores row r's pair, the odd lane row r + 1's (Ncols % 128 == 0: pairs are aligned)
        const int odd = lane & 1;
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const unsigned b0 = __builtin_bit_cast(unsigned short, (__bf16)acc[fm][fn][r]);
            const unsigned b1 = __builtin_bit_cast(unsigned short, (__bf16)acc[fm][fn][r + 1]);
            const unsigned recv = pmu_swap1(odd ? b0 : b1);
            const unsigned pair = odd ? (recv | (b1 << 16)) : (b0 | (recv << 16));
            const int m = m0 + wm * 128 + fm * 32 + acc_row(r + odd, lane);
            if (m < g.M) {
              PMU_DCHECK(col < g.Ncols, PMU_DBG_OUTPUT);
              *reinterpret_cast<unsigned*>(g.outb + (long long)m * g.Ncols + col - odd) = pair;
            }
          }
        continue;
      }
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 128 + fm * 32 + acc_row(r, lane);
          if (m < g.M) {
            PMU_DCHECK(col < g.Ncols, PMU_DBG_OUTPUT);
            g.out[(long long)m * g.Ncols + col] = acc[fm][fn][r];
          }
        }
    } else {
      const int ab = col / g.Cout, co = col - ab * g.Cout;
      float b = g.bias ? g.bias[co] : 0.f;
      // consumed here, unconditionally (see convT.hip: first consumed inside the per-output store
      // branches, the bias cost a vmcnt(0) — a wait for every earlier store — per store)
      asm volatile("" : "+v"(b));
      const int ldo = g.ldo;
      const long long cbase = (long long)(ab >> 1) * 2 * g.W * ldo + (ab & 1) * ldo + co;
      float* outc = g.out + cbase;
      unsigned short* outcb = g.outb + cbase;
      if (g.outb && g.pair) {
        // bf16 output as 4-byte channel pairs: lanes 2k and 2k+1 hold adjacent channels of the same two
        // rows (r, r + 1); one xor-1 shuffle gives the even lane row r's pair and the odd lane row
        // r + 1's, so each stores 4 bytes (half the store instructions of 2-byte stores)
        const int odd = lane & 1;
#define PMU_CT_PAIR(FM_, R_)                                                                                \
  const unsigned b0 = __builtin_bit_cast(unsigned short, (__bf16)(acc[FM_][fn][R_] + b));                   \
  const unsigned b1 = __builtin_bit_cast(unsigned short, (__bf16)(acc[FM_][fn][(R_) + 1] + b));             \
  const unsigned recv = pmu_swap1(odd ? b0 : b1);                                                         \
  const unsigned pair = odd ? (recv | (b1 << 16)) : (b0 | (recv << 16));
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          const int mf = m0 + wm * 128 + fm * 32;  // (uniform) the fragment's first input pixel
          if (g.w32) {
            // W % 32 == 0: the fragment's 32 pixels lie in one image row (it starts at a multiple of
            // 32), so (n, i, j0) is decoded once per fragment (scalar) and pixel mf + x lands 2x output
            // pixels further along the same output row — no per-store integer division
            const unsigned t = (unsigned)mf / (unsigned)g.W, j0 = (unsigned)mf - t * (unsigned)g.W;
            const unsigned n = t / (unsigned)g.H, i = t - n * (unsigned)g.H;
            unsigned short* fp = outcb + ((long long)(n * 2 * g.H + 2 * i) * (2 * g.W) + 2 * j0) * ldo - odd;
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              PMU_CT_PAIR(fm, r)
              const int x = acc_row(r + odd, lane);
              if (mf + x < g.M) *reinterpret_cast<unsigned*>(fp + (unsigned)(2 * x) * (unsigned)ldo) = pair;
            }
          } else {
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              PMU_CT_PAIR(fm, r)
              const int m = mf + acc_row(r + odd, lane);
              if (m < g.M) {
                const unsigned t = (unsigned)m / (unsigned)g.W, j = (unsigned)m - t * (unsigned)g.W;
                const unsigned n = t / (unsigned)g.H, i = t - n * (unsigned)g.H;
                const long long o = ((long long)(n * 2 * g.H + 2 * i) * (2 * g.W) + 2 * j) * ldo - odd;
                *reinterpret_cast<unsigned*>(outcb + o) = pair;
              }
            }
          }
        }
#undef PMU_CT_PAIR
      } else {
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm * 128 + fm * 32 + acc_row(r, lane);
            if (m < g.M) {
              const unsigned t = (unsigned)m / (unsigned)g.W, j = (unsigned)m - t * (unsigned)g.W;
              const unsigned n = t / (unsigned)g.H, i = t - n * (unsigned)g.H;
              const long long o = ((long long)(n * 2 * g.H + 2 * i) * (2 * g.W) + 2 * j) * ldo;
              if (g.outb) outcb[o] = __builtin_bit_cast(unsigned short, (__bf16)(acc[fm][fn][r] + b));
              else outc[o] = acc[fm][fn][r] + b;
            }
          }
      }
    }
  }
}

static int dma_wn(int Ncols) { return convT_dma_bn(Ncols) / 64; }

template <bool DGRAD>
static int launch(GArgs& g, void* stream) {
  const int wn = dma_wn(g.Ncols);
  const int BM = 128 * (NWV / wn), BN = 64 * wn;
  g.w32 = (!DGRAD && g.W % 32 == 0) ? 1 : 0;
  g.nnb = g.Ncols / BN;
  const long long blocks = (long long)pmu_cdiv(g.M, BM) * g.nnb;
  PMU_REQUIRE(blocks < (1LL << 31));
  if (wn == 4)
    hipLaunchKernelGGL((convT_dma_kernel<DGRAD, 4>), dim3((unsigned)blocks), dim3(NT), 0, (hipStream_t)stream, g);
  else
    hipLaunchKernelGGL((convT_dma_kernel<DGRAD, 2>), dim3((unsigned)blocks), dim3(NT), 0, (hipStream_t)stream, g);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

}  // namespace

extern "C" int pmu_convT2x2_dma_ok(int Cin, int Cout, int dgrad) {
  const int Ncols = dgrad ? Cin : 4 * Cout, K = dgrad ? 4 * Cout : Cin;
  return Cin % BK == 0 && Cout % BK == 0 && Ncols % 128 == 0 && K % BK == 0;
}

extern "C" size_t pmu_convT2x2_packed_size_dma(int Cin, int Cout) { return (size_t)4 * Cin * Cout * 2; }

extern "C" int pmu_convT2x2_pack_dma(const float* w, int Cin, int Cout, int dgrad, unsigned short* wp, void* stream) {
  PMU_REQUIRE(w && wp && pmu_convT2x2_dma_ok(Cin, Cout, dgrad));
  const int Ncols = dgrad ? Cin : 4 * Cout;
  const long long total = 4LL * Cin * Cout;
  long long gsz = (total + 255) / 256;
  if (gsz > 4096) gsz = 4096;
  hipLaunchKernelGGL(convT_pack_dma_kernel, dim3((unsigned)gsz), dim3(256), 0, (hipStream_t)stream, w, Cin, Cout, dgrad,
                     64 * dma_wn(Ncols), wp);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_convT2x2_fwd_dma(const unsigned short* xt, int Cip, int N, int H, int W, const unsigned short* wp,
                                    const float* bias, int Cin, int Cout, float* u, void* stream) {
  PMU_REQUIRE(xt && wp && u && N > 0 && H > 0 && W > 0 && Cip >= Cin && Cip % 8 == 0);
  PMU_REQUIRE(pmu_convT2x2_dma_ok(Cin, Cout, 0) && (long long)N * H * W < (1LL << 31));
  GArgs g{};
  g.a = xt; g.bp = wp; g.bias = bias; g.out = u;
  g.M = N * H * W; g.Ncols = 4 * Cout; g.K = Cin; g.lda = Cip;
  g.H = H; g.W = W; g.Cout = Cout; g.ldo = Cout;
  return launch<false>(g, stream);
}

// The forward written as bf16 (RNE) into channels [0, Cout) of a wider NHWC bf16 tensor (pixel stride
// ldo): the up-sampled half of the Up block's bf16 concat operand (unet_parts.py:52,66 under autocast),
// so the operand materialisation copies only the skip half and no fp32 u is written at all.
extern "C" int pmu_convT2x2_fwd_dma_ldb(const unsigned short* xt, int Cip, int N, int H, int W,
                                        const unsigned short* wp, const float* bias, int Cin, int Cout,
                                        unsigned short* ub, int ldo, void* stream) {
  PMU_REQUIRE(xt && wp && ub && N > 0 && H > 0 && W > 0 && Cip >= Cin && Cip % 8 == 0 && ldo >= Cout);
  PMU_REQUIRE(pmu_convT2x2_dma_ok(Cin, Cout, 0) && (long long)N * H * W < (1LL << 31));
  GArgs g{};
  g.a = xt; g.bp = wp; g.bias = bias; g.out = nullptr; g.outb = ub;
  g.M = N * H * W; g.Ncols = 4 * Cout; g.K = Cin; g.lda = Cip;
  g.H = H; g.W = W; g.Cout = Cout; g.ldo = ldo;
  g.pair = (ldo % 2 == 0 && (reinterpret_cast<uintptr_t>(ub) & 3) == 0) ? 1 : 0;
  return launch<false>(g, stream);
}

extern "C" int pmu_convT2x2_dgrad_dma(const unsigned short* dut, int Cop, int Hd, int Wd, int off_h, int off_w,
                                      const unsigned short* wp, int N, int H, int W, int Cin, int Cout, float* dx,
                                      void* stream) {
  PMU_REQUIRE(dut && wp && dx && N > 0 && H > 0 && W > 0 && Cop >= Cout && Cop % 8 == 0);
  PMU_REQUIRE(pmu_convT2x2_dma_ok(Cin, Cout, 1) && (long long)N * H * W < (1LL << 31));
  PMU_REQUIRE(off_h >= 0 && off_w >= 0 && off_h + 2 * H <= Hd && off_w + 2 * W <= Wd);
  GArgs g{};
  g.a = dut; g.bp = wp; g.out = dx;
  g.M = N * H * W; g.Ncols = Cin; g.K = 4 * Cout; g.lda = Cop;
  g.H = H; g.W = W; g.Cout = Cout; g.Hd = Hd; g.Wd = Wd; g.oh = off_h; g.ow = off_w;
  return launch<true>(g, stream);
}

// The input gradient stored as bf16 (RNE; the dtype torch.autocast's ConvTranspose2d backward returns it
// in): the consumer's BN backward reads it (pmu_bn_bwd_reduce_dxb, the BN-backward frames).
extern "C" int pmu_convT2x2_dgrad_dma_dxb(const unsigned short* dut, int Cop, int Hd, int Wd, int off_h, int off_w,
                                          const unsigned short* wp, int N, int H, int W, int Cin, int Cout,
                                          unsigned short* dx, void* stream) {
  PMU_REQUIRE(dut && wp && dx && N > 0 && H > 0 && W > 0 && Cop >= Cout && Cop % 8 == 0);
  PMU_REQUIRE(pmu_convT2x2_dma_ok(Cin, Cout, 1) && (long long)N * H * W < (1LL << 31));
  PMU_REQUIRE(off_h >= 0 && off_w >= 0 && off_h + 2 * H <= Hd && off_w + 2 * W <= Wd);
  GArgs g{};
  g.a = dut; g.bp = wp; g.out = nullptr; g.outb = dx;
  g.M = N * H * W; g.Ncols = Cin; g.K = 4 * Cout; g.lda = Cop;
  g.H = H; g.W = W; g.Cout = Cout; g.Hd = Hd; g.Wd = Wd; g.oh = off_h; g.ow = off_w;
  return launch<true>(g, stream);
}

static int convT_pack_dma_grid(int Cin, int Cout) {
  const long long g = (4LL * Cin * Cout + 255) / 256;
  return (int)(g > 4096 ? 4096 : g);
}

extern "C" int pmu_convT2x2_pack_dma_blocks(int Cin, int Cout, int dgrad) {
  (void)dgrad;
  return convT_pack_dma_grid(Cin, Cout);
}

// jobs[]: .Cout = the ConvTranspose2d's in_channels, .Cin = its out_channels
extern "C" int pmu_convT2x2_pack_dma_multi(const pmu_pack_job* jobs, int njobs, int blocks, int dgrad, void* stream) {
  PMU_REQUIRE(jobs && njobs > 0 && blocks > 0);
  hipLaunchKernelGGL(convT_pack_dma_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, jobs,
                     njobs, dgrad);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
